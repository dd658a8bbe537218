"""Diagnostic (GPU box): the 16-bit and fp32x3 MLP outputs of every bundled network on a fixed
point cloud, saved for offline fitting of the oracle's MFMA emulation (tools/mfma_model.py).

    python tools/dump_mlp.py out.npz"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import cudaneuralrender_amd as nr  # noqa: E402

GEOMS = ["plane_1", "plane_2", "plane_3", "car_1", "3a3d4a90a2db90b4203936772104a82d.obj"]
X = np.random.default_rng(11).uniform(-1.2, 1.2, size=(16384, 3)).astype(np.float32)
out = {"X": X}
with nr.Renderer(0) as r:
    for g in GEOMS:
        r.load_h5(nr.geometry_path(g))
        for prec in ("fp32x3", "bf16", "fp16", "fp32"):
            out[f"{g}/{prec}"] = r.set_precision(prec).mlp_forward(X)[:, 0]
np.savez_compressed(sys.argv[1], **out)
print("saved", len(out))
