"""Offline (no GPU): how well each of the oracle's MFMA summation models (nr_oracle.c mfma_sum)
reproduces the GPU's 16-bit and fp32x3 MLP outputs dumped by tools/dump_mlp.py.

    python tools/fit_emulation.py gpurun_out/mlp_dump.npz [--models 0,1,2:24,2:25,2:26]"""
import argparse
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import cudaneuralrender_amd as nr  # noqa: E402
import oracle  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("dump")
ap.add_argument("--models", default="0,1,2:24,2:25,2:26,2:27,2:28")
ap.add_argument("--n", type=int, default=4096)
a = ap.parse_args()
z = np.load(a.dump)
X = z["X"][: a.n]
geoms = sorted({k.split("/")[0] for k in z.files if "/" in k})
PREC = {"bf16": 1, "fp16": 2, "fp32x3": 4}
for spec in a.models.split(","):
    model, w = (int(spec.split(":")[0]), int(spec.split(":")[1])) if ":" in spec else (int(spec), 26)
    oracle.set_mfma_model(model, w)
    row = {"model": spec}
    for g in geoms:
        dims, K, B = nr.read_keras_h5(nr.geometry_path(g))
        pack = nr.pack_x3(dims, K, B)
        net = oracle.OracleNet(K, B, x3_pack=pack[:2])
        for prec, p in PREC.items():
            y = z[f"{g}/{prec}"][: a.n]
            e = net.forward(X, precision=p)[:, 0]
            row[f"{g[:8]}/{prec}"] = round(float((y == e).mean()), 4)
    print(json.dumps(row), flush=True)
oracle.set_mfma_model(3, 26)
