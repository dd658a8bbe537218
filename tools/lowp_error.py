"""Reduced-precision MLP error on the KAT points (tests/golden/mlp_kat.npz) of every bundled
geometry: max / mean |y - y_fp64| for bf16 and fp16 through nr_mlp_forward.  GPU box."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import cudaneuralrender_amd as nr  # noqa: E402

kat = np.load(os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests", "golden", "mlp_kat.npz"))
X = kat["X"]
r = nr.Renderer(0)
for g in sorted(k for k in kat.files if k != "X"):
    r.load_h5(nr.geometry_path(g))
    line = [g]
    for prec in ("fp32", "bf16", "fp16"):
        r.set_precision(prec)
        e = np.abs(r.mlp_forward(X)[:, 0].astype(np.float64) - kat[g])
        line.append(f"{prec} max {e.max():.2e} mean {e.mean():.2e}")
    print("  ".join(line), flush=True)
