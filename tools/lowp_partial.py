"""Diagnostic: the reduced-precision MLP on partial 64-point chunks (n = 1..64 points, so the
last chunk runs 1 or 2 of its 32-point tiles) against the same points inside full chunks."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import cudaneuralrender_amd as nr  # noqa: E402

X = np.random.default_rng(0).uniform(-1, 1, size=(64 * 64, 3)).astype(np.float32)
r = nr.Renderer(0).load_h5(nr.geometry_path("car_1"))
for prec in ("fp32", "bf16", "fp16"):
    r.set_precision(prec)
    full = r.mlp_forward(X)[:, 0]
    bad = []
    for n in range(1, 65):
        y = r.mlp_forward(X[:n])[:, 0]
        if not np.array_equal(y, full[:n]):
            bad.append((n, int((y != full[:n]).sum()), int(np.argmax(y != full[:n]))))
    print(prec, "partial chunks differing from full-chunk results (n, count, first):", bad[:12], flush=True)
