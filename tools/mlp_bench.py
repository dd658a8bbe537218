"""MLP microbenchmark: N = 2^22 points U[-1,1]^3 (default_rng(0)),
fp32 xyz in, fp32 SDF out, through nr_mlp_forward on device buffers.

Reports TFLOP/s over the whole network (14,592 FLOP per point) and the matrix-core
utilisation of the 7 hidden 32x32 layers (14,336 FLOP per point) against the dense
peak of the precision (MI355X_MICROARCH.md: f32 157.3, bf16/fp16 2516.6 TFLOP/s)."""
import argparse
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import cudaneuralrender_amd as nr  # noqa: E402

PEAK = {"fp32": 157.3, "bf16": 2516.6, "fp16": 2516.6, "fp32x3": 2516.6}
# matrix-core FLOP issued per algorithmic FLOP of the hidden layers (fp32x3: three fp16 terms)
ISSUED = {"fp32": 1, "bf16": 1, "fp16": 1, "fp32x3": 3}
ap = argparse.ArgumentParser()
ap.add_argument("--n", type=int, default=1 << 22)
ap.add_argument("--iters", type=int, default=20)
ap.add_argument("--precision", default="all")
ap.add_argument("--bpc", default="0", help="workgroups per CU (0: the library default: 12, or for bf16/fp16 3 with the dynamic tail)")
ap.add_argument("--debug", type=int, default=0, help="nr_set_debug flags (A/B of the bf16 ReLU forms: 512)")
a = ap.parse_args()
X = np.random.default_rng(0).uniform(-1, 1, size=(a.n, 3)).astype(np.float32)
dX = torch.from_numpy(X).cuda()
dY = torch.zeros(a.n, dtype=torch.float32, device="cuda")
r = nr.Renderer(0).load_h5(nr.geometry_path("plane_1"))
r.set_stream(torch.cuda.current_stream().cuda_stream)
r.set_debug(a.debug)
res = []
for prec in (["fp32", "bf16", "fp16"] if a.precision == "all" else a.precision.split(",")):
    for bpc in (int(b) for b in a.bpc.split(",")):
        r.set_occupancy(bpc)
        r.set_precision(prec)
        for _ in range(3):
            r.mlp_forward_device(dX.data_ptr(), dY.data_ptr(), a.n)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(a.iters):
            r.mlp_forward_device(dX.data_ptr(), dY.data_ptr(), a.n)
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / a.iters
        tf = a.n * 14592 / (ms * 1e-3) / 1e12
        util = a.n * 14336 * ISSUED[prec] / (ms * 1e-3) / 1e12 / PEAK[prec]
        res.append({"precision": prec, "debug": a.debug, "tile": "16" if prec == "fp32" else "32", "issued_per_flop": ISSUED[prec], "blocks_per_cu": bpc, "n": a.n, "ms": round(ms, 4), "TFLOPs": round(tf, 2),
                    "hidden_layer_mfma_util": round(util, 4), "Gpoints_per_s": round(a.n / ms / 1e6, 2)})
        print(json.dumps(res[-1]), flush=True)
