"""Interleaved A/B of the 16-bit k_mlp16's launch forms (GPU box): each round times every form once
(back-to-back launches after a warmup), rounds repeated, medians reported -- so that the clock's
drift over a run does not favour whichever form is measured first (a sequential A/B saw the first
form ~10 % slower whatever it was).

    python tools/mlp_ab.py [--n 16777216] [--rounds 7] [--iters 10] [--precision bf16]
Forms: "cuq" (one 12-wave workgroup per CU, LDS chunk queue: nr_set_debug bit 12), "gs3" / "gs12"
(grid-stride, 3 or 12 four-wave workgroups per CU, nr_set_occupancy; gs12 is the library default)."""
import argparse
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import cudaneuralrender_amd as nr  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--n", type=int, default=1 << 24)
ap.add_argument("--rounds", type=int, default=7)
ap.add_argument("--iters", type=int, default=10)
ap.add_argument("--precision", default="bf16,fp16")
ap.add_argument("--forms", default="cuq,gs3,gs12")
a = ap.parse_args()
X = torch.from_numpy(np.random.default_rng(0).uniform(-1, 1, size=(a.n, 3)).astype(np.float32)).cuda()
Y = torch.zeros(a.n, dtype=torch.float32, device="cuda")
r = nr.Renderer(0).load_h5(nr.geometry_path("plane_1"))
r.set_stream(torch.cuda.current_stream().cuda_stream)
FORMS = {"cuq": (4096, 0), "gs3": (0, 3), "gs12": (0, 12)}
for prec in a.precision.split(","):
    r.set_precision(prec)
    times = {f: [] for f in a.forms.split(",")}
    for rnd in range(a.rounds):
        for f in times:
            dbg, bpc = FORMS[f]
            r.set_debug(dbg)
            r.set_occupancy(bpc)
            for _ in range(3):
                r.mlp_forward_device(X.data_ptr(), Y.data_ptr(), a.n)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(a.iters):
                r.mlp_forward_device(X.data_ptr(), Y.data_ptr(), a.n)
            e1.record()
            torch.cuda.synchronize()
            times[f].append(e0.elapsed_time(e1) / a.iters)
    for f, t in times.items():
        ms = float(np.median(t))
        print(json.dumps({"precision": prec, "form": f, "ms_median": round(ms, 4), "ms_all": [round(x, 4) for x in t],
                          "TFLOPs": round(a.n * 14592 / (ms * 1e-3) / 1e12, 1),
                          "frac_of_peak": round(a.n * 14592 / (ms * 1e-3) / 1e12 / 2516.6, 4)}), flush=True)
r.set_debug(0)
r.set_occupancy(0)
