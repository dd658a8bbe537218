"""Diagnostic (GPU box): where a 16-bit k_mlp16 wave's time goes, from the per-wave s_memtime
stamps of a build with -DNR_MLP16_STAMPS=1 (NR_LIBRARY=build/stamps/libnr.so): cycles per
128-point chunk in the whole loop and in the MLP call, by workgroups per CU."""
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import cudaneuralrender_amd as nr  # noqa: E402

n = 1 << 24
X = torch.from_numpy(np.random.default_rng(0).uniform(-1, 1, size=(n, 3)).astype(np.float32)).cuda()
Y = torch.zeros(n, dtype=torch.float32, device="cuda")
r = nr.Renderer(0).load_h5(nr.geometry_path("plane_1"))
r.set_stream(torch.cuda.current_stream().cuda_stream)
for prec in sys.argv[1].split(",") if len(sys.argv) > 1 else ("bf16", "fp16"):
    r.set_precision(prec)
    for debug in (0, 2048):
        r.set_debug(debug)
        for bpc in (0, 3, 12):
            r.set_occupancy(bpc)
            for _ in range(3):
                Y.zero_()
                r.mlp_forward_device(X.data_ptr(), Y.data_ptr(), n)
            torch.cuda.synchronize()
            waves = min(256 * (bpc or 3), n // 512) * 4  # bpc 0: the persistent grid (3 per CU)
            st = Y[: 4 * waves].view(waves, 4).cpu().numpy().astype(np.float64)
            st = st[st[:, 2] > 0]
            per = st[:, 0] / st[:, 2]
            mlp = st[:, 1] / st[:, 2]
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            r.mlp_forward_device(X.data_ptr(), Y.data_ptr(), n)
            e1.record()
            torch.cuda.synchronize()
            ms = e0.elapsed_time(e1)
            st2 = Y[: 4 * waves].view(waves, 4).cpu().numpy().astype(np.float64)
            st2 = st2[st2[:, 2] > 0]
            clock = float(np.median(st2[:, 0] / (st2[:, 3] / 100e6))) / 1e9
            print(json.dumps({"precision": prec, "debug": debug, "bpc": bpc, "waves": int(len(st)),
                              "cycles_per_chunk_median": round(float(np.median(per))),
                              "mlp_cycles_per_chunk_median": round(float(np.median(mlp))),
                              "outside_mlp": round(float(np.median(per - mlp))),
                              "clock_GHz": round(clock, 3), "kernel_ms": round(ms, 4),
                              "loop_ms_max": round(float(st2[:, 3].max()) / 1e5, 4),
                              "loop_ms_median": round(float(np.median(st2[:, 3])) / 1e5, 4)}), flush=True)
r.set_debug(0)
