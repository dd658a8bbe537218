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
        for bpc in (1, 2, 3, 12):
            r.set_occupancy(bpc)
            for _ in range(3):
                Y.zero_()
                r.mlp_forward_device(X.data_ptr(), Y.data_ptr(), n)
            torch.cuda.synchronize()
            waves = min(256 * bpc, n // 512) * 4
            st = Y[: 4 * waves].view(waves, 4).cpu().numpy().astype(np.float64)
            st = st[st[:, 2] > 0]
            per = st[:, 0] / st[:, 2]
            mlp = st[:, 1] / st[:, 2]
            print(json.dumps({"precision": prec, "debug": debug, "bpc": bpc, "waves": int(len(st)),
                              "cycles_per_chunk_median": round(float(np.median(per))),
                              "mlp_cycles_per_chunk_median": round(float(np.median(mlp))),
                              "outside_mlp": round(float(np.median(per - mlp)))}), flush=True)
r.set_debug(0)
