"""Diagnostic: latency of one fp32 MLP evaluation for a lone wave (1-4 tiles of 16
points), in shader cycles (debug bit 6 of libnr).  Runs on the GPU box."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import cudaneuralrender_amd as nr  # noqa: E402

r = nr.Renderer(0).load_h5(nr.geometry_path("plane_1"))
X = torch.from_numpy(np.random.default_rng(0).uniform(-1, 1, (64, 3)).astype(np.float32)).cuda()
Y = torch.zeros(65, dtype=torch.float32, device="cuda")
# (the no-final-layer variant is meaningful for 1-2 tiles only: with more, the tiles whose
# outputs it drops are dead code)
# part bits: 1 no final layer, 2 the clamped-ReLU form (the tracers'), 4 hidden layers unrolled for 7
# (part 6: the hidden layers as the generated stream, nr_mlp16.h f32_hidden7_stream -- 1 or 2 tiles)
outs = {}
for part, name in [(0, "full"), (1, "no final layer"), (2, "clamped"), (6, "clamped, stream"),
                   (3, "clamped, no final")]:
    r.set_debug(64 | ((part & 1) << 7) | ((part >> 1) << 13))
    for nt in ((1, 2) if part == 6 else (1, 2, 3, 4)):
        r.set_wave_rays(16 * nt)
        for _ in range(2):
            r.mlp_forward_device(X.data_ptr(), Y.data_ptr(), 2000)
        torch.cuda.synchronize()
        cyc = float(Y[0].item())
        outs[(part, nt)] = Y[1:1 + 16 * nt].cpu().numpy().copy()
        same = ""
        if part == 6:
            same = "  outputs == clamped loop's: " + str(bool(np.array_equal(outs[(2, nt)].view(np.uint32),
                                                                              outs[(6, nt)].view(np.uint32))))
        print(f"{name:18s} tiles {nt}: {cyc:.0f} cycles per MLP ({cyc / nt:.0f} per tile; "
              f"MFMA issue floor {114 * 32 * nt}){same}", flush=True)

# the 16-bit MLP on 128 points (k_mlp16's form): the whole evaluation with the pipelined stream,
# with the builtin form (debug bit 11), and the stream alone
for prec in ("bf16", "fp16"):
    r.set_precision(prec)
    X2 = torch.from_numpy(np.random.default_rng(0).uniform(-1, 1, (130, 3)).astype(np.float32)).cuda()
    for flags, name in [(64, "whole, stream"), (64 | 2048, "whole, builtin"), (64 | 128, "stream alone")]:
        r.set_debug(flags)
        for _ in range(2):
            r.mlp_forward_device(X2.data_ptr(), Y.data_ptr(), 2000)
        torch.cuda.synchronize()
        cyc = float(Y[0].item())
        print(f"{prec} 128 points {name:16s}: {cyc:.0f} cycles (60 MFMA issue floor {60 * 32})", flush=True)
    # the tracer's form: 64 points, one per lane, on one or two 32-point tiles (wave_rays 16 / 32)
    for nt in (2, 1):
        r.set_wave_rays(16 * nt)
        for flags, name in [(64, "stream"), (64 | 2048, "builtin")]:
            r.set_debug(flags)
            for _ in range(2):
                r.mlp_forward_device(X2.data_ptr(), Y.data_ptr(), 2000)
            torch.cuda.synchronize()
            cyc = float(Y[0].item())
            print(f"{prec} tracer form, {nt} tile(s) {name:8s}: {cyc:.0f} cycles (MFMA issue floor {30 * nt * 32 // 2})",
                  flush=True)
    r.set_wave_rays(0)
r.set_debug(0)
