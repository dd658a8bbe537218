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
    for debug in (0,):
        r.set_debug(debug)
        for bpc in (3,):
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
            # per XCD (workgroup b runs on XCD b % 8): loop start / end on the 100 MHz clock
            se = Y[4 * waves: 6 * waves].view(waves, 2).cpu().numpy().astype(np.int64)
            base = se[:, 0].min()
            if se[:, 0].max() - base > (1 << 23):  # the low 24 bits wrapped inside the launch
                se = (se - (1 << 23)) % (1 << 24)
                base = se[:, 0].min()
            t0, t1 = (se[:, 0] - base) / 1e2, (se[:, 1] - base) / 1e2  # us
            xcd = (np.arange(waves) // 4) % 8
            by_xcd = {int(x): [round(float(np.median(t1[xcd == x])), 1), round(float(t1[xcd == x].max()), 1),
                               round(float(np.median(st2[xcd[: len(st2)] == x, 0] / np.maximum(st2[xcd[: len(st2)] == x, 2], 1))))]
                      for x in range(8)}
            hw = Y[6 * waves: 8 * waves].view(waves, 2).cpu().numpy().astype(np.int64)
            # HW_ID: wave 3:0, SIMD 5:4, CU 11:8, SH 12, SE 15:13 (gfx9); XCC from XCC_ID
            simd_key = ((hw[:, 1] >> 8) << 16) | (hw[:, 0] & 0xff30) | 0
            cu_key = ((hw[:, 1] >> 8) << 16) | (hw[:, 0] & 0xff00)
            _, inv, cnt = np.unique(simd_key, return_inverse=True, return_counts=True)
            waves_on_simd = cnt[inv]
            chunks = st2[:, 2] if len(st2) == waves else np.zeros(waves)
            by_load = {int(k): {"waves": int((waves_on_simd == k).sum()),
                                "end_us_median": round(float(np.median(t1[waves_on_simd == k])), 1),
                                "chunks_median": float(np.median(chunks[waves_on_simd == k]))}
                       for k in np.unique(waves_on_simd)}
            simds = len(np.unique(simd_key))
            cus = len(np.unique(cu_key))
            if os.environ.get("STAMPS_NPZ"):
                np.savez(os.environ["STAMPS_NPZ"] + f"_{prec}_{debug}_{bpc}.npz", st=st2, se=se, hw=hw)
            slot = (np.arange(waves) % 4)
            by_slot = {int(k): round(float(np.median(t1[slot == k])), 1) for k in range(4)}
            print(json.dumps({"precision": prec, "debug": debug, "bpc": bpc, "waves": int(len(st)),
                              "cycles_per_chunk_median": round(float(np.median(per))),
                              "mlp_cycles_per_chunk_median": round(float(np.median(mlp))),
                              "outside_mlp": round(float(np.median(per - mlp))),
                              "clock_GHz": round(clock, 3), "kernel_ms": round(ms, 4),
                              "loop_ms_max": round(float(st2[:, 3].max()) / 1e5, 4),
                              "loop_ms_median": round(float(np.median(st2[:, 3])) / 1e5, 4),
                              "start_us_max": round(float(t0.max()), 1), "end_us_p10_p50_p90_max":
                              [round(float(np.percentile(t1, q)), 1) for q in (10, 50, 90, 100)],
                              "by_xcd_end_median_max_us_cycles_per_chunk": by_xcd, "by_wave_slot_end_us": by_slot,
                              "cus": cus, "simds": simds, "by_waves_on_simd": by_load}), flush=True)
r.set_debug(0)
