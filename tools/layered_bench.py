"""Frame time of the layered schedule (any dense network) next to the fused schedules,
on the bench frame (plane_1 1024^2, 128 steps, default camera, Chrome matcap).
Runs on the GPU box: python3 tools/layered_bench.py"""
import os
import sys
import time

import numpy as np
import torch  # device buffers for the MLP timing; initialised before libnr

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import cudaneuralrender_amd as nr  # noqa: E402

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tests"))
from test_gpu_layered import random_net, widen  # noqa: E402


def timed(r, W, H, steps, reps=5):
    r.render(W, H, steps)  # warm (graph capture)
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        img, st = r.render(W, H, steps)
        ts.append(time.perf_counter() - t0)
    return float(np.median(ts)) * 1e3, st


def main():
    import argparse
    ap = argparse.ArgumentParser()
    ap.add_argument("--no-graph", action="store_true", help="layered launches one by one (debug bit 8)")
    args = ap.parse_args()
    W = H = 1024
    steps = 128
    r = nr.Renderer(0)
    if args.no_graph:
        r.set_debug(256)
    dims, K, B = nr.read_keras_h5(nr.geometry_path("plane_1"))
    iv, nm = nr.camera(0, 0, 2)
    r.set_view(iv, nm, 0).set_static(1, 3).set_scene("v1").set_matcap(nr.load_png(nr.matcap_path("Chrome")))
    rows = []
    r.load_mlp(dims, K, B)
    for sched in ("persistent", "wavefront", "layered"):
        r.set_schedule(sched)
        ms, st = timed(r, W, H, steps)
        rows.append((f"plane_1 {sched}", ms, st))
    r.set_schedule("persistent")
    K2, B2 = widen(K, B, 48)
    r.load_mlp([3] + [48] * 8 + [1], K2, B2)
    ms, st = timed(r, W, H, steps)
    rows.append(("plane_1 zero-padded to 48 (layered)", ms, st))
    for d in ([3, 64, 64, 64, 64, 1], [3, 128, 128, 128, 1], [3, 256, 256, 1]):
        Kr, Br = random_net(d, 5)
        r.load_mlp(d, Kr, Br)
        ms, st = timed(r, W, H, steps, reps=3)
        rows.append((f"random {d} (layered)", ms, st))
    # dense chain on 2^20 device-resident points (nr_mlp_forward, NR_DEVICE); the
    # [3, 32 x 8, 1] row is the fused kernel (k_mlp16) for comparison
    n = 1 << 20
    X = torch.rand((n, 3), device="cuda") * 2 - 1
    Y = torch.zeros((n, 1), device="cuda")
    mrows = []
    for d in ([3] + [32] * 8 + [1], [3, 64, 64, 64, 64, 1], [3, 128, 128, 128, 1], [3, 256, 256, 1],
              [3, 512, 512, 512, 1]):
        Kr, Br = random_net(d, 9)
        r.load_mlp(d, Kr, Br)
        flop = 2 * n * sum(a * b for a, b in zip(d[:-1], d[1:]))
        r.mlp_forward_device(X.data_ptr(), Y.data_ptr(), n)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(5):
            r.mlp_forward_device(X.data_ptr(), Y.data_ptr(), n)
        r.synchronize()
        torch.cuda.synchronize()
        ms = (time.perf_counter() - t0) / 5 * 1e3
        mrows.append((d, ms, flop / ms / 1e9))
    for name, ms, st in rows:
        print(f"{name:44s} {ms:9.2f} ms/frame  {st['ray_steps'] / ms / 1e3:9.1f} Mray-steps/s  "
              f"ray_steps {st['ray_steps']}  launches {st['launches']}")
    for d, ms, tf in mrows:
        print(f"mlp_forward 2^20 points {str(d):32s} {ms:9.3f} ms  {tf:8.1f} TFLOP/s")
    r.close()


if __name__ == "__main__":
    main()
