"""The reference's --spin sequence (main.cpp:470-477: frame i at viewRotation.y = i deg,
frameNumber i), one nr_render_shard launch per frame, timed for each nr_set_temporal_order mode
(0 plain, 1 previous frame's block order, 2 that order dilated over 3x3 blocks), without the
per-frame statistics read-back bench.py's config.spin includes.
Runs on the GPU box:  python tools/spin_bench.py [--frames 60] [--modes 0,1,2]"""
import argparse
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import cudaneuralrender_amd as nr  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--frames", type=int, default=60)
ap.add_argument("--modes", default="0,1,2")
ap.add_argument("--size", type=int, default=1024)
ap.add_argument("--precision", default="fp32")
a = ap.parse_args()
S = a.size
r = nr.Renderer(0).load_h5(nr.geometry_path("plane_1")).set_precision(a.precision)
r.set_static(1, 3).set_scene("v1").set_matcap(nr.load_png(nr.matcap_path("Chrome")))
buf = torch.zeros(S * S, dtype=torch.int32, device="cuda")
for mode in (int(m) for m in a.modes.split(",")):
    r.set_temporal_order(mode)
    for rep in range(2):  # the first pass warms up
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for i in range(a.frames):
            iv, nm = nr.camera(0.0, float(i % 360), 2.0)
            r.set_view(iv, nm, i)
            r.render_shard_device(buf.data_ptr(), S, S, 1, 1, 0, 128)
        r.synchronize()
        dt = (time.perf_counter() - t0) / a.frames * 1e3
    print(f"{a.precision} {S}^2 spin, temporal order mode {mode}: {dt:.3f} ms/frame", flush=True)
r.set_temporal_order(0)
