"""Occupancy / batching sweep of the reduced-precision tracer on C3 (car_1 2048^2, bf16,
256 steps) and C5 (plane_1 2048^2, fp16, 128 steps).  Runs on the GPU box.

For each blocks-per-CU setting: single-frame time (nr_render_device, HIP events around
the launch) and the per-frame time of a --batch-frame nr_render_batch launch, with a
bit-exactness check of every batch frame against the single frame."""
import argparse
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import cudaneuralrender_amd as nr  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--bpc", default="2,3")
ap.add_argument("--batch", type=int, default=8)
ap.add_argument("--frames", type=int, default=8)
a = ap.parse_args()
matcap = nr.load_png(nr.matcap_path("Chrome"))
iv, nm = nr.camera(0, 0, 2)
for name, geom, size, prec, steps in [("C3", "car_1", 2048, "bf16", 256), ("C5", "plane_1", 2048, "fp16", 128)]:
    r = nr.Renderer(0).load_h5(nr.geometry_path(geom)).set_precision(prec)
    r.set_view(iv, nm, 0).set_static(1, 3).set_scene("v1").set_matcap(matcap)
    one = torch.zeros(size * size, dtype=torch.int32, device="cuda")
    bufs = [torch.zeros(size * size, dtype=torch.int32, device="cuda") for _ in range(a.batch)]
    for bpc in (int(x) for x in a.bpc.split(",")):
        r.set_occupancy(bpc)
        ms = []
        for i in range(a.frames + 2):
            st = r.render_device(one.data_ptr(), size, size, steps, with_stats=True)
            if i >= 2:
                ms.append(st["ms_total"])
        ptrs = [t.data_ptr() for t in bufs]
        cams = [(iv, nm, 0)] * a.batch
        r.render_batch_device(ptrs, size, size, cams, steps, 8, 1, 0)
        r.synchronize()
        t0 = time.perf_counter()
        reps = 3
        for _ in range(reps):
            r.render_batch_device(ptrs, size, size, cams, steps, 8, 1, 0)
        r.synchronize()
        bt = (time.perf_counter() - t0) / (reps * a.batch) * 1e3
        same = all(torch.equal(b, one) for b in bufs)
        evals = st["ray_steps"] + st["shade_evals"]
        print(f"{name} {geom} {size}^2 {prec} {steps} steps bpc {bpc}: single {np.median(ms):.3f} ms "
              f"({st['ray_steps'] / np.median(ms) / 1e3:.0f} Mray-steps/s), batch {a.batch}: {bt:.3f} ms/frame "
              f"({st['ray_steps'] / bt / 1e3:.0f} Mray-steps/s, {evals * 14592 / bt / 1e9:.0f} TF/s)  identical {same}",
              flush=True)
    r.close()
