"""Scheduling sweep of the persistent tracer on the bench workload.  Runs on the GPU box.

    python tools/sched_sweep.py --grid "bpc,age,prio,temporal[,spread[,probe_steps[,probe_take]]]];..."
For each schedule: frame time (median and min over --frames renders, HIP events around
the k_trace launch) and a bit-exactness check against the first schedule's image --
scheduling changes only the order work is handed out, never a pixel."""
import argparse
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import cudaneuralrender_amd as nr  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--precision", default="fp32")
ap.add_argument("--size", type=int, default=1024)
ap.add_argument("--steps", type=int, default=128)
ap.add_argument("--frames", type=int, default=30)
ap.add_argument("--grid", default="2,0,0,0;3,0,0,0;2,32,2,0;3,32,2,0;3,16,2,0;3,48,2,0")
a = ap.parse_args()

matcap = nr.load_png(nr.matcap_path("Chrome"))
ref = None
out = torch.zeros(a.size * a.size, dtype=torch.int32, device="cuda")
for spec in a.grid.split(";"):
    v = [int(x) for x in spec.split(",")] + [16, 0, 16][len(spec.split(",")) - 4:]
    bpc, age, prio, temporal, spread, pst, ptake = v[:7]
    r = nr.Renderer(0).load_h5(nr.geometry_path("plane_1")).set_precision(a.precision)
    r.set_camera(0, 0, 2).set_static(1, 3).set_scene("v1").set_matcap(matcap)
    r.set_occupancy(bpc).set_temporal_order(temporal).set_pixel_spread(spread)
    r.set_cost_probe(pst, ptake)
    for _ in range(3):
        r.render_device(out.data_ptr(), a.size, a.size, a.steps)
    ms = []
    for _ in range(a.frames):
        st = r.render_device(out.data_ptr(), a.size, a.size, a.steps, with_stats=True)
        ms.append(st["ms_total"])
    img = out.cpu().numpy()
    if ref is None:
        ref = img
    same = bool(np.array_equal(img, ref))
    ms = np.array(ms)
    print(f"bpc {bpc} hold {age:3d}/{prio} temporal {temporal} spread {spread:3d} probe {pst:3d}/{ptake:2d}: "
          f"median {np.median(ms):.3f} ms  min {ms.min():.3f} ms  "
          f"Mray-steps/s {(st['ray_steps'] + st['shade_evals']) / np.median(ms) / 1e3:.0f}  identical {same}",
          flush=True)
    del r
