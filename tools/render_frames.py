"""Profiling driver: renders N frames of the benchmark workload (for rocprofv3 runs).

    python tools/render_frames.py [--frames 3] [--precision fp32] [--temporal 0] [--bpc 0]
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import cudaneuralrender_amd as nr  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--frames", type=int, default=3)
ap.add_argument("--precision", default="fp32")
ap.add_argument("--size", type=int, default=1024)
ap.add_argument("--steps", type=int, default=128)
ap.add_argument("--temporal", type=int, default=0)
ap.add_argument("--bpc", type=int, default=0)
ap.add_argument("--schedule", default="persistent")
a = ap.parse_args()
r = nr.Renderer(0).load_h5(nr.geometry_path("plane_1")).set_precision(a.precision)
r.set_camera(0, 0, 2).set_static(1, 3).set_scene("v1").set_matcap(nr.load_png(nr.matcap_path("Chrome")))
r.set_occupancy(a.bpc).set_temporal_order(a.temporal).set_schedule(a.schedule)
for i in range(a.frames):
    img, st = r.render(a.size, a.size, a.steps)
print(st)
