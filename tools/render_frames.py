"""Profiling driver: renders the benchmark workload for rocprofv3 runs.

    python tools/render_frames.py [--frames 3] [--batch 0] [--precision fp32] [--temporal 0] [--bpc 0] [--endgame T]
--batch B > 0 renders each of the --frames launches as one nr_render_batch of B frames
(the bench's batched kernel) into device buffers.
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import cudaneuralrender_amd as nr  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--frames", type=int, default=3)
ap.add_argument("--batch", type=int, default=0)
ap.add_argument("--precision", default="fp32")
ap.add_argument("--size", type=int, default=1024)
ap.add_argument("--steps", type=int, default=128)
ap.add_argument("--temporal", type=int, default=0)
ap.add_argument("--bpc", type=int, default=0)
ap.add_argument("--schedule", default="persistent")
ap.add_argument("--endgame", type=float, default=-1.0, help="nr_set_endgame threshold (-1: the library's default)")
a = ap.parse_args()
if a.batch > 0:
    # torch's HIP state first, then libnr's (the other order breaks torch kernels under
    # rocprofv3 --pmc)
    import torch
    torch.zeros(1, device="cuda")
r = nr.Renderer(0).load_h5(nr.geometry_path("plane_1")).set_precision(a.precision)
r.set_camera(0, 0, 2).set_static(1, 3).set_scene("v1").set_matcap(nr.load_png(nr.matcap_path("Chrome")))
r.set_occupancy(a.bpc).set_temporal_order(a.temporal).set_schedule(a.schedule)
if a.endgame >= 0:
    r.set_endgame(a.endgame)
if a.batch > 0:
    iv, nm = nr.camera(0, 0, 2)
    bufs = [torch.zeros(a.size * a.size, dtype=torch.int32, device="cuda") for _ in range(a.batch)]
    for i in range(a.frames):
        st = r.render_batch_device([b.data_ptr() for b in bufs], a.size, a.size, [(iv, nm, 0)] * a.batch, a.steps,
                                   with_stats=True)
else:
    for i in range(a.frames):
        img, st = r.render(a.size, a.size, a.steps)
print(st)
