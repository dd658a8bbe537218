"""Diagnostic: where does k_trace spend its time (bulk vs tail)?  Runs on the GPU box.

    python tools/tail_stamps.py [--precision fp32]
Prints the kernel span, when the pixel queue drained, and the distribution of wave end
times after that (from s_memrealtime stamps, 100 MHz)."""
import argparse
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import cudaneuralrender_amd as nr  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--precision", default="fp32")
ap.add_argument("--size", type=int, default=1024)
ap.add_argument("--steps", type=int, default=128)
ap.add_argument("--bpc", type=int, default=0)
ap.add_argument("--temporal", type=int, default=0)
ap.add_argument("--spread", type=int, default=0)
ap.add_argument("--hold", type=int, default=0)
a = ap.parse_args()
r = nr.Renderer(0).load_h5(nr.geometry_path("plane_1")).set_precision(a.precision)
r.set_camera(0, 0, 2).set_static(1, 3).set_scene("v1").set_matcap(nr.load_png(nr.matcap_path("Chrome")))
r.set_occupancy(a.bpc)
r.set_temporal_order(a.temporal)
r.set_pixel_spread(a.spread).set_age_hold(a.hold, 2)
for _ in range(3):
    r.render(a.size, a.size, a.steps)
r.set_debug(1)
img, st = r.render(a.size, a.size, a.steps)
s = r.debug_stamps().astype(np.int64)
s = s[s[:, 2] > 0]
t0 = s[:, 0].min()
start, empty, end, steps = (s[:, 0] - t0) / 100.0, s[:, 1], (s[:, 2] - t0) / 100.0, s[:, 3]
empty = np.where(empty > 0, (empty - t0) / 100.0, np.nan)
print(f"== bpc {a.bpc} temporal {a.temporal} spread {a.spread} hold {a.hold} precision {a.precision}: stats {st}")
print(f"waves {len(s)}  start spread {start.max():.1f} us  kernel span {end.max():.1f} us")
print(f"queue drained: first {np.nanmin(empty):.1f} us  median {np.nanmedian(empty):.1f} us  last {np.nanmax(empty):.1f} us")
q = np.percentile(end, [10, 50, 90, 99, 100])
print("wave end times us p10/50/90/99/100:", np.round(q, 1))
d = np.nanmax(empty)
print(f"tail after last drain: {end.max() - d:.1f} us ({(end.max() - d) / end.max() * 100:.1f}% of span);"
      f" steps after drain-ish: waves ending > drain+50us: {(end > d + 50).sum()}")
hist = np.histogram(end, bins=np.arange(0, end.max() + 100, 100))[0]
print("waves ending per 100us bin:", hist.tolist())
