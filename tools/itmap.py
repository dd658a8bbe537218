"""Diagnostic: per-pixel iteration counts of the bench workload (debug bit 3), saved to
gpurun_out/itmap_<size>.npy for offline schedule analysis.  Runs on the GPU box."""
import argparse
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import cudaneuralrender_amd as nr  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--size", type=int, default=1024)
ap.add_argument("--steps", type=int, default=128)
ap.add_argument("--geometry", default="plane_1")
a = ap.parse_args()
r = nr.Renderer(0).load_h5(nr.geometry_path(a.geometry))
r.set_camera(0, 0, 2).set_static(1, 3).set_scene("v1").set_matcap(nr.load_png(nr.matcap_path("Chrome")))
r.set_debug(8)
img, st = r.render(a.size, a.size, a.steps)
os.makedirs("gpurun_out", exist_ok=True)
np.save(f"gpurun_out/itmap_{a.geometry}_{a.size}.npy", img.astype(np.uint16))
h = np.bincount(img.reshape(-1), minlength=a.steps + 2)
print("stats", st)
print("pixels with >0 iterations:", int((img > 0).sum()), " sum:", int(img.sum()))
for lo, hi in [(1, 8), (8, 16), (16, 32), (32, 64), (64, 96), (96, 128), (128, 200)]:
    print(f"iters [{lo},{hi}): {int(h[lo:hi].sum())}")
