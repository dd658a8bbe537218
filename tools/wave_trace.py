"""One batch of 32 bench frames on the wavefront schedule (for rocprofv3 --kernel-trace):
python3 tools/wave_trace.py [--batch 32] [--bpc 0]"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402,F401  (HIP initialised by torch first)

import cudaneuralrender_amd as nr  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--batch", type=int, default=32)
ap.add_argument("--bpc", type=int, default=0)
ap.add_argument("--reps", type=int, default=2)
a = ap.parse_args()
iv, nm = nr.camera(0, 0, 2)
r = nr.Renderer(0).load_h5(nr.geometry_path("plane_1"))
r.set_view(iv, nm, 0).set_static(1, 3).set_scene("v1").set_matcap(nr.load_png(nr.matcap_path("Chrome")))
r.set_schedule("wavefront").set_occupancy(a.bpc)
bufs = [torch.zeros(1024 * 1024, dtype=torch.int32, device="cuda") for _ in range(a.batch)]
for _ in range(a.reps):
    r.render_batch_device([t.data_ptr() for t in bufs], 1024, 1024, [(iv, nm, 0)] * a.batch, 128, 8, 1, 0)
r.synchronize()
print("done")
