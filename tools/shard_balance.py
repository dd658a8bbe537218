"""Per-rank time of every shard of the bench batch (1024^2 plane_1, 128 steps, fp32,
32 frames per launch) for several band heights: the N-GPU bench waits for the slowest
rank, so max over shards is what scales.  Runs on the GPU box (one GPU renders each
shard in turn).

    python tools/shard_balance.py [--shards 8] [--bands 1,2,4,8] [--schedule persistent]
"""
import argparse
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import cudaneuralrender_amd as nr  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--shards", default="8")
ap.add_argument("--bands", default="1,2,4,8")
ap.add_argument("--schedule", default="persistent")
ap.add_argument("--batch", type=int, default=32)
ap.add_argument("--reps", type=int, default=3)
a = ap.parse_args()
iv, nm = nr.camera(0, 0, 2)
r = nr.Renderer(0).load_h5(nr.geometry_path("plane_1"))
r.set_view(iv, nm, 0).set_static(1, 3).set_scene("v1").set_matcap(nr.load_png(nr.matcap_path("Chrome")))
r.set_schedule(a.schedule)
bufs = [torch.zeros(1024 * 1024, dtype=torch.int32, device="cuda") for _ in range(a.batch)]
ptrs = [t.data_ptr() for t in bufs]
cams = [(iv, nm, 0)] * a.batch
for n in (int(x) for x in a.shards.split(",")):
    for band in (int(x) for x in a.bands.split(",")):
        per = []
        for s in range(n):
            r.render_batch_device(ptrs, 1024, 1024, cams, 128, band, n, s)
            r.synchronize()
            t0 = time.perf_counter()
            for _ in range(a.reps):
                r.render_batch_device(ptrs, 1024, 1024, cams, 128, band, n, s)
            r.synchronize()
            per.append((time.perf_counter() - t0) / (a.reps * a.batch) * 1e3)
        print(f"{a.schedule} shards {n} band {band}: max {max(per):.3f} mean {sum(per) / n:.3f} ms/frame  "
              + " ".join(f"{x:.3f}" for x in per), flush=True)
