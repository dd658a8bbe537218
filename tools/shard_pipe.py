"""Per-GPU throughput of one rank's shard (1024^2 plane_1, 128 steps, fp32) with 1-4
frames in flight on separate streams: what each GPU of the N-GPU bench sustains,
without the gather.  Runs on the GPU box."""
import argparse
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import cudaneuralrender_amd as nr  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--frames", type=int, default=40)
ap.add_argument("--rays", type=int, default=64)
ap.add_argument("--bpc", type=int, default=0)
a = ap.parse_args()
matcap = nr.load_png(nr.matcap_path("Chrome"))
for n in (1, 2, 4, 8):
    line = []
    for inflight in (1, 2, 3, 4):
        slots = []
        for _ in range(inflight):
            s = torch.cuda.Stream()
            r = nr.Renderer(0).load_h5(nr.geometry_path("plane_1"))
            r.set_camera(0, 0, 2).set_static(1, 3).set_scene("v1").set_matcap(matcap)
            r.set_wave_rays(a.rays).set_occupancy(a.bpc)
            r.set_stream(s.cuda_stream)
            buf = torch.zeros(1024 * 1024, dtype=torch.int32, device="cuda")
            slots.append((s, r, buf))
        for i in range(4):
            s, r, buf = slots[i % inflight]
            r.render_shard_device(buf.data_ptr(), 1024, 1024, 8, n, 0, 128)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for i in range(a.frames):
            s, r, buf = slots[i % inflight]
            r.render_shard_device(buf.data_ptr(), 1024, 1024, 8, n, 0, 128)
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t0) / a.frames * 1e3
        line.append(f"inflight {inflight}: {dt:.3f} ms")
        for s, r, buf in slots:
            r.close()
    print(f"n={n} rays {a.rays} bpc {a.bpc}: " + "  ".join(line), flush=True)
