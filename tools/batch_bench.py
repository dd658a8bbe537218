"""Per-GPU frame time of nr_render_batch on the bench frame (1024^2 plane_1, 128 steps,
fp32, default camera) for 1/2/4/8 row-band shards and several batch sizes -- what one
rank of the N-GPU bench sustains, without the gather.  Runs on the GPU box."""
import argparse
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import cudaneuralrender_amd as nr  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--frames", type=int, default=64)
ap.add_argument("--batches", default="1,4,16,32")
ap.add_argument("--bpc", type=int, default=0)
ap.add_argument("--rays", type=int, default=0, help="nr_set_wave_rays (0: automatic)")
ap.add_argument("--schedule", default="persistent")
ap.add_argument("--shards", default="1,2,4,8")
ap.add_argument("--precision", default="fp32")
ap.add_argument("--size", type=int, default=1024)
ap.add_argument("--steps", type=int, default=128)
ap.add_argument("--spread", type=int, default=-1, help="nr_set_pixel_spread (blocks per group, -1 auto)")
ap.add_argument("--queues", type=int, default=8, help="nr_set_queue_shards")
ap.add_argument("--temporal", type=int, default=0, help="nr_set_temporal_order")
ap.add_argument("--debug", type=int, default=0, help="nr_set_debug flags (1024: frame-major batch queue)")
ap.add_argument("--band", type=int, default=1, help="rows per band dealt round-robin (bench.py BAND)")
ap.add_argument("--probe", default="0,16", help="nr_set_cost_probe max_steps,rays_per_wave (0: off)")
ap.add_argument("--single", action="store_true",
                help="time one-frame launches through nr_render_shard (the one-frame k_trace instance) "
                     "instead of nr_render_batch")
a = ap.parse_args()
matcap = nr.load_png(nr.matcap_path("Chrome"))
iv, nm = nr.camera(0, 0, 2)
r = nr.Renderer(0).load_h5(nr.geometry_path("plane_1")).set_precision(a.precision)
r.set_view(iv, nm, 0).set_static(1, 3).set_scene("v1").set_matcap(matcap)
r.set_occupancy(a.bpc).set_wave_rays(a.rays).set_schedule(a.schedule)
r.set_pixel_spread(a.spread).set_queue_shards(a.queues).set_temporal_order(a.temporal)
r.set_debug(a.debug)
r.set_cost_probe(*(int(v) for v in a.probe.split(",")))
S = a.size
bufs = [torch.zeros(S * S, dtype=torch.int32, device="cuda") for _ in range(32)]
for n in (int(x) for x in a.shards.split(",")):
    line = []
    for b in (int(x) for x in a.batches.split(",")):
        cams = [(iv, nm, 0)] * b
        ptrs = [t.data_ptr() for t in bufs[:b]]
        def launch():
            if a.single and b == 1:
                r.render_shard_device(ptrs[0], S, S, a.band, n, 0, a.steps)
            else:
                r.render_batch_device(ptrs, S, S, cams, a.steps, a.band, n, 0)
        for _ in range(2):
            launch()
        r.synchronize()
        t0 = time.perf_counter()
        for _ in range(max(1, a.frames // b)):
            launch()
        r.synchronize()
        dt = (time.perf_counter() - t0) / (max(1, a.frames // b) * b) * 1e3
        line.append(f"{'single' if a.single and b == 1 else 'batch'} {b}: {dt:.3f} ms/frame")
    print(f"n={n} {a.precision} {S}^2 {a.schedule} bpc {a.bpc} rays {a.rays} spread {a.spread} queues {a.queues} temporal {a.temporal} probe {a.probe} debug {a.debug} band {a.band}: " + "  ".join(line), flush=True)
