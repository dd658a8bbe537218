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
ap.add_argument("--nshards", type=int, default=1)
ap.add_argument("--rays", type=int, default=0)
ap.add_argument("--queues", type=int, default=8)
ap.add_argument("--out", default="", help="save the per-wave stamps (npz)")
a = ap.parse_args()
r = nr.Renderer(0).load_h5(nr.geometry_path("plane_1")).set_precision(a.precision)
r.set_camera(0, 0, 2).set_static(1, 3).set_scene("v1").set_matcap(nr.load_png(nr.matcap_path("Chrome")))
r.set_occupancy(a.bpc)
r.set_temporal_order(a.temporal)
r.set_pixel_spread(a.spread).set_wave_rays(a.rays).set_queue_shards(a.queues)
for _ in range(3):
    r.render_shard(a.size, a.size, 8, a.nshards, 0, a.steps)
r.set_debug(1)
img, st = r.render_shard(a.size, a.size, 8, a.nshards, 0, a.steps)
s = r.debug_stamps().astype(np.int64)
s = s[s[:, 2] > 0]
t0 = s[:, 0].min()
nl_drain = s[:, 1] >> 56
s[:, 1] &= (1 << 56) - 1
start, empty, end = (s[:, 0] - t0) / 100.0, s[:, 1], (s[:, 2] - t0) / 100.0
wit, wit_tail = s[:, 3] & 0xffffffff, s[:, 3] >> 32
empty = np.where(empty > 0, (empty - t0) / 100.0, np.nan)
print(f"== bpc {a.bpc} temporal {a.temporal} spread {a.spread} rays {a.rays} queues {a.queues} "
      f"nshards {a.nshards} precision {a.precision}: stats {st}")
print(f"waves {len(s)}  start spread {start.max():.1f} us  kernel span {end.max():.1f} us")
print(f"queue drained: first {np.nanmin(empty):.1f} us  median {np.nanmedian(empty):.1f} us  last {np.nanmax(empty):.1f} us")
q = np.percentile(end, [10, 50, 90, 99, 100])
print("wave end times us p10/50/90/99/100:", np.round(q, 1))
d = np.nanmax(empty)
print(f"tail after last drain: {end.max() - d:.1f} us ({(end.max() - d) / end.max() * 100:.1f}% of span);"
      f" steps after drain-ish: waves ending > drain+50us: {(end > d + 50).sum()}")
hist = np.histogram(end, bins=np.arange(0, end.max() + 100, 100))[0]
print("waves ending per 100us bin:", hist.tolist())
last = np.argsort(end)[-8:]
for i in last:
    tail_us = end[i] - empty[i] if not np.isnan(empty[i]) else float("nan")
    print(f"  wave ending {end[i]:.1f} us: iterations {wit[i]} ({wit_tail[i]} after drain at {empty[i]:.1f} us), "
          f"{(end[i] - start[i]) / max(wit[i], 1):.2f} us/iter overall, {tail_us / max(wit_tail[i], 1):.2f} us/iter after drain")
ph = s[:, 4:9].astype(np.float64)
tot = ph.sum(axis=1)
print("phase share of wave cycles (refill, shading, MLP, scene, step), all waves:",
      np.round(ph.sum(axis=0) / tot.sum(), 3).tolist())
sub = s[:, 9:12].astype(np.float64).sum(axis=0)
print("within refill (reduced-precision tracers): reservation, bulk generation, dealing from the ring:",
      np.round(sub / tot.sum(), 3).tolist())
for i in last[-3:]:
    print(f"  wave ending {end[i]:.1f} us: cycles/iter refill {ph[i,0]/max(wit[i],1):.0f} shading {ph[i,1]/max(wit[i],1):.0f} "
          f"mlp {ph[i,2]/max(wit[i],1):.0f} scene {ph[i,3]/max(wit[i],1):.0f} step {ph[i,4]/max(wit[i],1):.0f}")
tl = s[:, 12:15].astype(np.float64)
tail_steps = s[:, 15] >> 32
s[:, 15] &= 0xffffffff
wt = np.maximum(wit_tail, 1)
print("after the drain, all waves: cycles per tail iteration refill+shading+step / MLP / scene:",
      np.round(tl.sum(axis=0) / wt.sum(), 0).tolist(), f" iterations with <= 4 rays: {int(s[:, 15].sum())} of {int(wit_tail.sum())}")
for i in last[-3:]:
    print(f"  wave ending {end[i]:.1f} us: tail cycles/iter other {tl[i,0]/wt[i]:.0f} mlp {tl[i,1]/wt[i]:.0f} scene {tl[i,2]/wt[i]:.0f}; "
          f"iterations with <= 4 rays {int(s[i, 15])} of {int(wit_tail[i])}")
print(f"live rays at the drain: total {int(nl_drain.sum())}, per wave p10/50/90/max",
      np.percentile(nl_drain, [10, 50, 90, 100]).tolist(), f"; ray-steps after the drain {int(tail_steps.sum())}")
if a.out:
    np.savez_compressed(a.out, start=start, empty=empty, end=end, wit=wit, wit_tail=wit_tail, nl_drain=nl_drain,
                        tail_steps=tail_steps, phases=ph, tail_phases=tl)
