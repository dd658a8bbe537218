"""Per-GPU frame time of one rank's row-band shard of the bench frame (1024^2 plane_1,
128 steps, fp32) for 1/2/4/8 shards, under schedule knobs.  Runs on the GPU box.

    python tools/shard_sweep.py --grid "bpc,age,prio,spread[,rays[,queues]]];..."
"""
import argparse
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import cudaneuralrender_amd as nr  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--size", type=int, default=1024)
ap.add_argument("--frames", type=int, default=20)
ap.add_argument("--grid", default="0,0,0,16")
a = ap.parse_args()
matcap = nr.load_png(nr.matcap_path("Chrome"))
out = torch.zeros(a.size * a.size, dtype=torch.int32, device="cuda")
for spec in a.grid.split(";"):
    v = [int(x) for x in spec.split(",")] + [64, 8][len(spec.split(",")) - 4:]
    bpc, age, prio, spread, rays, nq = v[:6]
    r = nr.Renderer(0).load_h5(nr.geometry_path("plane_1"))
    r.set_camera(0, 0, 2).set_static(1, 3).set_scene("v1").set_matcap(matcap)
    r.set_occupancy(bpc).set_pixel_spread(spread).set_wave_rays(rays).set_queue_shards(nq)
    line = []
    for n in (1, 2, 4, 8):
        ms = []
        for i in range(a.frames + 2):
            st = r.render_shard_device(out.data_ptr(), a.size, a.size, 8, n, 0, 128, with_stats=True)
            if i >= 2:
                ms.append(st["ms_total"])
        line.append(f"n={n}: {np.median(ms):.3f} ms")
    print(f"bpc {bpc} hold {age}/{prio} spread {spread} rays {rays} queues {nq}: " + "  ".join(line), flush=True)
    r.close()
