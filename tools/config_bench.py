"""Single-GPU timings of the BASELINE configs other than the headline (C3-C5), for
DESIGN.md / BASELINE.md.  Runs on the GPU box; prints one JSON object per config.

  C3  car_1 2048^2, bf16, 256 steps
  C4  plane_2 4096^2, bf16, 128 steps: the full frame on one GPU, and one rank's shard
      of the 8-way row-band split (what each GPU of the 8-GPU job renders)
  C5  each bundled geometry at 2048^2, fp16, 128 steps (one geometry per GPU)
Per config: median frame time over --frames renders (HIP events around the launch on
the context's stream, from nr_stats.ms_total), ray-steps, Mray-steps/s and the
matrix-core fraction of the precision's dense peak."""
import argparse
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import cudaneuralrender_amd as nr  # noqa: E402

PEAK = {"fp32": 157.3, "bf16": 2516.6, "fp16": 2516.6}
FLOP = 14592
ap = argparse.ArgumentParser()
ap.add_argument("--frames", type=int, default=10)
a = ap.parse_args()
matcap = nr.load_png(nr.matcap_path("Chrome"))


def run(name, geom, size, prec, steps, shard=None):
    r = nr.Renderer(0).load_h5(nr.geometry_path(geom)).set_precision(prec)
    r.set_camera(0, 0, 2).set_static(1, 3).set_scene("v1").set_matcap(matcap)
    rows = size if shard is None else nr.shard_rows(size, 8, 8, shard)
    out = torch.zeros(rows * size, dtype=torch.int32, device="cuda")
    ms = []
    for i in range(a.frames + 2):
        if shard is None:
            st = r.render_device(out.data_ptr(), size, size, steps, with_stats=True)
        else:
            st = r.render_shard_device(out.data_ptr(), size, size, 8, 8, shard, steps, with_stats=True)
        if i >= 2:
            ms.append(st["ms_total"])
    t = float(np.median(ms))
    evals = st["ray_steps"] + st["shade_evals"]
    res = {"config": name, "geometry": geom, "size": size, "precision": prec, "max_steps": steps,
           "shard": shard, "ms_per_frame": round(t, 4), "ray_steps": st["ray_steps"],
           "Mray_steps_per_s": round(st["ray_steps"] / t / 1e3, 1),
           "TFLOPs": round(evals * FLOP / t / 1e9, 2),
           "frac_of_peak": round(evals * FLOP / t / 1e9 / PEAK[prec], 4)}
    print(json.dumps(res), flush=True)
    r.close()


run("C3", "car_1", 2048, "bf16", 256)
run("C3-fp32", "car_1", 2048, "fp32", 256)
run("C4-full", "plane_2", 4096, "bf16", 128)
run("C4-shard0of8", "plane_2", 4096, "bf16", 128, shard=0)
for g in ["plane_1", "plane_2", "plane_3", "car_1", "3a3d4a90a2db90b4203936772104a82d.obj"]:
    run("C5", g, 2048, "fp16", 128)
