"""Single-GPU timings of the BASELINE configs other than the headline (C3-C5), for
DESIGN.md / BASELINE.md.  Runs on the GPU box; prints one JSON object per config.

  C3  car_1 2048^2, bf16, 256 steps
  C4  plane_2 4096^2, bf16, 128 steps: the full frame on one GPU, and one rank's shard
      of the 8-way row-band split (what each GPU of the 8-GPU job renders)
  C5  each bundled geometry at 2048^2, fp16, 128 steps (one geometry per GPU)
Per config, two schedules:
  single  median frame time over --frames renders, one nr_render launch per frame (HIP
          events around the launch on the context's stream, from nr_stats.ms_total);
  batch   --batch frames through one nr_render_batch launch (the bench's schedule: the
          pixel queue runs through the frames, so one frame's longest rays overlap the
          next frame's bulk), per-frame time = launch time / frames.
Ray-steps, Mray-steps/s and the fraction of the precision's dense matrix peak."""
import argparse
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import cudaneuralrender_amd as nr  # noqa: E402

PEAK = {"fp32": 157.3, "bf16": 2516.6, "fp16": 2516.6, "fp32x3": 2516.6}
FLOP = 14592
ap = argparse.ArgumentParser()
ap.add_argument("--frames", type=int, default=10)
ap.add_argument("--batch", type=int, default=8, help="frames per nr_render_batch launch (0: skip)")
ap.add_argument("--only", default="", help="comma-separated config names to run (default all)")
ap.add_argument("--bpc", type=int, default=0, help="nr_set_occupancy (0: the library's default)")
ap.add_argument("--debug", type=int, default=0, help="nr_set_debug flags (A/B of the bf16 ReLU forms: 512)")
ap.add_argument("--endgame", default="", help="comma-separated nr_set_endgame thresholds to run each 16-bit config "
                "with (default: the library's, NR_ENDGAME_DEFAULT; 0 = the pure 16-bit march)")
a = ap.parse_args()
matcap = nr.load_png(nr.matcap_path("Chrome"))


def report(name, geom, size, prec, steps, shard, sched, t, st, nframes=1, tau=None):
    evals = (st["ray_steps"] + st["shade_evals"]) / nframes
    rs = st["ray_steps"] / nframes
    res = {"config": name, "geometry": geom, "size": size, "precision": prec, "max_steps": steps,
           "shard": shard, "schedule": sched, "ms_per_frame": round(t, 4), "ray_steps": int(rs),
           "Mray_steps_per_s": round(rs / t / 1e3, 1),
           "TFLOPs": round(evals * FLOP / t / 1e9, 2),
           "frac_of_peak": round(evals * FLOP / t / 1e9 / PEAK[prec], 4)}
    if prec in ("bf16", "fp16"):
        res["endgame_tau"] = tau
        res["fp32x3_share"] = round(st.get("endgame_evals", 0) / max(st["ray_steps"], 1), 4)
    print(json.dumps(res), flush=True)


def run(name, geom, size, prec, steps, shard=None):
    if a.only and name not in a.only.split(","):
        return
    taus = [float(t) for t in a.endgame.split(",")] if a.endgame and prec in ("bf16", "fp16") else [None]
    for tau in taus:
        run1(name, geom, size, prec, steps, shard, tau)


def run1(name, geom, size, prec, steps, shard, tau):
    r = nr.Renderer(0).load_h5(nr.geometry_path(geom)).set_precision(prec)
    if tau is not None:
        r.set_endgame(tau)
    tau = nr.NR_ENDGAME_DEFAULT if tau is None else tau
    r.set_camera(0, 0, 2).set_static(1, 3).set_scene("v1").set_matcap(matcap)
    r.set_debug(a.debug)
    r.set_occupancy(a.bpc)
    band, nsh = (8, 8) if shard is not None else (8, 1)
    rows = nr.shard_rows(size, band, nsh, shard or 0)
    out = torch.zeros(max(a.batch, 1), rows * size, dtype=torch.int32, device="cuda")
    ms = []
    for i in range(a.frames + 2):
        st = r.render_shard_device(out[0].data_ptr(), size, size, band, nsh, shard or 0, steps, with_stats=True)
        if i >= 2:
            ms.append(st["ms_total"])
    report(name, geom, size, prec, steps, shard, "single", float(np.median(ms)), st, tau=tau)
    if a.batch > 0:
        iv, nm = nr.camera(0.0, 0.0, 2.0)
        cams = [(iv, nm, 0)] * a.batch
        ptrs = [out[i].data_ptr() for i in range(a.batch)]
        ms = []
        for i in range(4):
            st = r.render_batch_device(ptrs, size, size, cams, steps, band, nsh, shard or 0, with_stats=True)
            if i >= 1:
                ms.append(st["ms_total"])
        report(name, geom, size, prec, steps, shard, f"batch{a.batch}", float(np.median(ms)) / a.batch, st, a.batch, tau)
    r.close()


run("C3", "car_1", 2048, "bf16", 256)
run("C3-fp32", "car_1", 2048, "fp32", 256)
# the endgame's fine arithmetic on every evaluation (what a fine pass costs against the bulk form)
run("C3-fp32x3", "car_1", 2048, "fp32x3", 256)
run("C4-full", "plane_2", 4096, "bf16", 128)
run("C4-shard0of8", "plane_2", 4096, "bf16", 128, shard=0)
for g in ["plane_1", "plane_2", "plane_3", "car_1", "3a3d4a90a2db90b4203936772104a82d.obj"]:
    run("C5", g, 2048, "fp16", 128)
