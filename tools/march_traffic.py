"""Joins tools/march_traffic.sh's three runs: per k_march16 dispatch, HBM bytes (FETCH_SIZE x
1024 x 2 -- gfx950 tallies a wide read's 128-B requests at 64 B, MI355X_MICROARCH.md HBM section
-- plus WRITE_SIZE x 1024) and duration; reports the march's achieved GB/s against 8 TB/s and
bytes per ray-step against the algorithmic figure.

Algorithmic bytes per ray-step of k_march16: the ray is read from the
queue as two float4 ({p, tfar}, {d, tag}: 32 B) and a surviving ray is appended as the same
32 B (a converged one as 16 B to the shade queue); SURVEY.md section 8(d)'s minimal form is 44 B
(read p, d, t; write p, t).  The ray-steps of the profiled program are the ones its last
render_frames.py call printed, per launch of the batch.

    python tools/march_traffic.py OUTDIR BATCH PREC"""
import ast
import csv
import glob
import json
import sys

out, batch, prec = sys.argv[1], int(sys.argv[2]), sys.argv[3]
KN = "k_march16"


def counters(d, name):
    vals = {}
    for f in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if KN in r["Kernel_Name"] and r["Counter_Name"] == name:
                vals[int(r["Dispatch_Id"])] = vals.get(int(r["Dispatch_Id"]), 0.0) + float(r["Counter_Value"])
    return [vals[k] for k in sorted(vals)]


def durations(d):
    ds = []
    for f in glob.glob(f"{d}/**/*kernel_trace.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if KN in r["Kernel_Name"]:
                ds.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]) - int(r["Start_Timestamp"])))
    return [x[1] for x in sorted(ds)]


fetch, write, dur = counters(f"{out}/fetch", "FETCH_SIZE"), counters(f"{out}/write", "WRITE_SIZE"), durations(f"{out}/trace")
st = None
for line in open(f"{out}/trace.log"):
    line = line.strip()
    if line.startswith("{") and "ray_steps" in line:
        st = ast.literal_eval(line)
n = min(len(fetch), len(write), len(dur))
# the program renders 2 launches of the same batch: both halves are the same work; use all
fb = sum(fetch[:n]) * 1024 * 2
wb = sum(write[:n]) * 1024
t = sum(dur[:n]) * 1e-9
launches = 2
steps = st["ray_steps"] * launches if st else None
res = {
    "kernel": "k_march16 (wavefront schedule, one dispatch per march iteration)",
    "workload": f"plane_1 1024x1024, 128 steps, {prec}, {batch} frames per nr_render_batch call, 2 calls",
    "dispatches": [len(fetch), len(write), len(dur)],
    "fetch_bytes": int(fb), "write_bytes": int(wb), "hbm_bytes": int(fb + wb),
    "march_time_ms": round(t * 1e3, 3),
    "achieved_GBps": round((fb + wb) / t / 1e9, 1),
    "peak_GBps": 8000.0,
    "frac_of_hbm_peak": round((fb + wb) / t / 8e12, 4),
    "ray_steps": steps,
    "hbm_bytes_per_ray_step": round((fb + wb) / steps, 2) if steps else None,
    "algorithmic_bytes_per_ray_step": {"this_layout": 64, "survey_minimum": 44},
    "algorithmic_GBps": round(64 * steps / t / 1e9, 1) if steps else None,
    "correction": "bytes = FETCH_SIZE*1024*2 + WRITE_SIZE*1024 (MI355X_MICROARCH.md HBM section)",
    "bound": "MFMA (14,592 FLOP per ray-step against 64 B: 228 FLOP/B, above the f32 ridge of ~20 FLOP/B)",
}
print(json.dumps(res, indent=1))
