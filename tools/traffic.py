"""HBM traffic per k_trace launch (and per frame: bench.py scales it by its frames per launch) from tools/profile_round.sh's two --pmc passes.

gfx950 correction (MI355X_MICROARCH.md, HBM/rocprofv3 section): FETCH_SIZE is reported in
KiB and under-counts wide reads by 2x, so bytes = FETCH_SIZE * 1024 * 2; WRITE_SIZE in KiB.
Algorithmic bytes per launch for the fused tracer: the 4 B output pixel per pixel, plus
the staged weights (30 KB) and matcap (1 MiB) read once per workgroup at most."""
import csv
import glob
import json
import sys

out = sys.argv[1]
batch = int(sys.argv[2]) if len(sys.argv) > 2 else 0
# (prefixes of the demangled names: later template arguments follow)
kname = "k_trace<0, false, false, true, false, false" if batch else "k_trace<0, false, false, false, false, false"


def per_dispatch(counter_dir, name):
    vals = []
    for f in glob.glob(f"{counter_dir}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if kname in r["Kernel_Name"] and r["Counter_Name"] == name:
                vals.append(float(r["Counter_Value"]))
    return sum(vals) / len(vals), len(vals)


fetch, nf = per_dispatch(f"{out}/fetch", "FETCH_SIZE")
write, nw = per_dispatch(f"{out}/write", "WRITE_SIZE")
hbm = fetch * 1024 * 2 + write * 1024
print(json.dumps({
    "kernel": kname + " (fp32)",
    "frames_per_launch": batch if batch else 1,
    "workload": "plane_1 1024x1024, 128 march steps, fp32, Chrome.png, v1 scene, default camera",
    "collection": "rocprofv3 --pmc FETCH_SIZE and --pmc WRITE_SIZE, separate passes, tools/render_frames.py "
                  f"--frames 3 --batch {batch}",
    "dispatches": [nf, nw],
    "fetch_size_kb": round(fetch, 2),
    "write_size_kb": round(write, 2),
    "correction": "bytes = FETCH_SIZE*1024*2 (gfx950 under-reports wide reads 2x) + WRITE_SIZE*1024",
    "hbm_bytes_per_launch": int(hbm),
    "hbm_bytes_per_frame": int(hbm / max(batch, 1)),
    "algorithmic_bytes_per_launch": (1024 * 1024 * 4) * max(batch, 1) + 30 * 1024 + 1024 * 1024,
    "note": "output pixels are written 4 B at a time as rays finish (scattered), hence write > 4 MiB",
}, indent=1))
