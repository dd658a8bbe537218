"""Summarize tools/pmc_mfma.sh: per nr:: kernel, the MFMA-pipe busy fraction over all 1024
SIMDs, the effective shader clock and the instruction mix per dispatch."""
import collections
import csv
import glob
import sys

out = sys.argv[1]
for run in ("trace", "mlp"):
    ctr = collections.defaultdict(lambda: collections.defaultdict(float))
    dur = collections.defaultdict(list)
    for f in glob.glob(f"{out}/{run}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"].split("(")[0]
            if "nr::" not in k:
                continue
            ctr[(k, r.get("Dispatch_Id", r.get("Correlation_Id", "0")))][r["Counter_Name"]] += float(r["Counter_Value"])
    for f in glob.glob(f"{out}/{run}/**/*kernel_trace.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"].split("(")[0]
            if "nr::" in k:
                dur[k].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9)
    per = collections.defaultdict(list)
    for (k, _), v in ctr.items():
        per[k].append(v)
    for k, vs in per.items():
        if not vs or "GRBM_GUI_ACTIVE" not in vs[0]:
            continue
        v = {c: sum(x[c] for x in vs) / len(vs) for c in vs[0]}
        cyc = v["GRBM_GUI_ACTIVE"] / 8
        d = sorted(dur.get(k, [0.0]))[len(dur.get(k, [0.0])) // 2]
        print(f"{run}: {k[-60:]}  dispatches {len(vs)}  median {d * 1e3:.3f} ms")
        print(f"  MFMA busy {v['SQ_VALU_MFMA_BUSY_CYCLES'] / (1024 * cyc):.3f} of 1024 SIMDs x {cyc:.4g} cycles;"
              f"  clock {cyc / d / 1e9 if d else 0:.3f} GHz")
        print(f"  insts per dispatch: VALU {v['SQ_INSTS_VALU']:.4g}  MFMA {v['SQ_INSTS_MFMA']:.4g}"
              f"  VALU/MFMA {v['SQ_INSTS_VALU'] / max(v['SQ_INSTS_MFMA'], 1):.2f}")
        print(f"  SQ_BUSY {v['SQ_BUSY_CYCLES']:.4g}  WAVE {v['SQ_WAVE_CYCLES']:.4g}  ACTIVE_VALU {v['SQ_ACTIVE_INST_VALU']:.4g}"
              f"  WAIT_INST_ANY {v['SQ_WAIT_INST_ANY']:.4g}")
