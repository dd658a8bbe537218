"""Summarize tools/pmc_lowp.sh: per nr:: kernel of each program (mlp, trace), the counters of
both passes averaged per dispatch, and the derived figures:
  MFMA busy   = SQ_VALU_MFMA_BUSY_CYCLES / (1024 SIMDs x GRBM_GUI_ACTIVE / 8)
  clock       = GRBM_GUI_ACTIVE / 8 / median dispatch duration
  LDS share   = SQ_LDS_IDX_ACTIVE / (256 CUs x GRBM_GUI_ACTIVE / 8)   (LDS-array busy)
  conflicts   = SQ_LDS_BANK_CONFLICT / SQ_LDS_IDX_ACTIVE
(SQ_WAVE_CYCLES / SQ_WAIT_* / SQ_ACTIVE_INST_* count quad-cycles, MI355X_MICROARCH.md.)"""
import collections
import csv
import glob
import sys


def load(d):
    ctr = collections.defaultdict(lambda: collections.defaultdict(float))
    dur = collections.defaultdict(list)
    for f in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"].split("(")[0]
            if "nr::" in k:
                ctr[(k, r.get("Dispatch_Id", r.get("Correlation_Id", "0")))][r["Counter_Name"]] += float(r["Counter_Value"])
    for f in glob.glob(f"{d}/**/*kernel_trace.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"].split("(")[0]
            if "nr::" in k:
                dur[k].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9)
    per = collections.defaultdict(list)
    for (k, _), v in ctr.items():
        per[k].append(v)
    out = {}
    for k, vs in per.items():
        names = set().union(*[set(v) for v in vs])
        out[k] = ({c: sum(v.get(c, 0.0) for v in vs) / len(vs) for c in names}, len(vs),
                  sorted(dur.get(k, [0.0]))[len(dur.get(k, [0.0])) // 2])
    return out


def main(root):
    for prog in ("mlp", "trace"):
        merged = collections.defaultdict(dict)
        meta = {}
        for p in ("A", "B"):
            for k, (v, n, d) in load(f"{root}/{prog}_{p}").items():
                merged[k].update({c: x for c, x in v.items() if c != "GRBM_GUI_ACTIVE"})
                merged[k][f"GRBM_GUI_ACTIVE_{p}"] = v.get("GRBM_GUI_ACTIVE", 0.0)
                meta[k] = (n, d)
        for k, v in merged.items():
            n, d = meta[k]
            print(f"{prog}: {k[-70:]}  dispatches {n}  median {d * 1e3:.3f} ms")
            cyc = v.get("GRBM_GUI_ACTIVE_A", 0.0) / 8
            if cyc and "SQ_VALU_MFMA_BUSY_CYCLES" in v:
                print(f"  MFMA busy {v['SQ_VALU_MFMA_BUSY_CYCLES'] / (1024 * cyc):.3f}  clock {cyc / d / 1e9 if d else 0:.3f} GHz"
                      f"  VALU/MFMA {v['SQ_INSTS_VALU'] / max(v['SQ_INSTS_MFMA'], 1):.2f}"
                      f"  WAIT_INST_ANY/WAVE {v['SQ_WAIT_INST_ANY'] / max(v['SQ_WAVE_CYCLES'], 1):.3f}"
                      f"  ACTIVE_VALU/WAVE {v['SQ_ACTIVE_INST_VALU'] / max(v['SQ_WAVE_CYCLES'], 1):.3f}")
            cb = v.get("GRBM_GUI_ACTIVE_B", 0.0) / 8
            if cb and "SQ_LDS_IDX_ACTIVE" in v:
                print(f"  LDS busy {v['SQ_LDS_IDX_ACTIVE'] / (256 * cb):.3f}  conflicts/LDS cycles "
                      f"{v['SQ_LDS_BANK_CONFLICT'] / max(v['SQ_LDS_IDX_ACTIVE'], 1):.3f}"
                      f"  LDS insts/MFMA {v['SQ_INSTS_LDS'] / max(v.get('SQ_INSTS_MFMA', 1), 1):.2f}"
                      f"  SALU/MFMA {v['SQ_INSTS_SALU'] / max(v.get('SQ_INSTS_MFMA', 1), 1):.2f}"
                      f"  WAIT_ANY/ACTIVE_ANY {v['SQ_WAIT_ANY'] / max(v['SQ_ACTIVE_INST_ANY'], 1):.2f}"
                      f"  WAIT_INST_LDS {v['SQ_WAIT_INST_LDS']:.4g}")
            print("  " + "  ".join(f"{c} {x:.4g}" for c, x in sorted(v.items())))


if __name__ == "__main__":
    main(sys.argv[1])
