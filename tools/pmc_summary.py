"""Summarize tools/pmc.sh output: per-kernel average of each counter over dispatches."""
import collections
import csv
import glob
import sys

out = sys.argv[1]
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for f in sorted(glob.glob(f"{out}/p*/run_counter_collection.csv")):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].split("(")[0][-40:]
        agg[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, v in agg.items():
    if "nr::" not in k:
        continue
    print(k)
    for c, vals in sorted(v.items()):
        print(f"  {c:32s} {sum(vals) / len(vals):16.4g}")
