"""Per-dispatch WRITE_SIZE of tools/write_calib.py under rocprofv3 (argument: the -d directory)."""
import csv
import glob
import sys

rows = []
for f in glob.glob(f"{sys.argv[1]}/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if r["Counter_Name"] == "WRITE_SIZE":
            rows.append((int(r["Dispatch_Id"]), r["Kernel_Name"][:90], float(r["Counter_Value"])))
for d, k, v in sorted(rows):
    print(f"{d:5d} {v * 1024 / 2**20:10.2f} MiB  {k}")
