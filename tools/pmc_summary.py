"""Summarise rocprofv3 --pmc CSVs: per-counter average per dispatch of a kernel."""
import csv
import glob
import sys
from collections import defaultdict

tag = sys.argv[1]
kern = sys.argv[2] if len(sys.argv) > 2 else "resample"
vals = defaultdict(list)
for f in sorted(glob.glob(f"gpurun_out/{tag}_p*/run_counter_collection.csv")):
    per = defaultdict(float)
    for row in csv.DictReader(open(f)):
        if kern not in row["Kernel_Name"]:
            continue
        per[(row["Dispatch_Id"], row["Counter_Name"])] += float(row["Counter_Value"])
    for (d, c), v in per.items():
        vals[c].append(v)
for c, v in sorted(vals.items()):
    print(f"{c:28s} n={len(v):3d} avg={sum(v)/len(v):16.1f}")
