"""Mean value per dispatch of each counter, by kernel (name up to its template
arguments) and grid size, from a rocprofv3 --pmc counter_collection.csv.
  python tools/pmc_kernels.py FILE"""
import csv
import glob
import os
import sys
from collections import defaultdict


def main():
    path = sys.argv[1]
    if os.path.isdir(path):  # rocprofv3 -d DIR: the counter file may sit in a host / pid subdirectory
        path = sorted(glob.glob(os.path.join(path, "**", "*counter_collection.csv"), recursive=True))[0]
    rows = list(csv.DictReader(open(path)))
    per = defaultdict(float)  # (dispatch, kernel, grid, counter) -> summed over the row's instances
    for r in rows:
        short = r["Kernel_Name"].split("(")[0][:90]
        key = (r.get("Dispatch_Id", ""), short, r.get("Grid_Size", r.get("Grid_Size_X", "")), r["Counter_Name"])
        per[key] += float(r["Counter_Value"])
    acc = defaultdict(lambda: [0.0, 0])
    for (_, short, g, c), v in per.items():
        a = acc[(short, g, c)]
        a[0] += v
        a[1] += 1
    for (k, g, c), (v, n) in sorted(acc.items()):
        print(f"{c:12s} grid {g:>8s} dispatches {n:6d} mean {v / n:14.1f}  {k}")


if __name__ == "__main__":
    main()
