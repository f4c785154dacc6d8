"""HBM traffic per launch of the bench kernel from rocprofv3 --pmc passes.

Usage: python tools/pmc_traffic.py TAG OUT.json [kernel-substring]

Reads gpurun_out/TAG_p*/run_counter_collection.csv (tools/r03_measure.sh) and
applies the gfx950 corrections of MI355X_MICROARCH.md (HBM section):
FETCH_SIZE and WRITE_SIZE are in KiB; FETCH_SIZE counts half the bytes of a
streaming read, so it is doubled; WRITE_SIZE is exact for 16-B-per-lane
stores.  The result feeds bench.py's roofline.traffic.
"""
import csv
import glob
import json
import sys
from collections import defaultdict

tag, out = sys.argv[1], sys.argv[2]
kern = sys.argv[3] if len(sys.argv) > 3 else "resample_wave"
# Per kernel (name) the average over its dispatches, then the sum over the
# kernels: a batch of mixed sizes runs one launch per kernel shape, so a
# "launch" of the bench (one batch) is one dispatch of each kernel.
vals = defaultdict(lambda: defaultdict(list))
names = set()
for f in sorted(glob.glob(f"gpurun_out/{tag}_p*/run_counter_collection.csv")):
    per = defaultdict(float)
    for row in csv.DictReader(open(f)):
        if kern not in row["Kernel_Name"]:
            continue
        names.add(row["Kernel_Name"])
        per[(row["Kernel_Name"], row["Dispatch_Id"], row["Counter_Name"])] += float(row["Counter_Value"])
    for (k, d, c), v in per.items():
        vals[c][k].append(v)
avg = {c: sum(sum(v) / len(v) for v in ks.values()) for c, ks in vals.items()}
res = {
    "tag": tag,
    "kernels": sorted(names),
    "dispatches": {c: sum(len(v) for v in ks.values()) for c, ks in vals.items()},
    "counters_per_launch": avg,
}
if "FETCH_SIZE" in avg and "WRITE_SIZE" in avg:
    rd = avg["FETCH_SIZE"] * 1024 * 2
    wr = avg["WRITE_SIZE"] * 1024
    res.update({"hbm_read_bytes_per_launch": rd, "hbm_write_bytes_per_launch": wr,
                "hbm_bytes_per_launch": rd + wr,
                "correction": "read = FETCH_SIZE[KiB]*1024*2 (gfx950 half-count), write = WRITE_SIZE[KiB]*1024"})
json.dump(res, open(out, "w"), indent=1, sort_keys=True)
print(json.dumps({k: v for k, v in res.items() if k != "counters_avg_per_dispatch"}, indent=1))
for c in sorted(avg):
    print(f"{c:30s} {avg[c]:18.1f}")
