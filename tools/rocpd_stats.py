"""Per-kernel dispatch statistics from a rocprofv3 rocpd database (the
default output of `rocprofv3 --kernel-trace` on this image when no
--output-format is given): calls, average / min / max duration in ns by
kernel name (template arguments cut), like the --stats CSV.
  python tools/rocpd_stats.py DIR_OR_DB [--csv OUT]"""
import glob
import os
import sqlite3
import statistics
import sys
from collections import defaultdict


def main():
    path = sys.argv[1]
    if os.path.isdir(path):
        path = sorted(glob.glob(os.path.join(path, "**", "*.db"), recursive=True))[0]
    c = sqlite3.connect(path)
    names = {}
    cols = [r[1] for r in c.execute("pragma table_info(kernel_symbols)")]
    for row in c.execute("select * from kernel_symbols"):
        d = dict(zip(cols, row))
        names[d["id"]] = d.get("display_name") or d.get("kernel_name") or d.get("name")
    durs = defaultdict(list)
    for kid, s, e in c.execute("select kernel_id, start, end from rocpd_kernel_dispatch"):
        durs[names.get(kid, str(kid))].append(e - s)
    out = ["Name,Calls,TotalDurationNs,AverageNs,MinNs,MaxNs"]
    for n, v in sorted(durs.items(), key=lambda kv: -sum(kv[1])):
        short = n.replace("(anonymous namespace)::", "").split("(")[0].replace(",", ";")[:160]
        out.append(f"{short},{len(v)},{sum(v)},{statistics.mean(v):.1f},{min(v)},{max(v)}")
    text = "\n".join(out)
    if "--csv" in sys.argv:
        open(sys.argv[sys.argv.index("--csv") + 1], "w").write(text + "\n")
    print(text)


if __name__ == "__main__":
    main()
