#!/bin/bash
# PMC counters of jpeg_prog on a one-worker c4p run (instruction mix and
# wave cycles per launch): what bounds the serial per-lane decode.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-r05pmc}
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_SMEM SQ_WAVE_CYCLES SQ_WAIT_INST_ANY --output-format csv -d gpurun_out/${TAG} -o run -- python3 tools/bench_pipeline.py --datasets c4p --images 128 --workers 1 --variants device --min-seconds 1 > gpurun_out/${TAG}.log 2>&1
rc=$?
echo "rc=$rc"
python3 - "$TAG" <<'PY'
import csv, glob, sys, collections
tag = sys.argv[1]
f = glob.glob(f"gpurun_out/{tag}/**/*counter_collection.csv", recursive=True)
print(f)
agg = collections.defaultdict(lambda: collections.defaultdict(float)); n = collections.Counter()
for path in f:
    for r in csv.DictReader(open(path)):
        k = r.get("Kernel_Name", "")[:40]
        agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
        n[(k, r["Counter_Name"])] += 1
for k, d in agg.items():
    calls = max(n[(k, c)] for c in d)
    print(k, {c: round(v / max(1, n[(k, c)]), 1) for c, v in d.items()}, "records", calls)
PY
exit $rc
