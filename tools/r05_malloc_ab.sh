#!/bin/bash
# Round 5, late: does the allocator's trimming cost the load path page faults?
# C4 device batch at 1 and 16 workers, default glibc malloc vs no trimming /
# no mmap for large blocks, alternating.   tools/r05_malloc_ab.sh TAG
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-r05malloc}
NOTRIM="glibc.malloc.trim_threshold=1073741824:glibc.malloc.mmap_threshold=1073741824:glibc.malloc.top_pad=268435456"
P="python tools/bench_pipeline.py --datasets c4 --variants device --workers 1,16 --min-seconds 3 --images 1024 --stats"
: > gpurun_out/${TAG}.jsonl
for rep in 1 2 3; do
  for cfg in base notrim; do
    if [ $cfg = notrim ]; then E="GLIBC_TUNABLES=$NOTRIM"; else E="X=1"; fi
    env $E timeout -k 10 300 $P > gpurun_out/${TAG}_pt.log 2>&1 || { tail -5 gpurun_out/${TAG}_pt.log; exit 1; }
    grep '^{' gpurun_out/${TAG}_pt.log | sed "s/^{/{\"malloc\": \"$cfg\", /" | tee -a gpurun_out/${TAG}.jsonl
  done
done
