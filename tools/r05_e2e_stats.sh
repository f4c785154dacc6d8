#!/bin/bash
# Round 5: host-side time split of the JPEG device-batch pipeline
# (mxd_host_stats per image: batch-call wall, its device wait, marker parse)
# at 1 / 8 / 12 / 16 workers.   tools/r05_e2e_stats.sh TAG
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-r05stats}
timeout -k 10 400 python tools/bench_pipeline.py --datasets ${DATASETS:-c4,c1} --variants device \
  --workers ${WORKERS:-1,8,12,16} --min-seconds 3 --images 1024 --stats > gpurun_out/${TAG}.log 2>&1
rc=$?
grep '^{' gpurun_out/${TAG}.log > gpurun_out/${TAG}.jsonl
cat gpurun_out/${TAG}.jsonl
exit $rc
