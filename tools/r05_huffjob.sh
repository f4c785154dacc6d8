#!/bin/bash
# Round 5: device entropy decode job size A/B (MXD_TUNE_HUFF_JOB), one process,
# C4 / C1 / 12 MP; then rocprofv3 kernel traces of the same.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-r05m}
timeout -k 10 400 python tools/jpeg_batch_bench.py --datasets c4,c1,l12:4 --no-host --huff-job 0,500,333,250 \
  > gpurun_out/${TAG}_jobs.jsonl 2> gpurun_out/${TAG}_jobs.err || exit 1
cat gpurun_out/${TAG}_jobs.jsonl
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_prof -o run -- \
  python3 tools/jpeg_batch_bench.py --datasets c4,l12:1 --no-host --huff-job 0,333 > gpurun_out/${TAG}_prof.log 2>&1 || exit 1
exit 0
