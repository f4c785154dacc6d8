#!/bin/bash
# Round 5, late: entropy-decode knobs in the GPU-busy regime (C4 device batch
# at 16 workers), alternating: default, words from global memory (two jobs per
# CU), 500-subsequence jobs.   tools/r05_e2e_tune.sh TAG
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-r05tune}
P="python tools/bench_pipeline.py --datasets c4 --variants device --workers 16 --min-seconds 3 --images 1024 --stats"
: > gpurun_out/${TAG}.jsonl
for rep in 1 2; do
  for t in "" "--tune HUFF_GLOBAL=1" "--tune HUFF_JOB=500"; do
    timeout -k 10 200 $P $t > gpurun_out/${TAG}_pt.log 2>&1 || { tail -5 gpurun_out/${TAG}_pt.log; exit 1; }
    grep '^{' gpurun_out/${TAG}_pt.log | tee -a gpurun_out/${TAG}.jsonl
  done
done
