#!/bin/bash
# Round 5, late: VERDICT r4 next 7 re-measured after the host-side changes
# (staging helpers sized by the CPU quota, load straight into the parsed
# handle): device-batch JPEG pipeline at 16 workers with 4 vs 16 hardware
# queues, alternating, one process per point; --stats adds the host split.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
P="python -u tools/bench_pipeline.py --datasets c4,c1 --workers 16 --variants device --images 1024 --min-seconds 3 --stats"
for rep in 1 2; do
  for q in 4 16; do
    GPU_MAX_HW_QUEUES=$q timeout -k 10 200 $P | sed "s/^{/{\"hw_queues\": $q, \"rep\": $rep, /" || exit 1
  done
done
