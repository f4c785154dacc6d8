#!/bin/bash
# Round 5: the device-batch JPEG pipeline at 16 workers
# with HIP's 4 hardware queues -- one stream per host-path slot (default)
# against slots sharing n library streams (MXD_TUNE_HOST_STREAMS) -- and
# with 16 queues, alternating, one process per point.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
P="python -u tools/bench_pipeline.py --datasets c1,c4 --workers 16 --variants device --images 2048 --min-seconds 4"
for rep in 1 2; do
  for cfg in "4 0" "4 4" "4 2" "16 0"; do
    set -- $cfg
    T=""; [ "$2" != 0 ] && T="--tune HOST_STREAMS=$2"
    GPU_MAX_HW_QUEUES=$1 timeout -k 10 200 $P $T | sed "s/^{/{\"hw_queues\": $1, \"host_streams\": $2, \"rep\": $rep, /" || exit 1
  done
done
