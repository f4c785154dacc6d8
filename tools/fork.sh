#!/bin/bash
# c3 / c2 / c5 kernel time with and without the fork over helper streams.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
TAG=${1:-fk}
for w in c3 c5 c2; do
  for f in 0 1; do
    MXD_NO_FORK=$f timeout -k 10 120 python bench.py --workload $w --steps 30 --warmup 3 --no-cpu --no-e2e --no-copy > gpurun_out/${TAG}_${w}_nofork$f.log 2>&1 || exit $?
    echo "$w nofork=$f $(grep -o '"value": [0-9.]*' gpurun_out/${TAG}_${w}_nofork$f.log | head -1) $(grep -o '"kernel_ms_per_launch": [0-9.]*' gpurun_out/${TAG}_${w}_nofork$f.log) $(grep -o '"frac": [0-9.]*' gpurun_out/${TAG}_${w}_nofork$f.log)"
  done
done
