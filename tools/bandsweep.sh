#!/bin/bash
# Kernel time vs output rows per wave unit (MXD_BAND_ROWS; 0 = the host's
# capacity-based choice).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
TAG=${1:-band}
for b in ${BANDS:-0 21 23 28 32 45 56 75}; do
  MXD_BAND_ROWS=$b timeout -k 10 300 python bench.py --steps 30 --warmup 3 --no-cpu --no-e2e > gpurun_out/${TAG}_b$b.log 2>&1
  rc=$?
  echo "band=$b rc=$rc $(grep -o '"kernel_ms_per_launch": [0-9.]*' gpurun_out/${TAG}_b$b.log)"
  if [ $rc -ne 0 ]; then exit $rc; fi
done
