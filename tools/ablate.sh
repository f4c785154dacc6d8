#!/bin/bash
# Kernel ablations (MXD_WAVE_ABLATE, see wave.hip): full / no-V-math / no-loads / no-H.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
TAG=${1:-abl}
for m in ${MODES:-0 1 2 3 4 0}; do
  MXD_WAVE_ABLATE=$m timeout -k 10 300 python bench.py --steps 30 --warmup 3 --no-cpu --no-e2e > gpurun_out/${TAG}_m$m.log 2>&1
  rc=$?
  echo "mode=$m rc=$rc $(grep -o '"kernel_ms_per_launch": [0-9.]*\|"copy_ceiling_gbs": [0-9.]*' gpurun_out/${TAG}_m$m.log | tr '\n' ' ')"
  if [ $rc -ne 0 ]; then exit $rc; fi
done
