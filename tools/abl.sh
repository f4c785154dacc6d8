#!/bin/bash
# Ablation sweep of the C2 bench kernel, then the c3/c5 workloads:
#   tools/abl.sh TAG "modes"      (MXD_* env passes through to bench.py)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
TAG=${1:-abl}
for m in ${2:-0 1 2 5 6 7 8}; do
  MXD_WAVE_ABLATE=$m timeout -k 10 120 python bench.py --steps 30 --warmup 3 --no-cpu --no-e2e --no-copy > gpurun_out/${TAG}_m$m.log 2>&1
  rc=$?
  echo "mode=$m rc=$rc $(grep -o '"kernel_ms_per_launch": [0-9.]*' gpurun_out/${TAG}_m$m.log)"
  if [ $rc -ne 0 ]; then tail -5 gpurun_out/${TAG}_m$m.log; exit $rc; fi
done
if [ -z "${NO_WORKLOADS:-}" ]; then
  for w in c3 c5; do
    timeout -k 10 120 python bench.py --workload $w --steps 20 --warmup 3 --no-cpu --no-copy > gpurun_out/${TAG}_$w.log 2>&1 || exit $?
    echo "$w $(grep -o '"value": [0-9.]*' gpurun_out/${TAG}_$w.log | head -1) $(grep -o '"kernel_ms_per_launch": [0-9.]*' gpurun_out/${TAG}_$w.log) $(grep -o '"frac": [0-9.]*' gpurun_out/${TAG}_$w.log)"
  done
fi
