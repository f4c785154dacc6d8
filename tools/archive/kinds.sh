#!/bin/bash
# GPU session: parity tests, C2 kernel time per kernel kind (band / scatter /
# ring / gather), scatter ablations, c3/c5, the read/write probe, rocprofv3
# kernel stats of the default bench.   tools/kinds.sh TAG
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
TAG=${1:-k}
timeout -k 10 500 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/${TAG}_pytest.log 2>&1
rc=$?; tail -3 gpurun_out/${TAG}_pytest.log; [ $rc -le 1 ] || exit $rc
for kind in default scatter ring gather; do
  case $kind in
    default) envs="";;
    scatter) envs="MXD_NO_BAND=1";;
    ring) envs="MXD_NO_BAND=1 MXD_NO_SCATTER=1";;
    gather) envs="MXD_NO_BAND=1 MXD_NO_SCATTER=1 MXD_NO_RING=1";;
  esac
  env $envs MXD_DEBUG=1 timeout -k 10 120 python bench.py --steps 30 --warmup 3 --no-cpu --no-e2e --no-copy > gpurun_out/${TAG}_$kind.log 2>&1 || exit $?
  echo "$kind $(grep -o '"kernel_ms_per_launch": [0-9.]*' gpurun_out/${TAG}_$kind.log) $(grep -m1 'mxd: launch' gpurun_out/${TAG}_$kind.log)"
done
NO_WORKLOADS=1 bash tools/abl.sh ${TAG}abl "1 2 9" || exit $?
timeout -k 10 120 ./tools/membench > gpurun_out/${TAG}_mb.log 2>&1 || exit $?
cat gpurun_out/${TAG}_mb.log
export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_prof -o run -- python3 bench.py --steps 20 --warmup 3 --no-cpu --no-e2e --no-copy > gpurun_out/${TAG}_prof.log 2>&1 || exit $?
cut -c1-220 gpurun_out/${TAG}_prof/run_kernel_stats.csv
