#!/bin/bash
# One GPU-box session: parity tests, smoke, bench, rocprofv3 kernel stats.
# Each GPU step has its own time limit; a crash / abort / timeout ends the
# script (test failures, exit 1, do not).  Output goes to gpurun_out/.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
TAG=${1:-r01}
STEPS=${STEPS:-50}
step() {  # name, limit, command...
  local name=$1 lim=$2; shift 2
  echo "=== $name ($(date +%T))"
  timeout -k 10 "$lim" "$@" > "gpurun_out/${TAG}_${name}.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"; tail -n 30 "gpurun_out/${TAG}_${name}.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after rc=$rc"; exit $rc; fi
  return 0
}
rocminfo 2>/dev/null | grep -m1 -E "gfx9" > gpurun_out/${TAG}_agent.txt || true
step pytest_gpu 900 python -m pytest tests -x -q -m gpu
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
step bench 600 python bench.py --steps "$STEPS" --warmup 5
export TMPDIR=/tmp
step rocprof 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_prof -o run -- python3 bench.py --steps 20 --warmup 3 --no-cpu --no-e2e
exit 0
