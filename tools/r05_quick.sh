#!/bin/bash
# Round-5 quick session (one box): GPU tests + smoke, the default bench line,
# the C2 single-stream line, and rocprofv3 kernel stats of both commands (the
# roofline's per-launch events vs the profile's kernel average).
#   tools/r04_quick.sh TAG [skip-tests]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-r05}
run() {  # name limit cmd...
  local name=$1 lim=$2; shift 2
  timeout -k 10 "$lim" "$@" > gpurun_out/${TAG}_${name}.log 2>&1
  local rc=$?
  echo "== $name rc=$rc"; tail -n 2 gpurun_out/${TAG}_${name}.log | cut -c1-2500
  if [ $rc -ne 0 ]; then echo "stopping"; exit $rc; fi
}
if [ "${2:-}" != "skip-tests" ]; then
  run pytest_gpu 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread -p no:cacheprovider
  run smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
fi
run bench 400 python bench.py
run bench_1stream 300 python bench.py --streams 1 --no-cpu --no-e2e
run prof 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_prof -o run -- python3 bench.py --no-cpu --no-e2e
cut -c1-220 gpurun_out/${TAG}_prof/run_kernel_stats.csv
run prof_1stream 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_prof1 -o run -- python3 bench.py --streams 1 --no-cpu --no-e2e
cut -c1-220 gpurun_out/${TAG}_prof1/run_kernel_stats.csv
if [ -x tools/inflight_probe ]; then run inflight 300 tools/inflight_probe; cat gpurun_out/${TAG}_inflight.log; fi
exit 0
