#!/bin/bash
# Round 5: the multi-job device entropy decode -- JPEG GPU tests, the C ABI
# batch bench (C4 / C1 / a 12 MP no-restart photo), rocprofv3 kernel stats.
#   tools/r05_huff.sh TAG [skip-tests]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-r05h}
run() {  # name limit cmd...
  local name=$1 lim=$2; shift 2
  timeout -k 10 "$lim" "$@" > gpurun_out/${TAG}_${name}.log 2>&1
  local rc=$?
  echo "== $name rc=$rc"; tail -n 4 gpurun_out/${TAG}_${name}.log | cut -c1-3000
  if [ $rc -ne 0 ]; then echo "stopping"; exit $rc; fi
}
if [ "${2:-}" != "skip-tests" ]; then
  run tests 600 python -u -m pytest -x -q -p no:cacheprovider --timeout 240 --timeout-method thread \
    tests/test_gpu_jpeg_entropy.py tests/test_gpu_jpeg.py tests/test_gpu_c4_full.py
fi
run batch 400 python tools/jpeg_batch_bench.py --datasets c4,c1,l12:4
run prof 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_prof -o run -- python3 tools/jpeg_batch_bench.py --datasets c4,l12:4 --no-host
cut -c1-200 gpurun_out/${TAG}_prof/run_kernel_stats.csv
exit 0
