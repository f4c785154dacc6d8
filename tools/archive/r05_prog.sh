#!/bin/bash
# Round-5 progressive device decode session: its GPU tests, the other JPEG
# GPU tests, then the C4 pipeline on progressive files (c4p) with the device
# decode of every scan vs the host entropy decode (MXD_NO_DEVICE_PROGRESSIVE=1),
# and a rocprofv3 kernel trace of a short c4p run.
#   tools/r05_prog.sh TAG [tests-only]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
export GPU_MAX_HW_QUEUES=16  # (bench.py's own setting for its e2e_jpeg)
TAG=${1:-r05p}
run() {  # name limit cmd...
  local name=$1 lim=$2; shift 2
  timeout -k 10 "$lim" "$@" > gpurun_out/${TAG}_${name}.log 2>&1
  local rc=$?
  echo "== $name rc=$rc"; tail -n 4 gpurun_out/${TAG}_${name}.log | cut -c1-1500
  if [ $rc -ne 0 ]; then echo "stopping"; exit $rc; fi
}
run pytest_prog 300 python -u -m pytest tests/test_gpu_jpeg_progressive.py -x -v --timeout 120 --timeout-method thread -p no:cacheprovider
run pytest_jpeg 400 python -u -m pytest tests/test_gpu_jpeg.py tests/test_gpu_jpeg_entropy.py tests/test_gpu_c4_full.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider
if [ "${2:-}" = "tests-only" ]; then exit 0; fi
MXD_DEVICE_PROGRESSIVE=1 run pipe_dev 300 python tools/bench_pipeline.py --datasets c4p --images 256 --workers 1,16,32 --variants device --min-seconds 3 --stats
MXD_NO_DEVICE_PROGRESSIVE=1 run pipe_host 300 python tools/bench_pipeline.py --datasets c4p --images 256 --workers 1,16,32 --variants device --min-seconds 3 --stats
MXD_DEVICE_PROGRESSIVE=1 run prof 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_prof -o run -- python3 tools/bench_pipeline.py --datasets c4p --images 256 --workers 16 --variants device --min-seconds 2
cut -c1-250 gpurun_out/${TAG}_prof/run_kernel_stats.csv
exit 0
