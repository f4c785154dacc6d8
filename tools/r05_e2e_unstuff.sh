#!/bin/bash
# Round 5: JPEG GPU tests, then the device-batch pipeline with the stuffed
# bytes removed on the device (default) or by the host path
# (MXD_TUNE_HOST_UNSTUFF=1), alternating, with mxd_host_stats; then the
# kernel trace of the batch bench (jpeg_unstuff's time).   tools/r05_e2e_unstuff.sh TAG [skip-tests]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-r05us}
run() {  # name limit cmd...
  local name=$1 lim=$2; shift 2
  timeout -k 10 "$lim" "$@" > gpurun_out/${TAG}_${name}.log 2>&1
  local rc=$?
  echo "== $name rc=$rc"; tail -n 4 gpurun_out/${TAG}_${name}.log | cut -c1-1500
  if [ $rc -ne 0 ]; then echo "stopping"; exit $rc; fi
}
if [ "${2:-}" != "skip-tests" ]; then
  run tests 600 python -u -m pytest -x -q -p no:cacheprovider --timeout 240 --timeout-method thread \
    tests/test_gpu_jpeg_entropy.py tests/test_gpu_jpeg.py tests/test_gpu_c4_full.py
fi
P="python tools/bench_pipeline.py --datasets ${DATASETS:-c4,c1} --variants device --workers ${WORKERS:-1,16} --min-seconds 3 --images 1024 --stats"
for rep in 1 2; do
  run dev$rep 300 $P
  run host$rep 300 $P --tune HOST_UNSTUFF=1
done
(for f in dev1 host1 dev2 host2; do grep '^{' gpurun_out/${TAG}_$f.log | sed "s/^{/{\"build\": \"$f\", /"; done) > gpurun_out/${TAG}.jsonl
run prof 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_prof -o run -- python3 tools/jpeg_batch_bench.py --datasets c4,l12:4 --no-host
cut -c1-200 gpurun_out/${TAG}_prof/run_kernel_stats.csv
exit 0
