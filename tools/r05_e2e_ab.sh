#!/bin/bash
# Round 5: host-side A/B of the JPEG device-batch pipeline (C4 / C1 slice,
# bench_pipeline.py device variant) between the committed _pipeline build
# (tools/_pipeline_old.so, built here from HEAD) and the working tree's.
#   tools/r05_e2e_ab.sh TAG [skip-tests]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-r05e2e}
MOD=mlx-data_amd/mlx_data_amd/_pipeline.cpython-310-x86_64-linux-gnu.so
run() {  # name limit cmd...
  local name=$1 lim=$2; shift 2
  timeout -k 10 "$lim" "$@" > gpurun_out/${TAG}_${name}.log 2>&1
  local rc=$?
  echo "== $name rc=$rc"; tail -n 6 gpurun_out/${TAG}_${name}.log | cut -c1-600
  if [ $rc -ne 0 ]; then echo "stopping"; exit $rc; fi
}
if [ "${2:-}" != "skip-tests" ]; then
  run tests 600 python -u -m pytest -x -q -p no:cacheprovider --timeout 240 --timeout-method thread \
    tests/test_gpu_jpeg_entropy.py tests/test_gpu_jpeg.py
fi
cp $MOD /tmp/_pipeline_new.so
P="python tools/bench_pipeline.py --datasets ${DATASETS:-c4} --variants device --workers ${WORKERS:-1,16} --min-seconds 3 --images 1024"
run new1 300 $P
cp tools/_pipeline_old.so $MOD
run old1 300 $P
cp /tmp/_pipeline_new.so $MOD
run new2 300 $P
cp tools/_pipeline_old.so $MOD
run old2 300 $P
cp /tmp/_pipeline_new.so $MOD
exit 0
