#!/bin/bash
# Round-4 JPEG session: the device entropy decode against the host entropy
# decode -- C ABI batch calls (tools/jpeg_batch_bench.py), their rocprofv3
# kernel stats, and the operator-surface pipeline (tools/bench_pipeline.py,
# every point >= 5 s) with the Huffman decode on the device (default) and on
# the host (*_hostent), beside the CPU restatement.
#   tools/r04_jpeg.sh TAG [skip-pipeline]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-r04j}
run() {  # name limit cmd...
  local name=$1 lim=$2; shift 2
  timeout -k 10 "$lim" "$@" > gpurun_out/${TAG}_${name}.log 2>&1
  local rc=$?
  echo "== $name rc=$rc"; tail -n 4 gpurun_out/${TAG}_${name}.log | cut -c1-1500
  if [ $rc -ne 0 ]; then echo "stopping"; exit $rc; fi
}
run batch 300 python tools/jpeg_batch_bench.py
run prof 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_prof -o run -- python3 tools/jpeg_batch_bench.py --datasets c4
cut -c1-200 gpurun_out/${TAG}_prof/run_kernel_stats.csv
if [ "${2:-}" != "skip-pipeline" ]; then
  run pipeline 1000 python -u tools/bench_pipeline.py --images 4096 --variants device,device_hostent,fused,ref_form,cpu
  cat gpurun_out/${TAG}_pipeline.log
fi
exit 0
