#!/bin/bash
# Device entropy decode variants, one box: per library (the product, then the
# variant builds named on the command line) the entropy GPU tests, the
# rocprofv3 kernel stats of tools/jpeg_batch_bench.py (C4 and C1 batches of
# 128), and -- for the *stats builds -- tools/huff_stats.py (rounds, symbols,
# phase durations).  The product library is restored at the end.
#   tools/r04_huff_ab.sh TAG "VARIANTS" "STATS_VARIANTS"
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-r04h}
cp mlx-data_amd/libmxd_amd.so gpurun_out/.product.so
restore() { cp gpurun_out/.product.so mlx-data_amd/libmxd_amd.so; rm -f gpurun_out/.product.so; }
for v in product ${2:-}; do
  if [ $v != product ]; then cp tools/libmxd_amd_var_$v.so mlx-data_amd/libmxd_amd.so; fi
  timeout -k 10 300 python -u -m pytest tests/test_gpu_jpeg_entropy.py -x -q --timeout 120 --timeout-method thread > gpurun_out/${TAG}_${v}_tests.log 2>&1
  rc=$?; echo "== $v tests rc=$rc $(tail -1 gpurun_out/${TAG}_${v}_tests.log)"
  if [ $rc -ne 0 ]; then restore; exit $rc; fi
  timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_${v}_prof -o run -- python3 tools/jpeg_batch_bench.py --datasets c4,c1 > gpurun_out/${TAG}_${v}_prof.log 2>&1
  rc=$?; echo "== $v prof rc=$rc"
  if [ $rc -ne 0 ]; then restore; exit $rc; fi
  python3 -c "
import csv
for r in csv.DictReader(open('gpurun_out/${TAG}_${v}_prof/run_kernel_stats.csv')): print(r['Name'][:40], r['Calls'], r['AverageNs'])
"
  grep '^{' gpurun_out/${TAG}_${v}_prof.log | cut -c1-400
done
for v in ${3:-}; do
  cp tools/libmxd_amd_var_$v.so mlx-data_amd/libmxd_amd.so
  timeout -k 10 300 python tools/huff_stats.py > gpurun_out/${TAG}_${v}_stats.jsonl 2>&1
  rc=$?; echo "== $v stats rc=$rc"; cat gpurun_out/${TAG}_${v}_stats.jsonl
  if [ $rc -ne 0 ]; then restore; exit $rc; fi
done
restore
exit 0
