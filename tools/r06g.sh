#!/bin/bash
# Round 6 session g: the Huffman sync rounds' early exit (trails) -- JPEG GPU
# tests, then the product against the build without trails (-DMXD_HUFF_TRAILS=0,
# tools/variants.sh build notrail ... jpeghuff): batch-call wall time and
# rocprof kernel stats on the C4 files and the 12 MP no-restart photos.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${1:-r06g}
O=gpurun_out/r06/$TAG
mkdir -p gpurun_out/r06
timeout -k 10 400 python -u -m pytest tests/test_gpu_jpeg_entropy.py tests/test_gpu_jpeg.py tests/test_gpu_c4_full.py tests/test_gpu_jpeg_progressive.py -x -q --timeout 120 --timeout-method thread > ${O}_pytest_jpeg.txt 2>&1 || exit 1
cp mlx-data_amd/libmxd_amd.so gpurun_out/.product.so
rc=0
for rep in 1 2; do
for v in product notrail; do
  if [ $v = product ]; then cp gpurun_out/.product.so mlx-data_amd/libmxd_amd.so; else cp tools/libmxd_amd_var_$v.so mlx-data_amd/libmxd_amd.so; fi
  timeout -k 10 120 python3 tools/jpeg_batch_bench.py --datasets c4,l12:4 --no-host --seconds 2 >> ${O}_${v}_jpeg_batch.jsonl 2>&1 || { rc=1; break 2; }
  if [ $rep = 1 ]; then
    timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d ${O}_${v}_trace -o run -- python3 tools/jpeg_batch_bench.py --datasets c4,l12:4 --no-host --seconds 0.5 > ${O}_${v}_trace.log 2>&1 || { rc=1; break 2; }
  fi
done
done
cp gpurun_out/.product.so mlx-data_amd/libmxd_amd.so
rm -f gpurun_out/.product.so
exit $rc
