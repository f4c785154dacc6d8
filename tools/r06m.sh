#!/bin/bash
# Huffman trails A/B: SQ instruction counters per jpeg_huff dispatch, product
# vs the build without trails (one --pmc pass each, kernel-trace only).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${1:-r06m}
O=gpurun_out/r06/$TAG
mkdir -p gpurun_out/r06
cp mlx-data_amd/libmxd_amd.so gpurun_out/.product.so
rc=0
for v in product notrail; do
  if [ $v = product ]; then cp gpurun_out/.product.so mlx-data_amd/libmxd_amd.so; else cp tools/libmxd_amd_var_$v.so mlx-data_amd/libmxd_amd.so; fi
  d=${O}_${v}_sq
  timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_BRANCH --output-format csv -d $d -o run -- python3 tools/jpeg_batch_bench.py --datasets c4 --no-host --seconds 0.3 > $d.log 2>&1 || { rc=1; break; }
  python3 tools/pmc_kernels.py $d > $d.txt
done
cp gpurun_out/.product.so mlx-data_amd/libmxd_amd.so
rm -f gpurun_out/.product.so
exit $rc
