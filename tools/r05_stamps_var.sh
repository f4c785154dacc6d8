#!/bin/bash
# Phase stamps over several diagnostic builds (tools/variants.sh build NAME
# "-DMXD_HUFF_STAMPS ..." jpeghuff hostpath), C4 batch only.
#   tools/r05_stamps_var.sh TAG NAME...
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
TAG=$1; shift
cp mlx-data_amd/libmxd_amd.so gpurun_out/.product.so
rc=0
for v in "$@"; do
  cp tools/libmxd_amd_var_$v.so mlx-data_amd/libmxd_amd.so
  f=gpurun_out/${TAG}_$v.bin
  rm -f $f
  MXD_HUFF_STAMPS_FILE=$f timeout -k 10 200 python tools/jpeg_batch_bench.py --datasets ${DS:-c4} --no-host --seconds 0.3 \
    > /dev/null || { rc=1; break; }
  echo "== $v"; python tools/huff_stamps.py $f | tee gpurun_out/${TAG}_$v.json
  rm -f $f
done
cp gpurun_out/.product.so mlx-data_amd/libmxd_amd.so
rm -f gpurun_out/.product.so
exit $rc
