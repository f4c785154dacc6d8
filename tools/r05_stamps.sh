#!/bin/bash
# Phase stamps of the device entropy decode (diagnostic build from
#   tools/variants.sh build hstamps "-DMXD_HUFF_STAMPS" jpeghuff hostpath)
# over the C4 and 12 MP batches, summarised by tools/huff_stamps.py.
#   tools/r05_stamps.sh TAG [datasets]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
TAG=${1:-r05s}
cp mlx-data_amd/libmxd_amd.so gpurun_out/.product.so
cp tools/libmxd_amd_var_hstamps.so mlx-data_amd/libmxd_amd.so
rc=0
for ds in ${2:-c4 l12:4}; do
  f=gpurun_out/${TAG}_$(echo $ds | tr : _).bin
  rm -f $f
  MXD_HUFF_STAMPS_FILE=$f timeout -k 10 200 python tools/jpeg_batch_bench.py --datasets $ds --no-host --seconds 0.3 \
    || { rc=1; break; }
  python tools/huff_stamps.py $f | tee gpurun_out/${TAG}_$(echo $ds | tr : _).json
  rm -f $f
done
cp gpurun_out/.product.so mlx-data_amd/libmxd_amd.so
rm -f gpurun_out/.product.so
exit $rc
