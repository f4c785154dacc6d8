#!/bin/bash
# Compile-time variants of the band kernel against the product build, in one
# process per variant on one box (tools/band_sweep.py per variant).
#   tools/band_variants.sh build NAME "FLAGS"      (here: tools/libmxd_amd_band_NAME.so)
#   tools/band_variants.sh run "SWEEP ARGS" NAME... (GPU box; "product" = the in-tree build)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
if [ "$1" = build ]; then
  NAME=$2
  cd mlx-data_amd
  /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC -Wall -I../include -Icsrc --offload-arch=gfx950 -ffp-contract=fast \
    $3 -c csrc/band.hip -o build/band_$NAME.o || exit 1
  /opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 build/resample.o build/wave.o build/band_$NAME.o \
    build/band_plan.o build/pixmap.o build/capi.o build/plan.o build/batch.o build/hostpath.o build/taps.o build/jpeg.o build/jpegdev.o \
    -o ../tools/libmxd_amd_band_$NAME.so || exit 1
  exit 0
fi
ARGS=$2; shift 2
mkdir -p gpurun_out
cp mlx-data_amd/libmxd_amd.so gpurun_out/.product.so
rc=0
for v in "$@"; do
  if [ $v = product ]; then cp gpurun_out/.product.so mlx-data_amd/libmxd_amd.so; else cp tools/libmxd_amd_band_$v.so mlx-data_amd/libmxd_amd.so; fi
  timeout -k 10 200 python tools/band_sweep.py $ARGS | sed "s/^/{\"variant\": \"$v\", \"r\": /; s/$/}/" || { rc=1; break; }
done
cp gpurun_out/.product.so mlx-data_amd/libmxd_amd.so
rm -f gpurun_out/.product.so
exit $rc
