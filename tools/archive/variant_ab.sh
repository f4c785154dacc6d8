#!/bin/bash
# A/B of a compile-time variant of the wave kernel against the product build.
#   tools/variant_ab.sh build NAME "FLAGS"   (here: tools/libmxd_amd_NAME.so)
#   tools/variant_ab.sh run NAME             (GPU box: tools/quick_bench.sh, product vs variant, alternating)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
NAME=$2
if [ "$1" = build ]; then
  cd mlx-data_amd
  /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC -Wall -I../include -Icsrc --offload-arch=gfx950 -ffp-contract=fast \
    $3 -c csrc/wave.hip -o build/wave_$NAME.o || exit 1
  /opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 build/resample.o build/wave_$NAME.o build/pixmap.o \
    build/capi.o build/taps.o build/jpeg.o build/jpegdev.o -o ../tools/libmxd_amd_$NAME.so || exit 1
  exit 0
fi
mkdir -p gpurun_out
cp mlx-data_amd/libmxd_amd.so gpurun_out/.product.so
rc=0
for pass in 1 2; do
  for v in product $NAME; do
    if [ $v = product ]; then cp gpurun_out/.product.so mlx-data_amd/libmxd_amd.so; else cp tools/libmxd_amd_$NAME.so mlx-data_amd/libmxd_amd.so; fi
    tools/quick_bench.sh | sed "s/^/$v /" || { rc=1; break 2; }
  done
done
cp gpurun_out/.product.so mlx-data_amd/libmxd_amd.so
rm -f gpurun_out/.product.so
exit $rc
