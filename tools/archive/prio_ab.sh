#!/bin/bash
# A/B of the progress-based wave priority (wave.hip MXD_PRIO).
#   tools/prio_ab.sh build   (here: tools/libmxd_amd_noprio.so, -DMXD_PRIO=0)
#   tools/prio_ab.sh run     (GPU box: product vs no-priority build, tools/quick_bench.sh, alternating)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
if [ "$1" = build ]; then
  cd mlx-data_amd
  /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC -Wall -I../include -Icsrc --offload-arch=gfx950 -ffp-contract=fast \
    -DMXD_PRIO=0 -c csrc/wave.hip -o build/wave_noprio.o || exit 1
  /opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 build/resample.o build/wave_noprio.o build/pixmap.o \
    build/capi.o build/taps.o build/jpeg.o build/jpegdev.o -o ../tools/libmxd_amd_noprio.so || exit 1
  exit 0
fi
mkdir -p gpurun_out
cp mlx-data_amd/libmxd_amd.so gpurun_out/.product.so
rc=0
for pass in 1 2; do
  for v in prio noprio; do
    if [ $v = noprio ]; then cp tools/libmxd_amd_noprio.so mlx-data_amd/libmxd_amd.so; else cp gpurun_out/.product.so mlx-data_amd/libmxd_amd.so; fi
    tools/quick_bench.sh | sed "s/^/$v /" || { rc=1; break 2; }
  done
done
cp gpurun_out/.product.so mlx-data_amd/libmxd_amd.so
rm -f gpurun_out/.product.so
exit $rc
