#!/bin/bash
# Segment stamps of the band kernel (diagnostic build, -DMXD_BAND_STAMPS=1).
#   tools/band_stamps.sh build          (here: tools/libmxd_amd_bstamps.so)
#   tools/band_stamps.sh run [w[:knobs] ...]  (GPU box: swaps the build in, tools/band_stamps.py, restores)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
if [ "$1" = build ]; then
  cd mlx-data_amd
  /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC -Wall -I../include -Icsrc --offload-arch=gfx950 -ffp-contract=fast \
    -DMXD_BAND_STAMPS=1 ${STAMP_FLAGS:-} -c csrc/band.hip -o build/band_stamps.o || exit 1
  /opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 build/resample.o build/wave.o build/band_stamps.o \
    build/band_plan.o build/pixmap.o build/capi.o build/plan.o build/batch.o build/hostpath.o build/taps.o build/jpeg.o build/jpegdev.o \
    -o ../tools/libmxd_amd_bstamps.so || exit 1
  exit 0
fi
shift
mkdir -p gpurun_out
cp mlx-data_amd/libmxd_amd.so gpurun_out/.product.so
cp tools/libmxd_amd_bstamps.so mlx-data_amd/libmxd_amd.so
rc=0
for spec in ${@:-c2}; do
  w=${spec%%:*}; k=""; [ "$spec" != "$w" ] && k=${spec#*:}
  timeout -k 10 120 python tools/band_stamps.py $w 5 "$k" || { rc=$?; break; }
done
cp gpurun_out/.product.so mlx-data_amd/libmxd_amd.so
rm -f gpurun_out/.product.so
exit $rc
