#!/bin/bash
# Unit start/end stamps of the wave kernel (diagnostic build, -DMXD_STAMPS=1).
#   tools/stamps.sh build        (here: tools/libmxd_amd_stamps.so; extra flags in STAMP_FLAGS)
#   tools/stamps.sh run [w ...]  (GPU box: swaps the build in, tools/stamps.py per workload, restores)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
if [ "$1" = build ]; then
  mkdir -p tools/abl
  cd mlx-data_amd
  /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC -Wall -I../include -Icsrc --offload-arch=gfx950 -ffp-contract=fast \
    -DMXD_STAMPS=1 ${STAMP_FLAGS:-} -c csrc/wave.hip -o build/wave_stamps.o || exit 1
  /opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 build/resample.o build/wave_stamps.o build/band.o \
    build/band_plan.o build/pixmap.o build/capi.o build/plan.o build/batch.o build/hostpath.o build/taps.o \
    build/jpeg.o build/jpegdev.o build/jpeghuff.o -o ../tools/libmxd_amd_stamps.so || exit 1
  exit 0
fi
shift
mkdir -p gpurun_out
cp mlx-data_amd/libmxd_amd.so gpurun_out/.product.so
cp tools/libmxd_amd_stamps.so mlx-data_amd/libmxd_amd.so
rc=0
for w in ${@:-c2}; do
  timeout -k 10 120 python tools/stamps.py $w || { rc=$?; break; }
done
cp gpurun_out/.product.so mlx-data_amd/libmxd_amd.so
rm -f gpurun_out/.product.so
exit $rc
