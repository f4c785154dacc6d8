#!/bin/bash
# Timing-only ablation builds of the wave kernel (wave.hip MXD_ABLATE bits).
#   tools/ablate8.sh build      (here, on the CPU: tools/abl/libmxd_amd_<n>.so)
#   tools/ablate8.sh run TAG    (on the GPU box: swaps each build in, C2 bench)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
# variant name -> compile flags (ablations: wave.hip MXD_ABLATE bits; tuning: MXD_NT_STORE, MXD_MIN_WAVES)
declare -A FLAGS=( [a1]="-DMXD_ABLATE=1" [a2]="-DMXD_ABLATE=2" [a4]="-DMXD_ABLATE=4" [a8]="-DMXD_ABLATE=8"
                   [nt]="-DMXD_NT_STORE=1" [w2]="-DMXD_MIN_WAVES=2" [w4]="-DMXD_MIN_WAVES=4" [w5]="-DMXD_MIN_WAVES=5"
                   [ntw4]="-DMXD_NT_STORE=1 -DMXD_MIN_WAVES=4" [ww3]="-DMXD_MIN_WAVES_WIDE=3" [sync]="-DMXD_SYNC_STRIPS=1" )
MODES=${MODES:-"a1 a2 a4 a8"}
if [ "$1" = tune ]; then
  # product kernels, host code that reads the tuning environment (MXD_BAND_ROWS)
  cd mlx-data_amd
  /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC -Wall -I../include -Icsrc --offload-arch=gfx950 -DMXD_TUNING_ENV \
    -c csrc/capi.cpp -o build/capi_tune.o || exit 1
  /opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 build/resample.o build/wave.o build/pixmap.o \
    build/capi_tune.o build/taps.o build/jpeg.o -o ../tools/abl/libmxd_amd_tune.so || exit 1
  exit 0
fi
if [ "$1" = build ]; then
  cd mlx-data_amd
  for m in $MODES; do
    /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC -Wall -I../include -Icsrc --offload-arch=gfx950 -ffp-contract=fast \
      ${FLAGS[$m]} -c csrc/wave.hip -o build/wave_abl$m.o || exit 1
    /opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 build/resample.o build/wave_abl$m.o build/pixmap.o \
      build/capi.o build/plan.o build/batch.o build/hostpath.o build/taps.o build/jpeg.o -o ../tools/abl/libmxd_amd_$m.so || exit 1
  done
  exit 0
fi
TAG=${2:-abl}
mkdir -p gpurun_out
cp mlx-data_amd/libmxd_amd.so gpurun_out/.product.so
for m in 0 $MODES; do
  if [ $m != 0 ]; then cp tools/abl/libmxd_amd_$m.so mlx-data_amd/libmxd_amd.so; fi
  timeout -k 10 120 python bench.py --no-cpu --no-e2e --no-copy ${BENCH_ARGS:-} > gpurun_out/${TAG}_$m.log 2>&1 || { cp gpurun_out/.product.so mlx-data_amd/libmxd_amd.so; exit 1; }
  echo "ablate $m $(grep -o '"kernel_ms_per_launch": [0-9.]*' gpurun_out/${TAG}_$m.log)"
done
cp gpurun_out/.product.so mlx-data_amd/libmxd_amd.so
rm -f gpurun_out/.product.so
