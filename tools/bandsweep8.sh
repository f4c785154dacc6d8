#!/bin/bash
# Band-height sweep of the C2 kernel with the tuning library (tools/ablate8.sh tune).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
cp mlx-data_amd/libmxd_amd.so gpurun_out/.product.so
cp tools/abl/libmxd_amd_tune.so mlx-data_amd/libmxd_amd.so
for b in ${BANDS:-0 4 8 12 16 28}; do
  if [ $b = 0 ]; then unset MXD_BAND_ROWS; else export MXD_BAND_ROWS=$b; fi
  timeout -k 10 120 python bench.py --no-cpu --no-e2e --no-copy ${BENCH_ARGS:-} > gpurun_out/band_$b.log 2>&1 || { cp gpurun_out/.product.so mlx-data_amd/libmxd_amd.so; exit 1; }
  echo "band $b $(grep -o '"kernel_ms_per_launch": [0-9.]*' gpurun_out/band_$b.log)"
done
cp gpurun_out/.product.so mlx-data_amd/libmxd_amd.so
rm -f gpurun_out/.product.so
