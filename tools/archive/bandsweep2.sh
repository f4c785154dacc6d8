#!/bin/bash
# Band-height sweep with the tuning library, two passes: tools/bandsweep2.sh WORKLOAD "BANDS"
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
W=${1:-c2}; BANDS=${2:-"0 8 12 16 20 28"}
cp mlx-data_amd/libmxd_amd.so gpurun_out/.product.so
cp tools/abl/libmxd_amd_tune.so mlx-data_amd/libmxd_amd.so
for pass in 1 2; do
  for b in $BANDS; do
    if [ $b = 0 ]; then unset MXD_BAND_ROWS; else export MXD_BAND_ROWS=$b; fi
    timeout -k 10 120 python bench.py --workload $W --no-cpu --no-e2e --no-copy > gpurun_out/bs_${W}_$b.log 2>&1 || { cp gpurun_out/.product.so mlx-data_amd/libmxd_amd.so; exit 1; }
    echo "$pass $W band $b $(grep -o '"kernel_ms_per_launch": [0-9.]*' gpurun_out/bs_${W}_$b.log)"
  done
done
cp gpurun_out/.product.so mlx-data_amd/libmxd_amd.so
rm -f gpurun_out/.product.so
