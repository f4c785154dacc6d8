#!/bin/bash
# Band-height sweep with the tuning library (tools/libmxd_amd_tune.so: capi.cpp built with -DMXD_TUNING_ENV,
# which reads MXD_BAND_ROWS); 0 = the capacity-based choice.  BANDS / WL select the sweep.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
cp mlx-data_amd/libmxd_amd.so gpurun_out/.product.so
cp tools/libmxd_amd_tune.so mlx-data_amd/libmxd_amd.so
rc=0
for pass in 1 2; do
  for b in ${BANDS:-0 14 10 7}; do
    if [ $b = 0 ]; then unset MXD_BAND_ROWS; else export MXD_BAND_ROWS=$b; fi
    WL=${WL:-c2} tools/quick_bench.sh | head -1 | sed "s/^/band $b /" || { rc=1; break 2; }
  done
done
unset MXD_BAND_ROWS
cp gpurun_out/.product.so mlx-data_amd/libmxd_amd.so
rm -f gpurun_out/.product.so
exit $rc
