#!/bin/bash
# C4 band height sweep (tuning build with -DMXD_TUNING_ENV: MXD_BAND_ROWS
# forces the wave kernels' band height): per-launch time vs the planner's
# choice (10 rows: one occupancy round) -- profiles/r03/c4_rows.jsonl.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
cp mlx-data_amd/libmxd_amd.so gpurun_out/.product.so
cp tools/libmxd_amd_var_tenv.so mlx-data_amd/libmxd_amd.so
for w in c4 c2; do for r in 0 8 10 12 14 16 20 28; do
  if [ $r = 0 ]; then unset MXD_BAND_ROWS; else export MXD_BAND_ROWS=$r; fi
  timeout -k 10 120 python tools/band_sweep.py --workload $w --reps 5 --set policy=0 | sed "s/^/{\"rows\": $r, \"r\": /; s/$/}/" || break
done; done
unset MXD_BAND_ROWS
cp gpurun_out/.product.so mlx-data_amd/libmxd_amd.so
