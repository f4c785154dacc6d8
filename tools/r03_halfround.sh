#!/bin/bash
# Consecutive batches on 2-3 streams with full-round units (the planner's
# choice) against half-round units (forced band height, tuning build with
# -DMXD_TUNING_ENV): does co-residency of two launches hide the drain?
# (profiles/r03/halfround.jsonl)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
cp mlx-data_amd/libmxd_amd.so gpurun_out/.product.so
cp tools/libmxd_amd_var_tenv.so mlx-data_amd/libmxd_amd.so
run() {  # workload rows streams
  if [ $2 = 0 ]; then unset MXD_BAND_ROWS; else export MXD_BAND_ROWS=$2; fi
  timeout -k 10 120 python bench.py --workload $1 --streams $3 --steps 100 --warmup 10 --no-cpu --no-e2e --no-copy > gpurun_out/hr.log 2>&1 || { tail -3 gpurun_out/hr.log; return 1; }
  tail -1 gpurun_out/hr.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(json.dumps(dict(workload='$1', rows=$2, streams=$3, value=d['value'], ms_per_step=d['ms_per_step'], ms_per_launch=d['roofline']['kernel_ms_per_launch'])))"
}
for rep in 1 2; do
  for cfg in "c2 0 2" "c2 56 2" "c2 56 3" "c2 0 3" "c5 0 2" "c5 112 2" "c6 0 2" "c6 45 2" "c4 0 2" "c4 28 2"; do run $cfg || break 2; done
done
unset MXD_BAND_ROWS
cp gpurun_out/.product.so mlx-data_amd/libmxd_amd.so
