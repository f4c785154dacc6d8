#!/bin/bash
# C4 reads against band height: the
# tuning-environment build (tools/variants.sh build tenv "-DMXD_TUNING_ENV"
# plan) swapped in; per forced band height (0 = the planner's) a FETCH_SIZE
# and a WRITE_SIZE pass over single-stream C4 launches, then the per-launch
# time of every height round-robin in one process (tools/band_sweep.py).
#   tools/r04_c4rows.sh TAG
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-r04c}
cp mlx-data_amd/libmxd_amd.so gpurun_out/.product.so
cp tools/libmxd_amd_var_tenv.so mlx-data_amd/libmxd_amd.so
restore() { cp gpurun_out/.product.so mlx-data_amd/libmxd_amd.so; rm -f gpurun_out/.product.so; }
for rows in 0 16 23 32 56; do
  if [ $rows = 0 ]; then unset MXD_BAND_ROWS; else export MXD_BAND_ROWS=$rows; fi
  i=0
  for grp in FETCH_SIZE WRITE_SIZE; do
    i=$((i+1))
    timeout -s KILL 90 rocprofv3 --pmc $grp --output-format csv -d gpurun_out/${TAG}_rows${rows}_p$i -o run -- python3 bench.py --workload c4 --streams 1 --steps 10 --warmup 2 --no-cpu --no-e2e --no-copy > gpurun_out/${TAG}_rows${rows}_p$i.log 2>&1
    rc=$?
    echo "== rows $rows pass $i rc=$rc"
    if [ $rc -ne 0 ]; then tail -5 gpurun_out/${TAG}_rows${rows}_p$i.log; restore; exit $rc; fi
  done
  python3 tools/pmc_traffic.py ${TAG}_rows${rows} gpurun_out/${TAG}_rows${rows}_pmc.json resample_ | head -12
done
unset MXD_BAND_ROWS
timeout -k 10 300 python tools/band_sweep.py --workload c4 --launches 100 --reps 5 --set wrows=0 --set wrows=16 --set wrows=23 --set wrows=32 --set wrows=56 > gpurun_out/${TAG}_sweep.jsonl 2>&1
rc=$?
cat gpurun_out/${TAG}_sweep.jsonl
restore
exit $rc
