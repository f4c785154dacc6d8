#!/bin/bash
# Round 5: the real wave kernel at forced band heights that make the launch
# several occupancy rounds (the strip probe's "sweep" form: C2 148 -> 136.5 us
# at 4 rounds, profiles/r05/strip_probe.txt), round-robin in one process.
# Tuning-environment build: tools/variants.sh build tenv "-DMXD_TUNING_ENV" plan
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
cp mlx-data_amd/libmxd_amd.so gpurun_out/.product.so
cp tools/libmxd_amd_var_tenv.so mlx-data_amd/libmxd_amd.so
S="timeout -k 10 200 python tools/band_sweep.py --reps 5"
rc=0
$S --workload c2 --set wrows=0 --set wrows=14 --set wrows=7 --set wrows=9 --set wrows=4 --set wrows=5 || rc=1
[ $rc = 0 ] && { $S --workload c5 --set wrows=0 --set wrows=28 --set wrows=14 --set wrows=9 || rc=1; }
[ $rc = 0 ] && { $S --workload c3 --set wrows=0 --set wrows=14 --set wrows=7 --set wrows=10 || rc=1; }
[ $rc = 0 ] && { $S --workload c6 --set wrows=0 --set wrows=12 --set wrows=6 || rc=1; }
[ $rc = 0 ] && { $S --workload c4 --set wrows=0 --set wrows=7 --set wrows=5 || rc=1; }
cp gpurun_out/.product.so mlx-data_amd/libmxd_amd.so
exit $rc
