#!/bin/bash
# Occupancy / band-height check (profiles/r03/capacity.jsonl): what the
# occupancy API reports for each workload's wave kernel, then per-launch
# time of the planner's band height against forced heights, round-robin in
# one process (tuning build with -DMXD_TUNING_ENV: band_sweep's wrows knob).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 60 ./tools/capacity_probe || exit 1
cp mlx-data_amd/libmxd_amd.so gpurun_out/.product.so
cp tools/libmxd_amd_var_tenv.so mlx-data_amd/libmxd_amd.so
S="timeout -k 10 200 python tools/band_sweep.py --reps 5"
$S --workload c2 --set wrows=0 --set wrows=28 --set wrows=56 --set wrows=14 --set wrows=19
$S --workload c5 --set wrows=0 --set wrows=75 --set wrows=38 --set wrows=56
$S --workload c6 --set wrows=0 --set wrows=14 --set wrows=10 --set wrows=19
$S --workload c7 --set wrows=0 --set wrows=16 --set wrows=12 --set wrows=23
$S --workload c4 --set wrows=0 --set wrows=10 --set wrows=14 --set wrows=19
cp gpurun_out/.product.so mlx-data_amd/libmxd_amd.so
