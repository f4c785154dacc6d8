#!/bin/bash
# Round 3 kernel A/B (profiles/r03/kernel_ab_<w>.jsonl): per-launch time of
# the default choice (policy=0: wave kernel where its buckets fit) against the
# band kernel (policy=256, MXD_POLICY_PREFER_BAND; persistent grid, and
# grid=1: one workgroup per unit, rows=8: 8-row bands) on C2..C5, and the band
# kernel's knobs on the large-ratio workloads C6/C7 -- tools/band_sweep.py,
# settings round-robin after a warm-up, one box.
set -u
mkdir -p gpurun_out
S="timeout -k 10 200 python tools/band_sweep.py --reps 5"
$S --workload c2 --set policy=0 --set policy=256 --set policy=256,grid=1 --set policy=256,rows=8 --set policy=256,rows=8,grid=1 > gpurun_out/r03_ab_c2.jsonl 2>&1 || exit 1
for w in c3 c4 c5; do $S --workload $w --set policy=0 --set policy=256 --set policy=256,grid=1 > gpurun_out/r03_ab_$w.jsonl 2>&1 || exit 1; done
for w in c6 c7; do $S --workload $w --set rows=0 --set grid=1 --set la=3 --set rows=8 --set rows=24 > gpurun_out/r03_ab_$w.jsonl 2>&1 || exit 1; done
