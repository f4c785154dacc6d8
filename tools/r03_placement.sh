#!/bin/bash
# Placement probe (profiles/r03/placement.jsonl): per-launch time of C2 / C4
# over 6 independent allocations of the inputs in one process, and the same
# default setting in three separate processes.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for w in c2 c4; do timeout -k 10 200 python tools/placement_probe.py --workload $w --allocs 6 || exit 1; done
for k in 1 2 3; do timeout -k 10 120 python tools/band_sweep.py --workload c2 --reps 5 --set policy=0 || exit 1; done
