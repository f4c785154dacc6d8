#!/bin/bash
# C3's six shapes as separate 85-image launches (one process per shape) next
# to the mixed 512-image batch: how much of the mixed launch's time is the
# small launches themselves (profiles/r03/c3_parts.jsonl).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for s in 640x480 1280x720 1280x960 1920x1080 2560x1440 3840x2160; do
  timeout -k 10 150 python tools/band_sweep.py --workload c3 --c3-sizes $s --batch 85 --reps 5 --set policy=0 | sed "s/^/{\"shape\": \"$s\", \"batch\": 85, \"r\": /; s/$/}/" || exit 1
done
timeout -k 10 150 python tools/band_sweep.py --workload c3 --reps 5 --set policy=0 | sed "s/^/{\"shape\": \"mixed\", \"batch\": 512, \"r\": /; s/$/}/"
