#!/bin/bash
# C3 by shape (512 images of one size, u8): lane layouts the planner chooses
# between -- default, narrow pixel lanes (MXD_POLICY_NARROW = 4), no byte lanes
# (16), byte lanes where a kernel exists (32) -- round-robin in one process
# per shape (profiles/r03/c3_layouts.jsonl).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for s in 640x480 1280x720 1280x960 1920x1080 2560x1440 3840x2160; do
  timeout -k 10 150 python tools/band_sweep.py --workload c3 --c3-sizes $s --reps 5 --set policy=0 --set policy=4 --set policy=16 --set policy=32 | sed "s/^/{\"shape\": \"$s\", \"r\": /; s/$/}/" || exit 1
done
