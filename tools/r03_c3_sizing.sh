#!/bin/bash
# C3 mixed batch: launches over 1 / 2 / 4 streams x per-launch or joint band
# heights (MXD_TUNE_STREAMS, MXD_TUNE_SIZING), round-robin in one process
# (profiles/r03/c3_sizing.jsonl).  Joint sizing (sizing=2: units of equal
# work over all shapes, whole rounds of the device) measured 24-49 % slower and
# was removed with its knob after this run; the script is kept as the record.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python tools/band_sweep.py --workload c3 --reps 5 --set streams=4,sizing=1 --set streams=4,sizing=2 \
  --set streams=2,sizing=1 --set streams=2,sizing=2 --set streams=1,sizing=1 --set streams=1,sizing=2
