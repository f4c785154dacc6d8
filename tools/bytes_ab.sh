#!/bin/bash
# Byte lanes vs pixel lanes (MXD_POLICY_NO_BYTES = 16) per C3 source size:
# u8 batches of 256 images of one size, kernel ms per launch (one stream).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for sz in 640x480 1280x720 1280x960 1920x1080 2560x1440 3840x2160; do
  for pol in 0 16 0 16; do
    timeout -k 10 120 python bench.py --workload c3 --batch 256 --c3-sizes $sz --policy $pol --steps 30 --no-cpu --no-e2e --no-copy > gpurun_out/bab.log 2>&1 || exit 1
    python -c "import json;d=json.loads(open('gpurun_out/bab.log').read().strip().splitlines()[-1]);print('$sz policy $pol', d['roofline']['kernel_ms_per_launch'], d['ms_per_step'])"
  done
done
