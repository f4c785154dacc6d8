#!/bin/bash
# C3 by shape: 512 images of one C3 size per launch (u8 -> 224 crop), per-launch
# time and roofline fraction of each (profiles/r03/c3_shapes.jsonl), beside the
# mixed C3 line.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for s in 640x480 1280x720 1280x960 1920x1080 2560x1440 3840x2160 mixed; do
  a="--c3-sizes $s"; [ $s = mixed ] && a=""
  timeout -k 10 120 python bench.py --workload c3 $a --steps 20 --warmup 3 --no-cpu --no-e2e --no-copy --streams 1 > gpurun_out/c3s_$s.log 2>&1 || exit 1
  tail -1 gpurun_out/c3s_$s.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print(json.dumps(dict(shape='$s', ms_per_launch=r['kernel_ms_per_launch'], frac=r['frac'], alg_mb=round(r['alg_bytes_per_launch']/1e6,1), kernel=r['kernel'])))"
done
