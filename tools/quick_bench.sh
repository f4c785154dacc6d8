#!/bin/bash
# Device-resident bench lines, two passes per workload: value (two streams),
# ms per step and the single-stream kernel ms per launch.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for w in ${WL:-c2 c4 c5 c3}; do
  for pass in 1 2; do
    timeout -k 10 120 python bench.py --workload $w ${BENCH_ARGS:-} --no-cpu --no-e2e --no-copy > gpurun_out/qb.log 2>&1 || exit 1
    python -c "import json;d=json.loads(open('gpurun_out/qb.log').read().strip().splitlines()[-1]);r=d['roofline'];print('$w', d['value'], d['ms_per_step'], r['kernel_ms_per_launch'], r['frac'])"
  done
done
