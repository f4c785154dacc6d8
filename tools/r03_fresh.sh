#!/bin/bash
# Fresh-descriptor cost in the bench line (ms_per_launch_fresh_descriptors
# against kernel_ms_per_launch), C4 three times and C2 once
# (profiles/r03/fresh_<tag>.jsonl).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for w in c4 c4 c4 c2; do
  timeout -k 10 120 python bench.py --workload $w --no-cpu --no-e2e --no-copy --steps ${STEPS:-50} > gpurun_out/fr.log 2>&1 || exit 1
  tail -1 gpurun_out/fr.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print(json.dumps(dict(workload='$w', ms_per_launch=r['kernel_ms_per_launch'], fresh=r['ms_per_launch_fresh_descriptors'], host=r['host_ms_per_call'], host_fresh=r['host_ms_per_call_fresh'])))"
done
