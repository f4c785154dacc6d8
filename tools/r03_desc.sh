#!/bin/bash
# Descriptor upload modes (MXD_TUNE_DESC 1..4) with the submitting thread's
# time per call (profiles/r03/desc_host.jsonl).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for w in c4 c2; do for m in 1 3 4 6; do
  timeout -k 10 120 python bench.py --workload $w --no-cpu --no-e2e --no-copy --steps 100 --tune-desc $m > gpurun_out/desch_${w}_$m.log 2>&1 || exit 1
  tail -1 gpurun_out/desch_${w}_$m.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print(json.dumps(dict(workload='$w', desc_mode=$m, ms_per_launch=r['kernel_ms_per_launch'], fresh=r['ms_per_launch_fresh_descriptors'], host=r['host_ms_per_call'], host_fresh=r['host_ms_per_call_fresh'])))"
done; done
