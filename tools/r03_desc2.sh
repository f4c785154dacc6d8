#!/bin/bash
# Descriptor forms with slot reuse fenced every 4 written batches: C4 / C2
# cached vs fresh per-launch time, modes 4 (page-locked slot read in place)
# and 6 (host stores into HBM through the large BAR), three repetitions
# (profiles/r03/desc_host_d.jsonl).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for rep in 1 2 3; do for w in c4 c2; do for m in 4 6; do
  timeout -k 10 120 python bench.py --workload $w --no-cpu --no-e2e --no-copy --steps 100 --tune-desc $m > gpurun_out/desch.log 2>&1 || exit 1
  tail -1 gpurun_out/desch.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print(json.dumps(dict(workload='$w', desc_mode=$m, rep=$rep, ms_per_launch=r['kernel_ms_per_launch'], fresh=r['ms_per_launch_fresh_descriptors'], host=r['host_ms_per_call'], host_fresh=r['host_ms_per_call_fresh'])))"
done; done; done
