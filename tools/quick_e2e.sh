#!/bin/bash
# Host-path (PCIe-inclusive) and pipeline spot check: tools/quick_e2e.sh TAG
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
TAG=${1:-q}
timeout -k 10 200 python bench.py --no-cpu > gpurun_out/${TAG}_c2.log 2>&1 || exit 1
timeout -k 10 200 python bench.py --workload c4 --no-cpu > gpurun_out/${TAG}_c4.log 2>&1 || exit 1
timeout -k 10 300 python tools/bench_pipeline.py --datasets c4 --images 4096 --workers 8,16 --variants fused,device > gpurun_out/${TAG}_pipe.log 2>&1 || exit 1
for w in c2 c4; do
  tail -1 gpurun_out/${TAG}_$w.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$w', d['value'], d['roofline']['kernel_ms_per_launch'], d['e2e']['value'])"
done
cat gpurun_out/${TAG}_pipe.log
