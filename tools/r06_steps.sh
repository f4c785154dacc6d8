#!/bin/bash
# Round 6: C2 step time against the timed steps and the warm-up before them
# (bench.py --steps / --warmup, two streams), two repetitions, on one box.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r06
O=gpurun_out/r06/${1:-r06h}_steps.jsonl
: > $O
for rep in 1 2; do
  for cfg in "20 5" "50 5" "200 5" "20 200" "50 200" "20 1000"; do
    set -- $cfg
    line=$(timeout -k 10 120 python bench.py --steps $1 --warmup $2 --no-cpu --no-e2e --no-e2e-jpeg --no-others --no-copy | tail -1) || exit 1
    python3 -c "import json,sys;d=json.loads(sys.argv[1]);print(json.dumps({'steps':$1,'warmup':$2,'rep':$rep,'value':d['value'],'ms_per_step':d['ms_per_step']}))" "$line" | tee -a $O
  done
done
