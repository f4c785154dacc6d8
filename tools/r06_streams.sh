#!/bin/bash
# Round 6: C2 step time by the number of streams (and input / output sets)
# the bench's timed loop spreads its launches over (bench.py --streams /
# --sets), two repetitions, on one box.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r06
O=gpurun_out/r06/${1:-r06g}_streams.jsonl
: > $O
for rep in 1 2; do
  for cfg in "1 2" "2 2" "3 3" "4 4" "2 4"; do
    set -- $cfg
    line=$(timeout -k 10 120 python bench.py --streams $1 --sets $2 --steps 200 --no-cpu --no-e2e --no-e2e-jpeg --no-others --no-copy | tail -1) || exit 1
    python3 -c "import json,sys;d=json.loads(sys.argv[1]);print(json.dumps({'streams':$1,'sets':$2,'rep':$rep,'value':d['value'],'ms_per_step':d['ms_per_step']}))" "$line" | tee -a $O
  done
done
