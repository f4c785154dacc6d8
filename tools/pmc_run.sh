#!/bin/bash
# PMC passes over one bench.py command: tools/pmc_run.sh TAG "BENCH ARGS" "GROUP1" ["GROUP2" ...]
# One rocprofv3 --pmc pass per group (kernel-trace collection only, never
# combined with sys/runtime traces), each under its own time limit.  A pass
# that fails stops the script.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=$1; ARGS=$2; shift 2
i=0
for group in "$@"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $group --output-format csv -d gpurun_out/${TAG}_p$i -o run -- python3 bench.py $ARGS --no-cpu --no-e2e --no-copy > gpurun_out/${TAG}_p$i.log 2>&1
  rc=$?
  echo "pass $i rc=$rc: $group"
  if [ $rc -ne 0 ]; then echo "stopping"; exit $rc; fi
done
exit 0
