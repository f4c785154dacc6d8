#!/bin/bash
# Round-5 first session: the sweep / sibling strip probe
# and the default bench line of the current tree.
#   tools/r05_probe.sh TAG
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-r05a}
run() {  # name limit cmd...
  local name=$1 lim=$2; shift 2
  timeout -k 10 "$lim" "$@" > gpurun_out/${TAG}_${name}.log 2>&1
  local rc=$?
  echo "== $name rc=$rc"; tail -n 3 gpurun_out/${TAG}_${name}.log | cut -c1-2500
  if [ $rc -ne 0 ]; then echo "stopping"; exit $rc; fi
}
run strip 240 tools/strip_probe
cat gpurun_out/${TAG}_strip.log
run bench 400 python bench.py --no-e2e
exit 0
