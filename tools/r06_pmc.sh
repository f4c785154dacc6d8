#!/bin/bash
# Round-6 PMC session (traffic re-recorded from this
# build for every config): per workload C2..C7 three single-stream passes,
# each its own run with kernel-trace only: FETCH_SIZE, WRITE_SIZE, and the SQ
# group; then gpurun_out/TAG_traffic.json (tools/make_traffic.py) for
# profiles/traffic.json.
#   tools/r06_pmc.sh TAG [workloads]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-r06p}
WS=${2:-c2 c3 c4 c5 c6 c7}
for w in $WS; do
  i=0
  for grp in FETCH_SIZE WRITE_SIZE "GRBM_GUI_ACTIVE SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_INSTS_SALU"; do
    i=$((i+1))
    timeout -s KILL 90 rocprofv3 --pmc $grp --output-format csv -d gpurun_out/${TAG}_${w}pmc_p$i -o run -- python3 bench.py --workload $w --streams 1 --steps 10 --warmup 2 --no-cpu --no-e2e --no-e2e-jpeg --no-others --no-copy > gpurun_out/${TAG}_${w}pmc_p$i.log 2>&1
    rc=$?
    echo "== $w pass $i rc=$rc"
    if [ $rc -ne 0 ]; then tail -5 gpurun_out/${TAG}_${w}pmc_p$i.log; exit $rc; fi
  done
done
python3 tools/make_traffic.py $TAG r06/$TAG
