#!/bin/bash
# Round-end GPU session: parity tests, smoke, the default bench line (C2, with
# the CPU baseline), c3/c5 bench lines, rocprofv3 kernel stats of the default
# bench, and PMC FETCH_SIZE / WRITE_SIZE passes per workload (kernel-trace
# only).   tools/r1_final.sh TAG
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-fin}
run() {  # name limit cmd...
  local name=$1 lim=$2; shift 2
  timeout -k 10 "$lim" "$@" > gpurun_out/${TAG}_${name}.log 2>&1
  local rc=$?
  echo "== $name rc=$rc"; tail -n 2 gpurun_out/${TAG}_${name}.log | cut -c1-1500
  if [ $rc -ne 0 ]; then echo "stopping"; exit $rc; fi
}
run pytest 500 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread
run smoke 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')"
run bench 400 python bench.py
run bench_c3 300 python bench.py --workload c3 --steps 20 --warmup 3 --no-cpu
run bench_c4 300 python bench.py --workload c4 --steps 20 --warmup 3 --no-cpu
run bench_c5 300 python bench.py --workload c5 --steps 20 --warmup 3 --no-cpu
run prof 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_prof -o run -- python3 bench.py --steps 20 --warmup 3 --no-cpu --no-e2e --no-copy
cut -c1-220 gpurun_out/${TAG}_prof/run_kernel_stats.csv
for w in c2 c3 c5; do
  i=0
  for grp in FETCH_SIZE WRITE_SIZE "GRBM_GUI_ACTIVE SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_INSTS_SALU"; do
    i=$((i+1))
    run ${w}pmc_p$i 120 rocprofv3 --pmc $grp --output-format csv -d gpurun_out/${TAG}_${w}pmc_p$i -o run -- python3 bench.py --workload $w --steps 10 --warmup 2 --no-cpu --no-e2e --no-copy
  done
done
exit 0
