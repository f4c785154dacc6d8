#!/bin/bash
# Round-4 measurement session (one box): GPU tests + smoke, bench lines for
# every device-resident workload (default: two streams), the C2 single-stream
# line, rocprofv3 kernel stats of the default bench command (C2) and of the
# C4 / C6 single-stream runs, PMC FETCH/WRITE/SQ passes per workload (single
# stream, kernel-trace only, each pass its own run), profiles/traffic.json
# inputs, and optionally the operator-surface pipeline bench.  rocprof stats
# of C3 / C5 / C6 / C7 are single-stream runs of 20 launches.
#   tools/r04_measure.sh TAG [skip-pipeline] [skip-pmc] [skip-tests]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-r04}
run() {  # name limit cmd...
  local name=$1 lim=$2; shift 2
  timeout -k 10 "$lim" "$@" > gpurun_out/${TAG}_${name}.log 2>&1
  local rc=$?
  echo "== $name rc=$rc"; tail -n 2 gpurun_out/${TAG}_${name}.log | cut -c1-1500
  if [ $rc -ne 0 ]; then echo "stopping"; exit $rc; fi
}
if [ "${4:-}" != "skip-tests" ]; then
  run pytest_gpu 900 python -u -m pytest tests -x -q -m gpu --timeout 150 --timeout-method thread
  run smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
fi
run bench 400 python bench.py
run bench_c2_1stream 200 python bench.py --streams 1 --no-cpu --no-e2e
run bench_c3 300 python bench.py --workload c3 --steps 20 --warmup 3 --no-cpu
run bench_c4 300 python bench.py --workload c4 --steps 50 --warmup 5 --no-cpu
run bench_c5 300 python bench.py --workload c5 --steps 20 --warmup 3 --no-cpu
run bench_c6 300 python bench.py --workload c6 --steps 20 --warmup 3 --no-cpu --no-e2e
run bench_c7 300 python bench.py --workload c7 --steps 20 --warmup 3 --no-cpu --no-e2e
run prof 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_prof -o run -- python3 bench.py --no-cpu --no-e2e
cut -c1-220 gpurun_out/${TAG}_prof/run_kernel_stats.csv
run prof_1stream 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_prof1 -o run -- python3 bench.py --streams 1 --no-cpu --no-e2e
cut -c1-220 gpurun_out/${TAG}_prof1/run_kernel_stats.csv
run prof_c4 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_prof_c4 -o run -- python3 bench.py --workload c4 --streams 1 --no-cpu --no-e2e
cut -c1-220 gpurun_out/${TAG}_prof_c4/run_kernel_stats.csv
for w in c3 c5 c6 c7; do
  run prof_$w 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_prof_$w -o run -- python3 bench.py --workload $w --streams 1 --steps 20 --warmup 3 --no-cpu --no-e2e
  cut -c1-220 gpurun_out/${TAG}_prof_$w/run_kernel_stats.csv
done
if [ "${3:-}" != "skip-pmc" ]; then
for w in c2 c3 c4 c5 c6 c7; do
  i=0
  for grp in FETCH_SIZE WRITE_SIZE "GRBM_GUI_ACTIVE SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_INSTS_SALU"; do
    i=$((i+1))
    run ${w}pmc_p$i 120 rocprofv3 --pmc $grp --output-format csv -d gpurun_out/${TAG}_${w}pmc_p$i -o run -- python3 bench.py --workload $w --streams 1 --steps 10 --warmup 2 --no-cpu --no-e2e --no-copy
  done
done
python3 tools/make_traffic.py $TAG r04/$TAG > /dev/null
fi
if [ "${2:-}" != "skip-pipeline" ]; then
  run pipeline 1000 python -u tools/bench_pipeline.py --images 4096 --variants device,device_hostent,fused,ref_form,cpu
fi
exit 0
