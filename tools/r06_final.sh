#!/bin/bash
# Round-6 final records (one box): GPU tests + smoke, (LOAD_AB="c2 ..." adds) the load-policy
# A/B of the product build in one process per workload (MXD_TUNE_LOAD_POLICY
# auto / default / nt, tools/band_sweep.py), the default bench line, the C2
# single-stream line, and rocprofv3 kernel stats of both C2 commands.
#   tools/r06_quick.sh TAG [skip-tests]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r06
export TMPDIR=/tmp
TAG=${1:-r06z}
O=gpurun_out/r06/$TAG
run() {  # name limit cmd...
  local name=$1 lim=$2; shift 2
  timeout -k 10 "$lim" "$@" > ${O}_${name}.log 2>&1
  local rc=$?
  echo "== $name rc=$rc"; tail -n 2 ${O}_${name}.log | cut -c1-600
  if [ $rc -ne 0 ]; then echo "stopping"; exit $rc; fi
}
if [ "${2:-}" != "skip-tests" ]; then
  run pytest_gpu 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread -p no:cacheprovider
  run smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
fi
for w in ${LOAD_AB:-}; do
  run load_ab_$w 200 python tools/band_sweep.py --workload $w --reps 5 --set load=0 --set load=1 --set load=2
done
run bench 600 python bench.py
# the launcher the driver uses for N > 1, here with one rank (the only GPU)
run bench_torchrun 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 \
  --master-port 29517 bench.py --gpus 1 --steps 20 --warmup 3 --no-cpu --no-e2e --no-e2e-jpeg --no-others
run bench_1stream 300 python bench.py --streams 1 --no-cpu --no-e2e --no-e2e-jpeg --no-others
FLAGS="--no-cpu --no-e2e --no-e2e-jpeg --no-others"
run prof 300 rocprofv3 --kernel-trace --stats --output-format csv -d ${O}_prof -o run -- python3 bench.py $FLAGS
run prof_1stream 300 rocprofv3 --kernel-trace --stats --output-format csv -d ${O}_prof1 -o run -- python3 bench.py --streams 1 $FLAGS
exit 0
