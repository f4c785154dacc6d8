#!/bin/bash
# Round-2 GPU measurement session (one box, one run): bench lines for every
# device-resident workload, rocprofv3 kernel stats of the default bench
# command, PMC FETCH_SIZE / WRITE_SIZE / SQ passes per workload (kernel-trace
# only, each pass its own run), and the end-to-end pipeline bench.
#   tools/r02_measure.sh TAG [skip-pipeline]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-r02}
run() {  # name limit cmd...
  local name=$1 lim=$2; shift 2
  timeout -k 10 "$lim" "$@" > gpurun_out/${TAG}_${name}.log 2>&1
  local rc=$?
  echo "== $name rc=$rc"; tail -n 2 gpurun_out/${TAG}_${name}.log | cut -c1-1500
  if [ $rc -ne 0 ]; then echo "stopping"; exit $rc; fi
}
run bench 400 python bench.py
run bench_c3 300 python bench.py --workload c3 --steps 20 --warmup 3 --no-cpu
run bench_c4 300 python bench.py --workload c4 --steps 50 --warmup 5 --no-cpu
run bench_c5 300 python bench.py --workload c5 --steps 20 --warmup 3 --no-cpu
# the bench's own launches only (the e2e leg's chunked launches would mix into the average)
run prof 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_prof -o run -- python3 bench.py --no-cpu --no-e2e
cut -c1-220 gpurun_out/${TAG}_prof/run_kernel_stats.csv
run prof_c4 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_prof_c4 -o run -- python3 bench.py --workload c4 --no-cpu --no-e2e
cut -c1-220 gpurun_out/${TAG}_prof_c4/run_kernel_stats.csv
for w in c2 c3 c4 c5; do
  i=0
  for grp in FETCH_SIZE WRITE_SIZE "GRBM_GUI_ACTIVE SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_INSTS_SALU"; do
    i=$((i+1))
    run ${w}pmc_p$i 120 rocprofv3 --pmc $grp --output-format csv -d gpurun_out/${TAG}_${w}pmc_p$i -o run -- python3 bench.py --workload $w --steps 10 --warmup 2 --no-cpu --no-e2e --no-copy
  done
done
python3 tools/make_traffic.py $TAG r02/$TAG > /dev/null
# N>1 rehearsal on this one GPU: two ranks through torch.distributed.run, both on device 0
run dist2 240 env MXD_BENCH_DEVICE=0 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29513 bench.py --gpus 2 --steps 10 --warmup 3 --no-cpu
if [ "${2:-}" != "skip-pipeline" ]; then
  run pipeline 900 python tools/bench_pipeline.py --images 4096 --cpu-images 2048
fi
exit 0
