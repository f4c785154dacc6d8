#!/bin/bash
# GPU session: parity tests, ablation (mode 5), workloads c2/c3/c5, PMC passes.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
TAG=${1:-r1}
run() {  # name limit cmd...
  local name=$1 lim=$2; shift 2
  timeout -k 10 "$lim" "$@" > gpurun_out/${TAG}_${name}.log 2>&1
  local rc=$?
  echo "== $name rc=$rc"; tail -n 3 gpurun_out/${TAG}_${name}.log | cut -c1-600
  if [ $rc -gt 1 ]; then echo "stopping"; exit $rc; fi
}
run pytest 600 python -m pytest tests -x -q -m gpu
for m in 0 5 6 7 8 2; do
  MXD_WAVE_ABLATE=$m run abl_m$m 300 python bench.py --steps 30 --warmup 3 --no-cpu --no-e2e
done
for w in c3 c5; do run bench_$w 300 python bench.py --workload $w --steps 20 --warmup 3 --no-cpu; done
bash tools/gpu_pmc3.sh ${TAG}_c2pmc
