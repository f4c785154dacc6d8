#!/bin/bash
# Round 5: the host path's staging helpers sized by the cgroup CPU quota
# (default) against the affinity mask (MXD_HOST_CPUS set to it: the earlier
# sizing), JPEG device batch at 12 / 16 / 24 workers, alternating.
#   tools/r05_e2e_cpus.sh TAG
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-r05cpus}
DS=${DATASETS:-c4}
out=gpurun_out/${TAG}.jsonl
: > $out
{ cat /sys/fs/cgroup/cpu.max 2>&1; nproc; echo "OMP_NUM_THREADS=${OMP_NUM_THREADS:-}"; } > gpurun_out/${TAG}_cpus.txt
cat gpurun_out/${TAG}_cpus.txt
MASK=$(python -c "import os; print(len(os.sched_getaffinity(0)))")
point() {  # label workers [env...]
  local label=$1 w=$2; shift 2
  timeout -k 10 200 env "$@" python tools/bench_pipeline.py --datasets $DS --variants device --workers $w \
      --min-seconds 3 --images 1024 > gpurun_out/${TAG}_pt.log 2>&1
  local rc=$?
  if [ $rc -ne 0 ]; then echo "== $label rc=$rc"; tail -n 5 gpurun_out/${TAG}_pt.log; exit $rc; fi
  grep '^{' gpurun_out/${TAG}_pt.log | sed "s/^{/{\"label\": \"$label\", /" | tee -a $out
}
for rep in 1 2; do
  for w in ${WORKERS:-16 12 24}; do
    point quota $w X=1
    point mask $w MXD_HOST_CPUS=$MASK
  done
done
exit 0
