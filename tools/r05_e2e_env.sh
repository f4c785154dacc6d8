#!/bin/bash
# Round 5: JPEG device-batch pipeline (bench_pipeline.py device variant)
# under environment / worker-count variants, alternating, to find what bounds
# the host side at 16 workers.   tools/r05_e2e_env.sh TAG
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-r05env}
DS=${DATASETS:-c4}
NOTRIM="glibc.malloc.trim_threshold=1073741824:glibc.malloc.mmap_threshold=1073741824:glibc.malloc.top_pad=268435456"
out=gpurun_out/${TAG}.jsonl
: > $out
point() {  # label workers [env...]
  local label=$1 w=$2; shift 2
  timeout -k 10 200 env "$@" python tools/bench_pipeline.py --datasets $DS --variants device --workers $w \
      --min-seconds 3 --images 1024 > gpurun_out/${TAG}_pt.log 2>&1
  local rc=$?
  if [ $rc -ne 0 ]; then echo "== $label rc=$rc"; tail -n 5 gpurun_out/${TAG}_pt.log; exit $rc; fi
  grep '^{' gpurun_out/${TAG}_pt.log | sed "s/^{/{\"label\": \"$label\", /" | tee -a $out
}
for rep in 1 2; do
  point base 16 X=1
  point notrim 16 GLIBC_TUNABLES=$NOTRIM
  point w12 12 X=1
  point w24 24 X=1
done
exit 0
