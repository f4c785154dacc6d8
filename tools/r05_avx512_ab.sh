#!/bin/bash
# Round 5, late: AVX-512 byte scans (marker parse, unstuff) on the box CPU --
# the per-file probe with and without them, then the C4 / C1 device-batch
# pipeline at 16 workers alternating MXD_NO_AVX512=1 / default.
#   tools/r05_avx512_ab.sh TAG
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-r05avx}
python -c "
import sys, shutil, os
sys.path[:0]=['tools','mlx-data_amd']
import bench_pipeline as bp
fs=bp.make_files('/tmp/hp', 'c4', 128)
os.makedirs('/tmp/hpf', exist_ok=True)
[shutil.copy(f, '/tmp/hpf/%d.jpg' % i) for i, f in enumerate(fs)]
" || exit 1
MXD_NO_AVX512=1 tools/host_parse_probe /tmp/hpf | sed 's/^{/{"avx512": 0, /' > gpurun_out/${TAG}_probe.jsonl
tools/host_parse_probe /tmp/hpf | sed 's/^{/{"avx512": 1, /' >> gpurun_out/${TAG}_probe.jsonl
cat gpurun_out/${TAG}_probe.jsonl
P="python tools/bench_pipeline.py --datasets c4,c1 --variants device --workers 1,16 --min-seconds 3 --images 1024 --stats"
: > gpurun_out/${TAG}.jsonl
for rep in 1 2; do
  for v in 1 0; do
    MXD_NO_AVX512=$v timeout -k 10 300 $P > gpurun_out/${TAG}_pt.log 2>&1 || { tail -5 gpurun_out/${TAG}_pt.log; exit 1; }
    grep '^{' gpurun_out/${TAG}_pt.log | sed "s/^{/{\"no_avx512\": $v, /" | tee -a gpurun_out/${TAG}.jsonl
  done
done
