#!/bin/bash
# Split RGB lanes (variant build -DMXD_SPLIT_LANES=1: two contiguous 768-byte
# halves per window row instead of interleaved dwordx4 + dwordx2): bytes
# against the kernel-order oracle, then per-launch time on C2..C7 against the
# product, round-robin (profiles/r03/split.jsonl).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
cp mlx-data_amd/libmxd_amd.so gpurun_out/.product.so
cp tools/libmxd_amd_var_split.so mlx-data_amd/libmxd_amd.so
timeout -k 10 400 python -u -m pytest tests/test_gpu_vfirst.py tests/test_gpu_parity.py tests/test_gpu_border.py tests/test_gpu_band.py tests/test_gpu_host_path.py -x -q --timeout 150 --timeout-method thread > gpurun_out/split.log 2>&1
rc=$?
cp gpurun_out/.product.so mlx-data_amd/libmxd_amd.so
tail -2 gpurun_out/split.log
[ $rc = 0 ] || exit $rc
for w in c2 c5 c6 c7 c3; do bash tools/variants.sh run "--workload $w --reps 5 --set policy=0" product split || exit 1; done
