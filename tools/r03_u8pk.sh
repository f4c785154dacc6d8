#!/bin/bash
# u8 outputs through v_cvt_pk_u8_f32 (variant build -DMXD_U8_PK=1): bytes
# against the kernel-order oracle, then per-launch time on the u8 workloads
# C3 / C5 against the product (profiles/r03/u8pk.jsonl).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
cp mlx-data_amd/libmxd_amd.so gpurun_out/.product.so
cp tools/libmxd_amd_var_u8pk.so mlx-data_amd/libmxd_amd.so
timeout -k 10 300 python -u -m pytest tests/test_gpu_vfirst.py tests/test_gpu_parity.py tests/test_gpu_byte_lanes.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pk.log 2>&1
rc=$?
cp gpurun_out/.product.so mlx-data_amd/libmxd_amd.so
tail -2 gpurun_out/pk.log
[ $rc = 0 ] || exit $rc
for w in c5 c3; do bash tools/variants.sh run "--workload $w --reps 5 --set policy=0" product u8pk || exit 1; done
