#!/bin/bash
# Packed u8 stores (product, wave.hip MXD_U8_PACK) against byte stores
# (variant "nopack") and against byte stores with the narrow-lane rings
# (variant "ring": resample.h scatter_narrow_ring, 4 / 3 slots at DMAX 2 / 3,
# 8 waves per SIMD), one process per variant, same box; then the kernels'
# bit-exactness tests on the product build.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for w in "--workload c3 --c3-sizes 640x480" "--workload c3 --c3-sizes 1280x720" "--workload c3" "--workload c4 --launches 100" "--workload c5" "--workload c2"; do
  for rep in 1 2; do
    bash tools/variants.sh run "$w --reps 5" product nopack ring || exit 1
  done
done
timeout -k 10 600 python -u -m pytest tests/test_gpu_vfirst.py tests/test_gpu_kernels.py tests/test_gpu_parity.py -x -q --timeout 150 --timeout-method thread > gpurun_out/r04_ring_tests.log 2>&1; rc=$?
tail -2 gpurun_out/r04_ring_tests.log
exit $rc
