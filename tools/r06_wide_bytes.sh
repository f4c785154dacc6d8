#!/bin/bash
# Round 6, late: wide byte lanes (p = 24, a b128 + a b64 per lane) against
# the wide pixel lanes they replace (p = 8, MXD_POLICY_NO_BYTES = 16), in one
# process (tools/lib_ab.py), on every workload the scatter kernels serve;
# then the GPU tests of the kernel layouts.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r06
O=gpurun_out/r06/${1:-r06s}
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_kernels.py tests/test_gpu_byte_lanes.py tests/test_gpu_parity.py > ${O}_pytest.txt 2>&1 || { tail -30 ${O}_pytest.txt; exit 1; }
tail -2 ${O}_pytest.txt
timeout -k 10 500 python -u tools/lib_ab.py --workloads c2,c3,c5,c6,c7,c4 --variants product,product@policy=16 --reps 7 \
  > ${O}_lib_ab.jsonl || exit 1
cut -c1-150 ${O}_lib_ab.jsonl
