#!/bin/bash
# Round 6: work stealing between the units of a scatter wave launch
# (wave.hip Steal), on one box.
#   1. GPU tests of the stealing modes (byte-identical outputs) and the kernel
#      kinds
#   2. tools/lib_ab.py in ONE process, round-robin: the pre-stealing kernels
#      (tools/variants.sh build nosteal "-DMXD_STEAL=0" wave), the product with
#      stealing off / on / fewest blocks 1 and 4, on C2 / C3 / C4 / C5
# Output: gpurun_out/r06/<tag>_*.
# (Runs against the stealing builds only -- commits 2f4a86b and the one after
# it; the product reverted to the static units)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${1:-r06s}
VARS=${2:-nosteal,product@steal=1,product,product@steal_min=1,product@steal_min=4}
mkdir -p gpurun_out/r06
O=gpurun_out/r06/$TAG
timeout -k 10 400 python -u -m pytest -x -v --timeout 150 --timeout-method thread tests/test_gpu_steal.py \
  tests/test_gpu_kernels.py > ${O}_pytest.txt 2>&1 || { tail -30 ${O}_pytest.txt; exit 1; }
tail -3 ${O}_pytest.txt
timeout -k 10 600 python -u tools/lib_ab.py --workloads c2,c3,c4,c5 --variants $VARS --reps 5 > ${O}_lib_ab.jsonl || exit 1
cat ${O}_lib_ab.jsonl | cut -c1-160
exit 0
