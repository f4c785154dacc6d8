#!/bin/bash
# Round 6, VERDICT r5 next 1: cache-policy A/B of the resize kernels' source
# loads and the HBM ceilings by policy, on one box.
#   1. tools/nt_ceiling: copy / read / LDS-DMA read streams, default vs nt / sc1
#   2. tools/lib_ab.py: the product library and the load-policy variants
#      (tools/variants.sh build ntl "-DMXD_LOAD_AUX=2" wave, sc1 16, ntsc0 3,
#      ntsc1 18) in ONE process, round-robin, on C2 / C3 / C4 / C5
#   3. band.hip's MXD_BAND_LOAD_AUX=2 variant (bandnt) against the product
#      under MXD_POLICY_PREFER_BAND on C2 (tools/band_sweep.py policy 256)
# Output: gpurun_out/r06/<tag>_*.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${1:-r06a}
VARS=${2:-product,ntl,sc1,ntsc0,ntsc1}
mkdir -p gpurun_out/r06
O=gpurun_out/r06/$TAG
timeout -k 10 180 tools/nt_ceiling > ${O}_ceiling.jsonl || exit 1
timeout -k 10 600 python -u tools/lib_ab.py --workloads c2,c3,c4,c5 --variants $VARS --reps 5 > ${O}_lib_ab.jsonl || exit 1
if [ -f tools/libmxd_amd_var_bandnt.so ]; then
  timeout -k 10 300 python -u tools/lib_ab.py --workloads c2 --variants product,bandnt --reps 5 --policy 256 > ${O}_band_ab.jsonl || exit 1
fi
exit 0
