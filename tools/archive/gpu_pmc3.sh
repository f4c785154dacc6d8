#!/bin/bash
# PMC passes for the C2 bench kernel: tools/gpu_pmc3.sh TAG
# One rocprofv3 --pmc pass per group, kernel-trace only (never combined with
# sys/runtime traces).  Env (MXD_*) passes through to bench.py.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-pmc}
i=0
while read -r group; do
  [ -z "$group" ] && continue
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $group --output-format csv -d gpurun_out/${TAG}_p$i -o run -- python3 bench.py --steps 10 --warmup 2 --no-cpu --no-e2e --no-copy > gpurun_out/${TAG}_p$i.log 2>&1
  rc=$?
  echo "pass $i rc=$rc: $group"
  if [ $rc -eq 124 ] || [ $rc -eq 137 ] || [ $rc -ge 128 ]; then echo "stopping"; exit $rc; fi
done <<GROUPS
FETCH_SIZE
WRITE_SIZE
TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum
GRBM_GUI_ACTIVE SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_INSTS_SALU
SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU
TCC_HIT_sum TCC_MISS_sum TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum
TA_TA_BUSY_sum TD_TD_BUSY_sum TA_BUFFER_READ_WAVEFRONTS_sum
GROUPS
exit 0
