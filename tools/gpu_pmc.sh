#!/bin/bash
# PMC counter passes (one rocprofv3 --pmc pass per group, kernel-trace only;
# never combined with sys/runtime traces).  Usage: tools/gpu_pmc.sh TAG [bench args...]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-pmc}; shift || true
ARGS=${@:-"--steps 10 --warmup 2 --no-cpu --no-e2e"}
timeout -k 10 120 rocprofv3 -L > gpurun_out/${TAG}_counters.txt 2>&1 || true
i=0
while read -r group; do
  [ -z "$group" ] && continue
  i=$((i+1))
  echo "=== pass $i: $group"
  timeout -k 10 300 rocprofv3 --pmc $group --output-format csv -d gpurun_out/${TAG}_p$i -o run -- python3 bench.py $ARGS > gpurun_out/${TAG}_p$i.log 2>&1
  rc=$?
  echo "rc=$rc"; tail -n 3 gpurun_out/${TAG}_p$i.log
  if [ $rc -eq 124 ] || [ $rc -eq 137 ] || [ $rc -ge 128 ]; then echo "stopping"; exit $rc; fi
done <<GROUPS
FETCH_SIZE
WRITE_SIZE
GRBM_GUI_ACTIVE SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_INSTS_SALU
SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU
SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_VMEM
TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum
TA_BUSY_avr TA_TA_BUSY_sum TD_TD_BUSY_sum
GROUPS
exit 0
