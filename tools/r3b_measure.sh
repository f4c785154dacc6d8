set -u
export TMPDIR=/tmp
timeout -k 10 300 python tools/band_sweep.py --workload c2 --set "rows=0" --set "policy=128" --set "rows=38" --set "rows=25" --set "rows=19" --set "rows=150" --set "la=1" --set "la=2" --set "la=4" --set "la=5" --set "rows=38,la=2" --set "rows=38,la=5" > gpurun_out/r3b_sweep_c2.jsonl 2>&1 || exit 1
timeout -k 10 200 python tools/band_sweep.py --workload c4 --set "rows=0" --set "policy=128" --set "rows=14" --set "rows=56" --set "la=4" --set "la=12" > gpurun_out/r3b_sweep_c4.jsonl 2>&1 || exit 1
bash tools/pmc_run.sh r3b_c2pmc "--steps 10 --warmup 2" "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR GRBM_GUI_ACTIVE" "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT" "FETCH_SIZE" "WRITE_SIZE" || exit 1
