#!/bin/bash
# Round 3: the wave kernels' 24 / 32-tap scatter buckets (12 / 24 MP photos)
# -- parity, then per-launch A/B against the band kernel and the narrow lane
# width (profiles/r03/wave_large_<w>.jsonl), then the descriptor upload modes
# (MXD_TUNE_DESC 1..4) on C2 / C4 (profiles/r03/desc_modes.jsonl).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_vfirst.py tests/test_gpu_band.py tests/test_gpu_parity.py -x -q --timeout 150 --timeout-method thread > gpurun_out/wl_pytest.log 2>&1 || { tail -30 gpurun_out/wl_pytest.log; exit 1; }
tail -2 gpurun_out/wl_pytest.log
S="timeout -k 10 200 python tools/band_sweep.py --reps 5"
for w in c6 c7; do $S --workload $w --set policy=0 --set policy=4 --set policy=256 > gpurun_out/wl_$w.jsonl 2>&1 || { tail gpurun_out/wl_$w.jsonl; exit 1; }; cat gpurun_out/wl_$w.jsonl; done
for w in c2 c3 c4 c5; do $S --workload $w --set policy=0 > gpurun_out/wl_$w.jsonl 2>&1 || exit 1; cat gpurun_out/wl_$w.jsonl; done
for w in c2 c4; do for m in 1 2 3 4; do
  timeout -k 10 120 python bench.py --workload $w --no-cpu --no-e2e --tune-desc $m > gpurun_out/desc_${w}_$m.log 2>&1 || exit 1
  tail -1 gpurun_out/desc_${w}_$m.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print(json.dumps(dict(workload='$w', desc_mode=$m, ms_per_launch=r['kernel_ms_per_launch'], fresh=r['ms_per_launch_fresh_descriptors'], ms_per_step=d['ms_per_step'])))"
done; done
