set -u
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_band.py tests/test_gpu_vfirst.py > gpurun_out/r3j_pytest.log 2>&1 || { tail -30 gpurun_out/r3j_pytest.log; exit 1; }
tail -3 gpurun_out/r3j_pytest.log
for w in c2 c4 c3 c5; do
  timeout -k 10 200 python tools/band_sweep.py --workload $w --reps 3 --set rows=0 --set policy=128 --set rows=8 --set rows=4 > gpurun_out/r3j_sweep_$w.jsonl 2>&1 || exit 1
done
