set -u
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_band.py tests/test_gpu_vfirst.py > gpurun_out/r3k_pytest.log 2>&1 || { tail -30 gpurun_out/r3k_pytest.log; exit 1; }
tail -3 gpurun_out/r3k_pytest.log
for w in c2 c4; do
  timeout -k 10 200 python tools/band_sweep.py --workload $w --reps 3 --set rows=0 --set grid=1 --set rows=8 --set rows=8,grid=1 --set rows=16 --set policy=128 > gpurun_out/r3k_sweep_$w.jsonl 2>&1 || exit 1
done
for w in c6 c7; do
  timeout -k 10 200 python tools/band_sweep.py --workload $w --reps 3 --set rows=0 --set grid=1 --set policy=2 > gpurun_out/r3k_sweep_$w.jsonl 2>&1 || exit 1
done
bash tools/band_stamps.sh run c2:grid=1 c2 > gpurun_out/r3k_stamps.jsonl 2>&1
