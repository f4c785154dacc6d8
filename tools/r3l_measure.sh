set -u
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -q --timeout 150 --timeout-method thread -m gpu tests > gpurun_out/r3l_pytest.log 2>&1 || { tail -40 gpurun_out/r3l_pytest.log; exit 1; }
tail -3 gpurun_out/r3l_pytest.log
for w in c6 c7; do
  timeout -k 10 200 python tools/band_sweep.py --workload $w --reps 3 --set rows=0 --set rows=8 --set rows=32 --set grid=1 --set la=3 > gpurun_out/r3l_sweep_$w.jsonl 2>&1 || exit 1
done
