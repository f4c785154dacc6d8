set -u
timeout -k 10 300 python -u -m pytest -x -v --timeout 150 --timeout-method thread tests/test_gpu_surface.py tests/test_gpu_band.py > gpurun_out/r3f_pytest.log 2>&1 || { tail -20 gpurun_out/r3f_pytest.log; exit 1; }
MXD_BENCH_SPLIT_DEVICES=0,0 timeout -k 10 120 python bench.py --split-devices 2 --steps 10 --warmup 2 > gpurun_out/r3f_split_rehearsal.jsonl 2>&1 || exit 1
bash tools/r3e_measure.sh || exit 1
