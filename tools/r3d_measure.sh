set -u
bash tools/band_variants.sh run "--workload c2 --set rows=0 --set rows=25 --set la=2 --set rows=25,la=2 --set rows=38,la=2 --set policy=128" product noprio branchy > gpurun_out/r3d_variants_c2.jsonl 2>&1 || exit 1
timeout -k 10 200 python tools/band_sweep.py --workload c4 --set rows=0 --set policy=128 --set la=4 --set rows=14 > gpurun_out/r3d_sweep_c4.jsonl 2>&1 || exit 1
