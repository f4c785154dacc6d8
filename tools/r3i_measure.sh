set -u
bash tools/band_variants.sh run "--workload c2 --reps 3 --set la=2 --set rows=16,la=2 --set rows=8,la=2" ntload ntload12 product > gpurun_out/r3i_ntload_c2.jsonl 2>&1 || exit 1
for w in c3 c4 c5; do
  timeout -k 10 200 python tools/band_sweep.py --workload $w --reps 3 --set rows=0 --set policy=128 --set rows=16 --set la=2 --set rows=16,la=2 > gpurun_out/r3i_sweep_$w.jsonl 2>&1 || exit 1
done
