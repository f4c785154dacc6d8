set -u
bash tools/band_variants.sh run "--workload c2 --reps 3 --set la=2 --set rows=8,la=2 --set rows=12,la=2 --set rows=16,la=2 --set rows=25,la=2" abl12 abl14 product > gpurun_out/r3h_rows_c2.jsonl 2>&1 || exit 1
bash tools/band_stamps.sh run c2:rows=8,la=2 c2:rows=16,la=2 > gpurun_out/r3h_stamps.jsonl 2>&1 || exit 1
