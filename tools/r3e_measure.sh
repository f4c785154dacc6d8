set -u
bash tools/band_variants.sh run "--workload c2 --reps 3 --set rows=0 --set la=2 --set policy=128" product abl1 abl2 abl3 abl12 abl13 noprio product > gpurun_out/r3e_ablate_c2.jsonl 2>&1 || exit 1
