set -u
bash tools/band_variants.sh run "--workload c2 --reps 3 --set la=1 --set la=2 --set la=3 --set la=5 --set policy=128" abl14 abl12 abl6 nt0 product > gpurun_out/r3g_ablate_c2.jsonl 2>&1 || exit 1
