set -u
bash tools/r03_pmc.sh r03p || exit 1
for w in c2 c3 c4 c5 c6 c7; do
  bash tools/variants.sh run "--workload $w --reps 5 --set policy=0" product waves8 waves2 noprio > gpurun_out/var_$w.jsonl 2>&1 || { tail gpurun_out/var_$w.jsonl; exit 1; }
  cat gpurun_out/var_$w.jsonl
done
