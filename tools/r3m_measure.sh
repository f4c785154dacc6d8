set -u
mkdir -p gpurun_out
S="timeout -k 10 200 python tools/band_sweep.py --reps 5"
$S --workload c2 --set policy=0 --set policy=256 --set policy=256,grid=1 --set policy=256,rows=8 --set policy=256,rows=8,grid=1 > gpurun_out/r3m_c2.jsonl 2>&1 || exit 1
for w in c3 c4 c5; do $S --workload $w --set policy=0 --set policy=256 --set policy=256,grid=1 > gpurun_out/r3m_$w.jsonl 2>&1 || exit 1; done
for w in c6 c7; do $S --workload $w --set rows=0 --set grid=1 --set la=3 --set rows=8 --set rows=24 > gpurun_out/r3m_$w.jsonl 2>&1 || exit 1; done
