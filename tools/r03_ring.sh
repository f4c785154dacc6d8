set -u
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
for w in c2 c3 c4 c5 c6 c7; do
  bash tools/variants.sh run "--workload $w --reps 5 --set policy=0" product ring4 ring3 > gpurun_out/ring_$w.jsonl 2>&1 || { tail gpurun_out/ring_$w.jsonl; exit 1; }
  cat gpurun_out/ring_$w.jsonl
done
for w in c2 c4; do
  timeout -k 10 120 python bench.py --workload $w --no-cpu --no-e2e > gpurun_out/host_$w.log 2>&1 || exit 1
  tail -1 gpurun_out/host_$w.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print(json.dumps(dict(w='$w', k=r['kernel_ms_per_launch'], fresh=r['ms_per_launch_fresh_descriptors'], host=r['host_ms_per_call'], host_fresh=r['host_ms_per_call_fresh'])))"
done
