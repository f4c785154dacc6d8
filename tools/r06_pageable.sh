#!/bin/bash
# the pageable host path (bench.py `e2e`, C2
# host sources -> host f32 batch) against the staging helpers' CPU budget
# (MXD_HOST_CPUS; default = the cgroup quota / affinity), alternating the
# settings over two repetitions on one box.  One process per setting (the
# budget is read once per process).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r06
TAG=${1:-r06e}
O=gpurun_out/r06/${TAG}_pageable.jsonl
: > $O
for rep in 1 2; do
  for cpus in default 1 2 4 8 16 32; do
    if [ $cpus = default ]; then env_cpus=""; else env_cpus="MXD_HOST_CPUS=$cpus"; fi
    line=$(env $env_cpus timeout -k 10 120 python3 bench.py --steps 5 --warmup 2 --no-cpu --no-e2e-jpeg --no-others --no-copy | grep '^{') || exit 1
    python3 -c "import json,sys; d=json.loads(sys.argv[1]); e=d['e2e']; print(json.dumps({'rep': $rep, 'host_cpus': '$cpus', 'pageable': e['value'], 'pinned': e['pinned_value'], 'nproc': $(nproc)}))" "$line" >> $O
  done
done
cat $O
