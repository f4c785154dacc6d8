#!/bin/bash
# Host-path staging on persistent helper threads (product) against threads
# spawned per chunk (variant -DMXD_HOST_HELPERS=0): bench.py e2e (pageable and
# page-locked host batches) on C2 / C4, alternating, two rounds; host-path
# GPU tests first (profiles/r03/host_helpers.jsonl).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_host_path.py tests/test_gpu_jpeg.py tests/test_gpu_surface.py tests/test_gpu_pipeline.py -x -q --timeout 150 --timeout-method thread > gpurun_out/hh.log 2>&1 || { tail -5 gpurun_out/hh.log; exit 1; }
tail -1 gpurun_out/hh.log
cp mlx-data_amd/libmxd_amd.so gpurun_out/.product.so
for rep in 1 2; do for v in product spawn; do for w in c2 c4; do
  if [ $v = product ]; then cp gpurun_out/.product.so mlx-data_amd/libmxd_amd.so; else cp tools/libmxd_amd_var_spawn.so mlx-data_amd/libmxd_amd.so; fi
  timeout -k 10 120 python bench.py --workload $w --no-cpu --no-copy --steps 20 > gpurun_out/hh_b.log 2>&1 || { cp gpurun_out/.product.so mlx-data_amd/libmxd_amd.so; exit 1; }
  tail -1 gpurun_out/hh_b.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); e=d['e2e']; print(json.dumps(dict(variant='$v', workload='$w', rep=$rep, pageable=e['value'], pinned=e['pinned_value'], calls=e['steps'])))"
done; done; done
cp gpurun_out/.product.so mlx-data_amd/libmxd_amd.so
