#!/bin/bash
# Parity tests, then kernel timing with and without the scatter kernel.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
TAG=${1:-q}
timeout -k 10 600 python -m pytest tests -x -q -m gpu > gpurun_out/${TAG}_pytest.log 2>&1
rc=$?; tail -3 gpurun_out/${TAG}_pytest.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
for e in 0 1; do
  MXD_NO_RING=$e timeout -k 10 300 python bench.py --steps 30 --no-cpu --no-e2e > gpurun_out/${TAG}_bench_ns$e.log 2>&1 || exit $?
  echo "no_ring=$e $(grep -o '"kernel_ms_per_launch": [0-9.]*' gpurun_out/${TAG}_bench_ns$e.log)"
done
