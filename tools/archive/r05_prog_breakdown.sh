#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python3 tools/prog_breakdown.py > gpurun_out/${1:-r05pb}.log 2>&1; rc=$?
cat gpurun_out/${1:-r05pb}.log | tail -8
exit $rc
