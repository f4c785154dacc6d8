#!/bin/bash
# HBM bytes per kernel of the C4 JPEG call (128 files), with the fused plane
# source (MXD_TUNE_JPEG_RGB 0) and through the RGB frame (1): one rocprofv3
# --pmc pass per counter and mode (FETCH_SIZE and WRITE_SIZE cannot share a
# pass), summarised by tools/pmc_kernels.py.
#   tools/r05_pmc_jpeg.sh TAG
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-r05p}
for rgb in 0 1; do
  for ctr in FETCH_SIZE WRITE_SIZE; do
    d=gpurun_out/${TAG}_rgb${rgb}_${ctr}
    timeout -s KILL 120 rocprofv3 --pmc $ctr --output-format csv -d $d -o run -- python3 tools/jpeg_batch_bench.py \
      --datasets c4 --no-host --seconds 0.3 --jpeg-rgb $rgb > $d.log 2>&1
    rc=$?
    echo "rgb=$rgb $ctr rc=$rc"
    if [ $rc -ne 0 ]; then echo "stopping"; exit $rc; fi
    python3 tools/pmc_kernels.py $d/run_counter_collection.csv | tee $d.txt
  done
done
exit 0
