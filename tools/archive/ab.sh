#!/bin/bash
# A/B timing of library builds on one box: tools/ab.sh TAG "VARIANTS" "WORKLOADS"
# (variant 0 = the product libmxd_amd.so; others tools/abl/libmxd_amd_<v>.so),
# each workload's bench run per variant, twice in alternating order.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=$1; VARS=$2; WLS=${3:-c2}
mkdir -p gpurun_out
cp mlx-data_amd/libmxd_amd.so gpurun_out/.product.so
restore() { cp gpurun_out/.product.so mlx-data_amd/libmxd_amd.so; }
for pass in 1 2; do
  for w in $WLS; do
    for v in $VARS; do
      if [ $v = 0 ]; then restore; else cp ${ABL_DIR:-tools/abl}/libmxd_amd_$v.so mlx-data_amd/libmxd_amd.so || exit 1; fi
      timeout -k 10 120 python bench.py --workload $w --no-cpu --no-e2e --no-copy ${BENCH_ARGS:-} > gpurun_out/${TAG}_${w}_${v}_$pass.log 2>&1 || { restore; exit 1; }
      echo "$pass $w $v $(grep -o '"kernel_ms_per_launch": [0-9.]*' gpurun_out/${TAG}_${w}_${v}_$pass.log)"
    done
  done
done
restore
rm -f gpurun_out/.product.so
