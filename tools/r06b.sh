#!/bin/bash
# Round 6 session b: (1) per-shape cache-policy A/B of the wave kernels
# (product / nt loads / nt loads + nt-sc1 f32 stores / nt-sc1 stores / nt
# loads + nt buffer stores) on every single-shape workload; (2) the JPEG
# entropy-decode change (per-block zeroing in the write pass) against the
# round-5 kernel (variant oldhuff): JPEG GPU tests, call time and rocprof
# kernel stats, PMC FETCH_SIZE / WRITE_SIZE per kernel.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${1:-r06b}
O=gpurun_out/r06/$TAG
mkdir -p gpurun_out/r06
WL=c2,c3:640x480,c3:1280x720,c3:1280x960,c3:1920x1080,c3:2560x1440,c3:3840x2160,c3,c4,c5,c6,c7
timeout -k 10 900 python -u tools/lib_ab.py --workloads $WL --variants product,ntl,nts,sts,ntsn,bperm --reps 5 > ${O}_lib_ab.jsonl || exit 1
timeout -k 10 300 python -u -m pytest tests/test_gpu_jpeg_entropy.py tests/test_gpu_c4_full.py tests/test_gpu_jpeg.py -x -q --timeout 120 --timeout-method thread > ${O}_pytest_jpeg.txt 2>&1 || exit 1
cp mlx-data_amd/libmxd_amd.so gpurun_out/.product.so
rc=0
for v in product oldhuff; do
  if [ $v = product ]; then cp gpurun_out/.product.so mlx-data_amd/libmxd_amd.so; else cp tools/libmxd_amd_var_$v.so mlx-data_amd/libmxd_amd.so; fi
  timeout -k 10 120 python3 tools/jpeg_batch_bench.py --datasets c4 --no-host --seconds 2 > ${O}_${v}_jpeg_batch.jsonl 2>&1 || { rc=1; break; }
  timeout -k 10 120 rocprofv3 --kernel-trace --stats -d ${O}_${v}_trace -o run -- python3 tools/jpeg_batch_bench.py --datasets c4 --no-host --seconds 0.5 > ${O}_${v}_trace.log 2>&1 || { rc=1; break; }
  for ctr in FETCH_SIZE WRITE_SIZE; do
    d=${O}_${v}_${ctr}
    timeout -s KILL 120 rocprofv3 --pmc $ctr --output-format csv -d $d -o run -- python3 tools/jpeg_batch_bench.py \
      --datasets c4 --no-host --seconds 0.3 > $d.log 2>&1 || { rc=1; break 2; }
    python3 tools/pmc_kernels.py $d > $d.txt
  done
done
cp gpurun_out/.product.so mlx-data_amd/libmxd_amd.so
rm -f gpurun_out/.product.so
exit $rc
