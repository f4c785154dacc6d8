#!/bin/bash
# Compile-time variants of the fused stage against the product build, timed in
# one process per variant on one box (tools/band_sweep.py per variant).
#   tools/variants.sh build NAME "FLAGS" [SRC...]   (here; SRC default: wave plan
#        -- the kernel and the host schedule builder, which share resample.h's
#        ring geometry) -> tools/libmxd_amd_var_NAME.so
#   tools/variants.sh run "SWEEP ARGS" NAME...      (GPU box; "product" = the in-tree build)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
if [ "$1" = build ]; then
  NAME=$2 FLAGS=$3
  shift 3
  SRCS=${*:-wave plan}
  cd mlx-data_amd
  mkdir -p build/var_$NAME
  OBJS=""
  for o in resample wave band band_plan pixmap capi plan batch hostpath taps jpeg jpegdev jpeghuff; do
    if [[ " $SRCS " == *" $o "* ]]; then
      src=csrc/$o.hip; [ -f $src ] || src=csrc/$o.cpp
      if [ $o = jpeg ] || [ $o = band_plan ]; then  # host-only C++ (the Makefile's g++ rule)
        g++ -O3 -std=c++17 -fPIC -Wall -I../include -Icsrc $FLAGS -c $src -o build/var_$NAME/$o.o || exit 1
      else
        /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC -Wall -I../include -Icsrc --offload-arch=gfx950 -ffp-contract=fast \
          $FLAGS -c $src -o build/var_$NAME/$o.o || exit 1
      fi
      OBJS="$OBJS build/var_$NAME/$o.o"
    else
      OBJS="$OBJS build/$o.o"
    fi
  done
  /opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 $OBJS -o ../tools/libmxd_amd_var_$NAME.so || exit 1
  exit 0
fi
ARGS=$2; shift 2
mkdir -p gpurun_out
cp mlx-data_amd/libmxd_amd.so gpurun_out/.product.so
rc=0
for v in "$@"; do
  if [ $v = product ]; then cp gpurun_out/.product.so mlx-data_amd/libmxd_amd.so; else cp tools/libmxd_amd_var_$v.so mlx-data_amd/libmxd_amd.so; fi
  timeout -k 10 200 python tools/band_sweep.py $ARGS | sed "s/^/{\"variant\": \"$v\", \"r\": /; s/$/}/" || { rc=1; break; }
done
cp gpurun_out/.product.so mlx-data_amd/libmxd_amd.so
rm -f gpurun_out/.product.so
exit $rc
