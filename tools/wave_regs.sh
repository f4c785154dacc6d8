#!/bin/bash
# tools/wave_regs.sh [extra hipcc flags] -- compiles wave.hip with only C2's
# scatter kernels (-DMXD_ONLY_C2) and prints each kernel's VGPR / SGPR /
# spill counts (a register-pressure check in seconds instead of the full
# build's minutes; diagnostic, never the product library).
set -e
cd "$(dirname "$0")/../mlx-data_amd"
out=$(mktemp -d)
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC -I../include -Icsrc --offload-arch=gfx950 -ffp-contract=fast \
  -DMXD_ONLY_C2 "$@" --offload-device-only -S csrc/wave.hip -o "$out/w.s"
# C2's product kernel: resample_wave<3, 8, f32, 8, 2, scatter, 2, 4, no shift, RGB, nt>
grep -E "^\s+\.name:\s+_Z.*resample_wave|^\s+\.(vgpr_count|sgpr_count|vgpr_spill_count|sgpr_spill_count):" "$out/w.s" |
  grep -A4 "resample_waveILi3ELi8ELb1ELi8ELi2ELi2ELi2ELi4ELb0ELb0ELi2E"
rm -rf "$out"
