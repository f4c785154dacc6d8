#!/bin/bash
# VGPR / SGPR / spill counts of the gfx950 kernels in a host object built by
# hipcc (tools/kernel_regs.sh mlx-data_amd/build/wave.o [name-filter]).
set -e
OBJ=$1; PAT=${2:-.}
T=$(mktemp -d)
/opt/rocm/lib/llvm/bin/llvm-objcopy --dump-section .hip_fatbin=$T/fb.bin "$OBJ"
/opt/rocm/lib/llvm/bin/clang-offload-bundler --type=o --targets=hipv4-amdgcn-amd-amdhsa--gfx950 --input=$T/fb.bin --output=$T/k.hsaco --unbundle
/opt/rocm/lib/llvm/bin/llvm-readelf --notes $T/k.hsaco | python3 -c '
import re, sys
pat = sys.argv[1]
cur = {}
rows = []
for ln in sys.stdin:
    m = re.match(r"\s*-?\s*\.(\w+):\s+(\S+)", ln)
    if not m: continue
    k, v = m.groups()
    if k == "agpr_count" and cur: rows.append(cur); cur = {}
    cur[k] = v
if cur: rows.append(cur)
for r in rows:
    n = r.get("name", "?")
    if re.search(pat, n): print(r.get("vgpr_count"), r.get("agpr_count", "0"), r.get("sgpr_count"), r.get("vgpr_spill_count"), r.get("group_segment_fixed_size"), n)
' "$PAT"
rm -rf $T
