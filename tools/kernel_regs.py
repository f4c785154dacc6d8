"""tools/kernel_regs.py [LIB] [--match REGEX] -- VGPR / AGPR / SGPR / spill
counts of every kernel in a built library's gfx950 code objects (default:
the in-tree libmxd_amd.so, kernels matching resample_wave).  A linked
library's .hip_fatbin holds one offload bundle per object file: each is split
out and unbundled, and its code object's metadata notes are read."""
import argparse
import os
import re
import struct
import subprocess
import tempfile

LLVM = "/opt/rocm/lib/llvm/bin"
MAGIC = b"__CLANG_OFFLOAD_BUNDLE__"


def code_objects(lib, tmp):
    fat = os.path.join(tmp, "fat.bin")
    subprocess.run([f"{LLVM}/llvm-objcopy", f"--dump-section=.hip_fatbin={fat}", lib], check=True)
    data = open(fat, "rb").read()
    pos = data.find(MAGIC)
    while pos >= 0:
        n = struct.unpack_from("<Q", data, pos + len(MAGIC))[0]
        off = pos + len(MAGIC) + 8
        end = pos
        for _ in range(n):
            o, size, tlen = struct.unpack_from("<QQQ", data, off)
            triple = data[off + 24 : off + 24 + tlen].decode()
            off += 24 + tlen
            end = max(end, pos + o + size)
            if "gfx950" in triple:
                yield data[pos + o : pos + o + size]
        pos = data.find(MAGIC, max(end, pos + 1))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("lib", nargs="?", default=os.path.join(os.path.dirname(__file__), "..", "mlx-data_amd", "libmxd_amd.so"))
    ap.add_argument("--match", default="resample_wave")
    args = ap.parse_args()
    rx = re.compile(args.match)
    with tempfile.TemporaryDirectory() as tmp:
        for i, co in enumerate(code_objects(args.lib, tmp)):
            path = os.path.join(tmp, f"k{i}.co")
            open(path, "wb").write(co)
            notes = subprocess.run([f"{LLVM}/llvm-readelf", "--notes", path], capture_output=True, text=True).stdout
            cur = None
            for line in notes.splitlines():
                m = re.match(r"\s+\.(name|vgpr_count|sgpr_count|vgpr_spill_count|sgpr_spill_count|agpr_count):\s+(\S+)", line)
                if not m:
                    continue
                k, v = m.groups()
                if k == "name":
                    if cur and rx.search(cur["name"]):
                        print(cur)
                    cur = {"name": v}
                elif cur is not None:
                    cur[k] = int(v)
            if cur and rx.search(cur["name"]):
                print(cur)


if __name__ == "__main__":
    main()
