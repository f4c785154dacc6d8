"""Can the host write device memory directly (large BAR), and how fast?
Allocates 64 KB of device memory per flag (hipExtMallocWithFlags: 0 default,
1 fine-grained, 3 uncached), then in a child process (a failed access must
not take this one down) memmoves 13 KB into it from the CPU and reads it back
with hipMemcpy.  Prints one JSON line per flag: ok, us per 13 KB write.
python tools/bar_probe.py"""
import ctypes
import json
import os
import subprocess
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "mlx-data_amd"))

if len(sys.argv) > 1:  # child: flag
    from mlx_data_amd import capi
    capi.lib()
    hip = ctypes.CDLL("libamdhip64.so")
    flag = int(sys.argv[1])
    p = ctypes.c_void_p()
    assert hip.hipSetDevice(0) == 0
    rc = hip.hipExtMallocWithFlags(ctypes.byref(p), ctypes.c_size_t(65536), ctypes.c_uint(flag))
    if rc != 0:
        print(json.dumps({"flag": flag, "alloc_rc": rc}))
        sys.exit(0)
    n = 13312
    src = (ctypes.c_uint8 * n)(*[(i * 7) & 255 for i in range(n)])
    t0 = time.perf_counter()
    for _ in range(1000):
        ctypes.memmove(p, src, n)
    dt = (time.perf_counter() - t0) / 1000 * 1e6
    back = (ctypes.c_uint8 * n)()
    assert hip.hipDeviceSynchronize() == 0
    assert hip.hipMemcpy(back, p, ctypes.c_size_t(n), 2) == 0  # D2H
    print(json.dumps({"flag": flag, "ok": bytes(back) == bytes(src), "us_per_13KB_write": round(dt, 2)}))
    sys.exit(0)

for flag in (0, 1, 3):
    r = subprocess.run([sys.executable, __file__, str(flag)], capture_output=True, text=True, timeout=120)
    out = r.stdout.strip().splitlines()
    print(out[-1] if out and r.returncode == 0 else json.dumps({"flag": flag, "child_rc": r.returncode,
                                                                  "err": r.stderr.strip()[-200:]}))
