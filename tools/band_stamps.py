"""Where a band-kernel step spends its cycles (diagnostic; needs the
MXD_BAND_STAMPS build swapped in as mlx-data_amd/libmxd_amd.so,
tools/band_stamps.sh).  Runs one workload back to back on one stream, reads
the last launch's per-unit segment sums (wave 0 of each workgroup, shader
clock cycles) and prints the mean cycles per step of each segment, the setup
cycles, and how unit start/end times spread over the launch.
    python tools/band_stamps.py [c2|c4|c5] [launches] [rows=..,la=..]"""
import ctypes
import json
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "tools"), os.path.join(REPO, "mlx-data_amd")]
import band_sweep  # noqa: E402

w = sys.argv[1] if len(sys.argv) > 1 else "c2"
launches = int(sys.argv[2]) if len(sys.argv) > 2 else 5
kv = dict(p.split("=") for p in (sys.argv[3] if len(sys.argv) > 3 else "").split(",") if p)
capi, L, stream, sets, mode, alg, sizes, geoms, f32 = band_sweep.setup(w)
capi.set_tuning(capi.MXD_TUNE_BAND_ROWS, int(kv.get("rows", 0)))
capi.set_tuning(capi.MXD_TUNE_BAND_LA, int(kv.get("la", 0)))
capi.set_tuning(capi.MXD_TUNE_BAND_GRID, int(kv.get("grid", 0)))
hs = ctypes.c_void_p(stream.handle)
for i in range(launches):
    capi.check(L.mxd_resize_crop_batch(sets[i % 2][2], sets[i % 2][3], mode, 0, hs))
stream.synchronize()
K = 10
n = 8192
buf = (ctypes.c_ulonglong * (K * n))()
L.mxd_debug_band_stamps.argtypes = [ctypes.c_void_p, ctypes.c_int]
assert L.mxd_debug_band_stamps(buf, n) == 0
a = np.frombuffer(buf, dtype=np.uint64).reshape(n, K).astype(np.float64)
a = a[a[:, 7] > 0]
steps = a[:, 7]
names = ["setup", "wait", "barrier1", "hpass", "vpass", "barrier2", "write+issue"]
per = {nm: round(float((a[:, k] / steps).mean()), 1) for k, nm in enumerate(names) if k > 0}
t0 = a[:, 8].min()
start = (a[:, 8] - t0) / 100.0  # us (100 MHz realtime)
end = (a[:, 9] - t0) / 100.0
print(json.dumps({"workload": w, "set": kv, "units": int(len(a)), "steps_per_unit": float(steps.mean()),
                  "cycles_per_step": per, "setup_cycles": round(float(a[:, 0].mean()), 1),
                  "unit_start_us_pct": [round(float(np.percentile(start, q)), 2) for q in (0, 50, 90, 100)],
                  "unit_end_us_pct": [round(float(np.percentile(end, q)), 2) for q in (0, 10, 50, 90, 100)],
                  "unit_us_median": round(float(np.median(end - start)), 2)}), flush=True)
