"""Per-unit start/end stamps of the wave kernel (diagnostic; needs the
MXD_STAMPS build swapped in as mlx-data_amd/libmxd_amd.so, tools/stamps.sh).
Runs one workload's batch back to back on one stream, reads the last launch's
stamps and prints how the launch fills and drains: unit start / end
percentiles relative to the first start, and the count of running units over
time (the HBM-bound kernel needs most of its waves resident to keep HBM busy).
    python tools/stamps.py [c2|c4|c5] [launches]"""
import ctypes
import json
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "mlx-data_amd")]
import bench  # noqa: E402
from mlx_data_amd import capi  # noqa: E402

w = sys.argv[1] if len(sys.argv) > 1 else "c2"
launches = int(sys.argv[2]) if len(sys.argv) > 2 else 5
L = capi.lib()
B = bench.WORKLOADS[w]["batch"]
sizes, geoms, f32 = bench.make_workload(capi, w, B, 0)
elem = 4 if f32 else 1
offs, pitches, total = [], [], 0
for (sw, sh) in sizes:
    offs.append(total)
    pitches.append((sw * 3 + 15) // 16 * 16)
    total += (pitches[-1] * sh + 255) // 256 * 256
out_bytes = [g[4] * g[5] * 3 * elem for g in geoms]
src = capi.DeviceBuffer(total, 0)
dst = capi.DeviceBuffer(int(sum(out_bytes)), 0)
src.upload(np.random.default_rng(0).integers(0, 256, total, dtype=np.uint8))
oo = np.concatenate([[0], np.cumsum(out_bytes)[:-1]]).astype(np.int64)
entries = [dict(src=src.ptr + o, src_stride=pt, src_w=sw, src_h=sh, channels=3, resize_w=g[0], resize_h=g[1],
                crop_x=g[2], crop_y=g[3], crop_w=g[4], crop_h=g[5], flip=g[6], dst=dst.ptr + int(d),
                dst_stride=g[4] * 3 * elem) for (sw, sh), o, pt, g, d in zip(sizes, offs, pitches, geoms, oo)]
imgs, n = capi.make_images(entries)
stream = capi.Stream(0)
for _ in range(launches):
    capi.check(L.mxd_resize_crop_batch(imgs, n, capi.MXD_F32_DIV255 if f32 else capi.MXD_U8, 0,
                                       ctypes.c_void_p(stream.handle)))
stream.synchronize()
N = 32768
buf = (ctypes.c_ulonglong * (2 * N))()
assert L.mxd_debug_stamps(buf, N) == 0
a = np.frombuffer(buf, np.uint64).reshape(N, 2).astype(np.int64)
a = a[a[:, 0] > 0]
t0 = a[:, 0].min()
st, en = (a[:, 0] - t0) / 100.0, (a[:, 1] - t0) / 100.0  # us (100 MHz)
dur = en - st
span = en.max()
grid = np.arange(0, span + 1, 1.0)
running = [(int(((st <= t) & (en > t)).sum())) for t in grid]
peak = max(running)
res = {
    "workload": w, "units": int(len(a)), "span_us": round(float(span), 2),
    "start_us_pct": {p: round(float(np.percentile(st, p)), 2) for p in (0, 50, 90, 99, 100)},
    "end_us_pct": {p: round(float(np.percentile(en, p)), 2) for p in (0, 1, 10, 50, 90, 99, 100)},
    "unit_us_pct": {p: round(float(np.percentile(dur, p)), 2) for p in (0, 10, 50, 90, 100)},
    "peak_running": peak,
    "us_below_90pct_of_peak_at_end": round(float(span - max(t for t, r in zip(grid, running) if r >= 0.9 * peak)), 2),
    "us_below_50pct_of_peak_at_end": round(float(span - max(t for t, r in zip(grid, running) if r >= 0.5 * peak)), 2),
    "running_every_5us": running[::5],
}
# units are laid out XCD by XCD (wave.hip xcd_remap, kWaves = 8 waves per
# workgroup): unit u ran on XCD (u // 8) // ceil(blocks / 8) (blocks =
# ceil(units / 8)), roughly
WAVES = 8
nb = (len(a) + WAVES - 1) // WAVES
q = (nb + 7) // 8
ids = np.nonzero(np.frombuffer(buf, np.uint64).reshape(N, 2)[:, 0] > 0)[0]
xcd = np.minimum((ids // WAVES) // q, 7) if os.environ.get("NO_XCD_REMAP") is None else (ids // WAVES) % 8
img = ids // max(1, len(a) // bench.WORKLOADS[w]["batch"])
res["image_octile_unit_us_median"] = [round(float(np.median(dur[(img * 8 // bench.WORKLOADS[w]["batch"]) == k])), 1)
                                      for k in range(8)]
res["xcd_unit_us_median"] = [round(float(np.median(dur[xcd == x])), 1) for x in range(8)]
res["xcd_end_us_max"] = [round(float(en[xcd == x].max()), 1) for x in range(8)]
res["wave_in_block_median"] = [round(float(np.median(dur[ids % WAVES == k])), 1) for k in range(WAVES)]
# within one XCD: block order (dispatch order) vs duration
x0 = ids[xcd == 0]
res["xcd0_first_vs_last_blocks_us"] = [round(float(np.median(dur[(xcd == 0) & (ids < x0.min() + 128)])), 1),
                                       round(float(np.median(dur[(xcd == 0) & (ids >= x0.max() - 128)])), 1)]
print(json.dumps(res))
