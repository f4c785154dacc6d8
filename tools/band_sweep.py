"""Per-launch time of the fused stage over a grid of tuning settings, in one
process on one box (A/B without box-to-box spread).

  python tools/band_sweep.py [--workload c2] [--launches 20] \
      --set "rows=0,la=0,policy=0" --set "rows=38" ...

Settings are measured round-robin (rep 1 of every setting, then rep 2, ...)
after a --warm-s warm-up, so clock / cache drift does not favour any of them.
Each --set is a comma list of knob=value (rows -> MXD_TUNE_BAND_ROWS, la ->
MXD_TUNE_BAND_LA, grid -> MXD_TUNE_BAND_GRID, desc -> MXD_TUNE_DESC, streams ->
MXD_TUNE_STREAMS, load -> MXD_TUNE_LOAD_POLICY, policy -> mxd_set_kernel_policy).  Inputs are bench.py's
workload (two alternating source/output sets, resident in HBM); the time is
HIP events around `launches` back-to-back launches on one stream, after 3
warm-up launches, repeated `--reps` times (median reported).  Prints one JSON
line per setting."""
import argparse
import ctypes
import json
import os
import statistics
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "mlx-data_amd"))

import numpy as np  # noqa: E402

import bench  # noqa: E402


def setup(workload, nsets=2, c3_sizes=None, batch=0):
    """Two source/output sets of bench.py's workload, resident in HBM.
    Returns (capi, L, stream, sets [(src, dst, imgs, n)], mode, alg_bytes, sizes, geoms, f32)."""
    from mlx_data_amd import capi

    capi.lib()
    dev = 0
    capi.check(capi.lib().mxd_set_device(dev))
    B = batch or bench.WORKLOADS[workload]["batch"]
    sizes, geoms, f32 = bench.make_workload(capi, workload, B, 0, c3_sizes)
    C = bench.C
    elem = 4 if f32 else 1
    offs, pitches, total = [], [], 0
    for (sw, sh) in sizes:
        offs.append(total)
        pitches.append((sw * C + 15) // 16 * 16)
        total += (pitches[-1] * sh + 255) // 256 * 256
    out_bytes = [g[4] * g[5] * C * elem for g in geoms]
    out_offs = np.concatenate([[0], np.cumsum(out_bytes)[:-1]]).astype(np.int64)
    rng = np.random.default_rng(1000)
    host = rng.integers(0, 256, total, dtype=np.uint8)
    stream = capi.Stream(dev)
    sets = []
    for _ in range(nsets):
        src = capi.DeviceBuffer(total, dev)
        dst = capi.DeviceBuffer(int(sum(out_bytes)), dev)
        src.upload(host, stream=stream)
        entries = [dict(src=src.ptr + o, src_stride=pt, src_w=sw, src_h=sh, channels=C, resize_w=g[0], resize_h=g[1],
                        crop_x=g[2], crop_y=g[3], crop_w=g[4], crop_h=g[5], flip=g[6], dst=dst.ptr + int(oo),
                        dst_stride=g[4] * C * elem) for (sw, sh), o, pt, g, oo in zip(sizes, offs, pitches, geoms,
                                                                                     out_offs)]
        imgs, n = capi.make_images(entries)
        sets.append((src, dst, imgs, n))
    mode = capi.MXD_F32_DIV255 if f32 else capi.MXD_U8
    alg = sum(bench.footprint_bytes(capi, sw, sh, C, *g[:6]) for (sw, sh), g in zip(sizes, geoms)) + sum(out_bytes)
    return capi, capi.lib(), stream, sets, mode, alg, sizes, geoms, f32


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", default="c2", choices=sorted(bench.WORKLOADS))
    ap.add_argument("--launches", type=int, default=20)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--set", action="append", default=[])
    ap.add_argument("--warm-s", type=float, default=1.0)
    ap.add_argument("--c3-sizes", default="", help="C3 only: WxH,... pool (default bench.C3_SIZES)")
    ap.add_argument("--batch", type=int, default=0, help="images per launch (default: the workload's)")
    args = ap.parse_args()
    c3 = [tuple(int(v) for v in t.split("x")) for t in args.c3_sizes.split(",") if t] or None
    capi, L, stream, sets, mode, alg, sizes, geoms, f32 = setup(args.workload, c3_sizes=c3, batch=args.batch)
    dev = 0
    hs = ctypes.c_void_p(stream.handle)
    e0, e1 = capi.Event(), capi.Event()
    specs = args.set or ["rows=0"]

    def apply(spec):
        kv = dict(p.split("=") for p in spec.split(",") if p)
        capi.set_tuning(capi.MXD_TUNE_BAND_ROWS, int(kv.get("rows", 0)))
        capi.set_tuning(capi.MXD_TUNE_BAND_LA, int(kv.get("la", 0)))
        capi.set_tuning(capi.MXD_TUNE_BAND_GRID, int(kv.get("grid", 0)))
        capi.set_tuning(capi.MXD_TUNE_DESC, int(kv.get("desc", 0)))
        capi.set_tuning(capi.MXD_TUNE_STREAMS, int(kv.get("streams", 0)))
        capi.set_tuning(capi.MXD_TUNE_LOAD_POLICY, int(kv.get("load", 0)))
        capi.set_kernel_policy(int(kv.get("policy", 0)))
        # wrows: the wave kernels' band height, read from the environment by
        # tuning builds only (-DMXD_TUNING_ENV; tools/variants.sh build tenv)
        if int(kv.get("wrows", 0)) > 0:
            os.environ["MXD_BAND_ROWS"] = kv["wrows"]
        else:
            os.environ.pop("MXD_BAND_ROWS", None)
        return kv

    # Warm-up (clocks, caches, plans of every setting) before any timing;
    # then the reps go round-robin over the settings, so drift during the
    # run spreads over all of them instead of biasing the first.
    for spec in specs:
        apply(spec)
        for i in range(10):
            capi.check(L.mxd_resize_crop_batch(sets[i % 2][2], sets[i % 2][3], mode, dev, hs))
    apply(specs[0])
    stream.synchronize()
    t_end = time.time() + args.warm_s
    while time.time() < t_end:
        for i in range(20):
            capi.check(L.mxd_resize_crop_batch(sets[i % 2][2], sets[i % 2][3], mode, dev, hs))
        stream.synchronize()
    times = {spec: [] for spec in specs}
    for _ in range(args.reps):
        for spec in specs:
            apply(spec)
            for i in range(3):
                capi.check(L.mxd_resize_crop_batch(sets[i % 2][2], sets[i % 2][3], mode, dev, hs))
            stream.synchronize()
            e0.record(stream)
            for i in range(args.launches):
                capi.check(L.mxd_resize_crop_batch(sets[i % 2][2], sets[i % 2][3], mode, dev, hs))
            e1.record(stream)
            stream.synchronize()
            times[spec].append(e0.elapsed_ms(e1) / args.launches)
    for spec in specs:
        kv = apply(spec)
        ms = statistics.median(times[spec])
        print(json.dumps({"workload": args.workload, "set": spec, "ms_per_launch": round(ms, 5),
                          "frac": round(alg / (ms * 1e-3) / 8e12, 4), "reps": [round(t, 5) for t in times[spec]],
                          "kernel": bench.kernel_name(capi, sizes[0], geoms[0], f32, int(kv.get("policy", 0)))}),
              flush=True)
    capi.set_tuning(capi.MXD_TUNE_BAND_ROWS, 0)
    capi.set_tuning(capi.MXD_TUNE_BAND_LA, 0)
    capi.set_tuning(capi.MXD_TUNE_BAND_GRID, 0)
    capi.set_kernel_policy(0)


if __name__ == "__main__":
    main()
