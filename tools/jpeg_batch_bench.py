"""JPEG batch decode + resize through the C ABI, device entropy decode vs host
entropy decode (diagnostic).

For C4's file shapes (500x375 / 375x500 / 500x333, seed 2, Pillow q=90, like
bench.py's c4 workload) and C1's (300x200): the host time per image of
mxd_jpeg_coefs_parse (markers only: the device decodes the Huffman data) and
of mxd_jpeg_coefs_decode (the host entropy decode), then the wall time per
call of mxd_jpeg_resize_crop_to_device over a batch of each kind (decode
finish + resize 256 + center crop 224 + f32, results in HBM), over >= 2 s.
Prints one JSON line per dataset."""
import argparse
import ctypes
import io
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "mlx-data_amd"))

SIZES = {"c4": [(500, 375), (375, 500), (500, 333)], "c1": [(300, 200), (200, 300)],
         # round 5: a 12 MP photo without restart markers,
         # whose one segment the device decode spreads over many jobs
         "l12": [(4032, 3024)]}


def files(name, n):
    from PIL import Image

    rng = np.random.default_rng(2)
    out = []
    for i in range(n):
        w, h = SIZES[name][int(rng.integers(0, len(SIZES[name])))]
        gh, gw = h // 24 + 2, w // 24 + 2
        grid = rng.integers(0, 256, (gh, gw, 3)).astype(np.float32)
        yi = np.minimum(np.arange(h) * (gh - 1) // max(1, h - 1), gh - 2)
        xi = np.minimum(np.arange(w) * (gw - 1) // max(1, w - 1), gw - 2)
        f = grid[yi][:, xi] * 0.6 + grid[yi + 1][:, xi + 1] * 0.4 + rng.normal(0, 12, (h, w, 3))
        b = io.BytesIO()
        Image.fromarray(np.clip(f, 0, 255).astype(np.uint8)).save(b, "JPEG", quality=90)
        out.append(b.getvalue())
    return out


def per_image(fn, datas, min_s=1.0):
    k, t0 = 0, time.perf_counter()
    while k < len(datas) or time.perf_counter() - t0 < min_s:
        fn(datas[k % len(datas)])
        k += 1
    return (time.perf_counter() - t0) / k * 1e6


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=128)
    ap.add_argument("--datasets", default="c4,c1")
    ap.add_argument("--huff-bits", default="0", help="device entropy: subsequence lengths to time (0: default)")
    ap.add_argument("--huff-global", action="store_true", help="device entropy: also time every length with words read from device memory")
    ap.add_argument("--no-host", action="store_true", help="skip the host entropy decode runs")
    ap.add_argument("--huff-job", default="0", help="device entropy: own subsequences per job to time (0: default)")
    ap.add_argument("--seconds", type=float, default=2.0, help="timed loop length per run")
    ap.add_argument("--jpeg-rgb", type=int, default=0, help="MXD_TUNE_JPEG_RGB: 1 = always through an RGB frame")
    args = ap.parse_args()
    from mlx_data_amd import capi

    L = capi.lib()
    capi.check(L.mxd_set_device(0))
    capi.set_tuning(capi.MXD_TUNE_JPEG_RGB, args.jpeg_rgb)
    for spec in args.datasets.split(","):
        name, _, nb = spec.partition(":")  # "l12:4": a dataset's own batch size
        batch = int(nb) if nb else args.batch
        datas = files(name, batch)
        line = dict(dataset=name, batch=batch, mean_file_bytes=round(float(np.mean([len(d) for d in datas])), 1))
        runs = [(True, int(b), 0, int(j)) for b in args.huff_bits.split(",") for j in args.huff_job.split(",")]
        if args.huff_global:
            runs += [(True, int(b), 1, 0) for b in args.huff_bits.split(",")]
        if not args.no_host:
            runs.append((False, 0, 0, 0))
        for dev, bits, glob, job in runs:
            capi.set_tuning(capi.MXD_TUNE_HUFF_BITS, bits)
            capi.set_tuning(capi.MXD_TUNE_HUFF_GLOBAL, glob)
            capi.set_tuning(capi.MXD_TUNE_HUFF_JOB, job)
            tag = ("device_entropy" + (f"_bits{bits}" if bits else "") + ("_global" if glob else "") +
                   (f"_job{job}" if job else "")) if dev else "host_entropy"
            line[f"{tag}_host_us_per_image"] = round(per_image(lambda d: capi.JpegCoefs(d, dev).close(), datas), 1)
            coefs = [capi.JpegCoefs(d, dev) for d in datas]
            assert all(c.entropy_pending == dev for c in coefs)
            dst = capi.DeviceBuffer(batch * 224 * 224 * 12, 0)
            entries = []
            for i, c in enumerate(coefs):
                rw, rh = capi.resize_smallest_side_dims(c.width, c.height, 256)
                cx, cy = capi.center_crop_origin(rw, rh, 224, 224)
                entries.append(dict(coefs=c, win_x=0, win_y=0, win_w=c.width, win_h=c.height, resize_w=rw,
                                    resize_h=rh, crop_x=cx, crop_y=cy, crop_w=224, crop_h=224, flip=0,
                                    dst=dst.ptr + i * 224 * 224 * 12, dst_stride=224 * 12))
            arr, n = capi.make_jpeg_images(entries)
            for _ in range(3):
                capi.jpeg_resize_crop_to_device(arr, n, capi.MXD_F32_DIV255, 0)
            k, t0 = 0, time.perf_counter()
            while time.perf_counter() - t0 < args.seconds:
                capi.jpeg_resize_crop_to_device(arr, n, capi.MXD_F32_DIV255, 0)
                k += 1
            ms = (time.perf_counter() - t0) / k * 1e3
            line[f"{tag}_ms_per_batch_call"] = round(ms, 4)
            line[f"{tag}_images_per_s_per_call"] = round(batch / ms * 1e3, 1)
            dst.free()
            for c in coefs:
                c.close()
        capi.set_tuning(capi.MXD_TUNE_HUFF_BITS, 0)
        capi.set_tuning(capi.MXD_TUNE_HUFF_GLOBAL, 0)
        capi.set_tuning(capi.MXD_TUNE_HUFF_JOB, 0)
        print(json.dumps(line), flush=True)


if __name__ == "__main__":
    main()
