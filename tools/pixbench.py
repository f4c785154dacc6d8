"""Kernel timing of the pixel-map kernels (csrc/pixmap.hip), SURVEY.md §8f f4.

  gray:   N x 1920x1080 RGB u8 in HBM -> image_channel_reduction("default")
          algorithmic bytes/image = 3*W*H read + W*H written
  rotate: N x 1920x1080 RGB u8 in HBM -> image_rotate(30) (no crop)
          algorithmic bytes/image = source bytes the output samples (<= W*H*3,
          counted as the in-bounds output pixels * 3, each source byte at
          least once) + th*tw*3 written

HIP events around `--iters` back-to-back launches on one stream, inputs
resident.  Prints one JSON line per kernel.   python tools/pixbench.py
"""
import argparse
import json
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "mlx-data_amd"))
from mlx_data_amd import capi  # noqa: E402

HBM_PEAK_GBS = 8000.0


def run(kind, n, iters, w=1920, h=1080, angle=30.0):
    c = 3
    src = capi.DeviceBuffer(w * h * c * n)
    src.upload(np.random.default_rng(0).integers(0, 256, w * h * c * n, dtype=np.uint8))
    if kind == "gray":
        op, params, dw, dh, oc = capi.MXD_CHANNEL_REDUCTION, capi.channel_reduction_preset("default"), w, h, 1
        alg = n * (w * h * 3 + w * h)
    else:
        mx, dw, dh = capi.rotate_geometry(w, h, angle, False)
        op, params, oc = capi.MXD_AFFINE, mx, c
        # source pixels that some output samples: every in-bounds output maps
        # to a distinct-or-repeated source pixel; count the distinct ones
        ty, tx = np.meshgrid(np.arange(dh), np.arange(dw), indexing="ij")
        f = np.float32
        fx, fy = tx.astype(f) - f(dw / 2.0), ty.astype(f) - f(dh / 2.0)
        sx = (mx[0] * fx + mx[1] * fy) + mx[2]
        sy = (mx[3] * fx + mx[4] * fy) + mx[5]
        x = ((sx.astype(np.float64) + 0.5) + np.float64(f(w / 2.0))).astype(np.int64)
        y = ((sy.astype(np.float64) + 0.5) + np.float64(f(h / 2.0))).astype(np.int64)
        ok = (x >= 0) & (y >= 0) & (x < w) & (y < h)
        distinct = np.unique(y[ok] * w + x[ok]).size
        alg = n * (distinct * c + dw * dh * c)
    dst = capi.DeviceBuffer(dw * dh * oc * n)
    entries = [dict(src=src.ptr + i * w * h * c, src_stride=w * c, src_w=w, src_h=h, channels=c, dst_w=dw, dst_h=dh,
                    dst=dst.ptr + i * dw * dh * oc, dst_stride=dw * oc, params=params) for i in range(n)]
    arr, cnt = capi.make_pixmaps(entries)
    s = capi.Stream()
    for _ in range(3):
        capi.pixmap_batch(arr, cnt, op, 0, s.handle)
    e0, e1 = capi.Event(), capi.Event()
    e0.record(s)
    for _ in range(iters):
        capi.pixmap_batch(arr, cnt, op, 0, s.handle)
    e1.record(s)
    e1.synchronize()
    ms = e0.elapsed_ms(e1) / iters
    gbs = alg / (ms * 1e-3) / 1e9
    return {"kernel": kind, "images": n, "frame": f"{w}x{h}x3", "out": f"{dw}x{dh}x{oc}", "ms_per_launch": round(ms, 4),
            "images_per_s": round(n / (ms * 1e-3), 1), "alg_bytes_per_launch": int(alg),
            "achieved_gbs": round(gbs, 1), "frac_of_8TBs": round(gbs / HBM_PEAK_GBS, 4)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--images", type=int, default=64)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--kinds", default="gray,rotate")
    a = ap.parse_args()
    for k in a.kinds.split(","):
        print(json.dumps(run(k, a.images, a.iters)), flush=True)


if __name__ == "__main__":
    main()
