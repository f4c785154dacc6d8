"""Helpers for the GPU parity tests: run the fused kernel through the C ABI on
device buffers and compute the oracle's answer for the same geometry."""
import numpy as np

import oracle as O
from mlx_data_amd import capi


def run_device(images, geoms, f32=False, src_align=16, dst_pad=0, device=0, rgba_weighted=0, base_shift=0,
               src_pad=0):
    """images: list of (H, W, C) uint8; geoms: (rw, rh, cx, cy, cw, ch, flip).

    Sources are packed into one device buffer with row pitch rounded up to
    ``src_align`` bytes (1 = tightly packed, exercising the unaligned path),
    each image starting ``base_shift`` bytes past a 256-byte boundary, rows
    ``src_pad`` bytes longer than the pixels before rounding.
    Returns the list of outputs (uint8, or float32 when f32)."""
    elem = 4 if f32 else 1
    pitches, offs, total = [], [], 0
    for img in images:
        h, w, c = img.shape
        p = (w * c + src_pad + src_align - 1) // src_align * src_align
        pitches.append(p)
        offs.append(total + base_shift)
        total += (p * h + 255) // 256 * 256
    src = capi.DeviceBuffer(total + 256, device)
    host = np.zeros(total + 256, np.uint8)
    for img, p, o in zip(images, pitches, offs):
        h, w, c = img.shape
        host[o : o + p * h].reshape(h, p)[:, : w * c] = img.reshape(h, w * c)
    src.upload(host)
    douts, dsts, entries = [], [], []
    for img, g, p, o in zip(images, geoms, pitches, offs):
        rw, rh, cx, cy, cw, ch, flip = g
        c = img.shape[2]
        dpitch = cw * c * elem + dst_pad
        d = capi.DeviceBuffer(dpitch * ch, device)
        d.memset(0)
        dsts.append((d, dpitch))
        entries.append(dict(src=src.ptr + o, src_stride=p, src_w=img.shape[1], src_h=img.shape[0], channels=c,
                            resize_w=rw, resize_h=rh, crop_x=cx, crop_y=cy, crop_w=cw, crop_h=ch, flip=int(flip),
                            dst=d.ptr, dst_stride=dpitch, rgba_weighted=int(rgba_weighted)))
    arr, n = capi.make_images(entries)
    capi.resize_crop_batch(arr, n, capi.MXD_F32_DIV255 if f32 else capi.MXD_U8, device, None)
    for (d, dpitch), g, img in zip(dsts, geoms, images):
        cw, ch = g[4], g[5]
        c = img.shape[2]
        raw = d.download((ch, dpitch), np.uint8)
        row = raw[:, : cw * c * elem].copy()
        douts.append(row.view(np.float32).reshape(ch, cw, c) if f32 else row.reshape(ch, cw, c))
        d.free()
    src.free()
    return douts


def oracle_out(img, g, rgba_weighted=None):
    rw, rh, cx, cy, cw, ch, flip = g
    r = O.resize(img, rw, rh, rgba_weighted)
    out = O.crop(r, cx, cy, cw, ch)
    return O.hflip(out) if flip else out


def center_geom(img, size=256, cw=224, ch=224):
    h, w = img.shape[:2]
    tw, th = O.smallest_side_dims(w, h, size)
    x, y = O.center_crop_origin(tw, th, cw, ch)
    return (tw, th, x, y, cw, ch, 0)


def compare(gpu, ref):
    """(max abs diff, fraction of nonzero diffs)."""
    d = np.abs(gpu.astype(np.int32) - ref.astype(np.int32))
    return int(d.max()), float((d > 0).mean())


def synth(h, w, c, seed):
    rng = np.random.default_rng(seed)
    gh, gw = h // 32 + 2, w // 32 + 2
    grid = rng.integers(0, 256, (gh, gw, c)).astype(np.float32)
    yi = np.minimum((np.arange(h) * (gh - 1)) // max(1, h - 1), gh - 2)
    xi = np.minimum((np.arange(w) * (gw - 1)) // max(1, w - 1), gw - 2)
    f = grid[yi][:, xi] * 0.6 + grid[yi + 1][:, xi + 1] * 0.4
    f += rng.normal(0, 16, f.shape).astype(np.float32)
    return np.ascontiguousarray(np.clip(f, 0, 255).astype(np.uint8))
