"""TEST INFRASTRUCTURE ONLY -- ctypes/numpy face of the CPU oracle.

Only tests/, ``__graft_entry__.smoke()`` and bench.py's ``cpu_baseline`` leg
import this module.  The product path (mlx-data_amd/) never does.

* ``liboracle.so`` (stbir_oracle.c): CPU restatement of
  core::image::scale/resize/crop/hflip, array::batch and the /255 normalize
  (reference file:line citations in stbir_oracle.c).  Resize arithmetic is
  "parity unpinned" by the reference (stb_image_resize2 is not in this image);
  see DESIGN.md section "Oracle".
* ``_ref/libmlxref.so`` (ref_harness.cpp + the reference's own Array.cpp,
  Sample.cpp, core/BatchShape.cpp, core/State.cpp): crop bytes, batch layout
  and RNG draw streams computed by the reference's code itself.
"""
import ctypes
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
_u8p = ctypes.POINTER(ctypes.c_uint8)
_i64p = ctypes.POINTER(ctypes.c_int64)
_i32p = ctypes.POINTER(ctypes.c_int32)
_f32p = ctypes.POINTER(ctypes.c_float)

_lib = None
_ref = None


def lib():
    global _lib
    if _lib is None:
        path = os.path.join(HERE, "liboracle.so")
        if not os.path.exists(path):
            raise RuntimeError("oracle/liboracle.so missing: run `make -C oracle`")
        _lib = ctypes.CDLL(path)
    return _lib


def ref_lib():
    """The reference-code harness, or None when it was never built."""
    global _ref
    if _ref is None:
        path = os.path.join(HERE, "_ref", "libmlxref.so")
        if not os.path.exists(path):
            return None
        _ref = ctypes.CDLL(path)
    return _ref


def _ptr(a, t=_u8p):
    return a.ctypes.data_as(t)


def axis_coeffs(in_size, out_size):
    """(first, last, weights[out, width]) of the restated stbir triangle filter."""
    L = lib()
    cw = L.orc_axis_width(in_size, out_size)
    n0 = np.zeros(out_size, np.int32)
    n1 = np.zeros(out_size, np.int32)
    w = np.zeros((out_size, cw), np.float32)
    rc = L.orc_axis_coeffs(in_size, out_size, cw, _ptr(n0, _i32p), _ptr(n1, _i32p), _ptr(w, _f32p))
    if rc:
        raise ValueError("orc_axis_coeffs failed")
    return n0, n1, w


def resize(img, dw, dh, rgba_weighted=None):
    """stbir_resize_uint8_linear restated: (H, W, C) u8 -> (dh, dw, C) u8.
    C = 4 is alpha-weighted (STBIR_RGBA) unless rgba_weighted=False."""
    img = np.ascontiguousarray(img, np.uint8)
    h, w, c = img.shape
    out = np.zeros((dh, dw, c), np.uint8)
    weighted = (c == 4) if rgba_weighted is None else bool(rgba_weighted)
    if lib().orc_resize_u8_layout(_ptr(img), w, h, c, _ptr(out), dw, dh, int(weighted)):
        raise ValueError("orc_resize_u8 failed")
    return out


def resize_crop_vfirst(img, g):
    """Kernel-order restatement (orc_resize_crop_vfirst): the geometry tuple
    g = (rw, rh, cx, cy, cw, ch, flip) of a (H, W, C <= 4) uint8 image, summed
    vertical-first in byte units with fmaf chains in tap order -- what the HIP
    kernels must reproduce bit for bit."""
    rw, rh, cx, cy, cw, ch, flip = g
    img = np.ascontiguousarray(img)
    h, w, c = img.shape
    out = np.empty((ch, cw, c), np.uint8)
    if lib().orc_resize_crop_vfirst(_ptr(img), w, h, c, ctypes.c_int64(w * c), _ptr(out), rw, rh, cx, cy, cw, ch,
                                    int(bool(flip))):
        raise ValueError("orc_resize_crop_vfirst failed")
    return out


def resize_crop_vfirst_rgba(img, g):
    """Kernel-order restatement of the STBIR_RGBA form (orc_resize_crop_vfirst_rgba):
    a (H, W, 4) uint8 image, decoded, alpha-weighted, vertical pass first, in
    stbir's float operations -- what the general HIP kernel reproduces bit for bit."""
    rw, rh, cx, cy, cw, ch, flip = g
    img = np.ascontiguousarray(img)
    h, w, c = img.shape
    assert c == 4
    out = np.empty((ch, cw, 4), np.uint8)
    if lib().orc_resize_crop_vfirst_rgba(_ptr(img), w, h, ctypes.c_int64(w * 4), _ptr(out), rw, rh, cx, cy, cw, ch,
                                         int(bool(flip))):
        raise ValueError("orc_resize_crop_vfirst_rgba failed")
    return out


def smallest_side_dims(w, h, size):
    tw, th = ctypes.c_int64(), ctypes.c_int64()
    if lib().orc_resize_smallest_side_dims(
        ctypes.c_int64(w), ctypes.c_int64(h), ctypes.c_int64(size), ctypes.byref(tw), ctypes.byref(th)
    ):
        raise ValueError("ImageResizeSmallestSide: illegal target size")
    return tw.value, th.value


def center_crop_origin(w, h, cw, ch):
    if ch > h or cw > w:
        raise ValueError("ImageCenterCrop: target image size larger than input image")
    return (w - cw) // 2, (h - ch) // 2


def crop(img, x, y, cw, ch):
    img = np.ascontiguousarray(img, np.uint8)
    h, w, c = img.shape
    out = np.zeros((ch, cw, c), np.uint8)
    if lib().orc_crop_u8(_ptr(img), w, h, c, x, y, cw, ch, _ptr(out)):
        raise ValueError("crop out of bounds")
    return out


def hflip(img):
    img = np.ascontiguousarray(img, np.uint8)
    h, w, c = img.shape
    out = np.zeros_like(img)
    lib().orc_hflip_u8(_ptr(img), w, h, c, _ptr(out))
    return out


def normalize(q):
    q = np.ascontiguousarray(q, np.uint8)
    out = np.zeros(q.shape, np.float32)
    lib().orc_normalize_u8(_ptr(q), ctypes.c_size_t(q.size), _ptr(out, _f32p))
    return out


def resize_crop(img, size, cw, ch, crop_xy=None, flip=False):
    """resize_smallest_side(size) -> crop (centre unless crop_xy) -> optional hflip."""
    h, w = img.shape[:2]
    tw, th = smallest_side_dims(w, h, size)
    r = resize(img, tw, th)
    x, y = center_crop_origin(tw, th, cw, ch) if crop_xy is None else crop_xy
    out = crop(r, x, y, cw, ch)
    return hflip(out) if flip else out


def batch(arrs, pad=0):
    """array::batch: stack (H, W, C) u8 arrays into the padded NHWC batch."""
    shape = [len(arrs)] + [max(a.shape[d] for a in arrs) for d in range(3)]
    out = np.full(shape, pad, np.uint8)
    for i, a in enumerate(arrs):
        out[i, : a.shape[0], : a.shape[1], : a.shape[2]] = a
    return out


# ---- reference-code harness (oracle/_ref) ---------------------------------


def ref_crop(img, x, y, cw, ch):
    R = ref_lib()
    img = np.ascontiguousarray(img, np.uint8)
    h, w, c = img.shape
    out = np.zeros((ch, cw, c), np.uint8)
    if R.ref_crop_u8(_ptr(img), w, h, c, x, y, cw, ch, _ptr(out)):
        raise ValueError("array::sub raised")
    return out


def ref_batch(arrs, pad=0.0):
    R = ref_lib()
    arrs = [np.ascontiguousarray(a, np.uint8) for a in arrs]
    ptrs = (ctypes.POINTER(ctypes.c_uint8) * len(arrs))(*[_ptr(a) for a in arrs])
    shapes = np.array([a.shape for a in arrs], np.int64).reshape(-1)
    shape = [len(arrs)] + [max(a.shape[d] for a in arrs) for d in range(3)]
    out = np.zeros(shape, np.uint8)
    R.ref_batch_u8.restype = ctypes.c_int64
    n = R.ref_batch_u8(ptrs, _ptr(shapes, _i64p), len(arrs), ctypes.c_double(pad), _ptr(out), ctypes.c_int64(out.size))
    if n != out.size:
        raise ValueError("array::batch failed")
    return out


def ref_random_crop_flip(seed, sizes_wh, cw, ch, prob):
    """Per-sample (x, y, flip) draws of random_crop then random_h_flip after set_state(seed)."""
    R = ref_lib()
    wh = np.ascontiguousarray(np.asarray(sizes_wh, np.int64).reshape(-1))
    n = len(wh) // 2
    xy = np.zeros(2 * n, np.int64)
    fl = np.zeros(n, np.int32)
    R.ref_random_crop_flip_params(
        ctypes.c_int64(seed), n, _ptr(wh, _i64p), ctypes.c_int64(cw), ctypes.c_int64(ch), ctypes.c_float(prob),
        _ptr(xy, _i64p), _ptr(fl, _i32p)
    )
    return xy.reshape(n, 2), fl


def ref_random_area_crop(seed, sizes_wh, area_range, aspect_range, trials=10):
    """Per-sample (x, y, w, h) draws of image_random_area_crop after set_state(seed)
    (zeros: no crop found), from the reference's State (oracle/ref_harness.cpp)."""
    R = ref_lib()
    wh = np.ascontiguousarray(np.asarray(sizes_wh, np.int64).reshape(-1))
    n = len(wh) // 2
    out = np.zeros(4 * n, np.int64)
    R.ref_random_area_crop_params(
        ctypes.c_int64(seed), n, _ptr(wh, _i64p), ctypes.c_float(area_range[0]), ctypes.c_float(area_range[1]),
        ctypes.c_float(aspect_range[0]), ctypes.c_float(aspect_range[1]), int(trials), _ptr(out, _i64p)
    )
    return out.reshape(n, 4)


# ---- rotate / channel reduction -------------------------
CHANNEL_PRESETS = {  # op/ImageTransform.cpp:362-392 (float literals)
    "default": (0.0, (0.299, 0.587, 0.114)),
    "rec601": (0.0, (0.299, 0.587, 0.114)),
    "rec709": (0.0, (0.2126, 0.7152, 0.0722)),
    "rec2020": (0.0, (0.2627, 0.678, 0.0593)),
    "green": (0.0, (0.0, 1.0, 0.0)),
}


def rotate_geometry(w, h, angle, crop=False):
    mx = np.zeros(6, np.float32)
    tw, th = ctypes.c_int64(), ctypes.c_int64()
    bad = lib().orc_rotate_geometry(ctypes.c_int64(w), ctypes.c_int64(h), ctypes.c_double(angle), int(bool(crop)),
                                    _ptr(mx, _f32p), ctypes.byref(tw), ctypes.byref(th))
    return mx, tw.value, th.value, bool(bad)


def rotate(img, angle, crop=False):
    """core::image::rotate (core/image/ImageTransform.cpp:112-121)."""
    img = np.ascontiguousarray(img, np.uint8)
    h, w, c = img.shape
    mx, tw, th, bad = rotate_geometry(w, h, angle, crop)
    if bad:
        raise ValueError("image: cannot create image with 0 or negative dimension")
    out = np.zeros((th, tw, c), np.uint8)
    lib().orc_affine_u8(_ptr(img), ctypes.c_int64(w), ctypes.c_int64(h), ctypes.c_int64(c), _ptr(mx, _f32p),
                        ctypes.c_int64(tw), ctypes.c_int64(th), _ptr(out))
    return out


def channel_reduction(img, preset="default"):
    """core::image::channel_reduction (core/image/ImageTransform.cpp:142-180)."""
    img = np.ascontiguousarray(img, np.uint8)
    h, w, c = img.shape
    assert c == 3
    bias, m = CHANNEL_PRESETS[preset]
    mm = np.array(m, np.float32)
    out = np.zeros((h, w, 1), np.uint8)
    lib().orc_channel_reduction_u8(_ptr(img), ctypes.c_int64(w), ctypes.c_int64(h), ctypes.c_float(bias),
                                   _ptr(mm, _f32p), _ptr(out))
    return out
