"""Batched image functions over the C ABI (host numpy in, numpy out):
resize+crop (the hot path) and the pixel maps rotate / channel_reduction.

These are the functional counterparts of the reference's per-image
core::image::{scale, resize, crop, hflip} (mlx/data/core/image/ImageTransform.cpp)
applied to a whole batch in one fused kernel launch; geometry follows
ImageResizeSmallestSide / ImageCenterCrop (mlx/data/op/ImageTransform.cpp:78-126).
"""
import numpy as np

from . import capi


def _as_image(img):
    """The reference's checks (core/image/ImageTransform.cpp:17-31 verify_type,
    core/image/ImageIO.cpp:39-49 verify_image): HWC uint8, 1..4 channels; no
    silent casts or reshapes."""
    img = np.asarray(img)
    if img.dtype != np.uint8:
        raise TypeError("image must be of type UInt8")
    if img.ndim != 3:
        raise ValueError("verifyImage: image must be 3 dimension Array (HWC)")
    if img.shape[2] == 0 or img.shape[2] > 4:
        raise ValueError("verifyImage: channels must be 0 <= c <= 4")
    return np.ascontiguousarray(img)


def plan_resize_smallest_side_center_crop(w, h, size, cw, ch):
    """(resize_w, resize_h, crop_x, crop_y) exactly as the reference computes them."""
    tw, th = capi.resize_smallest_side_dims(w, h, size)
    x, y = capi.center_crop_origin(tw, th, cw, ch)
    return tw, th, x, y


def resize_crop(images, geoms, out_dtype="uint8", device=0):
    """Host-resident fused path.

    images: list of (H, W, C) uint8 arrays.
    geoms:  list of (resize_w, resize_h, crop_x, crop_y, crop_w, crop_h, flip).
    Returns a list of (crop_h, crop_w, C) arrays (uint8, or float32 q/255).
    """
    f32 = out_dtype in ("float32", np.float32)
    outs, entries = [], []
    keep = []
    for img, g in zip(images, geoms):
        img = _as_image(img)
        rw, rh, x, y, cw, ch, flip = g
        out = np.empty((ch, cw, img.shape[2]), np.float32 if f32 else np.uint8)
        keep.append(img)
        outs.append(out)
        entries.append(dict(src=img.ctypes.data, src_stride=img.strides[0], src_w=img.shape[1], src_h=img.shape[0],
                            channels=img.shape[2], resize_w=rw, resize_h=rh, crop_x=x, crop_y=y, crop_w=cw,
                            crop_h=ch, flip=int(bool(flip)), dst=out.ctypes.data, dst_stride=out.strides[0]))
    arr, n = capi.make_images(entries)
    capi.resize_crop_host(arr, n, capi.MXD_F32_DIV255 if f32 else capi.MXD_U8, device)
    return outs


def resize_smallest_side_center_crop(images, size, cw, ch, out_dtype="uint8", device=0):
    geoms = []
    for img in images:
        h, w = img.shape[:2]
        tw, th, x, y = plan_resize_smallest_side_center_crop(w, h, size, cw, ch)
        geoms.append((tw, th, x, y, cw, ch, 0))
    return resize_crop(images, geoms, out_dtype, device)


def _pixmap(images, op, params_of, dims_of, out_c, device):
    entries, outs, keep = [], [], []
    for img in images:
        img = _as_image(img)
        h, w, c = img.shape
        dw, dh = dims_of(w, h)
        out = np.empty((dh, dw, out_c(c)), np.uint8)
        keep.append(img)
        outs.append(out)
        entries.append(dict(src=img.ctypes.data, src_stride=img.strides[0], src_w=w, src_h=h, channels=c, dst_w=dw,
                            dst_h=dh, dst=out.ctypes.data, dst_stride=out.strides[0], params=params_of(w, h)))
    if entries:
        arr, n = capi.make_pixmaps(entries)
        capi.pixmap_host(arr, n, op, device)
    return outs


def rotate(images, angle, crop=False, device=0):
    """core::image::rotate (core/image/ImageTransform.cpp:112-121) of a batch:
    one pixel-map launch.  Returns a list of uint8 arrays."""
    geo = {}

    def g(w, h):
        if (w, h) not in geo:
            geo[(w, h)] = capi.rotate_geometry(w, h, angle, crop)
        return geo[(w, h)]

    return _pixmap(images, capi.MXD_AFFINE, lambda w, h: g(w, h)[0], lambda w, h: g(w, h)[1:], lambda c: c, device)


def channel_reduction(images, preset="default", device=0):
    """core::image::channel_reduction (core/image/ImageTransform.cpp:142-180)
    of a batch of RGB images: one launch.  Returns (H, W, 1) uint8 arrays."""
    p = capi.channel_reduction_preset(preset)
    return _pixmap(images, capi.MXD_CHANNEL_REDUCTION, lambda w, h: p, lambda w, h: (w, h), lambda c: 1, device)
