"""GPU: the host path (mxd_resize_crop_host) with page-locked memory.  Sources
and destinations that are page-locked are DMA'd in place (2-D copies of the
footprint rows / output rows) instead of being staged; a batch may mix both
kinds.  Results must equal the all-pageable call byte for byte."""
import ctypes

import numpy as np
import pytest

from gpu_util import synth
from mlx_data_amd import capi

pytestmark = pytest.mark.gpu


class Pinned:
    def __init__(self, nbytes):
        self.p = ctypes.c_void_p()
        capi.check(capi.lib().mxd_malloc_pinned(ctypes.byref(self.p), ctypes.c_size_t(nbytes)))
        self.a = np.ctypeslib.as_array((ctypes.c_uint8 * nbytes).from_address(self.p.value))

    def free(self):
        capi.check(capi.lib().mxd_free_pinned(self.p))


@pytest.mark.parametrize("f32", [False, True])
def test_pinned_and_pageable_mix(f32):
    elem = 4 if f32 else 1
    imgs = [synth(960, 1280, 3, 1), synth(375, 500, 3, 2), synth(200, 300, 3, 3), synth(333, 500, 3, 4),
            synth(61, 47, 3, 5)]
    geoms = []
    for im in imgs:
        h, w = im.shape[:2]
        rw, rh = capi.resize_smallest_side_dims(w, h, 64)
        cw, ch = min(rw, 56), min(rh, 56)
        geoms.append((rw, rh, (rw - cw) // 2, (rh - ch) // 2, cw, ch, 0))
    pins = []

    def run(pin_src, pin_dst):
        entries, outs = [], []
        for k, (im, g) in enumerate(zip(imgs, geoms)):
            h, w, c = im.shape
            pitch = w * c + (7 if k % 2 else 0)  # odd pitches too
            if pin_src[k]:
                ps = Pinned(pitch * h)
                pins.append(ps)
                src = ps.a.reshape(h, pitch)
                src_ptr = ps.p.value
            else:
                src = np.zeros((h, pitch), np.uint8)
                src_ptr = src.ctypes.data
            src[:, :w * c] = im.reshape(h, -1)
            row = g[4] * c * elem + (16 if k == 2 else 0)
            if pin_dst[k]:
                pd = Pinned(row * g[5])
                pins.append(pd)
                dst, dst_ptr = pd.a.reshape(g[5], row), pd.p.value
            else:
                dst = np.zeros((g[5], row), np.uint8)
                dst_ptr = dst.ctypes.data
            outs.append((dst, src))
            entries.append(dict(src=src_ptr, src_stride=pitch, src_w=w, src_h=h, channels=c, resize_w=g[0],
                                resize_h=g[1], crop_x=g[2], crop_y=g[3], crop_w=g[4], crop_h=g[5], flip=g[6],
                                dst=dst_ptr, dst_stride=row))
        arr, n = capi.make_images(entries)
        capi.resize_crop_host(arr, n, capi.MXD_F32_DIV255 if f32 else capi.MXD_U8, 0)
        return [d[:, :g[4] * im.shape[2] * elem].copy() for (d, _), g, im in zip(outs, geoms, imgs)]

    try:
        want = run([0] * 5, [0] * 5)
        for ps, pd in [([1] * 5, [1] * 5), ([1, 0, 1, 0, 1], [0, 1, 1, 0, 0]), ([0] * 5, [1] * 5)]:
            got = run(ps, pd)
            for a, b in zip(got, want):
                assert np.array_equal(a, b)
    finally:
        for p in pins:
            p.free()


@pytest.mark.parametrize("f32", [False, True])
def test_zero_copy_equals_dma(f32):
    """Zero copy (the kernel reads footprints and writes results over PCIe,
    in place in page-locked buffers or from / to the host path's page-locked
    staging) gives the bytes of the DMA form (MXD_POLICY_NO_ZERO_COPY)."""
    elem = 4 if f32 else 1
    imgs = [synth(960, 1280, 3, 11), synth(375, 500, 3, 12), synth(500, 333, 3, 13), synth(720, 1280, 3, 14)]
    geoms = []
    for k, im in enumerate(imgs):
        h, w = im.shape[:2]
        rw, rh = capi.resize_smallest_side_dims(w, h, 256)
        cx = 0 if k == 1 else rw - 224 if k == 2 else (rw - 224) // 2
        geoms.append((rw, rh, cx, (rh - 224) // 2, 224, 224, k % 2))
    pins = []

    def run(policy, pinned):
        prev = capi.set_kernel_policy(policy)
        try:
            entries, outs = [], []
            for im, g in zip(imgs, geoms):
                h, w, c = im.shape
                row = g[4] * c * elem
                if pinned:
                    ps, pd = Pinned(h * w * c), Pinned(row * g[5])
                    pins.extend([ps, pd])
                    src, sp = ps.a.reshape(h, w * c), ps.p.value
                    dst, dp = pd.a.reshape(g[5], row), pd.p.value
                else:
                    src = np.zeros((h, w * c), np.uint8)
                    dst = np.zeros((g[5], row), np.uint8)
                    sp, dp = src.ctypes.data, dst.ctypes.data
                src[:] = im.reshape(h, -1)
                outs.append((dst, src))
                entries.append(dict(src=sp, src_stride=w * c, src_w=w, src_h=h, channels=c, resize_w=g[0],
                                    resize_h=g[1], crop_x=g[2], crop_y=g[3], crop_w=g[4], crop_h=g[5], flip=g[6],
                                    dst=dp, dst_stride=row))
            arr, n = capi.make_images(entries)
            capi.resize_crop_host(arr, n, capi.MXD_F32_DIV255 if f32 else capi.MXD_U8, 0)
            return [d.copy() for d, _ in outs]
        finally:
            capi.set_kernel_policy(prev)

    try:
        want = run(capi.MXD_POLICY_NO_ZERO_COPY, False)
        for policy, pinned in [(0, False), (0, True), (capi.MXD_POLICY_NO_ZERO_COPY, True)]:
            for a, b in zip(run(policy, pinned), want):
                assert np.array_equal(a, b), (policy, pinned)
    finally:
        for p in pins:
            p.free()


@pytest.mark.parametrize("f32", [False, True])
def test_zero_copy_bottom_right_crops_of_page_aligned_buffers(f32):
    """a zero-copy source read in place must never be read past its
    last pixel.  Images whose bytes end exactly at a page boundary of their
    page-locked buffer (1024x768x3 = 576 pages; 768x1024x3), cropped at the
    bottom-right corner (the footprint reaches the last stored byte) with and
    without a mirror, and sources that start 1-3 bytes past a 4-byte boundary
    so the same end falls mid-dword: bytes equal the kernel-order oracle."""
    import oracle as O

    elem = 4 if f32 else 1
    cases = []
    for (h, w) in [(768, 1024), (1024, 768)]:
        for flip in (0, 1):
            for shift in (0, 1, 3):
                cases.append((h, w, flip, shift))
    pins = []
    try:
        entries, outs = [], []
        for k, (h, w, flip, shift) in enumerate(cases):
            im = synth(h, w, 3, 40 + k)
            nbytes = h * w * 3
            ps = Pinned(nbytes + shift)
            pins.append(ps)
            src = ps.a[shift:shift + nbytes]
            src[:] = im.reshape(-1)
            rw, rh = capi.resize_smallest_side_dims(w, h, 256)
            g = (rw, rh, rw - 224, rh - 224, 224, 224, flip)
            row = 224 * 3 * elem
            dst = np.zeros((224, row), np.uint8)
            outs.append((dst, im, g))
            entries.append(dict(src=ps.p.value + shift, src_stride=w * 3, src_w=w, src_h=h, channels=3, resize_w=rw,
                                resize_h=rh, crop_x=g[2], crop_y=g[3], crop_w=224, crop_h=224, flip=flip,
                                dst=dst.ctypes.data, dst_stride=row))
        arr, n = capi.make_images(entries)
        capi.resize_crop_host(arr, n, capi.MXD_F32_DIV255 if f32 else capi.MXD_U8, 0)
        lut = (np.arange(256, dtype=np.uint8).astype("float32") / 255).view(np.uint32)
        for dst, im, g in outs:
            want = O.resize_crop_vfirst(im, g)
            if f32:
                assert np.array_equal(dst.view(np.uint32).reshape(224, 224, 3), lut[want]), g
            else:
                assert np.array_equal(dst.reshape(224, 224, 3), want), g
    finally:
        for p in pins:
            p.free()


def test_narrow_return_equals_f32_over_the_link():
    """ABI 7: f32 results bound for pageable host memory cross the link as the
    kernels' u8 bytes and are expanded (x / 255, IEEE f32 division) on the host
    (MXD_TUNE_F32_LINK 0, the default): the bytes equal the f32-over-the-link
    form (MXD_TUNE_F32_LINK 1, with page-locked destinations the device's
    in-place f32 writes) and the numpy LUT of the u8 call, and
    mxd_narrow_returns counts the images, page-locked destinations included."""
    imgs = [synth(960, 1280, 3, 31), synth(375, 500, 3, 32), synth(61, 47, 3, 33), synth(720, 1280, 3, 34)]
    geoms = []
    for k, im in enumerate(imgs):
        h, w = im.shape[:2]
        rw, rh = capi.resize_smallest_side_dims(w, h, 256 if k != 2 else 40)
        cw, ch = min(rw, 224 if k != 2 else 33), min(rh, 224 if k != 2 else 37)
        geoms.append((rw, rh, (rw - cw) // 2, (rh - ch) // 2, cw, ch, k % 2))
    pins = []

    def run(dtype, link, pinned=False, pad=0):
        prev = capi.set_tuning(capi.MXD_TUNE_F32_LINK, link)
        try:
            elem = 4 if dtype == capi.MXD_F32_DIV255 else 1
            entries, outs = [], []
            for im, g in zip(imgs, geoms):
                h, w, c = im.shape
                row = g[4] * c * elem + pad
                if pinned:
                    pd = Pinned(row * g[5])
                    pins.append(pd)
                    dst, dp = pd.a.reshape(g[5], row), pd.p.value
                else:
                    dst = np.zeros((g[5], row), np.uint8)
                    dp = dst.ctypes.data
                outs.append((dst, g[4] * c * elem))
                entries.append(dict(src=im.ctypes.data, src_stride=w * c, src_w=w, src_h=h, channels=c,
                                    resize_w=g[0], resize_h=g[1], crop_x=g[2], crop_y=g[3], crop_w=g[4],
                                    crop_h=g[5], flip=g[6], dst=dp, dst_stride=row))
            arr, n = capi.make_images(entries)
            capi.resize_crop_host(arr, n, dtype, 0)
            return [d[:, :r].copy() for d, r in outs]
        finally:
            capi.set_tuning(capi.MXD_TUNE_F32_LINK, prev)

    lut = np.arange(256, dtype=np.uint8).astype(np.float32) / np.float32(255)
    try:
        u8 = run(capi.MXD_U8, 0)
        capi.narrow_returns(reset=True)
        narrow = run(capi.MXD_F32_DIV255, 0)
        assert capi.narrow_returns(reset=True) == len(imgs)
        wide = run(capi.MXD_F32_DIV255, 1)
        padded = run(capi.MXD_F32_DIV255, 0, pad=20)  # destination rows longer than the output row
        assert capi.narrow_returns(reset=True) == len(imgs)
        pinned = run(capi.MXD_F32_DIV255, 0, pinned=True)
        assert capi.narrow_returns(reset=True) == len(imgs)
        pinned_wide = run(capi.MXD_F32_DIV255, 1, pinned=True)
        assert capi.narrow_returns(reset=True) == 0
        # a share of the images narrowed (MXD_TUNE_F32_LINK 2..99): two
        # launches per chunk, one per output dtype
        half = run(capi.MXD_F32_DIV255, 50)
        half_pinned = run(capi.MXD_F32_DIV255, 50, pinned=True)
        assert capi.narrow_returns(reset=True) == 2 * (len(imgs) // 2)
        for a, b, c, d, e, f, g, u in zip(narrow, wide, padded, pinned, pinned_wide, half, half_pinned, u8):
            assert np.array_equal(a, b) and np.array_equal(a, c) and np.array_equal(a, d) and np.array_equal(a, e)
            assert np.array_equal(a, f) and np.array_equal(a, g)
            assert np.array_equal(a.view(np.float32), lut[u])
    finally:
        for p in pins:
            p.free()
