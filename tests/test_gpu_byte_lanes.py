"""GPU: byte-lane RGB scatter kernels (16 contiguous bytes per lane, V pass in
memory order, H pass at channel stride; csrc/wave.hip Lay<3, 16>) forced with
MXD_POLICY_BYTES give the bytes the pixel-lane kernels give
(MXD_POLICY_NO_BYTES) -- on whole device-resident images, crops at every
edge, mirrored crops, odd base addresses, and through the host path, where
only each image's staged footprint is on the device (the kernel's window
offsets and its last-chunk check then run against the footprint's pitch)."""
import numpy as np
import pytest

import oracle as O
from gpu_util import compare, oracle_out, run_device, synth
from mlx_data_amd import capi
from mlx_data_amd import image as mimg

pytestmark = pytest.mark.gpu


def _with_policy(policy, fn):
    prev = capi.set_kernel_policy(policy)
    try:
        return fn()
    finally:
        capi.set_kernel_policy(prev)


def _cases():
    imgs, geoms = [], []
    for (h, w), size, crop, seed in [((960, 1280), 256, 224, 1), ((720, 1280), 256, 224, 2),
                                     ((1080, 1920), 256, 224, 3), ((1440, 2560), 256, 224, 4),
                                     ((2160, 3840), 512, 448, 5), ((480, 640), 256, 224, 6)]:
        img = synth(h, w, 3, seed)
        rw, rh = O.smallest_side_dims(w, h, size)
        for cx, cy, flip in [((rw - crop) // 2, (rh - crop) // 2, 0), (0, 0, 1), (rw - crop, rh - crop, 0),
                             (rw - crop, 0, 1)]:
            imgs.append(img)
            geoms.append((rw, rh, cx, cy, crop, crop, flip))
    return imgs, geoms


@pytest.mark.parametrize("f32", [False, True])
def test_forced_byte_lanes_equal_pixel_lanes(f32):
    imgs, geoms = _cases()
    e = dict(src=256, src_stride=imgs[0].shape[1] * 3, src_w=imgs[0].shape[1], src_h=imgs[0].shape[0], channels=3,
             resize_w=geoms[0][0], resize_h=geoms[0][1], crop_x=geoms[0][2], crop_y=geoms[0][3], crop_w=224,
             crop_h=224, flip=0, dst=256, dst_stride=224 * 3)
    assert _with_policy(capi.MXD_POLICY_BYTES, lambda: capi.describe_plan(e))["p"] == 16
    got = _with_policy(capi.MXD_POLICY_BYTES, lambda: run_device(imgs, geoms, f32=f32))
    want = _with_policy(capi.MXD_POLICY_NO_BYTES, lambda: run_device(imgs, geoms, f32=f32))
    for i, (a, b) in enumerate(zip(got, want)):
        assert np.array_equal(a.view(np.uint8), b.view(np.uint8)), (i, geoms[i])
    if not f32:
        for k in (0, 2, 5, 18):
            m, frac = compare(got[k], oracle_out(imgs[k], geoms[k]))
            assert m <= 1 and frac < 2e-3, (geoms[k], m, frac)


@pytest.mark.parametrize("shift", [1, 2, 3])
def test_forced_byte_lanes_odd_base_addresses(shift):
    """Device sources whose first byte is 1-3 bytes past a 4-byte boundary
    (rows padded so the wave kernels still apply): byte lanes fold the offset
    into the H-pass positions; pixel lanes realign with alignbyte."""
    imgs, geoms = _cases()
    kw = dict(base_shift=shift, src_pad=16)
    got = _with_policy(capi.MXD_POLICY_BYTES, lambda: run_device(imgs, geoms, **kw))
    want = _with_policy(capi.MXD_POLICY_NO_BYTES, lambda: run_device(imgs, geoms, **kw))
    ref = _with_policy(capi.MXD_POLICY_NO_BYTES, lambda: run_device(imgs, geoms))
    for i, (a, b, r) in enumerate(zip(got, want, ref)):
        assert np.array_equal(a, b), (i, geoms[i])
        assert np.array_equal(a, r), (i, geoms[i])


def test_forced_byte_lanes_host_path():
    """Host path: pageable numpy sources (footprint staged), some of them views
    whose first byte is not 4-byte aligned."""
    imgs, geoms = _cases()
    srcs = []
    for k, im in enumerate(imgs):
        if k % 3 == 1:
            # a 1-byte-offset base: a view into a larger buffer
            h, w, c = im.shape
            buf = np.zeros(h * w * c + 64, np.uint8)
            v = buf[1:1 + h * w * c].reshape(h, w, c)
            v[...] = im
            srcs.append(v)
        else:
            srcs.append(im)
    got = _with_policy(capi.MXD_POLICY_BYTES, lambda: mimg.resize_crop(srcs, geoms))
    want = _with_policy(capi.MXD_POLICY_NO_BYTES, lambda: mimg.resize_crop(srcs, geoms))
    dev = _with_policy(capi.MXD_POLICY_NO_BYTES, lambda: run_device(imgs, geoms))
    for i, (a, b, d) in enumerate(zip(got, want, dev)):
        assert np.array_equal(a, b), (i, geoms[i])
        assert np.array_equal(a, d), (i, geoms[i])
