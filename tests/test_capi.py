"""CPU-side checks of the C ABI (no device work): the library loads, exports
every symbol include/mxd_amd.h declares, its host logic (geometry, tap tables,
argument validation) matches the reference rules and the oracle."""
import ctypes
import os
import re

import numpy as np
import pytest

import oracle as O
from mlx_data_amd import capi

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def header_symbols():
    text = open(os.path.join(REPO, "include", "mxd_amd.h")).read()
    return sorted(set(re.findall(r"^\s*(?:int|const char\*)\s+(mxd_\w+)\s*\(", text, re.M)))


def test_library_exports_every_header_symbol():
    L = capi.lib()
    syms = header_symbols()
    assert len(syms) >= 20
    for s in syms:
        assert hasattr(L, s), s
    assert sorted(capi.EXPORTS) == syms
    assert L.mxd_abi_version() == 7


@pytest.mark.parametrize("w,h,size", [(1280, 960, 256), (375, 500, 256), (500, 375, 256), (300, 200, 256),
                                      (3840, 2160, 512), (300, 300, 256), (1, 1, 256), (333, 500, 256),
                                      (641, 479, 224), (7, 1000, 256)])
def test_geometry_matches_oracle(w, h, size):
    assert capi.resize_smallest_side_dims(w, h, size) == O.smallest_side_dims(w, h, size)


def test_geometry_errors_use_reference_messages():
    with pytest.raises(capi.MxdError, match="ImageResizeSmallestSide: illegal target size: 0"):
        capi.resize_smallest_side_dims(10, 10, 0)
    with pytest.raises(capi.MxdError, match="ImageCenterCrop: target image size larger than input image"):
        capi.center_crop_origin(200, 300, 224, 224)
    assert capi.center_crop_origin(341, 256, 224, 224) == (58, 16)


GEOMS = [(1280, 341), (960, 256), (300, 384), (200, 256), (3840, 455), (2160, 256), (3840, 910), (2160, 512),
         (375, 256), (500, 341), (500, 333), (333, 256), (256, 256), (100, 256), (7, 3), (3, 7), (1, 5), (5, 1),
         (1000, 999), (999, 1000), (640, 341), (480, 256), (1080, 256), (1920, 455), (2560, 455), (1440, 256)]


@pytest.mark.parametrize("i,o", GEOMS)
def test_tap_tables_bitwise_equal_oracle(i, o):
    n0, n1, w = O.axis_coeffs(i, o)
    first, cnt, pw = capi.axis_taps(i, o)
    assert np.array_equal(first, n0)
    assert np.array_equal(cnt, n1 - n0 + 1)
    for j in range(o):
        k = cnt[j]
        assert np.array_equal(w[j, :k].view(np.uint32), pw[j, :k].view(np.uint32))
        assert not pw[j, k:].any()


def test_tap_window_is_slice_of_full_axis():
    f_full, c_full, w_full = capi.axis_taps(1280, 341)
    f, c, w = capi.axis_taps(1280, 341, 58, 224)
    assert np.array_equal(f, f_full[58:282]) and np.array_equal(c, c_full[58:282])
    assert np.array_equal(w[:, : w_full.shape[1]], w_full[58:282, : w.shape[1]])


def _one(**kw):
    e = dict(src=16, src_stride=3 * 100, src_w=100, src_h=80, channels=3, resize_w=100, resize_h=80, crop_x=0,
             crop_y=0, crop_w=50, crop_h=40, flip=0, dst=16, dst_stride=150)
    e.update(kw)
    return capi.make_images([e])


@pytest.mark.parametrize("kw,msg", [
    (dict(crop_w=200), "Array: sub: shape out of bound"),
    (dict(crop_x=100), "Array: sub: offset out of bound"),
    (dict(resize_w=0), "image: cannot create image with 0 or negative dimension"),
    (dict(crop_h=0), "image: cannot create image with 0 or negative dimension"),
    (dict(channels=0), "verifyImage: channels must be 0 <= c <= 4"),
    (dict(channels=5), "verifyImage: channels must be 0 <= c <= 4"),
    (dict(src=0), "null src/dst"),
])
def test_batch_validation_rejects_before_touching_the_device(kw, msg):
    arr, n = _one(**kw)
    with pytest.raises(capi.MxdError, match=msg):
        capi.resize_crop_batch(arr, n, capi.MXD_U8)


def test_channel_count_checked_like_verify_image():
    """1..4 channels (4 = STBIR_RGBA, tests/test_gpu_rgba.py); 5 is rejected
    with core/image/ImageIO.cpp:45-47's message before any device work."""
    arr, n = _one(channels=5, src_stride=500, dst_stride=250)
    with pytest.raises(capi.MxdError, match="channels must be 0 <= c <= 4") as e:
        capi.resize_crop_batch(arr, n, capi.MXD_U8)
    assert e.value.code == 1


def _entry(w=1280, h=960, stride=None, rw=341, rh=256, cx=58, cy=16, **kw):
    e = dict(src_w=w, src_h=h, src_stride=stride or w * 3, channels=3, resize_w=rw, resize_h=rh, crop_x=cx,
             crop_y=cy, crop_w=224, crop_h=224, flip=0, dst_stride=224 * 3 * 4)
    e.update(kw)
    return e


def _plan(entry, policy=0):
    prev = capi.set_kernel_policy(policy)
    try:
        return capi.describe_plan(entry, capi.MXD_F32_DIV255)
    finally:
        capi.set_kernel_policy(prev)


def test_rgb_scatter_lane_layouts():
    """RGB scatter plans (host only): byte lanes (p = 16: 16 contiguous bytes
    per lane, 1-KiB windows) when they need no more strips than pixel lanes at
    <= 2 output pixels per lane -- 720p -> 224, two strips -- and pixel lanes
    otherwise: C2's 960 -> 256 takes two 512-pixel strips with pixel lanes,
    three with byte lanes; ImageNet shapes (C4) two 256-pixel strips (one
    wide strip would run at 2-3 waves per SIMD, profiles/r03/onestrip.jsonl),
    one 1-KiB byte-lane strip when forced (profiles/r02/bytes_ab.txt).  MXD_POLICY_NO_BYTES keeps pixel lanes,
    MXD_POLICY_BYTES takes byte lanes wherever a kernel exists."""
    p = _plan(_entry())
    assert (p["wave"], p["kind"], p["taps"], p["s"], p["dmax"]) == (1, 2, 8, 2, 4)
    assert (p["p"], p["nstrips"], p["q"]) == (8, 2, 2)
    b = _plan(_entry(), capi.MXD_POLICY_BYTES)
    assert (b["p"], b["nstrips"], b["q"]) == (16, 3, 2)
    hd = _entry(1280, 720, 3840, 455, 256, cx=(455 - 224) // 2)
    assert (_plan(hd)["p"], _plan(hd)["nstrips"]) == (16, 2)
    assert _plan(hd, capi.MXD_POLICY_NO_BYTES)["p"] == 8
    c4 = _entry(500, 375, 1500, 341, 256)
    # one wide strip or two narrow ones: the narrow kernel (8 waves per SIMD)
    assert (_plan(c4)["p"], _plan(c4)["nstrips"], _plan(c4)["q"]) == (4, 2, 2)
    assert (_plan(c4, capi.MXD_POLICY_BYTES)["p"], _plan(c4, capi.MXD_POLICY_BYTES)["q"]) == (16, 4)


def test_byte_lanes_stay_inside_the_row():
    """A window reaching the last pixel of a tightly packed row would read its
    last 16-byte chunk past the row (and past the buffer on the last row):
    such crops keep pixel lanes, even when byte lanes are forced."""
    forced = capi.MXD_POLICY_BYTES
    assert _plan(_entry(500, 375, 1500, 341, 256), forced)["p"] == 16
    right = _entry(500, 375, 1500, 341, 256, cx=341 - 224)
    p = _plan(right, forced)
    assert p["wave"] == 1 and p["p"] != 16
    # the same crop with 16-byte padded rows fits
    assert _plan(dict(right, src_stride=1504), forced)["p"] == 16


def test_every_downscale_ratio_up_to_16_has_a_wave_kernel():
    """No cliff to the general kernel: RGB
    resize_smallest_side 256 -> center_crop 224 from every smaller side 257 ..
    4096 (up to 16:1) plans a wave scatter kernel whose tap bucket covers the
    horizontal taps and whose schedule depth covers the vertical shape (a
    deeper schedule runs bubble iterations); 12 MP and 24 MP photos take the
    24 / 32-tap buckets."""
    for side in list(range(257, 1200, 7)) + list(range(1200, 4097, 53)):
        w = side * 4 // 3
        rw, rh = capi.resize_smallest_side_dims(w, side, 256)
        cx, cy = capi.center_crop_origin(rw, rh, 224, 224)
        e = _entry(w, side, (w * 3 + 15) // 16 * 16, rw, rh, cx=cx, cy=cy)
        p = _plan(e)
        first, cnt, _ = capi.axis_taps(w, rw)
        assert p["wave"] == 1 and p["kind"] == 2, (side, p)
        assert p["taps"] >= cnt.max(), (side, p)
    p = _plan(_entry(4032, 3024, 4032 * 3, 341, 256, cx=58, cy=16))
    assert (p["taps"], p["dmax"], p["p"], p["nstrips"]) == (24, 12, 8, 6)
    p = _plan(_entry(6000, 4000, 6000 * 3, 384, 256, cx=80, cy=16))
    assert (p["taps"], p["dmax"]) == (32, 16)


def test_round6_knobs_and_counters_without_a_device():
    """ABI 6 (host side, no GPU call): MXD_TUNE_LOAD_POLICY and
    MXD_TUNE_DEVICE_TIMING are knobs (set returns the previous value, an
    unknown knob -1), mxd_device_stats reads and resets, and
    mxd_copy_bandwidth_policy refuses bad arguments with the ABI's status."""
    for knob in (capi.MXD_TUNE_LOAD_POLICY, capi.MXD_TUNE_DEVICE_TIMING, capi.MXD_TUNE_F32_LINK):
        assert capi.set_tuning(knob, 2) == 0
        assert capi.set_tuning(knob, 0) == 2
    assert capi.lib().mxd_set_tuning(capi.MXD_TUNE_F32_LINK + 1, 0) == -1  # MXD_TUNE_COUNT
    assert capi.device_stats(reset=True) == {"chunks": 0, "device_s": 0.0}
    g = ctypes.c_float()
    assert capi.lib().mxd_copy_bandwidth_policy(ctypes.c_size_t(1 << 20), 0, 1, 3, ctypes.byref(g)) == capi.MXD_ERR_INVALID
    assert capi.lib().mxd_copy_bandwidth_policy(ctypes.c_size_t(8), 0, 1, 0, ctypes.byref(g)) == capi.MXD_ERR_INVALID
