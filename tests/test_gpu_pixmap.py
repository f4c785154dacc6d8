"""GPU parity of the pixel-map kernels (csrc/pixmap.hip), SURVEY.md §8f row f4:
rotate (core::image::rotate -> affine, ImageTransform.cpp:75-121) and
channel_reduction (:142-180), through the C ABI (mxd_pixmap_batch /
mxd_pixmap_host) and through the operator surface (image_rotate,
image_channel_reduction).  Integer / byte work: bit-exact to the oracle and to
tests/golden/pixmap.npz.
"""
import os

import numpy as np
import pytest

import oracle as O
from mlx_data_amd import capi

pytestmark = pytest.mark.gpu

GOLD = np.load(os.path.join(os.path.dirname(__file__), "golden", "pixmap.npz"))


def run_device(jobs, src_align=16, dst_pad=0):
    """jobs: list of (img, op, params, dst_w, dst_h).  One launch for all."""
    pitches, offs, total = [], [], 0
    for img, *_ in jobs:
        h, w, c = img.shape
        p = (w * c + src_align - 1) // src_align * src_align
        pitches.append(p)
        offs.append(total)
        total += (p * h + 255) // 256 * 256
    src = capi.DeviceBuffer(total + 256)
    host = np.zeros(total, np.uint8)
    for (img, *_), p, o in zip(jobs, pitches, offs):
        h, w, c = img.shape
        host[o:o + p * h].reshape(h, p)[:, :w * c] = img.reshape(h, w * c)
    src.upload(host)
    ops = {j[1] for j in jobs}
    assert len(ops) == 1
    outs, entries = [], []
    for (img, op, params, dw, dh), p, o in zip(jobs, pitches, offs):
        h, w, c = img.shape
        oc = c if op == capi.MXD_AFFINE else 1
        dp = dw * oc + dst_pad
        d = capi.DeviceBuffer(dp * dh + 16)
        d.memset(7)
        outs.append((d, dp, dw, dh, oc))
        entries.append(dict(src=src.ptr + o, src_stride=p, src_w=w, src_h=h, channels=c, dst_w=dw, dst_h=dh,
                            dst=d.ptr, dst_stride=dp, params=params))
    arr, n = capi.make_pixmaps(entries)
    capi.pixmap_batch(arr, n, ops.pop())
    res = []
    for d, dp, dw, dh, oc in outs:
        flat = d.download((dp * dh,), np.uint8)
        res.append(flat.reshape(dh, dp)[:, :dw * oc].reshape(dh, dw, oc).copy())
        d.free()
    src.free()
    return res


def rotate_job(img, angle, crop):
    mx, tw, th = capi.rotate_geometry(img.shape[1], img.shape[0], angle, crop)
    return (img, capi.MXD_AFFINE, mx, tw, th)


def gray_job(img, preset):
    return (img, capi.MXD_CHANNEL_REDUCTION, capi.channel_reduction_preset(preset), img.shape[1], img.shape[0])


@pytest.mark.parametrize("src_align,dst_pad", [(16, 0), (1, 0), (1, 3), (4, 1)])
def test_rotate_batch_bit_exact(src_align, dst_pad):
    rng = np.random.default_rng(11)
    jobs, want = [], []
    shapes = [(37, 53, 3), (64, 48, 1), (21, 30, 4), (17, 17, 2), (240, 320, 3), (5, 3, 3)]
    for i, shp in enumerate(shapes):
        img = rng.integers(0, 256, shp, dtype=np.uint8)
        for a, crop in [(0.0, True), (17.5, False), (90.0, False), (-45.0, True), (333.0, False)]:
            jobs.append(rotate_job(img, a + i, crop))
            want.append(O.rotate(img, a + i, crop))
    got = run_device(jobs, src_align, dst_pad)
    for k, (g, w) in enumerate(zip(got, want)):
        assert g.shape == w.shape and np.array_equal(g, w), k


@pytest.mark.parametrize("src_align,dst_pad", [(16, 0), (1, 0), (1, 2)])
def test_channel_reduction_batch_bit_exact(src_align, dst_pad):
    rng = np.random.default_rng(12)
    jobs, want = [], []
    for shp, preset in [((37, 53, 3), "default"), ((480, 640, 3), "rec709"), ((7, 5, 3), "rec2020"),
                        ((1, 1, 3), "green"), ((256, 341, 3), "rec601")]:
        img = rng.integers(0, 256, shp, dtype=np.uint8)
        jobs.append(gray_job(img, preset))
        want.append(O.channel_reduction(img, preset))
    got = run_device(jobs, src_align, dst_pad)
    for g, w in zip(got, want):
        assert np.array_equal(g, w)


def test_large_frames():
    rng = np.random.default_rng(13)
    img = rng.integers(0, 256, (1080, 1920, 3), dtype=np.uint8)
    (g,) = run_device([rotate_job(img, 30.0, False)])
    assert np.array_equal(g, O.rotate(img, 30.0, False))
    (g,) = run_device([gray_job(img, "default")])
    assert np.array_equal(g, O.channel_reduction(img, "default"))


def test_golden_fixtures_host_path():
    for name in GOLD.files:
        if name.startswith("in_"):
            continue
        kind, k, arg = name.split("_", 2)
        img = GOLD[f"in_{k}"]
        if kind == "gray":
            job = gray_job(img, arg)
            oc = 1
        else:
            job = rotate_job(img, float(arg), kind == "rotc")
            oc = img.shape[2]
        _, op, params, dw, dh = job
        out = np.full((dh, dw, oc), 7, np.uint8)
        arr, n = capi.make_pixmaps([dict(src=img.ctypes.data, src_stride=img.shape[1] * img.shape[2],
                                         src_w=img.shape[1], src_h=img.shape[0], channels=img.shape[2], dst_w=dw,
                                         dst_h=dh, dst=out.ctypes.data, dst_stride=dw * oc, params=params)])
        capi.pixmap_host(arr, n, op)
        assert np.array_equal(out, GOLD[name]), name


def test_errors():
    img = np.zeros((4, 4, 1), np.uint8)
    out = np.zeros((4, 4, 1), np.uint8)
    arr, n = capi.make_pixmaps([dict(src=img.ctypes.data, src_stride=4, src_w=4, src_h=4, channels=1, dst_w=4,
                                     dst_h=4, dst=out.ctypes.data, dst_stride=4, params=[0, 1, 0, 0])])
    with pytest.raises(capi.MxdError, match="expected a 3 channel uint8 array"):
        capi.pixmap_host(arr, n, capi.MXD_CHANNEL_REDUCTION)


def test_pipeline_rotate_and_gray():
    from mlx_data_amd import data as dx

    rng = np.random.default_rng(14)
    imgs = [rng.integers(0, 256, s, dtype=np.uint8) for s in [(200, 300, 3), (375, 500, 3), (64, 64, 3)]]
    b = dx.buffer_from_vector([dict(image=i) for i in imgs])
    r = b.image_rotate("image", 30.0, output_key="r").image_channel_reduction("image", "rec709", output_key="g")
    for k, img in enumerate(imgs):
        s = r[k]
        assert np.array_equal(np.asarray(s["r"]), O.rotate(img, 30.0, False))
        assert np.array_equal(np.asarray(s["g"]), O.channel_reduction(img, "rec709"))
    # rotate after a pending resize + crop plan: the plan materialises first
    c = b.image_resize_smallest_side("image", 256).image_center_crop("image", 224, 224).image_rotate("image", 45.0, True)
    base = np.asarray(b.image_resize_smallest_side("image", 256).image_center_crop("image", 224, 224)[0]["image"])
    got = np.asarray(c[0]["image"])
    assert np.array_equal(got, O.rotate(base, 45.0, True))


def test_functional_batch_api():
    from mlx_data_amd import image

    rng = np.random.default_rng(15)
    imgs = [rng.integers(0, 256, s, dtype=np.uint8) for s in [(37, 53, 3), (64, 48, 3), (120, 90, 3)]]
    for a, crop in [(30.0, False), (-12.5, True)]:
        for got, img in zip(image.rotate(imgs, a, crop), imgs):
            assert np.array_equal(got, O.rotate(img, a, crop))
    for got, img in zip(image.channel_reduction(imgs, "rec2020"), imgs):
        assert np.array_equal(got, O.channel_reduction(img, "rec2020"))
