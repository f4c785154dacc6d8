"""CPU tests of SURVEY.md §8f row f4 (rotate / affine, channel reduction).

Reference: core::image::affine / rotate / channel_reduction
(mlx/data/core/image/ImageTransform.cpp:75-121,142-180) and the op presets
(mlx/data/op/ImageTransform.cpp:362-421).  That file needs stb_image_resize2.h
and cannot be built here, so the oracle (oracle/stbir_oracle.c) is checked
against an independent numpy restatement of the same per-pixel arithmetic,
against the committed fixtures (tests/golden/pixmap.npz), and the product's
host-side geometry (mxd_rotate_geometry, mxd_channel_reduction_preset) against
the oracle bit for bit.  No GPU compute here.
"""
import os

import numpy as np
import pytest

import oracle as O
from mlx_data_amd import capi

GOLD = np.load(os.path.join(os.path.dirname(__file__), "golden", "pixmap.npz"))
ANGLES = (0.0, 1.0, 17.5, 30.0, 45.0, 90.0, -45.0, 135.0, 180.0, 270.0, 333.0, 359.9)


def np_affine(img, mx, tw, th):
    """Independent restatement of core::image::affine's inner loop
    (ImageTransform.cpp:94-107): float products/sums, `+ 0.5 + wh` in double,
    truncating int64 conversion, zero outside the source."""
    h, w, c = img.shape
    f = np.float32
    twh, thh, wh, hh = f(tw / 2.0), f(th / 2.0), f(w / 2.0), f(h / 2.0)
    ty, tx = np.meshgrid(np.arange(th), np.arange(tw), indexing="ij")
    fx = tx.astype(f) - twh
    fy = ty.astype(f) - thh
    sx = (mx[0] * fx + mx[1] * fy) + mx[2]
    sy = (mx[3] * fx + mx[4] * fy) + mx[5]
    x = ((sx.astype(np.float64) + 0.5) + np.float64(wh)).astype(np.int64)
    y = ((sy.astype(np.float64) + 0.5) + np.float64(hh)).astype(np.int64)
    ok = (x >= 0) & (y >= 0) & (x < w) & (y < h)
    out = np.zeros((th, tw, c), np.uint8)
    out[ok] = img[y[ok], x[ok]]
    return out


def np_channel_reduction(img, preset):
    bias, m = O.CHANNEL_PRESETS[preset]
    scale = np.float32(65536)
    mi = (np.array(m, np.float32) * scale).astype(np.int64)
    ib = int(np.float32(bias) * scale)
    v = img[..., 0].astype(np.int64) * mi[0] + img[..., 1] * mi[1] + img[..., 2] * mi[2] + ib
    q = np.sign(v) * (np.abs(v) // 65536)  # C integer division truncates toward zero
    return np.clip(q, 0, 255).astype(np.uint8)[..., None]


@pytest.mark.parametrize("shape", [(37, 53, 3), (64, 48, 1), (21, 30, 4), (17, 17, 2), (120, 200, 3)])
@pytest.mark.parametrize("crop", [False, True])
def test_oracle_affine_matches_numpy(shape, crop):
    img = np.random.default_rng(sum(shape)).integers(0, 256, shape, dtype=np.uint8)
    for a in ANGLES:
        mx, tw, th, bad = O.rotate_geometry(shape[1], shape[0], a, crop)
        assert not bad
        got = O.rotate(img, a, crop)
        assert got.shape == (th, tw, shape[2])
        assert np.array_equal(got, np_affine(img, mx, tw, th)), a


@pytest.mark.parametrize("preset", sorted(O.CHANNEL_PRESETS))
def test_oracle_channel_reduction_matches_numpy(preset):
    img = np.random.default_rng(5).integers(0, 256, (63, 91, 3), dtype=np.uint8)
    img[0, :8] = [[0, 0, 0], [255, 255, 255], [255, 0, 0], [0, 255, 0], [0, 0, 255], [1, 2, 3], [254, 255, 255], [128] * 3]
    assert np.array_equal(O.channel_reduction(img, preset), np_channel_reduction(img, preset))


def test_known_answers():
    img = np.random.default_rng(1).integers(0, 256, (9, 14, 3), dtype=np.uint8)
    # crop=True at 0 degrees is the identity
    assert np.array_equal(O.rotate(img, 0.0, True), img)
    # the reference sizes the uncropped output th = h|sin| + w|cos|
    # (ImageTransform.cpp:84-85), so 0 degrees on a 14x9 image gives 14x14
    assert O.rotate(img, 0.0, False).shape == (14, 14, 3)
    # "green" keeps the G channel exactly; white stays white under every preset
    assert np.array_equal(O.channel_reduction(img, "green")[..., 0], img[..., 1])
    white = np.full((2, 5, 3), 255, np.uint8)
    for p in ("default", "rec601", "rec709"):
        assert O.channel_reduction(white, p).max() <= 255


def test_golden_fixtures_reproduce():
    for k in "abcd":
        img = GOLD[f"in_{k}"]
        for name in GOLD.files:
            if name.startswith(f"rot_{k}_") or name.startswith(f"rotc_{k}_"):
                a = float(name.split("_")[2])
                assert np.array_equal(O.rotate(img, a, name.startswith("rotc")), GOLD[name]), name
            if name.startswith(f"gray_{k}_"):
                assert np.array_equal(O.channel_reduction(img, name.split("_", 2)[2]), GOLD[name]), name


@pytest.mark.parametrize("crop", [False, True])
def test_product_rotate_geometry_matches_oracle(crop):
    for (w, h) in [(1, 1), (53, 37), (1280, 960), (960, 1280), (3840, 2160), (7, 300)]:
        for a in ANGLES + (0.25, 89.999, 1e3, -720.0):
            mx, tw, th = capi.rotate_geometry(w, h, a, crop)
            omx, otw, oth, bad = O.rotate_geometry(w, h, a, crop)
            assert not bad
            assert np.array_equal(mx.view(np.uint32), omx.view(np.uint32)), (w, h, a)
            assert (tw, th) == (otw, oth), (w, h, a)


def test_product_presets():
    for name, (bias, m) in O.CHANNEL_PRESETS.items():
        p = capi.channel_reduction_preset(name)
        assert np.array_equal(p, np.array([bias, *m], np.float32)), name
    with pytest.raises(capi.MxdError, match="ImageChannelReduction: unable to find preset sepia"):
        capi.channel_reduction_preset("sepia")


def test_pipeline_ops_construct_and_check():
    from mlx_data_amd import data as dx

    b = dx.buffer_from_vector([dict(image=np.zeros((4, 4, 3), np.uint8))])
    with pytest.raises(RuntimeError, match="ImageChannelReduction: unable to find preset nope"):
        b.image_channel_reduction("image", "nope")
    b.image_rotate("image", 30.0)
    b.image_rotate("image", angle=30.0, crop=True, output_key="r")
    b.image_channel_reduction("image", preset="rec709", output_key="g")
    assert b.image_rotate_if(False, "image", 10.0) is b
    with pytest.raises(RuntimeError, match="expected a 3 channel uint8 array"):
        dx.buffer_from_vector([dict(image=np.zeros((4, 4, 1), np.uint8))]).image_channel_reduction("image")[0]


def test_video_channel_check_on_cpu():
    from mlx_data_amd import data as dx

    v = np.zeros((2, 4, 4, 5), np.uint8)
    with pytest.raises(RuntimeError, match="verifyVideo: channels must be 0 <= c <= 4"):
        dx.buffer_from_vector([dict(video=v)]).image_center_crop("video", 2, 2)[0]
