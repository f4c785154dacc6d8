"""Pins the CPU oracle (oracle/) before it is trusted as the GPU parity checker.

* crop / batch / RNG draws: against the reference's OWN code (oracle/_ref, built
  from /root/reference/mlx/data/{Array,Sample}.cpp, core/{BatchShape,State}.cpp)
  live when present, and against the committed fixtures it produced.
* resize arithmetic (stb_image_resize2, absent from this image: parity unpinned
  by the reference): against two independent implementations of the same
  triangle filter -- torch antialiased bilinear (f32) and Pillow BILINEAR -- on
  the crop window the hot path keeps, tolerance +-1 per uint8 channel.
* normalize: numpy x.astype("float32") / 255 exactly (mlx_data.py:46).
"""
import hashlib
import os

import numpy as np
import pytest

import oracle as O

HERE = os.path.dirname(os.path.abspath(__file__))
GOLD = np.load(os.path.join(HERE, "golden", "golden.npz"))
NAMES = sorted(k[4:] for k in GOLD.files if k.startswith("img_"))


def synth(h, w, c, seed):
    rng = np.random.default_rng(seed)
    gh, gw = h // 16 + 2, w // 16 + 2
    grid = rng.integers(0, 256, (gh, gw, c)).astype(np.float32)
    yi = np.minimum((np.arange(h) * (gh - 1)) // max(1, h - 1), gh - 2)
    xi = np.minimum((np.arange(w) * (gw - 1)) // max(1, w - 1), gw - 2)
    f = grid[yi][:, xi] * 0.5 + grid[yi + 1][:, xi + 1] * 0.5
    f += rng.normal(0, 12, f.shape)
    return np.clip(f, 0, 255).astype(np.uint8)


@pytest.mark.parametrize("name", NAMES)
def test_golden_resize_crop_regression(name):
    img = GOLD[f"img_{name}"]
    got = O.resize_crop(img, 256, 224, 224)
    assert np.array_equal(got, GOLD[f"rc_{name}"])


@pytest.mark.parametrize("name", NAMES)
def test_golden_crop_matches_reference_array_sub(name):
    # the fixture's digest came from the reference's array::sub on the same window
    got = GOLD[f"rc_{name}"]
    assert hashlib.sha256(got.tobytes()).digest() == GOLD[f"refcrop_sha_{name}"].tobytes()


def test_crop_live_reference():
    if O.ref_lib() is None:
        pytest.skip("oracle/_ref not built")
    rng = np.random.default_rng(7)
    for _ in range(20):
        h, w = rng.integers(1, 90, 2)
        c = int(rng.integers(1, 5))
        img = rng.integers(0, 256, (h, w, c), dtype=np.uint8)
        cw, ch = int(rng.integers(1, w + 1)), int(rng.integers(1, h + 1))
        x, y = int(rng.integers(0, w - cw + 1)), int(rng.integers(0, h - ch + 1))
        assert np.array_equal(O.crop(img, x, y, cw, ch), O.ref_crop(img, x, y, cw, ch))


def test_batch_matches_reference():
    shapes = GOLD["refbatch_shapes"]
    crops = [GOLD["rc_caltech_200x300"], GOLD["rc_small_97x131"][:200, :210], GOLD["rc_tiny_48x64"][:150, :224]]
    assert [list(c.shape) for c in crops] == shapes.tolist()
    assert np.array_equal(O.batch(crops, 0), GOLD["refbatch"])
    if O.ref_lib() is not None:
        assert np.array_equal(O.ref_batch(crops, 0.0), GOLD["refbatch"])


def test_rng_draws_fixture_matches_live_reference():
    if O.ref_lib() is None:
        pytest.skip("oracle/_ref not built")
    xy, fl = O.ref_random_crop_flip(1234, [(910, 512)] * 64, 448, 448, 0.5)
    assert np.array_equal(xy, GOLD["rng_xy"]) and np.array_equal(fl, GOLD["rng_flip"])


def test_normalize_lut_exact():
    q = np.arange(256, dtype=np.uint8)
    assert np.array_equal(O.normalize(q).view(np.uint32), GOLD["lut"].view(np.uint32))
    assert np.array_equal((q.astype("float32") / 255).view(np.uint32), GOLD["lut"].view(np.uint32))


def test_identity_resize_is_exact():
    img = synth(37, 53, 3, 1)
    assert np.array_equal(O.resize(img, 53, 37), img)


def test_geometry_matches_reference_rules():
    # ImageResizeSmallestSide: scale by the smaller side; square uses h (op/ImageTransform.cpp:87-92)
    assert O.smallest_side_dims(1280, 960, 256) == (341, 256)
    assert O.smallest_side_dims(375, 500, 256) == (256, 341)
    assert O.smallest_side_dims(300, 200, 256) == (384, 256)
    assert O.smallest_side_dims(3840, 2160, 512) == (910, 512)
    assert O.smallest_side_dims(300, 300, 256) == (256, 256)
    assert O.center_crop_origin(341, 256, 224, 224) == (58, 16)
    assert O.center_crop_origin(384, 256, 224, 224) == (80, 16)
    with pytest.raises(ValueError):
        O.center_crop_origin(200, 256, 224, 224)


CROSS = [(960, 1280), (200, 300), (375, 500), (500, 375), (480, 640), (1080, 1920), (300, 300), (100, 150),
         (333, 500)]


@pytest.mark.parametrize("h,w", CROSS)
def test_resize_vs_torch_antialias(h, w):
    torch = pytest.importorskip("torch")
    F = torch.nn.functional
    img = synth(h, w, 3, h * 7 + w)
    tw, th = O.smallest_side_dims(w, h, 256)
    ours = O.resize(img, tw, th).astype(np.int32)
    t = torch.from_numpy(img.astype(np.float32) / 255).permute(2, 0, 1)[None]
    r = F.interpolate(t, size=(th, tw), mode="bilinear", align_corners=False, antialias=True)
    tq = np.clip(np.floor(r[0].permute(1, 2, 0).numpy() * 255 + 0.5), 0, 255).astype(np.int32)
    x, y = O.center_crop_origin(tw, th, 224, 224)
    d = np.abs(ours - tq)[y : y + 224, x : x + 224]
    assert d.max() <= 1
    assert (d > 0).mean() < 1e-3  # float-order noise only


@pytest.mark.parametrize("h,w", CROSS[:5])
def test_resize_vs_pillow_bilinear(h, w):
    Image = pytest.importorskip("PIL.Image")
    img = synth(h, w, 3, h * 5 + w)
    tw, th = O.smallest_side_dims(w, h, 256)
    ours = O.resize(img, tw, th).astype(np.int32)
    pil = np.asarray(Image.fromarray(img).resize((tw, th), Image.BILINEAR)).astype(np.int32)
    x, y = O.center_crop_origin(tw, th, 224, 224)
    assert np.abs(ours - pil)[y : y + 224, x : x + 224].max() <= 1


def test_vfirst_restatement_within_one_of_stbir_order():
    """The kernel-order restatement (vertical first, byte units, fmaf chains)
    differs from the stbir-order one only by f32 rounding: +-1, rarely."""
    rng = np.random.default_rng(4)
    for (h, w, rw, rh, cx, cy, cw, ch) in [(96, 128, 43, 32, 5, 3, 30, 28), (50, 75, 96, 64, 10, 4, 56, 56),
                                          (210, 380, 45, 25, 0, 0, 45, 25)]:
        img = rng.integers(0, 256, (h, w, 3), dtype=np.uint8)
        a = O.resize_crop_vfirst(img, (rw, rh, cx, cy, cw, ch, 0))
        b = O.crop(O.resize(img, rw, rh), cx, cy, cw, ch)
        d = np.abs(a.astype(int) - b.astype(int))
        assert d.max() <= 1 and (d > 0).mean() < 0.01
        m = O.resize_crop_vfirst(img, (rw, rh, cx, cy, cw, ch, 1))
        assert np.array_equal(m, a[:, ::-1])


def test_rgba_kernel_order_within_one_of_stbir_order():
    """The STBIR_RGBA kernel-order restatement (vertical pass first, what the
    general HIP kernel reproduces bit for bit) stays within +-1 of the
    horizontal-first stbir-order restatement on whole windows, transparent
    and faint regions included; crops of a same-size resize are unchanged
    where alpha is opaque."""
    rng = np.random.default_rng(5)
    for k in range(6):
        h, w = int(rng.integers(20, 300)), int(rng.integers(20, 300))
        img = rng.integers(0, 256, (h, w, 4), dtype=np.uint8)
        img[: h // 3, : w // 3, 3] = 0
        img[h // 2:, w // 2:, 3] //= 4
        rw, rh = int(rng.integers(8, 200)), int(rng.integers(8, 200))
        cw, ch = int(rng.integers(1, rw + 1)), int(rng.integers(1, rh + 1))
        g = (rw, rh, int(rng.integers(0, rw - cw + 1)), int(rng.integers(0, rh - ch + 1)), cw, ch, k % 2)
        a = O.resize_crop_vfirst_rgba(img, g)
        r = O.crop(O.resize(img, rw, rh, True), g[2], g[3], cw, ch)
        if g[6]:
            r = r[:, ::-1]
        d = np.abs(a.astype(int) - r.astype(int))
        assert d.max() <= 1 and (d > 0).mean() < 5e-3, (g, d.max(), (d > 0).mean())
