"""GPU: the geometries whose outputs reach the resize's borders (VERDICT r1
weak 1), against the oracle -- itself cross-checked on whole frames by three
independent statements of clamp-edge resampling in
tests/test_border_evidence.py -- and against the float64 restatement
directly.

- C5: 3840x2160 -> 910x512, random_crop 448 lands anywhere, including x = 0,
  y = 0, x = W' - 448 and y = H' - 448 (with and without the mirror).
- f3: random_area_crop -> image_resize(224, 224) keeps the WHOLE resized
  frame; here whole frames of crop windows of several shapes.
- Constant frames: exactly the constant on every output pixel (u8 and f32).
Anchor: /root/reference/mlx/data/core/image/ImageTransform.cpp:49-60."""
import numpy as np
import pytest

import oracle as O
import stbir_f64 as F
from gpu_util import compare, oracle_out, run_device, synth

pytestmark = pytest.mark.gpu


def rand(h, w, c, seed):
    return np.random.default_rng(seed).integers(0, 256, (h, w, c), dtype=np.uint8)


@pytest.mark.parametrize("flip", [0, 1])
def test_c5_crops_at_frame_edges(flip):
    img = rand(2160, 3840, 3, 3)
    origins = [(0, 0), (462, 64), (0, 64), (462, 0), (231, 32), (1, 63)]
    geoms = [(910, 512, x, y, 448, 448, flip) for x, y in origins]
    outs = run_device([img] * len(geoms), geoms)
    full = O.resize(img, 910, 512)
    f64 = F.resize(img, 910, 512)
    for g, o in zip(geoms, outs):
        x, y = g[2], g[3]
        want = full[y:y + 448, x:x + 448]
        want = want[:, ::-1] if flip else want
        m, frac = compare(o, want)
        assert m <= 1 and frac < 1e-3, (g, m, frac)
        w64 = f64[y:y + 448, x:x + 448]
        m, frac = compare(o, w64[:, ::-1] if flip else w64)
        assert m <= 1 and frac < 2e-3, (g, m, frac)


# whole frames: (src h, src w) -> (dst w, dst h)
FRAMES = [((512, 731), (224, 224)), ((203, 97), (224, 224)), ((960, 1280), (224, 224)), ((333, 500), (224, 224)),
          ((200, 300), (384, 256)), ((375, 500), (341, 256)), ((999, 1000), (1000, 999)), ((3, 7), (5, 9)),
          ((5, 1), (3, 2)), ((65, 129), (64, 130))]


@pytest.mark.parametrize("f32", [False, True])
def test_whole_frames_f3_and_odd_shapes(f32):
    imgs = [rand(h, w, 3, 11 + k) for k, ((h, w), _) in enumerate(FRAMES)]
    geoms = [(dw, dh, 0, 0, dw, dh, k % 2) for k, (_, (dw, dh)) in enumerate(FRAMES)]
    outs = run_device(imgs, geoms, f32=f32)
    lut = (np.arange(256, dtype=np.uint8).astype(np.float32) / 255).view(np.uint32)
    for img, g, o in zip(imgs, geoms, outs):
        if f32:
            q = np.round(o * 255).astype(np.uint8)
            assert np.array_equal(o.view(np.uint32), lut[q])
            o = q
        ref = oracle_out(img, g)
        m, frac = compare(o, ref)
        assert m <= 1 and (frac < 2e-3 or ref.size < 4096), (g, m, frac)
        f64 = F.resize(img, g[0], g[1])
        m, _ = compare(o, f64[:, ::-1] if g[6] else f64)
        assert m <= 1, g


@pytest.mark.parametrize("f32", [False, True])
def test_constant_frames_exact_everywhere(f32):
    shapes = [((960, 1280), (341, 256)), ((200, 300), (384, 256)), ((2160, 3840), (910, 512)), ((3, 7), (5, 9)),
              ((512, 731), (224, 224))]
    values = [0, 1, 128, 254, 255]
    imgs, geoms = [], []
    for k, ((h, w), (dw, dh)) in enumerate(shapes):
        for v in values:
            imgs.append(np.full((h, w, 3), v, np.uint8))
            geoms.append((dw, dh, 0, 0, dw, dh, 0))
    outs = run_device(imgs, geoms, f32=f32)
    for img, o in zip(imgs, outs):
        v = img[0, 0, 0]
        assert (o == (np.float32(v) / np.float32(255) if f32 else v)).all(), (img.shape, v)


def test_crop_window_borders_are_the_window_edges():
    """A crop-then-resize clamps at the crop window's edges, not the frame's
    (core::image::crop gives stbir a w x h view): a bright frame outside a
    dark window must not leak in."""
    frame = np.full((400, 600, 3), 255, np.uint8)
    frame[100:300, 150:450] = synth(200, 300, 3, 5)
    win = np.ascontiguousarray(frame[100:300, 150:450])
    from mlx_data_amd import data as dx

    b = dx.buffer_from_vector([dict(image=frame)])
    out = b.image_center_crop("image", 300, 200).image_resize("image", 224, 224)[0]["image"]
    ref = O.resize(win, 224, 224)
    m, frac = compare(out, ref)
    assert m <= 1 and frac < 2e-3
