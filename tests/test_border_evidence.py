"""Independent evidence for the resize's border arithmetic.

stb_image_resize2 is absent, so the oracle (oracle/stbir_oracle.c) and the
product tap builder (csrc/taps.cpp) cannot be pinned to stbir itself.  What
this file adds is evidence that does not come from the same recollection:

1. oracle/stbir_f64.py -- a third restatement written from SURVEY.md
   Appendix A's text alone: float64, dense-then-sparse weight matrices,
   clamp folding by index clamping.
2. torch (``interpolate(bilinear, antialias=True)``) and Pillow (mode "F"
   BILINEAR) run on sources replicate-padded by in/gcd(in, out) pixels, with
   the output cropped back by out/gcd(in, out): replicate padding is the
   implementation-independent statement of STBIR_EDGE_CLAMP (every
   out-of-range tap reads the edge pixel), and at that pad the output grid
   lines up exactly with the unpadded one, so neither library's own border
   renormalisation is ever reached.

All three agree with the oracle on WHOLE frames, borders included, within
+-1 and with few nonzero differences; the GPU kernel is then held to the
oracle on border-reaching geometries in tests/test_gpu_border.py.  Still
unpinned (stbir-internal, not observable by any of these): the exact
renormalisation epsilon and the float32 casts of the scale (Appendix A items
1 and 6).  Anchor: /root/reference/mlx/data/core/image/ImageTransform.cpp:7-10,49-60."""
import math

import numpy as np
import pytest

import oracle as O
import stbir_f64 as F
from mlx_data_amd import capi

# (src w, src h, dst w, dst h): C1 upsample, C2, C4 shapes, C3 sizes, f3 area
# crop -> 224, non-integer up/down mixes, tiny frames, identity axes.
GEOMS = [
    (300, 200, 384, 256), (1280, 960, 341, 256), (500, 375, 341, 256), (375, 500, 256, 341),
    (500, 333, 384, 256), (640, 480, 341, 256), (1280, 720, 455, 256), (731, 512, 224, 224),
    (97, 203, 224, 224), (1000, 999, 999, 1000), (7, 3, 5, 9), (3, 7, 9, 5), (1, 5, 3, 2),
    (256, 300, 256, 200), (300, 256, 200, 256), (129, 65, 64, 130),
]


def rand(h, w, c, seed):
    return np.random.default_rng(seed).integers(0, 256, (h, w, c), dtype=np.uint8)


def border_mask(h, w, k=2):
    m = np.zeros((h, w), bool)
    m[:k] = m[-k:] = True
    m[:, :k] = m[:, -k:] = True
    return m


def stats(a, b):
    d = np.abs(a.astype(np.int32) - b.astype(np.int32))
    return int(d.max()), float((d > 0).mean()), d


def pads(n_in, n_out):
    g = math.gcd(n_in, n_out)
    return n_in // g, n_out // g  # source pad, output offset


def torch_clamp(img, dw, dh):
    import torch

    h, w, c = img.shape
    px, mx = pads(w, dw)
    py, my = pads(h, dh)
    t = torch.from_numpy(img.astype(np.float64) / 255.0).permute(2, 0, 1)[None]
    t = torch.nn.functional.pad(t, (px, px, py, py), mode="replicate")
    o = torch.nn.functional.interpolate(t, size=(dh + 2 * my, dw + 2 * mx), mode="bilinear", antialias=True,
                                        align_corners=False)
    return F.encode(o[0, :, my:my + dh, mx:mx + dw].permute(1, 2, 0).numpy())


def pillow_clamp(img, dw, dh):
    Image = pytest.importorskip("PIL.Image")
    h, w, c = img.shape
    px, mx = pads(w, dw)
    py, my = pads(h, dh)
    p = np.pad(img.astype(np.float32) / 255.0, ((py, py), (px, px), (0, 0)), mode="edge")
    planes = [np.asarray(Image.fromarray(p[:, :, k], mode="F").resize((dw + 2 * mx, dh + 2 * my), Image.BILINEAR))
              for k in range(c)]
    return F.encode(np.stack(planes, -1)[my:my + dh, mx:mx + dw].astype(np.float64))


def _gate(ref, other, dw, dh):
    m, frac, d = stats(ref, other)
    assert m <= 1, m
    if dw * dh >= 64 * 64:
        assert frac < 2e-3, frac
    return d


@pytest.mark.parametrize("w,h,dw,dh", GEOMS)
def test_f64_restatement_whole_frame(w, h, dw, dh):
    img = rand(h, w, 3, w * 7 + h)
    ref = O.resize(img, dw, dh)
    d = _gate(ref, F.resize(img, dw, dh), dw, dh)
    assert d[border_mask(dh, dw)].max() <= 1


@pytest.mark.parametrize("w,h,dw,dh", GEOMS)
def test_clamp_is_replicate_padding_torch(w, h, dw, dh):
    img = rand(h, w, 3, w * 5 + h)
    _gate(O.resize(img, dw, dh), torch_clamp(img, dw, dh), dw, dh)


@pytest.mark.parametrize("w,h,dw,dh", GEOMS)
def test_clamp_is_replicate_padding_pillow(w, h, dw, dh):
    img = rand(h, w, 3, w * 3 + h)
    _gate(O.resize(img, dw, dh), pillow_clamp(img, dw, dh), dw, dh)


def test_c5_frame_edges_f64():
    """C5 (3840x2160 -> 910x512), whose random 448 crops reach x = 0, y = 0
    and the far edges: the whole frame against the float64 restatement."""
    img = rand(2160, 3840, 3, 3)
    ref = O.resize(img, 910, 512)
    m, frac, d = stats(ref, F.resize(img, 910, 512))
    assert m <= 1 and frac < 1e-3
    for x, y in [(0, 0), (462, 64), (0, 64), (462, 0)]:
        assert d[y:y + 448, x:x + 448].max() <= 1


def test_edge_vs_interior_differs_from_renormalising_filters():
    """Sanity of the method: plain torch antialias (which renormalises over
    in-range taps instead of clamping) does differ at the border of a
    downsample with an edge gradient, so the agreement above is not vacuous."""
    import torch

    h, w = 240, 320
    edge = np.zeros((h, w, 3), np.uint8)
    edge[:, :2] = 255  # a bright 2-px stripe on the left border
    t = torch.from_numpy(edge.astype(np.float64) / 255).permute(2, 0, 1)[None]
    plain = F.encode(torch.nn.functional.interpolate(t, size=(64, 85), mode="bilinear", antialias=True,
                                                     align_corners=False)[0].permute(1, 2, 0).numpy())
    ref = O.resize(edge, 85, 64)
    assert np.abs(plain.astype(int) - ref).max() > 10  # 119 vs 136 at x = 0
    assert np.abs(torch_clamp(edge, 85, 64).astype(int) - ref).max() <= 1


@pytest.mark.parametrize("w,h,dw,dh", GEOMS)
@pytest.mark.parametrize("value", [0, 1, 128, 254, 255])
def test_constant_image_is_exact_everywhere(w, h, dw, dh, value):
    """Weights sum to 1 and the encode rounds: a constant frame stays that
    constant on every output pixel, borders included (oracle and f64)."""
    img = np.full((h, w, 3), value, np.uint8)
    assert (O.resize(img, dw, dh) == value).all()
    assert (F.resize(img, dw, dh) == value).all()


@pytest.mark.parametrize("n_in,n_out", sorted({(g[0], g[2]) for g in GEOMS} | {(g[1], g[3]) for g in GEOMS}))
def test_product_weights_sum_to_one(n_in, n_out):
    """Every output's weights (the product tables, float32) sum to 1 within
    float32 rounding, and cover only in-range source pixels (clamp folded)."""
    first, cnt, w = capi.axis_taps(n_in, n_out)
    sums = w.astype(np.float64).sum(axis=1)
    assert np.abs(sums - 1).max() < 1e-5
    assert first.min() >= 0 and (first + cnt).max() <= n_in
    # and the same matrix as the float64 restatement, up to the float32 scale
    # and weight arithmetic of Appendix A item 1 (a few 1e-6 per weight)
    dense = np.zeros((n_out, n_in))
    for j in range(n_out):
        dense[j, first[j]:first[j] + cnt[j]] = w[j, :cnt[j]]
    assert np.abs(dense - F.axis_matrix(n_in, n_out)).max() < 5e-5


@pytest.mark.parametrize("w,h", [(256, 300), (341, 256), (7, 3)])
def test_identity_axes_are_exact(w, h):
    """Item 10: out == in returns the bytes, per axis and on both."""
    img = rand(h, w, 3, w + h)
    assert np.array_equal(O.resize(img, w, h), img)
    assert np.array_equal(F.resize(img, w, h), img)
    # x identity: every row is resampled in y only
    assert np.array_equal(O.resize(img, w, 2 * h + 1)[:, 3 % w], O.resize(img[:, 3 % w:3 % w + 1], 1, 2 * h + 1)[:, 0])
