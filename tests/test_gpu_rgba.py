"""GPU: 4-channel images (`(stbir_pixel_layout)c` with
c = 4 = STBIR_RGBA at core/image/ImageTransform.cpp:49-58).

A resize is alpha-weighted: colours are premultiplied by alpha for filtering
and divided by the filtered alpha after it.  This follows SURVEY.md Appendix
A item 9, restated in the oracle in stbir's float operations -- stb is absent,
so the weighting itself is parity unpinned.  The GPU is bit-exact to the
kernel-order restatement (orc_resize_crop_vfirst_rgba: decode, weight,
vertical then horizontal pass, x 1/alpha, unfused v * 255 + 0.5) and within
+-1 of stbir's horizontal-first order (orc_resize_u8_layout).
A crop or flip without a resize is array::sub / hflip in the reference (no
stbir): bit-exact copies, transparent pixels keep their colour."""
import numpy as np
import pytest

import oracle as O
from gpu_util import compare, oracle_out, run_device, synth

pytestmark = pytest.mark.gpu


def rgba(h, w, seed, holes=True):
    img = synth(h, w, 4, seed)
    if holes:
        a = img[:, :, 3]
        a[: h // 3, : w // 3] = 0          # fully transparent block
        a[h // 2:, w // 2:] //= 4           # faint region
        a[:, ::7] = 255
    return img


@pytest.mark.parametrize("f32,src_align", [(False, 16), (True, 16), (False, 1), (True, 1)])
def test_rgba_resize_alpha_weighted(f32, src_align):
    imgs = [rgba(200, 300, 1), rgba(375, 500, 2), rgba(960, 1280, 3), rgba(61, 47, 4), rgba(90, 70, 5)]
    geoms = []
    for k, im in enumerate(imgs):
        h, w = im.shape[:2]
        tw, th = O.smallest_side_dims(w, h, 64 if k < 4 else 160)  # the last one upsamples
        cw, ch = min(tw, 56), min(th, 56)
        geoms.append((tw, th, (tw - cw) // 2, (th - ch) // 2, cw, ch, k % 2))
    outs = run_device(imgs, geoms, f32=f32, rgba_weighted=1, src_align=src_align)
    lut = (np.arange(256, dtype=np.uint8).astype("float32") / 255).view(np.uint32)
    for im, g, o in zip(imgs, geoms, outs):
        ref = oracle_out(im, g)
        if f32:
            q = np.round(o * 255).astype(np.uint8)
            assert np.array_equal(o.view(np.uint32), lut[q])
            o = q
        assert np.array_equal(o, O.resize_crop_vfirst_rgba(im, g)), g
        m, frac = compare(o, ref)
        assert m <= 1 and frac < 5e-3, (g, m, frac)
        # colour under zero alpha is not the unweighted colour
        if (ref[:, :, 3] == 0).any():
            unweighted = oracle_out(im, g, rgba_weighted=False)
            assert not np.array_equal(ref, unweighted)


def test_rgba_crop_and_flip_are_exact_copies():
    img = rgba(120, 90, 7)
    h, w = img.shape[:2]
    geoms = [(w, h, 5, 9, 60, 70, 0), (w, h, 0, 0, w, h, 1), (w, h, 30, 50, 60, 70, 1)]
    outs = run_device([img] * 3, geoms, rgba_weighted=0)
    for g, o in zip(geoms, outs):
        rw, rh, cx, cy, cw, ch, flip = g
        want = img[cy:cy + ch, cx:cx + cw]
        assert np.array_equal(o, want[:, ::-1] if flip else want)


def test_rgba_through_operator_surface():
    """(H, W, 4) through the pipeline: resize -> alpha-weighted, crop / flip
    alone -> exact (those ops used to reject RGBA)."""
    from mlx_data_amd import data as dx

    img = rgba(80, 100, 9)
    b = dx.buffer_from_vector([dict(image=img)])
    crop = b.image_center_crop("image", 50, 40)[0]["image"]
    assert np.array_equal(crop, img[20:60, 25:75])
    dx.set_state(3)
    flipped = b.image_random_h_flip("image", 1.0)[0]["image"]
    assert np.array_equal(flipped, img[:, ::-1])
    rs = b.image_resize_smallest_side("image", 40)[0]["image"]
    ref = O.resize(img, *O.smallest_side_dims(100, 80, 40))
    m, frac = compare(rs, ref)
    assert rs.shape == ref.shape and m <= 1 and frac < 5e-3
    # a same-size resize still runs stbir: transparent colour goes to 0
    same = b.image_resize("image", 100, 80)[0]["image"]
    ref = O.resize(img, 100, 80)
    clear = img[:, :, 3] == 0
    assert clear.any() and (ref[clear][:, :3] == 0).all() and np.array_equal(ref[~clear], img[~clear])
    assert np.array_equal(same, ref)
