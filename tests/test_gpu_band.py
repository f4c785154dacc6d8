"""GPU: the band kernel (mlx-data_amd/csrc/band.hip -- persistent workgroups
streaming image bands' source rows into LDS by LDS-DMA; MXD_POLICY_PREFER_BAND
selects it where a wave kernel also fits, and it is the default past the wave
kernels' buckets) gives the bytes the wave kernels give (MXD_POLICY_NO_BAND)
on the same inputs: both sum each output
row's vertical taps in tap order from 0 and each pixel's horizontal taps the
same way, then encode like stbir (core/image/ImageTransform.cpp:41-62).  Cases
cover the band kernel's classes (upsampling .. 12 MP sources), strips, crops
at every edge, mirrored crops, odd source bases, ragged batches and the
tuning knobs (band height, lookahead), which must never change a byte."""
import numpy as np
import pytest

import oracle as O
from gpu_util import center_geom, compare, oracle_out, run_device, synth
from mlx_data_amd import capi

pytestmark = pytest.mark.gpu


def _with(policy, fn):
    prev = capi.set_kernel_policy(policy)
    try:
        return fn()
    finally:
        capi.set_kernel_policy(prev)


def _band_and_wave(imgs, geoms, **kw):
    band = _with(capi.MXD_POLICY_PREFER_BAND, lambda: run_device(imgs, geoms, **kw))
    wave = _with(capi.MXD_POLICY_NO_BAND, lambda: run_device(imgs, geoms, **kw))
    return band, wave


def _entry(img, g, f32, stride=None):
    rw, rh, cx, cy, cw, ch, flip = g
    h, w, c = img.shape
    return dict(src_w=w, src_h=h, src_stride=stride or (w * c + 15) // 16 * 16, channels=c, resize_w=rw,
                resize_h=rh, crop_x=cx, crop_y=cy, crop_w=cw, crop_h=ch, flip=flip,
                dst_stride=cw * c * (4 if f32 else 1))


def _assert_band_planned(imgs, geoms, f32):
    for img, g in zip(imgs, geoms):
        p = capi.describe_band_plan(_entry(img, g, f32), capi.MXD_F32_DIV255 if f32 else capi.MXD_U8)
        assert p["band"] == 1, (img.shape, g, p)


SIZES = [(960, 1280), (375, 500), (500, 333), (480, 640), (720, 1280), (1080, 1920), (1440, 2560), (2160, 3840),
         (200, 300), (300, 300)]


@pytest.mark.parametrize("f32", [False, True])
def test_center_crops_all_classes(f32):
    imgs = [synth(h, w, 3, 40 + i) for i, (h, w) in enumerate(SIZES)]
    geoms = [center_geom(i) for i in imgs]
    _assert_band_planned(imgs, geoms, f32)
    band, wave = _band_and_wave(imgs, geoms, f32=f32)
    for img, g, b, w in zip(imgs, geoms, band, wave):
        assert np.array_equal(b.view(np.uint8), w.view(np.uint8)), (img.shape, g)
    for img, g, b in zip(imgs[:4], geoms[:4], band[:4]):
        q = np.round(b * 255).astype(np.uint8) if f32 else b
        m, frac = compare(q, oracle_out(img, g))
        assert m <= 1 and frac < 2e-3, (img.shape, m, frac)


def test_c5_edge_crops_and_mirror():
    """4K -> 512, 448 x 448 random crops at every edge, mirrored or not (two
    strips per row, class taps 10)."""
    img = synth(2160, 3840, 3, 7)
    tw, th = O.smallest_side_dims(3840, 2160, 512)
    geoms = [(tw, th, x, y, 448, 448, f) for (x, y) in [(0, 0), (tw - 448, 0), (0, th - 448), (tw - 448, th - 448),
                                                        (231, 17)] for f in (0, 1)]
    imgs = [img] * len(geoms)
    _assert_band_planned(imgs, geoms, False)
    band, wave = _band_and_wave(imgs, geoms)
    for g, b, w in zip(geoms, band, wave):
        assert np.array_equal(b, w), g
    m, frac = compare(band[1], oracle_out(img, geoms[1]))
    assert m <= 1 and frac < 2e-3


@pytest.mark.parametrize("shift", [1, 2, 3])
def test_odd_source_base(shift):
    """Sources starting 1-3 bytes past a 4-byte boundary (random area crops
    hand the kernel such windows): realigned through the byte shift."""
    imgs = [synth(960, 1280, 3, 3), synth(500, 333, 3, 4)]
    geoms = [center_geom(i) for i in imgs]
    band, wave = _band_and_wave(imgs, geoms, base_shift=shift, f32=True)
    for b, w in zip(band, wave):
        assert np.array_equal(b.view(np.uint32), w.view(np.uint32))


def test_random_windows_and_sizes():
    """Arbitrary crop windows of arbitrary resizes (f3-style area crops, small
    and wide outputs, heights of 1-3 rows): identical bytes."""
    rng = np.random.default_rng(5)
    imgs, geoms = [], []
    for k in range(24):
        h, w = int(rng.integers(64, 1500)), int(rng.integers(64, 1500))
        rw, rh = int(rng.integers(32, 400)), int(rng.integers(8, 400))
        cw, ch = int(rng.integers(1, min(rw, 256) + 1)), int(rng.integers(1, rh + 1))
        cx, cy = int(rng.integers(0, rw - cw + 1)), int(rng.integers(0, rh - ch + 1))
        imgs.append(synth(h, w, 3, 100 + k))
        geoms.append((rw, rh, cx, cy, cw, ch, int(rng.integers(0, 2))))
    for f32 in (False, True):
        band, wave = _band_and_wave(imgs, geoms, f32=f32)
        for g, b, w in zip(geoms, band, wave):
            assert np.array_equal(b.view(np.uint8), w.view(np.uint8)), g


@pytest.mark.parametrize("rows,la,grid", [(1, 0, 0), (7, 0, 0), (224, 0, 0), (0, 1, 0), (0, 2, 0), (0, 8, 0),
                                          (13, 5, 0), (0, 0, 1), (3, 0, 1), (0, 3, 7), (5, 1, 2)])
def test_tuning_knobs_keep_bytes(rows, la, grid):
    """Band height, lookahead and the persistent grid (grid > 0: workgroups
    running streams of units, 7 and 2 make uneven streams) never change a byte."""
    imgs = [synth(960, 1280, 3, 1), synth(1080, 1920, 3, 2), synth(375, 500, 3, 9), synth(3024, 4032, 3, 12)]
    geoms = [center_geom(i) for i in imgs]
    pol = capi.set_kernel_policy(capi.MXD_POLICY_PREFER_BAND)
    want = run_device(imgs, geoms, f32=True)
    p0 = capi.set_tuning(capi.MXD_TUNE_BAND_ROWS, rows)
    p1 = capi.set_tuning(capi.MXD_TUNE_BAND_LA, la)
    p2 = capi.set_tuning(capi.MXD_TUNE_BAND_GRID, grid)
    try:
        got = run_device(imgs, geoms, f32=True)
    finally:
        capi.set_tuning(capi.MXD_TUNE_BAND_ROWS, p0)
        capi.set_tuning(capi.MXD_TUNE_BAND_LA, p1)
        capi.set_tuning(capi.MXD_TUNE_BAND_GRID, p2)
        capi.set_kernel_policy(pol)
    for g, w in zip(got, want):
        assert np.array_equal(g.view(np.uint32), w.view(np.uint32))


@pytest.mark.parametrize("h,w", [(3024, 4032), (4000, 6000), (4032, 3024), (6000, 8000)])
def test_large_downscale(h, w):
    """12 MP, 24 MP and 48 MP photos -> 256 -> 224 (11.8:1 .. 31:1; 24 .. 64
    taps per axis; an output row's new source rows span several groups):
    the default choice (the wave kernels' 24 / 32-tap scatter buckets up to
    16:1), the band kernel, the wave kernels at both lane widths and the
    general kernel against the kernel-order oracle, bit for bit."""
    img = synth(h, w, 3, 11)
    g = center_geom(img)
    if max(h, w) <= 6000:
        _assert_band_planned([img], [g], True)
        p = capi.describe_plan(_entry(img, g, True), capi.MXD_F32_DIV255)
        assert p["wave"] == 1 and p["kind"] == 2, p
    lut = (np.arange(256, dtype=np.uint8).astype("float32") / 255).view(np.uint32)
    want = lut[O.resize_crop_vfirst(img, g)]
    for pol in (capi.MXD_POLICY_AUTO, capi.MXD_POLICY_PREFER_BAND, capi.MXD_POLICY_NO_BAND,
                capi.MXD_POLICY_NARROW, capi.MXD_POLICY_NO_WAVE):
        got = _with(pol, lambda: run_device([img], [g], f32=True))[0]
        assert np.array_equal(got.view(np.uint32), want), pol


def test_constant_frames_exact():
    for v in (0, 1, 127, 254, 255):
        imgs = [np.full((960, 1280, 3), v, np.uint8), np.full((2160, 3840, 3), v, np.uint8)]
        out = run_device(imgs, [center_geom(i) for i in imgs])
        for o in out:
            assert (o == v).all(), v


@pytest.mark.parametrize("shift,f32", [(0, True), (1, False), (2, True), (3, False)])
def test_large_ratio_windows_mirrors_and_shifts(shift, f32):
    """12 MP and 24 MP photos through the 24 / 32-tap wave buckets (and every
    other kernel) with random crop windows of the 256-resize, mirrors, and
    sources 1-3 bytes past a 4-byte boundary (the realigning kernel
    variants): bit-exact to the kernel-order oracle."""
    rng = np.random.default_rng(100 + shift)
    imgs, geoms = [], []
    for (h, w) in [(3024, 4032), (4000, 6000), (4032, 3024)]:
        img = synth(h, w, 3, int(rng.integers(0, 1000)))
        rw, rh = O.smallest_side_dims(w, h, 256)
        cw, ch = int(rng.integers(32, min(rw, 300) + 1)), int(rng.integers(16, rh + 1))
        imgs.append(img)
        geoms.append((rw, rh, int(rng.integers(0, rw - cw + 1)), int(rng.integers(0, rh - ch + 1)), cw, ch,
                      int(rng.integers(0, 2))))
    lut = (np.arange(256, dtype=np.uint8).astype("float32") / 255).view(np.uint32)
    want = [O.resize_crop_vfirst(i, g) for i, g in zip(imgs, geoms)]
    for pol in (capi.MXD_POLICY_AUTO, capi.MXD_POLICY_NARROW, capi.MXD_POLICY_PREFER_BAND):
        outs = _with(pol, lambda: run_device(imgs, geoms, f32=f32, base_shift=shift))
        for o, wv, g in zip(outs, want, geoms):
            if f32:
                assert np.array_equal(o.view(np.uint32), lut[wv]), (pol, g)
            else:
                assert np.array_equal(o, wv), (pol, g)
