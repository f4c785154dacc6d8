"""GPU parity: the HIP path (through the C ABI) against the CPU oracle on the
same seeded inputs.  Bar (BASELINE.json north_star): crop geometry exact,
resize within +-1 per uint8 channel; the f32 output is bit-exact q/255.0f of
the kernel's own uint8 result.  Mismatch fractions are asserted small too, so
a systematic +-1 bias cannot hide under the tolerance."""
import os

import numpy as np
import pytest

import oracle as O
from gpu_util import center_geom, compare, oracle_out, run_device, synth
from mlx_data_amd import capi

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))
GOLD = np.load(os.path.join(HERE, "golden", "golden.npz"))
LUT = GOLD["lut"]
MAX_FRAC = 2e-3  # fraction of channels allowed to differ by exactly 1


def check(gpu, ref, frac=MAX_FRAC):
    m, f = compare(gpu, ref)
    assert m <= 1, f"max diff {m}"
    assert f <= frac, f"{f:.5f} of values differ by 1"


def test_device_present():
    assert capi.device_count() >= 1


@pytest.mark.parametrize("name", sorted(k[4:] for k in GOLD.files if k.startswith("img_")))
def test_golden_u8_and_f32(name):
    img = GOLD[f"img_{name}"]
    g = center_geom(img)
    u8 = run_device([img], [g])[0]
    check(u8, GOLD[f"rc_{name}"])
    f32 = run_device([img], [g], f32=True)[0]
    assert np.array_equal(f32.view(np.uint32), LUT[u8].view(np.uint32))


def test_c2_1280x960_batch():
    imgs = [synth(960, 1280, 3, s) for s in range(6)]
    geoms = [center_geom(i) for i in imgs]
    assert geoms[0] == (341, 256, 58, 16, 224, 224, 0)
    outs = run_device(imgs, geoms)
    for img, g, o in zip(imgs, geoms, outs):
        check(o, oracle_out(img, g))
    f32 = run_device(imgs, geoms, f32=True)
    for o, f in zip(outs, f32):
        assert np.array_equal(f.view(np.uint32), LUT[o].view(np.uint32))


def test_4k_resize_256_and_512_random_crop_flip():
    img = synth(2160, 3840, 3, 99)
    check(run_device([img], [center_geom(img)])[0], oracle_out(img, center_geom(img)))
    # config 5: resize 512 -> random_crop 448 -> hflip(0.5), draws from the reference's RNG (fixture)
    tw, th = O.smallest_side_dims(3840, 2160, 512)
    geoms = [(tw, th, int(x), int(y), 448, 448, int(f)) for (x, y), f in zip(GOLD["rng_xy"][:4], GOLD["rng_flip"][:4])]
    assert any(g[6] for g in geoms) and not all(g[6] for g in geoms)
    outs = run_device([img] * 4, geoms)
    for g, o in zip(geoms, outs):
        check(o, oracle_out(img, g))


def test_ragged_mixed_resolution_batch():
    sizes = [(480, 640), (720, 1280), (960, 1280), (1080, 1920), (1440, 2560), (2160, 3840), (375, 500), (500, 375),
             (200, 300), (333, 500)]
    imgs = [synth(h, w, 3, i) for i, (h, w) in enumerate(sizes)]
    geoms = [center_geom(i) for i in imgs]
    outs = run_device(imgs, geoms)
    for img, g, o in zip(imgs, geoms, outs):
        check(o, oracle_out(img, g))


@pytest.mark.parametrize("f32", [False, True])
def test_mixed_row_alignment_batch(f32):
    """Tightly packed rows: 500- and 1280-wide rows stay 4-byte aligned, 375-
    and 333-wide rows do not -- one call, split between the wave and the
    general kernels by image."""
    sizes = [(375, 500), (500, 375), (500, 333), (960, 1280), (200, 333), (375, 500)]
    imgs = [synth(h, w, 3, 40 + i) for i, (h, w) in enumerate(sizes)]
    geoms = [center_geom(i) for i in imgs]
    outs = run_device(imgs, geoms, f32=f32, src_align=1)
    lut = (np.arange(256, dtype=np.uint8).astype("float32") / 255).view(np.uint32)
    for img, g, o in zip(imgs, geoms, outs):
        ref = oracle_out(img, g)
        if f32:
            q = np.rint(o * 255).astype(np.uint8)
            assert np.array_equal(o.view(np.uint32), lut[q])
            check(q, ref)
        else:
            check(o, ref)


@pytest.mark.parametrize("c", [1, 2, 3])
def test_channels_and_unaligned_rows(c):
    img = synth(301, 457, c, c)  # odd width: rows not 16-byte aligned -> byte path
    g = center_geom(img)
    check(run_device([img], [g], src_align=1)[0], oracle_out(img, g))
    check(run_device([img], [g], src_align=16)[0], oracle_out(img, g))


@pytest.mark.parametrize("shape,geom", [
    ((1, 1, 3), (256, 256, 16, 16, 224, 224, 0)),          # 1x1 upsample
    ((256, 256, 3), (256, 256, 16, 16, 224, 224, 0)),      # identity axis -> exact crop
    ((200, 300, 3), (384, 256, 0, 0, 384, 256, 0)),        # whole resized image: borders in the window
    ((960, 1280, 3), (341, 256, 0, 0, 341, 256, 1)),       # whole image, flipped
    ((64, 48, 3), (7, 9, 3, 4, 1, 1, 0)),                  # 1x1 output
    ((97, 131, 3), (1000, 740, 3, 5, 997, 731, 0)),        # big upsample, odd sizes
    ((50, 2000, 3), (5120, 128, 0, 0, 5120, 128, 0)),      # very wide output: many strips
])
def test_edge_geometries(shape, geom):
    img = synth(*shape, seed=sum(shape))
    out = run_device([img], [geom])[0]
    check(out, oracle_out(img, geom))
    if shape == (256, 256, 3):
        assert np.array_equal(out, img[16:240, 16:240])


def test_padded_dst_stride_and_host_path():
    imgs = [synth(375, 500, 3, 5), synth(500, 375, 3, 6)]
    geoms = [center_geom(i) for i in imgs]
    padded = run_device(imgs, geoms, dst_pad=37)
    host = capi  # host-resident convenience path
    from mlx_data_amd import image

    hout = image.resize_crop(imgs, geoms)
    for p, h, img, g in zip(padded, hout, imgs, geoms):
        assert np.array_equal(p, h)
        check(h, oracle_out(img, g))
    hf = image.resize_crop(imgs, geoms, out_dtype="float32")
    for h, f in zip(hout, hf):
        assert np.array_equal(f.view(np.uint32), LUT[h].view(np.uint32))
    del host


def test_full_size_c2_batch_properties():
    """BASELINE config 2 at full size: 256 x 1280x960 -> f32 224x224 in one launch.
    Size-independent checks: determinism, f32 == LUT[u8] everywhere, sampled
    images against the oracle."""
    n = 256
    rng = np.random.default_rng(0)
    imgs = [rng.integers(0, 256, (960, 1280, 3), dtype=np.uint8) for _ in range(n)]
    geoms = [center_geom(imgs[0])] * n
    u8 = run_device(imgs, geoms)
    u8b = run_device(imgs, geoms)
    f32 = run_device(imgs, geoms, f32=True)
    for a, b, f in zip(u8, u8b, f32):
        assert np.array_equal(a, b)
        assert np.array_equal(f.view(np.uint32), LUT[a].view(np.uint32))
    for i in (0, 77, 255):
        check(u8[i], oracle_out(imgs[i], geoms[i]))


def test_full_size_c3_mixed_batch_properties():
    """BASELINE config 3 at full size: 512 images of six resolutions (480p-4K,
    seed 1 like bench.py) -> 256 -> center 224 u8 in one call: one launch per
    kernel shape.  Checks: determinism, per-size constant images exact, and
    one image of every size against the oracle."""
    sizes = [(640, 480), (1280, 720), (1280, 960), (1920, 1080), (2560, 1440), (3840, 2160)]
    pick = np.random.default_rng(1).integers(0, len(sizes), 512)
    base = {s: synth(s[1], s[0], 3, 10 + k) for k, s in enumerate(sizes)}
    imgs = [base[sizes[k]] for k in pick]
    # every 16th image is a constant frame of its size
    for j in range(0, 512, 16):
        w, h = sizes[pick[j]]
        imgs[j] = np.full((h, w, 3), 37 + j % 200, np.uint8)
    geoms = [center_geom(im) for im in imgs]
    a = run_device(imgs, geoms)
    b = run_device(imgs, geoms)
    for x, y in zip(a, b):
        assert np.array_equal(x, y)
    for j in range(0, 512, 16):
        assert (a[j] == imgs[j][0, 0, 0]).all()
    done = set()
    for j, k in enumerate(pick):
        if k not in done and j % 16:
            check(a[j], oracle_out(imgs[j], geoms[j]))
            done.add(k)
    assert len(done) == len(sizes)


def test_full_size_c5_random_crop_flip_batch():
    """BASELINE config 5 at full size: 128 x 3840x2160 -> 512 -> random 448 +
    mirror (the bench's draws), u8, one launch; every 32nd frame against the
    oracle, all frames deterministic."""
    rng = np.random.default_rng(3)
    frame = synth(2160, 3840, 3, 5)
    imgs = [frame] * 128
    rw, rh = O.smallest_side_dims(3840, 2160, 512)
    geoms = [(rw, rh, int(rng.integers(0, rw - 448 + 1)), int(rng.integers(0, rh - 448 + 1)), 448, 448,
              int(rng.random() <= 0.5)) for _ in range(128)]
    a = run_device(imgs, geoms)
    b = run_device(imgs, geoms)
    full = O.resize(frame, rw, rh)
    for j, (x, y, g) in enumerate(zip(a, b, geoms)):
        assert np.array_equal(x, y)
        if j % 32 == 0:
            want = full[g[3]:g[3] + 448, g[2]:g[2] + 448]
            check(x, want[:, ::-1] if g[6] else want)
