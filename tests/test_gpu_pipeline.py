"""GPU parity of the operator surface: mlx.data-style pipelines whose image ops
run as fused batch launches, checked image by image against the oracle
(resize: max |diff| <= 1 and < 0.2 % differing; crop / flip / batch layout /
f32 normalize: exact).  Reference anchors as in test_pipeline.py; the Caltech
stand-in follows benchmarks/comparative/caltech101/mlx_data.py:22-45.
"""
import os

import numpy as np
import pytest

import oracle as O
from gpu_util import compare, synth
from mlx_data_amd import data as dx

pytestmark = pytest.mark.gpu

GOLD = np.load(os.path.join(os.path.dirname(__file__), "golden", "golden.npz"))
MAX_FRAC = 2e-3


def oracle_center(img, size=256, cw=224, ch=224):
    h, w = img.shape[:2]
    tw, th = O.smallest_side_dims(w, h, size)
    x, y = O.center_crop_origin(tw, th, cw, ch)
    return O.crop(O.resize(img, tw, th), x, y, cw, ch)


def check(got, ref):
    assert got.shape == ref.shape, (got.shape, ref.shape)
    mx, frac = compare(got, ref)
    assert mx <= 1 and frac < MAX_FRAC, (mx, frac)


def test_center_crop_batch_c2_shapes():
    imgs = [synth(960, 1280, 3, s) for s in range(6)] + [synth(1280, 960, 3, 9)]
    b = dx.buffer_from_vector([dict(image=im, label=i) for i, im in enumerate(imgs)])
    t = b.image_resize_smallest_side("image", 256).image_center_crop("image", 224, 224).batch(4)
    got = [s for s in t]
    assert [s["image"].shape for s in got] == [(4, 224, 224, 3), (3, 224, 224, 3)]
    for k, im in enumerate(imgs):
        check(got[k // 4]["image"][k % 4], oracle_center(im))
    assert got[1]["label"].tolist() == [4, 5, 6]


def test_unbatched_access_materialises():
    im = synth(375, 500, 3, 1)
    b = dx.buffer_from_vector([dict(image=im)]).image_resize_smallest_side("image", 256)
    out = b[0]["image"]
    tw, th = O.smallest_side_dims(500, 375, 256)
    check(out, O.resize(im, tw, th))
    c = dx.buffer_from_vector([dict(image=im)]).image_resize_smallest_side("image", 256).image_center_crop(
        "image", 224, 224)
    check(c[0]["image"], oracle_center(im))


def test_golden_images_through_pipeline():
    names = [k[4:] for k in GOLD.files if k.startswith("img_") and f"rc_{k[4:]}" in GOLD.files]
    samples = [dict(image=np.ascontiguousarray(GOLD[f"img_{n}"])) for n in names]
    rc = [GOLD[f"rc_{n}"] for n in names]
    for s, r, n in zip(samples, rc, names):
        got = dx.buffer_from_vector([s]).image_resize_smallest_side("image", 256).image_center_crop(
            "image", 224, 224)[0]["image"]
        check(got, r)


def test_random_crop_flip_c5():
    """Config 5 shape, scaled: 1080x1920 -> 512 -> random_crop 448 + hflip."""
    imgs = [synth(1080, 1920, 3, 20 + i) for i in range(6)]
    b = dx.buffer_from_vector([dict(image=im) for im in imgs])
    t = (b.image_resize_smallest_side("image", 512).image_random_crop("image", 448, 448)
         .image_random_h_flip("image", 0.5).batch(6))
    dx.set_state(1234)
    out = t[0]["image"]
    # The draws are the reference's (pinned by the CPU test); recompute the
    # expected pixels from the geometry the pipeline recorded.
    from mlx_data_amd import _pipeline as P

    g = b.image_resize_smallest_side("image", 512).image_random_crop("image", 448, 448).image_random_h_flip(
        "image", 0.5)
    dx.set_state(1234)
    plans = [P._plan(g, i, "image") for i in range(6)]
    assert any(p["flip"] for p in plans) and not all(p["flip"] for p in plans)
    for k, (im, p) in enumerate(zip(imgs, plans)):
        rw, rh = p["resize"]
        x, y, cw, ch = p["crop"]
        ref = O.crop(O.resize(im, rw, rh), x, y, cw, ch)
        if p["flip"]:
            ref = O.hflip(ref)
        check(out[k], ref)


def test_ragged_batch_pads():
    """Pending plans of different shapes in one launch: each image lands at
    its slot, the rest is the pad value (Array.cpp:484-485)."""
    a = synth(300, 200, 3, 3)  # portrait -> 64 x 96
    b = synth(200, 300, 3, 4)  # landscape -> 96 x 64
    buf = dx.buffer_from_vector([dict(image=a), dict(image=b)]).image_resize_smallest_side("image", 64)
    out = buf.batch(2, pad={"image": 255})[0]["image"]
    assert out.shape == (2, 96, 96, 3)
    check(out[0, :, :64], O.resize(a, 64, 96))
    check(out[1, :64, :], O.resize(b, 96, 64))
    assert (out[0, :, 64:] == 255).all() and (out[1, 64:, :] == 255).all()
    # crops alone (identity resize) are exact bytes
    r = dx.buffer_from_vector([dict(image=a), dict(image=b)]).image_center_crop("image", 100, 60).batch(2)[0]["image"]
    assert np.array_equal(r[0], a[120:180, 50:150])
    assert np.array_equal(r[1], b[70:130, 100:200])
    # images materialised one by one (a key_transform read them) batch by copy
    m = dx.buffer_from_vector([dict(image=a)]).image_resize("image", 20, 30)[0]["image"]
    mixed = dx.buffer_from_vector([dict(image=np.ascontiguousarray(m)), dict(image=b)])
    mixed = mixed.image_center_crop("image", 20, 30).key_transform("image", lambda v: v).batch(2)[0]["image"]
    assert np.array_equal(mixed[0], m)
    assert np.array_equal(mixed[1], b[85:115, 140:160])


def test_crop_then_resize_and_resize_twice():
    im = synth(480, 640, 3, 5)
    b = dx.buffer_from_vector([dict(image=im)])
    got = b.image_center_crop("image", 400, 300).image_resize("image", 200, 150)[0]["image"]
    ref = O.resize(np.ascontiguousarray(im[90:390, 120:520]), 200, 150)
    check(got, ref)
    got2 = b.image_resize("image", 320, 240).image_resize("image", 100, 80)[0]["image"]
    first = b.image_resize("image", 320, 240)[0]["image"]
    check(got2, O.resize(np.ascontiguousarray(first), 100, 80))


def test_caltech_like_jpeg_pipeline(tmp_path):
    """C1 stand-in: Pillow JPEGs (q=90, ~300x200) through the benchmark's
    exact chain, prefetch and ordered_prefetch; every image equals the oracle
    on the decoded pixels, and the f32 batch is exactly u8/255."""
    from PIL import Image

    files = []
    for i in range(40):
        h, w = (200, 300) if i % 3 else (300, 200)
        arr = synth(h, w, 3, 100 + i)
        d = tmp_path / f"class{i % 4}"
        d.mkdir(exist_ok=True)
        p = d / f"img{i}.jpg"
        Image.fromarray(arr).save(p, quality=90)
        files.append(str(p))
    decoded = {f: np.asarray(Image.open(f).convert("RGB")) for f in files}
    samples = [dict(image=f.encode("ascii"), label=i) for i, f in enumerate(files)]

    dx.set_state(42)
    dset = (dx.buffer_from_vector(samples).to_stream().load_image("image")
            .image_resize_smallest_side("image", 256).image_center_crop("image", 224, 224)
            .batch(8).key_transform("image", lambda x: x.astype("float32") / 255).prefetch(4, 4))
    seen = 0
    for s in dset:
        img = s["image"]
        assert img.dtype == np.float32 and img.shape[1:] == (224, 224, 3)
        q = np.rint(img * 255).astype(np.uint8)
        assert np.array_equal(q.astype(np.float32) / 255, img)
        for k, lab in enumerate(s["label"].tolist()):
            check(q[k], oracle_center(decoded[files[lab]]))
            seen += 1
    assert seen == len(files)

    ordered = (dx.buffer_from_vector(samples).load_image("image").image_resize_smallest_side("image", 256)
               .image_center_crop("image", 224, 224).batch(8).ordered_prefetch(3, 3))
    labels = [v for s in ordered for v in s["label"].tolist()]
    assert labels == list(range(len(files)))


def test_prefetch_threads_share_devices():
    imgs = [synth(480, 640, 3, 200 + i) for i in range(32)]
    b = dx.buffer_from_vector([dict(image=im, i=k) for k, im in enumerate(imgs)])
    s = (b.to_stream().image_resize_smallest_side("image", 256).image_center_crop("image", 224, 224)
         .batch(4).prefetch(8, 8))
    n = 0
    for x in s:
        for k, i in enumerate(x["i"].tolist()):
            check(x["image"][k], oracle_center(imgs[i]))
            n += 1
    assert n == 32


@pytest.mark.parametrize("flip", [False, True])
def test_random_area_crop_resize(flip):
    """Inception-style train augmentation:
    image_random_area_crop((0.08, 1), (3/4, 4/3)) -> image_resize(224, 224)
    [-> random_h_flip(1.0)] -> batch.  The crop is the resize's source window
    at any x (byte-shifted wave path), checked against the oracle resize of
    the numpy crop."""
    from mlx_data_amd import _pipeline as P

    sizes = [(960, 1280), (375, 500), (500, 333), (1080, 1920), (2160, 3840), (300, 200), (720, 1280), (481, 641)]
    imgs = [synth(h, w, 3, 40 + i) for i, (h, w) in enumerate(sizes)]
    b = dx.buffer_from_vector([dict(image=im) for im in imgs])
    t = b.image_random_area_crop("image", (0.08, 1.0), (0.75, 4 / 3)).image_resize("image", 224, 224)
    if flip:
        t = t.image_random_h_flip("image", 1.0)
    dx.set_state(99)
    plans = [P._plan(t, i, "image") for i in range(len(imgs))]
    dx.set_state(99)
    got = [s for s in t.batch(len(imgs))][0]["image"]
    assert got.shape == (len(imgs), 224, 224, 3)
    shifted = 0
    for k, (im, p) in enumerate(zip(imgs, plans)):
        x, y, w, h = p["window"]
        shifted += (x * 3) % 4 != 0
        ref = O.resize(np.ascontiguousarray(im[y:y + h, x:x + w]), 224, 224)
        check(got[k], ref[:, ::-1] if flip else ref)
    assert shifted > 0  # some windows start off a 4-byte boundary
