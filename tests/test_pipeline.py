"""CPU tests of the operator surface (mlx_data_amd.data): dataset plumbing,
batch semantics, plan geometry, RNG draw order and error behaviour.

Nothing here reads pixels of a resized image (that needs the GPU; see
test_gpu_pipeline.py).  Expected values come from the reference's own code
(golden fixtures made with oracle/_ref) or from the oracle's geometry.
Reference anchors: op/ImageTransform.cpp:78-158,317-332, Array.cpp:465-541,
stream/{Batch,Prefetch,OrderedPrefetch}.cpp, buffer/{Batch,Shuffle}.cpp,
op/LoadImage.cpp:23-48.
"""
import os

import numpy as np
import pytest

import oracle as O
from mlx_data_amd import data as dx
from mlx_data_amd import _pipeline as P

GOLD = np.load(os.path.join(os.path.dirname(__file__), "golden", "golden.npz"))


def has_gpu():
    return len(dx.devices()) > 0


def test_sample_conversion():
    b = dx.buffer_from_vector([dict(a=3, f=2.5, s=b"abc", n=np.arange(4, dtype=np.int32), u=np.ones((2, 2), np.uint8))])
    s = b[0]
    assert s["a"].dtype == np.int64 and s["a"].shape == () and int(s["a"]) == 3
    assert s["f"].dtype == np.float64 and float(s["f"]) == 2.5
    assert s["s"].dtype == np.int8 and bytes(s["s"]) == b"abc"
    assert s["n"].dtype == np.int32 and list(s["n"]) == [0, 1, 2, 3]
    assert s["u"].dtype == np.uint8 and s["u"].shape == (2, 2)
    with pytest.raises(ValueError, match="Cannot convert strings"):
        dx.buffer_from_vector([dict(a="x")])
    with pytest.raises(RuntimeError, match="unexpected empty sample"):
        dx.buffer_from_vector([dict()])
    with pytest.raises(RuntimeError, match="Contiguous array expected"):
        dx.buffer_from_vector([dict(a=np.zeros((4, 4))[:, ::2])])


def test_batch_matches_reference_array_batch():
    """Ragged uint8 crops batched with pad 0: bytes equal the reference's
    array::batch output (golden refbatch, made by oracle/_ref)."""
    shapes = GOLD["refbatch_shapes"]
    crops = [GOLD["rc_caltech_200x300"], GOLD["rc_small_97x131"][:200, :210], GOLD["rc_tiny_48x64"][:150, :224]]
    assert [c.shape for c in crops] == [tuple(s) for s in shapes]
    b = dx.buffer_from_vector([dict(image=np.ascontiguousarray(c)) for c in crops]).batch(3)
    out = b[0]["image"]
    assert out.shape == GOLD["refbatch"].shape
    assert np.array_equal(out, GOLD["refbatch"])


def test_batch_pad_and_dim():
    xs = [np.arange(n, dtype=np.int64) + 10 * n for n in (1, 3, 2)]
    b = dx.buffer_from_vector([dict(x=x, y=float(i)) for i, x in enumerate(xs)])
    s = b.batch(3, pad={"x": -7})[0]
    assert s["x"].tolist() == [[10, -7, -7], [30, 31, 32], [20, 21, -7]]
    assert s["y"].tolist() == [0.0, 1.0, 2.0]
    # dim: concatenation along an existing axis (Array.cpp:500-541)
    m = [np.full((2, n), n, np.int32) for n in (1, 3)]
    s = dx.buffer_from_vector([dict(m=a) for a in m]).batch(2, dim={"m": 1})[0]
    assert s["m"].tolist() == [[1, 3, 3, 3], [1, 3, 3, 3]]
    s = dx.buffer_from_vector([dict(m=a) for a in [np.ones((1, 2), np.int32), np.ones((2, 1), np.int32)]]).batch(
        2, dim={"m": 0}, pad={"m": 5})[0]
    assert s["m"].tolist() == [[1, 1], [1, 5], [1, 5]]
    with pytest.raises(RuntimeError, match="consistent shapes"):
        dx.buffer_from_vector([dict(x=np.zeros(2)), dict(x=np.zeros((2, 2)))]).batch(2)[0]
    with pytest.raises(RuntimeError, match="different types"):
        dx.buffer_from_vector([dict(x=np.zeros(2)), dict(x=np.zeros(2, np.int32))]).batch(2)[0]
    with pytest.raises(RuntimeError, match="inconsistent sample keys"):
        dx.buffer_from_vector([dict(x=1), dict(y=1)]).batch(2)[0]
    with pytest.raises(RuntimeError, match="batch size must be positive"):
        dx.buffer_from_vector([dict(x=1)]).batch(0)


def test_buffer_batch_sizes_and_short_last():
    b = dx.buffer_from_vector([dict(i=i) for i in range(10)]).batch(4)
    assert len(b) == 3
    assert [s["i"].tolist() for s in b] == [[0, 1, 2, 3], [4, 5, 6, 7], [8, 9]]
    with pytest.raises(RuntimeError, match="index out of range"):
        b[3]


def test_stream_batch_prefetch_and_reset():
    s = dx.buffer_from_vector([dict(i=i) for i in range(11)]).to_stream().batch(3)
    assert [x["i"].tolist() for x in s] == [[0, 1, 2], [3, 4, 5], [6, 7, 8], [9, 10]]
    assert s.next() == {}
    s.reset()
    assert s.next()["i"].tolist() == [0, 1, 2]
    # prefetch: every batch exactly once (order between workers is free)
    p = dx.buffer_from_vector([dict(i=i) for i in range(100)]).to_stream().batch(7).prefetch(4, 3)
    got = sorted(v for x in p for v in x["i"].tolist())
    assert got == list(range(100))
    # ordered_prefetch keeps buffer order
    o = dx.buffer_from_vector([dict(i=i) for i in range(50)]).batch(4).ordered_prefetch(3, 4)
    assert [v for x in o for v in x["i"].tolist()] == list(range(50))
    o.reset()
    assert o.next()["i"].tolist() == [0, 1, 2, 3]


def test_shuffle_is_seeded_permutation():
    b = dx.buffer_from_vector([dict(i=i) for i in range(64)])
    dx.set_state(7)
    a = [int(s["i"]) for s in b.shuffle()]
    dx.set_state(7)
    c = [int(s["i"]) for s in b.shuffle()]
    assert a == c and sorted(a) == list(range(64)) and a != list(range(64))


def test_key_transform_and_if_variants():
    b = dx.buffer_from_vector([dict(x=np.arange(3, dtype=np.float32))])
    t = b.key_transform("x", lambda v: v * 2, output_key="y")
    s = t[0]
    assert s["x"].tolist() == [0, 1, 2] and s["y"].tolist() == [0, 2, 4]
    assert b.key_transform_if(False, "x", lambda v: v + 1)[0]["x"].tolist() == [0, 1, 2]
    assert b.key_transform_if(True, "x", lambda v: v + 1)[0]["x"].tolist() == [1, 2, 3]
    with pytest.raises(RuntimeError, match="key <nope> expected"):
        b.key_transform("nope", lambda v: v)[0]


IMGS = sorted(k[4:] for k in GOLD.files if k.startswith("img_"))


@pytest.mark.parametrize("name", IMGS)
def test_plan_geometry_matches_oracle(name):
    img = np.ascontiguousarray(GOLD[f"img_{name}"])
    h, w = img.shape[:2]
    b = dx.buffer_from_vector([dict(image=img)])
    t = b.image_resize_smallest_side("image", 256)
    tw, th = O.smallest_side_dims(w, h, 256)
    p = P._plan(t, 0, "image")
    assert p["resize"] == (tw, th) and p["window"] == (0, 0, w, h) and p["shape"] == [th, tw, img.shape[2]]
    if tw >= 224 and th >= 224:
        c = t.image_center_crop("image", 224, 224)
        x, y = O.center_crop_origin(tw, th, 224, 224)
        p = P._plan(c, 0, "image")
        assert p["crop"] == (x, y, 224, 224) and p["shape"] == [224, 224, img.shape[2]] and not p["flip"]


def test_random_crop_flip_draws_match_reference():
    """set_state(1234) then random_crop(448) + random_h_flip(0.5) on 910x512
    images: the (x, y, flip) stream equals the reference's (golden rng_*)."""
    img = np.zeros((512, 910, 3), np.uint8)
    b = dx.buffer_from_vector([dict(image=img)] * 64)
    t = b.image_random_crop("image", 448, 448).image_random_h_flip("image", 0.5)
    dx.set_state(1234)
    got = [P._plan(t, i, "image") for i in range(64)]
    xy = [g["crop"][:2] for g in got]
    fl = [int(g["flip"]) for g in got]
    assert np.array_equal(np.array(xy), GOLD["rng_xy"])
    assert np.array_equal(np.array(fl), GOLD["rng_flip"])


def test_plan_composition():
    img = np.zeros((100, 200, 3), np.uint8)
    b = dx.buffer_from_vector([dict(image=img)])
    # crop -> resize: the crop becomes the source window
    p = P._plan(b.image_center_crop("image", 50, 40).image_resize("image", 25, 20), 0, "image")
    assert p["window"] == (75, 30, 50, 40) and p["resize"] == (25, 20) and p["crop"] == (0, 0, 25, 20)
    # crop of a mirrored view maps back into unmirrored coordinates
    b2 = dx.buffer_from_vector([dict(image=img)] * 2)
    dx.set_state(0)
    f = b2.image_random_h_flip("image", 1.0).image_center_crop("image", 60, 100)
    p = P._plan(f, 0, "image")
    assert p["flip"] and p["crop"] == (70, 0, 60, 100)
    g = P._plan(b.image_random_h_flip("image", 1.0).image_random_crop("image", 10, 10), 0, "image")
    assert g["flip"]
    # flip twice = identity mirror
    p = P._plan(b.image_random_h_flip("image", 1.0).image_random_h_flip("image", 1.0), 0, "image")
    assert not p["flip"]


def test_image_op_errors():
    img = np.zeros((20, 30, 3), np.uint8)
    b = dx.buffer_from_vector([dict(image=img)])
    with pytest.raises(RuntimeError, match="ImageResizeSmallestSide: illegal target size: 0"):
        b.image_resize_smallest_side("image", 0)[0]
    with pytest.raises(RuntimeError, match="ImageCenterCrop: target image size larger than input image"):
        b.image_center_crop("image", 31, 10)[0]
    with pytest.raises(RuntimeError, match="ImageRandomCrop: target image size larger than input image"):
        b.image_random_crop("image", 10, 21)[0]
    with pytest.raises(RuntimeError, match="cannot create image with 0 or negative dimension"):
        b.image_resize("image", 0, 5)[0]
    with pytest.raises(RuntimeError, match="image must be 3 dimension"):
        dx.buffer_from_vector([dict(image=np.zeros((4, 4), np.uint8))]).image_resize("image", 2, 2)[0]
    with pytest.raises(RuntimeError, match="channels must be 0 <= c <= 4"):
        dx.buffer_from_vector([dict(image=np.zeros((4, 4, 5), np.uint8))]).image_resize("image", 2, 2)[0]
    with pytest.raises(ValueError, match="UInt8"):
        dx.buffer_from_vector([dict(image=np.zeros((4, 4, 3), np.float32))]).image_resize("image", 2, 2)[0]


def test_non_uint8_crop_is_a_sub_array():
    a = np.arange(4 * 6 * 2, dtype=np.float32).reshape(4, 6, 2)
    s = dx.buffer_from_vector([dict(image=a)]).image_center_crop("image", 2, 2)[0]
    assert np.array_equal(s["image"], a[1:3, 2:4])


@pytest.mark.skipif(has_gpu(), reason="checks the no-GPU behaviour")
def test_pixels_need_the_gpu():
    img = np.zeros((20, 30, 3), np.uint8)
    b = dx.buffer_from_vector([dict(image=img)] * 2)
    with pytest.raises(RuntimeError, match="no HIP device"):
        b.image_resize("image", 10, 10)[0]
    with pytest.raises(RuntimeError, match="no HIP device"):
        b.image_center_crop("image", 10, 10).batch(2)[0]


def test_load_image(tmp_path):
    from PIL import Image

    rng = np.random.default_rng(3)
    arr = rng.integers(0, 256, (40, 60, 3), dtype=np.uint8)
    Image.fromarray(arr).save(tmp_path / "a.jpg", quality=90)
    Image.fromarray(arr[:, :, 0]).save(tmp_path / "g.png")
    Image.fromarray(arr).save(tmp_path / "c.png")
    expect = np.asarray(Image.open(tmp_path / "a.jpg").convert("RGB"))
    b = dx.buffer_from_vector([dict(f=b"a.jpg"), dict(f=b"g.png"), dict(f=b"c.png")])
    s = b.load_image("f", prefix=str(tmp_path), output_key="image")
    assert np.array_equal(s[0]["image"], expect)
    assert s[1]["image"].shape == (40, 60, 1) and np.array_equal(s[1]["image"][:, :, 0], arr[:, :, 0])
    assert np.array_equal(s[2]["image"], arr)
    info = b.load_image("f", prefix=str(tmp_path), info=True)[0]["f"]
    assert info.tolist() == [60, 40]
    raw = (tmp_path / "a.jpg").read_bytes()
    m = dx.buffer_from_vector([dict(f=np.frombuffer(raw, np.uint8))]).load_image("f", from_memory=True)
    assert np.array_equal(m[0]["f"], expect)
    # core/image/ImageJPEG.cpp:77-80 (check_signature's fopen) names the path
    with pytest.raises(RuntimeError, match=r"load_jpeg: could not load <.*missing.jpg>"):
        dx.buffer_from_vector([dict(f=b"missing.jpg")]).load_image("f", prefix=str(tmp_path))[0]
    with pytest.raises(RuntimeError, match=r"char array \(int8\) expected"):
        dx.buffer_from_vector([dict(f=np.zeros(3, np.uint8))]).load_image("f")[0]


def test_load_image_info_reads_headers_only(tmp_path):
    """info=True is core::image::info -> stbi_info (core/image/ImageIO.cpp:26-32):
    (0, 0) for a file that cannot be opened (no exception), the frame size of a
    JPEG whose APP segments push its frame header far into the file, and the
    non-JPEG formats through the stb_image hook."""
    from PIL import Image

    rng = np.random.default_rng(4)
    arr = rng.integers(0, 256, (30, 50, 3), dtype=np.uint8)
    Image.fromarray(arr).save(tmp_path / "a.jpg", quality=90)
    Image.fromarray(arr).save(tmp_path / "c.png")
    raw = (tmp_path / "a.jpg").read_bytes()
    # five 60 KB APP15 segments (~300 KB) between SOI and the frame header
    app = b"".join(b"\xff\xef" + (60002).to_bytes(2, "big") + bytes(60000) for _ in range(5))
    (tmp_path / "big.jpg").write_bytes(raw[:2] + app + raw[2:])
    b = dx.buffer_from_vector([dict(f=b"missing.jpg"), dict(f=b"a.jpg"), dict(f=b"big.jpg"), dict(f=b"c.png")])
    info = b.load_image("f", prefix=str(tmp_path), info=True)
    assert [info[i]["f"].tolist() for i in range(4)] == [[0, 0], [50, 30], [50, 30], [50, 30]]
    big = dx.buffer_from_vector([dict(f=b"big.jpg")]).load_image("f", prefix=str(tmp_path))[0]["f"]
    assert np.array_equal(big, np.asarray(Image.open(tmp_path / "a.jpg").convert("RGB")))


AREA = np.load(os.path.join(os.path.dirname(__file__), "golden", "rng_area.npz"))
AREA_CASES = sorted({int(k.split("_")[1]) for k in AREA.files})


@pytest.mark.parametrize("case", AREA_CASES)
def test_random_area_crop_draws_match_reference(case):
    """image_random_area_crop (op/ImageTransform.cpp:214-291) after set_state:
    the crop windows equal the reference State's draws (golden rng_area.npz);
    where no crop was found the image passes unchanged."""
    seed, trials, a0, a1, r0, r1 = AREA[f"area_{case}_in"]
    wh = AREA[f"area_{case}_wh"]
    ref = AREA[f"area_{case}_out"]
    b = dx.buffer_from_vector([dict(image=np.zeros((h, w, 3), np.uint8)) for w, h in wh])
    t = b.image_random_area_crop("image", (a0, a1), (r0, r1), num_trial=int(trials))
    dx.set_state(int(seed))
    for i, (w, h) in enumerate(wh):
        p = P._plan(t, i, "image")
        if ref[i][2] == 0:  # unchanged: the source array itself, no plan
            assert p is None or p["crop"] == (0, 0, int(w), int(h)), (i, w, h, p)
        else:
            assert p is not None and p["crop"] == tuple(int(v) for v in ref[i]), (i, w, h, p, ref[i])


def test_random_area_crop_then_resize_plan():
    """Inception-style random_area_crop -> image_resize: the crop becomes the
    resize's source window (one fused launch)."""
    img = np.zeros((375, 500, 3), np.uint8)
    t = dx.buffer_from_vector([dict(image=img)]).image_random_area_crop("image", (0.08, 1.0), (0.75, 4 / 3))
    dx.set_state(1234)
    c = P._plan(t, 0, "image")["crop"]
    r = t.image_resize("image", 224, 224)
    dx.set_state(1234)
    p = P._plan(r, 0, "image")
    assert p["window"] == c and p["resize"] == (224, 224) and p["crop"] == (0, 0, 224, 224)


def test_random_area_crop_errors():
    b = dx.buffer_from_vector([dict(image=np.zeros((8, 8, 3), np.uint8))])
    cases = [
        (((0.0, 1.0), (1.0, 1.0), 10), "invalid area range"),
        (((0.6, 0.5), (1.0, 1.0), 10), "invalid area range"),
        (((0.5, 1.1), (1.0, 1.0), 10), "invalid area range"),
        (((0.5, 1.0), (0.0, 1.0), 10), "invalid aspect ratio range"),
        (((0.5, 1.0), (2.0, 1.0), 10), "invalid aspect ratio range"),
        (((0.6, 1.0), (2.0, 3.0), 10), "cannot be fullfilled"),
        (((0.5, 1.0), (0.1, 0.4), 10), "cannot be fullfilled"),
        (((0.5, 1.0), (1.0, 1.0), 0), "number of trial must be positive"),
    ]
    for (a, r, n), msg in cases:
        with pytest.raises(RuntimeError, match=msg):
            b.image_random_area_crop("image", a, r, num_trial=n)


def test_worker_errors_reach_the_consumer():
    """SURVEY.md §5 failure handling: an exception raised inside a prefetch
    worker (stream/Prefetch.cpp:48 future::get) surfaces at the consumer's
    next(), with its message; ordered_prefetch likewise; the pipeline can be
    dropped afterwards without hanging (Prefetch::~Prefetch drains)."""
    def boom(x):
        if int(x[0]) == 5:
            raise ValueError("bad sample 5")
        return x

    samples = [dict(i=np.array([k], np.int64)) for k in range(12)]
    s = dx.buffer_from_vector(samples).to_stream().key_transform("i", boom).prefetch(4, 4)
    with pytest.raises(ValueError, match="bad sample 5"):
        for _ in s:
            pass
    del s
    o = dx.buffer_from_vector(samples).key_transform("i", boom).ordered_prefetch(3, 3)
    seen = []
    with pytest.raises(ValueError, match="bad sample 5"):
        for x in o:
            seen.append(int(x["i"][0]))
    assert seen == [0, 1, 2, 3, 4]
    del o
    # a missing file through load_image: the reference's message, via a worker
    m = dx.buffer_from_vector([dict(f=b"/nonexistent/x.jpg")]).to_stream().load_image("f").prefetch(2, 2)
    with pytest.raises(RuntimeError, match="could not load"):
        next(iter(m))


def test_dropping_a_busy_prefetch_does_not_deadlock():
    """Prefetch::~Prefetch joins its workers (stream/Prefetch.cpp:21-27); when
    they run a Python key_transform they need the GIL, so the last reference
    must be dropped with the GIL released (module.cpp nogil_owned)."""
    import gc
    import threading
    import time

    def slow(x):
        time.sleep(0.01)
        return x

    samples = [dict(i=np.array([k], np.int64)) for k in range(64)]
    s = dx.buffer_from_vector(samples).to_stream().key_transform("i", slow).prefetch(8, 4)
    # workers now busy in `slow` (which sample a future gets is up to the
    # threads: each calls the upstream next(), stream/Prefetch.cpp:38-49)
    assert 0 <= int(next(iter(s))["i"][0]) < 64
    done = threading.Event()

    def drop():
        nonlocal s
        del s
        gc.collect()
        done.set()

    t = threading.Thread(target=drop)
    t.start()
    t.join(timeout=20)
    assert done.is_set()


def test_split_batch_routing():
    """pipeline.cpp split_batch: below 64 images per
    device slice a batch goes whole to one device, consecutive batches
    rotating over the devices; larger batches are cut into contiguous slices
    (op/Shard.cpp:11-20), k = min(devices, n // 64), covering [0, n) in order."""
    from mlx_data_amd import _pipeline as P

    assert P._MIN_SLICE_IMAGES == 64
    # Caltech: batch 32 on 8 devices -> one call, device = the rotation counter
    for first in range(10):
        assert P._split_batch(32, 8, first) == [(first % 8, 0, 32)]
    assert P._split_batch(127, 8, 0) == [(0, 0, 127)]
    assert P._split_batch(128, 8, 3) == [(3, 0, 64), (4, 64, 128)]
    # C4: 1024 over 8 devices -> 8 slices of 128, one per device
    sl = P._split_batch(1024, 8, 6)
    assert [d for d, _, _ in sl] == [6, 7, 0, 1, 2, 3, 4, 5]
    assert [(b, e) for _, b, e in sl] == [(128 * k, 128 * (k + 1)) for k in range(8)]
    for n in (1, 63, 64, 65, 200, 511, 513, 4096):
        for nd in (1, 2, 3, 8):
            sl = P._split_batch(n, nd, 0)
            assert len(sl) == max(1, min(nd, n // 64))
            assert sl[0][1] == 0 and sl[-1][2] == n
            assert all(a[2] == b[1] for a, b in zip(sl, sl[1:]))
            assert all(e - b >= min(n, 64) for _, b, e in sl)
    assert P._split_batch(0, 8, 0) == []
