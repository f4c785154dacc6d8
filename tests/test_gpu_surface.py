"""GPU: operator-surface additions of round 2.

- image_to_float: the fused normalize (VERDICT r1 missing 3).  The batch is
  LUT[u8] bit for bit, and the Caltech chain (benchmarks/comparative/
  caltech101/mlx_data.py:34,46) gives identical tensors with the op in place
  of its trailing ``key_transform(lambda x: x.astype("float32") / 255)``.
- batch with mixed channel counts pads the channel dim like array::batch
  (Array.cpp:465-498, BatchShape::add), pending or materialised.
- one batch split over several devices: contiguous slices of >= 64 images
  in one host thread each, identical to the single-device batch (VERDICT r1
  missing 2); smaller batches go whole to one device, rotating (VERDICT r3
  weak 6).
"""
import numpy as np
import pytest

import oracle as O
from gpu_util import compare, synth
from mlx_data_amd import data as dx

pytestmark = pytest.mark.gpu

LUT = np.arange(256, dtype=np.uint8).astype(np.float32) / np.float32(255)


@pytest.fixture(autouse=True)
def one_device():
    before = dx.devices()
    yield
    dx.set_devices(before)


def c2_samples(n, seed=0):
    shapes = [(960, 1280), (375, 500), (500, 375), (200, 300), (2160, 3840)]
    return [dict(image=synth(*shapes[i % len(shapes)], 3, seed + i), label=i) for i in range(n)]


def test_to_float_batch_is_lut_of_u8_batch():
    samples = c2_samples(10)
    b = dx.buffer_from_vector(samples).image_resize_smallest_side("image", 256).image_center_crop("image", 224, 224)
    u8 = b.batch(10)[0]["image"]
    f = b.image_to_float("image").batch(10)[0]["image"]
    assert f.dtype == np.float32 and f.shape == u8.shape
    assert np.array_equal(f.view(np.uint32), LUT[u8].view(np.uint32))


def test_to_float_unbatched_materialised_and_video():
    img = synth(120, 160, 3, 4)
    b = dx.buffer_from_vector([dict(image=img)])
    # materialised input: one identity launch
    f = b.image_to_float("image")[0]["image"]
    assert f.dtype == np.float32 and np.array_equal(f.view(np.uint32), LUT[img].view(np.uint32))
    # pending input read without batch, output_key keeps the u8 image
    s = b.image_resize("image", 64, 48).image_to_float("image", output_key="f")[0]
    assert s["image"].dtype == np.uint8
    assert np.array_equal(s["f"].view(np.uint32), LUT[s["image"]].view(np.uint32))
    # video: every frame converted in one launch
    video = np.stack([synth(40, 50, 3, k) for k in range(3)])
    v = dx.buffer_from_vector([dict(v=video)]).image_center_crop("v", 30, 20).image_to_float("v")[0]["v"]
    assert v.shape == (3, 20, 30, 3) and np.array_equal(v.view(np.uint32), LUT[video[:, 10:30, 10:40]].view(np.uint32))
    # float images are not images for the resize ops (verify_type)
    with pytest.raises(ValueError, match="image must be of type UInt8"):
        b.image_to_float("image").image_resize("image", 10, 10)[0]


def test_caltech_chain_identical_without_lambda(tmp_path):
    from PIL import Image

    files = []
    for i in range(24):
        h, w = (200, 300) if i % 3 else (300, 200)
        p = tmp_path / f"img{i}.jpg"
        Image.fromarray(synth(h, w, 3, 300 + i)).save(p, quality=90)
        files.append(dict(image=str(p).encode(), label=i))

    def chain(fused):
        d = (dx.buffer_from_vector(files).to_stream().load_image("image")
             .image_resize_smallest_side("image", 256).image_center_crop("image", 224, 224))
        d = d.image_to_float("image").batch(8) if fused else d.batch(8).key_transform(
            "image", lambda x: x.astype("float32") / 255)
        # prefetch threads share the stream, so batches interleave samples:
        # compare per sample
        return {int(lab): img for s in d.prefetch(2, 2) for lab, img in zip(s["label"], s["image"])}

    a, b = chain(False), chain(True)
    assert a.keys() == b.keys() == set(range(24))
    for k in a:
        assert a[k].dtype == b[k].dtype == np.float32
        assert np.array_equal(a[k].view(np.uint32), b[k].view(np.uint32))


def test_mixed_channel_batch_pads_channels():
    grey = synth(90, 120, 1, 1)
    rgb = synth(100, 100, 3, 2)
    b = dx.buffer_from_vector([dict(image=grey), dict(image=rgb)]).image_center_crop("image", 80, 60)
    got = b.batch(2, pad={"image": 7})[0]["image"]
    assert got.shape == (2, 60, 80, 3)
    assert np.array_equal(got[0, :, :, :1], grey[15:75, 20:100])
    assert (got[0, :, :, 1:] == 7).all()
    assert np.array_equal(got[1], rgb[20:80, 10:90])
    assert np.array_equal(got, O.ref_batch([grey[15:75, 20:100], rgb[20:80, 10:90]], pad=7.0))


def test_mixed_channel_batch_pending_and_materialised():
    """random_h_flip leaves unflipped images materialised and makes flipped
    ones pending: over a few seeds every combination of a 1-channel and a
    3-channel image, pending or not, lands in one batch."""
    grey, rgb = synth(60, 80, 1, 1), synth(60, 80, 3, 2)
    b = dx.buffer_from_vector([dict(image=grey), dict(image=rgb)]).image_random_h_flip("image", 0.5)
    seen = set()
    for seed in range(12):
        dx.set_state(seed)
        got = b.batch(2, pad={"image": 9})[0]["image"]
        fg = not np.array_equal(got[0, :, :, :1], grey)
        fr = not np.array_equal(got[1], rgb)
        seen.add((fg, fr))
        assert np.array_equal(got[0, :, :, :1], grey[:, ::-1] if fg else grey)
        assert (got[0, :, :, 1:] == 9).all()
        assert np.array_equal(got[1], rgb[:, ::-1] if fr else rgb)
    assert len(seen) == 4, seen


def test_mixed_channel_resized_batch():
    imgs = [synth(300, 400, 1, 3), synth(400, 300, 3, 4), synth(250, 250, 2, 5)]
    b = dx.buffer_from_vector([dict(image=i) for i in imgs]).image_resize("image", 64, 48)
    got = b.batch(3)[0]["image"]
    assert got.shape == (3, 48, 64, 3)
    for k, img in enumerate(imgs):
        c = img.shape[2]
        m, frac = compare(got[k, :, :, :c], O.resize(img, 64, 48))
        assert m <= 1 and frac < 5e-3
        assert (got[k, :, :, c:] == 0).all()


def small_samples(n, seed=0):
    """n small images of mixed shapes (split tests need >= 64 images a slice)."""
    shapes = [(48, 64), (75, 100), (100, 75), (60, 90), (97, 131)]
    return [dict(image=synth(*shapes[i % len(shapes)], 3, seed + i), idx=np.int64(i)) for i in range(n)]


def test_batch_split_over_devices_matches_single_device():
    """set_devices([0, 0, 0]) with a 200-image batch: three slices (>= 64
    images each, pipeline.cpp split_batch) from three host threads onto the
    same card; the batch equals the one-device batch byte for byte, and a
    failing slice surfaces its message."""
    from mlx_data_amd import _pipeline

    samples = small_samples(200, seed=40)
    assert len(_pipeline._split_batch(200, 3)) == 3

    def run(devs):
        dx.set_devices(devs)
        d = (dx.buffer_from_vector(samples).image_resize_smallest_side("image", 72)
             .image_random_crop("image", 64, 64).image_random_h_flip("image", 0.5))
        dx.set_state(7)
        u = d.batch(200)[0]["image"]
        dx.set_state(7)
        return u, d.image_to_float("image").batch(200)[0]["image"]

    u1, f1 = run([0])
    u3, f3 = run([0, 0, 0])
    assert np.array_equal(u1, u3) and np.array_equal(f1.view(np.uint32), f3.view(np.uint32))
    assert np.array_equal(f1.view(np.uint32), LUT[u1].view(np.uint32))
    # a failing slice (device 99 does not exist) surfaces its message
    dx.set_devices([0, 99])
    bad = dx.buffer_from_vector(samples[:128]).image_resize("image", 32, 32)
    with pytest.raises(RuntimeError, match="invalid device 99"):
        bad.batch(128)[0]


def test_small_batches_route_whole_to_one_device():
    """Caltech's shape on eight devices: batch 32 under prefetch(8, 8) with
    set_devices([0] * 8).  A 32-image batch is below the 64-image slice
    threshold, so each batch is one call on one device, consecutive batches
    rotating over the devices (split_batch) -- and every
    image equals its one-device form (prefetch interleaves the pulls, so
    batches are compared image by image, keyed by a per-sample index)."""
    from mlx_data_amd import _pipeline

    assert _pipeline._split_batch(32, 8, 5) == [(5, 0, 32)]
    samples = small_samples(256, seed=43)
    dx.set_devices([0])
    want = (dx.buffer_from_vector(samples).image_resize_smallest_side("image", 72)
            .image_center_crop("image", 64, 64).image_to_float("image").batch(256))[0]["image"]
    dx.set_devices([0] * 8)
    s = (dx.buffer_from_vector(samples).to_stream().image_resize_smallest_side("image", 72)
         .image_center_crop("image", 64, 64).image_to_float("image").batch(32).prefetch(8, 8))
    seen = []
    for b in s:
        for k, i in enumerate(b["idx"].tolist()):
            assert np.array_equal(b["image"][k].view(np.uint32), want[i].view(np.uint32)), i
            seen.append(i)
    assert sorted(seen) == list(range(256))


def test_batch_split_over_every_visible_device():
    """One batch split over range(device_count()) (op/Shard.cpp:11-20's
    contiguous slices, one per device, on persistent per-device workers):
    byte-identical to the one-device batch.  Needs two or more devices."""
    from mlx_data_amd import capi

    n = capi.device_count()
    if n < 2:
        pytest.skip("one device visible")
    samples = small_samples(64 * n + 1, seed=41)

    def run(devs):
        dx.set_devices(devs)
        d = (dx.buffer_from_vector(samples).image_resize_smallest_side("image", 72)
             .image_center_crop("image", 64, 64).image_to_float("image"))
        return d.batch(len(samples))[0]["image"]

    one = run([0])
    every = run(list(range(n)))
    assert np.array_equal(one.view(np.uint32), every.view(np.uint32))


def test_split_batches_under_prefetch_reuse_workers():
    """Many split batches from prefetch threads at once (128-image batches
    over [0, 0, 0]: two slices each, slice 1 on the per-device workers, at most
    four per device): every image equals its one-device form (compared image
    by image, keyed by a per-sample index)."""
    samples = small_samples(768, seed=42)
    dx.set_devices([0])
    want = (dx.buffer_from_vector(samples).image_resize_smallest_side("image", 72)
            .image_center_crop("image", 64, 64).batch(768))[0]["image"]
    dx.set_devices([0, 0, 0])
    s = (dx.buffer_from_vector(samples).to_stream().image_resize_smallest_side("image", 72)
         .image_center_crop("image", 64, 64).batch(128).prefetch(4, 4))
    seen = []
    for b in s:
        for k, i in enumerate(b["idx"].tolist()):
            assert np.array_equal(b["image"][k], want[i]), i
            seen.append(i)
    assert sorted(seen) == list(range(768))
