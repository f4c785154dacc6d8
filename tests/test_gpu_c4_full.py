"""GPU: configuration 4 at one GPU's full slice (BASELINE.json configs[3]:
1024 ImageNet-shape JPEG files over 8 GPUs = 128 per GPU), through the
operator surface the reference benchmarks (benchmarks/comparative/caltech101/
mlx_data.py: load_image -> image_resize_smallest_side(256) ->
image_center_crop(224, 224) -> /255 -> batch), VERDICT r3 weak 7.

* 128 JPEG files of the bench's shapes (500x375 / 375x500 / 500x333 drawn
  with seed 2, like bench.py's c4 workload), encoded by Pillow;
* the batch with the device-side decode finish (the default with a GPU
  visible) equals the batch decoded whole on the host byte for byte;
* every image equals the kernel-order oracle (orc_resize_crop_vfirst) on the
  decoded pixels bit for bit, and the stbir-order restatement within +-1 on
  < 0.2 % of channels (the parity bar of tests/test_gpu_parity.py); the
  decoded pixels themselves are Pillow's libjpeg-turbo decode (the
  reference's decoder, ImageJPEG.cpp:99-146), checked on a sample here and
  pinned in full by tests/test_jpeg.py;
* /255 is the numpy LUT bit for bit."""
import io

import numpy as np
import pytest

import oracle as O
from gpu_util import compare, synth

pytestmark = pytest.mark.gpu

C4_SIZES = [(500, 375), (375, 500), (500, 333)]  # (w, h), bench.py
N = 128
LUT = np.arange(256, dtype=np.uint8).astype(np.float32) / np.float32(255)


@pytest.fixture(scope="module")
def c4_files(tmp_path_factory):
    from PIL import Image

    d = tmp_path_factory.mktemp("c4")
    rng = np.random.default_rng(2)
    sizes = [C4_SIZES[i] for i in rng.integers(0, len(C4_SIZES), N)]
    files, decoded = [], []
    for i, (w, h) in enumerate(sizes):
        b = io.BytesIO()
        Image.fromarray(synth(h, w, 3, 1000 + i)).save(b, "JPEG", quality=90)
        p = d / f"{i:04d}.jpg"
        p.write_bytes(b.getvalue())
        files.append(str(p))
        decoded.append(np.asarray(Image.open(io.BytesIO(b.getvalue())).convert("RGB")))
    return files, decoded


def _batch(files, device_decode):
    from mlx_data_amd import data as dx

    before = dx.device_decode()
    dx.set_device_decode(device_decode)
    try:
        d = (dx.buffer_from_vector([dict(image=f.encode(), idx=np.int64(i)) for i, f in enumerate(files)])
             .load_image("image").image_resize_smallest_side("image", 256).image_center_crop("image", 224, 224)
             .image_to_float("image").batch(N))
        b = d[0]
        assert b["idx"].tolist() == list(range(N))
        return b["image"]
    finally:
        dx.set_device_decode(before)


def test_c4_slice_device_decode_equals_host_decode_and_oracle(c4_files):
    from mlx_data_amd import capi

    files, decoded = c4_files
    on = _batch(files, True)
    off = _batch(files, False)
    assert on.shape == (N, 224, 224, 3) and on.dtype == np.float32
    assert np.array_equal(on.view(np.uint32), off.view(np.uint32))
    # the float batch is the LUT of its u8 values (exact /255)
    q = np.rint(on * 255).astype(np.uint8)
    assert np.array_equal(on.view(np.uint32), LUT[q].view(np.uint32))
    # the native decoder equals Pillow's libjpeg-turbo on a sample
    for i in range(0, N, 16):
        with open(files[i], "rb") as f:
            assert np.array_equal(capi.jpeg_decode(f.read()), decoded[i]), i
    worst, frac = 0, 0.0
    for i, img in enumerate(decoded):
        h, w = img.shape[:2]
        tw, th = O.smallest_side_dims(w, h, 256)
        cx, cy = O.center_crop_origin(tw, th, 224, 224)
        assert np.array_equal(q[i], O.resize_crop_vfirst(img, (tw, th, cx, cy, 224, 224, 0))), i
        m, f = compare(q[i], O.crop(O.resize(img, tw, th), cx, cy, 224, 224))
        worst, frac = max(worst, m), max(frac, f)
    assert worst <= 1 and frac < 0.002, (worst, frac)


@pytest.fixture(scope="module")
def c4_files_1024(tmp_path_factory):
    """configs[3]'s whole batch: 1024 ImageNet-shape files (seed 2 shapes),
    Pillow q=90, baseline: every file takes the device entropy decode."""
    from PIL import Image

    d = tmp_path_factory.mktemp("c4_1024")
    rng = np.random.default_rng(2)
    sizes = [C4_SIZES[i] for i in rng.integers(0, len(C4_SIZES), 1024)]
    files = []
    base = synth(500, 500, 3, 7)
    for i, (w, h) in enumerate(sizes):
        y, x = (i * 37) % (500 - h + 1), (i * 53) % (500 - w + 1)
        p = d / f"{i:04d}.jpg"
        Image.fromarray(np.ascontiguousarray(np.roll(base, i, axis=1)[y:y + h, x:x + w])).save(p, quality=90)
        files.append(str(p))
    return files


def test_c4_batch_split_over_eight_devices(c4_files_1024):
    """C4's multi-GPU form rehearsed on one card --
    set_devices([0] * 8) with the 1024-file batch, device entropy decode on:
    eight slices of 128 (op/Shard.cpp:11-20's contiguous split), each one
    fused JPEG call (Huffman + IDCT + colour + resize on the GPU), and the
    batch byte-identical to set_devices([0])."""
    from mlx_data_amd import _pipeline
    from mlx_data_amd import data as dx

    assert dx.device_entropy() and dx.device_decode()
    assert _pipeline._split_batch(1024, 8) == [(k, 128 * k, 128 * (k + 1)) for k in range(8)]
    before = dx.devices()

    def run(devs):
        dx.set_devices(devs)
        d = (dx.buffer_from_vector([dict(image=f.encode(), idx=np.int64(i)) for i, f in enumerate(c4_files_1024)])
             .load_image("image").image_resize_smallest_side("image", 256).image_center_crop("image", 224, 224)
             .image_to_float("image"))
        _pipeline._run_on_stats(True)
        b = d.batch(1024)[0]
        calls, jpegs = _pipeline._run_on_stats(True)
        assert b["idx"].tolist() == list(range(1024))
        return b["image"], calls, jpegs

    try:
        one, calls1, j1 = run([0])
        eight, calls8, j8 = run([0] * 8)
    finally:
        dx.set_devices(before)
    assert (calls1, j1) == (1, 1024)
    assert (calls8, j8) == (8, 1024)
    assert eight.shape == (1024, 224, 224, 3)
    assert np.array_equal(one.view(np.uint32), eight.view(np.uint32))
    q = np.rint(eight * 255).astype(np.uint8)
    assert np.array_equal(eight.view(np.uint32), LUT[q].view(np.uint32))
