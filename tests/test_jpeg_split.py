"""The split JPEG decode (include/mxd_amd.h mxd_jpeg_coefs_*; SURVEY.md §8f
f1, "later a device-side decode"), host side: the entropy decode keeps the
quantised coefficients and the host finish (IDCT, upsampling, colour) gives
exactly the bytes of the one-shot decode -- and so of Pillow's libjpeg-turbo
(tests/golden/jpeg.npz, plus a live Pillow sweep).  Errors come from the
entropy decode with the one-shot decoder's messages.  The GPU finish is
tests/test_gpu_jpeg.py."""
import io
import os

import numpy as np
import pytest

from mlx_data_amd import capi

GOLD = np.load(os.path.join(os.path.dirname(__file__), "golden", "jpeg.npz"))
CASES = sorted(k[:-4] for k in GOLD.files if k.endswith("_jpg"))


@pytest.mark.parametrize("case", CASES)
def test_host_finish_equals_decode(case):
    data = GOLD[f"{case}_jpg"]
    c = capi.JpegCoefs(data)
    want = GOLD[f"{case}_rgb"]
    assert (c.height, c.width) == want.shape[:2]
    assert c.device_ok  # (CMYK too, since round 6; only lossless files finish on the host alone)
    got = c.finish()
    assert np.array_equal(got, want)
    assert np.array_equal(c.finish(), got)  # the handle stays valid
    c.close()


@pytest.mark.parametrize("seed", range(6))
def test_live_pillow_sweep(seed):
    Image = pytest.importorskip("PIL.Image")
    rng = np.random.default_rng(100 + seed)
    for _ in range(6):
        h, w = int(rng.integers(1, 160)), int(rng.integers(1, 160))
        grey = rng.random() < 0.2
        a = rng.integers(0, 256, (h, w, 1 if grey else 3)).astype(np.uint8)
        kw = dict(quality=int(rng.integers(5, 101)), progressive=bool(rng.random() < 0.5))
        if not grey:
            kw["subsampling"] = int(rng.integers(0, 3))
        if rng.random() < 0.3:
            kw["restart_marker_blocks"] = int(rng.integers(1, 6))
        b = io.BytesIO()
        Image.fromarray(a[:, :, 0] if grey else a).save(b, "JPEG", **kw)
        want = np.asarray(Image.open(io.BytesIO(b.getvalue())).convert("RGB"))
        assert np.array_equal(capi.JpegCoefs(b.getvalue()).finish(), want), (h, w, kw)


def _segment(marker, payload):
    return bytes([0xFF, marker]) + (len(payload) + 2).to_bytes(2, "big") + payload


def test_errors_from_the_entropy_decode():
    with pytest.raises(capi.MxdError, match="Not a JPEG file"):
        capi.JpegCoefs(b"\x89PNG\r\n\x1a\n" + bytes(32))
    sof7 = b"\xff\xd8" + _segment(0xC7, bytes([8, 0, 8, 0, 8, 1, 1, 0x11, 0]))  # differential lossless
    with pytest.raises(capi.MxdError, match="Unsupported JPEG process: SOF type 0xc7"):
        capi.JpegCoefs(sof7)
    sof9 = b"\xff\xd8" + _segment(0xC9, bytes([8, 0, 8, 0, 8, 1, 1, 0x11, 0]))  # arithmetic, no scan
    with pytest.raises(capi.MxdError, match="Premature end of JPEG file"):
        capi.JpegCoefs(sof9)
    data = bytes(GOLD["sub2_prog0_jpg"])
    for cut in (data.index(b"\xff\xc0") + 6, data.index(b"\xff\xda") + 4):
        with pytest.raises(capi.MxdError) as a:
            capi.JpegCoefs(data[:cut])
        with pytest.raises(capi.MxdError) as b:
            capi.jpeg_decode(data[:cut]) if cut > data.index(b"\xff\xc0") + 20 else capi.jpeg_info(data[:cut])
        assert str(a.value) == str(b.value)


def test_load_image_lazy_decode_reads_back_on_host():
    """With the device finish switched on, load_image keeps the coefficients;
    reading the sample (no batch) runs the host finish: the fixture bytes."""
    from mlx_data_amd import data as dx

    before = dx.device_decode()
    dx.set_device_decode(True)
    try:
        cases = ["caltech_300x200", "grey", "cmyk", "sub0_prog1", "tiny_1x1"]
        b = dx.buffer_from_vector([dict(m=GOLD[f"{c}_jpg"]) for c in cases]).load_image("m", from_memory=True)
        for i, c in enumerate(cases):
            got = b[i]["m"]
            assert got.shape == GOLD[f"{c}_rgb"].shape
            assert np.array_equal(got, GOLD[f"{c}_rgb"]), c
    finally:
        dx.set_device_decode(before)
