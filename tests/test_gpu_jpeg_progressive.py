"""GPU: progressive JPEGs through the device route.  Round 5 decoded every
scan of a complete progressive file on the GPU (jpeg_prog, one serial chain
per component); it lost to the host entropy decode at 16 pipeline workers
and was retired in round 6, so with
mxd_jpeg_coefs_parse(device_entropy=1) a progressive file is entropy-decoded
on the host (jpeg.cpp, libjpeg-turbo's jdphuff.c semantics) and its
coefficients -- natural order -- are finished (IDCT, upsampling, colour) and
resized on the GPU.

Bit-exact against the host decoder (pinned to libjpeg-turbo through Pillow by
tests/test_jpeg.py) and against Pillow's decode of the same file, at identity
geometry: the committed progressive fixtures, seeded Pillow progressive
encodes (sizes 1..600, qualities 5..100, 4:4:4 / 4:2:2 / 4:2:0 / grey,
restart intervals), corrupt scan data, scans whose data runs out before
their last block, batches that mix progressive, sequential and host-decoded
files, and large photos."""
import io
import os

import numpy as np
import pytest

from mlx_data_amd import capi

pytestmark = pytest.mark.gpu

GOLD = np.load(os.path.join(os.path.dirname(__file__), "golden", "jpeg.npz"))

from test_gpu_jpeg_entropy import _check_identity, _decode_gpu, _encode, _smooth  # noqa: E402


def _sweep(seed, n=16, max_side=600):
    rng = np.random.default_rng(seed)
    datas = []
    for i in range(n):
        h, w = int(rng.integers(1, max_side)), int(rng.integers(1, max_side))
        grey = i % 6 == 5
        kw = dict(quality=int(rng.integers(5, 101)), progressive=True, optimize=bool(rng.random() < 0.5))
        if not grey:
            kw["subsampling"] = i % 3
        if rng.random() < 0.25:
            kw["restart_marker_blocks"] = int(rng.integers(1, 8))
        datas.append(_encode(_smooth(rng, h, w, 1 if grey else 3), **kw))
    return datas


def _scans(d):
    """(SOS offset, data start, data end) of every scan of a file."""
    out, i = [], 2
    while True:
        i = d.find(b"\xff\xda", i)
        if i < 0:
            return out
        start = i + 2 + int.from_bytes(d[i + 2:i + 4], "big")
        e = start
        while True:
            e = d.index(b"\xff", e)
            if d[e + 1] == 0x00 or 0xD0 <= d[e + 1] <= 0xD7:
                e += 2
                continue
            break
        out.append((i, start, e))
        i = e


def test_progressive_fixtures_identity():
    keys = [k[:-4] for k in GOLD.files if k.endswith("_jpg") and "prog" in k and "trunc" not in k]
    datas = [GOLD[f"{k}_jpg"].tobytes() for k in keys]
    coefs = _check_identity(datas, pillow=False)
    _, got = _decode_gpu(datas)
    for k, g, c in zip(keys, got, coefs):
        if f"{k}_rgb" in GOLD.files:
            assert np.array_equal(g.reshape(c.height, c.width, 3), GOLD[f"{k}_rgb"]), k
    for k, c in zip(keys, coefs):
        assert not c.entropy_pending or "prog0" in k, k


@pytest.mark.parametrize("seed", [1, 2, 3])
def test_progressive_sweep_matches_pillow(seed):
    datas = _sweep(seed)
    coefs = _check_identity(datas)
    assert not any(c.entropy_pending for c in coefs)


def test_progressive_corrupt_scan_data():
    """Bytes overwritten inside the scans (bad codes, runs past the band,
    EOB runs over the end): the device decode still equals the host
    decoder, which follows libjpeg's C paths on such data."""
    rng = np.random.default_rng(11)
    datas = []
    for i in range(12):
        d = bytearray(_encode(_smooth(rng, 90 + 7 * i, 120), quality=85, progressive=True,
                              subsampling=i % 3))
        for _ in range(3):
            _, s, e = _scans(bytes(d))[int(rng.integers(0, len(_scans(bytes(d)))))]
            if e - s > 4:
                at = int(rng.integers(s, e - 1))
                if d[at - 1] != 0xFF:
                    d[at] = int(rng.integers(0, 0xFF))
        datas.append(bytes(d))
    coefs = _check_identity(datas, pillow=False)
    assert not any(c.entropy_pending for c in coefs)


def test_progressive_scan_data_runs_out():
    """A scan whose data stops before its last block (bytes cut from its
    middle) while the later scans still arrive: the rest of that scan is
    skipped (libjpeg's insufficient data), the file still decodes on the
    device, and equals the host decoder."""
    rng = np.random.default_rng(12)
    datas = []
    for i in range(10):
        d = _encode(_smooth(rng, 80 + 9 * i, 100), quality=90, progressive=True, subsampling=i % 3)
        sc = _scans(d)
        _, s, e = sc[int(rng.integers(0, len(sc)))]
        if e - s < 8:
            continue
        cut = int(rng.integers(s + 1, e - 2))
        keep = int(rng.integers(cut + 1, e))
        if d[cut - 1] == 0xFF:
            cut += 1
        datas.append(d[:cut] + d[keep:] if d[keep - 1] != 0xFF else d)
    coefs = _check_identity(datas, pillow=False)
    assert not any(c.entropy_pending for c in coefs)


def test_progressive_mixed_batch_and_resize():
    """Progressive, sequential and host-decoded (arithmetic) files in one
    batch call, resized and cropped: each equals the host decode resized the
    same way (jpeg_resize_crop_host on decoded pixels)."""
    import jpeg_arith_enc as A

    rng = np.random.default_rng(13)
    datas = _sweep(21, n=6, max_side=400) + [_encode(_smooth(rng, 300, 200), quality=90),
                                              A.encode_progressive(_smooth(rng, 64, 96), q=2)]
    coefs, got = _decode_gpu(datas)
    for i, (d, g, c) in enumerate(zip(datas, got, coefs)):
        assert np.array_equal(g.reshape(c.height, c.width, 3), capi.jpeg_decode(d)), i
    geoms = []
    for c in coefs:
        s = min(c.width, c.height)
        rw, rh = max(1, c.width * 64 // s), max(1, c.height * 64 // s)
        cw, ch = min(56, rw), min(56, rh)
        geoms.append((0, 0, c.width, c.height, rw, rh, (rw - cw) // 2, (rh - ch) // 2, cw, ch, 0))
    want, entries = [], []
    for d, (wx, wy, ww, wh, rw, rh, cx, cy, cw, ch, flip) in zip(datas, geoms):
        win = np.ascontiguousarray(capi.jpeg_decode(d))
        o = np.zeros((ch, cw * 3), np.uint8)
        want.append((o, win))
        entries.append(dict(src=win.ctypes.data, src_stride=ww * 3, src_w=ww, src_h=wh, channels=3, resize_w=rw,
                            resize_h=rh, crop_x=cx, crop_y=cy, crop_w=cw, crop_h=ch, flip=flip, dst=o.ctypes.data,
                            dst_stride=cw * 3))
    arr, n = capi.make_images(entries)
    capi.resize_crop_host(arr, n, capi.MXD_U8, 0)
    _, dev = _decode_gpu(datas, geoms)
    for i, (g, (w_, _)) in enumerate(zip(dev, want)):
        assert np.array_equal(g, w_), i


def test_progressive_large_images():
    """1600x1200 and 2400x1800 progressive photos, one grey with restart
    markers, finished on the device: equal to the host decoder and Pillow."""
    rng = np.random.default_rng(14)
    datas = [_encode(_smooth(rng, 1200, 1600), quality=95, progressive=True, subsampling=2),
             _encode(_smooth(rng, 1800, 2400), quality=92, progressive=True, subsampling=0),
             _encode(_smooth(rng, 1200, 1600, 1), quality=97, progressive=True, restart_marker_blocks=5)]
    coefs = _check_identity(datas)
    assert not any(c.entropy_pending for c in coefs)
