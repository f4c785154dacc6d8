"""The native JPEG decoder behind load_image (SURVEY.md §8f row f1;
mlx-data_amd/csrc/jpeg.cpp) against libjpeg-turbo, which the reference links
(core/image/ImageJPEG.cpp:99-146, libjpeg defaults: ISLOW IDCT, fancy
upsampling, RGB out, grey replicated, CMYK -> first three raw channels).

Pinned two ways: the committed fixtures (tests/golden/jpeg.npz, encoded and
decoded by Pillow's bundled libjpeg-turbo; generator make_jpeg_golden.py) and,
on hosts with Pillow, a seeded sweep decoded live by Pillow.  Bit-exact
everywhere, including libjpeg's block smoothing of progressive files whose
scans leave low-frequency coefficients inexact (truncated progressive data;
fixtures `prog_trunc_*` and a live sweep of files cut at and inside scans)."""
import io
import os

import numpy as np
import pytest

from mlx_data_amd import capi

GOLD_PATH = os.path.join(os.path.dirname(__file__), "golden", "jpeg.npz")
GOLD = np.load(GOLD_PATH)
CASES = sorted(k[:-4] for k in GOLD.files if k.endswith("_jpg"))


@pytest.mark.parametrize("case", CASES)
def test_fixture_bit_exact(case):
    data = GOLD[f"{case}_jpg"]
    want = GOLD[f"{case}_rgb"]
    got = capi.jpeg_decode(data)
    assert got.shape == want.shape
    assert np.array_equal(got, want), (case, int(np.abs(got.astype(int) - want.astype(int)).max()))


def test_info_and_signature():
    data = GOLD["sub2_prog0_jpg"]
    w, h, c = capi.jpeg_info(data)
    assert (h, w, c) == (*GOLD["sub2_prog0_rgb"].shape[:2], 3)
    assert capi.jpeg_info(GOLD["grey_jpg"])[2] == 1
    assert capi.jpeg_info(GOLD["cmyk_jpg"])[2] == 4
    assert capi.lib().mxd_is_jpeg(bytes(data[:3]), 3) == 1
    assert capi.lib().mxd_is_jpeg(b"\x89PNG", 4) == 0


def _smooth(rng, h, w, c):
    x = np.linspace(0, 6, w)[None, :, None]
    y = np.linspace(0, 4, h)[:, None, None]
    base = (np.sin(x * 1.3 + y * 0.7) + np.cos(y * 2.1 - x * 0.4)) * 60 + 128
    return np.clip(base + rng.normal(0, 25, (h, w, c)) + np.arange(c)[None, None, :] * 20, 0, 255).astype(np.uint8)


@pytest.mark.parametrize("seed", range(12))
def test_live_pillow_sweep(seed):
    Image = pytest.importorskip("PIL.Image")
    rng = np.random.default_rng(seed)
    for _ in range(6):
        h, w = int(rng.integers(1, 140)), int(rng.integers(1, 140))
        grey = rng.random() < 0.2
        a = _smooth(rng, h, w, 1 if grey else 3)
        kw = dict(quality=int(rng.integers(5, 101)), progressive=bool(rng.random() < 0.5),
                  optimize=bool(rng.random() < 0.5))
        if not grey:
            kw["subsampling"] = int(rng.integers(0, 3))
        if rng.random() < 0.3:
            kw["restart_marker_blocks"] = int(rng.integers(1, 6))
        b = io.BytesIO()
        Image.fromarray(a[:, :, 0] if grey else a).save(b, "JPEG", **kw)
        data = b.getvalue()
        want = np.asarray(Image.open(io.BytesIO(data)).convert("RGB"))
        assert np.array_equal(capi.jpeg_decode(data), want), (h, w, kw)


def _cut_progressive(data, rng):
    """Cuts a progressive file after a whole scan or inside a scan's entropy-coded data."""
    sos = [i for i in range(len(data) - 1) if data[i] == 0xFF and data[i + 1] == 0xDA]
    k = int(rng.integers(1, len(sos)))
    if rng.random() < 0.4:
        return data[:sos[k]]
    p = sos[k - 1]
    s = p + 2 + int.from_bytes(data[p + 2:p + 4], "big")
    e = s
    while not (data[e] == 0xFF and data[e + 1] != 0 and not 0xD0 <= data[e + 1] <= 0xD7):
        e += 1
    if e - s < 3:
        return data[:sos[k]]
    m = int(rng.integers(s + 1, e))
    while data[m - 1] == 0xFF:
        m += 1
    return data[:m]


@pytest.mark.parametrize("seed", range(6))
def test_truncated_progressive_block_smoothing(seed):
    """Progressive files cut after / inside a scan: libjpeg-turbo estimates
    the missing low-frequency AC coefficients (and, with no AC data at all,
    the DC) from the 5x5 DC neighbourhood, rows past the last complete iMCU
    row with the progression status from before the cut scan; Pillow appends
    the EOI libjpeg's memory source fakes for the reference."""
    Image = pytest.importorskip("PIL.Image")
    ImageFile = pytest.importorskip("PIL.ImageFile")
    rng = np.random.default_rng(500 + seed)
    prev = ImageFile.LOAD_TRUNCATED_IMAGES
    ImageFile.LOAD_TRUNCATED_IMAGES = True
    try:
        for i in range(10):
            h, w = int(rng.integers(1, 130)), int(rng.integers(1, 130))
            grey = i % 5 == 4
            kw = dict(quality=int(rng.integers(10, 96)), progressive=True)
            if not grey:
                kw["subsampling"] = i % 3
            b = io.BytesIO()
            a = _smooth(rng, h, w, 1 if grey else 3)
            Image.fromarray(a[:, :, 0] if grey else a).save(b, "JPEG", **kw)
            data = _cut_progressive(b.getvalue(), rng)
            want = np.asarray(Image.open(io.BytesIO(data)).convert("RGB"))
            assert np.array_equal(capi.jpeg_decode(data), want), (i, h, w, kw, len(data))
    finally:
        ImageFile.LOAD_TRUNCATED_IMAGES = prev


def _segment(marker, payload):
    return bytes([0xFF, marker]) + (len(payload) + 2).to_bytes(2, "big") + payload


def test_errors_carry_libjpeg_messages():
    with pytest.raises(capi.MxdError, match="Not a JPEG file"):
        capi.jpeg_info(b"\x89PNG\r\n\x1a\n" + bytes(32))
    # a hierarchical (differential) frame, which libjpeg-turbo does not decode
    sof13 = b"\xff\xd8" + _segment(0xCD, bytes([8, 0, 8, 0, 8, 1, 1, 0x11, 0]))
    with pytest.raises(capi.MxdError, match="Unsupported JPEG process: SOF type 0xcd"):
        capi.jpeg_info(sof13)
    # 12-bit precision
    sof1_12 = b"\xff\xd8" + _segment(0xC1, bytes([12, 0, 8, 0, 8, 1, 1, 0x11, 0]))
    with pytest.raises(capi.MxdError, match="precision"):
        capi.jpeg_info(sof1_12)
    # header cut inside the frame
    data = bytes(GOLD["sub2_prog0_jpg"])
    sof = data.index(b"\xff\xc0")
    with pytest.raises(capi.MxdError):
        capi.jpeg_info(data[:sof + 6])


def test_load_image_uses_native_decoder(tmp_path):
    """load_image on JPEG bytes (from_memory) and files: the fixture pixels, in
    the reference's (H, W, 3) layout; info=True gives (w, h)."""
    from mlx_data_amd import data as dx

    raw = GOLD["caltech_300x200_jpg"]
    want = GOLD["caltech_300x200_rgb"]
    (tmp_path / "x.jpg").write_bytes(raw.tobytes())
    b = dx.buffer_from_vector([dict(f=b"x.jpg", m=raw)])
    s = b.load_image("f", prefix=str(tmp_path), output_key="img").load_image("m", from_memory=True)[0]
    assert np.array_equal(s["img"], want) and np.array_equal(s["m"], want)
    info = b.load_image("f", prefix=str(tmp_path), info=True)[0]["f"]
    assert info.tolist() == [want.shape[1], want.shape[0]]
    grey = dx.buffer_from_vector([dict(m=GOLD["grey_jpg"])]).load_image("m", from_memory=True)[0]["m"]
    assert np.array_equal(grey, GOLD["grey_rgb"]) and grey.shape[2] == 3
    bad = np.frombuffer(bytes(raw[:200]) + b"\xff\xd9", np.uint8)
    bad = np.concatenate([bad[:2], np.frombuffer(b"\xff\xcd\x00\x0b\x08\x00\x08\x00\x08\x01\x01\x11\x00", np.uint8),
                          bad[2:]])
    with pytest.raises(RuntimeError, match=r"load_jpeg: could not load from memory \(Unsupported JPEG process"):
        dx.buffer_from_vector([dict(m=bad)]).load_image("m", from_memory=True)[0]


def test_host_and_pipeline_stats_count(tmp_path):
    """The diagnostics bench_pipeline --stats reads: mxd_host_stats counts
    marker parses / loads (and resets), the pipeline's stage timers count
    load_image calls and time the batch's fetches."""
    from mlx_data_amd import _pipeline
    from mlx_data_amd import data as dx

    raw = GOLD["caltech_300x200_jpg"]
    (tmp_path / "x.jpg").write_bytes(raw.tobytes())
    capi.host_stats(reset=True)
    capi.JpegCoefs(raw.tobytes(), device_entropy=True)
    capi.JpegCoefs.load(str(tmp_path / "x.jpg"))
    hs = capi.host_stats(reset=True)
    assert hs["parses"] == 2 and hs["parse_s"] > 0
    assert capi.host_stats()["parses"] == 0
    _pipeline._pipe_stats(True)
    d = dx.buffer_from_vector([dict(f=b"x.jpg")] * 6).to_stream().load_image("f", prefix=str(tmp_path)).batch(3)
    assert sum(1 for _ in d) == 2
    ps = _pipeline._pipe_stats(True)
    assert ps[5] == 6 and ps[0] > 0 and ps[2] >= ps[0] and ps[1] >= ps[0]
    assert _pipeline._pipe_stats(False)[5] == 0


def _arith_cases(seed, n, progressive):
    import jpeg_arith_enc as A

    rng = np.random.default_rng(seed)
    for t in range(n):
        h, w = int(rng.integers(1, 90)), int(rng.integers(1, 90))
        grey = t % 4 == 3
        if t % 2:
            img = rng.integers(0, 256, (h, w) if grey else (h, w, 3), dtype=np.uint8)
        else:
            img = _smooth(rng, h, w, 1 if grey else 3)
            img = img[:, :, 0] if grey else img
        kw = dict(q=int(rng.integers(1, 30)))
        if t % 3 == 0:
            kw["restart_mcus"] = int(rng.integers(1, 5))
        if t % 5 == 0:  # DAC conditioning other than the defaults
            kw["dac"] = (int(rng.integers(0, 4)), int(rng.integers(4, 16)), int(rng.integers(1, 63)))
        yield (A.encode_progressive if progressive else A.encode)(img, **kw), kw


@pytest.mark.parametrize("progressive", [False, True])
def test_arithmetic_coded_files_match_pillow(progressive):
    """Arithmetic-coded JPEGs (SOF9 sequential, SOF10 progressive; the
    reference's libjpeg-turbo build decodes them, super/CMakeLists.txt):
    tests/jpeg_arith_enc.py writes them from T.81's QM coder and statistical
    models -- Pillow decodes every one to the pixels of the same
    coefficients Huffman-coded (the encoder is right) -- and the host decoder
    gives Pillow's bytes: noise and smooth images, grey and 4:4:4, restart
    intervals, DAC conditioning.  They are entropy-decoded on the host on the
    device route too (parse_coefs)."""
    Image = pytest.importorskip("PIL.Image")

    for i, (data, kw) in enumerate(_arith_cases(31 + progressive, 24, progressive)):
        pil = np.asarray(Image.open(io.BytesIO(data)).convert("RGB"))
        assert np.array_equal(capi.jpeg_decode(data), pil), (i, kw)
        if i < 4:  # the encoder: the same coefficients Huffman-coded decode alike
            c = capi.JpegCoefs(data, device_entropy=True)
            assert not c.entropy_pending and np.array_equal(c.finish(), pil), (i, kw)


def test_truncated_progressive_arithmetic_files_match_pillow():
    """Progressive arithmetic-coded files cut between scans and inside their
    entropy-coded data (an EOI appended, as libjpeg's memory source fakes
    one): past a cut the decoder reads zeros (T.81 allows a marker inside
    arithmetic-coded data) and block smoothing fills what later scans would
    have held; Pillow's bytes for every cut between scans.  A cut inside a
    scan decodes the rest of it from zeros, which can leave coefficients far
    outside any 8-bit image's range; where the IDCT's 16-bit SIMD
    dequantisation in Pillow's libjpeg-turbo then departs from jidctint.c
    (test_gpu_jpeg_entropy.py's out-of-range test) a few pixels differ, so
    those cuts must match in all but a few percent of files."""
    Image = pytest.importorskip("PIL.Image")
    ImageFile = pytest.importorskip("PIL.ImageFile")
    import jpeg_arith_enc as A

    prev = ImageFile.LOAD_TRUNCATED_IMAGES
    ImageFile.LOAD_TRUNCATED_IMAGES = True
    try:
        rng = np.random.default_rng(9)
        between = inside = inside_bad = 0
        for t in range(12):
            h, w = int(rng.integers(16, 120)), int(rng.integers(16, 120))
            d = A.encode_progressive(_smooth(rng, h, w, 3), q=int(rng.integers(1, 12)),
                                     restart_mcus=3 if t % 3 == 0 else 0)
            sos = [i for i in range(len(d) - 1) if d[i] == 0xFF and d[i + 1] == 0xDA]
            hdr = [i + 2 + int.from_bytes(d[i + 2:i + 4], "big") for i in sos]  # each scan's data start
            for cut in sos[1:]:
                m = d[:cut] + b"\xff\xd9"
                want = np.asarray(Image.open(io.BytesIO(m)).convert("RGB"))
                assert np.array_equal(capi.jpeg_decode(m), want), (t, cut)
                between += 1
            for a, b in zip(hdr, sos[1:] + [len(d) - 2]):
                if b - a <= 3:
                    continue
                m = d[:int(rng.integers(a + 1, b - 1))] + b"\xff\xd9"
                want = np.asarray(Image.open(io.BytesIO(m)).convert("RGB"))
                inside += 1
                inside_bad += not np.array_equal(capi.jpeg_decode(m), want)
        assert between > 100 and inside > 100
        assert inside_bad <= 0.03 * inside, (inside_bad, inside)
    finally:
        ImageFile.LOAD_TRUNCATED_IMAGES = prev


def test_lossless_files_match_pillow():
    """Lossless Huffman-coded JPEGs (SOF3, 8-bit; libjpeg-turbo 3.x, the
    reference's build, decodes them): tests/jpeg_enc.py encode_lossless writes
    every predictor 1..7, point transforms, restart intervals, grey and
    three-component files; the decoder gives Pillow's bytes on each, on files
    cut inside their data (the row the data runs out in decodes on from zero
    bits, later rows are uniform grey, as jdlhuff.c does), and refuses a
    JFIF-marked (YCbCr) one as libjpeg-turbo does (no colour conversion in
    lossless mode).  Such files finish on the host on the device route."""
    Image = pytest.importorskip("PIL.Image")
    ImageFile = pytest.importorskip("PIL.ImageFile")
    import jpeg_enc as J

    rng = np.random.default_rng(5)
    cut_files = []
    for t in range(28):
        h, w = int(rng.integers(1, 60)), int(rng.integers(1, 60))
        grey = t % 3 == 2
        if t % 2:
            img = rng.integers(0, 256, (h, w) if grey else (h, w, 3), dtype=np.uint8)
        else:
            img = _smooth(rng, h, w, 1 if grey else 3)
            img = img[:, :, 0] if grey else img
        kw = dict(psv=1 + t % 7, pt=int(rng.integers(1, 4)) if t % 4 == 0 else 0,
                  restart_rows=int(rng.integers(1, 4)) if t % 5 == 0 and h > 1 else 0)
        data = J.encode_lossless(img, **kw)
        pil = np.asarray(Image.open(io.BytesIO(data)).convert("RGB"))
        assert np.array_equal(capi.jpeg_decode(data), pil), (t, kw)
        if t % 2 == 0 and h >= 8:
            cut_files.append(data)
        if t < 3:
            c = capi.JpegCoefs(data, device_entropy=True)
            assert not c.entropy_pending and not c.device_ok and np.array_equal(c.finish(), pil)
    prev = ImageFile.LOAD_TRUNCATED_IMAGES
    ImageFile.LOAD_TRUNCATED_IMAGES = True
    try:
        for data in cut_files:
            sos = data.index(b"\xff\xda")
            for cut in rng.integers(sos + 14, len(data) - 2, 4):
                m = data[:int(cut)] + b"\xff\xd9"
                assert np.array_equal(capi.jpeg_decode(m), np.asarray(Image.open(io.BytesIO(m)).convert("RGB")))
    finally:
        ImageFile.LOAD_TRUNCATED_IMAGES = prev
    jfif = _segment(0xE0, b"JFIF\x00\x01\x01\x00\x00\x01\x00\x01\x00\x00")
    with pytest.raises(capi.MxdError, match="Unsupported color conversion request"):
        capi.jpeg_decode(J.encode_lossless(_smooth(rng, 9, 9, 3), markers=jfif))


def test_device_entropy_parse_routes_and_host_finish():
    """mxd_jpeg_coefs_parse(device_entropy=1) (CPU half of the device entropy
    decode, csrc/jpeghuff.h): baseline one-scan files are only parsed
    (entropy_pending), every other file -- progressive ones included (round
    6: the device progressive decode was retired) -- is entropy-decoded on
    the host; either way the host finish gives the decoder's bytes (Pillow's
    libjpeg-turbo)."""
    Image = pytest.importorskip("PIL.Image")
    rng = np.random.default_rng(77)
    for i in range(24):
        h, w = int(rng.integers(1, 160)), int(rng.integers(1, 160))
        grey = i % 5 == 4
        prog = i % 4 == 1
        kw = dict(quality=int(rng.integers(5, 101)), progressive=prog, optimize=bool(rng.random() < 0.4))
        if not grey:
            kw["subsampling"] = i % 3
        if i % 3 == 2:
            kw["restart_marker_blocks"] = int(rng.integers(1, 5))
        b = io.BytesIO()
        a = _smooth(rng, h, w, 1 if grey else 3)
        Image.fromarray(a[:, :, 0] if grey else a).save(b, "JPEG", **kw)
        data = b.getvalue()
        c = capi.JpegCoefs(data, device_entropy=True)
        assert c.entropy_pending == (not prog), (i, kw)
        assert np.array_equal(c.finish(), np.asarray(Image.open(io.BytesIO(data)).convert("RGB"))), (i, kw)
    # fixtures: CMYK / truncated files are decoded on the host
    for k in [k[:-4] for k in GOLD.files if k.endswith("_jpg")]:
        data = bytes(GOLD[f"{k}_jpg"])
        c = capi.JpegCoefs(data, device_entropy=True)
        if "trunc" in k or ("prog" in k and "prog0" not in k):
            assert not c.entropy_pending, k
        if "cmyk" in k:  # (round 6: four-component sequential files decode on the device too)
            assert c.entropy_pending and c.device_ok, k
        if c.device_ok:
            assert np.array_equal(c.finish(), GOLD[f"{k}_rgb"]), k


def test_coefs_load_reads_files_like_parse(tmp_path):
    """mxd_jpeg_coefs_load (the pipeline's LoadImage on device decode): the
    file read straight into the handle gives mxd_jpeg_coefs_parse's routes and
    bytes; a file without the JPEG signature gives no handle (the caller's
    other decoders take it); unreadable / broken files are errors."""
    Image = pytest.importorskip("PIL.Image")
    rng = np.random.default_rng(78)
    for i, kw in enumerate([dict(quality=90), dict(quality=70, progressive=True), dict(quality=85, subsampling=0,
                                                                                       restart_marker_blocks=2)]):
        b = io.BytesIO()
        Image.fromarray(_smooth(rng, 60 + i, 83, 3)).save(b, "JPEG", **kw)
        p = tmp_path / f"f{i}.jpg"
        p.write_bytes(b.getvalue())
        for dev in (True, False):
            c = capi.JpegCoefs.load(str(p), device_entropy=dev)
            ref = capi.JpegCoefs(b.getvalue(), device_entropy=dev)
            assert (c.width, c.height, c.entropy_pending) == (ref.width, ref.height, ref.entropy_pending), (i, dev)
            assert np.array_equal(c.finish(), ref.finish()), (i, dev)
    png = tmp_path / "x.png"
    Image.fromarray(_smooth(rng, 8, 8, 3)).save(png)
    assert capi.JpegCoefs.load(str(png)) is None
    with pytest.raises(capi.MxdError, match="could not load"):
        capi.JpegCoefs.load(str(tmp_path / "missing.jpg"))
    bad = tmp_path / "bad.jpg"
    bad.write_bytes(b"\xff\xd8\xff\xe0\x00\x10JFIF" + bytes(40))
    with pytest.raises(capi.MxdError):
        capi.JpegCoefs.load(str(bad))


def test_device_entropy_tables_after_the_scan_go_to_the_host():
    """a DHT or DRI between the recorded scan and EOI must not
    reach the device decode (the host decodes the scan at its SOS with the
    tables and interval in force there).  Such files are entropy-decoded on
    the host and give Pillow's bytes."""
    Image = pytest.importorskip("PIL.Image")
    rng = np.random.default_rng(5)
    b = io.BytesIO()
    Image.fromarray(_smooth(rng, 48, 64, 3)).save(b, "JPEG", quality=80)
    data = b.getvalue()
    assert capi.JpegCoefs(data, device_entropy=True).entropy_pending
    i = data.index(b"\xff\xc4")
    n = int.from_bytes(data[i + 2:i + 4], "big")
    dht = data[i:i + 2 + n]
    # a DC table 0 of other codes: the device would decode with it
    other = b"\xff\xc4\x00\x1f\x00" + bytes([0, 1, 5, 1, 1, 1, 1, 1, 1, 0, 0, 0, 0, 0, 0, 0]) + bytes(range(11, -1, -1))
    dri = b"\xff\xdd\x00\x04\x00\x02"
    for tail in (dht, other, dri, other + dri):
        mod = data[:-2] + tail + data[-2:]
        c = capi.JpegCoefs(mod, device_entropy=True)
        assert not c.entropy_pending, tail[:2]
        assert np.array_equal(c.finish(), np.asarray(Image.open(io.BytesIO(mod)).convert("RGB")))


def test_device_entropy_parse_errors_match_host():
    """The markers-only parse reports the host decode's errors (a DC table
    with a category above 15 is libjpeg's "Bogus Huffman table definition")."""
    data = bytearray(GOLD["sub2_prog0_jpg"].tobytes())
    dht = data.index(b"\xff\xc4")
    # first DHT: class/index byte, 16 counts, then the values: make a DC value 16
    tc = data[dht + 4]
    assert tc >> 4 == 0  # a DC table first (Pillow writes DC 0 first)
    vals = dht + 5 + 16
    data[vals] = 16
    for dev in (False, True):
        with pytest.raises(capi.MxdError, match="Bogus Huffman table definition"):
            capi.JpegCoefs(bytes(data), device_entropy=dev)


def test_deep_huffman_tables_host_decode_matches_pillow():
    """Huffman tables with many codes longer than 11 bits low in the code
    space (tests/jpeg_enc.py): the host decoder's slow path equals Pillow's
    libjpeg-turbo, and the device-entropy parse still takes such files (the
    GPU decoder searches their tables; tests/test_gpu_jpeg_entropy.py)."""
    import jpeg_enc as J
    from PIL import Image

    rng = np.random.default_rng(32)
    for a, rs in [(rng.integers(0, 256, (45, 61), dtype=np.uint8), 0),
                  (rng.integers(0, 256, (70, 90, 3), dtype=np.uint8), 5)]:
        d = J.encode(a, restart_mcus=rs, q=1)
        want = np.asarray(Image.open(io.BytesIO(d)).convert("RGB"))
        assert np.array_equal(capi.jpeg_decode(d), want)
        c = capi.JpegCoefs(d, device_entropy=True)
        assert c.entropy_pending
        assert np.array_equal(c.finish(), want)


def test_scalar_byte_scans_match_avx512(tmp_path):
    """The marker parse's and unstuff's AVX-512 forms (chosen when the CPU
    has them) and the scalar ones (MXD_NO_AVX512=1, in a child process) give
    the same segment split and the same decodes: every fixture, through the
    markers-only parse and the host finish, digested in both processes."""
    import subprocess
    import sys

    script = (
        "import hashlib, sys, numpy as np\n"
        "sys.path.insert(0, %r)\n"
        "from mlx_data_amd import capi\n"
        "g = np.load(%r)\n"
        "h = hashlib.sha256()\n"
        "for k in sorted(f for f in g.files if f.endswith('_jpg')):\n"
        "    d = g[k].tobytes()\n"
        "    try:\n"
        "        c = capi.JpegCoefs(d, device_entropy=True)\n"
        "        h.update(bytes([c.entropy_pending])); h.update(c.finish().tobytes())\n"
        "    except capi.MxdError as e:\n"
        "        h.update(str(e).encode())\n"
        "print(h.hexdigest())\n") % (os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                        "mlx-data_amd"), GOLD_PATH)
    out = {}
    for flag in ("0", "1"):
        env = dict(os.environ, MXD_NO_AVX512=flag)
        out[flag] = subprocess.run([sys.executable, "-c", script], env=env, capture_output=True, text=True,
                                   check=True, timeout=300).stdout.strip()
    assert out["0"] == out["1"] and len(out["0"]) == 64


def test_ycck_and_cmyk_decode_like_libjpeg():
    """Four-component files (Adobe transform 2 = YCCK, 0 = CMYK; tests/
    jpeg_enc.py) decode to the first three channels of libjpeg's CMYK output
    (ImageJPEG.cpp:112-124): YCCK through jdcolor.c ycck_cmyk_convert (C, M,
    Y = 255 - R, G, B).  Pinned to libjpeg-turbo through Pillow, whose Adobe
    CMYK comes un-inverted (255 - libjpeg's raw values)."""
    Image = pytest.importorskip("PIL.Image")
    import jpeg_enc as J

    rng = np.random.default_rng(43)
    for i in range(8):
        h, w = int(rng.integers(1, 90)), int(rng.integers(1, 90))
        d = J.encode(_smooth(rng, h, w, 4), q=int(rng.integers(1, 8)), adobe=2 if i % 2 == 0 else 0,
                     restart_mcus=2 if i % 4 == 3 else 0)
        pil = Image.open(io.BytesIO(d))
        assert pil.mode == "CMYK"
        assert np.array_equal(capi.jpeg_decode(d), 255 - np.asarray(pil)[:, :, :3]), i
        c = capi.JpegCoefs(d, device_entropy=True)
        assert c.device_ok and c.entropy_pending, i
        assert np.array_equal(c.finish(), 255 - np.asarray(pil)[:, :, :3]), i
