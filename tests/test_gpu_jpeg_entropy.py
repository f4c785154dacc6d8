"""GPU: the device-side entropy (Huffman) decode of sequential JPEG scans
(csrc/jpeghuff.hip; SURVEY.md §8f f1 "later a device-side decode", VERDICT r3
missing 1).  With mxd_jpeg_coefs_parse(device_entropy=1) a qualifying file is
only parsed on the host; its entropy-coded segments are decoded on the GPU in
parallel subsequences that synchronise, then finished (IDCT, upsampling,
colour) and resized there.

Every check is bit-exact against the host decoder (tests/test_jpeg.py pins it
to libjpeg-turbo through Pillow), at identity geometry (the decoded image):

* the committed fixtures (tests/golden/jpeg.npz: every sampling layout, grey,
  restart markers, odd sizes; progressive / CMYK / truncated ones fall back to
  the host entropy decode and must still match);
* seeded Pillow encodes: sizes 1..700, qualities 5..100, 4:4:4 / 4:2:2 /
  4:2:0 / grey, optimised tables, restart intervals in blocks and rows;
* short subsequences (MXD_TUNE_HUFF_BITS 32 / 64 / 96): hundreds of
  subsequences per image that must find their symbol boundaries, block and
  coefficient position by propagation;
* corrupt entropy data (bytes overwritten: bad codes, runs past 63) and data
  that runs out before the last MCU while the file still ends with EOI
  (libjpeg's insufficient-data rule: the rest of the interval stays zero);
* batches across several jobs / images, resize + crop windows, device
  destinations;
* both word sources: LDS (jobs whose words fit it, the default) and device
  memory through the prefetching reader (MXD_TUNE_HUFF_GLOBAL = 1, what
  jobs too large for LDS use)."""
import io
import os

import numpy as np
import pytest

from mlx_data_amd import capi

pytestmark = pytest.mark.gpu

GOLD = np.load(os.path.join(os.path.dirname(__file__), "golden", "jpeg.npz"))
CASES = sorted(k[:-4] for k in GOLD.files if k.endswith("_jpg"))


def _encode(a, **kw):
    from PIL import Image

    b = io.BytesIO()
    Image.fromarray(a if a.shape[2] == 3 else a[:, :, 0]).save(b, "JPEG", **kw)
    return b.getvalue()


def _smooth(rng, h, w, c=3):
    gh, gw = h // 16 + 2, w // 16 + 2
    grid = rng.integers(0, 256, (gh, gw, c)).astype(np.float32)
    yi = np.minimum(np.arange(h) * (gh - 1) // max(1, h - 1), gh - 2)
    xi = np.minimum(np.arange(w) * (gw - 1) // max(1, w - 1), gw - 2)
    f = grid[yi][:, xi] * 0.6 + grid[yi + 1][:, xi + 1] * 0.4 + rng.normal(0, 14, (h, w, c))
    return np.clip(f, 0, 255).astype(np.uint8)


def _decode_gpu(datas, geoms=None, f32=False, device_dst=False):
    """mxd_jpeg_resize_crop_host / _to_device over device-entropy coefs;
    geoms default to identity (the decoded image)."""
    coefs = [capi.JpegCoefs(d, device_entropy=True) for d in datas]
    if geoms is None:
        geoms = [(0, 0, c.width, c.height, c.width, c.height, 0, 0, c.width, c.height, 0) for c in coefs]
    elem = 4 if f32 else 1
    outs, entries, bufs = [], [], []
    for c, (wx, wy, ww, wh, rw, rh, cx, cy, cw, ch, flip) in zip(coefs, geoms):
        row = cw * 3 * elem
        if device_dst:
            d = capi.DeviceBuffer(row * ch, 0)
            d.memset(0)
            bufs.append((d, row, ch))
            ptr = d.ptr
        else:
            o = np.zeros((ch, row), np.uint8)
            outs.append(o)
            ptr = o.ctypes.data
        entries.append(dict(coefs=c, win_x=wx, win_y=wy, win_w=ww, win_h=wh, resize_w=rw, resize_h=rh, crop_x=cx,
                            crop_y=cy, crop_w=cw, crop_h=ch, flip=flip, dst=ptr, dst_stride=row))
    arr, n = capi.make_jpeg_images(entries)
    dt = capi.MXD_F32_DIV255 if f32 else capi.MXD_U8
    if device_dst:
        capi.jpeg_resize_crop_to_device(arr, n, dt, 0)
        for d, row, ch in bufs:
            outs.append(d.download((ch, row), np.uint8))
            d.free()
    else:
        capi.jpeg_resize_crop_host(arr, n, dt, 0)
    return coefs, outs


def _pillow(d):
    from PIL import Image

    return np.asarray(Image.open(io.BytesIO(d)).convert("RGB"))


def _check_identity(datas, pillow=True):
    """The device decode equals the host decoder and (pillow) Pillow's
    libjpeg-turbo decode of the same file (the reference's decoder,
    ImageJPEG.cpp:99-146) -- directly, not only through the host decoder
    (VERDICT r4 weak 1)."""
    coefs, got = _decode_gpu(datas)
    for i, (d, g, c) in enumerate(zip(datas, got, coefs)):
        img = g.reshape(c.height, c.width, 3)
        assert np.array_equal(img, capi.jpeg_decode(d)), (i, c.entropy_pending)
        if pillow:
            assert np.array_equal(img, _pillow(d)), (i, c.entropy_pending)
    return coefs


def _sweep(seed, n=16, max_side=700):
    rng = np.random.default_rng(seed)
    datas = []
    for i in range(n):
        h, w = int(rng.integers(1, max_side)), int(rng.integers(1, max_side))
        grey = i % 7 == 6
        kw = dict(quality=int(rng.integers(5, 101)), optimize=bool(rng.random() < 0.3))
        if not grey:
            kw["subsampling"] = i % 3
        r = rng.random()
        if r < 0.2:
            kw["restart_marker_blocks"] = int(rng.integers(1, 8))
        elif r < 0.35:
            kw["restart_marker_rows"] = int(rng.integers(1, 4))
        datas.append(_encode(_smooth(rng, h, w, 1 if grey else 3), **kw))
    return datas


def test_fixtures_identity():
    keys = [k for k in CASES if not k.startswith("cmyk")]
    datas = [GOLD[f"{k}_jpg"].tobytes() for k in keys]
    coefs = _check_identity(datas, pillow=False)
    _, got = _decode_gpu(datas)
    for k, g, c in zip(keys, got, coefs):  # the fixtures' committed libjpeg-turbo decodes
        if f"{k}_rgb" in GOLD.files and "trunc" not in k:
            assert np.array_equal(g.reshape(c.height, c.width, 3), GOLD[f"{k}_rgb"]), k
    assert sum(c.entropy_pending for c in coefs) >= 5  # the baseline fixtures go to the device


@pytest.fixture(params=[0, 1], ids=["lds_words", "global_words"])
def word_source(request):
    prev = capi.set_tuning(capi.MXD_TUNE_HUFF_GLOBAL, request.param)
    yield request.param
    capi.set_tuning(capi.MXD_TUNE_HUFF_GLOBAL, prev)


def test_fill_bytes_before_markers(word_source):
    """0xFF fill bytes before restart markers and EOI (legal padding no
    Pillow file carries) are dropped like jdhuff.c drops them: the device
    decode equals the host decoder and Pillow."""
    rng = np.random.default_rng(12)
    datas = []
    for i in range(4):
        d = _encode(_smooth(rng, 120 + 40 * i, 170), quality=80 + 4 * i, subsampling=i % 3,
                    restart_marker_blocks=1 + i)
        s, e = _ecs_range(d)
        body = bytearray()
        k = s
        while k < e:  # before every RSTn marker: one to three fill bytes
            if d[k] == 0xFF and 0xD0 <= d[k + 1] <= 0xD7:
                body += b"\xff" * (1 + (k % 3))
                body += d[k:k + 2]
                k += 2
                continue
            body.append(d[k])
            k += 1
        datas.append(d[:s] + bytes(body) + b"\xff\xff" + d[e:])
    coefs = _check_identity(datas)
    assert all(c.entropy_pending for c in coefs)


@pytest.mark.parametrize("seed", range(4))
def test_encoded_sweep_identity(seed, word_source):
    coefs = _check_identity(_sweep(seed))
    assert all(c.entropy_pending for c in coefs)  # baseline, one scan: every file qualifies


@pytest.mark.parametrize("bits", [32, 64, 96])
def test_short_subsequences_synchronise(bits, word_source):
    prev = capi.set_tuning(capi.MXD_TUNE_HUFF_BITS, bits)
    try:
        _check_identity(_sweep(100 + bits, n=10, max_side=400))
    finally:
        capi.set_tuning(capi.MXD_TUNE_HUFF_BITS, prev)


def _ecs_range(d):
    """(start, end) of the entropy-coded data of a one-scan file (after SOS, up to EOI)."""
    sos = d.find(b"\xff\xda")
    start = sos + 2 + int.from_bytes(d[sos + 2:sos + 4], "big")
    end = d.rfind(b"\xff\xd9")
    return start, end


@pytest.mark.parametrize("bits", [0, 64])
def test_corrupt_and_short_entropy_data(bits, word_source):
    rng = np.random.default_rng(9)
    datas = []
    for i in range(12):
        h, w = int(rng.integers(16, 300)), int(rng.integers(16, 300))
        kw = dict(quality=int(rng.integers(30, 96)), subsampling=i % 3)
        if i % 4 == 3:
            kw["restart_marker_blocks"] = 2
        d = bytearray(_encode(_smooth(rng, h, w), **kw))
        s, e = _ecs_range(bytes(d))
        if i % 2 == 0:
            # overwrite bytes (never creating or breaking an 0xFF pair)
            for p in rng.integers(s, e, 6):
                if d[p] != 0xFF and d[p - 1] != 0xFF and d[p + 1] != 0x00:
                    d[p] = int(rng.integers(0, 0xFF))
        else:
            # cut entropy bytes out of the middle of the last segment: the data
            # runs out before the last MCUs, the file still ends with EOI
            last = max([s] + [bytes(d).rfind(bytes([0xFF, 0xD0 + m]), s, e) + 2 for m in range(8)])
            a = last + (e - last) // 3
            b = a + (e - last) // 3
            while d[a - 1] == 0xFF:  # never leave a dangling 0xFF (a marker) behind
                a += 1
            while b < e and d[b - 1] == 0xFF:
                b += 1
            del d[a:max(a, b)]
        datas.append(bytes(d))
    prev = capi.set_tuning(capi.MXD_TUNE_HUFF_BITS, bits)
    try:
        coefs = _check_identity(datas, pillow=False)  # corrupt data: host-decoder parity only
    finally:
        capi.set_tuning(capi.MXD_TUNE_HUFF_BITS, prev)
    assert sum(c.entropy_pending for c in coefs) >= 10


@pytest.mark.parametrize("f32,device_dst", [(False, False), (True, False), (True, True)])
def test_resize_crop_windows(f32, device_dst):
    """Resize / crop / mirror windows of device-entropy images equal the same
    geometry on the host-decoded pixels (mxd_resize_crop_host)."""
    rng = np.random.default_rng(21)
    datas, geoms, pixels = [], [], []
    for i in range(20):
        h, w = int(rng.integers(40, 700)), int(rng.integers(40, 700))
        d = _encode(_smooth(rng, h, w), quality=90, subsampling=i % 3)
        datas.append(d)
        pixels.append(capi.jpeg_decode(d))
        ww, wh = int(rng.integers(8, w + 1)), int(rng.integers(8, h + 1))
        wx, wy = int(rng.integers(0, w - ww + 1)), int(rng.integers(0, h - wh + 1))
        rw, rh = int(rng.integers(16, 400)), int(rng.integers(16, 400))
        cw, ch = int(rng.integers(1, rw + 1)), int(rng.integers(1, rh + 1))
        cx, cy = int(rng.integers(0, rw - cw + 1)), int(rng.integers(0, rh - ch + 1))
        geoms.append((wx, wy, ww, wh, rw, rh, cx, cy, cw, ch, i % 2))
    elem = 4 if f32 else 1
    want, entries = [], []
    for im, (wx, wy, ww, wh, rw, rh, cx, cy, cw, ch, flip) in zip(pixels, geoms):
        win = np.ascontiguousarray(im[wy:wy + wh, wx:wx + ww])
        o = np.zeros((ch, cw * 3 * elem), np.uint8)
        want.append((o, win))
        entries.append(dict(src=win.ctypes.data, src_stride=ww * 3, src_w=ww, src_h=wh, channels=3, resize_w=rw,
                            resize_h=rh, crop_x=cx, crop_y=cy, crop_w=cw, crop_h=ch, flip=flip, dst=o.ctypes.data,
                            dst_stride=cw * 3 * elem))
    arr, n = capi.make_images(entries)
    capi.resize_crop_host(arr, n, capi.MXD_F32_DIV255 if f32 else capi.MXD_U8, 0)
    _, got = _decode_gpu(datas, geoms, f32, device_dst)
    for g, (w_, _) in zip(got, want):
        assert np.array_equal(g, w_)


def test_large_image_many_jobs(word_source):
    """A 3000x2000 image with restart markers every block: thousands of
    segments, packed into several jobs; and a 2400x1800 one without restart
    markers (one segment of ~1024 subsequences)."""
    rng = np.random.default_rng(5)
    a = _encode(_smooth(rng, 2000, 3000), quality=92, subsampling=2, restart_marker_blocks=1)
    b = _encode(_smooth(rng, 1800, 2400), quality=97, subsampling=0)
    coefs = _check_identity([a, b])
    assert all(c.entropy_pending for c in coefs)


@pytest.mark.parametrize("bits", [0, 32])
def test_deep_tables_take_the_searching_decoder(bits, word_source):
    """Tables whose codes longer than 11 bits reach below the top 1/64 of the
    code space (tests/jpeg_enc.py; no Pillow file has one) need the searching
    decoder (HuffDev::search): a batch mixing such files -- grey, 4:4:4,
    restart intervals, a noise image long enough for several jobs -- with
    Pillow files, equal to the host decoder and to Pillow."""
    import jpeg_enc as J

    assert J.first_long_prefix(J.DEEP_DC[0]) < 2016 and J.first_long_prefix(J.DEEP_AC[0]) < 2016
    rng = np.random.default_rng(31)
    datas = [J.encode(rng.integers(0, 256, (37, 53), dtype=np.uint8)),
             J.encode(_smooth(rng, 120, 97), restart_mcus=3),
             J.encode(_smooth(rng, 200, 330)[:, :, 0], q=1),
             J.encode(rng.integers(0, 256, (384, 512, 3), dtype=np.uint8), q=1),
             _encode(_smooth(rng, 150, 170), quality=85)]
    prev = capi.set_tuning(capi.MXD_TUNE_HUFF_BITS, bits)
    try:
        coefs = _check_identity(datas)
    finally:
        capi.set_tuning(capi.MXD_TUNE_HUFF_BITS, prev)
    assert all(c.entropy_pending for c in coefs)


def test_out_of_range_coefficients_take_the_wide_idct():
    """Dequantised blocks outside the 32-bit IDCT's range (|x| >= 2^14 in
    either pass: no encoder of real pixels writes them, tests/jpeg_enc.py
    writes them directly) take jpeg_idct's JLONG path (idct_block_wide) and
    still equal the host decoder, which follows jidctint.c's JLONG
    arithmetic.  Pillow is not compared: libjpeg-turbo's SIMD IDCT
    dequantises in 16 bits, so on such data it leaves jidctint.c's results."""
    import jpeg_enc as J

    rng = np.random.default_rng(47)
    datas = []
    for h, w, nc, amp, qlo in [(40, 56, 1, 1023, 1), (64, 48, 3, 60, 150), (24, 200, 3, 400, 20)]:
        rows, cols = -(-h // 8), -(-w // 8)
        planes = []
        for _ in range(nc):
            z = rng.integers(-amp, amp + 1, (rows, cols, 64))
            z[:, :, 0] = rng.integers(-900, 901, (rows, cols))
            z[rng.random((rows, cols)) < 0.3] //= 64  # blocks inside the 32-bit range beside them
            planes.append(z)
        q = rng.integers(qlo, 256, 64)
        datas.append(J.encode(np.zeros((h, w, nc) if nc == 3 else (h, w), np.uint8), q=q, coefs=planes))
    datas.append(_encode(_smooth(rng, 90, 70), quality=90))
    _check_identity(datas, pillow=False)


def test_arithmetic_coded_files_finish_on_the_device():
    """Arithmetic-coded files (tests/jpeg_arith_enc.py, SOF9 and SOF10) are
    entropy-decoded on the host (parse_coefs routes them there) and finished
    by the batch launch beside device-entropy files: equal to the host
    decoder and to Pillow."""
    import jpeg_arith_enc as A

    rng = np.random.default_rng(33)
    datas = [A.encode(_smooth(rng, 70, 90), q=3, restart_mcus=4),
             A.encode_progressive(_smooth(rng, 64, 100), q=2),
             _encode(_smooth(rng, 80, 60), quality=90),
             A.encode(_smooth(rng, 33, 47)[:, :, 0], q=5, dac=(1, 6, 9))]
    coefs = _check_identity(datas)
    assert [c.entropy_pending for c in coefs] == [False, False, True, False]


def _segment_bytes(d):
    """Unstuffed bytes of each restart interval of a one-scan file (what
    jpeg.cpp record_segments counts: stuffed 0x00 and fill 0xFF dropped)."""
    i = 2
    while True:
        m, n = d[i + 1], d[i + 2] * 256 + d[i + 3]
        if m == 0xDA:
            p = i + 2 + n
            break
        i += 2 + n
    out, cur = [], 0
    while True:
        if d[p] == 0xFF:
            m = d[p + 1]
            if m == 0x00:
                cur, p = cur + 1, p + 2
            elif 0xD0 <= m <= 0xD7:
                out.append(cur)
                cur, p = 0, p + 2
            elif m == 0xFF:
                p += 1
            else:
                out.append(cur)
                return out
        else:
            cur, p = cur + 1, p + 1


def _job_sizes(subs, cap, move=32, warm=24):
    """hostpath.cpp jpeg_chunk's job split (subsequences per job, warm-up
    included) for segments of `subs` subsequences at a per-job cap."""
    import bisect

    sf = [0]
    for s in subs:
        sf.append(sf[-1] + s)
    n = sf[-1]
    njob = -(-n // cap)
    cuts = [0]
    for q in range(1, njob):
        cut = q * n // njob
        g = bisect.bisect_right(sf, cut) - 1
        if cut - sf[g] <= move and sf[g] > cuts[-1]:
            cut = sf[g]
        cuts.append(cut)
    cuts.append(n)
    return [b - a + min(warm, a - sf[bisect.bisect_right(sf, a) - 1]) for a, b in zip(cuts, cuts[1:])]


def test_cut_moved_to_a_segment_start_stays_within_a_workgroup():
    """a job cut moved back to a restart-segment start (no
    warm-up) lengthens the next job by up to 32 subsequences; with the old
    per-job cap of 1000 that job could hold 1025..1032 subsequences, past the
    1024-thread workgroup -- its tail never decoded and the next job waiting
    for a state that never came.  Search (seeded) for a restart-interval file
    and subsequence length where the old split overflows, then decode it on
    the device with that length: bit-exact to the host decoder and Pillow."""
    rng = np.random.default_rng(7)
    found = None
    for _ in range(60):
        h, w = 64 * int(rng.integers(2, 8)), 64 * int(rng.integers(2, 8))
        a = rng.integers(0, 256, (h, w, 3), dtype=np.uint8)
        d = _encode(a, quality=int(rng.integers(60, 100)), subsampling=2,
                    restart_marker_blocks=int(rng.integers(4, 40)))
        sb = _segment_bytes(d)
        for bits in range(32, 2049, 32):
            subs = [max(1, -(-8 * b // bits)) for b in sb]
            if max(_job_sizes(subs, 1000)) > 1024:
                found = (d, bits, subs)
                break
        if found:
            break
    assert found, "no overflowing split found"
    d, bits, subs = found
    assert max(_job_sizes(subs, 1024 - 32)) <= 1024  # the fixed cap
    prev = capi.set_tuning(capi.MXD_TUNE_HUFF_BITS, bits)
    try:
        coefs = _check_identity([d])
    finally:
        capi.set_tuning(capi.MXD_TUNE_HUFF_BITS, prev)
    assert coefs[0].entropy_pending
