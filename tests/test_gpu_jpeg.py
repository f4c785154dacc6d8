"""GPU: the device-side finish of the split JPEG decode (csrc/jpegdev.hip,
mxd_jpeg_resize_crop_host / _to_device).

* identity geometry: the GPU-decoded image equals the host decode byte for
  byte (and so Pillow's libjpeg-turbo: tests/test_jpeg.py pins the host
  decoder) -- committed fixtures and Pillow-encoded images of every sampling
  layout, progressive, restart intervals, odd sizes;
* resize + crop + mirror, u8 and f32, windows (random_area_crop): equal to
  mxd_resize_crop_host on the host-decoded pixels (same kernels, same bytes);
* batches spanning several staging chunks, device destinations;
* the operator surface: load_image -> resize -> crop -> batch gives the same
  batches with the device finish on and off."""
import io
import os

import numpy as np
import pytest

from mlx_data_amd import capi

pytestmark = pytest.mark.gpu

GOLD = np.load(os.path.join(os.path.dirname(__file__), "golden", "jpeg.npz"))
CASES = sorted(k[:-4] for k in GOLD.files if k.endswith("_jpg") and not k.startswith("cmyk"))


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


def _host_ref(pixels, geoms, f32):
    """mxd_resize_crop_host on host-decoded pixels: the expected bytes."""
    elem = 4 if f32 else 1
    outs, entries = [], []
    for im, (wx, wy, ww, wh, rw, rh, cx, cy, cw, ch, flip) in zip(pixels, geoms):
        win = np.ascontiguousarray(im[wy:wy + wh, wx:wx + ww])
        o = np.zeros((ch, cw * 3 * elem), np.uint8)
        outs.append((o, win))
        entries.append(dict(src=win.ctypes.data, src_stride=ww * 3, src_w=ww, src_h=wh, channels=3, resize_w=rw,
                            resize_h=rh, crop_x=cx, crop_y=cy, crop_w=cw, crop_h=ch, flip=flip, dst=o.ctypes.data,
                            dst_stride=cw * 3 * elem))
    arr, n = capi.make_images(entries)
    capi.resize_crop_host(arr, n, capi.MXD_F32_DIV255 if f32 else capi.MXD_U8, 0)
    return [o for o, _ in outs]


def _gpu(coefs, geoms, f32, device_dst=False):
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
    return outs


def _identity(c):
    return (0, 0, c.width, c.height, c.width, c.height, 0, 0, c.width, c.height, 0)


def test_fixtures_identity_decode():
    coefs = [capi.JpegCoefs(GOLD[f"{k}_jpg"]) for k in CASES]
    got = _gpu(coefs, [_identity(c) for c in coefs], False)
    for k, g, c in zip(CASES, got, coefs):
        assert np.array_equal(g.reshape(c.height, c.width, 3), GOLD[f"{k}_rgb"]), k


@pytest.mark.parametrize("seed", range(4))
def test_encoded_layouts_identity_decode(seed):
    rng = np.random.default_rng(seed)
    datas = []
    for i in range(12):
        h, w = int(rng.integers(1, 300)), int(rng.integers(1, 300))
        grey = i % 6 == 5
        kw = dict(quality=int(rng.integers(10, 101)), progressive=bool(rng.random() < 0.4))
        if not grey:
            kw["subsampling"] = i % 3
        if rng.random() < 0.3:
            kw["restart_marker_blocks"] = int(rng.integers(1, 5))
        datas.append(_encode(_smooth(rng, h, w, 1 if grey else 3), **kw))
    coefs = [capi.JpegCoefs(d) for d in datas]
    got = _gpu(coefs, [_identity(c) for c in coefs], False)
    for d, g, c in zip(datas, got, coefs):
        assert np.array_equal(g.reshape(c.height, c.width, 3), capi.jpeg_decode(d))


@pytest.mark.parametrize("f32", [False, True])
@pytest.mark.parametrize("device_dst", [False, True])
def test_resize_crop_windows_equal_host_pixels(f32, device_dst):
    rng = np.random.default_rng(7)
    datas, geoms = [], []
    for i in range(24):
        h, w = int(rng.integers(40, 700)), int(rng.integers(40, 700))
        datas.append(_encode(_smooth(rng, h, w), quality=90, subsampling=i % 3, progressive=i % 5 == 0))
        ww, wh = int(rng.integers(8, w + 1)), int(rng.integers(8, h + 1))
        wx, wy = int(rng.integers(0, w - ww + 1)), int(rng.integers(0, h - wh + 1))
        rw, rh = int(rng.integers(16, 400)), int(rng.integers(16, 400))
        cw, ch = int(rng.integers(1, rw + 1)), int(rng.integers(1, rh + 1))
        cx, cy = int(rng.integers(0, rw - cw + 1)), int(rng.integers(0, rh - ch + 1))
        geoms.append((wx, wy, ww, wh, rw, rh, cx, cy, cw, ch, i % 2))
    coefs = [capi.JpegCoefs(d) for d in datas]
    want = _host_ref([capi.jpeg_decode(d) for d in datas], geoms, f32)
    got = _gpu(coefs, geoms, f32, device_dst)
    for g, w_ in zip(got, want):
        assert np.array_equal(g, w_)


def _smallest_side(w, h, size):
    return capi.resize_smallest_side_dims(w, h, size)


@pytest.mark.parametrize("f32,device_dst", [(False, False), (True, False), (True, True)])
def test_plane_sources_equal_rgb_frames(f32, device_dst):
    """4:2:0 images whose resize runs on a scatter wave
    kernel are resized straight from their sample planes (wave.hip YccSrc:
    fancy upsampling + YCbCr -> RGB in registers, no RGB frame).  Every
    output equals mxd_resize_crop_host on the host-decoded pixels and the
    same call through the RGB frame (MXD_TUNE_JPEG_RGB = 1) byte for byte:
    odd and tiny sizes, restart intervals, windows (x a multiple of 4, any
    y), mirrored crops, downscales of every scatter shape and upscales."""
    rng = np.random.default_rng(11)
    datas, geoms = [], []
    for i in range(28):
        h, w = int(rng.integers(17, 900)), int(rng.integers(17, 900))
        kw = dict(quality=int(rng.integers(30, 98)), subsampling=2)
        if i % 5 == 4:
            kw["restart_marker_blocks"] = 3
        datas.append(_encode(_smooth(rng, h, w), **kw))
        if i % 3 == 0:  # a window: x a multiple of 4, any y
            ww, wh = int(rng.integers(16, w + 1)), int(rng.integers(16, h + 1))
            wx = int(rng.integers(0, (w - ww) // 4 + 1)) * 4
            wy = int(rng.integers(0, h - wh + 1))
        else:
            wx, wy, ww, wh = 0, 0, w, h
        size = int(rng.choice([64, 128, 224, 256, 384]))
        rw, rh = _smallest_side(ww, wh, size)
        cw, ch = min(rw, int(rng.integers(1, 257))), min(rh, int(rng.integers(1, 257)))
        cx, cy = capi.center_crop_origin(rw, rh, cw, ch)
        geoms.append((wx, wy, ww, wh, rw, rh, cx, cy, cw, ch, i % 2))
    coefs = [capi.JpegCoefs(d) for d in datas]
    want = _host_ref([capi.jpeg_decode(d) for d in datas], geoms, f32)
    capi.jpeg_plane_sources(reset=True)
    got = _gpu(coefs, geoms, f32, device_dst)
    fused = capi.jpeg_plane_sources(reset=True)
    prev = capi.set_tuning(capi.MXD_TUNE_JPEG_RGB, 1)
    try:
        rgb = _gpu(coefs, geoms, f32, device_dst)
    finally:
        capi.set_tuning(capi.MXD_TUNE_JPEG_RGB, prev)
    assert capi.jpeg_plane_sources(reset=True) == 0
    assert fused >= 14, fused  # most of them take the plane source
    for i, (g, r, w_) in enumerate(zip(got, rgb, want)):
        assert np.array_equal(g, w_), (i, geoms[i])
        assert np.array_equal(g, r), i


def test_chunked_batch_of_large_images():
    """~150 MB of coefficients: several staging chunks over both slots."""
    rng = np.random.default_rng(3)
    base = [_encode(_smooth(rng, 960, 1280), quality=85, subsampling=s) for s in (0, 2)]
    datas = [base[i % 2] for i in range(40)]
    coefs = [capi.JpegCoefs(d) for d in datas]
    geoms = []
    for i, c in enumerate(coefs):
        rw, rh = capi.resize_smallest_side_dims(c.width, c.height, 256)
        cx, cy = capi.center_crop_origin(rw, rh, 224, 224)
        geoms.append((0, 0, c.width, c.height, rw, rh, cx, cy, 224, 224, i % 3 == 0))
    want = _host_ref([capi.jpeg_decode(d) for d in datas], geoms, True)
    got = _gpu(coefs, geoms, True)
    for g, w_ in zip(got, want):
        assert np.array_equal(g, w_)


def _cmyk_files(seed):
    """Four-component files: Pillow CMYK (Adobe transform 0, 1x1 sampling;
    baseline, restart intervals, progressive), and tests/jpeg_enc.py files
    with an Adobe marker of transform 2 (YCCK) and 0 (CMYK), with restarts."""
    import jpeg_enc as J
    from PIL import Image

    rng = np.random.default_rng(seed)
    out = [bytes(GOLD["cmyk_jpg"])]
    for i in range(6):
        h, w = int(rng.integers(1, 300)), int(rng.integers(1, 300))
        kw = dict(quality=int(rng.integers(20, 101)), progressive=i % 3 == 2)
        if i % 3 == 1:
            kw["restart_marker_blocks"] = int(rng.integers(1, 6))
        b = io.BytesIO()
        Image.fromarray(_smooth(rng, h, w, 4), "CMYK").save(b, "JPEG", **kw)
        out.append(b.getvalue())
    for i in range(4):
        h, w = int(rng.integers(8, 200)), int(rng.integers(8, 200))
        out.append(J.encode(_smooth(rng, h, w, 4), q=int(rng.integers(1, 6)), adobe=2 if i % 2 == 0 else 0,
                            restart_mcus=3 if i >= 2 else 0))
    return out


def test_cmyk_and_ycck_finish_on_the_device():
    """four-component JPEGs (CMYK and YCCK) finish on the
    device -- their first three components through the IDCT and the colour
    step (YCCK: YCbCr -> RGB inverted, jdcolor.c ycck_cmyk_convert), the
    reference's first three channels of libjpeg's CMYK output
    (ImageJPEG.cpp:112-124) -- with the sequential ones' Huffman data decoded
    on the device too (K decoded and dropped).  Identity geometry: equal to
    the host decoder and to libjpeg's raw output through Pillow (255 - Pillow's
    un-inverted Adobe CMYK), then resized + cropped like the host bytes."""
    from PIL import Image

    datas = _cmyk_files(41)
    coefs = [capi.JpegCoefs(d, device_entropy=True) for d in datas]
    assert all(c.device_ok for c in coefs)
    assert sum(c.entropy_pending for c in coefs) >= 6  # the sequential ones
    got = _gpu(coefs, [_identity(c) for c in coefs], False)
    for i, (d, g, c) in enumerate(zip(datas, got, coefs)):
        img = g.reshape(c.height, c.width, 3)
        assert np.array_equal(img, capi.jpeg_decode(d)), i
        pil = Image.open(io.BytesIO(d))
        assert pil.mode == "CMYK"
        assert np.array_equal(img, 255 - np.asarray(pil)[:, :, :3]), i
    geoms = []
    for c in coefs:
        rw, rh = capi.resize_smallest_side_dims(c.width, c.height, 48)
        cw, ch = min(40, rw), min(40, rh)
        geoms.append((0, 0, c.width, c.height, rw, rh, (rw - cw) // 2, (rh - ch) // 2, cw, ch, 1))
    for f32 in (False, True):
        want = _host_ref([capi.jpeg_decode(d) for d in datas], geoms, f32)
        for g, w_ in zip(_gpu(coefs, geoms, f32), want):
            assert np.array_equal(g, w_)


def test_lossless_files_are_refused_on_the_device():
    import jpeg_enc as J

    c = capi.JpegCoefs(J.encode_lossless(_smooth(np.random.default_rng(3), 20, 30), psv=1))
    assert not c.device_ok
    with pytest.raises(capi.MxdError, match="host"):
        _gpu([c], [_identity(c)], False)


@pytest.mark.parametrize("variant", ["u8", "f32", "device"])
def test_pipeline_device_decode_on_off(variant, tmp_path):
    from mlx_data_amd import data as dx

    rng = np.random.default_rng(11)
    samples = []
    for i in range(37):
        h, w = int(rng.integers(120, 520)), int(rng.integers(120, 520))
        p = tmp_path / f"{i}.jpg"
        if i % 9 == 4:  # grey
            p.write_bytes(_encode(_smooth(rng, h, w, 1), quality=88))
        elif i % 9 == 7:  # arithmetic-coded (tests/jpeg_arith_enc.py): host entropy decode
            import jpeg_arith_enc as A

            img = _smooth(rng, h // 4 + 8, w // 4 + 8)
            p.write_bytes(A.encode_progressive(img, q=3) if i % 2 else A.encode(img, q=3, restart_mcus=5))
        elif i % 9 == 8:  # lossless (SOF3): the host finishes it
            import jpeg_enc as J

            p.write_bytes(J.encode_lossless(_smooth(rng, h // 4 + 8, w // 4 + 8), psv=1 + i % 7))
        else:
            p.write_bytes(_encode(_smooth(rng, h, w), quality=88, subsampling=i % 3, progressive=i % 4 == 1))
        samples.append(dict(image=str(p).encode(), label=i))
    samples.append(dict(image=os.path.join(str(tmp_path), "cmyk.jpg").encode(), label=99))
    (tmp_path / "cmyk.jpg").write_bytes(GOLD["cmyk_jpg"].tobytes())

    def run(on):
        before = dx.device_decode()
        dx.set_device_decode(on)
        try:
            dx.set_state(5)
            d = (dx.buffer_from_vector(samples).load_image("image").image_random_area_crop("image", (0.3, 1.0),
                                                                                         (0.75, 1.33))
                 .image_resize("image", 96, 80).image_random_h_flip("image", 0.5))
            d = d.image_to_float("image") if variant != "u8" else d
            d = d.batch(8, device=0) if variant == "device" else d.batch(8)
            batches = [d[i] for i in range(len(d))]
            return [np.asarray(b["image"].numpy() if variant == "device" else b["image"]) for b in batches]
        finally:
            dx.set_device_decode(before)

    on, off = run(True), run(False)
    assert len(on) == len(off) == 5
    for a, b in zip(on, off):
        assert a.dtype == b.dtype and np.array_equal(a, b)
