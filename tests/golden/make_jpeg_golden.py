"""Generates tests/golden/jpeg.npz: small JPEG files (encoded by Pillow's
libjpeg-turbo) and the pixels libjpeg-turbo decodes from them with the
reference's settings (core/image/ImageJPEG.cpp:99-146: libjpeg defaults, RGB
out, grey replicated to 3 channels, CMYK -> the first three raw channels).

Cases: 4:4:4 / 4:2:2 / 4:2:0 chroma, greyscale, progressive (spectral
selection + successive approximation), optimised Huffman tables, restart
markers (every block, every MCU row), an RGB JPEG (Adobe transform 0), an
Adobe CMYK JPEG, odd / tiny sizes, a baseline file truncated inside a
restart interval (libjpeg's insufficient-data rule), and progressive files
truncated after 1-3 whole scans or inside a DC / AC scan (`prog_trunc_*`:
libjpeg's block smoothing, jdcoefct.c decompress_smooth_data, which
jpeg_start_decompress applies by default; Pillow's decoder appends the EOI
that libjpeg's memory source fakes for the reference).

    python tests/golden/make_jpeg_golden.py
"""
import io
import os

import numpy as np
from PIL import Image, ImageFile, features

HERE = os.path.dirname(os.path.abspath(__file__))


def smooth(rng, h, w, c):
    x = np.linspace(0, 6, w)[None, :, None]
    y = np.linspace(0, 4, h)[:, None, None]
    base = (np.sin(x * 1.3 + y * 0.7) + np.cos(y * 2.1 - x * 0.4)) * 60 + 128
    return np.clip(base + rng.normal(0, 25, (h, w, c)) + np.arange(c)[None, None, :] * 20, 0, 255).astype(np.uint8)


def encode(a, mode=None, **kw):
    b = io.BytesIO()
    Image.fromarray(a, mode).save(b, "JPEG", **kw) if mode else Image.fromarray(a).save(b, "JPEG", **kw)
    return b.getvalue()


def reference_pixels(data):
    im = Image.open(io.BytesIO(data))
    if im.mode == "CMYK":
        # Pillow un-inverts Adobe CMYK; libjpeg's raw output is the stored (inverted) values
        return 255 - np.asarray(im)[:, :, :3]
    return np.asarray(im.convert("RGB"))


def main():
    rng = np.random.default_rng(2024)
    cases = {}
    rgb = smooth(rng, 61, 83, 3)
    for sub in (0, 1, 2):
        for prog in (False, True):
            cases[f"sub{sub}_prog{int(prog)}"] = encode(rgb, quality=85, subsampling=sub, progressive=prog)
    cases["sub2_q30_opt"] = encode(rgb, quality=30, subsampling=2, optimize=True)
    cases["sub2_q100"] = encode(rgb, quality=100, subsampling=2)
    cases["grey"] = encode(rgb[:, :, 0], quality=90)
    cases["grey_prog"] = encode(rgb[:, :, 0], quality=90, progressive=True)
    cases["rst_blocks1"] = encode(rgb, quality=80, subsampling=2, restart_marker_blocks=1)
    cases["rst_rows1_prog"] = encode(rgb, quality=80, subsampling=1, restart_marker_rows=1, progressive=True)
    cases["rgb_adobe0"] = encode(rgb, quality=90, keep_rgb=True, subsampling=0)
    cases["cmyk"] = encode(smooth(rng, 29, 37, 4), "CMYK", quality=90)
    cases["tiny_1x1"] = encode(rgb[:1, :1], quality=90, subsampling=2)
    cases["tiny_3x2"] = encode(rgb[:2, :3], quality=90, subsampling=2)
    cases["tall_40x3"] = encode(smooth(rng, 40, 3, 3), quality=90, subsampling=2)
    big = smooth(rng, 200, 300, 3)
    cases["caltech_300x200"] = encode(big, quality=90, subsampling=2)
    full = encode(big, quality=90, subsampling=2, restart_marker_blocks=2)
    ImageFile.LOAD_TRUNCATED_IMAGES = True
    cases["truncated_rst"] = full[: len(full) * 6 // 10]
    # progressive files cut at scan boundaries and inside scans (block smoothing)
    trng = np.random.default_rng(77)
    for name, (h, w, c, kw, cut) in {
        "prog_trunc_s1": (61, 83, 3, dict(subsampling=2), ("scan", 1)),
        "prog_trunc_s2": (61, 83, 3, dict(subsampling=2), ("scan", 2)),
        "prog_trunc_s3": (61, 83, 3, dict(subsampling=1), ("scan", 3)),
        "prog_trunc_dc_mid": (90, 70, 3, dict(subsampling=0), ("mid", 1)),
        "prog_trunc_ac_mid": (97, 120, 3, dict(subsampling=2), ("mid", 2)),
        "prog_trunc_ac_mid2": (75, 64, 3, dict(subsampling=1), ("mid", 4)),
        "prog_trunc_grey_mid": (70, 50, 1, {}, ("mid", 2)),
        "prog_trunc_w10": (40, 10, 3, dict(subsampling=1), ("scan", 2)),
    }.items():
        a = smooth(trng, h, w, c)
        data = encode(a if c == 3 else a[:, :, 0], quality=75, progressive=True, **kw)
        sos = [i for i in range(len(data) - 1) if data[i] == 0xFF and data[i + 1] == 0xDA]
        if cut[0] == "scan":
            cases[name] = data[: sos[cut[1]]]  # the first cut[1] scans, whole
        else:
            # inside scan cut[1] (1-based): halfway through its entropy-coded data
            p = sos[cut[1] - 1]
            s = p + 2 + int.from_bytes(data[p + 2:p + 4], "big")
            e = s
            while not (data[e] == 0xFF and data[e + 1] != 0 and not 0xD0 <= data[e + 1] <= 0xD7):
                e += 1
            m = (s + e) // 2
            while data[m - 1] == 0xFF:
                m += 1
            cases[name] = data[:m]
    out = {"libjpeg_version": np.array(features.version("libjpeg_turbo") or "", dtype="U16")}
    for k, data in cases.items():
        out[f"{k}_jpg"] = np.frombuffer(data, np.uint8)
        out[f"{k}_rgb"] = reference_pixels(data)
    np.savez_compressed(os.path.join(HERE, "jpeg.npz"), **out)
    print({k: len(v) for k, v in cases.items()})


if __name__ == "__main__":
    main()
