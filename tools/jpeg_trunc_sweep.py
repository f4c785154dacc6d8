"""Truncated progressive JPEGs decoded by the native decoder against Pillow's
libjpeg-turbo (block smoothing): seeded Pillow encodes (sizes
1..199, qualities 10..95, 4:4:4 / 4:2:2 / 4:2:0 / grey) cut at every scan
boundary (`sos`) or at a random point inside every scan's entropy-coded data
(`mid`).  Prints the mismatching files and a count.

    python tools/jpeg_trunc_sweep.py {sos|mid} SEED
"""
import io
import os
import sys

import numpy as np
from PIL import Image, ImageFile

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "mlx-data_amd"))
from mlx_data_amd import capi  # noqa: E402

ImageFile.LOAD_TRUNCATED_IMAGES = True


def smooth(rng, h, w, c=3):
    gh, gw = h // 16 + 2, w // 16 + 2
    grid = rng.integers(0, 256, (gh, gw, c)).astype(np.float32)
    yi = np.minimum(np.arange(h) * (gh - 1) // max(1, h - 1), gh - 2)
    xi = np.minimum(np.arange(w) * (gw - 1) // max(1, w - 1), gw - 2)
    f = grid[yi][:, xi] * 0.6 + grid[yi + 1][:, xi + 1] * 0.4 + rng.normal(0, 14, (h, w, c))
    return np.clip(f, 0, 255).astype(np.uint8)


def main():
    mode = sys.argv[1] if len(sys.argv) > 1 else "sos"
    rng = np.random.default_rng(int(sys.argv[2]) if len(sys.argv) > 2 else 0)
    bad = tot = 0
    for it in range(40):
        h, w = int(rng.integers(1, 200)), int(rng.integers(1, 200))
        grey = it % 5 == 4
        a = smooth(rng, h, w, 1 if grey else 3)
        kw = dict(quality=int(rng.integers(10, 96)), progressive=True)
        if not grey:
            kw["subsampling"] = it % 3
        b = io.BytesIO()
        Image.fromarray(a if not grey else a[:, :, 0]).save(b, "JPEG", **kw)
        d = b.getvalue()
        pos = [i for i in range(len(d) - 1) if d[i] == 0xFF and d[i + 1] == 0xDA]
        for k in range(1, len(pos)):
            if mode == "sos":
                t = d[:pos[k]]
            else:
                s = pos[k - 1] + 2 + int.from_bytes(d[pos[k - 1] + 2:pos[k - 1] + 4], "big")
                e = s
                while not (d[e] == 0xFF and d[e + 1] != 0 and not 0xD0 <= d[e + 1] <= 0xD7):
                    e += 1
                if e - s < 4:
                    continue
                cut = int(rng.integers(s + 1, e - 1))
                while d[cut - 1] == 0xFF:
                    cut += 1
                t = d[:cut]
            ref = np.asarray(Image.open(io.BytesIO(t)).convert("RGB"))
            mine = capi.jpeg_decode(t)
            tot += 1
            if not np.array_equal(ref, mine):
                bad += 1
                df = np.abs(ref.astype(int) - mine.astype(int))
                print("diff", it, (w, h), kw, "scan", k, "max", int(df.max()), "frac", round(float((df > 0).mean()), 4))
    print(mode, "mismatching", bad, "of", tot)


if __name__ == "__main__":
    main()
