"""Decode speed of the native JPEG decoder vs Pillow (libjpeg-turbo) on
seeded synthetic images, single thread: python tools/jpeg_speed.py [reps]"""
import io
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "mlx-data_amd"), os.path.join(REPO, "tools")]
from PIL import Image  # noqa: E402

from bench_pipeline import smooth  # noqa: E402
from mlx_data_amd import capi  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 100
rng = np.random.default_rng(0)
cases = [((300, 200), dict(quality=90)), ((500, 375), dict(quality=90)),
         ((1280, 960), dict(quality=85)), ((500, 375), dict(quality=90, subsampling=0)),
         ((500, 375), dict(quality=90, progressive=True))]
for (w, h), kw in cases:
    b = io.BytesIO()
    Image.fromarray(smooth(rng, h, w)).save(b, "JPEG", **kw)
    data = b.getvalue()
    buf = np.frombuffer(data, np.uint8)
    want = np.asarray(Image.open(io.BytesIO(data)).convert("RGB"))
    assert np.array_equal(capi.jpeg_decode(buf), want)
    res = []
    for f in (lambda: capi.jpeg_decode(buf), lambda: np.asarray(Image.open(io.BytesIO(data)).convert("RGB"))):
        f()
        t = time.perf_counter()
        for _ in range(reps):
            f()
        res.append((time.perf_counter() - t) / reps * 1e3)
    print(f"{w}x{h} {kw}: ours {res[0]:.3f} ms  pillow {res[1]:.3f} ms  ratio {res[0] / res[1]:.2f}")
