"""Generates tests/golden/pixmap.npz (committed) -- run in the dev container.

Fixtures for SURVEY.md §8f row f4 (data only: inputs and expected outputs):
  in_<k>        seeded HWC uint8 inputs
  rot_<k>_<a>   core::image::rotate(in_k, angle a, crop=False)   (oracle restatement)
  rotc_<k>_<a>  core::image::rotate(in_k, angle a, crop=True)
  gray_<k>_<p>  core::image::channel_reduction(in_k, preset p)   (3-channel inputs)

The reference's core/image/ImageTransform.cpp needs stb_image_resize2.h and is
not buildable here, so these outputs come from oracle/stbir_oracle.c, which
tests/test_pixmap.py cross-checks against an independent numpy restatement.

Requires oracle/liboracle.so (`make -C oracle`).
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(REPO, "oracle"))
import oracle as O  # noqa: E402

SHAPES = {"a": (37, 53, 3), "b": (64, 48, 1), "c": (21, 30, 4), "d": (40, 40, 3)}
ANGLES = (0.0, 17.5, 90.0, -45.0, 180.0, 333.0)
PRESETS = ("default", "rec709", "rec2020", "green")


def main():
    rng = np.random.default_rng(77)
    out = {}
    for k, shp in SHAPES.items():
        img = rng.integers(0, 256, shp, dtype=np.uint8)
        out[f"in_{k}"] = img
        for a in ANGLES:
            out[f"rot_{k}_{a:g}"] = O.rotate(img, a, False)
            out[f"rotc_{k}_{a:g}"] = O.rotate(img, a, True)
        if shp[2] == 3:
            for p in PRESETS:
                out[f"gray_{k}_{p}"] = O.channel_reduction(img, p)
    np.savez_compressed(os.path.join(HERE, "pixmap.npz"), **out)
    print("wrote", len(out), "arrays")


if __name__ == "__main__":
    main()
