"""Generates tests/golden/golden.npz (committed) -- run in the dev container.

Fixtures (data only: inputs and expected outputs):
  img_<name>            seeded synthetic HWC uint8 inputs (smooth field + noise)
  rc_<name>             oracle resize_smallest_side(256) -> center_crop(224, 224)
  refcrop_sha_<name>    SHA-256 (32 bytes) of the SAME crop window cut from the
                        oracle's resized image by the reference's own array::sub
                        (oracle/_ref, Array.cpp:544-583); asserted equal to rc_<name>
  refbatch              array::batch (Array.cpp:465-498) of three ragged crops, pad 0
  refbatch_shapes       their shapes
  rng_xy, rng_flip      (x, y, flip) draws of image_random_crop(448, 448) then
                        image_random_h_flip(0.5) after set_state(1234), 64 samples of
                        a 910x512 resized frame, from the reference's State.cpp
  lut                   numpy x.astype("float32") / 255 for x = 0..255
                        (benchmarks/comparative/caltech101/mlx_data.py:46)

Requires oracle/liboracle.so and oracle/_ref/libmlxref.so (`make -C oracle`).
"""
import hashlib
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(REPO, "oracle"))
import oracle as O  # noqa: E402

SIZES = {
    "caltech_200x300": (200, 300, 3),
    "imagenet_375x500": (375, 500, 3),
    "portrait_500x375": (500, 375, 3),
    "odd_333x500": (333, 500, 3),
    "square_256": (256, 256, 3),
    "square_300": (300, 300, 3),
    "small_97x131": (97, 131, 3),
    "tiny_48x64": (48, 64, 3),
    "gray_240x320": (240, 320, 3),
    "c1_120x160": (120, 160, 1),
}


def synth(h, w, c, seed):
    """Smooth random field (bilinear-upsampled coarse grid) plus noise, uint8."""
    rng = np.random.default_rng(seed)
    gh, gw = max(2, h // 16 + 2), max(2, w // 16 + 2)
    grid = rng.integers(0, 256, (gh, gw, c)).astype(np.float64)
    ys = np.linspace(0, gh - 1.001, h)
    xs = np.linspace(0, gw - 1.001, w)
    y0, x0 = np.floor(ys).astype(int), np.floor(xs).astype(int)
    fy, fx = (ys - y0)[:, None, None], (xs - x0)[None, :, None]
    a = grid[y0][:, x0]
    b = grid[y0][:, x0 + 1]
    cc = grid[y0 + 1][:, x0]
    d = grid[y0 + 1][:, x0 + 1]
    f = a * (1 - fy) * (1 - fx) + b * (1 - fy) * fx + cc * fy * (1 - fx) + d * fy * fx
    f += rng.normal(0, 10, f.shape)
    return np.clip(np.rint(f), 0, 255).astype(np.uint8)


def main():
    out = {}
    for i, (name, (h, w, c)) in enumerate(SIZES.items()):
        img = synth(h, w, c, 1000 + i)
        if name.startswith("gray"):
            img[:, :, 1] = img[:, :, 0]
            img[:, :, 2] = img[:, :, 0]
        out[f"img_{name}"] = img
        tw, th = O.smallest_side_dims(w, h, 256)
        resized = O.resize(img, tw, th)
        x, y = O.center_crop_origin(tw, th, 224, 224)
        out[f"rc_{name}"] = O.crop(resized, x, y, 224, 224)
        ref = O.ref_crop(resized, x, y, 224, 224)
        assert np.array_equal(ref, out[f"rc_{name}"]), name
        out[f"refcrop_sha_{name}"] = np.frombuffer(hashlib.sha256(ref.tobytes()).digest(), np.uint8)
    crops = [out["rc_caltech_200x300"], out["rc_small_97x131"][:200, :210], out["rc_tiny_48x64"][:150, :224]]
    out["refbatch"] = O.ref_batch(crops, 0.0)
    out["refbatch_shapes"] = np.array([a.shape for a in crops], np.int64)
    xy, fl = O.ref_random_crop_flip(1234, [(910, 512)] * 64, 448, 448, 0.5)
    out["rng_xy"] = xy
    out["rng_flip"] = fl
    out["lut"] = np.arange(256, dtype=np.uint8).astype("float32") / 255
    path = os.path.join(HERE, "golden.npz")
    np.savez_compressed(path, **out)
    manifest = {k: hashlib.sha256(np.ascontiguousarray(v).tobytes()).hexdigest() for k, v in sorted(out.items())}
    with open(os.path.join(HERE, "manifest.json"), "w") as f:
        json.dump(manifest, f, indent=1, sort_keys=True)
    print(f"wrote {path} ({os.path.getsize(path)} bytes, {len(out)} arrays)")


if __name__ == "__main__":
    main()
