"""Writes tests/golden/rng_area.npz: the (x, y, w, h) draws of
image_random_area_crop after set_state(seed), made by the reference's own
State (core/State.cpp, compiled from /root/reference by oracle/Makefile) driving
the restated generate_random_crop_ (op/ImageTransform.cpp:214-280) in
oracle/ref_harness.cpp.  Run here (the reference tree is present):
    python tests/golden/make_rng_golden.py
Arrays per case k: area_k_in = [seed, trials] + ranges (f32), area_k_wh
(sizes), area_k_out (n, 4) int64; zeros = no crop found (image unchanged)."""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "..", "oracle"))
import oracle as O  # noqa: E402

CASES = [
    # seed, area range, aspect range, trials, sizes
    (1234, (0.08, 1.0), (3 / 4, 4 / 3), 10, "mixed"),
    (7, (0.5, 1.0), (1.0, 1.0), 10, "mixed"),
    (11, (0.5, 0.75), (1.0, 1.5), 10, "mixed"),
    (3, (0.5, 0.55), (0.5, 0.6), 3, "mixed"),  # mostly rejected trials
    (5, (0.2, 0.4), (2.0, 3.0), 1, "mixed"),  # one trial: unconstrained fall-through
]


def sizes(seed):
    rng = np.random.default_rng(seed)
    fixed = [(500, 375), (375, 500), (1280, 960), (300, 200), (3840, 2160), (64, 64), (1, 1), (2, 7)]
    rand = [(int(w), int(h)) for w, h in rng.integers(1, 1200, (40, 2))]
    return fixed + rand


def main():
    out = {}
    for k, (seed, a, r, trials, _) in enumerate(CASES):
        wh = sizes(100 + k)
        out[f"area_{k}_in"] = np.array([seed, trials, a[0], a[1], r[0], r[1]], np.float64)
        out[f"area_{k}_wh"] = np.array(wh, np.int64)
        out[f"area_{k}_out"] = O.ref_random_area_crop(seed, wh, a, r, trials)
    path = os.path.join(HERE, "rng_area.npz")
    np.savez_compressed(path, **out)
    print(f"wrote {path}")
    for k in range(len(CASES)):
        o = out[f"area_{k}_out"]
        print(k, "no-crop:", int((o[:, 2] == 0).sum()), "of", len(o))


if __name__ == "__main__":
    main()
