"""GPU: the wave-kernel kinds of mlx-data_amd/csrc/wave.hip -- band workgroups,
scatter, register ring, gather -- give bit-identical outputs on the same inputs
(each sums an output row's taps in the same order from 0), and the default
choice (scatter) matches the oracle (+-1 per channel, < 0.2 % of channels
differing).  The kind is chosen through MXD_BAND (opt-in) / MXD_NO_SCATTER /
MXD_NO_RING, which the C ABI reads on every call."""
import numpy as np
import pytest

import oracle as O
from gpu_util import center_geom, compare, oracle_out, run_device, synth

pytestmark = pytest.mark.gpu

SWITCHES = ("MXD_BAND", "MXD_NO_BAND", "MXD_NO_SCATTER", "MXD_NO_RING")
KINDS = [
    ("band", {"MXD_BAND": "1"}),
    ("default", {}),
    ("ring", {"MXD_NO_SCATTER": "1"}),
    ("gather", {"MXD_NO_SCATTER": "1", "MXD_NO_RING": "1"}),
]


def c2():
    imgs = [synth(960, 1280, 3, s) for s in range(3)]
    return imgs, [center_geom(i) for i in imgs]


def mixed():
    sizes = [(480, 640), (720, 1280), (1080, 1920), (1440, 2560), (2160, 3840), (375, 500), (500, 333), (200, 300)]
    imgs = [synth(h, w, 3, 20 + i) for i, (h, w) in enumerate(sizes)]
    return imgs, [center_geom(i) for i in imgs]


def c5():
    img = synth(2160, 3840, 3, 7)
    tw, th = O.smallest_side_dims(3840, 2160, 512)
    return [img, img], [(tw, th, 100, 30, 448, 448, 1), (tw, th, tw - 448, 0, 448, 448, 0)]


CASES = {"c2": c2, "mixed": mixed, "c5": c5}


def run_kinds(monkeypatch, imgs, geoms, f32):
    outs = {}
    for name, env in KINDS:
        for k in SWITCHES:
            if k in env:
                monkeypatch.setenv(k, env[k])
            else:
                monkeypatch.delenv(k, raising=False)
        outs[name] = run_device(imgs, geoms, f32=f32)
    for k in SWITCHES:
        monkeypatch.delenv(k, raising=False)
    return outs


@pytest.mark.parametrize("f32", [False, True])
@pytest.mark.parametrize("case", sorted(CASES))
def test_kernel_kinds_bit_identical(monkeypatch, case, f32):
    imgs, geoms = CASES[case]()
    outs = run_kinds(monkeypatch, imgs, geoms, f32)
    for name, got in outs.items():
        for i, (a, b) in enumerate(zip(outs["gather"], got)):
            assert np.array_equal(a.view(np.uint8), b.view(np.uint8)), (case, name, i)
    if not f32:
        for img, g, o in zip(imgs, geoms, outs["default"]):
            m, frac = compare(o, oracle_out(img, g))
            assert m <= 1 and frac < 2e-3, (case, g, m, frac)
