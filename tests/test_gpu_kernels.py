"""GPU: the kernels of the fused stage -- the wave kernels of
mlx-data_amd/csrc/wave.hip (scatter schedule with byte lanes or pixel lanes,
gather) and the general tile
kernel of resample.hip -- give bit-identical outputs on the same inputs (each
sums an output row's taps in the same order from 0), in both source-load
cache policies of the scatter kernels, and the default choice
matches the oracle (+-1 per channel, < 0.2 % of channels differing).  The
kernel is chosen through mxd_set_kernel_policy (include/mxd_amd.h)."""
import numpy as np
import pytest

import oracle as O
from gpu_util import center_geom, compare, oracle_out, run_device, synth

pytestmark = pytest.mark.gpu

from mlx_data_amd import capi

# (name, kernel policy, source-load policy: MXD_TUNE_LOAD_POLICY 0 auto /
# 1 default / 2 streaming (nt) -- round 6's second form of every scatter
# kernel, which the planner takes for calls with >= 128 MiB of sources)
KINDS = [
    ("default", capi.MXD_POLICY_AUTO, 1),
    ("pixel_lanes", capi.MXD_POLICY_NO_BYTES, 1),
    ("byte_lanes", capi.MXD_POLICY_BYTES, 1),
    ("gather", capi.MXD_POLICY_NO_SCATTER, 1),
    ("general", capi.MXD_POLICY_NO_WAVE, 1),
    ("nt_default", capi.MXD_POLICY_AUTO, 2),
    ("nt_pixel_lanes", capi.MXD_POLICY_NO_BYTES, 2),
    ("nt_byte_lanes", capi.MXD_POLICY_BYTES, 2),
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


def run_kinds(imgs, geoms, f32):
    outs = {}
    try:
        for name, policy, load in KINDS:
            capi.set_kernel_policy(policy)
            capi.set_tuning(capi.MXD_TUNE_LOAD_POLICY, load)
            outs[name] = run_device(imgs, geoms, f32=f32)
    finally:
        capi.set_kernel_policy(capi.MXD_POLICY_AUTO)
        capi.set_tuning(capi.MXD_TUNE_LOAD_POLICY, 0)
    return outs


@pytest.mark.parametrize("f32", [False, True])
@pytest.mark.parametrize("case", sorted(CASES))
def test_kernel_kinds_bit_identical(case, f32):
    imgs, geoms = CASES[case]()
    outs = run_kinds(imgs, geoms, f32)
    for name, got in outs.items():
        for i, (a, b) in enumerate(zip(outs["gather"], got)):
            assert np.array_equal(a.view(np.uint8), b.view(np.uint8)), (case, name, i)
    if not f32:
        for img, g, o in zip(imgs, geoms, outs["default"]):
            m, frac = compare(o, oracle_out(img, g))
            assert m <= 1 and frac < 2e-3, (case, g, m, frac)
