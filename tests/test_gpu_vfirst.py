"""GPU: every resample kernel is bit-exact to the kernel-order oracle
(oracle/stbir_oracle.c orc_resize_crop_vfirst: the shared tap tables, vertical
pass first in byte units, fmaf chains in tap order from 0, stbir's encode) --
SURVEY.md §8(c)2's "bit-exact when coefficient tables are shared" gate.  The
stbir-order restatement (horizontal first, decoded to [0, 1]) stays the
reference-semantics check at +-1 (tests/test_gpu_parity.py); what is still
unpinned about stbir itself is listed in DESIGN.md §3.

Full-size workloads: C2 (1280x960 -> 256 -> 224), C3's six sizes, C4's
ImageNet shapes, C5 (4K -> 512, random 448 crops, mirrored), Caltech
upsampling, arbitrary windows and 12 / 24 MP photos; each on the default
choice, the band kernel (MXD_POLICY_PREFER_BAND), the wave kernels
(MXD_POLICY_NO_BAND), the 256-pixel-window wave kernels (MXD_POLICY_NARROW)
and the general kernel (MXD_POLICY_NO_WAVE)."""
import numpy as np
import pytest

import oracle as O
from gpu_util import center_geom, run_device, synth
from mlx_data_amd import capi

pytestmark = pytest.mark.gpu

POLICIES = [("default", capi.MXD_POLICY_AUTO), ("band", capi.MXD_POLICY_PREFER_BAND),
            ("wave", capi.MXD_POLICY_NO_BAND), ("narrow", capi.MXD_POLICY_NARROW),
            ("general", capi.MXD_POLICY_NO_WAVE)]


def _cases():
    out = {}
    imgs = [synth(960, 1280, 3, s) for s in range(2)]
    out["c2"] = (imgs, [center_geom(i) for i in imgs])
    sizes = [(480, 640), (720, 1280), (960, 1280), (1080, 1920), (1440, 2560), (2160, 3840)]
    imgs = [synth(h, w, 3, 60 + i) for i, (h, w) in enumerate(sizes)]
    out["c3"] = (imgs, [center_geom(i) for i in imgs])
    imgs = [synth(375, 500, 3, 70), synth(500, 375, 3, 71), synth(333, 500, 3, 72), synth(200, 300, 3, 73)]
    out["c4_caltech"] = (imgs, [center_geom(i) for i in imgs])
    img = synth(2160, 3840, 3, 74)
    tw, th = O.smallest_side_dims(3840, 2160, 512)
    out["c5"] = ([img] * 4, [(tw, th, 0, 0, 448, 448, 1), (tw, th, tw - 448, th - 448, 448, 448, 0),
                             (tw, th, 201, 33, 448, 448, 1), (tw, th, tw - 448, 0, 448, 448, 1)])
    rng = np.random.default_rng(9)
    imgs, geoms = [], []
    for k in range(10):
        h, w = int(rng.integers(40, 1200)), int(rng.integers(40, 1200))
        rw, rh = int(rng.integers(16, 380)), int(rng.integers(16, 380))
        cw, ch = int(rng.integers(1, min(rw, 256) + 1)), int(rng.integers(1, rh + 1))
        imgs.append(synth(h, w, 3, 80 + k))
        geoms.append((rw, rh, int(rng.integers(0, rw - cw + 1)), int(rng.integers(0, rh - ch + 1)), cw, ch,
                      int(rng.integers(0, 2))))
    out["windows"] = (imgs, geoms)
    imgs = [synth(3024, 4032, 3, 90), synth(4000, 6000, 3, 91)]
    out["photos_12_24mp"] = (imgs, [center_geom(i) for i in imgs])
    return out


CASES = _cases()


@pytest.mark.parametrize("case", sorted(CASES))
def test_kernels_bit_exact_to_vfirst_oracle(case):
    imgs, geoms = CASES[case]
    want = [O.resize_crop_vfirst(i, g) for i, g in zip(imgs, geoms)]
    lut = (np.arange(256, dtype=np.uint8).astype("float32") / 255).view(np.uint32)
    for name, policy in POLICIES:
        prev = capi.set_kernel_policy(policy)
        try:
            u8 = run_device(imgs, geoms)
            f32 = run_device(imgs, geoms, f32=True)
        finally:
            capi.set_kernel_policy(prev)
        for g, w, a, f in zip(geoms, want, u8, f32):
            diff = int((a != w).sum())
            assert diff == 0, (name, case, g, diff)
            assert np.array_equal(f.view(np.uint32), lut[w]), (name, case, g)


@pytest.mark.parametrize("streams", [1, 2, 3, 4])
def test_mixed_batch_launch_layouts_keep_bytes(streams):
    """C3's six shapes in one batch with its six launches over 1 .. 4 streams
    (MXD_TUNE_STREAMS; default 2) -- bit-exact to the kernel-order oracle."""
    imgs, geoms = CASES["c3"]
    ps = capi.set_tuning(capi.MXD_TUNE_STREAMS, streams)
    try:
        outs = run_device(imgs, geoms)
    finally:
        capi.set_tuning(capi.MXD_TUNE_STREAMS, ps)
    for img, g, o in zip(imgs, geoms, outs):
        assert np.array_equal(o, O.resize_crop_vfirst(img, g)), g
