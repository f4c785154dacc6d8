"""GPU: work stealing between the units of a scatter wave launch (round 6,
mlx-data_amd/csrc/wave.hip `Steal`) never changes a byte.

A wave that finishes its band takes the last blocks of the band furthest
behind and runs them from the same schedule; the owner stops before them.
The tests run the same inputs with stealing off (MXD_TUNE_STEAL 1), on (2)
and in the test mode (3: the owners of odd units start ~80 us late, so that
thieves run the ends of half the bands, and owners read limits lowered
while they slept), and require byte-identical outputs:

* C2 at its full launch shape (256 x 1280x960 -> 224^2 f32: 4,096 units,
  one occupancy round), and the u8 form;
* a mixed-resolution batch (several scatter launches on two streams);
* the C4 JPEG slice through the operator surface (scatter kernels reading
  JPEG sample planes), against the host decode as well.
The steal-off output is the product's pre-stealing path, which the parity
suites pin to the oracle."""
import io

import numpy as np
import pytest

from gpu_util import center_geom, run_device, synth

pytestmark = pytest.mark.gpu

from mlx_data_amd import capi

MODES = [1, 2, 3]


def _run_modes(imgs, geoms, f32):
    outs = {}
    try:
        for m in MODES:
            capi.set_tuning(capi.MXD_TUNE_STEAL, m)
            outs[m] = run_device(imgs, geoms, f32=f32)
    finally:
        capi.set_tuning(capi.MXD_TUNE_STEAL, 0)
    return outs


def _same(outs, tag):
    for m in MODES[1:]:
        for i, (a, b) in enumerate(zip(outs[MODES[0]], outs[m])):
            assert np.array_equal(a.view(np.uint8), b.view(np.uint8)), (tag, m, i)


@pytest.mark.parametrize("f32", [True, False])
def test_c2_full_launch_steal_modes_identical(f32):
    base = [synth(960, 1280, 3, 300 + s) for s in range(8)]
    imgs = [base[i % 8] if i % 3 else np.ascontiguousarray(base[i % 8][::-1]) for i in range(256)]
    geoms = [center_geom(i) for i in imgs]
    _same(_run_modes(imgs, geoms, f32), ("c2", f32))


def test_mixed_batch_steal_modes_identical():
    sizes = [(480, 640), (720, 1280), (1080, 1920), (1440, 2560), (2160, 3840), (375, 500), (500, 333), (960, 1280)]
    imgs = [synth(h, w, 3, 40 + i) for i, (h, w) in enumerate(sizes * 4)]
    geoms = [center_geom(i) for i in imgs]
    _same(_run_modes(imgs, geoms, False), "mixed")


def test_c4_jpeg_planes_steal_modes_identical(tmp_path):
    from PIL import Image

    from mlx_data_amd import data as dx

    rng = np.random.default_rng(5)
    files = []
    for i in range(64):
        w, h = [(500, 375), (375, 500), (500, 333)][int(rng.integers(0, 3))]
        b = io.BytesIO()
        Image.fromarray(synth(h, w, 3, 700 + i)).save(b, "JPEG", quality=90)
        p = tmp_path / f"{i:03d}.jpg"
        p.write_bytes(b.getvalue())
        files.append(str(p))

    def batch(device_decode):
        before = dx.device_decode()
        dx.set_device_decode(device_decode)
        try:
            d = (dx.buffer_from_vector([dict(image=f.encode()) for f in files]).load_image("image")
                 .image_resize_smallest_side("image", 256).image_center_crop("image", 224, 224)
                 .image_to_float("image").batch(len(files)))
            return np.asarray(d[0]["image"])
        finally:
            dx.set_device_decode(before)

    host = batch(False)
    try:
        for m in MODES:
            capi.set_tuning(capi.MXD_TUNE_STEAL, m)
            got = batch(True)
            assert np.array_equal(got.view(np.uint8), host.view(np.uint8)), m
    finally:
        capi.set_tuning(capi.MXD_TUNE_STEAL, 0)
