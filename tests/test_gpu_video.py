"""GPU parity of the image ops on (F, H, W, C) videos: op/ImageTransform.cpp
ImageTransformOp::apply_video (:33-70, per-frame apply_image, frames stacked),
ImageRandomCrop / ImageRandomAreaCrop::apply_video (:160-182, :293-315, ONE
draw for all frames) and ImageRandomHFlip::apply_video (:334-356, one draw).
Pending frame plans materialise in one batched launch (pipeline stack_frames).
"""
import numpy as np
import pytest

import oracle as O
from gpu_util import compare, synth
from mlx_data_amd import data as dx

pytestmark = pytest.mark.gpu


def video(f=4, h=120, w=160, seed=0):
    return np.stack([synth(h, w, 3, seed + i) for i in range(f)])


def test_resize_center_crop_video():
    v = video()
    b = dx.buffer_from_vector([dict(video=v)])
    out = np.asarray(b.image_resize_smallest_side("video", 64).image_center_crop("video", 56, 56)[0]["video"])
    assert out.shape == (4, 56, 56, 3)
    tw, th = O.smallest_side_dims(160, 120, 64)
    x, y = O.center_crop_origin(tw, th, 56, 56)
    for i in range(4):
        m, frac = compare(out[i], O.crop(O.resize(v[i], tw, th), x, y, 56, 56))
        assert m <= 1 and frac < 2e-3, (i, m, frac)


def test_random_crop_video_one_draw():
    v = video(5, 90, 130, 7)
    b = dx.buffer_from_vector([dict(video=v)])
    dx.set_state(99)
    out = np.asarray(b.image_random_crop("video", 64, 48)[0]["video"])
    # the same draw on a single frame of the same size
    dx.set_state(99)
    one = np.asarray(dx.buffer_from_vector([dict(image=v[0])]).image_random_crop("image", 64, 48)[0]["image"])
    assert out.shape == (5, 48, 64, 3)
    assert np.array_equal(out[0], one)
    hits = [(x, y) for y in range(90 - 48 + 1) for x in range(130 - 64 + 1)
            if np.array_equal(v[0, y:y + 48, x:x + 64], one)]
    assert hits
    x, y = hits[0]
    for i in range(5):
        assert np.array_equal(out[i], v[i, y:y + 48, x:x + 64]), i


def test_hflip_video_all_or_none():
    v = video(3, 40, 50, 3)
    b = dx.buffer_from_vector([dict(video=v)])
    out = np.asarray(b.image_random_h_flip("video", 1.0)[0]["video"])
    assert np.array_equal(out, v[:, :, ::-1])
    out = np.asarray(b.image_random_h_flip("video", -1.0)[0]["video"])
    assert np.array_equal(out, v)


def test_rotate_and_gray_video():
    v = video(3, 37, 53, 11)
    b = dx.buffer_from_vector([dict(video=v)])
    s = b.image_rotate("video", 30.0, output_key="r").image_channel_reduction("video", "rec709", output_key="g")[0]
    r, g = np.asarray(s["r"]), np.asarray(s["g"])
    for i in range(3):
        assert np.array_equal(r[i], O.rotate(v[i], 30.0, False))
        assert np.array_equal(g[i], O.channel_reduction(v[i], "rec709"))


def test_random_area_crop_video_one_draw():
    v = video(3, 80, 100, 21)
    b = dx.buffer_from_vector([dict(video=v)])
    dx.set_state(5)
    out = np.asarray(b.image_random_area_crop("video", (0.2, 0.5), (0.75, 1.33))[0]["video"])
    assert out.shape[0] == 3
    h, w = out.shape[1:3]
    hits = [(x, y) for y in range(80 - h + 1) for x in range(100 - w + 1) if np.array_equal(v[0, y:y + h, x:x + w], out[0])]
    assert hits
    x, y = hits[0]
    for i in range(3):
        assert np.array_equal(out[i], v[i, y:y + h, x:x + w])
