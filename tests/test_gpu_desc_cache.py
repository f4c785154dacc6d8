"""GPU: the descriptor-slot cache of mxd_resize_crop_batch (batch.cpp
upload_descs: 16 slots per (device, stream), reuse fenced every 8 batches
that wrote a slot).  24 distinct batches -- more than the slots -- launched
back to back on one stream with no host sync in between: first a long run of
cache hits only (which records no fence), then evictions whose fence
wait_batch must record on demand, mixed with more hits and fresh uploads.
Every batch writes its own output buffers, and each batch's images are crops
of different windows, so a launch that read another batch's (or a
half-overwritten) descriptor array would leave wrong bytes behind."""
import ctypes

import numpy as np
import pytest

import oracle as O
from gpu_util import synth
from mlx_data_amd import capi

pytestmark = pytest.mark.gpu


SLOTS = 16    # Workspace::kSlots (batch.cpp)
NBATCH = 24   # distinct batches: more than the slots


def test_slot_reuse_under_back_to_back_launches():
    imgs = [synth(300 + 20 * i, 400 + 30 * i, 3, 50 + i) for i in range(4)]
    pitch = [(im.shape[1] * 3 + 15) // 16 * 16 for im in imgs]
    src = [capi.DeviceBuffer(p * im.shape[0], 0) for p, im in zip(pitch, imgs)]
    for b, p, im in zip(src, pitch, imgs):
        host = np.zeros((im.shape[0], p), np.uint8)
        host[:, :im.shape[1] * 3] = im.reshape(im.shape[0], -1)
        b.upload(host)
    batches = []  # (descriptor array, n, [(dst buffer, expected)])
    for k in range(NBATCH):
        entries, outs = [], []
        for i, im in enumerate(imgs):
            h, w = im.shape[:2]
            rw, rh = O.smallest_side_dims(w, h, 96 + 4 * k)
            cw, ch = 48, 40
            cx, cy = (rw - cw) * (k % 8 + 1) // 9, (rh - ch) * (7 - k % 8) // 9 + k // 8
            flip = (k + i) % 2
            d = capi.DeviceBuffer(cw * ch * 3, 0)
            d.memset(0)
            want = O.crop(O.resize(im, rw, rh), cx, cy, cw, ch)
            outs.append((d, O.hflip(want) if flip else want))
            entries.append(dict(src=src[i].ptr, src_stride=pitch[i], src_w=w, src_h=h, channels=3, resize_w=rw,
                                resize_h=rh, crop_x=cx, crop_y=cy, crop_w=cw, crop_h=ch, flip=flip, dst=d.ptr,
                                dst_stride=cw * 3))
        arr, n = capi.make_images(entries)
        batches.append((arr, n, outs))
    capi.check(capi.lib().mxd_stream_synchronize(ctypes.c_void_p(None)))  # the memsets above
    stream = capi.Stream(0)
    fill = list(range(SLOTS))                       # every slot written once
    hits = [k % 5 for k in range(60)]                 # hits only: no fence recorded
    evict = [16, 0, 17, 18, 1, 19, 20, 2, 21, 22, 23]  # evictions right behind the hits
    mixed = [0, 16, 5, 23, 9, 12, 3, 20, 14, 7, 18, 1] * 3
    order = fill + hits + evict + mixed + list(range(NBATCH))
    for k in order:
        arr, n, _ = batches[k]
        capi.resize_crop_batch(arr, n, capi.MXD_U8, 0, stream.handle)
    stream.synchronize()
    for arr, n, outs in batches:
        for d, want in outs:
            got = d.download(want.shape, np.uint8)
            assert np.abs(got.astype(int) - want.astype(int)).max() <= 1
            d.free()
    for b in src:
        b.free()


@pytest.mark.parametrize("mode", [1, 2, 3, 4, 6])
def test_fresh_descriptor_arrays_every_launch(mode):
    """Every launch carries a new descriptor array (its own output buffers),
    40 launches back to back on one stream through the 16 slots, under each
    upload mode (MXD_TUNE_DESC; 6 = the default, the host stores the array
    into the device slot through the large PCI BAR, 4 without a large BAR:
    the kernels read a non-coherent page-locked slot in place): a launch that read a stale or half-written
    slot would write another launch's geometry into its buffers, or nothing."""
    imgs = [synth(200 + 30 * i, 260 + 20 * i, 3, 70 + i) for i in range(3)]
    pitch = [(im.shape[1] * 3 + 15) // 16 * 16 for im in imgs]
    src = [capi.DeviceBuffer(p * im.shape[0], 0) for p, im in zip(pitch, imgs)]
    for b, p, im in zip(src, pitch, imgs):
        host = np.zeros((im.shape[0], p), np.uint8)
        host[:, :im.shape[1] * 3] = im.reshape(im.shape[0], -1)
        b.upload(host)
    want = {}
    launches = []
    for k in range(40):
        g = k % 5
        entries, outs = [], []
        for i, im in enumerate(imgs):
            h, w = im.shape[:2]
            rw, rh = O.smallest_side_dims(w, h, 64 + 16 * g)
            cw, ch = 40, 32
            cx, cy = (rw - cw) * g // 5, (rh - ch) * (4 - g) // 5
            key = (g, i)
            if key not in want:
                want[key] = O.crop(O.resize(im, rw, rh), cx, cy, cw, ch)
            d = capi.DeviceBuffer(cw * ch * 3, 0)
            d.memset(0)
            outs.append((d, key))
            entries.append(dict(src=src[i].ptr, src_stride=pitch[i], src_w=w, src_h=h, channels=3, resize_w=rw,
                                resize_h=rh, crop_x=cx, crop_y=cy, crop_w=cw, crop_h=ch, flip=0, dst=d.ptr,
                                dst_stride=cw * 3))
        arr, n = capi.make_images(entries)
        launches.append((arr, n, outs))
    capi.check(capi.lib().mxd_stream_synchronize(ctypes.c_void_p(None)))
    prev = capi.set_tuning(capi.MXD_TUNE_DESC, mode)
    try:
        stream = capi.Stream(0)
        for arr, n, _ in launches:
            capi.resize_crop_batch(arr, n, capi.MXD_U8, 0, stream.handle)
        stream.synchronize()
    finally:
        capi.set_tuning(capi.MXD_TUNE_DESC, prev)
    for _, _, outs in launches:
        for d, key in outs:
            got = d.download(want[key].shape, np.uint8)
            assert np.abs(got.astype(int) - want[key].astype(int)).max() <= 1, key
            d.free()
    for b in src:
        b.free()
