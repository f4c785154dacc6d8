"""GPU: device-resident batches (reference stream/Batch.cpp:25-39
-> core/Utils.cpp:209-252 merge_batch, which always builds host arrays).

``batch(n, device=d)`` makes the image keys' batch tensors in device memory:
pending images are written there by the fused kernel from staged host
footprints (mxd_resize_crop_to_device; no D2H), anything else is batched on
the host and uploaded once.  The result is a DeviceArray -- a DLPack producer
(kDLROCM) -- whose bytes equal the host batch exactly."""
import ctypes
import json
import os
import subprocess
import sys

import numpy as np
import pytest

from gpu_util import synth
from mlx_data_amd import data as dx

pytestmark = pytest.mark.gpu
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def samples(n, seed=0):
    shapes = [(960, 1280), (375, 500), (200, 300), (500, 375)]
    return [dict(image=synth(*shapes[i % 4], 3, seed + i), label=i) for i in range(n)]


def chain(b):
    return b.image_resize_smallest_side("image", 256).image_center_crop("image", 224, 224)


def test_device_batch_equals_host_batch():
    b = chain(dx.buffer_from_vector(samples(6)))
    host = b.batch(6)[0]
    dev = b.batch(6, device=0)[0]
    img = dev["image"]
    assert isinstance(img, dx.DeviceArray) and isinstance(dev["label"], np.ndarray)
    assert img.shape == (6, 224, 224, 3) and img.dtype == np.uint8 and img.device == 0
    assert img.nbytes == 6 * 224 * 224 * 3 and img.data_ptr != 0
    assert np.array_equal(img.numpy(), host["image"]) and np.array_equal(np.asarray(img), host["image"])
    assert np.array_equal(dev["label"], host["label"])
    # fused normalize straight into the device tensor
    f = b.image_to_float("image").batch(6, device=0)[0]["image"]
    assert f.dtype == np.float32
    lut = np.arange(256, dtype=np.uint8).astype(np.float32) / np.float32(255)
    assert np.array_equal(f.numpy().view(np.uint32), lut[host["image"]].view(np.uint32))


def test_ragged_and_listed_keys_upload_the_host_batch():
    raw = [dict(image=synth(40 + 7 * i, 50 + 5 * i, 3, i), label=i) for i in range(5)]
    b = dx.buffer_from_vector(raw).image_random_h_flip("image", 0.5)
    dx.set_state(3)
    host = b.batch(5, pad={"image": 11})[0]
    dx.set_state(3)
    dev = b.batch(5, pad={"image": 11}, device=0, device_keys=["image", "label"])[0]
    assert isinstance(dev["label"], dx.DeviceArray)
    assert np.array_equal(dev["image"].numpy(), host["image"])
    assert np.array_equal(dev["label"].numpy(), host["label"])


def test_stream_prefetch_device_batches():
    s = chain(dx.buffer_from_vector(samples(12, seed=5)).to_stream()).batch(4, device=0).prefetch(3, 3)
    ref = {int(lab): img for x in chain(dx.buffer_from_vector(samples(12, seed=5))).batch(4)
           for lab, img in zip(x["label"], x["image"])}
    seen = 0
    for x in s:
        imgs = x["image"].numpy()
        for lab, img in zip(x["label"], imgs):
            assert np.array_equal(img, ref[int(lab)])
            seen += 1
    assert seen == 12


class _DLDevice(ctypes.Structure):
    _fields_ = [("device_type", ctypes.c_int32), ("device_id", ctypes.c_int32)]


class _DLDataType(ctypes.Structure):
    _fields_ = [("code", ctypes.c_uint8), ("bits", ctypes.c_uint8), ("lanes", ctypes.c_uint16)]


class _DLTensor(ctypes.Structure):
    _fields_ = [("data", ctypes.c_void_p), ("device", _DLDevice), ("ndim", ctypes.c_int32),
                ("dtype", _DLDataType), ("shape", ctypes.POINTER(ctypes.c_int64)),
                ("strides", ctypes.POINTER(ctypes.c_int64)), ("byte_offset", ctypes.c_uint64)]


def test_dlpack_capsule_describes_the_device_tensor():
    img = chain(dx.buffer_from_vector(samples(3))).image_to_float("image").batch(3, device=0)[0]["image"]
    assert img.__dlpack_device__() == (10, 0)  # kDLROCM
    cap = img.__dlpack__()
    get = ctypes.pythonapi.PyCapsule_GetPointer
    get.restype = ctypes.c_void_p
    get.argtypes = [ctypes.py_object, ctypes.c_char_p]
    t = _DLTensor.from_address(get(cap, b"dltensor"))
    assert t.data == img.data_ptr and t.device.device_type == 10 and t.device.device_id == 0
    assert t.ndim == 4 and [t.shape[i] for i in range(4)] == [3, 224, 224, 3]
    assert (t.dtype.code, t.dtype.bits, t.dtype.lanes) == (2, 32, 1) and not t.strides
    del cap  # unconsumed: the capsule frees its tensor


def test_image_ops_refuse_device_arrays():
    dev = chain(dx.buffer_from_vector(samples(2))).batch(2, device=0)
    with pytest.raises(RuntimeError, match="device-resident"):
        dev.image_center_crop("image", 10, 10)[0]
    with pytest.raises(RuntimeError, match="cannot batch device-resident"):
        dev.batch(1)[0]


TORCH_CONSUMER = r"""
import json, sys
import numpy as np
import torch                      # torch first: its HIP runtime is the one libmxd_amd.so binds
torch.zeros(1, device="cuda")
sys.path[:0] = [{repo!r}, {repo!r} + "/tests", {repo!r} + "/oracle", {repo!r} + "/mlx-data_amd"]
from mlx_data_amd import data as dx
from gpu_util import synth
imgs = [dict(image=synth(300 + 40 * i, 400, 3, i)) for i in range(4)]
b = dx.buffer_from_vector(imgs).image_resize_smallest_side("image", 256).image_center_crop("image", 224, 224)
host = b.image_to_float("image").batch(4)[0]["image"]
dev = b.image_to_float("image").batch(4, device=0)[0]["image"]
t = torch.from_dlpack(dev)
ok = t.is_cuda and t.shape == (4, 224, 224, 3) and t.dtype == torch.float32
same = bool(np.array_equal(t.cpu().numpy().view(np.uint32), host.view(np.uint32)))
s = float((t * 2).sum().item())   # a torch kernel reading the batch in place
print(json.dumps(dict(ok=bool(ok), same=same, sum_ok=abs(s - 2 * float(host.astype(np.float64).sum())) < 1e-2 * s)))
"""


@pytest.mark.timeout(300)
def test_torch_consumes_device_batch_via_dlpack():
    """torch.from_dlpack on a device batch, zero copy, in a process that
    imported torch first (the one-HIP-runtime configuration)."""
    code = TORCH_CONSUMER.format(repo=REPO)
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-2000:]
    res = json.loads(r.stdout.strip().splitlines()[-1])
    assert res == dict(ok=True, same=True, sum_ok=True), res


POOL_REUSE = r"""
import json, sys
import numpy as np
import torch                      # torch first (the one-HIP-runtime configuration)
torch.zeros(1, device="cuda")
sys.path[:0] = [{repo!r}, {repo!r} + "/tests", {repo!r} + "/oracle", {repo!r} + "/mlx-data_amd"]
from mlx_data_amd import data as dx
from gpu_util import synth
imgs = [dict(image=synth(300 + 40 * (i % 4), 400, 3, 5 + i)) for i in range(8)]
b = dx.buffer_from_vector(imgs).image_resize_smallest_side("image", 256).image_center_crop("image", 224, 224)
host = b.batch(8)[0]["image"]
want = float(host.astype(np.float64).sum())
side = torch.cuda.Stream()
sums = []
for _ in range(12):
    dev = b.batch(8, device=0)[0]["image"]
    t = torch.from_dlpack(dev)
    with torch.cuda.stream(side):
        acc = torch.zeros((), device=t.device, dtype=torch.float64)
        for _ in range(20):           # the side stream reads the block 20 times
            acc = acc + t.double().sum()
        sums.append(acc / 20)
    del t, dev                        # the block returns to the pool while the side stream may still read it
torch.cuda.synchronize()
ok = all(abs(float(x.item()) - want) < 1e-6 * want for x in sums)
again = b.batch(8, device=0)[0]["image"]
print(json.dumps(dict(sums_ok=bool(ok), again=bool(np.array_equal(again.numpy(), host)))))
"""


@pytest.mark.timeout(300)
def test_device_batch_blocks_recycled_safely():
    """Device batch tensors come from a per-device pool (pipeline.cpp
    DevicePool): a released block is reused only after a device
    synchronisation that followed its release.  A torch consumer enqueues 20
    reads of each batch on a stream of its own and drops the tensor at once;
    the next batches (same size: reuse) must not disturb what it reads, and a
    later batch must equal the host batch."""
    code = POOL_REUSE.format(repo=REPO)
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-2000:]
    res = json.loads(r.stdout.strip().splitlines()[-1])
    assert res == dict(sums_ok=True, again=True), res


def test_device_pool_stays_bounded_over_changing_shapes():
    """Batches whose byte size changes every time: each released
    block waits for a device synchronisation before reuse; the pool drains its
    pending blocks once they pass half its cap, so idle + pending stays within
    the 2 GiB cap (plus the block in use) however many shapes go by."""
    from mlx_data_amd import _pipeline

    cap = 2 << 30
    peak = 0
    for mb in range(1, 81):  # 1..80 MiB per batch: 3.2 GiB of distinct sizes in all
        a = np.full(((mb << 20) // 3072, 1024, 3), mb % 251, np.uint8)
        d = dx.buffer_from_vector([dict(image=a)]).batch(1, device=0, device_keys=["image"])[0]["image"]
        assert isinstance(d, dx.DeviceArray)
        if mb % 20 == 0:
            assert np.array_equal(d.numpy()[0, -1], a[-1])
        del d
        peak = max(peak, _pipeline._device_pool_bytes(0))
        assert _pipeline._device_pool_bytes(0) <= cap + (mb << 20), (mb, _pipeline._device_pool_bytes(0))
    assert peak > cap // 2  # the drain was exercised
