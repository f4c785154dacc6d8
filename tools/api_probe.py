"""Host cost of the HIP runtime calls a batch submission makes (us per call,
median of 5 x 2000 calls) on one device: hipEventRecord / hipEventQuery /
hipEventSynchronize of a completed event, hipStreamWaitEvent, a 13 KB
page-locked -> device hipMemcpyAsync, and a memcpy of 13 KB into page-locked
memory.  python tools/api_probe.py"""
import ctypes
import json
import os
import statistics
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "mlx-data_amd"))
from mlx_data_amd import capi  # noqa: E402

capi.lib()  # binds /opt/rocm's HIP runtime
hip = ctypes.CDLL("libamdhip64.so")
vp = ctypes.c_void_p


def ok(rc):
    assert rc == 0, rc


ok(hip.hipSetDevice(0))
s = vp()
ok(hip.hipStreamCreateWithFlags(ctypes.byref(s), 1))
s2 = vp()
ok(hip.hipStreamCreateWithFlags(ctypes.byref(s2), 1))
ev = vp()
ok(hip.hipEventCreateWithFlags(ctypes.byref(ev), 2))  # hipEventDisableTiming
n = 13312
hostp = vp()
ok(hip.hipHostMalloc(ctypes.byref(hostp), ctypes.c_size_t(n), 0))
devp = vp()
ok(hip.hipMalloc(ctypes.byref(devp), ctypes.c_size_t(n)))
src = (ctypes.c_uint8 * n)()


def per_call(fn, k=2000):
    fn()
    hip.hipStreamSynchronize(s)
    t = []
    for _ in range(5):
        t0 = time.perf_counter()
        for _ in range(k):
            fn()
        t.append((time.perf_counter() - t0) / k * 1e6)
        hip.hipStreamSynchronize(s)
    return round(statistics.median(t), 2)


out = {
    "python_ctypes_noop": per_call(lambda: hip.hipGetLastError()),
    "hipEventRecord": per_call(lambda: hip.hipEventRecord(ev, s)),
    "hipEventQuery_done": per_call(lambda: hip.hipEventQuery(ev)),
    "hipEventSynchronize_done": per_call(lambda: hip.hipEventSynchronize(ev)),
    "hipStreamWaitEvent": per_call(lambda: hip.hipStreamWaitEvent(s2, ev, 0)),
    "hipMemcpyAsync_13KB_pinned_h2d": per_call(lambda: hip.hipMemcpyAsync(devp, hostp, ctypes.c_size_t(n), 1, s), 500),
    "memmove_13KB_to_pinned": per_call(lambda: ctypes.memmove(hostp, src, n)),
}
print(json.dumps(out))
