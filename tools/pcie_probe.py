"""PCIe copy probe (diagnostic): one large pinned H2D / D2H copy vs many
per-image 2-D copies of C4-sized footprints, on one stream."""
import ctypes
import sys
import time

sys.path.insert(0, "mlx-data_amd")
from mlx_data_amd import capi  # noqa: E402

capi.lib()
hip = ctypes.CDLL("libamdhip64.so")
hip.hipHostMalloc.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_size_t, ctypes.c_uint]
hip.hipMalloc.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_size_t]
hip.hipMemcpyAsync.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int, ctypes.c_void_p]
hip.hipMemcpy2DAsync.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_size_t,
                                 ctypes.c_size_t, ctypes.c_int, ctypes.c_void_p]
hip.hipStreamSynchronize.argtypes = [ctypes.c_void_p]
N = 256 << 20
h, d = ctypes.c_void_p(), ctypes.c_void_p()
assert hip.hipHostMalloc(ctypes.byref(h), N, 0) == 0
assert hip.hipMalloc(ctypes.byref(d), N) == 0
ctypes.memset(h, 1, N)
s = capi.Stream(0)
sh = ctypes.c_void_p(s.handle)


def timed(f, reps=5):
    f()
    s.synchronize()
    t = time.perf_counter()
    for _ in range(reps):
        f()
    s.synchronize()
    return (time.perf_counter() - t) / reps


for mb in (24, 96, 256):
    b = mb << 20
    t = timed(lambda: hip.hipMemcpyAsync(d, h, b, 1, sh))
    print(f"H2D {mb} MB one copy: {b / t / 1e9:.1f} GB/s")
    t = timed(lambda: hip.hipMemcpyAsync(h, d, b, 2, sh))
    print(f"D2H {mb} MB one copy: {b / t / 1e9:.1f} GB/s")
    t = timed(lambda: (hip.hipMemcpyAsync(d, h, b, 1, sh), hip.hipMemcpyAsync(ctypes.c_void_p(h.value + b), ctypes.c_void_p(d.value + b), b // 2, 2, sh)))
    print(f"H2D {mb} MB then D2H {mb // 2} MB same stream: {1.5 * b / t / 1e9:.1f} GB/s")
# C4-like footprints: 128 images, 256 rows x 1000 B from a 1500-B pitch
rows, width, pitch = 256, 1000, 1500
t = timed(lambda: [hip.hipMemcpy2DAsync(ctypes.c_void_p(d.value + i * rows * 1008), 1008,
                                        ctypes.c_void_p(h.value + i * rows * pitch), pitch, width, rows, 1, sh)
                   for i in range(128)])
print(f"128 x 2D H2D ({rows}x{width} B): {t * 1e3:.3f} ms, {128 * rows * width / t / 1e9:.1f} GB/s")
t = timed(lambda: hip.hipMemcpyAsync(d, h, 128 * rows * width, 1, sh))
print(f"same bytes one H2D: {t * 1e3:.3f} ms")
