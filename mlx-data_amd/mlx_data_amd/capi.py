"""ctypes binding of the C ABI in include/mxd_amd.h (libmxd_amd.so).

This is the Python-side stub a maintainer would add to bind the library
(INTEGRATION.md); the C++ pipeline binds the same symbols directly.  Loading
fails loudly when the library is missing: there is no CPU fallback.
"""
import ctypes
import os

import numpy as np

PKG_ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB_PATH = os.path.join(PKG_ROOT, "libmxd_amd.so")

MXD_OK = 0
MXD_ERR_INVALID = 1
MXD_ERR_UNSUPPORTED = 2
MXD_ERR_DEVICE = 3
MXD_ERR_NOMEM = 4
MXD_U8 = 0
MXD_F32_DIV255 = 1

# Every symbol include/mxd_amd.h declares.
EXPORTS = (
    "mxd_abi_version", "mxd_last_error", "mxd_device_count", "mxd_device_properties",
    "mxd_resize_smallest_side_dims", "mxd_center_crop_origin", "mxd_axis_taps",
    "mxd_resize_crop_batch", "mxd_set_kernel_policy", "mxd_set_tuning", "mxd_describe_plan",
    "mxd_describe_band_plan", "mxd_copy_bandwidth",
    "mxd_set_device", "mxd_malloc_device", "mxd_free_device", "mxd_malloc_pinned", "mxd_free_pinned",
    "mxd_memcpy_h2d_async", "mxd_memcpy_d2h_async", "mxd_memcpy2d_h2d_async", "mxd_memset_async",
    "mxd_stream_create", "mxd_stream_destroy", "mxd_stream_synchronize", "mxd_device_synchronize",
    "mxd_event_create", "mxd_event_destroy", "mxd_event_record", "mxd_event_synchronize", "mxd_event_elapsed_ms",
    "mxd_resize_crop_host", "mxd_resize_crop_to_device", "mxd_memcpy_h2d", "mxd_memcpy_d2h",
    "mxd_release_host_buffers",
    "mxd_rotate_geometry", "mxd_channel_reduction_preset", "mxd_pixmap_batch", "mxd_pixmap_host",
    "mxd_is_jpeg", "mxd_jpeg_info", "mxd_jpeg_decode",
    "mxd_jpeg_coefs_decode", "mxd_jpeg_coefs_parse", "mxd_jpeg_coefs_load", "mxd_jpeg_coefs_entropy_pending", "mxd_jpeg_coefs_free",
    "mxd_jpeg_coefs_info", "mxd_jpeg_coefs_finish",
    "mxd_jpeg_resize_crop_host", "mxd_jpeg_resize_crop_to_device", "mxd_jpeg_plane_sources", "mxd_host_stats", "mxd_device_stats", "mxd_copy_bandwidth_policy",
    "mxd_narrow_returns",
)

MXD_AFFINE = 0
MXD_CHANNEL_REDUCTION = 1

MXD_POLICY_AUTO = 0
MXD_POLICY_NO_SCATTER = 1
MXD_POLICY_NO_WAVE = 2
MXD_POLICY_NARROW = 4
MXD_POLICY_NO_DESC_CACHE = 8
MXD_POLICY_NO_BYTES = 16
MXD_POLICY_BYTES = 32
MXD_POLICY_NO_ZERO_COPY = 64
MXD_POLICY_NO_BAND = 128
MXD_POLICY_PREFER_BAND = 256

MXD_TUNE_BAND_ROWS = 0
MXD_TUNE_BAND_LA = 1
MXD_TUNE_BAND_GRID = 2
MXD_TUNE_DESC = 3
MXD_TUNE_STREAMS = 4
MXD_TUNE_HUFF_BITS = 5
MXD_TUNE_HUFF_GLOBAL = 6
MXD_TUNE_HOST_WAIT = 7
MXD_TUNE_HOST_STREAMS = 8
MXD_TUNE_HUFF_JOB = 9
MXD_TUNE_JPEG_RGB = 10
MXD_TUNE_DEVICE_TIMING = 11
MXD_TUNE_LOAD_POLICY = 12
MXD_TUNE_F32_LINK = 13


class MxdImage(ctypes.Structure):
    """struct mxd_image (include/mxd_amd.h)."""

    _fields_ = [
        ("src", ctypes.c_void_p),
        ("src_stride", ctypes.c_int64),
        ("src_w", ctypes.c_int32),
        ("src_h", ctypes.c_int32),
        ("channels", ctypes.c_int32),
        ("resize_w", ctypes.c_int32),
        ("resize_h", ctypes.c_int32),
        ("crop_x", ctypes.c_int32),
        ("crop_y", ctypes.c_int32),
        ("crop_w", ctypes.c_int32),
        ("crop_h", ctypes.c_int32),
        ("flip", ctypes.c_int32),
        ("dst", ctypes.c_void_p),
        ("dst_stride", ctypes.c_int64),
        ("rgba_weighted", ctypes.c_int32),
        ("reserved", ctypes.c_int32),
    ]


class MxdPixmap(ctypes.Structure):
    """struct mxd_pixmap (include/mxd_amd.h): rotate / channel reduction."""

    _fields_ = [
        ("src", ctypes.c_void_p),
        ("src_stride", ctypes.c_int64),
        ("src_w", ctypes.c_int32),
        ("src_h", ctypes.c_int32),
        ("channels", ctypes.c_int32),
        ("dst_w", ctypes.c_int32),
        ("dst_h", ctypes.c_int32),
        ("dst", ctypes.c_void_p),
        ("dst_stride", ctypes.c_int64),
        ("params", ctypes.c_float * 6),
    ]


class MxdJpegImage(ctypes.Structure):
    """struct mxd_jpeg_image (include/mxd_amd.h): decode + resize + crop."""

    _fields_ = [
        ("coefs", ctypes.c_void_p),
        ("win_x", ctypes.c_int32),
        ("win_y", ctypes.c_int32),
        ("win_w", ctypes.c_int32),
        ("win_h", ctypes.c_int32),
        ("resize_w", ctypes.c_int32),
        ("resize_h", ctypes.c_int32),
        ("crop_x", ctypes.c_int32),
        ("crop_y", ctypes.c_int32),
        ("crop_w", ctypes.c_int32),
        ("crop_h", ctypes.c_int32),
        ("flip", ctypes.c_int32),
        ("reserved", ctypes.c_int32),
        ("dst", ctypes.c_void_p),
        ("dst_stride", ctypes.c_int64),
    ]


class MxdError(RuntimeError):
    def __init__(self, code, msg):
        super().__init__(msg)
        self.code = code


_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise ImportError(f"{LIB_PATH} not built: run __graft_entry__.build() or `make -C mlx-data_amd`")
        L = ctypes.CDLL(LIB_PATH)
        L.mxd_last_error.restype = ctypes.c_char_p
        for name in ("mxd_malloc_pinned", "mxd_free_pinned", "mxd_memcpy_h2d_async", "mxd_memcpy_d2h_async",
                     "mxd_memset_async"):
            getattr(L, name).restype = ctypes.c_int
        _lib = L
    return _lib


def check(rc):
    if rc != MXD_OK:
        raise MxdError(rc, lib().mxd_last_error().decode())
    return rc


def device_properties(device=0):
    """(name, gcnArchName, compute units) of a device."""
    name, arch, cus = ctypes.create_string_buffer(256), ctypes.create_string_buffer(64), ctypes.c_int32()
    check(lib().mxd_device_properties(device, name, ctypes.c_size_t(256), arch, ctypes.c_size_t(64), ctypes.byref(cus)))
    return name.value.decode(), arch.value.decode(), cus.value


def resize_smallest_side_dims(w, h, size):
    tw, th = ctypes.c_int64(), ctypes.c_int64()
    check(lib().mxd_resize_smallest_side_dims(ctypes.c_int64(w), ctypes.c_int64(h), ctypes.c_int64(size),
                                              ctypes.byref(tw), ctypes.byref(th)))
    return tw.value, th.value


def center_crop_origin(w, h, cw, ch):
    x, y = ctypes.c_int64(), ctypes.c_int64()
    check(lib().mxd_center_crop_origin(ctypes.c_int64(w), ctypes.c_int64(h), ctypes.c_int64(cw),
                                       ctypes.c_int64(ch), ctypes.byref(x), ctypes.byref(y)))
    return x.value, y.value


def axis_taps(in_size, out_size, off=0, length=None):
    """(first[len], ntaps[len], weights[len, width]) of the product tap builder."""
    length = out_size - off if length is None else length
    need = ctypes.c_int32()
    L = lib()
    rc = L.mxd_axis_taps(in_size, out_size, off, length, 0, None, None, None, ctypes.byref(need))
    width = need.value
    if rc != MXD_OK and width <= 0:
        check(rc)
    first = np.zeros(length, np.int32)
    cnt = np.zeros(length, np.int32)
    w = np.zeros((length, width), np.float32)
    check(L.mxd_axis_taps(in_size, out_size, off, length, width,
                          first.ctypes.data_as(ctypes.POINTER(ctypes.c_int32)),
                          cnt.ctypes.data_as(ctypes.POINTER(ctypes.c_int32)),
                          w.ctypes.data_as(ctypes.POINTER(ctypes.c_float)), None))
    return first, cnt, w


def make_images(entries):
    """entries: iterable of dicts with the mxd_image fields -> ctypes array."""
    entries = list(entries)
    arr = (MxdImage * max(1, len(entries)))()
    for i, e in enumerate(entries):
        for k, v in e.items():
            setattr(arr[i], k, v)
    return arr, len(entries)


def resize_crop_batch(images, n, out_dtype, device=0, stream=None):
    check(lib().mxd_resize_crop_batch(images, n, out_dtype, device, ctypes.c_void_p(stream)))


def set_kernel_policy(policy):
    """Process-wide choice between kernels with identical results; returns the previous policy."""
    return lib().mxd_set_kernel_policy(int(policy))


def set_tuning(knob, value):
    """Process-wide tuning knob (MXD_TUNE_*; 0 = automatic); returns the previous value."""
    return lib().mxd_set_tuning(int(knob), int(value))


PLAN_FIELDS = ("wave", "kind", "taps", "s", "dmax", "q", "nstrips", "p")


def describe_plan(entry, out_dtype=MXD_U8, device=0):
    """The wave-kernel plan of one image (what runs when the band kernel declines it; host only)."""
    arr, _ = make_images([dict(entry, src=entry.get("src", 256), dst=entry.get("dst", 256))])
    info = (ctypes.c_int32 * 8)()
    check(lib().mxd_describe_plan(arr, out_dtype, device, info))
    return dict(zip(PLAN_FIELDS, list(info)))


BAND_FIELDS = ("band", "taps", "db", "s", "nq", "nstrips", "tx", "prologue", "dmax", "la", "lds_bytes")


def describe_band_plan(entry, out_dtype=MXD_U8):
    """The band-kernel plan of one image under the current policy (host only)."""
    arr, _ = make_images([dict(entry, src=entry.get("src", 256), dst=entry.get("dst", 256))])
    info = (ctypes.c_int32 * 12)()
    check(lib().mxd_describe_band_plan(arr, out_dtype, info))
    return dict(zip(BAND_FIELDS, list(info)))


def resize_crop_host(images, n, out_dtype, device=0):
    check(lib().mxd_resize_crop_host(images, n, out_dtype, device))


def resize_crop_to_device(images, n, out_dtype, device=0):
    """Host sources, device destinations (mxd_resize_crop_to_device)."""
    check(lib().mxd_resize_crop_to_device(images, n, out_dtype, device))


def jpeg_info(data):
    """(width, height, components) of a JPEG (bytes / uint8 array)."""
    buf = np.frombuffer(bytes(data), np.uint8) if not isinstance(data, np.ndarray) else np.ascontiguousarray(data)
    w, h, c = ctypes.c_int32(), ctypes.c_int32(), ctypes.c_int32()
    check(lib().mxd_jpeg_info(buf.ctypes.data_as(ctypes.c_void_p), ctypes.c_size_t(buf.nbytes), ctypes.byref(w),
                              ctypes.byref(h), ctypes.byref(c)))
    return w.value, h.value, c.value


def jpeg_decode(data):
    """The native decoder: (H, W, 3) uint8, libjpeg ISLOW + fancy upsampling output."""
    buf = np.frombuffer(bytes(data), np.uint8) if not isinstance(data, np.ndarray) else np.ascontiguousarray(data)
    w, h, _ = jpeg_info(buf)
    out = np.empty((h, w, 3), np.uint8)
    check(lib().mxd_jpeg_decode(buf.ctypes.data_as(ctypes.c_void_p), ctypes.c_size_t(buf.nbytes),
                                out.ctypes.data_as(ctypes.c_void_p), ctypes.c_int64(w * 3), w, h))
    return out


class JpegCoefs:
    """An entropy-decoded JPEG (mxd_jpeg_coefs_decode): the host half of the
    split decode; finish() runs the rest on the host, make_jpeg_images() hands
    it to the GPU finish.  device_entropy=True: mxd_jpeg_coefs_parse, the
    Huffman decode too is left to the GPU when the file qualifies
    (``entropy_pending``)."""

    def __init__(self, data, device_entropy=False, _handle=None):
        h = ctypes.c_void_p(_handle)
        if _handle is not None:
            pass
        elif device_entropy:
            buf = np.frombuffer(bytes(data), np.uint8) if not isinstance(data, np.ndarray) else np.ascontiguousarray(data)
            check(lib().mxd_jpeg_coefs_parse(buf.ctypes.data_as(ctypes.c_void_p), ctypes.c_size_t(buf.nbytes), 1,
                                             ctypes.byref(h)))
        else:
            buf = np.frombuffer(bytes(data), np.uint8) if not isinstance(data, np.ndarray) else np.ascontiguousarray(data)
            check(lib().mxd_jpeg_coefs_decode(buf.ctypes.data_as(ctypes.c_void_p), ctypes.c_size_t(buf.nbytes),
                                              ctypes.byref(h)))
        self.handle = h.value
        pend = ctypes.c_int32()
        check(lib().mxd_jpeg_coefs_entropy_pending(ctypes.c_void_p(self.handle), ctypes.byref(pend)))
        self.entropy_pending = bool(pend.value)
        w, hh, ok = ctypes.c_int32(), ctypes.c_int32(), ctypes.c_int32()
        check(lib().mxd_jpeg_coefs_info(ctypes.c_void_p(self.handle), ctypes.byref(w), ctypes.byref(hh),
                                        ctypes.byref(ok)))
        self.width, self.height, self.device_ok = w.value, hh.value, bool(ok.value)

    @classmethod
    def load(cls, path, device_entropy=True):
        """mxd_jpeg_coefs_load: the file at `path` read straight into the
        handle; None when it does not start with the JPEG signature."""
        h = ctypes.c_void_p()
        check(lib().mxd_jpeg_coefs_load(os.fsencode(path), 1 if device_entropy else 0, ctypes.byref(h)))
        return None if not h.value else cls(None, _handle=h.value)

    def finish(self):
        """Host finish: (H, W, 3) uint8, the bytes jpeg_decode gives."""
        out = np.empty((self.height, self.width, 3), np.uint8)
        check(lib().mxd_jpeg_coefs_finish(ctypes.c_void_p(self.handle), out.ctypes.data_as(ctypes.c_void_p),
                                          ctypes.c_int64(self.width * 3)))
        return out

    def close(self):
        if self.handle:
            lib().mxd_jpeg_coefs_free(ctypes.c_void_p(self.handle))
            self.handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def make_jpeg_images(entries):
    """entries: dicts with the mxd_jpeg_image fields (coefs: a JpegCoefs; the
    window defaults to the whole image) -> ctypes array."""
    entries = list(entries)
    arr = (MxdJpegImage * max(1, len(entries)))()
    for i, e in enumerate(entries):
        c = e["coefs"]
        e = dict(dict(win_x=0, win_y=0, win_w=c.width, win_h=c.height), **e)
        for k, v in e.items():
            setattr(arr[i], k, c.handle if k == "coefs" else v)
    return arr, len(entries)


def jpeg_resize_crop_host(images, n, out_dtype, device=0):
    check(lib().mxd_jpeg_resize_crop_host(images, n, out_dtype, device))


def jpeg_plane_sources(reset=False):
    """Images resized straight from their JPEG sample planes since the last
    reset (mxd_jpeg_plane_sources)."""
    c = ctypes.c_int64()
    check(lib().mxd_jpeg_plane_sources(ctypes.byref(c), 1 if reset else 0))
    return c.value


def narrow_returns(reset=False):
    """Images whose f32 results a host-ending call returned over the link as
    u8 and expanded on the host since the last reset (mxd_narrow_returns)."""
    c = ctypes.c_int64()
    check(lib().mxd_narrow_returns(ctypes.byref(c), 1 if reset else 0))
    return c.value


def host_stats(reset=False):
    """Host-side time split since the last reset (mxd_host_stats): a dict of
    host-path calls, images, wall / device-wait seconds, coefficient parses
    and their seconds (summed over threads)."""
    v = (ctypes.c_int64 * 6)()
    check(lib().mxd_host_stats(v, 1 if reset else 0))
    return {"calls": v[0], "images": v[1], "call_s": v[2] * 1e-9, "wait_s": v[3] * 1e-9,
            "parses": v[4], "parse_s": v[5] * 1e-9}


def device_stats(reset=False):
    """Device time of the host-path calls' chunks since the last reset
    (mxd_device_stats; counted while MXD_TUNE_DEVICE_TIMING is 1): a dict of
    timed chunks and their summed seconds from first kernel to last."""
    v = (ctypes.c_int64 * 2)()
    check(lib().mxd_device_stats(v, 1 if reset else 0))
    return {"chunks": v[0], "device_s": v[1] * 1e-9}


def jpeg_resize_crop_to_device(images, n, out_dtype, device=0):
    check(lib().mxd_jpeg_resize_crop_to_device(images, n, out_dtype, device))


def rotate_geometry(w, h, angle, crop=False):
    """(mx[6] float32, out_w, out_h) of core::image::rotate for a w x h image."""
    mx = np.zeros(6, np.float32)
    tw, th = ctypes.c_int64(), ctypes.c_int64()
    check(lib().mxd_rotate_geometry(ctypes.c_int64(w), ctypes.c_int64(h), ctypes.c_double(angle), int(bool(crop)),
                                    mx.ctypes.data_as(ctypes.POINTER(ctypes.c_float)), ctypes.byref(tw),
                                    ctypes.byref(th)))
    return mx, tw.value, th.value


def channel_reduction_preset(preset):
    p = np.zeros(4, np.float32)
    check(lib().mxd_channel_reduction_preset(preset.encode(), p.ctypes.data_as(ctypes.POINTER(ctypes.c_float))))
    return p


def make_pixmaps(entries):
    """entries: iterable of dicts with the mxd_pixmap fields -> ctypes array."""
    entries = list(entries)
    arr = (MxdPixmap * max(1, len(entries)))()
    for i, e in enumerate(entries):
        for k, v in e.items():
            if k == "params":
                for j, x in enumerate(v):
                    arr[i].params[j] = float(x)
            else:
                setattr(arr[i], k, v)
    return arr, len(entries)


def pixmap_batch(images, n, op, device=0, stream=None):
    check(lib().mxd_pixmap_batch(images, n, op, device, ctypes.c_void_p(stream)))


def pixmap_host(images, n, op, device=0):
    check(lib().mxd_pixmap_host(images, n, op, device))


class Stream:
    """A HIP stream owned through the C ABI (NULL = the device's null stream)."""

    def __init__(self, device=0):
        self.device = device
        h = ctypes.c_void_p()
        check(lib().mxd_stream_create(device, ctypes.byref(h)))
        self.handle = h.value

    def synchronize(self):
        check(lib().mxd_stream_synchronize(ctypes.c_void_p(self.handle)))

    def close(self):
        if self.handle:
            check(lib().mxd_stream_destroy(ctypes.c_void_p(self.handle)))
            self.handle = None


class Event:
    def __init__(self):
        h = ctypes.c_void_p()
        check(lib().mxd_event_create(ctypes.byref(h)))
        self.handle = h.value

    def record(self, stream):
        check(lib().mxd_event_record(ctypes.c_void_p(self.handle), ctypes.c_void_p(stream.handle if stream else None)))

    def synchronize(self):
        check(lib().mxd_event_synchronize(ctypes.c_void_p(self.handle)))

    def elapsed_ms(self, end):
        ms = ctypes.c_float()
        check(lib().mxd_event_elapsed_ms(ctypes.byref(ms), ctypes.c_void_p(self.handle), ctypes.c_void_p(end.handle)))
        return ms.value

    def close(self):
        if self.handle:
            check(lib().mxd_event_destroy(ctypes.c_void_p(self.handle)))
            self.handle = None


class DeviceBuffer:
    """Raw device allocation with numpy upload/download helpers."""

    def __init__(self, nbytes, device=0):
        self.device = device
        self.nbytes = int(nbytes)
        p = ctypes.c_void_p()
        check(lib().mxd_malloc_device(ctypes.byref(p), ctypes.c_size_t(max(1, self.nbytes)), device))
        self.ptr = p.value

    def upload(self, arr, offset=0, stream=None):
        arr = np.ascontiguousarray(arr)
        check(lib().mxd_memcpy_h2d_async(ctypes.c_void_p(self.ptr + offset), arr.ctypes.data_as(ctypes.c_void_p),
                                         ctypes.c_size_t(arr.nbytes), ctypes.c_void_p(stream.handle if stream else None)))
        if stream is not None:
            stream.synchronize()
        else:
            check(lib().mxd_stream_synchronize(ctypes.c_void_p(None)))

    def download(self, shape, dtype, offset=0, stream=None):
        out = np.empty(shape, dtype)
        check(lib().mxd_memcpy_d2h_async(out.ctypes.data_as(ctypes.c_void_p), ctypes.c_void_p(self.ptr + offset),
                                         ctypes.c_size_t(out.nbytes), ctypes.c_void_p(stream.handle if stream else None)))
        if stream is not None:
            stream.synchronize()
        else:
            check(lib().mxd_stream_synchronize(ctypes.c_void_p(None)))
        return out

    def memset(self, value, stream=None):
        check(lib().mxd_memset_async(ctypes.c_void_p(self.ptr), value, ctypes.c_size_t(self.nbytes),
                                     ctypes.c_void_p(stream.handle if stream else None)))

    def free(self):
        if self.ptr:
            check(lib().mxd_free_device(ctypes.c_void_p(self.ptr), self.device))
            self.ptr = None

    def __del__(self):
        try:
            self.free()
        except Exception:
            pass


def copy_bandwidth(nbytes=1 << 30, device=0, iters=20, policy=0):
    """Streaming copy rate in GB/s (read + written bytes); policy 0 default,
    1 nontemporal, 2 nontemporal + sc1 (mxd_copy_bandwidth_policy)."""
    g = ctypes.c_float()
    check(lib().mxd_copy_bandwidth_policy(ctypes.c_size_t(nbytes), device, iters, policy, ctypes.byref(g)))
    return g.value


def device_count():
    n = ctypes.c_int()
    rc = lib().mxd_device_count(ctypes.byref(n))
    return n.value if rc == MXD_OK else 0
