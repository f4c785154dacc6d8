"""The mlx.data operator surface for the image path, over the gfx950 kernels.

Same names, keyword arguments and error behaviour as mlx-data 0.2.0
(``python/src/wrap_dataset.h``, ``wrap_buffer.cpp``, ``wrap_stream.cpp``):

    dset = (buffer_from_vector(samples)
            .shuffle().to_stream()
            .load_image("image")
            .image_resize_smallest_side("image", 256)
            .image_center_crop("image", 224, 224)
            .batch(32)
            .key_transform("image", lambda x: x.astype("float32") / 255)
            .prefetch(8, 8))

The image ops only record geometry; ``batch`` runs the resize, crop and
mirror of the whole batch as one fused GPU launch and writes the stacked
(B, H, W, C) uint8 tensor.  ``image_to_float(key)`` before ``batch`` (this
build's one addition to the surface) replaces the trailing
``key_transform(..., lambda x: x.astype("float32") / 255)``: the same launch
then writes the float32 batch, bit-identical to that lambda.  With several
devices (``set_devices``) a batch of at least 64 images per device is split
into contiguous slices, one per device; smaller batches go whole to one
device, consecutive batches rotating over the devices.  ``batch(n, device=d)`` builds the image keys' batches in device
memory instead (``DeviceArray``: DLPack producer, ``numpy()`` copies back);
import torch before this package when torch consumes them, so both share one
HIP runtime.  Reading an unbatched image materialises it with its own launch.
There is no CPU resize: without a visible GPU the image ops raise.

``load_image`` decodes JPEG natively (``csrc/jpeg.cpp``, the reference's
libjpeg path, ``core/image/ImageJPEG.cpp``).  With a device visible it only
parses the markers of a sequential file and the batch launch runs the whole
decode on the GPU -- Huffman (``csrc/jpeghuff.hip``), IDCT, upsampling,
colour (``csrc/jpegdev.hip``) -- before resizing, with the same bytes;
progressive and other files are entropy-decoded on the host first.
``set_device_entropy(False)`` keeps the Huffman decode on the host for every
file, ``set_device_decode(False)`` decodes whole on the host.
Other formats go to a Pillow hook that follows the reference's stb_image
rules (``core/image/ImageSTBI.cpp``: 1/2/3 channels kept, 4 -> 3, 16-bit >> 8).
"""
import io

import numpy as np

from . import capi  # noqa: F401  (loads libmxd_amd.so before anything else binds a HIP runtime)
from . import _pipeline  # noqa: F401
from ._pipeline import (Buffer, DeviceArray, Stream, buffer_from_vector, device_decode, device_entropy, devices,
                        set_device_decode, set_device_entropy, set_devices, set_image_decoder, set_state)

__all__ = ["Buffer", "Stream", "DeviceArray", "buffer_from_vector", "set_state", "set_devices", "devices",
           "set_device_decode", "device_decode", "set_device_entropy", "device_entropy"]


def _decode(path, data, from_memory, info):
    """Non-JPEG images (the reference's stb_image fallback, core/image/ImageSTBI.cpp:14-58):
    channels = min(stbi channels, 3) -- grey 1, grey+alpha 2, RGB 3, RGBA -> RGB;
    16-bit samples are scaled to 8 bits with >> 8 (stbi__convert_16_to_8); 1-bit
    images are expanded to 0/255 grey."""
    from PIL import Image

    try:
        im = Image.open(io.BytesIO(data.tobytes()) if from_memory else path)
        if info:
            return np.array([im.width, im.height], dtype=np.int64)
        if im.mode in ("L", "RGB", "LA"):
            a = np.asarray(im)
        elif im.mode in ("I;16", "I;16B", "I;16L", "I"):
            a = (np.asarray(im).astype(np.int64) >> 8).clip(0, 255).astype(np.uint8)
        elif im.mode == "1":
            a = np.asarray(im.convert("L"))
        else:  # palette, RGBA, CMYK, ...
            a = np.asarray(im.convert("RGB"))
    except (OSError, ValueError, SyntaxError):
        return None
    if a.ndim == 2:
        a = a[:, :, None]
    return np.ascontiguousarray(a, dtype=np.uint8)


set_image_decoder(_decode)


def _add_if_variants(cls):
    """``<op>_if(cond, ...)``: the op when ``cond`` holds, else the dataset
    unchanged (``Dataset::*_if``, ``Dataset.cpp``)."""
    for name in ("key_transform", "load_image", "image_resize_smallest_side", "image_resize",
                 "image_center_crop", "image_random_crop", "image_random_h_flip", "image_random_area_crop",
                 "image_rotate", "image_channel_reduction", "image_to_float"):
        def op_if(self, cond, *args, _name=name, **kwargs):
            return getattr(self, _name)(*args, **kwargs) if cond else self

        op_if.__name__ = name + "_if"
        setattr(cls, name + "_if", op_if)


def _stream_iter(self):
    return self


def _stream_next(self):
    s = self.next()
    if not s:
        raise StopIteration
    return s


def _buffer_iter(self):
    for i in range(len(self)):
        yield self[i]


_add_if_variants(Buffer)
_add_if_variants(Stream)
Stream.__iter__ = _stream_iter
Stream.__next__ = _stream_next
Buffer.__iter__ = _buffer_iter

