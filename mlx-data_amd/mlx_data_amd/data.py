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
(B, H, W, C) uint8 tensor.  Reading an unbatched image materialises it with
its own launch.  There is no CPU resize: without a visible GPU the image ops
raise.

``load_image`` decodes with Pillow (libjpeg-turbo) into host memory, following
the channel rules of ``core/image/ImageIO.cpp:10-33`` (JPEG -> 3 channels; other
formats keep 1/2/3 channels, 4 -> 3).
"""
import io

import numpy as np

from . import capi  # noqa: F401  (loads libmxd_amd.so before anything else binds a HIP runtime)
from . import _pipeline  # noqa: F401
from ._pipeline import Buffer, Stream, buffer_from_vector, devices, set_devices, set_image_decoder, set_state

__all__ = ["Buffer", "Stream", "buffer_from_vector", "set_state", "set_devices", "devices"]


def _decode(path, data, from_memory, info):
    from PIL import Image

    try:
        im = Image.open(io.BytesIO(data.tobytes()) if from_memory else path)
        if info:
            return np.array([im.width, im.height], dtype=np.int64)
        if im.format == "JPEG":
            im = im.convert("RGB")
        elif im.mode in ("L", "RGB"):
            pass
        elif im.mode == "LA":
            pass
        elif im.mode in ("I;16", "I", "F"):
            im = im.convert("L")
        else:
            im = im.convert("RGB")
        a = np.asarray(im)
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
                 "image_rotate", "image_channel_reduction"):
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

