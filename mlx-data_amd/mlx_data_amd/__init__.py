"""mlx_data_amd -- MI355X-native image resize/crop stage for the mlx-data pipeline.

The hot path (image_resize_smallest_side + image_center_crop, optional f32/255)
runs as hand-written gfx950 HIP kernels behind the C ABI in
include/mxd_amd.h (libmxd_amd.so, built in-tree).  ``capi`` binds that ABI;
``image`` exposes batched functional forms.
"""
from . import capi, image  # noqa: F401

__version__ = "0.1.0"
