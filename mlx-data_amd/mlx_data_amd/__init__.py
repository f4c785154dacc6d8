"""mlx_data_amd -- MI355X-native image resize/crop stage for the mlx-data pipeline.

The hot path (image_resize_smallest_side + image_center_crop, optional f32/255)
runs as hand-written gfx950 HIP kernels behind the C ABI in
include/mxd_amd.h (libmxd_amd.so, built in-tree).  ``capi`` binds that ABI;
``image`` exposes batched functional forms.
"""
import os

# Hardware queues per process for the HIP runtime (read once, when HIP
# initialises; a value the user set wins).  The pipeline's prefetch workers
# each launch on a stream of their own, and with HIP's default of 4 queues
# their small device calls serialise: JPEG pipeline into device batches at 16
# workers, C4 106 k -> 138 k img/s and C1 122 k -> 152 k with 16 queues
# (profiles/r04/hwq_*.jsonl).  No effect when another
# library initialised HIP first.
os.environ.setdefault("GPU_MAX_HW_QUEUES", "16")

from . import capi, image  # noqa: E402,F401

__version__ = "0.1.0"
