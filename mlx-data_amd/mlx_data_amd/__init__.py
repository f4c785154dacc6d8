"""mlx_data_amd -- MI355X-native image resize/crop stage for the mlx-data pipeline.

The hot path (image_resize_smallest_side + image_center_crop, optional f32/255)
runs as hand-written gfx950 HIP kernels behind the C ABI in
include/mxd_amd.h (libmxd_amd.so, built in-tree).  ``capi`` binds that ABI;
``image`` exposes batched functional forms.
"""
import os


def _raise_hw_queues():
    """Hardware queues per process for the HIP runtime (read once, when HIP
    initialises).  The pipeline's prefetch workers each launch on a stream of
    their own; with HIP's default of 4 queues their small device calls
    serialise: JPEG pipeline into device batches at 16 workers, C4 95-106 k ->
    138-142 k img/s and C1 122 k -> 152 k with 16 queues
    (profiles/r04/hwq_*.jsonl).

    A ``GPU_MAX_HW_QUEUES`` the environment already sets is the user's (or
    the machine's) choice and is left alone.  When it is unset, the package
    sets it to ``MXD_HW_QUEUES`` (default 16, at most 32; 0: leave HIP's
    default).  An explicit ``MXD_HW_QUEUES`` is the opt-in for raising an
    exported value; the change is then logged to stderr.  No effect when
    another library initialised HIP first."""
    explicit = "MXD_HW_QUEUES" in os.environ
    try:
        want = min(int(os.environ.get("MXD_HW_QUEUES", "16")), 32)
    except ValueError:
        raise ValueError("MXD_HW_QUEUES must be an integer") from None
    if want <= 0:
        return
    have = os.environ.get("GPU_MAX_HW_QUEUES")
    if have is None:
        os.environ["GPU_MAX_HW_QUEUES"] = str(want)
        return
    if not explicit:
        return  # the exported setting wins
    try:
        cur = int(have)
    except ValueError:
        cur = 0
    if cur < want:
        os.environ["GPU_MAX_HW_QUEUES"] = str(want)
        import sys

        print("mlx_data_amd: GPU_MAX_HW_QUEUES %s -> %d (MXD_HW_QUEUES)" % (have, want), file=sys.stderr)


_raise_hw_queues()

from . import capi, image  # noqa: E402,F401

__version__ = "0.1.0"
