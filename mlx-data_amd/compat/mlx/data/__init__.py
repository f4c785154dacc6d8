"""``import mlx.data`` compatibility package for the image path.

Put ``mlx-data_amd/compat`` (and ``mlx-data_amd``) on ``sys.path`` and scripts
written for mlx-data, e.g. ``benchmarks/comparative/caltech101/mlx_data.py``,
run unchanged on the MI355X implementation: ``mlx.data.buffer_from_vector``
returns a ``mlx_data_amd`` Buffer whose image ops run on the GPU.  Only the
image-path surface exists ("Out of scope").
"""
import numpy  # noqa: F401  (import numpy in the main thread first, as mlx.data does)

from mlx_data_amd.data import Buffer, Stream, buffer_from_vector  # noqa: F401

from . import core  # noqa: F401

__version__ = "0.2.0+mi355x"
