import os
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (REPO, os.path.join(REPO, "oracle"), os.path.join(REPO, "mlx-data_amd")):
    if p not in sys.path:
        sys.path.insert(0, p)

# Bind the product library (and with it /opt/rocm's HIP runtime) before any
# test module imports torch, which bundles its own libamdhip64.so.7.
try:
    from mlx_data_amd import capi as _capi  # noqa: E402

    _capi.lib()
except ImportError:
    pass


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (run on the GPU box with -m gpu)")
