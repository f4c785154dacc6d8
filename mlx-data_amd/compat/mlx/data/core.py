"""mlx.data.core for the image path: the RNG state (core/State.cpp:9-22)."""
from mlx_data_amd.data import set_state  # noqa: F401
