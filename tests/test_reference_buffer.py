"""The reference's own Buffer tests (python/tests/test_buffer.py:12-67),
restated against this package's operator surface (`import mlx.data as dx`
resolves to mlx-data_amd/compat).  CPU only: no image ops."""
import array
import os
import sys

import numpy as np
import pytest

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "mlx-data_amd", "compat"))
import mlx.data as dx  # noqa: E402


def test_getitem():
    n = 5
    b = dx.buffer_from_vector(list(dict(i=i) for i in range(n)))
    for i in range(n):
        assert b[i]["i"] == i
        i += 1
        assert np.array_equal(b[-i]["i"], b[n - i]["i"])
    with pytest.raises(IndexError):
        _ = b[n]
    with pytest.raises(IndexError):
        _ = b[-(n + 1)]


@pytest.mark.parametrize("num_threads,prefetch_size,n", [(8, 16, 160), (4, 12, 6)])
def test_ordered_prefetch(num_threads, prefetch_size, n):
    buffer = dx.buffer_from_vector(list(dict(i=i) for i in range(n)))
    stream = buffer.ordered_prefetch(prefetch_size, num_threads)
    count = 0
    for i, e in enumerate(stream):
        assert i == e["i"]
        count += 1
    assert count == n


def test_passing_python_objects():
    with pytest.raises(ValueError):
        dx.buffer_from_vector([{"a": "hello"}])
    with pytest.raises(ValueError):
        dx.buffer_from_vector([{"a": object()}])
    x = array.array("f")
    x.append(10)
    x.append(-2.5)
    y = np.random.randn(10)
    b = dx.buffer_from_vector([{"a": 1, "b": 1.2, "c": b"Hello world", "d": y, "e": x}])
    assert -2.5 == b[0]["e"][1]
    assert 1 == b[0]["a"]
    assert np.all(y == b[0]["d"])
    assert np.all(x == b[0]["e"])
    # numpy inputs are taken without a copy ...
    y[0] = 0
    assert np.all(y == b[0]["d"])
    # ... and Python buffers by copy (python/tests/test_buffer.py:71-77)
    x[0] = 0
    assert 10 == b[0]["e"][0]


def test_non_contiguous_buffer_rejected():
    """wrap.cpp:27-41: a strided buffer is refused with the reference's message."""
    m = memoryview(np.arange(16, dtype=np.uint8).reshape(4, 4)[:, ::2])
    with pytest.raises(ValueError, match="Contiguous buffer expected"):
        dx.buffer_from_vector([{"a": m}])
