"""TEST INFRASTRUCTURE ONLY -- never imported by the product path.

A third, independent statement of the resize arithmetic (SURVEY.md Appendix
A, items 1-7 and 10), written from that text alone in float64 numpy as dense
per-axis weight matrices.  It shares no code, no table layout and no
precision with the product tap builder (mlx-data_amd/csrc/taps.cpp) or the C
oracle (oracle/stbir_oracle.c): weights are evaluated in float64 at the exact
rational scale, out-of-range taps are folded onto the edge pixel by index
clamping (item 5), each row is renormalised to sum to 1 (item 6) and the
separable product is taken in float64 before the encode (item 7).

It exists to give the border behaviour (item 5, marked † in the survey)
evidence that does not come from the same recollection as the oracle:
tests/test_border_evidence.py compares it, and torch / Pillow run on
replicate-padded sources (a second, implementation-independent statement of
clamp folding), with the oracle on whole frames, borders included.

Call site being restated: /root/reference/mlx/data/core/image/ImageTransform.cpp:49-60
(stbir_resize_uint8_linear, STBIR_FILTER_TRIANGLE at :7-9, default
STBIR_EDGE_CLAMP)."""
import numpy as np
from scipy import sparse


def tent(x):
    """Appendix A item 2: k(x) = max(0, 1 - |x|)."""
    return np.maximum(0.0, 1.0 - np.abs(x))


def axis_matrix(n_in, n_out):
    """(n_out, n_in) float64 weights of one axis, clamp-folded and
    row-normalised (Appendix A items 3-6)."""
    s = n_out / n_in
    j = np.arange(n_out, dtype=np.float64)[:, None]
    if s >= 1.0:
        # item 3: c = (j + 0.5) / s; weight of n is k((n + 0.5) - c)
        centre = (j + 0.5) / s
        lo = np.floor(centre - 1.0).astype(np.int64) - 1
        span = 4
        n = lo + np.arange(span)[None, :]
        w = tent((n + 0.5) - centre)
    else:
        # item 4: weight of n is s * k((j + 0.5) - (n + 0.5) * s), support 1/s
        centre = (j + 0.5) / s
        radius = 1.0 / s
        lo = np.floor(centre - radius).astype(np.int64) - 1
        span = int(np.ceil(2 * radius)) + 4
        n = lo + np.arange(span)[None, :]
        w = s * tent((j + 0.5) - (n + 0.5) * s)
    # item 5: fold taps outside [0, n_in) onto the edge pixel
    idx = np.clip(n, 0, n_in - 1)
    m = np.zeros((n_out, n_in), np.float64)
    rows = np.broadcast_to(np.arange(n_out)[:, None], idx.shape)
    np.add.at(m, (rows, idx), w)
    # item 6: every output's weights sum to 1
    m /= m.sum(axis=1, keepdims=True)
    return m


def resize_float(img, dw, dh):
    """(dh, dw, C) float64 values in [0, 1] (before the encode)."""
    h, w, c = img.shape
    mx = axis_matrix(w, dw)
    my = axis_matrix(h, dh)
    # sparse products (the matrices are band-diagonal); exact float64 sums
    mx, my = sparse.csr_matrix(mx), sparse.csr_matrix(my)
    v = img.astype(np.float64) / 255.0  # item 7 decode
    t = (mx @ v.transpose(1, 0, 2).reshape(w, h * c)).reshape(dw, h, c)  # horizontal: (dw, H, C)
    t = t.transpose(1, 0, 2).reshape(h, dw * c)
    return (my @ t).reshape(dh, dw, c)  # vertical


def encode(v):
    """Appendix A item 7: trunc(clamp(255 v + 0.5, 0, 255))."""
    return np.trunc(np.clip(v * 255.0 + 0.5, 0, 255)).astype(np.uint8)


def resize(img, dw, dh):
    return encode(resize_float(img, dw, dh))
