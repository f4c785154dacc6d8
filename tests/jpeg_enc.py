"""A minimal baseline JPEG encoder with caller-chosen Huffman tables (test
infrastructure): Pillow / libjpeg-turbo always writes either the Annex K
tables or optimised ones, whose codes longer than 11 bits all lie in the top
1/64 of the 16-bit code space -- so no Pillow file reaches the device entropy
decoder's searching path (jpeghuff.hip Dec::step, HuffDev::search).  This
writes files whose tables put long codes far below that (DEEP_DC / DEEP_AC),
so the tests can decode them on the GPU and compare with the host decoder and
with Pillow.  Pixels go through a float DCT and a flat quantiser; the result
only has to be a valid JPEG (every decoder reads the same file)."""
import numpy as np

ZIGZAG = np.array([
    0, 1, 8, 16, 9, 2, 3, 10, 17, 24, 32, 25, 18, 11, 4, 5, 12, 19, 26, 33, 40, 48, 41, 34, 27, 20, 13, 6, 7, 14, 21,
    28, 35, 42, 49, 56, 57, 50, 43, 36, 29, 22, 15, 23, 30, 37, 44, 51, 58, 59, 52, 45, 38, 31, 39, 46, 53, 60, 61,
    54, 47, 55, 62, 63])

# DC categories 0..11: three 2-bit codes, one 3-bit code, the other eight
# 12-bit codes starting at 1110 0000 0000 (11-bit prefix 1792 < 2016).
DEEP_DC = ([0, 3, 1, 0, 0, 0, 0, 0, 0, 0, 0, 8, 0, 0, 0, 0], [0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11])
# AC: EOB / 0x01 / 0x02 at 2 bits, six 5-bit codes, the other 153 symbols at
# 12 bits starting at 1111 0000 0000 (11-bit prefix 1920 < 2016).
_AC_SHORT = [0x00, 0x01, 0x02, 0x03, 0x11, 0x04, 0x21, 0x05, 0xF0]
_AC_ALL = [0x00, 0xF0] + [(r << 4) | s for r in range(16) for s in range(1, 11)]
DEEP_AC = ([0, 3, 0, 0, 6, 0, 0, 0, 0, 0, 0, 153, 0, 0, 0, 0], _AC_SHORT + [v for v in _AC_ALL if v not in _AC_SHORT])


def first_long_prefix(counts):
    """The 11-bit prefix of the first code longer than 11 bits (2048: none) --
    the device decoder searches a table when it is below 2016."""
    code = 0
    for n in range(1, 17):
        if n > 11 and counts[n - 1]:
            return (code << (16 - n)) >> 5
        code = (code + counts[n - 1]) << 1
    return 2048


def _codes(table):
    counts, vals = table
    out, code, k = {}, 0, 0
    for n in range(1, 17):
        for _ in range(counts[n - 1]):
            out[vals[k]] = (code, n)
            code += 1
            k += 1
        code <<= 1
    return out


class _Bits:
    def __init__(self):
        self.out, self.acc, self.n = bytearray(), 0, 0

    def put(self, v, n):
        self.acc = (self.acc << n) | (v & ((1 << n) - 1))
        self.n += n
        while self.n >= 8:
            self.n -= 8
            b = (self.acc >> self.n) & 0xFF
            self.out.append(b)
            if b == 0xFF:
                self.out.append(0)
        self.acc &= (1 << self.n) - 1

    def flush(self):
        if self.n:
            self.put((1 << (8 - self.n)) - 1, 8 - self.n)


def _category(v):
    return int(abs(int(v))).bit_length()


def _dct_blocks(plane, q):
    """(rows, cols, 64) quantised coefficients in zigzag order."""
    h, w = plane.shape
    ph, pw = -(-h // 8) * 8, -(-w // 8) * 8
    p = np.pad(plane.astype(np.float64), ((0, ph - h), (0, pw - w)), mode="edge") - 128.0
    k = np.arange(8)
    c = np.cos((2 * k[None, :] + 1) * k[:, None] * np.pi / 16) * np.where(k == 0, np.sqrt(1 / 8), 0.5)[:, None]
    b = p.reshape(ph // 8, 8, pw // 8, 8).transpose(0, 2, 1, 3)
    f = np.einsum("ij,rcjk,lk->rcil", c, b, c)
    z = np.rint(f / q).astype(np.int64).reshape(ph // 8, pw // 8, 64)[:, :, ZIGZAG]
    return np.clip(z, -1023, 1023)


def encode(pixels, dc=DEEP_DC, ac=DEEP_AC, q=2, restart_mcus=0, coefs=None, adobe=None):
    """pixels: (H, W) or (H, W, 3) uint8 -> baseline JPEG bytes (4:4:4 when
    three components, which are written as given: Y, Cb, Cr).  q: the flat
    quantiser (int) or a 64-entry table in natural order.  coefs: the
    quantised blocks to write instead of the pixels' -- per component a
    (rows, cols, 64) zig-zag array (DC within +-2047 of its neighbour, AC
    within +-1023) -- pixels then only gives the frame size.  adobe: write an
    Adobe APP14 marker with this colour transform (0: RGB / CMYK as stored,
    1: YCbCr, 2: YCCK for four components)."""
    a = pixels if pixels.ndim == 3 else pixels[:, :, None]
    h, w, nc = a.shape
    qt = np.full(64, q, np.int64) if np.isscalar(q) else np.asarray(q, np.int64)
    planes = coefs if coefs is not None else [_dct_blocks(a[:, :, i], qt.reshape(8, 8)) for i in range(nc)]
    rows, cols = planes[0].shape[:2]
    dcc, acc = _codes(dc), _codes(ac)
    bits, pred = _Bits(), [0] * nc
    segs, mcu = [], 0
    for r in range(rows):
        for cidx in range(cols):
            if restart_mcus and mcu and mcu % restart_mcus == 0:
                bits.flush()
                segs.append(bytes(bits.out))
                bits, pred = _Bits(), [0] * nc
            for i in range(nc):
                z = planes[i][r, cidx]
                d = int(z[0]) - pred[i]
                pred[i] = int(z[0])
                s = _category(d)
                bits.put(*dcc[s])
                if s:
                    bits.put(d if d > 0 else d - 1, s)
                run = 0
                nz = np.flatnonzero(z[1:])
                last = nz[-1] + 1 if len(nz) else 0
                for k in range(1, last + 1):
                    v = int(z[k])
                    if v == 0:
                        run += 1
                        continue
                    while run > 15:
                        bits.put(*acc[0xF0])
                        run -= 16
                    s = _category(v)
                    bits.put(*acc[(run << 4) | s])
                    bits.put(v if v > 0 else v - 1, s)
                    run = 0
                if last < 63:
                    bits.put(*acc[0x00])
            mcu += 1
    bits.flush()
    segs.append(bytes(bits.out))

    def seg(marker, body):
        return bytes([0xFF, marker]) + (len(body) + 2).to_bytes(2, "big") + body

    out = bytearray(b"\xff\xd8")
    if adobe is not None:
        out += seg(0xEE, b"Adobe" + (100).to_bytes(2, "big") + bytes(4) + bytes([adobe]))
    out += seg(0xDB, bytes([0]) + bytes(qt[ZIGZAG].astype(np.uint8).tolist()))
    out += seg(0xC0, bytes([8]) + h.to_bytes(2, "big") + w.to_bytes(2, "big") + bytes([nc]) +
               b"".join(bytes([i + 1, 0x11, 0]) for i in range(nc)))
    out += seg(0xC4, bytes([0x00]) + bytes(dc[0]) + bytes(dc[1]) + bytes([0x10]) + bytes(ac[0]) + bytes(ac[1]))
    if restart_mcus:
        out += seg(0xDD, restart_mcus.to_bytes(2, "big"))
    out += seg(0xDA, bytes([nc]) + b"".join(bytes([i + 1, 0x00]) for i in range(nc)) + bytes([0, 63, 0]))
    for i, s in enumerate(segs):
        if i:
            out += bytes([0xFF, 0xD0 + (i - 1) % 8])
        out += s
    out += b"\xff\xd9"
    return bytes(out)


# Lossless difference categories 0..16, all 5-bit codes.
LOSSLESS_DC = ([0, 0, 0, 0, 17, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0], list(range(17)))


def encode_lossless(pixels, psv=1, pt=0, restart_rows=0, table=LOSSLESS_DC, markers=b""):
    """pixels: (H, W) or (H, W, 3) uint8 -> lossless Huffman-coded JPEG
    (SOF3, 8-bit, 1x1 sampling, one interleaved scan; T.81 H.1): predictor
    `psv` (1..7), point transform `pt`, a restart interval of `restart_rows`
    rows of MCUs, `markers` (e.g. an APP segment) after SOI."""
    a = pixels if pixels.ndim == 3 else pixels[:, :, None]
    h, w, nc = a.shape
    x = a.astype(np.int64) >> pt
    codes = _codes(table)
    segs, bits = [], _Bits()
    r0 = 0
    for r in range(h):
        if restart_rows and r and r % restart_rows == 0:
            bits.flush()
            segs.append(bytes(bits.out))
            bits, r0 = _Bits(), r
        for c in range(w):
            for i in range(nc):
                if r == r0:
                    px = (1 << (8 - pt - 1)) if c == 0 else x[r, c - 1, i]
                elif c == 0:
                    px = x[r - 1, c, i]
                else:
                    ra, rb, rc = x[r, c - 1, i], x[r - 1, c, i], x[r - 1, c - 1, i]
                    px = {1: ra, 2: rb, 3: rc, 4: ra + rb - rc, 5: ra + ((rb - rc) >> 1), 6: rb + ((ra - rc) >> 1),
                          7: (ra + rb) >> 1}[psv]
                d = (int(x[r, c, i]) - int(px)) & 0xFFFF
                d = d - 0x10000 if d >= 0x8000 else d
                s = 0 if d == 0 else 16 if d == -32768 else abs(d).bit_length()
                bits.put(*codes[s])
                if 0 < s < 16:
                    bits.put(d if d > 0 else d - 1, s)
    bits.flush()
    segs.append(bytes(bits.out))

    def seg(marker, body):
        return bytes([0xFF, marker]) + (len(body) + 2).to_bytes(2, "big") + body

    out = bytearray(b"\xff\xd8") + markers
    out += seg(0xC3, bytes([8]) + h.to_bytes(2, "big") + w.to_bytes(2, "big") + bytes([nc]) +
               b"".join(bytes([i + 1, 0x11, 0]) for i in range(nc)))
    out += seg(0xC4, bytes([0x00]) + bytes(table[0]) + bytes(table[1]))
    if restart_rows:
        out += seg(0xDD, (restart_rows * w).to_bytes(2, "big"))
    out += seg(0xDA, bytes([nc]) + b"".join(bytes([i + 1, 0x00]) for i in range(nc)) + bytes([psv, 0, pt]))
    for i, s in enumerate(segs):
        if i:
            out += bytes([0xFF, 0xD0 + (i - 1) % 8])
        out += s
    out += b"\xff\xd9"
    return bytes(out)
