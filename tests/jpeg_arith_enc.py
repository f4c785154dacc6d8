"""A minimal arithmetic-coded JPEG encoder (test infrastructure): ITU-T T.81
Annex D's QM coder, Annex F.1.4's DC / AC statistical models (sequential,
SOF9) and Annex G.1.3's progressive procedures (SOF10: DC first / refine, AC
first / refine), so the host decoder's arithmetic path can be checked
against Pillow's libjpeg-turbo decode of the same files (nothing here writes
arithmetic-coded JPEGs otherwise).  Pixels go through jpeg_enc's float DCT
and flat quantiser, or the caller passes quantised blocks."""
import numpy as np

from jpeg_enc import ZIGZAG, _dct_blocks

# T.81 Table D.2: (Qe, next index after MPS, next index after LPS, switch MPS)
QE = [
    (0x5A1D, 1, 1, 1), (0x2586, 2, 14, 0), (0x1114, 3, 16, 0), (0x080B, 4, 18, 0), (0x03D8, 5, 20, 0),
    (0x01DA, 6, 23, 0), (0x00E5, 7, 25, 0), (0x006F, 8, 28, 0), (0x0036, 9, 30, 0), (0x001A, 10, 33, 0),
    (0x000D, 11, 35, 0), (0x0006, 12, 9, 0), (0x0003, 13, 10, 0), (0x0001, 13, 12, 0), (0x5A7F, 15, 15, 1),
    (0x3F25, 16, 36, 0), (0x2CF2, 17, 38, 0), (0x207C, 18, 39, 0), (0x17B9, 19, 40, 0), (0x1182, 20, 42, 0),
    (0x0CEF, 21, 43, 0), (0x09A1, 22, 45, 0), (0x072F, 23, 46, 0), (0x055C, 24, 48, 0), (0x0406, 25, 49, 0),
    (0x0303, 26, 51, 0), (0x0240, 27, 52, 0), (0x01B1, 28, 54, 0), (0x0144, 29, 56, 0), (0x00F5, 30, 57, 0),
    (0x00B7, 31, 59, 0), (0x008A, 32, 60, 0), (0x0068, 33, 62, 0), (0x004E, 34, 63, 0), (0x003B, 35, 32, 0),
    (0x002C, 9, 33, 0), (0x5AE1, 37, 37, 1), (0x484C, 38, 64, 0), (0x3A0D, 39, 65, 0), (0x2EF1, 40, 67, 0),
    (0x261F, 41, 68, 0), (0x1F33, 42, 69, 0), (0x19A8, 43, 70, 0), (0x1518, 44, 72, 0), (0x1177, 45, 73, 0),
    (0x0E74, 46, 74, 0), (0x0BFB, 47, 75, 0), (0x09F8, 48, 77, 0), (0x0861, 49, 78, 0), (0x0706, 50, 79, 0),
    (0x05CD, 51, 48, 0), (0x04DE, 52, 50, 0), (0x040F, 53, 50, 0), (0x0363, 54, 51, 0), (0x02D4, 55, 52, 0),
    (0x025C, 56, 53, 0), (0x01F8, 57, 54, 0), (0x01A4, 58, 55, 0), (0x0160, 59, 56, 0), (0x0125, 60, 57, 0),
    (0x00F6, 61, 58, 0), (0x00CB, 62, 59, 0), (0x00AB, 63, 61, 0), (0x008F, 32, 61, 0), (0x5B12, 65, 65, 1),
    (0x4D04, 66, 80, 0), (0x412C, 67, 81, 0), (0x37D8, 68, 82, 0), (0x2FE8, 69, 83, 0), (0x293C, 70, 84, 0),
    (0x2379, 71, 86, 0), (0x1EDF, 72, 87, 0), (0x1AA9, 73, 87, 0), (0x174E, 74, 72, 0), (0x1424, 75, 72, 0),
    (0x119C, 76, 74, 0), (0x0F6B, 77, 74, 0), (0x0D51, 78, 75, 0), (0x0BB6, 79, 77, 0), (0x0A40, 48, 77, 0),
    (0x5832, 81, 80, 1), (0x4D1C, 82, 88, 0), (0x438E, 83, 89, 0), (0x3BDD, 84, 90, 0), (0x34EE, 85, 91, 0),
    (0x2EAE, 86, 92, 0), (0x299A, 87, 93, 0), (0x2516, 71, 86, 0), (0x5570, 89, 88, 1), (0x4CA9, 90, 95, 0),
    (0x44D9, 91, 96, 0), (0x3E22, 92, 97, 0), (0x3824, 93, 99, 0), (0x32B4, 94, 99, 0), (0x2E17, 86, 93, 0),
    (0x56A8, 96, 95, 1), (0x4F46, 97, 101, 0), (0x47E5, 98, 102, 0), (0x41CF, 99, 103, 0), (0x3C3D, 100, 104, 0),
    (0x375E, 93, 99, 0), (0x5231, 102, 105, 0), (0x4C0F, 103, 106, 0), (0x4639, 104, 107, 0), (0x415E, 99, 103, 0),
    (0x5627, 106, 105, 1), (0x50E7, 107, 108, 0), (0x4B85, 103, 109, 0), (0x5597, 109, 110, 0), (0x504F, 107, 111, 0),
    (0x5A10, 111, 110, 1), (0x5522, 109, 112, 0), (0x59EB, 111, 112, 1),
    (0x5A1D, 113, 113, 0),  # 113: the fixed 0.5 estimate of the AC sign (Table F.5 SS)
]


class _QM:
    """T.81 D.1 encoder: C (code register with 3 spacer bits), A (interval),
    CT (shifts to the next output byte), carry propagation through stacked
    0xFF bytes, 0xFF 0x00 stuffing."""

    def __init__(self):
        self.out = bytearray()
        self.c, self.a, self.ct = 0, 0x10000, 11
        self.sc = self.zc = 0
        self.buffer = -1

    def _emit_pending(self, byte):
        self.out += b"\x00" * self.zc
        self.zc = 0
        self.out.append(byte)
        if byte == 0xFF:
            self.out.append(0)

    def _byte_out(self):
        temp = self.c >> 19
        if temp > 0xFF:  # carry into the buffered byte; stacked 0xFF bytes become 0x00
            if self.buffer >= 0:
                self._emit_pending(self.buffer + 1)
            self.zc += self.sc
            self.sc = 0
            self.buffer = temp & 0xFF
        elif temp == 0xFF:
            self.sc += 1
        else:
            if self.buffer == 0:
                self.zc += 1
            elif self.buffer >= 0:
                self._emit_pending(self.buffer)
            if self.sc:
                self.out += b"\x00" * self.zc
                self.zc = 0
                self.out += b"\xff\x00" * self.sc
                self.sc = 0
            self.buffer = temp & 0xFF
        self.c &= 0x7FFFF
        self.ct += 8

    def encode(self, stats, i, bit):
        sv = stats[i]
        qe, nmps, nlps, switch = QE[sv & 0x7F]
        mps = sv >> 7
        self.a -= qe
        if bit != mps:
            if self.a >= qe:  # the LPS takes the lower interval unless it is the larger one
                self.c += self.a
                self.a = qe
            stats[i] = ((mps ^ switch) << 7) | nlps
        else:
            if self.a >= 0x8000:
                return
            if self.a < qe:
                self.c += self.a
                self.a = qe
            stats[i] = (mps << 7) | nmps
        while True:
            self.a <<= 1
            self.c <<= 1
            self.ct -= 1
            if self.ct == 0:
                self._byte_out()
            if self.a >= 0x8000:
                break

    def flush(self):
        temp = (self.a - 1 + self.c) & 0xFFFF0000
        self.c = temp + 0x8000 if temp < self.c else temp
        self.c <<= self.ct
        if self.c & 0xF8000000:
            if self.buffer >= 0:
                self._emit_pending(self.buffer + 1)
            self.zc += self.sc
            self.sc = 0
        else:
            if self.buffer == 0:
                self.zc += 1
            elif self.buffer >= 0:
                self._emit_pending(self.buffer)
            if self.sc:
                self.out += b"\x00" * self.zc
                self.zc = 0
                self.out += b"\xff\x00" * self.sc
                self.sc = 0
        if self.c & 0x7FFF800:  # the final bytes, unless zero
            self._emit_pending((self.c >> 19) & 0xFF)
            if self.c & 0x7F800:
                b = (self.c >> 11) & 0xFF
                self.out.append(b)
                if b == 0xFF:
                    self.out.append(0)
        return bytes(self.out)


def _encode_block(qm, z, comp, dc_stats, ac_stats, fixed, L, U, K):
    """F.1.4.4: one block's DC difference and AC coefficients (z in zig-zag order)."""
    st = dc_stats
    s0 = comp["ctx"]
    v = int(z[0]) - comp["pred"]
    comp["pred"] = int(z[0])
    if v == 0:
        qm.encode(st, s0, 0)
        comp["ctx"] = 0
    else:
        qm.encode(st, s0, 1)
        if v > 0:
            qm.encode(st, s0 + 1, 0)
            i = s0 + 2
            comp["ctx"] = 4
        else:
            v = -v
            qm.encode(st, s0 + 1, 1)
            i = s0 + 3
            comp["ctx"] = 8
        m = 0
        v -= 1
        if v:
            qm.encode(st, i, 1)
            m = 1
            v2 = v
            i = 20
            v2 >>= 1
            while v2:
                qm.encode(st, i, 1)
                m <<= 1
                i += 1
                v2 >>= 1
        qm.encode(st, i, 0)
        if m < (1 << L) >> 1:
            comp["ctx"] = 0
        elif m > (1 << U) >> 1:
            comp["ctx"] += 8
        i += 14
        m >>= 1
        while m:
            qm.encode(st, i, 1 if (m & v) else 0)
            m >>= 1
    nz = np.flatnonzero(z[1:])
    ke = int(nz[-1]) + 1 if len(nz) else 0
    k = 1
    while k <= ke:
        i = 3 * (k - 1)
        qm.encode(ac_stats, i, 0)  # not EOB
        while int(z[k]) == 0:
            qm.encode(ac_stats, i + 1, 0)
            i += 3
            k += 1
        qm.encode(ac_stats, i + 1, 1)
        v = int(z[k])
        if v > 0:
            qm.encode(fixed, 0, 0)
        else:
            v = -v
            qm.encode(fixed, 0, 1)
        i += 2
        m = 0
        v -= 1
        if v:
            qm.encode(ac_stats, i, 1)
            m = 1
            v2 = v >> 1
            if v2:
                qm.encode(ac_stats, i, 1)
                m <<= 1
                i = 189 if k <= K else 217
                v2 >>= 1
                while v2:
                    qm.encode(ac_stats, i, 1)
                    m <<= 1
                    i += 1
                    v2 >>= 1
        qm.encode(ac_stats, i, 0)
        i += 14
        m >>= 1
        while m:
            qm.encode(ac_stats, i, 1 if (m & v) else 0)
            m >>= 1
        k += 1
    if k <= 63:
        qm.encode(ac_stats, 3 * (k - 1), 1)  # EOB


def encode(pixels, q=2, restart_mcus=0, coefs=None, dac=None):
    """pixels: (H, W) or (H, W, 3) uint8 -> sequential arithmetic-coded JPEG
    bytes (SOF9, 4:4:4 when three components, one DC / AC conditioning table
    set shared).  q: flat quantiser or a 64-entry natural-order table.
    coefs: per component (rows, cols, 64) zig-zag blocks instead of the
    pixels'.  dac: (L, U, K) conditioning written in a DAC segment (default
    none: L=0, U=1, K=5)."""
    a = pixels if pixels.ndim == 3 else pixels[:, :, None]
    h, w, nc = a.shape
    qt = np.full(64, q, np.int64) if np.isscalar(q) else np.asarray(q, np.int64)
    planes = coefs if coefs is not None else [_dct_blocks(a[:, :, i], qt.reshape(8, 8)) for i in range(nc)]
    rows, cols = planes[0].shape[:2]
    L, U, K = dac if dac is not None else (0, 1, 5)

    def fresh():
        return (bytearray(64), bytearray(256), bytearray([113]),
                [dict(pred=0, ctx=0) for _ in range(nc)], _QM())

    segs = []
    dc_stats, ac_stats, fixed, comps, qm = fresh()
    mcu = 0
    for r in range(rows):
        for c in range(cols):
            if restart_mcus and mcu and mcu % restart_mcus == 0:
                segs.append(qm.flush())
                dc_stats, ac_stats, fixed, comps, qm = fresh()
            for i in range(nc):
                _encode_block(qm, planes[i][r, c], comps[i], dc_stats, ac_stats, fixed, L, U, K)
            mcu += 1
    segs.append(qm.flush())

    def seg(marker, body):
        return bytes([0xFF, marker]) + (len(body) + 2).to_bytes(2, "big") + body

    out = bytearray(b"\xff\xd8")
    out += seg(0xDB, bytes([0]) + bytes(qt[ZIGZAG].astype(np.uint8).tolist()))
    out += seg(0xC9, bytes([8]) + h.to_bytes(2, "big") + w.to_bytes(2, "big") + bytes([nc]) +
               b"".join(bytes([i + 1, 0x11, 0]) for i in range(nc)))
    if dac is not None:
        out += seg(0xCC, bytes([0x00, (U << 4) | L, 0x10, K]))
    if restart_mcus:
        out += seg(0xDD, restart_mcus.to_bytes(2, "big"))
    out += seg(0xDA, bytes([nc]) + b"".join(bytes([i + 1, 0x00]) for i in range(nc)) + bytes([0, 63, 0]))
    for i, s in enumerate(segs):
        if i:
            out += bytes([0xFF, 0xD0 + (i - 1) % 8])
        out += s
    out += b"\xff\xd9"
    return bytes(out)


def _dc_first(qm, dc_val, comp, st, L, U):
    """F.1.4.4.1 on a (point-transformed) DC value."""
    s0 = comp["ctx"]
    v = dc_val - comp["pred"]
    comp["pred"] = dc_val
    if v == 0:
        qm.encode(st, s0, 0)
        comp["ctx"] = 0
        return
    qm.encode(st, s0, 1)
    if v > 0:
        qm.encode(st, s0 + 1, 0)
        i = s0 + 2
        comp["ctx"] = 4
    else:
        v = -v
        qm.encode(st, s0 + 1, 1)
        i = s0 + 3
        comp["ctx"] = 8
    m = 0
    v -= 1
    if v:
        qm.encode(st, i, 1)
        m = 1
        v2 = v >> 1
        i = 20
        while v2:
            qm.encode(st, i, 1)
            m <<= 1
            i += 1
            v2 >>= 1
    qm.encode(st, i, 0)
    if m < (1 << L) >> 1:
        comp["ctx"] = 0
    elif m > (1 << U) >> 1:
        comp["ctx"] += 8
    i += 14
    m >>= 1
    while m:
        qm.encode(st, i, 1 if (m & v) else 0)
        m >>= 1


def _shifted(v, al):
    """|v| >> al with v's sign (the point transform of an AC coefficient)."""
    return (v >> al) if v >= 0 else -((-v) >> al)


def _ac_first(qm, z, ss, se, al, st, fixed, K):
    """G.1.3.2: coefficients ss..se of zig-zag block z, point transform al."""
    ke = se
    while ke > 0 and _shifted(int(z[ke]), al) == 0:
        ke -= 1
    k = ss
    while k <= ke:
        i = 3 * (k - 1)
        qm.encode(st, i, 0)
        while True:
            v = _shifted(int(z[k]), al)
            if v:
                qm.encode(st, i + 1, 1)
                qm.encode(fixed, 0, 0 if v > 0 else 1)
                v = abs(v)
                break
            qm.encode(st, i + 1, 0)
            i += 3
            k += 1
        i += 2
        m = 0
        v -= 1
        if v:
            qm.encode(st, i, 1)
            m = 1
            v2 = v >> 1
            if v2:
                qm.encode(st, i, 1)
                m <<= 1
                i = 189 if k <= K else 217
                v2 >>= 1
                while v2:
                    qm.encode(st, i, 1)
                    m <<= 1
                    i += 1
                    v2 >>= 1
        qm.encode(st, i, 0)
        i += 14
        m >>= 1
        while m:
            qm.encode(st, i, 1 if (m & v) else 0)
            m >>= 1
        k += 1
    if k <= se:
        qm.encode(st, 3 * (k - 1), 1)


def _ac_refine(qm, z, ss, se, ah, al, st, fixed):
    """G.1.3.3: the next bit (al) of coefficients ss..se, earlier bits from ah up."""
    ke = se
    while ke > 0 and _shifted(int(z[ke]), al) == 0:
        ke -= 1
    kex = ke
    while kex > 0 and _shifted(int(z[kex]), ah) == 0:
        kex -= 1
    k = ss
    while k <= ke:
        i = 3 * (k - 1)
        if k > kex:
            qm.encode(st, i, 0)
        while True:
            v = _shifted(int(z[k]), al)
            if v:
                a = abs(v)
                if a >> 1:
                    qm.encode(st, i + 2, a & 1)
                else:
                    qm.encode(st, i + 1, 1)
                    qm.encode(fixed, 0, 0 if v > 0 else 1)
                break
            qm.encode(st, i + 1, 0)
            i += 3
            k += 1
        k += 1
    if k <= se:
        qm.encode(st, 3 * (k - 1), 1)


# A libjpeg-style progressive script: (components, Ss, Se, Ah, Al)
DEFAULT_SCRIPT = [("all", 0, 0, 0, 1), ("each", 1, 5, 0, 2), ("each", 6, 63, 0, 2), ("each", 1, 63, 2, 1),
                  ("all", 0, 0, 1, 0), ("each", 1, 63, 1, 0)]


def encode_progressive(pixels, q=2, restart_mcus=0, coefs=None, dac=None, script=None):
    """encode()'s frame as a progressive arithmetic-coded JPEG (SOF10) with
    `script` (DEFAULT_SCRIPT: DC first, two AC bands, AC refinement, DC
    refinement, AC refinement; "all" = one interleaved DC scan, "each" = one
    scan per component)."""
    a = pixels if pixels.ndim == 3 else pixels[:, :, None]
    h, w, nc = a.shape
    qt = np.full(64, q, np.int64) if np.isscalar(q) else np.asarray(q, np.int64)
    planes = coefs if coefs is not None else [_dct_blocks(a[:, :, i], qt.reshape(8, 8)) for i in range(nc)]
    rows, cols = planes[0].shape[:2]
    L, U, K = dac if dac is not None else (0, 1, 5)

    def seg(marker, body):
        return bytes([0xFF, marker]) + (len(body) + 2).to_bytes(2, "big") + body

    out = bytearray(b"\xff\xd8")
    out += seg(0xDB, bytes([0]) + bytes(qt[ZIGZAG].astype(np.uint8).tolist()))
    out += seg(0xCA, bytes([8]) + h.to_bytes(2, "big") + w.to_bytes(2, "big") + bytes([nc]) +
               b"".join(bytes([i + 1, 0x11, 0]) for i in range(nc)))
    if dac is not None:
        out += seg(0xCC, bytes([0x00, (U << 4) | L, 0x10, K]))
    if restart_mcus:
        out += seg(0xDD, restart_mcus.to_bytes(2, "big"))
    scans = []
    for comps, ss, se, ah, al in (script or DEFAULT_SCRIPT):
        if comps == "all" and ss == 0:
            scans.append((list(range(nc)), ss, se, ah, al))
        else:
            scans += [([c], ss, se, ah, al) for c in range(nc)]
    for cl, ss, se, ah, al in scans:
        out += seg(0xDA, bytes([len(cl)]) + b"".join(bytes([c + 1, 0x00]) for c in cl) + bytes([ss, se, (ah << 4) | al]))

        def fresh():
            return bytearray(64), bytearray(256), bytearray([113]), [dict(pred=0, ctx=0) for _ in range(nc)], _QM()

        dc_stats, ac_stats, fixed, cs, qm = fresh()
        segs = []
        units = [(r, c) for r in range(rows) for c in range(cols)]
        for n, (r, c) in enumerate(units):
            if restart_mcus and n and n % restart_mcus == 0:
                segs.append(qm.flush())
                dc_stats, ac_stats, fixed, cs, qm = fresh()
            for ci in cl:
                z = planes[ci][r, c]
                if ss == 0 and ah == 0:
                    _dc_first(qm, int(z[0]) >> al, cs[ci], dc_stats, L, U)
                elif ss == 0:
                    qm.encode(fixed, 0, (int(z[0]) >> al) & 1)
                elif ah == 0:
                    _ac_first(qm, z, ss, se, al, ac_stats, fixed, K)
                else:
                    _ac_refine(qm, z, ss, se, ah, al, ac_stats, fixed)
        segs.append(qm.flush())
        for i, sgm in enumerate(segs):
            if i:
                out += bytes([0xFF, 0xD0 + (i - 1) % 8])
            out += sgm
    out += b"\xff\xd9"
    return bytes(out)
