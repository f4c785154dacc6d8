// jpeg.cpp -- from-scratch JPEG decoder for load_image.
//
// The reference decodes with libjpeg(-turbo) defaults and always hands back
// H x W x 3 (core/image/ImageJPEG.cpp:99-146): 3 components -> RGB, 1 -> grey
// replicated, 4 -> the first three channels of libjpeg's CMYK output.  The
// libjpeg defaults that shape the pixels, restated here (file names are
// libjpeg-turbo's):
//   * entropy decoding: Huffman, baseline / extended sequential (SOF0, SOF1)
//     and progressive (SOF2) with successive approximation (jdhuff.c,
//     jdphuff.c), restart markers; after data runs out (a marker where entropy
//     bits were needed) the rest of the restart interval decodes as zeros
//     (uniform grey), as jdhuff.c does for "insufficient data";
//   * dequantize + inverse DCT: JDCT_ISLOW, 13-bit fixed point, two passes with
//     PASS1_BITS = 2 (jidctint.c), outputs clamped to 0..255 as libjpeg-turbo's
//     SIMD IDCTs do (range_limit below);
//   * block smoothing of progressive files whose scans leave low-frequency AC
//     coefficients inexact (jdcoefct.c decompress_smooth_data, on by default);
//   * chroma upsampling: "fancy" triangle upsampling h2v1 / h1v2 / h2v2
//     (jdsample.c) with edge columns special-cased and the rows above the
//     first / below the last real row replicated (jdmainct.c context rows);
//     plain replication for other integral factors;
//   * colour: YCbCr -> RGB with 16-bit fixed-point tables (jdcolor.c); YCCK ->
//     CMYK; colour space from JFIF / Adobe markers / component ids
//     (jdapimin.c default_decompress_parms).
// Arithmetic coding, 12-bit and lossless JPEGs are rejected (the reference's
// 8-bit libjpeg API rejects or does not produce them either).
#include "jpeg.h"

#include "jpeghuff.h"

#include <fcntl.h>
#include <sys/stat.h>
#include <unistd.h>

#include <immintrin.h>

#include <algorithm>
#include <cerrno>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <string>
#include <vector>

namespace mxd {
namespace jpeg {
namespace {

// Zig-zag -> natural order, with 16 extra entries so a corrupt run past 63
// lands on 63 (jutils.c jpeg_natural_order).
const int kNatural[80] = {0,  1,  8,  16, 9,  2,  3,  10, 17, 24, 32, 25, 18, 11, 4,  5,  12, 19, 26, 33,
                          40, 48, 41, 34, 27, 20, 13, 6,  7,  14, 21, 28, 35, 42, 49, 56, 57, 50, 43, 36,
                          29, 22, 15, 23, 30, 37, 44, 51, 58, 59, 52, 45, 38, 31, 39, 46, 53, 60, 61, 54,
                          47, 55, 62, 63, 63, 63, 63, 63, 63, 63, 63, 63, 63, 63, 63, 63, 63, 63, 63, 63};

struct Error {
  std::string msg;
};

[[noreturn]] void fail(const std::string& m) { throw Error{m}; }

// parse_coefs: the file is not one the device entropy decode covers.
struct NotDevice {};

std::string hex2(int v) {
  static const char* d = "0123456789abcdef";
  return std::string("0x") + d[(v >> 4) & 15] + d[v & 15];
}

// SOF markers other than 0xC0-0xC2 and 0xC9-0xCA (sequential / progressive
// arithmetic coding): lossless and hierarchical processes are not decoded
// here.
[[noreturn]] void unsupported_sof(int m) {
  fail("Unsupported JPEG process: SOF type " + hex2(m));
}

// ---------------------------------------------------------------- Huffman
constexpr int kLook = 9;

// AC fast path: for a kLook-bit lookahead whose code AND magnitude bits both
// fit in it, the decoded coefficient, its zero run and the bits to consume
// (stb_image's fast-AC idea).  run == kEob marks an end-of-block-class symbol
// (size 0, run != 15); len == 0: take the general path.
constexpr uint8_t kEob = 0xFF;
struct FastAC {
  int16_t val;
  uint8_t run;
  uint8_t len;
};

struct Huff {
  bool present = false;
  int nvals = 0;
  uint16_t look[1 << kLook];  // (length << 8) | symbol, 0 = longer code
  int32_t maxcode[18];
  int32_t valoffset[18];
  uint8_t vals[256];
  FastAC fac[1 << kLook];
};

// jdhuff.c jpeg_make_d_derived_tbl
void build_huff(Huff& h, const uint8_t* bits /* [17], bits[0] unused */, const uint8_t* vals, int nvals) {
  int32_t size[257], code[257];
  int p = 0;
  for (int l = 1; l <= 16; l++)
    for (int i = 0; i < bits[l]; i++) {
      if (p >= 256) fail("Bogus Huffman table definition");
      size[p++] = l;
    }
  size[p] = 0;
  const int n = p;
  if (n != nvals) fail("Bogus Huffman table definition");
  int32_t c = 0;
  int si = size[0];
  p = 0;
  while (size[p]) {
    while (size[p] == si) code[p++] = c++;
    if (c >= (1 << si)) fail("Bogus Huffman table definition");
    c <<= 1;
    si++;
  }
  p = 0;
  for (int l = 1; l <= 16; l++) {
    if (bits[l]) {
      h.valoffset[l] = p - code[p];
      p += bits[l];
      h.maxcode[l] = code[p - 1];
    } else {
      h.maxcode[l] = -1;
    }
  }
  h.maxcode[17] = 0xFFFFF;
  std::memset(h.look, 0, sizeof h.look);
  p = 0;
  for (int l = 1; l <= kLook; l++)
    for (int i = 1; i <= bits[l]; i++, p++) {
      const int lookbits = code[p] << (kLook - l);
      for (int ctr = 1 << (kLook - l); ctr > 0; ctr--) h.look[lookbits + ctr - 1] = (uint16_t)((l << 8) | vals[p]);
    }
  std::memcpy(h.vals, vals, n);
  h.nvals = n;
  for (int i = 0; i < (1 << kLook); i++) {
    FastAC f{0, 0, 0};
    if (const int e = h.look[i]) {
      const int l = e >> 8, rs = e & 0xff, r = rs >> 4, sz = rs & 15;
      if (sz == 0) {
        f = FastAC{0, (uint8_t)(r == 15 ? 15 : kEob), (uint8_t)l};
      } else if (l + sz <= kLook) {
        const int v = (i >> (kLook - l - sz)) & ((1 << sz) - 1);
        f = FastAC{(int16_t)(v < (1 << (sz - 1)) ? v - (1 << sz) + 1 : v), (uint8_t)r, (uint8_t)(l + sz)};
      }
    }
    h.fac[i] = f;
  }
  h.present = true;
}

// build_huff through a small per-thread cache keyed by the DHT's counts and
// values: files from one encoder carry the same tables, and deriving them is
// about half of a markers-only parse (mxd_jpeg_coefs_parse).
void cached_huff(Huff& h, const uint8_t* bits, const uint8_t* vals, int nvals) {
  struct Entry {
    uint8_t bits[17];
    uint8_t vals[256];
    int nvals = -1;
    Huff h;
  };
  constexpr int kEntries = 8;
  thread_local std::unique_ptr<Entry[]> cache;
  thread_local int next = 0;
  if (!cache) cache.reset(new Entry[kEntries]);
  for (int i = 0; i < kEntries; i++) {
    const Entry& e = cache[i];
    if (e.nvals == nvals && std::memcmp(e.bits + 1, bits + 1, 16) == 0 && std::memcmp(e.vals, vals, nvals) == 0) {
      h = e.h;
      return;
    }
  }
  build_huff(h, bits, vals, nvals);  // throws on a bogus table: nothing cached
  Entry& e = cache[next];
  next = (next + 1) % kEntries;
  std::memcpy(e.bits, bits, 17);
  std::memcpy(e.vals, vals, nvals);
  e.nvals = nvals;
  e.h = h;
}

inline int extend(int v, int s) { return v < (1 << (s - 1)) ? v - (1 << s) + 1 : v; }

// Entropy-coded segment reader: stops at a marker; bits needed past it are
// zeros and set `insufficient` (jdhuff.c jpeg_fill_bit_buffer).
struct Bits {
  const uint8_t* p = nullptr;
  const uint8_t* end = nullptr;
  uint64_t buf = 0;
  int cnt = 0;
  bool at_marker = false;
  bool insufficient = false;

  void fill() {
    // Fast path: the next 8 bytes hold no 0xFF (no stuffing, no marker).
    if (cnt <= 56 && !at_marker && end - p >= 8) {
      uint64_t w;
      std::memcpy(&w, p, 8);
      const uint64_t x = ~w;
      if (((x - 0x0101010101010101ull) & ~x & 0x8080808080808080ull) == 0) {
        const int k = (64 - cnt) >> 3;
        const uint64_t be = __builtin_bswap64(w);
        buf |= (be >> (64 - 8 * k)) << (64 - cnt - 8 * k);
        p += k;
        cnt += 8 * k;
        return;
      }
    }
    while (cnt <= 56) {
      if (at_marker || p >= end) return;
      const uint8_t b = *p;
      if (b == 0xFF) {
        if (p + 1 >= end) {
          at_marker = true;
          return;
        }
        const uint8_t b2 = p[1];
        if (b2 == 0x00) {
          p += 2;
        } else if (b2 == 0xFF) {
          p++;  // fill byte
          continue;
        } else {
          at_marker = true;
          return;
        }
      } else {
        p++;
      }
      buf |= (uint64_t)b << (56 - cnt);
      cnt += 8;
    }
  }
  int peek(int n) const { return (int)(buf >> (64 - n)); }
  void skip(int n) {
    buf <<= n;
    cnt -= n;
  }
  int get(int n) {
    if (n == 0) return 0;
    if (cnt < n) fill();
    const int v = peek(n);
    consume(n);
    return v;
  }
  // Consumes n bits; bits past the end of the segment are zeros and mark the
  // data insufficient (only when they are actually used).
  void consume(int n) {
    if (n > cnt) {
      insufficient = true;
      cnt = 64;
    }
    skip(n);
  }
  int decode(const Huff& h) {
    if (cnt < 16) fill();
    const int look = peek(kLook);
    const int e = h.look[look];
    if (e) {
      consume(e >> 8);
      return e & 0xff;
    }
    int l = kLook + 1;
    int32_t code = peek(l);
    while (code > h.maxcode[l]) {
      l++;
      if (l > 16) {
        // jdhuff.c jpeg_huff_decode: corrupt data, return a zero
        consume(16);
        return 0;
      }
      code = peek(l);
    }
    consume(l);
    return h.vals[(code + h.valoffset[l]) & 0xff];
  }
  // Codes longer than the lookahead (and short ones whose value bits did not
  // fit the AC fast table), on a bit buffer held by the caller.
  static int decode_slow(const Huff& h, uint64_t& b, int& n) {
    const int e = h.look[b >> (64 - kLook)];
    if (e) {
      b <<= e >> 8;
      n -= e >> 8;
      return e & 0xff;
    }
    int l = kLook + 1;
    int32_t code = (int32_t)(b >> (64 - l));
    while (code > h.maxcode[l]) {
      if (++l > 16) {
        // jdhuff.c jpeg_huff_decode: corrupt data, return a zero
        b <<= 16;
        n -= 16;
        return 0;
      }
      code = (int32_t)(b >> (64 - l));
    }
    b <<= l;
    n -= l;
    return h.vals[(code + h.valoffset[l]) & 0xff];
  }

  // One block of a sequential scan (DC difference + AC run/levels, into blk,
  // which the caller zeroed), with the bit buffer in registers: refilled to
  // >= 57 bits whenever fewer than 32 remain (a symbol and its value bits
  // take <= 27), 8 bytes at a time where they hold no 0xFF.  Bits past the
  // end of the segment are zeros and mark the data insufficient, as in
  // consume(); the flag is only read between MCUs.
  void block_seq(const Huff& hd, const Huff& ha, int& pred, int16_t* blk) {
    uint64_t b = buf;
    int n = cnt;
    auto refill = [&]() {
      if (!at_marker && end - p >= 8 && n >= 0) {
        uint64_t w;
        std::memcpy(&w, p, 8);
        const uint64_t x = ~w;
        if (((x - 0x0101010101010101ull) & ~x & 0x8080808080808080ull) == 0) {
          const int k = (64 - n) >> 3;
          b |= (__builtin_bswap64(w) >> (64 - 8 * k)) << (64 - n - 8 * k);
          p += k;
          n += 8 * k;
          return;
        }
      }
      if (n < 0) return;  // past the end: only zeros follow
      buf = b;
      cnt = n;
      fill();
      b = buf;
      n = cnt;
    };
    if (n < 32) refill();
    int s = decode_slow(hd, b, n);
    if (s) {
      const int v = (int)(b >> (64 - s));
      b <<= s;
      n -= s;
      s = extend(v, s);
    }
    pred += s;
    blk[0] = (int16_t)pred;
    for (int k = 1; k < 64; k++) {
      if (n < 32) refill();
      const FastAC f = ha.fac[b >> (64 - kLook)];
      if (f.len) {
        b <<= f.len;
        n -= f.len;
        if (f.run == kEob) break;
        k += f.run;
        blk[kNatural[k]] = f.val;
        continue;
      }
      const int rs = decode_slow(ha, b, n);
      const int r = rs >> 4, sz = rs & 15;
      if (sz) {
        k += r;
        const int v = (int)(b >> (64 - sz));
        b <<= sz;
        n -= sz;
        blk[kNatural[k]] = (int16_t)extend(v, sz);
      } else {
        if (r != 15) break;
        k += 15;
      }
    }
    if (n < 0) {
      insufficient = true;
      n = 0;
      b = 0;
    }
    buf = b;
    cnt = n;
  }

  // One block of a progressive AC refinement scan (jdphuff.c
  // decode_mcu_AC_refine: new coefficients of +-p1 / m1 placed after r
  // still-zero ones, a correction bit for every nonzero one passed, EOB runs
  // correcting the rest of the band) with the bit buffer in registers as in
  // block_seq: refilled to >= 57 bits whenever fewer than 32 remain (a symbol,
  // its sign and an EOB run's bits take <= 30), per correction bit when
  // empty.  Bits past the segment's end are zeros and mark the data
  // insufficient, as consume() does.
  void block_refine(const Huff& ha, int16_t* blk, int ss, int se, int p1, int m1, int& eobrun) {
    uint64_t b = buf;
    int n = cnt;
    auto refill = [&]() {
      if (!at_marker && end - p >= 8 && n >= 0) {
        uint64_t w;
        std::memcpy(&w, p, 8);
        const uint64_t x = ~w;
        if (((x - 0x0101010101010101ull) & ~x & 0x8080808080808080ull) == 0) {
          const int k = (64 - n) >> 3;
          b |= (__builtin_bswap64(w) >> (64 - 8 * k)) << (64 - n - 8 * k);
          p += k;
          n += 8 * k;
          return;
        }
      }
      if (n < 0) return;  // past the end: only zeros follow
      buf = b;
      cnt = n;
      fill();
      b = buf;
      n = cnt;
    };
    auto bit = [&]() {
      if (n < 1) refill();
      const int v = (int)(b >> 63);
      b <<= 1;
      n -= 1;
      return v;
    };
    auto fix = [&](int16_t& co) {
      if (bit() && (co & p1) == 0) co = (int16_t)(co >= 0 ? co + p1 : co + m1);
    };
    int k = ss;
    if (eobrun == 0) {
      for (; k <= se; k++) {
        if (n < 32) refill();
        const int rs = decode_slow(ha, b, n);
        int r = rs >> 4;
        int s = rs & 15;
        if (s) {
          s = (int)(b >> 63) ? p1 : m1;
          b <<= 1;
          n -= 1;
        } else if (r != 15) {
          eobrun = 1 << r;
          if (r) {
            eobrun += (int)(b >> (64 - r));
            b <<= r;
            n -= r;
          }
          break;
        }
        do {
          int16_t& co = blk[kNatural[k]];
          if (co != 0) {
            fix(co);
          } else {
            if (--r < 0) break;
          }
          k++;
        } while (k <= se);
        if (s) blk[kNatural[k]] = (int16_t)s;
      }
    }
    if (eobrun > 0) {
      for (; k <= se; k++) {
        int16_t& co = blk[kNatural[k]];
        if (co != 0) fix(co);
      }
      eobrun--;
    }
    if (n < 0) {
      insufficient = true;
      n = 0;
      b = 0;
    }
    buf = b;
    cnt = n;
  }

  // Next marker from p: p at its 0xFF, returns its code; 0xD9 (EOI) at the
  // end of the data, as libjpeg's sources insert a fake EOI there.
  int find_marker() {
    for (;;) {
      while (p < end && *p != 0xFF) p++;
      if (p + 1 >= end) {
        p = end;
        return 0xD9;
      }
      if (p[1] != 0x00 && p[1] != 0xFF) return p[1];
      p += p[1] == 0x00 ? 2 : 1;
    }
  }
  // End of a restart interval (jdhuff.c process_restart, jdmarker.c
  // read_restart_marker + jpeg_resync_to_restart): drop the buffered bits,
  // expect RST<expected>.  The wanted marker (or one too far off to place) is
  // consumed and the out-of-data flag cleared; one of the next two markers or
  // a non-RST marker is left in place (the next segment is empty, and the
  // flag stays as it was); an older RST or a non-marker is skipped.
  void restart(int expected) {
    buf = 0;
    cnt = 0;
    for (;;) {
      const int m = at_marker && p + 1 < end ? p[1] : find_marker();
      at_marker = true;
      int action;
      if (m < 0xC0) action = 2;
      else if (m < 0xD0 || m > 0xD7) action = 3;
      else if (m == 0xD0 + ((expected + 1) & 7) || m == 0xD0 + ((expected + 2) & 7)) action = 3;
      else if (m == 0xD0 + ((expected - 1) & 7) || m == 0xD0 + ((expected - 2) & 7)) action = 2;
      else action = 1;
      if (action == 1) {
        p += 2;
        at_marker = false;
        insufficient = false;
        return;
      }
      if (action == 3) return;
      p += 2;
      at_marker = false;
    }
  }
};


// ---------------------------------------------------------------- IDCT
// ---------------------------------------------------------------- arithmetic
// T.81 Table D.2 (Qe, next state after an MPS, after an LPS, MPS switch on
// an LPS) and a 114th state: Table F.5's fixed estimate for the AC sign.
struct QeState {
  uint16_t qe;
  uint8_t nmps, nlps, sw;
};
constexpr QeState kQe[114] = {
    {0x5A1D, 1, 1, 1},    {0x2586, 2, 14, 0},   {0x1114, 3, 16, 0},   {0x080B, 4, 18, 0},   {0x03D8, 5, 20, 0},
    {0x01DA, 6, 23, 0},   {0x00E5, 7, 25, 0},   {0x006F, 8, 28, 0},   {0x0036, 9, 30, 0},   {0x001A, 10, 33, 0},
    {0x000D, 11, 35, 0},  {0x0006, 12, 9, 0},   {0x0003, 13, 10, 0},  {0x0001, 13, 12, 0},  {0x5A7F, 15, 15, 1},
    {0x3F25, 16, 36, 0},  {0x2CF2, 17, 38, 0},  {0x207C, 18, 39, 0},  {0x17B9, 19, 40, 0},  {0x1182, 20, 42, 0},
    {0x0CEF, 21, 43, 0},  {0x09A1, 22, 45, 0},  {0x072F, 23, 46, 0},  {0x055C, 24, 48, 0},  {0x0406, 25, 49, 0},
    {0x0303, 26, 51, 0},  {0x0240, 27, 52, 0},  {0x01B1, 28, 54, 0},  {0x0144, 29, 56, 0},  {0x00F5, 30, 57, 0},
    {0x00B7, 31, 59, 0},  {0x008A, 32, 60, 0},  {0x0068, 33, 62, 0},  {0x004E, 34, 63, 0},  {0x003B, 35, 32, 0},
    {0x002C, 9, 33, 0},   {0x5AE1, 37, 37, 1},  {0x484C, 38, 64, 0},  {0x3A0D, 39, 65, 0},  {0x2EF1, 40, 67, 0},
    {0x261F, 41, 68, 0},  {0x1F33, 42, 69, 0},  {0x19A8, 43, 70, 0},  {0x1518, 44, 72, 0},  {0x1177, 45, 73, 0},
    {0x0E74, 46, 74, 0},  {0x0BFB, 47, 75, 0},  {0x09F8, 48, 77, 0},  {0x0861, 49, 78, 0},  {0x0706, 50, 79, 0},
    {0x05CD, 51, 48, 0},  {0x04DE, 52, 50, 0},  {0x040F, 53, 50, 0},  {0x0363, 54, 51, 0},  {0x02D4, 55, 52, 0},
    {0x025C, 56, 53, 0},  {0x01F8, 57, 54, 0},  {0x01A4, 58, 55, 0},  {0x0160, 59, 56, 0},  {0x0125, 60, 57, 0},
    {0x00F6, 61, 58, 0},  {0x00CB, 62, 59, 0},  {0x00AB, 63, 61, 0},  {0x008F, 32, 61, 0},  {0x5B12, 65, 65, 1},
    {0x4D04, 66, 80, 0},  {0x412C, 67, 81, 0},  {0x37D8, 68, 82, 0},  {0x2FE8, 69, 83, 0},  {0x293C, 70, 84, 0},
    {0x2379, 71, 86, 0},  {0x1EDF, 72, 87, 0},  {0x1AA9, 73, 87, 0},  {0x174E, 74, 72, 0},  {0x1424, 75, 72, 0},
    {0x119C, 76, 74, 0},  {0x0F6B, 77, 74, 0},  {0x0D51, 78, 75, 0},  {0x0BB6, 79, 77, 0},  {0x0A40, 48, 77, 0},
    {0x5832, 81, 80, 1},  {0x4D1C, 82, 88, 0},  {0x438E, 83, 89, 0},  {0x3BDD, 84, 90, 0},  {0x34EE, 85, 91, 0},
    {0x2EAE, 86, 92, 0},  {0x299A, 87, 93, 0},  {0x2516, 71, 86, 0},  {0x5570, 89, 88, 1},  {0x4CA9, 90, 95, 0},
    {0x44D9, 91, 96, 0},  {0x3E22, 92, 97, 0},  {0x3824, 93, 99, 0},  {0x32B4, 94, 99, 0},  {0x2E17, 86, 93, 0},
    {0x56A8, 96, 95, 1},  {0x4F46, 97, 101, 0}, {0x47E5, 98, 102, 0}, {0x41CF, 99, 103, 0}, {0x3C3D, 100, 104, 0},
    {0x375E, 93, 99, 0},  {0x5231, 102, 105, 0}, {0x4C0F, 103, 106, 0}, {0x4639, 104, 107, 0}, {0x415E, 99, 103, 0},
    {0x5627, 106, 105, 1}, {0x50E7, 107, 108, 0}, {0x4B85, 103, 109, 0}, {0x5597, 109, 110, 0}, {0x504F, 107, 111, 0},
    {0x5A10, 111, 110, 1}, {0x5522, 109, 112, 0}, {0x59EB, 111, 112, 1}, {0x5A1D, 113, 113, 0}};
constexpr uint8_t kFixedState = 113;

// The QM decoder (T.81 D.2: INITDEC, DECODE with its conditional exchanges,
// RENORMD, BYTEIN) over one scan's data.  A statistics bin is a byte: the MPS
// in bit 7, the state index below.  C holds the code bits aligned to A << CT;
// CT < 0 at a segment's start takes the first two bytes in.  At a marker (or
// the end of the data) the input is zeros from then on, as T.81 allows and
// jdarith.c does.  `failed`: a spectral or magnitude overflow in this
// interval (corrupt data) -- its remaining blocks are left zero.
struct Arith {
  const uint8_t* p = nullptr;
  const uint8_t* end = nullptr;
  bool at_marker = false;  // p at the 0xFF of the marker the data ran into
  uint64_t c = 0;
  uint32_t a = 0;
  int ct = -16;
  bool failed = false;
  uint8_t dc_stats[16][64], ac_stats[16][256];
  uint8_t fixed = kFixedState;

  int byte_in() {
    if (at_marker || p >= end) {
      at_marker = true;
      return 0;
    }
    const uint8_t b = *p;
    if (b != 0xFF) {
      p++;
      return b;
    }
    const uint8_t* q = p + 1;
    while (q < end && *q == 0xFF) q++;  // fill bytes
    if (q < end && *q == 0x00) {
      p = q + 1;
      return 0xFF;  // stuffed
    }
    p = q - 1;  // the marker's 0xFF
    at_marker = true;
    return 0;
  }
  void reset() {
    c = 0;
    a = 0;
    ct = -16;
    failed = false;
  }
  int decode(uint8_t& st) {
    while (a < 0x8000) {
      if (--ct < 0) {
        c = (c << 8) | (uint64_t)byte_in();
        ct += 8;
        if (ct < 0 && ++ct == 0) a = 0x8000;  // both initial bytes in: A = 0x10000 below
      }
      a <<= 1;
    }
    int sv = st;
    const QeState& q = kQe[sv & 0x7F];
    const uint8_t mps_next = (uint8_t)q.nmps, lps_next = (uint8_t)(q.nlps | (q.sw << 7));
    a -= q.qe;
    const uint64_t t = (uint64_t)a << ct;
    if (c >= t) {  // the lower sub-interval: the LPS, unless it is the larger one
      c -= t;
      if (a < q.qe) {
        st = (uint8_t)((sv & 0x80) ^ mps_next);
      } else {
        st = (uint8_t)((sv & 0x80) ^ lps_next);
        sv ^= 0x80;
      }
      a = q.qe;
    } else if (a < 0x8000) {  // the upper one, renormalising: the MPS, unless exchanged
      if (a < q.qe) {
        st = (uint8_t)((sv & 0x80) ^ lps_next);
        sv ^= 0x80;
      } else {
        st = (uint8_t)((sv & 0x80) ^ mps_next);
      }
    }
    return sv >> 7;
  }
  // The bins of the scan's tables to state 0 / MPS 0 (scan start, restart).
  void clear_stats(const int* dc_tbls, const int* ac_tbls, int n) {
    for (int i = 0; i < n; i++) {
      if (dc_tbls[i] >= 0) std::memset(dc_stats[dc_tbls[i]], 0, sizeof dc_stats[0]);
      if (ac_tbls[i] >= 0) std::memset(ac_stats[ac_tbls[i]], 0, sizeof ac_stats[0]);
    }
  }
  // End of a restart interval: the RST marker (Bits::restart's resync
  // rules), then a fresh coder.
  void restart(int expected) {
    Bits b;
    b.p = p;
    b.end = end;
    b.at_marker = at_marker;
    b.restart(expected);
    p = b.p;
    at_marker = b.at_marker;
    reset();
  }
  // Magnitude category and bits of a nonzero value (F.2.4.3, Figures F.23 /
  // F.24): the first decision in bin `first`, the next ones from `x2` on
  // (first + 0 again for AC: X1 = SP), the bits 14 bins past the last
  // category bin.  Returns |v| - 1 (*cat: its top bit, 0 for |v| = 1), or -1
  // on a magnitude overflow.
  int magnitude(uint8_t* stats, int first, int x2, bool ac, int* cat) {
    int i = first;
    int m = decode(stats[i]);
    if (m) {
      if (ac) {
        if (!decode(stats[i])) goto bits;
        m <<= 1;
      }
      i = x2;
      while (decode(stats[i])) {
        if ((m <<= 1) == 0x8000) return -1;
        i++;
      }
    }
  bits:
    *cat = m;
    int v = m;
    i += 14;
    while (m >>= 1)
      if (decode(stats[i])) v |= m;
    return v;
  }
};

constexpr int kConstBits = 13;
constexpr int kPass1Bits = 2;
constexpr int32_t FIX_0_298631336 = 2446, FIX_0_390180644 = 3196, FIX_0_541196100 = 4433, FIX_0_765366865 = 6270,
                  FIX_0_899976223 = 7373, FIX_1_175875602 = 9633, FIX_1_501321110 = 12299,
                  FIX_1_847759065 = 15137, FIX_1_961570560 = 16069, FIX_2_053119869 = 16819,
                  FIX_2_562915447 = 20995, FIX_3_072711026 = 25172;

using JLONG = int64_t;  // libjpeg-turbo's JLONG (long on LP64)

inline int32_t descale(JLONG x, int n) { return (int32_t)((x + ((JLONG)1 << (n - 1))) >> n); }

// Output range limit.  jidctint.c indexes jdmaster.c's post-IDCT table with
// (x & 1023) -- out-of-range values wrap past +-384 -- while libjpeg-turbo's
// SIMD IDCTs (the build Pillow ships; x86 AVX2 / ARM NEON builds of the
// reference's libjpeg-turbo) narrow with signed saturation, i.e. clamp.  The
// two agree on every value a well-formed file produces; they part on the
// blocks truncated or corrupt data and block smoothing can drive out of
// range, where the saturating form is what Pillow's decodes (the pinned
// fixtures) hold.
inline uint8_t range_limit(int32_t x) {
  x += 128;
  return (uint8_t)(x < 0 ? 0 : x > 255 ? 255 : x);
}

// jidctint.c jpeg_idct_islow: dequantize + 8x8 inverse DCT into out (stride).
void idct_islow(const int16_t* in, const uint16_t* q, uint8_t* out, int stride) {
  int32_t ws[64];  // (int) workspace of pass 1
  for (int c = 0; c < 8; c++) {
    const int16_t* ip = in + c;
    const uint16_t* qp = q + c;
    int32_t* wp = ws + c;
    if (ip[8] == 0 && ip[16] == 0 && ip[24] == 0 && ip[32] == 0 && ip[40] == 0 && ip[48] == 0 && ip[56] == 0) {
      const int32_t dc = (JLONG)ip[0] * qp[0] * (1 << kPass1Bits);
      for (int r = 0; r < 8; r++) wp[8 * r] = dc;
      continue;
    }
    JLONG z2 = (JLONG)ip[16] * qp[16], z3 = (JLONG)ip[48] * qp[48];
    JLONG z1 = (z2 + z3) * FIX_0_541196100;
    JLONG tmp2 = z1 + z3 * -FIX_1_847759065;
    JLONG tmp3 = z1 + z2 * FIX_0_765366865;
    z2 = (JLONG)ip[0] * qp[0];
    z3 = (JLONG)ip[32] * qp[32];
    JLONG tmp0 = (z2 + z3) * (1 << kConstBits);
    JLONG tmp1 = (z2 - z3) * (1 << kConstBits);
    const JLONG tmp10 = tmp0 + tmp3, tmp13 = tmp0 - tmp3, tmp11 = tmp1 + tmp2, tmp12 = tmp1 - tmp2;
    tmp0 = (JLONG)ip[56] * qp[56];
    tmp1 = (JLONG)ip[40] * qp[40];
    tmp2 = (JLONG)ip[24] * qp[24];
    tmp3 = (JLONG)ip[8] * qp[8];
    z1 = tmp0 + tmp3;
    z2 = tmp1 + tmp2;
    z3 = tmp0 + tmp2;
    JLONG z4 = tmp1 + tmp3;
    const JLONG z5 = (z3 + z4) * FIX_1_175875602;
    tmp0 *= FIX_0_298631336;
    tmp1 *= FIX_2_053119869;
    tmp2 *= FIX_3_072711026;
    tmp3 *= FIX_1_501321110;
    z1 *= -FIX_0_899976223;
    z2 *= -FIX_2_562915447;
    z3 *= -FIX_1_961570560;
    z4 *= -FIX_0_390180644;
    z3 += z5;
    z4 += z5;
    tmp0 += z1 + z3;
    tmp1 += z2 + z4;
    tmp2 += z2 + z3;
    tmp3 += z1 + z4;
    constexpr int s = kConstBits - kPass1Bits;
    wp[0] = descale(tmp10 + tmp3, s);
    wp[56] = descale(tmp10 - tmp3, s);
    wp[8] = descale(tmp11 + tmp2, s);
    wp[48] = descale(tmp11 - tmp2, s);
    wp[16] = descale(tmp12 + tmp1, s);
    wp[40] = descale(tmp12 - tmp1, s);
    wp[24] = descale(tmp13 + tmp0, s);
    wp[32] = descale(tmp13 - tmp0, s);
  }
  for (int r = 0; r < 8; r++) {
    const int32_t* wp = ws + 8 * r;
    uint8_t* op = out + (size_t)r * stride;
    if (wp[1] == 0 && wp[2] == 0 && wp[3] == 0 && wp[4] == 0 && wp[5] == 0 && wp[6] == 0 && wp[7] == 0) {
      const uint8_t v = range_limit(descale(wp[0], kPass1Bits + 3));
      for (int c = 0; c < 8; c++) op[c] = v;
      continue;
    }
    JLONG z2 = wp[2], z3 = wp[6];
    JLONG z1 = (z2 + z3) * FIX_0_541196100;
    JLONG tmp2 = z1 + z3 * -FIX_1_847759065;
    JLONG tmp3 = z1 + z2 * FIX_0_765366865;
    JLONG tmp0 = ((JLONG)wp[0] + wp[4]) * (1 << kConstBits);
    JLONG tmp1 = ((JLONG)wp[0] - wp[4]) * (1 << kConstBits);
    const JLONG tmp10 = tmp0 + tmp3, tmp13 = tmp0 - tmp3, tmp11 = tmp1 + tmp2, tmp12 = tmp1 - tmp2;
    tmp0 = wp[7];
    tmp1 = wp[5];
    tmp2 = wp[3];
    tmp3 = wp[1];
    z1 = tmp0 + tmp3;
    z2 = tmp1 + tmp2;
    z3 = tmp0 + tmp2;
    JLONG z4 = tmp1 + tmp3;
    const JLONG z5 = (z3 + z4) * FIX_1_175875602;
    tmp0 *= FIX_0_298631336;
    tmp1 *= FIX_2_053119869;
    tmp2 *= FIX_3_072711026;
    tmp3 *= FIX_1_501321110;
    z1 *= -FIX_0_899976223;
    z2 *= -FIX_2_562915447;
    z3 *= -FIX_1_961570560;
    z4 *= -FIX_0_390180644;
    z3 += z5;
    z4 += z5;
    tmp0 += z1 + z3;
    tmp1 += z2 + z4;
    tmp2 += z2 + z3;
    tmp3 += z1 + z4;
    constexpr int s = kConstBits + kPass1Bits + 3;
    op[0] = range_limit(descale(tmp10 + tmp3, s));
    op[7] = range_limit(descale(tmp10 - tmp3, s));
    op[1] = range_limit(descale(tmp11 + tmp2, s));
    op[6] = range_limit(descale(tmp11 - tmp2, s));
    op[2] = range_limit(descale(tmp12 + tmp1, s));
    op[5] = range_limit(descale(tmp12 - tmp1, s));
    op[3] = range_limit(descale(tmp13 + tmp0, s));
    op[4] = range_limit(descale(tmp13 - tmp0, s));
  }
}

// The same transform in 32-bit lanes, vectorised across the 8 columns (pass
// 1) and, after a transpose, the 8 rows (pass 2).  Exact whenever no
// intermediate leaves int32: the dequantised inputs and the pass-1 outputs
// are checked below 2^14 in magnitude (every product then stays below 2^31),
// otherwise the block goes to idct_islow.  The post-IDCT range table is
// applied as its arithmetic equivalent: wrap to 10 bits, +128, clamp.
template <int S>
inline void idct_1d8(const int32_t* in, int32_t* out) {
  // in[k * 8 + l], out[k * 8 + l]: lane l, coefficient / sample k
  for (int l = 0; l < 8; l++) {
    const int32_t z2a = in[16 + l], z3a = in[48 + l];
    const int32_t z1a = (z2a + z3a) * FIX_0_541196100;
    const int32_t t2 = z1a + z3a * -FIX_1_847759065;
    const int32_t t3 = z1a + z2a * FIX_0_765366865;
    const int32_t t0 = (in[l] + in[32 + l]) * (1 << kConstBits);
    const int32_t t1 = (in[l] - in[32 + l]) * (1 << kConstBits);
    const int32_t t10 = t0 + t3, t13 = t0 - t3, t11 = t1 + t2, t12 = t1 - t2;
    int32_t o0 = in[56 + l], o1 = in[40 + l], o2 = in[24 + l], o3 = in[8 + l];
    int32_t z1 = o0 + o3, z2 = o1 + o2, z3 = o0 + o2, z4 = o1 + o3;
    const int32_t z5 = (z3 + z4) * FIX_1_175875602;
    o0 *= FIX_0_298631336;
    o1 *= FIX_2_053119869;
    o2 *= FIX_3_072711026;
    o3 *= FIX_1_501321110;
    z1 *= -FIX_0_899976223;
    z2 *= -FIX_2_562915447;
    z3 = z3 * -FIX_1_961570560 + z5;
    z4 = z4 * -FIX_0_390180644 + z5;
    o0 += z1 + z3;
    o1 += z2 + z4;
    o2 += z2 + z3;
    o3 += z1 + z4;
    constexpr int32_t r = 1 << (S - 1);
    out[l] = (t10 + o3 + r) >> S;
    out[56 + l] = (t10 - o3 + r) >> S;
    out[8 + l] = (t11 + o2 + r) >> S;
    out[48 + l] = (t11 - o2 + r) >> S;
    out[16 + l] = (t12 + o1 + r) >> S;
    out[40 + l] = (t12 - o1 + r) >> S;
    out[24 + l] = (t13 + o0 + r) >> S;
    out[32 + l] = (t13 - o0 + r) >> S;
  }
}

__attribute__((target_clones("avx2", "default"))) bool idct_islow32(const int16_t* in, const uint16_t* q,
                                                                    uint8_t* out, int stride) {
  int32_t d[64], ws[64], wt[64], o[64];
  int32_t m = 0;
  for (int i = 0; i < 64; i++) {
    d[i] = (int32_t)in[i] * (int32_t)q[i];
    m |= d[i] >= 0 ? d[i] : -d[i];
  }
  if (m >= (1 << 14)) return false;
  idct_1d8<kConstBits - kPass1Bits>(d, ws);  // ws[k * 8 + c]: row k of column c
  m = 0;
  for (int i = 0; i < 64; i++) m |= ws[i] >= 0 ? ws[i] : -ws[i];
  if (m >= (1 << 14)) return false;
  for (int r = 0; r < 8; r++)
    for (int c = 0; c < 8; c++) wt[c * 8 + r] = ws[r * 8 + c];
  idct_1d8<kConstBits + kPass1Bits + 3>(wt, o);  // o[c * 8 + r]: column c of row r
  for (int i = 0; i < 64; i++) {
    const int32_t v = o[i] + 128;
    o[i] = v < 0 ? 0 : v > 255 ? 255 : v;
  }
  for (int r = 0; r < 8; r++)
    for (int c = 0; c < 8; c++) out[(size_t)r * stride + c] = (uint8_t)o[c * 8 + r];
  return true;
}

inline void idct_block(const int16_t* in, const uint16_t* q, uint8_t* out, int stride) {
  if (!idct_islow32(in, q, out, stride)) idct_islow(in, q, out, stride);
}

// ---------------------------------------------------------------- colour
// jdsample.c h2v2_fancy_upsample for one output row from its two input rows
// (in0 nearer): column sums first, then the 3:1 horizontal blend -- the same
// integer formula, laid out without a loop-carried dependency.
__attribute__((target_clones("avx2", "default"))) void h2v2_fancy_row(const uint8_t* in0, const uint8_t* in1,
                                                                      int dw, uint8_t* t, int16_t* cs) {
  for (int x = 0; x < dw; x++) cs[x] = (int16_t)(in0[x] * 3 + in1[x]);
  t[0] = (uint8_t)((cs[0] * 4 + 8) >> 4);
  t[1] = (uint8_t)((cs[0] * 3 + cs[1] + 7) >> 4);
  for (int x = 1; x < dw - 1; x++) {
    t[2 * x] = (uint8_t)((cs[x] * 3 + cs[x - 1] + 8) >> 4);
    t[2 * x + 1] = (uint8_t)((cs[x] * 3 + cs[x + 1] + 7) >> 4);
  }
  t[2 * dw - 2] = (uint8_t)((cs[dw - 1] * 3 + cs[dw - 2] + 8) >> 4);
  t[2 * dw - 1] = (uint8_t)((cs[dw - 1] * 4 + 7) >> 4);
}

// jdcolor.c ycc_rgb_convert for one row, in the integer arithmetic its tables
// hold (FIX(x) = round(x * 2^16); Cr->R and Cb->B rounded by ONE_HALF, the G
// term shifted after summing), so it vectorises; YCCK -> CMYK inverts.
constexpr int32_t kFixCrR = 91881, kFixCbB = 116130, kFixCrG = 46802, kFixCbG = 22554, kHalf16 = 1 << 15;

__attribute__((target_clones("avx2", "default"))) void ycc_rgb_row(const uint8_t* Y, const uint8_t* Cb,
                                                                   const uint8_t* Cr, uint8_t* o, int W,
                                                                   bool invert) {
  for (int x = 0; x < W; x++) {
    const int32_t y = Y[x], cb = Cb[x] - 128, cr = Cr[x] - 128;
    int32_t r = y + ((kFixCrR * cr + kHalf16) >> 16);
    int32_t g = y + ((-kFixCbG * cb + kHalf16 - kFixCrG * cr) >> 16);
    int32_t b = y + ((kFixCbB * cb + kHalf16) >> 16);
    r = r < 0 ? 0 : r > 255 ? 255 : r;
    g = g < 0 ? 0 : g > 255 ? 255 : g;
    b = b < 0 ? 0 : b > 255 ? 255 : b;
    if (invert) {
      r = 255 - r;
      g = 255 - g;
      b = 255 - b;
    }
    o[3 * x] = (uint8_t)r;
    o[3 * x + 1] = (uint8_t)g;
    o[3 * x + 2] = (uint8_t)b;
  }
}


// ---------------------------------------------------------------- byte scans
// Entropy-coded data's 0xFF bytes, classified by the byte after each (T.81
// B.1.1.5): 0xFF 0x00 is a stuffed 0xFF (the 0x00 dropped), 0xFF 0xFF a fill
// byte (the first dropped), anything else a marker.  The marker parse counts
// the dropped bytes up to each marker and unstuff() removes them: both ran a
// memchr per 0xFF (one about every 160 bytes), ~6 us per 80 KB file each on
// the GPU boxes' EPYC 9575F.  With AVX-512 (BW + VBMI2, checked at run time)
// 64 bytes go at a time with mask arithmetic and a byte compress, branching
// only at a marker.

// The first marker at or after p (size when none before the end), adding to
// *dropped the bytes dropped before it.
size_t scan_to_marker_scalar(const uint8_t* data, size_t p, size_t size, int64_t* dropped) {
  for (;;) {
    const uint8_t* f = static_cast<const uint8_t*>(std::memchr(data + p, 0xFF, size - p));
    if (!f || (size_t)(f - data) + 1 >= size) return size;
    p = (size_t)(f - data);
    const uint8_t m = data[p + 1];
    if (m != 0x00 && m != 0xFF) return p;
    ++*dropped;
    p += m == 0x00 ? 2 : 1;
  }
}

__attribute__((target("avx512f,avx512bw,avx512vbmi2,popcnt,bmi")))
size_t scan_to_marker_avx512(const uint8_t* data, size_t p, size_t size, int64_t* dropped) {
  const __m512i ff = _mm512_set1_epi8((char)0xFF), zero = _mm512_setzero_si512();
  int64_t d = 0;
  for (; p + 65 <= size; p += 64) {
    const __m512i x = _mm512_loadu_si512(data + p), y = _mm512_loadu_si512(data + p + 1);
    const uint64_t isff = _mm512_cmpeq_epi8_mask(x, ff);
    const uint64_t drops = isff & (_mm512_cmpeq_epi8_mask(y, zero) | _mm512_cmpeq_epi8_mask(y, ff));
    if (const uint64_t marks = isff & ~drops) {
      const int j = __builtin_ctzll(marks);
      *dropped += d + __builtin_popcountll(drops & ((1ull << j) - 1));
      return p + (size_t)j;
    }
    d += __builtin_popcountll(drops);
  }
  *dropped += d;
  return scan_to_marker_scalar(data, p, size, dropped);
}

bool have_avx512_bytes() {  // (MXD_NO_AVX512=1: the scalar forms, for A/Bs)
  static const bool ok = __builtin_cpu_supports("avx512bw") && __builtin_cpu_supports("avx512vbmi2") &&
                         !(std::getenv("MXD_NO_AVX512") && std::atoi(std::getenv("MXD_NO_AVX512")) == 1);
  return ok;
}

size_t scan_to_marker(const uint8_t* data, size_t p, size_t size, int64_t* dropped) {
  return have_avx512_bytes() ? scan_to_marker_avx512(data, p, size, dropped)
                             : scan_to_marker_scalar(data, p, size, dropped);
}

// ---------------------------------------------------------------- decoder
struct Component {
  int id = 0, h = 1, v = 1, tq = 0;
  int dc_tbl = 0, ac_tbl = 0;
  int dw = 0, dh = 0;          // downsampled width / height (samples)
  int bw = 0, bh = 0;          // blocks per row / column in the MCU-padded grid
  int wib = 0, hib = 0;        // width / height in blocks of the component proper
  int64_t off = 0;             // first coefficient in Decoder::coefbuf (progressive / deferred IDCT)
  std::vector<uint8_t> plane;  // bw*8 x bh*8 samples (sequential, IDCT at once)
  int dc_pred = 0;
  bool coded = false;          // a scan carried it (sequential: else its samples stay 0)
  uint16_t q[64];              // quantisation table latched for it
};

struct Decoder {
  const uint8_t* data;
  size_t size;
  size_t pos = 0;
  int width = 0, height = 0, ncomp = 0;
  bool progressive = false, baseline_seen = false;
  bool arith = false;     // arithmetic-coded frame (SOF9 / SOF10)
  bool lossless = false;  // lossless Huffman-coded frame (SOF3): samples, no DCT
  // DAC conditioning (T.81 F.1.4.4.1.4 / F.1.4.4.2.1), defaults L = 0, U = 1, Kx = 5
  uint8_t arith_dc_l[16], arith_dc_u[16], arith_ac_k[16];
  bool jfif = false, adobe = false;
  int adobe_transform = -1;
  int restart_interval = 0;
  int max_h = 1, max_v = 1, mcux = 0, mcuy = 0;
  uint16_t qt[4][64];
  bool qt_present[4] = {false, false, false, false};
  Huff dc[4], ac[4];
  Component comp[4];
  bool frame = false, any_scan = false;
  int eobrun = 0;
  // defer: keep the coefficients of sequential scans too (decode_coefs) and
  // run no IDCT while parsing.
  bool defer = false;
  // device_entropy (parse_coefs): the first sequential scan is not decoded
  // but its entropy-coded segments recorded (pending); a file the device
  // decode does not cover throws NotDevice and is decoded on the host.
  bool device_entropy = false;
  bool pending = false;
  int scans = 0;
  bool eoi = false;
  std::vector<int64_t> seg_begin, seg_end;
  std::vector<int64_t> seg_bytes;  // unstuffed bytes of each segment (what unstuff() writes)
  int scan_ns = 0;
  int scan_comp[4] = {0, 0, 0, 0};  // frame index of each scan component (SOS order)
  int64_t scan_mcus = 0;
  std::vector<int16_t> coefbuf;  // every component's bw*bh blocks of 64, natural order
  int64_t coef_total = 0;        // its size (also while the entropy decode is pending)
  // Progression status of the first 10 zigzag coefficients (jdphuff.c
  // start_pass_phuff_decoder's coef_bits): [ci] the Al of the component's
  // latest scan of each (-1: none yet), [4 + ci] the values before that scan.
  int coef_bits[8][10];
  int input_scans = 0;
  // iMCU row of the last MCU that started with data left (jdcoefct.c
  // consume_data's last_good_iMCU_row): rows past it use the progression
  // status from before the last scan when smoothing
  int64_t last_good_imcu = INT64_MAX;

  int16_t* cblk(const Component& c, int bx, int by) {
    return coefbuf.data() + c.off + ((int64_t)by * c.bw + bx) * 64;
  }

  Decoder(const uint8_t* d, size_t n) : data(d), size(n) {
    std::memset(arith_dc_l, 0, sizeof arith_dc_l);
    std::memset(arith_dc_u, 1, sizeof arith_dc_u);
    std::memset(arith_ac_k, 5, sizeof arith_ac_k);
  }

  int u8() {
    if (pos >= size) fail("Premature end of JPEG file");
    return data[pos++];
  }
  int u16() {
    const int a = u8();
    return (a << 8) | u8();
  }

  // Next marker code (after 0xFF fill bytes), skipping garbage like libjpeg.
  int next_marker() {
    for (;;) {
      while (pos < size && data[pos] != 0xFF) pos++;
      if (pos >= size) return -1;
      while (pos < size && data[pos] == 0xFF) pos++;
      if (pos >= size) return -1;
      const int m = data[pos++];
      if (m != 0) return m;
    }
  }

  void read_dqt() {
    int len = u16() - 2;
    while (len > 0) {
      const int pq = u8();
      const int t = pq & 15, prec = pq >> 4;
      if (t > 3) fail("Bogus DQT index");
      for (int i = 0; i < 64; i++) qt[t][kNatural[i]] = (uint16_t)(prec ? u16() : u8());
      qt_present[t] = true;
      len -= 1 + 64 * (prec ? 2 : 1);
    }
    if (len < 0) fail("Bogus marker length");
  }

  void read_dht() {
    int len = u16() - 2;
    while (len > 16) {
      const int tc = u8();
      uint8_t bits[17] = {0};
      int count = 0;
      for (int i = 1; i <= 16; i++) {
        bits[i] = (uint8_t)u8();
        count += bits[i];
      }
      len -= 17;
      if (count > 256 || count > len) fail("Bogus Huffman table definition");
      uint8_t vals[256];
      for (int i = 0; i < count; i++) vals[i] = (uint8_t)u8();
      len -= count;
      const int cls = tc >> 4, idx = tc & 15;
      if (idx > 3) fail("Bogus DHT index");
      cached_huff(cls ? ac[idx] : dc[idx], bits, vals, count);
    }
    if (len != 0) fail("Bogus marker length");
  }

  // jdmarker.c get_dac: (Tc Tb, value) pairs; DC values are U << 4 | L.
  void read_dac() {
    int len = u16() - 2;
    while (len > 0) {
      const int index = u8(), val = u8();
      len -= 2;
      if (index >= 32) fail("Bogus DAC index " + std::to_string(index));
      if (index >= 16) {
        arith_ac_k[index - 16] = (uint8_t)val;
      } else {
        arith_dc_l[index] = (uint8_t)(val & 15);
        arith_dc_u[index] = (uint8_t)(val >> 4);
        if (arith_dc_l[index] > arith_dc_u[index]) fail("Bogus DAC value " + hex2(val));
      }
    }
    if (len != 0) fail("Bogus marker length");
  }

  void read_sof(int marker) {
    if (frame) fail("Invalid JPEG file structure: two SOF markers");
    const int len = u16();
    const int prec = u8();
    height = u16();
    width = u16();
    ncomp = u8();
    if (prec != 8) fail("Unsupported JPEG data precision " + std::to_string(prec));
    if (width <= 0 || height <= 0 || ncomp <= 0 || ncomp > 4) fail("Empty JPEG image (DNL not supported)");
    if (len != 8 + 3 * ncomp) fail("Bogus marker length");
    progressive = marker == 0xC2 || marker == 0xCA;
    arith = marker == 0xC9 || marker == 0xCA;
    lossless = marker == 0xC3;
    // progressive files: every scan's entropy decode on the host (round 5's
    // device form, one serial chain per component, lost to the host decode
    // at 16 workers and was retired in round 6: DESIGN.md section 8)
    if ((arith || lossless || progressive) && device_entropy) throw NotDevice{};
    for (int i = 0; i < ncomp; i++) {
      Component& c = comp[i];
      c.id = u8();
      const int hv = u8();
      c.h = hv >> 4;
      c.v = hv & 15;
      c.tq = u8();
      if (c.h < 1 || c.h > 4 || c.v < 1 || c.v > 4 || c.tq > 3) fail("Bogus sampling factors");
      max_h = std::max(max_h, c.h);
      max_v = std::max(max_v, c.v);
    }
    mcux = (width + 8 * max_h - 1) / (8 * max_h);
    mcuy = (height + 8 * max_v - 1) / (8 * max_v);
    int64_t total = 0;
    for (int i = 0; i < ncomp; i++) {
      Component& c = comp[i];
      c.dw = (int)(((int64_t)width * c.h + max_h - 1) / max_h);
      c.dh = (int)(((int64_t)height * c.v + max_v - 1) / max_v);
      c.wib = (c.dw + 7) / 8;
      c.hib = (c.dh + 7) / 8;
      c.bw = mcux * c.h;
      c.bh = mcuy * c.v;
      c.off = total;
      total += (int64_t)c.bw * c.bh * 64;
      if ((lossless || (!progressive && !defer)) && !device_entropy) c.plane.assign((size_t)c.bw * 8 * c.bh * 8, 0);
    }
    coef_total = lossless ? 0 : total;
    if ((progressive || defer) && !lossless && !device_entropy) coefbuf.assign((size_t)total, 0);
    for (auto& row : coef_bits)
      for (int& b : row) b = -1;
    frame = true;
  }

  void read_app(int marker) {
    const int len = u16();
    if (len < 2 || pos + len - 2 > size) fail("Bogus marker length");
    const uint8_t* d = data + pos;
    const int n = len - 2;
    if (marker == 0xE0 && n >= 5 && std::memcmp(d, "JFIF\0", 5) == 0) jfif = true;
    if (marker == 0xEE && n >= 12 && std::memcmp(d, "Adobe", 5) == 0) {
      adobe = true;
      adobe_transform = d[11];
    }
    pos += n;
  }

  void skip_segment() {
    const int len = u16();
    if (len < 2) fail("Bogus marker length");
    pos += len - 2;
    if (pos > size) pos = size;
  }

  const uint16_t* quant(const Component& c) const {
    if (!qt_present[c.tq]) fail("Quantization table 0x0" + std::to_string(c.tq) + " was not defined");
    return qt[c.tq];
  }

  // ---- scans
  void read_sos() {
    if (!frame) fail("Invalid JPEG file structure: SOS before SOF");
    const int len = u16();
    const int ns = u8();
    if (ns < 1 || ns > 4 || len != 6 + 2 * ns) fail("Bogus marker length");
    Component* sc[4];
    for (int i = 0; i < ns; i++) {
      const int id = u8(), t = u8();
      Component* c = nullptr;
      for (int k = 0; k < ncomp; k++)
        if (comp[k].id == id && !c) c = &comp[k];
      if (!c) fail("Invalid component ID " + std::to_string(id) + " in SOS");
      c->dc_tbl = t >> 4;
      c->ac_tbl = t & 15;
      sc[i] = c;
    }
    const int ss = u8(), se = u8(), a = u8();
    const int ah = a >> 4, al = a & 15;
    if (device_entropy) {
      record_scan(sc, ns);
      any_scan = true;
      return;
    }
    if (progressive) {
      if (ss > se || se > 63 || (ss == 0 && se != 0) || (ss > 0 && ns != 1) || ah > 13 || al > 13)
        fail("Invalid progressive parameters");
      // progression status, updated when the scan starts (whatever its data holds)
      input_scans++;
      for (int i = 0; i < ns; i++) {
        const int ci = (int)(sc[i] - comp);
        for (int k = std::min(ss, 1); k <= std::min(std::max(se, 9), 9); k++)
          coef_bits[4 + ci][k] = input_scans > 1 ? coef_bits[ci][k] : 0;
        for (int k = ss; k <= std::min(se, 9); k++) coef_bits[ci][k] = al;
      }
    } else if (ss != 0 || se != 63 || ah != 0 || al != 0) {
      // libjpeg only warns here; sequential decoding ignores the fields
    }
    any_scan = true;
    for (int i = 0; i < ns; i++) sc[i]->dc_pred = 0;
    eobrun = 0;
    if (lossless) {
      // jdlossls.c start_pass: a predictor 1..7, Se 0, Ah 0, Al below the precision
      if (ss < 1 || ss > 7 || se != 0 || ah != 0 || al >= 8) fail("Invalid progressive parameters");
      Bits bits;
      bits.p = data + pos;
      bits.end = data + size;
      decode_scan_lossless(bits, sc, ns, ss, al);
      pos = (size_t)(bits.p - data);
      return;
    }
    if (arith) {
      if (progressive && ah != 0 && al != ah - 1) fail("Invalid progressive parameters");
      Arith ar;
      ar.p = data + pos;
      ar.end = data + size;
      decode_scan_arith(ar, sc, ns, ss, se, ah, al);
      pos = (size_t)(ar.p - data);
      return;
    }
    Bits bits;
    bits.p = data + pos;
    bits.end = data + size;
    decode_scan(bits, sc, ns, ss, se, ah, al);
    // resume marker parsing where the entropy data ended
    pos = (size_t)(bits.p - data);
  }

  // jdhuff.c jpeg_make_d_derived_tbl: DC symbols (difference categories)
  // above 15 are a bogus table.
  void check_dc_table(const Huff& h) const {
    for (int i = 0; i < h.nvals; i++)
      if (h.vals[i] > 15) fail("Bogus Huffman table definition");
  }

  // Device entropy decode: the scan's segments are recorded, not decoded.
  // Covered: the first and only scan of a sequential file, carrying every
  // component of a grey (1) or YCbCr / RGB (3) image, its entropy-coded data
  // ending at a marker, restart markers RST0..7 in sequence, one per interval.
  void record_scan(Component** sc, int ns) {
    if (scans++ > 0 || progressive || ns != ncomp || (ncomp != 1 && ncomp != 3 && ncomp != 4)) throw NotDevice{};
    int bpm = 0;
    for (int i = 0; i < ns; i++) {
      if (sc[i]->dc_tbl > 3 || sc[i]->ac_tbl > 3 || !dc[sc[i]->dc_tbl].present || !ac[sc[i]->ac_tbl].present)
          fail("Huffman table was not defined");
      check_dc_table(dc[sc[i]->dc_tbl]);
      std::memcpy(sc[i]->q, quant(*sc[i]), sizeof sc[i]->q);  // latched at the scan
      sc[i]->coded = true;
      scan_comp[i] = (int)(sc[i] - comp);
      bpm += ns == 1 ? 1 : sc[i]->h * sc[i]->v;
    }
    if (bpm > 10) throw NotDevice{};  // libjpeg: "Sampling factors too large for interleaved scan"
    scan_ns = ns;
    scan_mcus = ns == 1 ? (int64_t)sc[0]->wib * sc[0]->hib : (int64_t)mcux * mcuy;
    record_segments(scan_mcus);
    pending = true;
  }

  // The entropy-coded data from pos split at its restart markers (RST0..7 in
  // sequence, one per interval) into seg_begin / seg_end / seg_bytes; pos
  // left at the marker after the data.  Data not ending at a marker, or
  // markers out of sequence: NotDevice.
  void record_segments(int64_t mcus) {
    const int64_t nseg = restart_interval ? (mcus + restart_interval - 1) / restart_interval : 1;
    const int64_t seg0 = (int64_t)seg_begin.size();
    size_t p = pos, b = pos;
    int next_rst = 0;
    int64_t dropped = 0;  // bytes unstuff() drops: the 0x00 of 0xFF 0x00, fill 0xFF bytes
    for (;;) {
      p = scan_to_marker(data, p, size, &dropped);
      if (p + 1 >= size) throw NotDevice{};  // no marker after the data: truncated
      const uint8_t m = data[p + 1];
      // the device decoder keeps a segment's bit count and word offsets in
      // int32: segments past 2^28 bytes go to the host decoder
      if (p - b >= ((size_t)1 << 28)) throw NotDevice{};
      seg_begin.push_back((int64_t)b);
      seg_end.push_back((int64_t)p);
      seg_bytes.push_back((int64_t)(p - b) - dropped);
      dropped = 0;
      if (m >= 0xD0 && m <= 0xD7) {
        if (!restart_interval || m != 0xD0 + next_rst || (int64_t)seg_begin.size() - seg0 >= nseg) throw NotDevice{};
        next_rst = (next_rst + 1) & 7;
        p += 2;
        b = p;
        continue;
      }
      break;  // the marker after the scan
    }
    if ((int64_t)seg_begin.size() - seg0 != nseg) throw NotDevice{};
    pos = seg_end.back();  // marker parsing resumes at the marker
  }

  // R: Bits or Arith (restart(), insufficient)
  template <class R, class F>
  void for_each_mcu(R& bits, Component** sc, int ns, F&& decode_block) {
    int restarts_left = restart_interval, next_rst = 0;
    auto restart_check = [&]() {
      if (restart_interval) {
        if (restarts_left == 0) {
          bits.restart(next_rst);
          next_rst = (next_rst + 1) & 7;
          for (int i = 0; i < ns; i++) sc[i]->dc_pred = 0;
          eobrun = 0;
          restarts_left = restart_interval;
        }
        restarts_left--;
      }
    };
    if (ns == 1) {
      // non-interleaved: MCU = one block of the component proper
      Component& c = *sc[0];
      for (int by = 0; by < c.hib; by++)
        for (int bx = 0; bx < c.wib; bx++) {
          restart_check();
          if (!bits.insufficient) last_good_imcu = by / c.v;
          decode_block(c, bx, by, bits.insufficient);
        }
    } else {
      for (int my = 0; my < mcuy; my++)
        for (int mx = 0; mx < mcux; mx++) {
          restart_check();
          const bool skip = bits.insufficient;
          if (!skip) last_good_imcu = my;
          for (int i = 0; i < ns; i++) {
            Component& c = *sc[i];
            for (int v = 0; v < c.v; v++)
              for (int h = 0; h < c.h; h++) decode_block(c, mx * c.h + h, my * c.v + v, skip);
          }
        }
    }
  }

  void decode_scan(Bits& bits, Component** sc, int ns, int ss, int se, int ah, int al) {
    if (!progressive) {
      for (int i = 0; i < ns; i++) {
        if (sc[i]->dc_tbl > 3 || sc[i]->ac_tbl > 3 || !dc[sc[i]->dc_tbl].present || !ac[sc[i]->ac_tbl].present)
          fail("Huffman table was not defined");
        check_dc_table(dc[sc[i]->dc_tbl]);
        std::memcpy(sc[i]->q, quant(*sc[i]), sizeof sc[i]->q);  // latched at the scan
        sc[i]->coded = true;
      }
      int16_t local[64];
      for_each_mcu(bits, sc, ns, [&](Component& c, int bx, int by, bool skip) {
        // deferred blocks are zero from the allocation (each is written once)
        int16_t* blk = defer ? cblk(c, bx, by) : local;
        if (!defer) std::memset(blk, 0, 64 * sizeof(int16_t));
        if (!skip) bits.block_seq(dc[c.dc_tbl], ac[c.ac_tbl], c.dc_pred, blk);
        if (!defer) idct_block(blk, c.q, c.plane.data() + ((size_t)by * 8 * c.bw * 8) + (size_t)bx * 8, c.bw * 8);
      });
      return;
    }
    // progressive (jdphuff.c)
    if (ss == 0) {
      if (ah == 0)
        for (int i = 0; i < ns; i++) {
          if (sc[i]->dc_tbl > 3 || !dc[sc[i]->dc_tbl].present) fail("Huffman table was not defined");
          check_dc_table(dc[sc[i]->dc_tbl]);  // (jdphuff.c derives DC tables with the DC check too)
        }
      for_each_mcu(bits, sc, ns, [&](Component& c, int bx, int by, bool skip) {
        int16_t* blk = cblk(c, bx, by);
        if (ah == 0) {
          if (skip) return;
          int s = bits.decode(dc[c.dc_tbl]);
          if (s) s = extend(bits.get(s), s);
          s += c.dc_pred;
          c.dc_pred = s;
          blk[0] = (int16_t)(s * (1 << al));
        } else if (bits.get(1)) {
          blk[0] |= (int16_t)(1 << al);
        }
      });
      return;
    }
    Component& c0 = *sc[0];
    if (c0.ac_tbl > 3 || !ac[c0.ac_tbl].present) fail("Huffman table was not defined");
    const Huff& ha = ac[c0.ac_tbl];
    if (ah == 0) {
      for_each_mcu(bits, sc, ns, [&](Component& c, int bx, int by, bool skip) {
        if (skip) return;
        int16_t* blk = cblk(c, bx, by);
        if (eobrun > 0) {
          eobrun--;
          return;
        }
        for (int k = ss; k <= se; k++) {
          if (bits.cnt < 16) bits.fill();
          const FastAC f = ha.fac[bits.peek(kLook)];
          if (f.len && f.run != kEob) {
            bits.consume(f.len);
            k += f.run;
            blk[kNatural[k]] = (int16_t)(f.val * (1 << al));
            continue;
          }
          const int rs = bits.decode(ha);
          int r = rs >> 4;
          const int s = rs & 15;
          if (s) {
            k += r;
            blk[kNatural[k]] = (int16_t)(extend(bits.get(s), s) * (1 << al));
          } else if (r == 15) {
            k += 15;
          } else {
            eobrun = 1 << r;
            if (r) eobrun += bits.get(r);
            eobrun--;
            break;
          }
        }
      });
      return;
    }
    const int p1 = 1 << al, m1 = -1 * (1 << al);
    for_each_mcu(bits, sc, ns, [&](Component& c, int bx, int by, bool skip) {
      if (!skip) bits.block_refine(ha, cblk(c, bx, by), ss, se, p1, m1, eobrun);
    });
  }

  // One lossless scan (T.81 H.1.2; jdlossls.c / jdlhuff.c / jdpred.c): per
  // sample a Huffman-coded difference category (DC tables, 0..16; 16 is
  // 32768 with no extra bits) and value, added modulo 2^16 to the
  // prediction from the component's reconstructed neighbours -- Ra (left), Rb
  // (above), Rc (above left) through predictor `psv` -- except on the first
  // line of the scan or of a restart interval (Ra; its first sample
  // 2^(P - Pt - 1)) and in the first column (Rb).  The output sample is the
  // reconstruction << Pt (8 bits).  An MCU holds h x v samples of each
  // component (interleaved) or one sample (one component).
  void decode_scan_lossless(Bits& bits, Component** sc, int ns, int psv, int pt) {
    for (int i = 0; i < ns; i++) {
      if (sc[i]->dc_tbl > 3 || !dc[sc[i]->dc_tbl].present) fail("Huffman table was not defined");
      const Huff& h = dc[sc[i]->dc_tbl];
      for (int k = 0; k < h.nvals; k++)
        if (h.vals[k] > 16) fail("Bogus Huffman table definition");
      sc[i]->coded = true;
    }
    const int mx_n = ns == 1 ? sc[0]->dw : (width + max_h - 1) / max_h;
    const int my_n = ns == 1 ? sc[0]->dh : (height + max_v - 1) / max_v;
    // reconstructed samples per component, on its MCU-padded sample grid
    std::vector<int32_t> rec[4];
    int gw[4], row0[4];
    for (int i = 0; i < ns; i++) {
      const int hh = ns == 1 ? 1 : sc[i]->h, vv = ns == 1 ? 1 : sc[i]->v;
      gw[i] = mx_n * hh;
      rec[i].assign((size_t)gw[i] * my_n * vv, 0);
      row0[i] = 0;
    }
    const int init = 1 << (8 - pt - 1);
    auto predict = [&](int i, int x, int y) -> int {
      const int32_t* r = rec[i].data();
      const int w = gw[i];
      if (y == row0[i]) return x == 0 ? init : r[(size_t)y * w + x - 1];
      if (x == 0) return r[(size_t)(y - 1) * w];
      const int ra = r[(size_t)y * w + x - 1], rb = r[(size_t)(y - 1) * w + x], rc = r[(size_t)(y - 1) * w + x - 1];
      switch (psv) {
        case 1: return ra;
        case 2: return rb;
        case 3: return rc;
        case 4: return ra + rb - rc;
        case 5: return ra + ((rb - rc) >> 1);
        case 6: return rb + ((ra - rc) >> 1);
        default: return (ra + rb) >> 1;
      }
    };
    // Data running out (jdlhuff.c decode_mcus, per MCU row): the row it runs
    // out in decodes on from zero bits; every later row (until a restart
    // marker clears the flag) gets zero differences with the predictor
    // restarted, i.e. uniform grey.
    int restarts_left = restart_interval, next_rst = 0;
    bool skip = false;
    for (int my = 0; my < my_n; my++)
      for (int mx = 0; mx < mx_n; mx++) {
        if (restart_interval) {
          if (restarts_left == 0) {
            bits.restart(next_rst);
            next_rst = (next_rst + 1) & 7;
            for (int i = 0; i < ns; i++) row0[i] = my * (ns == 1 ? 1 : sc[i]->v);
            restarts_left = restart_interval;
          }
          restarts_left--;
        }
        if (mx == 0) {
          skip = bits.insufficient;
          if (skip)
            for (int i = 0; i < ns; i++) row0[i] = my * (ns == 1 ? 1 : sc[i]->v);
        }
        for (int i = 0; i < ns; i++) {
          const int hh = ns == 1 ? 1 : sc[i]->h, vv = ns == 1 ? 1 : sc[i]->v;
          const Huff& h = dc[sc[i]->dc_tbl];
          for (int v = 0; v < vv; v++)
            for (int u = 0; u < hh; u++) {
              const int x = mx * hh + u, y = my * vv + v;
              int diff = 0;
              if (!skip) {
                const int s = bits.decode(h);
                if (s == 16) diff = -32768;
                else if (s) diff = extend(bits.get(s), s);
              }
              rec[i][(size_t)y * gw[i] + x] = (predict(i, x, y) + diff) & 0xFFFF;
            }
        }
      }
    // the samples (<< Pt, 8 bits) into the planes the output reads
    for (int i = 0; i < ns; i++) {
      Component& c = *sc[i];
      const int rows = (int)(rec[i].size() / gw[i]);
      const int stride = c.bw * 8;
      for (int y = 0; y < rows && y < c.bh * 8; y++)
        for (int x = 0; x < gw[i] && x < stride; x++)
          c.plane[(size_t)y * stride + x] = (uint8_t)(rec[i][(size_t)y * gw[i] + x] << pt);
    }
  }

  // One arithmetic-coded scan (T.81 F.2.4 / G.2: jdarith.c's decode_mcu,
  // decode_mcu_DC_first / _AC_first / _DC_refine / _AC_refine).  The
  // statistics of the scan's tables, the DC predictions and contexts start
  // over at the scan and at every restart; a spectral or magnitude overflow
  // (corrupt data) leaves the rest of its restart interval's blocks alone.
  void decode_scan_arith(Arith& ar, Component** sc, int ns, int ss, int se, int ah, int al) {
    const bool dc_stats = !progressive || (ss == 0 && ah == 0);
    const bool ac_stats = !progressive || ss != 0;
    int dct[4], act[4];
    for (int i = 0; i < ns; i++) {
      dct[i] = dc_stats ? sc[i]->dc_tbl : -1;
      act[i] = ac_stats ? sc[i]->ac_tbl : -1;
      if (!progressive) {
        std::memcpy(sc[i]->q, quant(*sc[i]), sizeof sc[i]->q);  // latched at the scan
        sc[i]->coded = true;
      }
    }
    int dc_ctx[4] = {0, 0, 0, 0};
    int gen = 0, seen = -1;  // restarts seen by the coder / by the block loop
    struct Restarting {
      Arith& ar;
      int& gen;
      bool insufficient = false;
      void restart(int expected) {
        ar.restart(expected);
        gen++;
      }
    } rd{ar, gen};
    auto fresh = [&]() {
      if (seen == gen) return;
      seen = gen;
      ar.clear_stats(dct, act, ns);
      for (int i = 0; i < 4; i++) dc_ctx[i] = 0;
    };
    // F.2.4.1: a DC difference in the context of the component's last one
    auto dc_diff = [&](Component& c) -> bool {
      const int ci = (int)(&c - comp), t = c.dc_tbl;
      uint8_t* st = ar.dc_stats[t];
      const int s0 = dc_ctx[ci];
      if (!ar.decode(st[s0])) {
        dc_ctx[ci] = 0;
        return true;
      }
      const int sign = ar.decode(st[s0 + 1]);
      int cat;
      const int v = ar.magnitude(st, s0 + 2 + sign, 20, false, &cat);
      if (v < 0) return false;
      if (cat < (1 << arith_dc_l[t]) >> 1) dc_ctx[ci] = 0;
      else if (cat > (1 << arith_dc_u[t]) >> 1) dc_ctx[ci] = 12 + 4 * sign;
      else dc_ctx[ci] = 4 + 4 * sign;
      c.dc_pred = (c.dc_pred + (sign ? -(v + 1) : v + 1)) & 0xffff;
      return true;
    };
    // F.2.4.2 / G.2: the AC coefficients k0..k1 of a first (or only) scan
    auto ac_first = [&](Component& c, int16_t* blk, int k0, int k1, int shift) -> bool {
      const int t = c.ac_tbl;
      uint8_t* st = ar.ac_stats[t];
      int k = k0 - 1;
      do {
        int i = 3 * k;
        if (ar.decode(st[i])) break;  // end of block
        for (;;) {
          k++;
          if (ar.decode(st[i + 1])) break;
          i += 3;
          if (k >= k1) return false;  // spectral overflow
        }
        const int sign = ar.decode(ar.fixed);
        int cat;
        const int v = ar.magnitude(st, i + 2, k <= arith_ac_k[t] ? 189 : 217, true, &cat);
        if (v < 0) return false;
        blk[kNatural[k]] = (int16_t)((uint32_t)(sign ? -(v + 1) : v + 1) << shift);
      } while (k < k1);
      return true;
    };
    if (!progressive) {
      int16_t local[64];
      for_each_mcu(rd, sc, ns, [&](Component& c, int bx, int by, bool) {
        fresh();
        int16_t* blk = defer ? cblk(c, bx, by) : local;
        if (!defer) std::memset(blk, 0, 64 * sizeof(int16_t));
        if (!ar.failed) {
          if (!dc_diff(c)) ar.failed = true;
          else {
            blk[0] = (int16_t)c.dc_pred;
            if (!ac_first(c, blk, 1, 63, 0)) ar.failed = true;  // (a sequential scan's Ss / Se / Al are ignored)
          }
        }
        if (!defer) idct_block(blk, c.q, c.plane.data() + ((size_t)by * 8 * c.bw * 8) + (size_t)bx * 8, c.bw * 8);
      });
      return;
    }
    const int p1 = 1 << al, m1 = -1 * (1 << al);
    for_each_mcu(rd, sc, ns, [&](Component& c, int bx, int by, bool) {
      fresh();
      if (ar.failed) return;
      int16_t* blk = cblk(c, bx, by);
      if (ss == 0 && ah == 0) {
        if (!dc_diff(c)) ar.failed = true;
        else blk[0] = (int16_t)((uint32_t)c.dc_pred << al);
      } else if (ss == 0) {
        if (ar.decode(ar.fixed)) blk[0] = (int16_t)(blk[0] | p1);
      } else if (ah == 0) {
        if (!ac_first(c, blk, ss, se, al)) ar.failed = true;
      } else {
        uint8_t* st = ar.ac_stats[c.ac_tbl];
        int kex = se;  // the previous stage's end of block
        while (kex > 0 && !blk[kNatural[kex]]) kex--;
        for (int k = ss - 1; k < se; k++) {
          int i = 3 * k;
          if (k >= kex && ar.decode(st[i])) break;  // end of block
          for (;;) {
            int16_t& co = blk[kNatural[k + 1]];
            if (co) {  // already nonzero: a correction bit
              if (ar.decode(st[i + 2])) co = (int16_t)(co < 0 ? co + m1 : co + p1);
              break;
            }
            if (ar.decode(st[i + 1])) {  // newly nonzero
              co = (int16_t)(ar.decode(ar.fixed) ? m1 : p1);
              break;
            }
            i += 3;
            k++;
            if (k >= se) {
              ar.failed = true;  // spectral overflow
              return;
            }
          }
        }
      }
    });
  }

  void parse() {
    if (size < 3 || data[0] != 0xFF || data[1] != 0xD8) fail("Not a JPEG file");
    pos = 2;
    for (;;) {
      const int m = next_marker();
      if (m < 0) {
        if (!any_scan) fail("Premature end of JPEG file");
        return;  // libjpeg warns and finishes with what it has
      }
      switch (m) {
        case 0xC0:
        case 0xC1:
        case 0xC2:
        case 0xC3:
        case 0xC9:
        case 0xCA:
          read_sof(m);
          break;
        case 0xC5: case 0xC6: case 0xC7: case 0xCB: case 0xCD: case 0xCE:
        case 0xCF:
          unsupported_sof(m);
        case 0xC4:
          // a table defined after the recorded scan (before EOI): the host
          // decoded that scan at its SOS with the earlier tables, the device
          // would read the later ones -- decode such files on the host
          if (pending) throw NotDevice{};
          read_dht();
          break;
        case 0xCC:
          read_dac();
          break;
        case 0xDB:
          read_dqt();
          break;
        case 0xDD:
          if (pending) throw NotDevice{};  // likewise a restart interval after the recorded scan
          if (u16() != 4) fail("Bogus marker length");
          restart_interval = u16();
          break;
        case 0xDA:
          read_sos();
          break;
        case 0xD9:
          if (!any_scan) fail("Premature end of JPEG file");
          eoi = true;
          return;
        case 0xD8:
          fail("Invalid JPEG file structure: two SOI markers");
        default:
          if (m >= 0xD0 && m <= 0xD7) break;  // stray RST
          if (m >= 0xE0 && m <= 0xEF) read_app(m);
          else skip_segment();
      }
    }
  }

  int color_space() const;  // 0 grey, 1 YCbCr, 2 RGB, 3 CMYK, 4 YCCK

  // Row y of component c upsampled to full width (jdsample.c), into o (>= width
  // bytes; scratch >= 2 * dw + 2 bytes); returns the row (o, or the plane row
  // itself when c is full size).
  const uint8_t* upsample_row(const Component& c, const uint8_t* pl, int y, uint8_t* o, uint8_t* scratch) const {
    const int W = width;
    const int stride = c.bw * 8;
    const int hx = max_h / c.h, vx = max_v / c.v;
    const bool h2 = c.h * 2 == max_h, v2 = c.v * 2 == max_v;
    auto row = [&](int yy) { return pl + (size_t)std::min(std::max(yy, 0), c.dh - 1) * stride; };
    if (c.h == max_h && c.v == max_v) return pl + (size_t)y * stride;
    if (h2 && c.v == max_v) {
      // h2v1_fancy_upsample (or h2v1_upsample when dw <= 2)
      const uint8_t* in = pl + (size_t)y * stride;
      uint8_t* t = scratch;
      if (c.dw > 2) {
        int v = in[0];
        t[0] = (uint8_t)v;
        t[1] = (uint8_t)((v * 3 + in[1] + 2) >> 2);
        for (int x = 1; x < c.dw - 1; x++) {
          v = in[x] * 3;
          t[2 * x] = (uint8_t)((v + in[x - 1] + 1) >> 2);
          t[2 * x + 1] = (uint8_t)((v + in[x + 1] + 2) >> 2);
        }
        v = in[c.dw - 1];
        t[2 * c.dw - 2] = (uint8_t)((v * 3 + in[c.dw - 2] + 1) >> 2);
        t[2 * c.dw - 1] = (uint8_t)v;
      } else {
        for (int x = 0; x < c.dw; x++) t[2 * x] = t[2 * x + 1] = in[x];
      }
      return t;
    }
    if (c.h == max_h && v2) {
      // h1v2_fancy_upsample
      const int iy = y >> 1;
      const bool below = y & 1;
      const uint8_t* in0 = row(iy);
      const uint8_t* in1 = row(below ? iy + 1 : iy - 1);
      const int bias = below ? 2 : 1;
      for (int x = 0; x < W; x++) o[x] = (uint8_t)((in0[x] * 3 + in1[x] + bias) >> 2);
      return o;
    }
    if (h2 && v2 && c.dw > 2) {
      // h2v2_fancy_upsample
      const int iy = y >> 1;
      const bool below = y & 1;
      const uint8_t* in0 = row(iy);
      const uint8_t* in1 = row(below ? iy + 1 : iy - 1);
      h2v2_fancy_row(in0, in1, c.dw, scratch, reinterpret_cast<int16_t*>(scratch + 2 * c.dw + 2));
      return scratch;
    }
    if (max_h % c.h != 0 || max_v % c.v != 0) fail("Fractional sampling not implemented yet");
    // int_upsample / h2v1_upsample / h2v2_upsample: replication.  Source rows
    // come from the padded plane (not clamped), like the row groups libjpeg
    // replicates.
    const uint8_t* in = pl + (size_t)(y / vx) * stride;
    for (int x = 0; x < W; x++) o[x] = in[x / hx];
    return o;
  }

  // After parse(): a progressive image latches every component's table now
  // (they may change between scans); sequential scans latched theirs.
  void finalize() {
    if (!progressive) return;
    finalize_quant();
    smooth_blocks();
  }
  void finalize_quant() {
    for (int i = 0; i < ncomp; i++) {
      std::memcpy(comp[i].q, quant(comp[i]), sizeof comp[i].q);
      comp[i].coded = true;
    }
  }

  // ---- block smoothing (libjpeg's do_block_smoothing, on by default and
  // reached through jpeg_start_decompress, ImageJPEG.cpp:100-101)
  //
  // A progressive file whose scans leave some of the first nine AC
  // coefficients inexact (truncated files, or files that never send them)
  // gets them estimated from the DC values of the 5x5 block neighbourhood,
  // as libjpeg-turbo's jdcoefct.c decompress_smooth_data does (its 5x5
  // extension of ITU T.81 Annex K.8): an estimate replaces a coefficient
  // only while it is still zero, limited to the bits below its Al; with no
  // AC data at all for a component the DC itself is re-estimated too and
  // four more coefficients are filled.  Pinned by Pillow's libjpeg-turbo
  // decodes of truncated progressive files (tests/golden/jpeg.npz, prog_trunc*).

  // jdcoefct.c smoothing_ok: DC known for every component, the ten
  // quantisers nonzero, and some of the nine AC coefficients inexact.
  bool smoothing_ok() const {
    static const int kPos[10] = {0, 1, 8, 16, 9, 2, 3, 10, 17, 24};
    bool useful = false;
    for (int ci = 0; ci < ncomp; ci++) {
      for (int k = 0; k < 10; k++)
        if (comp[ci].q[kPos[k]] == 0) return false;
      if (coef_bits[ci][0] < 0) return false;
      for (int k = 1; k < 10; k++)
        if (coef_bits[ci][k] != 0) useful = true;
    }
    return useful;
  }

  static int smooth_pred(int64_t num, int64_t q, int al, bool limit) {
    int pred = (int)(((q << 7) + (num >= 0 ? num : -num)) / (q << 8));
    if (limit && al > 0 && pred >= (1 << al)) pred = (1 << al) - 1;
    return num >= 0 ? pred : -pred;
  }

  void smooth_blocks() {
    if (coefbuf.empty() || !smoothing_ok()) return;
    std::vector<int16_t> out(coefbuf);
    for (int ci = 0; ci < ncomp; ci++) {
      const Component& c = comp[ci];
      int prev[10];
      for (int k = 0; k < 10; k++) prev[k] = input_scans > 1 ? coef_bits[4 + ci][k] : -1;
      const int64_t Q00 = c.q[0], Q01 = c.q[1], Q10 = c.q[8], Q20 = c.q[16], Q11 = c.q[9], Q02 = c.q[2],
                    Q03 = c.q[3], Q12 = c.q[10], Q21 = c.q[17], Q30 = c.q[24];
      auto dc = [&](int row, int col) { return (int)coefbuf[c.off + ((int64_t)row * c.bw + col) * 64]; };
      const int last_col = c.wib - 1;
      for (int m = 0; m < mcuy; m++) {
        // block rows of this iMCU row (the last one: the rows of the component proper)
        int block_rows = c.v;
        if (m == mcuy - 1 && c.hib % c.v) block_rows = c.hib % c.v;
        const int64_t image_rows = (int64_t)block_rows * mcuy;
        const int* bits = m > last_good_imcu ? prev : coef_bits[ci];
        bool change_dc = true;
        for (int k = 1; k < 10; k++) change_dc = change_dc && bits[k] == -1;
        for (int br = 0; br < block_rows; br++) {
          const int r = m * c.v + br;
          const int64_t ir = (int64_t)m * block_rows + br;
          const int rp = ir > 0 ? r - 1 : r, rpp = ir > 1 ? r - 2 : rp;
          const int rn = ir < image_rows - 1 ? r + 1 : r, rnn = ir < image_rows - 2 ? r + 2 : rn;
          const int rows[5] = {rpp, rp, r, rn, rnn};
          // D[i][j]: DC of row i, column block - 2 + j clamped to the component's blocks
          int D[5][5];
          for (int b = 0; b <= last_col; b++) {
            for (int i = 0; i < 5; i++)
              for (int j = 0; j < 5; j++) D[i][j] = dc(rows[i], std::min(std::max(b - 2 + j, 0), last_col));
            const int DC01 = D[0][0], DC02 = D[0][1], DC03 = D[0][2], DC04 = D[0][3], DC05 = D[0][4];
            const int DC06 = D[1][0], DC07 = D[1][1], DC08 = D[1][2], DC09 = D[1][3], DC10 = D[1][4];
            const int DC11 = D[2][0], DC12 = D[2][1], DC13 = D[2][2], DC14 = D[2][3], DC15 = D[2][4];
            const int DC16 = D[3][0], DC17 = D[3][1], DC18 = D[3][2], DC19 = D[3][3], DC20 = D[3][4];
            const int DC21 = D[4][0], DC22 = D[4][1], DC23 = D[4][2], DC24 = D[4][3], DC25 = D[4][4];
            int16_t* w = out.data() + c.off + ((int64_t)r * c.bw + b) * 64;
            if (bits[1] != 0 && w[1] == 0)
              w[1] = (int16_t)smooth_pred(
                  Q00 * (change_dc ? (-DC01 - DC02 + DC04 + DC05 - 3 * DC06 + 13 * DC07 - 13 * DC09 + 3 * DC10 -
                                      3 * DC11 + 38 * DC12 - 38 * DC14 + 3 * DC15 - 3 * DC16 + 13 * DC17 -
                                      13 * DC19 + 3 * DC20 - DC21 - DC22 + DC24 + DC25)
                                   : (-7 * DC11 + 50 * DC12 - 50 * DC14 + 7 * DC15)),
                  Q01, bits[1], true);
            if (bits[2] != 0 && w[8] == 0)
              w[8] = (int16_t)smooth_pred(
                  Q00 * (change_dc ? (-DC01 - 3 * DC02 - 3 * DC03 - 3 * DC04 - DC05 - DC06 + 13 * DC07 +
                                      38 * DC08 + 13 * DC09 - DC10 + DC16 - 13 * DC17 - 38 * DC18 - 13 * DC19 +
                                      DC20 + DC21 + 3 * DC22 + 3 * DC23 + 3 * DC24 + DC25)
                                   : (-7 * DC03 + 50 * DC08 - 50 * DC18 + 7 * DC23)),
                  Q10, bits[2], true);
            if (bits[3] != 0 && w[16] == 0)
              w[16] = (int16_t)smooth_pred(
                  Q00 * (change_dc ? (DC03 + 2 * DC07 + 7 * DC08 + 2 * DC09 - 5 * DC12 - 14 * DC13 - 5 * DC14 +
                                      2 * DC17 + 7 * DC18 + 2 * DC19 + DC23)
                                   : (-DC03 + 13 * DC08 - 24 * DC13 + 13 * DC18 - DC23)),
                  Q20, bits[3], true);
            if (bits[4] != 0 && w[9] == 0)
              w[9] = (int16_t)smooth_pred(
                  Q00 * (change_dc ? (-DC01 + DC05 + 9 * DC07 - 9 * DC09 - 9 * DC17 + 9 * DC19 + DC21 - DC25)
                                   : (DC10 + DC16 - 10 * DC17 + 10 * DC19 - DC02 - DC20 + DC22 - DC24 + DC04 -
                                      DC06 + 10 * DC07 - 10 * DC09)),
                  Q11, bits[4], true);
            if (bits[5] != 0 && w[2] == 0)
              w[2] = (int16_t)smooth_pred(
                  Q00 * (change_dc ? (2 * DC07 - 5 * DC08 + 2 * DC09 + DC11 + 7 * DC12 - 14 * DC13 + 7 * DC14 +
                                      DC15 + 2 * DC17 - 5 * DC18 + 2 * DC19)
                                   : (-DC11 + 13 * DC12 - 24 * DC13 + 13 * DC14 - DC15)),
                  Q02, bits[5], true);
            if (change_dc) {
              if (bits[6] != 0 && w[3] == 0)
                w[3] = (int16_t)smooth_pred(Q00 * (DC07 - DC09 + 2 * DC12 - 2 * DC14 + DC17 - DC19), Q03, bits[6],
                                            true);
              if (bits[7] != 0 && w[10] == 0)
                w[10] = (int16_t)smooth_pred(Q00 * (DC07 - 3 * DC08 + DC09 - DC17 + 3 * DC18 - DC19), Q12,
                                             bits[7], true);
              if (bits[8] != 0 && w[17] == 0)
                w[17] = (int16_t)smooth_pred(Q00 * (DC07 - DC09 - 3 * DC12 + 3 * DC14 + DC17 - DC19), Q21,
                                             bits[8], true);
              if (bits[9] != 0 && w[24] == 0)
                w[24] = (int16_t)smooth_pred(Q00 * (DC07 + 2 * DC08 + DC09 - DC17 - 2 * DC18 - DC19), Q30,
                                             bits[9], true);
              w[0] = (int16_t)smooth_pred(
                  Q00 * (-2 * DC01 - 6 * DC02 - 8 * DC03 - 6 * DC04 - 2 * DC05 - 6 * DC06 + 6 * DC07 + 42 * DC08 +
                         6 * DC09 - 6 * DC10 - 8 * DC11 + 42 * DC12 + 152 * DC13 + 42 * DC14 - 8 * DC15 -
                         6 * DC16 + 6 * DC17 + 42 * DC18 + 6 * DC19 - 6 * DC20 - 2 * DC21 - 6 * DC22 - 8 * DC23 -
                         6 * DC24 - 2 * DC25),
                  Q00, 0, false);
            }
          }
        }
      }
    }
    coefbuf.swap(out);
  }

  // Components output() reads: grey -> 1; CMYK -> 3 (K is dropped).
  int used_components() const { return ncomp == 1 ? 1 : ncomp == 4 && color_space() == 3 ? 3 : ncomp; }

  // Samples of component i: the plane decoded in place (sequential), else the
  // IDCT of its coefficients into `store` (zeros for a component no scan
  // carried, as the in-place planes keep).
  const uint8_t* samples(int i, std::vector<uint8_t>& store) const {
    const Component& c = comp[i];
    if (lossless || (!progressive && !defer)) return c.plane.data();
    store.assign((size_t)c.bw * 8 * c.bh * 8, 0);
    if (c.coded)
      for (int by = 0; by < c.bh; by++)
        for (int bx = 0; bx < c.bw; bx++) {
          idct_block(coefbuf.data() + c.off + ((int64_t)by * c.bw + bx) * 64, c.q,
                     store.data() + (size_t)by * 8 * c.bw * 8 + (size_t)bx * 8, c.bw * 8);
        }
    return store.data();
  }

  void output(uint8_t* dst, int64_t dst_stride) const {
    std::vector<uint8_t> store[4];
    const uint8_t* pl[4] = {nullptr, nullptr, nullptr, nullptr};
    for (int i = 0; i < used_components(); i++) pl[i] = samples(i, store[i]);
    const int cs = color_space();
    const int W = width, H = height;
    if (ncomp == 1) {
      const Component& c = comp[0];
      for (int y = 0; y < H; y++) {
        const uint8_t* in = pl[0] + (size_t)y * c.bw * 8;
        uint8_t* o = dst + (size_t)y * dst_stride;
        for (int x = 0; x < W; x++) o[3 * x] = o[3 * x + 1] = o[3 * x + 2] = in[x];
      }
      return;
    }
    const int nuse = ncomp == 4 && cs == 3 ? 3 : ncomp;  // CMYK: K is dropped by the caller
    // per component: an output row, and scratch = 2 dw + 2 upsampled bytes +
    // dw int16 column sums (dw <= W)
    const size_t rb = ((size_t)W + 63) & ~(size_t)63, sb = ((size_t)4 * W + 64) & ~(size_t)63;
    std::vector<uint8_t> buf(3 * (rb + sb) + 64);
    uint8_t* base = reinterpret_cast<uint8_t*>(((uintptr_t)buf.data() + 63) & ~(uintptr_t)63);
    uint8_t* rowbuf[3];
    uint8_t* scratch[3];
    for (int i = 0; i < 3; i++) {
      rowbuf[i] = base + (size_t)i * (rb + sb);
      scratch[i] = rowbuf[i] + rb;
    }
    for (int y = 0; y < H; y++) {
      const uint8_t* r3[3];
      for (int i = 0; i < 3 && i < nuse; i++) r3[i] = upsample_row(comp[i], pl[i], y, rowbuf[i], scratch[i]);
      uint8_t* o = dst + (size_t)y * dst_stride;
      if (cs == 1 || cs == 4) ycc_rgb_row(r3[0], r3[1], r3[2], o, W, cs == 4);
      else
        for (int x = 0; x < W; x++) {
          o[3 * x] = r3[0][x];
          o[3 * x + 1] = r3[1][x];
          o[3 * x + 2] = r3[2][x];
        }
    }
  }
};

// jdapimin.c default_decompress_parms
int Decoder::color_space() const {
  if (ncomp == 1) return 0;
  if (lossless) {
    // libjpeg-turbo: no colour conversion in lossless mode -- RGB / CMYK
    // unless a JFIF or Adobe marker declares YCbCr / YCCK, which it refuses
    if (jfif || (adobe && adobe_transform != 0)) fail("Unsupported color conversion request");
    return ncomp == 3 ? 2 : ncomp == 4 ? 3 : -1;
  }
  if (ncomp == 3) {
    if (jfif) return 1;
    if (adobe) return adobe_transform == 0 ? 2 : 1;
    if (comp[0].id == 1 && comp[1].id == 2 && comp[2].id == 3) return 1;
    if (comp[0].id == 82 && comp[1].id == 71 && comp[2].id == 66) return 2;
    return 1;
  }
  if (ncomp == 4) {
    if (adobe) return adobe_transform == 0 ? 3 : 4;
    return 3;
  }
  return -1;
}

}  // namespace

struct Coefs {
  Decoder d;
  // parse_coefs / load_coefs with a pending entropy decode: the file, for the
  // segments (not value-initialised: load_coefs reads straight into it)
  std::unique_ptr<uint8_t[]> file;
  size_t file_size = 0;
  Coefs(const uint8_t* data, size_t size) : d(data, size) {}
};

Coefs* decode_coefs(const uint8_t* data, size_t size, std::string* err) {
  try {
    auto c = std::make_unique<Coefs>(data, size);
    Decoder& d = c->d;
    d.defer = true;
    d.parse();
    if (!d.frame) fail("Invalid JPEG file structure: missing SOF marker");
    if (d.ncomp == 2 || d.color_space() < 0) fail("unhandled format");
    d.finalize();
    // output()'s one failure, checked here so it comes from the decode call
    // (upsampling reaches it exactly for non-integral factors)
    if (d.ncomp > 1)
      for (int i = 0; i < d.used_components(); i++)
        if (d.max_h % d.comp[i].h != 0 || d.max_v % d.comp[i].v != 0) fail("Fractional sampling not implemented yet");
    d.data = nullptr;
    d.size = 0;
    return c.release();
  } catch (const Error& e) {
    if (err) *err = e.msg;
    return nullptr;
  } catch (const std::bad_alloc&) {
    if (err) *err = "Insufficient memory";
    return nullptr;
  }
}

namespace {
// parse_coefs on a Coefs that already holds the file (c->file, c->file_size).
Coefs* parse_held(std::unique_ptr<Coefs> c, std::string* err) {
  const uint8_t* data = c->file.get();
  const size_t size = c->file_size;
  try {
    Decoder& d = c->d;
    d.data = data;
    d.size = size;
    d.device_entropy = true;
    d.parse();
    if (!d.frame) fail("Invalid JPEG file structure: missing SOF marker");
    if (d.color_space() < 0) fail("unhandled format");
    if (!d.pending) throw NotDevice{};  // no scan
    // decode_coefs' check: output() reaches it exactly for non-integral factors
    if (d.ncomp > 1)
      for (int i = 0; i < d.used_components(); i++)
        if (d.max_h % d.comp[i].h != 0 || d.max_v % d.comp[i].v != 0) fail("Fractional sampling not implemented yet");
    return c.release();
  } catch (const NotDevice&) {
    return decode_coefs(data, size, err);
  } catch (const Error& e) {
    if (err) *err = e.msg;
    return nullptr;
  } catch (const std::bad_alloc&) {
    if (err) *err = "Insufficient memory";
    return nullptr;
  }
}
}  // namespace

Coefs* parse_coefs(const uint8_t* data, size_t size, bool device_entropy, std::string* err) {
  if (!device_entropy) return decode_coefs(data, size, err);
  std::unique_ptr<Coefs> c;
  try {
    c = std::make_unique<Coefs>(nullptr, 0);
    c->file.reset(new uint8_t[size ? size : 1]);
  } catch (const std::bad_alloc&) {
    if (err) *err = "Insufficient memory";
    return nullptr;
  }
  std::memcpy(c->file.get(), data, size);
  c->file_size = size;
  return parse_held(std::move(c), err);
}

Coefs* load_coefs(const char* path, bool device_entropy, bool* not_jpeg, std::string* err) {
  *not_jpeg = false;
  const int fd = ::open(path, O_RDONLY | O_CLOEXEC);
  if (fd < 0) {
    if (err) *err = "could not load <" + std::string(path) + ">";
    return nullptr;
  }
  struct Close {
    int fd;
    ~Close() { ::close(fd); }
  } close_fd{fd};
  struct stat st;
  if (::fstat(fd, &st) != 0 || !S_ISREG(st.st_mode) || st.st_size < 3) {
    if (err) *err = "not a regular file";
    return nullptr;  // the caller's general path reads it
  }
  std::unique_ptr<Coefs> c;
  try {
    c = std::make_unique<Coefs>(nullptr, 0);
    c->file.reset(new uint8_t[(size_t)st.st_size]);
  } catch (const std::bad_alloc&) {
    if (err) *err = "Insufficient memory";
    return nullptr;
  }
  uint8_t* buf = c->file.get();
  size_t got = 0;
  while (got < (size_t)st.st_size) {
    const ssize_t r = ::read(fd, buf + got, (size_t)st.st_size - got);
    if (r < 0 && errno == EINTR) continue;
    if (r <= 0) break;
    got += (size_t)r;
    if (got >= 3 && got - (size_t)r < 3 && !is_jpeg(buf, got)) {
      *not_jpeg = true;
      return nullptr;
    }
  }
  if (got != (size_t)st.st_size) {
    if (err) *err = "short read";
    return nullptr;
  }
  c->file_size = got;
  if (!device_entropy) return decode_coefs(buf, got, err);
  return parse_held(std::move(c), err);
}

void free_coefs(Coefs* c) { delete c; }

EntropyScan entropy_scan(const Coefs* c) {
  const Decoder& d = c->d;
  EntropyScan e{};
  e.nseg = (int)d.seg_begin.size();
  e.seg_begin = d.seg_begin.data();
  e.seg_end = d.seg_end.data();
  e.seg_bytes = d.seg_bytes.data();
  e.data = d.data;
  e.mcus = d.scan_mcus;
  e.restart_interval = d.restart_interval;
  e.interleaved = d.scan_ns > 1 ? 1 : 0;
  e.mcux = d.scan_ns > 1 ? d.mcux : d.comp[d.scan_comp[0]].wib;
  // tables: distinct (class, index) pairs in first-use order
  auto table = [&](int cls, int id) {
    for (int t = 0; t < e.ntables; t++)
      if (e.table_class[t] == cls && e.table_id[t] == id) return t;
    e.table_class[e.ntables] = cls;
    e.table_id[e.ntables] = id;
    return e.ntables++;
  };
  for (int i = 0; i < d.scan_ns; i++) {
    const int ci = d.scan_comp[i];
    const Component& k = d.comp[ci];
    const int nh = d.scan_ns > 1 ? k.h : 1, nv = d.scan_ns > 1 ? k.v : 1;
    for (int v = 0; v < nv; v++)
      for (int h = 0; h < nh; h++) {
        e.blk_comp[e.bpm] = ci;
        e.blk_dx[e.bpm] = h;
        e.blk_dy[e.bpm] = v;
        e.blk_dc[e.bpm] = table(0, k.dc_tbl);
        e.blk_ac[e.bpm] = table(1, k.ac_tbl);
        e.bpm++;
      }
  }
  return e;
}

uint64_t device_table(const Coefs* c, int cls, int table_id, void* huff_dev) {
  const Huff& h = cls ? c->d.ac[table_id] : c->d.dc[table_id];
  // per-thread cache of built tables (a batch's files mostly share theirs),
  // keyed by the class and the derived code: maxcode, valoffset and the symbol values
  struct Entry {
    int32_t maxcode[18], valoffset[18];
    uint8_t vals[256];
    int nvals = -1, cls = -1;
    uint64_t serial = 0;  // this thread's build number: equal serials, equal tables
    HuffDev d;
  };
  constexpr int kEntries = 8;
  thread_local std::unique_ptr<Entry[]> cache;
  thread_local int next = 0;
  thread_local uint64_t builds = 0;
  if (!cache) cache.reset(new Entry[kEntries]);
  for (int k = 0; k < kEntries; k++) {
    const Entry& e = cache[k];
    if (e.nvals == h.nvals && e.cls == cls && std::memcmp(e.maxcode, h.maxcode, sizeof e.maxcode) == 0 &&
        std::memcmp(e.valoffset, h.valoffset, sizeof e.valoffset) == 0 &&
        std::memcmp(e.vals, h.vals, (size_t)h.nvals) == 0) {
      if (huff_dev) *static_cast<HuffDev*>(huff_dev) = e.d;
      return e.serial;
    }
  }
  // built in the cache entry it replaces
  Entry& e = cache[next];
  next = (next + 1) % kEntries;
  e.nvals = -1;
  HuffDev& o = e.d;
  std::memset(&o, 0, sizeof o);
  // The code starting a 16-bit pattern: its length and symbol, jdhuff.c
  // jpeg_huff_decode's search (the shortest l whose l-bit prefix is <=
  // maxcode[l]; canonical codes); none (corrupt data): 16 bits, symbol 0.
  auto code_at = [&](uint32_t p16, int* len, int* sym) {
    for (int l = 1; l <= 16; l++) {
      const int32_t code = (int32_t)(p16 >> (16 - l));
      if (code <= h.maxcode[l]) {
        *len = l;
        *sym = h.vals[(code + h.valoffset[l]) & 0xff];
        return;
      }
    }
    *len = 16;
    *sym = 0;
  };
  // step table over kHuffLook bits (0: a longer code or none)
  uint16_t one[1 << kHuffLook];
  int first_long = 1 << kHuffLook;  // the first kHuffLook-bit prefix without a code that fits it
  for (int i = 0; i < (1 << kHuffLook); i++) {
    int len, sym;
    code_at((uint32_t)i << (16 - kHuffLook), &len, &sym);
    const bool fits = len <= kHuffLook && (int32_t)(i >> (kHuffLook - len)) <= h.maxcode[len];
    one[i] = fits ? huff_step_entry(cls, len, sym) : 0;
    if (!fits && first_long == (1 << kHuffLook)) first_long = i;
  }
  // AC pairs: a symbol other than EOB and the whole next one inside the
  // kHuffLook bits (the next one's entry is that of the remaining bits
  // shifted up: its code and value bits lie in them)
  for (int i = 0; i < (1 << kHuffLook); i++) {
    o.step[i] = huff_step_single(one[i]);
    const int s1 = one[i] & 31, a1 = (one[i] >> 5) & 127;
    if (!cls || !one[i] || a1 == 64 || s1 >= kHuffLook) continue;
    const uint16_t e2 = one[(i << s1) & ((1 << kHuffLook) - 1)];
    if (e2 && (e2 & 31) <= kHuffLook - s1) o.step[i] = huff_step_pair(one[i], e2);
  }
  // longer codes (canonical: every prefix from first_long up to the top has
  // none that fits) over the top kHuffLong 16-bit patterns, indexed from
  // 65536 - kHuffLong (the kernel's constant base), when they lie there
  const int32_t base = first_long << (16 - kHuffLook);
  o.long_base = 65536;
  o.search = 1;
  if (65536 - base <= kHuffLong) {
    bool ok = true;
    for (int i = first_long; i < (1 << kHuffLook); i++) ok = ok && one[i] == 0;
    if (ok) {
      o.search = 0;
      o.long_base = base;
      for (int32_t v = base; v < 65536; v++) {
        int len, sym;
        code_at((uint32_t)v, &len, &sym);
        o.step_long[v - (65536 - kHuffLong)] = huff_step_single(huff_step_entry(cls, len, sym));
      }
    }
  }
  std::memcpy(o.maxcode, h.maxcode, sizeof o.maxcode);
  std::memcpy(o.valoffset, h.valoffset, sizeof o.valoffset);
  std::memcpy(o.vals, h.vals, sizeof o.vals);
  std::memcpy(e.maxcode, h.maxcode, sizeof e.maxcode);
  std::memcpy(e.valoffset, h.valoffset, sizeof e.valoffset);
  std::memcpy(e.vals, h.vals, (size_t)h.nvals);
  e.nvals = h.nvals;
  e.cls = cls;
  e.serial = ++builds;
  if (huff_dev) *static_cast<HuffDev*>(huff_dev) = o;
  return e.serial;
}

namespace {
// Mirrors Bits::fill's byte rules on a segment that ends at its marker's 0xFF.
int64_t unstuff_scalar(const uint8_t* b, const uint8_t* e, uint8_t* o) {
  uint8_t* const o0 = o;
  while (b < e) {
    const uint8_t* f = static_cast<const uint8_t*>(std::memchr(b, 0xFF, (size_t)(e - b)));
    if (!f) {
      std::memcpy(o, b, (size_t)(e - b));
      o += e - b;
      break;
    }
    std::memcpy(o, b, (size_t)(f - b));
    o += f - b;
    if (f + 1 < e && f[1] == 0x00) {
      *o++ = 0xFF;  // stuffed byte
      b = f + 2;
    } else {
      b = f + 1;  // fill byte (0xFF 0xFF ...)
    }
  }
  return (int64_t)(o - o0);
}

// 64 bytes at a time: byte j is dropped when it is 0x00 after an 0xFF, or an
// 0xFF not followed by 0x00 (the same rules, which need only each byte's
// neighbours); the kept bytes are compressed together and stored whole (the
// output never passes the input position, so a full 64-byte store stays
// inside the segment's room).
__attribute__((target("avx512f,avx512bw,avx512vbmi2,popcnt")))
int64_t unstuff_avx512(const uint8_t* b, const uint8_t* e, uint8_t* dst) {
  const __m512i ff = _mm512_set1_epi8((char)0xFF), zero = _mm512_setzero_si512();
  uint8_t* o = dst;
  uint64_t prev_ff = 0;  // the byte before the block was 0xFF
  for (; e - b >= 65; b += 64) {
    const __m512i x = _mm512_loadu_si512(b), y = _mm512_loadu_si512(b + 1);
    const uint64_t isff = _mm512_cmpeq_epi8_mask(x, ff), is00 = _mm512_cmpeq_epi8_mask(x, zero);
    const uint64_t next00 = _mm512_cmpeq_epi8_mask(y, zero);
    const uint64_t drop = (is00 & ((isff << 1) | prev_ff)) | (isff & ~next00);
    _mm512_storeu_si512(o, _mm512_maskz_compress_epi8(~drop, x));
    o += __builtin_popcountll(~drop);
    prev_ff = isff >> 63;
  }
  if (prev_ff && b < e && *b == 0x00) b++;  // the stuffed pair's 0x00 across the block edge
  return (int64_t)(o - dst) + unstuff_scalar(b, e, o);
}
}  // namespace

int64_t unstuff(const uint8_t* b, const uint8_t* e, uint8_t* dst) {
  return have_avx512_bytes() ? unstuff_avx512(b, e, dst) : unstuff_scalar(b, e, dst);
}

CoefInfo coef_info(const Coefs* c) {
  const Decoder& d = c->d;
  CoefInfo r{};
  r.width = d.width;
  r.height = d.height;
  r.ncomp = d.ncomp;
  r.used = d.used_components();
  r.color_space = d.color_space();
  r.max_h = d.max_h;
  r.max_v = d.max_v;
  r.coef = d.pending ? nullptr : d.coefbuf.data();
  r.coef_count = d.coef_total;
  r.entropy_pending = d.pending;
  for (int i = 0; i < d.ncomp; i++) {
    const Component& k = d.comp[i];
    CoefPlane& p = r.comp[i];
    p.h = k.h;
    p.v = k.v;
    p.dw = k.dw;
    p.dh = k.dh;
    p.bw = k.bw;
    p.bh = k.bh;
    p.coded = k.coded;
    p.off = k.off;
    p.q = k.q;
  }
  // grey, YCbCr, RGB, and (round 6) CMYK / YCCK: their first three output
  // channels come from the first three components (ImageJPEG.cpp:112-124
  // keeps C, M, Y of libjpeg's CMYK output; K is never read)
  r.device_ok = !d.lossless && (d.ncomp == 1 || (d.ncomp == 3 && (r.color_space == 1 || r.color_space == 2)) ||
                                (d.ncomp == 4 && (r.color_space == 3 || r.color_space == 4)));
  return r;
}


bool finish(const Coefs* c, uint8_t* dst, int64_t dst_stride, std::string* err) {
  try {
    if (c->d.pending) {
      // the entropy decode was left to the device: run it here now
      std::unique_ptr<Coefs> h(decode_coefs(c->file.get(), c->file_size, err));
      if (!h) return false;
      h->d.output(dst, dst_stride);
      return true;
    }
    c->d.output(dst, dst_stride);
    return true;
  } catch (const Error& e) {
    if (err) *err = e.msg;
    return false;
  } catch (const std::bad_alloc&) {
    if (err) *err = "Insufficient memory";
    return false;
  }
}

bool is_jpeg(const uint8_t* data, size_t size) {
  return size >= 3 && data[0] == 0xFF && data[1] == 0xD8 && data[2] == 0xFF;
}

bool info(const uint8_t* data, size_t size, int* width, int* height, int* components, std::string* err) {
  try {
    Decoder d(data, size);
    if (!is_jpeg(data, size)) fail("Not a JPEG file");
    d.pos = 2;
    for (;;) {
      const int m = d.next_marker();
      if (m < 0) fail("Premature end of JPEG file");
      if (m == 0xC0 || m == 0xC1 || m == 0xC2 || m == 0xC3 || m == 0xC9 || m == 0xCA) {
        d.read_sof(m);
        break;
      }
      if (m == 0xD9 || m == 0xDA) fail("Invalid JPEG file structure: SOS before SOF");
      if (m >= 0xD0 && m <= 0xD7) continue;
      if (m >= 0xC5 && m <= 0xCF && m != 0xC8 && m != 0xC9 && m != 0xCA && m != 0xCC) unsupported_sof(m);
      d.skip_segment();
    }
    *width = d.width;
    *height = d.height;
    *components = d.ncomp;
    return true;
  } catch (const Error& e) {
    if (err) *err = e.msg;
    return false;
  }
}

bool decode(const uint8_t* data, size_t size, uint8_t* dst, int64_t dst_stride, int width, int height,
            std::string* err) {
  try {
    Decoder d(data, size);
    d.parse();
    if (!d.frame) fail("Invalid JPEG file structure: missing SOF marker");
    if (d.width != width || d.height != height) fail("mxd: output buffer does not match the image size");
    if (d.ncomp == 2 || d.color_space() < 0) fail("unhandled format");
    d.finalize();
    d.output(dst, dst_stride);
    return true;
  } catch (const Error& e) {
    if (err) *err = e.msg;
    return false;
  } catch (const std::bad_alloc&) {
    if (err) *err = "Insufficient memory";
    return false;
  }
}

}  // namespace jpeg
}  // namespace mxd
