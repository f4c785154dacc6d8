// jpeghuff.hip -- device-side Huffman (entropy) decode of sequential JPEG
// scans: the half of load_image's decode (ImageJPEG.cpp:99-146, libjpeg's
// jdhuff.c) that round 3 still ran on the host (VERDICT r3 missing 1).  The
// algorithm and data layout are described in jpeghuff.h; the arithmetic is
// jpeg.cpp's host block decoder (Bits::block_seq), symbol by symbol, so the
// coefficients are the host decoder's bit for bit (tests/test_gpu_jpeg_entropy.py).
//
// One workgroup per job (segments of one image, <= kHuffThreads
// subsequences), one thread per subsequence:
//   0. the image's Huffman tables into LDS; its coefficient blocks zeroed;
//   1. synchronisation rounds: every subsequence whose start state changed
//      decodes to its end; each hands its exit state to the next one of its
//      segment; repeat until no state changes;
//   2. block counts prefix-summed per segment -> each subsequence's first block;
//   3. write pass: decode again, storing AC coefficients and DC differences;
//   4. DC: per-component sums of the differences prefix-summed per segment,
//      then each subsequence turns its blocks' differences into values.
#include <hip/hip_runtime.h>

#include "jpeghuff.h"

namespace mxd {
namespace {


// Diagnostic builds only (-DMXD_HUFF_STATS=1; never in the product library):
// per job, the synchronisation rounds and the symbols decoded in them and in
// the write pass, and the durations of the phases (s_memrealtime ticks, 10 ns:
// staging, synchronisation, write pass, DC), read back with
// mxd_debug_huff_stats (kStatInts per job).
#ifndef MXD_HUFF_STATS
#define MXD_HUFF_STATS 0
#endif
// One decode path for DC and AC symbols (default; tuning builds
// -DMXD_HUFF_UNIFIED=0 keep separate DC / fast-AC / general paths, whose
// divergence cost 28 % more kernel time: 1.48 vs 1.15 ms per C4 batch of
// 128, profiles/r04/r04h_*).
#ifndef MXD_HUFF_UNIFIED
#define MXD_HUFF_UNIFIED 1
#endif
// The symbol step without per-kind branches (default; tuning builds
// -DMXD_HUFF_LEAN=0 keep the if / else chain of the unified step): code and
// value bits consumed by one shift, the next coefficient index and block
// selected arithmetically, one word refilled per step.
#ifndef MXD_HUFF_LEAN
#define MXD_HUFF_LEAN 1
#endif
// Branch-free refill in the lean step and the synchronisation loop's exit on
// the subsequence end alone (default; tuning builds -DMXD_HUFF_LEAN2=0).
#ifndef MXD_HUFF_LEAN2
#define MXD_HUFF_LEAN2 1
#endif
// The LDS reader loads each word one refill ahead (default; tuning builds
// -DMXD_HUFF_PREFETCH=0 load it when needed, on the symbol loop's dependency
// chain: kernel 0.961 vs 1.094 ms per batch-bench call, profiles/r04/r04x_*).
#ifndef MXD_HUFF_PREFETCH
#define MXD_HUFF_PREFETCH 1
#endif
// The lean step's next coefficient index by one select and every symbol's
// store unconditional (tuning builds -DMXD_HUFF_LEAN3=1).
#ifndef MXD_HUFF_LEAN3
#define MXD_HUFF_LEAN3 0
#endif
// The class-specific step table (HuffDev::step; default): one lookup gives
// the bits consumed, the index advance and the value bits, and implies
// LEAN3's write-pass form (every symbol stores; tuning builds
// -DMXD_HUFF_LEAN4=0 -DMXD_HUFF_LEAN3=0 restore the earlier step: kernel
// 0.761 vs 0.692 (LEAN3) vs 0.634 ms (LEAN4) per batch-bench call,
// profiles/r04/r04ag_*).
#ifndef MXD_HUFF_LEAN4
#define MXD_HUFF_LEAN4 1
#endif
// The synchronisation loop runs MXD_HUFF_UNROLL steps per check while the
// subsequence's end is further than UNROLL - 1 steps (2, default, or 4; 1
// checks every step: kernel 0.633 (1) vs 0.564 ms (2) per batch-bench call,
// profiles/r04/r04ah_*); the write pass likewise runs MXD_HUFF_WUNROLL.
// Byte-swapping the words once while they are staged into LDS instead of at
// every refill measured nothing (0.632 ms) and is not kept.
#ifndef MXD_HUFF_UNROLL
#define MXD_HUFF_UNROLL 2
#endif
#ifndef MXD_HUFF_WUNROLL
#define MXD_HUFF_WUNROLL 1
#endif
// The LDS reader takes words past its segment from the segment's zero
// padding (default; tuning builds -DMXD_HUFF_ZPAD=0 select zero instead:
// 0.568 vs 0.535 ms, profiles/r04/r04aj_*).
#ifndef MXD_HUFF_ZPAD
#define MXD_HUFF_ZPAD 1
#endif
#if !(MXD_HUFF_UNIFIED && MXD_HUFF_LEAN)
// the earlier steps keep the earlier write-pass form
#undef MXD_HUFF_LEAN3
#define MXD_HUFF_LEAN3 0
#undef MXD_HUFF_LEAN4
#define MXD_HUFF_LEAN4 0
#elif MXD_HUFF_LEAN4
#undef MXD_HUFF_LEAN3
#define MXD_HUFF_LEAN3 1
#endif

#if MXD_HUFF_STATS
constexpr int kStatJobs = 1 << 16;
constexpr int kStatInts = 16;
__device__ int g_huff_stats[kStatJobs * kStatInts];
__device__ __forceinline__ uint64_t stat_clock() { return __builtin_amdgcn_s_memrealtime(); }
__device__ __forceinline__ uint64_t stat_cycles() { return __builtin_amdgcn_s_memtime(); }
#endif

// Bit readers over one segment's unstuffed bytes (32-bit words, big-endian
// byte order); words past the segment read as zeros (libjpeg's zeros past
// the data).  After refill() at least 33 bits are buffered.
//
// LdsReader: the job's words staged in LDS.
struct LdsReader {
  const uint32_t* w;
  int32_t nw;
  uint64_t buf;
  int32_t cnt, wi;
#if MXD_HUFF_PREFETCH
  uint32_t nxt;  // w[wi] (clamped into the segment), loaded one refill ahead
#endif

  // base: the job's words in LDS; w0 / nw: the segment's first word and words
  __device__ __forceinline__ void init(const void* base, int32_t w0, int32_t nwords) {
    w = static_cast<const uint32_t*>(base) + w0;
    nw = nwords;
  }

#if MXD_HUFF_PREFETCH
  static __device__ __forceinline__ uint32_t order(uint32_t x) { return __builtin_bswap32(x); }
#if MXD_HUFF_ZPAD
  // w[nw] is a zero word: every segment is staged with >= 4 zero bytes past
  // its data, rounded up to 16 (hostpath.cpp), so words past the segment
  // read as w[nw] without a separate zero select
  __device__ __forceinline__ uint32_t word(int32_t i) const { return w[min(i, nw)]; }
  __device__ __forceinline__ bool inside() const { return true; }
#else
  __device__ __forceinline__ uint32_t word(int32_t i) const { return w[i < nw ? i : max(nw - 1, 0)]; }
  __device__ __forceinline__ bool inside() const { return wi < nw; }
#endif
  // one word (the caller knows cnt <= 32)
  __device__ __forceinline__ void refill1() {
    const uint32_t x = inside() ? order(nxt) : 0u;
    buf |= (uint64_t)x << (32 - cnt);
    cnt += 32;
    wi++;
    nxt = word(wi);
  }
  // refill1 when cnt <= 32, without a branch (the word load is issued either way)
  __device__ __forceinline__ void refill_if() {
    const bool need = cnt <= 32;
    const uint32_t x = need && inside() ? order(nxt) : 0u;
    buf |= (uint64_t)x << (need ? 32 - cnt : 0);
    cnt += need ? 32 : 0;
    wi += need ? 1 : 0;
    nxt = word(wi);
  }
  __device__ __forceinline__ void refill() {
    while (cnt <= 32) {
      const uint32_t x = inside() ? order(nxt) : 0u;
      buf |= (uint64_t)x << (32 - cnt);
      cnt += 32;
      wi++;
      nxt = word(wi);  // for the next refill: its latency overlaps this step's decode
    }
  }
  __device__ __forceinline__ void seek(int32_t bit) {
    wi = bit >> 5;
    nxt = word(wi);
    buf = 0;
    cnt = 0;
    refill();
    const int s = bit & 31;
    buf <<= s;
    cnt -= s;
  }
#else
  __device__ __forceinline__ void refill1() {
    const uint32_t x = wi < nw ? __builtin_bswap32(w[wi]) : 0u;
    buf |= (uint64_t)x << (32 - cnt);
    cnt += 32;
    wi++;
  }
  __device__ __forceinline__ void refill_if() {
    if (cnt <= 32) refill1();
  }
  __device__ __forceinline__ void refill() {
    while (cnt <= 32) {
      const uint32_t x = wi < nw ? __builtin_bswap32(w[wi]) : 0u;
      buf |= (uint64_t)x << (32 - cnt);
      cnt += 32;
      wi++;
    }
  }
  __device__ __forceinline__ void seek(int32_t bit) {
    wi = bit >> 5;
    buf = 0;
    cnt = 0;
    refill();
    const int s = bit & 31;
    buf <<= s;
    cnt -= s;
  }
#endif
  __device__ __forceinline__ int32_t pos() const { return wi * 32 - cnt; }
  __device__ __forceinline__ uint32_t take(int n) {  // n <= 16 bits (n = 0: 0)
    const uint32_t v = n ? (uint32_t)(buf >> (64 - n)) : 0u;
    buf <<= n;
    cnt -= n;
    return v;
  }
};

// GlobalReader: the job's words in device memory (jobs whose words do not
// fit LDS), read in 16-byte chunks two chunks ahead of the one being
// consumed, so a chunk's load latency hides behind ~256 bits of decoding
// instead of stalling every word.  Chunks past the segment are not loaded.
struct GlobalReader {
  const uint4* chunks;  // the job's words (16-byte aligned)
  int32_t w0, nw;       // the segment's first word (relative to the job's) and its words
  int32_t last_chunk;   // the segment's last chunk
  uint64_t buf;
  int32_t cnt, wi;      // wi: next word, relative to the segment
  int32_t ca;           // chunk held in A; B, C: the next two
  uint4 A, B, C;

  // base: the job's words in device memory
  __device__ __forceinline__ void init(const void* base, int32_t w0_, int32_t nwords) {
    chunks = static_cast<const uint4*>(base);
    w0 = w0_;
    nw = nwords;
    last_chunk = (w0_ + nwords - 1) >> 2;
  }

  __device__ __forceinline__ uint4 fetch(int32_t ch) const {
    return ch <= last_chunk ? chunks[ch] : uint4{0u, 0u, 0u, 0u};
  }
  __device__ __forceinline__ void refill1() {
    const int32_t a = w0 + wi;
    if ((a >> 2) != ca) {
      A = B;
      B = C;
      ca++;
      C = fetch(ca + 2);
    }
    const int i = a & 3;
    const uint32_t v = i == 0 ? A.x : i == 1 ? A.y : i == 2 ? A.z : A.w;
    const uint32_t x = wi < nw ? __builtin_bswap32(v) : 0u;
    buf |= (uint64_t)x << (32 - cnt);
    cnt += 32;
    wi++;
  }
  __device__ __forceinline__ void refill_if() {
    if (cnt <= 32) refill1();
  }
  __device__ __forceinline__ void refill() {
    while (cnt <= 32) {
      const int32_t a = w0 + wi;
      if ((a >> 2) != ca) {  // words are consumed in order: the next chunk
        A = B;
        B = C;
        ca++;
        C = fetch(ca + 2);
      }
      const int i = a & 3;
      const uint32_t v = i == 0 ? A.x : i == 1 ? A.y : i == 2 ? A.z : A.w;
      const uint32_t x = wi < nw ? __builtin_bswap32(v) : 0u;
      buf |= (uint64_t)x << (32 - cnt);
      cnt += 32;
      wi++;
    }
  }
  __device__ __forceinline__ void seek(int32_t bit) {
    wi = bit >> 5;
    ca = (w0 + wi) >> 2;
    A = fetch(ca);
    B = fetch(ca + 1);
    C = fetch(ca + 2);
    buf = 0;
    cnt = 0;
    refill();
    const int s = bit & 31;
    buf <<= s;
    cnt -= s;
  }
  __device__ __forceinline__ int32_t pos() const { return wi * 32 - cnt; }
  __device__ __forceinline__ uint32_t take(int n) {
    const uint32_t v = n ? (uint32_t)(buf >> (64 - n)) : 0u;
    buf <<= n;
    cnt -= n;
    return v;
  }
};

// jdhuff.c jpeg_huff_decode on a buffer of >= 16 bits: a code longer than 16
// bits (corrupt data) consumes 16 bits and decodes as 0.
template <class Reader>
__device__ __forceinline__ int huff_symbol(const HuffDev& t, Reader& r) {
  const int e = t.look[(uint32_t)(r.buf >> (64 - kHuffLook))];
  if (e) {
    r.buf <<= e >> 8;
    r.cnt -= e >> 8;
    return e & 0xff;
  }
  int l = kHuffLook + 1;
  int32_t code = (int32_t)(r.buf >> (64 - l));
  while (code > t.maxcode[l]) {
    if (++l > 16) {
      r.buf <<= 16;
      r.cnt -= 16;
      return 0;
    }
    code = (int32_t)(r.buf >> (64 - l));
  }
  r.buf <<= l;
  r.cnt -= l;
  return t.vals[(code + t.valoffset[l]) & 0xff];
}

// A code longer than kHuffLook bits without a loop: its length is the
// shortest l in kHuffLook+1..16 whose l-bit prefix is <= maxcode[l] (canonical
// codes; jdhuff.c jpeg_huff_decode's search); none (corrupt data) consumes 16
// bits and decodes as 0, as huff_symbol does.
template <class Reader>
[[maybe_unused]] __device__ __forceinline__ int huff_long(const HuffDev& t, Reader& r) {
  const uint32_t p16 = (uint32_t)(r.buf >> 48);
  int len = 17;
#pragma unroll
  for (int l = 16; l > kHuffLook; l--)
    if ((int32_t)(p16 >> (16 - l)) <= t.maxcode[l]) len = l;
  if (len > 16) {
    r.buf <<= 16;
    r.cnt -= 16;
    return 0;
  }
  const int32_t code = (int32_t)(p16 >> (16 - len));
  r.buf <<= len;
  r.cnt -= len;
  return t.vals[(code + t.valoffset[len]) & 0xff];
}

// huff_long's search without consuming: the code's length (16 for corrupt
// data, whose symbol is 0) and its symbol.
[[maybe_unused]] __device__ __forceinline__ void huff_long_peek(const HuffDev& t, uint64_t buf, int& len, int& sym) {
  const uint32_t p16 = (uint32_t)(buf >> 48);
  int l = 17;
#pragma unroll
  for (int ll = 16; ll > kHuffLook; ll--)
    if ((int32_t)(p16 >> (16 - ll)) <= t.maxcode[ll]) l = ll;
  if (l > 16) {
    len = 16;
    sym = 0;
  } else {
    len = l;
    sym = t.vals[((int32_t)(p16 >> (16 - l)) + t.valoffset[l]) & 0xff];
  }
}

__device__ __forceinline__ int extend(uint32_t v, int s) {
  return s == 0 ? 0 : (int)v < (1 << (s - 1)) ? (int)v + ((-1) << s) + 1 : (int)v;
}

// One segment of the job in LDS.
struct SegLds {
  int32_t word;  // first word, relative to the job's first word
  int32_t bits;
  int32_t mcu0, mcus;
};

// Per-job shared state (static part; the tables, segment records and, when
// they fit, the job's words follow in dynamic LDS: jpeg_huff_lds_bytes).
struct Shared {
  HuffImgDev img;
  int32_t seg_sub0[kHuffThreads];  // first subsequence of each segment of the job
  int32_t in_pos[kHuffThreads], out_pos[kHuffThreads];
  int8_t in_b[kHuffThreads], in_k[kHuffThreads], out_b[kHuffThreads], out_k[kHuffThreads];
  int32_t done[kHuffThreads];      // blocks a subsequence completes (sync pass)
  int64_t blk_off[kHuffMaxBlocks];  // block j of an MCU: offset of MCU (0, 0)'s block j in the coefficients,
  int32_t blk_mxs[kHuffMaxBlocks];  // and its steps per MCU column / row (non-interleaved: per block)
  int32_t blk_mys[kHuffMaxBlocks];
  int16_t sub_seg[kHuffThreads];   // segment of each subsequence
  int16_t list[kHuffThreads];      // this round's subsequences to decode (compacted)
  int32_t scan[kHuffThreads / 64];
  int32_t flag[2];
};

// Block-wide exclusive prefix sum of v (every thread of the workgroup calls it).
__device__ int block_exclusive_scan(int v, int* totals, int* total_out) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, nw = (blockDim.x + 63) >> 6;
  int x = v;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const int y = __shfl_up(x, d, 64);
    if (lane >= d) x += y;
  }
  if (lane == 63) totals[wave] = x;
  __syncthreads();
  if (wave == 0) {
    int t = lane < nw ? totals[lane] : 0;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
      const int y = __shfl_up(t, d, 64);
      if (lane >= d) t += y;
    }
    if (lane < nw) totals[lane] = t;  // inclusive wave totals
  }
  __syncthreads();
  const int before = wave > 0 ? totals[wave - 1] : 0;
  const int total = totals[nw - 1];
  __syncthreads();  // totals may be reused by the next call
  if (total_out) *total_out = total;
  return before + x - v;
}

// Decoder state machine over one segment: block b of the MCU, next
// coefficient k (0 = the DC difference), symbols from Reader r.
struct Dec {
  const HuffImgDev* im;
  const HuffDev* tab;
  int b, k;
  // per-block table indices and components in registers instead of LDS
  // reads per symbol
  uint32_t dpack, apack;  // the DC / AC table of each block of the MCU (bits 3b..3b+2)
  uint32_t cpack;         // component of each block of the MCU (bits 2b..2b+1)
  int bpm;

  __device__ __forceinline__ void init(const HuffImgDev* im_, const HuffDev* tab_) {
    im = im_;
    tab = tab_;
    b = k = 0;
    bpm = im_->bpm;
    dpack = apack = cpack = 0;
    for (int j = 0; j < bpm; j++) {
      dpack |= (uint32_t)(im_->blk_dc[j] & 7) << (3 * j);
      apack |= (uint32_t)(im_->blk_ac[j] & 7) << (3 * j);
      cpack |= (uint32_t)(im_->blk_comp[j] & 3) << (2 * j);
    }
  }
  // component of the current block
  __device__ __forceinline__ int comp() const { return (cpack >> (2 * b)) & 3; }

  // Decodes one symbol.  Returns true at the end of a block (b, k advanced to
  // the next block's start).  For the write pass, on_dc(diff) / on_ac(pos,
  // value) receive the block's values.
#if MXD_HUFF_UNIFIED && MXD_HUFF_LEAN
  template <class Reader, class OnDc, class OnAc>
  __device__ __forceinline__ bool step(Reader& r, OnDc&& on_dc, OnAc&& on_ac) {
#if MXD_HUFF_LEAN2
    r.refill_if();  // >= 33 bits buffered: a step consumes <= 16 + 15
#else
    if (r.cnt <= 32) r.refill1();
#endif
    const bool dc = k == 0;
    const HuffDev& t = tab[((dc ? dpack : apack) >> (3 * b)) & 7];
#if MXD_HUFF_LEAN4
    // one lookup gives the bits to consume, the index advance and the value
    // bits (HuffDev::step, built for the table's class)
    int st = t.step[(uint32_t)(r.buf >> (64 - kHuffLook))];
    if (!st) {
      int len, sym;
      huff_long_peek(t, r.buf, len, sym);
      st = huff_step_entry(dc ? 0 : 1, len, sym);
    }
    const int shift = st & 31, adv = (st >> 5) & 127, sz = st >> 12;
    // value bits: the sz bits after the code, in the buffer's top 32 bits (shift <= 31)
    const uint32_t hi = (uint32_t)(r.buf >> 32);
    const uint32_t raw = sz ? (hi >> (32 - shift)) & ((1u << sz) - 1u) : 0u;
    r.buf <<= shift;
    r.cnt -= shift;
    const int v = extend(raw, sz);
    // the index advance: DC 1, a coefficient run + 1 (stored at k + run), ZRL
    // 16 (its zero at k + 15), EOB 64 (its zero at 63): every position stored
    // is one of the block's not yet written
    const int knew = k + adv;
    on_ac(min(knew - 1, 63), v);
    on_dc(dc, v);
#else
    const int e = t.look[(uint32_t)(r.buf >> (64 - kHuffLook))];
    int len, sym;
    if (e) {
      len = e >> 8;
      sym = e & 0xff;
    } else {
      huff_long_peek(t, r.buf, len, sym);
    }
    const int sz = dc ? sym : sym & 15;
    const int run = dc ? 0 : sym >> 4;
    const uint32_t raw = sz ? (uint32_t)((r.buf << len) >> (64 - sz)) : 0u;
    r.buf <<= len + sz;
    r.cnt -= len + sz;
    const int v = extend(raw, sz);
    const int kpos = k + run;  // an AC coefficient's index (sz != 0)
#if MXD_HUFF_LEAN3
    // next index: kpos + 1 after the DC (k = run = 0), a coefficient or a ZRL
    // (run 15: k + 16); 64 after an EOB.  Every symbol stores: the DC at 0, a
    // coefficient at kpos (a corrupt run past 63 lands on 63), and an EOB / ZRL
    // its zero at an index of the block not yet written -- so no branch.
    const int knew = (dc || sz != 0 || run == 15) ? kpos + 1 : 64;
    on_ac(min(kpos, 63), v);
    on_dc(dc, v);
#else
    // next index: after the DC 1; after a coefficient kpos + 1; ZRL k + 16; EOB 64
    const int knew = dc ? 1 : sz ? kpos + 1 : run == 15 ? k + 16 : 64;
    if (dc) on_dc(v);
    else if (sz) on_ac(kpos, v);
#endif
#endif  // MXD_HUFF_LEAN4
    const bool end = knew >= 64;
    k = end ? 0 : knew;
    b = end ? (b + 1 == bpm ? 0 : b + 1) : b;
    return end;
  }
#elif MXD_HUFF_UNIFIED
  // One path for DC and AC symbols: the
  // block's DC or AC table is selected, one lookup gives the symbol (codes
  // past the lookahead without a loop), the value bits follow; the lanes of a
  // wave, whichever symbol kind each decodes, run the same instructions.
  template <class Reader, class OnDc, class OnAc>
  __device__ __forceinline__ bool step(Reader& r, OnDc&& on_dc, OnAc&& on_ac) {
    if (r.cnt < 32) r.refill();
    const bool dc = k == 0;
    const HuffDev& t = tab[((dc ? dpack : apack) >> (3 * b)) & 7];
    const int e = t.look[(uint32_t)(r.buf >> (64 - kHuffLook))];
    int sym;
    if (e) {
      r.buf <<= e >> 8;
      r.cnt -= e >> 8;
      sym = e & 0xff;
    } else {
      sym = huff_long(t, r);
    }
    const int run = dc ? 0 : sym >> 4, sz = dc ? sym : sym & 15;
    const int v = extend(r.take(sz), sz);
    bool end = false;
    if (dc) {
      on_dc(v);
      k = 1;
    } else if (sz) {
      k += run;
      on_ac(k, v);
      end = ++k >= 64;
    } else if (run == 15) {
      k += 16;
      end = k >= 64;
    } else {
      end = true;
    }
    if (end) {
      k = 0;
      b = b + 1 == bpm ? 0 : b + 1;
    }
    return end;
  }
#else
  template <class Reader, class OnDc, class OnAc>
  __device__ __forceinline__ bool step(Reader& r, OnDc&& on_dc, OnAc&& on_ac) {
    if (r.cnt < 32) r.refill();
    if (k == 0) {
      const int s = huff_symbol(tab[im->blk_dc[b]], r);
      on_dc(extend(r.take(s), s));
      k = 1;
      return false;
    }
    const HuffDev& t = tab[im->blk_ac[b]];
    const uint32_t f = t.fac[(uint32_t)(r.buf >> (64 - kHuffFacLook))];
    bool end;
    if (f >> 24) {
      r.buf <<= f >> 24;
      r.cnt -= f >> 24;
      const int run = (f >> 16) & 0xff;
      if (run == 0xff) {
        end = true;
      } else {
        k += run;
        on_ac(k, (int)(int16_t)(f & 0xffff));
        end = ++k >= 64;
      }
    } else {
      const int rs = huff_symbol(t, r);
      const int run = rs >> 4, sz = rs & 15;
      if (sz) {
        k += run;
        on_ac(k, extend(r.take(sz), sz));
        end = ++k >= 64;
      } else if (run == 15) {
        k += 16;
        end = k >= 64;
      } else {
        end = true;
      }
    }
    if (end) {
      k = 0;
      b = b + 1 == im->bpm ? 0 : b + 1;
    }
    return end;
  }
#endif
};

// Coefficient offset of block g (decode order) of the image: blocks number
// < 2^31 (the host refuses larger images), so 32-bit divisions.
__device__ __forceinline__ int64_t block_addr(const HuffImgDev& im, int64_t g64) {
  const uint32_t g = (uint32_t)g64;
  if (!im.interleaved) {
    const uint32_t by = g / (uint32_t)im.mcux, bx = g - by * (uint32_t)im.mcux;
    return im.coef + im.plane[0] + ((int64_t)by * im.bw[0] + bx) * 64;
  }
  const uint32_t m = g / (uint32_t)im.bpm;
  const int j = (int)(g - m * (uint32_t)im.bpm);
  const int c = im.blk_comp[j];
  const uint32_t my = m / (uint32_t)im.mcux, mx = m - my * (uint32_t)im.mcux;
  const int64_t bx = (int64_t)mx * im.comp_h[c] + im.blk_dx[j], by = (int64_t)my * im.comp_v[c] + im.blk_dy[j];
  return im.coef + im.plane[c] + (by * im.bw[c] + bx) * 64;
}

// Dynamic LDS of a job: its tables, its segment records, then (job.lds)
// its words.
__host__ __device__ constexpr int64_t lds_tables_bytes(int ntables) { return (int64_t)ntables * sizeof(HuffDev); }
__host__ __device__ constexpr int64_t lds_words_at(int ntables, int nseg) {
  return (lds_tables_bytes(ntables) + (int64_t)nseg * sizeof(SegLds) + 15) / 16 * 16;
}

// One thread's subsequence: its segment (in LDS form), its index in the
// segment and its bit range.
struct Sub {
  SegLds sg;
  int j;
  bool active, first, last;
  int32_t start, end;
};

// Subsequence `id` of the job (its segment from sh.sub_seg).
__device__ __forceinline__ Sub sub_of(const Shared& sh, const SegLds* seg, int sub_bits, int id, int nsub) {
  Sub v;
  const int si = sh.sub_seg[id];
  v.sg = seg[si];
  v.j = id - sh.seg_sub0[si];
  const int nseg_sub = max(1, (v.sg.bits + sub_bits - 1) / sub_bits);
  v.active = id < nsub;
  v.first = v.j == 0;
  v.last = v.j == nseg_sub - 1;
  v.start = v.j * sub_bits;
  v.end = v.last ? 0x7fffffff : v.start + sub_bits;
  return v;
}

// Each round's subsequences packed onto the first threads (default; tuning
// builds -DMXD_HUFF_COMPACT=0 let every thread decode its own: 0.824 vs
// 0.750 ms per batch-bench call with the lean step, profiles/r04/r04ad_*).
#ifndef MXD_HUFF_COMPACT
#define MXD_HUFF_COMPACT 1
#endif
// Tuning builds (-DMXD_HUFF_OVERLAP=<bits>): round 0 decodes that many bits
// before each subsequence's start from the guessed state.
#ifndef MXD_HUFF_OVERLAP
#define MXD_HUFF_OVERLAP 0
#endif

#if MXD_HUFF_STATS
struct Stats {
  int sync_syms = 0, write_syms = 0, rounds = 0;
  uint64_t t[4] = {0, 0, 0, 0};  // thread 0: staged, synchronised, written, done
  uint64_t c[2] = {0, 0};        // thread 0: shader clock at the write pass's start and end
  uint64_t r[2] = {0, 0};        // and the real-time clock there
  int chg = 0, chg_pos = 0, chg_k = 0;  // start-state changes after round 0: all, same bit position, same (position, k)
};
#else
struct Stats {};
#endif

// Passes 1-3 over the job with bit reader `rd` (LdsReader or GlobalReader):
// synchronisation rounds, each subsequence's first block, the write pass.
// Leaves the subsequence's per-component DC-difference sums in dcsum and the
// blocks whose DC it decoded in [dc0, dc1).
template <class R>
__device__ __forceinline__ void decode_passes(const void* wbase, Shared& sh, const HuffImgDev& im, const HuffDev* tab,
                                              const SegLds* seg, int sub_bits, int nsub, const Sub& u,
                                              int16_t* coef, int (&dcsum)[3], int64_t& dc0, int64_t& dc1,
                                              Stats& st) {
  const int t = threadIdx.x;
  Dec dec;
  dec.init(&im, tab);
  const auto nop_dc = [](auto...) {};
  const auto nop_ac = [](auto...) {};
  R rd;

  // 1. synchronisation rounds (the last subsequence of a segment hands its
  // state to nobody: it decodes only in the write pass)
  bool need = u.active && !u.last;
  for (int round = 0;; round++) {
#if MXD_HUFF_STATS
    st.rounds = round + 1;
#endif
    // this round's subsequences: compacted onto the first threads, so a
    // round in which few start states changed runs few waves
#if MXD_HUFF_COMPACT
    int nact = 0;
    const int slot = block_exclusive_scan(need ? 1 : 0, sh.scan, &nact);
    if (need) sh.list[slot] = (int16_t)t;
    __syncthreads();
    const bool work = t < nact;
    const int id = work ? sh.list[t] : t;
#else
    const bool work = need;
    const int id = t;
#endif
    if (work) {
      const Sub v = sub_of(sh, seg, sub_bits, id, nsub);
      rd.init(wbase, v.sg.word, (v.sg.bits + 31) >> 5);
#if MXD_HUFF_OVERLAP > 0
      // round 0: start the guess MXD_HUFF_OVERLAP bits early, so the decoder
      // has had that long to fall into step when it reaches the subsequence
      if (round == 0 && !v.first) {
        rd.seek(max(0, v.start - MXD_HUFF_OVERLAP));
        dec.b = 0;
        dec.k = 0;
        while (rd.pos() < v.start) dec.step(rd, nop_dc, nop_ac);
        sh.in_pos[id] = rd.pos();
        sh.in_b[id] = (int8_t)dec.b;
        sh.in_k[id] = (int8_t)dec.k;
      } else
#endif
      {
        rd.seek(sh.in_pos[id]);
        dec.b = sh.in_b[id];
        dec.k = sh.in_k[id];
      }
      int done = 0;
#if MXD_HUFF_UNROLL > 1
      // a step consumes <= 31 bits: while the end is further than UNROLL - 1
      // steps can reach, the next UNROLL steps all start before it
      while (rd.pos() + 31 * (MXD_HUFF_UNROLL - 1) < v.end) {
#pragma unroll
        for (int i = 0; i < MXD_HUFF_UNROLL; i++) done += dec.step(rd, nop_dc, nop_ac) ? 1 : 0;
#if MXD_HUFF_STATS
        st.sync_syms += MXD_HUFF_UNROLL;
#endif
      }
#endif
      for (;;) {
        const int32_t p = rd.pos();
        // the segment's end can only stop the last subsequence, which the rounds never decode
#if MXD_HUFF_LEAN2
        if (p >= v.end) break;
#else
        if (p >= v.end || (dec.b == 0 && dec.k == 0 && p > v.sg.bits)) break;
#endif
        done += dec.step(rd, nop_dc, nop_ac) ? 1 : 0;
#if MXD_HUFF_STATS
        st.sync_syms++;
#endif
      }
      sh.out_pos[id] = rd.pos();
      sh.out_b[id] = (int8_t)dec.b;
      sh.out_k[id] = (int8_t)dec.k;
      sh.done[id] = done;
    }
    need = false;
    __syncthreads();
    if (t == 0) sh.flag[(round + 1) & 1] = 0;
    if (u.active && !u.first) {
      const int32_t p = sh.out_pos[t - 1];
      const int8_t b = sh.out_b[t - 1], k = sh.out_k[t - 1];
      if (p != sh.in_pos[t] || b != sh.in_b[t] || k != sh.in_k[t]) {
#if MXD_HUFF_STATS
        if (round > 0) {
          st.chg++;
          st.chg_pos += p == sh.in_pos[t] ? 1 : 0;
          st.chg_k += p == sh.in_pos[t] && k == sh.in_k[t] ? 1 : 0;
        }
#endif
        sh.in_pos[t] = p;
        sh.in_b[t] = b;
        sh.in_k[t] = k;
        need = !u.last;
        sh.flag[round & 1] = 1;
      }
    }
    __syncthreads();
    if (!sh.flag[round & 1]) break;
  }
#if MXD_HUFF_STATS
  st.t[1] = stat_clock();
#endif

  // 2. first block of each subsequence: the blocks completed before it in its segment
  const int before = block_exclusive_scan(u.active && !u.last ? sh.done[t] : 0, sh.scan, nullptr);
  __syncthreads();
  sh.done[t] = before;  // reuse: exclusive prefix (over the whole job)
  __syncthreads();
  const int64_t seg_block0 = (int64_t)u.sg.mcu0 * im.bpm, seg_block1 = ((int64_t)u.sg.mcu0 + u.sg.mcus) * im.bpm;
  int64_t g = seg_block0 + (u.active ? before - sh.done[t - u.j] : 0);

  // 3. write pass
#if MXD_HUFF_STATS
  __syncthreads();
  st.c[0] = stat_cycles();
  st.r[0] = stat_clock();
#endif
  if (u.active) {
    rd.init(wbase, u.sg.word, (u.sg.bits + 31) >> 5);
    rd.seek(sh.in_pos[t]);
    dec.b = sh.in_b[t];
    dec.k = sh.in_k[t];
    // block cursor: (MCU column, row, block of the MCU), advanced without divisions
    const uint32_t bpm = (uint32_t)im.bpm, mcux = (uint32_t)im.mcux;
    const uint32_t g0 = (uint32_t)min(g, seg_block1 - 1), m0 = g0 / bpm;
    uint32_t cj = g0 - m0 * bpm, cmy = m0 / mcux, cmx = m0 - cmy * mcux;
    auto addr = [&]() {
      return coef + im.coef + sh.blk_off[cj] + (int64_t)cmy * sh.blk_mys[cj] + (int64_t)cmx * sh.blk_mxs[cj];
    };
    int16_t* blk = addr();
    auto wstep = [&]() {
#if MXD_HUFF_LEAN3
      const bool fin = dec.step(
          rd,
          [&](bool dc, int diff) {
            const int c = dec.comp();
            dcsum[0] += dc && c == 0 ? diff : 0;
            dcsum[1] += dc && c == 1 ? diff : 0;
            dcsum[2] += dc && c == 2 ? diff : 0;
            dc0 = dc && dc0 < 0 ? g : dc0;
            dc1 = dc ? g + 1 : dc1;
          },
          // zig-zag order (jpeg_idct reorders)
          [&](int kk, int v) { blk[kk] = (int16_t)v; });
#else
      const bool fin = dec.step(
          rd,
          [&](int diff) {
            blk[0] = (int16_t)diff;
            const int c = (dec.cpack >> (2 * dec.b)) & 3;
            dcsum[0] += c == 0 ? diff : 0;
            dcsum[1] += c == 1 ? diff : 0;
            dcsum[2] += c == 2 ? diff : 0;
            if (dc0 < 0) dc0 = g;
            dc1 = g + 1;
          },
          [&](int kk, int v) {
            // zig-zag order (jpeg_idct reorders); a corrupt run past 63 lands on 63, as
            // jpeg_natural_order's extra entries put it
            blk[min(kk, 63)] = (int16_t)v;
          });
#endif
      if (fin) {
        g++;
        cj++;
        const bool wrap = cj == bpm;
        cj = wrap ? 0 : cj;
        cmx += wrap ? 1 : 0;
        const bool row = cmx == mcux;
        cmx = row ? 0 : cmx;
        cmy += row ? 1 : 0;
        blk = addr();  // past the segment's last block when g == seg_block1: never stored through
      }
#if MXD_HUFF_STATS
      st.write_syms++;
#endif
    };
#if MXD_HUFF_WUNROLL > 1
    // WUNROLL steps per check while none of them can reach the subsequence's
    // end, the segment's last block or the bits past the data (a step
    // consumes <= 31 bits and finishes <= 1 block)
    const int32_t lim = min(u.end, u.sg.bits + 1);
    while (rd.pos() + 31 * (MXD_HUFF_WUNROLL - 1) < lim && g + (MXD_HUFF_WUNROLL - 1) < seg_block1) {
#pragma unroll
      for (int i = 0; i < MXD_HUFF_WUNROLL; i++) wstep();
    }
#endif
    for (;;) {
      const int32_t p = rd.pos();
      if (p >= u.end || g >= seg_block1 || (dec.b == 0 && dec.k == 0 && p > u.sg.bits)) break;
      wstep();
    }
  }
}

__global__ __launch_bounds__(kHuffThreads) void jpeg_huff(const uint32_t* __restrict__ words,
                                                          const HuffDev* __restrict__ tables,
                                                          const HuffImgDev* __restrict__ imgs,
                                                          const HuffSegDev* __restrict__ segs,
                                                          const HuffJobDev* __restrict__ jobs, int16_t* coef) {
  __shared__ Shared sh;
  extern __shared__ __attribute__((aligned(16))) uint4 dyn[];
#if MXD_HUFF_STATS
  const uint64_t t_kernel = stat_clock();
#endif
  const int t = threadIdx.x;
  const HuffJobDev job = jobs[blockIdx.x];
  if (t == 0) sh.img = imgs[segs[job.seg0].img];
  __syncthreads();
  const HuffImgDev& im = sh.img;
  if (t < im.bpm) {  // the block cursor's tables (read after stage 0's barrier)
    if (!im.interleaved) {
      sh.blk_off[0] = im.plane[0];
      sh.blk_mxs[0] = 64;
      sh.blk_mys[0] = im.bw[0] * 64;
    } else {
      const int c = im.blk_comp[t];
      sh.blk_off[t] = im.plane[c] + ((int64_t)im.blk_dy[t] * im.bw[c] + im.blk_dx[t]) * 64;
      sh.blk_mxs[t] = im.comp_h[c] * 64;
      sh.blk_mys[t] = im.comp_v[c] * im.bw[c] * 64;
    }
  }
  HuffDev* tab = reinterpret_cast<HuffDev*>(dyn);
  SegLds* seg = reinterpret_cast<SegLds*>(reinterpret_cast<char*>(dyn) + lds_tables_bytes(im.ntables));
  const int64_t word0 = segs[job.seg0].word;  // the job's first word (16-byte aligned)
  const int sub_bits = segs[job.seg0].sub_bits;

  // 0. tables, segment records and (job.lds) words into LDS; zero the job's
  // coefficient blocks
  {
    const uint4* src = reinterpret_cast<const uint4*>(tables + im.tables);
    const int n16 = im.ntables * (int)(sizeof(HuffDev) / 16);
    for (int i = t; i < n16; i += blockDim.x) dyn[i] = src[i];
  }
  uint32_t* lds_words = reinterpret_cast<uint32_t*>(reinterpret_cast<char*>(dyn) + lds_words_at(im.ntables, job.nseg));
  if (job.lds) {
    const uint4* src = reinterpret_cast<const uint4*>(words + word0);
    uint4* dst = reinterpret_cast<uint4*>(lds_words);
    for (int i = t; i < job.words16; i += blockDim.x) dst[i] = src[i];
  }
  int nsub_mine = 0;
  if (t < job.nseg) {
    const HuffSegDev g = segs[job.seg0 + t];
    seg[t] = SegLds{(int32_t)(g.word - word0), g.bits, (int32_t)g.mcu0, g.mcus};
    nsub_mine = max(1, (g.bits + sub_bits - 1) / sub_bits);
  }
  int nsub = 0;
  const int sub0 = block_exclusive_scan(nsub_mine, sh.scan, &nsub);
  if (t < job.nseg) sh.seg_sub0[t] = sub0;
  {
    const HuffSegDev& s0 = segs[job.seg0];
    const HuffSegDev& s1 = segs[job.seg0 + job.nseg - 1];
    const int64_t b0 = s0.mcu0 * im.bpm, b1 = (s1.mcu0 + (int64_t)s1.mcus) * im.bpm;
    for (int64_t g = b0 + (t >> 3); g < b1; g += blockDim.x >> 3)
      reinterpret_cast<uint4*>(coef + block_addr(im, g))[t & 7] = uint4{0, 0, 0, 0};
  }
  if (t == 0) sh.flag[0] = sh.flag[1] = 0;
  __syncthreads();
#if MXD_HUFF_STATS
  const uint64_t t_start = stat_clock();
#endif

  // this thread's subsequence: its segment (binary search of seg_sub0) and bit range
  int si = 0;
  if (t < nsub) {
    int lo = 0, hi = job.nseg - 1;
    while (lo < hi) {
      const int mid = (lo + hi + 1) >> 1;
      if (sh.seg_sub0[mid] <= t) lo = mid;
      else hi = mid - 1;
    }
    si = lo;
  }
  Sub u;
  u.sg = seg[si];
  u.j = t - sh.seg_sub0[si];  // index inside the segment
  const int nseg_sub = max(1, (u.sg.bits + sub_bits - 1) / sub_bits);
  u.active = t < nsub;
  u.first = u.j == 0;
  u.last = u.j == nseg_sub - 1;
  u.start = u.j * sub_bits;
  u.end = u.last ? 0x7fffffff : u.start + sub_bits;
  if (u.active) {
    sh.in_pos[t] = u.start;
    sh.in_b[t] = 0;
    sh.in_k[t] = 0;
    sh.done[t] = 0;
    sh.sub_seg[t] = (int16_t)si;
  }
  __syncthreads();  // sub_seg of every subsequence before any round reads it

  int dcsum[3] = {0, 0, 0};
  int64_t dc0 = -1, dc1 = -1;  // blocks whose DC this subsequence decoded: [dc0, dc1)
  Stats st;
#if MXD_HUFF_STATS
  st.t[0] = t_start;
#endif
  if (job.lds)  // uniform over the workgroup
    decode_passes<LdsReader>(lds_words, sh, im, tab, seg, sub_bits, nsub, u, coef, dcsum, dc0, dc1, st);
  else
    decode_passes<GlobalReader>(words + word0, sh, im, tab, seg, sub_bits, nsub, u, coef, dcsum, dc0, dc1, st);

#if MXD_HUFF_STATS
  __syncthreads();
  st.c[1] = stat_cycles();
  st.r[1] = stat_clock();
  if (t == 0) sh.flag[0] = 0;
  __syncthreads();
  atomicMax(&sh.flag[0], st.write_syms);  // an LDS atomic: the busiest thread's write-pass symbols
  __syncthreads();
  const int stat_wmax = sh.flag[0];
  __syncthreads();
#endif
  // 4. DC values: per component, the differences before this subsequence in its segment
  for (int c = 0; c < 3; c++) {
    const int ex = block_exclusive_scan(u.active ? dcsum[c] : 0, sh.scan, nullptr);
#if MXD_HUFF_STATS
    if (c == 0) st.t[2] = stat_clock();
#endif
    __syncthreads();
    sh.done[t] = ex;
    __syncthreads();
    dcsum[c] = u.active ? ex - sh.done[t - u.j] : 0;  // this subsequence's predictor start
    __syncthreads();
  }
#if MXD_HUFF_STATS
  int stat_sync = 0, stat_write = 0, stat_chg = 0, stat_chg_pos = 0, stat_chg_k = 0;
  {
    const int a = block_exclusive_scan(st.sync_syms, sh.scan, &stat_sync);
    const int b = block_exclusive_scan(st.write_syms, sh.scan, &stat_write);
    const int c = block_exclusive_scan(st.chg, sh.scan, &stat_chg);
    const int d = block_exclusive_scan(st.chg_pos, sh.scan, &stat_chg_pos);
    const int e = block_exclusive_scan(st.chg_k, sh.scan, &stat_chg_k);
    (void)a;
    (void)b;
    (void)c;
    (void)d;
    (void)e;
  }
#endif
  if (u.active && dc0 >= 0) {
    int pred[3] = {dcsum[0], dcsum[1], dcsum[2]};
    for (int64_t b = dc0; b < dc1; b++) {
      const int bj = (int)(b % im.bpm);
      const int c = im.blk_comp[bj];
      int16_t* d = coef + block_addr(im, b);
      pred[c] += d[0];
      d[0] = (int16_t)pred[c];
    }
  }
#if MXD_HUFF_STATS
  __syncthreads();
  st.t[3] = stat_clock();
  // wave 0's lanes 0..7 (vector stores); thread 0's clocks
  const uint64_t t0 = __shfl(st.t[0], 0, 64), t1 = __shfl(st.t[1], 0, 64), t2 = __shfl(st.t[2], 0, 64),
                 t3 = __shfl(st.t[3], 0, 64), tk = __shfl(t_kernel, 0, 64);
  const uint64_t c0 = __shfl(st.c[0], 0, 64), c1 = __shfl(st.c[1], 0, 64);
  const uint64_t r0 = __shfl(st.r[0], 0, 64), r1 = __shfl(st.r[1], 0, 64);
  if (blockIdx.x < kStatJobs && t < kStatInts) {
    // write-pass shader cycles, the busiest thread's write symbols, and thread 0's
    const int v[kStatInts] = {st.rounds,      nsub,           stat_sync,         stat_write,
                              (int)(t1 - t0), (int)(t2 - t1), (int)(t3 - t2),    (int)(t0 - tk),
                              (int)(c1 - c0), stat_wmax,      __shfl(st.write_syms, 0, 64), (int)(r1 - r0),
                              stat_chg,       stat_chg_pos,   stat_chg_k,        0};
    g_huff_stats[blockIdx.x * kStatInts + t] = v[t];
  }
#endif
}

}  // namespace

int64_t jpeg_huff_lds_budget() { return 160 * 1024 - (int64_t)sizeof(Shared) - 1024; }

int64_t jpeg_huff_lds_bytes(int ntables, int nseg, int64_t words) {
  return lds_words_at(ntables, nseg) + words * 4;
}

int launch_jpeg_huff(const uint32_t* words, const HuffDev* tables, const HuffImgDev* imgs, const HuffSegDev* segs,
                     const HuffJobDev* jobs, int32_t njobs, int32_t threads, int64_t lds_bytes, int16_t* coef,
                     void* stream) {
  if (njobs <= 0) return 0;
  threads = (threads + 63) / 64 * 64;
  threads = threads < 64 ? 64 : threads > kHuffThreads ? kHuffThreads : threads;
  auto k = jpeg_huff;
  if (hipFuncSetAttribute(reinterpret_cast<const void*>(k), hipFuncAttributeMaxDynamicSharedMemorySize,
                          (int)lds_bytes) != hipSuccess)
    return -1;
  hipLaunchKernelGGL(k, dim3(njobs), dim3(threads), (size_t)lds_bytes, reinterpret_cast<hipStream_t>(stream), words,
                     tables, imgs, segs, jobs, coef);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

}  // namespace mxd

#if MXD_HUFF_STATS
// (rounds, subsequences, sync-pass symbols, write-pass symbols) of the last
// launch's first n jobs.
extern "C" int mxd_debug_huff_stats(int* host, int n) {
  if (n > mxd::kStatJobs) n = mxd::kStatJobs;
  return hipMemcpyFromSymbol(host, HIP_SYMBOL(mxd::g_huff_stats), sizeof(int) * mxd::kStatInts * n, 0,
                             hipMemcpyDeviceToHost) ==
                 hipSuccess
             ? 0
             : -1;
}
#endif
