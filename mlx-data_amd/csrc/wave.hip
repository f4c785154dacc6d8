// wave.hip -- the fast paths of the fused resize + crop (+ hflip) (+ /255) stage.
//
// Arithmetic (shared with resample.hip): stbir triangle taps from the shared
// tables, vertical pass first in byte units, f32 FMA accumulation in tap order
// starting from 0, stbir's encode, exact q/255.
//
// A UNIT = (image, band of output rows, strip of output columns) is run by one
// wave.  The wave covers a 1024-byte window of each source row: lane l holds
// the four dwords at bytes 4l + 256j (j = 0..3) of the window, loaded with
// buffer_load_dword through a descriptor spanning the image (row offset in the
// scalar soffset; dwords outside the strip's footprint are not fetched, reads
// past the image return 0).  The vertical (V) pass yields 16 f32 per lane for
// an output row; they go to an LDS row (four ds_write_b128, lanes 16 B apart:
// conflict-free).  The horizontal (H) pass gives lane l the output elements
// 4l..4l+3 of the strip row (C channels interleaved) from the LDS row with
// their T horizontal taps (in registers for the whole band, paired for
// v_pk_fma_f32), rounds like stbir's encode and stores 4 f32 (exact q/255, one
// 16-byte store) or 4 u8.
//
// Four ways to run a band (KIND):
//   kGather  each output row loads its T tap rows, double-buffered one output
//            row ahead.  Any geometry (upsampling included).
//   kRing    every source row of the band is loaded once, kLook rows ahead,
//            into a register ring; when a row is the last tap of an output row
//            the T ring rows ending there are converted and summed
//            (right-aligned taps).  Downsampling, <= 1 output row per source row.
//   kScatter every source row is loaded once and converted to f32 ONCE, then
//            FMA'd into each open output row whose taps contain it, following
//            a host-built schedule (below).  About half the VALU work of kRing.
//   kBand    kScatter's V pass with the H pass and every store moved to a
//            fourth wave of the workgroup (resample_band, below): the vertical
//            waves' vmcnt then counts only their own row loads.
//
// Scatter schedule (capi.cpp builds it per image crop and band height): a
// sequence of GROUPS of DMAX iterations.  An iteration carries one source row
// (or -1, a bubble), its weights for the output rows of groups g, g+1, ...,
// g+S-1, and the row to load for the iteration R-1 ahead; group g completes one
// output row (or none).  Group g accumulates in slot g mod S, so with the group
// loop unrolled by a multiple of S every accumulator index is static.  Rows
// are loaded R-1 iterations ahead into a ring of R register slots, and the
// unrolled block is a multiple of R iterations, so every ring slot index is
// static too.  Rows are visited in ascending order, so each output row's sum
// runs in tap order from 0 exactly as in kGather / kRing: all kinds give
// bit-identical results.
// Per band: word 0 = groups to run (a multiple of the block's groups), words
// 1.. = the output row each group completes (-1: none), then at word
// ImgDev::group the iteration entries, scatter_entry_words(S) words each:
// row to prefetch, row, S f32 weights (one scalar burst per group).
#include <hip/hip_runtime.h>

#include <type_traits>
#include <utility>

#include "resample.h"

namespace mxd {
namespace {

constexpr int kWaves = 4;
constexpr int kLanes = 64;
constexpr int kChunk = 16;                  // source bytes per lane per row
constexpr int kRowBytes = kLanes * kChunk;  // 1024 source bytes per wave row
constexpr int kOutPerLane = 4;              // output elements per lane per row

#define GLOBAL_PTR(T, p) ((__attribute__((address_space(1))) T*)(p))
using cgfloat = const __attribute__((address_space(1))) float;
// Constant address space: uniform loads through it are scalar (s_load).
using kfloat = const __attribute__((address_space(4))) float;
using kint = const __attribute__((address_space(4))) int;
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x2 __attribute__((ext_vector_type(2)));
using Rsrc = __amdgpu_buffer_rsrc_t;

enum Kind { kGather = 0, kRing = 1, kScatter = 2, kBand = 3 };

__device__ __forceinline__ int xcd_remap(int b, int n) {
  const int q = n >> 3, r = n & 7;
  const int xcd = b & 7, idx = b >> 3;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + idx;
}

// Exact f32 q/255.0f for q in 0..255 (checked for all 256 values).
__device__ __forceinline__ float div255(float q) {
  const float inv = 1.0f / 255.0f;
  const float r = q * inv;
  const float e = __builtin_fmaf(-r, 255.0f, q);
  return __builtin_fmaf(e, inv, r);
}

// stbir encode: (uint8)trunc(clamp(v*255 + 0.5, 0, 255)), v in byte units here.
__device__ __forceinline__ float encode(float v) { return truncf(fminf(fmaxf(v + 0.5f, 0.0f), 255.0f)); }

// A uniform pointer held in scalar registers.
template <class P>
__device__ __forceinline__ P uniform_ptr(const void* p) {
  const uint64_t v = reinterpret_cast<uint64_t>(p);
  return (P)(((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)(v >> 32)) << 32) |
             (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)v));
}

struct Chunk {
  uint32_t d[4];
};

// A voffset past any image (images are < 2^31 bytes): the buffer range check
// turns the load into a zero without a memory request.
constexpr int kNoLoad = 0x7ffffff0;

// Source descriptor spanning the image, and a dead one (no records: every
// load through it returns zeros without a memory request).
struct Src {
  Rsrc live, dead;
  int stride;
};

__device__ __forceinline__ Src make_src(const ImgDev& im) {
  void* base = uniform_ptr<void*>(im.src);
  const int stride = __builtin_amdgcn_readfirstlane((int)im.src_stride);
  const int rows = __builtin_amdgcn_readfirstlane(im.src_h);
  return Src{__builtin_amdgcn_make_buffer_rsrc(base, (short)0, stride * rows, 0x00020000),
             __builtin_amdgcn_make_buffer_rsrc(base, (short)0, 0, 0x00020000), stride};
}

// The lane's 4 dwords of source row r (byte offsets voff[j] of the row,
// kNoLoad for dwords outside the strip's footprint); four zeros without a
// memory request when r < 0 (uniform; the descriptor is chosen in SGPRs).
__device__ __forceinline__ Chunk load_row(const Src& src, const int* voff, int r) {
  const bool live = r >= 0;
  const Rsrc rs = live ? src.live : src.dead;
  const int soff = live ? r * src.stride : 0;
  Chunk c;
#pragma unroll
  for (int j = 0; j < 4; j++) c.d[j] = __builtin_amdgcn_raw_buffer_load_b32(rs, voff[j], soff, 0);
  return c;
}

// Bytes -> f32 in pairs: x[2j] = bytes 0,1 of dword j, x[2j+1] = bytes 2,3.
__device__ __forceinline__ void chunk_to_f32(const Chunk& v, f32x2* x) {
#pragma unroll
  for (int j = 0; j < 4; j++) {
    x[2 * j] = f32x2{(float)(v.d[j] & 0xffu), (float)((v.d[j] >> 8) & 0xffu)};
    x[2 * j + 1] = f32x2{(float)((v.d[j] >> 16) & 0xffu), (float)(v.d[j] >> 24)};
  }
}

// acc += w * x over the lane's 16 bytes (8 v_pk_fma_f32).
__device__ __forceinline__ void fma_row(f32x2* acc, float w, const f32x2* x) {
  const f32x2 ww = {w, w};
#pragma unroll
  for (int p = 0; p < 8; p++) acc[p] = __builtin_elementwise_fma(ww, x[p], acc[p]);
}

__device__ __forceinline__ void fma_chunk(f32x2* acc, float w, const Chunk& v) {
  f32x2 x[8];
  chunk_to_f32(v, x);
  fma_row(acc, w, x);
}

__device__ __forceinline__ void zero_row(f32x2* acc) {
#pragma unroll
  for (int p = 0; p < 8; p++) acc[p] = f32x2{0.0f, 0.0f};
}

// Timing-only ablation (MODE 1): keep the loads live without the V math.
__device__ __forceinline__ void touch_chunk(f32x2* acc, const Chunk& v) {
#pragma unroll
  for (int j = 0; j < 4; j++) acc[j].x += __uint_as_float(v.d[j] & 0x3fffffffu);
}

__device__ __forceinline__ Chunk fake_chunk(int lane, int r) {
  return Chunk{{(uint32_t)(lane * 7 + r), (uint32_t)(r * 3), (uint32_t)lane, (uint32_t)(r ^ lane)}};
}

// V sums (16 f32 per lane) -> an LDS row: floats of bytes 4l + 256j .. +3 go
// to row[4l + 256j], lanes 16 B apart per store (conflict-free).
__device__ __forceinline__ void write_vrow(float* row, const f32x2* acc, int lane) {
#pragma unroll
  for (int j = 0; j < 4; j++)
    *reinterpret_cast<float4*>(row + 4 * lane + 256 * j) =
        make_float4(acc[2 * j].x, acc[2 * j].y, acc[2 * j + 1].x, acc[2 * j + 1].y);
}

__device__ __forceinline__ void wave_lds_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// LDS-only workgroup barrier.  No fence: a workgroup release fence waits for
// vmcnt(0) on gfx9 and would drain the ring's row loads at every output row.
__device__ __forceinline__ void band_barrier() {
  asm volatile("" ::: "memory");
  __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0): this wave's LDS writes have landed
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

// Calls f(std::integral_constant<int, I>) for I = 0..N-1 (guaranteed unrolled,
// so register-array indices derived from I are static).
template <class F, int... Is>
__device__ __forceinline__ void static_for_impl(F&& f, std::integer_sequence<int, Is...>) {
  (f(std::integral_constant<int, Is>{}), ...);
}
template <int N, class F>
__device__ __forceinline__ void static_for(F&& f) {
  static_for_impl(f, std::make_integer_sequence<int, N>{});
}

// The image a unit belongs to (units are numbered through ImgDev::tile_begin).
__device__ __forceinline__ const ImgDev& find_image(const ImgDev* imgs, int nimgs, int unit) {
  int lo = 0, hi = nimgs - 1;
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (imgs[mid].tile_begin <= unit) lo = mid; else hi = mid - 1;
  }
  return imgs[lo];
}

// Source footprint of output columns [ox0, ox1) (taps are monotone in the crop
// column): first byte fb0 (4-byte aligned) and byte count (<= kRowBytes).
template <int C>
__device__ __forceinline__ void strip_footprint(cgfloat* xtab, int xs, int crop_w, int flip, int shift, int ox0,
                                                int ox1, int* fb0, int* need) {
  const int xa = flip ? crop_w - ox1 : ox0;
  const int xb = flip ? crop_w - 1 - ox0 : ox1 - 1;
  const int px_lo = __float_as_int(xtab[xa * xs]);
  const int px_hi = __float_as_int(xtab[xb * xs]) + __float_as_int(xtab[xb * xs + 1]) - 1;
  *fb0 = (px_lo * C + shift) & ~3;
  *need = (px_hi + 1) * C + shift - *fb0;
}

// Per-lane byte offsets of the strip window: only the dwords that hold
// footprint bytes are fetched.
__device__ __forceinline__ void window_offsets(int fb0, int need, int lane, int* voff) {
#pragma unroll
  for (int j = 0; j < 4; j++) voff[j] = 4 * lane + 256 * j < need ? fb0 + 4 * lane + 256 * j : kNoLoad;
}

// Horizontal pass of one strip: the lane's 4 output elements (taps paired for
// v_pk_fma_f32, positions in the strip's LDS row).
template <int C, bool F32, int T>
struct HStrip {
  f32x2 wx[2][T];
  int pos[kOutPerLane];
  int ox0, nout;

  __device__ __forceinline__ void init(cgfloat* xtab, int xs, int crop_w, int flip, int shift, int ox0_, int ox1,
                                       int fb0, int lane) {
    ox0 = ox0_;
    nout = (ox1 - ox0) * C;
#pragma unroll
    for (int j = 0; j < kOutPerLane; j++) {
      const int o = min(kOutPerLane * lane + j, nout - 1);
      const int px = o / C;
      const int c = o - px * C;
      const int ox = ox0 + px;
      const int xc = flip ? crop_w - 1 - ox : ox;
      cgfloat* xe = xtab + xc * xs;
      pos[j] = __float_as_int(xe[0]) * C + shift - fb0 + c;
#pragma unroll
      for (int k = 0; k < T; k++) wx[j >> 1][k][j & 1] = xe[kTapHeader + k];  // zero padded past the tap count
    }
  }

  // H taps of an output row from its LDS row, stbir encode, store into drow
  // (the output row).  MODE 9 (timing only): no stores (`never` is false).
  template <int MODE>
  __device__ __forceinline__ void run(const float* vrow, char* drow, int lane, bool never) const {
    f32x2 s0 = {0.0f, 0.0f}, s1 = {0.0f, 0.0f};
#pragma unroll
    for (int k = 0; k < T; k++) {
      s0 = __builtin_elementwise_fma(wx[0][k], f32x2{vrow[pos[0] + k * C], vrow[pos[1] + k * C]}, s0);
      s1 = __builtin_elementwise_fma(wx[1][k], f32x2{vrow[pos[2] + k * C], vrow[pos[3] + k * C]}, s1);
    }
    const float out[kOutPerLane] = {encode(s0.x), encode(s0.y), encode(s1.x), encode(s1.y)};
    const int o0 = kOutPerLane * lane;
    if (MODE == 9 && !never) return;
    if (o0 + kOutPerLane <= nout) {  // one store instruction per row (lanes past nout masked)
      if constexpr (F32) {
        f32x4 v = {div255(out[0]), div255(out[1]), div255(out[2]), div255(out[3])};
        *reinterpret_cast<__attribute__((address_space(1))) f32x4*>(GLOBAL_PTR(float, drow) + ox0 * C + o0) = v;
      } else {
        *reinterpret_cast<__attribute__((address_space(1))) uint32_t*>(GLOBAL_PTR(uint8_t, drow) + ox0 * C + o0) =
            (uint32_t)out[0] | ((uint32_t)out[1] << 8) | ((uint32_t)out[2] << 16) | ((uint32_t)out[3] << 24);
      }
    } else if (o0 < nout) {  // ragged strip end
#pragma unroll
      for (int j = 0; j < kOutPerLane; j++) {
        if (o0 + j < nout) {
          if constexpr (F32) GLOBAL_PTR(float, drow)[ox0 * C + o0 + j] = div255(out[j]);
          else GLOBAL_PTR(uint8_t, drow)[ox0 * C + o0 + j] = (uint8_t)out[j];
        }
      }
    }
  }
};

// Runs a band's scatter schedule (see the top of the file); on_row(acc, y) is
// called with the V sums of every completed output row y.
template <int S, int DMAX, int MODE, class OnRow>
__device__ __forceinline__ void scatter_band(kint* sched, int entry_off, const Src& src, const int* voff, int lane,
                                             OnRow&& on_row) {
  constexpr int R = scatter_ring_slots(DMAX);
  constexpr int LA = R - 1;  // iterations loaded ahead
  constexpr int BG = scatter_block_groups(S, DMAX);
  constexpr int E = scatter_entry_words(S);
  const int ngroups = sched[0];
  kint* gout = sched + 1;
  kint* itab = sched + entry_off;
  auto load = [&](int r) {
    if constexpr (MODE == 2) return fake_chunk(lane, r);
    return load_row(src, voff, r);
  };
  f32x2 acc[S][8];
#pragma unroll
  for (int s = 0; s < S; s++) zero_row(acc[s]);
  Chunk ring[R];
  static_for<LA>([&](auto ic) {
    __builtin_amdgcn_sched_barrier(0);  // issue in ring order: the loop's counted waits assume it
    ring[decltype(ic)::value] = load(itab[decltype(ic)::value * E + 1]);
  });
  __builtin_amdgcn_sched_barrier(0);
  for (int gb = 0; gb < ngroups; gb += BG) {
    kint* blk = itab + gb * DMAX * E;
    static_for<BG>([&](auto gc) {
      constexpr int gi = decltype(gc)::value;
      // the group's entries in one scalar burst
      int ent[DMAX * E];
#pragma unroll
      for (int q = 0; q < DMAX * E; q++) ent[q] = blk[gi * DMAX * E + q];
      static_for<DMAX>([&](auto jc) {
        constexpr int j = decltype(jc)::value;
        constexpr int i = gi * DMAX + j;
        __builtin_amdgcn_sched_barrier(0);  // keep each row's work (and its load) in place
        // slot (i + LA) % R was consumed by the previous iteration
        ring[(i + LA) % R] = load(ent[j * E]);
        if (ent[j * E + 1] >= 0) {
          if constexpr (MODE == 1) {
            touch_chunk(acc[gi % S], ring[i % R]);
          } else {
            f32x2 x[8];
            chunk_to_f32(ring[i % R], x);
            static_for<S>([&](auto kc) {
              constexpr int k = decltype(kc)::value;
              const int wbits = ent[j * E + 2 + k];
              if (k == 0 || wbits != 0) fma_row(acc[(gi + k) % S], __int_as_float(wbits), x);
            });
          }
        }
      });
      const int y = gout[gb + gi];
      if (y >= 0) on_row(acc[gi % S], y);
      zero_row(acc[gi % S]);
    });
  }
}

// Timing-only ablations (MXD_WAVE_ABLATE, instantiated for the C2 scatter
// kernel only): 1 = no V math, 2 = no source loads, 9 = no stores,
// 16 = stores folded onto each image's first 8 rows (they stay in L2).
template <int C, bool F32, int T, int KIND, int S, int DMAX, int MODE>
__global__ __launch_bounds__(kWaves* kLanes, KIND == kScatter && T <= 12 ? 3 : 1) void resample_wave(
    const ImgDev* __restrict__ imgs, int nimgs, int nunits, int rowf) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  const int lane = threadIdx.x & (kLanes - 1);
  const int unit = __builtin_amdgcn_readfirstlane(xcd_remap(blockIdx.x, gridDim.x) * kWaves + (threadIdx.x >> 6));
  float* __restrict__ vrow = smem + (threadIdx.x >> 6) * rowf;
  for (int i = kRowBytes + lane; i < rowf; i += kLanes) vrow[i] = 0.0f;  // zeroed tail for padded taps
  if (unit >= nunits) return;

  const ImgDev& im = find_image(imgs, nimgs, unit);
  const int nstrips = __builtin_amdgcn_readfirstlane(im.nstrips);
  const int crop_w = __builtin_amdgcn_readfirstlane(im.crop_w);
  const int crop_h = __builtin_amdgcn_readfirstlane(im.crop_h);
  const int flip_shift = __builtin_amdgcn_readfirstlane(im.flip);
  const int flip = flip_shift & 1, shift = flip_shift >> 8;  // see ImgDev::flip
  const int band_rows = __builtin_amdgcn_readfirstlane(im.ty);
  const int strip_cols = __builtin_amdgcn_readfirstlane(im.tx);
  const int xs = kTapHeader + __builtin_amdgcn_readfirstlane(im.xwidth);
  const int ys = kTapHeader + __builtin_amdgcn_readfirstlane(im.ywidth);
  cgfloat* xtab = GLOBAL_PTR(const float, im.xtab);
  // The vertical taps / schedule are read with scalar loads (lgkmcnt), which
  // never wait on the vector loads of the next rows.
  kfloat* ytab = uniform_ptr<kfloat*>(im.ytab);
  char* dst = reinterpret_cast<char*>(im.dst);
  const int64_t dstride = im.dst_stride;
  const int local = unit - __builtin_amdgcn_readfirstlane(im.tile_begin);
  const int band = local / nstrips;
  const int strip = local - band * nstrips;
  const int oy0 = band * band_rows;
  const int oy1 = min(oy0 + band_rows, crop_h);
  const int ox0 = strip * strip_cols;
  const int ox1 = min(ox0 + strip_cols, crop_w);

  int fb0, need;
  strip_footprint<C>(xtab, xs, crop_w, flip, shift, ox0, ox1, &fb0, &need);
  const Src src = make_src(im);
  int voff[4];
  window_offsets(fb0, need, lane, voff);

  HStrip<C, F32, T> hs;
  hs.init(xtab, xs, crop_w, flip, shift, ox0, ox1, fb0, lane);
  // The horizontal weights are loaded once; retire them here so the waits the
  // compiler places in the row loop only ever cover the row loads.
  __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0)

  // V row of output row y done (16 f32 per lane): H pass and store.
  auto finish_row = [&](const f32x2* acc, int y) {
    write_vrow(vrow, acc, lane);
    wave_lds_sync();
    hs.template run<MODE>(vrow, dst + (int64_t)(MODE == 16 ? (y & 7) : y) * dstride, lane, nimgs < 0);
    wave_lds_sync();
  };

  if constexpr (KIND == kGather) {
    // ---- gather: each output row sums its T source rows, loaded for it ----
    auto load_rows = [&](Chunk* R, int y, bool live) {
      const int n0 = __float_as_int(ytab[y * ys]);
#pragma unroll
      for (int k = 0; k < T; k++) R[k] = load_row(src, voff, live ? n0 + k : -1);
    };
    auto step = [&](const Chunk* R, int y) {
      kfloat* ye = ytab + y * ys;
      f32x2 acc[8];
      zero_row(acc);
#pragma unroll
      for (int k = 0; k < T; k++) fma_chunk(acc, ye[kTapHeader + k], R[k]);  // zero padded past the tap count
      finish_row(acc, y);
    };
    // Double-buffered rows: the loads of row y+1 are issued before row y is
    // computed, so they fly during the whole V+H of row y.  The prefetch is
    // unconditional (clamped to the last output row) so every path through
    // the loop has the same loads in flight and the compiler's counted waits
    // stay partial.
    Chunk RA[T], RB[T];
    load_rows(RA, oy0, true);
    for (int y = oy0;; y += 2) {
      load_rows(RB, min(y + 1, crop_h - 1), y + 1 < oy1);
      step(RA, y);
      if (y + 1 >= oy1) break;
      load_rows(RA, min(y + 2, crop_h - 1), y + 2 < oy1);
      step(RB, y + 1);
      if (y + 2 >= oy1) break;
    }
  } else if constexpr (KIND == kRing) {
    // ---- ring: every source row of the band is loaded once, kLook rows
    // ahead, into a register ring of kRing = T + kLook slots; the source-row
    // loop is unrolled by kRing so every slot index is static.  When row r is
    // the last tap of output row y, y's taps are exactly the T rows ending at
    // r (right-aligned weights, zero for the rows before y's first tap), all
    // resident in the ring: convert and sum them (V), then H and store.
    // Requires the last taps of consecutive output rows to strictly increase
    // (at most one output row ends per source row); the host checks it.
    constexpr int kLook = 6;
    constexpr int kRing = T + kLook;
    kfloat* rtab = ytab;  // right-aligned vertical table: {last row, count, w[T]} per output row
    auto last_of = [&](int y) { return __float_as_int(rtab[min(y, crop_h - 1) * ys]); };
    const int rs = last_of(oy0) - (T - 1);
    const int re = last_of(oy1 - 1);
    int y = oy0;
    int ly = last_of(y);
    Chunk ring[kRing];
    static_for<kLook>([&](auto ic) {
      constexpr int i = decltype(ic)::value;
      __builtin_amdgcn_sched_barrier(0);  // issue in ring order: the loop's counted waits assume it
      ring[i] = load_row(src, voff, rs + i <= re ? rs + i : -1);
    });
    for (int base = rs; base <= re; base += kRing) {
      static_for<kRing>([&](auto ic) {
        constexpr int i = decltype(ic)::value;
        __builtin_amdgcn_sched_barrier(0);  // keep each row's work (and its load) in place
        const int r = base + i;
        if (r > re) return;
        // keep kLook rows in flight: slot (i + kLook) % kRing is free (its row
        // left the tap window of every open output row)
        ring[(i + kLook) % kRing] = load_row(src, voff, r + kLook <= re ? r + kLook : -1);
        if (r == ly) {  // output row y ends at source row r (at most one: checked on the host)
          kfloat* we = rtab + y * ys + kTapHeader;
          f32x2 acc[8];
          zero_row(acc);
#pragma unroll
          for (int k = 0; k < T; k++) fma_chunk(acc, we[k], ring[(i + kRing - (T - 1) + k) % kRing]);
          finish_row(acc, y);
          ++y;
          ly = y < oy1 ? last_of(y) : 0x7fffffff;
        }
      });
    }
  } else {
    // ---- scatter: follow the band's schedule ----
    kint* sched = reinterpret_cast<kint*>(ytab) + band * __builtin_amdgcn_readfirstlane(im.ywidth);
    scatter_band<S, DMAX, MODE>(sched, __builtin_amdgcn_readfirstlane(im.group), src, voff, lane, finish_row);
  }
}

// ---- kBand: one WORKGROUP per (image, band) ----
// Waves 0..2 run the scatter schedule of strips 0..2 (a wave without a strip
// only keeps the barrier count) and hand every finished V row to wave 3
// through a double-buffered LDS slot, one s_barrier per output row; wave 3
// runs the horizontal pass of every strip and issues all global stores.  On
// gfx9 a store retires in order with the loads issued after it, so a store in
// a vertical wave would hold back the wait for each later row; here the
// vertical waves' vmcnt counts their own row loads only, and the H pass is
// off their critical path.
template <int C, bool F32, int T, int S, int DMAX>
__global__ __launch_bounds__(kWaves* kLanes, 4) void resample_band(const ImgDev* __restrict__ imgs, int nimgs,
                                                                    int nunits, int rowf) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  constexpr int kV = kWaves - 1;  // vertical waves = most strips per workgroup
  const int lane = threadIdx.x & (kLanes - 1);
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int unit = __builtin_amdgcn_readfirstlane(xcd_remap(blockIdx.x, gridDim.x));
  auto slot = [&](int parity, int s) { return smem + (parity * kV + s) * rowf; };
  if (wave < kV)
    for (int par = 0; par < 2; par++)
      for (int i = kRowBytes + lane; i < rowf; i += kLanes) slot(par, wave)[i] = 0.0f;  // zeroed tails
  if (unit >= nunits) return;  // the whole workgroup

  const ImgDev& im = find_image(imgs, nimgs, unit);
  const int nstrips = __builtin_amdgcn_readfirstlane(im.nstrips);
  const int crop_w = __builtin_amdgcn_readfirstlane(im.crop_w);
  const int flip_shift = __builtin_amdgcn_readfirstlane(im.flip);
  const int flip = flip_shift & 1, shift = flip_shift >> 8;  // see ImgDev::flip
  const int strip_cols = __builtin_amdgcn_readfirstlane(im.tx);
  const int xs = kTapHeader + __builtin_amdgcn_readfirstlane(im.xwidth);
  cgfloat* xtab = GLOBAL_PTR(const float, im.xtab);
  const int band = unit - __builtin_amdgcn_readfirstlane(im.tile_begin);
  kint* sched = uniform_ptr<kint*>(im.ytab) + band * __builtin_amdgcn_readfirstlane(im.ywidth);
  const int entry_off = __builtin_amdgcn_readfirstlane(im.group);

  if (wave < kV) {
    // ---- vertical wave of strip `wave` ----
    int fb0 = 0, need = 0;  // a wave without a strip loads nothing
    if (wave < nstrips)
      strip_footprint<C>(xtab, xs, crop_w, flip, shift, wave * strip_cols, min((wave + 1) * strip_cols, crop_w), &fb0, &need);
    const Src src = make_src(im);
    int voff[4];
    window_offsets(fb0, need, lane, voff);
    __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0): the footprint reads
    scatter_band<S, DMAX, 0>(sched, entry_off, src, voff, lane, [&](const f32x2* acc, int y) {
      write_vrow(slot(y & 1, wave), acc, lane);
      band_barrier();
    });
  } else {
    // ---- store wave: H pass and stores of every strip ----
    char* dst = reinterpret_cast<char*>(im.dst);
    const int64_t dstride = im.dst_stride;
    HStrip<C, F32, T> hs[kV];
    static_for<kV>([&](auto sc) {
      constexpr int s = decltype(sc)::value;
      if (s < nstrips) {
        const int ox0 = s * strip_cols, ox1 = min(ox0 + strip_cols, crop_w);
        int fb0, need;
        strip_footprint<C>(xtab, xs, crop_w, flip, shift, ox0, ox1, &fb0, &need);
        hs[s].init(xtab, xs, crop_w, flip, shift, ox0, ox1, fb0, lane);
      }
    });
    const int ngroups = sched[0];
    for (int g = 0; g < ngroups; g++) {
      const int y = sched[1 + g];
      if (y < 0) continue;
      band_barrier();
      static_for<kV>([&](auto sc) {
        constexpr int s = decltype(sc)::value;
        if (s < nstrips) hs[s].template run<0>(slot(y & 1, s), dst + (int64_t)y * dstride, lane, false);
      });
    }
  }
}

using WaveKernel = void (*)(const ImgDev*, int, int, int);

template <int C, bool F32, int T>
WaveKernel select_gr(const WaveCfg& cfg) {
  if (cfg.kind == kRing) return resample_wave<C, F32, T, kRing, 1, 1, 0>;
  return resample_wave<C, F32, T, kGather, 1, 1, 0>;
}

template <int C, bool F32>
WaveKernel select_c(const WaveCfg& cfg) {
  switch (cfg.taps) {
    case 2: return select_gr<C, F32, 2>(cfg);
    case 3: return select_gr<C, F32, 3>(cfg);
    case 4: return select_gr<C, F32, 4>(cfg);
    case 5: return select_gr<C, F32, 5>(cfg);
    case 6: return select_gr<C, F32, 6>(cfg);
    case 8: return select_gr<C, F32, 8>(cfg);
    case 9: return select_gr<C, F32, 9>(cfg);
    case 10: return select_gr<C, F32, 10>(cfg);
    case 12: return select_gr<C, F32, 12>(cfg);
    case 14: return select_gr<C, F32, 14>(cfg);
    case 17: return select_gr<C, F32, 17>(cfg);
    default: return nullptr;
  }
}

// Scatter / band kernels exist for RGB and the (S, DMAX, horizontal taps)
// shapes of resize_smallest_side 256/512 from 200p..4K sources: downsampling
// by the tent filter reaches each source row from at most two output rows
// (S = 2), DMAX = ceil(in / out).
template <bool F32>
WaveKernel select_scatter(const WaveCfg& cfg) {
  if (cfg.channels != 3) return nullptr;
  if (cfg.kind == kBand) {
#define MXD_BAND(S_, D_, T_) \
  if (cfg.s == S_ && cfg.dmax == D_ && cfg.taps == T_) return resample_band<3, F32, T_, S_, D_>;
    MXD_BAND(2, 4, 8)  // 960 -> 256
    MXD_BAND(2, 3, 6)  // 720 -> 256
    MXD_BAND(2, 2, 4)  // 480 -> 256
    MXD_BAND(2, 2, 3)  // 375 / 333 -> 256
#undef MXD_BAND
    return nullptr;
  }
#define MXD_SCATTER(S_, D_, T_) \
  if (cfg.s == S_ && cfg.dmax == D_ && cfg.taps == T_) return resample_wave<3, F32, T_, kScatter, S_, D_, 0>;
  if (cfg.s == 2 && cfg.dmax == 4 && cfg.taps == 8) {  // C2 (960 -> 256): ablation builds
    if (cfg.mode == 1) return resample_wave<3, F32, 8, kScatter, 2, 4, 1>;
    if (cfg.mode == 2) return resample_wave<3, F32, 8, kScatter, 2, 4, 2>;
    if (cfg.mode == 9) return resample_wave<3, F32, 8, kScatter, 2, 4, 9>;
    if (cfg.mode == 16) return resample_wave<3, F32, 8, kScatter, 2, 4, 16>;
  }
  MXD_SCATTER(2, 4, 8)   // 960 -> 256
  MXD_SCATTER(2, 5, 9)   // 1080 -> 256, 2160 -> 512
  MXD_SCATTER(2, 6, 12)  // 1440 -> 256
  MXD_SCATTER(2, 9, 17)  // 2160 -> 256
  MXD_SCATTER(2, 3, 6)   // 720 -> 256
  MXD_SCATTER(2, 2, 4)   // 480 -> 256
  MXD_SCATTER(2, 2, 3)   // 375 / 333 -> 256
  MXD_SCATTER(3, 1, 2)   // upsampling (200 -> 256)
#undef MXD_SCATTER
  return nullptr;
}

WaveKernel select_kernel(const WaveCfg& cfg) {
  if (cfg.kind == kScatter || cfg.kind == kBand) return cfg.f32 ? select_scatter<true>(cfg) : select_scatter<false>(cfg);
  switch (cfg.channels * 2 + (cfg.f32 ? 1 : 0)) {
    case 2: return select_c<1, false>(cfg);
    case 3: return select_c<1, true>(cfg);
    case 4: return select_c<2, false>(cfg);
    case 5: return select_c<2, true>(cfg);
    case 6: return select_c<3, false>(cfg);
    case 7: return select_c<3, true>(cfg);
    default: return nullptr;
  }
}

// LDS per workgroup: one row per wave, or (kBand) two slots per vertical wave.
int lds_bytes(const WaveCfg& cfg) {
  const int rows = cfg.kind == kBand ? 2 * (kWaves - 1) : kWaves;
  return rows * wave_row_floats(cfg.taps, cfg.channels) * (int)sizeof(float);
}

// Units per workgroup: one per wave, or (kBand) one per workgroup.
int units_per_block(const WaveCfg& cfg) { return cfg.kind == kBand ? 1 : kWaves; }

}  // namespace

int wave_taps_bucket(int taps) {
  static const int kB[] = {2, 3, 4, 5, 6, 8, 9, 10, 12, 14, 17};
  for (int b : kB)
    if (taps <= b) return b;
  return -1;
}

int wave_row_floats(int taps, int channels) { return (kRowBytes + taps * channels + 3) & ~3; }

int wave_row_bytes() { return kRowBytes; }

int wave_max_outputs() { return kLanes * kOutPerLane; }

int wave_band_strips() { return kWaves - 1; }

bool wave_has_kernel(const WaveCfg& cfg) { return select_kernel(cfg) != nullptr; }

// Streaming copy (16 B per lane, grid-stride): the measured HBM ceiling that
// bench.py reports next to the spec peak.
// Each thread moves 4 x 16 B per iteration (4 loads in flight before the
// stores); blocks own contiguous 16 KiB pieces.
__global__ __launch_bounds__(256) void copy_f4(const float4* __restrict__ a, float4* __restrict__ b, size_t n) {
  const size_t per_block = 256 * 4;
  for (size_t base = blockIdx.x * per_block; base < n; base += (size_t)gridDim.x * per_block) {
    float4 v[4];
#pragma unroll
    for (int i = 0; i < 4; i++) {
      const size_t j = base + i * 256 + threadIdx.x;
      if (j < n) v[i] = a[j];
    }
#pragma unroll
    for (int i = 0; i < 4; i++) {
      const size_t j = base + i * 256 + threadIdx.x;
      if (j < n) b[j] = v[i];
    }
  }
}

int launch_copy(const void* src, void* dst, size_t bytes, void* stream) {
  const size_t n = bytes / 16;
  hipLaunchKernelGGL(copy_f4, dim3(256 * 8), dim3(256), 0, reinterpret_cast<hipStream_t>(stream),
                     reinterpret_cast<const float4*>(src), reinterpret_cast<float4*>(dst), n);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

int launch_wave(const WaveCfg& cfg, const ImgDev* imgs, void* stream) {
  const WaveKernel k = select_kernel(cfg);
  if (!k) return -2;
  const int per = units_per_block(cfg);
  const int blocks = (cfg.nunits + per - 1) / per;
  hipLaunchKernelGGL(k, dim3(blocks), dim3(kWaves * kLanes), lds_bytes(cfg), reinterpret_cast<hipStream_t>(stream),
                     imgs, cfg.nimgs, cfg.nunits, wave_row_floats(cfg.taps, cfg.channels));
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

int wave_capacity(const WaveCfg& cfg, int device) {
  const WaveKernel k = select_kernel(cfg);
  if (!k) return 0;
  int blocks = 0, cus = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&blocks, reinterpret_cast<const void*>(k), kWaves * kLanes,
                                                   lds_bytes(cfg)) != hipSuccess)
    return 0;
  if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device) != hipSuccess) return 0;
  return blocks * units_per_block(cfg) * cus;
}

}  // namespace mxd
