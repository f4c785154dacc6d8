// wave.hip -- the fast path of the fused resize + crop (+ hflip) (+ /255) stage.
//
// Same arithmetic as resample.hip (stbir triangle taps from the shared tables,
// vertical pass first in byte units, f32 FMA accumulation, stbir encode), but
// organised so that no workgroup barrier is ever needed:
//
//   one WAVE owns one unit = (image, band of output rows, strip of output
//   columns).  The wave covers a 1024-byte window of each source row: lane l
//   holds the four dwords at bytes 4l + 256j (j = 0..3) of the window, loaded
//   with buffer_load_dword through a descriptor spanning the whole image (row
//   offset in the scalar soffset, so no per-load address arithmetic; reads
//   past the image return 0).  For each output row y of the band:
//     V  lane sums its 16 byte columns over the T vertical taps of y from the
//        T consecutive source rows it holds in registers and writes 16 f32 to
//        the wave's private LDS row (four ds_write_b128, lanes 16 bytes apart:
//        conflict-free).  Then it moves on to y+1: the rows shared by the taps
//        of y and y+1 stay in registers (shifted by the uniform row advance d),
//        only the d new rows are loaded, and those loads are in flight during
//     H  lane l produces output elements 4l..4l+3 of the strip row (C
//        channels interleaved) from the LDS row with their T horizontal taps
//        (weights in registers for the whole band), rounds like stbir's encode
//        and stores 4 f32 (exact q/255, one 16-byte store) or 4 u8.
//   Waves never wait for each other; the CU interleaves the waves of many
//   units so that loads of their next rows are always in flight.
// Tap counts are padded to the template T with zero weights; padded taps read
// real neighbouring rows/columns (or zeros), so every value is finite.
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
using gfloat = __attribute__((address_space(1))) float;
using cgfloat = const __attribute__((address_space(1))) float;
// Constant address space: uniform loads through it are scalar (s_load).
using kfloat = const __attribute__((address_space(4))) float;
typedef float f32x4 __attribute__((ext_vector_type(4)));

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

struct Chunk {
  uint32_t d[4];
};

// A voffset past any image (images are < 2^31 bytes): the buffer range check
// turns the load into a zero without a memory request.
constexpr int kNoLoad = 0x7ffffff0;

// The lane's 4 dwords of source row `row_off / stride` (byte offsets voff[j]
// of the row, kNoLoad for dwords outside the strip's footprint), or four
// zeros without memory traffic when !live (uniform).
template <int AUX = 0>
__device__ __forceinline__ Chunk load_chunk_if(__amdgpu_buffer_rsrc_t rsrc, const int* voff, int row_off, bool live) {
  Chunk r;
#pragma unroll
  for (int j = 0; j < 4; j++) r.d[j] = __builtin_amdgcn_raw_buffer_load_b32(rsrc, live ? voff[j] : kNoLoad, row_off, AUX);
  return r;
}

__device__ __forceinline__ void fma16(float* acc, float w, const Chunk& v) {
#pragma unroll
  for (int i = 0; i < 4; i++) {
    acc[4 * i + 0] = __builtin_fmaf(w, (float)(v.d[i] & 0xffu), acc[4 * i + 0]);
    acc[4 * i + 1] = __builtin_fmaf(w, (float)((v.d[i] >> 8) & 0xffu), acc[4 * i + 1]);
    acc[4 * i + 2] = __builtin_fmaf(w, (float)((v.d[i] >> 16) & 0xffu), acc[4 * i + 2]);
    acc[4 * i + 3] = __builtin_fmaf(w, (float)(v.d[i] >> 24), acc[4 * i + 3]);
  }
}

// Diagnostic (MODE 5): one 16-byte load per lane instead of four dwords --
// same bytes per wave, wrong lane order (timing only).
__device__ __forceinline__ Chunk load_x4_if(__amdgpu_buffer_rsrc_t rsrc, int off, int row_off, bool live) {
  typedef int i32x4 __attribute__((ext_vector_type(4)));
  const i32x4 v = __builtin_amdgcn_raw_buffer_load_b128(rsrc, live ? off : kNoLoad, row_off, 0);
  return Chunk{{(uint32_t)v.x, (uint32_t)v.y, (uint32_t)v.z, (uint32_t)v.w}};
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

template <int C, bool F32, int T, int MODE = 0, bool RING = false>
__global__ __launch_bounds__(kWaves* kLanes) void resample_wave(const ImgDev* __restrict__ imgs, int nimgs,
                                                               int nunits, int rowf) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  const int lane = threadIdx.x & (kLanes - 1);
  const int unit = __builtin_amdgcn_readfirstlane(xcd_remap(blockIdx.x, gridDim.x) * kWaves + (threadIdx.x >> 6));
  float* __restrict__ vrow = smem + (threadIdx.x >> 6) * rowf;
  for (int i = kRowBytes + lane; i < rowf; i += kLanes) vrow[i] = 0.0f;  // zeroed tail for padded taps
  if (unit >= nunits) return;

  int lo = 0, hi = nimgs - 1;
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (imgs[mid].tile_begin <= unit) lo = mid; else hi = mid - 1;
  }
  const ImgDev& im = imgs[lo];
  const int nstrips = __builtin_amdgcn_readfirstlane(im.nstrips);
  const int crop_w = __builtin_amdgcn_readfirstlane(im.crop_w);
  const int crop_h = __builtin_amdgcn_readfirstlane(im.crop_h);
  const int flip = __builtin_amdgcn_readfirstlane(im.flip);
  const int band_rows = __builtin_amdgcn_readfirstlane(im.ty);
  const int strip_cols = __builtin_amdgcn_readfirstlane(im.tx);
  const int xs = kTapHeader + __builtin_amdgcn_readfirstlane(im.xwidth);
  const int ys = kTapHeader + __builtin_amdgcn_readfirstlane(im.ywidth);
  cgfloat* xtab = GLOBAL_PTR(const float, im.xtab);
  // Uniform pointer: the vertical taps are read with scalar loads (lgkmcnt),
  // which never wait on the vector loads of the next rows.
  const uint64_t yb = reinterpret_cast<uint64_t>(im.ytab);
  kfloat* ytab = (kfloat*)(((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)(yb >> 32)) << 32) |
                           (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)yb));
  char* dst = reinterpret_cast<char*>(im.dst);
  const int sstride = __builtin_amdgcn_readfirstlane((int)im.src_stride);
  const int src_h = __builtin_amdgcn_readfirstlane(im.src_h);
  const int64_t dstride = im.dst_stride;
  const int local = unit - __builtin_amdgcn_readfirstlane(im.tile_begin);
  const int band = local / nstrips;
  const int strip = local - band * nstrips;
  const int oy0 = band * band_rows;
  const int oy1 = min(oy0 + band_rows, crop_h);
  const int ox0 = strip * strip_cols;
  const int ox1 = min(ox0 + strip_cols, crop_w);

  // Source footprint of the strip (taps are monotone in the crop column).
  const int xa = flip ? crop_w - ox1 : ox0;
  const int xb = flip ? crop_w - 1 - ox0 : ox1 - 1;
  const int px_lo = __float_as_int(xtab[xa * xs]);
  const int px_hi = __float_as_int(xtab[xb * xs]) + __float_as_int(xtab[xb * xs + 1]) - 1;
  const int fb0 = (px_lo * C) & ~3;
  const int need = (px_hi + 1) * C - fb0;  // footprint bytes of the strip (<= kRowBytes)
  const uint64_t sbase = reinterpret_cast<uint64_t>(im.src);
  const uint64_t sb = ((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)(sbase >> 32)) << 32) |
                      (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)sbase);
  const __amdgpu_buffer_rsrc_t rsrc = __builtin_amdgcn_make_buffer_rsrc(
      reinterpret_cast<void*>(sb), (short)0, sstride * src_h, 0x00020000);
  // Only the dwords that hold footprint bytes are fetched.
  int voff[4];
#pragma unroll
  for (int j = 0; j < 4; j++) voff[j] = 4 * lane + 256 * j < need ? fb0 + 4 * lane + 256 * j : kNoLoad;

  // Horizontal taps of this lane's 4 output elements, for the whole band.
  const int nout = (ox1 - ox0) * C;
  const bool partial = (nout & (kOutPerLane - 1)) != 0;
  float wx[kOutPerLane][T];
  int pos[kOutPerLane];
#pragma unroll
  for (int j = 0; j < kOutPerLane; j++) {
    const int o = min(kOutPerLane * lane + j, nout - 1);
    const int px = o / C;
    const int c = o - px * C;
    const int ox = ox0 + px;
    const int xc = flip ? crop_w - 1 - ox : ox;
    cgfloat* xe = xtab + xc * xs;
    pos[j] = __float_as_int(xe[0]) * C - fb0 + c;
#pragma unroll
    for (int k = 0; k < T; k++) wx[j][k] = xe[kTapHeader + k];  // zero padded past the tap count
  }

  // The horizontal weights are loaded once; retire them here so the waits the
  // compiler places in the row loop only ever cover the row loads.
  __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0)

  auto load_rows = [&](Chunk* R, int y, bool live) {
    const int n0 = __float_as_int(ytab[y * ys]);
#pragma unroll
    for (int k = 0; k < T; k++) {
      if constexpr (MODE == 2) {
        R[k] = Chunk{{(uint32_t)(lane * 7 + k + n0), (uint32_t)(k * 3), (uint32_t)lane, (uint32_t)(k ^ lane)}};
      } else if constexpr (MODE == 4) {
        if (k >= T / 2) R[k] = load_chunk_if(rsrc, voff, (n0 + k) * sstride, live);
        else R[k] = Chunk{{(uint32_t)(lane * 7 + k + n0), (uint32_t)(k * 3), (uint32_t)lane, (uint32_t)(k ^ lane)}};
      } else {
        R[k] = load_chunk_if(rsrc, voff, (n0 + k) * sstride, live);
      }
    }
  };

  // V result (16 f32 per lane) -> the wave's LDS row: floats of bytes
  // 4l + 256j .. +3 go to vrow[4l + 256j], lanes 16 B apart per store.
  auto write_vrow = [&](const float* acc) {
#pragma unroll
    for (int j = 0; j < 4; j++)
      *reinterpret_cast<float4*>(vrow + 4 * lane + 256 * j) =
          make_float4(acc[4 * j], acc[4 * j + 1], acc[4 * j + 2], acc[4 * j + 3]);
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  };

  // H: horizontal taps of output row y from the LDS row, encode, store.
  auto h_store = [&](int y) {
    float out[kOutPerLane];
#pragma unroll
    for (int j = 0; j < kOutPerLane; j++) {
      float s = 0.0f;
      if constexpr (MODE == 3) {
        s = wx[j][0] * vrow[pos[j]];
      } else {
#pragma unroll
        for (int k = 0; k < T; k++) s = __builtin_fmaf(wx[j][k], vrow[pos[j] + k * C], s);
      }
      out[j] = encode(s);
    }
    const int o0 = kOutPerLane * lane;
    char* drow = dst + (int64_t)y * dstride;
    // MODE 9/10 (timing only): no stores (nimgs is never negative)
    if ((MODE != 9 && MODE != 10) || nimgs < 0)
    if (o0 + kOutPerLane <= nout) {  // one store instruction per row (lanes past nout masked)
      if constexpr (F32) {
        f32x4 v = {div255(out[0]), div255(out[1]), div255(out[2]), div255(out[3])};
        const int ob = (ox0 * C + o0) * 4;  // MODE 14: only whole 128-B lines of the strip's row segment
        if (MODE != 14 || (ob >= ((ox0 * C * 4 + 127) & ~127) && ob + 16 <= ((ox1 * C * 4) & ~127))) {
          if constexpr (MODE == 11 || MODE == 13)
            __builtin_nontemporal_store(v, reinterpret_cast<f32x4*>(reinterpret_cast<float*>(drow) + ox0 * C + o0));
          else
            *reinterpret_cast<__attribute__((address_space(1))) f32x4*>(GLOBAL_PTR(float, drow) + ox0 * C + o0) = v;
        }
      } else {
        *reinterpret_cast<__attribute__((address_space(1))) uint32_t*>(GLOBAL_PTR(uint8_t, drow) + ox0 * C + o0) =
            (uint32_t)out[0] | ((uint32_t)out[1] << 8) | ((uint32_t)out[2] << 16) | ((uint32_t)out[3] << 24);
      }
    }
    if (partial && o0 < nout && o0 + kOutPerLane > nout) {  // ragged strip end (uniform `partial`)
#pragma unroll
      for (int j = 0; j < kOutPerLane; j++) {
        if (o0 + j < nout) {
          if constexpr (F32) GLOBAL_PTR(float, drow)[ox0 * C + o0 + j] = div255(out[j]);
          else GLOBAL_PTR(uint8_t, drow)[ox0 * C + o0 + j] = (uint8_t)out[j];
        }
      }
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  };

  if constexpr (!RING) {
    // ---- gather: each output row sums its T source rows, loaded for it ----
    auto step = [&](const Chunk* R, int y) {
      kfloat* ye = ytab + y * ys;
      float acc[kChunk];
#pragma unroll
      for (int i = 0; i < kChunk; i++) acc[i] = 0.0f;
      if constexpr (MODE == 1) {
#pragma unroll
        for (int k = 0; k < T; k++)
#pragma unroll
          for (int i = 0; i < 4; i++) acc[4 * i] += __uint_as_float(R[k].d[i] & 0x3fffffffu);
      } else {
#pragma unroll
        for (int k = 0; k < T; k++) fma16(acc, ye[kTapHeader + k], R[k]);  // zero padded past the tap count
      }
      write_vrow(acc);
      h_store(y);
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
  } else {
    // ---- ring: every source row of the band is loaded once, kLook rows
    // ahead, into a register ring of kRing = T + kLook slots; the source-row
    // loop is unrolled by kRing so every slot index is static.  When row r is
    // the last tap of output row y, y's taps are exactly the T rows ending at
    // r (right-aligned weights, zero for the rows before y's first tap), all
    // resident in the ring: gather them (V), then H and store.  Requires the
    // last taps of consecutive output rows to strictly increase (at most one
    // output row ends per source row: downsampling); the host checks it.
    // rows loaded ahead (MODE 6/7/8: lookahead experiments)
    constexpr int kLook = MODE == 6 ? 9 : MODE == 7 ? 4 : MODE == 8 ? 12 : 6;
    constexpr int kRing = T + kLook;
    // right-aligned vertical table: {last row, count, w[T]} per output row
    kfloat* rtab = ytab;
    auto last_of = [&](int y) { return __float_as_int(rtab[min(y, crop_h - 1) * ys]); };
    const int rs = last_of(oy0) - (T - 1);
    const int re = last_of(oy1 - 1);
    int y = oy0;
    int ly = last_of(y);
    Chunk ring[kRing];
#pragma unroll
    for (int i = 0; i < kLook; i++) {
      if constexpr (MODE == 2) ring[i] = Chunk{{(uint32_t)(lane * 7 + i), (uint32_t)(rs * 3), (uint32_t)lane, (uint32_t)(i ^ lane)}};
      else if constexpr (MODE == 5) ring[i] = load_x4_if(rsrc, fb0 + 16 * lane, min(rs + i, re) * sstride, rs + i <= re);
      else ring[i] = load_chunk_if<(MODE == 12 || MODE == 13) ? 2 : 0>(rsrc, voff, min(rs + i, re) * sstride, rs + i <= re);
    }
    for (int base = rs; base <= re; base += kRing) {
      static_for<kRing>([&](auto ic) {
        constexpr int i = decltype(ic)::value;
        __builtin_amdgcn_sched_barrier(0);  // keep each row's work (and its load) in place
        const int r = base + i;
        if (r > re) return;
        // keep kLook rows in flight: slot (i + kLook) % kRing is free (its row
        // left the tap window of every open output row)
        if constexpr (MODE == 2) ring[(i + kLook) % kRing].d[0] = (uint32_t)(r + lane);
        else if constexpr (MODE == 5)
          ring[(i + kLook) % kRing] = load_x4_if(rsrc, fb0 + 16 * lane, min(r + kLook, re) * sstride, r + kLook <= re);
        else ring[(i + kLook) % kRing] = load_chunk_if<(MODE == 12 || MODE == 13) ? 2 : 0>(rsrc, voff, min(r + kLook, re) * sstride, r + kLook <= re);
        if (r == ly) {  // output row y ends at source row r (at most one: checked on the host)
          kfloat* we = rtab + y * ys + kTapHeader;
          float acc[kChunk];
#pragma unroll
          for (int q = 0; q < kChunk; q++) acc[q] = 0.0f;
#pragma unroll
          for (int k = 0; k < T; k++) {
            const Chunk& c = ring[(i + kRing - (T - 1) + k) % kRing];
            if constexpr (MODE == 1 || MODE == 10) {
#pragma unroll
              for (int q = 0; q < 4; q++) acc[4 * q] += __uint_as_float(c.d[q] & 0x3fffffffu);
            } else {
              fma16(acc, we[k], c);
            }
          }
          write_vrow(acc);
          h_store(y);
          ++y;
          ly = y < oy1 ? last_of(y) : 0x7fffffff;
        }
      });
    }
  }
}

using WaveKernel = void (*)(const ImgDev*, int, int, int);

template <int C, bool F32, int T>
WaveKernel select_ct(const WaveCfg& cfg) {
  if (cfg.ring) {
    if constexpr (C == 3 && F32 && T == 8) {
      if (cfg.mode == 1) return resample_wave<C, F32, T, 1, true>;
      if (cfg.mode == 2) return resample_wave<C, F32, T, 2, true>;
      if (cfg.mode == 3) return resample_wave<C, F32, T, 3, true>;
      if (cfg.mode == 5) return resample_wave<C, F32, T, 5, true>;
      if (cfg.mode == 6) return resample_wave<C, F32, T, 6, true>;
      if (cfg.mode == 7) return resample_wave<C, F32, T, 7, true>;
      if (cfg.mode == 8) return resample_wave<C, F32, T, 8, true>;
      if (cfg.mode == 9) return resample_wave<C, F32, T, 9, true>;
      if (cfg.mode == 10) return resample_wave<C, F32, T, 10, true>;
      if (cfg.mode == 11) return resample_wave<C, F32, T, 11, true>;
      if (cfg.mode == 12) return resample_wave<C, F32, T, 12, true>;
      if (cfg.mode == 13) return resample_wave<C, F32, T, 13, true>;
      if (cfg.mode == 14) return resample_wave<C, F32, T, 14, true>;
    }
    return resample_wave<C, F32, T, 0, true>;
  }
  if constexpr (C == 3 && F32 && T == 8) {
    if (cfg.mode == 1) return resample_wave<C, F32, T, 1>;
    if (cfg.mode == 2) return resample_wave<C, F32, T, 2>;
    if (cfg.mode == 3) return resample_wave<C, F32, T, 3>;
    if (cfg.mode == 4) return resample_wave<C, F32, T, 4>;
  }
  return resample_wave<C, F32, T, 0>;
}

template <int C, bool F32>
WaveKernel select_c(const WaveCfg& cfg) {
  switch (cfg.taps) {
    case 2: return select_ct<C, F32, 2>(cfg);
    case 3: return select_ct<C, F32, 3>(cfg);
    case 4: return select_ct<C, F32, 4>(cfg);
    case 5: return select_ct<C, F32, 5>(cfg);
    case 6: return select_ct<C, F32, 6>(cfg);
    case 8: return select_ct<C, F32, 8>(cfg);
    case 9: return select_ct<C, F32, 9>(cfg);
    case 10: return select_ct<C, F32, 10>(cfg);
    case 12: return select_ct<C, F32, 12>(cfg);
    case 14: return select_ct<C, F32, 14>(cfg);
    case 17: return select_ct<C, F32, 17>(cfg);
    default: return nullptr;
  }
}

WaveKernel select_kernel(const WaveCfg& cfg) {
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

int lds_bytes(const WaveCfg& cfg) { return kWaves * wave_row_floats(cfg.taps, cfg.channels) * (int)sizeof(float); }

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
  const int blocks = (cfg.nunits + kWaves - 1) / kWaves;
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
  return blocks * kWaves * cus;
}

}  // namespace mxd
