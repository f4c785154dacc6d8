// wave.hip -- the fast path of the fused resize + crop (+ hflip) (+ /255) stage.
//
// Same arithmetic as resample.hip (stbir triangle taps from the shared tables,
// vertical pass first in byte units, f32 FMA accumulation, stbir encode), but
// organised so that no workgroup barrier is ever needed:
//
//   one WAVE owns one unit = (image, band of output rows, strip of output
//   columns).  Lane l holds 16 source bytes of the strip's footprint, so one
//   wave spans 1024 source bytes of a row (one dwordx4 load per lane, 1 KiB
//   per wave-instruction).  For each output row y of the band:
//     V  lane sums its 16 byte columns over the T vertical taps of y from the
//        T source rows it holds in registers and writes 16 f32 to the wave's
//        private LDS row.  Then it moves on to y+1: source rows shared by the
//        taps of y and y+1 (about half of them when downsampling) stay in
//        registers (shifted by the uniform row advance d); only the new rows
//        are loaded, and those loads are in flight during
//     H  lane l produces output elements 4l..4l+3 of the strip row (C
//        channels interleaved) from the LDS row with their T horizontal taps
//        (weights in registers for the whole band), rounds like stbir's encode
//        and stores 4 f32 (exact q/255, one 16-byte store) or 4 u8.
//   Waves never wait for each other; the CU interleaves the waves of many
//   units so that loads of their next rows are always in flight.
// Tap counts are padded to the template T with zero weights and clamped row
// indices; the LDS row has a zeroed tail so padded taps read finite values.
#include <hip/hip_runtime.h>

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

struct alignas(4) Chunk {
  uint32_t d[4];
};

// Loads the lane's 16 bytes; only the first nd dwords when the chunk would
// cross src_stride (the last lane of a strip at the right edge of the image,
// where the bytes past the row may be past the end of the buffer).
__device__ __forceinline__ Chunk load_chunk(const uint8_t* p, int nd) {
  const __attribute__((address_space(1))) uint32_t* q = GLOBAL_PTR(const uint32_t, p);
  Chunk r;
  if (nd == 4) {
    r.d[0] = q[0];
    r.d[1] = q[1];
    r.d[2] = q[2];
    r.d[3] = q[3];
  } else {
#pragma unroll
    for (int i = 0; i < 4; i++) r.d[i] = i < nd ? q[i] : 0u;
  }
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

// R[k] <- R[k + D] for k < m (m uniform): rows shared by consecutive outputs.
template <int T, int D>
__device__ __forceinline__ void shift_rows(Chunk* R, int m) {
#pragma unroll
  for (int k = 0; k + D < T; k++)
    if (k < m) R[k] = R[k + D];
}

template <int T>
__device__ __forceinline__ void shift_rows_dyn(Chunk* R, int d, int m) {
  switch (d) {
#define MXD_SHIFT_CASE(D)                        \
  case D:                                        \
    if constexpr (D < T) shift_rows<T, D>(R, m); \
    break;
    MXD_SHIFT_CASE(1)
    MXD_SHIFT_CASE(2)
    MXD_SHIFT_CASE(3)
    MXD_SHIFT_CASE(4)
    MXD_SHIFT_CASE(5)
    MXD_SHIFT_CASE(6)
    MXD_SHIFT_CASE(7)
    MXD_SHIFT_CASE(8)
    MXD_SHIFT_CASE(9)
    MXD_SHIFT_CASE(10)
    MXD_SHIFT_CASE(11)
    MXD_SHIFT_CASE(12)
    MXD_SHIFT_CASE(13)
    MXD_SHIFT_CASE(14)
    MXD_SHIFT_CASE(15)
    MXD_SHIFT_CASE(16)
#undef MXD_SHIFT_CASE
    default:
      break;
  }
}

// MODE: 0 = the product kernel.  Diagnostic ablations (selected only through
// the MXD_WAVE_ABLATE environment variable, C=3/f32/T=8 only):
//   1 = no vertical arithmetic (loads kept live with one op per dword),
//   2 = no source loads (rows synthesised from the lane id),
//   3 = no horizontal pass (encode of the LDS value at the tap base only).
template <int C, bool F32, int T, int MODE = 0>
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
  cgfloat* ytab = GLOBAL_PTR(const float, im.ytab);
  const uint8_t* src = im.src;
  char* dst = reinterpret_cast<char*>(im.dst);
  const int64_t sstride = im.src_stride;
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
  const bool vact = fb0 + lane * kChunk < (px_hi + 1) * C;
  const int nd = vact ? (int)min<int64_t>(4, (sstride - (fb0 + lane * kChunk)) / 4) : 0;

  // Horizontal taps of this lane's 4 output elements, for the whole band.
  const int nout = (ox1 - ox0) * C;
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
    const int ntx = __float_as_int(xe[1]);
    pos[j] = __float_as_int(xe[0]) * C - fb0 + c;
#pragma unroll
    for (int k = 0; k < T; k++) wx[j][k] = k < ntx ? xe[kTapHeader + k] : 0.0f;
  }

  const uint8_t* __restrict__ col = src + fb0 + lane * kChunk;
  Chunk R[T];
  // Loads rows n0 + min(k, nt-1) for k in [m, T).
  auto load_rows = [&](int n0, int nt, int m) {
#pragma unroll
    for (int k = 0; k < T; k++) {
      if (k >= m) {
        const int row = n0 + min(k, nt - 1);
        if constexpr (MODE == 2) {
          R[k] = Chunk{{(uint32_t)(lane * 7 + row), (uint32_t)(row * 3), (uint32_t)lane, (uint32_t)(row ^ lane)}};
        } else {
          if (vact) R[k] = load_chunk(col + row * sstride, nd);
          else R[k] = Chunk{{0u, 0u, 0u, 0u}};
        }
      }
    }
  };

  cgfloat* ye = ytab + oy0 * ys;
  int n0 = __float_as_int(ye[0]);
  int nt = __float_as_int(ye[1]);
  load_rows(n0, nt, 0);
  for (int y = oy0; y < oy1; y++) {
    // ---- V: vertical taps of row y -> LDS ----
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
      for (int k = 0; k < T; k++) fma16(acc, k < nt ? ye[kTapHeader + k] : 0.0f, R[k]);
    }
    float4* dv = reinterpret_cast<float4*>(vrow + lane * kChunk);
    dv[0] = make_float4(acc[0], acc[1], acc[2], acc[3]);
    dv[1] = make_float4(acc[4], acc[5], acc[6], acc[7]);
    dv[2] = make_float4(acc[8], acc[9], acc[10], acc[11]);
    dv[3] = make_float4(acc[12], acc[13], acc[14], acc[15]);

    // ---- rows for y+1: keep the shared ones, load the rest (in flight during H) ----
    if (y + 1 < oy1) {
      cgfloat* yn = ye + ys;
      const int n0n = __float_as_int(yn[0]);
      const int ntn = __float_as_int(yn[1]);
      const int d = n0n - n0;
      const int m = (d > 0) ? min(max(nt - d, 0), ntn) : (d == 0 ? min(nt, ntn) : 0);
      if (d > 0) shift_rows_dyn<T>(R, d, m);
      load_rows(n0n, ntn, m);
      ye = yn;
      n0 = n0n;
      nt = ntn;
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");

    // ---- H: horizontal taps from LDS, encode, store ----
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
    if (o0 < nout) {
      char* drow = dst + (int64_t)y * dstride;
      if constexpr (F32) {
        gfloat* d = GLOBAL_PTR(float, drow) + ox0 * C + o0;
        if (o0 + kOutPerLane <= nout) {
          f32x4 v = {div255(out[0]), div255(out[1]), div255(out[2]), div255(out[3])};
          *reinterpret_cast<__attribute__((address_space(1))) f32x4*>(d) = v;
        } else {
#pragma unroll
          for (int j = 0; j < kOutPerLane; j++)
            if (o0 + j < nout) d[j] = div255(out[j]);
        }
      } else {
        __attribute__((address_space(1))) uint8_t* d = GLOBAL_PTR(uint8_t, drow) + ox0 * C + o0;
        if (o0 + kOutPerLane <= nout) {
          *reinterpret_cast<__attribute__((address_space(1))) uint32_t*>(d) =
              (uint32_t)out[0] | ((uint32_t)out[1] << 8) | ((uint32_t)out[2] << 16) | ((uint32_t)out[3] << 24);
        } else {
#pragma unroll
          for (int j = 0; j < kOutPerLane; j++)
            if (o0 + j < nout) d[j] = (uint8_t)out[j];
        }
      }
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  }
}

template <int C, bool F32, int T, int MODE = 0>
int launch_ct(const WaveCfg& cfg, const ImgDev* imgs, hipStream_t s) {
  if constexpr (MODE == 0 && C == 3 && F32 && T == 8) {
    switch (cfg.mode) {
      case 1: return launch_ct<C, F32, T, 1>(cfg, imgs, s);
      case 2: return launch_ct<C, F32, T, 2>(cfg, imgs, s);
      case 3: return launch_ct<C, F32, T, 3>(cfg, imgs, s);
      default: break;
    }
  }
  const int rowf = wave_row_floats(cfg.taps, C);
  const int blocks = (cfg.nunits + kWaves - 1) / kWaves;
  hipLaunchKernelGGL((resample_wave<C, F32, T, MODE>), dim3(blocks), dim3(kWaves * kLanes),
                     kWaves * rowf * (int)sizeof(float), s, imgs, cfg.nimgs, cfg.nunits, rowf);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

template <int C, bool F32>
int launch_c(const WaveCfg& cfg, const ImgDev* imgs, hipStream_t s) {
  switch (cfg.taps) {
    case 2: return launch_ct<C, F32, 2>(cfg, imgs, s);
    case 3: return launch_ct<C, F32, 3>(cfg, imgs, s);
    case 4: return launch_ct<C, F32, 4>(cfg, imgs, s);
    case 5: return launch_ct<C, F32, 5>(cfg, imgs, s);
    case 6: return launch_ct<C, F32, 6>(cfg, imgs, s);
    case 8: return launch_ct<C, F32, 8>(cfg, imgs, s);
    case 9: return launch_ct<C, F32, 9>(cfg, imgs, s);
    case 10: return launch_ct<C, F32, 10>(cfg, imgs, s);
    case 12: return launch_ct<C, F32, 12>(cfg, imgs, s);
    case 14: return launch_ct<C, F32, 14>(cfg, imgs, s);
    case 17: return launch_ct<C, F32, 17>(cfg, imgs, s);
    default: return -2;
  }
}

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
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  switch (cfg.channels * 2 + (cfg.f32 ? 1 : 0)) {
    case 2: return launch_c<1, false>(cfg, imgs, s);
    case 3: return launch_c<1, true>(cfg, imgs, s);
    case 4: return launch_c<2, false>(cfg, imgs, s);
    case 5: return launch_c<2, true>(cfg, imgs, s);
    case 6: return launch_c<3, false>(cfg, imgs, s);
    case 7: return launch_c<3, true>(cfg, imgs, s);
    default: return -2;
  }
}

}  // namespace mxd
