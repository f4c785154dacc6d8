// wave.hip -- the fast path of the fused resize + crop (+ hflip) (+ /255) stage.
//
// Same arithmetic as resample.hip (stbir triangle taps from the shared tables,
// vertical pass first in byte units, f32 FMA accumulation, stbir encode), but
// organised so that no workgroup barrier is ever needed:
//
//   one WAVE owns one unit = (image, band of output rows, strip of <= 64
//   output columns).  Lane l holds 12 source bytes (4 RGB pixels) of the
//   strip's footprint, so one wave spans 768 source bytes per row.
//   For each output row y of the band:
//     V  lane sums its 12 byte columns over the T vertical taps of y straight
//        from HBM (dwordx3 loads, one per tap, issued together; rows beyond the
//        tap count are clamped and weighted 0), and writes 12 f32 to the
//        wave's private LDS row;
//        the loads for row y+1 are issued right after, so they fly during
//     H  lane l produces output pixel l of the strip (C channels) from the LDS
//        row with its T horizontal taps (weights kept in registers for the
//        whole band), rounds like stbir and stores C f32 (exact q/255) or u8.
//   Waves never wait for each other; 16 waves per CU keep the loads of their
//   next rows in flight while others compute.
// Tap counts are padded to the template T with zero weights; the LDS row has
// a zeroed tail so padded taps read finite values.
#include <hip/hip_runtime.h>

#include "resample.h"

namespace mxd {
namespace {

constexpr int kWaves = 4;
constexpr int kLanes = 64;
constexpr int kChunk = 12;                    // source bytes per lane per row
constexpr int kRowBytes = kLanes * kChunk;    // 768 source bytes per wave row

__device__ __forceinline__ int xcd_remap(int b, int n) {
  const int q = n >> 3, r = n & 7;
  const int xcd = b & 7, idx = b >> 3;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + idx;
}

__device__ __forceinline__ float div255(float q) {
  const float inv = 1.0f / 255.0f;
  const float r = q * inv;
  const float e = __builtin_fmaf(-r, 255.0f, q);
  return __builtin_fmaf(e, inv, r);
}

__device__ __forceinline__ float encode(float v) { return truncf(fminf(fmaxf(v + 0.5f, 0.0f), 255.0f)); }

// Image data, tap tables and outputs live in global memory; pointers that come
// out of the descriptor table are generic, so cast them explicitly (otherwise
// hipcc emits flat_* accesses, which also count on lgkmcnt and serialise).
#define GLOBAL_PTR(T, p) ((__attribute__((address_space(1))) T*)(p))

struct alignas(4) B12 {
  uint32_t a, b, c;
};

__device__ __forceinline__ B12 load12(const uint8_t* p) {
  const __attribute__((address_space(1))) uint32_t* q = GLOBAL_PTR(const uint32_t, p);
  B12 r;
  r.a = q[0];
  r.b = q[1];
  r.c = q[2];
  return r;
}

__device__ __forceinline__ void fma12(float* acc, float w, const B12& v) {
  const uint32_t d[3] = {v.a, v.b, v.c};
#pragma unroll
  for (int i = 0; i < 3; i++) {
    acc[4 * i + 0] = __builtin_fmaf(w, (float)(d[i] & 0xffu), acc[4 * i + 0]);
    acc[4 * i + 1] = __builtin_fmaf(w, (float)((d[i] >> 8) & 0xffu), acc[4 * i + 1]);
    acc[4 * i + 2] = __builtin_fmaf(w, (float)((d[i] >> 16) & 0xffu), acc[4 * i + 2]);
    acc[4 * i + 3] = __builtin_fmaf(w, (float)(d[i] >> 24), acc[4 * i + 3]);
  }
}

template <int C, bool F32, int T>
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
  const int tile_begin = __builtin_amdgcn_readfirstlane(im.tile_begin);
  const int nstrips = __builtin_amdgcn_readfirstlane(im.nstrips);
  const int crop_w = __builtin_amdgcn_readfirstlane(im.crop_w);
  const int crop_h = __builtin_amdgcn_readfirstlane(im.crop_h);
  const int flip = __builtin_amdgcn_readfirstlane(im.flip);
  const int band_rows = __builtin_amdgcn_readfirstlane(im.ty);
  const int strip_cols = __builtin_amdgcn_readfirstlane(im.tx);
  const int xs = kTapHeader + __builtin_amdgcn_readfirstlane(im.xwidth);
  const int ys = kTapHeader + __builtin_amdgcn_readfirstlane(im.ywidth);
  const __attribute__((address_space(1))) float* xtab = GLOBAL_PTR(const float, im.xtab);
  const __attribute__((address_space(1))) float* ytab = GLOBAL_PTR(const float, im.ytab);
  const uint8_t* src = im.src;
  char* dst = reinterpret_cast<char*>(im.dst);
  const int64_t sstride = im.src_stride;
  const int64_t dstride = im.dst_stride;
  const int local = unit - tile_begin;
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
  const int fb0 = (px_lo * C) / kChunk * kChunk;
  const bool vact = fb0 + lane * kChunk < (px_hi + 1) * C;

  // Horizontal taps of this lane's output column, for the whole band.
  const int ox = ox0 + lane;
  const bool hact = ox < ox1;
  const int xc = flip ? crop_w - 1 - min(ox, ox1 - 1) : min(ox, ox1 - 1);
  const __attribute__((address_space(1))) float* xe = xtab + xc * xs;
  const int ntx = __float_as_int(xe[1]);
  const int pos = __float_as_int(xe[0]) * C - fb0;
  float wx[T];
#pragma unroll
  for (int k = 0; k < T; k++) wx[k] = k < ntx ? xe[kTapHeader + k] : 0.0f;

  const uint8_t* __restrict__ col = src + fb0 + lane * kChunk;
  B12 R[T];
  auto prefetch = [&](int y) {
    const __attribute__((address_space(1))) float* ye = ytab + y * ys;
    const int n0 = __float_as_int(ye[0]);
    const int last = n0 + __float_as_int(ye[1]) - 1;
#pragma unroll
    for (int k = 0; k < T; k++) {
      const int row = min(n0 + k, last);
      if (vact) R[k] = load12(col + row * sstride);
      else R[k] = B12{0u, 0u, 0u};
    }
  };

  prefetch(oy0);
  for (int y = oy0; y < oy1; y++) {
    // ---- V: vertical taps of row y -> LDS ----
    const __attribute__((address_space(1))) float* ye = ytab + y * ys;
    const int nty = __float_as_int(ye[1]);
    float acc[kChunk];
#pragma unroll
    for (int i = 0; i < kChunk; i++) acc[i] = 0.0f;
#pragma unroll
    for (int k = 0; k < T; k++) fma12(acc, k < nty ? ye[kTapHeader + k] : 0.0f, R[k]);
    float4* dv = reinterpret_cast<float4*>(vrow + lane * kChunk);
    dv[0] = make_float4(acc[0], acc[1], acc[2], acc[3]);
    dv[1] = make_float4(acc[4], acc[5], acc[6], acc[7]);
    dv[2] = make_float4(acc[8], acc[9], acc[10], acc[11]);
    if (y + 1 < oy1) prefetch(y + 1);
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");

    // ---- H: horizontal taps from LDS, encode, store ----
    float out[C];
#pragma unroll
    for (int c = 0; c < C; c++) {
      float s = 0.0f;
#pragma unroll
      for (int k = 0; k < T; k++) s = __builtin_fmaf(wx[k], vrow[pos + k * C + c], s);
      out[c] = encode(s);
    }
    if (hact) {
      char* drow = dst + (int64_t)y * dstride;
      if constexpr (F32) {
        __attribute__((address_space(1))) float* d = GLOBAL_PTR(float, drow) + ox * C;
#pragma unroll
        for (int c = 0; c < C; c++) d[c] = div255(out[c]);
      } else {
        __attribute__((address_space(1))) uint8_t* d = GLOBAL_PTR(uint8_t, drow) + ox * C;
#pragma unroll
        for (int c = 0; c < C; c++) d[c] = (uint8_t)out[c];
      }
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  }
}

template <int C, bool F32, int T>
int launch_ct(const WaveCfg& cfg, const ImgDev* imgs, hipStream_t s) {
  const int rowf = wave_row_floats(cfg.taps, C);
  const int blocks = (cfg.nunits + kWaves - 1) / kWaves;
  hipLaunchKernelGGL((resample_wave<C, F32, T>), dim3(blocks), dim3(kWaves * kLanes),
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
    case 20: return launch_ct<C, F32, 20>(cfg, imgs, s);
    case 24: return launch_ct<C, F32, 24>(cfg, imgs, s);
    default: return -2;
  }
}

}  // namespace

int wave_taps_bucket(int taps) {
  static const int kB[] = {2, 3, 4, 5, 6, 8, 9, 10, 12, 14, 17, 20, 24};
  for (int b : kB)
    if (taps <= b) return b;
  return -1;
}

int wave_row_floats(int taps, int channels) { return (kRowBytes + taps * channels + 3) & ~3; }

int wave_row_bytes() { return kRowBytes; }

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
