// resample.hip -- fused resize (stbir triangle filter) + crop (+ hflip)
// (+ u8 -> f32 /255) for gfx950.
//
// Replaces, per image, core::image::resize -> stbir_resize_uint8_linear
// (mlx/data/core/image/ImageTransform.cpp:41-62), core::image::crop
// (:64-73 -> array::sub, Array.cpp:544-583), core::image::hflip (:123-140) and
// the benchmark's x.astype("float32")/255, in one pass that reads only the
// source pixels the kept crop window depends on.
//
// Work decomposition: one 256-thread workgroup per tile = (image, band of
// output rows, strip of output columns).  Per group of G output rows:
//   V phase  every thread owns 16-byte columns of the tile's source footprint
//            and sums the tile's vertical taps straight from HBM
//            (global_load_dwordx4, coalesced along the row), converting bytes
//            to f32 once per load; the G f32 rows land in LDS.
//   H phase  every thread produces 4 consecutive output elements of a row from
//            the LDS rows with the horizontal taps (tap table staged in LDS),
//            rounds like stbir's encode (trunc(v+0.5) clamped), and writes u8
//            or the exact f32 q/255.0f with 16-byte (f32) / 4-byte (u8) stores.
// Arithmetic is in byte units (v = sum w*p), f32 accumulation with FMA.
// 4 channels with ALPHA (stb_image_resize2's STBIR_RGBA, the layout
// core::image::resize passes for c = 4, ImageTransform.cpp:49-58) follow
// stbir's float operations instead: every byte decoded to [0, 1] (b * 1/255),
// colours multiplied by their decoded alpha, both passes, colours multiplied
// by 1 / filtered alpha unless that alpha is below stbir's tiny threshold,
// then encoded as (uint8)trunc(clamp(v * 255 + 0.5)) with an unfused multiply
// and add -- bit-exact to oracle/stbir_oracle.c orc_resize_crop_vfirst_rgba.
// Workgroup ids are remapped so that tiles of the same image run on the same
// XCD (blocks b, b+8, ... share an XCD): the vertical halo of adjacent bands
// then hits that XCD's L2.
#include <hip/hip_runtime.h>

#include "resample.h"

namespace mxd {
namespace {

constexpr int kThreads = 256;

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

__device__ __forceinline__ float encode(float v) {
  // stbir encode: (uint8)trunc(clamp(v*255 + 0.5, 0, 255)); here v is in byte units.
  return truncf(fminf(fmaxf(v + 0.5f, 0.0f), 255.0f));
}

constexpr float kInv255 = 1.0f / 255.0f;
// stbir's "small float" below which a filtered alpha counts as zero (colours
// then stay premultiplied, i.e. ~0): 1 / 2^120.
constexpr float kTinyAlpha = 7.52316384526264e-37f;

// ALPHA: the chunk holds whole RGBA pixels (16-byte chunks of a 4-channel row
// start on a pixel); colours enter premultiplied.
template <int VEC, bool ALPHA>
struct Chunk;

template <bool ALPHA>
struct Chunk<16, ALPHA> {
  uint4 v;
  __device__ __forceinline__ void load(const uint8_t* p) { v = *reinterpret_cast<const uint4*>(p); }
  __device__ __forceinline__ void fma_into(float* acc, float w) const {
    const uint32_t d[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
    for (int i = 0; i < 4; i++) {
      if constexpr (ALPHA) {
        const float a = (float)(d[i] >> 24) * kInv255;
        acc[4 * i + 0] = __builtin_fmaf(w, (float)(d[i] & 0xffu) * kInv255 * a, acc[4 * i + 0]);
        acc[4 * i + 1] = __builtin_fmaf(w, (float)((d[i] >> 8) & 0xffu) * kInv255 * a, acc[4 * i + 1]);
        acc[4 * i + 2] = __builtin_fmaf(w, (float)((d[i] >> 16) & 0xffu) * kInv255 * a, acc[4 * i + 2]);
        acc[4 * i + 3] = __builtin_fmaf(w, a, acc[4 * i + 3]);
      } else {
        acc[4 * i + 0] = __builtin_fmaf(w, (float)(d[i] & 0xffu), acc[4 * i + 0]);
        acc[4 * i + 1] = __builtin_fmaf(w, (float)((d[i] >> 8) & 0xffu), acc[4 * i + 1]);
        acc[4 * i + 2] = __builtin_fmaf(w, (float)((d[i] >> 16) & 0xffu), acc[4 * i + 2]);
        acc[4 * i + 3] = __builtin_fmaf(w, (float)(d[i] >> 24), acc[4 * i + 3]);
      }
    }
  }
};

// One byte; ALPHA: byte `c` of an RGBA pixel, its alpha 3 - c bytes on.
template <bool ALPHA>
struct Chunk<1, ALPHA> {
  float v;
  __device__ __forceinline__ void load(const uint8_t* p, int c = 3) {
    v = (float)*p;
    if constexpr (ALPHA) {
      v = v * kInv255;
      if (c < 3) v = v * ((float)p[3 - c] * kInv255);
    }
  }
  __device__ __forceinline__ void fma_into(float* acc, float w) const { acc[0] = __builtin_fmaf(w, v, acc[0]); }
};

template <int VEC, int C, bool F32, bool ALPHA>
__global__ __launch_bounds__(kThreads) void resample_tiles(const ImgDev* __restrict__ imgs, int nimgs, int vw,
                                                           int xs, int ys, int x_off, int y_off) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  const int tid = threadIdx.x;
  const int t = xcd_remap(blockIdx.x, gridDim.x);
  int lo = 0, hi = nimgs - 1;
  while (lo < hi) {  // image owning logical tile t
    const int mid = (lo + hi + 1) >> 1;
    if (imgs[mid].tile_begin <= t) lo = mid; else hi = mid - 1;
  }
  const ImgDev im = imgs[lo];
  const int local = t - im.tile_begin;
  const int band = local / im.nstrips;
  const int strip = local - band * im.nstrips;
  struct {
    int oy0, oy1, ox0, ox1, fb0, nchunks, group;
  } tile;
  tile.oy0 = band * im.ty;
  tile.oy1 = min(tile.oy0 + im.ty, im.crop_h);
  tile.ox0 = strip * im.tx;
  tile.ox1 = min(tile.ox0 + im.tx, im.crop_w);
  tile.group = im.group;
  {
    // Source footprint of the strip: taps are monotone in the crop column.
    const int xa = im.flip ? im.crop_w - tile.ox1 : tile.ox0;
    const int xb = im.flip ? im.crop_w - 1 - tile.ox0 : tile.ox1 - 1;
    const float* ea = im.xtab + (size_t)xa * (kTapHeader + im.xwidth);
    const float* eb = im.xtab + (size_t)xb * (kTapHeader + im.xwidth);
    const int px_lo = __float_as_int(ea[0]);
    const int px_hi = __float_as_int(eb[0]) + __float_as_int(eb[1]) - 1;
    tile.fb0 = (px_lo * C) & ~(VEC - 1);
    tile.nchunks = ((px_hi + 1) * C - tile.fb0 + VEC - 1) / VEC;
  }
  float* __restrict__ vbuf = smem;
  float* __restrict__ xinf = smem + x_off;
  float* __restrict__ yinf = smem + y_off;
  const int tw = tile.ox1 - tile.ox0;
  const int th = tile.oy1 - tile.oy0;
  const int G = tile.group;
  const int nchunks = tile.nchunks;

  // Stage the tile's tap tables in LDS.  x entries hold the LDS position of
  // (first tap, channel 0) instead of the source index.
  for (int i = tid; i < tw * xs; i += kThreads) {
    const int xl = i / xs, k = i - xl * xs;
    const int ox = tile.ox0 + xl;
    const int x = im.flip ? im.crop_w - 1 - ox : ox;
    const float* e = im.xtab + (size_t)x * (kTapHeader + im.xwidth);
    float v;
    if (k == 0)
      v = __int_as_float(__float_as_int(e[0]) * C - tile.fb0);
    else if (k < kTapHeader + im.xwidth)
      v = e[k];
    else
      v = 0.0f;
    xinf[i] = v;
  }
  for (int i = tid; i < th * ys; i += kThreads) {
    const int yl = i / ys, k = i - yl * ys;
    const float* e = im.ytab + (size_t)(tile.oy0 + yl) * (kTapHeader + im.ywidth);
    yinf[i] = k < kTapHeader + im.ywidth ? e[k] : 0.0f;
  }
  __syncthreads();

  const uint8_t* __restrict__ src = im.src + tile.fb0;
  const int64_t sstride = im.src_stride;
  const int nout = tw * C;
  const int nq = (nout + 3) >> 2;
  const bool vec_store =
      ((reinterpret_cast<uintptr_t>(im.dst) | (uintptr_t)im.dst_stride) & (F32 ? 15 : 3)) == 0 &&
      ((tile.ox0 * C) & 3) == 0;

  for (int oy = tile.oy0; oy < tile.oy1; oy += G) {
    const int ng = min(G, tile.oy1 - oy);

    // ---- V phase: vertical taps over the footprint, HBM -> LDS (f32) ----
    for (int it = tid; it < ng * nchunks; it += kThreads) {
      const int g = it / nchunks;
      const int ch = it - g * nchunks;
      const float* yi = yinf + (oy - tile.oy0 + g) * ys;
      const int n0 = __float_as_int(yi[0]);
      const int nt = __float_as_int(yi[1]);
      const uint8_t* p = src + (int64_t)n0 * sstride + ch * VEC;
      float acc[VEC];
#pragma unroll
      for (int i = 0; i < VEC; i++) acc[i] = 0.0f;
      int k = 0;
      if constexpr (VEC == 1) {
        const int c = (tile.fb0 + ch) % C;  // fb0 starts a pixel
        for (; k < nt; k++) {
          Chunk<1, ALPHA> c0;
          c0.load(p + k * sstride, c);
          c0.fma_into(acc, yi[kTapHeader + k]);
        }
      } else {
        for (; k + 4 <= nt; k += 4) {
          Chunk<VEC, ALPHA> c0, c1, c2, c3;
          c0.load(p + (k + 0) * sstride);
          c1.load(p + (k + 1) * sstride);
          c2.load(p + (k + 2) * sstride);
          c3.load(p + (k + 3) * sstride);
          c0.fma_into(acc, yi[kTapHeader + k + 0]);
          c1.fma_into(acc, yi[kTapHeader + k + 1]);
          c2.fma_into(acc, yi[kTapHeader + k + 2]);
          c3.fma_into(acc, yi[kTapHeader + k + 3]);
        }
        for (; k < nt; k++) {
          Chunk<VEC, ALPHA> c0;
          c0.load(p + k * sstride);
          c0.fma_into(acc, yi[kTapHeader + k]);
        }
      }
      float* dstv = vbuf + g * vw + ch * VEC;
      if constexpr (VEC % 4 == 0) {
#pragma unroll
        for (int i = 0; i < VEC; i += 4)
          *reinterpret_cast<float4*>(dstv + i) = make_float4(acc[i], acc[i + 1], acc[i + 2], acc[i + 3]);
      } else {
#pragma unroll
        for (int i = 0; i < VEC; i++) dstv[i] = acc[i];
      }
    }
    __syncthreads();

    // ---- H phase: horizontal taps from LDS, encode, store ----
    for (int it = tid; it < ng * nq; it += kThreads) {
      const int g = it / nq;
      const int q = it - g * nq;
      const float* vr = vbuf + g * vw;
      float res[4];
#pragma unroll
      for (int j = 0; j < 4; j++) {
        const int o = 4 * q + j;
        float s = 0.0f;
        if (o < nout) {
          const int xl = o / C;
          const int c = o - xl * C;
          const float* xi = xinf + xl * xs;
          const int base = __float_as_int(xi[0]) + c;
          const int nt = __float_as_int(xi[1]);
          for (int k = 0; k < nt; k++) s = __builtin_fmaf(xi[kTapHeader + k], vr[base + k * C], s);
        }
        res[j] = s;
      }
      if constexpr (ALPHA) {
        // the thread's 4 elements are one RGBA pixel (tiles start on a pixel)
        if (res[3] >= kTinyAlpha) {
          const float ia = 1.0f / res[3];
#pragma unroll
          for (int j = 0; j < 3; j++) res[j] = res[j] * ia;
        }
        {
#pragma clang fp contract(off)  // v * 255, then + 0.5 (built with -ffp-contract=on: the pragma holds)
#pragma unroll
          for (int j = 0; j < 4; j++) res[j] = encode(res[j] * 255.0f);
        }
      } else {
#pragma unroll
        for (int j = 0; j < 4; j++) res[j] = encode(res[j]);
      }
      const int64_t row = (int64_t)(oy + g) * im.dst_stride;
      const int o0 = tile.ox0 * C + 4 * q;
      if constexpr (F32) {
        float* d = reinterpret_cast<float*>(reinterpret_cast<char*>(im.dst) + row) + o0;
        const float4 f = make_float4(div255(res[0]), div255(res[1]), div255(res[2]), div255(res[3]));
        if (vec_store && 4 * q + 4 <= nout) {
          *reinterpret_cast<float4*>(d) = f;
        } else {
          const float fv[4] = {f.x, f.y, f.z, f.w};
          for (int j = 0; j < 4 && 4 * q + j < nout; j++) d[j] = fv[j];
        }
      } else {
        uint8_t* d = reinterpret_cast<uint8_t*>(im.dst) + row + o0;
        if (vec_store && 4 * q + 4 <= nout) {
          const uint32_t packed = (uint32_t)res[0] | ((uint32_t)res[1] << 8) | ((uint32_t)res[2] << 16) |
                                  ((uint32_t)res[3] << 24);
          *reinterpret_cast<uint32_t*>(d) = packed;
        } else {
          for (int j = 0; j < 4 && 4 * q + j < nout; j++) d[j] = (uint8_t)res[j];
        }
      }
    }
    __syncthreads();
  }
}

template <int VEC, int C, bool F32>
int launch_t(const LaunchCfg& cfg, const ImgDev* imgs, int vw, int xs, int ys, int x_off, int y_off, hipStream_t s) {
  if constexpr (C == 4) {
    if (cfg.alpha) {
      hipLaunchKernelGGL((resample_tiles<VEC, C, F32, true>), dim3(cfg.ntiles), dim3(kThreads),
                         resample_smem_bytes(cfg), s, imgs, cfg.nimgs, vw, xs, ys, x_off, y_off);
      return hipGetLastError() == hipSuccess ? 0 : -1;
    }
  }
  hipLaunchKernelGGL((resample_tiles<VEC, C, F32, false>), dim3(cfg.ntiles), dim3(kThreads), resample_smem_bytes(cfg),
                     s, imgs, cfg.nimgs, vw, xs, ys, x_off, y_off);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

template <int VEC>
int launch_v(const LaunchCfg& cfg, const ImgDev* i, int vw, int xs, int ys, int xo, int yo, hipStream_t s) {
  switch (cfg.channels * 2 + (cfg.f32 ? 1 : 0)) {
    case 2: return launch_t<VEC, 1, false>(cfg, i, vw, xs, ys, xo, yo, s);
    case 3: return launch_t<VEC, 1, true>(cfg, i, vw, xs, ys, xo, yo, s);
    case 4: return launch_t<VEC, 2, false>(cfg, i, vw, xs, ys, xo, yo, s);
    case 5: return launch_t<VEC, 2, true>(cfg, i, vw, xs, ys, xo, yo, s);
    case 6: return launch_t<VEC, 3, false>(cfg, i, vw, xs, ys, xo, yo, s);
    case 7: return launch_t<VEC, 3, true>(cfg, i, vw, xs, ys, xo, yo, s);
    case 8: return launch_t<VEC, 4, false>(cfg, i, vw, xs, ys, xo, yo, s);
    case 9: return launch_t<VEC, 4, true>(cfg, i, vw, xs, ys, xo, yo, s);
    default: return -2;
  }
}

}  // namespace

int resample_smem_bytes(const LaunchCfg& cfg) {
  const int vw = cfg.max_vw;
  const int xs = kTapHeader + cfg.max_xw;
  const int ys = kTapHeader + cfg.max_yw;
  const int x_off = cfg.max_group * vw;
  const int y_off = x_off + ((cfg.max_tx * xs + 3) & ~3);
  return (y_off + cfg.max_ty * ys) * (int)sizeof(float);
}

int launch_resample(const LaunchCfg& cfg, const ImgDev* imgs, void* stream) {
  const int vw = cfg.max_vw;  // floats per LDS row (multiple of 4)
  const int xs = kTapHeader + cfg.max_xw;
  const int ys = kTapHeader + cfg.max_yw;
  const int x_off = cfg.max_group * vw;
  const int y_off = x_off + ((cfg.max_tx * xs + 3) & ~3);
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  if (cfg.vec == 16) return launch_v<16>(cfg, imgs, vw, xs, ys, x_off, y_off, s);
  if (cfg.vec == 1) return launch_v<1>(cfg, imgs, vw, xs, ys, x_off, y_off, s);
  return -2;
}

}  // namespace mxd
