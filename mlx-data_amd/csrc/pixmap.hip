// pixmap.hip -- pixel-map kernels for gfx950: nearest-pixel affine (rotate)
// and RGB -> gray channel reduction.  SURVEY.md §8f row f4.
//
//   affine             mlx/data/core/image/ImageTransform.cpp:75-110
//   channel_reduction  mlx/data/core/image/ImageTransform.cpp:142-180
//
// Both are byte-level HBM-bound maps (no MFMA work).  blockIdx.y selects the
// image.  Affine: a thread owns 4 consecutive output pixels (one 4*C-byte
// store), a workgroup a 64 x 16 output tile (compact rotated source
// footprint).  Reduction: a thread owns 16 pixels (3 x 16-B loads, 1 x 16-B
// store), lanes in row order.
//
// The affine inverse map repeats the reference's arithmetic step for step:
// float products and sums (no contraction), then `+ 0.5 + wh` in double and a
// truncating int64 conversion, so every output byte matches the CPU code.
#include <hip/hip_runtime.h>

#include "pixmap.h"

namespace mxd {
namespace {

constexpr int kThreads = 256;

__device__ __forceinline__ void put_byte(uint32_t* w, int b, uint32_t v) { w[b >> 2] |= v << (8 * (b & 3)); }

// Affine: a workgroup owns an output tile of 16 rows x 64 px; wave w covers
// rows 4w..4w+3 of it (16 lanes per row, 4 px per lane, one 4*C-byte store).
// Measured on 64 1080p frames at 30 degrees (profiles/r01/pixmap_*): this
// shape (1.23 ms) beat 8 x 32 and 16 x 16 px per wave (1.46 / 1.86 ms), 1 x 256
// px per wave with XCD-contiguous tile ranges (1.91 ms) and an LDS-assembled
// 16 x 128 tile with 16-byte row stores (2.30 ms), although the last two cut
// HBM traffic: the gather is bound by its load/store instruction stream, not
// by bytes.
constexpr int kAffThreads = 256, kTileRows = 16, kTileGroups = 16;

template <int C>
__device__ void affine_tiles(const PixDev& d) {
#pragma clang fp contract(off)
  const int32_t tiles_x = (d.groups + kTileGroups - 1) / kTileGroups;
  const int32_t ntiles = tiles_x * ((d.dst_h + kTileRows - 1) / kTileRows);
  const int32_t r = threadIdx.x / kTileGroups, gq = threadIdx.x % kTileGroups;
  // Gathers: every pixel of the thread's group is read with one unconditional
  // 12-byte load from a 4-byte aligned word at or before it, clamped to end at
  // the aligned word holding the source's last byte (a dword never straddles
  // a page, so that word is always readable); out-of-range pixels read the
  // first word and are masked.  A thread's four loads are thus in flight
  // together.  Sources under 12 bytes take byte loads.
  const uint8_t* base = reinterpret_cast<const uint8_t*>(reinterpret_cast<uintptr_t>(d.src) & ~(uintptr_t)3);
  const int64_t skew = d.src - base;
  const int64_t total = skew + (int64_t)(d.src_h - 1) * d.src_stride + (int64_t)d.src_w * C;
  const int64_t end4 = (total + 3) & ~(int64_t)3;
  const bool tiny = end4 < 12;
  const int64_t last = end4 - 12;
  for (int32_t t = blockIdx.x; t < ntiles; t += gridDim.x) {
    const int32_t tyb = t / tiles_x;
    const int32_t ty = tyb * kTileRows + r;
    const int32_t g = (t - tyb * tiles_x) * kTileGroups + gq;
    if (ty >= d.dst_h || g >= d.groups) continue;
    const int32_t tx0 = g * 4;
    const float fy = (float)ty - d.thh;
    const float by = d.mx[1] * fy;
    const float ey = d.mx[4] * fy;
    uint32_t w[C] = {};
    const int cnt = min(4, d.dst_w - tx0);
    int64_t off[4];
    bool ok[4];
#pragma unroll
    for (int k = 0; k < 4; k++) {
      const float fx = (float)(tx0 + k) - d.twh;
      const float sx = d.mx[0] * fx + by + d.mx[2];
      const float sy = d.mx[3] * fx + ey + d.mx[5];
      // (int64_t) of the double sum, as v_cvt_i32_f64 (truncating; it
      // saturates only far outside any image, where both are rejected)
      const int32_t x = __double2int_rz((double)sx + 0.5 + (double)d.wh);
      const int32_t y = __double2int_rz((double)sy + 0.5 + (double)d.hh);
      ok[k] = k < cnt && x >= 0 && y >= 0 && x < d.src_w && y < d.src_h;
      off[k] = ok[k] ? skew + (int64_t)y * d.src_stride + (int64_t)x * C : skew;
    }
    if (!tiny) {
      uint32_t q[4][3];
#pragma unroll
      for (int k = 0; k < 4; k++) {
        const int64_t a = min(off[k] & ~(int64_t)3, last);
        const uint32_t* p = reinterpret_cast<const uint32_t*>(base + a);
        q[k][0] = p[0];
        q[k][1] = p[1];
        q[k][2] = p[2];
        off[k] -= a;  // byte position of the pixel in the 12 loaded bytes
      }
#pragma unroll
      for (int k = 0; k < 4; k++) {
        if (ok[k]) {
          const int32_t sh = (int32_t)off[k];
#pragma unroll
          for (int ch = 0; ch < C; ch++) {
            const int32_t bpos = sh + ch;
            const uint32_t dw = bpos < 4 ? q[k][0] : (bpos < 8 ? q[k][1] : q[k][2]);
            put_byte(w, k * C + ch, (dw >> (8 * (bpos & 3))) & 255);
          }
        }
      }
    } else {
#pragma unroll
      for (int k = 0; k < 4; k++)
        if (ok[k])
#pragma unroll
          for (int ch = 0; ch < C; ch++) put_byte(w, k * C + ch, base[off[k] + ch]);
    }
    uint8_t* out = d.dst + (int64_t)ty * d.dst_stride + (int64_t)tx0 * C;
    if (d.fast && cnt == 4) {
#pragma unroll
      for (int j = 0; j < C; j++) reinterpret_cast<uint32_t*>(out)[j] = w[j];
    } else {
      for (int b = 0; b < cnt * C; b++) out[b] = (uint8_t)(w[b >> 2] >> (8 * (b & 3)));
    }
  }
}

__device__ __forceinline__ uint32_t gray(const PixDev& d, uint32_t r, uint32_t g, uint32_t b) {
  int v = ((int)r * d.m[0] + (int)g * d.m[1] + (int)b * d.m[2] + d.bias) / (256 * 256);
  v = v <= 255 ? v : 255;
  v = v >= 0 ? v : 0;
  return (uint32_t)v;
}

// Channel reduction: a thread owns 16 consecutive pixels of a row -- three
// 16-byte loads (48 source bytes) and one 16-byte store when rows are 16-byte
// aligned; lanes of a wave cover 1024 consecutive pixels.
constexpr int kGrayGroup = 16;

__device__ void reduce_rows(const PixDev& d) {
  const int32_t units = d.dst_h * d.groups;
  const int32_t step = gridDim.x * kThreads;
  for (int32_t u = blockIdx.x * kThreads + threadIdx.x; u < units; u += step) {
    const int32_t ty = u / d.groups;
    const int32_t tx0 = (u - ty * d.groups) * kGrayGroup;
    const int cnt = min(kGrayGroup, d.dst_w - tx0);
    const uint8_t* in = d.src + (int64_t)ty * d.src_stride + (int64_t)tx0 * 3;
    uint8_t* out = d.dst + (int64_t)ty * d.dst_stride + tx0;
    if (d.fast && cnt == kGrayGroup) {
      const uint4* q = reinterpret_cast<const uint4*>(in);
      const uint4 a = q[0], b = q[1], c = q[2];
      const uint32_t wv[12] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w, c.x, c.y, c.z, c.w};
      uint32_t o[4] = {0, 0, 0, 0};
#pragma unroll
      for (int k = 0; k < kGrayGroup; k++) {
        const uint32_t rr = (wv[(3 * k) >> 2] >> (8 * ((3 * k) & 3))) & 255;
        const uint32_t gg = (wv[(3 * k + 1) >> 2] >> (8 * ((3 * k + 1) & 3))) & 255;
        const uint32_t bb = (wv[(3 * k + 2) >> 2] >> (8 * ((3 * k + 2) & 3))) & 255;
        o[k >> 2] |= gray(d, rr, gg, bb) << (8 * (k & 3));
      }
      *reinterpret_cast<uint4*>(out) = make_uint4(o[0], o[1], o[2], o[3]);
    } else {
      for (int k = 0; k < cnt; k++) out[k] = (uint8_t)gray(d, in[3 * k], in[3 * k + 1], in[3 * k + 2]);
    }
  }
}

__global__ __launch_bounds__(kThreads) void reduce_kernel(const PixDev* __restrict__ imgs) {
  reduce_rows(imgs[blockIdx.y]);
}

__global__ __launch_bounds__(kAffThreads) void affine_kernel(const PixDev* __restrict__ imgs) {
  const PixDev d = imgs[blockIdx.y];
  switch (d.c) {
    case 1: affine_tiles<1>(d); break;
    case 2: affine_tiles<2>(d); break;
    case 3: affine_tiles<3>(d); break;
    default: affine_tiles<4>(d); break;
  }
}

}  // namespace

int launch_pixmap(int op, const PixDev* imgs, int n, int64_t max_units, void* stream) {
  if (n <= 0 || max_units <= 0) return 0;
  // max_units: per image, output pixels (affine) or 16-px groups (reduction).
  // Enough blocks per image to fill the chip when the batch is small; each
  // block strides over its image's rows (reduction) or tiles (affine).
  const int threads = op == 1 ? kThreads : kAffThreads;
  const int64_t per_unit = op == 1 ? 1 : 4;  // affine: a thread covers 4 px
  int64_t per_img = (max_units + (int64_t)threads * per_unit - 1) / ((int64_t)threads * per_unit);
  const int64_t want = (32 * 256 * 256 / threads + n - 1) / n;  // ~32 x 256-thread blocks per CU
  if (per_img > want) per_img = want;
  dim3 grid((unsigned)per_img, (unsigned)n);
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  if (op == 1)
    hipLaunchKernelGGL(reduce_kernel, grid, dim3(kThreads), 0, s, imgs);
  else
    hipLaunchKernelGGL(affine_kernel, grid, dim3(kAffThreads), 0, s, imgs);
  return hipGetLastError() == hipSuccess ? 0 : 1;
}

}  // namespace mxd
