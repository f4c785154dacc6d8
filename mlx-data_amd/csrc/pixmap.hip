// pixmap.hip -- pixel-map kernels for gfx950: nearest-pixel affine (rotate)
// and RGB -> gray channel reduction.  SURVEY.md §8f row f4.
//
//   affine             mlx/data/core/image/ImageTransform.cpp:75-110
//   channel_reduction  mlx/data/core/image/ImageTransform.cpp:142-180
//
// Both are byte-level HBM-bound maps (no MFMA work).  One thread owns a group
// of 4 consecutive output pixels of a row, so a full group is one 4*C-byte
// (affine) or one 4-byte (reduction) store, and the reduction reads its 12
// source bytes as 3 dwords when rows are 4-byte aligned.  blockIdx.y selects
// the image; blocks stride over the image's groups.
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

template <int C>
__device__ void affine_rows(const PixDev& d, int64_t units) {
#pragma clang fp contract(off)
  const int64_t step = (int64_t)gridDim.x * kThreads;
  for (int64_t u = (int64_t)blockIdx.x * kThreads + threadIdx.x; u < units; u += step) {
    const int32_t ty = (int32_t)(u / d.groups);
    const int32_t tx0 = (int32_t)(u - (int64_t)ty * d.groups) * 4;
    const float fy = (float)ty - d.thh;
    const float by = d.mx[1] * fy;
    const float ey = d.mx[4] * fy;
    uint32_t w[C] = {};
    const int cnt = min(4, d.dst_w - tx0);
#pragma unroll
    for (int k = 0; k < 4; k++) {
      if (k < cnt) {
        const float fx = (float)(tx0 + k) - d.twh;
        const float sx = d.mx[0] * fx + by + d.mx[2];
        const float sy = d.mx[3] * fx + ey + d.mx[5];
        const int64_t x = (int64_t)((double)sx + 0.5 + (double)d.wh);
        const int64_t y = (int64_t)((double)sy + 0.5 + (double)d.hh);
        if (x >= 0 && y >= 0 && x < d.src_w && y < d.src_h) {
          const uint8_t* p = d.src + y * d.src_stride + x * C;
#pragma unroll
          for (int ch = 0; ch < C; ch++) put_byte(w, k * C + ch, p[ch]);
        }
      }
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

__device__ void reduce_rows(const PixDev& d, int64_t units) {
  const int64_t step = (int64_t)gridDim.x * kThreads;
  for (int64_t u = (int64_t)blockIdx.x * kThreads + threadIdx.x; u < units; u += step) {
    const int32_t ty = (int32_t)(u / d.groups);
    const int32_t tx0 = (int32_t)(u - (int64_t)ty * d.groups) * 4;
    const int cnt = min(4, d.dst_w - tx0);
    const uint8_t* in = d.src + (int64_t)ty * d.src_stride + (int64_t)tx0 * 3;
    uint8_t* out = d.dst + (int64_t)ty * d.dst_stride + tx0;
    if (d.fast && cnt == 4) {
      const uint32_t* q = reinterpret_cast<const uint32_t*>(in);
      const uint32_t a = q[0], b = q[1], c = q[2];
      // bytes: a = r0 g0 b0 r1, b = g1 b1 r2 g2, c = b2 r3 g3 b3
      const uint32_t v0 = gray(d, a & 255, (a >> 8) & 255, (a >> 16) & 255);
      const uint32_t v1 = gray(d, a >> 24, b & 255, (b >> 8) & 255);
      const uint32_t v2 = gray(d, (b >> 16) & 255, b >> 24, c & 255);
      const uint32_t v3 = gray(d, (c >> 8) & 255, (c >> 16) & 255, c >> 24);
      *reinterpret_cast<uint32_t*>(out) = v0 | (v1 << 8) | (v2 << 16) | (v3 << 24);
    } else {
      for (int k = 0; k < cnt; k++) out[k] = (uint8_t)gray(d, in[3 * k], in[3 * k + 1], in[3 * k + 2]);
    }
  }
}

__global__ __launch_bounds__(kThreads) void pixmap_kernel(int op, const PixDev* __restrict__ imgs) {
  const PixDev d = imgs[blockIdx.y];
  const int64_t units = (int64_t)d.dst_h * d.groups;
  if (op == 1) {
    reduce_rows(d, units);
    return;
  }
  switch (d.c) {
    case 1: affine_rows<1>(d, units); break;
    case 2: affine_rows<2>(d, units); break;
    case 3: affine_rows<3>(d, units); break;
    default: affine_rows<4>(d, units); break;
  }
}

}  // namespace

int launch_pixmap(int op, const PixDev* imgs, int n, int64_t max_units, void* stream) {
  if (n <= 0 || max_units <= 0) return 0;
  // Enough blocks per image to fill the chip when the batch is small; each
  // block strides over its image's groups.
  int64_t per_img = (max_units + kThreads - 1) / kThreads;
  const int64_t want = (4 * 256 + n - 1) / n;  // ~4 blocks per CU over the batch
  if (per_img > want) per_img = want;
  dim3 grid((unsigned)(per_img < 1 ? 1 : per_img), (unsigned)n);
  hipLaunchKernelGGL(pixmap_kernel, grid, dim3(kThreads), 0, reinterpret_cast<hipStream_t>(stream), op, imgs);
  return hipGetLastError() == hipSuccess ? 0 : 1;
}

}  // namespace mxd
