// devutil.h -- small device helpers shared by the resample kernels
// (wave.hip, band.hip).  Header-only, device code.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>
#include <type_traits>
#include <utility>

#include "resample.h"

namespace mxd {
namespace dev {

#define MXD_GLOBAL_PTR(T, p) ((__attribute__((address_space(1))) T*)(p))
using cgfloat = const __attribute__((address_space(1))) float;
// Constant address space: uniform loads through it are scalar (s_load).
using kfloat = const __attribute__((address_space(4))) float;
using kint = const __attribute__((address_space(4))) int;

// Workgroup ids remapped so that blocks the dispatcher places on one XCD
// (b, b + 8, b + 16, ...) get consecutive ids: neighbouring units (bands of
// one image, whose halo rows overlap) then share that XCD's L2.
__device__ __forceinline__ int xcd_remap(int b, int n) {
#ifdef MXD_NO_XCD_REMAP  // diagnostic builds: consecutive blocks on consecutive XCDs
  return b;
#endif
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

// Window of output columns [ox0, ox1): first and last source pixel their taps
// read (tables: first tap index as int bits, tap count, weights).
__device__ __forceinline__ void strip_span(cgfloat* xtab, int xs, int crop_w, int flip, int ox0, int ox1, int* lo,
                                           int* hi) {
  const int xa = flip ? crop_w - ox1 : ox0;
  const int xb = flip ? crop_w - 1 - ox0 : ox1 - 1;
  *lo = __float_as_int(xtab[xa * xs]);
  *hi = __float_as_int(xtab[xb * xs]) + __float_as_int(xtab[xb * xs + 1]) - 1;
}

// Bytes of the stored source region a buffer descriptor may cover: from the
// 4-byte aligned base (`shift` bytes below the first stored byte) to the end
// of the last stored row's pixels (never past the stored allocation: a staged
// footprint's row, or the caller's image row, ends within one stride),
// rounded up to a whole dword -- the range check drops a dword that is only
// partly inside, and an end that is not page aligned has its page's bytes up
// to the next 4-byte boundary mapped.
__device__ __forceinline__ int src_records(int shift, int rows, int stride, int row_bytes) {
  return (shift + (rows - 1) * stride + (row_bytes < stride ? row_bytes : stride) + 3) & ~3;
}

}  // namespace dev
}  // namespace mxd
