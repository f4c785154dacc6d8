// jpegycc.h -- jdcolor.c's YCbCr -> RGB in 16-bit fixed point (the host
// decoder's jpeg.cpp ycc_rgb), shared by jpegdev.hip's jpeg_color and the
// wave kernels that read JPEG sample planes directly (wave.hip YccSrc).
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

namespace mxd {

constexpr int kFixCrR = 91881, kFixCbB = 116130, kFixCrG = 46802, kFixCbG = 22554, kHalf16 = 1 << 15;

__device__ __forceinline__ uint32_t jpeg_clamp255(int v) { return (uint32_t)(v < 0 ? 0 : v > 255 ? 255 : v); }

__device__ __forceinline__ void jpeg_ycc_to_rgb(int y, int cb, int cr, uint32_t* px) {
  cb -= 128;
  cr -= 128;
  px[0] = jpeg_clamp255(y + ((kFixCrR * cr + kHalf16) >> 16));
  px[1] = jpeg_clamp255(y + ((-kFixCbG * cb + kHalf16 - kFixCrG * cr) >> 16));
  px[2] = jpeg_clamp255(y + ((kFixCbB * cb + kHalf16) >> 16));
}

}  // namespace mxd
