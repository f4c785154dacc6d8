// taps.h -- resampling taps of one image axis, stb_image_resize2 semantics.
//
// mlx-data resizes with stbir_resize_uint8_linear and forces the triangle
// filter for both directions (mlx/data/core/image/ImageTransform.cpp:7-10,
// 49-60).  This builds, on the host, the per-output (first input, tap count,
// f32 weights) tables the HIP kernels consume, restricted to the output window
// the crop keeps.  Tables are computed once per (in, out, window) geometry and
// cached on the device by capi.cpp.
#pragma once

#include <cstdint>
#include <vector>

namespace mxd {

struct AxisTaps {
  int32_t in_size = 0, out_size = 0;
  int32_t off = 0, len = 0;     // output window [off, off+len)
  int32_t width = 0;            // max taps over the window
  std::vector<int32_t> first;   // [len] first input index of each output
  std::vector<int32_t> count;   // [len] taps of each output (>= 1)
  std::vector<float> weight;    // [len][width], zero padded
  int32_t lo() const;           // smallest input index touched by the window
  int32_t hi() const;           // largest input index touched by the window
};

// Builds taps for outputs [off, off+len) of an in_size -> out_size resize.
// Returns false if the arguments are invalid.
bool build_axis_taps(int32_t in_size, int32_t out_size, int32_t off, int32_t len, AxisTaps* out);

// core::image::scale dims: lround(scale * w), lround(scale * h) in double.
void smallest_side_dims(int64_t w, int64_t h, int64_t size, int64_t* tw, int64_t* th);

}  // namespace mxd
