// pixmap.h -- device descriptors and launchers of the pixel-map kernels
// (rotate / affine, channel reduction).  SURVEY.md §8f row f4.
#pragma once
#include <cstddef>
#include <cstdint>

namespace mxd {

// One image of a pixel-map launch, as the kernels read it.  Built by capi.cpp
// from mxd_pixmap; the affine constants and the 16.16 channel weights are
// derived on the host exactly as the reference derives them.
struct PixDev {
  const uint8_t* src;
  uint8_t* dst;
  int64_t src_stride, dst_stride;
  int32_t src_w, src_h, dst_w, dst_h, c;
  int32_t groups;  // groups of 4 output pixels per output row
  int32_t fast;    // 4-byte aligned rows: dword loads/stores for full groups
  int32_t pad;
  float mx[6];     // affine matrix (core::image::affine)
  float twh, thh, wh, hh;
  int32_t m[3], bias;  // channel reduction, 16.16 fixed point
};

// op: 0 affine, 1 channel reduction.  c: 1..4 (affine), 3 (reduction).
// max_units = max over images of dst_h * dst_w (affine) or dst_h * groups.
int launch_pixmap(int op, const PixDev* imgs, int n, int64_t max_units, void* stream);

}  // namespace mxd
