// oracle/ref_harness.cpp -- TEST INFRASTRUCTURE ONLY.
//
// A thin extern "C" driver around the parts of the reference that DO compile
// in this image, built from the reference's own sources where they lie
// (/root/reference/mlx/data/{Array,Sample}.cpp, core/{BatchShape,State}.cpp)
// by oracle/Makefile into oracle/_ref/libmlxref.so.  It pins, with the
// reference's own code:
//   - crop bytes:  array::sub            (Array.cpp:544-583), as called by
//                  core::image::crop     (core/image/ImageTransform.cpp:64-73)
//   - batching:    array::batch          (Array.cpp:465-498), pad + NHWC copy
//   - RNG streams: core::set_state / get_state (core/State.cpp:9-22) driving the
//                  draws of ImageRandomCrop::generate_random_crop_
//                  (op/ImageTransform.cpp:135-150) and ImageRandomHFlip
//                  (:323-332), in the per-sample order a pipeline applies them.
// core/image/ImageTransform.cpp itself (resize/hflip) needs stb_image_resize2.h,
// which this image lacks, so it is not built.
#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <random>
#include <stdexcept>
#include <vector>

#include "mlx/data/Array.h"
#include "mlx/data/core/State.h"

using mlx::data::Array;
using mlx::data::ArrayType;

namespace {
std::shared_ptr<Array> wrap_u8(const uint8_t* p, int64_t h, int64_t w, int64_t c) {
  std::shared_ptr<void> data(const_cast<uint8_t*>(p), [](void*) {});
  return std::make_shared<Array>(ArrayType::UInt8, std::vector<int64_t>{h, w, c}, data);
}
}  // namespace

extern "C" {

// core::image::crop(img, x, y, cw, ch) == array::sub(img, {y, x, 0}, {ch, cw, -1})
int ref_crop_u8(const uint8_t* src, int w, int h, int c, int x, int y, int cw, int ch, uint8_t* dst) {
  try {
    auto res = mlx::data::array::sub(wrap_u8(src, h, w, c), {y, x, 0}, {ch, cw, -1});
    std::memcpy(dst, res->data(), (size_t)res->size());
    return 0;
  } catch (const std::exception&) {
    return -1;
  }
}

// array::batch of n u8 images (shapes[i] = {h, w, c}); dst receives the padded
// NHWC batch of shape {n, max h, max w, max c}; returns its byte size or -1.
int64_t ref_batch_u8(const uint8_t* const* srcs, const int64_t* shapes, int n, double pad, uint8_t* dst,
                     int64_t dst_cap) {
  try {
    std::vector<std::shared_ptr<Array>> arrs;
    for (int i = 0; i < n; i++) arrs.push_back(wrap_u8(srcs[i], shapes[3 * i], shapes[3 * i + 1], shapes[3 * i + 2]));
    auto res = mlx::data::array::batch(arrs, pad);
    if (res->size() > dst_cap) return -1;
    std::memcpy(dst, res->data(), (size_t)res->size());
    return res->size();
  } catch (const std::exception&) {
    return -1;
  }
}

// Per sample, the draws a stream .image_random_crop(cw, ch).image_random_h_flip(p)
// makes on one thread after mlx.data.core.set_state(seed): x, y, then u <= p.
void ref_random_crop_flip_params(int64_t seed, int n, const int64_t* wh, int64_t cw, int64_t ch, float prob,
                                 int64_t* out_xy, int32_t* out_flip) {
  mlx::data::core::set_state(seed);
  for (int i = 0; i < n; i++) {
    auto state = mlx::data::core::get_state();
    std::uniform_int_distribution<int64_t> xu{0, wh[2 * i] - cw};
    std::uniform_int_distribution<int64_t> yu{0, wh[2 * i + 1] - ch};
    out_xy[2 * i] = xu(state->randomGenerator);
    out_xy[2 * i + 1] = yu(state->randomGenerator);
    std::uniform_real_distribution<float> u{0, 1.0};
    out_flip[i] = u(state->randomGenerator) <= prob ? 1 : 0;
  }
}

// Per sample, the draws of ImageRandomAreaCrop::generate_random_crop_
// (op/ImageTransform.cpp:214-280) after set_state(seed), restated on the
// reference's own State: out[4i..4i+3] = (x, y, w, h), zeros when none.
void ref_random_area_crop_params(int64_t seed, int n, const int64_t* wh, float a0, float a1, float r0, float r1,
                                 int trials, int64_t* out) {
  mlx::data::core::set_state(seed);
  for (int i = 0; i < n; i++) {
    const int64_t w = wh[2 * i], h = wh[2 * i + 1];
    int64_t* o = out + 4 * i;
    o[0] = o[1] = o[2] = o[3] = 0;
    if (w == 0 || h == 0) continue;
    const float wf = (float)w, hf = (float)h, r = wf / hf;
    auto state = mlx::data::core::get_state();
    int64_t wmin = std::ceil(std::sqrt(a0 * r0) * wf);
    int64_t wmax = std::floor(std::min(std::sqrt(a1 * r1) * wf, wf));
    if (wmin > wmax) continue;
    std::uniform_int_distribution<int64_t> wu{wmin, wmax};
    int64_t tw = 0, th = 0;
    for (int t = 0; t < trials; t++) {
      tw = wu(state->randomGenerator);
      int64_t hmin = std::ceil(std::max(1.0f / (r * r1) * tw, a0 * wf * hf / tw));
      int64_t hmax = std::floor(std::min(std::min(1.0f / (r * r0) * tw, a1 * wf * hf / tw), hf));
      if (hmin > hmax) continue;
      std::uniform_int_distribution<int64_t> hu{hmin, hmax};
      th = hu(state->randomGenerator);
      float tr = (float)tw / (float)th;
      if (a0 * w * h > tw * th || a1 * w * h < tw * th) continue;
      if (r0 * r > tr || r1 * r < tr) continue;
      if (tw <= 0 || tw > w || th <= 0 || th > h) continue;
      break;
    }
    if (tw == 0 || th == 0) continue;
    std::uniform_int_distribution<int64_t> xu{0, w - tw};
    std::uniform_int_distribution<int64_t> yu{0, h - th};
    o[0] = xu(state->randomGenerator);
    o[1] = yu(state->randomGenerator);
    o[2] = tw;
    o[3] = th;
  }
}

}  // extern "C"
