// band_plan.h -- host planning of the band kernel (band.h): kernel class,
// strips, LDS-DMA window, lookahead and the per-band scatter schedule.
// Host only; no device calls (tested on CPU through mxd_describe_plan).
#pragma once

#include <cstdint>
#include <vector>

#include "band.h"

namespace mxd {

// One axis' taps over the WHOLE resized axis (index = resized coordinate).
struct AxisView {
  const int32_t* first;
  const int32_t* count;
  const float* w;  // [out][width]
  int32_t width;
  int32_t padded;  // weights per entry of the device table (>= the class taps it may serve)
};

// What the planner needs to know about one image (stored region as the
// kernel will address it: x0 / y0 = source pixel / row at the stored base,
// shift = the base's misalignment below a 4-byte boundary).
struct BandImage {
  int32_t channels, f32;
  int32_t crop_x, crop_y, crop_w, crop_h, flip;
  int32_t src_w, x0, shift;
  int64_t stride;        // bytes between stored rows
  int64_t dst_stride;    // bytes between output rows
  uintptr_t dst;         // output base address (alignment only)
};

struct BandPlan {
  bool ok = false;
  int32_t cls = -1;      // index into kBandClasses
  int32_t taps = 0, db = 0, s = 0;
  int32_t nq = 0;        // KiB of source window per strip row
  int32_t nstrips = 0, tx = 0;
  int32_t prologue = 0;  // groups before the one completing a band's first output row (at crop row 0)
  int32_t dmax = 0;      // most source rows new for one output row
  int32_t la = 0;        // groups loaded ahead
  double rows_per_out = 0;  // mean source rows per output row
};

// Scatter shape of crop rows [off, off+len): dmax, and whether the taps are
// monotone (first and last tap nondecreasing).
bool band_vertical_shape(const AxisView& yt, int32_t off, int32_t len, int32_t* dmax);

// Plans one image; plan.ok = false when the band kernel cannot take it (the
// caller falls back to wave.hip / resample.hip).  la_override > 0 forces the
// lookahead (tuning).
BandPlan band_plan_image(const AxisView& xt, const AxisView& yt, const BandImage& im, int32_t la_override = 0);

// Accumulator slots (open output rows a source row's weights reach) the
// schedule of crop rows [off, off+len) needs, bands starting at any row
// (cached per table window).
int32_t band_slots(const AxisView& yt, int32_t off, int32_t len);

// Schedule words for crop rows [crop_y, crop_y + crop_h) in bands of ty rows:
// per band `band_words` words = header [groups, 0, 0, 0], then the groups,
// each a header [flags, 0, 0, 0] (kBandRowDone: completes the oldest open
// output row) and db entries {source row or -1, s weights, zero padded to 4
// words}.  The rows new for an output row fill ceil(new / db) groups (at
// least one), the last completing it; a band has at least min_groups groups
// (empty ones appended).  Returns false if some source row's weights do not
// fit the s slots.
bool band_schedule(const AxisView& yt, int32_t crop_y, int32_t crop_h, int32_t ty, int32_t db, int32_t s,
                   int32_t min_groups, std::vector<int32_t>* words, int32_t* band_words);

}  // namespace mxd
