// taps.cpp -- see taps.h.
//
// The reference's resize arithmetic is stb_image_resize2 (FetchContent pin
// nothings/stb@f0569113, CMakeLists.txt:19-26), called with the triangle
// filter, clamp edges and packed uint8 (core/image/ImageTransform.cpp:49-60).
// The filter construction it performs, restated:
//   scale = (float)(out/in), inv = (float)(1/(out/in)) computed in double;
//   out == in        -> point sampling (identity);
//   upsample  (s>=1) -> per output n, centre c=(n+.5)*inv, taps over the input
//                       pixels whose centres lie within 1 of c, w = tri(c - (i+.5));
//   downsample (s<1) -> per input i (swept from -margin), w = s*tri((n+.5) - (i+.5)*s)
//                       for the outputs n it reaches (support 1/s input pixels);
//   each output's weights are rescaled to sum to 1; when out/in reduces to
//   num/den with num < out the first `num` outputs are built and repeated
//   with the input shifted by `den` (polyphase); out-of-range taps are folded
//   onto pixel 0 / in-1 (clamp) and zero taps trimmed.
#include "taps.h"

#include <algorithm>
#include <cmath>
#include <cstring>
#include <numeric>

namespace mxd {
namespace {

constexpr float kTiny = (float)1 / (1 << 20) / (1 << 20) / (1 << 20) / (1 << 20) / (1 << 20) / (1 << 20);

inline float tent(float x) {
  x = x < 0.0f ? -x : x;
  return x <= 1.0f ? 1.0f - x : 0.0f;
}

// A contiguous run of taps [n0, n1] with weights w[0..n1-n0].
struct Run {
  int32_t n0 = 0, n1 = -1;
  std::vector<float> w;
  float& at(int32_t px) { return w[px - n0]; }
  // Add weight v to pixel px, growing the run as needed.
  void add(int32_t px, float v) {
    if (px >= n0 && px <= n1) {
      at(px) += v;
    } else if (px > n1) {
      w.resize(px - n0 + 1, 0.0f);
      w[px - n0] = v;
      n1 = px;
    } else {
      w.insert(w.begin(), n0 - px, 0.0f);
      w[0] = v;
      n0 = px;
    }
  }
};

void normalise(Run& r) {
  float total = 0.0f;
  for (float v : r.w) total += v;
  if (total < kTiny && total > -kTiny) {
    r.n1 = r.n0;
    r.w.assign(1, 0.0f);
  } else if (total < 1.0f - kTiny || total > 1.0f + kTiny) {
    const float f = 1.0f / total;
    for (float& v : r.w) v *= f;
  }
}

// Folds taps outside [0, in-1] onto the edge pixels the way stbir's clamp
// edge inserts them (left: pixel -1 down to n0, right: in .. n1).
void clamp_edges(Run& r, int32_t in) {
  if (r.n0 < 0) {
    Run f;
    f.n0 = 0;
    f.n1 = r.n1;
    f.w.assign(r.n1 + 1, 0.0f);
    for (int32_t px = 0; px <= r.n1; px++) f.w[px] = r.at(px);
    // stbir accumulates -1, -2, ..., n0+1 into pixel 0 first, then n0.
    for (int32_t px = -1; px >= r.n0; px--) f.w[0] += r.at(px);
    r = std::move(f);
  }
  if (r.n1 > in - 1) {
    const int32_t old_n1 = r.n1;
    std::vector<float> tail(r.w.begin() + (in - r.n0), r.w.end());
    r.w.resize(in - r.n0);
    r.n1 = in - 1;
    for (int32_t px = in; px <= old_n1; px++) r.at(in - 1) += tail[px - in];
  }
  while (r.n1 > r.n0 && r.w.front() == 0.0f) {
    r.w.erase(r.w.begin());
    r.n0++;
  }
  while (r.n1 > r.n0 && r.w.back() == 0.0f) {
    r.w.pop_back();
    r.n1--;
  }
}

std::vector<Run> upsample_runs(int32_t in, int32_t nbuild, float scale, float inv) {
  std::vector<Run> runs(nbuild);
  for (int32_t n = 0; n < nbuild; n++) {
    const float centre = (float)n + 0.5f;
    const float src_centre = centre * inv;
    int32_t first = (int32_t)std::floor((centre - scale) * inv + 0.5f);
    int32_t last = (int32_t)std::floor((centre + scale) * inv - 0.5f);
    if (last < first) last = first;
    Run& r = runs[n];
    int32_t last_nz = -1;
    std::vector<float> w;
    for (int32_t px = first; px <= last; px++) {
      float v = tent(src_centre - ((float)px + 0.5f));
      if (v < kTiny && v > -kTiny) {
        if (w.empty()) {  // leading zero taps are dropped
          first = px + 1;
          continue;
        }
        v = 0.0f;
      } else {
        last_nz = px;
      }
      w.push_back(v);
    }
    r.n0 = first;
    r.n1 = last_nz;
    w.resize(std::max<int32_t>(last_nz - first + 1, 0));
    r.w = std::move(w);
  }
  (void)in;
  return runs;
}

std::vector<Run> downsample_runs(int32_t in, int32_t out, int32_t nbuild, float scale, float inv) {
  std::vector<Run> runs(nbuild);
  std::vector<char> seen(nbuild, 0);
  const int32_t margin = ((int32_t)std::ceil(2.0f / scale)) / 2;
  for (int32_t px = -margin; px < in + margin; px++) {
    const float pc = (float)px + 0.5f;
    const float dst_centre = pc * scale;
    int32_t o0 = (int32_t)std::floor((pc - inv) * scale + 0.5f);
    int32_t o1 = (int32_t)std::floor((pc + inv) * scale - 0.5f);
    o0 = std::max(o0, 0);
    o1 = std::min(o1, out - 1);
    if (o0 > o1) continue;
    if (nbuild < out) {
      if (o0 == nbuild) break;
      o1 = std::min(o1, nbuild - 1);
    }
    for (int32_t o = o0; o <= o1; o++) {
      float v = tent(((float)o + 0.5f) - dst_centre) * scale;
      if (v < kTiny && v > -kTiny) v = 0.0f;
      Run& r = runs[o];
      if (!seen[o]) {
        seen[o] = 1;
        r.n0 = r.n1 = px;
        r.w.assign(1, v);
      } else {
        if (r.w.front() == 0.0f && r.w.size() == 1) {  // zero first tap is replaced
          r.n0 = px;
          r.w.clear();
        }
        r.n1 = px;
        r.w.resize(px - r.n0 + 1, 0.0f);
        r.w[px - r.n0] = v;
      }
    }
  }
  return runs;
}

}  // namespace

int32_t AxisTaps::lo() const {
  int32_t v = first.empty() ? 0 : first[0];
  for (size_t i = 0; i < first.size(); i++) v = std::min(v, first[i]);
  return v;
}

int32_t AxisTaps::hi() const {
  int32_t v = first.empty() ? 0 : first[0];
  for (size_t i = 0; i < first.size(); i++) v = std::max(v, first[i] + count[i] - 1);
  return v;
}

bool build_axis_taps(int32_t in, int32_t out, int32_t off, int32_t len, AxisTaps* t) {
  if (in <= 0 || out <= 0 || len <= 0 || off < 0 || off + len > out) return false;
  t->in_size = in;
  t->out_size = out;
  t->off = off;
  t->len = len;
  std::vector<Run> all;
  if (in == out) {
    all.resize(out);
    for (int32_t n = 0; n < out; n++) {
      all[n].n0 = all[n].n1 = n;
      all[n].w.assign(1, 1.0f);
    }
  } else {
    const double s = (double)out / (double)in;
    const float scale = (float)s, inv = (float)(1.0 / s);
    const int32_t g = std::gcd(out, in);
    const int32_t num = out / g, den = in / g;
    const int32_t nbuild = num < out ? num : out;
    all = scale >= 1.0f ? upsample_runs(in, nbuild, scale, inv) : downsample_runs(in, out, nbuild, scale, inv);
    for (auto& r : all) normalise(r);
    all.resize(out);
    for (int32_t n = nbuild; n < out; n++) {
      all[n] = all[n - nbuild];
      all[n].n0 += den;
      all[n].n1 += den;
    }
    for (auto& r : all) clamp_edges(r, in);
  }
  int32_t width = 1;
  for (int32_t i = 0; i < len; i++) width = std::max<int32_t>(width, all[off + i].n1 - all[off + i].n0 + 1);
  t->width = width;
  t->first.assign(len, 0);
  t->count.assign(len, 0);
  t->weight.assign((size_t)len * width, 0.0f);
  for (int32_t i = 0; i < len; i++) {
    const Run& r = all[off + i];
    t->first[i] = r.n0;
    t->count[i] = r.n1 - r.n0 + 1;
    std::memcpy(&t->weight[(size_t)i * width], r.w.data(), sizeof(float) * r.w.size());
  }
  return true;
}

void smallest_side_dims(int64_t w, int64_t h, int64_t size, int64_t* tw, int64_t* th) {
  const double scale = h > w ? (double)size / (double)w : (double)size / (double)h;
  *tw = std::lround(scale * (double)w);
  *th = std::lround(scale * (double)h);
}

}  // namespace mxd
