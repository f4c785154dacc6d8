// band_plan.cpp -- see band_plan.h.
#include "band_plan.h"

#include <algorithm>
#include <cmath>
#include <cstring>
#include <map>
#include <mutex>
#include <tuple>

namespace mxd {
namespace {

constexpr int32_t kNumClasses = (int32_t)(sizeof(kBandClasses) / sizeof(kBandClasses[0]));
// Groups loaded ahead (measured on C2/C3/C4: 2 beats 3..8 once four
// workgroups share a CU); LDS per workgroup is capped so that at least two
// workgroups fit a CU, and one ring area (a group's rows) at kAreaCap.
constexpr int32_t kDefaultLookahead = 2;
constexpr int32_t kMaxLookahead = 8;
constexpr int32_t kLdsCap = 80 * 1024;
constexpr int32_t kAreaCap = 16 * 1024;

int32_t lds_bytes(int32_t la, int32_t db, int32_t nq) {
  BandCfg c{};
  c.la = la;
  c.db = db;
  c.nq = nq;
  return band_lds_bytes(c);
}

}  // namespace

bool band_vertical_shape(const AxisView& yt, int32_t off, int32_t len, int32_t* dmax) {
  int32_t d = 1;
  for (int32_t u = 1; u < len; u++) {
    const int32_t f0 = yt.first[off + u - 1], f1 = yt.first[off + u];
    const int32_t l0 = f0 + yt.count[off + u - 1] - 1, l1 = f1 + yt.count[off + u] - 1;
    if (f1 < f0 || l1 < l0) return false;
    d = std::max(d, l1 - l0);
  }
  *dmax = d;
  return true;
}

int32_t band_slots(const AxisView& yt, int32_t off, int32_t len) {
  static std::mutex mu;
  static std::map<std::tuple<const int32_t*, int32_t, int32_t>, int32_t> cache;
  const auto key = std::make_tuple(yt.first, off, len);
  {
    std::lock_guard<std::mutex> lk(mu);
    auto it = cache.find(key);
    if (it != cache.end()) return it->second;
  }
  auto first = [&](int32_t u) { return yt.first[off + u]; };
  auto last = [&](int32_t u) { return yt.first[off + u] + yt.count[off + u] - 1; };
  // Source row r joins the groups that complete output row b; its weights
  // reach the open rows b .. u for every u whose taps contain r.
  auto reach = [&](int32_t b, int32_t r) {
    int32_t s = 1;
    for (int32_t u = b; u < len && first(u) <= r; u++)
      if (r <= last(u)) s = std::max(s, u - b + 1);
    return s;
  };
  int32_t s = 1;
  for (int32_t b = 0; b < len; b++) {
    // b as a band's first output row: all its taps
    for (int32_t r = first(b); r <= last(b); r++) s = std::max(s, reach(b, r));
    // b as a later row: the rows new for it
    if (b > 0)
      for (int32_t r = last(b - 1) + 1; r <= last(b); r++) s = std::max(s, reach(b, r));
  }
  std::lock_guard<std::mutex> lk(mu);
  cache[key] = s;
  return s;
}

bool band_schedule(const AxisView& yt, int32_t crop_y, int32_t crop_h, int32_t ty, int32_t db, int32_t s,
                   int32_t min_groups, std::vector<int32_t>* words, int32_t* band_words) {
  constexpr int32_t E = kBandEntryWords;
  const int32_t gw = (1 + db) * E;
  const int32_t nb = (crop_h + ty - 1) / ty;
  auto first = [&](int32_t y) { return yt.first[crop_y + y]; };
  auto last = [&](int32_t y) { return yt.first[crop_y + y] + yt.count[crop_y + y] - 1; };
  // groups of every band first (their count sizes the band stride)
  std::vector<std::vector<int32_t>> bands(nb);
  int32_t maxg = 0;
  for (int32_t b = 0; b < nb; b++) {
    std::vector<int32_t>& w = bands[b];
    const int32_t y0 = b * ty, n = std::min(ty, crop_h - y0);
    int32_t ng = 0;
    auto new_group = [&](int32_t flags) {
      w.resize((size_t)(ng + 1) * gw, 0);
      int32_t* g = w.data() + (size_t)ng * gw;
      g[0] = flags;
      for (int32_t j = 0; j < db; j++) g[(1 + j) * E] = -1;
      return ng++;
    };
    for (int32_t u = 0; u < n; u++) {
      const int32_t r0 = u == 0 ? first(y0) : last(y0 + u - 1) + 1, r1 = last(y0 + u);
      const int32_t nr = std::max(0, r1 - r0 + 1);
      const int32_t ngr = std::max(1, (nr + db - 1) / db);  // an upsampled row may bring no new rows
      for (int32_t k = 0; k < ngr; k++) {
        const int32_t g = new_group(k == ngr - 1 ? kBandRowDone : 0);
        for (int32_t j = 0; j < db && r0 + k * db + j <= r1; j++) {
          const int32_t r = r0 + k * db + j;
          int32_t* e = w.data() + (size_t)g * gw + (1 + j) * E;
          e[0] = r;
          // weight slot i = output row u + i of the band (u = the oldest open row)
          for (int32_t v = u; v < n && first(y0 + v) <= r; v++) {
            if (r > last(y0 + v)) continue;
            if (v - u >= s) return false;
            const float wt = yt.w[(size_t)(crop_y + y0 + v) * yt.width + (r - first(y0 + v))];
            std::memcpy(&e[1 + v - u], &wt, sizeof(float));
          }
        }
      }
    }
    while (ng < min_groups) new_group(0);  // the stream needs la + 2 groups per unit
    maxg = std::max(maxg, ng);
  }
  const int32_t bw = E + maxg * gw;
  *band_words = bw;
  words->assign((size_t)nb * bw, 0);
  for (int32_t b = 0; b < nb; b++) {
    int32_t* w = words->data() + (size_t)b * bw;
    w[0] = (int32_t)(bands[b].size() / gw);
    std::copy(bands[b].begin(), bands[b].end(), w + E);
  }
  return true;
}

BandPlan band_plan_image(const AxisView& xt, const AxisView& yt, const BandImage& im, int32_t la_override) {
  BandPlan p;
  const int32_t c = im.channels;
  if (c != 3) return p;
  if ((im.stride & 3) != 0) return p;
  if (im.f32 && ((im.dst | (uintptr_t)im.dst_stride) & 3) != 0) return p;
  int32_t dmax = 0;
  if (!band_vertical_shape(yt, im.crop_y, im.crop_h, &dmax)) return p;
  int32_t xw = 1;
  for (int32_t i = 0; i < im.crop_w; i++) xw = std::max(xw, xt.count[im.crop_x + i]);
  const int32_t slots = band_slots(yt, im.crop_y, im.crop_h);
  int32_t ci = -1;
  for (int32_t k = 0; k < kNumClasses; k++)
    if (kBandClasses[k].taps >= xw && kBandClasses[k].taps <= xt.padded && slots <= kBandClasses[k].s) {
      ci = k;
      break;
    }
  if (ci < 0) return p;
  const BandClass& cl = kBandClasses[ci];
  // Strips: the fewest whose source window (+ the zero-padded taps the
  // horizontal pass reads past the last one) fits the largest window whose
  // ring area stays within kAreaCap, at most one output pixel per thread.
  const int32_t ds = std::max(cl.db, 4);
  const int32_t max_nq = std::max(1, std::min(kBandMaxNq, kAreaCap / (ds * kBandChunk)));
  int32_t ns = (im.crop_w + kBandThreads - 1) / kBandThreads, nq = 0, tx = 0;
  for (; ns <= im.crop_w; ns++) {
    tx = (im.crop_w + ns - 1) / ns;
    if ((im.crop_w + tx - 1) / tx != ns) continue;  // equal strips of tx columns give another count
    int32_t need = 0;
    for (int32_t ox0 = 0; ox0 < im.crop_w; ox0 += tx) {
      const int32_t ox1 = std::min(ox0 + tx, im.crop_w);
      const int32_t xa = im.flip ? im.crop_w - ox1 : ox0;
      const int32_t xb = im.flip ? im.crop_w - 1 - ox0 : ox1 - 1;
      const int32_t lo = xt.first[im.crop_x + xa];
      const int32_t hi = xt.first[im.crop_x + xb] + xt.count[im.crop_x + xb] - 1;
      const int64_t b0 = ((int64_t)(lo - im.x0) * c + im.shift) & ~(int64_t)15;
      need = (int32_t)std::max<int64_t>(need, (int64_t)(hi + cl.taps - im.x0) * c + im.shift - b0);
    }
    nq = (need + kBandChunk - 1) / kBandChunk;
    if (nq <= max_nq) break;
  }
  if (ns > im.crop_w || nq < 1 || nq > max_nq) return p;
  int32_t la = la_override > 0 ? la_override : kDefaultLookahead;
  la = std::min(std::max(la, 1), kMaxLookahead);
  while (la > 1 && lds_bytes(la, cl.db, nq) > kLdsCap) la--;
  if (lds_bytes(la, cl.db, nq) > 160 * 1024) return p;
  const int32_t y_lo = yt.first[im.crop_y];
  const int32_t y_hi = yt.first[im.crop_y + im.crop_h - 1] + yt.count[im.crop_y + im.crop_h - 1] - 1;
  p.ok = true;
  p.cls = ci;
  p.taps = cl.taps;
  p.db = cl.db;
  p.s = cl.s;
  p.nq = nq;
  p.nstrips = ns;
  p.tx = tx;
  p.prologue = (yt.count[im.crop_y] + cl.db - 1) / cl.db - 1;
  p.dmax = dmax;
  p.la = la;
  p.rows_per_out = (double)(y_hi - y_lo + 1) / im.crop_h;
  return p;
}

}  // namespace mxd
