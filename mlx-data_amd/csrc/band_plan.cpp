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
// Bytes of source rows each workgroup keeps in flight (sizes the lookahead);
// LDS per workgroup is capped so that at least two workgroups fit a CU.
constexpr double kTargetInflight = 24.0 * 1024;
constexpr int32_t kMaxLookahead = 8;
constexpr int32_t kLdsCap = 80 * 1024;

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

int32_t band_slots(const AxisView& yt, int32_t off, int32_t len, int32_t db) {
  static std::mutex mu;
  static std::map<std::tuple<const int32_t*, int32_t, int32_t, int32_t>, int32_t> cache;
  const auto key = std::make_tuple(yt.first, off, len, db);
  {
    std::lock_guard<std::mutex> lk(mu);
    auto it = cache.find(key);
    if (it != cache.end()) return it->second;
  }
  auto first = [&](int32_t u) { return yt.first[off + u]; };
  auto last = [&](int32_t u) { return yt.first[off + u] + yt.count[off + u] - 1; };
  int32_t s = 1;
  for (int32_t b = 0; b < len; b++) {
    // a band starting at output b: its first row's taps (prologue groups)
    for (int32_t r = first(b); r <= last(b); r++)
      for (int32_t u = b; u < len && first(u) <= r; u++)
        if (r <= last(u)) s = std::max(s, u - b + (last(b) - r) / db + 1);
    // rows new for output b as a later row of a band
    if (b > 0)
      for (int32_t r = last(b - 1) + 1; r <= last(b); r++)
        for (int32_t u = b; u < len && first(u) <= r; u++)
          if (r <= last(u)) s = std::max(s, u - b + 1);
  }
  std::lock_guard<std::mutex> lk(mu);
  cache[key] = s;
  return s;
}

int32_t band_prologue(const AxisView& yt, int32_t off, int32_t len, int32_t db) {
  int32_t p = 0;
  for (int32_t u = 0; u < len; u++) p = std::max(p, (yt.count[off + u] + db - 1) / db - 1);
  return p;
}

bool band_schedule(const AxisView& yt, int32_t crop_y, int32_t crop_h, int32_t ty, int32_t db, int32_t s,
                   int32_t prologue, std::vector<int32_t>* words, int32_t* band_words) {
  constexpr int32_t E = kBandEntryWords;
  const int32_t P = prologue;
  const int32_t groups = P + ty + 1;  // + one all-absent group
  const int32_t bw = E + groups * db * E;
  const int32_t nb = (crop_h + ty - 1) / ty;
  *band_words = bw;
  words->assign((size_t)nb * bw, 0);
  auto first = [&](int32_t y) { return yt.first[crop_y + y]; };
  auto last = [&](int32_t y) { return yt.first[crop_y + y] + yt.count[crop_y + y] - 1; };
  for (int32_t b = 0; b < nb; b++) {
    int32_t* w = words->data() + (size_t)b * bw;
    const int32_t y0 = b * ty, n = std::min(ty, crop_h - y0);
    w[0] = P;
    int32_t* ent = w + E;
    for (int32_t i = 0; i < groups * db; i++) ent[i * E] = -1;
    std::vector<int32_t> fill(groups, 0);
    bool ok = true;
    // Source row r joins group g; weight slot k of it = output row P + u - g
    // of the band for every output u whose taps contain r.
    auto add_row = [&](int32_t g, int32_t r) {
      if (g < 0 || g >= groups - 1 || fill[g] >= db) return void(ok = false);
      int32_t* e = ent + (size_t)(g * db + fill[g]++) * E;
      e[0] = r;
      for (int32_t u = 0; u < n; u++) {
        if (r < first(y0 + u) || r > last(y0 + u)) continue;
        const int32_t k = P + u - g;
        if (k < 0 || k >= s) return void(ok = false);
        const float wt = yt.w[(size_t)(crop_y + y0 + u) * yt.width + (r - first(y0 + u))];
        std::memcpy(&e[1 + k], &wt, sizeof(float));
      }
    };
    for (int32_t r = first(y0); r <= last(y0); r++) add_row(P - (last(y0) - r) / db, r);
    for (int32_t u = 1; u < n; u++)
      for (int32_t r = last(y0 + u - 1) + 1; r <= last(y0 + u); r++) add_row(P + u, r);
    if (!ok) return false;
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
  int32_t ci = -1;
  for (int32_t k = 0; k < kNumClasses; k++)
    if (kBandClasses[k].taps >= xw && kBandClasses[k].db >= dmax && kBandClasses[k].taps <= xt.padded &&
        band_slots(yt, im.crop_y, im.crop_h, kBandClasses[k].db) <= kBandClasses[k].s) {
      ci = k;
      break;
    }
  if (ci < 0) return p;
  const BandClass& cl = kBandClasses[ci];
  // Strips: the fewest whose source window (+ the zero-padded taps the
  // horizontal pass reads past the last one) fits kBandMaxNq KiB, at most
  // one output pixel per thread.
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
    if (nq <= kBandMaxNq) break;
  }
  if (ns > im.crop_w || nq < 1 || nq > kBandMaxNq) return p;
  const int32_t y_lo = yt.first[im.crop_y];
  const int32_t y_hi = yt.first[im.crop_y + im.crop_h - 1] + yt.count[im.crop_y + im.crop_h - 1] - 1;
  const double rows = (double)(y_hi - y_lo + 1) / im.crop_h;
  int32_t la = la_override > 0 ? la_override
                                : (int32_t)std::ceil(kTargetInflight / (std::max(rows, 1.0) * nq * kBandChunk));
  la = std::min(std::max(la, 1), kMaxLookahead);
  while (la > 1 && lds_bytes(la, cl.db, nq) > kLdsCap) la--;
  if (lds_bytes(la, cl.db, nq) > 160 * 1024) return p;
  p.ok = true;
  p.cls = ci;
  p.taps = cl.taps;
  p.db = cl.db;
  p.s = cl.s;
  p.nq = nq;
  p.nstrips = ns;
  p.tx = tx;
  p.prologue = band_prologue(yt, im.crop_y, im.crop_h, cl.db);
  p.dmax = dmax;
  p.la = la;
  p.rows_per_out = rows;
  return p;
}

}  // namespace mxd
