// plan.cpp -- tap tables, kernel planning and schedule caches of the fused
// resize + crop stage (capi_internal.h).  Host only: planning needs no device
// (host_tables), uploads happen on first use of a table or schedule.
#include "capi_internal.h"

namespace mxd {
namespace capi {

TableCache& tables() {
  static TableCache* c = new TableCache();  // leaked on purpose: outlives static teardown
  return *c;
}

TableCache& host_tables() {
  static TableCache* c = new TableCache(false);
  return *c;
}




ScatterShape scatter_shape_uncached(const DevTable& t, int32_t off, int32_t len) {
  ScatterShape sh;
  auto first = [&](int32_t u) { return t.first[off + u]; };
  auto last = [&](int32_t u) { return t.first[off + u] + t.count[off + u] - 1; };
  int32_t dmax = 1;
  for (int32_t u = 1; u < len; u++) {
    if (first(u) < first(u - 1) || last(u) < last(u - 1)) return sh;
    dmax = std::max(dmax, last(u) - last(u - 1));
  }
  int32_t p = 0;
  for (int32_t u = 0; u < len; u++) p = std::max(p, (t.count[off + u] + dmax - 1) / dmax - 1);
  int32_t s = 1;
  for (int32_t b = 0; b < len; b++) {
    // prologue rows of a band starting at b: slot = (output - b) + (last(b) - r) / dmax
    for (int32_t r = first(b); r <= last(b); r++)
      for (int32_t u = b; u < len && first(u) <= r; u++)
        if (r <= last(u)) s = std::max(s, u - b + (last(b) - r) / dmax + 1);
    // rows new for output b (b > 0 as a non-first output): slot = output - b
    if (b > 0)
      for (int32_t r = last(b - 1) + 1; r <= last(b); r++)
        for (int32_t u = b; u < len && first(u) <= r; u++)
          if (r <= last(u)) s = std::max(s, u - b + 1);
  }
  sh.s = s;
  sh.dmax = dmax;
  sh.p = p;
  return sh;
}

// Cached per (table, crop rows): computing the shape walks every crop row.
ScatterShape scatter_shape(const DevTable& t, int32_t off, int32_t len) {
  static std::mutex mu;
  static std::map<std::tuple<const DevTable*, int32_t, int32_t>, ScatterShape> cache;
  const auto key = std::make_tuple(&t, off, len);
  std::lock_guard<std::mutex> lock(mu);
  auto it = cache.find(key);
  if (it != cache.end()) return it->second;
  return cache[key] = scatter_shape_uncached(t, off, len);
}


class SchedCache {
 public:
  int get(int32_t device, const DevTable& yt, int32_t src_h, int32_t resize_h, int32_t crop_y, int32_t crop_h,
          int32_t ty, const ScatterShape& sh, const DevSched** out) {
    std::lock_guard<std::mutex> lock(mu_);
    const auto key = std::make_tuple(device, src_h, resize_h, crop_y, crop_h, ty, sh.s, sh.dmax, sh.p, sh.lane_bytes);
    auto it = map_.find(key);
    if (it != map_.end()) {
      *out = it->second.get();
      return MXD_OK;
    }
    auto sched = std::make_unique<DevSched>();
    std::vector<int32_t> words;
    if (!build(yt, crop_y, crop_h, ty, sh, &words, sched.get()))
      return fail(MXD_ERR_INVALID, "mxd: scatter schedule does not fit its shape");
    DeviceGuard g(device);
    MXD_HIP(hipMalloc(reinterpret_cast<void**>(&sched->ptr), words.size() * sizeof(int32_t)));
    MXD_HIP(hipMemcpy(sched->ptr, words.data(), words.size() * sizeof(int32_t), hipMemcpyHostToDevice));
    *out = sched.get();
    map_[key] = std::move(sched);
    return MXD_OK;
  }

 private:
  static bool build(const DevTable& yt, int32_t crop_y, int32_t crop_h, int32_t ty, const ScatterShape& sh,
                    std::vector<int32_t>* words, DevSched* d) {
    const int32_t S = sh.s, D = sh.dmax, P = sh.p;
    const int32_t la = mxd::scatter_ring_slots(D, sh.lane_bytes) - 1,
                  bg = mxd::scatter_block_groups(S, D, sh.lane_bytes);
    const int32_t E = mxd::scatter_entry_words(S);
    const int32_t nb = (crop_h + ty - 1) / ty;
    const int32_t gmax = (P + ty + bg - 1) / bg * bg;
    const int32_t gwords = (1 + gmax + 3) & ~3;
    const int32_t iters = gmax * D + la;
    d->band_words = gwords + iters * E;
    d->entry_off = gwords;
    words->assign((size_t)nb * d->band_words, 0);
    auto first = [&](int32_t y) { return yt.first[crop_y + y]; };
    auto last = [&](int32_t y) { return yt.first[crop_y + y] + yt.count[crop_y + y] - 1; };
    for (int32_t b = 0; b < nb; b++) {
      int32_t* w = words->data() + (size_t)b * d->band_words;
      const int32_t y0 = b * ty, n = std::min(ty, crop_h - y0);
      w[0] = (P + n + bg - 1) / bg * bg;
      for (int32_t g = 0; g < gmax; g++) w[1 + g] = g >= P && g - P < n ? y0 + g - P : -1;
      int32_t* ent = w + gwords;
      for (int32_t i = 0; i < iters; i++) ent[i * E] = ent[i * E + 1] = -1;
      std::vector<int32_t> fill(gmax, 0);
      bool ok = true;
      auto add_row = [&](int32_t g, int32_t r) {
        if (g < 0 || g >= gmax || fill[g] >= D) return void(ok = false);
        int32_t* e = ent + (size_t)(g * D + fill[g]++) * E;
        e[1] = r;
        for (int32_t u = 0; u < n; u++) {
          if (r < first(y0 + u) || r > last(y0 + u)) continue;
          const int32_t k = P + u - g;
          if (k < 0 || k >= S) return void(ok = false);
          const float wt = yt.w[(size_t)(crop_y + y0 + u) * yt.width + (r - first(y0 + u))];
          std::memcpy(&e[2 + k], &wt, sizeof(float));
        }
      };
      for (int32_t r = first(y0); r <= last(y0); r++) add_row(P - (last(y0) - r) / D, r);
      for (int32_t u = 1; u < n; u++)
        for (int32_t r = last(y0 + u - 1) + 1; r <= last(y0 + u); r++) add_row(P + u, r);
      if (!ok) return false;
      // word 0 of iteration i: the row iteration i + la loads into the ring
      for (int32_t i = 0; i + la < iters; i++) ent[i * E] = ent[(i + la) * E + 1];
    }
    return true;
  }

  std::mutex mu_;
  std::map<std::tuple<int32_t, int32_t, int32_t, int32_t, int32_t, int32_t, int32_t, int32_t, int32_t, int32_t>,
           std::unique_ptr<DevSched>>
      map_;
};

SchedCache& schedules() {
  static SchedCache* c = new SchedCache();
  return *c;
}

mxd::AxisView axis_view(const DevTable& t) {
  return mxd::AxisView{t.first.data(), t.count.data(), t.w.data(), t.width, t.padded};
}

// Band-kernel schedules (layout: band_plan.h) in device memory, one per
// (device, vertical geometry, crop rows, band height, class, least groups per band).
class BandSchedCache {
 public:
  int get(int32_t device, const DevTable& yt, int32_t src_h, int32_t resize_h, int32_t crop_y, int32_t crop_h,
          int32_t ty, int32_t db, int32_t s, int32_t min_groups, const DevSched** out) {
    std::lock_guard<std::mutex> lock(mu_);
    const auto key = std::make_tuple(device, src_h, resize_h, crop_y, crop_h, ty, db, s, min_groups);
    auto it = map_.find(key);
    if (it != map_.end()) {
      *out = it->second.get();
      return MXD_OK;
    }
    auto sched = std::make_unique<DevSched>();
    std::vector<int32_t> words;
    if (!mxd::band_schedule(axis_view(yt), crop_y, crop_h, ty, db, s, min_groups, &words, &sched->band_words))
      return fail(MXD_ERR_INVALID, "mxd: band schedule does not fit its class");
    DeviceGuard g(device);
    MXD_HIP(hipMalloc(reinterpret_cast<void**>(&sched->ptr), words.size() * sizeof(int32_t)));
    MXD_HIP(hipMemcpy(sched->ptr, words.data(), words.size() * sizeof(int32_t), hipMemcpyHostToDevice));
    *out = sched.get();
    map_[key] = std::move(sched);
    return MXD_OK;
  }

 private:
  std::mutex mu_;
  std::map<std::tuple<int32_t, int32_t, int32_t, int32_t, int32_t, int32_t, int32_t, int32_t, int32_t>,
           std::unique_ptr<DevSched>>
      map_;
};

BandSchedCache& band_schedules() {
  static BandSchedCache* c = new BandSchedCache();
  return *c;
}

// Wave path strips: q output pixels per lane (strip_cols <= 64 q) and every
// strip's source window (start aligned down to wave_window_align()) within
// wave_window_px() pixels.  Fewest strips first (least halo re-reading and
// fewest units), then the smallest q.
bool wave_strips(const DevTable& xt, const mxd_image& im, int32_t pp, int32_t* nstrips, int32_t* tx, int32_t* q) {
  const int32_t c = im.channels, wpx = mxd::wave_window_px(c, pp), al = mxd::wave_window_align(c);
  int32_t best = 0;
  for (int32_t qq : {1, 2, 4}) {
    const int32_t max_tx = mxd::wave_lanes() * qq;
    for (int32_t ns = (im.crop_w + max_tx - 1) / max_tx; ns <= im.crop_w && (best == 0 || ns < best); ns++) {
      const int32_t t = (im.crop_w + ns - 1) / ns;
      if ((im.crop_w + t - 1) / t != ns) continue;  // equal strips of t columns give another count
      bool ok = true;
      for (int32_t ox0 = 0; ox0 < im.crop_w && ok; ox0 += t) {
        const int32_t ox1 = std::min(ox0 + t, im.crop_w);
        const int32_t xa = im.flip ? im.crop_w - ox1 : ox0;
        const int32_t xb = im.flip ? im.crop_w - 1 - ox0 : ox1 - 1;
        const int32_t lo = xt.first[im.crop_x + xa] & ~(al - 1);
        const int32_t hi = xt.first[im.crop_x + xb] + xt.count[im.crop_x + xb] - 1;
        ok = hi + 1 - lo <= wpx;
      }
      if (ok) {
        best = ns;
        *nstrips = ns;
        *tx = t;
        *q = qq;
        break;
      }
    }
  }
  return best > 0;
}

// Output rows per wave unit.  The units of one launch all do about the same
// work, so the launch runs best as whole "rounds" of the device's concurrent
// wave slots: a last round that is only partly filled leaves the HBM queue
// short of loads while it drains.  Pick the fewest rounds whose band height
// stays <= kMaxBand, then the smallest band height whose unit count fits them.
int32_t band_rows(const std::vector<std::pair<int32_t, int32_t>>& strips, int32_t capacity, int32_t kMaxBand) {
  constexpr int32_t kMinBand = 8;
#ifdef MXD_TUNING_ENV  // tuning builds only (tools/ablate8.sh): never read by the product library
  if (const char* e = std::getenv("MXD_BAND_ROWS")) return std::max(1, std::atoi(e));
#endif
  int64_t rows = 0;
  int32_t max_h = 1;
  for (auto& s : strips) {
    rows += (int64_t)s.first * s.second;
    max_h = std::max(max_h, s.second);
  }
  auto units = [&](int32_t ty) {
    int64_t u = 0;
    for (auto& s : strips) u += (int64_t)s.first * ((s.second + std::min(ty, s.second) - 1) / std::min(ty, s.second));
    return u;
  };
  if (capacity <= 0) capacity = 4096;
  kMaxBand = std::max(kMaxBand, kMinBand);
  for (int64_t rounds = 1;; rounds++) {
    const int64_t slots = rounds * capacity;
    int32_t ty = (int32_t)std::max<int64_t>(kMinBand, (rows + slots - 1) / slots);
    if (ty > kMaxBand) continue;
    while (ty < max_h && ty < kMaxBand && units(ty) > slots) ty++;
    if (units(ty) <= slots || ty >= max_h) return std::min(ty, max_h);
  }
}

int32_t band_capacity_cached(const mxd::BandCfg& cfg, int32_t device) {
  static std::mutex mu;
  static std::map<std::tuple<int, int, int, int, int, int, int, int>, int32_t> cache;
  const auto key = std::make_tuple(device, cfg.channels, cfg.f32, cfg.nq, cfg.taps, cfg.s, cfg.db, cfg.la);
  std::lock_guard<std::mutex> lk(mu);
  auto it = cache.find(key);
  if (it != cache.end()) return it->second;
  DeviceGuard g(device);
  const int32_t c = mxd::band_capacity(cfg, device);
  cache[key] = c;
  return c;
}

int32_t wave_capacity_cached(const mxd::WaveCfg& cfg, int32_t device) {
  static std::mutex mu;
  static std::map<std::tuple<int, int, int, int, int, int, int, int, int, int>, int32_t> cache;
  const auto key =
      std::make_tuple(device, cfg.channels, cfg.f32, cfg.taps, cfg.kind, cfg.s, cfg.dmax, cfg.q, cfg.shift, cfg.p);
  std::lock_guard<std::mutex> lk(mu);
  auto it = cache.find(key);
  if (it != cache.end()) return it->second;
  DeviceGuard g(device);
  const int32_t c = mxd::wave_capacity(cfg, device);
  cache[key] = c;
  return c;
}

Stored whole(const mxd_image& im) { return Stored{im.src, im.src_stride, 0, 0, im.src_h}; }

// The wave path reads through the 4-byte aligned address below the stored
// base and shifts its column bytes by the remainder (a source window at any
// x, e.g. random_area_crop); rows must stay 4-byte aligned.  f32 outputs are
// stored per pixel (4-byte aligned), u8 outputs per byte.
bool wave_layout_ok(const mxd_image& im, const Stored& st, int32_t out_dtype) {
  const uintptr_t o = reinterpret_cast<uintptr_t>(im.dst) | (uintptr_t)im.dst_stride;
  const int64_t row = (int64_t)(im.src_w - st.x0) * im.channels;
  return im.channels <= 3 && (st.stride & 3) == 0 && (out_dtype != MXD_F32_DIV255 || (o & 3) == 0) &&
         (int64_t)(reinterpret_cast<uintptr_t>(st.base) & 3) + std::min(row, st.stride) <= st.stride &&
         st.stride * (int64_t)st.rows < ((int64_t)1 << 31);
}

// Byte-lane strips (RGB, wave_byte_lanes): every strip's source span, from
// the 16-byte boundary at or below its first byte (relative to the 4-byte
// aligned stored base), fits the byte window, and its 16-byte chunks rounded
// up stay inside the row stride (so the last stored row never reads past the
// buffer's records).  Fewest strips first, then the smallest q.
bool wave_strips_bytes(const DevTable& xt, const mxd_image& im, const Stored& st, int32_t* nstrips, int32_t* tx,
                       int32_t* q) {
  const int32_t c = im.channels, win = mxd::wave_byte_window();
  const int32_t shift = (int32_t)(reinterpret_cast<uintptr_t>(st.base) & 3);
  int32_t best = 0;
  for (int32_t qq : {1, 2, 4}) {
    const int32_t max_tx = mxd::wave_lanes() * qq;
    for (int32_t ns = (im.crop_w + max_tx - 1) / max_tx; ns <= im.crop_w && (best == 0 || ns < best); ns++) {
      const int32_t t = (im.crop_w + ns - 1) / ns;
      if ((im.crop_w + t - 1) / t != ns) continue;
      bool ok = true;
      for (int32_t ox0 = 0; ox0 < im.crop_w && ok; ox0 += t) {
        const int32_t ox1 = std::min(ox0 + t, im.crop_w);
        const int32_t xa = im.flip ? im.crop_w - ox1 : ox0;
        const int32_t xb = im.flip ? im.crop_w - 1 - ox0 : ox1 - 1;
        const int32_t lo = xt.first[im.crop_x + xa];
        const int32_t hi = xt.first[im.crop_x + xb] + xt.count[im.crop_x + xb] - 1;
        const int64_t b0 = ((int64_t)(lo - st.x0) * c + shift) & ~(int64_t)15;
        const int64_t nb = (int64_t)(hi + 1 - st.x0) * c + shift - b0;
        ok = nb <= win && b0 + (nb + 15) / 16 * 16 <= st.stride;
      }
      if (ok) {
        best = ns;
        *nstrips = ns;
        *tx = t;
        *q = qq;
        break;
      }
    }
  }
  return best > 0;
}

// The band kernel (band.hip) for one image when its class, strips and
// layout fit (p.band = false: wave or general kernel).  Any wave-kernel
// policy bit turns it off, so those policies keep selecting what they name.
constexpr int32_t kWavePolicies = MXD_POLICY_NO_SCATTER | MXD_POLICY_NO_WAVE | MXD_POLICY_NARROW |
                                  MXD_POLICY_NO_BYTES | MXD_POLICY_BYTES;
void plan_band(const mxd_image& im, const Stored& st, int32_t f32, ImgPlan& p) {
  p.band = false;
  if (g_policy.load() & (MXD_POLICY_NO_BAND | kWavePolicies)) return;
  const int64_t c = im.channels, elem = f32 ? 4 : 1;
  const int64_t shift = (int64_t)(reinterpret_cast<uintptr_t>(st.base) & 3);
  const int64_t row = (int64_t)(im.src_w - st.x0) * c;
  const int64_t src_records = shift + (int64_t)(st.rows - 1) * st.stride + std::min(row, st.stride);
  const int64_t dst_records = (int64_t)(im.crop_h - 1) * im.dst_stride + (int64_t)im.crop_w * c * elem;
  if (st.stride <= 0 || src_records >= ((int64_t)1 << 31) || im.dst_stride < 0 ||
      dst_records >= ((int64_t)1 << 31))
    return;
  mxd::BandImage bi{};
  bi.channels = im.channels;
  bi.f32 = f32;
  bi.crop_x = im.crop_x;
  bi.crop_y = im.crop_y;
  bi.crop_w = im.crop_w;
  bi.crop_h = im.crop_h;
  bi.flip = im.flip ? 1 : 0;
  bi.src_w = im.src_w;
  bi.x0 = st.x0;
  bi.shift = (int32_t)shift;
  bi.stride = st.stride;
  bi.dst_stride = im.dst_stride;
  bi.dst = reinterpret_cast<uintptr_t>(im.dst);
  p.bp = mxd::band_plan_image(axis_view(*p.xt), axis_view(*p.yt), bi, g_tune[MXD_TUNE_BAND_LA].load());
  p.band = p.bp.ok;
}

constexpr int32_t kMaxScatterDepth = 16;  // deepest scatter schedule (wave.hip select_scatter)

// The scatter kernel for a vertical shape: the smallest instantiated tap
// bucket >= xw and schedule depth >= sh.dmax (a deeper schedule runs the same
// rows with bubble iterations, so any downscale ratio up to 16:1 reaches a
// kernel instead of the general path).
bool scatter_kernel_for(int32_t c, int32_t f32, int32_t xw, const ScatterShape& sh, int32_t q, int32_t shift,
                        int32_t pp, int32_t* taps, int32_t* dmax) {
  if (sh.s <= 0) return false;
  for (int32_t t = mxd::wave_taps_bucket(xw); t > 0; t = mxd::wave_taps_bucket(t + 1))
    for (int32_t d = sh.dmax; d <= kMaxScatterDepth; d++)
      if (mxd::wave_has_kernel(mxd::WaveCfg{c, f32, t, 0, 0, 2, sh.s, d, q, shift, pp})) {
        *taps = t;
        *dmax = d;
        return true;
      }
  return false;
}

// Chooses the wave kernel of one image (p.wave = false: the general kernel):
// over the lane widths available for its channel count, the one that cuts
// the crop into the fewest strips (narrow strips read more halo and more,
// shorter row pieces), then the narrower lane width.
void plan_wave(const mxd_image& im, const Stored& st, int32_t f32, int32_t out_dtype, ImgPlan& p) {
  p.wave = false;
  p.ycc = false;
  const bool ycc = st.ycc != nullptr;
  if (ycc) {
    // JPEG planes: the RGB-row layout rules do not apply, only the output's
    const uintptr_t o = reinterpret_cast<uintptr_t>(im.dst) | (uintptr_t)im.dst_stride;
    if (im.channels != 3 || ((reinterpret_cast<uintptr_t>(st.base) | (uintptr_t)st.stride) & 3) != 0 ||
        (out_dtype == MXD_F32_DIV255 && (o & 3) != 0))
      return;
  } else if (!wave_layout_ok(im, st, out_dtype)) {
    return;
  }
  const int32_t c = im.channels;
  const int32_t shift = (reinterpret_cast<uintptr_t>(st.base) & 3) != 0 ? 1 : 0;
  // Scatter when the vertical axis downsamples into a shape with a kernel,
  // else gather.
  const ScatterShape sh =
      (g_policy.load() & MXD_POLICY_NO_SCATTER) ? ScatterShape{} : scatter_shape(*p.yt, im.crop_y, im.crop_h);
  const int32_t gb = mxd::wave_taps_bucket(std::max(p.xt->width, p.yt->width));
  const int32_t dp = mxd::wave_default_p(c);
  const int32_t policy = g_policy.load();
  const int32_t widths[2] = {dp, c == 3 && !(policy & MXD_POLICY_NARROW) ? 8 : dp};
  for (int32_t pp : widths) {
    if (p.wave && pp == p.pp) continue;
    if (ycc && pp != 4) continue;  // plane sources: four RGB pixels per lane
    int32_t ns = 0, tx = 0, q = 0;
    if (!wave_strips(*p.xt, im, pp, &ns, &tx, &q)) continue;
    if (p.wave && ns >= p.nstrips) continue;
    // A crop the wide lanes take in one strip that narrow lanes take in two
    // (ImageNet shapes, 480p) keeps the narrow kernel: at 64-78 VGPRs it runs
    // 8 waves per SIMD where the wide one-strip kernels (132-146 VGPRs) run 2-3
    // -- C4 0.0237 -> 0.0229 ms per launch, C3 unchanged
    // (profiles/r03/onestrip.jsonl).
    if (p.wave && p.nstrips == 2 && ns == 1 && pp == 8) continue;
    ImgPlan cand = p;
    cand.nstrips = ns;
    cand.tx = tx;
    cand.q = q;
    cand.pp = pp;
    cand.shift = shift;
    int32_t tb = 0, td = 0;
    if (scatter_kernel_for(c, f32, p.xt->width, sh, q, shift, pp, &tb, &td)) {
      cand.kind = 2;
      cand.bucket = tb;
      cand.s = sh.s;
      cand.dmax = td;
      cand.p = sh.p;
    } else if (!ycc && gb > 0 && mxd::wave_has_kernel(mxd::WaveCfg{c, f32, gb, 0, 0, 0, 0, 0, q, shift, pp})) {
      cand.kind = 0;
      cand.bucket = gb;
    } else {
      continue;
    }
    cand.wave = true;
    cand.ycc = ycc;
    p = cand;
  }
  if (ycc) return;
  // RGB scatter: byte lanes (one 1-KiB contiguous load per wave and row)
  // instead of wide pixel lanes when they cut the crop into no more strips,
  // at <= 2 output pixels per lane (measured: 720p -> 224 with two strips 4 %
  // faster; with more strips -- their narrower 341-pixel window -- or a single
  // 224-column strip (C4) pixel lanes were 2-10 % faster;
  // profiles/r02/bytes_ab.txt).  Never instead of the narrow kernel (480p:
  // 0.0908 vs 0.0977 ms, profiles/r03/c3_layouts.jsonl).
  if (c == 3 && sh.s > 0 && !(policy & (MXD_POLICY_NO_BYTES | MXD_POLICY_NARROW))) {
    int32_t ns = 0, tx = 0, q = 0, bt = 0, bd = 0;
    if (wave_strips_bytes(*p.xt, im, st, &ns, &tx, &q) &&
        ((policy & MXD_POLICY_BYTES) || !p.wave || p.kind != 2 || (p.pp == 8 && ns <= p.nstrips && q <= 2)) &&
        scatter_kernel_for(c, f32, p.xt->width, sh, q, 0, 16, &bt, &bd)) {
      p.wave = true;
      p.nstrips = ns;
      p.tx = tx;
      p.q = q;
      p.pp = 16;
      p.shift = 0;
      p.kind = 2;
      p.bucket = bt;
      p.s = sh.s;
      p.dmax = bd;
      p.p = sh.p;
    }
  }
}

PlanKey plan_key(const mxd_image& im, const Stored& st) {
  const uint64_t ss = (uint64_t)st.stride, ds = (uint64_t)im.dst_stride;
  return PlanKey{{im.src_w, im.src_h, im.channels, im.resize_w, im.resize_h, im.crop_x, im.crop_y, im.crop_w,
                  im.crop_h, im.flip ? 1 : 0, im.rgba_weighted, st.x0, st.rows, (int32_t)ss, (int32_t)(ss >> 32),
                  (int32_t)ds, (int32_t)(ds >> 32), (int32_t)(reinterpret_cast<uintptr_t>(st.base) & 15),
                  (int32_t)(reinterpret_cast<uintptr_t>(im.dst) & 15), st.ycc ? 1 : 0}};
}

bool ycc_plan_ok(const mxd_image& im, const Stored& st, int32_t out_dtype, int32_t device) {
  if (!st.ycc || (g_policy.load() & MXD_POLICY_NO_WAVE)) return false;
  ImgPlan p;
  if (tables().get(device, im.src_w, im.resize_w, &p.xt) != MXD_OK) return false;
  if (tables().get(device, im.src_h, im.resize_h, &p.yt) != MXD_OK) return false;
  plan_wave(im, st, out_dtype == MXD_F32_DIV255 ? 1 : 0, out_dtype, p);
  return p.wave && p.ycc;
}


int scatter_schedule(int32_t device, const DevTable& yt, int32_t src_h, int32_t resize_h, int32_t crop_y,
                     int32_t crop_h, int32_t ty, const ScatterShape& sh, const DevSched** out) {
  return schedules().get(device, yt, src_h, resize_h, crop_y, crop_h, ty, sh, out);
}

int band_schedule_dev(int32_t device, const DevTable& yt, int32_t src_h, int32_t resize_h, int32_t crop_y, int32_t crop_h,
                  int32_t ty, int32_t db, int32_t s, int32_t min_groups, const DevSched** out) {
  return band_schedules().get(device, yt, src_h, resize_h, crop_y, crop_h, ty, db, s, min_groups, out);
}

}  // namespace capi
}  // namespace mxd
