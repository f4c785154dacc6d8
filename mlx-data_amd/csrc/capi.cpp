// capi.cpp -- the C ABI declared in include/mxd_amd.h.
//
// Host side of the fused resize+crop stage: validation with the reference's
// error conditions, per-device caches of the axis tap tables, tiling, a
// per-stream descriptor workspace, and the launch.  No exceptions cross the
// ABI: every entry point returns a status and leaves a thread-local message.
#include <hip/hip_runtime.h>
#include <sched.h>

#include <algorithm>
#include <numeric>
#include <atomic>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <condition_variable>
#include <cstring>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <tuple>
#include <unordered_map>
#include <vector>

#include "mxd_amd.h"
#include "band.h"
#include "band_plan.h"
#include "jpeg.h"
#include "jpegdev.h"
#include "pixmap.h"
#include "resample.h"
#include "taps.h"

using mxd::ImgDev;
using mxd::LaunchCfg;

namespace {

thread_local std::string g_error;

int fail(int code, const std::string& msg) {
  g_error = msg;
  return code;
}

// Every entry point that takes a device ordinal refuses one that does not
// exist (DeviceGuard would otherwise leave the work on the current device).
int check_device(int32_t device) {
  static const int count = [] {
    int n = 0;
    return hipGetDeviceCount(&n) == hipSuccess ? n : 0;
  }();
  if (device < 0 || device >= count)
    return fail(MXD_ERR_INVALID, "mxd: invalid device " + std::to_string(device) + " (" + std::to_string(count) +
                                     " visible)");
  return MXD_OK;
}

#define MXD_HIP(expr)                                                                                    \
  do {                                                                                                   \
    hipError_t e_ = (expr);                                                                              \
    if (e_ != hipSuccess) return fail(MXD_ERR_DEVICE, std::string(#expr) + ": " + hipGetErrorString(e_)); \
  } while (0)

// Restores the calling thread's current device on scope exit.
struct DeviceGuard {
  int prev = -1;
  explicit DeviceGuard(int dev) {
    if (hipGetDevice(&prev) != hipSuccess) prev = -1;
    if (prev != dev) (void)hipSetDevice(dev);
  }
  ~DeviceGuard() {
    int cur = -1;
    if (prev >= 0 && hipGetDevice(&cur) == hipSuccess && cur != prev) (void)hipSetDevice(prev);
  }
};

// ---------------------------------------------------------------------------
// Device tap tables: one per (device, in_size, out_size), covering every
// output pixel of the axis, so any crop window is a pointer offset into it.
struct DevTable {
  float* ptr = nullptr;
  int32_t width = 0;     // max taps of any output
  int32_t padded = 0;    // weights per entry in device memory (>= kMinTabWidth)
  std::vector<int32_t> first, count;  // host copy for tiling decisions
  std::vector<float> w;               // host copy of the weights, `width` per output (scatter schedules)
};

class TableCache {
 public:
  // upload = false: host copies only (ptr stays null), for planning without a device.
  explicit TableCache(bool upload = true) : upload_(upload) {}
  int get(int32_t device, int32_t in, int32_t out, const DevTable** out_tab) {
    std::lock_guard<std::mutex> lock(mu_);
    auto key = std::make_tuple(device, in, out);
    auto it = map_.find(key);
    if (it != map_.end()) {
      *out_tab = it->second.get();
      return MXD_OK;
    }
    mxd::AxisTaps taps;
    if (!mxd::build_axis_taps(in, out, 0, out, &taps))
      return fail(MXD_ERR_INVALID, "image: cannot create image with 0 or negative dimension");
    const int32_t padded = std::max<int32_t>(taps.width, mxd::kMinTabWidth);
    const int32_t stride = mxd::kTapHeader + padded;
    std::vector<float> host((size_t)out * stride, 0.0f);
    for (int32_t i = 0; i < out; i++) {
      float* e = &host[(size_t)i * stride];
      std::memcpy(&e[0], &taps.first[i], 4);
      std::memcpy(&e[1], &taps.count[i], 4);
      std::memcpy(&e[2], &taps.weight[(size_t)i * taps.width], sizeof(float) * taps.width);
    }
    auto tab = std::make_unique<DevTable>();
    tab->width = taps.width;
    tab->padded = padded;
    tab->first = taps.first;
    tab->count = taps.count;
    tab->w = taps.weight;
    if (upload_) {
      DeviceGuard g(device);
      MXD_HIP(hipMalloc(&tab->ptr, host.size() * sizeof(float)));
      MXD_HIP(hipMemcpy(tab->ptr, host.data(), host.size() * sizeof(float), hipMemcpyHostToDevice));
    }
    *out_tab = tab.get();
    map_[key] = std::move(tab);
    return MXD_OK;
  }

 private:
  bool upload_;
  std::mutex mu_;
  std::map<std::tuple<int32_t, int32_t, int32_t>, std::unique_ptr<DevTable>> map_;
};

TableCache& tables() {
  static TableCache* c = new TableCache();  // leaked on purpose: outlives static teardown
  return *c;
}

TableCache& host_tables() {
  static TableCache* c = new TableCache(false);
  return *c;
}

// ---------------------------------------------------------------------------
// Per-(device, stream) descriptor workspace: pinned staging + device copy of
// the ImgDev array.  Re-uploads are skipped when the batch is unchanged.
// Kernel policy (mxd_set_kernel_policy): a process-wide tuning / test switch
// between kernels that compute identical results.
std::atomic<int32_t> g_policy{0};
// Tuning knobs (mxd_set_tuning): 0 = automatic.
std::atomic<int32_t> g_tune[MXD_TUNE_COUNT] = {};

struct Workspace {
  std::mutex mu;
  // Descriptor slots: each launch reads its descriptors from one slot's
  // device copy.  A batch whose descriptors a slot holds reuses it; a new one
  // takes the least recently used slot once the launches that read it are
  // done, and uploads on a copy stream while the previous launch computes.
  // Launches wait for their slot's upload, so consecutive batches never
  // serialize behind an H2D copy.
  static constexpr int kSlots = 4;
  struct Slot {
    ImgDev* host = nullptr;  // pinned
    ImgDev* dev = nullptr;
    size_t cap = 0, count = 0;
    hipEvent_t copied = nullptr, used = nullptr;
    uint64_t last_use = 0;
    bool unrecorded_hits = false;  // launched from since `used` was last recorded
  } slot[kSlots];
  int cur = -1;
  uint64_t clock = 0;
  hipStream_t copy = nullptr;
  // Fork/join helpers: the launches of a mixed batch (one per kernel shape)
  // run concurrently on these streams, so one launch's tail overlaps the
  // next instead of idling the CUs between serialized launches.
  static constexpr int kHelpers = 3;
  hipStream_t helper[kHelpers] = {};
  hipEvent_t fork = nullptr, join[kHelpers] = {};
};

class WorkspacePool {
 public:
  Workspace* get(int32_t device, void* stream) {
    std::lock_guard<std::mutex> lock(mu_);
    auto& w = map_[std::make_pair(device, stream)];
    if (!w) w = std::make_unique<Workspace>();
    return w.get();
  }

 private:
  std::mutex mu_;
  std::map<std::pair<int32_t, void*>, std::unique_ptr<Workspace>> map_;
};

WorkspacePool& workspaces() {
  static WorkspacePool* p = new WorkspacePool();
  return *p;
}

// ---------------------------------------------------------------------------
// Tiling.
constexpr int32_t kTileRows = 32;          // output rows per tile
constexpr int32_t kStripBytes = 1536;      // target source-footprint bytes per strip row
constexpr int32_t kLdsBudget = 40 * 1024;  // bytes of LDS for the f32 row group
constexpr int32_t kBandMaxRows = 16;       // band kernel: most output rows per unit (short units keep the
                                           // device on few images at a time; the stream makes them cheap)

int32_t strip_chunks(const DevTable& xt, int32_t crop_x, int32_t crop_w, int32_t ox0, int32_t ox1, bool flip,
                     int32_t c, int32_t vec) {
  const int32_t xa = flip ? crop_w - ox1 : ox0;
  const int32_t xb = flip ? crop_w - 1 - ox0 : ox1 - 1;
  const int32_t lo = xt.first[crop_x + xa];
  const int32_t hi = xt.first[crop_x + xb] + xt.count[crop_x + xb] - 1;
  const int32_t fb0 = (lo * c) & ~(vec - 1);
  return ((hi + 1) * c - fb0 + vec - 1) / vec;
}

int validate(const mxd_image& im, int32_t i) {
  const std::string at = " (image " + std::to_string(i) + ")";
  if (!im.src || !im.dst) return fail(MXD_ERR_INVALID, "mxd: null src/dst pointer" + at);
  if (im.src_w <= 0 || im.src_h <= 0)
    return fail(MXD_ERR_INVALID, "image: cannot create image with 0 or negative dimension" + at);
  if (im.channels <= 0 || im.channels > 4)
    return fail(MXD_ERR_INVALID, "verifyImage: channels must be 0 <= c <= 4" + at);
  if (im.resize_w <= 0 || im.resize_h <= 0 || im.crop_w <= 0 || im.crop_h <= 0)
    return fail(MXD_ERR_INVALID, "image: cannot create image with 0 or negative dimension" + at);
  if (im.crop_x < 0 || im.crop_y < 0 || im.crop_x >= im.resize_w || im.crop_y >= im.resize_h)
    return fail(MXD_ERR_INVALID, "Array: sub: offset out of bound" + at);
  if (im.crop_x + im.crop_w > im.resize_w || im.crop_y + im.crop_h > im.resize_h)
    return fail(MXD_ERR_INVALID, "Array: sub: shape out of bound" + at);
  if (im.src_stride < (int64_t)im.src_w * im.channels)
    return fail(MXD_ERR_INVALID, "mxd: src_stride smaller than a row" + at);
  return MXD_OK;
}

// Uploads descs to the stream's workspace (skipped when unchanged) and returns
// the device copy.
int upload_descs(const std::vector<ImgDev>& descs, int32_t device, void* stream, ImgDev** dev_out,
                 std::unique_lock<std::mutex>* hold, Workspace** ws_out = nullptr, bool* hit = nullptr) {
  if (hit) *hit = false;
  Workspace* ws = workspaces().get(device, stream);
  if (ws_out) *ws_out = ws;
  *hold = std::unique_lock<std::mutex>(ws->mu);
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  const size_t n = descs.size();
  const size_t bytes = sizeof(ImgDev) * n;
  // A batch whose descriptors a slot already holds (a loop over fixed device
  // buffers) launches from that slot's device copy: no upload, no
  // cross-stream wait once the copy has landed.  Slots are immutable while
  // cached, so concurrent readers are safe.
  if (!(g_policy.load() & MXD_POLICY_NO_DESC_CACHE))
    for (int k = 0; k < Workspace::kSlots; k++) {
      Workspace::Slot& c = ws->slot[k];
      if (c.count == n && c.host && std::memcmp(c.host, descs.data(), bytes) == 0) {
        ws->cur = k;
        c.last_use = ++ws->clock;
        if (hipEventQuery(c.copied) != hipSuccess) MXD_HIP(hipStreamWaitEvent(s, c.copied, 0));
        // No per-launch event (it costs ~2.5 us between kernels): the slot's
        // readers are fenced when it is next overwritten (below).
        c.unrecorded_hits = true;
        *dev_out = c.dev;
        if (hit) *hit = true;
        return MXD_OK;
      }
    }
  if (!ws->copy) MXD_HIP(hipStreamCreateWithFlags(&ws->copy, hipStreamNonBlocking));
  // the least recently used slot takes the new batch
  int victim = 0;
  for (int k = 1; k < Workspace::kSlots; k++)
    if (ws->slot[k].last_use < ws->slot[victim].last_use) victim = k;
  ws->cur = victim;
  ws->slot[victim].last_use = ++ws->clock;
  Workspace::Slot& c = ws->slot[ws->cur];
  if (!c.copied) {
    MXD_HIP(hipEventCreateWithFlags(&c.copied, hipEventDisableTiming));
    MXD_HIP(hipEventCreateWithFlags(&c.used, hipEventDisableTiming));
  } else {
    // Launched from by cache hits since `used` was recorded: fence them now
    // (after every launch enqueued so far).  Only a working-set change evicts
    // such a slot; a stream of fresh batches never has hits.
    if (c.unrecorded_hits) {
      MXD_HIP(hipEventRecord(c.used, s));
      c.unrecorded_hits = false;
    }
    // Host-side wait: the launches that read this slot are done.  (Ordering
    // the upload after them on the GPU instead, with a wait of the copy
    // stream on the compute stream, measured ms-long stalls.)
    MXD_HIP(hipEventSynchronize(c.used));
  }
  if (n > c.cap) {
    if (c.dev) MXD_HIP(hipFree(c.dev));
    if (c.host) MXD_HIP(hipHostFree(c.host));
    c.dev = nullptr;
    c.host = nullptr;
    const size_t cap = std::max<size_t>(n, 64);
    MXD_HIP(hipMalloc(reinterpret_cast<void**>(&c.dev), sizeof(ImgDev) * cap));
    MXD_HIP(hipHostMalloc(reinterpret_cast<void**>(&c.host), sizeof(ImgDev) * cap, hipHostMallocDefault));
    c.cap = cap;
  }
  std::memcpy(c.host, descs.data(), bytes);
  c.count = n;
  MXD_HIP(hipMemcpyAsync(c.dev, c.host, bytes, hipMemcpyHostToDevice, ws->copy));
  MXD_HIP(hipEventRecord(c.copied, ws->copy));
  MXD_HIP(hipStreamWaitEvent(s, c.copied, 0));
  *dev_out = c.dev;
  return MXD_OK;
}

// After the launches of a batch: the slot is free again once they finish.
int release_descs(Workspace* ws, void* stream) {
  MXD_HIP(hipEventRecord(ws->slot[ws->cur].used, reinterpret_cast<hipStream_t>(stream)));
  return MXD_OK;
}

struct ImgPlan {
  const DevTable* xt = nullptr;
  const DevTable* yt = nullptr;
  bool band = false;     // runs on the band kernel (band.hip)
  mxd::BandPlan bp;      // its plan
  bool wave = false;     // runs on a wave kernel (wave.hip), else the general tile kernel
  int32_t bucket = -1;   // wave kernel tap bucket
  int32_t kind = 0;      // wave kernel: 0 gather, 2 scatter
  int32_t s = 0, dmax = 0, p = 0;  // scatter shape (ScatterShape)
  int32_t nstrips = 0, tx = 0, q = 0, shift = 0;
  int32_t pp = 0;  // source pixels per lane
};


// Shape of the scatter schedule for crop rows [off, off+len) of a vertical
// table, valid for bands starting at any row: dmax = most source rows that are
// new for one output row (after the previous row's last tap), p = prologue
// groups (the first output of a band needs all its taps), s = most output rows
// a source row's weights must reach from its group (accumulator slots).
// s = 0: taps not monotone (not a geometry the scatter kernel handles).
struct ScatterShape {
  int32_t s = 0, dmax = 0, p = 0;
};

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

// Scatter schedules (layout: wave.hip) in device memory, one per
// (device, vertical geometry, crop rows, band height, shape).
struct DevSched {
  int32_t* ptr = nullptr;
  int32_t band_words = 0;  // words per band
  int32_t entry_off = 0;   // word offset of the iteration entries in a band
};

class SchedCache {
 public:
  int get(int32_t device, const DevTable& yt, int32_t src_h, int32_t resize_h, int32_t crop_y, int32_t crop_h,
          int32_t ty, const ScatterShape& sh, const DevSched** out) {
    std::lock_guard<std::mutex> lock(mu_);
    const auto key = std::make_tuple(device, src_h, resize_h, crop_y, crop_h, ty, sh.s, sh.dmax, sh.p);
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
    const int32_t la = mxd::scatter_ring_slots(D) - 1, bg = mxd::scatter_block_groups(S, D);
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
  std::map<std::tuple<int32_t, int32_t, int32_t, int32_t, int32_t, int32_t, int32_t, int32_t, int32_t>,
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
int32_t band_rows(const std::vector<std::pair<int32_t, int32_t>>& strips, int32_t capacity, int32_t kMaxBand = 64) {
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
  for (int64_t rounds = 1;; rounds++) {
    const int64_t slots = rounds * capacity;
    int32_t ty = (int32_t)std::max<int64_t>(kMinBand, (rows + slots - 1) / slots);
    if (ty > kMaxBand) continue;
    while (ty < max_h && units(ty) > slots) ty++;
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

// Where an image's source bytes live: the whole image at mxd_image::src, or
// (host path) only its staged footprint: `rows` rows from source row y0 and
// columns from source pixel x0 at base, `stride` bytes apart.
struct Stored {
  const uint8_t* base;
  int64_t stride;
  int32_t x0, y0, rows;
};

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

// Chooses the wave kernel of one image (p.wave = false: the general kernel):
// over the lane widths available for its channel count, the one that cuts
// the crop into the fewest strips (narrow strips read more halo and more,
// shorter row pieces), then the narrower lane width.
void plan_wave(const mxd_image& im, const Stored& st, int32_t f32, int32_t out_dtype, ImgPlan& p) {
  p.wave = false;
  if (!wave_layout_ok(im, st, out_dtype)) return;
  const int32_t c = im.channels;
  const int32_t shift = (reinterpret_cast<uintptr_t>(st.base) & 3) != 0 ? 1 : 0;
  // Scatter when the vertical axis downsamples into a shape with a kernel,
  // else gather.
  const ScatterShape sh =
      (g_policy.load() & MXD_POLICY_NO_SCATTER) ? ScatterShape{} : scatter_shape(*p.yt, im.crop_y, im.crop_h);
  const int32_t xb = mxd::wave_taps_bucket(p.xt->width);
  const int32_t gb = mxd::wave_taps_bucket(std::max(p.xt->width, p.yt->width));
  const int32_t dp = mxd::wave_default_p(c);
  const int32_t policy = g_policy.load();
  const int32_t widths[2] = {dp, c == 3 && !(policy & MXD_POLICY_NARROW) ? 8 : dp};
  for (int32_t pp : widths) {
    if (p.wave && pp == p.pp) continue;
    int32_t ns = 0, tx = 0, q = 0;
    if (!wave_strips(*p.xt, im, pp, &ns, &tx, &q)) continue;
    if (p.wave && ns >= p.nstrips) continue;
    ImgPlan cand = p;
    cand.nstrips = ns;
    cand.tx = tx;
    cand.q = q;
    cand.pp = pp;
    cand.shift = shift;
    if (sh.s > 0 && xb > 0 &&
        mxd::wave_has_kernel(mxd::WaveCfg{c, f32, xb, 0, 0, 2, sh.s, sh.dmax, q, shift, pp})) {
      cand.kind = 2;
      cand.bucket = xb;
      cand.s = sh.s;
      cand.dmax = sh.dmax;
      cand.p = sh.p;
    } else if (gb > 0 && mxd::wave_has_kernel(mxd::WaveCfg{c, f32, gb, 0, 0, 0, 0, 0, q, shift, pp})) {
      cand.kind = 0;
      cand.bucket = gb;
    } else {
      continue;
    }
    cand.wave = true;
    p = cand;
  }
  // RGB scatter: byte lanes (one 1-KiB contiguous load per wave and row)
  // when they cut the crop into no more strips than pixel lanes do, at <= 2
  // output pixels per lane (measured: 720p -> 224 with two strips 4 % faster;
  // with more strips -- their narrower 341-pixel window -- or a single 224-column
  // strip (C4) pixel lanes were 2-10 % faster; profiles/r02/bytes_ab.txt).
  if (c == 3 && sh.s > 0 && xb > 0 && !(policy & (MXD_POLICY_NO_BYTES | MXD_POLICY_NARROW))) {
    int32_t ns = 0, tx = 0, q = 0;
    if (wave_strips_bytes(*p.xt, im, st, &ns, &tx, &q) &&
        ((policy & MXD_POLICY_BYTES) || !p.wave || p.kind != 2 || (ns <= p.nstrips && q <= 2)) &&
        mxd::wave_has_kernel(mxd::WaveCfg{c, f32, xb, 0, 0, 2, sh.s, sh.dmax, q, 0, 16})) {
      p.wave = true;
      p.nstrips = ns;
      p.tx = tx;
      p.q = q;
      p.pp = 16;
      p.shift = 0;
      p.kind = 2;
      p.bucket = xb;
      p.s = sh.s;
      p.dmax = sh.dmax;
      p.p = sh.p;
    }
  }
}

// What a plan depends on: geometry, the stored region's layout and the
// alignments of source and destination.
struct PlanKey {
  int32_t v[20];
  bool operator==(const PlanKey& o) const { return std::memcmp(v, o.v, sizeof v) == 0; }
};
struct PlanKeyHash {
  size_t operator()(const PlanKey& k) const {
    uint64_t h = 1469598103934665603ull;  // FNV-1a over the words
    for (int32_t x : k.v) h = (h ^ (uint32_t)x) * 1099511628211ull;
    return (size_t)h;
  }
};
PlanKey plan_key(const mxd_image& im, const Stored& st) {
  const uint64_t ss = (uint64_t)st.stride, ds = (uint64_t)im.dst_stride;
  return PlanKey{{im.src_w, im.src_h, im.channels, im.resize_w, im.resize_h, im.crop_x, im.crop_y, im.crop_w,
                  im.crop_h, im.flip ? 1 : 0, im.rgba_weighted, st.x0, st.rows, (int32_t)ss, (int32_t)(ss >> 32),
                  (int32_t)ds, (int32_t)(ds >> 32), (int32_t)(reinterpret_cast<uintptr_t>(st.base) & 15),
                  (int32_t)(reinterpret_cast<uintptr_t>(im.dst) & 15), 0}};
}

int run_batch(const mxd_image* images, int32_t n, int32_t out_dtype, int32_t device, void* stream,
              const Stored* stored = nullptr) {
  if (n < 0 || (n > 0 && !images)) return fail(MXD_ERR_INVALID, "mxd: bad image array");
  if (out_dtype != MXD_U8 && out_dtype != MXD_F32_DIV255) return fail(MXD_ERR_INVALID, "mxd: bad out_dtype");
  if (n == 0) return MXD_OK;
  const int64_t elem = out_dtype == MXD_F32_DIV255 ? 4 : 1;
  const int32_t channels = images[0].channels;
  bool mixed = false;
  for (int32_t i = 0; i < n; i++) {
    if (int rc = validate(images[i], i)) return rc;
    mixed = mixed || images[i].channels != channels;
    if (images[i].dst_stride < (int64_t)images[i].crop_w * images[i].channels * elem)
      return fail(MXD_ERR_INVALID, "mxd: dst_stride smaller than an output row");
  }
  if (int rc = check_device(device)) return rc;
  if (mixed) {
    // one channel count per launch: one sub-batch per count, in order
    for (int32_t c = 1; c <= 4; c++) {
      std::vector<mxd_image> sub;
      std::vector<Stored> ssub;
      for (int32_t i = 0; i < n; i++)
        if (images[i].channels == c) {
          sub.push_back(images[i]);
          if (stored) ssub.push_back(stored[i]);
        }
      if (!sub.empty())
        if (int rc = run_batch(sub.data(), (int32_t)sub.size(), out_dtype, device, stream, stored ? ssub.data() : nullptr))
          return rc;
    }
    return MXD_OK;
  }
  if (channels == 4) {
    // one alpha mode per general-kernel launch: split a mixed batch
    int32_t nw = 0;
    for (int32_t i = 0; i < n; i++) nw += images[i].rgba_weighted ? 1 : 0;
    if (nw > 0 && nw < n) {
      std::vector<mxd_image> a, b;
      std::vector<Stored> sa, sb;
      for (int32_t i = 0; i < n; i++) {
        (images[i].rgba_weighted ? a : b).push_back(images[i]);
        if (stored) (images[i].rgba_weighted ? sa : sb).push_back(stored[i]);
      }
      if (int rc = run_batch(a.data(), (int32_t)a.size(), out_dtype, device, stream, stored ? sa.data() : nullptr))
        return rc;
      return run_batch(b.data(), (int32_t)b.size(), out_dtype, device, stream, stored ? sb.data() : nullptr);
    }
  }
  const int32_t f32 = out_dtype == MXD_F32_DIV255 ? 1 : 0;
  const bool no_wave = (g_policy.load() & MXD_POLICY_NO_WAVE) != 0;
  std::vector<ImgPlan> plans(n);
  std::vector<int32_t> slow;  // images for the general kernel
  // Images of one geometry, layout and alignment share a plan (and later a
  // schedule): planning walks tap tables, and a batch rarely holds more than
  // a few shapes.  rep[i] = the first image with image i's key.
  std::vector<int32_t> rep(n);
  {
    std::unordered_map<PlanKey, int32_t, PlanKeyHash> first_of;
    first_of.reserve(16);
    for (int32_t i = 0; i < n; i++) {
      const mxd_image& im = images[i];
      const Stored st = stored ? stored[i] : whole(im);
      const auto ins = first_of.emplace(plan_key(im, st), i);
      rep[i] = ins.first->second;
      ImgPlan& p = plans[i];
      if (!ins.second) {
        p = plans[rep[i]];
      } else {
        if (int rc = tables().get(device, im.src_w, im.resize_w, &p.xt)) return rc;
        if (int rc = tables().get(device, im.src_h, im.resize_h, &p.yt)) return rc;
        if (!no_wave) {
          if (g_policy.load() & MXD_POLICY_PREFER_BAND) {
            plan_band(im, st, f32, p);
            if (!p.band) plan_wave(im, st, f32, out_dtype, p);
          } else {
            plan_wave(im, st, f32, out_dtype, p);
            if (!p.wave) plan_band(im, st, f32, p);
          }
        }
      }
      if (!p.band && !p.wave) slow.push_back(i);
    }
  }
  DeviceGuard guard(device);
  auto fill = [&](ImgDev& d, int32_t i, const ImgPlan& p) {
    const mxd_image& im = images[i];
    const Stored st = stored ? stored[i] : whole(im);
    d = ImgDev{};
    d.src = st.base;
    d.src_stride = st.stride;
    d.src_w = im.src_w;
    d.src_h = st.rows;
    d.src_x0 = st.x0;
    d.src_y0 = st.y0;
    d.dst = im.dst;
    d.dst_stride = im.dst_stride;
    d.xwidth = p.xt->padded;
    d.ywidth = p.yt->padded;
    d.xtab = p.xt->ptr + (size_t)im.crop_x * (mxd::kTapHeader + p.xt->padded);
    d.ytab = p.yt->ptr + (size_t)im.crop_y * (mxd::kTapHeader + p.yt->padded);
    d.crop_w = im.crop_w;
    d.crop_h = im.crop_h;
    d.flip = im.flip ? 1 : 0;
  };

  // Descriptors of one upload: band-kernel images first, then wave-kernel
  // images, then the general kernel's.
  std::vector<ImgDev> descs(n);

  // Band launches: one per (class, window KiB, lookahead).
  auto bkey = [&](int32_t i) {
    const mxd::BandPlan& b = plans[i].bp;
    return std::make_tuple(b.cls, b.nq, b.la);
  };
  std::vector<int32_t> border;
  for (int32_t i = 0; i < n; i++)
    if (plans[i].band) border.push_back(i);
  std::stable_sort(border.begin(), border.end(), [&](int32_t a, int32_t b) { return bkey(a) < bkey(b); });
  const int32_t nbd = (int32_t)border.size();
  struct BandGroup {
    int32_t first, count, units;
    mxd::BandCfg cfg;
    int32_t table = -1;  // descriptor slot of the unit -> image table (per_img == 0)
  };
  std::vector<BandGroup> bgroups;
  for (int32_t k = 0; k < nbd; k++) {
    const mxd::BandPlan& b = plans[border[k]].bp;
    if (bgroups.empty() || bkey(border[bgroups.back().first]) != bkey(border[k]))
      bgroups.push_back({k, 0, 0, mxd::BandCfg{channels, f32, b.nq, b.taps, b.s, b.db, b.la, 0, 0, 0, 0}});
    bgroups.back().count++;
  }
  for (BandGroup& g : bgroups) {
    g.cfg.nimgs = g.count;
    std::vector<std::pair<int32_t, int32_t>> strips;  // (nstrips, crop_h) per image
    for (int32_t k = g.first; k < g.first + g.count; k++)
      strips.push_back({plans[border[k]].bp.nstrips, images[border[k]].crop_h});
    const int32_t forced = g_tune[MXD_TUNE_BAND_ROWS].load();
    const int32_t capacity = band_capacity_cached(g.cfg, device);
    const int32_t ty = forced > 0 ? forced : band_rows(strips, capacity, kBandMaxRows);
    std::unordered_map<int32_t, const DevSched*> sched_of;  // by rep[] (one geometry, one band height)
    for (int32_t k = g.first; k < g.first + g.count; k++) {
      const int32_t i = border[k];
      const mxd_image& im = images[i];
      const ImgPlan& p = plans[i];
      ImgDev& d = descs[k];
      fill(d, i, p);
      const uintptr_t a = reinterpret_cast<uintptr_t>(d.src);
      d.src = reinterpret_cast<const uint8_t*>(a & ~(uintptr_t)3);
      d.flip |= (int32_t)(a & 3) << 8;
      d.ty = std::min(ty, im.crop_h);
      const DevSched*& sc = sched_of[rep[i]];
      if (!sc)
        if (int rc = band_schedules().get(device, *p.yt, im.src_h, im.resize_h, im.crop_y, im.crop_h, d.ty, p.bp.db,
                                          p.bp.s, p.bp.la + 2, &sc))
          return rc;
      d.ytab = reinterpret_cast<const float*>(sc->ptr);
      d.ywidth = sc->band_words;
      d.group = 0;
      d.tile_begin = g.units;
      d.nstrips = p.bp.nstrips;
      d.tx = p.bp.tx;
      const int32_t u = d.nstrips * ((im.crop_h + d.ty - 1) / d.ty);
      g.cfg.per_img = k == g.first ? u : (g.cfg.per_img == u ? u : 0);
      g.units += u;
    }
    g.cfg.nunits = g.units;
    // A persistent grid: as many workgroups as the device holds at once,
    // each running an equal share of units (measured on C2 / 12 MP / 24 MP:
    // 0.158 / 0.195 / 0.367 ms against 0.17-0.19 / 0.224 / 0.383 with one
    // workgroup per unit); MXD_TUNE_BAND_GRID overrides.
    const int32_t knob = g_tune[MXD_TUNE_BAND_GRID].load();
    int32_t grid = knob == 1 ? g.units : knob > 1 ? knob : (capacity > 0 ? capacity : 1024);
    grid = std::max(1, std::min(g.units, grid));
    g.cfg.grid = (g.units + (g.units + grid - 1) / grid - 1) / ((g.units + grid - 1) / grid);
  }
  // Unit -> image tables of the band launches whose images differ in unit
  // count, after every descriptor (ImgDev-sized blocks of int32).
  std::vector<int32_t> unit_tables;
  for (BandGroup& g : bgroups) {
    if (g.cfg.per_img > 0) continue;
    g.table = (int32_t)unit_tables.size();
    for (int32_t k = g.first; k < g.first + g.count; k++) {
      const ImgDev& d = descs[k];
      const int32_t u = d.nstrips * ((images[border[k]].crop_h + d.ty - 1) / d.ty);
      unit_tables.insert(unit_tables.end(), u, k - g.first);
    }
    unit_tables.resize((unit_tables.size() * 4 + sizeof(ImgDev) - 1) / sizeof(ImgDev) * sizeof(ImgDev) / 4, 0);
  }

  // Wave launches: one per kernel (kind, tap bucket, scatter shape, q,
  // shift).
  auto key = [&](int32_t i) {
    const ImgPlan& p = plans[i];
    return std::make_tuple(p.kind, p.bucket, p.s, p.dmax, p.q, p.shift, p.pp);
  };
  std::vector<int32_t> order;
  for (int32_t i = 0; i < n; i++)
    if (plans[i].wave) order.push_back(i);
  std::stable_sort(order.begin(), order.end(), [&](int32_t a, int32_t b) { return key(a) < key(b); });
  const int32_t nw = (int32_t)order.size();
  const int32_t wbase = nbd;  // first wave descriptor
  struct Group {
    int32_t first, count, units, ty;
    mxd::WaveCfg cfg;
  };
  std::vector<Group> groups;
  for (int32_t k = 0; k < nw; k++) {
    const ImgPlan& p = plans[order[k]];
    if (groups.empty() || key(order[groups.back().first]) != key(order[k]))
      groups.push_back(
          {k, 0, 0, 0, mxd::WaveCfg{channels, f32, p.bucket, 0, 0, p.kind, p.s, p.dmax, p.q, p.shift, p.pp}});
    groups.back().count++;
  }
  for (Group& g : groups) {
    g.cfg.nimgs = g.count;
    std::vector<std::pair<int32_t, int32_t>> strips;  // (nstrips, crop_h) per image
    for (int32_t k = g.first; k < g.first + g.count; k++) strips.push_back({plans[order[k]].nstrips, images[order[k]].crop_h});
    g.ty = band_rows(strips, wave_capacity_cached(g.cfg, device));
    std::unordered_map<int32_t, const DevSched*> sched_of;  // by rep[]
    for (int32_t k = g.first; k < g.first + g.count; k++) {
      const int32_t i = order[k];
      const mxd_image& im = images[i];
      const ImgPlan& p = plans[i];
      ImgDev& d = descs[wbase + k];
      fill(d, i, p);
      // aligned base + byte shift (ImgDev::flip bits 8..)
      const uintptr_t a = reinterpret_cast<uintptr_t>(d.src);
      d.src = reinterpret_cast<const uint8_t*>(a & ~(uintptr_t)3);
      d.flip |= (int32_t)(a & 3) << 8;
      d.ty = std::min(g.ty, im.crop_h);
      if (p.kind == 2) {
        const DevSched*& sc = sched_of[rep[i]];
        if (!sc)
          if (int rc = schedules().get(device, *p.yt, im.src_h, im.resize_h, im.crop_y, im.crop_h, d.ty,
                                       ScatterShape{p.s, p.dmax, p.p}, &sc))
            return rc;
        d.ytab = reinterpret_cast<const float*>(sc->ptr);
        d.ywidth = sc->band_words;
        d.group = sc->entry_off;
      } else {
        d.group = 1;
      }
      d.tile_begin = g.units;
      d.nstrips = p.nstrips;
      d.tx = p.tx;
      const int32_t u = d.nstrips * ((im.crop_h + d.ty - 1) / d.ty);
      g.cfg.per_img = k == g.first ? u : (g.cfg.per_img == u ? u : 0);
      g.units += u;
    }
    g.cfg.nunits = g.units;
  }

  // General path (any alignment, any tap count): workgroup tiles, resample.hip.
  LaunchCfg cfg{};
  int32_t tiles = 0;
  if (!slow.empty()) {
    // The tile kernel addresses rows from the image's row 0: a staged
    // footprint is reached through the (never dereferenced) address its
    // row 0 would have; the kernel only reads footprint rows and columns.
    auto base0 = [&](int32_t i) {
      const Stored st = stored ? stored[i] : whole(images[i]);
      return st.base - (int64_t)st.y0 * st.stride - (int64_t)st.x0 * images[i].channels;
    };
    bool aligned16 = true;
    for (int32_t i : slow) {
      const Stored st = stored ? stored[i] : whole(images[i]);
      const uintptr_t a = reinterpret_cast<uintptr_t>(base0(i)) | (uintptr_t)st.stride;
      aligned16 = aligned16 && (a & 15) == 0;
    }
    const int32_t vec = aligned16 ? 16 : 1;
    cfg.vec = vec;
    cfg.channels = channels;
    cfg.alpha = channels == 4 && images[slow[0]].rgba_weighted ? 1 : 0;
    cfg.f32 = f32;
    cfg.nimgs = (int32_t)slow.size();
    for (size_t k = 0; k < slow.size(); k++) {
      const int32_t i = slow[k];
      const mxd_image& im = images[i];
      const DevTable* xt = plans[i].xt;
      const DevTable* yt = plans[i].yt;
      const bool flip = im.flip != 0;
      // Column strips: enough that one strip row's footprint is ~kStripBytes.
      const int32_t full = strip_chunks(*xt, im.crop_x, im.crop_w, 0, im.crop_w, flip, channels, 1);
      int32_t nstrips = std::max<int32_t>(1, (full + kStripBytes - 1) / kStripBytes);
      int32_t tx = (im.crop_w + nstrips - 1) / nstrips;
      tx = std::min<int32_t>(im.crop_w, (tx + 3) & ~3);
      nstrips = (im.crop_w + tx - 1) / tx;
      int32_t max_chunks = 0;
      for (int32_t s = 0; s < nstrips; s++) {
        const int32_t ox0 = s * tx, ox1 = std::min(ox0 + tx, im.crop_w);
        max_chunks = std::max(max_chunks, strip_chunks(*xt, im.crop_x, im.crop_w, ox0, ox1, flip, channels, vec));
      }
      const int32_t vw = (max_chunks * vec + 3) & ~3;
      const int32_t ty = std::min(kTileRows, im.crop_h);
      int32_t group = std::max<int32_t>(1, std::min<int32_t>(8, 512 / std::max(1, max_chunks)));
      group = std::max<int32_t>(1, std::min<int32_t>(group, kLdsBudget / (vw * 4)));
      group = std::min(group, ty);
      const int32_t nbands = (im.crop_h + ty - 1) / ty;
      ImgDev& d = descs[wbase + nw + k];
      fill(d, i, plans[i]);
      d.src = base0(i);
      d.src_h = im.src_h;
      d.src_x0 = d.src_y0 = 0;
      d.tile_begin = tiles;
      d.nstrips = nstrips;
      d.ty = ty;
      d.tx = tx;
      d.group = group;
      tiles += nbands * nstrips;
      cfg.max_tx = std::max(cfg.max_tx, tx);
      cfg.max_ty = std::max(cfg.max_ty, ty);
      cfg.max_xw = std::max(cfg.max_xw, xt->padded);
      cfg.max_yw = std::max(cfg.max_yw, yt->padded);
      cfg.max_vw = std::max(cfg.max_vw, vw);
      cfg.max_group = std::max(cfg.max_group, group);
    }
    cfg.ntiles = tiles;
    if (mxd::resample_smem_bytes(cfg) > 160 * 1024) return fail(MXD_ERR_UNSUPPORTED, "mxd: tile does not fit in LDS");
  }

  ImgDev* dev = nullptr;
  std::unique_lock<std::mutex> hold;
  Workspace* ws = nullptr;
  bool hit = false;
  if (!unit_tables.empty()) {
    const size_t at = descs.size();
    descs.resize(at + unit_tables.size() * 4 / sizeof(ImgDev));
    std::memcpy(reinterpret_cast<void*>(descs.data() + at), unit_tables.data(), unit_tables.size() * 4);
  }
  if (int rc = upload_descs(descs, device, stream, &dev, &hold, &ws, &hit)) return rc;
  const int32_t* tables_dev = reinterpret_cast<const int32_t*>(dev + n);
  // Several launches: fork them over the caller's stream and the workspace's
  // helper streams (largest first), join back before return, so one launch's
  // tail overlaps the next.
  struct Launch {
    int64_t units;
    int32_t kind;   // 0 band, 1 wave, 2 general
    int32_t group;
  };
  std::vector<Launch> launches;
  // (a band unit is a workgroup, ~4 wave units)
  for (size_t g = 0; g < bgroups.size(); g++) launches.push_back({4 * (int64_t)bgroups[g].units, 0, (int32_t)g});
  for (size_t g = 0; g < groups.size(); g++) launches.push_back({groups[g].units, 1, (int32_t)g});
  if (!slow.empty()) launches.push_back({tiles, 2, -1});
  std::stable_sort(launches.begin(), launches.end(), [](const Launch& a, const Launch& b) { return a.units > b.units; });
  const int nfork = std::min<int>((int)launches.size() - 1, Workspace::kHelpers);
  if (nfork > 0) {
    if (!ws->fork) {
      MXD_HIP(hipEventCreateWithFlags(&ws->fork, hipEventDisableTiming));
      for (int h = 0; h < Workspace::kHelpers; h++) {
        MXD_HIP(hipStreamCreateWithFlags(&ws->helper[h], hipStreamNonBlocking));
        MXD_HIP(hipEventCreateWithFlags(&ws->join[h], hipEventDisableTiming));
      }
    }
    MXD_HIP(hipEventRecord(ws->fork, reinterpret_cast<hipStream_t>(stream)));
    for (int h = 0; h < nfork; h++) MXD_HIP(hipStreamWaitEvent(ws->helper[h], ws->fork, 0));
  }
  for (size_t k = 0; k < launches.size(); k++) {
    const int lane = nfork > 0 ? (int)(k % (size_t)(nfork + 1)) : 0;
    void* s = lane == 0 ? stream : reinterpret_cast<void*>(ws->helper[lane - 1]);
    int rc = 0;
    if (launches[k].kind == 0) {
      const BandGroup& g = bgroups[launches[k].group];
      rc = mxd::launch_band(g.cfg, dev + g.first, g.table >= 0 ? tables_dev + g.table : nullptr, s);
    } else if (launches[k].kind == 1) {
      const Group& g = groups[launches[k].group];
      rc = mxd::launch_wave(g.cfg, dev + wbase + g.first, s);
    } else {
      rc = mxd::launch_resample(cfg, dev + wbase + nw, s);
    }
    if (rc)
      return fail(MXD_ERR_DEVICE, std::string("resample launch failed: ") + hipGetErrorString(hipGetLastError()) +
                                      " rc=" + std::to_string(rc));
  }
  for (int h = 0; h < nfork; h++) {
    MXD_HIP(hipEventRecord(ws->join[h], ws->helper[h]));
    MXD_HIP(hipStreamWaitEvent(reinterpret_cast<hipStream_t>(stream), ws->join[h], 0));
  }
  return hit ? MXD_OK : release_descs(ws, stream);
}

// ---------------------------------------------------------------------------
// Pixel maps (rotate / channel reduction): validation with the reference's
// messages, host-side derivation of the per-image constants, descriptor upload
// through a per-(device, stream) pinned/device pair guarded like Workspace.
struct PixWorkspace {
  std::mutex mu;
  mxd::PixDev* host = nullptr;
  mxd::PixDev* dev = nullptr;
  size_t cap = 0;
  hipEvent_t copied = nullptr;
};

PixWorkspace* pix_workspace(int32_t device, void* stream) {
  static std::mutex mu;
  static auto* map = new std::map<std::pair<int32_t, void*>, std::unique_ptr<PixWorkspace>>();
  std::lock_guard<std::mutex> lk(mu);
  auto& w = (*map)[std::make_pair(device, stream)];
  if (!w) w = std::make_unique<PixWorkspace>();
  return w.get();
}

int pix_validate(const mxd_pixmap& im, int32_t op, int32_t i) {
  const std::string at = " (image " + std::to_string(i) + ")";
  if (!im.src || !im.dst) return fail(MXD_ERR_INVALID, "mxd: null src/dst pointer" + at);
  if (op != MXD_AFFINE && op != MXD_CHANNEL_REDUCTION) return fail(MXD_ERR_INVALID, "mxd: unknown pixmap op" + at);
  if (im.src_w <= 0 || im.src_h <= 0 || im.dst_w <= 0 || im.dst_h <= 0)
    return fail(MXD_ERR_INVALID, "image: cannot create image with 0 or negative dimension" + at);
  if (im.channels <= 0 || im.channels > 4)
    return fail(MXD_ERR_INVALID, "image: channels must be 0 < c <= 4" + at);
  if (op == MXD_CHANNEL_REDUCTION) {
    if (im.channels != 3)
      return fail(MXD_ERR_INVALID, "image::channelReduction: expected a 3 channel uint8 array" + at);
    if (im.dst_w != im.src_w || im.dst_h != im.src_h)
      return fail(MXD_ERR_INVALID, "mxd: channel reduction keeps the image size" + at);
  }
  if (im.src_stride < (int64_t)im.src_w * im.channels)
    return fail(MXD_ERR_INVALID, "mxd: src_stride smaller than a row" + at);
  if ((int64_t)im.dst_w * im.dst_h >= ((int64_t)1 << 31))
    return fail(MXD_ERR_UNSUPPORTED, "mxd: pixel map output of 2^31 pixels or more" + at);
  const int64_t out_row = (int64_t)im.dst_w * (op == MXD_AFFINE ? im.channels : 1);
  if (im.dst_stride < out_row) return fail(MXD_ERR_INVALID, "mxd: dst_stride smaller than a row" + at);
  return MXD_OK;
}

mxd::PixDev pix_desc(const mxd_pixmap& im, int32_t op) {
  mxd::PixDev d{};
  d.src = im.src;
  d.dst = static_cast<uint8_t*>(im.dst);
  d.src_stride = im.src_stride;
  d.dst_stride = im.dst_stride;
  d.src_w = im.src_w;
  d.src_h = im.src_h;
  d.dst_w = im.dst_w;
  d.dst_h = im.dst_h;
  d.c = im.channels;
  // affine: 4-pixel groups, dword stores; reduction: 16-pixel groups, 16-B
  // loads and stores (pixmap.hip)
  const int gp = op == MXD_AFFINE ? 4 : 16;
  d.groups = (im.dst_w + gp - 1) / gp;
  const uintptr_t am = op == MXD_AFFINE ? 3 : 15;  // dword stores / 16-byte loads and stores
  const bool dst_al = ((uintptr_t)im.dst & am) == 0 && ((uintptr_t)im.dst_stride & am) == 0;
  const bool src_al = ((uintptr_t)im.src & am) == 0 && ((uintptr_t)im.src_stride & am) == 0;
  d.fast = op == MXD_AFFINE ? dst_al : (dst_al && src_al);
  if (op == MXD_AFFINE) {
    // core/image/ImageTransform.cpp:88-91 (double halves narrowed to float)
    for (int k = 0; k < 6; k++) d.mx[k] = im.params[k];
    d.twh = (float)(im.dst_w / 2.0);
    d.thh = (float)(im.dst_h / 2.0);
    d.wh = (float)(im.src_w / 2.0);
    d.hh = (float)(im.src_h / 2.0);
  } else {
    // core/image/ImageTransform.cpp:158-163: float * 65536 truncated to int
    const int scale = 256 * 256;
    d.bias = (int)(im.params[0] * scale);
    for (int k = 0; k < 3; k++) d.m[k] = (int)(im.params[1 + k] * scale);
  }
  return d;
}

int run_pixmap(const mxd_pixmap* images, int32_t n, int32_t op, int32_t device, void* stream) {
  if (n < 0 || (n > 0 && !images)) return fail(MXD_ERR_INVALID, "mxd: bad image array");
  if (n == 0) return MXD_OK;
  for (int32_t i = 0; i < n; i++)
    if (int rc = pix_validate(images[i], op, i)) return rc;
  DeviceGuard g(device);
  PixWorkspace* ws = pix_workspace(device, stream);
  std::lock_guard<std::mutex> lk(ws->mu);
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  if (ws->copied) MXD_HIP(hipEventSynchronize(ws->copied));  // staging free again
  if ((size_t)n > ws->cap) {
    if (ws->dev) {
      MXD_HIP(hipStreamSynchronize(s));
      MXD_HIP(hipFree(ws->dev));
      MXD_HIP(hipHostFree(ws->host));
      ws->dev = nullptr;
      ws->host = nullptr;
    }
    const size_t cap = std::max<size_t>(n, 64);
    MXD_HIP(hipMalloc(reinterpret_cast<void**>(&ws->dev), sizeof(mxd::PixDev) * cap));
    MXD_HIP(hipHostMalloc(reinterpret_cast<void**>(&ws->host), sizeof(mxd::PixDev) * cap, hipHostMallocDefault));
    ws->cap = cap;
  }
  if (!ws->copied) MXD_HIP(hipEventCreateWithFlags(&ws->copied, hipEventDisableTiming));
  int64_t max_units = 0;
  for (int32_t i = 0; i < n; i++) {
    ws->host[i] = pix_desc(images[i], op);
    const int64_t u = op == MXD_AFFINE ? (int64_t)ws->host[i].dst_h * ws->host[i].dst_w
                                       : (int64_t)ws->host[i].dst_h * ws->host[i].groups;
    max_units = std::max(max_units, u);
  }
  MXD_HIP(hipMemcpyAsync(ws->dev, ws->host, sizeof(mxd::PixDev) * n, hipMemcpyHostToDevice, s));
  MXD_HIP(hipEventRecord(ws->copied, s));
  if (mxd::launch_pixmap(op, ws->dev, n, max_units, stream))
    return fail(MXD_ERR_DEVICE, std::string("pixmap launch: ") + hipGetErrorString(hipGetLastError()));
  return MXD_OK;
}

// ---------------------------------------------------------------------------
// Host-resident path.  Each call borrows a context from its device's pool
// (at most kCtxPerDevice, so pinned / device memory is bounded no matter how
// many threads call), and runs the batch in chunks over the context's two
// slots: while the GPU copies in, computes and copies out chunk k on one
// slot's stream, the calling thread stages chunk k+1 into the other slot's
// pinned buffer and copies chunk k-1's results out.
struct Slot {
  hipStream_t stream = nullptr;
  hipEvent_t done = nullptr;
  uint8_t* pin_in = nullptr;
  size_t pin_in_cap = 0;
  uint8_t* pin_out = nullptr;
  size_t pin_out_cap = 0;
  uint8_t* dev_in = nullptr;
  size_t dev_in_cap = 0;
  uint8_t* dev_out = nullptr;
  size_t dev_out_cap = 0;
  uint8_t* dev_mid = nullptr;  // JPEG chunks: IDCT samples + decoded RGB images
  size_t dev_mid_cap = 0;
};

struct HostCtx {
  Slot slot[2];
};

int grow_pinned(uint8_t** p, size_t* cap, size_t need) {
  if (need <= *cap) return MXD_OK;
  if (*p) MXD_HIP(hipHostFree(*p));
  *p = nullptr;
  *cap = 0;
  const size_t c = (need + (1 << 20) - 1) & ~(size_t)((1 << 20) - 1);
  MXD_HIP(hipHostMalloc(reinterpret_cast<void**>(p), c, hipHostMallocDefault));
  *cap = c;
  return MXD_OK;
}

int grow_device(uint8_t** p, size_t* cap, size_t need) {
  if (need <= *cap) return MXD_OK;
  if (*p) MXD_HIP(hipFree(*p));
  *p = nullptr;
  *cap = 0;
  const size_t c = (need + (1 << 20) - 1) & ~(size_t)((1 << 20) - 1);
  MXD_HIP(hipMalloc(reinterpret_cast<void**>(p), c));
  *cap = c;
  return MXD_OK;
}

void free_slot_buffers(Slot& s) {
  if (s.pin_in) (void)hipHostFree(s.pin_in);
  if (s.pin_out) (void)hipHostFree(s.pin_out);
  if (s.dev_in) (void)hipFree(s.dev_in);
  if (s.dev_out) (void)hipFree(s.dev_out);
  if (s.dev_mid) (void)hipFree(s.dev_mid);
  s.pin_in = s.pin_out = s.dev_in = s.dev_out = s.dev_mid = nullptr;
  s.pin_in_cap = s.pin_out_cap = s.dev_in_cap = s.dev_out_cap = s.dev_mid_cap = 0;
}

constexpr int kCtxPerDevice = 4;

// Host-side byte moves of the host path (footprint staging into pinned
// memory, copy-out of results) are bound by one core's memory bandwidth;
// they are split over helper threads, fewer when several host-path calls run
// at once (prefetch workers already spread the work).
std::atomic<int> g_host_calls{0};

template <class F>
void parallel_items(int32_t first, int32_t end, int64_t bytes, F&& f) {
  const int32_t n = end - first;
  static const int hw = [] {  // the cores this process may run on (a container's share, not the machine)
    cpu_set_t set;
    CPU_ZERO(&set);
    if (sched_getaffinity(0, sizeof set, &set) == 0) return std::max(1, CPU_COUNT(&set));
    return std::max(1, (int)std::thread::hardware_concurrency());
  }();
  int t = std::min<int64_t>({8, hw / std::max(1, g_host_calls.load()), n, bytes >> 20});
  if (t <= 1) {
    for (int32_t i = first; i < end; i++) f(i);
    return;
  }
  std::atomic<int32_t> next{first};
  auto work = [&] {
    for (int32_t i; (i = next.fetch_add(1)) < end;) f(i);
  };
  std::vector<std::thread> ts;
  for (int k = 1; k < t; k++) ts.emplace_back(work);
  work();
  for (auto& th : ts) th.join();
}

class HostPool {
 public:
  HostCtx* acquire(int32_t device) {
    std::unique_lock<std::mutex> lk(mu_);
    Dev& d = devs_[device];
    cv_.wait(lk, [&] { return !d.idle.empty() || (int)d.all.size() < kCtxPerDevice; });
    if (!d.idle.empty()) {
      HostCtx* c = d.idle.back();
      d.idle.pop_back();
      return c;
    }
    d.all.push_back(std::make_unique<HostCtx>());
    return d.all.back().get();
  }
  void release(int32_t device, HostCtx* c) {
    {
      std::lock_guard<std::mutex> lk(mu_);
      devs_[device].idle.push_back(c);
    }
    cv_.notify_one();
  }
  // Frees the buffers of every idle context (streams stay).
  void trim() {
    std::lock_guard<std::mutex> lk(mu_);
    for (auto& kv : devs_) {
      DeviceGuard g(kv.first);
      for (HostCtx* c : kv.second.idle)
        for (Slot& s : c->slot) free_slot_buffers(s);
    }
  }

 private:
  struct Dev {
    std::vector<std::unique_ptr<HostCtx>> all;
    std::vector<HostCtx*> idle;
  };
  std::mutex mu_;
  std::condition_variable cv_;
  std::map<int32_t, Dev> devs_;
};

HostPool& host_pool() {
  static HostPool* p = new HostPool();
  return *p;
}

// Borrowed context, returned to the pool on scope exit.
struct CtxLease {
  int32_t device;
  HostCtx* ctx;
  explicit CtxLease(int32_t d) : device(d), ctx(host_pool().acquire(d)) {}
  ~CtxLease() { host_pool().release(device, ctx); }
};

int init_slot(Slot& s) {
  if (!s.stream) MXD_HIP(hipStreamCreateWithFlags(&s.stream, hipStreamNonBlocking));
  if (!s.done) MXD_HIP(hipEventCreateWithFlags(&s.done, hipEventDisableTiming));
  return MXD_OK;
}

// Source footprint of an image's crop window (rows [y_lo, y_hi], pixels
// [x_lo, x_hi]): taps are monotone, so the window's ends bound it.
void footprint(const DevTable& xt, const DevTable& yt, const mxd_image& im, int32_t* x_lo, int32_t* x_hi,
               int32_t* y_lo, int32_t* y_hi) {
  const int32_t xa = im.crop_x, xb = im.crop_x + im.crop_w - 1;
  const int32_t ya = im.crop_y, yb = im.crop_y + im.crop_h - 1;
  *x_lo = xt.first[xa];
  *x_hi = xt.first[xb] + xt.count[xb] - 1;
  *y_lo = yt.first[ya];
  *y_hi = yt.first[yb] + yt.count[yb] - 1;
}

}  // namespace

extern "C" {

int mxd_abi_version(void) { return MXD_ABI_VERSION; }

const char* mxd_last_error(void) { return g_error.c_str(); }


int mxd_device_properties(int32_t device, char* name, size_t name_len, char* arch, size_t arch_len, int32_t* cus) {
  if (int rc = check_device(device)) return rc;
  hipDeviceProp_t p{};
  MXD_HIP(hipGetDeviceProperties(&p, device));
  auto put = [](char* dst, size_t n, const char* src) {
    if (!dst || n == 0) return;
    std::strncpy(dst, src, n - 1);
    dst[n - 1] = 0;
  };
  put(name, name_len, p.name);
  put(arch, arch_len, p.gcnArchName);
  if (cus) *cus = p.multiProcessorCount;
  return MXD_OK;
}

int mxd_device_count(int* count) {
  if (!count) return fail(MXD_ERR_INVALID, "mxd: null count");
  MXD_HIP(hipGetDeviceCount(count));
  return MXD_OK;
}

int mxd_resize_smallest_side_dims(int64_t w, int64_t h, int64_t size, int64_t* out_w, int64_t* out_h) {
  if (!out_w || !out_h) return fail(MXD_ERR_INVALID, "mxd: null output");
  if (size <= 0)
    return fail(MXD_ERR_INVALID, "ImageResizeSmallestSide: illegal target size: " + std::to_string(size));
  if (w <= 0 || h <= 0) return fail(MXD_ERR_INVALID, "image: cannot create image with 0 or negative dimension");
  mxd::smallest_side_dims(w, h, size, out_w, out_h);
  return MXD_OK;
}

int mxd_center_crop_origin(int64_t w, int64_t h, int64_t cw, int64_t ch, int64_t* x, int64_t* y) {
  if (!x || !y) return fail(MXD_ERR_INVALID, "mxd: null output");
  if (ch > h || cw > w) return fail(MXD_ERR_INVALID, "ImageCenterCrop: target image size larger than input image");
  *x = (w - cw) / 2;
  *y = (h - ch) / 2;
  return MXD_OK;
}

int mxd_axis_taps(int32_t in_size, int32_t out_size, int32_t crop_off, int32_t crop_len, int32_t max_taps,
                  int32_t* first, int32_t* ntaps, float* weights, int32_t* taps_needed) {
  mxd::AxisTaps t;
  if (!mxd::build_axis_taps(in_size, out_size, crop_off, crop_len, &t))
    return fail(MXD_ERR_INVALID, "mxd: invalid axis geometry");
  if (taps_needed) *taps_needed = t.width;
  if (t.width > max_taps) return fail(MXD_ERR_INVALID, "mxd: max_taps too small");
  if (!first || !ntaps || !weights) return fail(MXD_ERR_INVALID, "mxd: null output");
  for (int32_t i = 0; i < crop_len; i++) {
    first[i] = t.first[i];
    ntaps[i] = t.count[i];
    for (int32_t k = 0; k < max_taps; k++)
      weights[(size_t)i * max_taps + k] = k < t.width ? t.weight[(size_t)i * t.width + k] : 0.0f;
  }
  return MXD_OK;
}

int mxd_resize_crop_batch(const mxd_image* images, int32_t n, int32_t out_dtype, int32_t device, void* stream) {
  return run_batch(images, n, out_dtype, device, stream);
}

int mxd_set_kernel_policy(int32_t policy) { return g_policy.exchange(policy); }

int mxd_set_tuning(int32_t knob, int32_t value) {
  if (knob < 0 || knob >= MXD_TUNE_COUNT) return -1;
  return g_tune[knob].exchange(value);
}

int mxd_describe_band_plan(const mxd_image* image, int32_t out_dtype, int32_t* info12) {
  if (!image || !info12) return fail(MXD_ERR_INVALID, "mxd: null argument");
  if (int rc = validate(*image, 0)) return rc;
  ImgPlan p;
  if (int rc = host_tables().get(0, image->src_w, image->resize_w, &p.xt)) return rc;
  if (int rc = host_tables().get(0, image->src_h, image->resize_h, &p.yt)) return rc;
  const int32_t f32 = out_dtype == MXD_F32_DIV255 ? 1 : 0;
  plan_band(*image, whole(*image), f32, p);
  const mxd::BandPlan& b = p.bp;
  mxd::BandCfg cfg{};
  cfg.nq = b.nq;
  cfg.db = b.db;
  cfg.la = b.la;
  const int32_t v[12] = {p.band ? 1 : 0, b.taps, b.db, b.s, b.nq, b.nstrips, b.tx, b.prologue, b.dmax, b.la,
                         b.ok ? mxd::band_lds_bytes(cfg) : 0, 0};
  std::memcpy(info12, v, sizeof v);
  return MXD_OK;
}

int mxd_describe_plan(const mxd_image* image, int32_t out_dtype, int32_t device, int32_t* info8) {
  if (!image || !info8) return fail(MXD_ERR_INVALID, "mxd: null argument");
  if (int rc = validate(*image, 0)) return rc;
  ImgPlan p;
  if (int rc = host_tables().get(device, image->src_w, image->resize_w, &p.xt)) return rc;
  if (int rc = host_tables().get(device, image->src_h, image->resize_h, &p.yt)) return rc;
  if (!(g_policy.load() & MXD_POLICY_NO_WAVE)) plan_wave(*image, whole(*image), out_dtype == MXD_F32_DIV255, out_dtype, p);
  const int32_t v[8] = {p.wave ? 1 : 0, p.kind, p.bucket, p.s, p.dmax, p.q, p.nstrips, p.pp};
  std::memcpy(info8, v, sizeof v);
  return MXD_OK;
}

int mxd_copy_bandwidth(size_t bytes, int32_t device, int32_t iters, float* gbps) {
  if (!gbps || bytes < 16 || iters <= 0) return fail(MXD_ERR_INVALID, "mxd: bad copy_bandwidth arguments");
  if (int rc = check_device(device)) return rc;
  DeviceGuard g(device);
  void *a = nullptr, *b = nullptr;
  hipStream_t s = nullptr;
  hipEvent_t e0 = nullptr, e1 = nullptr;
  MXD_HIP(hipMalloc(&a, bytes));
  MXD_HIP(hipMalloc(&b, bytes));
  MXD_HIP(hipMemset(a, 1, bytes));
  MXD_HIP(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  MXD_HIP(hipEventCreate(&e0));
  MXD_HIP(hipEventCreate(&e1));
  mxd::launch_copy(a, b, bytes, s);
  MXD_HIP(hipEventRecord(e0, s));
  for (int32_t i = 0; i < iters; i++) mxd::launch_copy(a, b, bytes, s);
  MXD_HIP(hipEventRecord(e1, s));
  MXD_HIP(hipEventSynchronize(e1));
  float ms = 0.0f;
  MXD_HIP(hipEventElapsedTime(&ms, e0, e1));
  *gbps = (float)(2.0 * (double)(bytes / 16 * 16) * iters / (ms * 1e-3) / 1e9);
  (void)hipEventDestroy(e0);
  (void)hipEventDestroy(e1);
  (void)hipStreamDestroy(s);
  (void)hipFree(a);
  (void)hipFree(b);
  return MXD_OK;
}

int mxd_set_device(int32_t device) {
  if (int rc = check_device(device)) return rc;
  MXD_HIP(hipSetDevice(device));
  return MXD_OK;
}

int mxd_malloc_device(void** ptr, size_t bytes, int32_t device) {
  if (int rc = check_device(device)) return rc;
  if (!ptr) return fail(MXD_ERR_INVALID, "mxd: null ptr");
  DeviceGuard g(device);
  MXD_HIP(hipMalloc(ptr, bytes));
  return MXD_OK;
}

int mxd_free_device(void* ptr, int32_t device) {
  if (int rc = check_device(device)) return rc;
  DeviceGuard g(device);
  MXD_HIP(hipFree(ptr));
  return MXD_OK;
}

int mxd_malloc_pinned(void** ptr, size_t bytes) {
  if (!ptr) return fail(MXD_ERR_INVALID, "mxd: null ptr");
  MXD_HIP(hipHostMalloc(ptr, bytes, hipHostMallocDefault));
  return MXD_OK;
}

int mxd_free_pinned(void* ptr) {
  MXD_HIP(hipHostFree(ptr));
  return MXD_OK;
}

int mxd_memcpy_h2d_async(void* dst, const void* src, size_t bytes, void* stream) {
  MXD_HIP(hipMemcpyAsync(dst, src, bytes, hipMemcpyHostToDevice, reinterpret_cast<hipStream_t>(stream)));
  return MXD_OK;
}

int mxd_memcpy_d2h_async(void* dst, const void* src, size_t bytes, void* stream) {
  MXD_HIP(hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToHost, reinterpret_cast<hipStream_t>(stream)));
  return MXD_OK;
}

int mxd_memcpy2d_h2d_async(void* dst, size_t dpitch, const void* src, size_t spitch, size_t width, size_t rows,
                           void* stream) {
  MXD_HIP(hipMemcpy2DAsync(dst, dpitch, src, spitch, width, rows, hipMemcpyHostToDevice,
                           reinterpret_cast<hipStream_t>(stream)));
  return MXD_OK;
}

int mxd_memset_async(void* dst, int value, size_t bytes, void* stream) {
  MXD_HIP(hipMemsetAsync(dst, value, bytes, reinterpret_cast<hipStream_t>(stream)));
  return MXD_OK;
}

int mxd_stream_create(int32_t device, void** stream) {
  if (int rc = check_device(device)) return rc;
  if (!stream) return fail(MXD_ERR_INVALID, "mxd: null stream");
  DeviceGuard g(device);
  hipStream_t s = nullptr;
  MXD_HIP(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  *stream = s;
  return MXD_OK;
}

int mxd_stream_destroy(void* stream) {
  MXD_HIP(hipStreamDestroy(reinterpret_cast<hipStream_t>(stream)));
  return MXD_OK;
}

int mxd_stream_synchronize(void* stream) {
  MXD_HIP(hipStreamSynchronize(reinterpret_cast<hipStream_t>(stream)));
  return MXD_OK;
}

int mxd_event_create(void** event) {
  if (!event) return fail(MXD_ERR_INVALID, "mxd: null event");
  hipEvent_t e = nullptr;
  MXD_HIP(hipEventCreate(&e));
  *event = e;
  return MXD_OK;
}

int mxd_event_destroy(void* event) {
  MXD_HIP(hipEventDestroy(reinterpret_cast<hipEvent_t>(event)));
  return MXD_OK;
}

int mxd_event_record(void* event, void* stream) {
  MXD_HIP(hipEventRecord(reinterpret_cast<hipEvent_t>(event), reinterpret_cast<hipStream_t>(stream)));
  return MXD_OK;
}

int mxd_event_synchronize(void* event) {
  MXD_HIP(hipEventSynchronize(reinterpret_cast<hipEvent_t>(event)));
  return MXD_OK;
}

int mxd_event_elapsed_ms(float* ms, void* start, void* stop) {
  if (!ms) return fail(MXD_ERR_INVALID, "mxd: null ms");
  MXD_HIP(hipEventElapsedTime(ms, reinterpret_cast<hipEvent_t>(start), reinterpret_cast<hipEvent_t>(stop)));
  return MXD_OK;
}

namespace {
int host_path(const mxd_image* images, int32_t n, int32_t out_dtype, int32_t device, bool dst_device,
              const mxd_jpeg_image* jpeg = nullptr);
}  // namespace

int mxd_resize_crop_host(const mxd_image* images, int32_t n, int32_t out_dtype, int32_t device) {
  return host_path(images, n, out_dtype, device, false);
}

int mxd_resize_crop_to_device(const mxd_image* images, int32_t n, int32_t out_dtype, int32_t device) {
  return host_path(images, n, out_dtype, device, true);
}

int mxd_memcpy_h2d(void* dst, const void* src, size_t bytes, int32_t device) {
  if (!dst || !src) return fail(MXD_ERR_INVALID, "mxd: null pointer");
  if (int rc = check_device(device)) return rc;
  DeviceGuard g(device);
  MXD_HIP(hipMemcpy(dst, src, bytes, hipMemcpyHostToDevice));
  return MXD_OK;
}

int mxd_memcpy_d2h(void* dst, const void* src, size_t bytes, int32_t device) {
  if (!dst || !src) return fail(MXD_ERR_INVALID, "mxd: null pointer");
  if (int rc = check_device(device)) return rc;
  DeviceGuard g(device);
  MXD_HIP(hipMemcpy(dst, src, bytes, hipMemcpyDeviceToHost));
  return MXD_OK;
}

namespace {
// The host path: host sources (footprints staged through pinned memory),
// results to host (dst_device false: D2H + copy-out) or straight into device
// destinations (dst_device true).
// Page-locked host memory of this HIP runtime (hipHostMalloc'd or
// registered): the DMA engines can read / write it in place.
bool host_pinned(const void* p) {
  hipPointerAttribute_t a{};
  if (hipPointerGetAttributes(&a, p) != hipSuccess) {
    (void)hipGetLastError();  // pageable memory is not an error here
    return false;
  }
  return a.type == hipMemoryTypeHost;
}

// The device-side address of page-locked host memory (kernels read it over
// PCIe), or null when the runtime gives none.
const uint8_t* host_device_ptr(const void* p) {
  hipPointerAttribute_t a{};
  if (hipPointerGetAttributes(&a, p) != hipSuccess || a.type != hipMemoryTypeHost || !a.devicePointer) {
    (void)hipGetLastError();
    return nullptr;
  }
  return static_cast<const uint8_t*>(a.devicePointer);
}

// Chunk tables of a JPEG chunk (device-side finish, jpegdev.h): where the
// coefficients, descriptors and quantisation tables sit in the staged input,
// and the decoded images in the slot's dev_mid buffer.
struct JpegChunk {
  std::vector<mxd::JpegPlaneDev> planes;
  std::vector<mxd::JpegImgDev> imgs;
  std::vector<uint16_t> qtabs;
  int64_t planes_off = 0, imgs_off = 0, q_off = 0, end = 0;  // in the staged input
  int64_t samples = 0, rgb_off = 0, mid_bytes = 0;             // in dev_mid
  int64_t nblocks = 0, max_quad_rows = 0;
};

const mxd::jpeg::Coefs* coefs_of(const mxd_jpeg_coefs* c) { return reinterpret_cast<const mxd::jpeg::Coefs*>(c); }

int64_t rgb_pitch(int32_t w) { return (((int64_t)w * 3 + 63) & ~(int64_t)63) + 64; }

// Lays out the chunk [first, end) of a JPEG batch whose coefficients are staged
// at in_off[i]; the tables follow at `tables_at`.
void jpeg_chunk(const mxd_jpeg_image* jimg, int32_t first, int32_t end, const std::vector<int64_t>& in_off,
                int64_t tables_at, JpegChunk* out) {
  JpegChunk& c = *out;
  c = JpegChunk();
  auto up = [](int64_t v, int64_t a) { return (v + a - 1) / a * a; };
  for (int32_t i = first; i < end; i++) {
    const mxd::jpeg::CoefInfo info = mxd::jpeg::coef_info(coefs_of(jimg[i].coefs));
    mxd::JpegImgDev m{};
    m.ncomp = info.ncomp == 1 ? 1 : 3;
    m.rgb = info.color_space == 2 ? 1 : 0;
    m.width = info.width;
    m.height = info.height;
    m.pitch = (int32_t)rgb_pitch(info.width);
    m.quads = (info.width + 3) / 4;
    for (int k = 0; k < m.ncomp; k++) {
      const mxd::jpeg::CoefPlane& cp = info.comp[k];
      mxd::JpegPlaneDev p{};
      p.coef = (in_off[i] + cp.off * 2) / 2;
      p.out = c.samples;
      p.first_block = c.nblocks;
      p.bw = cp.bw;
      p.bh = cp.bh;
      p.qtab = (int32_t)c.qtabs.size();
      p.coded = cp.coded ? 1 : 0;
      c.qtabs.insert(c.qtabs.end(), cp.q, cp.q + 64);
      c.planes.push_back(p);
      m.plane[k] = c.samples;
      m.stride[k] = cp.bw * 8;
      m.dw[k] = cp.dw;
      m.dh[k] = cp.dh;
      m.hx[k] = info.max_h / cp.h;
      m.vx[k] = info.max_v / cp.v;
      // jpeg.cpp upsample_row's choice
      const bool h2 = cp.h * 2 == info.max_h, v2 = cp.v * 2 == info.max_v;
      const bool hf = cp.h == info.max_h, vf = cp.v == info.max_v;
      m.mode[k] = hf && vf                ? mxd::kUpFull
                  : h2 && vf              ? (cp.dw > 2 ? mxd::kUpH2V1 : mxd::kUpRep)
                  : hf && v2              ? mxd::kUpH1V2
                  : h2 && v2 && cp.dw > 2 ? mxd::kUpH2V2
                                          : mxd::kUpRep;
      c.samples += up((int64_t)cp.bw * 8 * cp.bh * 8, 256);
      c.nblocks += (int64_t)cp.bw * cp.bh;
    }
    m.out = c.mid_bytes;  // relative to rgb_off, fixed below
    c.mid_bytes += up((int64_t)m.pitch * m.height, 256);
    c.max_quad_rows = std::max<int64_t>(c.max_quad_rows, (int64_t)m.height * m.quads);
    c.imgs.push_back(m);
  }
  c.rgb_off = c.samples;
  c.mid_bytes += c.samples;
  c.planes_off = up(tables_at, 256);
  c.imgs_off = up(c.planes_off + (int64_t)(c.planes.size() * sizeof(mxd::JpegPlaneDev)), 256);
  c.q_off = up(c.imgs_off + (int64_t)(c.imgs.size() * sizeof(mxd::JpegImgDev)), 256);
  c.end = c.q_off + (int64_t)(c.qtabs.size() * sizeof(uint16_t));
}

// jpeg != nullptr: images[i] is jpeg[i] as an mxd_image (3 channels, the
// window as the source); its "source" is the image's coefficients, staged
// whole, and the chunk's kernels first decode them into dev_mid.
int host_path(const mxd_image* images, int32_t n, int32_t out_dtype, int32_t device, bool dst_device,
              const mxd_jpeg_image* jpeg) {
  if (n < 0 || (n > 0 && !images)) return fail(MXD_ERR_INVALID, "mxd: bad image array");
  if (out_dtype != MXD_U8 && out_dtype != MXD_F32_DIV255) return fail(MXD_ERR_INVALID, "mxd: bad out_dtype");
  if (n == 0) return MXD_OK;
  const int64_t elem = out_dtype == MXD_F32_DIV255 ? 4 : 1;
  for (int32_t i = 0; i < n; i++)
    if (int rc = validate(images[i], i)) return rc;
  if (int rc = check_device(device)) return rc;
  DeviceGuard g(device);
  g_host_calls.fetch_add(1);
  struct CallCount {
    ~CallCount() { g_host_calls.fetch_sub(1); }
  } call_count;
  // Per image: the staged footprint (columns from x0, 16-byte aligned so both
  // kernel families read it as they would the whole image) and its offsets.
  struct Stage {
    int32_t x0, y0, rows;
    int64_t pitch, copy, in_off, out_off, out_row;
    int64_t in_size;              // staged bytes (footprint rows, or a JPEG's coefficients)
    bool src_pinned, dst_pinned;  // page-locked host memory: DMA'd directly, no staging copy
    const uint8_t* src_dev;       // zero copy: the kernel reads the page-locked source in place
    uint8_t* dst_dev;             // zero copy: the kernel writes the page-locked destination in place
  };
  std::vector<Stage> st(n);
  for (int32_t i = 0; i < n; i++) {
    const mxd_image& im = images[i];
    if (jpeg) {
      Stage& s = st[i];
      const mxd::jpeg::CoefInfo info = mxd::jpeg::coef_info(coefs_of(jpeg[i].coefs));
      s.x0 = s.y0 = 0;
      s.rows = im.src_h;
      s.pitch = s.copy = 0;
      s.in_size = info.coef_count * 2;
      s.out_row = (int64_t)im.crop_w * im.channels * elem;
      s.src_pinned = false;
      s.src_dev = nullptr;
      s.dst_pinned = !dst_device && host_pinned(im.dst);
      s.dst_dev = s.dst_pinned && !(g_policy.load() & MXD_POLICY_NO_ZERO_COPY)
                      ? const_cast<uint8_t*>(host_device_ptr(im.dst)) : nullptr;
      if (!dst_device && im.dst_stride < s.out_row)
        return fail(MXD_ERR_INVALID, "mxd: dst_stride smaller than an output row");
      continue;
    }
    const DevTable *xt = nullptr, *yt = nullptr;
    if (int rc = tables().get(device, im.src_w, im.resize_w, &xt)) return rc;
    if (int rc = tables().get(device, im.src_h, im.resize_h, &yt)) return rc;
    int32_t xl, xh, yl, yh;
    footprint(*xt, *yt, im, &xl, &xh, &yl, &yh);
    const int32_t c = im.channels;
    const int32_t m = 16 / std::gcd(c, 16);  // x0 * c is a multiple of 16
    Stage& s = st[i];
    s.x0 = xl - xl % m;
    s.y0 = yl;
    s.rows = yh - yl + 1;
    const int64_t want = (int64_t)(xh + 1 - s.x0) * c + 32;  // + the kernels' read-ahead inside a row
    s.copy = std::min<int64_t>((int64_t)(im.src_w - s.x0) * c, want);
    s.pitch = (want + 15) & ~(int64_t)15;
    s.in_size = s.pitch * s.rows;
    s.out_row = (int64_t)im.crop_w * c * elem;
    s.src_pinned = host_pinned(im.src);
    // Page-locked sources are read in place by the kernel (PCIe reads): 2-D
    // DMA of short footprint rows measured 3.4x slower than one contiguous
    // copy of the same bytes (tools/pcie_probe.py).
    s.src_dev = s.src_pinned && !(g_policy.load() & MXD_POLICY_NO_ZERO_COPY) ? host_device_ptr(im.src) : nullptr;
    s.dst_pinned = !dst_device && host_pinned(im.dst);
    s.dst_dev = s.dst_pinned && !(g_policy.load() & MXD_POLICY_NO_ZERO_COPY)
                    ? const_cast<uint8_t*>(host_device_ptr(im.dst)) : nullptr;
    if (!dst_device && im.dst_stride < s.out_row)
      return fail(MXD_ERR_INVALID, "mxd: dst_stride smaller than an output row");
  }
  // Chunks of about kChunk staged bytes (at least one image each).
  constexpr int64_t kChunk = 24 << 20;
  // (and at most 65535 images: the JPEG colour kernel puts one image per grid row)
  constexpr int32_t kChunkImages = 65535;
  std::vector<std::pair<int32_t, int32_t>> chunks;  // [first, end)
  for (int32_t i = 0; i < n;) {
    int32_t j = i;
    int64_t bytes = 0;
    while (j < n && j - i < kChunkImages && (j == i || bytes + st[j].in_size <= kChunk)) {
      bytes += st[j].in_size;
      j++;
    }
    chunks.push_back({i, j});
    i = j;
  }
  CtxLease lease(device);
  HostCtx& ctx = *lease.ctx;
  // On every exit (an error return included) the context goes back to the
  // pool idle: no kernel of this call may still read its slot buffers or
  // write the caller's destinations once the call has returned.
  struct Drain {
    HostCtx& c;
    ~Drain() {
      for (Slot& sl : c.slot)
        if (sl.stream) (void)hipStreamSynchronize(sl.stream);
    }
  } drain{ctx};
  for (Slot& sl : ctx.slot)
    if (int rc = init_slot(sl)) return rc;
  int pending[2] = {-1, -1};  // chunk in flight on each slot
  auto copy_out = [&](int k) -> int {
    Slot& sl = ctx.slot[k & 1];
    MXD_HIP(hipEventSynchronize(sl.done));
    pending[k & 1] = -1;
    if (dst_device) return MXD_OK;  // the kernel wrote the destinations
    int64_t bytes = 0;
    for (int32_t i = chunks[k].first; i < chunks[k].second; i++) bytes += st[i].out_row * images[i].crop_h;
    parallel_items(chunks[k].first, chunks[k].second, bytes, [&](int32_t i) {
      if (st[i].dst_pinned) return;  // DMA'd straight into place
      const mxd_image& im = images[i];
      uint8_t* d = static_cast<uint8_t*>(im.dst);
      const uint8_t* src = sl.pin_out + st[i].out_off;
      if (im.dst_stride == st[i].out_row) {
        std::memcpy(d, src, (size_t)st[i].out_row * im.crop_h);
      } else {
        for (int32_t r = 0; r < im.crop_h; r++)
          std::memcpy(d + (size_t)r * im.dst_stride, src + (size_t)r * st[i].out_row, st[i].out_row);
      }
    });
    return MXD_OK;
  };
  for (int k = 0; k < (int)chunks.size(); k++) {
    Slot& sl = ctx.slot[k & 1];
    if (pending[k & 1] >= 0)
      if (int rc = copy_out(pending[k & 1])) return rc;
    // Staged images first (one H2D / D2H each way covers them), directly
    // DMA'd ones after them.
    int64_t in_bytes = 0, out_bytes = 0;
    for (int pass = 0; pass < 2; pass++)
      for (int32_t i = chunks[k].first; i < chunks[k].second; i++)
        if (st[i].src_pinned == (pass == 1) && !st[i].src_dev) {
          st[i].in_off = in_bytes;
          in_bytes += (st[i].in_size + 255) & ~(int64_t)255;
        }
    int64_t in_staged = 0, out_staged = 0;
    for (int32_t i = chunks[k].first; i < chunks[k].second; i++)
      if (!st[i].src_pinned) in_staged = std::max(in_staged, st[i].in_off + st[i].in_size);
    JpegChunk jc;
    if (jpeg) {
      std::vector<int64_t> off(n, 0);
      for (int32_t i = chunks[k].first; i < chunks[k].second; i++) off[i] = st[i].in_off;
      jpeg_chunk(jpeg, chunks[k].first, chunks[k].second, off, in_bytes, &jc);
      in_bytes = in_staged = jc.end;  // coefficients, then the chunk's tables, in one copy
      if (int rc = grow_device(&sl.dev_mid, &sl.dev_mid_cap, jc.mid_bytes)) return rc;
    }
    for (int pass = 0; pass < 2; pass++)
      for (int32_t i = chunks[k].first; i < chunks[k].second; i++)
        if (st[i].dst_pinned == (pass == 1) && !st[i].dst_dev) {
          st[i].out_off = out_bytes;
          // page-locked destinations back to back (one copy per contiguous run)
          const int64_t b = st[i].out_row * images[i].crop_h;
          out_bytes += pass == 1 && (st[i].out_row & 3) == 0 ? b : (b + 255) & ~(int64_t)255;
        }
    for (int32_t i = chunks[k].first; i < chunks[k].second; i++)
      if (!st[i].dst_pinned) out_staged = std::max(out_staged, st[i].out_off + st[i].out_row * images[i].crop_h);
    if (int rc = grow_pinned(&sl.pin_in, &sl.pin_in_cap, in_bytes)) return rc;
    if (int rc = grow_device(&sl.dev_in, &sl.dev_in_cap, in_bytes)) return rc;
    if (!dst_device) {
      if (int rc = grow_pinned(&sl.pin_out, &sl.pin_out_cap, out_bytes)) return rc;
      if (int rc = grow_device(&sl.dev_out, &sl.dev_out_cap, out_bytes)) return rc;
    }
    // Zero copy through the staging buffers too: the kernel reads staged
    // footprints from the page-locked slot buffer and writes results into its
    // page-locked output buffer (no H2D / D2H DMA step in between).
    const bool zc = !(g_policy.load() & MXD_POLICY_NO_ZERO_COPY) && !jpeg;
    const uint8_t* pin_in_dev = zc ? host_device_ptr(sl.pin_in) : nullptr;
    uint8_t* pin_out_dev = zc && !dst_device && sl.pin_out ? const_cast<uint8_t*>(host_device_ptr(sl.pin_out)) : nullptr;
    const int32_t cn = chunks[k].second - chunks[k].first;
    std::vector<mxd_image> dev_imgs(images + chunks[k].first, images + chunks[k].second);
    std::vector<Stored> where(cn);
    parallel_items(chunks[k].first, chunks[k].second, in_staged, [&](int32_t i) {
      const mxd_image& im = images[i];
      const Stage& s = st[i];
      if (jpeg) {
        std::memcpy(sl.pin_in + s.in_off, mxd::jpeg::coef_info(coefs_of(jpeg[i].coefs)).coef, s.in_size);
        return;
      }
      if (s.src_pinned) return;
      uint8_t* stage = sl.pin_in + s.in_off;
      const uint8_t* from = im.src + (int64_t)s.y0 * im.src_stride + (int64_t)s.x0 * im.channels;
      for (int32_t r = 0; r < s.rows; r++) std::memcpy(stage + r * s.pitch, from + (int64_t)r * im.src_stride, s.copy);
    });
    if (jpeg) {
      std::memcpy(sl.pin_in + jc.planes_off, jc.planes.data(), jc.planes.size() * sizeof(mxd::JpegPlaneDev));
      for (auto& m : jc.imgs) m.out += jc.rgb_off;
      std::memcpy(sl.pin_in + jc.imgs_off, jc.imgs.data(), jc.imgs.size() * sizeof(mxd::JpegImgDev));
      std::memcpy(sl.pin_in + jc.q_off, jc.qtabs.data(), jc.qtabs.size() * sizeof(uint16_t));
    }
    for (int32_t j = 0; j < cn; j++) {
      const int32_t i = chunks[k].first + j;
      const mxd_image& im = images[i];
      const Stage& s = st[i];
      if (jpeg) {
        const mxd::JpegImgDev& m = jc.imgs[j];
        const uint8_t* win = sl.dev_mid + m.out + (int64_t)jpeg[i].win_y * m.pitch + (int64_t)jpeg[i].win_x * 3;
        where[j] = Stored{win, m.pitch, 0, 0, im.src_h};
        dev_imgs[j].src = win;
        dev_imgs[j].src_stride = m.pitch;
        if (!dst_device && !s.dst_dev) {
          dev_imgs[j].dst = sl.dev_out + s.out_off;
          dev_imgs[j].dst_stride = s.out_row;
        } else if (s.dst_dev) {
          dev_imgs[j].dst = s.dst_dev;  // written in place over PCIe
        }
        continue;
      }
      if (s.src_dev) {
        // zero copy: the footprint rows in place in the page-locked source
        const uint8_t* base = s.src_dev + (int64_t)s.y0 * im.src_stride + (int64_t)s.x0 * im.channels;
        where[j] = Stored{base, im.src_stride, s.x0, s.y0, s.rows};
        dev_imgs[j].src = base;
      } else {
        const uint8_t* in = pin_in_dev ? pin_in_dev : sl.dev_in;
        where[j] = Stored{in + s.in_off, s.pitch, s.x0, s.y0, s.rows};
        dev_imgs[j].src = in + s.in_off;  // checked by validate() only; `where` says what is stored
      }
      dev_imgs[j].src_stride = std::max<int64_t>(s.pitch, (int64_t)im.src_w * im.channels);
      if (!dst_device && !s.dst_dev) {
        dev_imgs[j].dst = (pin_out_dev ? pin_out_dev : sl.dev_out) + s.out_off;
        dev_imgs[j].dst_stride = s.out_row;
      } else if (s.dst_dev) {
        dev_imgs[j].dst = s.dst_dev;  // written in place over PCIe
      }
    }
    if (in_staged > 0 && !pin_in_dev)
      MXD_HIP(hipMemcpyAsync(sl.dev_in, sl.pin_in, in_staged, hipMemcpyHostToDevice, sl.stream));
    if (jpeg) {
      mxd::launch_jpeg_idct(reinterpret_cast<const int16_t*>(sl.dev_in),
                            reinterpret_cast<const uint16_t*>(sl.dev_in + jc.q_off),
                            reinterpret_cast<const mxd::JpegPlaneDev*>(sl.dev_in + jc.planes_off),
                            (int32_t)jc.planes.size(), jc.nblocks, sl.dev_mid, sl.stream);
      mxd::launch_jpeg_color(sl.dev_mid, reinterpret_cast<const mxd::JpegImgDev*>(sl.dev_in + jc.imgs_off), cn,
                             jc.max_quad_rows, sl.dev_mid, sl.stream);
      MXD_HIP(hipGetLastError());
    }
    for (int32_t i = chunks[k].first; i < chunks[k].second; i++) {
      const Stage& s = st[i];
      if (!s.src_pinned || s.src_dev) continue;
      const mxd_image& im = images[i];
      const uint8_t* from = im.src + (int64_t)s.y0 * im.src_stride + (int64_t)s.x0 * im.channels;
      MXD_HIP(hipMemcpy2DAsync(sl.dev_in + s.in_off, s.pitch, from, im.src_stride, s.copy, s.rows,
                               hipMemcpyHostToDevice, sl.stream));
    }
    if (int rc = run_batch(dev_imgs.data(), cn, out_dtype, device, sl.stream, where.data())) return rc;
    if (!dst_device) {
      if (out_staged > 0 && !pin_out_dev)
        MXD_HIP(hipMemcpyAsync(sl.pin_out, sl.dev_out, out_staged, hipMemcpyDeviceToHost, sl.stream));
      // Page-locked destinations: straight from the device.  Images packed
      // back to back both here and in the destination (a batch tensor) go as
      // one copy; strided ones as 2-D copies.
      for (int32_t i = chunks[k].first; i < chunks[k].second;) {
        const Stage& s = st[i];
        if (!s.dst_pinned || s.dst_dev) {
          i++;
          continue;
        }
        const int64_t bytes_i = s.out_row * images[i].crop_h;
        if (images[i].dst_stride != s.out_row) {
          MXD_HIP(hipMemcpy2DAsync(images[i].dst, images[i].dst_stride, sl.dev_out + s.out_off, s.out_row, s.out_row,
                                   images[i].crop_h, hipMemcpyDeviceToHost, sl.stream));
          i++;
          continue;
        }
        int32_t j = i + 1;
        int64_t run = bytes_i;
        while (j < chunks[k].second && st[j].dst_pinned && images[j].dst_stride == st[j].out_row &&
               static_cast<uint8_t*>(images[j].dst) == static_cast<uint8_t*>(images[i].dst) + run &&
               st[j].out_off == s.out_off + run) {
          run += st[j].out_row * images[j].crop_h;
          j++;
        }
        MXD_HIP(hipMemcpyAsync(images[i].dst, sl.dev_out + s.out_off, run, hipMemcpyDeviceToHost, sl.stream));
        i = j;
      }
    }
    MXD_HIP(hipEventRecord(sl.done, sl.stream));
    pending[k & 1] = k;
    // results of the previous chunk, while this one runs
    const int prev = pending[(k + 1) & 1];
    if (prev >= 0)
      if (int rc = copy_out(prev)) return rc;
  }
  for (int k = 0; k < 2; k++)
    if (pending[k] >= 0)
      if (int rc = copy_out(pending[k])) return rc;
  return MXD_OK;
}
}  // namespace

namespace {
int jpeg_path(const mxd_jpeg_image* jimg, int32_t n, int32_t out_dtype, int32_t device, bool dst_device) {
  if (n < 0 || (n > 0 && !jimg)) return fail(MXD_ERR_INVALID, "mxd: bad image array");
  std::vector<mxd_image> imgs(n);
  for (int32_t i = 0; i < n; i++) {
    const mxd_jpeg_image& j = jimg[i];
    const std::string at = " (image " + std::to_string(i) + ")";
    if (!j.coefs) return fail(MXD_ERR_INVALID, "mxd: null coefs" + at);
    const mxd::jpeg::CoefInfo info = mxd::jpeg::coef_info(coefs_of(j.coefs));
    if (!info.device_ok)
      return fail(MXD_ERR_UNSUPPORTED, "mxd: CMYK / YCCK JPEGs finish on the host (mxd_jpeg_coefs_finish)" + at);
    if (j.win_w <= 0 || j.win_h <= 0)
      return fail(MXD_ERR_INVALID, "image: cannot create image with 0 or negative dimension" + at);
    if (j.win_x < 0 || j.win_y < 0 || (int64_t)j.win_x + j.win_w > info.width ||
        (int64_t)j.win_y + j.win_h > info.height)
      return fail(MXD_ERR_INVALID, "mxd: source window outside the image" + at);
    mxd_image& m = imgs[i];
    m.src = reinterpret_cast<const uint8_t*>(j.coefs);  // validated, never read: host_path decodes the coefficients
    m.src_stride = (int64_t)j.win_w * 3;
    m.src_w = j.win_w;
    m.src_h = j.win_h;
    m.channels = 3;
    m.resize_w = j.resize_w;
    m.resize_h = j.resize_h;
    m.crop_x = j.crop_x;
    m.crop_y = j.crop_y;
    m.crop_w = j.crop_w;
    m.crop_h = j.crop_h;
    m.flip = j.flip;
    m.dst = j.dst;
    m.dst_stride = j.dst_stride;
  }
  return host_path(imgs.data(), n, out_dtype, device, dst_device, jimg);
}
}  // namespace

int mxd_jpeg_coefs_decode(const uint8_t* data, size_t size, mxd_jpeg_coefs** out) {
  if (!data || !out) return fail(MXD_ERR_INVALID, "mxd: null argument");
  std::string err;
  mxd::jpeg::Coefs* c = mxd::jpeg::decode_coefs(data, size, &err);
  if (!c) return fail(MXD_ERR_INVALID, "load_jpeg: " + err);
  *out = reinterpret_cast<mxd_jpeg_coefs*>(c);
  return MXD_OK;
}

int mxd_jpeg_coefs_free(mxd_jpeg_coefs* coefs) {
  mxd::jpeg::free_coefs(reinterpret_cast<mxd::jpeg::Coefs*>(coefs));
  return MXD_OK;
}

int mxd_jpeg_coefs_info(const mxd_jpeg_coefs* coefs, int32_t* width, int32_t* height, int32_t* device_ok) {
  if (!coefs || !width || !height || !device_ok) return fail(MXD_ERR_INVALID, "mxd: null argument");
  const mxd::jpeg::CoefInfo info = mxd::jpeg::coef_info(coefs_of(coefs));
  *width = info.width;
  *height = info.height;
  *device_ok = info.device_ok ? 1 : 0;
  return MXD_OK;
}

int mxd_jpeg_coefs_finish(const mxd_jpeg_coefs* coefs, uint8_t* dst, int64_t dst_stride) {
  if (!coefs || !dst) return fail(MXD_ERR_INVALID, "mxd: null argument");
  const mxd::jpeg::CoefInfo info = mxd::jpeg::coef_info(coefs_of(coefs));
  if (dst_stride < (int64_t)info.width * 3) return fail(MXD_ERR_INVALID, "mxd: dst_stride smaller than a row");
  std::string err;
  if (!mxd::jpeg::finish(coefs_of(coefs), dst, dst_stride, &err)) return fail(MXD_ERR_INVALID, "load_jpeg: " + err);
  return MXD_OK;
}

int mxd_jpeg_resize_crop_host(const mxd_jpeg_image* images, int32_t n, int32_t out_dtype, int32_t device) {
  return jpeg_path(images, n, out_dtype, device, false);
}

int mxd_jpeg_resize_crop_to_device(const mxd_jpeg_image* images, int32_t n, int32_t out_dtype, int32_t device) {
  return jpeg_path(images, n, out_dtype, device, true);
}

int mxd_release_host_buffers(void) {
  host_pool().trim();
  return MXD_OK;
}

int mxd_rotate_geometry(int64_t w, int64_t h, double angle, int32_t crop, float* mx6, int64_t* out_w,
                        int64_t* out_h) {
#pragma clang fp contract(off)
  if (!mx6 || !out_w || !out_h) return fail(MXD_ERR_INVALID, "mxd: null output");
  // core/image/ImageTransform.cpp:112-121: pi, the radian angle, cos and sin in float
  const float pi = std::atan(1.0) * 4;
  const float rangle = angle * pi / 180.;
  const float c = std::cos(rangle);
  const float s = std::sin(rangle);
  const float mx[6] = {c, s, 0, -s, c, 0};
  for (int k = 0; k < 6; k++) mx6[k] = mx[k];
  // :81-86 (float products, truncated to int64)
  int64_t tw = w, th = h;
  if (!crop) {
    tw = (int64_t)((float)w * std::fabs(mx[0]) + (float)h * std::fabs(mx[1]));
    th = (int64_t)((float)h * std::fabs(mx[3]) + (float)w * std::fabs(mx[4]));
  }
  *out_w = tw;
  *out_h = th;
  if (tw <= 0 || th <= 0) return fail(MXD_ERR_INVALID, "image: cannot create image with 0 or negative dimension");
  return MXD_OK;
}

int mxd_channel_reduction_preset(const char* preset, float* params4) {
  if (!preset || !params4) return fail(MXD_ERR_INVALID, "mxd: null argument");
  // op/ImageTransform.cpp:362-392
  struct P {
    const char* name;
    float bias, m[3];
  };
  static const P presets[] = {{"default", 0, {0.299, 0.587, 0.114}},
                              {"rec601", 0, {0.299, 0.587, 0.114}},
                              {"rec709", 0, {0.2126, 0.7152, 0.0722}},
                              {"rec2020", 0, {0.2627, 0.678, 0.0593}},
                              {"green", 0, {0, 1, 0}}};
  for (const P& p : presets)
    if (std::strcmp(p.name, preset) == 0) {
      params4[0] = p.bias;
      for (int k = 0; k < 3; k++) params4[1 + k] = p.m[k];
      return MXD_OK;
    }
  return fail(MXD_ERR_INVALID, std::string("ImageChannelReduction: unable to find preset ") + preset);
}

int mxd_is_jpeg(const uint8_t* data, size_t size) { return data && mxd::jpeg::is_jpeg(data, size) ? 1 : 0; }

int mxd_jpeg_info(const uint8_t* data, size_t size, int32_t* width, int32_t* height, int32_t* components) {
  if (!data || !width || !height || !components) return fail(MXD_ERR_INVALID, "mxd: null argument");
  int w = 0, h = 0, c = 0;
  std::string err;
  if (!mxd::jpeg::info(data, size, &w, &h, &c, &err)) return fail(MXD_ERR_INVALID, "load_jpeg: " + err);
  *width = w;
  *height = h;
  *components = c;
  return MXD_OK;
}

int mxd_jpeg_decode(const uint8_t* data, size_t size, uint8_t* dst, int64_t dst_stride, int32_t width,
                    int32_t height) {
  if (!data || !dst) return fail(MXD_ERR_INVALID, "mxd: null argument");
  if (dst_stride < (int64_t)width * 3) return fail(MXD_ERR_INVALID, "mxd: dst_stride smaller than a row");
  std::string err;
  if (!mxd::jpeg::decode(data, size, dst, dst_stride, width, height, &err))
    return fail(MXD_ERR_INVALID, "load_jpeg: " + err);
  return MXD_OK;
}

int mxd_pixmap_batch(const mxd_pixmap* images, int32_t n, int32_t op, int32_t device, void* stream) {
  if (n > 0 && images)
    for (int32_t i = 0; i < n; i++)
      if (int rc = pix_validate(images[i], op, i)) return rc;
  if (n > 0)
    if (int rc = check_device(device)) return rc;
  return run_pixmap(images, n, op, device, stream);
}

int mxd_pixmap_host(const mxd_pixmap* images, int32_t n, int32_t op, int32_t device) {
  if (n < 0 || (n > 0 && !images)) return fail(MXD_ERR_INVALID, "mxd: bad image array");
  if (n == 0) return MXD_OK;
  for (int32_t i = 0; i < n; i++)
    if (int rc = pix_validate(images[i], op, i)) return rc;
  if (int rc = check_device(device)) return rc;
  DeviceGuard g(device);
  CtxLease lease(device);
  Slot& ctx = lease.ctx->slot[0];
  if (int rc = init_slot(ctx)) return rc;
  std::vector<size_t> in_off(n), out_off(n);
  std::vector<int64_t> in_pitch(n), out_pitch(n);
  size_t in_bytes = 0, out_bytes = 0;
  for (int32_t i = 0; i < n; i++) {
    const mxd_pixmap& im = images[i];
    const int64_t oc = op == MXD_AFFINE ? im.channels : 1;
    in_pitch[i] = ((int64_t)im.src_w * im.channels + 15) & ~(int64_t)15;
    out_pitch[i] = ((int64_t)im.dst_w * oc + 15) & ~(int64_t)15;
    in_off[i] = in_bytes;
    in_bytes += ((size_t)in_pitch[i] * im.src_h + 255) & ~(size_t)255;
    out_off[i] = out_bytes;
    out_bytes += ((size_t)out_pitch[i] * im.dst_h + 255) & ~(size_t)255;
  }
  if (int rc = grow_pinned(&ctx.pin_in, &ctx.pin_in_cap, in_bytes)) return rc;
  if (int rc = grow_pinned(&ctx.pin_out, &ctx.pin_out_cap, out_bytes)) return rc;
  if (int rc = grow_device(&ctx.dev_in, &ctx.dev_in_cap, in_bytes)) return rc;
  if (int rc = grow_device(&ctx.dev_out, &ctx.dev_out_cap, out_bytes)) return rc;
  std::vector<mxd_pixmap> dev_imgs(images, images + n);
  for (int32_t i = 0; i < n; i++) {
    const mxd_pixmap& im = images[i];
    const size_t row = (size_t)im.src_w * im.channels;
    uint8_t* stage = ctx.pin_in + in_off[i];
    for (int32_t r = 0; r < im.src_h; r++)
      std::memcpy(stage + (size_t)r * in_pitch[i], im.src + (size_t)r * im.src_stride, row);
    dev_imgs[i].src = ctx.dev_in + in_off[i];
    dev_imgs[i].src_stride = in_pitch[i];
    dev_imgs[i].dst = ctx.dev_out + out_off[i];
    dev_imgs[i].dst_stride = out_pitch[i];
  }
  MXD_HIP(hipMemcpyAsync(ctx.dev_in, ctx.pin_in, in_bytes, hipMemcpyHostToDevice, ctx.stream));
  if (int rc = run_pixmap(dev_imgs.data(), n, op, device, ctx.stream)) return rc;
  MXD_HIP(hipMemcpyAsync(ctx.pin_out, ctx.dev_out, out_bytes, hipMemcpyDeviceToHost, ctx.stream));
  MXD_HIP(hipStreamSynchronize(ctx.stream));
  for (int32_t i = 0; i < n; i++) {
    const mxd_pixmap& im = images[i];
    const size_t row = (size_t)im.dst_w * (op == MXD_AFFINE ? im.channels : 1);
    uint8_t* d = static_cast<uint8_t*>(im.dst);
    const uint8_t* s = ctx.pin_out + out_off[i];
    for (int32_t r = 0; r < im.dst_h; r++) std::memcpy(d + (size_t)r * im.dst_stride, s + (size_t)r * out_pitch[i], row);
  }
  return MXD_OK;
}

}  // extern "C"
