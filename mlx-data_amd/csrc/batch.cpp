// batch.cpp -- run_batch (capi_internal.h): per-stream descriptor
// workspaces and the fused launches of one batch (band, wave and general
// kernels, forked over helper streams when a batch needs several).
#include <atomic>
#include <deque>

#include "capi_internal.h"

namespace mxd {
namespace capi {
namespace {

// A call whose wave-kernel sources total at least this many bytes loads them
// with the streaming (nt) policy (half the 256 MB Infinity Cache).
constexpr int64_t kNtSourceBytes = (int64_t)128 << 20;

struct Workspace {
  std::mutex mu;
  // Descriptor slots: each launch reads its descriptors from one slot.  A
  // batch whose descriptors a slot holds reuses it; a new one takes the least
  // recently used slot once the launches that read it are done.
  // Reuse is fenced without an event per launch (an event between kernels
  // costs the GPU a few microseconds): batches are numbered in stream order,
  // every slot remembers the last batch that read it, and one event is
  // recorded every kFenceEvery batches; reusing a slot waits on the first
  // fence recorded after its last batch (recording one then if none is).
  // With 16 slots the fence a reuse needs was recorded >= 8 batches earlier
  // and has normally completed.
  static constexpr int kSlots = 16;
  static constexpr uint64_t kFenceEvery = 8;
  static constexpr size_t kMaxFences = 8;
  struct Slot {
    ImgDev* host = nullptr;  // pageable copy (cache key; copy modes' source)
    ImgDev* dev = nullptr;
    ImgDev* zc = nullptr;          // pinned, read by the kernels in place (zero-copy modes)
    bool zc_nc = false;            // zc allocated non-coherent
    const ImgDev* launch = nullptr;  // what the batch's kernels read (dev or zc)
    size_t cap = 0, count = 0;
    hipEvent_t copied = nullptr;   // mode 1: the copy-stream upload landed
    uint64_t last_use = 0;         // LRU clock
    uint64_t last_batch = 0;       // the last batch that read it (0: none)
  } slot[kSlots];
  int cur = -1;
  uint64_t clock = 0;
  uint64_t batch = 0;    // batches launched on this stream
  uint64_t written = 0;  // of them, batches that wrote a slot
  struct Fence {
    hipEvent_t ev;
    uint64_t covers;  // every batch <= covers has finished once ev has
  };
  std::deque<Fence> fences;
  std::vector<hipEvent_t> spare;
  hipStream_t copy = nullptr;
  // Fork/join helpers: the launches of a mixed batch (one per kernel shape)
  // run concurrently on these streams, so one launch's tail overlaps the
  // next instead of idling the CUs between serialized launches.
  static constexpr int kHelpers = 3;
  hipStream_t helper[kHelpers] = {};
  hipEvent_t fork = nullptr, join[kHelpers] = {};
};

// Records a fence covering every batch launched so far on the stream.
int record_fence(Workspace* ws, hipStream_t s) {
  hipEvent_t ev = nullptr;
  if (!ws->spare.empty()) {
    ev = ws->spare.back();
    ws->spare.pop_back();
  } else {
    MXD_HIP(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
  }
  MXD_HIP(hipEventRecord(ev, s));
  ws->fences.push_back({ev, ws->batch});
  while (ws->fences.size() > Workspace::kMaxFences) {
    // a later fence covers everything the oldest did
    ws->spare.push_back(ws->fences.front().ev);
    ws->fences.pop_front();
  }
  return MXD_OK;
}

// Blocks until batch `b` of the stream has finished.
int wait_batch(Workspace* ws, uint64_t b, hipStream_t s) {
  if (b == 0) return MXD_OK;
  for (const Workspace::Fence& f : ws->fences)
    if (f.covers >= b) {
      MXD_HIP(hipEventSynchronize(f.ev));
      return MXD_OK;
    }
  if (int rc = record_fence(ws, s)) return rc;
  MXD_HIP(hipEventSynchronize(ws->fences.back().ev));
  return MXD_OK;
}

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

}  // namespace

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
  // the message is built only on failure (this runs for every image of every batch)
  auto at = [i](const char* msg) { return fail(MXD_ERR_INVALID, std::string(msg) + " (image " + std::to_string(i) + ")"); };
  if (!im.src || !im.dst) return at("mxd: null src/dst pointer");
  if (im.src_w <= 0 || im.src_h <= 0) return at("image: cannot create image with 0 or negative dimension");
  if (im.channels <= 0 || im.channels > 4) return at("verifyImage: channels must be 0 <= c <= 4");
  if (im.resize_w <= 0 || im.resize_h <= 0 || im.crop_w <= 0 || im.crop_h <= 0)
    return at("image: cannot create image with 0 or negative dimension");
  if (im.crop_x < 0 || im.crop_y < 0 || im.crop_x >= im.resize_w || im.crop_y >= im.resize_h)
    return at("Array: sub: offset out of bound");
  if (im.crop_x + im.crop_w > im.resize_w || im.crop_y + im.crop_h > im.resize_h)
    return at("Array: sub: shape out of bound");
  if (im.src_stride < (int64_t)im.src_w * im.channels) return at("mxd: src_stride smaller than a row");
  return MXD_OK;
}

// Whether the host can store into the device's memory directly (large PCI
// BAR: the whole HBM mapped for the CPU), cached per device.
bool large_bar(int32_t device) {
  static std::mutex mu;
  static std::map<int32_t, bool> known;
  std::lock_guard<std::mutex> lock(mu);
  auto it = known.find(device);
  if (it != known.end()) return it->second;
  hipDeviceProp_t prop{};
  const bool ok = hipGetDeviceProperties(&prop, device) == hipSuccess && prop.isLargeBar != 0;
  known[device] = ok;
  return ok;
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
        c.last_batch = ws->batch + 1;  // the batch about to launch
        if (c.copied && hipEventQuery(c.copied) != hipSuccess) MXD_HIP(hipStreamWaitEvent(s, c.copied, 0));
        *dev_out = const_cast<ImgDev*>(c.launch);
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
  // Host-side wait: the launches that read this slot are done.  (Ordering
  // the upload after them on the GPU instead, with a wait of the copy stream
  // on the compute stream, measured ms-long stalls.)
  if (int rc = wait_batch(ws, c.last_batch, s)) return rc;
  c.last_batch = ws->batch + 1;
  if (n > c.cap) {
    // empty first: a failed allocation below leaves an empty slot (cap 0),
    // never a stale capacity over null buffers
    c.cap = c.count = 0;
    c.launch = nullptr;
    if (c.dev) MXD_HIP(hipFree(c.dev));
    std::free(c.host);
    if (c.zc) MXD_HIP(hipHostFree(c.zc));
    c.dev = nullptr;
    c.host = nullptr;
    c.zc = nullptr;
    const size_t cap = std::max<size_t>(n, 64);
    MXD_HIP(hipMalloc(reinterpret_cast<void**>(&c.dev), sizeof(ImgDev) * cap));
    // the host copy only answers "does a slot hold these descriptors" (and is
    // the source of the copy modes 1 / 2): pageable, so 16 slots per stream
    // cost no page-locked allocations
    c.host = static_cast<ImgDev*>(std::malloc(sizeof(ImgDev) * cap));
    if (!c.host) {
      c.cap = c.count = 0;
      return fail(MXD_ERR_NOMEM, "mxd: out of host memory for descriptors");
    }
    c.cap = cap;
  }
  std::memcpy(c.host, descs.data(), bytes);
  c.count = n;
  // Upload modes (MXD_TUNE_DESC): 1 = copy stream + cross-stream wait, 2 =
  // copy on the launch stream, 3 / 4 = the kernels read the pinned slot in
  // place (coherent / non-coherent allocation), 6 = the host stores into the
  // device slot through the large PCI BAR.  Default 6 (4 without a large
  // BAR): no copy, no cross-stream wait, and the kernels read their
  // descriptors from HBM like a cached batch.  With slot reuse fenced every 4
  // written batches (8 slots), fresh batches cost C2 +0.2-1.5 % and C4
  // -3..+1.5 % over cached descriptors in mode 6, C2 +1.3 % and C4 +3..18 %
  // in mode 4 (profiles/r03/desc_host_d.jsonl, three repetitions); with 16
  // slots fenced every 8, C2 -1.5..0 % and C4 -3..+4.6 %
  // (profiles/r03/fresh_slots16.jsonl); against +3.9 % / +5 %
  // with an event per launch (desc_host.jsonl) and +6.5 % / +31 % for the
  // round-2 copy stream.  A copy kernel on the launch stream bringing the slot
  // into HBM (mode 5 of profiles/r03/desc_host_b.jsonl) measured no better and
  // was dropped.
  int32_t mode = g_tune[MXD_TUNE_DESC].load() > 0 ? g_tune[MXD_TUNE_DESC].load() : 6;
  if (mode == 6 && !large_bar(device)) mode = 4;
  if (mode == 6) {
    // the host stores the array straight into the device slot through the
    // large PCI BAR (~1 us for 13 KB); the fence drains the write-combining
    // buffers before the launch's doorbell, and the kernel-start acquire
    // drops the slot's lines from the L2s.  Kernels read HBM, no PCIe trip.
    std::memcpy(c.dev, descs.data(), bytes);
    std::atomic_thread_fence(std::memory_order_seq_cst);
    c.launch = c.dev;
  } else if (mode >= 3) {
    const bool nc = mode == 4;
    if (!c.zc || c.zc_nc != nc || n > c.cap) {
      if (c.zc) MXD_HIP(hipHostFree(c.zc));
      MXD_HIP(hipHostMalloc(reinterpret_cast<void**>(&c.zc), sizeof(ImgDev) * c.cap,
                            nc ? hipHostMallocNonCoherent : hipHostMallocDefault));
      c.zc_nc = nc;
    }
    std::memcpy(c.zc, descs.data(), bytes);
    c.launch = c.zc;
  } else if (mode == 2) {
    MXD_HIP(hipMemcpyAsync(c.dev, c.host, bytes, hipMemcpyHostToDevice, s));
    c.launch = c.dev;
  } else {
    if (!c.copied) MXD_HIP(hipEventCreateWithFlags(&c.copied, hipEventDisableTiming));
    MXD_HIP(hipMemcpyAsync(c.dev, c.host, bytes, hipMemcpyHostToDevice, ws->copy));
    MXD_HIP(hipEventRecord(c.copied, ws->copy));
    MXD_HIP(hipStreamWaitEvent(s, c.copied, 0));
    c.launch = c.dev;
  }
  *dev_out = const_cast<ImgDev*>(c.launch);
  return MXD_OK;
}

// After the launches of a batch: count it, and every kFenceEvery batches that
// wrote a slot record a fence for slot reuse (a loop of cache hits records
// none: an eviction after it records its fence on demand).
int release_descs(Workspace* ws, void* stream, bool hit) {
  ws->batch++;
  if (!hit && ++ws->written % Workspace::kFenceEvery == 0)
    return record_fence(ws, reinterpret_cast<hipStream_t>(stream));
  return MXD_OK;
}

int run_batch(const mxd_image* images, int32_t n, int32_t out_dtype, int32_t device, void* stream,
              const Stored* stored) {
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
        if (st.ycc) {
          // JPEG planes (the host path checked ycc_plan_ok): a wave kernel or nothing
          plan_wave(im, st, f32, out_dtype, p);
          if (!p.wave) return fail(MXD_ERR_UNSUPPORTED, "mxd: no wave kernel for a JPEG plane source");
        } else if (!no_wave) {
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
    d.ycc = st.ycc;
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
        if (int rc = band_schedule_dev(device, *p.yt, im.src_h, im.resize_h, im.crop_y, im.crop_h, d.ty, p.bp.db,
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
    return std::make_tuple(p.kind, p.bucket, p.s, p.dmax, p.q, p.shift, p.pp, p.ycc);
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
          {k, 0, 0, 0, mxd::WaveCfg{channels, f32, p.bucket, 0, 0, p.kind, p.s, p.dmax, p.q, p.shift, p.pp, 0, 1,
                                    p.ycc ? 1 : 0}});
    groups.back().count++;
  }
  // Source load policy (wave.hip LAUX): streaming (nt) loads when the
  // call's sources are far past what the 256 MB Infinity Cache could hold
  // for a re-read (sources just written by a decode or a copy stay there,
  // and nt loads would bypass them: C4's 128 small images measured 45 %
  // slower with nt, C2 / C3 / C5 2-7 % faster; profiles/r06/README.md).
  // MXD_TUNE_LOAD_POLICY: 1 = default policy always, 2 = nt always.
  int64_t src_bytes = 0;
  for (int32_t i : order) src_bytes += (int64_t)images[i].src_w * images[i].src_h * images[i].channels;
  const int32_t load_knob = g_tune[MXD_TUNE_LOAD_POLICY].load();
  const int32_t nt = load_knob == 2 ? 1 : load_knob == 1 ? 0 : src_bytes >= kNtSourceBytes ? 1 : 0;
  for (Group& g : groups) {
    g.cfg.nimgs = g.count;
    g.cfg.nt = g.cfg.ycc ? 0 : nt;
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
          if (int rc = scatter_schedule(device, *p.yt, im.src_h, im.resize_h, im.crop_y, im.crop_h, d.ty,
                                       ScatterShape{p.s, p.dmax, p.p,
                                                    p.ycc ? mxd::kYccLaneBytes : p.pp == 16 ? 16 : p.pp * channels},
                                       &sc))
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
  // Streams: the caller's and one helper by default.  C3's six launches
  // measured 0.465 ms on one stream, 0.429 on two and 0.455 on four
  // (profiles/r03/c3_sizing.jsonl); MXD_TUNE_STREAMS overrides.
  const int32_t knob_streams = g_tune[MXD_TUNE_STREAMS].load();
  const int32_t nstreams = knob_streams > 0 ? knob_streams : 2;
  const int nfork = std::min<int>({(int)launches.size() - 1, nstreams - 1, Workspace::kHelpers});
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
  int launch_rc = MXD_OK;
  for (size_t k = 0; k < launches.size(); k++) {
    const int lane = nfork > 0 ? (int)(k % (size_t)(nfork + 1)) : 0;
    void* s = lane == 0 ? stream : reinterpret_cast<void*>(ws->helper[lane - 1]);
    int rc = 0;
    if (launches[k].kind == 0) {
      const BandGroup& g = bgroups[launches[k].group];
      rc = mxd::launch_band(g.cfg, dev + g.first, g.table >= 0 ? tables_dev + g.table : nullptr, s);
    } else if (launches[k].kind == 1) {
      Group& g = groups[launches[k].group];
      g.cfg.prio = nfork == 0 ? 1 : 0;  // priorities only where launches never overlap
      rc = mxd::launch_wave(g.cfg, dev + wbase + g.first, s);
    } else {
      rc = mxd::launch_resample(cfg, dev + wbase + nw, s);
    }
    if (rc) {
      launch_rc = fail(MXD_ERR_DEVICE, std::string("resample launch failed: ") + hipGetErrorString(hipGetLastError()) +
                                           " rc=" + std::to_string(rc));
      break;
    }
  }
  // Every helper stream that may hold kernels of this batch joins the
  // caller's stream and the batch is counted -- on a failed launch too, so the
  // slot's fence covers the kernels already queued and a caller syncing its
  // own stream waits for their writes.
  for (int h = 0; h < nfork; h++) {
    if (hipEventRecord(ws->join[h], ws->helper[h]) != hipSuccess ||
        hipStreamWaitEvent(reinterpret_cast<hipStream_t>(stream), ws->join[h], 0) != hipSuccess)
      if (launch_rc == MXD_OK) launch_rc = fail(MXD_ERR_DEVICE, "mxd: joining helper streams failed");
  }
  const int rel = release_descs(ws, stream, hit);
  return launch_rc != MXD_OK ? launch_rc : rel;
}


}  // namespace capi
}  // namespace mxd
