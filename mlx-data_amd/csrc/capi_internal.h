// capi_internal.h -- what the translation units of the C ABI share:
// capi.cpp (extern "C" entry points, pixel maps, process-wide state),
// plan.cpp (tap tables, kernel planning, schedule caches), batch.cpp
// (descriptor workspaces, run_batch: one fused launch per kernel shape) and
// hostpath.cpp (host-resident and JPEG batches staged through page-locked
// memory).  Host only.
#pragma once
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
#include "jpeghuff.h"
#include "pixmap.h"
#include "resample.h"
#include "taps.h"



#define MXD_HIP(expr)                                                                                    \
  do {                                                                                                   \
    hipError_t e_ = (expr);                                                                              \
    if (e_ != hipSuccess) return fail(MXD_ERR_DEVICE, std::string(#expr) + ": " + hipGetErrorString(e_)); \
  } while (0)

namespace mxd {
namespace capi {

using mxd::ImgDev;
using mxd::LaunchCfg;

// Error message of the calling thread's last failed entry point.
extern thread_local std::string g_error;
int fail(int code, const std::string& msg);
// Every entry point that takes a device ordinal refuses one that does not exist.
int check_device(int32_t device);

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


// Kernel policy (mxd_set_kernel_policy) and tuning knobs (mxd_set_tuning).
extern std::atomic<int32_t> g_policy;
extern std::atomic<int32_t> g_tune[MXD_TUNE_COUNT];

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

TableCache& tables();
TableCache& host_tables();  // host copies only (planning without a device)

// ---------------------------------------------------------------------------
// Tiling.
constexpr int32_t kTileRows = 32;          // output rows per tile
constexpr int32_t kStripBytes = 1536;      // target source-footprint bytes per strip row
constexpr int32_t kLdsBudget = 40 * 1024;  // bytes of LDS for the f32 row group
constexpr int32_t kBandMaxRows = 16;       // band kernel: most output rows per unit (short units keep the
                                           // device on few images at a time; the stream makes them cheap)


int32_t strip_chunks(const DevTable& xt, int32_t crop_x, int32_t crop_w, int32_t ox0, int32_t ox1, bool flip,
                     int32_t c, int32_t vec);
int validate(const mxd_image& im, int32_t i);

// ---------------------------------------------------------------------------
// Planning (plan.cpp).
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
  bool ycc = false;  // reads JPEG sample planes (Stored::ycc)
};

// Shape of the scatter schedule for crop rows [off, off+len) of a vertical
// table, valid for bands starting at any row: dmax = most source rows that are
// new for one output row (after the previous row's last tap), p = prologue
// groups (the first output of a band needs all its taps), s = most output rows
// a source row's weights must reach from its group (accumulator slots).
// s = 0: taps not monotone (not a geometry the scatter kernel handles).
struct ScatterShape {
  int32_t s = 0, dmax = 0, p = 0;
  int32_t lane_bytes = 0;  // of the kernel that runs it (its ring: resample.h scatter_ring_slots)
};
ScatterShape scatter_shape(const DevTable& t, int32_t off, int32_t len);

// Scatter schedules (layout: wave.hip) in device memory, one per
// (device, vertical geometry, crop rows, band height, shape).
struct DevSched {
  int32_t* ptr = nullptr;
  int32_t band_words = 0;  // words per band
  int32_t entry_off = 0;   // word offset of the iteration entries in a band
};
// Device copies of the wave kernels' scatter schedule and of the band
// kernel's schedule, built once per geometry and cached.
int scatter_schedule(int32_t device, const DevTable& yt, int32_t src_h, int32_t resize_h, int32_t crop_y,
                     int32_t crop_h, int32_t ty, const ScatterShape& sh, const DevSched** out);
int band_schedule_dev(int32_t device, const DevTable& yt, int32_t src_h, int32_t resize_h, int32_t crop_y, int32_t crop_h,
                  int32_t ty, int32_t db, int32_t s, int32_t min_groups, const DevSched** out);
mxd::AxisView axis_view(const DevTable& t);

bool wave_strips(const DevTable& xt, const mxd_image& im, int32_t pp, int32_t* nstrips, int32_t* tx, int32_t* q);
int32_t band_rows(const std::vector<std::pair<int32_t, int32_t>>& strips, int32_t capacity, int32_t kMaxBand = 64);
int32_t band_capacity_cached(const mxd::BandCfg& cfg, int32_t device);
int32_t wave_capacity_cached(const mxd::WaveCfg& cfg, int32_t device);

// Where an image's source bytes live: the whole image at mxd_image::src, or
// (host path) only its staged footprint: `rows` rows from source row y0 and
// columns from source pixel x0 at base, `stride` bytes apart.
// ycc: a JPEG image's sample planes instead (base = its Y plane; wave.hip
// YccSrc): only a scatter wave kernel with RGB pixel lanes runs it.
struct Stored {
  const uint8_t* base;
  int64_t stride;
  int32_t x0, y0, rows;
  const mxd::YccDev* ycc = nullptr;
};

Stored whole(const mxd_image& im);
bool wave_layout_ok(const mxd_image& im, const Stored& st, int32_t out_dtype);
void plan_band(const mxd_image& im, const Stored& st, int32_t f32, ImgPlan& p);
void plan_wave(const mxd_image& im, const Stored& st, int32_t f32, int32_t out_dtype, ImgPlan& p);
// Whether run_batch would resize image im from the JPEG planes st.ycc
// describes (a scatter wave kernel with RGB pixel lanes takes it).
bool ycc_plan_ok(const mxd_image& im, const Stored& st, int32_t out_dtype, int32_t device);

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
PlanKey plan_key(const mxd_image& im, const Stored& st);

// ---------------------------------------------------------------------------
// Batches (batch.cpp): one fused launch per kernel shape over a batch whose
// sources are in device memory (or, from the host path, staged: stored[i]).
int run_batch(const mxd_image* images, int32_t n, int32_t out_dtype, int32_t device, void* stream,
              const Stored* stored = nullptr);

// ---------------------------------------------------------------------------
// Host-resident batches (hostpath.cpp).
int host_path(const mxd_image* images, int32_t n, int32_t out_dtype, int32_t device, bool dst_device,
              const mxd_jpeg_image* jpeg = nullptr);
int jpeg_path(const mxd_jpeg_image* jimg, int32_t n, int32_t out_dtype, int32_t device, bool dst_device);
// mxd_host_stats counters: host-path calls, images, wall ns, device-wait ns,
// coefficient parses, parse ns
extern std::atomic<int64_t> g_host_stats[6];
extern std::atomic<int64_t> g_device_stats[2];  // mxd_device_stats: timed chunks, device ns
int64_t now_ns();
extern std::atomic<int64_t> g_plane_sources;  // images resized from their JPEG sample planes (mxd_jpeg_plane_sources)
extern std::atomic<int64_t> g_narrow_images;  // f32 results returned to the host as u8 (mxd_narrow_returns)
const mxd::jpeg::Coefs* coefs_of(const mxd_jpeg_coefs* c);
// Frees the buffers of every idle host-path context (mxd_release_host_buffers).
void host_trim();

// ---------------------------------------------------------------------------
// Pixel maps (capi.cpp; host images: hostpath.cpp).
int pix_validate(const mxd_pixmap& im, int32_t op, int32_t i);
int run_pixmap(const mxd_pixmap* images, int32_t n, int32_t op, int32_t device, void* stream);
int pixmap_host(const mxd_pixmap* images, int32_t n, int32_t op, int32_t device);

}  // namespace capi
}  // namespace mxd
