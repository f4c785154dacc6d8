// capi.cpp -- the C ABI declared in include/mxd_amd.h: the extern "C" entry
// points (validation with the reference's error conditions, no exceptions
// across the ABI: every entry point returns a status and leaves a
// thread-local message), pixel-map dispatch and the process-wide state.  The
// fused stage's planning, batches and host path live in plan.cpp, batch.cpp
// and hostpath.cpp (capi_internal.h).
#include "capi_internal.h"

namespace mxd {
namespace capi {

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

// ---------------------------------------------------------------------------
// Per-(device, stream) descriptor workspace: pinned staging + device copy of
// the ImgDev array.  Re-uploads are skipped when the batch is unchanged.
// Kernel policy (mxd_set_kernel_policy): a process-wide tuning / test switch
// between kernels that compute identical results.
std::atomic<int32_t> g_policy{0};
// Tuning knobs (mxd_set_tuning): 0 = automatic.
std::atomic<int32_t> g_tune[MXD_TUNE_COUNT] = {};


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

}  // namespace capi
}  // namespace mxd

using namespace mxd::capi;

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
  // hipDeviceProp_t::name came back empty on some boxes:
  // then hipDeviceGetName, then the architecture and CU count.
  std::string nm = p.name;
  if (nm.empty()) {
    char buf[256] = {0};
    if (hipDeviceGetName(buf, sizeof buf - 1, device) == hipSuccess) nm = buf;
  }
  if (nm.empty()) nm = std::string(p.gcnArchName).substr(0, std::string(p.gcnArchName).find(':')) + " (" +
                       std::to_string(p.multiProcessorCount) + " CUs)";
  put(name, name_len, nm.c_str());
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
  return mxd_copy_bandwidth_policy(bytes, device, iters, 0, gbps);
}

int mxd_copy_bandwidth_policy(size_t bytes, int32_t device, int32_t iters, int32_t policy, float* gbps) {
  if (!gbps || bytes < 16 || iters <= 0 || policy < 0 || policy > 2)
    return fail(MXD_ERR_INVALID, "mxd: bad copy_bandwidth arguments");
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
  mxd::launch_copy(a, b, bytes, s, policy);
  MXD_HIP(hipEventRecord(e0, s));
  for (int32_t i = 0; i < iters; i++) mxd::launch_copy(a, b, bytes, s, policy);
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

int mxd_device_synchronize(int32_t device) {
  if (int rc = check_device(device)) return rc;
  DeviceGuard g(device);
  MXD_HIP(hipDeviceSynchronize());
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


int mxd_jpeg_coefs_decode(const uint8_t* data, size_t size, mxd_jpeg_coefs** out) {
  if (!data || !out) return fail(MXD_ERR_INVALID, "mxd: null argument");
  std::string err;
  mxd::jpeg::Coefs* c = mxd::jpeg::decode_coefs(data, size, &err);
  if (!c) return fail(MXD_ERR_INVALID, "load_jpeg: " + err);
  *out = reinterpret_cast<mxd_jpeg_coefs*>(c);
  return MXD_OK;
}

int mxd_jpeg_coefs_parse(const uint8_t* data, size_t size, int32_t device_entropy, mxd_jpeg_coefs** out) {
  if (!data || !out) return fail(MXD_ERR_INVALID, "mxd: null argument");
  std::string err;
  const int64_t t0 = now_ns();
  mxd::jpeg::Coefs* c = mxd::jpeg::parse_coefs(data, size, device_entropy != 0, &err);
  g_host_stats[4].fetch_add(1, std::memory_order_relaxed);
  g_host_stats[5].fetch_add(now_ns() - t0, std::memory_order_relaxed);
  if (!c) return fail(MXD_ERR_INVALID, "load_jpeg: " + err);
  *out = reinterpret_cast<mxd_jpeg_coefs*>(c);
  return MXD_OK;
}

int mxd_jpeg_coefs_load(const char* path, int32_t device_entropy, mxd_jpeg_coefs** out) {
  if (!path || !out) return fail(MXD_ERR_INVALID, "mxd: null argument");
  *out = nullptr;
  std::string err;
  bool not_jpeg = false;
  const int64_t t0 = now_ns();
  mxd::jpeg::Coefs* c = mxd::jpeg::load_coefs(path, device_entropy != 0, &not_jpeg, &err);
  g_host_stats[4].fetch_add(1, std::memory_order_relaxed);
  g_host_stats[5].fetch_add(now_ns() - t0, std::memory_order_relaxed);
  if (not_jpeg) return MXD_OK;
  if (!c) return fail(MXD_ERR_INVALID, "load_jpeg: " + err);
  *out = reinterpret_cast<mxd_jpeg_coefs*>(c);
  return MXD_OK;
}

int mxd_jpeg_coefs_entropy_pending(const mxd_jpeg_coefs* coefs, int32_t* pending) {
  if (!coefs || !pending) return fail(MXD_ERR_INVALID, "mxd: null argument");
  const mxd::jpeg::CoefInfo info = mxd::jpeg::coef_info(coefs_of(coefs));
  *pending = info.entropy_pending ? 1 : 0;
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

int mxd_host_stats(int64_t* out6, int32_t reset) {
  if (!out6) return fail(MXD_ERR_INVALID, "mxd: null out6");
  for (int i = 0; i < 6; i++) out6[i] = reset ? g_host_stats[i].exchange(0) : g_host_stats[i].load();
  return MXD_OK;
}

int mxd_device_stats(int64_t* out2, int32_t reset) {
  if (!out2) return fail(MXD_ERR_INVALID, "mxd: null out2");
  for (int i = 0; i < 2; i++) out2[i] = reset ? g_device_stats[i].exchange(0) : g_device_stats[i].load();
  return MXD_OK;
}

int mxd_jpeg_plane_sources(int64_t* count, int32_t reset) {
  if (!count) return fail(MXD_ERR_INVALID, "mxd: null count");
  *count = reset ? g_plane_sources.exchange(0) : g_plane_sources.load();
  return MXD_OK;
}

int mxd_narrow_returns(int64_t* count, int32_t reset) {
  if (!count) return fail(MXD_ERR_INVALID, "mxd: null count");
  *count = reset ? g_narrow_images.exchange(0) : g_narrow_images.load();
  return MXD_OK;
}

int mxd_release_host_buffers(void) {
  host_trim();
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
  return pixmap_host(images, n, op, device);
}

}  // extern "C"
