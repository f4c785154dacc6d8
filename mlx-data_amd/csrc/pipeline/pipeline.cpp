// pipeline.cpp -- see pipeline.h.  Host-side control only: every pixel of the
// resize / crop / mirror path is produced by the gfx950 kernels behind
// mxd_resize_crop_host (include/mxd_amd.h); there is no CPU pixel path for
// uint8 images.
#include "pipeline.h"

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cmath>
#include <condition_variable>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <functional>
#include <future>
#include <map>
#include <mutex>
#include <numeric>
#include <stdexcept>
#include <thread>

#include "mxd_amd.h"

#include <fcntl.h>
#include <sys/stat.h>
#include <unistd.h>

#include <cerrno>
#include <cstdint>

namespace mxd {
namespace pipe {

struct JpegSource {
  mxd_jpeg_coefs* coefs;
  explicit JpegSource(mxd_jpeg_coefs* c) : coefs(c) {}
  ~JpegSource() { (void)mxd_jpeg_coefs_free(coefs); }
  JpegSource(const JpegSource&) = delete;
  JpegSource& operator=(const JpegSource&) = delete;
};

int64_t itemsize(DType t) {
  switch (t) {
    case DType::UInt8:
    case DType::Int8:
      return 1;
    case DType::Int32:
    case DType::Float:
      return 4;
    case DType::Int64:
    case DType::Double:
      return 8;
    default:
      return 0;
  }
}

namespace {

int64_t shape_size(const std::vector<int64_t>& s) {
  int64_t n = 1;
  for (auto d : s) n *= d;
  return n;
}

std::shared_ptr<void> alloc_bytes(int64_t n) {
  // 64-byte alignment: batch tensors are handed to numpy / torch as is.
  void* p = nullptr;
  if (posix_memalign(&p, 64, std::max<int64_t>(n, 1)) != 0) throw std::bad_alloc();
  return std::shared_ptr<void>(p, std::free);
}

// Image batch tensors (tens of MB each) come from a pool of page-locked
// blocks: the host path DMAs results straight into them (no staging copy-out)
// and a recycled block costs no page faults, where a fresh allocation of that
// size is first-touched page by page.  Blocks are recycled by size (the batch
// shape of a pipeline repeats); at most kMaxCached bytes wait unused.  Without
// a device (CPU-only runs) the pool turns itself off.
class BatchPool {
 public:
  std::shared_ptr<void> get(int64_t n) {
    const size_t cap = ((size_t)n + (1 << 20) - 1) & ~(size_t)((1 << 20) - 1);
    void* p = nullptr;
    {
      std::lock_guard<std::mutex> lk(mu_);
      if (off_) return nullptr;
      auto it = free_.find(cap);
      if (it != free_.end() && !it->second.empty()) {
        p = it->second.back();
        it->second.pop_back();
        cached_ -= cap;
      }
    }
    if (!p && mxd_malloc_pinned(&p, cap) != MXD_OK) {
      std::lock_guard<std::mutex> lk(mu_);
      off_ = true;
      return nullptr;
    }
    return std::shared_ptr<void>(p, [this, cap](void* q) { put(q, cap); });
  }

 private:
  static constexpr size_t kMaxCached = (size_t)2 << 30;
  // Returns a block; over the cap, blocks of OTHER sizes are freed first (a
  // pipeline whose batch shape changed keeps its new shape's blocks).
  void put(void* p, size_t cap) {
    std::vector<void*> drop;
    {
      std::lock_guard<std::mutex> lk(mu_);
      free_[cap].push_back(p);
      cached_ += cap;
      for (auto it = free_.begin(); cached_ > kMaxCached && it != free_.end(); ++it) {
        if (it->first == cap) continue;
        while (cached_ > kMaxCached && !it->second.empty()) {
          drop.push_back(it->second.back());
          it->second.pop_back();
          cached_ -= it->first;
        }
      }
      if (cached_ > kMaxCached) {
        drop.push_back(free_[cap].back());
        free_[cap].pop_back();
        cached_ -= cap;
      }
    }
    for (void* q : drop) (void)mxd_free_pinned(q);
  }
  std::mutex mu_;
  std::map<size_t, std::vector<void*>> free_;
  size_t cached_ = 0;
  bool off_ = false;
};

BatchPool& batch_pool() {
  static BatchPool* p = new BatchPool();  // never destroyed: outlives every Array
  return *p;
}

std::shared_ptr<void> alloc_batch_bytes(int64_t n) {
  if (n >= (4 << 20) && !devices().empty())
    if (auto p = batch_pool().get(n)) return p;
  return alloc_bytes(n);
}

void check(int rc) {
  if (rc != MXD_OK) throw std::runtime_error(mxd_last_error());
}

// ------------------------------------------------------------ device choice
std::mutex g_dev_mu;
std::vector<int> g_devices;
bool g_devices_set = false;
std::atomic<uint64_t> g_rr{0};

int next_device() {
  std::vector<int> d = devices();
  if (d.empty()) throw std::runtime_error("mxd: no HIP device visible (the image path runs only on the GPU)");
  return d[g_rr.fetch_add(1) % d.size()];
}

mxd_image plan_desc(const ImagePlan& p, void* dst, int64_t dst_stride) {
  const Array& s = *p.src;
  const int64_t c = s.shape(2);
  const int64_t stride = s.shape(1) * c;
  mxd_image d{};
  d.src = static_cast<const uint8_t*>(s.data()) + p.sy * stride + p.sx * c;
  d.src_stride = stride;
  d.src_w = (int32_t)p.sw;
  d.src_h = (int32_t)p.sh;
  d.channels = (int32_t)c;
  d.resize_w = (int32_t)p.resize_w;
  d.resize_h = (int32_t)p.resize_h;
  d.crop_x = (int32_t)p.crop_x;
  d.crop_y = (int32_t)p.crop_y;
  d.crop_w = (int32_t)p.crop_w;
  d.crop_h = (int32_t)p.crop_h;
  d.flip = p.flip ? 1 : 0;
  d.rgba_weighted = p.resampled && c == 4 ? 1 : 0;
  d.dst = dst;
  d.dst_stride = dst_stride;
  return d;
}

// An image plan and where its result goes.
struct Job {
  ImagePlan plan;
  void* dst;
  int64_t stride;
};

mxd_jpeg_image jpeg_desc(const ImagePlan& p, const JpegSource& j, void* dst, int64_t dst_stride) {
  mxd_jpeg_image d{};
  d.coefs = j.coefs;
  d.win_x = (int32_t)p.sx;
  d.win_y = (int32_t)p.sy;
  d.win_w = (int32_t)p.sw;
  d.win_h = (int32_t)p.sh;
  d.resize_w = (int32_t)p.resize_w;
  d.resize_h = (int32_t)p.resize_h;
  d.crop_x = (int32_t)p.crop_x;
  d.crop_y = (int32_t)p.crop_y;
  d.crop_w = (int32_t)p.crop_w;
  d.crop_h = (int32_t)p.crop_h;
  d.flip = p.flip ? 1 : 0;
  d.dst = dst;
  d.dst_stride = dst_stride;
  return d;
}

// One device's share of the jobs: plans over entropy-decoded JPEGs in one
// decode + resize call (the GPU finishes the decode), the rest in one resize
// call.  Returns the C ABI status (message in mxd_last_error()).
std::atomic<int64_t> g_run_calls{0}, g_run_jpeg{0};  // diagnostics (run_on_stats)

// Diagnostics (pipe_stats): ns summed over threads -- LoadImage::apply_key,
// every StreamTransform op (LoadImage included), StreamBatch's upstream
// fetches, its merge_batch, FromBuffer::next -- and the LoadImage count.
// One cache line of counters per thread (up to 64 lines, shared beyond), so
// prefetch workers do not contend on them.
struct alignas(64) PipeLine {
  std::atomic<int64_t> v[6];
};
PipeLine g_pipe_ns[64];
std::atomic<int> g_pipe_threads{0};
std::atomic<int64_t>* pipe_counters() {
  thread_local const int k = g_pipe_threads.fetch_add(1) & 63;
  return g_pipe_ns[k].v;
}
int64_t pipe_now() {
  return std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now().time_since_epoch())
      .count();
}
struct PipeTimer {
  int slot;
  int64_t t0 = pipe_now();
  explicit PipeTimer(int k) : slot(k) {}
  ~PipeTimer() { pipe_counters()[slot].fetch_add(pipe_now() - t0, std::memory_order_relaxed); }
};

int run_on(const Job* jobs, size_t n, int32_t dtype, int device, bool dst_device) {
  g_run_calls.fetch_add(1);
  std::vector<mxd_image> plain;
  std::vector<mxd_jpeg_image> jp;
  std::vector<std::shared_ptr<const JpegSource>> keep;  // alive for the call
  for (size_t i = 0; i < n; i++) {
    const Job& j = jobs[i];
    if (auto src = j.plan.src->jpeg()) {
      jp.push_back(jpeg_desc(j.plan, *src, j.dst, j.stride));
      keep.push_back(std::move(src));
    } else {
      plain.push_back(plan_desc(j.plan, j.dst, j.stride));
    }
  }
  g_run_jpeg.fetch_add((int64_t)jp.size());
  if (!jp.empty()) {
    const int rc = dst_device ? mxd_jpeg_resize_crop_to_device(jp.data(), (int32_t)jp.size(), dtype, device)
                              : mxd_jpeg_resize_crop_host(jp.data(), (int32_t)jp.size(), dtype, device);
    if (rc != MXD_OK) return rc;
  }
  if (plain.empty()) return MXD_OK;
  return dst_device ? mxd_resize_crop_to_device(plain.data(), (int32_t)plain.size(), dtype, device)
                    : mxd_resize_crop_host(plain.data(), (int32_t)plain.size(), dtype, device);
}

// Persistent host workers per device for the slices of split batches: a
// batch split over D devices hands D - 1 slices to the slice devices'
// workers (started on first use, at most kWorkersPerDevice each, matching the
// C ABI's per-device host-path contexts) instead of spawning threads per
// batch.  Workers live for the process (never joined: no teardown-order
// hazards at exit).
class DeviceWorkers {
 public:
  static constexpr size_t kWorkersPerDevice = 4;
  std::future<std::string> submit(int device, std::function<std::string()> fn) {
    auto task = std::make_shared<std::packaged_task<std::string()>>(std::move(fn));
    std::future<std::string> f = task->get_future();
    Dev* d;
    {
      std::lock_guard<std::mutex> lk(mu_);
      std::unique_ptr<Dev>& slot = devs_[device];
      if (!slot) slot = std::make_unique<Dev>();
      d = slot.get();
    }
    {
      std::lock_guard<std::mutex> lk(d->mu);
      d->q.push_back([task] { (*task)(); });
      // one more worker while every started one is busy (up to the cap)
      if (d->idle == 0 && d->threads < kWorkersPerDevice) {
        d->threads++;
        std::thread([d] { d->loop(); }).detach();
      }
    }
    d->cv.notify_one();
    return f;
  }

 private:
  struct Dev {
    std::mutex mu;
    std::condition_variable cv;
    std::deque<std::function<void()>> q;
    size_t threads = 0, idle = 0;
    void loop() {
      for (;;) {
        std::function<void()> t;
        {
          std::unique_lock<std::mutex> lk(mu);
          idle++;
          cv.wait(lk, [&] { return !q.empty(); });
          idle--;
          t = std::move(q.front());
          q.pop_front();
        }
        t();
      }
    }
  };
  std::mutex mu_;
  std::map<int, std::unique_ptr<Dev>> devs_;
};

DeviceWorkers& device_workers() {
  static DeviceWorkers* w = new DeviceWorkers();  // leaked on purpose: outlives static teardown
  return *w;
}

}  // namespace

// Slices of an n-image batch over `ndev` devices, starting at device index
// `first` (round-robin counter): a batch whose per-device slice would hold
// fewer than kMinSliceImages images is not split -- the whole batch goes to
// one device and consecutive batches rotate over the devices (Caltech's batch
// 32 on 8 GPUs: 8 prefetch workers, each batch one call on its own device,
// instead of every batch as 8 synchronous calls of 4 images); larger batches
// are cut into contiguous slices [s n / k, (s + 1) n / k) (op/Shard.cpp:11-20's
// contiguous split; the order of the batch is kept), k = min(ndev,
// n / kMinSliceImages) (C4's 1024 over 8 GPUs: 8 slices of 128).
std::vector<Slice> split_batch(int64_t n, int64_t ndev, uint64_t first) {
  std::vector<Slice> out;
  if (n <= 0 || ndev <= 0) return out;
  const int64_t k = std::max<int64_t>(1, std::min<int64_t>(ndev, n / kMinSliceImages));
  for (int64_t s = 0; s < k; s++)
    out.push_back(Slice{(int64_t)((first + (uint64_t)s) % (uint64_t)ndev), s * n / k, (s + 1) * n / k});
  return out;
}

namespace {

// Runs the jobs into host destinations (one fused launch per device and
// source kind) over split_batch's slices: slice 0 on the calling thread, the
// others on their devices' persistent workers; the first failing slice's
// message wins.
void run_host(const std::vector<Job>& jobs, int32_t dtype) {
  if (jobs.empty()) return;
  const std::vector<int> devs = devices();
  if (devs.empty()) throw std::runtime_error("mxd: no HIP device visible (the image path runs only on the GPU)");
  const size_t n = jobs.size();
  const size_t k = (size_t)std::max<int64_t>(1, std::min<int64_t>((int64_t)devs.size(), (int64_t)n / kMinSliceImages));
  const std::vector<Slice> sl = split_batch((int64_t)n, (int64_t)devs.size(), g_rr.fetch_add(k));
  if (sl.size() == 1) {
    check(run_on(jobs.data(), n, dtype, devs[sl[0].device], false));
    return;
  }
  auto slice = [&jobs, dtype, &devs, &sl](size_t s) -> std::string {
    if (run_on(jobs.data() + sl[s].begin, (size_t)(sl[s].end - sl[s].begin), dtype, devs[sl[s].device], false) !=
        MXD_OK)
      return mxd_last_error();  // thread-local: read on the failing thread
    return std::string();
  };
  std::vector<std::future<std::string>> pending;
  for (size_t s = 1; s < sl.size(); s++)
    pending.push_back(device_workers().submit(devs[sl[s].device], [&slice, s] { return slice(s); }));
  std::string err;
  try {
    err = slice(0);
  } catch (const std::exception& ex) {  // still wait: the slices read `jobs`
    err = ex.what();
  }
  for (auto& f : pending) {
    std::string e = f.get();  // every slice done before `jobs` goes out of scope
    if (err.empty()) err = std::move(e);
  }
  if (!err.empty()) throw std::runtime_error(err);
}

int32_t out_dtype(DType t) { return t == DType::Float ? MXD_F32_DIV255 : MXD_U8; }

std::atomic<int> g_device_decode{-1};  // -1: not set (on when a device is visible)

}  // namespace

void set_device_decode(bool on) { g_device_decode.store(on ? 1 : 0); }

std::atomic<bool> g_device_entropy{true};
void set_device_entropy(bool on) { g_device_entropy.store(on); }
bool device_entropy() { return g_device_entropy.load(); }

bool device_decode() {
  const int v = g_device_decode.load();
  return v < 0 ? !devices().empty() : v == 1;
}

int64_t ImagePlan::channels() const { return src->shape(2); }

// ------------------------------------------------------------------ Array
Array::Array(DType type, std::vector<int64_t> shape) : type_(type), shape_(std::move(shape)) {
  if (type_ == DType::Any && size() != 0) throw std::runtime_error("Array: cannot create a tensor of undetermined type");
  if (size() > 0) {
    data_ = alloc_bytes(nbytes());
    std::memset(data_.get(), 0, nbytes());
  }
}

Array::Array(DType type, std::vector<int64_t> shape, std::shared_ptr<void> data)
    : type_(type), shape_(std::move(shape)), data_(std::move(data)) {}

Array::Array(DType type, std::vector<int64_t> shape, std::shared_ptr<void> data, int device)
    : type_(type), shape_(std::move(shape)), data_(std::move(data)), device_(device) {}

Array::Array(std::shared_ptr<const ImagePlan> plan)
    : type_(plan->f32 ? DType::Float : DType::UInt8),
      shape_({plan->crop_h, plan->crop_w, plan->channels()}),
      plan_(std::move(plan)) {}

Array::Array(std::shared_ptr<const JpegSource> jpeg, int64_t height, int64_t width)
    : type_(DType::UInt8), shape_({height, width, 3}), jpeg_(std::move(jpeg)) {}

std::shared_ptr<const JpegSource> Array::jpeg() const {
  std::lock_guard<std::mutex> lk(mu_);
  return data_ ? nullptr : jpeg_;
}

int64_t Array::shape(int d) const {
  if (d < 0) d += ndim();
  if (d < 0 || d >= ndim()) throw std::runtime_error("Array: out of bound dimension");
  return shape_[d];
}

int64_t Array::size() const { return shape_size(shape_); }

bool Array::pending() const {
  std::lock_guard<std::mutex> lk(mu_);
  return plan_ && !data_;
}

void* Array::data() const {
  std::lock_guard<std::mutex> lk(mu_);
  if (!data_ && plan_) {
    auto buf = alloc_bytes(nbytes());
    const int64_t row = shape_[1] * shape_[2] * itemsize(type_);
    run_host({Job{*plan_, buf.get(), row}}, out_dtype(type_));
    data_ = buf;
  }
  if (!data_ && jpeg_) {
    // host finish of a lazy decode read directly
    auto buf = alloc_bytes(nbytes());
    check(mxd_jpeg_coefs_finish(jpeg_->coefs, static_cast<uint8_t*>(buf.get()), shape_[1] * 3));
    data_ = buf;
    jpeg_.reset();
  }
  return data_.get();
}

std::shared_ptr<Array> check_key(const Sample& s, const std::string& key) {
  auto it = s.find(key);
  if (it == s.end()) throw std::runtime_error("key <" + key + "> expected");
  return it->second;
}

void set_devices(const std::vector<int>& d) {
  std::lock_guard<std::mutex> lk(g_dev_mu);
  g_devices = d;
  g_devices_set = true;
}

std::vector<int> devices() {
  std::lock_guard<std::mutex> lk(g_dev_mu);
  if (!g_devices_set) {
    int n = 0;
    if (mxd_device_count(&n) != MXD_OK) n = 0;
    g_devices.clear();
    for (int i = 0; i < n; i++) g_devices.push_back(i);
    g_devices_set = true;
  }
  return g_devices;
}

// ------------------------------------------------------------------ state
// core/State.cpp:9-22: a global generator; each thread takes a copy of it
// whenever set_state() bumped the version.
namespace {
State g_state{std::mt19937(), 0};
std::mutex g_state_mu;
}  // namespace

void set_state(int64_t seed) {
  std::lock_guard<std::mutex> lk(g_state_mu);
  g_state.gen = std::mt19937(seed);
  g_state.version++;
}

std::shared_ptr<State> get_state() {
  static thread_local std::shared_ptr<State> st;
  std::lock_guard<std::mutex> lk(g_state_mu);
  if (!st || st->version != g_state.version) st = std::make_shared<State>(g_state);
  return st;
}

// ------------------------------------------------------------------ ops
Sample KeyTransformOp::apply(const Sample& sample) const {
  auto x = check_key(sample, ikey_);
  Sample res = sample;
  res[okey_.empty() ? ikey_ : okey_] = apply_key(x);
  return res;
}

namespace {

// The image (H, W, C) as a plan: a pending one as is, a materialised one as
// the identity plan over all of it.
ImagePlan view(const std::shared_ptr<Array>& img) {
  if (img->type() != DType::UInt8) throw std::invalid_argument("image must be of type UInt8");
  if (img->plan() && img->pending()) return *img->plan();
  ImagePlan p;
  p.src = img;
  p.sw = p.resize_w = p.crop_w = img->shape(1);
  p.sh = p.resize_h = p.crop_h = img->shape(0);
  return p;
}

void verify_dimensions(int64_t w, int64_t h, int64_t c) {
  // core/image/ImageTransform.cpp:23-31
  if (h <= 0 || w <= 0) throw std::runtime_error("image: cannot create image with 0 or negative dimension");
  if (c <= 0 || c > 4) throw std::runtime_error("image: channels must be 0 < c <= 4");
}

std::shared_ptr<Array> make(const ImagePlan& p) { return std::make_shared<Array>(std::make_shared<const ImagePlan>(p)); }

// core::image::resize (core/image/ImageTransform.cpp:41-62).
std::shared_ptr<Array> plan_resize(const std::shared_ptr<Array>& img, int64_t dw, int64_t dh) {
  verify_dimensions(dw, dh, img->shape(2));
  ImagePlan p = view(img);
  // (an alpha-weighted same-size resize is not the identity: it zeroes the
  // colour of transparent pixels, so it runs before the next one)
  const bool identity_so_far =
      p.resize_w == p.sw && p.resize_h == p.sh && !p.flip && !(p.resampled && p.channels() == 4);
  if (identity_so_far) {
    // crop-then-resize: the crop becomes the source window.
    p.sx += p.crop_x;
    p.sy += p.crop_y;
    p.sw = p.crop_w;
    p.sh = p.crop_h;
  } else {
    // resize of a resized (or mirrored) image: run the first one, resample
    // its output.
    img->data();
    p = view(img);
  }
  p.resize_w = p.crop_w = dw;
  p.resize_h = p.crop_h = dh;
  p.crop_x = p.crop_y = 0;
  p.flip = false;
  p.resampled = true;
  return make(p);
}

// core::image::crop -> array::sub (Array.cpp:544-583), in the coordinates of
// the current view.
std::shared_ptr<Array> plan_crop(const std::shared_ptr<Array>& img, int64_t x, int64_t y, int64_t w, int64_t h) {
  verify_dimensions(w, h, 3);
  const int64_t W = img->shape(1), H = img->shape(0);
  if (y < 0 || x < 0 || y >= H || x >= W) throw std::runtime_error("Array: sub: offset out of bound");
  if (y + h > H || x + w > W) throw std::runtime_error("Array: sub: shape out of bound");
  if (img->type() != DType::UInt8) {
    // Not the image path (the resize kernel is uint8 only, like the
    // reference's resize): a plain strided sub-array copy.
    const int64_t c = img->ndim() > 2 ? img->shape(2) : 1, isz = itemsize(img->type());
    auto out = std::make_shared<Array>(img->type(), std::vector<int64_t>{h, w, c});
    const auto* s = static_cast<const uint8_t*>(img->data());
    auto* d = static_cast<uint8_t*>(out->data());
    for (int64_t r = 0; r < h; r++) std::memcpy(d + r * w * c * isz, s + ((y + r) * W + x) * c * isz, w * c * isz);
    return out;
  }
  ImagePlan p = view(img);
  p.crop_x = p.flip ? p.crop_x + p.crop_w - x - w : p.crop_x + x;
  p.crop_y += y;
  p.crop_w = w;
  p.crop_h = h;
  return make(p);
}

}  // namespace

// op/ImageTransform.cpp:22-31 + core/image/ImageIO.cpp:39-49 + core/video/Video.cpp:69-79
std::shared_ptr<Array> ImageOp::apply_key(const std::shared_ptr<Array>& x) const {
  if (x->device() >= 0) throw std::runtime_error("image: device-resident array (batch(..., device=)) expected on host");
  if (x->ndim() == 4) {
    if (x->shape(3) == 0 || x->shape(3) > 4) throw std::runtime_error("verifyVideo: channels must be 0 <= c <= 4");
    return apply_video(x);
  }
  if (x->ndim() != 3) throw std::runtime_error("verifyImage: image must be 3 dimension Array (HWC)");
  if (x->shape(2) == 0 || x->shape(2) > 4) throw std::runtime_error("verifyImage: channels must be 0 <= c <= 4");
  return apply_image(x);
}

std::shared_ptr<Array> video_frame(const std::shared_ptr<Array>& video, int64_t i) {
  const int64_t h = video->shape(1), w = video->shape(2), c = video->shape(3);
  const int64_t bytes = h * w * c * itemsize(video->type());
  auto* base = static_cast<uint8_t*>(video->data()) + i * bytes;
  return std::make_shared<Array>(video->type(), std::vector<int64_t>{h, w, c},
                                 std::shared_ptr<void>(video, static_cast<void*>(base)));
}

std::shared_ptr<Array> stack_frames(const std::vector<std::shared_ptr<Array>>& frames) {
  const auto& f0 = frames.at(0);
  const int64_t h = f0->shape(0), w = f0->shape(1), c = f0->shape(2);
  for (const auto& f : frames)
    if (f->shape(0) != h || f->shape(1) != w)
      throw std::runtime_error("applyVideo: frame size inconsistent during transform");
  auto out = std::make_shared<Array>(f0->type(), std::vector<int64_t>{(int64_t)frames.size(), h, w, c});
  const int64_t isz = itemsize(f0->type()), bytes = h * w * c * isz;
  auto* dst = static_cast<uint8_t*>(out->data());
  std::vector<Job> jobs;
  for (size_t i = 0; i < frames.size(); i++) {
    const auto& f = frames[i];
    if (f->type() != f0->type()) throw std::runtime_error("applyVideo: frame type inconsistent during transform");
    if (f->plan() && f->pending())
      jobs.push_back(Job{*f->plan(), dst + i * bytes, w * c * isz});
    else
      std::memcpy(dst + i * bytes, f->data(), bytes);
  }
  run_host(jobs, out_dtype(f0->type()));  // every pending frame in one launch
  return out;
}

std::shared_ptr<Array> ImageOp::apply_video(const std::shared_ptr<Array>& video) const {
  std::vector<std::shared_ptr<Array>> frames;
  for (int64_t i = 0; i < video->shape(0); i++) frames.push_back(apply_image(video_frame(video, i)));
  if (frames.empty()) throw std::runtime_error("applyVideo: empty video");
  return stack_frames(frames);
}

// op/ImageTransform.cpp:78-94 + core::image::scale :33-39
std::shared_ptr<Array> ImageResizeSmallestSide::apply_image(const std::shared_ptr<Array>& img) const {
  if (size_ <= 0) throw std::runtime_error("ImageResizeSmallestSide: illegal target size: " + std::to_string(size_));
  const int64_t w = img->shape(1), h = img->shape(0);
  const double scale = h > w ? (double)size_ / w : (double)size_ / h;
  return plan_resize(img, std::lround(scale * w), std::lround(scale * h));
}

// op/ImageTransform.cpp:103-106
std::shared_ptr<Array> ImageResize::apply_image(const std::shared_ptr<Array>& img) const {
  return plan_resize(img, w_, h_);
}

// op/ImageTransform.cpp:115-126
std::shared_ptr<Array> ImageCenterCrop::apply_image(const std::shared_ptr<Array>& img) const {
  const int64_t w = img->shape(1), h = img->shape(0);
  if (h_ > h || w_ > w) throw std::runtime_error("ImageCenterCrop: target image size larger than input image");
  return plan_crop(img, (w - w_) / 2, (h - h_) / 2, w_, h_);
}

// op/ImageTransform.cpp:135-158 (x drawn before y, int64 uniform ints)
std::shared_ptr<Array> ImageRandomCrop::apply_image(const std::shared_ptr<Array>& img) const {
  const int64_t w = img->shape(1), h = img->shape(0);
  if (h_ > h || w_ > w) throw std::runtime_error("ImageRandomCrop: target image size larger than input image");
  std::uniform_int_distribution<int64_t> xu{0, w - w_};
  std::uniform_int_distribution<int64_t> yu{0, h - h_};
  auto st = get_state();
  const int64_t x = xu(st->gen);
  const int64_t y = yu(st->gen);
  return plan_crop(img, x, y, w_, h_);
}

// op/ImageTransform.cpp:160-182: one draw, the same window for every frame
std::shared_ptr<Array> ImageRandomCrop::apply_video(const std::shared_ptr<Array>& video) const {
  const int64_t w = video->shape(2), h = video->shape(1);
  if (h_ > h || w_ > w) throw std::runtime_error("ImageRandomCrop: target image size larger than input image");
  std::uniform_int_distribution<int64_t> xu{0, w - w_};
  std::uniform_int_distribution<int64_t> yu{0, h - h_};
  auto st = get_state();
  const int64_t x = xu(st->gen);
  const int64_t y = yu(st->gen);
  if (w_ == 0 || h_ == 0) return video;
  std::vector<std::shared_ptr<Array>> frames;
  for (int64_t i = 0; i < video->shape(0); i++) frames.push_back(plan_crop(video_frame(video, i), x, y, w_, h_));
  return stack_frames(frames);
}

// op/ImageTransform.cpp:334-356: one draw, every frame mirrored or none
std::shared_ptr<Array> ImageRandomHFlip::apply_video(const std::shared_ptr<Array>& video) const {
  std::uniform_real_distribution<float> u{0, 1.0};
  auto st = get_state();
  if (!(u(st->gen) <= prob_)) return video;
  std::vector<std::shared_ptr<Array>> frames;
  for (int64_t i = 0; i < video->shape(0); i++) {
    auto f = video_frame(video, i);
    verify_dimensions(f->shape(1), f->shape(0), f->shape(2));
    ImagePlan p = view(f);
    p.flip = !p.flip;
    frames.push_back(make(p));
  }
  return stack_frames(frames);
}

// op/ImageTransform.cpp:323-332 + core::image::hflip :123-140
std::shared_ptr<Array> ImageRandomHFlip::apply_image(const std::shared_ptr<Array>& img) const {
  std::uniform_real_distribution<float> u{0, 1.0};
  auto st = get_state();
  if (u(st->gen) <= prob_) {
    verify_dimensions(img->shape(1), img->shape(0), img->shape(2));
    ImagePlan p = view(img);
    p.flip = !p.flip;
    return make(p);
  }
  return img;
}

std::shared_ptr<Array> ImageToFloat::apply_image(const std::shared_ptr<Array>& img) const {
  verify_dimensions(img->shape(1), img->shape(0), img->shape(2));
  ImagePlan p = view(img);
  p.f32 = true;
  return make(p);
}

namespace {
// A materialised, contiguous (H, W, C) uint8 image through one pixel-map
// launch on the next device.
std::shared_ptr<Array> run_pixmap(const std::shared_ptr<Array>& img, int32_t op, const float* params, int64_t dw,
                                  int64_t dh, int64_t dc) {
  if (img->type() != DType::UInt8) throw std::invalid_argument("image must be of type UInt8");
  const int64_t w = img->shape(1), h = img->shape(0), c = img->shape(2);
  auto out = std::make_shared<Array>(DType::UInt8, std::vector<int64_t>{dh, dw, dc});
  mxd_pixmap d{};
  d.src = static_cast<const uint8_t*>(img->data());
  d.src_stride = w * c;
  d.src_w = (int32_t)w;
  d.src_h = (int32_t)h;
  d.channels = (int32_t)c;
  d.dst_w = (int32_t)dw;
  d.dst_h = (int32_t)dh;
  d.dst = out->data();
  d.dst_stride = dw * dc;
  for (int k = 0; k < 6; k++) d.params[k] = params[k];
  check(mxd_pixmap_host(&d, 1, op, next_device()));
  return out;
}
}  // namespace

// op/ImageTransform.cpp:334-343 -> core/image/ImageTransform.cpp:75-121
std::shared_ptr<Array> ImageRotate::apply_image(const std::shared_ptr<Array>& img) const {
  const int64_t w = img->shape(1), h = img->shape(0), c = img->shape(2);
  float mx[6];
  int64_t tw = 0, th = 0;
  (void)mxd_rotate_geometry(w, h, angle_, crop_ ? 1 : 0, mx, &tw, &th);  // dims are set even when invalid
  verify_dimensions(tw, th, c);
  return run_pixmap(img, MXD_AFFINE, mx, tw, th, c);
}

// op/ImageTransform.cpp:394-421 -> core/image/ImageTransform.cpp:142-180
ImageChannelReduction::ImageChannelReduction(std::string ikey, const std::string& preset, std::string okey)
    : ImageOp(std::move(ikey), std::move(okey)) {
  if (mxd_channel_reduction_preset(preset.c_str(), params_) != MXD_OK)
    throw std::runtime_error(std::string("ImageChannelReduction: unable to find preset ") + preset);
}

std::shared_ptr<Array> ImageChannelReduction::apply_image(const std::shared_ptr<Array>& img) const {
  const int64_t w = img->shape(1), h = img->shape(0), c = img->shape(2);
  if (c != 3) throw std::runtime_error("image::channelReduction: expected a 3 channel uint8 array");
  verify_dimensions(w, h, 1);
  const float p[6] = {params_[0], params_[1], params_[2], params_[3], 0, 0};
  return run_pixmap(img, MXD_CHANNEL_REDUCTION, p, w, h, 1);
}

// op/ImageTransform.cpp:184-212 (constructor checks, same messages)
ImageRandomAreaCrop::ImageRandomAreaCrop(std::string ikey, std::pair<float, float> area_range,
                                         std::pair<float, float> aspect_ratio_range, int num_trial, std::string okey)
    : ImageOp(std::move(ikey), std::move(okey)), area_(area_range), aspect_(aspect_ratio_range), trials_(num_trial) {
  const char* bad = nullptr;
  if (area_.first <= 0 || area_.first > area_.second || area_.second > 1.0)
    bad = "ImageRandomAreaCrop: invalid area range";
  else if (aspect_.first <= 0 || aspect_.first > aspect_.second)
    bad = "ImageRandomAreaCrop: invalid aspect ratio range";
  else if (area_.first * aspect_.first > 1 || area_.first > aspect_.second)
    bad = "ImageRandomAreaCrop: provided area range and aspect ratio range cannot be fullfilled";
  else if (trials_ <= 0)
    bad = "ImageRandomAreaCrop: number of trial must be positive";
  if (bad) throw std::runtime_error(bad);
}

// op/ImageTransform.cpp:214-280 (generate_random_crop_).  The arithmetic keeps
// the reference's types step for step -- float ranges times float image sizes,
// int64 draws from std::uniform_int_distribution on the thread's mt19937 --
// so the draws and the accept/reject decisions are the same.  Order of draws:
// per trial a width, then (if its height range is non-empty) a height; after
// the trials x, then y.
std::array<int64_t, 4> ImageRandomAreaCrop::draw(int64_t w, int64_t h) const {
  const std::array<int64_t, 4> none{0, 0, 0, 0};
  if (w == 0 || h == 0) return none;
  const float fw = static_cast<float>(w), fh = static_cast<float>(h);
  const float ratio = fw / fh;
  auto st = get_state();
  const int64_t lo_w = std::ceil(std::sqrt(area_.first * aspect_.first) * fw);
  const int64_t hi_w = std::floor(std::min(std::sqrt(area_.second * aspect_.second) * fw, fw));
  if (lo_w > hi_w) return none;
  std::uniform_int_distribution<int64_t> wdist{lo_w, hi_w};
  int64_t cw = 0, ch = 0;
  for (int t = 0; t < trials_; t++) {
    cw = wdist(st->gen);
    const float h_by_aspect_lo = 1.0f / (ratio * aspect_.second) * cw;
    const float h_by_aspect_hi = 1.0f / (ratio * aspect_.first) * cw;
    const float h_by_area_lo = area_.first * fw * fh / cw;
    const float h_by_area_hi = area_.second * fw * fh / cw;
    const int64_t lo_h = std::ceil(std::max(h_by_aspect_lo, h_by_area_lo));
    const int64_t hi_h = std::floor(std::min(std::min(h_by_aspect_hi, h_by_area_hi), fh));
    if (lo_h > hi_h) continue;
    ch = std::uniform_int_distribution<int64_t>{lo_h, hi_h}(st->gen);
    const float crop_ratio = static_cast<float>(cw) / static_cast<float>(ch);
    const bool area_ok = !(area_.first * w * h > cw * ch) && !(area_.second * w * h < cw * ch);
    const bool aspect_ok = !(aspect_.first * ratio > crop_ratio) && !(aspect_.second * ratio < crop_ratio);
    if (area_ok && aspect_ok && cw > 0 && cw <= w && ch > 0 && ch <= h) break;
  }
  if (cw == 0 || ch == 0) return none;
  const int64_t x = std::uniform_int_distribution<int64_t>{0, w - cw}(st->gen);
  const int64_t y = std::uniform_int_distribution<int64_t>{0, h - ch}(st->gen);
  return {x, y, cw, ch};
}

// op/ImageTransform.cpp:282-291
std::shared_ptr<Array> ImageRandomAreaCrop::apply_image(const std::shared_ptr<Array>& img) const {
  const auto c = draw(img->shape(1), img->shape(0));
  if (c[2] == 0 || c[3] == 0) return img;
  return plan_crop(img, c[0], c[1], c[2], c[3]);
}

// op/ImageTransform.cpp:293-315: one draw, the same window for every frame
std::shared_ptr<Array> ImageRandomAreaCrop::apply_video(const std::shared_ptr<Array>& video) const {
  const auto c = draw(video->shape(2), video->shape(1));
  if (c[2] == 0 || c[3] == 0) return video;
  std::vector<std::shared_ptr<Array>> frames;
  for (int64_t i = 0; i < video->shape(0); i++) frames.push_back(plan_crop(video_frame(video, i), c[0], c[1], c[2], c[3]));
  return stack_frames(frames);
}

// ------------------------------------------------------------------ load
namespace {
std::mutex g_dec_mu;
ImageDecoder g_decoder;
}  // namespace

void set_image_decoder(ImageDecoder dec) {
  std::lock_guard<std::mutex> lk(g_dec_mu);
  g_decoder = std::move(dec);
}

LoadImage::LoadImage(std::string ikey, std::string prefix, bool info, std::string format, bool from_memory,
                     std::string okey)
    : KeyTransformOp(std::move(ikey), std::move(okey)),
      prefix_(std::move(prefix)),
      info_(info),
      format_(std::move(format)),
      from_memory_(from_memory) {}

namespace {
// File reads with POSIX calls straight into a buffer sized from fstat: the
// earlier stdio loop (64 KB chunks appended to a growing vector, after a
// separate open for the signature) cost several times the read itself on an
// 80 KB JPEG.
struct Fd {
  int fd;
  explicit Fd(const std::string& path) : fd(::open(path.c_str(), O_RDONLY | O_CLOEXEC)) {}
  ~Fd() {
    if (fd >= 0) ::close(fd);
  }
  Fd(const Fd&) = delete;
  Fd& operator=(const Fd&) = delete;
};

// Appends the file's bytes from the current offset to *out until EOF or until
// *out holds `limit` bytes; false on a read error.  A regular file is read to
// the size fstat gives; anything else until read() returns 0.
bool read_to(int fd, size_t limit, std::vector<uint8_t>* out) {
  struct stat st;
  const bool regular = ::fstat(fd, &st) == 0 && S_ISREG(st.st_mode);
  size_t got = out->size();
  const size_t want = regular ? std::min(limit, std::max(got, (size_t)st.st_size)) : limit;
  if (regular) out->resize(want);
  while (got < limit) {
    if (got == out->size()) {
      if (regular) break;  // fstat's size reached
      out->resize(std::min(limit, got + std::max<size_t>(got, 1 << 16)));
    }
    const ssize_t r = ::read(fd, out->data() + got, out->size() - got);
    if (r < 0) {
      if (errno == EINTR) continue;
      return false;
    }
    if (r == 0) break;
    got += (size_t)r;
  }
  out->resize(got);
  return true;
}

// The whole file (the reference's check_signature fopen failure message).
std::vector<uint8_t> read_file(const std::string& path) {
  Fd f(path);
  std::vector<uint8_t> data;
  if (f.fd < 0 || !read_to(f.fd, SIZE_MAX, &data)) throw std::runtime_error("load_jpeg: could not load <" + path + ">");
  return data;
}

// Up to `n` leading bytes of a file; false when it cannot be opened.
bool read_prefix(const std::string& path, size_t n, std::vector<uint8_t>* out) {
  Fd f(path);
  out->clear();
  return f.fd >= 0 && read_to(f.fd, n, out);
}

// libjpeg's message without the C ABI's "load_jpeg: " prefix.
std::string jpeg_error() {
  std::string m = mxd_last_error();
  const std::string pre = "load_jpeg: ";
  return m.compare(0, pre.size(), pre) == 0 ? m.substr(pre.size()) : m;
}
}  // namespace

// op/LoadImage.cpp:23-48 -> core/image/ImageIO.cpp:10-24: JPEG (signature
// FF D8 FF) through the native decoder (ImageJPEG.cpp:99-232 semantics),
// anything else through the installed stb_image-rules hook.
std::shared_ptr<Array> LoadImage::apply_key(const std::shared_ptr<Array>& x) const {
  PipeTimer timer(0);
  pipe_counters()[5].fetch_add(1, std::memory_order_relaxed);
  if (x->device() >= 0) throw std::runtime_error("LoadImage: device-resident array expected on host");
  std::string path;
  if (!from_memory_) {
    if (x->type() != DType::Int8) throw std::runtime_error("LoadImage: char array (int8) expected");
    std::string filename(static_cast<const char*>(x->data()), x->size());
    path = prefix_;
    if (!filename.empty() && filename[0] == '/') path = filename;  // std::filesystem::path operator/
    else if (!path.empty()) path = (path.back() == '/' ? path : path + "/") + filename;
    else path = filename;
  }
  // The deferred image of a parsed JPEG (the GPU finishes it in the batch).
  auto deferred = [](mxd_jpeg_coefs* c) {
    auto src = std::make_shared<const JpegSource>(c);
    int32_t cw = 0, ch = 0, dev_ok = 0;
    check(mxd_jpeg_coefs_info(c, &cw, &ch, &dev_ok));
    auto out = std::make_shared<Array>(src, ch, cw);
    if (!dev_ok) out->data();  // CMYK / YCCK: the host finishes it now
    return out;
  };
  if (!from_memory_ && !info_ && device_decode()) {
    // the file read straight into the parsed handle; anything unusual (not
    // readable, not a regular file, a parse error) takes the general path
    // below, which gives the reference's messages
    mxd_jpeg_coefs* c = nullptr;
    if (mxd_jpeg_coefs_load(path.c_str(), device_entropy() ? 1 : 0, &c) == MXD_OK) {
      if (c) return deferred(c);
      goto not_jpeg;
    }
  }
  {
    std::vector<uint8_t> file;
    const uint8_t* bytes = nullptr;
    size_t nbytes = 0;
    if (from_memory_) {
      bytes = static_cast<const uint8_t*>(x->data());
      nbytes = (size_t)x->nbytes();
    } else if (info_) {
      // core::image::info -> stbi_info (ImageIO.cpp:26-32): the header only;
      // (0, 0) when the file cannot be opened or parsed.  A JPEG's frame header
      // follows its APP segments, so a short prefix is read first.
      constexpr size_t kHead = 1 << 18;
      if (!read_prefix(path, kHead, &file)) {
        auto out = std::make_shared<Array>(DType::Int64, std::vector<int64_t>{2});
        static_cast<int64_t*>(out->data())[0] = static_cast<int64_t*>(out->data())[1] = 0;
        return out;
      }
      int32_t w = 0, h = 0, c = 0;
      if (mxd_is_jpeg(file.data(), file.size()) && file.size() == kHead &&
          mxd_jpeg_info(file.data(), file.size(), &w, &h, &c) != MXD_OK)
        file = read_file(path);  // frame header past the prefix
      bytes = file.data();
      nbytes = file.size();
    } else {
      // load_jpeg's signature check (ImageJPEG.cpp:74-86) first: only JPEGs are
      // read here, anything else goes to the stb_image hook by path.
      // One open: the signature, then (a JPEG) the rest of the file.
      Fd f(path);
      if (f.fd < 0 || !read_to(f.fd, 3, &file)) throw std::runtime_error("load_jpeg: could not load <" + path + ">");
      if (mxd_is_jpeg(file.data(), file.size())) {
        if (!read_to(f.fd, SIZE_MAX, &file)) throw std::runtime_error("load_jpeg: could not load <" + path + ">");
        bytes = file.data();
        nbytes = file.size();
      }
    }
    const std::string where = from_memory_ ? std::string("from memory") : "<" + path + ">";
    if (bytes && mxd_is_jpeg(bytes, nbytes)) {
      int32_t w = 0, h = 0, c = 0;
      const bool ok = mxd_jpeg_info(bytes, nbytes, &w, &h, &c) == MXD_OK;
      if (info_) {
        // stbi_info: (w, h), zeros when the header cannot be read
        auto out = std::make_shared<Array>(DType::Int64, std::vector<int64_t>{2});
        static_cast<int64_t*>(out->data())[0] = ok ? w : 0;
        static_cast<int64_t*>(out->data())[1] = ok ? h : 0;
        return out;
      }
      if (!ok) throw std::runtime_error("load_jpeg: could not load " + where + " (" + jpeg_error() + ")");
      if (device_decode()) {
        // markers only (the Huffman decode too runs on the GPU, csrc/jpeghuff.hip)
        // when the file qualifies, else the entropy decode here; the GPU
        // finishes it in the batch launch
        mxd_jpeg_coefs* c = nullptr;
        if (mxd_jpeg_coefs_parse(bytes, nbytes, device_entropy() ? 1 : 0, &c) != MXD_OK)
          throw std::runtime_error("load_jpeg: could not load " + where + " (" + jpeg_error() + ")");
        return deferred(c);
      }
      auto out = std::make_shared<Array>(DType::UInt8, std::vector<int64_t>{h, w, 3}, alloc_bytes((int64_t)h * w * 3));
      if (mxd_jpeg_decode(bytes, nbytes, static_cast<uint8_t*>(out->data()), (int64_t)w * 3, w, h) != MXD_OK) {
        const std::string e = jpeg_error();
        throw std::runtime_error("load_jpeg: could not load " + where + " (" +
                                 (e == "unhandled format" ? e : e) + ")");
      }
      return out;
    }
  }
not_jpeg:
  ImageDecoder dec;
  {
    std::lock_guard<std::mutex> lk(g_dec_mu);
    dec = g_decoder;
  }
  if (!dec) throw std::runtime_error("LoadImage: no image decoder installed");
  auto out = dec(path, x, from_memory_, info_);
  if (!out) throw std::runtime_error("LoadImage: unable to load image <" + (from_memory_ ? std::string("stream") : path) + ">");
  return out;
}

// ------------------------------------------------------------------ batch
namespace {

// array_copy_linear_to_strided (Array.cpp:405-463): `src` (dense, shape
// `shape`) into `dst` at element offset `off` with per-dim strides `stride`.
void copy_to_strided(uint8_t* dst, int64_t off, const uint8_t* src, const std::vector<int64_t>& shape,
                     const std::vector<int64_t>& stride, int64_t isz) {
  const int nd = (int)shape.size();
  if (nd == 0) {
    std::memcpy(dst + off * isz, src, isz);
    return;
  }
  const int64_t run = shape[nd - 1] * isz;
  int64_t rows = 1;
  for (int d = 0; d < nd - 1; d++) rows *= shape[d];
  std::vector<int64_t> idx(std::max(nd - 1, 0), 0);
  for (int64_t r = 0; r < rows; r++) {
    int64_t o = off;
    for (int d = 0; d < nd - 1; d++) o += idx[d] * stride[d];
    std::memcpy(dst + o * isz, src + r * run, run);
    for (int d = nd - 2; d >= 0; d--) {
      if (++idx[d] < shape[d]) break;
      idx[d] = 0;
    }
  }
}

template <class T>
void fill_t(void* p, int64_t n, double v) {
  std::fill_n(static_cast<T*>(p), n, static_cast<T>(v));
}

void fill(Array& a, double v) {
  void* p = a.data();
  const int64_t n = a.size();
  switch (a.type()) {
    case DType::UInt8: fill_t<uint8_t>(p, n, v); break;
    case DType::Int8: fill_t<int8_t>(p, n, v); break;
    case DType::Int32: fill_t<int32_t>(p, n, v); break;
    case DType::Int64: fill_t<int64_t>(p, n, v); break;
    case DType::Float: fill_t<float>(p, n, v); break;
    case DType::Double: fill_t<double>(p, n, v); break;
    default: break;
  }
}

}  // namespace

namespace {
// An array whose pixels a batch launch produces: a pending plan, or a lazy
// JPEG decode (as the identity plan over it).
bool deferred(const Array& a) { return a.pending() || (a.type() == DType::UInt8 && a.jpeg()); }

ImagePlan deferred_plan(const std::shared_ptr<Array>& a) {
  if (a->plan() && a->pending()) return *a->plan();
  ImagePlan p;
  p.src = a;
  p.sw = p.resize_w = p.crop_w = a->shape(1);
  p.sh = p.resize_h = p.crop_h = a->shape(0);
  return p;
}

// Device batch tensors (batch(..., device=d)), recycled by size like
// BatchPool: a device allocation and its release (hipMalloc / hipFree, which
// waits for the whole device) per batch serialised the prefetch workers of a
// device pipeline.  A released block may still be read by work its consumer
// (e.g. torch through DLPack) enqueued on a stream of its own, so it is only
// reused after a device synchronisation that followed its release: blocks
// released since the last one wait in `pending`.  A request that finds no
// idle block of its size synchronises the device once and makes every
// pending block idle when a pending block has its size, or when the pending
// blocks hold more than half of kMaxCached (batches of changing shapes: their
// blocks would otherwise wait forever); idle blocks past kMaxCached are then
// freed, other sizes first.  So at most kMaxCached bytes (plus one block)
// stay cached per device, idle and pending together.
class DevicePool {
 public:
  std::shared_ptr<void> get(int device, int64_t n) {
    const size_t cap = ((size_t)std::max<int64_t>(n, 1) + (1 << 20) - 1) & ~(size_t)((1 << 20) - 1);
    void* p = take(device, cap);
    if (!p && must_drain(device, cap)) {
      std::vector<std::pair<size_t, void*>> now;
      {
        std::lock_guard<std::mutex> lk(mu_);
        Dev& d = devs_[device];
        now.swap(d.pending);
        d.pending_bytes = 0;
      }
      check(mxd_device_synchronize(device));  // everything released before this point is idle
      std::vector<void*> drop;
      {
        std::lock_guard<std::mutex> lk(mu_);
        Dev& d = devs_[device];
        for (auto& b : now) d.idle[b.first].push_back(b.second);
        evict(d, cap, &drop);
      }
      for (void* q : drop) (void)mxd_free_device(q, device);
      p = take(device, cap);
    }
    if (!p) check(mxd_malloc_device(&p, cap, device));
    return std::shared_ptr<void>(p, [this, device, cap](void* q) { put(device, q, cap); });
  }

  // Bytes the pool holds for `device` (idle + pending): tests bound it.
  size_t cached(int device) {
    std::lock_guard<std::mutex> lk(mu_);
    return devs_[device].cached;
  }

 private:
  static constexpr size_t kMaxCached = (size_t)2 << 30;
  struct Dev {
    std::map<size_t, std::vector<void*>> idle;
    std::vector<std::pair<size_t, void*>> pending;
    size_t cached = 0, pending_bytes = 0;
  };
  void* take(int device, size_t cap) {
    std::lock_guard<std::mutex> lk(mu_);
    Dev& d = devs_[device];
    auto it = d.idle.find(cap);
    if (it == d.idle.end() || it->second.empty()) return nullptr;
    void* p = it->second.back();
    it->second.pop_back();
    d.cached -= cap;
    return p;
  }
  bool must_drain(int device, size_t cap) {
    std::lock_guard<std::mutex> lk(mu_);
    const Dev& d = devs_[device];
    if (d.pending.empty()) return false;
    if (d.pending_bytes > kMaxCached / 2) return true;
    for (auto& b : d.pending)
      if (b.first == cap) return true;
    return false;
  }
  // Frees idle blocks (other sizes than `keep` first) while over the cap.
  static void evict(Dev& d, size_t keep, std::vector<void*>* drop) {
    for (int pass = 0; pass < 2 && d.cached > kMaxCached; pass++)
      for (auto it = d.idle.begin(); d.cached > kMaxCached && it != d.idle.end(); ++it) {
        if ((pass == 0) == (it->first == keep)) continue;
        while (d.cached > kMaxCached && !it->second.empty()) {
          drop->push_back(it->second.back());
          it->second.pop_back();
          d.cached -= it->first;
        }
      }
  }
  void put(int device, void* p, size_t cap) {
    std::vector<void*> drop;
    {
      std::lock_guard<std::mutex> lk(mu_);
      Dev& d = devs_[device];
      d.pending.emplace_back(cap, p);
      d.pending_bytes += cap;
      d.cached += cap;
      evict(d, cap, &drop);  // over the cap: idle blocks of other sizes go first
    }
    for (void* q : drop) (void)mxd_free_device(q, device);
  }
  std::mutex mu_;
  std::map<int, Dev> devs_;
};

DevicePool& device_pool() {
  static DevicePool* p = new DevicePool();  // leaked on purpose: outlives static teardown
  return *p;
}

}  // namespace

size_t device_pool_bytes(int device) { return device_pool().cached(device); }

std::vector<int64_t> pipe_stats(bool reset) {
  std::vector<int64_t> r(6, 0);
  for (PipeLine& l : g_pipe_ns)
    for (int i = 0; i < 6; i++) r[i] += reset ? l.v[i].exchange(0) : l.v[i].load();
  return r;
}

std::pair<int64_t, int64_t> run_on_stats(bool reset) {
  const std::pair<int64_t, int64_t> r{g_run_calls.load(), g_run_jpeg.load()};
  if (reset) {
    g_run_calls = 0;
    g_run_jpeg = 0;
  }
  return r;
}

namespace {
// batch_arrays into device memory.  The fused case -- every array a pending
// image filling the batch's pixel slots, nothing to pad -- has the kernel
// write the batch in place; otherwise the host batch is built and uploaded.
std::shared_ptr<Array> device_batch(const std::vector<std::shared_ptr<Array>>& arrs,
                                    const std::vector<int64_t>& bshape, const std::vector<int64_t>& stride,
                                    int64_t item, bool ragged, double pad_value, int dim, bool has_dim, int device) {
  const auto type = arrs.front()->type();
  const int64_t isz = itemsize(type), bytes = shape_size(bshape) * isz;
  std::shared_ptr<void> mem = device_pool().get(device, bytes);
  void* ptr = mem.get();
  auto res = std::make_shared<Array>(type, bshape, mem, device);
  bool fused = !has_dim && !ragged && arrs.front()->ndim() == 3;
  for (const auto& a : arrs) fused = fused && deferred(*a) && a->shape(2) == bshape[3];
  if (fused) {
    std::vector<Job> jobs;
    auto* base = static_cast<uint8_t*>(ptr);
    for (size_t i = 0; i < arrs.size(); i++)
      jobs.push_back(Job{deferred_plan(arrs[i]), base + (int64_t)i * item * isz, stride[0] * isz});
    check(run_on(jobs.data(), jobs.size(), out_dtype(type), device, true));
    return res;
  }
  auto host = batch_arrays(arrs, pad_value, dim, has_dim, -1);
  check(mxd_memcpy_h2d(ptr, host->data(), bytes, device));
  return res;
}
}  // namespace

// array::batch (Array.cpp:465-541) + BatchShape::add (core/BatchShape.cpp:26-66).
std::shared_ptr<Array> batch_arrays(const std::vector<std::shared_ptr<Array>>& arrs, double pad_value, int dim,
                                    bool has_dim, int device) {
  const auto type = arrs.front()->type();
  for (const auto& a : arrs)
    if (a->device() >= 0) throw std::runtime_error("Array: cannot batch device-resident arrays");
  const int nd = arrs.front()->ndim();
  if (has_dim) {
    if (dim < 0) dim += nd;
    if (dim < 0 || dim >= nd) throw std::runtime_error("Array: out of bound dimension");
  }
  std::vector<int64_t> bshape;
  for (size_t i = 0; i < arrs.size(); i++) {
    const auto& a = arrs[i];
    if (a->type() != type) throw std::runtime_error("Array: unexpected different types of arrays in batch");
    const auto& s = a->shape();
    if (!has_dim) {
      if (i == 0) {
        bshape.assign(1, 0);
        bshape.insert(bshape.end(), s.begin(), s.end());
      } else if (s.size() + 1 != bshape.size()) {
        throw std::runtime_error("BatchShape: batched arrays expected to have consistent shapes");
      } else {
        for (size_t d = 0; d < s.size(); d++) bshape[d + 1] = std::max(bshape[d + 1], s[d]);
      }
      bshape[0]++;
    } else {
      if (dim >= (int)s.size()) throw std::runtime_error("BatchShape: dimension out of bound");
      if (i == 0) {
        bshape = s;
      } else if (s.size() != bshape.size()) {
        throw std::runtime_error("BatchShape: batched arrays expected to have consistent shapes");
      } else {
        for (size_t d = 0; d < s.size(); d++) bshape[d] = d == (size_t)dim ? bshape[d] + s[d] : std::max(bshape[d], s[d]);
      }
    }
  }
  // Per-array element strides into the result and the per-array step.
  const int rd = (int)bshape.size();
  std::vector<int64_t> full_stride(rd);
  int64_t acc = 1;
  for (int d = rd - 1; d >= 0; d--) {
    full_stride[d] = acc;
    acc *= bshape[d];
  }
  std::vector<int64_t> stride(nd);
  int64_t item = 1;
  if (!has_dim) {
    for (int d = 0; d < nd; d++) stride[d] = full_stride[d + 1];
    item = full_stride[0];
  } else {
    for (int d = 0; d < nd; d++) stride[d] = full_stride[d];
    item = full_stride[dim];
  }

  bool ragged = false;
  for (const auto& a : arrs)
    for (int d = 0; d < nd; d++)
      if (a->shape()[d] != (has_dim ? bshape[d] : bshape[d + 1]) && !(has_dim && d == dim)) ragged = true;
  const int64_t isz = itemsize(type);
  if (device >= 0) return device_batch(arrs, bshape, stride, item, ragged, pad_value, dim, has_dim, device);
  bool images = false;
  for (const auto& a : arrs) images = images || deferred(*a);
  const int64_t total = shape_size(bshape) * isz;
  auto res = std::make_shared<Array>(type, bshape, images ? alloc_batch_bytes(total) : alloc_bytes(total));
  if (ragged) fill(*res, pad_value);

  auto* base = static_cast<uint8_t*>(res->data());
  std::vector<Job> launch;
  int64_t off = 0;
  for (const auto& a : arrs) {
    // Pending HWC images (and lazy JPEG decodes) in the default stacking
    // layout whose pixels fill the batch's pixel slots (same channel count)
    // go to the fused kernels, which write rows straight into the batch; the
    // rest (and a channel count the batch pads) are materialised and copied.
    if (!has_dim && deferred(*a) && nd == 3 && a->shape(2) == bshape[3]) {
      launch.push_back(Job{deferred_plan(a), base + off * isz, stride[0] * isz});
    } else {
      copy_to_strided(base, off, static_cast<const uint8_t*>(a->data()), a->shape(), stride, isz);
    }
    off += has_dim ? item * a->shape(dim) : item;
  }
  run_host(launch, out_dtype(type));
  return res;
}

// core::merge_batch (core/Utils.cpp:209-252)
Sample merge_batch(const std::vector<Sample>& samples, const std::unordered_map<std::string, double>& pad,
                   const std::unordered_map<std::string, int>& dims, const DeviceOut& dev) {
  std::vector<std::string> keys;
  std::vector<std::vector<std::shared_ptr<Array>>> values;
  for (const auto& s : samples) {
    if (keys.empty()) {
      for (const auto& kv : s) keys.push_back(kv.first);
      values.resize(keys.size());
    }
    for (size_t k = 0; k < keys.size(); k++) {
      auto it = s.find(keys[k]);
      if (it == s.end())
        throw std::runtime_error("mergeBatch: inconsistent sample keys in batch (unknown key: <" + keys[k] + ">)");
      values[k].push_back(it->second);
    }
  }
  Sample out;
  for (size_t k = 0; k < keys.size(); k++) {
    auto p = pad.find(keys[k]);
    auto d = dims.find(keys[k]);
    int device = -1;
    if (dev.device >= 0) {
      bool on = false;
      if (dev.keys.empty())
        for (const auto& a : values[k]) on = on || deferred(*a);
      else
        on = std::find(dev.keys.begin(), dev.keys.end(), keys[k]) != dev.keys.end();
      device = on ? dev.device : -1;
    }
    out[keys[k]] = batch_arrays(values[k], p == pad.end() ? 0.0 : p->second, d == dims.end() ? 0 : d->second,
                                d != dims.end(), device);
  }
  return out;
}

// ------------------------------------------------------------------ pool
ThreadPool::ThreadPool(int n) : st_(std::make_shared<State>()) {
  n = std::max(n, 1);
  for (int i = 0; i < n; i++) {
    workers_.emplace_back([st = st_] {
      for (;;) {
        std::packaged_task<Sample()> task;
        {
          std::unique_lock<std::mutex> lk(st->mu);
          st->cv.wait(lk, [&] { return st->stop || !st->tasks.empty(); });
          if (st->stop && st->tasks.empty()) return;
          task = std::move(st->tasks.front());
          st->tasks.pop();
        }
        task();
        // `task` is released here, possibly destroying this pool (see the
        // class comment): only `st` is touched afterwards
      }
    });
  }
}

ThreadPool::~ThreadPool() {
  {
    std::lock_guard<std::mutex> lk(st_->mu);
    st_->stop = true;
  }
  st_->cv.notify_all();
  const auto self = std::this_thread::get_id();
  for (auto& w : workers_) {
    if (w.get_id() == self)
      w.detach();  // destroyed from its own worker: it exits once this returns
    else
      w.join();
  }
}

bool ThreadPool::on_worker() const {
  const auto self = std::this_thread::get_id();
  for (const auto& w : workers_)
    if (w.get_id() == self) return true;
  return false;
}

std::future<Sample> ThreadPool::enqueue(std::function<Sample()> fn) {
  std::packaged_task<Sample()> task(std::move(fn));
  auto fut = task.get_future();
  {
    std::lock_guard<std::mutex> lk(st_->mu);
    if (st_->stop) throw std::runtime_error("ThreadPool: enqueue on stopped pool");
    st_->tasks.push(std::move(task));
  }
  st_->cv.notify_one();
  return fut;
}

// ------------------------------------------------------------------ buffers
// buffer/FromVector.cpp
Sample FromVector::get(int64_t idx) const {
  if (idx < 0 || idx >= (int64_t)data_.size()) throw std::out_of_range("FromVector: index out of range");
  return data_[idx];
}

Perm::Perm(std::shared_ptr<Buffer> b, std::vector<int64_t> perm) : b_(std::move(b)), perm_(std::move(perm)) {
  for (auto i : perm_)
    if (i < 0 || i >= b_->size()) throw std::runtime_error("Perm: index out of range");
}

Sample Perm::get(int64_t idx) const {
  if (idx < 0 || idx >= (int64_t)perm_.size()) throw std::runtime_error("Perm: index out of range");
  return b_->get(perm_[idx]);
}

// buffer/Shuffle.cpp:13-24
std::shared_ptr<Buffer> shuffle_buffer(const std::shared_ptr<Buffer>& b) {
  std::vector<int64_t> perm(b->size());
  std::iota(perm.begin(), perm.end(), 0);
  auto st = get_state();
  std::shuffle(perm.begin(), perm.end(), st->gen);
  return std::make_shared<Perm>(b, std::move(perm));
}

// buffer/Transform.cpp:21-33
Sample BufferTransform::get(int64_t idx) const {
  Sample s = b_->get(idx);
  if (s.empty()) throw std::runtime_error("Transform: cannot return empty sample");
  s = op_->apply(s);
  if (s.empty()) throw std::runtime_error("Transform: cannot return empty sample");
  return s;
}

// buffer/Batch.cpp:10-25,52-68
BufferBatch::BufferBatch(std::shared_ptr<Buffer> b, int64_t batch_size, std::unordered_map<std::string, double> pad,
                         std::unordered_map<std::string, int> dims, DeviceOut out)
    : b_(std::move(b)), bs_(batch_size), pad_(std::move(pad)), dims_(std::move(dims)), out_(std::move(out)) {
  if (bs_ <= 0) throw std::runtime_error("Batch: batch size must be positive");
  size_ = (b_->size() + bs_ - 1) / bs_;
}

Sample BufferBatch::get(int64_t idx) const {
  if (idx < 0 || idx >= size_) throw std::runtime_error("Batch: index out of range");
  const int64_t n = std::min(bs_, b_->size() - idx * bs_);
  std::vector<Sample> samples(n);
  for (int64_t i = 0; i < n; i++) samples[i] = b_->get(idx * bs_ + i);
  return merge_batch(samples, pad_, dims_, out_);
}

// ------------------------------------------------------------------ streams
// stream/FromBuffer.cpp:12-30
Sample FromBuffer::next() const {
  PipeTimer timer(4);
  int64_t idx = -1;
  {
    std::lock_guard<std::mutex> lk(mu_);
    if (idx_ < b_->size()) idx = idx_++;
  }
  return idx < 0 ? Sample() : b_->get(idx);
}

void FromBuffer::reset() {
  std::lock_guard<std::mutex> lk(mu_);
  idx_ = 0;
}

// stream/Transform.cpp:21-47: skip samples an op drops.
Sample StreamTransform::next() const {
  Sample res;
  while (res.empty()) {
    Sample s = s_->next();
    if (s.empty()) break;
    PipeTimer timer(1);
    res = op_->apply(s);
  }
  return res;
}

// stream/Batch.cpp:10-39
StreamBatch::StreamBatch(std::shared_ptr<Stream> s, int64_t batch_size, std::unordered_map<std::string, double> pad,
                         std::unordered_map<std::string, int> dims, DeviceOut out)
    : s_(std::move(s)), bs_(batch_size), pad_(std::move(pad)), dims_(std::move(dims)), out_(std::move(out)) {
  if (bs_ <= 0) throw std::runtime_error("Batch: batch size must be positive");
}

Sample StreamBatch::next() const {
  std::vector<Sample> samples;
  {
    PipeTimer timer(2);
    for (int64_t i = 0; i < bs_; i++) {
      Sample s = s_->next();
      if (s.empty()) break;
      samples.push_back(std::move(s));
    }
  }
  PipeTimer timer(3);
  return samples.empty() ? Sample() : merge_batch(samples, pad_, dims_, out_);
}

// stream/Prefetch.cpp:9-66
Prefetch::Prefetch(std::shared_ptr<Stream> s, int prefetch_size, int num_threads)
    : s_(std::move(s)), pool_(std::make_unique<ThreadPool>(num_threads)), size_(prefetch_size) {
  if (size_ < 0) throw std::runtime_error("Prefetch: prefetch size must be positive");
}

Prefetch::~Prefetch() {
  std::lock_guard<std::mutex> lk(mu_);
  // Destroyed from one of its own workers (ThreadPool): the outstanding tasks
  // hold their upstream, not this node, so they are left to the pool's other
  // workers instead of waited for here (with one worker that would deadlock).
  if (pool_->on_worker()) return;
  while (!cache_.empty()) {
    cache_.front().wait();
    cache_.pop();
  }
}

Sample Prefetch::next() const {
  std::lock_guard<std::mutex> lk(mu_);
  if (size_ == 0) return s_->next();
  if ((int)cache_.size() < size_)
    for (int i = 0; i < size_; i++) cache_.push(pool_->enqueue([s = s_] { return s->next(); }));
  Sample res;
  for (int i = 0; i < size_; i++) {
    auto f = std::move(cache_.front());
    cache_.pop();
    cache_.push(pool_->enqueue([s = s_] { return s->next(); }));
    res = f.get();
    if (!res.empty()) break;
  }
  return res;
}

void Prefetch::reset() {
  std::lock_guard<std::mutex> lk(mu_);
  while (!cache_.empty()) {
    cache_.front().wait();
    cache_.pop();
  }
  s_->reset();
}

// stream/OrderedPrefetch.cpp:8-80
OrderedPrefetch::OrderedPrefetch(std::shared_ptr<Buffer> b, int prefetch_size, int num_threads)
    : b_(std::move(b)), pool_(std::make_unique<ThreadPool>(num_threads)), size_(prefetch_size) {
  if (size_ <= 0) throw std::runtime_error("Prefetch: prefetch size must be strictly positive");
}

OrderedPrefetch::~OrderedPrefetch() {
  std::lock_guard<std::mutex> lk(mu_);
  if (pool_->on_worker()) return;  // as in ~Prefetch
  for (auto& f : cache_)
    if (f.valid()) f.wait();
  cache_.clear();
}

Sample OrderedPrefetch::next() const {
  std::unique_lock<std::mutex> lk(mu_);
  const int64_t n = b_->size();
  if (cache_.empty()) {
    cache_.resize(size_);
    for (int64_t i = idx_; i < std::min<int64_t>(idx_ + size_, n); i++)
      cache_[i % size_] = pool_->enqueue([b = b_, i] { return b->get(i); });
  }
  if (idx_ >= n) return Sample();
  const int64_t idx = idx_++;
  auto f = std::move(cache_[idx % size_]);
  const int64_t nxt = idx + size_;
  if (nxt < n) cache_[idx % size_] = pool_->enqueue([b = b_, nxt] { return b->get(nxt); });
  lk.unlock();
  return f.get();
}

void OrderedPrefetch::reset() {
  std::lock_guard<std::mutex> lk(mu_);
  for (auto& f : cache_)
    if (f.valid()) f.wait();
  cache_.clear();
  idx_ = 0;
}

}  // namespace pipe
}  // namespace mxd
