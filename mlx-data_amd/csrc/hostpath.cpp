// hostpath.cpp -- host-resident batches (capi_internal.h): sources staged
// through page-locked memory (or read in place over PCIe), results copied out
// or written to device destinations, JPEG batches finished on the device.
#include "capi_internal.h"

#include <array>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <functional>

#include <immintrin.h>
#include <sched.h>

namespace mxd {
namespace capi {
namespace {

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
  int32_t* huff_err = nullptr;  // page-locked: the entropy decode's error word, copied back with the chunk
  // MXD_TUNE_DEVICE_TIMING: events around the chunk's kernels (timed: this
  // chunk recorded them)
  hipEvent_t k0 = nullptr, k1 = nullptr;
  bool timed = false;
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
  if (s.huff_err) (void)hipHostFree(s.huff_err);
  s.huff_err = nullptr;
  s.pin_in = s.pin_out = s.dev_in = s.dev_out = s.dev_mid = nullptr;
  s.pin_in_cap = s.pin_out_cap = s.dev_in_cap = s.dev_out_cap = s.dev_mid_cap = 0;
}

// Concurrent host-path calls per device (each context holds its staging
// buffers): enough for the 16 prefetch workers of the largest measured
// pipeline, which 4 contexts serialised.
constexpr int kCtxPerDevice = 16;

// Host-side byte moves of the host path (footprint staging into pinned
// memory, copy-out of results) are bound by one core's memory bandwidth;
// they are split over helper threads, fewer when several host-path calls run
// at once (prefetch workers already spread the work).
std::atomic<int> g_host_calls{0};

// Persistent helper threads for parallel_items (MXD_HOST_HELPERS=1, the
// default; 0 spawns threads per call as before): a chunk's staging used to
// start and join up to 7 std::threads, ~20 us each, for every ~24 MB chunk.
#ifndef MXD_HOST_HELPERS
#define MXD_HOST_HELPERS 1
#endif

class Helpers {
 public:
  static Helpers& get() {
    static Helpers* h = new Helpers();  // leaked on purpose: its threads live until exit
    return *h;
  }
  // Runs `work` on the calling thread and on up to `extra` helpers; returns
  // once every helper that took part has finished it (helpers that had not
  // started by then never will).
  void run(int extra, const std::function<void()>& work) {
    auto job = std::make_shared<Job>();
    job->work = &work;
    job->pending = extra;
    {
      // the pool grows to the helpers every call in flight asks for (capped),
      // so concurrent calls (prefetch workers, split devices) each get theirs
      std::lock_guard<std::mutex> lk(mu_);
      outstanding_ += extra;
      while ((int)threads_.size() < std::min(outstanding_, kMaxHelpers)) threads_.emplace_back([this] { loop(); });
      for (int k = 0; k < extra; k++) queue_.push_back(job);
    }
    cv_.notify_all();
    work();
    int unclaimed = 0;
    {
      std::lock_guard<std::mutex> lk(mu_);
      outstanding_ -= extra;
      for (auto it = queue_.begin(); it != queue_.end();)
        if (*it == job) {
          it = queue_.erase(it);
          unclaimed++;
        } else {
          ++it;
        }
    }
    std::unique_lock<std::mutex> lk(job->mu);
    job->pending -= unclaimed;
    job->cv.wait(lk, [&] { return job->pending == 0; });
  }

 private:
  static constexpr int kMaxHelpers = 16;
  struct Job {
    const std::function<void()>* work = nullptr;
    int pending = 0;
    std::mutex mu;
    std::condition_variable cv;
  };
  void loop() {
    for (;;) {
      std::shared_ptr<Job> job;
      {
        std::unique_lock<std::mutex> lk(mu_);
        cv_.wait(lk, [&] { return !queue_.empty(); });
        job = queue_.front();
        queue_.pop_front();
      }
      (*job->work)();
      std::lock_guard<std::mutex> lk(job->mu);
      if (--job->pending == 0) job->cv.notify_all();
    }
  }
  std::mutex mu_;
  std::condition_variable cv_;
  std::deque<std::shared_ptr<Job>> queue_;
  std::vector<std::thread> threads_;
  int outstanding_ = 0;  // helpers asked for by the calls in flight
};

// The CPUs this process may keep busy: the affinity mask, capped by a cgroup
// CPU quota (v2 cpu.max, v1 cpu.cfs_quota_us) -- a container's share, which
// the mask does not show: the GPU boxes give every process the whole
// machine's mask and a 16-CPU quota, and sizing helpers by the mask put
// 16 prefetch workers x 8 staging threads on 16 CPUs -- and by
// OMP_NUM_THREADS when the environment sets it above 1 (the boxes' per-GPU
// share; torchrun and similar launchers export 1 to every rank by default,
// which says nothing about the host's CPUs and is ignored).
// MXD_HOST_CPUS overrides all of it (tuning knobs).
int host_cpu_budget() {
  if (const char* e = std::getenv("MXD_HOST_CPUS"))
    if (std::atoi(e) > 0) return std::atoi(e);
  int n = (int)std::thread::hardware_concurrency();
  cpu_set_t set;
  CPU_ZERO(&set);
  if (sched_getaffinity(0, sizeof set, &set) == 0) n = CPU_COUNT(&set);
  auto cap = [&](double quota, double period) {
    if (quota > 0 && period > 0) n = std::min(n, std::max(1, (int)std::ceil(quota / period)));
  };
  if (FILE* f = std::fopen("/sys/fs/cgroup/cpu.max", "r")) {
    char q[32] = {0};
    double period = 0;
    if (std::fscanf(f, "%31s %lf", q, &period) == 2 && std::strcmp(q, "max") != 0) cap(std::atof(q), period);
    std::fclose(f);
  } else if (FILE* g = std::fopen("/sys/fs/cgroup/cpu/cpu.cfs_quota_us", "r")) {
    double quota = -1, period = 0;
    if (std::fscanf(g, "%lf", &quota) != 1) quota = -1;
    std::fclose(g);
    if (FILE* h = std::fopen("/sys/fs/cgroup/cpu/cpu.cfs_period_us", "r")) {
      if (std::fscanf(h, "%lf", &period) != 1) period = 0;
      std::fclose(h);
    }
    cap(quota, period);
  }
  if (const char* e = std::getenv("OMP_NUM_THREADS")) {
    const int k = std::atoi(e);
    if (k > 1) n = std::min(n, k);
  }
  return std::max(1, n);
}

// dst[j] = src[j] / 255 in f32 (IEEE division: the bytes of the kernels'
// MXD_F32_DIV255 output and of the reference's astype(float32) / 255 for the
// same u8 value; multiplying by 1/255 differs for 126 of the 256 values).
// The f32 rows are written with streaming (non-temporal) stores from the
// first 32-byte boundary on: the batch is written once here and read by the
// consumer later, and ordinary stores would first read every destination
// line into the cache (the pass is bound by host memory traffic).
__attribute__((target("avx2"))) void div255_avx2(const uint8_t* src, float* dst, int64_t n) {
  const __m256 k = _mm256_set1_ps(255.0f);
  int64_t j = 0;
  for (; j < n && (reinterpret_cast<uintptr_t>(dst + j) & 31) != 0; j++) dst[j] = (float)src[j] / 255.0f;
  for (; j + 16 <= n; j += 16) {
    const __m128i b = _mm_loadu_si128(reinterpret_cast<const __m128i*>(src + j));
    _mm256_stream_ps(dst + j, _mm256_div_ps(_mm256_cvtepi32_ps(_mm256_cvtepu8_epi32(b)), k));
    _mm256_stream_ps(dst + j + 8, _mm256_div_ps(_mm256_cvtepi32_ps(_mm256_cvtepu8_epi32(_mm_srli_si128(b, 8))), k));
  }
  for (; j < n; j++) dst[j] = (float)src[j] / 255.0f;
}

void div255_row(const uint8_t* src, float* dst, int64_t n) {
  static const bool avx2 = __builtin_cpu_supports("avx2");
  if (avx2) return div255_avx2(src, dst, n);
  for (int64_t j = 0; j < n; j++) dst[j] = (float)src[j] / 255.0f;
}

template <class F>
void parallel_items(int32_t first, int32_t end, int64_t bytes, F&& f) {
  const int32_t n = end - first;
  static const int hw = host_cpu_budget();
  int t = std::min<int64_t>({8, hw / std::max(1, g_host_calls.load()), n, bytes >> 20});
  if (t <= 1) {
    for (int32_t i = first; i < end; i++) f(i);
    return;
  }
  std::atomic<int32_t> next{first};
  auto work = [&] {
    for (int32_t i; (i = next.fetch_add(1)) < end;) f(i);
  };
  if constexpr (MXD_HOST_HELPERS != 0) {
    const std::function<void()> fn = work;
    Helpers::get().run(t - 1, fn);
  } else {
    std::vector<std::thread> ts;
    for (int k = 1; k < t; k++) ts.emplace_back(work);
    work();
    for (auto& th : ts) th.join();
  }
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

// MXD_TUNE_HOST_STREAMS > 0: host-path slots share that many library
// streams per device (round robin as slots are first set up) instead of
// owning one each, so 16 prefetch workers do not spread their device calls
// over 32 streams when HIP maps a process's streams onto fewer hardware
// queues (GPU_MAX_HW_QUEUES, 4 by default).  Read when a slot is first set up.
int shared_stream(hipStream_t* out, int32_t n) {
  static std::mutex mu;
  static std::map<int, std::pair<std::vector<hipStream_t>, int64_t>> pools;
  int dev = 0;
  MXD_HIP(hipGetDevice(&dev));
  std::lock_guard<std::mutex> lk(mu);
  auto& pl = pools[dev];
  if ((int32_t)pl.first.size() < n) {
    hipStream_t st = nullptr;
    MXD_HIP(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
    pl.first.push_back(st);
    *out = st;
    return MXD_OK;
  }
  *out = pl.first[(size_t)(pl.second++ % (int64_t)pl.first.size())];
  return MXD_OK;
}

int init_slot(Slot& s) {
  if (!s.stream) {
    const int32_t shared = g_tune[MXD_TUNE_HOST_STREAMS].load();
    if (shared > 0) {
      if (int rc = shared_stream(&s.stream, shared)) return rc;
    } else {
      MXD_HIP(hipStreamCreateWithFlags(&s.stream, hipStreamNonBlocking));
    }
  }
  // the calling thread sleeps on the chunk's event instead of polling
  // (MXD_TUNE_HOST_WAIT 2: polling): with 16 prefetch workers on 16 cores the
  // polling waits took the cores the other workers' parsing and staging need
  // (JPEG device batch at 16 workers, C4 137 k -> 156-161 k img/s, C1
  // 176-192 k -> 205-208 k; profiles/r04/host_wait_ab.jsonl)
  if (!s.done)
    MXD_HIP(hipEventCreateWithFlags(
        &s.done, hipEventDisableTiming | (g_tune[MXD_TUNE_HOST_WAIT].load() == 2 ? 0 : hipEventBlockingSync)));
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
  std::vector<mxd::YccDev> ycc;  // per image: its planes as a resize source (used when JpegImgDev::skip)
  int64_t planes_off = 0, imgs_off = 0, q_off = 0, ycc_off = 0, end = 0;  // in the staged input
  int64_t samples = 0, rgb_off = 0, mid_bytes = 0;             // in dev_mid
  int64_t nblocks = 0, max_quad_rows = 0;  // max_quad_rows: the colour kernel's threads per image (8 pixels each)
  // Device entropy decode of the chunk's pending images (jpeghuff.h): their
  // unstuffed segments (words_off..), tables, image / segment / job records in
  // the staged input; their coefficients in dev_in past the staged bytes
  // ([coef_off, dev_end), written by the decode, never copied).
  std::vector<mxd::HuffDev> htabs;
  struct TableSet {
    std::array<uint64_t, 8> key;  // device_table serials
    int n;
    int32_t first;                // in htabs
  };
  std::vector<TableSet> table_sets;
  std::vector<mxd::HuffImgDev> himgs;
  std::vector<mxd::HuffSegDev> hsegs;
  std::vector<mxd::HuffJobDev> hjobs;
  struct Raw {
    const uint8_t *b, *e;  // raw segment bytes
    int64_t at;            // staged byte offset (relative to words_off)
  };
  std::vector<Raw> raw;              // per staged segment (hsegs entries)
  std::vector<int32_t> seg_first;    // per chunk image: its first raw entry (-1: not pending)
  std::vector<int32_t> seg_count;    // and their number
  int64_t words_off = 0, words_bytes = 0, htabs_off = 0, himgs_off = 0, hsegs_off = 0, hjobs_off = 0;
  int64_t coef_off = 0, dev_end = 0;
  int64_t pub_off = 0;  // the jobs' publication records + launch control, zeroed with the coefficients
  int32_t huff_threads = 0;
  int64_t huff_lds = 0;  // the largest job's dynamic LDS (its words included when they fit)
  bool huff_search = false;  // some table needs the searching kernel (HuffDev::search)
};

std::atomic<int64_t> g_plane_sources{0};
std::atomic<int64_t> g_narrow_images{0};
std::atomic<int64_t> g_host_stats[6] = {};
std::atomic<int64_t> g_device_stats[2] = {};
int64_t now_ns() {
  return std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now().time_since_epoch())
      .count();
}

const mxd::jpeg::Coefs* coefs_of(const mxd_jpeg_coefs* c) { return reinterpret_cast<const mxd::jpeg::Coefs*>(c); }

int64_t rgb_pitch(int32_t w) { return (((int64_t)w * 3 + 63) & ~(int64_t)63) + 64; }

// Lays out the chunk [first, end) of a JPEG batch whose coefficients are staged
// at in_off[i]; the tables follow at `tables_at`.
// foot[i]: image i's resize footprint (x0, x1, y0, y1, inclusive, in image
// pixels; the whole image when unknown).
void jpeg_chunk(const mxd_jpeg_image* jimg, int32_t first, int32_t end, const std::vector<int64_t>& in_off,
                int64_t tables_at, const std::vector<std::array<int32_t, 4>>& foot, JpegChunk* out) {
  JpegChunk& c = *out;
  c = JpegChunk();
  auto up = [](int64_t v, int64_t a) { return (v + a - 1) / a * a; };
  int64_t coef_rel = 0;  // pending images' coefficients, relative to coef_off
  std::vector<int64_t> pend_rel(end - first, -1);
  c.seg_first.assign(end - first, -1);
  c.seg_count.assign(end - first, 0);
  for (int32_t i = first; i < end; i++) {
    const mxd::jpeg::CoefInfo info = mxd::jpeg::coef_info(coefs_of(jimg[i].coefs));
    if (!info.entropy_pending) continue;
    const mxd::jpeg::EntropyScan es = mxd::jpeg::entropy_scan(coefs_of(jimg[i].coefs));
    pend_rel[i - first] = coef_rel;
    mxd::HuffImgDev h{};
    h.coef = coef_rel / 2;  // coef_off added below
    for (int k = 0; k < info.ncomp && k < 4; k++) {
      h.plane[k] = info.comp[k].off;
      h.bw[k] = info.comp[k].bw;
      h.comp_h[k] = (int8_t)info.comp[k].h;
      h.comp_v[k] = (int8_t)info.comp[k].v;
    }
    h.ntables = es.ntables;
    h.bpm = es.bpm;
    h.mcux = es.mcux;
    h.interleaved = es.interleaved;
    h.rst_mcus = es.restart_interval > 0 ? es.restart_interval : (int32_t)std::min<int64_t>(es.mcus, INT32_MAX);
    h.mcus = es.mcus;
    for (int j = 0; j < es.bpm; j++) {
      h.blk_comp[j] = (int8_t)es.blk_comp[j];
      h.blk_dc[j] = (int8_t)es.blk_dc[j];
      h.blk_ac[j] = (int8_t)es.blk_ac[j];
      h.blk_dx[j] = (int8_t)es.blk_dx[j];
      h.blk_dy[j] = (int8_t)es.blk_dy[j];
    }
    // the image's tables (consecutive from h.tables): a set an earlier image
    // of the chunk already staged is shared (files from one encoder carry the
    // same tables: one set per C4 batch instead of 128 x ~50 KB staged)
    {
      std::array<uint64_t, 8> key{};
      for (int t = 0; t < es.ntables; t++)
        key[t] = mxd::jpeg::device_table(coefs_of(jimg[i].coefs), es.table_class[t], es.table_id[t], nullptr);
      int32_t at = -1;
      for (const auto& ts : c.table_sets)
        if (ts.n == es.ntables && ts.key == key) at = ts.first;
      if (at < 0) {
        at = (int32_t)c.htabs.size();
        c.table_sets.push_back({key, es.ntables, at});
        for (int t = 0; t < es.ntables; t++) {
          c.htabs.emplace_back();
          mxd::jpeg::device_table(coefs_of(jimg[i].coefs), es.table_class[t], es.table_id[t], &c.htabs.back());
          c.huff_search = c.huff_search || c.htabs.back().search != 0;
        }
      }
      h.tables = at;
    }
    // subsequence length: kHuffMinBits (MXD_TUNE_HUFF_BITS overrides it;
    // a multiple of 32); segments of any length split over several jobs
    const int32_t knob = g_tune[MXD_TUNE_HUFF_BITS].load();
    const int32_t sub_bits = (int32_t)up(knob > 0 ? knob : kHuffMinBits, 32);
    h.sub_bits = sub_bits;
    c.seg_first[i - first] = (int32_t)c.raw.size();
    c.seg_count[i - first] = es.nseg;
    const int32_t img_index = (int32_t)c.himgs.size();
    const int32_t seg_base = (int32_t)c.hsegs.size();
    std::vector<int64_t> sub_first;  // per segment: its first subsequence (image-wide numbering)
    int64_t nsub_img = 0;
    for (int sgi = 0; sgi < es.nseg; sgi++) {
      const int64_t raw = es.seg_end[sgi] - es.seg_begin[sgi];
      mxd::HuffSegDev sd{};
      sd.word = c.words_bytes / 4;
      sd.bits = (int32_t)(8 * es.seg_bytes[sgi]);
      sd.img = img_index;
      sd.mcu0 = (int64_t)sgi * h.rst_mcus;
      sd.mcus = (int32_t)std::min<int64_t>(h.rst_mcus, es.mcus - sd.mcu0);
      sd.nsub = (int32_t)std::max<int64_t>(1, (sd.bits + sub_bits - 1) / sub_bits);
      c.raw.push_back({es.data + es.seg_begin[sgi], es.data + es.seg_end[sgi], c.words_bytes});
      // zero padding past the data: a partial last word's tail and >= 1 zero word,
      // which jpeghuff.hip's LDS reader reads for every word past the segment
      c.words_bytes += up(raw + 4, 16);
      sub_first.push_back(nsub_img);
      nsub_img += sd.nsub;
      c.hsegs.push_back(sd);
    }
    sub_first.push_back(nsub_img);
    // jobs: runs of at most kHuffThreads - kJobSlack own subsequences, evenly
    // sized; a cut inside a segment gives the next job a warm-up of up to
    // kHuffWarm subsequences before its own (jpeghuff.h); cuts within
    // kCutMove subsequences of a segment start move there (restart markers: no
    // warm-up), which lengthens the job after the cut by up to kCutMove.  The
    // slack covers both, so no job exceeds one workgroup's kHuffThreads.
    constexpr int64_t kCutMove = 32;
    constexpr int64_t kJobSlack = std::max<int64_t>(mxd::kHuffWarm, kCutMove);
    const int32_t job_knob = g_tune[MXD_TUNE_HUFF_JOB].load();
    const int64_t cap = job_knob > 0 ? std::min<int64_t>(job_knob, mxd::kHuffThreads - kJobSlack)
                                     : mxd::kHuffThreads - kJobSlack;
    const int64_t njob = (nsub_img + cap - 1) / cap;
    std::vector<int64_t> cuts{0};
    for (int64_t q = 1; q < njob; q++) {
      int64_t cut = q * nsub_img / njob;
      const int64_t sgi = std::upper_bound(sub_first.begin(), sub_first.end(), cut) - sub_first.begin() - 1;
      if (cut - sub_first[sgi] <= kCutMove && sub_first[sgi] > cuts.back()) cut = sub_first[sgi];
      cuts.push_back(cut);
    }
    cuts.push_back(nsub_img);
    for (size_t q = 0; q + 1 < cuts.size(); q++) {
      const int64_t a0 = cuts[q], b0 = cuts[q + 1];
      const int64_t sa = std::upper_bound(sub_first.begin(), sub_first.end(), a0) - sub_first.begin() - 1;
      const int64_t ja = a0 - sub_first[sa];  // the first own subsequence's index in its segment
      const int64_t warm = std::min<int64_t>(mxd::kHuffWarm, ja);
      const int64_t sl = std::upper_bound(sub_first.begin(), sub_first.end(), b0 - 1) - sub_first.begin() - 1;
      const int64_t jl = b0 - 1 - sub_first[sl];  // the last subsequence's index in its segment
      const mxd::HuffSegDev& s0 = c.hsegs[seg_base + sa];
      const mxd::HuffSegDev& s1 = c.hsegs[seg_base + sl];
      mxd::HuffJobDev jb{};
      jb.seg0 = (int32_t)(seg_base + sa);
      jb.nseg = (int32_t)(sl - sa + 1);
      jb.sub0 = (int32_t)(ja - warm);
      jb.nsub = (int32_t)(b0 - a0 + warm);
      jb.warm = (int32_t)warm;
      jb.pred = ja > 0 ? 1 : 0;
      jb.word0 = s0.word + (((int64_t)jb.sub0 * sub_bits / 32) & ~(int64_t)3);
      // words staged: to the last segment's staged end when the job reaches
      // it, else 4 words past its last subsequence (a step reads <= 2 past)
      const int64_t seg_end = s1.word + up(es.seg_end[sl] - es.seg_begin[sl] + 4, 16) / 4;
      const int64_t end = jl == s1.nsub - 1 ? seg_end : std::min(seg_end, s1.word + (jl + 1) * sub_bits / 32 + 4);
      jb.words16 = (int32_t)((end - jb.word0 + 3) / 4);
      const int64_t with = mxd::jpeg_huff_lds_bytes(es.ntables, jb.nseg, 4 * (int64_t)jb.words16);
      jb.lds = with <= mxd::jpeg_huff_lds_budget() && g_tune[MXD_TUNE_HUFF_GLOBAL].load() == 0 ? 1 : 0;
      c.huff_lds = std::max(c.huff_lds, jb.lds ? with : mxd::jpeg_huff_lds_bytes(es.ntables, jb.nseg, 0));
      c.huff_threads = std::max(c.huff_threads, jb.nsub);
      c.hjobs.push_back(jb);
    }
    c.himgs.push_back(h);
    coef_rel += up(info.coef_count * 2, 256);
  }
  for (int32_t i = first; i < end; i++) {
    const mxd::jpeg::CoefInfo info = mxd::jpeg::coef_info(coefs_of(jimg[i].coefs));
    mxd::JpegImgDev m{};
    m.ncomp = info.ncomp == 1 ? 1 : 3;
    // 0 YCbCr -> RGB; 1 the components as they are (RGB, CMYK's C M Y);
    // 2 YCCK: YCbCr -> RGB inverted (jdcolor.c ycck_cmyk_convert's C M Y)
    m.rgb = info.color_space == 2 || info.color_space == 3 ? 1 : info.color_space == 4 ? 2 : 0;
    m.width = info.width;
    m.height = info.height;
    m.pitch = (int32_t)rgb_pitch(info.width);
    m.skip = 0;
    for (int k = 0; k < m.ncomp; k++) {
      const mxd::jpeg::CoefPlane& cp = info.comp[k];
      mxd::JpegPlaneDev p{};
      // host-decoded coefficients: staged at in_off[i]; pending: in the
      // device-only region (coef_off added below)
      p.coef = pend_rel[i - first] >= 0 ? (pend_rel[i - first] + cp.off * 2) / 2 : (in_off[i] + cp.off * 2) / 2;
      p.out = c.samples;
      p.first_block = c.nblocks;
      p.bw = cp.bw;
      p.bh = cp.bh;
      p.qtab = (int32_t)c.qtabs.size();
      p.coded = cp.coded ? 1 : 0;
      p.zigzag = pend_rel[i - first] >= 0 ? 1 : 0;  // decoded by jpeg_huff: zig-zag order
      {
        // the footprint on this component's sample grid, one sample wider on
        // each side (fancy upsampling reads a neighbour), in whole blocks
        const int hx = info.max_h / cp.h, vx = info.max_v / cp.v;
        const std::array<int32_t, 4>& f = foot[i];
        p.bx0 = std::max(0, (f[0] / hx - 1) / 8);
        p.bx1 = std::min(cp.bw, (f[1] / hx + 1) / 8 + 1);
        p.by0 = std::max(0, (f[2] / vx - 1) / 8);
        p.by1 = std::min(cp.bh, (f[3] / vx + 1) / 8 + 1);
      }
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
      // jpeg_idct's threads: the plane's needed rectangle, padded to a wave
      // (a wave stays in one plane)
      c.nblocks += ((int64_t)std::max(0, p.bx1 - p.bx0) * std::max(0, p.by1 - p.by0) + 63) & ~(int64_t)63;
    }
    m.out = c.mid_bytes;  // relative to rgb_off, fixed below
    c.mid_bytes += up((int64_t)m.pitch * m.height, 256);
    c.max_quad_rows = std::max<int64_t>(c.max_quad_rows, (int64_t)m.height * ((info.width + 7) / 8));
    c.imgs.push_back(m);
  }
  c.rgb_off = c.samples;
  c.mid_bytes += c.samples;
  c.words_off = up(tables_at, 256);
  c.htabs_off = up(c.words_off + c.words_bytes, 256);
  c.himgs_off = up(c.htabs_off + (int64_t)(c.htabs.size() * sizeof(mxd::HuffDev)), 256);
  c.hsegs_off = up(c.himgs_off + (int64_t)(c.himgs.size() * sizeof(mxd::HuffImgDev)), 256);
  c.hjobs_off = up(c.hsegs_off + (int64_t)(c.hsegs.size() * sizeof(mxd::HuffSegDev)), 256);
  c.planes_off = up(c.hjobs_off + (int64_t)(c.hjobs.size() * sizeof(mxd::HuffJobDev)), 256);
  c.imgs_off = up(c.planes_off + (int64_t)(c.planes.size() * sizeof(mxd::JpegPlaneDev)), 256);
  c.q_off = up(c.imgs_off + (int64_t)(c.imgs.size() * sizeof(mxd::JpegImgDev)), 256);
  c.ycc.assign(c.imgs.size(), mxd::YccDev{});
  c.ycc_off = up(c.q_off + (int64_t)(c.qtabs.size() * sizeof(uint16_t)), 16);
  c.end = c.ycc_off + (int64_t)(c.ycc.size() * sizeof(mxd::YccDev));
  c.pub_off = up(c.end, 256);
  c.coef_off = up(c.pub_off + (int64_t)(c.hjobs.size() * sizeof(mxd::HuffPubDev)) + (int64_t)sizeof(mxd::HuffCtlDev),
                  256);
  c.dev_end = c.coef_off + coef_rel;
  for (mxd::HuffImgDev& h : c.himgs) h.coef += c.coef_off / 2;
  for (size_t k = 0, pi = 0; k < (size_t)(end - first); k++) {
    const mxd::jpeg::CoefInfo info = mxd::jpeg::coef_info(coefs_of(jimg[first + k].coefs));
    const int np = info.ncomp == 1 ? 1 : 3;
    if (pend_rel[k] >= 0)
      for (int q = 0; q < np; q++) c.planes[pi + q].coef += c.coef_off / 2;
    pi += np;
  }
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
  // Narrow return (round 6): f32 results bound for host memory cross the link
  // as the u8 bytes the same kernels compute before their exact /255 (the
  // f32 output is LUT[u8] bit for bit), and the host expands them while it
  // copies them into place -- a quarter of the link bytes (150 instead of 602
  // KB per 224x224 RGB image), for page-locked destinations too (instead of
  // the kernels writing f32 into them over PCIe: the pipeline's host batches
  // are page-locked, and that write was the host-ending C4 bound, 43 GB/s).
  // MXD_TUNE_F32_LINK 1: the f32 results cross the link; 2..99: that
  // percentage of the images is narrowed, spread evenly, the rest cross the
  // link as f32 (the link and the host's writes share the work).
  const int32_t link_knob = g_tune[MXD_TUNE_F32_LINK].load();
  const int32_t narrow_pct = link_knob == 1 ? 0 : link_knob >= 2 && link_knob < 100 ? link_knob : 100;
  const bool narrow_any = out_dtype == MXD_F32_DIV255 && !dst_device && narrow_pct > 0;
  auto narrow_of = [&](int32_t i) { return narrow_any && (narrow_pct == 100 || (i * narrow_pct) % 100 < narrow_pct); };
  DeviceGuard g(device);
  g_host_calls.fetch_add(1);
  struct CallCount {
    int64_t t0 = now_ns(), n;
    ~CallCount() {
      g_host_calls.fetch_sub(1);
      g_host_stats[0].fetch_add(1, std::memory_order_relaxed);
      g_host_stats[1].fetch_add(n, std::memory_order_relaxed);
      g_host_stats[2].fetch_add(now_ns() - t0, std::memory_order_relaxed);
    }
  } call_count{now_ns(), n};
  auto waited = [](int64_t t0) { g_host_stats[3].fetch_add(now_ns() - t0, std::memory_order_relaxed); };
  // Per image: the staged footprint (columns from x0, 16-byte aligned so both
  // kernel families read it as they would the whole image) and its offsets.
  struct Stage {
    int32_t x0, y0, rows;
    int64_t pitch, copy, in_off, out_off, out_row;
    int64_t stage_row;            // an output row as staged (u8 for a narrow return)
    bool narrow = false;          // f32 results returned as u8, expanded on the host
    int64_t in_size;              // staged bytes (footprint rows, or a JPEG's coefficients)
    bool src_pinned, dst_pinned;  // page-locked host memory: DMA'd directly, no staging copy
    bool pending = false;         // JPEG whose entropy decode runs on the device (nothing staged at in_off)
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
      s.in_size = info.coef_count * 2;  // chunk sizing (device memory); staged only when decoded on the host
      s.pending = info.entropy_pending;
      s.out_row = (int64_t)im.crop_w * im.channels * elem;
      s.src_pinned = false;
      s.src_dev = nullptr;
      s.dst_pinned = !dst_device && host_pinned(im.dst);
      s.dst_dev = s.dst_pinned && !(g_policy.load() & MXD_POLICY_NO_ZERO_COPY)
                      ? const_cast<uint8_t*>(host_device_ptr(im.dst)) : nullptr;
      s.narrow = narrow_of(i);
      if (s.narrow) s.dst_pinned = false, s.dst_dev = nullptr;  // staged, then expanded into place
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
    s.narrow = narrow_of(i);
    if (s.narrow) s.dst_pinned = false, s.dst_dev = nullptr;  // staged, then expanded into place
    if (!dst_device && im.dst_stride < s.out_row)
      return fail(MXD_ERR_INVALID, "mxd: dst_stride smaller than an output row");
  }
  int64_t nnarrow = 0;
  for (int32_t i = 0; i < n; i++) {
    st[i].stage_row = st[i].narrow ? st[i].out_row / 4 : st[i].out_row;
    nnarrow += st[i].narrow ? 1 : 0;
  }
  if (nnarrow) g_narrow_images.fetch_add(nnarrow, std::memory_order_relaxed);
  auto launch_dtype = [&](int32_t i) { return st[i].narrow ? MXD_U8 : out_dtype; };
  // Chunks of about kChunk staged bytes (at least one image each).  A JPEG
  // whose entropy decode runs on the device stages only its compressed
  // segments, and counts an eighth of its coefficient bytes (device memory):
  // ~300 ImageNet-size files a chunk, so a 128-file batch is one entropy
  // launch over the whole GPU rather than three of ~40 files on ~80 CUs
  // (round 5).
  constexpr int64_t kChunk = 24 << 20;
  // (and at most 65535 images: the JPEG colour kernel puts one image per grid row)
  constexpr int32_t kChunkImages = 65535;
  std::vector<std::pair<int32_t, int32_t>> chunks;  // [first, end)
  for (int32_t i = 0; i < n;) {
    int32_t j = i;
    int64_t bytes = 0;
    auto size = [&](int32_t q) { return st[q].pending ? st[q].in_size / 8 : st[q].in_size; };
    while (j < n && j - i < kChunkImages && (j == i || bytes + size(j) <= kChunk)) {
      bytes += size(j);
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
      const int64_t t0 = now_ns();
      for (Slot& sl : c.slot)
        if (sl.stream) (void)hipStreamSynchronize(sl.stream);
      g_host_stats[3].fetch_add(now_ns() - t0, std::memory_order_relaxed);
    }
  } drain{ctx};
  for (Slot& sl : ctx.slot)
    if (int rc = init_slot(sl)) return rc;
  int pending[2] = {-1, -1};  // chunk in flight on each slot
  auto copy_out = [&](int k) -> int {
    Slot& sl = ctx.slot[k & 1];
    const int64_t t0 = now_ns();
    MXD_HIP(hipEventSynchronize(sl.done));
    waited(t0);
    pending[k & 1] = -1;
    if (sl.timed) {
      float ms = 0.0f;
      if (hipEventElapsedTime(&ms, sl.k0, sl.k1) == hipSuccess && ms > 0.0f) {
        g_device_stats[0].fetch_add(1, std::memory_order_relaxed);
        g_device_stats[1].fetch_add((int64_t)((double)ms * 1e6), std::memory_order_relaxed);
      }
      sl.timed = false;
    }
    if (sl.huff_err && *sl.huff_err) {
      *sl.huff_err = 0;
      return fail(MXD_ERR_DEVICE, "jpeg entropy decode: a job never received its predecessor's state");
    }
    if (dst_device) return MXD_OK;  // the kernel wrote the destinations
    int64_t bytes = 0;
    for (int32_t i = chunks[k].first; i < chunks[k].second; i++) bytes += st[i].out_row * images[i].crop_h;
    parallel_items(chunks[k].first, chunks[k].second, bytes, [&](int32_t i) {
      if (st[i].dst_pinned) return;  // DMA'd straight into place
      const mxd_image& im = images[i];
      uint8_t* d = static_cast<uint8_t*>(im.dst);
      const uint8_t* src = sl.pin_out + st[i].out_off;
      if (st[i].narrow) {
        for (int32_t r = 0; r < im.crop_h; r++)
          div255_row(src + (size_t)r * st[i].stage_row, reinterpret_cast<float*>(d + (size_t)r * im.dst_stride),
                     st[i].stage_row);
        _mm_sfence();  // the streaming stores are visible before the call returns
      } else if (im.dst_stride == st[i].out_row) {
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
        if (st[i].src_pinned == (pass == 1) && !st[i].src_dev && !st[i].pending) {
          st[i].in_off = in_bytes;
          in_bytes += (st[i].in_size + 255) & ~(int64_t)255;
        }
    int64_t in_staged = 0, out_staged = 0;
    for (int32_t i = chunks[k].first; i < chunks[k].second; i++)
      if (!st[i].src_pinned && !st[i].pending) in_staged = std::max(in_staged, st[i].in_off + st[i].in_size);
    JpegChunk jc;
    int64_t dev_in_bytes = 0;
    if (jpeg) {
      std::vector<int64_t> off(n, 0);
      std::vector<std::array<int32_t, 4>> foot(n);
      for (int32_t i = chunks[k].first; i < chunks[k].second; i++) {
        off[i] = st[i].in_off;
        // the resize's source footprint in the window, as image pixels
        const mxd_image& im = images[i];
        const DevTable *xt = nullptr, *yt = nullptr;
        int32_t xl = 0, xh = im.src_w - 1, yl = 0, yh = im.src_h - 1;
        if (tables().get(device, im.src_w, im.resize_w, &xt) == MXD_OK &&
            tables().get(device, im.src_h, im.resize_h, &yt) == MXD_OK)
          footprint(*xt, *yt, im, &xl, &xh, &yl, &yh);
        foot[i] = {jpeg[i].win_x + xl, jpeg[i].win_x + xh, jpeg[i].win_y + yl, jpeg[i].win_y + yh};
      }
      jpeg_chunk(jpeg, chunks[k].first, chunks[k].second, off, in_bytes, foot, &jc);
      // coefficients, then the chunk's tables, then the entropy decode's
      // publication records and launch control (zeros), in one copy
      in_bytes = in_staged = jc.hjobs.empty() ? jc.end : jc.coef_off;
      dev_in_bytes = jc.dev_end;      // + the device-decoded coefficients
      if (int rc = grow_device(&sl.dev_mid, &sl.dev_mid_cap, jc.mid_bytes)) return rc;
    }
    for (int pass = 0; pass < 2; pass++)
      for (int32_t i = chunks[k].first; i < chunks[k].second; i++)
        if (st[i].dst_pinned == (pass == 1) && !st[i].dst_dev) {
          st[i].out_off = out_bytes;
          // page-locked destinations back to back (one copy per contiguous run)
          const int64_t b = st[i].stage_row * images[i].crop_h;
          out_bytes += pass == 1 && (st[i].stage_row & 3) == 0 ? b : (b + 255) & ~(int64_t)255;
        }
    for (int32_t i = chunks[k].first; i < chunks[k].second; i++)
      if (!st[i].dst_pinned) out_staged = std::max(out_staged, st[i].out_off + st[i].stage_row * images[i].crop_h);
    if (int rc = grow_pinned(&sl.pin_in, &sl.pin_in_cap, in_bytes)) return rc;
    if (int rc = grow_device(&sl.dev_in, &sl.dev_in_cap, std::max(in_bytes, dev_in_bytes))) return rc;
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
        if (s.pending) {
          // the image's entropy-coded segments, unstuffed, zero padded (the
          // marker parse counted the bytes: HuffSegDev::bits; removing the
          // stuffing on the device instead measured slower)
          const int32_t f = jc.seg_first[i - chunks[k].first];
          for (int32_t q = f; q < f + jc.seg_count[i - chunks[k].first]; q++) {
            const JpegChunk::Raw& r = jc.raw[q];
            uint8_t* to = sl.pin_in + jc.words_off + r.at;
            const int64_t n = mxd::jpeg::unstuff(r.b, r.e, to);
            std::memset(to + n, 0, (size_t)(((r.e - r.b + 4 + 15) & ~(int64_t)15) - n));
          }
          return;
        }
        std::memcpy(sl.pin_in + s.in_off, mxd::jpeg::coef_info(coefs_of(jpeg[i].coefs)).coef, s.in_size);
        return;
      }
      if (s.src_pinned) return;
      uint8_t* stage = sl.pin_in + s.in_off;
      const uint8_t* from = im.src + (int64_t)s.y0 * im.src_stride + (int64_t)s.x0 * im.channels;
      for (int32_t r = 0; r < s.rows; r++) std::memcpy(stage + r * s.pitch, from + (int64_t)r * im.src_stride, s.copy);
    });
    if (jpeg) {
      if (!jc.hjobs.empty()) {
        std::memcpy(sl.pin_in + jc.htabs_off, jc.htabs.data(), jc.htabs.size() * sizeof(mxd::HuffDev));
        std::memcpy(sl.pin_in + jc.himgs_off, jc.himgs.data(), jc.himgs.size() * sizeof(mxd::HuffImgDev));
        std::memcpy(sl.pin_in + jc.hsegs_off, jc.hsegs.data(), jc.hsegs.size() * sizeof(mxd::HuffSegDev));
        std::memcpy(sl.pin_in + jc.hjobs_off, jc.hjobs.data(), jc.hjobs.size() * sizeof(mxd::HuffJobDev));
      }
      std::memcpy(sl.pin_in + jc.planes_off, jc.planes.data(), jc.planes.size() * sizeof(mxd::JpegPlaneDev));
      for (auto& m : jc.imgs) m.out += jc.rgb_off;
      std::memcpy(sl.pin_in + jc.q_off, jc.qtabs.data(), jc.qtabs.size() * sizeof(uint16_t));
    }
    for (int32_t j = 0; j < cn; j++) {
      const int32_t i = chunks[k].first + j;
      const mxd_image& im = images[i];
      const Stage& s = st[i];
      if (jpeg) {
        mxd::JpegImgDev& m = jc.imgs[j];
        const uint8_t* win = sl.dev_mid + m.out + (int64_t)jpeg[i].win_y * m.pitch + (int64_t)jpeg[i].win_x * 3;
        where[j] = Stored{win, m.pitch, 0, 0, im.src_h};
        dev_imgs[j].src = win;
        dev_imgs[j].src_stride = m.pitch;
        if (!dst_device && !s.dst_dev) {
          dev_imgs[j].dst = sl.dev_out + s.out_off;
          dev_imgs[j].dst_stride = s.stage_row;
        } else if (s.dst_dev) {
          dev_imgs[j].dst = s.dst_dev;  // written in place over PCIe
        }
        // 4:2:0 YCbCr resized straight from its sample planes when a scatter
        // wave kernel takes it: no RGB frame (jpeg_color skips the image)
        const bool h2v2 = m.ncomp == 3 && !m.rgb && m.mode[0] == mxd::kUpFull && m.mode[1] == mxd::kUpH2V2 &&
                          m.mode[2] == mxd::kUpH2V2 && m.stride[1] == m.stride[2] && m.dw[1] == m.dw[2] &&
                          m.dh[1] == m.dh[2] && m.plane[0] < m.plane[1] && m.plane[1] < m.plane[2];
        if (h2v2 && g_tune[MXD_TUNE_JPEG_RGB].load() != 1 && (jpeg[i].win_x & 3) == 0) {
          mxd::YccDev& y = jc.ycc[j];
          y.cb = m.plane[1] - m.plane[0];
          y.cr = m.plane[2] - m.plane[0];
          y.ystride = m.stride[0];
          y.cstride = m.stride[1];
          y.dw = m.dw[1];
          y.dh = m.dh[1];
          y.win_x = jpeg[i].win_x;
          y.win_y = jpeg[i].win_y;
          y.records = (int32_t)std::min<int64_t>(y.cr + (int64_t)y.cstride * y.dh, INT32_MAX);
          const Stored planes{sl.dev_mid + m.plane[0], m.stride[0], 0, 0, im.src_h,
                              reinterpret_cast<const mxd::YccDev*>(sl.dev_in + jc.ycc_off) + j};
          if (y.cr + (int64_t)y.cstride * y.dh < INT32_MAX && ycc_plan_ok(dev_imgs[j], planes, launch_dtype(i), device)) {
            where[j] = planes;  // (dev_imgs[j] keeps the RGB frame's geometry, which run_batch validates)
            m.skip = 1;
            g_plane_sources.fetch_add(1, std::memory_order_relaxed);
          }
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
        dev_imgs[j].dst_stride = s.stage_row;
      } else if (s.dst_dev) {
        dev_imgs[j].dst = s.dst_dev;  // written in place over PCIe
      }
    }
    if (jpeg) {  // (after the fused-source decisions above)
      std::memcpy(sl.pin_in + jc.imgs_off, jc.imgs.data(), jc.imgs.size() * sizeof(mxd::JpegImgDev));
      std::memcpy(sl.pin_in + jc.ycc_off, jc.ycc.data(), jc.ycc.size() * sizeof(mxd::YccDev));
      if (!jc.hjobs.empty()) {
        // the entropy decode's publication records and launch control, staged
        // zero (one copy with the rest instead of a fill), the error word's
        // page-locked host twin in the control record
        if (!sl.huff_err) {
          MXD_HIP(hipHostMalloc(reinterpret_cast<void**>(&sl.huff_err), 64, hipHostMallocDefault));
        }
        // cleared for every staged chunk: a call that left early (another
        // chunk's error, a failed launch) never read the word back, and a job
        // that gave up there must not fail this call
        *sl.huff_err = 0;
        std::memset(sl.pin_in + jc.pub_off, 0, (size_t)(jc.coef_off - jc.pub_off));
        mxd::HuffCtlDev ctl{};
        ctl.err_host = const_cast<int32_t*>(reinterpret_cast<const int32_t*>(host_device_ptr(sl.huff_err)));
        std::memcpy(sl.pin_in + jc.pub_off + jc.hjobs.size() * sizeof(mxd::HuffPubDev), &ctl, sizeof ctl);
      }
    }
    if (in_staged > 0 && !pin_in_dev)
      MXD_HIP(hipMemcpyAsync(sl.dev_in, sl.pin_in, in_staged, hipMemcpyHostToDevice, sl.stream));
    sl.timed = g_tune[MXD_TUNE_DEVICE_TIMING].load() == 1;
    if (sl.timed) {
      if (!sl.k0) MXD_HIP(hipEventCreate(&sl.k0));
      if (!sl.k1) MXD_HIP(hipEventCreate(&sl.k1));
      if (jpeg) MXD_HIP(hipEventRecord(sl.k0, sl.stream));  // (else after the source row copies below)
    }
    if (jpeg) {
      if (!jc.hjobs.empty()) {
        // jpeg_chunk's job sizing keeps every job within one workgroup; a
        // larger one would leave subsequences undecoded and never publish
        if (jc.huff_threads > mxd::kHuffThreads)
          return fail(MXD_ERR_DEVICE, "jpeg entropy decode: a job of " + std::to_string(jc.huff_threads) +
                                          " subsequences exceeds a workgroup");
        // (the publication records and the ticket came zero with the staged
        // copy; the decode zeroes every block it starts, and the blocks
        // insufficient data leaves undecoded)
        auto* pub = reinterpret_cast<mxd::HuffPubDev*>(sl.dev_in + jc.pub_off);
        auto* ctl = reinterpret_cast<mxd::HuffCtlDev*>(pub + jc.hjobs.size());
        if (mxd::launch_jpeg_huff(reinterpret_cast<const uint32_t*>(sl.dev_in + jc.words_off),
                                  reinterpret_cast<const mxd::HuffDev*>(sl.dev_in + jc.htabs_off),
                                  reinterpret_cast<const mxd::HuffImgDev*>(sl.dev_in + jc.himgs_off),
                                  reinterpret_cast<const mxd::HuffSegDev*>(sl.dev_in + jc.hsegs_off),
                                  reinterpret_cast<const mxd::HuffJobDev*>(sl.dev_in + jc.hjobs_off),
                                  (int32_t)jc.hjobs.size(), jc.huff_threads, jc.huff_lds, pub, ctl,
                                  reinterpret_cast<int16_t*>(sl.dev_in), jc.huff_search, sl.stream))
          return fail(MXD_ERR_DEVICE, std::string("jpeg entropy decode launch: ") + hipGetErrorString(hipGetLastError()));
        // (a job that gives up sets *sl.huff_err itself: no copy back)
#ifdef MXD_HUFF_STAMPS
        // diagnostic build: the jobs' phase stamps (jpeghuff.hip) appended to $MXD_HUFF_STAMPS_FILE
        if (const char* path = getenv("MXD_HUFF_STAMPS_FILE")) {
          std::vector<mxd::HuffPubDev> rec(jc.hjobs.size());
          MXD_HIP(hipStreamSynchronize(sl.stream));
          MXD_HIP(hipMemcpy(rec.data(), pub, rec.size() * sizeof(mxd::HuffPubDev), hipMemcpyDeviceToHost));
          static std::mutex mu;
          std::lock_guard<std::mutex> lk(mu);
          if (FILE* f = fopen(path, "ab")) {
            const int64_t n = (int64_t)rec.size(), words = mxd::kHuffPubWords - 8;
            fwrite(&n, 8, 1, f);
            fwrite(&words, 8, 1, f);
            for (const auto& r : rec) fwrite(&r.w[8], 8, mxd::kHuffPubWords - 8, f);
            for (const auto& j : jc.hjobs) fwrite(&j, sizeof(j), 1, f);
            fclose(f);
          }
        }
#endif
      }
      mxd::launch_jpeg_idct(reinterpret_cast<const int16_t*>(sl.dev_in),
                            reinterpret_cast<const uint16_t*>(sl.dev_in + jc.q_off),
                            reinterpret_cast<const mxd::JpegPlaneDev*>(sl.dev_in + jc.planes_off),
                            (int32_t)jc.planes.size(), jc.nblocks, sl.dev_mid, sl.stream);
      bool rgb_frames = false;  // some image still needs its RGB frame
      for (const auto& m : jc.imgs) rgb_frames = rgb_frames || !m.skip;
      if (rgb_frames)
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
    if (sl.timed && !jpeg) MXD_HIP(hipEventRecord(sl.k0, sl.stream));
    // one launch per output dtype (a chunk mixes them only when a share of
    // its images is narrowed)
    {
      const int32_t first = chunks[k].first;
      bool mixed = false;
      for (int32_t i = first + 1; i < chunks[k].second; i++) mixed = mixed || st[i].narrow != st[first].narrow;
      int rc = MXD_OK;
      if (!mixed) {
        rc = run_batch(dev_imgs.data(), cn, launch_dtype(first), device, sl.stream, where.data());
      } else {
        for (int part = 0; part < 2 && rc == MXD_OK; part++) {
          std::vector<mxd_image> pi;
          std::vector<Stored> pw;
          for (int32_t j = 0; j < cn; j++)
            if (st[first + j].narrow == (part == 0)) {
              pi.push_back(dev_imgs[j]);
              pw.push_back(where[j]);
            }
          if (!pi.empty())
            rc = run_batch(pi.data(), (int32_t)pi.size(), part == 0 ? MXD_U8 : out_dtype, device, sl.stream, pw.data());
        }
      }
      if (rc) {
        sl.timed = false;  // (k1 not recorded for this chunk)
        return rc;
      }
    }
    if (sl.timed) MXD_HIP(hipEventRecord(sl.k1, sl.stream));
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
int jpeg_path(const mxd_jpeg_image* jimg, int32_t n, int32_t out_dtype, int32_t device, bool dst_device) {
  if (n < 0 || (n > 0 && !jimg)) return fail(MXD_ERR_INVALID, "mxd: bad image array");
  std::vector<mxd_image> imgs(n);
  for (int32_t i = 0; i < n; i++) {
    const mxd_jpeg_image& j = jimg[i];
    const std::string at = " (image " + std::to_string(i) + ")";
    if (!j.coefs) return fail(MXD_ERR_INVALID, "mxd: null coefs" + at);
    const mxd::jpeg::CoefInfo info = mxd::jpeg::coef_info(coefs_of(j.coefs));
    if (!info.device_ok)
      return fail(MXD_ERR_UNSUPPORTED, "mxd: this JPEG finishes on the host (mxd_jpeg_coefs_finish)" + at);
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

void host_trim() { host_pool().trim(); }

// Pixel maps of host images through a borrowed context (mxd_pixmap_host).
int pixmap_host(const mxd_pixmap* images, int32_t n, int32_t op, int32_t device) {
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


}  // namespace capi
}  // namespace mxd
