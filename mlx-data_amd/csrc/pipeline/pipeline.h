// pipeline.h -- the mlx-data Buffer/Stream operator surface for the image
// path, with the pixel work of image_resize_smallest_side / image_resize /
// image_center_crop / image_random_crop / image_random_h_flip deferred to the
// batch and executed by the fused gfx950 kernel through the C ABI
// (include/mxd_amd.h).
//
// Mirrors (semantics, error conditions, RNG draw order) of mlx-data 0.2.0:
//   Array / batch         mlx/data/Array.{h,cpp} (batch :465-498, sub :544-583)
//   Sample, check_key     mlx/data/Sample.{h,cpp}:13,18-29
//   Op / KeyTransformOp   mlx/data/op/{Op,KeyTransform}.{h,cpp}
//   image ops             mlx/data/op/ImageTransform.cpp:22-158,317-332
//   LoadImage             mlx/data/op/LoadImage.cpp:23-48
//   buffers               mlx/data/buffer/{FromVector,Perm,Shuffle,Transform,Batch}.cpp
//   streams               mlx/data/stream/{FromBuffer,Transform,Batch,Prefetch,OrderedPrefetch}.cpp
//   state                 mlx/data/core/State.cpp:9-22
//   merge_batch           mlx/data/core/Utils.cpp:209-252, BatchShape.cpp:26-66
#pragma once

#include <array>
#include <condition_variable>
#include <cstdint>
#include <functional>
#include <future>
#include <memory>
#include <mutex>
#include <queue>
#include <random>
#include <string>
#include <thread>
#include <unordered_map>
#include <vector>

namespace mxd {
namespace pipe {

// Same order as mlx::data::ArrayType.
enum class DType { Any, UInt8, Int8, Int32, Int64, Float, Double };
int64_t itemsize(DType t);

class Array;

// An entropy-decoded JPEG (mxd_jpeg_coefs_decode): load_image's output when
// the device finish is on (set_device_decode).  Its pixels come from the host
// finish on first direct access, or from the GPU finish inside the batch
// launch that resizes / crops it (mxd_jpeg_resize_crop_*); the bytes are the
// same either way.
struct JpegSource;

// Pixel work that has not run yet: take the window (sx, sy, sw, sh) of `src`,
// resize it to resize_w x resize_h (identity when equal), keep the crop window
// of that, mirror it if `flip`.  The output is `crop_h x crop_w x C` uint8.
// It materialises on the GPU -- one launch for a whole batch when the batch
// node sees plans, one launch per image when something reads it directly.
struct ImagePlan {
  std::shared_ptr<Array> src;  // (H, W, C) uint8, materialised
  int64_t sx = 0, sy = 0, sw = 0, sh = 0;
  int64_t resize_w = 0, resize_h = 0;
  int64_t crop_x = 0, crop_y = 0, crop_w = 0, crop_h = 0;
  bool flip = false;
  // Went through core::image::resize (stbir): 4-channel images are then
  // alpha-weighted (STBIR_RGBA); crops and mirrors alone never are.
  bool resampled = false;
  // image_to_float: the kernel writes float32 q / 255 (MXD_F32_DIV255)
  // instead of the uint8 q; the array's type is then Float.
  bool f32 = false;
  int64_t channels() const;
};

class Array {
 public:
  Array(DType type, std::vector<int64_t> shape);                      // zero-initialised storage
  Array(DType type, std::vector<int64_t> shape, std::shared_ptr<void> data);
  // Device-resident storage (a batch made with batch(..., device=d)):
  // data() is then a device pointer on `device`.
  Array(DType type, std::vector<int64_t> shape, std::shared_ptr<void> data, int device);
  explicit Array(std::shared_ptr<const ImagePlan> plan);              // lazy image
  Array(std::shared_ptr<const JpegSource> jpeg, int64_t height, int64_t width);  // lazy decode, (H, W, 3)

  DType type() const { return type_; }
  const std::vector<int64_t>& shape() const { return shape_; }
  int64_t shape(int d) const;
  int ndim() const { return (int)shape_.size(); }
  int64_t size() const;
  int64_t nbytes() const { return size() * itemsize(type_); }
  // Materialises a pending image plan (one GPU launch) on first use.
  void* data() const;
  const std::shared_ptr<const ImagePlan>& plan() const { return plan_; }
  bool pending() const;
  // The entropy-decoded JPEG of a lazy decode not materialised yet, else null.
  std::shared_ptr<const JpegSource> jpeg() const;
  // -1: host memory; else the HIP device holding data().
  int device() const { return device_; }

 private:
  DType type_;
  std::vector<int64_t> shape_;
  mutable std::shared_ptr<void> data_;
  std::shared_ptr<const ImagePlan> plan_;
  mutable std::shared_ptr<const JpegSource> jpeg_;
  int device_ = -1;
  mutable std::mutex mu_;
};

using Sample = std::unordered_map<std::string, std::shared_ptr<Array>>;

std::shared_ptr<Array> check_key(const Sample& s, const std::string& key);

// Devices the fused kernel may use (default: all visible).  With several,
// one batch is split into contiguous slices, one per device, each launched
// from its own host thread (the reference's shard / partition analogue,
// op/Shard.cpp:11-20, stream/Partition.cpp:23-35); outputs land at the same
// offsets, so the batch is identical to a single-device one.
void set_devices(const std::vector<int>& devices);
std::vector<int> devices();
// How run_host splits a batch of n images over ndev devices (pipeline.cpp).
constexpr int64_t kMinSliceImages = 64;
struct Slice {
  int64_t device;      // index into devices()
  int64_t begin, end;  // images [begin, end) of the batch
};
std::vector<Slice> split_batch(int64_t n, int64_t ndev, uint64_t first);

// load_image's JPEG route: on (the default when a device is visible), only
// the entropy decode runs in load_image and the GPU finishes the decode inside
// the batch launch; off, load_image decodes whole on the
// host.  Identical bytes either way.
void set_device_decode(bool on);
// With the device decode on: the Huffman decode too runs on the GPU for the
// files it covers (mxd_jpeg_coefs_parse; default on).  Off: the host
// entropy-decodes every file (round 3's split).
void set_device_entropy(bool on);
bool device_entropy();
bool device_decode();
// Bytes the device batch pool holds for `device` (idle and pending blocks).
size_t device_pool_bytes(int device);
// Per-device batch calls made (fused launches, one per device slice) and the
// JPEG images they carried since the last reset (diagnostics, tests).
std::pair<int64_t, int64_t> run_on_stats(bool reset);
std::vector<int64_t> pipe_stats(bool reset);  // diagnostics: see pipeline.cpp g_pipe_ns

// ---------------------------------------------------------------- state
struct State {
  std::mt19937 gen;
  int64_t version = 0;
};
void set_state(int64_t seed);
std::shared_ptr<State> get_state();

// ---------------------------------------------------------------- ops
class Op {
 public:
  virtual ~Op() = default;
  virtual Sample apply(const Sample& sample) const = 0;
};

class KeyTransformOp : public Op {
 public:
  KeyTransformOp(std::string ikey, std::string okey) : ikey_(std::move(ikey)), okey_(std::move(okey)) {}
  Sample apply(const Sample& sample) const override;
  virtual std::shared_ptr<Array> apply_key(const std::shared_ptr<Array>& x) const = 0;

 protected:
  std::string ikey_, okey_;
};

class KeyTransform : public KeyTransformOp {
 public:
  using Fn = std::function<std::shared_ptr<Array>(const std::shared_ptr<Array>&)>;
  KeyTransform(std::string ikey, Fn fn, std::string okey) : KeyTransformOp(std::move(ikey), std::move(okey)), fn_(std::move(fn)) {}
  std::shared_ptr<Array> apply_key(const std::shared_ptr<Array>& x) const override { return fn_(x); }

 private:
  Fn fn_;
};

class ImageOp : public KeyTransformOp {
 public:
  using KeyTransformOp::KeyTransformOp;
  std::shared_ptr<Array> apply_key(const std::shared_ptr<Array>& x) const override;
  virtual std::shared_ptr<Array> apply_image(const std::shared_ptr<Array>& img) const = 0;
  // (F, H, W, C) video: op/ImageTransform.cpp:33-70 -- apply_image per frame,
  // every frame the size of the first; pending frame plans run as one batched
  // launch writing straight into the result.
  virtual std::shared_ptr<Array> apply_video(const std::shared_ptr<Array>& video) const;
};

// Frame i of a materialised (F, H, W, C) video, sharing its storage.
std::shared_ptr<Array> video_frame(const std::shared_ptr<Array>& video, int64_t i);
// Stacks per-frame results (pending plans in one launch) into (F, h, w, c).
std::shared_ptr<Array> stack_frames(const std::vector<std::shared_ptr<Array>>& frames);

class ImageResizeSmallestSide : public ImageOp {
 public:
  ImageResizeSmallestSide(std::string ikey, int64_t size, std::string okey)
      : ImageOp(std::move(ikey), std::move(okey)), size_(size) {}
  std::shared_ptr<Array> apply_image(const std::shared_ptr<Array>& img) const override;

 private:
  int64_t size_;
};

class ImageResize : public ImageOp {
 public:
  ImageResize(std::string ikey, int64_t w, int64_t h, std::string okey)
      : ImageOp(std::move(ikey), std::move(okey)), w_(w), h_(h) {}
  std::shared_ptr<Array> apply_image(const std::shared_ptr<Array>& img) const override;

 private:
  int64_t w_, h_;
};

class ImageCenterCrop : public ImageOp {
 public:
  ImageCenterCrop(std::string ikey, int64_t w, int64_t h, std::string okey)
      : ImageOp(std::move(ikey), std::move(okey)), w_(w), h_(h) {}
  std::shared_ptr<Array> apply_image(const std::shared_ptr<Array>& img) const override;

 private:
  int64_t w_, h_;
};

class ImageRandomCrop : public ImageOp {
 public:
  ImageRandomCrop(std::string ikey, int64_t w, int64_t h, std::string okey)
      : ImageOp(std::move(ikey), std::move(okey)), w_(w), h_(h) {}
  std::shared_ptr<Array> apply_video(const std::shared_ptr<Array>& video) const override;
  std::shared_ptr<Array> apply_image(const std::shared_ptr<Array>& img) const override;

 private:
  int64_t w_, h_;
};

class ImageRandomHFlip : public ImageOp {
 public:
  ImageRandomHFlip(std::string ikey, float prob, std::string okey)
      : ImageOp(std::move(ikey), std::move(okey)), prob_(prob) {}
  std::shared_ptr<Array> apply_image(const std::shared_ptr<Array>& img) const override;
  std::shared_ptr<Array> apply_video(const std::shared_ptr<Array>& video) const override;

 private:
  float prob_;
};

// Fused normalize: the reference's post-batch
// `key_transform(key, lambda x: x.astype("float32") / 255)`
// (benchmarks/comparative/caltech101/mlx_data.py:34,46) as an image op ahead
// of batch.  A pending image (resize / crop / mirror not run yet) only
// records it, so batch writes the float32 tensor from the same launch; a
// materialised uint8 image is converted by one identity launch.  Values are
// exactly float(q) / 255.0f.  UInt8 input only ("image must be of type
// UInt8", core/image/ImageTransform.cpp:17-21).
class ImageToFloat : public ImageOp {
 public:
  ImageToFloat(std::string ikey, std::string okey) : ImageOp(std::move(ikey), std::move(okey)) {}
  std::shared_ptr<Array> apply_image(const std::shared_ptr<Array>& img) const override;
};

// op/ImageTransform.h:139-152 ImageRotate: nearest-pixel rotation about the
// centre (core::image::rotate -> affine), one GPU pixel-map launch.
class ImageRotate : public ImageOp {
 public:
  ImageRotate(std::string ikey, double angle, bool crop, std::string okey)
      : ImageOp(std::move(ikey), std::move(okey)), angle_(angle), crop_(crop) {}
  std::shared_ptr<Array> apply_image(const std::shared_ptr<Array>& img) const override;

 private:
  double angle_;
  bool crop_;
};

// op/ImageTransform.h:154-167 ImageChannelReduction: RGB -> (H, W, 1) gray in
// 16.16 fixed point with a named preset; unknown presets throw at construction.
class ImageChannelReduction : public ImageOp {
 public:
  ImageChannelReduction(std::string ikey, const std::string& preset, std::string okey);
  std::shared_ptr<Array> apply_image(const std::shared_ptr<Array>& img) const override;

 private:
  float params_[4];  // bias, m0, m1, m2
};

// op/ImageTransform.h ImageRandomAreaCrop: a crop whose area and aspect ratio
// are drawn by rejection sampling (Inception-style); the image unchanged when
// no trial meets the constraints.
class ImageRandomAreaCrop : public ImageOp {
 public:
  ImageRandomAreaCrop(std::string ikey, std::pair<float, float> area_range, std::pair<float, float> aspect_ratio_range,
                      int num_trial, std::string okey);
  std::shared_ptr<Array> apply_image(const std::shared_ptr<Array>& img) const override;
  std::shared_ptr<Array> apply_video(const std::shared_ptr<Array>& video) const override;
  // (x, y, w, h) of the crop for a w x h image, all 0 when none was found.
  std::array<int64_t, 4> draw(int64_t w, int64_t h) const;

 private:
  std::pair<float, float> area_, aspect_;
  int trials_;
};

// Decoder hook: (path or encoded bytes, from_memory) -> (H, W, 3) uint8, or
// nullptr when the image cannot be decoded.  Installed by the binding.
using ImageDecoder = std::function<std::shared_ptr<Array>(const std::string& path, const std::shared_ptr<Array>& bytes,
                                                          bool from_memory, bool info)>;
void set_image_decoder(ImageDecoder dec);

class LoadImage : public KeyTransformOp {
 public:
  LoadImage(std::string ikey, std::string prefix, bool info, std::string format, bool from_memory, std::string okey);
  std::shared_ptr<Array> apply_key(const std::shared_ptr<Array>& x) const override;

 private:
  std::string prefix_;
  bool info_;
  std::string format_;
  bool from_memory_;
};

// ---------------------------------------------------------------- batching
// array::batch semantics (pad with pad_value to the max shape; optional
// concatenation dim).  Pending image plans of one key become one fused launch.
// device >= 0: the batch is made in that device's memory:
// pending images are written there by the kernel (host sources staged, no
// D2H); anything else is batched on the host and uploaded once.
std::shared_ptr<Array> batch_arrays(const std::vector<std::shared_ptr<Array>>& arrs, double pad_value, int dim,
                                    bool has_dim, int device = -1);

// Where merge_batch puts each key: device < 0 everything on the host; else
// the listed keys on `device`, or (empty list) every key with a pending image.
struct DeviceOut {
  int device = -1;
  std::vector<std::string> keys;
};
Sample merge_batch(const std::vector<Sample>& samples, const std::unordered_map<std::string, double>& pad,
                   const std::unordered_map<std::string, int>& dims, const DeviceOut& out = {});

// ---------------------------------------------------------------- threads
// Workers share the queue state with the pool, so the pool may be destroyed
// from one of its own workers: a finished task's result can hold the last
// reference to the pipeline that owns the pool (an exception carrying a
// Python traceback, released on the worker).  That worker is detached
// instead of joined and leaves its loop through the shared state.
class ThreadPool {
 public:
  explicit ThreadPool(int n);
  ~ThreadPool();
  std::future<Sample> enqueue(std::function<Sample()> fn);
  // Whether the calling thread is one of this pool's workers.
  bool on_worker() const;

 private:
  struct State {
    std::queue<std::packaged_task<Sample()>> tasks;
    std::mutex mu;
    std::condition_variable cv;
    bool stop = false;
  };
  std::shared_ptr<State> st_;
  std::vector<std::thread> workers_;
};

// ---------------------------------------------------------------- buffers
class Buffer {
 public:
  virtual ~Buffer() = default;
  virtual int64_t size() const = 0;
  virtual Sample get(int64_t idx) const = 0;
};

class FromVector : public Buffer {
 public:
  explicit FromVector(std::vector<Sample> data) : data_(std::move(data)) {}
  int64_t size() const override { return (int64_t)data_.size(); }
  Sample get(int64_t idx) const override;

 private:
  std::vector<Sample> data_;
};

class Perm : public Buffer {
 public:
  Perm(std::shared_ptr<Buffer> b, std::vector<int64_t> perm);
  int64_t size() const override { return (int64_t)perm_.size(); }
  Sample get(int64_t idx) const override;

 private:
  std::shared_ptr<Buffer> b_;
  std::vector<int64_t> perm_;
};
std::shared_ptr<Buffer> shuffle_buffer(const std::shared_ptr<Buffer>& b);

class BufferTransform : public Buffer {
 public:
  BufferTransform(std::shared_ptr<Buffer> b, std::shared_ptr<Op> op) : b_(std::move(b)), op_(std::move(op)) {}
  int64_t size() const override { return b_->size(); }
  Sample get(int64_t idx) const override;

 private:
  std::shared_ptr<Buffer> b_;
  std::shared_ptr<Op> op_;
};

class BufferBatch : public Buffer {
 public:
  BufferBatch(std::shared_ptr<Buffer> b, int64_t batch_size, std::unordered_map<std::string, double> pad,
              std::unordered_map<std::string, int> dims, DeviceOut out = {});
  int64_t size() const override { return size_; }
  Sample get(int64_t idx) const override;

 private:
  std::shared_ptr<Buffer> b_;
  int64_t bs_, size_;
  std::unordered_map<std::string, double> pad_;
  std::unordered_map<std::string, int> dims_;
  DeviceOut out_;
};

// ---------------------------------------------------------------- streams
class Stream {
 public:
  virtual ~Stream() = default;
  virtual Sample next() const = 0;
  virtual void reset() = 0;
};

class FromBuffer : public Stream {
 public:
  explicit FromBuffer(std::shared_ptr<Buffer> b) : b_(std::move(b)) {}
  Sample next() const override;
  void reset() override;

 private:
  std::shared_ptr<Buffer> b_;
  mutable std::mutex mu_;
  mutable int64_t idx_ = 0;
};

class StreamTransform : public Stream {
 public:
  StreamTransform(std::shared_ptr<Stream> s, std::shared_ptr<Op> op) : s_(std::move(s)), op_(std::move(op)) {}
  Sample next() const override;
  void reset() override { s_->reset(); }

 private:
  std::shared_ptr<Stream> s_;
  std::shared_ptr<Op> op_;
};

class StreamBatch : public Stream {
 public:
  StreamBatch(std::shared_ptr<Stream> s, int64_t batch_size, std::unordered_map<std::string, double> pad,
              std::unordered_map<std::string, int> dims, DeviceOut out = {});
  Sample next() const override;
  void reset() override { s_->reset(); }

 private:
  std::shared_ptr<Stream> s_;
  int64_t bs_;
  std::unordered_map<std::string, double> pad_;
  std::unordered_map<std::string, int> dims_;
  DeviceOut out_;
};

class Prefetch : public Stream {
 public:
  Prefetch(std::shared_ptr<Stream> s, int prefetch_size, int num_threads);
  ~Prefetch() override;
  Sample next() const override;
  void reset() override;

 private:
  std::shared_ptr<Stream> s_;
  std::unique_ptr<ThreadPool> pool_;
  int size_;
  mutable std::mutex mu_;
  mutable std::queue<std::future<Sample>> cache_;
};

class OrderedPrefetch : public Stream {
 public:
  OrderedPrefetch(std::shared_ptr<Buffer> b, int prefetch_size, int num_threads);
  ~OrderedPrefetch() override;
  Sample next() const override;
  void reset() override;

 private:
  std::shared_ptr<Buffer> b_;
  std::unique_ptr<ThreadPool> pool_;
  int size_;
  mutable std::mutex mu_;
  mutable std::vector<std::future<Sample>> cache_;
  mutable int64_t idx_ = 0;
};

}  // namespace pipe
}  // namespace mxd
