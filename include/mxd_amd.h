/*
 * mxd_amd.h -- C ABI of the MI355X image resample/crop stage for the mlx-data
 * Buffer/Stream pipeline.
 *
 * The library (mlx-data_amd/libmxd_amd.so) replaces, for the per-pixel hot path
 * only, these reference interfaces (file:line into ml-explore/mlx-data 0.2.0):
 *
 *   core::image::scale(img, double)          mlx/data/core/image/ImageTransform.cpp:33-39
 *   core::image::resize(img, dw, dh)         mlx/data/core/image/ImageTransform.cpp:41-62
 *     -> stbir_resize_uint8_linear(...)       (stb_image_resize2, triangle filter, :7-10,49-60)
 *   core::image::crop(img, x, y, w, h)       mlx/data/core/image/ImageTransform.cpp:64-73
 *   core::image::hflip(img)                  mlx/data/core/image/ImageTransform.cpp:123-140
 *   op::ImageResizeSmallestSide::apply_image mlx/data/op/ImageTransform.cpp:78-94
 *   op::ImageCenterCrop::apply_image         mlx/data/op/ImageTransform.cpp:115-126
 *   op::ImageRandomCrop / ImageRandomHFlip   mlx/data/op/ImageTransform.cpp:135-158,323-332
 *   array::batch (NHWC stack + pad)          mlx/data/Array.cpp:465-498
 *   x.astype("float32") / 255 (normalize)    benchmarks/comparative/caltech101/mlx_data.py:46
 *
 * Conventions: plain pointers and sizes only; every function returns an int
 * status (MXD_OK == 0) and never throws.  On failure the thread-local message
 * returned by mxd_last_error() holds the reason, using the reference's own
 * error strings where the reference has one.  All functions are thread-safe.
 * Streams are HIP streams passed as void* (NULL = the device's null stream).
 */
#ifndef MXD_AMD_H
#define MXD_AMD_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* 5: the round-4 additions (numbered in round 5): mxd_jpeg_coefs_parse (device
 * entropy decode pending), mxd_jpeg_coefs_entropy_pending,
 * mxd_device_synchronize, and the tuning knobs MXD_TUNE_HUFF_BITS,
 * MXD_TUNE_HUFF_GLOBAL, MXD_TUNE_HOST_WAIT; round 5: MXD_TUNE_HOST_STREAMS,
 * MXD_TUNE_HUFF_JOB, MXD_TUNE_JPEG_RGB, mxd_jpeg_plane_sources,
 * mxd_host_stats, mxd_jpeg_coefs_load.
 * 6 (round 6): the knobs MXD_TUNE_DEVICE_TIMING, MXD_TUNE_LOAD_POLICY,
 * mxd_device_stats and mxd_copy_bandwidth_policy; CMYK / YCCK files finish (and sequential ones
 * entropy-decode) on the device; mxd_jpeg_coefs_entropy_pending no longer
 * reports 2 (progressive files are
 * entropy-decoded on the host).
 * 7 (round 6, later): f32 results bound for host memory cross the link as
 * u8 and are expanded (x / 255) on the host -- the knob MXD_TUNE_F32_LINK and
 * the counter mxd_narrow_returns. */
#define MXD_ABI_VERSION 7

enum mxd_status {
  MXD_OK = 0,
  MXD_ERR_INVALID = 1,     /* bad argument (reference: std::runtime_error / invalid_argument) */
  MXD_ERR_UNSUPPORTED = 2, /* valid for the reference, not supported by this build */
  MXD_ERR_DEVICE = 3,      /* HIP runtime failure */
  MXD_ERR_NOMEM = 4
};

/* Output element type of a resample launch. */
enum mxd_dtype {
  MXD_U8 = 0,          /* uint8, as core::image::resize + crop produce */
  MXD_F32_DIV255 = 1   /* float32 q/255.0f of the uint8 result, bit-exact to the
                          NumPy x.astype("float32")/255 the reference benchmark runs */
};

/*
 * One image of a batch: source HWC uint8 in device memory, the resize target
 * (the dims core::image::scale / resize would produce), the crop window inside
 * the resized image, and where the (crop_h x crop_w x channels) result goes.
 *
 *   src          device pointer to the first byte of row 0; the buffer must span
 *                src_stride * src_h bytes (the kernels read whole 4-byte words
 *                of a row up to src_stride, never past it)
 *   src_stride   bytes between source rows (>= src_w*channels)
 *   resize_w/h   resized dims, >= 1 (reference: verify_dimensions, ImageTransform.cpp:23-31)
 *   crop_x/y/w/h window in resized coordinates; must lie inside the resized image
 *                (reference: ImageCenterCrop :119-122, array::sub Array.cpp:558-566)
 *   flip         nonzero: mirror the cropped result horizontally (core::image::hflip)
 *   dst          device pointer to row 0 of the output image
 *   dst_stride   bytes between output rows
 *   rgba_weighted  4 channels only: nonzero = the resample is stbir's STBIR_RGBA
 *                (colours weighted by alpha while filtering), as
 *                core::image::resize does for c = 4 (ImageTransform.cpp:49-58);
 *                zero = channels filtered independently, which an identity
 *                resize turns into the exact copy a pure crop / flip is
 *                (array::sub / hflip never call stbir)
 */
typedef struct mxd_image {
  const uint8_t* src;
  int64_t src_stride;
  int32_t src_w, src_h, channels;
  int32_t resize_w, resize_h;
  int32_t crop_x, crop_y, crop_w, crop_h;
  int32_t flip;
  void* dst;
  int64_t dst_stride;
  int32_t rgba_weighted;
  int32_t reserved;
} mxd_image;

/* ---- library / errors ------------------------------------------------- */
int mxd_abi_version(void);
const char* mxd_last_error(void);
int mxd_device_count(int* count);
/* Run manifest (SURVEY.md §5 metrics): marketing name, gcnArchName and
 * compute-unit count of `device`; strings are NUL-terminated, truncated to
 * their buffer. */
int mxd_device_properties(int32_t device, char* name, size_t name_len, char* arch, size_t arch_len, int32_t* cus);

/* ---- reference geometry (host only, no device needed) ------------------ */

/* ImageResizeSmallestSide + core::image::scale: target dims of resizing the
 * smaller side of (w, h) to `size` (lround of a double scale). */
int mxd_resize_smallest_side_dims(int64_t w, int64_t h, int64_t size, int64_t* out_w, int64_t* out_h);

/* ImageCenterCrop: origin of a (cw x ch) centre crop of a (w x h) image. */
int mxd_center_crop_origin(int64_t w, int64_t h, int64_t cw, int64_t ch, int64_t* x, int64_t* y);

/* Resampling taps of one axis for output pixels [crop_off, crop_off+crop_len)
 * of an in_size -> out_size resize: first input index, tap count and weights
 * (row-major [crop_len][max_taps], zero padded).  *taps_needed receives the
 * widest tap count; if it exceeds max_taps nothing is written and
 * MXD_ERR_INVALID is returned. */
int mxd_axis_taps(int32_t in_size, int32_t out_size, int32_t crop_off, int32_t crop_len, int32_t max_taps,
                  int32_t* first, int32_t* ntaps, float* weights, int32_t* taps_needed);

/* ---- the hot path -------------------------------------------------------- */

/* Fused resize + crop (+ flip) (+ /255 normalize) of n images on `device`,
 * enqueued on `stream`.  One kernel launch per call; inputs and outputs are in
 * device memory.  Asynchronous: returns once the work is enqueued. */
int mxd_resize_crop_batch(const mxd_image* images, int32_t n, int32_t out_dtype, int32_t device, void* stream);

/* Kernel policy: a process-wide switch between kernels that compute
 * bit-identical results (for tests and tuning; default 0 = automatic choice:
 * a wave kernel -- one wave streams an image band's row pieces -- wherever
 * its tap buckets fit (every measured configuration C2..C5 runs fastest
 * there), else the band kernel -- persistent workgroups stream image bands'
 * source rows into LDS by LDS-DMA, any downscale ratio up to 32 taps per
 * axis -- else the general kernel).  MXD_POLICY_PREFER_BAND: the band kernel
 * first wherever its classes fit; MXD_POLICY_NO_BAND: never the band kernel
 * (any of the wave-kernel bits below implies it).  MXD_POLICY_NO_SCATTER: wave kernels gather every
 * output row's taps instead of following a scatter schedule; MXD_POLICY_NO_WAVE: every image takes the
 * general workgroup-tile kernel; MXD_POLICY_NARROW: wave kernels keep the
 * narrow per-lane window (no wide RGB strips, no byte lanes);
 * MXD_POLICY_NO_DESC_CACHE: every batch uploads its descriptor array even
 * when a cached slot holds the same bytes (measures the per-batch upload of
 * fresh descriptors); MXD_POLICY_NO_BYTES: RGB scatter kernels keep whole
 * pixels per lane instead of 16 contiguous bytes per lane (by default byte
 * lanes run where they need no more strips); MXD_POLICY_BYTES: byte lanes
 * wherever a kernel exists; MXD_POLICY_NO_ZERO_COPY: the host path DMAs
 * page-locked sources' footprint rows to the device (2-D copies) and results
 * back to page-locked destinations instead of letting the kernel read and
 * write them in place over PCIe.  Returns the previous policy. */
enum mxd_policy {
  MXD_POLICY_AUTO = 0,
  MXD_POLICY_NO_SCATTER = 1,
  MXD_POLICY_NO_WAVE = 2,
  MXD_POLICY_NARROW = 4,
  MXD_POLICY_NO_DESC_CACHE = 8,
  MXD_POLICY_NO_BYTES = 16,
  MXD_POLICY_BYTES = 32,
  MXD_POLICY_NO_ZERO_COPY = 64,
  MXD_POLICY_NO_BAND = 128,
  MXD_POLICY_PREFER_BAND = 256
};
int mxd_set_kernel_policy(int32_t policy);

/* Tuning knobs (process-wide, for measurements; 0 = automatic).  Returns the
 * previous value, or -1 for an unknown knob.
 * MXD_TUNE_BAND_ROWS: output rows per band-kernel unit;
 * MXD_TUNE_BAND_LA: row groups the band kernel keeps in flight per unit;
 * MXD_TUNE_BAND_GRID: band-kernel workgroups (0: as many as the device holds
 * at once, each running a stream of units; 1: one per unit; n > 1: n);
 * MXD_TUNE_DESC: how a batch's new descriptor array reaches the kernels (1:
 * copy stream + cross-stream wait; 2: copy on the launch stream; 3: kernels
 * read the page-locked slot in place; 4: as 3, non-coherent allocation; 6
 * (the default): the host stores the array into device memory through the
 * large PCI BAR, falling back to 4 without one);
 * MXD_TUNE_STREAMS: streams the launches of a mixed batch (one per kernel
 * shape) spread over (1: all on the caller's stream; default 2, at most 4);
 * MXD_TUNE_HUFF_BITS: shortest subsequence (bits, a multiple of 32) of the
 * device entropy decode (default 512; tests force short ones so many
 * subsequences must synchronise);
 * MXD_TUNE_HUFF_GLOBAL: 1 = the device entropy decode reads every job's
 * entropy-coded words from device memory (default: from LDS for the jobs
 * whose words fit it);
 * MXD_TUNE_HOST_WAIT: how a host-path call waits for its chunks (read when
 * a host-path context's events are first created): 0 / 1 = events created
 * with hipEventBlockingSync, the waiting thread sleeps (default); 2 = HIP's
 * default polling wait;
 * MXD_TUNE_HOST_STREAMS: streams per device the host-path calls launch on
 * (read when a host-path context is first set up): 0 = every context slot
 * owns one (default); n > 0 = the slots share n library streams;
 * MXD_TUNE_HUFF_JOB: most own subsequences per device entropy-decode job
 * (workgroup); 0 = kHuffThreads - kHuffWarm (1000);
 * MXD_TUNE_JPEG_RGB: 1 = every device-finished JPEG goes through an RGB
 * frame (jpeg_color) before the resize; 0 (default) = a 4:2:0 image whose
 * resize runs on a scatter wave kernel is resized straight from its sample
 * planes (no RGB frame);
 * MXD_TUNE_DEVICE_TIMING: 1 = every host-path chunk records two timing events
 * on its stream, before its first kernel and after its last, and
 * mxd_device_stats sums the span between them (diagnostics: what the batch
 * calls cost the device; read when a chunk is launched);
 * MXD_TUNE_LOAD_POLICY: cache policy of the scatter wave kernels' source
 * loads (0 = automatic: streaming (nt) when the call's sources total >= 128
 * MiB, else the default policy; 1 = default policy always; 2 = nt always);
 * MXD_TUNE_F32_LINK (ABI 7): how a host-ending call returns MXD_F32_DIV255
 * results staged through page-locked memory (0 = automatic: the kernels'
 * u8 bytes cross the link and the host writes u8 / 255 -- the same f32 bytes,
 * a quarter of the link traffic, page-locked destinations included; 1 = the
 * f32 results cross the link, and page-locked destinations are written by
 * the device in place; 2..99 = that percentage of a call's images narrowed,
 * spread evenly, the rest as with 1). */
enum mxd_tune {
  MXD_TUNE_BAND_ROWS = 0,
  MXD_TUNE_BAND_LA = 1,
  MXD_TUNE_BAND_GRID = 2,
  MXD_TUNE_DESC = 3,
  MXD_TUNE_STREAMS = 4,
  MXD_TUNE_HUFF_BITS = 5,
  MXD_TUNE_HUFF_GLOBAL = 6,
  MXD_TUNE_HOST_WAIT = 7,
  MXD_TUNE_HOST_STREAMS = 8,
  MXD_TUNE_HUFF_JOB = 9,
  MXD_TUNE_JPEG_RGB = 10,
  MXD_TUNE_DEVICE_TIMING = 11,
  MXD_TUNE_LOAD_POLICY = 12,
  MXD_TUNE_F32_LINK = 13,
  MXD_TUNE_COUNT = 14
};
int mxd_set_tuning(int32_t knob, int32_t value);

/* The wave-kernel plan of one image on `device`, i.e. what runs when the
 * band kernel declines it or is off (diagnostics, tests): info[0] = 1 wave
 * kernel / 0 general kernel, then kind
 * (0 gather, 2 scatter), tap bucket, scatter S, scatter DMAX, output pixels
 * per lane, strips, source pixels per lane (RGB 16: byte lanes, 16 bytes per
 * lane).  Host only: needs no device. */
int mxd_describe_plan(const mxd_image* image, int32_t out_dtype, int32_t device, int32_t* info8);

/* The band-kernel plan of one image (host only): info[0] = 1 when the band
 * kernel takes it (under the current policy), then horizontal tap class, row
 * slots per group (DB), accumulator slots, source window KiB per strip row,
 * strips, strip columns, prologue groups, most new source rows per output
 * row, groups in flight, LDS bytes per workgroup, 0. */
int mxd_describe_band_plan(const mxd_image* image, int32_t out_dtype, int32_t* info12);

/* Measured device-memory ceiling: a 16-byte-per-lane streaming copy of `bytes`
 * (read + write counted), averaged over `iters` launches, in GB/s. */
int mxd_copy_bandwidth(size_t bytes, int32_t device, int32_t iters, float* gbps);
/* The same copy with a cache policy on its loads and stores (ABI 6): 0 the
 * default (= mxd_copy_bandwidth), 1 nontemporal, 2 nontemporal + sc1. */
int mxd_copy_bandwidth_policy(size_t bytes, int32_t device, int32_t iters, int32_t policy, float* gbps);

/* ---- device memory / streams / events (so a C or C++ host needs no torch) */
int mxd_set_device(int32_t device);
int mxd_malloc_device(void** ptr, size_t bytes, int32_t device);
int mxd_free_device(void* ptr, int32_t device);
int mxd_malloc_pinned(void** ptr, size_t bytes);
int mxd_free_pinned(void* ptr);
int mxd_memcpy_h2d_async(void* dst, const void* src, size_t bytes, void* stream);
int mxd_memcpy_d2h_async(void* dst, const void* src, size_t bytes, void* stream);
/* 2-D copy: rows of `width` bytes, host pitch spitch -> device pitch dpitch. */
int mxd_memcpy2d_h2d_async(void* dst, size_t dpitch, const void* src, size_t spitch, size_t width, size_t rows,
                           void* stream);
int mxd_memset_async(void* dst, int value, size_t bytes, void* stream);
int mxd_stream_create(int32_t device, void** stream);
int mxd_stream_destroy(void* stream);
int mxd_stream_synchronize(void* stream);
/* Waits for all work on every stream of `device` (hipDeviceSynchronize). */
int mxd_device_synchronize(int32_t device);
int mxd_event_create(void** event);
int mxd_event_destroy(void* event);
int mxd_event_record(void* event, void* stream);
int mxd_event_synchronize(void* event);
int mxd_event_elapsed_ms(float* ms, void* start, void* stop);

/* ---- host-resident convenience path ------------------------------------ */

/* Host image in, host result out; synchronous.  `images[i].src` and
 * `images[i].dst` are HOST pointers here.  Only each image's source footprint
 * (the rows and columns its crop window's taps touch) is read, zero copy:
 * page-locked sources and destinations are read and written in place by the
 * kernel over PCIe; pageable sources are staged into the call's page-locked
 * buffers by helper threads (the kernel reads them there) and pageable
 * destinations written into page-locked buffers and copied out (no H2D / D2H
 * DMA step; MXD_POLICY_NO_ZERO_COPY restores the DMA form).  The batch runs in
 * chunks over two slots so staging, kernel and copy-out overlap.  Calls
 * borrow one of a bounded number of per-device contexts (threads beyond that
 * wait), so pinned and device memory stay bounded.  This is the path the C++
 * pipeline ops use when samples live in host memory (mlx-data's default). */
int mxd_resize_crop_host(const mxd_image* images, int32_t n, int32_t out_dtype, int32_t device);

/* Host image in, DEVICE result out (the device-resident
 * batch): as mxd_resize_crop_host, but `images[i].dst` are device pointers on
 * `device` (e.g. one (B, H, W, C) batch tensor) that the kernel writes
 * directly -- no D2H, no host copy-out.  Returns once the results are
 * complete on the device, so any stream (or another library sharing this HIP
 * runtime) may read them.  Replaces, for device consumers, the host batch of
 * stream/Batch.cpp:25-39 -> core/Utils.cpp:209-252 (merge_batch). */
int mxd_resize_crop_to_device(const mxd_image* images, int32_t n, int32_t out_dtype, int32_t device);

/* Synchronous copies for device-resident batches (fill, read back). */
int mxd_memcpy_h2d(void* dst, const void* src, size_t bytes, int32_t device);
int mxd_memcpy_d2h(void* dst, const void* src, size_t bytes, int32_t device);

/* Frees the pinned and device buffers of idle host-path contexts. */
int mxd_release_host_buffers(void);

/* ---- JPEG decode (load_image's producer) ---------------
 *
 *   core::image::load_jpeg(contents)         mlx/data/core/image/ImageJPEG.cpp:99-146,197-232
 *   op::LoadImage::apply_key                 mlx/data/op/LoadImage.cpp:23-48
 *
 * A from-scratch decoder with libjpeg's default output: ISLOW inverse DCT,
 * fancy chroma upsampling, YCbCr -> RGB; the result is always H x W x 3
 * (grey replicated, CMYK: its first three channels).  Host only. */

/* Nonzero when the bytes start with the reference's JPEG signature FF D8 FF. */
int mxd_is_jpeg(const uint8_t* data, size_t size);

/* Image size and component count from the frame header. */
int mxd_jpeg_info(const uint8_t* data, size_t size, int32_t* width, int32_t* height, int32_t* components);

/* Decodes into dst: height rows of width*3 bytes, dst_stride bytes apart (any
 * host memory, e.g. pinned staging from mxd_malloc_pinned).  width/height
 * must be mxd_jpeg_info's.  Baseline, extended, progressive and (8-bit)
 * lossless frames, Huffman or arithmetic coded (SOF0-3, SOF9-10).
 * MXD_ERR_INVALID with
 * libjpeg's message on corrupt or unsupported data. */
int mxd_jpeg_decode(const uint8_t* data, size_t size, uint8_t* dst, int64_t dst_stride, int32_t width,
                    int32_t height);

/* ---- split JPEG decode with the device-side finish (SURVEY.md §8f f1,
 * "later a device-side decode") ---------------------------------------------
 *
 * The same decode in two halves: mxd_jpeg_coefs_decode runs the host part
 * (markers + Huffman or arithmetic entropy decode, every error
 * mxd_jpeg_decode reports)
 * and keeps the quantised DCT coefficients; dequantisation + ISLOW IDCT,
 * chroma upsampling and colour conversion run later -- on the host
 * (mxd_jpeg_coefs_finish) or on the GPU inside mxd_jpeg_resize_crop_host /
 * _to_device, which decode, resize, crop and mirror a whole batch in one call
 * (what load_image -> image_resize_smallest_side -> image_center_crop ->
 * batch do per sample: ImageJPEG.cpp:99-146 + the resize/crop rows above).
 * Every route gives the bytes mxd_jpeg_decode (then mxd_resize_crop_*) gives. */
typedef struct mxd_jpeg_coefs mxd_jpeg_coefs;

/* Entropy-decodes `data` (which may be freed afterwards) into *out; release
 * with mxd_jpeg_coefs_free.  MXD_ERR_INVALID with libjpeg's message. */
int mxd_jpeg_coefs_decode(const uint8_t* data, size_t size, mxd_jpeg_coefs** out);
/* The same with the Huffman decode optionally left to the GPU
 * (device_entropy != 0): a baseline / extended-sequential file whose one scan
 * carries every component (grey, YCbCr or RGB), complete up to a marker after
 * its entropy-coded data, with its restart markers in sequence, is only
 * parsed here; mxd_jpeg_resize_crop_host / _to_device then decode its
 * segments on the device (csrc/jpeghuff.hip), mxd_jpeg_coefs_finish on the
 * host.  Any other file is entropy-decoded here, as by mxd_jpeg_coefs_decode.
 * The bytes are copied (`data` may be freed after the call); every route
 * gives mxd_jpeg_decode's bytes. */
int mxd_jpeg_coefs_parse(const uint8_t* data, size_t size, int32_t device_entropy, mxd_jpeg_coefs** out);
/* mxd_jpeg_coefs_parse of the regular file at `path`, read straight into the
 * handle's own copy (one open, one read sized by fstat: the file-loading
 * half of op/LoadImage.cpp:23-48 for JPEGs).  MXD_OK with *out = NULL when
 * the file does not start with the JPEG signature (FF D8 FF; the caller's
 * other decoders take it); MXD_ERR_INVALID when it cannot be read or parsed,
 * or is not a regular file -- read it and call mxd_jpeg_coefs_parse for the
 * reference's exact message. */
int mxd_jpeg_coefs_load(const char* path, int32_t device_entropy, mxd_jpeg_coefs** out);
/* *pending = 1 when the coefficients will come from the device entropy decode
 * of a sequential file's one scan, 0 when the host decoded them (progressive
 * files always: round 5's value 2, every scan of a progressive file decoded
 * on the device, was retired in round 6 -- DESIGN.md section 8). */
int mxd_jpeg_coefs_entropy_pending(const mxd_jpeg_coefs* coefs, int32_t* pending);
int mxd_jpeg_coefs_free(mxd_jpeg_coefs* coefs);

/* Image size; *device_ok = 1 when the GPU can finish it (grey, YCbCr, RGB
 * and, since ABI 6, CMYK / YCCK -- their first three output channels; lossless
 * files finish on the host only). */
int mxd_jpeg_coefs_info(const mxd_jpeg_coefs* coefs, int32_t* width, int32_t* height, int32_t* device_ok);

/* Host finish: height rows of width*3 bytes at dst_stride (thread-safe; the
 * handle stays valid). */
int mxd_jpeg_coefs_finish(const mxd_jpeg_coefs* coefs, uint8_t* dst, int64_t dst_stride);

/* One image of a decode + resize + crop batch: the window (win_x, win_y,
 * win_w, win_h) of the decoded image is the source of an mxd_image with
 * channels 3 (the whole image: 0, 0, width, height); the rest as mxd_image. */
typedef struct mxd_jpeg_image {
  const mxd_jpeg_coefs* coefs;
  int32_t win_x, win_y, win_w, win_h;
  int32_t resize_w, resize_h;
  int32_t crop_x, crop_y, crop_w, crop_h;
  int32_t flip;
  int32_t reserved;
  void* dst;
  int64_t dst_stride;
} mxd_jpeg_image;

/* Host destinations (like mxd_resize_crop_host): coefficients staged through
 * pinned memory, IDCT + colour + resample kernels on `device`, results back. */
int mxd_jpeg_resize_crop_host(const mxd_jpeg_image* images, int32_t n, int32_t out_dtype, int32_t device);

/* Device destinations on `device` (like mxd_resize_crop_to_device). */
int mxd_jpeg_resize_crop_to_device(const mxd_jpeg_image* images, int32_t n, int32_t out_dtype, int32_t device);

/* Diagnostics: *count = the images the two calls above resized straight from
 * their sample planes (4:2:0 on a scatter wave kernel, MXD_TUNE_JPEG_RGB 0:
 * no RGB frame) since the last reset; reset != 0 zeroes it after reading. */
int mxd_jpeg_plane_sources(int64_t* count, int32_t reset);

/* Diagnostics (ABI 7): images whose MXD_F32_DIV255 results a host-ending
 * call (mxd_resize_crop_host, mxd_jpeg_resize_crop_host) returned over the
 * link as u8 and expanded on the host (see MXD_TUNE_F32_LINK) since the last
 * reset; reset != 0 zeroes it after reading. */
int mxd_narrow_returns(int64_t* count, int32_t reset);

/* Diagnostics: where a host-side pipeline's time goes, summed over every
 * thread since the last reset (reset != 0 zeroes them after reading).
 * out[0] host-path calls (the mxd_*_host / *_to_device batch calls above),
 * out[1] their images, out[2] their wall time in ns, out[3] the part of it
 * spent waiting for the device (chunk events and the final drain),
 * out[4] mxd_jpeg_coefs_parse / mxd_jpeg_coefs_load calls, out[5] their time
 * in ns (a load's includes its file read). */
int mxd_host_stats(int64_t* out6, int32_t reset);

/* Diagnostics (ABI 6): with MXD_TUNE_DEVICE_TIMING 1, out[0] = host-path
 * chunks timed, out[1] = the summed device time in ns from each chunk's
 * first kernel to the end of its last (entropy decode, IDCT, colour, resize;
 * the staged input copy before them and the result copy after them are
 * outside), since the last reset (reset != 0 zeroes them after reading). */
int mxd_device_stats(int64_t* out2, int32_t reset);

/* ---- pixel maps: rotate / affine and channel reduction --
 *
 *   core::image::affine(img, mx, crop)       mlx/data/core/image/ImageTransform.cpp:75-110
 *   core::image::rotate(img, angle, crop)    mlx/data/core/image/ImageTransform.cpp:112-121
 *   core::image::channel_reduction(img,b,m)  mlx/data/core/image/ImageTransform.cpp:142-180
 *   op::ImageRotate / ImageChannelReduction  mlx/data/op/ImageTransform.cpp:334-421
 *
 * One uint8 image of a pixel-map launch.  Affine: dst is dst_h x dst_w x
 * channels, dst(tx,ty) = src(x,y) at the reference's nearest-pixel inverse map
 * (0 outside the source).  Channel reduction: channels must be 3, dst is
 * src_h x src_w x 1.  params: affine mx[0..5]; channel reduction
 * {bias, m0, m1, m2} as floats (the reference's 16.16 fixed point is derived
 * from them exactly as core::image::channel_reduction does). */
typedef struct mxd_pixmap {
  const uint8_t* src;
  int64_t src_stride;
  int32_t src_w, src_h, channels;
  int32_t dst_w, dst_h;
  void* dst;
  int64_t dst_stride;
  float params[6];
} mxd_pixmap;

enum mxd_pixop { MXD_AFFINE = 0, MXD_CHANNEL_REDUCTION = 1 };

/* core::image::rotate's matrix and core::image::affine's output dims for a
 * (w x h) image rotated by `angle` degrees (crop: keep w x h). */
int mxd_rotate_geometry(int64_t w, int64_t h, double angle, int32_t crop, float* mx6, int64_t* out_w,
                        int64_t* out_h);

/* op::ImageChannelReduction presets (op/ImageTransform.cpp:362-392):
 * "default", "rec601", "rec709", "rec2020", "green" -> {bias, m0, m1, m2}.
 * Unknown name: MXD_ERR_INVALID with the reference's message. */
int mxd_channel_reduction_preset(const char* preset, float* params4);

/* n pixel maps of kind `op` on `device`, one kernel launch, enqueued on
 * `stream`; src/dst are device pointers. */
int mxd_pixmap_batch(const mxd_pixmap* images, int32_t n, int32_t op, int32_t device, void* stream);

/* Host pointers in and out (pinned staging, synchronous), like
 * mxd_resize_crop_host. */
int mxd_pixmap_host(const mxd_pixmap* images, int32_t n, int32_t op, int32_t device);

#ifdef __cplusplus
}
#endif

#endif /* MXD_AMD_H */
