// resample.h -- device-side descriptors shared by capi.cpp and resample.hip.
#pragma once

#include <cstddef>
#include <cstdint>

namespace mxd {

// One entry of a per-axis tap table in device memory: the first input index
// and tap count stored as int bits, then `width` f32 weights, zero padded to
// at least kMinTabWidth so the wave and band kernels can read T <=
// kMinTabWidth weights of any entry unconditionally (both read up to their
// largest tap bucket / class, 32).
constexpr int kTapHeader = 2;
constexpr int kMinTabWidth = 32;

// Per-image parameters, resolved by the host (geometry already validated).
// Each image is cut into nbands x nstrips tiles of ty output rows x tx output
// columns; tiles of all images are numbered consecutively from tile_begin.
struct ImgDev {
  const uint8_t* src;
  int64_t src_stride;
  void* dst;
  int64_t dst_stride;
  const float* ytab;  // crop_h entries of (kTapHeader + ywidth) floats
  const float* xtab;  // crop_w entries of (kTapHeader + xwidth) floats
  int32_t ywidth, xwidth;
  int32_t crop_w, crop_h;
  int32_t flip;  // bit 0: mirror; wave path: bits 8.. = byte offset of the
                 // source window past the 4-byte aligned `src` (0..3)
  int32_t tile_begin;
  int32_t nstrips, ty, tx, group;
  int32_t src_w, src_h;  // src_h: rows stored at src (the whole image, or a staged footprint)
  int32_t src_x0, src_y0;  // source pixel at src (0, 0 unless only a footprint is stored)
  const struct YccDev* ycc;  // wave kernels: the source is JPEG sample planes, not RGB (null: RGB at src)
};
static_assert(sizeof(ImgDev) == 112, "ImgDev layout");

// A JPEG image's sample planes as a wave kernel's source (the fused decode
// finish): 4:2:0 YCbCr as jpeg_idct writes them; the kernel
// makes the RGB pixels of the rows it reads in registers, by jpeg_color's
// rules (h2v2 fancy upsampling, jdcolor's fixed-point YCbCr -> RGB).
// ImgDev::src is the Y plane's first byte; the source image is the window
// from (win_x, win_y) (win_x a multiple of 4) of win_w x win_h =
// ImgDev::src_w x src_h pixels.
struct YccDev {
  int64_t cb, cr;          // Cb / Cr plane: byte offset from the Y plane
  int32_t ystride, cstride;
  int32_t dw, dh;          // chroma plane samples per row / rows (jdsample's downsampled size)
  int32_t win_x, win_y;
  int32_t records;         // bytes from the Y plane to the Cr plane's end (the buffer's range)
  int32_t pad;
};
static_assert(sizeof(YccDev) == 48, "YccDev layout");

struct LaunchCfg {
  int32_t vec;        // bytes per thread per source row: 16 (16-byte aligned rows) or 1
  int32_t channels;   // 1..4
  int32_t alpha;      // channels == 4: STBIR_RGBA alpha weighting
  int32_t f32;        // output f32 /255
  int32_t nimgs;
  int32_t ntiles;
  int32_t max_tx, max_ty, max_xw, max_yw, max_vw, max_group;
};

// Wave-per-unit fast paths (wave.hip): source rows 4-byte aligned (a window
// may start at any byte: ImgDev::flip bits 8.. hold the base's misalignment),
// f32 outputs 4-byte aligned, every strip's source window <= wave_window_px()
// pixels (start aligned to wave_window_align()), strip_cols <= 64 q, taps <=
// 17.  Units are numbered through ImgDev::tile_begin exactly like tiles; ty =
// band rows, tx = strip columns.  kind: 0 = gather, 2 = scatter (ImgDev::ytab
// is the schedule, ywidth its words per band, group the offset of its
// iteration entries).  taps = horizontal (and, for gather, vertical) tap
// bucket; s / dmax = scatter shape; q = output pixels per lane; shift = some
// image of the launch has a misaligned base.
struct WaveCfg {
  int32_t channels, f32, taps, nimgs, nunits;
  int32_t kind;
  int32_t s, dmax;
  int32_t q, shift;
  int32_t p;  // source pixels per lane (wave_default_p, or 8 for wide RGB windows; RGB 16 = byte lanes)
  int32_t per_img = 0;  // units of every image when all images of the launch have the same count, else 0
  int32_t prio = 1;     // progress-based wave priority (off for the concurrent launches of a mixed batch)
  int32_t ycc = 0;      // sources are JPEG sample planes (ImgDev::ycc; scatter, p = 4, no shift)
  int32_t nt = 0;       // streaming (nt) source loads (scatter kernels; wave.hip LAUX)
};

// Scatter schedule geometry, shared by the kernel and the host builder:
// register ring slots for DMAX iterations per group, groups per unrolled
// block (a multiple of S whose iterations are a multiple of the ring), words
// per iteration entry (row + S weights).
constexpr int scatter_gcd(int a, int b) { return b ? scatter_gcd(b, a % b) : a; }
// Ring target: 6 (4 slots at DMAX 4) keeps the C2 kernel at 118 VGPRs, i.e.
// 4 waves per SIMD; 12 (166 VGPRs, 3 waves) measured 3 % slower on C2 and
// 1-2 % on C4/C5 (tools/ab.sh, profiles/r02/ring_ab.txt).  Tuning builds
// override it with -DMXD_RING=<n> (kernel and host together).
#ifndef MXD_RING
#define MXD_RING 6
#endif
// Past DMAX 9 (large downscale ratios) a ring of DMAX slots would hold 12-16
// rows of registers: the ring is the smallest size in [MXD_RING, 2 MXD_RING]
// that divides two groups (the block then stays S = 2 groups long).
// Tuning builds: -DMXD_RING_FIXED=<n> uses n slots at every DMAX >= 2.
#ifndef MXD_RING_FIXED
#define MXD_RING_FIXED 0
#endif
// DMAX 5 (1080p / 4K -> 512, C5) takes 4 slots: its RGB u8 kernel then fits
// 124 VGPRs (4 waves per SIMD instead of 3 at 5 slots), C5 0.3244 -> 0.3204 ms
// per launch (profiles/r03/ring_variants.jsonl, variant ring4).
// (Narrow-lane rings of 4 / 3 slots at DMAX 2 / 3, 8 waves per SIMD, were
// measured in round 4 and lost: 480p 0.0935 vs 0.0903 ms per launch, C4
// 0.0236 vs 0.0227, profiles/r04/ring_pack_b.jsonl.)
// JPEG plane sources (wave.hip YccSrc) hold 9 dwords per ring slot: their
// ring is the smallest that keeps the unrolled block at S = 2 groups (3 slots
// at DMAX 1, 4 at DMAX 2, DMAX up to 6, then 6 or 4).
constexpr int kYccLaneBytes = 36;
constexpr int scatter_ring_slots(int dmax, int lane_bytes = 0) {
  if (lane_bytes == kYccLaneBytes)
    return dmax == 1 ? 3 : dmax == 2 ? 4 : dmax <= 6 ? dmax : (2 * dmax) % 6 == 0 ? 6 : 4;
  if (MXD_RING_FIXED > 0 && dmax >= 2) return MXD_RING_FIXED;
  if (dmax == 5 && MXD_RING == 6) return 4;
  if (MXD_RING % dmax == 0) return MXD_RING;
  if (2 * dmax <= MXD_RING) return 2 * dmax;
  if (dmax > 9)
    for (int r = MXD_RING; r <= 2 * MXD_RING; r++)
      if ((2 * dmax) % r == 0) return r;
  return dmax;
}
constexpr int scatter_block_groups(int s, int dmax, int lane_bytes = 0) {
  return scatter_ring_slots(dmax, lane_bytes) / scatter_gcd(scatter_ring_slots(dmax, lane_bytes), s * dmax) * s;
}
constexpr int scatter_entry_words(int s) { return s <= 2 ? 4 : 8; }  // prefetch row, row, s weights

int wave_taps_bucket(int taps);            // supported padded tap count >= taps, or -1
int wave_default_p(int channels);          // source pixels per lane of the gather kernels
int wave_window_px(int channels, int p);   // source pixels one wave covers per row
int wave_window_align(int channels);       // window start alignment (pixels)
// RGB with p = 16: byte lanes (16 bytes per lane, a wave_byte_window()-byte
// window starting at a 16-byte boundary past the 4-byte aligned base).
bool wave_byte_lanes(int channels, int p);
int wave_byte_window();
int wave_plane_floats(int channels, int p);  // LDS floats per wave
int wave_lanes();
int launch_wave(const WaveCfg& cfg, const ImgDev* imgs, void* stream);
bool wave_has_kernel(const WaveCfg& cfg);
// Waves of this configuration the device runs at once (occupancy x CUs), 0 if unknown.
int wave_capacity(const WaveCfg& cfg, int device);
// Diagnostics: the occupancy API's blocks per CU, the kernel's VGPRs and LDS
// bytes per block; returns waves per block (-1: no kernel / error).
int wave_kernel_info(const WaveCfg& cfg, int device, int* api_blocks, int* vgprs, int* lds);
// policy: 0 default (16-B loads / stores per thread), 1 nt, 2 nt sc1 (buffer forms)
int launch_copy(const void* src, void* dst, size_t bytes, void* stream, int policy = 0);

// Dynamic LDS bytes the kernel needs for cfg.
int resample_smem_bytes(const LaunchCfg& cfg);

// Enqueues the fused kernel; imgs is a device pointer to cfg.nimgs entries.
int launch_resample(const LaunchCfg& cfg, const ImgDev* imgs, void* stream);

}  // namespace mxd
