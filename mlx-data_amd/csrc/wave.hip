// wave.hip -- the fast path of the fused resize + crop (+ hflip) (+ /255) stage.
//
// Arithmetic (shared with resample.hip): stbir triangle taps from the shared
// tables, vertical pass first in byte units, f32 FMA accumulation in tap order
// starting from 0, stbir's encode, exact q/255.
//
// A UNIT = (image, band of output rows, strip of output columns) is run by one
// wave; units never synchronise with each other (no workgroup barriers).
//
// Channel-planar layout.  The wave covers a window of WPX = 64 P source
// pixels of each row; lane l owns pixels [P l, P l + P) of it, i.e. the P*C
// bytes at byte offset P*C*l (one buffer_load_dwordx3/x4 per row: 12 bytes for
// RGB).  The vertical (V) pass converts those bytes to f32 once per source row
// and FMAs them into the open output rows; a finished V row goes to LDS as C
// channel PLANES (plane c holds channel c of the window's pixels): lane l
// writes its P floats of plane c with one ds_write_b128 per 4 pixels, lanes
// 16 B apart -- conflict-free.  The horizontal (H) pass gives lane l the
// output pixels l, l + 64, ... (Q of them) of the strip row: output pixel x
// reads its T taps of plane c at consecutive floats (ds_read2_b32 with
// immediate offsets), consecutive lanes read addresses ~1/scale apart, so the
// tap reads are (nearly) conflict-free as well.  It then rounds like stbir's
// encode and stores the pixel's C channels contiguously (f32 exact q/255, or
// u8).
//
// Two ways to run a band (KIND):
//   kGather  each output row loads its T tap rows, double-buffered one output
//            row ahead.  Any geometry (upsampling included).
//   kScatter every source row of the band is loaded once and converted to f32
//            once, then FMA'd into each open output row whose taps contain it,
//            following a host-built schedule (below).
//
// Scatter schedule (capi.cpp builds it per image crop and band height): a
// sequence of GROUPS of DMAX iterations.  An iteration carries one source row
// (or -1, a bubble), its weights for the output rows of groups g, g+1, ...,
// g+S-1, and the row to load for the iteration R-1 ahead; group g completes one
// output row (or none).  Group g accumulates in slot g mod S, so with the group
// loop unrolled by a multiple of S every accumulator index is static.  Rows
// are loaded R-1 iterations ahead into a ring of R register slots, and the
// unrolled block is a multiple of R iterations, so every ring slot index is
// static too.  Rows are visited in ascending order, so each output row's sum
// runs in tap order from 0 exactly as in kGather: both kinds give
// bit-identical results.
// Per band: word 0 = groups to run (a multiple of the block's groups), words
// 1.. = the output row each group completes (-1: none), then at word
// ImgDev::group the iteration entries, scatter_entry_words(S) words each:
// row to prefetch, row, S f32 weights (one scalar burst per group).
#include <hip/hip_runtime.h>

#include <type_traits>
#include <utility>

#include "devutil.h"
#include "jpegycc.h"
#include "resample.h"

namespace mxd {
namespace {

using namespace dev;

// Waves per workgroup (tuning builds: -DMXD_WAVES=<1|2|4|8>).  8 measured
// 0.2-2.6 % faster than 4 on C2..C7 (profiles/r03/wave_variants.jsonl).
#ifndef MXD_WAVES
#define MXD_WAVES 8
#endif
constexpr int kWaves = MXD_WAVES;
constexpr int kLanes = 64;

// Timing-only ablations, compiled in only when the library is built with
// -DMXD_ABLATE=<n> (tools/ablate8.sh; never in the product library):
// 1 = no source loads, 2 = no output stores, 4 = no H pass (LDS), 8 = no V math.
#ifndef MXD_ABLATE
#define MXD_ABLATE 0
#endif
// f32 output stores are nontemporal (MXD_NT_STORE, default 1; tuning builds
// -DMXD_NT_STORE=0): results are written once and never read back here, and
// with plain stores the dirty lines they leave in each XCD's L2 are written
// back at the kernel's end -- C4 (77 MB of f32 per launch) measured 0.0325 ->
// 0.0263 ms per launch, C2 0.1536 -> 0.1505 (profiles/r02/nt_store_ab.txt).
// Tuning builds (-DMXD_MIN_WAVES=<n>): minimum waves per SIMD the register
// allocation must allow.
#ifndef MXD_NT_STORE
#define MXD_NT_STORE 1
#endif
#ifndef MXD_MIN_WAVES
#define MXD_MIN_WAVES 3
#endif
#ifndef MXD_SPLIT_LANES
#define MXD_SPLIT_LANES 1
#endif
#ifndef MXD_MIN_WAVES_WIDE
#define MXD_MIN_WAVES_WIDE 2
#endif
// Tuning build (-DMXD_SYNC_STRIPS=1): when a workgroup's four waves are the
// four strips of one band, an s_barrier after every group keeps them loading
// the same source rows at the same time.
#ifndef MXD_SYNC_STRIPS
#define MXD_SYNC_STRIPS 0
#endif
constexpr int kPad = 32;  // floats after each plane: padded taps read zeros there

// Progress-based wave priority (tuning builds: -DMXD_PRIO=0 turns it off).
// All units of a launch do about the same work and start together, but the
// SIMD arbiter issues oldest-first, so without it a CU's first workgroup
// finishes its band in ~95 us and its last in ~141 us (C2, tools/stamps.sh):
// the launch then drains for ~60 us with ever fewer waves feeding HBM.  Each
// wave lowers its s_setprio level as it completes quarters of its band, so
// waves that are behind win the arbiter and the band ends line up.  Only for
// a batch that is one launch (`on`): launches of a mixed batch run
// concurrently, and there the priorities of one launch's waves starve the
// others' (C3 0.440 -> 0.423 ms without them, profiles/r03/wave_variants.jsonl).
#ifndef MXD_PRIO
#define MXD_PRIO 1
#endif

// Tuning builds (-DMXD_PRIO_MODE=<n>, round 6; the unit stamps show a
// workgroup's waves 4-7 finishing ~3 % after waves 0-3): 1 = waves 4-7 one
// level above the others at equal progress (capped at 3); 2 = levels in
// eighths of the band, cycling 3, 2, 1, 0, 3, 2, 1, 0 (a wave that falls
// behind its neighbours wins ties within the cycle).
#ifndef MXD_PRIO_MODE
#define MXD_PRIO_MODE 0
#endif
__device__ __forceinline__ void progress_prio(bool on, int done, int total) {
  if (!on) return;
  if constexpr (MXD_PRIO != 0) {
    int level = 3 - (4 * done) / (total + 1);  // 3 at the start .. 0 in the last quarter
    if constexpr (MXD_PRIO_MODE == 1) level = min(3, level + ((threadIdx.x >> 6) >= kWaves / 2 ? 1 : 0));
    if constexpr (MXD_PRIO_MODE == 2) level = 3 - ((8 * done) / (total + 1)) % 4;
    switch (level) {
      case 3: __builtin_amdgcn_s_setprio(3); break;
      case 2: __builtin_amdgcn_s_setprio(2); break;
      case 1: __builtin_amdgcn_s_setprio(1); break;
      default: __builtin_amdgcn_s_setprio(0); break;
    }
  }
}

// Diagnostic builds only (-DMXD_STAMPS=1, tools/stamps.sh; never in the
// product library): every unit's start and end time (s_memrealtime, 100 MHz)
// from its wave's lane 0, read back with mxd_debug_stamps.
#ifndef MXD_STAMPS
#define MXD_STAMPS 0
#endif
#if MXD_STAMPS
constexpr int kMaxStamped = 32768;
__device__ unsigned long long g_stamps[2 * kMaxStamped];
#endif

#define GLOBAL_PTR(T, p) MXD_GLOBAL_PTR(T, p)
typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef float f32x3 __attribute__((ext_vector_type(3)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
typedef uint32_t u32x3 __attribute__((ext_vector_type(3)));
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
using Rsrc = __amdgpu_buffer_rsrc_t;

enum Kind { kGather = 0, kScatter = 2 };

// Lane layouts.  Pixel lanes (planar): P source pixels (P*C bytes) per lane;
// the default P fills 16 bytes (12 for RGB), P = 8 widens an RGB window to
// 512 pixels (fewer, wider strips per row); the V pass keeps C channel planes.
// Byte lanes (RGB with P = 16, `B`): lane l owns the 16 bytes at 16 l of a
// 1-KiB window, so every row load is one b128 per lane and 1 KiB contiguous
// per wave-instruction; the V pass runs on bytes in memory order (it is
// per-byte anyway) and the LDS row keeps that order, so the H pass reads
// channel c of pixel x at float C x + c.
template <int C_, int P_ = (C_ == 1 ? 16 : C_ == 2 ? 8 : 4)>
struct Lay {
  static constexpr int C = C_;
  static constexpr int P = P_;
  static constexpr bool B = C == 3 && P == 16;  // byte lanes
  static constexpr int VC = B ? 1 : C;          // V-pass planes
  static constexpr int LB = B ? 16 : P * C;     // bytes per lane
  static constexpr int ND = LB / 4;             // dwords per lane
  static constexpr int VP = LB / VC;            // V-pass values per lane and plane
  static constexpr int WPX = kLanes * VP;       // window pixels (byte lanes: bytes)
  static constexpr int PAD = B ? 64 : kPad;     // zeroed floats past each plane (padded taps)
  static constexpr int PL = WPX + PAD;          // floats per plane
  static constexpr int HS = B ? C : 1;          // floats between adjacent pixels of a plane
  static constexpr int CS = B ? 1 : PL;         // floats between the channels of a pixel
  // Split RGB lanes (default; tuning builds -DMXD_SPLIT_LANES=0 interleave): at
  // P = 8 lane l owns pixels 4l..4l+3 and 256+4l..256+4l+3, loaded by two
  // dwordx3 loads that each cover one contiguous 768-byte half of the window,
  // instead of a dwordx4 and a dwordx2 interleaved over all of it.  Same bytes;
  // C3 0.468 -> 0.451 ms per launch, C2 / C5 / C6 / C7 unchanged
  // (profiles/r03/split.jsonl).
  static constexpr bool SPLIT = MXD_SPLIT_LANES != 0 && C == 3 && P == 8;
  static constexpr int HALF = kLanes * 4 * C;   // bytes per window half (SPLIT)
};

// One f32 output store (vector memory; nontemporal unless MXD_NT_STORE == 0).
template <class V, class T>
__device__ __forceinline__ void store_out(V* p, T v) {
  if constexpr (MXD_NT_STORE != 0)
    __builtin_nontemporal_store(v, p);
  else
    *p = v;
}

// Tuning builds (-DMXD_STORE_AUX=<n>, e.g. 18 = nt sc1): the f32 output
// stores as buffer stores with that cache policy instead of store_out.
#ifndef MXD_STORE_AUX
#define MXD_STORE_AUX 0
#endif
template <int C>
__device__ __forceinline__ void store_row_px(char* drow, int px, const float (&s)[C]) {
  const Rsrc rs = __builtin_amdgcn_make_buffer_rsrc(drow, (short)0, 0x7ffffff0, 0x00020000);
  if constexpr (C == 3) {
    const u32x3 v = {__float_as_uint(s[0]), __float_as_uint(s[1]), __float_as_uint(s[2])};
    __builtin_amdgcn_raw_buffer_store_b96(v, rs, px * 12, 0, MXD_STORE_AUX);
  } else if constexpr (C == 4) {
    const u32x4 v = {__float_as_uint(s[0]), __float_as_uint(s[1]), __float_as_uint(s[2]), __float_as_uint(s[3])};
    __builtin_amdgcn_raw_buffer_store_b128(v, rs, px * 16, 0, MXD_STORE_AUX);
  } else if constexpr (C == 2) {
    const u32x2 v = {__float_as_uint(s[0]), __float_as_uint(s[1])};
    __builtin_amdgcn_raw_buffer_store_b64(v, rs, px * 8, 0, MXD_STORE_AUX);
  } else {
    __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(s[0]), rs, px * 4, 0, MXD_STORE_AUX);
  }
}

// Cache policy of the source row loads (the aux operand of the buffer loads).
// Kernels come in two forms (template argument LAUX): the default policy,
// and nt (2, streaming) for calls whose sources are far larger than the
// Infinity Cache -- the planner's choice (batch.cpp, MXD_TUNE_LOAD_POLICY).
// Measured in one process (profiles/r06/README.md): nt reads stream at
// 7.0-7.2 TB/s against 6.2-6.4 default (tools/nt_ceiling.hip), and the wave
// kernels gain 2-7 % on C2 / C3 / C5, while C4's 128 small images, which the
// Infinity Cache holds, lose 45 % with nt.  Tuning builds: -DMXD_LOAD_AUX=<n>
// replaces the default form's policy (1 = sc0, 16 = sc1, ...).
#ifndef MXD_LOAD_AUX
#define MXD_LOAD_AUX 0
#endif
constexpr int kLoadNt = 2;

// A voffset past any image (images are < 2^31 bytes): the buffer range check
// turns the load into zeros without a memory request.
constexpr int kNoLoad = 0x7ffffff0;

// The lane's raw bytes of one source row.
template <int ND>
struct Raw {
  uint32_t d[ND];
};

// Raw bytes -> f32 planes: x[c][p] = byte C*p + c (p pixels of the lane).
template <int C, int P>
__device__ __forceinline__ void to_planes(const Raw<P * C / 4>& v, float (&x)[C][P]) {
#pragma unroll
  for (int i = 0; i < P * C; i++) x[i % C][i / C] = (float)((v.d[i >> 2] >> (8 * (i & 3))) & 0xffu);
}

// n consecutive dwords of a buffer row into w[0..n) (cache policy AUX).
template <int N, int AUX>
__device__ __forceinline__ void load_dwords(Rsrc rs, int voff, int soff, uint32_t* w) {
  if constexpr (N >= 4) {
    const u32x4 v = __builtin_amdgcn_raw_buffer_load_b128(rs, voff, soff, AUX);
    w[0] = v.x, w[1] = v.y, w[2] = v.z, w[3] = v.w;
    if constexpr (N > 4) load_dwords<N - 4, AUX>(rs, voff + 16, soff, w + 4);
  } else if constexpr (N == 3) {
    const u32x3 v = __builtin_amdgcn_raw_buffer_load_b96(rs, voff, soff, AUX);
    w[0] = v.x, w[1] = v.y, w[2] = v.z;
  } else if constexpr (N == 2) {
    const u32x2 v = __builtin_amdgcn_raw_buffer_load_b64(rs, voff, soff, AUX);
    w[0] = v.x, w[1] = v.y;
  } else if constexpr (N == 1) {
    w[0] = __builtin_amdgcn_raw_buffer_load_b32(rs, voff, soff, AUX);
  }
}

// Source rows of one image: a descriptor spanning the image and a dead one (no
// records: every load through it returns zeros without a memory request).
// SHIFT: the window starts `sh` bytes past a 4-byte boundary (a source window
// at any x); one more dword is loaded and the bytes are realigned.
// Row offsets go into the VGPR offset (r - y0) * stride + lane offset, which
// the buffer range check covers (the scalar offset is not checked): rows
// outside the stored region read zeros, never other memory.
template <class L, bool SHIFT, int AUX>
struct Src {
  using RawT = Raw<L::ND>;
  static constexpr int kLaneBytes = L::LB;  // (its scatter ring: resample.h scatter_ring_slots)
  Rsrc live, dead;
  int stride, voff, voff2, sh, y0;  // voff2: the second window half (L::SPLIT)

  __device__ __forceinline__ void planes(const RawT& v, float (&x)[L::VC][L::VP]) const { to_planes<L::VC, L::VP>(v, x); }
  __device__ __forceinline__ Raw<L::ND> load(int r) const {
    constexpr int ND = L::ND;
    const bool ok = r >= 0 && !(MXD_ABLATE & 1);
    const Rsrc rs = ok ? live : dead;
    const uint32_t roff = ok ? (uint32_t)((r - y0) * stride) : 0u;
    // unsigned: a row above the region wraps to a huge (out-of-range) offset
    const int off = (int)((uint32_t)voff + roff);
    Raw<ND> x;
    if constexpr (L::SPLIT) {
      const int off2 = (int)((uint32_t)voff2 + roff);
      constexpr int NH = ND / 2;
      if constexpr (!SHIFT) {
        load_dwords<NH, AUX>(rs, off, 0, x.d);
        load_dwords<NH, AUX>(rs, off2, 0, x.d + NH);
      } else {
        uint32_t w[NH + 1], v[NH + 1];
        load_dwords<NH + 1, AUX>(rs, off, 0, w);
        load_dwords<NH + 1, AUX>(rs, off2, 0, v);
#pragma unroll
        for (int j = 0; j < NH; j++) {
          x.d[j] = __builtin_amdgcn_alignbyte(w[j + 1], w[j], sh);
          x.d[NH + j] = __builtin_amdgcn_alignbyte(v[j + 1], v[j], sh);
        }
      }
      return x;
    }
    if constexpr (!SHIFT) {
      load_dwords<ND, AUX>(rs, off, 0, x.d);
    } else {
      uint32_t w[ND + 1];
      load_dwords<ND + 1, AUX>(rs, off, 0, w);
#pragma unroll
      for (int j = 0; j < ND; j++) x.d[j] = __builtin_amdgcn_alignbyte(w[j + 1], w[j], sh);
    }
    return x;
  }
};

// JPEG sample planes as the source of RGB pixel lanes (P = 4; resample.h
// YccDev): a row load fetches the lane's four Y samples and, per chroma
// component, the samples c - 1 .. c + 2 (c: the chroma column of its first
// pixel) of the two chroma rows the row's fancy upsampling blends; planes()
// makes the four RGB pixels from them with jpegdev.hip jpeg_color's
// arithmetic (jpeg.cpp upsample_row h2v2, jdcolor.c), so the resampled bytes
// are those of the RGB frame jpeg_color would have written.
struct YccRaw {
  uint32_t y;
  uint32_t c[2][2][2];  // [Cb / Cr][near / far row][two dwords from the lane's chroma dword]
};

struct YccSrc {
  using RawT = YccRaw;
  static constexpr int kLaneBytes = kYccLaneBytes;
  Rsrc live, dead;
  int ystride, cstride, cb, cr, dw, dh, wy;
  int yoff;  // the lane's Y byte in window row 0 (kNoLoad: a lane past the window)
  int coff;  // its chroma dword's byte offset in a chroma row (kNoLoad likewise)
  int e;     // byte of sample c - 1 in the two chroma dwords (-1 at the left edge: c = 0)
  int ci;    // c

  __device__ __forceinline__ YccRaw load(int r) const {
    const bool ok = r >= 0 && !(MXD_ABLATE & 1);
    const Rsrc rs = ok ? live : dead;
    const int ry = wy + (ok ? r : 0);  // image row
    const int iy = ry >> 1;
    const uint32_t c0 = (uint32_t)(min(iy, dh - 1) * cstride) + (uint32_t)coff;
    const uint32_t c1 = (uint32_t)(min(max((ry & 1) ? iy + 1 : iy - 1, 0), dh - 1) * cstride) + (uint32_t)coff;
    YccRaw v;
    v.y = __builtin_amdgcn_raw_buffer_load_b32(rs, (int)((uint32_t)yoff + (uint32_t)((ok ? r : 0) * ystride)), 0, MXD_LOAD_AUX);
    const uint32_t offs[2][2] = {{c0 + (uint32_t)cb, c1 + (uint32_t)cb}, {c0 + (uint32_t)cr, c1 + (uint32_t)cr}};
#pragma unroll
    for (int k = 0; k < 2; k++)
#pragma unroll
      for (int j = 0; j < 2; j++) {
        const u32x2 t = __builtin_amdgcn_raw_buffer_load_b64(rs, (int)offs[k][j], 0, MXD_LOAD_AUX);
        v.c[k][j][0] = t.x;
        v.c[k][j][1] = t.y;
      }
    return v;
  }

  __device__ __forceinline__ void planes(const YccRaw& v, float (&x)[3][4]) const {
    int cs[2][4];  // chroma samples c - 1 .. c + 2: near * 3 + far
#pragma unroll
    for (int k = 0; k < 2; k++) {
      const uint32_t n = e < 0 ? v.c[k][0][0] << 8 : __builtin_amdgcn_alignbyte(v.c[k][0][1], v.c[k][0][0], e);
      const uint32_t f = e < 0 ? v.c[k][1][0] << 8 : __builtin_amdgcn_alignbyte(v.c[k][1][1], v.c[k][1][0], e);
#pragma unroll
      for (int q = 0; q < 4; q++) cs[k][q] = (int)((n >> (8 * q)) & 255u) * 3 + (int)((f >> (8 * q)) & 255u);
      // the row's edges: the first sample's left neighbour and the last
      // one's right neighbour are the sample itself (jpeg.cpp's (4 s + 8) >> 4
      // and (4 s + 7) >> 4); pixels past the row end are never read
      cs[k][0] = ci == 0 ? cs[k][1] : cs[k][0];
      cs[k][2] = ci == dw - 1 ? cs[k][1] : cs[k][2];
      cs[k][3] = ci + 1 >= dw - 1 ? cs[k][2] : cs[k][3];
    }
#pragma unroll
    for (int j = 0; j < 4; j++) {
      const int q = 1 + (j >> 1);
      int ch[2];
#pragma unroll
      for (int k = 0; k < 2; k++)
        ch[k] = (j & 1) ? (cs[k][q] * 3 + cs[k][q + 1] + 7) >> 4 : (cs[k][q] * 3 + cs[k][q - 1] + 8) >> 4;
      uint32_t px[3];
      jpeg_ycc_to_rgb((int)((v.y >> (8 * j)) & 255u), ch[0], ch[1], px);
#pragma unroll
      for (int c = 0; c < 3; c++) x[c][j] = (float)px[c];
    }
  }
};

// acc += w * x (pairs of pixels per v_pk_fma_f32).
template <int C, int P>
__device__ __forceinline__ void fma_planes(float (&acc)[C][P], float w, const float (&x)[C][P]) {
  const f32x2 ww = {w, w};
#pragma unroll
  for (int c = 0; c < C; c++)
#pragma unroll
    for (int p = 0; p < P; p += 2) {
      f32x2 a = {acc[c][p], acc[c][p + 1]};
      a = __builtin_elementwise_fma(ww, f32x2{x[c][p], x[c][p + 1]}, a);
      acc[c][p] = a.x, acc[c][p + 1] = a.y;
    }
}

template <int C, int P>
__device__ __forceinline__ void zero_planes(float (&acc)[C][P]) {
#pragma unroll
  for (int c = 0; c < C; c++)
#pragma unroll
    for (int p = 0; p < P; p++) acc[c][p] = 0.0f;
}

// V sums -> the wave's LDS planes (lane l: pixels P l .. P l + P - 1).
template <class L>
__device__ __forceinline__ void write_planes(float* planes, const float (&acc)[L::VC][L::VP], int lane) {
  constexpr int C = L::VC, P = L::VP;
#pragma unroll
  for (int c = 0; c < C; c++)
#pragma unroll
    for (int p = 0; p < P; p += 4)
      *reinterpret_cast<f32x4*>(planes + c * L::PL + (L::SPLIT ? (p / 4) * 4 * kLanes + 4 * lane : P * lane + p)) =
          f32x4{acc[c][p], acc[c][p + 1], acc[c][p + 2], acc[c][p + 3]};
}

__device__ __forceinline__ void wave_lds_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// u8 outputs are stored one byte per channel: dword stores of 4 packed bytes
// gathered across lanes through LDS measured no better (round 4,
// profiles/r04/ring_pack_b.jsonl: 480p 0.0898 vs 0.0903 ms per launch, C5
// 0.3249 vs 0.3203).  Tuning builds (-DMXD_U8_BPERM=1, round 6): RGB u8
// rows packed across lanes with ds_bpermute (no LDS memory): lane l gathers
// the two pixels its output dword at byte 4 l overlaps and stores one dword,
// 48 lanes x 4 bytes per instruction instead of 3 x 64 single bytes.
#ifndef MXD_U8_BPERM
#define MXD_U8_BPERM 0
#endif

// Horizontal pass of one strip: lane l owns output pixels l + 64 q (q < Q).
template <class L, bool F32, int T, int Q>
struct HStrip {
  static constexpr int C = L::C;
  float wx[Q][T];
  int pos[Q];  // first tap, in pixels from the window start
  int npx;     // output pixels of the strip

  // base: pos = first tap * HS - base is the first tap's float in a plane
  __device__ __forceinline__ void init(cgfloat* xtab, int xs, int crop_w, int flip, int ox0, int ox1, int base,
                                       int lane) {
    npx = ox1 - ox0;
#pragma unroll
    for (int q = 0; q < Q; q++) {
      const int px = min(lane + kLanes * q, npx - 1);
      const int ox = ox0 + px;
      const int xc = flip ? crop_w - 1 - ox : ox;
      cgfloat* xe = xtab + xc * xs;
      pos[q] = __float_as_int(xe[0]) * L::HS - base;
#pragma unroll
      for (int k = 0; k < T; k++) wx[q][k] = xe[kTapHeader + k];  // zero padded past the tap count
    }
  }

  // H taps of an output row from the LDS planes, stbir encode, store into
  // drow (the output row, pixel ox0 first).
  __device__ __forceinline__ void run(const float* planes, char* drow, int lane) const {
#pragma unroll
    for (int q = 0; q < Q; q++) {
      const int px = lane + kLanes * q;
      float s[C];
#pragma unroll
      for (int c = 0; c < C; c++) {
        const float* pl = planes + c * L::CS + pos[q];
        float a = 0.0f;
#pragma unroll
        for (int k = 0; k < T; k++) a = __builtin_fmaf(wx[q][k], pl[k * L::HS], a);
        s[c] = encode(a);
      }
      if (q > 0 && kLanes * q >= npx) break;  // uniform: no lane has pixels left
      if ((MXD_ABLATE & 2) && s[0] != -1.0f) continue;
      if constexpr (!F32 && C == 3 && MXD_U8_BPERM != 0) {
        char* row = drow + kLanes * q * 3;  // the chunk's 192 bytes (4-aligned when drow is)
        if ((reinterpret_cast<uintptr_t>(drow) & 3) == 0) {  // uniform
          const int pk = (int)((uint32_t)s[0] | ((uint32_t)s[1] << 8) | ((uint32_t)s[2] << 16));
          const int p0 = (4 * lane) / 3, r = 4 * lane - 3 * p0;
          const uint32_t a = (uint32_t)__builtin_amdgcn_ds_bpermute(4 * min(p0, kLanes - 1), pk);
          const uint32_t b = (uint32_t)__builtin_amdgcn_ds_bpermute(4 * min(p0 + 1, kLanes - 1), pk);
          const uint32_t w = (uint32_t)((((uint64_t)b << 24) | a) >> (8 * r));
          const int nbytes = 3 * min(kLanes, npx - kLanes * q);
          if (4 * lane + 4 <= nbytes) {
            *GLOBAL_PTR(uint32_t, row + 4 * lane) = w;
          } else if (4 * lane < nbytes) {
            for (int i = 0; i < nbytes - 4 * lane; i++) GLOBAL_PTR(uint8_t, row)[4 * lane + i] = (uint8_t)(w >> (8 * i));
          }
          continue;
        }
      }
      if (px < npx) {
        if constexpr (F32 && MXD_STORE_AUX != 0) {
          float q[C];
#pragma unroll
          for (int c = 0; c < C; c++) q[c] = div255(s[c]);
          store_row_px<C>(drow, px, q);
        } else if constexpr (F32) {
          auto* d = GLOBAL_PTR(float, drow) + px * C;
          if constexpr (C == 1) {
            store_out(d, div255(s[0]));
          } else if constexpr (C == 2) {
            store_out(reinterpret_cast<__attribute__((address_space(1))) f32x2*>(d), f32x2{div255(s[0]), div255(s[1])});
          } else if constexpr (C == 3) {
            store_out(reinterpret_cast<__attribute__((address_space(1))) f32x3*>(d),
                      f32x3{div255(s[0]), div255(s[1]), div255(s[2])});
          } else {
            store_out(reinterpret_cast<__attribute__((address_space(1))) f32x4*>(d),
                      f32x4{div255(s[0]), div255(s[1]), div255(s[2]), div255(s[3])});
          }
        } else {
          auto* d = GLOBAL_PTR(uint8_t, drow) + px * C;
#pragma unroll
          for (int c = 0; c < C; c++) d[c] = (uint8_t)s[c];  // byte stores: nontemporal measured no better
        }
      }
    }
  }
};

// Runs a band's scatter schedule (see the top of the file); on_row(acc, y) is
// called with the V sums of every completed output row y.
template <class L, int S, int DMAX, class SrcT, class OnRow, class Start>
__device__ __forceinline__ void scatter_band(kint* sched, int entry_off, const SrcT& src, OnRow&& on_row,
                                             Start&& start, bool prio, bool sync = false) {
  constexpr int C = L::VC;
  constexpr int R = scatter_ring_slots(DMAX, SrcT::kLaneBytes);
  constexpr int LA = R - 1;  // iterations loaded ahead
  constexpr int BG = scatter_block_groups(S, DMAX, SrcT::kLaneBytes);
  constexpr int E = scatter_entry_words(S);
  constexpr int P = L::VP;
  const int ngroups = sched[0];
  kint* gout = sched + 1;
  kint* itab = sched + entry_off;
  float acc[S][C][P];
#pragma unroll
  for (int s = 0; s < S; s++) zero_planes<C, P>(acc[s]);
  typename SrcT::RawT ring[R];
  static_for<LA>([&](auto ic) {
    __builtin_amdgcn_sched_barrier(0);  // issue in ring order: the loop's counted waits assume it
    ring[decltype(ic)::value] = src.load(itab[decltype(ic)::value * E + 1]);
  });
  __builtin_amdgcn_sched_barrier(0);
  start();  // after the prologue loads (see resample_wave)
  __builtin_amdgcn_sched_barrier(0);
  for (int gb = 0; gb < ngroups; gb += BG) {
    kint* blk = itab + gb * DMAX * E;
    static_for<BG>([&](auto gc) {
      constexpr int gi = decltype(gc)::value;
      // the group's entries in one scalar burst
      int ent[DMAX * E];
#pragma unroll
      for (int q = 0; q < DMAX * E; q++) ent[q] = blk[gi * DMAX * E + q];
      static_for<DMAX>([&](auto jc) {
        constexpr int j = decltype(jc)::value;
        constexpr int i = gi * DMAX + j;
        __builtin_amdgcn_sched_barrier(0);  // keep each row's work (and its load) in place
        // slot (i + LA) % R was consumed by the previous iteration
        ring[(i + LA) % R] = src.load(ent[j * E]);
        if (ent[j * E + 1] >= 0) {
          if constexpr ((MXD_ABLATE & 8) != 0) {
            acc[gi % S][0][0] += __uint_as_float(ring[i % R].d[0] & 0x3fffffffu);
            return;
          }
          float x[C][P];
          src.planes(ring[i % R], x);
          static_for<S>([&](auto kc) {
            constexpr int k = decltype(kc)::value;
            const int wbits = ent[j * E + 2 + k];
            if (k == 0 || wbits != 0) fma_planes<C, P>(acc[(gi + k) % S], __int_as_float(wbits), x);
          });
        }
      });
      const int y = gout[gb + gi];
      if (y >= 0) on_row(acc[gi % S], y);
      zero_planes<C, P>(acc[gi % S]);
      if constexpr (MXD_SYNC_STRIPS != 0)
        if (sync) __builtin_amdgcn_s_barrier();
    });
    progress_prio(prio, gb + BG, ngroups);
  }
}

// bytes per lane of Lay<c, p> (a plain function: template arguments do not
// parse inside __launch_bounds__)
constexpr int lane_bytes(int c, int p) { return c == 3 && p == 16 ? 16 : p * c; }

// Minimum waves per SIMD the register allocation must allow, by lane width.
constexpr int min_waves(int c, int p, int kind, int dmax) {
  (void)kind;
  (void)dmax;
  return lane_bytes(c, p) > 16 ? MXD_MIN_WAVES_WIDE : MXD_MIN_WAVES;
}

// One unit (image, band, strip) by the calling wave; planes = its LDS rows.
template <int C, int P, bool F32, int T, int Q, int KIND, int S, int DMAX, bool SHIFT, bool YCC, int LAUX>
__device__ __forceinline__ void run_unit(const ImgDev* __restrict__ imgs, int nimgs, int per_img, int unit,
                                         float* __restrict__ planes, int lane, bool prio) {
  using L = Lay<C, P>;
  constexpr int VC = L::VC, VP = L::VP;
  progress_prio(prio, 0, 1);
#if MXD_STAMPS
  const unsigned long long t_start = __builtin_amdgcn_s_memrealtime();
#endif

  // per_img > 0: every image has per_img units (no search: the wave issues
  // its first row loads one dependent descriptor load after it starts)
  const ImgDev& im = per_img > 0 ? imgs[unit / per_img] : find_image(imgs, nimgs, unit);
  const int nstrips = __builtin_amdgcn_readfirstlane(im.nstrips);
  const int crop_w = __builtin_amdgcn_readfirstlane(im.crop_w);
  const int crop_h = __builtin_amdgcn_readfirstlane(im.crop_h);
  const int flip_shift = __builtin_amdgcn_readfirstlane(im.flip);
  const int flip = flip_shift & 1, shift = flip_shift >> 8;  // see ImgDev::flip
  const int band_rows = __builtin_amdgcn_readfirstlane(im.ty);
  const int strip_cols = __builtin_amdgcn_readfirstlane(im.tx);
  const int xs = kTapHeader + __builtin_amdgcn_readfirstlane(im.xwidth);
  const int ys = kTapHeader + __builtin_amdgcn_readfirstlane(im.ywidth);
  cgfloat* xtab = GLOBAL_PTR(const float, im.xtab);
  // The vertical taps / schedule are read with scalar loads (lgkmcnt), which
  // never wait on the vector loads of the next rows.
  kfloat* ytab = uniform_ptr<kfloat*>(im.ytab);
  char* dst = reinterpret_cast<char*>(im.dst);
  const int64_t dstride = im.dst_stride;
  const int local = unit - __builtin_amdgcn_readfirstlane(im.tile_begin);
  const int band = local / nstrips;
  const int strip = local - band * nstrips;
  const int oy0 = band * band_rows;
  const int oy1 = min(oy0 + band_rows, crop_h);
  const int ox0 = strip * strip_cols;
  const int ox1 = min(ox0 + strip_cols, crop_w);

  int lo, hi;
  strip_span(xtab, xs, crop_w, flip, ox0, ox1, &lo, &hi);
  const int sx0 = __builtin_amdgcn_readfirstlane(im.src_x0);
  Src<L, SHIFT, LAUX> src;
  int hbase;  // HStrip base (see HStrip::init)
  {
    void* base = uniform_ptr<void*>(im.src);
    const int stride = __builtin_amdgcn_readfirstlane((int)im.src_stride);
    const int rows = __builtin_amdgcn_readfirstlane(im.src_h);
    // records end at the last stored row's last pixel (a page-locked source
    // read in place must not be read past its image)
    src.live = __builtin_amdgcn_make_buffer_rsrc(
        base, (short)0, src_records(shift, rows, stride, (__builtin_amdgcn_readfirstlane(im.src_w) - sx0) * C),
        0x00020000);
    src.dead = __builtin_amdgcn_make_buffer_rsrc(base, (short)0, 0, 0x00020000);
    src.stride = stride;
    src.y0 = __builtin_amdgcn_readfirstlane(im.src_y0);
    if constexpr (L::B) {
      // byte lanes: window = the span's bytes from a 16-byte boundary past the
      // 4-byte aligned base (the host checked it fits 1 KiB and, 16-byte chunks
      // rounded up, stays inside the row's stride)
      const int b0 = ((lo - sx0) * C + shift) & ~15;
      const int nb = (hi + 1 - sx0) * C + shift - b0;
      src.sh = 0;
      src.voff = L::LB * lane < nb ? b0 + L::LB * lane : kNoLoad;
      hbase = sx0 * C - shift + b0;
    } else {
      constexpr int A = C == 2 ? 2 : C == 4 ? 1 : 4;  // wp0 * C a multiple of 4
      const int wp0 = lo & ~(A - 1);
      const int npx = hi + 1 - wp0;
      // window start, bytes past the 4-byte aligned base of the stored region
      const int fbyte = (wp0 - sx0) * C + shift;
      src.sh = fbyte & 3;
      if constexpr (L::SPLIT) {
        src.voff = 4 * lane < npx ? (fbyte & ~3) + 4 * C * lane : kNoLoad;
        src.voff2 = 4 * kLanes + 4 * lane < npx ? (fbyte & ~3) + L::HALF + 4 * C * lane : kNoLoad;
      } else {
        src.voff = P * lane < npx ? (fbyte & ~3) + L::LB * lane : kNoLoad;
      }
      hbase = wp0;
    }
  }
  HStrip<L, F32, T, Q> hs;
  // The horizontal weights are loaded once, right after the band's first row
  // loads (their latencies overlap), and retired together with those rows, so
  // the waits the compiler places in the row loop only ever cover row loads.
  auto start = [&] {
    hs.init(xtab, xs, crop_w, flip, ox0, ox1, hbase, lane);
    __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0)
  };

  char* dcol = dst + (int64_t)ox0 * C * (F32 ? 4 : 1);
  // V row of output row y done: planes to LDS, H pass and store.
  auto finish_row = [&](const float (&acc)[VC][VP], int y) {
    if constexpr ((MXD_ABLATE & 4) != 0) {
      float t = 0.0f;
#pragma unroll
      for (int c = 0; c < VC; c++)
#pragma unroll
        for (int p = 0; p < VP; p++) t += acc[c][p];
      if (t == -1.0f) planes[lane] = t;
      GLOBAL_PTR(float, dcol + (int64_t)y * dstride)[lane] = 0.0f;
      return;
    }
    write_planes<L>(planes, acc, lane);
    wave_lds_sync();
    hs.run(planes, dcol + (int64_t)y * dstride, lane);
    wave_lds_sync();
  };

  if constexpr (KIND == kGather) {
    // ---- gather: each output row sums its T source rows, loaded for it ----
    auto load_rows = [&](Raw<L::ND>* R, int y, bool live) {
      const int n0 = __float_as_int(ytab[y * ys]);
#pragma unroll
      for (int k = 0; k < T; k++) R[k] = src.load(live ? n0 + k : -1);
    };
    auto step = [&](const Raw<L::ND>* R, int y) {
      kfloat* ye = ytab + y * ys;
      float acc[VC][VP];
      zero_planes<VC, VP>(acc);
#pragma unroll
      for (int k = 0; k < T; k++) {  // zero padded past the tap count
        float x[VC][VP];
        to_planes<VC, VP>(R[k], x);
        fma_planes<VC, VP>(acc, ye[kTapHeader + k], x);
      }
      finish_row(acc, y);
    };
    // Double-buffered rows: the loads of row y+1 are issued before row y is
    // computed, so they fly during the whole V+H of row y.  The prefetch is
    // unconditional (clamped to the last output row) so every path through
    // the loop has the same loads in flight and the compiler's counted waits
    // stay partial.
    Raw<L::ND> RA[T], RB[T];
    load_rows(RA, oy0, true);
    start();
    for (int y = oy0;; y += 2) {
      progress_prio(prio, y - oy0, oy1 - oy0);
      load_rows(RB, min(y + 1, crop_h - 1), y + 1 < oy1);
      step(RA, y);
      if (y + 1 >= oy1) break;
      load_rows(RA, min(y + 2, crop_h - 1), y + 2 < oy1);
      step(RB, y + 1);
      if (y + 2 >= oy1) break;
    }
  } else {
    // ---- scatter: follow the band's schedule ----
    kint* sched = reinterpret_cast<kint*>(ytab) + band * __builtin_amdgcn_readfirstlane(im.ywidth);
    const bool sync = nstrips == kWaves && ((unit - local + band * nstrips) & (kWaves - 1)) == 0;
    if constexpr (YCC) {
      static_assert(C == 3 && P == 4 && !SHIFT, "JPEG plane sources: RGB pixel lanes, P = 4, aligned windows");
      // the same window as the RGB source would have (hbase = wp0), read from the planes
      const YccDev* yd = uniform_ptr<const YccDev*>(im.ycc);
      YccSrc ys;
      const int records = __builtin_amdgcn_readfirstlane(yd->records);
      ys.live = __builtin_amdgcn_make_buffer_rsrc(uniform_ptr<void*>(im.src), (short)0, records, 0x00020000);
      ys.dead = __builtin_amdgcn_make_buffer_rsrc(uniform_ptr<void*>(im.src), (short)0, 0, 0x00020000);
      ys.ystride = __builtin_amdgcn_readfirstlane(yd->ystride);
      ys.cstride = __builtin_amdgcn_readfirstlane(yd->cstride);
      ys.cb = __builtin_amdgcn_readfirstlane((int)yd->cb);
      ys.cr = __builtin_amdgcn_readfirstlane((int)yd->cr);
      ys.dw = __builtin_amdgcn_readfirstlane(yd->dw);
      ys.dh = __builtin_amdgcn_readfirstlane(yd->dh);
      ys.wy = __builtin_amdgcn_readfirstlane(yd->win_y);
      const int wx = __builtin_amdgcn_readfirstlane(yd->win_x);
      const int xl = wx + hbase + 4 * lane;  // the lane's first pixel (image column)
      const bool on = 4 * lane < hi + 1 - hbase;
      const int c = xl >> 1, d = c > 0 ? (c - 1) >> 2 : 0;
      ys.yoff = on ? ys.wy * ys.ystride + xl : kNoLoad;
      ys.coff = on ? 4 * d : kNoLoad;
      ys.e = c - 1 - 4 * d;
      ys.ci = c;
      scatter_band<L, S, DMAX>(sched, __builtin_amdgcn_readfirstlane(im.group), ys, finish_row, start, prio, sync);
    } else {
      scatter_band<L, S, DMAX>(sched, __builtin_amdgcn_readfirstlane(im.group), src, finish_row, start, prio, sync);
    }
  }
#if MXD_STAMPS
  if (lane == 0 && unit < kMaxStamped) {
    g_stamps[2 * unit] = t_start;
    g_stamps[2 * unit + 1] = __builtin_amdgcn_s_memrealtime();
  }
#endif
}

template <int C, int P, bool F32, int T, int Q, int KIND, int S, int DMAX, bool SHIFT, bool YCC = false,
          int LAUX = MXD_LOAD_AUX>
__global__ __launch_bounds__(kWaves* kLanes, min_waves(C, P, KIND, DMAX)) void resample_wave(
    const ImgDev* __restrict__ imgs, int nimgs, int nunits, int per_img, int prio) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  using L = Lay<C, P>;
  constexpr int PL = L::PL;
  const int lane = threadIdx.x & (kLanes - 1);
  const int unit = __builtin_amdgcn_readfirstlane(xcd_remap(blockIdx.x, gridDim.x) * kWaves + (threadIdx.x >> 6));
  float* __restrict__ planes = smem + (threadIdx.x >> 6) * (L::VC * PL);
#pragma unroll
  for (int c = 0; c < L::VC; c++)
#pragma unroll
    for (int i = 0; i < L::PAD; i += kLanes)
      if (i + lane < L::PAD) planes[c * PL + L::WPX + i + lane] = 0.0f;  // padded taps read zeros
  if (unit < nunits)
    run_unit<C, P, F32, T, Q, KIND, S, DMAX, SHIFT, YCC, LAUX>(imgs, nimgs, per_img, unit, planes, lane,
                                                    __builtin_amdgcn_readfirstlane(prio) != 0);
}

using WaveKernel = void (*)(const ImgDev*, int, int, int, int);

constexpr int default_p(int c) { return c == 1 ? 16 : c == 2 ? 8 : 4; }

template <int C, bool F32, int T, int Q>
WaveKernel select_gather(const WaveCfg& cfg) {
  constexpr int P = default_p(C);
  if (cfg.shift) return resample_wave<C, P, F32, T, Q, kGather, 1, 1, true>;
  return resample_wave<C, P, F32, T, Q, kGather, 1, 1, false>;
}

template <int C, bool F32, int Q>
WaveKernel select_taps(const WaveCfg& cfg) {
  switch (cfg.taps) {
    case 2: return select_gather<C, F32, 2, Q>(cfg);
    case 3: return select_gather<C, F32, 3, Q>(cfg);
    case 4: return select_gather<C, F32, 4, Q>(cfg);
    case 6: return select_gather<C, F32, 6, Q>(cfg);
    case 8: return select_gather<C, F32, 8, Q>(cfg);
    case 10: return select_gather<C, F32, 10, Q>(cfg);
    case 12: return select_gather<C, F32, 12, Q>(cfg);
    case 17: return select_gather<C, F32, 17, Q>(cfg);
    default: return nullptr;
  }
}

template <int C, bool F32>
WaveKernel select_q(const WaveCfg& cfg) {
  if (cfg.p != default_p(C)) return nullptr;
  switch (cfg.q) {
    case 1: return select_taps<C, F32, 1>(cfg);
    case 2: return select_taps<C, F32, 2>(cfg);
    case 4: return select_taps<C, F32, 4>(cfg);
    default: return nullptr;
  }
}

// Scatter kernels exist for RGB and the (S, DMAX, horizontal taps, Q, P)
// shapes of resize_smallest_side 256/512 from 200p..4K sources: downsampling
// by the tent filter reaches each source row from at most two output rows
// (S = 2), DMAX = ceil(in / out).
template <bool F32>
WaveKernel select_scatter(const WaveCfg& cfg) {
  if (cfg.channels != 3) return nullptr;
#define MXD_SCATTER(S_, D_, T_, Q_, P_)                                                           \
  if (cfg.s == S_ && cfg.dmax == D_ && cfg.taps == T_ && cfg.q == Q_ && cfg.p == P_)              \
    return cfg.ycc ? (P_ == 4 && !cfg.shift ? resample_wave<3, 4, F32, T_, Q_, kScatter, S_, D_, false, true> \
                                            : nullptr)                                            \
           : cfg.shift ? (cfg.nt ? resample_wave<3, P_, F32, T_, Q_, kScatter, S_, D_, true, false, kLoadNt> \
                                 : resample_wave<3, P_, F32, T_, Q_, kScatter, S_, D_, true>)     \
                       : (cfg.nt ? resample_wave<3, P_, F32, T_, Q_, kScatter, S_, D_, false, false, kLoadNt> \
                                 : resample_wave<3, P_, F32, T_, Q_, kScatter, S_, D_, false>);
  // byte lanes (P = 16): any base alignment, no realignment variant
#define MXD_SCATTER_B(S_, D_, T_, Q_)                                                             \
  if (cfg.s == S_ && cfg.dmax == D_ && cfg.taps == T_ && cfg.q == Q_ && cfg.p == 16 && !cfg.ycc)  \
    return cfg.nt ? resample_wave<3, 16, F32, T_, Q_, kScatter, S_, D_, false, false, kLoadNt>    \
                  : resample_wave<3, 16, F32, T_, Q_, kScatter, S_, D_, false>;
  MXD_SCATTER(2, 4, 8, 2, 8)    // 960 -> 256 (C2)
#ifndef MXD_ONLY_C2  // register-count checks of one kernel (tools/wave_regs.sh)
  MXD_SCATTER(2, 4, 8, 1, 4)
  MXD_SCATTER(2, 5, 10, 2, 8)   // 1080 -> 256, 2160 -> 512 (C5)
  MXD_SCATTER(2, 5, 10, 1, 4)
  MXD_SCATTER(2, 6, 12, 2, 8)   // 1440 -> 256
  MXD_SCATTER(2, 6, 12, 1, 4)
  MXD_SCATTER(2, 9, 17, 1, 8)   // 2160 -> 256
  MXD_SCATTER(2, 9, 17, 1, 4)
  MXD_SCATTER(2, 3, 6, 2, 8)    // 720 -> 256
  MXD_SCATTER(2, 3, 6, 2, 4)
  MXD_SCATTER(2, 2, 4, 2, 4)    // 480 -> 256
  MXD_SCATTER(2, 2, 4, 4, 8)
  MXD_SCATTER(2, 2, 3, 2, 4)    // 375 / 333 -> 256 (C4)
  MXD_SCATTER(2, 2, 3, 4, 8)
  MXD_SCATTER(3, 1, 2, 4, 4)    // upsampling (200 -> 256)
  MXD_SCATTER(2, 12, 24, 1, 8)  // 8.5..12:1 (12 MP -> 256, C6)
  MXD_SCATTER(2, 12, 24, 1, 4)
  MXD_SCATTER(2, 16, 32, 1, 8)  // 12..16:1 (24 MP -> 256, C7)
  MXD_SCATTER(2, 16, 32, 1, 4)
  // byte lanes: 1 KiB windows (341 RGB pixels) per strip row
  MXD_SCATTER_B(2, 4, 8, 2)     // 960 -> 256 (C2: 3 strips of 75)
  MXD_SCATTER_B(2, 4, 8, 1)
  MXD_SCATTER_B(2, 5, 10, 2)    // 1080 -> 256, 2160 -> 512 (C5: 6 strips of 75)
  MXD_SCATTER_B(2, 5, 10, 1)
  MXD_SCATTER_B(2, 6, 12, 1)    // 1440 -> 256 (4 strips of 56)
  MXD_SCATTER_B(2, 6, 12, 2)
  MXD_SCATTER_B(2, 9, 17, 1)    // 2160 -> 256 (6 strips of 38)
  MXD_SCATTER_B(2, 3, 6, 2)     // 720 -> 256 (2 strips of 112)
  MXD_SCATTER_B(2, 2, 4, 2)     // 480 -> 256
  MXD_SCATTER_B(2, 2, 4, 4)
  MXD_SCATTER_B(2, 2, 3, 4)     // 375 / 333 -> 256 (C4: one strip)
  MXD_SCATTER_B(2, 2, 3, 2)
  MXD_SCATTER_B(3, 1, 2, 4)     // upsampling (200 -> 256)
#endif
#undef MXD_SCATTER_B
#undef MXD_SCATTER
  return nullptr;
}

WaveKernel select_kernel(const WaveCfg& cfg) {
#ifdef MXD_ONLY_C2
  return cfg.kind == kScatter && cfg.f32 ? select_scatter<true>(cfg) : nullptr;
#endif
  if (cfg.kind == kScatter) return cfg.f32 ? select_scatter<true>(cfg) : select_scatter<false>(cfg);
  if (cfg.ycc) return nullptr;  // JPEG plane sources: scatter kernels only
  switch (cfg.channels * 2 + (cfg.f32 ? 1 : 0)) {
    case 2: return select_q<1, false>(cfg);
    case 3: return select_q<1, true>(cfg);
    case 4: return select_q<2, false>(cfg);
    case 5: return select_q<2, true>(cfg);
    case 6: return select_q<3, false>(cfg);
    case 7: return select_q<3, true>(cfg);
    default: return nullptr;
  }
}

int lds_bytes(const WaveCfg& cfg) { return kWaves * wave_plane_floats(cfg.channels, cfg.p) * (int)sizeof(float); }

template <int C, int P>
constexpr int plane_floats() {
  return Lay<C, P>::VC * Lay<C, P>::PL;
}

}  // namespace

int wave_taps_bucket(int taps) {
  static const int kB[] = {2, 3, 4, 6, 8, 10, 12, 17, 24, 32};
  for (int b : kB)
    if (taps <= b) return b;
  return -1;
}

int wave_default_p(int channels) { return default_p(channels); }

int wave_window_px(int channels, int p) { return kLanes * p; }

int wave_window_align(int channels) { return channels == 2 ? 2 : channels == 4 ? 1 : 4; }

bool wave_byte_lanes(int channels, int p) { return channels == 3 && p == 16; }

int wave_byte_window() { return kLanes * 16; }

int wave_plane_floats(int channels, int p) {
  if (wave_byte_lanes(channels, p)) return plane_floats<3, 16>();
  return channels * (kLanes * p + kPad);
}

int wave_lanes() { return kLanes; }

bool wave_has_kernel(const WaveCfg& cfg) { return select_kernel(cfg) != nullptr; }

// Streaming copy: one 16-B load and store per thread, one block per 4 KiB
// (no grid-stride loop): the form that measured fastest on MI355X
// (tools/membench2.hip, 6.2 TB/s over 1 GiB).  bench.py reports it as the
// measured HBM ceiling next to the spec peak.
__global__ __launch_bounds__(256) void copy_f4(const f32x4* __restrict__ a, f32x4* __restrict__ b, size_t n) {
  const size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
  if (i < n) b[i] = a[i];
}

// The same copy with a cache policy on both sides (buffer loads / stores,
// one 4-KiB window per block): AUX 2 = nt, 18 = nt sc1 -- the streaming forms
// tools/nt_ceiling.hip measured fastest (round 6), so bench.py can quote the
// ceiling the nt-load kernels are held to on the box it runs on.
template <int AUX>
__global__ __launch_bounds__(256) void copy_policy(const char* __restrict__ a, char* __restrict__ b, size_t bytes) {
  const size_t base = (size_t)blockIdx.x * 4096;
  const int n = (int)min((size_t)4096, bytes - base);
  const Rsrc ra = __builtin_amdgcn_make_buffer_rsrc(const_cast<char*>(a) + base, (short)0, n, 0x00020000);
  const Rsrc rb = __builtin_amdgcn_make_buffer_rsrc(b + base, (short)0, n, 0x00020000);
  const u32x4 v = __builtin_amdgcn_raw_buffer_load_b128(ra, threadIdx.x * 16, 0, AUX);
  __builtin_amdgcn_raw_buffer_store_b128(v, rb, threadIdx.x * 16, 0, AUX);
}

int launch_copy(const void* src, void* dst, size_t bytes, void* stream, int policy) {
  const size_t n = bytes / 16;
  const auto s = reinterpret_cast<hipStream_t>(stream);
  if (policy == 0) {
    hipLaunchKernelGGL(copy_f4, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s,
                       reinterpret_cast<const f32x4*>(src), reinterpret_cast<f32x4*>(dst), n);
  } else {
    const unsigned blocks = (unsigned)((n * 16 + 4095) / 4096);
    const auto* a = static_cast<const char*>(src);
    auto* b = static_cast<char*>(dst);
    if (policy == 1) hipLaunchKernelGGL(copy_policy<2>, dim3(blocks), dim3(256), 0, s, a, b, n * 16);
    else hipLaunchKernelGGL(copy_policy<18>, dim3(blocks), dim3(256), 0, s, a, b, n * 16);
  }
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

int launch_wave(const WaveCfg& cfg, const ImgDev* imgs, void* stream) {
  const WaveKernel k = select_kernel(cfg);
  if (!k) return -2;
  const int blocks = (cfg.nunits + kWaves - 1) / kWaves;
  hipLaunchKernelGGL(k, dim3(blocks), dim3(kWaves * kLanes), lds_bytes(cfg), reinterpret_cast<hipStream_t>(stream),
                     imgs, cfg.nimgs, cfg.nunits, cfg.per_img, cfg.prio);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

int wave_kernel_info(const WaveCfg& cfg, int device, int* api_blocks, int* vgprs, int* lds) {
  const WaveKernel k = select_kernel(cfg);
  if (!k) return -1;
  hipFuncAttributes a{};
  if (hipFuncGetAttributes(&a, reinterpret_cast<const void*>(k)) != hipSuccess) return -1;
  *vgprs = a.numRegs;
  *lds = lds_bytes(cfg);
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(api_blocks, reinterpret_cast<const void*>(k), kWaves * kLanes,
                                                   *lds) != hipSuccess)
    return -1;
  (void)device;
  return kWaves;
}

int wave_capacity(const WaveCfg& cfg, int device) {
  const WaveKernel k = select_kernel(cfg);
  if (!k) return 0;
  int blocks = 0, cus = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&blocks, reinterpret_cast<const void*>(k), kWaves * kLanes,
                                                   lds_bytes(cfg)) != hipSuccess)
    return 0;
  if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device) != hipSuccess) return 0;
  return blocks * kWaves * cus;
}

}  // namespace mxd

#if MXD_STAMPS
// Copies the first n units' (start, end) stamps of the last stamped launches.
extern "C" int mxd_debug_stamps(unsigned long long* host, int n) {
  if (n > mxd::kMaxStamped) n = mxd::kMaxStamped;
  return hipMemcpyFromSymbol(host, HIP_SYMBOL(mxd::g_stamps), sizeof(unsigned long long) * 2 * n, 0,
                             hipMemcpyDeviceToHost) == hipSuccess ? 0 : -1;
}
#endif
