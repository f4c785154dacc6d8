// band.hip -- the row-stream kernel of the fused resize + crop (+ hflip) (+ /255)
// stage; structure and LDS layout in band.h.
//
// Reference arithmetic replaced: core::image::resize -> stbir_resize_uint8_linear
// (mlx/data/core/image/ImageTransform.cpp:41-62, triangle filter :7-9), then
// core::image::crop / hflip (:64-73, :123-140) and the benchmark's
// astype(float32) / 255 (benchmarks/comparative/caltech101/mlx_data.py:46).
//
// Why this shape (measured on the wave kernel): ~4,000 waves
// each streaming its own band of 1.5-KiB row pieces sat at the probe floor of
// that access pattern (~0.15 ms for C2).  Here one workgroup streams whole
// contiguous footprint rows (1 KiB per LDS-DMA instruction) of one band, the
// loads need no VGPRs, and every output row leaves as one contiguous run of
// 12-byte (f32 RGB) stores.
#include <hip/hip_runtime.h>

#include "band.h"
#include "devutil.h"

namespace mxd {
namespace {

using namespace dev;

constexpr int kThreads = kBandThreads;
constexpr int kLanes = 64;
constexpr int kWaves = kThreads / kLanes;
constexpr int kChunk = kBandChunk;
constexpr int E = kBandEntryWords;
// A voffset past any buffer: the range check drops the access (loads: no
// request, zeros; stores: nothing written).
constexpr int kNoLoad = 0x7ffffff0;
using lds_u8 = __attribute__((address_space(3))) uint8_t;
typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
typedef uint32_t u32x3 __attribute__((ext_vector_type(3)));
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

// f32 results are stored nontemporally (written once, never read here; the
// wave kernel measured 0.0325 -> 0.0263 ms on C4 from it).  Tuning builds:
// -DMXD_BAND_NT=0.
#ifndef MXD_BAND_NT
#define MXD_BAND_NT 1
#endif
constexpr int kStoreAux = MXD_BAND_NT ? 2 : 0;  // gfx950 cache-policy bits: 2 = nt
// Cache policy of the source LDS-DMA (tuning builds: -DMXD_BAND_LOAD_AUX=2 = nt).
#ifndef MXD_BAND_LOAD_AUX
#define MXD_BAND_LOAD_AUX 0
#endif
// Progress-based priority (as wave.hip's progress_prio; tuning builds
// -DMXD_BAND_PRIO=0): the SIMD arbiter issues oldest-first, so the workgroups
// sharing a CU would otherwise finish in age order (C2 stamps: units of one
// launch ending between 120 and 161 us); each unit lowers its s_setprio level
// as it completes quarters of its band, so units behind win the arbiter.
#ifndef MXD_BAND_PRIO
#define MXD_BAND_PRIO 1
#endif
__device__ __forceinline__ void band_prio(int done, int total) {
  if constexpr (MXD_BAND_PRIO != 0) {
    switch (3 - (4 * done) / (total + 1)) {
      case 3: __builtin_amdgcn_s_setprio(3); break;
      case 2: __builtin_amdgcn_s_setprio(2); break;
      case 1: __builtin_amdgcn_s_setprio(1); break;
      default: __builtin_amdgcn_s_setprio(0); break;
    }
  }
}

// Timing-only ablations (tools/band_variants.sh builds, never the product
// library): 1 = no source loads, 2 = no output stores, 4 = no horizontal
// arithmetic, 8 = no vertical arithmetic.
#ifndef MXD_BAND_ABLATE
#define MXD_BAND_ABLATE 0
#endif

// Branch-free vertical pass (see vpass); tuning builds: -DMXD_BAND_BRANCHLESS=0.
#ifndef MXD_BAND_BRANCHLESS
#define MXD_BAND_BRANCHLESS 1
#endif

// Tuning builds: -DMXD_BAND_PPW_ALIGN=32 rounds each wave's pixel run up to
// whole 128-byte lines of f32 RGB output.
#ifndef MXD_BAND_PPW_ALIGN
#define MXD_BAND_PPW_ALIGN 1
#endif

#define RFL(x) __builtin_amdgcn_readfirstlane(x)

// Diagnostic builds only (-DMXD_BAND_STAMPS=1, tools/band_stamps.sh; never
// the product library): wave 0 of every unit sums the shader-clock cycles of
// each segment of its steps, read back with mxd_debug_band_stamps.
#ifndef MXD_BAND_STAMPS
#define MXD_BAND_STAMPS 0
#endif
[[maybe_unused]] constexpr int kStampSegs = 10;  // setup, wait, barrier 1, H, V, barrier 2, write+issue, steps, start, end
#if MXD_BAND_STAMPS
constexpr int kMaxStamped = 8192;
__device__ unsigned long long g_band_stamps[kStampSegs * kMaxStamped];
#define MXD_STAMP(var) const unsigned long long var = __builtin_amdgcn_s_memtime()
#define MXD_SEG(k, a, b) seg[k] += (b) - (a)
#else
#define MXD_STAMP(var)
#define MXD_SEG(k, a, b)
#endif

// s_waitcnt vmcnt(n) for a run-time, wave-uniform n (the count is an
// immediate); n > 63 waits for 63 (more than asked: always safe).
__device__ __forceinline__ void wait_vmcnt(int n) {
#define MXD_VMC(k) \
  case k:          \
    asm volatile("s_waitcnt vmcnt(" #k ")" ::: "memory"); \
    break;
#define MXD_VMC8(b) MXD_VMC(b) MXD_VMC(b + 1) MXD_VMC(b + 2) MXD_VMC(b + 3) MXD_VMC(b + 4) MXD_VMC(b + 5) \
    MXD_VMC(b + 6) MXD_VMC(b + 7)
  switch (n < 63 ? n : 63) {
    MXD_VMC8(0) MXD_VMC8(8) MXD_VMC8(16) MXD_VMC8(24) MXD_VMC8(32) MXD_VMC8(40) MXD_VMC8(48) MXD_VMC8(56)
    default:
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
#undef MXD_VMC8
#undef MXD_VMC
}

// Workgroup barrier for LDS hand-offs: this wave's LDS writes done, then
// s_barrier.  LDS-DMA data is covered by each wave's own wait_vmcnt before it
// (a __syncthreads() would also wait vmcnt(0) and drain the ring).
__device__ __forceinline__ void barrier_lds() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

// One output pixel's C encoded channels to the buffer (vector stores; SW of
// them per wave and output row, the same in every wave: inactive lanes carry
// an out-of-range offset).
template <int C, bool F32>
constexpr int store_instrs() {
  return (!F32 && C == 3) ? 3 : 1;
}

template <int C, bool F32>
__device__ __forceinline__ void store_pixel(__amdgpu_buffer_rsrc_t rs, int voff, const float (&q)[C]) {
  if constexpr (F32) {
    if constexpr (C == 1) {
      __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(div255(q[0])), rs, voff, 0, kStoreAux);
    } else if constexpr (C == 2) {
      __builtin_amdgcn_raw_buffer_store_b64(u32x2{__float_as_uint(div255(q[0])), __float_as_uint(div255(q[1]))}, rs,
                                            voff, 0, kStoreAux);
    } else if constexpr (C == 3) {
      __builtin_amdgcn_raw_buffer_store_b96(
          u32x3{__float_as_uint(div255(q[0])), __float_as_uint(div255(q[1])), __float_as_uint(div255(q[2]))}, rs,
          voff, 0, kStoreAux);
    } else {
      __builtin_amdgcn_raw_buffer_store_b128(u32x4{__float_as_uint(div255(q[0])), __float_as_uint(div255(q[1])),
                                                   __float_as_uint(div255(q[2])), __float_as_uint(div255(q[3]))},
                                             rs, voff, 0, kStoreAux);
    }
  } else {
    const uint32_t b0 = (uint32_t)q[0];
    if constexpr (C == 1) {
      __builtin_amdgcn_raw_buffer_store_b8((uint8_t)b0, rs, voff, 0, 0);
    } else if constexpr (C == 2) {
      __builtin_amdgcn_raw_buffer_store_b16((uint16_t)(b0 | ((uint32_t)q[1] << 8)), rs, voff, 0, 0);
    } else if constexpr (C == 3) {
      // byte stores (a pixel's 3 bytes are not 2-byte aligned every other
      // pixel); an out-of-range voffset stays out of range 1 or 2 bytes on
      __builtin_amdgcn_raw_buffer_store_b8((uint8_t)b0, rs, voff, 0, 0);
      __builtin_amdgcn_raw_buffer_store_b8((uint8_t)(uint32_t)q[1], rs, voff + 1, 0, 0);
      __builtin_amdgcn_raw_buffer_store_b8((uint8_t)(uint32_t)q[2], rs, voff + 2, 0, 0);
    } else {
      __builtin_amdgcn_raw_buffer_store_b32(b0 | ((uint32_t)q[1] << 8) | ((uint32_t)q[2] << 16) | ((uint32_t)q[3] << 24),
                                            rs, voff, 0, 0);
    }
  }
}

// What the cursors of the stream need of one unit (wave-uniform: SGPRs).
struct Unit {
  __amdgpu_buffer_rsrc_t src, dst;
  kint* sched;  // the band's first group
  int ng;       // groups (0: no unit -- past the last one)
  int b0, bend, y0, stride;  // source window of the strip (LDS-DMA)
  int dstride, oy0;          // output rows
  int vboff;                 // vertical-row float index of source pixel 0, channel 0 (minus first tap * C)
};

// The horizontal pass's per-lane state of one unit, and the raw table words
// it is made from (loaded ahead; unpacked when the unit becomes current).
template <int T>
struct Lanes {
  float wx[T];
  int vb;     // vertical-row float index of the pixel's tap 0, channel 0
  int scol;   // output byte column, kNoLoad for lanes without a pixel
};
template <int T>
constexpr int raw_words() {
  return (kTapHeader + T + 3) / 4;  // 16-byte table loads per lane
}

template <int C, bool F32>
__device__ __forceinline__ Unit load_unit(const ImgDev* imgs, kint* unit_img, int per_img, int u, int nunits,
                                          int* npx_out, int* ox0_out, int* xs_out, cgfloat** xtab_out, int* crop_w_out,
                                          int* flip_out) {
  constexpr int ELEM = F32 ? 4 : 1;
  Unit U;
  if (u >= nunits) {
    U.src = U.dst = __builtin_amdgcn_make_buffer_rsrc((void*)nullptr, (short)0, 0, 0x00020000);
    U.sched = nullptr;
    U.ng = 0;
    U.b0 = U.bend = U.y0 = U.stride = U.dstride = U.oy0 = U.vboff = 0;
    *npx_out = *ox0_out = *xs_out = *crop_w_out = *flip_out = 0;
    *xtab_out = nullptr;
    return U;
  }
  const int ii = per_img > 0 ? u / per_img : unit_img[u];
  const ImgDev& im = imgs[ii];
  const int nstrips = RFL(im.nstrips);
  const int crop_w = RFL(im.crop_w);
  const int crop_h = RFL(im.crop_h);
  const int fl = RFL(im.flip);
  const int flip = fl & 1, shift = fl >> 8;  // see ImgDev::flip
  const int band_rows = RFL(im.ty);
  const int strip_cols = RFL(im.tx);
  const int xs = kTapHeader + RFL(im.xwidth);
  cgfloat* xtab = MXD_GLOBAL_PTR(const float, im.xtab);
  const int local = u - RFL(im.tile_begin);
  const int band = local / nstrips;
  const int strip = local - band * nstrips;
  const int ox0 = strip * strip_cols;
  const int npx = min(strip_cols, crop_w - ox0);
  // the strip's first and last source pixel, by scalar loads (a vector load
  // here would make the wave wait for the LDS-DMA in flight)
  kint* xti = uniform_ptr<kint*>(im.xtab);
  const int xa = flip ? crop_w - (ox0 + npx) : ox0;
  const int xb = flip ? crop_w - 1 - ox0 : ox0 + npx - 1;
  const int lo = xti[xa * xs];
  const int hi = xti[xb * xs] + xti[xb * xs + 1] - 1;
  const int sx0 = RFL(im.src_x0);
  U.y0 = RFL(im.src_y0);
  U.stride = RFL((int)im.src_stride);
  const int rows = RFL(im.src_h), srcw = RFL(im.src_w);
  U.src = __builtin_amdgcn_make_buffer_rsrc(uniform_ptr<void*>(im.src), (short)0,
                                            src_records(shift, rows, U.stride, (srcw - sx0) * C), 0x00020000);
  U.b0 = ((lo - sx0) * C + shift) & ~15;  // window start: 16-byte boundary past the aligned base
  U.bend = (hi + 1 - sx0) * C + shift;    // one past the strip's last source byte
  U.vboff = -sx0 * C + shift - U.b0;
  U.dstride = RFL((int)im.dst_stride);
  U.dst = __builtin_amdgcn_make_buffer_rsrc(uniform_ptr<void*>(im.dst), (short)0,
                                            (crop_h - 1) * U.dstride + crop_w * C * ELEM, 0x00020000);
  U.oy0 = band * band_rows;
  kint* hdr = uniform_ptr<kint*>(im.ytab) + band * RFL(im.ywidth);
  U.ng = hdr[0];
  U.sched = hdr + E;
  *npx_out = npx;
  *ox0_out = ox0;
  *xs_out = xs;
  *xtab_out = xtab;
  *crop_w_out = crop_w;
  *flip_out = flip;
  return U;
}

template <int C, bool F32, int NQ, int T, int S, int DB>
__global__ __launch_bounds__(kThreads, 2) void resample_band(const ImgDev* __restrict__ imgs,
                                                             const int* __restrict__ unit_img_p, int nunits,
                                                             int per_img, int la) {
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  constexpr int DS = DB > 4 ? DB : 4;     // row slots per area (>= 4: NQ KiB of floats fit)
  constexpr int AREA = DS * NQ * kChunk;  // bytes per ring area
  constexpr int KW = (DB * NQ + kWaves - 1) / kWaves;  // LDS-DMA instructions per wave and group
  constexpr int SW = store_instrs<C, F32>();
  constexpr int LW = raw_words<T>();      // table loads per lane when a unit is loaded ahead
  constexpr int ELEM = F32 ? 4 : 1;
  constexpr int NX = 4 * NQ;              // source bytes per thread and row
  constexpr int GW = (1 + DB) * E;        // schedule words per group

  const int tid = threadIdx.x;
  const int lane = tid & (kLanes - 1);
  const int wave = RFL(tid >> 6);
  const int G = gridDim.x;
  int ucur = RFL(xcd_remap(blockIdx.x, G));
  if (ucur >= nunits) return;  // the whole workgroup
  const int nmine = (nunits - ucur + G - 1) / G;  // units of this workgroup's stream
  int kdone = 0;                                  // of them finished (progress priority)
  kint* unit_img = uniform_ptr<kint*>(unit_img_p);
#if MXD_BAND_STAMPS
  unsigned long long seg[kStampSegs] = {};
  const unsigned long long t_real0 = __builtin_amdgcn_s_memrealtime();
  MXD_STAMP(t_setup0);
#endif

  // A unit's horizontal lanes: thread = one output pixel of the strip row
  // (pixels in contiguous runs per wave, so each wave's stores are one
  // contiguous run).  Issues the LW table loads of the lane's pixel.
  using u32x4v = u32x4;
  auto lane_loads = [&](int npx, int ox0, int xs, cgfloat* xtab, int crop_w, int flip, u32x4v (&raw)[LW],
                        int* scol) {
    const int ppw = ((npx + kWaves - 1) / kWaves + MXD_BAND_PPW_ALIGN - 1) / MXD_BAND_PPW_ALIGN * MXD_BAND_PPW_ALIGN;
    const int px = wave * ppw + lane;
    const bool hact = lane < ppw && px < npx;
    const int ox = ox0 + min(px, max(npx, 1) - 1);
    const int xc = flip ? crop_w - 1 - ox : ox;
    const __amdgpu_buffer_rsrc_t xt =
        __builtin_amdgcn_make_buffer_rsrc(uniform_ptr<void*>((const void*)xtab), (short)0, crop_w * xs * 4, 0x00020000);
#pragma unroll
    for (int i = 0; i < LW; i++) raw[i] = __builtin_amdgcn_raw_buffer_load_b128(xt, xc * xs * 4 + 16 * i, 0, 0);
    *scol = hact ? (ox0 + px) * C * ELEM : kNoLoad;
  };
  auto unpack = [&](const u32x4v (&raw)[LW], int vboff, Lanes<T>& L) {
    float w[4 * LW];
#pragma unroll
    for (int i = 0; i < LW; i++) {
      // every loaded word stays live until here: a dead one's register would
      // be reused while its load is in flight, which costs a wait at the load
      asm volatile("" ::"v"(raw[i]));
      w[4 * i] = __uint_as_float(raw[i].x);
      w[4 * i + 1] = __uint_as_float(raw[i].y);
      w[4 * i + 2] = __uint_as_float(raw[i].z);
      w[4 * i + 3] = __uint_as_float(raw[i].w);
    }
    L.vb = __float_as_int(w[0]) * C + vboff;
#pragma unroll
    for (int k = 0; k < T; k++) L.wx[k] = w[kTapHeader + k];  // zero padded past the tap count
  };

  // Current unit c (horizontal and vertical passes; its groups are steps
  // [cstart, cstart + c.ng) of the stream) and the next one n (loaded ahead
  // when the LDS-DMA cursor reaches it).
  Unit c, n;
  Lanes<T> cl;
  u32x4v nraw[LW];
  int nscol = kNoLoad;
  {
    int npx, ox0, xs, crop_w, flip;
    cgfloat* xtab;
    c = load_unit<C, F32>(imgs, unit_img, per_img, ucur, nunits, &npx, &ox0, &xs, &xtab, &crop_w, &flip);
    u32x4v raw[LW];
    lane_loads(npx, ox0, xs, xtab, crop_w, flip, raw, &cl.scol);
    __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0): table loads done before the ring starts counting
    unpack(raw, c.vboff, cl);
  }
  n = c;
  n.ng = 0;

  const int rg = la + 1;
  const uint32_t sink = (uint32_t)(rg * AREA);  // 1 KiB for loads of absent rows

  // LDS-DMA of a group's rows into area a: item i = wave + 4 m is row slot
  // i / NQ, 1-KiB piece i % NQ; lane = 16 bytes of the piece.
  auto dma_rows = [&](const Unit& U, int l, int (&dr)[KW]) {
    static_for<KW>([&](auto mc) {
      constexpr int m = decltype(mc)::value;
      const int j = (wave + kWaves * m) / NQ;
      dr[m] = (j < DB && l < U.ng) ? U.sched[l * GW + (1 + j) * E] : -1;
    });
  };
  auto issue = [&](const Unit& U, const int (&dr)[KW], int a) {
    static_for<KW>([&](auto mc) {
      constexpr int m = decltype(mc)::value;
      const int i = wave + kWaves * m;
      const int j = i / NQ, k = i - (i / NQ) * NQ;
      const int row = dr[m];
      const int cb = U.b0 + kChunk * k + 16 * lane;
      const int voff = (row >= 0 && cb < U.bend && !(MXD_BAND_ABLATE & 1)) ? (row - U.y0) * U.stride + cb : kNoLoad;
      const uint32_t to = row >= 0 ? (uint32_t)(a * AREA + (j * NQ + k) * kChunk) : sink;
      __builtin_amdgcn_raw_ptr_buffer_load_lds(U.src, (lds_u8*)(smem + to), 16, voff, 0, 0, MXD_BAND_LOAD_AUX);
    });
  };

  // acc[s] = open output row (oldest + s); a completed row leaves slot 0 and
  // the slots shift down.
  float acc[S][NX];
#pragma unroll
  for (int s = 0; s < S; s++)
#pragma unroll
    for (int i = 0; i < NX; i++) acc[s][i] = 0.0f;

  // Vertical pass of one group (entries eg) from area a: thread t converts
  // dwords t, t + 256, ... of each row slot.  Row slots and their schedule
  // entries are read in batches of up to 4 before any use, and
  // (MXD_BAND_BRANCHLESS) every slot is converted and FMA'd into every
  // accumulator unconditionally: absent rows and unused slots carry weight 0,
  // and fma(0, x, acc) == acc for the finite x a byte converts to (a zero may
  // change sign, which the encode cannot see), so the batch is one branch-free
  // block the compiler can schedule.
  auto vpass = [&](kint* eg, int a) {
    constexpr int JB = DB < 4 ? DB : 4;
    const uint32_t* rb = reinterpret_cast<const uint32_t*>(smem + a * AREA);
    static_for<(DB + JB - 1) / JB>([&](auto bc) {
      constexpr int j0 = decltype(bc)::value * JB;
      constexpr int JN = DB - j0 < JB ? DB - j0 : JB;
      int ev[JN * E];
#pragma unroll
      for (int q = 0; q < JN * E; q++) ev[q] = eg[j0 * E + q];
      uint32_t d[JN][NQ];
#pragma unroll
      for (int j = 0; j < JN; j++)
#pragma unroll
        for (int k = 0; k < NQ; k++) d[j][k] = rb[((j0 + j) * NQ + k) * (kChunk / 4) + tid];
      static_for<JN>([&](auto jc) {
        constexpr int j = decltype(jc)::value;
        const int* e = ev + j * E;
        if (MXD_BAND_BRANCHLESS || e[0] >= 0) {
          if constexpr ((MXD_BAND_ABLATE & 8) != 0) {
            acc[0][0] += __uint_as_float(d[j][0] & 0x3fffffffu);
            return;
          }
          float x[NX];
#pragma unroll
          for (int i = 0; i < NX; i++) x[i] = (float)((d[j][i >> 2] >> (8 * (i & 3))) & 0xffu);
          static_for<S>([&](auto sc) {
            constexpr int s = decltype(sc)::value;
            const float w = __int_as_float(e[1 + s]);
            if (MXD_BAND_BRANCHLESS || s == 0 || w != 0.0f) {
#pragma unroll
              for (int i = 0; i < NX; i++) acc[s][i] = __builtin_fmaf(w, x[i], acc[s][i]);
            }
          });
        }
      });
    });
  };

  // Completed vertical row (slot 0) -> area a as f32 in byte order, then the
  // slots shift.  The stores are inline asm: hipcc would otherwise wait
  // vmcnt(0) before them (an LDS store after in-flight LDS-DMA it cannot prove
  // disjoint), which drains the ring; the areas in flight are never this one.
  auto vwrite = [&](int a) {
    const uint32_t addr = (uint32_t)(uintptr_t)(smem + a * AREA) + 16u * tid;
#pragma unroll
    for (int k = 0; k < NQ; k++) {
      const f32x4 v = {acc[0][4 * k], acc[0][4 * k + 1], acc[0][4 * k + 2], acc[0][4 * k + 3]};
      asm volatile("ds_write_b128 %0, %1" ::"v"(addr + (uint32_t)(k * kChunk * 4)), "v"(v) : "memory");
    }
#pragma unroll
    for (int s = 0; s + 1 < S; s++)
#pragma unroll
      for (int i = 0; i < NX; i++) acc[s][i] = acc[s + 1][i];
#pragma unroll
    for (int i = 0; i < NX; i++) acc[S - 1][i] = 0.0f;
  };

  // Horizontal pass of output row y of the current unit from the vertical
  // row in area a.
  auto hpass = [&](int a, int y) {
    const float* vf = reinterpret_cast<const float*>(smem + a * AREA) + cl.vb;
    float q[C];
#pragma unroll
    for (int ch = 0; ch < C; ch++) {
      float h = 0.0f;
      if constexpr ((MXD_BAND_ABLATE & 4) != 0) {
        h = vf[ch];
      } else {
#pragma unroll
        for (int k = 0; k < T; k++) h = __builtin_fmaf(cl.wx[k], vf[k * C + ch], h);
      }
      q[ch] = encode(h);
    }
    store_pixel<C, F32>(c.dst, cl.scol != kNoLoad && !(MXD_BAND_ABLATE & 2) ? y * c.dstride + cl.scol : kNoLoad, q);
  };

  for (int g = 0; g < la; g++) {
    int dr[KW];
    dma_rows(c, g, dr);
    issue(c, dr, g);
  }
  int acur = 0, aprev = rg - 1;  // areas of groups t and t - 1
  int cstart = 0;                // stream step of the current unit's group 0
  int vrows = 0;                 // output rows the vertical pass completed in its unit
  int hrow = -1;                 // output row the next step's horizontal pass writes (-1: none)
  int tx_loads = -(1 << 20);     // step that loaded a unit's tables ahead (its LW loads)
#if MXD_BAND_STAMPS
  MXD_STAMP(t_loop0);
  MXD_SEG(0, t_setup0, t_loop0);
#endif
  for (int t = 0;; t++) {
    const int cend = cstart + c.ng;
    const int tcross = cend - la;  // the step whose LDS-DMA starts the next unit
    if ((t & 7) == 0) band_prio(kdone * c.ng + t - cstart, nmine * c.ng);
    int npx = 0, ox0 = 0, xs = 0, crop_w = 0, flip = 0;
    cgfloat* xtab = nullptr;
    if (t == tcross)
      n = load_unit<C, F32>(imgs, unit_img, per_img, ucur + G, nunits, &npx, &ox0, &xs, &xtab, &crop_w, &flip);
    const int gd = t + la;  // the group this step's LDS-DMA brings
    const bool dcur = gd < cend;
    int dr[KW];
    if (dcur)
      dma_rows(c, gd - cstart, dr);
    else
      dma_rows(n, gd - cend, dr);
    // Vector-memory ops this wave issued after group t's LDS-DMA: the DMA of
    // the la - 1 groups after it, the stores of the steps since, and a
    // unit's table loads issued in those steps.
    MXD_STAMP(ta);
    wait_vmcnt((la - 1) * KW + SW * min(t, la - 1) + (tx_loads > t - la && tx_loads < t ? LW : 0));
    MXD_STAMP(tb);
    barrier_lds();  // group t's rows and the previous step's vertical row visible
    MXD_STAMP(tc);
    if (hrow >= 0) {
      hpass(aprev, c.oy0 + hrow);
    } else {
      const float z[C] = {};
      store_pixel<C, F32>(c.dst, kNoLoad, z);  // every step issues SW stores (the counts above)
    }
    MXD_STAMP(td);
    const bool vcur = t < cend;  // else: group 0 of the next unit
    kint* vg = vcur ? c.sched + (t - cstart) * GW : n.sched;
    const bool vany = vcur || n.ng > 0;
    int flags = 0;
    if (vany) {
      flags = vg[0];
      vpass(vg + E, acur);
    }
    MXD_STAMP(te);
    barrier_lds();  // area acur's rows and area aprev's vertical row consumed
    MXD_STAMP(tf);
    const bool done = (flags & kBandRowDone) != 0;
    if (done) vwrite(acur);
    const int vr = vcur ? vrows : 0;
    hrow = done ? vr : -1;
    vrows = vr + (done ? 1 : 0);
    if (t == tcross && n.ng > 0) {
      lane_loads(npx, ox0, xs, xtab, crop_w, flip, nraw, &nscol);
      tx_loads = t;
    }
    issue(dcur ? c : n, dr, aprev);  // group t + la: (t + la) mod (la + 1) == (t - 1) mod (la + 1)
#if MXD_BAND_STAMPS
    MXD_STAMP(tg);
    MXD_SEG(1, ta, tb);
    MXD_SEG(2, tb, tc);
    MXD_SEG(3, tc, td);
    MXD_SEG(4, td, te);
    MXD_SEG(5, te, tf);
    MXD_SEG(6, tf, tg);
    seg[7] += 1;
#endif
    aprev = acur;
    acur = acur + 1 == rg ? 0 : acur + 1;
    if (t >= cend) {
      // the current unit's last row went out this step: the next one takes over
      if (n.ng <= 0) break;
      c = n;
      cl.scol = nscol;
      unpack(nraw, c.vboff, cl);
      cstart = cend;
      ucur += G;
      kdone++;
      n.ng = 0;
    }
  }
  // no LDS-DMA may land after the workgroup's LDS is reassigned
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#if MXD_BAND_STAMPS
  seg[8] = t_real0;
  seg[9] = __builtin_amdgcn_s_memrealtime();
  const int sid = RFL(xcd_remap(blockIdx.x, G));
  if (wave == 0 && lane == 0 && sid < kMaxStamped)
    for (int k = 0; k < kStampSegs; k++) g_band_stamps[kStampSegs * sid + k] = seg[k];
#endif
}

using BandKernel = void (*)(const ImgDev*, const int*, int, int, int);

constexpr int kNumClasses = sizeof(kBandClasses) / sizeof(kBandClasses[0]);

int class_index(const BandCfg& cfg) {
  for (int i = 0; i < kNumClasses; i++)
    if (kBandClasses[i].taps == cfg.taps && kBandClasses[i].db == cfg.db && kBandClasses[i].s == cfg.s) return i;
  return -1;
}

// Variant / diagnostic builds may instantiate one class and window only
// (-DMXD_BAND_ONLY_CLASS=<index> -DMXD_BAND_ONLY_NQ=<KiB>, for fast A/B builds).
template <int CI, int NQ>
constexpr bool built() {
#if defined(MXD_BAND_ONLY_CLASS) && defined(MXD_BAND_ONLY_NQ)
  return CI == MXD_BAND_ONLY_CLASS && NQ == MXD_BAND_ONLY_NQ;
#else
  return true;
#endif
}

template <int C, bool F32, int NQ, int CI>
BandKernel class_kernel() {
  if constexpr (built<CI, NQ>())
    return resample_band<C, F32, NQ, kBandClasses[CI].taps, kBandClasses[CI].s, kBandClasses[CI].db>;
  else
    return nullptr;
}

template <int C, bool F32, int NQ, int... CI>
BandKernel pick_class(int ci, std::integer_sequence<int, CI...>) {
  BandKernel k = nullptr;
  ((ci == CI ? (k = class_kernel<C, F32, NQ, CI>(), 0) : 0), ...);
  return k;
}

template <int C, bool F32>
BandKernel pick_nq(int nq, int ci) {
  const auto seq = std::make_integer_sequence<int, kNumClasses>{};
  switch (nq) {
    case 1: return pick_class<C, F32, 1>(ci, seq);
    case 2: return pick_class<C, F32, 2>(ci, seq);
    case 3: return pick_class<C, F32, 3>(ci, seq);
    case 4: return pick_class<C, F32, 4>(ci, seq);
    default: return nullptr;
  }
}

// Kernels are built for RGB (what load_image produces for JPEG and the
// configurations measure); other channel counts take wave.hip / resample.hip.
BandKernel select_kernel(const BandCfg& cfg) {
  const int ci = class_index(cfg);
  if (ci < 0 || cfg.channels != 3 || cfg.la < 1) return nullptr;
  return cfg.f32 ? pick_nq<3, true>(cfg.nq, ci) : pick_nq<3, false>(cfg.nq, ci);
}

}  // namespace

int band_lds_bytes(const BandCfg& cfg) {
  const int ds = cfg.db > 4 ? cfg.db : 4;
  return (cfg.la + 1) * ds * cfg.nq * kChunk + kChunk;
}

bool band_has_kernel(const BandCfg& cfg) { return select_kernel(cfg) != nullptr; }

int band_capacity(const BandCfg& cfg, int device) {
  const BandKernel k = select_kernel(cfg);
  if (!k) return 0;
  int blocks = 0, cus = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&blocks, reinterpret_cast<const void*>(k), kThreads,
                                                   band_lds_bytes(cfg)) != hipSuccess)
    return 0;
  if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device) != hipSuccess) return 0;
  return blocks * cus;
}

int launch_band(const BandCfg& cfg, const ImgDev* imgs, const int32_t* unit_img, void* stream) {
  const BandKernel k = select_kernel(cfg);
  if (!k) return -2;
  if (cfg.grid < 1 || cfg.grid > cfg.nunits || (cfg.per_img <= 0 && !unit_img)) return -3;
  hipLaunchKernelGGL(k, dim3(cfg.grid), dim3(kThreads), band_lds_bytes(cfg), reinterpret_cast<hipStream_t>(stream),
                     imgs, unit_img, cfg.nunits, cfg.per_img, cfg.la);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

}  // namespace mxd

#if MXD_BAND_STAMPS
// Copies the first n units' segment sums of the last stamped launch.
extern "C" int mxd_debug_band_stamps(unsigned long long* host, int n) {
  if (n > mxd::kMaxStamped) n = mxd::kMaxStamped;
  return hipMemcpyFromSymbol(host, HIP_SYMBOL(mxd::g_band_stamps),
                             sizeof(unsigned long long) * mxd::kStampSegs * n, 0, hipMemcpyDeviceToHost) == hipSuccess
             ? 0
             : -1;
}
#endif
