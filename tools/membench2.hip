// tools/membench2.hip -- HBM ceilings on this box (diagnostic, not product).
//
//  copy / read / write sweeps over 1 GiB buffers (16 B per lane), grid-stride
//  and one-chunk-per-block forms, plain and nontemporal; then the C2 access
//  mix: 256 images of 960 x 3840 B, each reading its 844-row x 2532-B source
//  footprint and writing 224 rows x 2688 B of f32 output, with one wave per
//  (image, band) reading whole footprint rows (3 x 1 KiB dwordx4 loads) or
//  three waves per row (one 1 KiB strip each).
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <functional>

#define CHECK(x)                                                    \
  do {                                                              \
    hipError_t e = (x);                                             \
    if (e != hipSuccess) {                                          \
      fprintf(stderr, "%s failed: %s\n", #x, hipGetErrorString(e)); \
      exit(1);                                                      \
    }                                                               \
  } while (0)

typedef float f4 __attribute__((ext_vector_type(4)));
typedef float f32x3 __attribute__((ext_vector_type(3)));
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
using Rsrc = __amdgpu_buffer_rsrc_t;

template <int U, bool NT>
__global__ __launch_bounds__(256) void copy_gs(const f4* __restrict__ a, f4* __restrict__ b, size_t n) {
  const size_t step = (size_t)gridDim.x * 256 * U;
  for (size_t i = (size_t)blockIdx.x * 256 * U + threadIdx.x; i + 256 * (U - 1) < n; i += step) {
    f4 v[U];
#pragma unroll
    for (int u = 0; u < U; u++) v[u] = NT ? __builtin_nontemporal_load(&a[i + 256 * u]) : a[i + 256 * u];
#pragma unroll
    for (int u = 0; u < U; u++) {
      if (NT) __builtin_nontemporal_store(v[u], &b[i + 256 * u]);
      else b[i + 256 * u] = v[u];
    }
  }
}

template <int U, bool NT>
__global__ __launch_bounds__(256) void copy_flat(const f4* __restrict__ a, f4* __restrict__ b) {
  const size_t i = (size_t)blockIdx.x * 256 * U + threadIdx.x;
  f4 v[U];
#pragma unroll
  for (int u = 0; u < U; u++) v[u] = NT ? __builtin_nontemporal_load(&a[i + 256 * u]) : a[i + 256 * u];
#pragma unroll
  for (int u = 0; u < U; u++) {
    if (NT) __builtin_nontemporal_store(v[u], &b[i + 256 * u]);
    else b[i + 256 * u] = v[u];
  }
}

template <int U>
__global__ __launch_bounds__(256) void read_gs(const f4* __restrict__ a, f4* __restrict__ out, size_t n) {
  const size_t step = (size_t)gridDim.x * 256 * U;
  float acc = 0.0f;
  for (size_t i = (size_t)blockIdx.x * 256 * U + threadIdx.x; i + 256 * (U - 1) < n; i += step) {
    f4 v[U];
#pragma unroll
    for (int u = 0; u < U; u++) v[u] = a[i + 256 * u];
#pragma unroll
    for (int u = 0; u < U; u++) acc += v[u].x + v[u].y + v[u].z + v[u].w;
  }
  if (acc == 1234.5f) out[threadIdx.x] = f4{acc, acc, acc, acc};
}

template <int U>
__global__ __launch_bounds__(256) void write_gs(f4* __restrict__ b, size_t n) {
  const size_t step = (size_t)gridDim.x * 256 * U;
  const float f = (float)threadIdx.x;
  for (size_t i = (size_t)blockIdx.x * 256 * U + threadIdx.x; i + 256 * (U - 1) < n; i += step) {
#pragma unroll
    for (int u = 0; u < U; u++) b[i + 256 * u] = f4{f, f, f, (float)u};
  }
}

// ---- C2 access mix ----
constexpr int kRows = 960, kStride = 3840, kImgs = 256;
constexpr int kFy0 = 56, kFy1 = 900, kFb0 = 640, kNeed = 2532;  // footprint rows / bytes
constexpr int kOutRows = 224, kOutRow = 2688;                      // f32 output row bytes
constexpr int kNoLoad = 0x7ffffff0;

// One wave per (image, band): NW dwordx4 loads per lane cover NW KiB of each
// footprint row (whole row: NW = 3), DEPTH rows in flight; every time the
// running row count crosses an output-row boundary (3.768 rows per output
// row) the wave stores one output row's share (row bytes / strips).
template <int NW, int DEPTH>
__global__ __launch_bounds__(256) void c2_mix(const uint8_t* __restrict__ base, float* __restrict__ out, int nbands,
                                              int strips, int write) {
  const int nunits_all = kImgs * nbands * strips;
  const int lane = threadIdx.x & 63;
  const int unit = __builtin_amdgcn_readfirstlane(blockIdx.x * 4 + (threadIdx.x >> 6));
  const int per_img = nbands * strips;
  if (unit >= kImgs * per_img) return;
  const int img = unit / per_img;
  const int rest = unit - img * per_img;
  const int band = rest / strips, strip = rest - band * strips;
  const uint8_t* p = base + (size_t)img * kRows * kStride;
  const Rsrc r = __builtin_amdgcn_make_buffer_rsrc((void*)p, (short)0, kRows * kStride, 0x00020000);
  const int swidth = (kNeed + strips - 1) / strips;
  int off[NW];
#pragma unroll
  for (int j = 0; j < NW; j++) {
    const int b = 16 * lane + 1024 * j;
    off[j] = b < swidth && write != 5 ? kFb0 + strip * swidth + b : kNoLoad;
  }
  const int oy0 = band * kOutRows / nbands, oy1 = (band + 1) * kOutRows / nbands;
  const int r0 = kFy0 + (int)(oy0 * 3.768f), r1 = min(kFy1, kFy0 + (int)(oy1 * 3.768f) + 4);
  const int orow_share = kOutRow / strips;  // bytes
  float* o = out + ((size_t)img * kOutRows) * (kOutRow / 4) + strip * (orow_share / 4);
  u32x4 ring[DEPTH][NW];
#pragma unroll
  for (int d = 0; d < DEPTH; d++)
#pragma unroll
    for (int j = 0; j < NW; j++)
      ring[d][j] = __builtin_amdgcn_raw_buffer_load_b128(r, off[j], min(r0 + d, r1 - 1) * kStride, 0);
  float acc[4] = {0, 0, 0, 0};
  int oy = oy0;
  for (int row = r0; row < r1; row += DEPTH) {
#pragma unroll
    for (int d = 0; d < DEPTH; d++) {
#pragma unroll
      for (int j = 0; j < NW; j++) {
        acc[0] += (float)(ring[d][j].x & 255);
        acc[1] += (float)(ring[d][j].y >> 24);
        acc[2] += (float)(ring[d][j].z & 255);
        acc[3] += (float)(ring[d][j].w >> 24);
        ring[d][j] = __builtin_amdgcn_raw_buffer_load_b128(r, off[j], min(row + d + DEPTH, r1 - 1) * kStride, 0);
      }
      const int want = (int)((row + d - r0) / 3.768f) + oy0;
      if (write && want > oy && oy < oy1) {
        const f4 v = {acc[0], acc[1], acc[2], acc[3]};
        if (write == 1 || write == 5) {
          f4* orow = reinterpret_cast<f4*>(o + (size_t)oy * (kOutRow / 4));
          for (int b = lane; b < orow_share / 16; b += 64) orow[b] = v;
        } else if (write == 2) {
          f4* orow = reinterpret_cast<f4*>(out) + ((size_t)(oy - oy0) * nunits_all + unit) * (orow_share / 16);
          for (int b = lane; b < orow_share / 16; b += 64) orow[b] = v;
        } else if (write == 3) {
          f4* orow = reinterpret_cast<f4*>(o + (size_t)oy * (kOutRow / 4));
          for (int b = lane; b < orow_share / 16; b += 64) __builtin_nontemporal_store(v, &orow[b]);
        } else if (write == 4 && ((oy - oy0) & 3) == 3) {
          f4* orow = reinterpret_cast<f4*>(o + (size_t)(oy - 3) * (kOutRow / 4));
          for (int b = lane; b < 4 * orow_share / 16; b += 64) orow[b] = v;
        }
        oy++;
      }
    }
  }
  if (acc[0] == -1.0f) out[lane] = acc[1];
}


// Kernel-shaped mix: unit = (image, band, strip); the strip reads a window of
// `wb` bytes (LB bytes per lane: 12 = dwordx3, 16 = dwordx4) at step `step`,
// the band reads its rows plus `halo` rows; every 3.768 rows it stores one
// strip-row of `ob` bytes (SB bytes per lane) at out + row*2688 + strip*ob.
template <int LB, int SB, int DEPTH>
__global__ __launch_bounds__(256) void c2_kmix(const uint8_t* __restrict__ base, float* __restrict__ out, int nbands,
                                               int strips, int wb, int step, int ob, int halo, int write) {
  typedef unsigned uv __attribute__((ext_vector_type(LB / 4)));
  const int lane = threadIdx.x & 63;
  const int unit = __builtin_amdgcn_readfirstlane(blockIdx.x * 4 + (threadIdx.x >> 6));
  const int per_img = nbands * strips;
  if (unit >= kImgs * per_img) return;
  const int img = unit / per_img;
  const int rest = unit - img * per_img;
  const int band = rest / strips, strip = rest - band * strips;
  const uint8_t* p = base + (size_t)img * kRows * kStride;
  const Rsrc r = __builtin_amdgcn_make_buffer_rsrc((void*)p, (short)0, kRows * kStride, 0x00020000);
  const int voff = LB * lane < wb ? kFb0 + strip * step + LB * lane : kNoLoad;
  const int oy0 = band * kOutRows / nbands, oy1 = (band + 1) * kOutRows / nbands;
  const int r0 = kFy0 + (int)(oy0 * 3.768f), r1 = min(kFy1, kFy0 + (int)(oy1 * 3.768f) + halo);
  char* o = reinterpret_cast<char*>(out) + (size_t)img * kOutRows * kOutRow + strip * ob;
  uv ring[DEPTH];
#pragma unroll
  for (int d = 0; d < DEPTH; d++) {
    if constexpr (LB == 12) ring[d] = __builtin_amdgcn_raw_buffer_load_b96(r, voff, min(r0 + d, r1 - 1) * kStride, 0);
    else ring[d] = __builtin_amdgcn_raw_buffer_load_b128(r, voff, min(r0 + d, r1 - 1) * kStride, 0);
  }
  float acc[4] = {0, 0, 0, 0};
  int oy = oy0;
  for (int row = r0; row < r1; row += DEPTH) {
#pragma unroll
    for (int d = 0; d < DEPTH; d++) {
      acc[0] += (float)(ring[d].x & 255);
      acc[1] += (float)(ring[d].y >> 24);
      acc[2] += (float)(ring[d].z & 255);
      if constexpr (LB == 12) ring[d] = __builtin_amdgcn_raw_buffer_load_b96(r, voff, min(row + d + DEPTH, r1 - 1) * kStride, 0);
      else ring[d] = __builtin_amdgcn_raw_buffer_load_b128(r, voff, min(row + d + DEPTH, r1 - 1) * kStride, 0);
      const int want = (int)((row + d - r0) / 3.768f) + oy0;
      if (write == 1 && want > oy && oy < oy1) {
        char* orow = o + (size_t)oy * kOutRow;
        for (int b = lane; b * SB < ob; b += 64) {
          if constexpr (SB == 12) *reinterpret_cast<f32x3*>(orow + 12 * b) = f32x3{acc[0], acc[1], acc[2]};
          else *reinterpret_cast<f4*>(orow + 16 * b) = f4{acc[0], acc[1], acc[2], acc[3]};
        }
        oy++;
      }
    }
  }
  // write == 2: the band's stores deferred until all its reads are done (a
  // single-round launch then reads chip-wide first and writes after)
  if (write == 2)
    for (oy = oy0; oy < oy1; oy++) {
      char* orow = o + (size_t)oy * kOutRow;
      for (int b = lane; b * SB < ob; b += 64) {
        if constexpr (SB == 12) *reinterpret_cast<f32x3*>(orow + 12 * b) = f32x3{acc[0], acc[1], acc[2]};
        else *reinterpret_cast<f4*>(orow + 16 * b) = f4{acc[0], acc[1], acc[2], acc[3]};
      }
    }
  if (acc[0] == -1.0f) out[lane] = acc[1];
}

// Lane-ownership probe (mode 'l'): unit = (image, band, strip) as in the wave
// kernel.  MODE 0: lane l owns 24 B at 24 l of a window starting 12-B aligned
// (the P = 8 RGB layout: one b128 + one b64 per lane and row, each instruction
// touching every line of the window).  MODE 1: lane l owns the 16 B at 16 l of
// a window aligned down to 16 B (one b128 per lane and row: 1 KiB contiguous
// per instruction).  Lanes past the strip's bytes issue no request.  Output
// strip rows of `ob` bytes, 12 B per lane, every 3.768 source rows.
template <int MODE, int DEPTH>
__global__ __launch_bounds__(256) void c2_lanes(const uint8_t* __restrict__ base, float* __restrict__ out, int nbands,
                                                int strips, int write) {
  constexpr int LB = MODE == 0 ? 24 : 16;
  const int lane = threadIdx.x & 63;
  const int unit = __builtin_amdgcn_readfirstlane(blockIdx.x * 4 + (threadIdx.x >> 6));
  const int per_img = nbands * strips;
  if (unit >= kImgs * per_img) return;
  const int img = unit / per_img;
  const int rest = unit - img * per_img;
  const int band = rest / strips, strip = rest - band * strips;
  const uint8_t* p = base + (size_t)img * kRows * kStride;
  const Rsrc r = __builtin_amdgcn_make_buffer_rsrc((void*)p, (short)0, kRows * kStride, 0x00020000);
  // strip window: output columns [224 s / strips, 224 (s+1) / strips) need
  // source pixels ~[x0 * 3.768 - 4, x1 * 3.768 + 4) of the footprint
  const int ox0 = 224 * strip / strips, ox1 = 224 * (strip + 1) / strips;
  const int px0 = max(0, (int)(ox0 * 3.768f) - 4), px1 = min(844, (int)(ox1 * 3.768f) + 4);
  int b0 = kFb0 + 3 * px0;
  b0 = MODE == 0 ? b0 - (b0 % 12) : b0 & ~15;
  const int wbytes = kFb0 + 3 * px1 - b0;
  const int voff = LB * lane < wbytes ? b0 + LB * lane : kNoLoad;
  const int oy0 = band * kOutRows / nbands, oy1 = (band + 1) * kOutRows / nbands;
  const int r0 = kFy0 + max(0, (int)(oy0 * 3.768f) - 4), r1 = min(kFy1, kFy0 + (int)(oy1 * 3.768f) + 4);
  const int ob = (ox1 - ox0) * 12;
  char* o = reinterpret_cast<char*>(out) + (size_t)img * kOutRows * kOutRow + ox0 * 12;
  u32x4 ra[DEPTH];
  unsigned rb[DEPTH][2];
  auto load = [&](int d, int row) {
    ra[d] = __builtin_amdgcn_raw_buffer_load_b128(r, voff, row * kStride, 0);
    if constexpr (MODE == 0) {
      typedef unsigned u2 __attribute__((ext_vector_type(2)));
      const u2 v = __builtin_amdgcn_raw_buffer_load_b64(r, voff + 16, row * kStride, 0);
      rb[d][0] = v.x, rb[d][1] = v.y;
    }
  };
#pragma unroll
  for (int d = 0; d < DEPTH; d++) load(d, min(r0 + d, r1 - 1));
  float acc[4] = {0, 0, 0, 0};
  int oy = oy0;
  for (int row = r0; row < r1; row += DEPTH) {
#pragma unroll
    for (int d = 0; d < DEPTH; d++) {
      acc[0] += (float)(ra[d].x & 255);
      acc[1] += (float)(ra[d].y >> 24);
      acc[2] += (float)(ra[d].z & 255) + (float)(ra[d].w >> 24);
      if constexpr (MODE == 0) acc[3] += (float)(rb[d][0] & 255) + (float)(rb[d][1] >> 24);
      load(d, min(row + d + DEPTH, r1 - 1));
      const int want = (int)((row + d - r0) / 3.768f) + oy0;
      if (write && want > oy && oy < oy1) {
        char* orow = o + (size_t)oy * kOutRow;
        for (int b = lane; b * 12 < ob; b += 64)
          *reinterpret_cast<f32x3*>(orow + 12 * b) = f32x3{acc[0], acc[1], acc[2] + acc[3]};
        oy++;
      }
    }
  }
  if (acc[0] == -1.0f) out[lane] = acc[1];
}

int g_iter = 0;  // launches alternate source / output buffers on g_iter's parity


// Workgroup = (image, band): wave w reads strip w's window (LB bytes per lane,
// strips x wb bytes at step `step`); every K output rows the workgroup writes
// the K full output rows (K x 2688 B, contiguous) with 16 B per lane, between
// two barriers (the K-row burst a workgroup-staged kernel would produce).
template <int K, int DEPTH>
__global__ __launch_bounds__(256) void c2_wgmix(const uint8_t* __restrict__ base, float* __restrict__ out, int nbands,
                                                int wb, int step, int halo, int write) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int unit = blockIdx.x;
  if (unit >= kImgs * nbands) return;
  const int img = unit / nbands, band = unit - img * nbands;
  const uint8_t* p = base + (size_t)img * kRows * kStride;
  const Rsrc r = __builtin_amdgcn_make_buffer_rsrc((void*)p, (short)0, kRows * kStride, 0x00020000);
  const int voff = 12 * lane < wb ? kFb0 + wave * step + 12 * lane : kNoLoad;
  const int oy0 = band * kOutRows / nbands, oy1 = (band + 1) * kOutRows / nbands;
  const int r0 = kFy0 + (int)(oy0 * 3.768f), r1 = min(kFy1, kFy0 + (int)(oy1 * 3.768f) + halo);
  char* o = reinterpret_cast<char*>(out) + (size_t)img * kOutRows * kOutRow;
  typedef unsigned uv __attribute__((ext_vector_type(3)));
  uv ring[DEPTH];
#pragma unroll
  for (int d = 0; d < DEPTH; d++) ring[d] = __builtin_amdgcn_raw_buffer_load_b96(r, voff, min(r0 + d, r1 - 1) * kStride, 0);
  float acc[4] = {0, 0, 0, 0};
  int oy = oy0, pend = 0;
  for (int row = r0; row < r1; row += DEPTH) {
#pragma unroll
    for (int d = 0; d < DEPTH; d++) {
      acc[0] += (float)(ring[d].x & 255);
      acc[1] += (float)(ring[d].y >> 24);
      acc[2] += (float)(ring[d].z & 255);
      ring[d] = __builtin_amdgcn_raw_buffer_load_b96(r, voff, min(row + d + DEPTH, r1 - 1) * kStride, 0);
      const int want = (int)((row + d - r0) / 3.768f) + oy0;
      if (want > oy && oy < oy1) {
        oy++;
        if (++pend == K || oy == oy1) {
          if (write) {
            __syncthreads();
            f4* dst = reinterpret_cast<f4*>(o + (size_t)(oy - pend) * kOutRow);
            for (int b = threadIdx.x; b < pend * kOutRow / 16; b += 256) dst[b] = f4{acc[0], acc[1], acc[2], acc[3]};
            __syncthreads();
          }
          pend = 0;
        }
      }
    }
  }
  if (acc[0] == -1.0f) out[lane] = acc[1];
}

int g_iter_dummy;

// DRAM mix probes (one workgroup per chunk of consecutive "rows"):
//   mode 0: read `rb` bytes of each of `nrows` rows spaced `rstride` apart,
//           write 2688 B to a sequential output every `ratio` rows.
template <int U>
__global__ __launch_bounds__(256) void mixprobe(const uint8_t* __restrict__ base, f4* __restrict__ out, int nrows,
                                                int rstride, int rb, float ratio, int rows_per_block, int write) {
  const int r0 = blockIdx.x * rows_per_block;
  const int r1 = min(r0 + rows_per_block, nrows);
  float acc = 0.0f;
  int wrote = (int)(r0 / ratio);
  for (int r = r0; r < r1; r += U) {
    u32x4 v[U];
#pragma unroll
    for (int u = 0; u < U; u++) {
      const int rr = min(r + u, nrows - 1);
      const int off = 16 * threadIdx.x;
      v[u] = off < rb ? *reinterpret_cast<const u32x4*>(base + (size_t)rr * rstride + off) : u32x4{0, 0, 0, 0};
    }
#pragma unroll
    for (int u = 0; u < U; u++) acc += (float)(v[u].x & 255) + (float)(v[u].w >> 24);
    const int want = (int)((r + U) / ratio);
    if (write) {
      for (; wrote < want; wrote++) {
        f4* o = out + (size_t)wrote * (2688 / 16);
        if (threadIdx.x < 2688 / 16) o[threadIdx.x] = f4{acc, acc, acc, acc};
      }
    }
  }
  if (acc == -1.0f) out[0] = f4{acc, acc, acc, acc};
}

double timeit(const char* name, double bytes, std::function<void()> f) {
  hipEvent_t a, b;
  CHECK(hipEventCreate(&a));
  CHECK(hipEventCreate(&b));
  for (int w = 0; w < 3; w++, g_iter++) f();
  CHECK(hipEventRecord(a));
  const int iters = 20;
  for (int i = 0; i < iters; i++, g_iter++) f();
  CHECK(hipEventRecord(b));
  CHECK(hipEventSynchronize(b));
  CHECK(hipGetLastError());
  float ms;
  CHECK(hipEventElapsedTime(&ms, a, b));
  const double us = ms / iters * 1e3;
  printf("%-46s %9.1f us  %7.1f GB/s\n", name, us, bytes / (us * 1e-6) / 1e9);
  fflush(stdout);
  return us;
}

int main(int argc, char** argv) {
  const bool only_c2 = argc > 1;
  const size_t bytes = (size_t)1 << 30, n = bytes / 16;
  f4 *a, *b;
  CHECK(hipMalloc(&a, bytes));
  CHECK(hipMalloc(&b, bytes));
  CHECK(hipMemset(a, 1, bytes));
  CHECK(hipMemset(b, 2, bytes));
  char name[128];
  for (int k : {2, 4, 8, 16, 32}) {
    if (only_c2) break;
    const int g = 256 * k;
    snprintf(name, sizeof name, "copy gs U=1 blocks=%d", g);
    timeit(name, 2.0 * bytes, [&] { copy_gs<1, false><<<g, 256>>>(a, b, n); });
    snprintf(name, sizeof name, "copy gs U=4 blocks=%d", g);
    timeit(name, 2.0 * bytes, [&] { copy_gs<4, false><<<g, 256>>>(a, b, n); });
    snprintf(name, sizeof name, "copy gs U=4 nt blocks=%d", g);
    timeit(name, 2.0 * bytes, [&] { copy_gs<4, true><<<g, 256>>>(a, b, n); });
  }
  if (!only_c2) {
  timeit("copy flat U=1", 2.0 * bytes, [&] { copy_flat<1, false><<<n / 256, 256>>>(a, b); });
  timeit("copy flat U=4", 2.0 * bytes, [&] { copy_flat<4, false><<<n / 1024, 256>>>(a, b); });
  timeit("copy flat U=8", 2.0 * bytes, [&] { copy_flat<8, false><<<n / 2048, 256>>>(a, b); });
  timeit("copy flat U=4 nt", 2.0 * bytes, [&] { copy_flat<4, true><<<n / 1024, 256>>>(a, b); });
  timeit("hipMemcpyDtoD", 2.0 * bytes, [&] { CHECK(hipMemcpyAsync(b, a, bytes, hipMemcpyDeviceToDevice, 0)); });
  for (int k : {4, 8, 16}) {
    snprintf(name, sizeof name, "read gs U=4 blocks=%d", 256 * k);
    timeit(name, 1.0 * bytes, [&] { read_gs<4><<<256 * k, 256>>>(a, b, n); });
    snprintf(name, sizeof name, "read gs U=8 blocks=%d", 256 * k);
    timeit(name, 1.0 * bytes, [&] { read_gs<8><<<256 * k, 256>>>(a, b, n); });
    snprintf(name, sizeof name, "write gs U=4 blocks=%d", 256 * k);
    timeit(name, 1.0 * bytes, [&] { write_gs<4><<<256 * k, 256>>>(b, n); });
  }
  }

  if (argc > 1 && argv[1][0] == 'm') {
    uint8_t* src2;
    f4* out2;
    CHECK(hipMalloc(&src2, bytes));
    CHECK(hipMalloc(&out2, bytes));
    const uint8_t* srcs[2] = {reinterpret_cast<const uint8_t*>(a), src2};
    f4* outs[2] = {b, out2};
    const int nrows = 256 * 844;  // C2 footprint rows
    struct V { const char* n; int rstride, rb; };
    const V vs[] = {{"contiguous 2560B rows", 2560, 2560}, {"2560B of 3840B rows", 3840, 2560},
                    {"full 3840B rows", 3840, 3840}};
    for (const V& v : vs)
      for (int write : {0, 1})
        for (int rpb : {16, 64}) {
          snprintf(name, sizeof name, "%s rows/block=%d write=%d", v.n, rpb, write);
          const double by = (double)nrows * v.rb + write * (double)nrows / 3.768 * 2688;
          timeit(name, by, [&] {
            mixprobe<4><<<(nrows + rpb - 1) / rpb, 256>>>(srcs[g_iter & 1], outs[g_iter & 1], nrows, v.rstride, v.rb,
                                                          3.768f, rpb, write);
          });
        }
    return 0;
  }
  if (argc > 1 && argv[1][0] == 'l') {
    uint8_t* src2;
    float* out2;
    CHECK(hipMalloc(&src2, bytes));
    CHECK(hipMalloc(&out2, bytes));
    CHECK(hipMemset(src2, 3, bytes));
    const uint8_t* srcs[2] = {reinterpret_cast<const uint8_t*>(a), src2};
    float* outs[2] = {reinterpret_cast<float*>(b), out2};
    const double rd = (double)kImgs * (kFy1 - kFy0) * kNeed, wr = (double)kImgs * kOutRows * kOutRow;
    struct V { const char* n; int mode, ns, nb; };
    const V vs[] = {{"24B lanes (P=8 now) 2 strips x 8 bands", 0, 2, 8},
                    {"16B lanes aligned 3 strips x 5 bands", 1, 3, 5},
                    {"16B lanes aligned 3 strips x 6 bands", 1, 3, 6},
                    {"16B lanes aligned 3 strips x 10 bands", 1, 3, 10},
                    {"16B lanes aligned 4 strips x 4 bands", 1, 4, 4},
                    {"24B lanes (P=8 now) 2 strips x 8 bands (again)", 0, 2, 8}};
    for (const V& v : vs)
      for (int write : {0, 1}) {
        const int units = kImgs * v.nb * v.ns;
        snprintf(name, sizeof name, "%s w=%d", v.n, write);
        timeit(name, rd + (write ? wr : 0), [&] {
          const uint8_t* src = srcs[g_iter & 1];
          float* out = outs[g_iter & 1];
          if (v.mode == 0) c2_lanes<0, 6><<<(units + 3) / 4, 256>>>(src, out, v.nb, v.ns, write);
          else c2_lanes<1, 6><<<(units + 3) / 4, 256>>>(src, out, v.nb, v.ns, write);
        });
      }
    return 0;
  }
  if (argc > 1 && argv[1][0] == 'k') {
    // two source sets and two output sets, alternating (no Infinity Cache reuse between launches)
    uint8_t *src2;
    float* out2;
    CHECK(hipMalloc(&src2, bytes));
    CHECK(hipMalloc(&out2, bytes));
    CHECK(hipMemset(src2, 3, bytes));
    const uint8_t* srcs[2] = {reinterpret_cast<const uint8_t*>(a), src2};
    float* outs[2] = {reinterpret_cast<float*>(b), out2};
    const double rd = (double)kImgs * (kFy1 - kFy0) * kNeed, wr = (double)kImgs * kOutRows * kOutRow;
    struct V { const char* n; int lb, sb, nb, ns, wb, step, ob, halo; };
    const V vs[] = {
      {"1 strip (whole 2532B rows) x4 bands", 16, 16, 4, 1, 2532, 0, 2688, 4},
      {"2 strips 1266B x4 bands", 16, 16, 4, 2, 1280, 1266, 1344, 4},
      {"kernel-like 4x4 x3/x3 768B 672B halo4", 12, 12, 4, 4, 768, 633, 672, 4},
      {"4x4 x3 loads, 672B x4-less? (x3) halo0", 12, 12, 4, 4, 768, 633, 672, 0},
      {"4x4 window 633B (no overlap)", 12, 12, 4, 4, 633, 633, 672, 4},
      {"4x4 x4 loads 768B", 16, 12, 4, 4, 768, 633, 672, 4},
      {"4x4 stores x4 672B", 12, 16, 4, 4, 768, 633, 672, 4},
      {"3x4 strips 896B out, 1KiB window", 16, 16, 4, 3, 1024, 844, 896, 4},
      {"3x4 strips 896B out, 844B window", 16, 16, 4, 3, 844, 844, 896, 0},
      {"4x8 bands", 12, 12, 8, 4, 768, 633, 672, 4},
      {"4x2 bands", 12, 12, 2, 4, 768, 633, 672, 4},
    };
    const bool defer_only = argv[1][1] == 'd';
    for (int k : {1, 4, 8, 16}) {
      if (defer_only) break;
      for (int nb : {4, 8}) {
        snprintf(name, sizeof name, "wg burst K=%d nb=%d (4 strips, full-row writes)", k, nb);
        auto go = [&] {
          const uint8_t* src = srcs[g_iter & 1];
          float* out = outs[g_iter & 1];
          if (k == 1) c2_wgmix<1, 8><<<kImgs * nb, 256>>>(src, out, nb, 768, 633, 4, 1);
          if (k == 4) c2_wgmix<4, 8><<<kImgs * nb, 256>>>(src, out, nb, 768, 633, 4, 1);
          if (k == 8) c2_wgmix<8, 8><<<kImgs * nb, 256>>>(src, out, nb, 768, 633, 4, 1);
          if (k == 16) c2_wgmix<16, 8><<<kImgs * nb, 256>>>(src, out, nb, 768, 633, 4, 1);
        };
        timeit(name, rd + wr, go);
      }
    }
    for (const V& v : vs) {
      if (v.wb > 1024) continue;
      for (int write : {0, 1, 2}) {
        if (defer_only && write == 0) continue;
        const int units = kImgs * v.nb * v.ns;
        snprintf(name, sizeof name, "%s w=%d", v.n, write);
        auto go = [&] {
          const uint8_t* src = srcs[g_iter & 1];
          float* out = outs[g_iter & 1];
          if (v.lb == 12 && v.sb == 12) c2_kmix<12, 12, 8><<<(units + 3) / 4, 256>>>(src, out, v.nb, v.ns, v.wb, v.step, v.ob, v.halo, write);
          else if (v.lb == 16 && v.sb == 12) c2_kmix<16, 12, 8><<<(units + 3) / 4, 256>>>(src, out, v.nb, v.ns, v.wb, v.step, v.ob, v.halo, write);
          else if (v.lb == 12 && v.sb == 16) c2_kmix<12, 16, 8><<<(units + 3) / 4, 256>>>(src, out, v.nb, v.ns, v.wb, v.step, v.ob, v.halo, write);
          else c2_kmix<16, 16, 8><<<(units + 3) / 4, 256>>>(src, out, v.nb, v.ns, v.wb, v.step, v.ob, v.halo, write);
        };
        timeit(name, rd + (write ? wr : 0), go);
      }
    }
    return 0;
  }
  // C2 mix: sources in `a` (256 x 3.69 MB = 944 MB), outputs in `b`.
  const uint8_t* src = reinterpret_cast<const uint8_t*>(a);
  float* out = reinterpret_cast<float*>(b);
  const double rd = (double)kImgs * (kFy1 - kFy0) * kNeed, wr = (double)kImgs * kOutRows * kOutRow;
  const char* wname[] = {"none", "nhwc", "interleaved", "nt", "burst4", "write-only"};
  for (int write : {0, 1, 2, 3, 4, 5}) {
    for (int nb : {4, 8}) {
      const int units = kImgs * nb;
      const double by = (write == 5 ? 0 : rd) + (write ? wr : 0);
      snprintf(name, sizeof name, "c2 row-wave nb=%d d=8 %s", nb, wname[write]);
      timeit(name, by, [&] { c2_mix<3, 8><<<(units + 3) / 4, 256>>>(src, out, nb, 1, write); });
      snprintf(name, sizeof name, "c2 strip-wave nb=%d d=8 %s", nb, wname[write]);
      timeit(name, by, [&] { c2_mix<1, 8><<<(units * 3 + 3) / 4, 256>>>(src, out, nb, 3, write); });
    }
  }
  return 0;
}
