// tools/c2_floor.hip -- the floor of C2's access pattern on this box
// (diagnostic, not product; round 6).
//
// The product's C2 launch (resample_wave<3, 8, true, 8, 2, kScatter, 2, 4>,
// split pixel lanes) with its arithmetic removed: 256 images of 960 rows x
// 3840 B; 4,096 units = image x 8 bands x 2 strips, one 64-lane wave each, 8
// waves per 512-thread workgroup (2 per CU, one occupancy round), XCD-
// contiguous workgroup order as wave.hip's xcd_remap; per unit the band's
// ~109 source rows (its 28 output rows x 3.768 + the 8-tap halo), each row one
// 1,536-B window per wave read as two dwordx3 loads per lane over two
// contiguous 768-B halves, a 4-slot register ring (3 rows ahead); per output
// row a 1,344-B strip row of f32 stored as f32x3 per lane (2 per lane).  The
// same bytes as the kernel (547 MB read, 154 MB written per launch).
// Variants: source-load policy (default / nt), stores (nt / none), loads
// (on / none), and a light "V pass" (convert + 2 FMAs per byte) to see how
// much of the kernel's VALU the pattern hides.  Median of 7 x 20 launches
// over two alternating source / output sets.
//
//   hipcc --offload-arch=gfx950 -O3 tools/c2_floor.hip -o tools/c2_floor && tools/c2_floor
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CHECK(x)                                                    \
  do {                                                              \
    hipError_t e = (x);                                             \
    if (e != hipSuccess) {                                          \
      fprintf(stderr, "%s failed: %s\n", #x, hipGetErrorString(e)); \
      exit(1);                                                      \
    }                                                               \
  } while (0)

typedef unsigned u32x3 __attribute__((ext_vector_type(3)));
typedef float f32x3 __attribute__((ext_vector_type(3)));
using Rsrc = __amdgpu_buffer_rsrc_t;

constexpr int kImgs = 256, kRows = 960, kStride = 3840;
constexpr int kBands = 8, kStrips = 2, kOutRows = 224, kOutRowBytes = 224 * 12;
constexpr int kFy0 = 58, kFy1 = 902;                 // footprint rows [58, 902)
constexpr int kFx0 = 218 * 3;                        // footprint's first byte in a row
constexpr int kWin = 1536, kHalf = 768;              // bytes per wave row window, per half
constexpr int kStripStep = 422 * 3;                  // the second strip's window start (bytes)
constexpr int kWaves = 8, kUnits = kImgs * kBands * kStrips;

__device__ __forceinline__ int xcd_remap(int b, int n) {
  const int q = n >> 3, r = n & 7;
  const int xcd = b & 7, idx = b >> 3;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + idx;
}

typedef float f32x4 __attribute__((ext_vector_type(4)));

// STORES: 0 none, 1 f32x3 per pixel (the kernel's: 12 B per lane, 2 stores per
// strip row), 2 the same bytes as 16 B per lane (84 x 16 B per strip row: one
// full-wave and one 20-lane store)
// MAP (round 6, later): how units map to workgroups -- 0 the kernel's (a
// workgroup = 4 bands x 2 strips of one image, XCD-contiguous workgroups);
// 1 a workgroup = the 8 bands of one strip; 2 as 0 without the XCD remap;
// 3 a workgroup = one band x 2 strips of 4 consecutive images
// RING: register ring slots (rows loaded RING - 1 ahead; the kernel's 4)
// STRIDE: bytes between source rows (the 1280-pixel frame's 3,840; 2,560 =
// the 844-pixel footprint rows nearly back to back, a diagnostic layout)
template <int AUX, bool LOADS, int STORES, bool VALU, int MAP = 0, int RING = 4, int STRIDE = kStride>
__global__ __launch_bounds__(512, 2) void c2_floor(const unsigned char* __restrict__ src, float* __restrict__ out) {
  const int lane = threadIdx.x & 63;
  const int wg = MAP == 2 ? (int)blockIdx.x : xcd_remap(blockIdx.x, gridDim.x);
  const int unit = __builtin_amdgcn_readfirstlane(wg * kWaves + (threadIdx.x >> 6));
  if (unit >= kUnits) return;
  int img = unit / (kBands * kStrips), rest = unit % (kBands * kStrips);
  int band = rest / kStrips, strip = rest % kStrips;
  if constexpr (MAP == 1) {
    strip = rest / kBands;
    band = rest % kBands;
  } else if constexpr (MAP == 3) {
    // workgroup w: images 4 (w / 4) .. + 3, band w % 4 * 2 + (wave >> 2 & 1)?  simpler:
    // unit u -> group of 64 units = 4 images x 8 bands x 2 strips, band-major
    const int grp = unit / 64, r = unit % 64;
    band = r / 8;
    img = grp * 4 + (r % 8) / 2;
    strip = r % 2;
  }
  const Rsrc r = __builtin_amdgcn_make_buffer_rsrc((void*)(src + (size_t)img * kRows * STRIDE), (short)0,
                                                   kRows * STRIDE, 0x00020000);
  const int w0 = (STRIDE == kStride ? kFx0 : 0) + strip * kStripStep;
  const int v0 = w0 + 12 * lane, v1 = w0 + kHalf + 12 * lane;
  const int oy0 = band * (kOutRows / kBands), oy1 = oy0 + kOutRows / kBands;
  const int r0 = kFy0 + (int)(oy0 * 3.768f), r1 = min(kFy1, kFy0 + (int)(oy1 * 3.768f) + 4);
  float* orow0 = out + ((size_t)img * kOutRows) * (kOutRowBytes / 4) + strip * (kOutRowBytes / 8);
  constexpr int R = RING;
  u32x3 ring[R][2];
  auto load = [&](int row, u32x3 (&d)[2]) {
    if constexpr (LOADS) {
      d[0] = __builtin_amdgcn_raw_buffer_load_b96(r, v0 + row * STRIDE, 0, AUX);
      d[1] = __builtin_amdgcn_raw_buffer_load_b96(r, v1 + row * STRIDE, 0, AUX);
    } else {
      d[0] = u32x3{(unsigned)row, 0u, 0u};
      d[1] = d[0];
    }
  };
#pragma unroll
  for (int d = 0; d < R - 1; d++) load(min(r0 + d, r1 - 1), ring[d]);
  float acc[2][12] = {};
  int oy = oy0;
  for (int row = r0; row < r1; row += R) {
#pragma unroll
    for (int d = 0; d < R; d++) {
      load(min(row + d + R - 1, r1 - 1), ring[(d + R - 1) % R]);
      const u32x3* x = ring[d];
      if constexpr (VALU) {
#pragma unroll
        for (int h = 0; h < 2; h++)
#pragma unroll
          for (int i = 0; i < 12; i++) {
            const float f = (float)((x[h][i >> 2] >> (8 * (i & 3))) & 255u);
            acc[h][i] = __builtin_fmaf(f, 0.25f, acc[h][i]);
            acc[(h + 1) & 1][i] = __builtin_fmaf(f, 0.125f, acc[(h + 1) & 1][i]);
          }
      } else if constexpr (STORES == 0) {
        // no stores: every loaded dword kept live by an xor (minimal VALU)
        const uint32_t k = x[0].x ^ x[0].y ^ x[0].z ^ x[1].x ^ x[1].y ^ x[1].z;
        acc[0][0] = __uint_as_float(__float_as_uint(acc[0][0]) ^ k);
      } else {
        acc[0][0] += (float)(x[0].x & 255u);
        acc[1][0] += (float)(x[1].y >> 24);
      }
      const int want = (int)((row + d - r0) / 3.768f) + oy0;
      if (want > oy && oy < oy1) {
        if constexpr (STORES == 1) {
          float* o = orow0 + (size_t)oy * (kOutRowBytes / 4);
#pragma unroll
          for (int q = 0; q < 2; q++) {
            const int px = lane + 64 * q;
            if (px < 112)
              __builtin_nontemporal_store(f32x3{acc[0][q], acc[1][q], acc[0][q + 2]},
                                          reinterpret_cast<f32x3*>(o + 3 * px));
          }
        } else if constexpr (STORES == 2) {
          float* o = orow0 + (size_t)oy * (kOutRowBytes / 4);
#pragma unroll
          for (int q = 0; q < 2; q++) {
            const int c = lane + 64 * q;  // 16-B chunk of the 1,344-B strip row
            if (c < 84)
              __builtin_nontemporal_store(f32x4{acc[0][q], acc[1][q], acc[0][q + 2], acc[1][q + 2]},
                                          reinterpret_cast<f32x4*>(o + 4 * c));
          }
        }
        oy++;
      }
    }
  }
  // keeps every accumulated byte live without storing (no-store variants)
  float t = 0.0f;
#pragma unroll
  for (int h = 0; h < 2; h++)
#pragma unroll
    for (int i = 0; i < 12; i++) t += acc[h][i];
  if (t == -1.0f) out[lane] = acc[1][1];
}

// The same units and rows, read as two b128 loads per lane (2 KiB per wave
// per row, 16 B per lane) instead of two b96 (1.5 KiB): is the load width
// part of the pattern's ceiling?  Minimal VALU, no stores; reports its own
// byte count.
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
__global__ __launch_bounds__(512, 2) void c2_read128(const unsigned char* __restrict__ src, float* __restrict__ out) {
  const int lane = threadIdx.x & 63;
  const int unit = __builtin_amdgcn_readfirstlane(xcd_remap(blockIdx.x, gridDim.x) * kWaves + (threadIdx.x >> 6));
  if (unit >= kUnits) return;
  const int img = unit / (kBands * kStrips), rest = unit % (kBands * kStrips);
  const int band = rest / kStrips, strip = rest % kStrips;
  const Rsrc r = __builtin_amdgcn_make_buffer_rsrc((void*)(src + (size_t)img * kRows * kStride), (short)0,
                                                   kRows * kStride, 0x00020000);
  const int v0 = (kFx0 & ~15) + strip * 1280 + 16 * lane, v1 = v0 + 1024;
  const int oy0 = band * (kOutRows / kBands), oy1 = oy0 + kOutRows / kBands;
  const int r0 = kFy0 + (int)(oy0 * 3.768f), r1 = min(kFy1, kFy0 + (int)(oy1 * 3.768f) + 4);
  constexpr int R = 4;
  u32x4 ring[R][2];
  auto load = [&](int row, u32x4 (&d)[2]) {
    d[0] = __builtin_amdgcn_raw_buffer_load_b128(r, v0 + row * kStride, 0, 2);
    d[1] = __builtin_amdgcn_raw_buffer_load_b128(r, v1 + row * kStride, 0, 2);
  };
#pragma unroll
  for (int d = 0; d < R - 1; d++) load(min(r0 + d, r1 - 1), ring[d]);
  uint32_t k = 0;
  for (int row = r0; row < r1; row += R) {
#pragma unroll
    for (int d = 0; d < R; d++) {
      load(min(row + d + R - 1, r1 - 1), ring[(d + R - 1) % R]);
      const u32x4* x = ring[d];
      k ^= x[0].x ^ x[0].y ^ x[0].z ^ x[0].w ^ x[1].x ^ x[1].y ^ x[1].z ^ x[1].w;
    }
  }
  if (k == 0x12345678u) out[lane] = 1.0f;
}

// The kernel's bytes (1.5 KiB per wave-row, two strips) read as one b128
// (the first KiB, 16 B per lane) and one b64 (the last 512 B, 8 B per lane)
// per lane instead of two b96 halves: a byte-order lane layout's loads.
typedef unsigned u32x2 __attribute__((ext_vector_type(2)));
template <bool FULL = false>  // FULL: + the V-pass stand-in and the f32 output stores
__global__ __launch_bounds__(512, 2) void c2_read_b128_b64(const unsigned char* __restrict__ src, float* __restrict__ out) {
  const int lane = threadIdx.x & 63;
  const int unit = __builtin_amdgcn_readfirstlane(xcd_remap(blockIdx.x, gridDim.x) * kWaves + (threadIdx.x >> 6));
  if (unit >= kUnits) return;
  const int img = unit / (kBands * kStrips), rest = unit % (kBands * kStrips);
  const int band = rest / kStrips, strip = rest % kStrips;
  const Rsrc r = __builtin_amdgcn_make_buffer_rsrc((void*)(src + (size_t)img * kRows * kStride), (short)0,
                                                   kRows * kStride, 0x00020000);
  const int w0 = ((kFx0 + strip * kStripStep) & ~15);
  const int v0 = w0 + 16 * lane, v1 = w0 + 1024 + 8 * lane;
  const int oy0 = band * (kOutRows / kBands), oy1 = oy0 + kOutRows / kBands;
  const int r0 = kFy0 + (int)(oy0 * 3.768f), r1 = min(kFy1, kFy0 + (int)(oy1 * 3.768f) + 4);
  constexpr int R = 4;
  u32x4 a[R];
  u32x2 b[R];
  auto load = [&](int row, int slot) {
    a[slot] = __builtin_amdgcn_raw_buffer_load_b128(r, v0 + row * kStride, 0, 2);
    b[slot] = __builtin_amdgcn_raw_buffer_load_b64(r, v1 + row * kStride, 0, 2);
  };
#pragma unroll
  for (int d = 0; d < R - 1; d++) load(min(r0 + d, r1 - 1), d);
  uint32_t k = 0;
  float acc[2][12] = {};
  int oy = oy0;
  float* orow0 = out + ((size_t)img * kOutRows) * (kOutRowBytes / 4) + strip * (kOutRowBytes / 8);
  for (int row = r0; row < r1; row += R) {
#pragma unroll
    for (int d = 0; d < R; d++) {
      load(min(row + d + R - 1, r1 - 1), (d + R - 1) % R);
      if constexpr (FULL) {
        const uint32_t w[6] = {a[d].x, a[d].y, a[d].z, a[d].w, b[d].x, b[d].y};
#pragma unroll
        for (int i = 0; i < 24; i++) {
          const float f = (float)((w[i >> 2] >> (8 * (i & 3))) & 255u);
          acc[i / 12][i % 12] = __builtin_fmaf(f, 0.25f, acc[i / 12][i % 12]);
          acc[(i / 12 + 1) & 1][i % 12] = __builtin_fmaf(f, 0.125f, acc[(i / 12 + 1) & 1][i % 12]);
        }
        const int want = (int)((row + d - r0) / 3.768f) + oy0;
        if (want > oy && oy < oy1) {
          float* o = orow0 + (size_t)oy * (kOutRowBytes / 4);
#pragma unroll
          for (int q = 0; q < 2; q++) {
            const int px = lane + 64 * q;
            if (px < 112)
              __builtin_nontemporal_store(f32x3{acc[0][q], acc[1][q], acc[0][q + 2]}, reinterpret_cast<f32x3*>(o + 3 * px));
          }
          oy++;
        }
      } else {
        k ^= a[d].x ^ a[d].y ^ a[d].z ^ a[d].w ^ b[d].x ^ b[d].y;
      }
    }
  }
  float t = 0.0f;
#pragma unroll
  for (int h = 0; h < 2; h++)
#pragma unroll
    for (int i = 0; i < 12; i++) t += acc[h][i];
  if (k == 0x12345678u || t == -1.0f) out[lane] = 1.0f;
}

template <class K>
static float time_us(K kernel, unsigned char** src, float** out, int iters = 20, int reps = 7) {
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  const unsigned blocks = kUnits / kWaves;
  for (int i = 0; i < 4; i++) hipLaunchKernelGGL(kernel, dim3(blocks), dim3(512), 0, 0, src[i & 1], out[i & 1]);
  std::vector<float> t;
  for (int r = 0; r < reps; r++) {
    CHECK(hipEventRecord(e0));
    for (int i = 0; i < iters; i++) hipLaunchKernelGGL(kernel, dim3(blocks), dim3(512), 0, 0, src[i & 1], out[i & 1]);
    CHECK(hipEventRecord(e1));
    CHECK(hipEventSynchronize(e1));
    float ms;
    CHECK(hipEventElapsedTime(&ms, e0, e1));
    t.push_back(ms * 1000.0f / iters);
  }
  std::sort(t.begin(), t.end());
  return t[t.size() / 2];
}

int main(int argc, char** argv) {
  unsigned char* src[2];
  float* out[2];
  const size_t sb = (size_t)kImgs * kRows * kStride, ob = (size_t)kImgs * kOutRows * kOutRowBytes;
  for (int i = 0; i < 2; i++) {
    CHECK(hipMalloc(&src[i], sb));
    CHECK(hipMalloc(&out[i], ob));
    CHECK(hipMemset(src[i], 7 + i, sb));
  }
  CHECK(hipDeviceSynchronize());
  const double alg = 256.0 * (844.0 * 844 * 3 + 224.0 * 224 * 3 * 4);
  auto report = [&](const char* name, float us) {
    printf("{\"probe\": \"%s\", \"us\": %.1f, \"alg_TBps\": %.3f, \"frac_of_8TBps\": %.3f}\n", name, us,
           alg / (us * 1e-6) / 1e12, alg / (us * 1e-6) / 8e12);
    fflush(stdout);
  };
  const bool only16 = argc > 1 && argv[1][0] == 's';  // round 6, later: the store-width A/B only
  if (argc > 1 && argv[1][0] == 'w') {  // round 6, later: load widths for the kernel's 1.5-KiB wave-rows
    for (int round = 0; round < 3; round++) {
      report("2 x b96 (the kernel's), loads only (xor)", time_us(c2_floor<2, true, 0, false, 0, 4, 3840>, src, out));
      report("b128 + b64, loads only (xor)", time_us(c2_read_b128_b64<false>, src, out));
      report("2 x b96 + V-pass + stores (the kernel's floor)", time_us(c2_floor<2, true, 1, true, 0, 4, 3840>, src, out));
      report("b128 + b64 + V-pass + stores", time_us(c2_read_b128_b64<true>, src, out));
    }
    return 0;
  }
  if (argc > 1 && argv[1][0] == 'l') {  // round 6, later: the read pattern with minimal VALU
    for (int round = 0; round < 2; round++) {
      {
        const float us = time_us(c2_read128, src, out);  // (2 KiB wave-rows)
        // rows per unit as the kernel computes them, 2 KiB per wave per row
        double bytes = 0;
        for (int b = 0; b < kBands; b++) {
          const int oy0 = b * (kOutRows / kBands), oy1 = oy0 + kOutRows / kBands;
          const int r0 = kFy0 + (int)(oy0 * 3.768f), r1 = std::min(kFy1, kFy0 + (int)(oy1 * 3.768f) + 4);
          bytes += (double)(r1 - r0) * 2048.0 * kStrips * kImgs;
        }
        printf("{\"probe\": \"b128 loads, 2 KiB per wave-row (xor)\", \"us\": %.1f, \"read_TBps\": %.3f}\n", us,
               bytes / (us * 1e-6) / 1e12);
        double b96 = bytes * 1536.0 / 2048.0;
        printf("{\"probe\": \"(b96 pattern's bytes for comparison)\", \"bytes\": %.0f}\n", b96);
        fflush(stdout);
      }
      report("loads only (xor, minimal VALU)", time_us(c2_floor<2, true, 0, false, 0, 4, 3840>, src, out));
      report("loads + V-pass VALU", time_us(c2_floor<2, true, 0, true, 0, 4, 3840>, src, out));
      report("loads only (xor), footprint-row stride", time_us(c2_floor<2, true, 0, false, 0, 4, 2560>, src, out));
    }
    return 0;
  }
  if (argc > 1 && argv[1][0] == 'p') {  // round 6, later: row stride (DRAM page use), loads only
    for (int round = 0; round < 2; round++) {
      report("stride 3840 (frame), loads + VALU", time_us(c2_floor<2, true, 0, true, 0, 4, 3840>, src, out));
      report("stride 2560 (footprint rows), loads + VALU", time_us(c2_floor<2, true, 0, true, 0, 4, 2560>, src, out));
      report("stride 3840 (frame), loads + stores + VALU", time_us(c2_floor<2, true, 1, true, 0, 4, 3840>, src, out));
      report("stride 2560 (footprint rows), loads + stores + VALU", time_us(c2_floor<2, true, 1, true, 0, 4, 2560>, src, out));
    }
    return 0;
  }
  if (argc > 1 && argv[1][0] == 'r') {  // round 6, later: rows in flight per wave, loads only
    for (int round = 0; round < 2; round++) {
      report("ring 2, loads + VALU", time_us(c2_floor<2, true, 0, true, 0, 2>, src, out));
      report("ring 4 (kernel's), loads + VALU", time_us(c2_floor<2, true, 0, true, 0, 4>, src, out));
      report("ring 6, loads + VALU", time_us(c2_floor<2, true, 0, true, 0, 6>, src, out));
      report("ring 8, loads + VALU", time_us(c2_floor<2, true, 0, true, 0, 8>, src, out));
      report("ring 8, loads + stores + VALU", time_us(c2_floor<2, true, 1, true, 0, 8>, src, out));
      report("ring 4, loads + stores + VALU", time_us(c2_floor<2, true, 1, true, 0, 4>, src, out));
    }
    return 0;
  }
  if (argc > 1 && argv[1][0] == 'm') {  // round 6, later: unit -> workgroup maps, loads only
    for (int round = 0; round < 2; round++) {
      report("map 0 (kernel's), loads + VALU", time_us(c2_floor<2, true, 0, true, 0>, src, out));
      report("map 1 (strip-major WG), loads + VALU", time_us(c2_floor<2, true, 0, true, 1>, src, out));
      report("map 2 (no XCD remap), loads + VALU", time_us(c2_floor<2, true, 0, true, 2>, src, out));
      report("map 3 (4 images per band group), loads + VALU", time_us(c2_floor<2, true, 0, true, 3>, src, out));
      report("map 1, loads + stores + VALU", time_us(c2_floor<2, true, 1, true, 1>, src, out));
      report("map 3, loads + stores + VALU", time_us(c2_floor<2, true, 1, true, 3>, src, out));
      report("map 0, loads + stores + VALU", time_us(c2_floor<2, true, 1, true, 0>, src, out));
    }
    return 0;
  }
  for (int round = 0; round < 2; round++) {
    if (!only16) {
      report("nt loads + nt stores", time_us(c2_floor<2, true, 1, false>, src, out));
      report("default loads + nt stores", time_us(c2_floor<0, true, 1, false>, src, out));
      report("nt loads, no stores", time_us(c2_floor<2, true, 0, false>, src, out));
      report("no loads, nt stores", time_us(c2_floor<2, false, 1, false>, src, out));
      report("nt loads + nt stores + V-pass VALU", time_us(c2_floor<2, true, 1, true>, src, out));
    }
    report("nt loads + V-pass VALU, no stores", time_us(c2_floor<2, true, 0, true>, src, out));
    report("default loads + V-pass VALU, no stores", time_us(c2_floor<0, true, 0, true>, src, out));
    report("no loads, nt stores 12 B / lane", time_us(c2_floor<2, false, 1, false>, src, out));
    report("no loads, nt stores 16 B / lane", time_us(c2_floor<2, false, 2, false>, src, out));
    report("nt loads + nt stores 12 B / lane + V-pass VALU", time_us(c2_floor<2, true, 1, true>, src, out));
    report("nt loads + nt stores 16 B / lane + V-pass VALU", time_us(c2_floor<2, true, 2, true>, src, out));
  }
  return 0;
}
