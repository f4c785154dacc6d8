// tools/inflight_probe.hip -- diagnostic (not product): does the number of
// source rows a wave keeps in flight bound the C2 kernel's access pattern?
//
// The C2 pattern of resample_wave (wave.hip): 256 images of 960 rows x 3840 B
// (1280x960 RGB), one wave per unit = (image, band of output rows, strip),
// 2 strips, each strip reading a 1284-byte window of every footprint row as
// two 768-byte halves (P = 8 split lanes: one dwordx3 per lane per half),
// converting the 24 bytes of a lane to f32 and FMA-ing them into two open
// rows of accumulators (48 floats, packed FMAs), and every 3.768 source rows
// storing one f32 strip row (112 pixels x 12 B, nontemporal f32x3 stores).
// No horizontal pass: the probe isolates the row stream.
//
// Two ways to keep D rows in flight per wave:
//   reg  a register ring of D rows (what the product kernel does, D = 4),
//   lds  a wave-private LDS ring of D slots filled by LDS-DMA
//        (buffer_load_dwordx3 ... lds), no workgroup barrier: each wave waits
//        on its own vmcnt, then reads the slot back with ds_read_b96.
// Occupancy is pinned with dynamic LDS per workgroup (8 waves each), so the
// rows in flight per CU vary only with D.  Prints us per launch and GB/s of
// (footprint reads + f32 writes) for every (mode, D, workgroups per CU).
//
// Build: hipcc -O3 --offload-arch=gfx950 -std=c++17 tools/inflight_probe.hip -o /tmp/inflight_probe
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

typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef float f32x3 __attribute__((ext_vector_type(3)));
typedef unsigned u32x3 __attribute__((ext_vector_type(3)));
using Rsrc = __amdgpu_buffer_rsrc_t;
typedef __attribute__((address_space(3))) void lds_void;

constexpr int kNoLoad = 0x7ffffff0;
constexpr int kWaves = 8;
constexpr int kHalf = 768;  // bytes one dwordx3-per-lane wave instruction covers
constexpr int kSlot = 2 * kHalf;  // LDS bytes per ring slot (one row, two halves)

// Source / output geometry of one workload shape.
struct Geo {
  const char* name;
  int imgs, rows, stride;  // images of rows x stride bytes
  int fy0, fy1, fb0;       // footprint rows [fy0, fy1), first footprint byte
  int strips, win, step;   // strips per row, window bytes per strip (<= 2 kHalf), strip step bytes
  float ratio;             // source rows per output row
  int out_px, out_elem;    // output pixels per strip row, bytes per channel (4 f32, 1 u8)
  double bytes;            // algorithmic bytes per launch
};

__device__ __forceinline__ void wait_vm(int n) {
#define VMC(k)                                              \
  case k:                                                   \
    asm volatile("s_waitcnt vmcnt(" #k ")" ::: "memory"); \
    break;
  switch (n) {
    VMC(0) VMC(1) VMC(2) VMC(3) VMC(4) VMC(5) VMC(6) VMC(7) VMC(8) VMC(9) VMC(10) VMC(11) VMC(12) VMC(13) VMC(14)
    VMC(15) VMC(16) VMC(17) VMC(18) VMC(19) VMC(20) VMC(21) VMC(22) VMC(23) VMC(24) VMC(25) VMC(26) VMC(27) VMC(28)
    VMC(29) VMC(30) VMC(31)
    default: asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
#undef VMC
}

struct Row {
  unsigned d[6];
};

__device__ __forceinline__ void consume(const Row& r, float (&acc)[2][24], float w0, float w1) {
  float x[24];
#pragma unroll
  for (int i = 0; i < 24; i++) x[i] = (float)((r.d[i >> 2] >> (8 * (i & 3))) & 0xffu);
#pragma unroll
  for (int i = 0; i < 24; i += 2) {
    f32x2 a = {acc[0][i], acc[0][i + 1]}, b = {acc[1][i], acc[1][i + 1]};
    a = __builtin_elementwise_fma(f32x2{w0, w0}, f32x2{x[i], x[i + 1]}, a);
    b = __builtin_elementwise_fma(f32x2{w1, w1}, f32x2{x[i], x[i + 1]}, b);
    acc[0][i] = a.x, acc[0][i + 1] = a.y, acc[1][i] = b.x, acc[1][i + 1] = b.y;
  }
}

template <int MODE, int D>
__global__ __launch_bounds__(kWaves * 64) void probe(const uint8_t* __restrict__ base, float* __restrict__ out,
                                                     int nbands, Geo g) {
  const int kStrips = g.strips, kRows = g.rows, kStride = g.stride, kImgs = g.imgs, kFy0 = g.fy0, kFy1 = g.fy1;
  const int kOutRows = 224, kOutRow = 224 * 3 * g.out_elem;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int unit = __builtin_amdgcn_readfirstlane(blockIdx.x * kWaves + wave);
  const int per_img = nbands * kStrips;
  if (unit >= kImgs * per_img) return;
  const int img = unit / per_img;
  const int rest = unit - img * per_img;
  const int band = rest / kStrips, strip = rest - band * kStrips;
  const uint8_t* p = base + (size_t)img * kRows * kStride;
  const Rsrc rs = __builtin_amdgcn_make_buffer_rsrc((void*)p, (short)0, kRows * kStride, 0x00020000);
  const int b0 = g.fb0 + strip * g.step;
  const int va = 12 * lane < g.win ? b0 + 12 * lane : kNoLoad;
  const int vb = 12 * lane + kHalf < g.win ? b0 + kHalf + 12 * lane : kNoLoad;
  const int oy0 = band * kOutRows / nbands, oy1 = (band + 1) * kOutRows / nbands;
  const int r0 = kFy0 + (int)(oy0 * g.ratio), r1 = min(kFy1, kFy0 + (int)(oy1 * g.ratio) + 4);
  char* o = reinterpret_cast<char*>(out) + (size_t)img * kOutRows * kOutRow + strip * (g.out_px * 3 * g.out_elem);
  char* ring = smem + wave * (D * kSlot);  // MODE 1: this wave's slots
  float acc[2][24];
#pragma unroll
  for (int s = 0; s < 2; s++)
#pragma unroll
    for (int i = 0; i < 24; i++) acc[s][i] = 0.0f;
  Row reg[D];
  auto issue = [&](int slot, int row) {
    row = min(row, r1 - 1);
    if constexpr (MODE == 0) {
      const u32x3 a = __builtin_amdgcn_raw_buffer_load_b96(rs, va, row * kStride, 0);
      const u32x3 b = __builtin_amdgcn_raw_buffer_load_b96(rs, vb, row * kStride, 0);
      reg[slot].d[0] = a.x, reg[slot].d[1] = a.y, reg[slot].d[2] = a.z;
      reg[slot].d[3] = b.x, reg[slot].d[4] = b.y, reg[slot].d[5] = b.z;
    } else {
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (lds_void*)(ring + slot * kSlot), 12, va, row * kStride, 0, 0);
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (lds_void*)(ring + slot * kSlot + kHalf), 12, vb, row * kStride, 0, 0);
    }
  };
  auto fetch = [&](int slot) {
    if constexpr (MODE == 0) {
      return reg[slot];
    } else {
      Row r;
      const u32x3 a = *reinterpret_cast<const u32x3*>(ring + slot * kSlot + 12 * lane);
      const u32x3 b = *reinterpret_cast<const u32x3*>(ring + slot * kSlot + kHalf + 12 * lane);
      r.d[0] = a.x, r.d[1] = a.y, r.d[2] = a.z, r.d[3] = b.x, r.d[4] = b.y, r.d[5] = b.z;
      return r;
    }
  };
#pragma unroll
  for (int d = 0; d < D; d++) issue(d, r0 + d);
  int oy = oy0;
  for (int row = r0; row < r1; row += D) {
#pragma unroll
    for (int d = 0; d < D; d++) {
      if constexpr (MODE == 1) wait_vm(2 * (D - 1));  // this slot's two loads landed
      const Row r = fetch(d);
      if constexpr (MODE == 1) asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // read out before refilling
      issue(d, row + d + D);
      consume(r, acc, 0.25f, 0.125f);
      const int want = (int)((row + d - r0) / g.ratio) + oy0;
      if (want > oy && oy < oy1) {
        char* orow = o + (size_t)oy * kOutRow;
        float sum[3] = {0.0f, 0.0f, 0.0f};  // every accumulator feeds the stores (none is dead code)
#pragma unroll
        for (int i = 0; i < 24; i++) sum[i % 3] += acc[0][i];
#pragma unroll
        for (int q = 0; q < 4; q++) {
          const int px = lane + 64 * q;
          if (px < g.out_px) {
            if (g.out_elem == 4) {
              __builtin_nontemporal_store(f32x3{sum[0] + q, sum[1], sum[2]}, reinterpret_cast<f32x3*>(orow + 12 * px));
            } else {  // u8: three byte stores per pixel, like the product kernel
              orow[3 * px] = (char)sum[0], orow[3 * px + 1] = (char)sum[1], orow[3 * px + 2] = (char)(sum[2] + q);
            }
          }
        }
#pragma unroll
        for (int i = 0; i < 24; i++) acc[0][i] = acc[1][i], acc[1][i] = 0.0f;
        oy++;
      }
    }
  }
  if (MODE == 1) wait_vm(0);
  float t = 0.0f;
#pragma unroll
  for (int i = 0; i < 24; i++) t += acc[1][i];
  if (t == -1.0f) out[lane] = t;
}

int g_iter = 0;

double timeit(const char* name, double bytes, const std::function<void()>& f) {
  hipEvent_t a, b;
  CHECK(hipEventCreate(&a));
  CHECK(hipEventCreate(&b));
  for (int w = 0; w < 4; w++, g_iter++) f();
  const int iters = 40;
  CHECK(hipEventRecord(a));
  for (int i = 0; i < iters; i++, g_iter++) f();
  CHECK(hipEventRecord(b));
  CHECK(hipEventSynchronize(b));
  CHECK(hipGetLastError());
  float ms;
  CHECK(hipEventElapsedTime(&ms, a, b));
  const double us = ms / iters * 1e3;
  printf("%-58s %8.1f us  %7.1f GB/s\n", name, us, bytes / (us * 1e-6) / 1e9);
  fflush(stdout);
  return us;
}

template <int MODE, int D>
void run(const uint8_t* const* srcs, float* const* outs, const Geo& g, int cus) {
  const double bytes = g.bytes;
  const int kImgs = g.imgs, kStrips = g.strips;
  const int lds_need = MODE == 1 ? kWaves * D * kSlot : 0;
  for (int wgs : {1, 2, 3, 4}) {  // workgroups (of 8 waves) per CU
    const int lds = 160 * 1024 / wgs - 64;
    if (lds < lds_need) continue;
    auto k = probe<MODE, D>;
    int occ = 0;
    CHECK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, reinterpret_cast<const void*>(k), kWaves * 64, lds));
    if (occ < wgs) continue;  // registers allow fewer
    // units fill exactly one round of the resident waves (the product planner's rule)
    const int waves = wgs * kWaves * cus;
    int nbands = waves / (kImgs * kStrips);
    if (nbands < 1) nbands = 1;
    const int units = kImgs * kStrips * nbands;
    char name[128];
    snprintf(name, sizeof name, "%-12s %s D=%-2d %d WG/CU (%2d waves/CU) bands=%d", g.name, MODE ? "lds" : "reg", D,
             wgs, wgs * kWaves, nbands);
    CHECK(hipFuncSetAttribute(reinterpret_cast<const void*>(k), hipFuncAttributeMaxDynamicSharedMemorySize, lds));
    timeit(name, bytes, [&] {
      hipLaunchKernelGGL(k, dim3((units + kWaves - 1) / kWaves), dim3(kWaves * 64), lds, 0, srcs[g_iter & 1],
                         outs[g_iter & 1], nbands, g);
    });
  }
}

int main(int argc, char** argv) {
  // C2: 256 x 1280x960 -> 341x256 -> 224 f32: footprint 844 rows x 844 px,
  // two strips of 1284 B (P = 8 split lanes), 3.768 source rows per output row.
  const Geo c2{"c2", 256, 960, 3840, 56, 900, 640, 2, 1284, 1248, 3.768f, 112, 4,
               256.0 * (844.0 * 844 * 3 + 224.0 * 224 * 12)};
  // C3's 480p shape: 512 x 640x480 -> 341x256 -> 224 u8: footprint ~424 x 424 px,
  // narrow lanes (P = 4): two strips of 636 B; 1.875 source rows per output row.
  const Geo p480{"480p-2strip", 512, 480, 1920, 28, 452, 174, 2, 636, 636, 1.875f, 112, 1,
                 512.0 * (424.0 * 424 * 3 + 224.0 * 224 * 3)};
  // the same shape read as one 1272-B strip per row (wide lanes, 4 pixels per lane out)
  const Geo p480w{"480p-1strip", 512, 480, 1920, 28, 452, 174, 1, 1272, 0, 1.875f, 224, 1,
                  512.0 * (424.0 * 424 * 3 + 224.0 * 224 * 3)};
  const bool only480 = argc > 1 && argv[1][0] == '4';
  const size_t sbytes = (size_t)512 * 480 * 1920 > (size_t)256 * 960 * 3840 ? (size_t)512 * 480 * 1920
                                                                            : (size_t)256 * 960 * 3840;
  const size_t obytes = (size_t)256 * 224 * 224 * 12;
  uint8_t *s0, *s1;
  float *o0, *o1;
  CHECK(hipMalloc(&s0, sbytes));
  CHECK(hipMalloc(&s1, sbytes));
  CHECK(hipMalloc(&o0, obytes));
  CHECK(hipMalloc(&o1, obytes));
  CHECK(hipMemset(s0, 1, sbytes));
  CHECK(hipMemset(s1, 2, sbytes));
  int cus = 0;
  CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  const uint8_t* srcs[2] = {s0, s1};
  float* outs[2] = {o0, o1};
  printf("# %d CUs\n", cus);
  for (const Geo* g : {&p480, &p480w, &c2}) {
    if (only480 && g == &c2) continue;
    printf("# %s: algorithmic bytes per launch %.0f\n", g->name, g->bytes);
    run<0, 2>(srcs, outs, *g, cus);
    run<0, 3>(srcs, outs, *g, cus);
    run<0, 4>(srcs, outs, *g, cus);
    run<0, 6>(srcs, outs, *g, cus);
    run<0, 8>(srcs, outs, *g, cus);
    run<0, 12>(srcs, outs, *g, cus);
    run<1, 2>(srcs, outs, *g, cus);
    run<1, 4>(srcs, outs, *g, cus);
    run<1, 6>(srcs, outs, *g, cus);
    run<1, 8>(srcs, outs, *g, cus);
    run<1, 12>(srcs, outs, *g, cus);
    run<1, 16>(srcs, outs, *g, cus);
  }
  return 0;
}
