// tools/strip_probe.hip -- diagnostic (not product): how the length of the
// row piece each wave reads sets the rate of the resize kernels' access
// pattern, and whether a wave can give the DRAM whole rows while computing
// only its strip.
//
// Follows tools/inflight_probe.hip (whose finding: rows in flight per wave do
// not matter for C2's pattern, 147-153 us for any depth or ring kind) with the
// strip count as the variable: unit = (image, band, strip), one wave each, 8
// waves per workgroup, the strips of one band in adjacent waves; a strip row
// is NH dwordx3 loads per lane (768 B per instruction, lanes past the strip's
// window masked), converted and FMA'd into two open rows of accumulators, and
// every `ratio` source rows one output strip row is stored (f32x3
// nontemporal, or three byte stores per pixel for u8).
//
// PF (prefetch of the sibling strips): 0 = none; 1 = every wave also issues
// LDS-DMA loads of the WHOLE footprint row (into an 768-byte per-wave sink
// nobody reads) D rows ahead of its own register loads, so the DRAM sees one
// contiguous row request and the strips' own loads hit L2; 2 = only strip 0
// does.
//
// Build: hipcc -O3 --offload-arch=gfx950 -std=c++17 tools/strip_probe.hip -o tools/strip_probe
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
constexpr int kInst = 768;  // bytes of one dwordx3-per-lane wave instruction

struct Geo {
  const char* name;
  int imgs, rows, stride;   // images of rows x stride bytes
  int fy0, fy1, fb0, fw;    // footprint rows [fy0, fy1), footprint bytes [fb0, fb0 + fw)
  float ratio;              // source rows per output row
  int out_elem;             // 4: f32 output, 1: u8
  double bytes;             // algorithmic bytes per launch
};

// The product's blockIdx -> XCD-contiguous remap (csrc/devutil.h xcd_remap):
// XCD k runs a contiguous range of units, in dispatch order.
__device__ __forceinline__ int remap_xcd(int b, int n) {
  const int q = n >> 3, r = n & 7;
  const int xcd = b & 7, idx = b >> 3;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + idx;
}

template <int NH, int D, int PF>
__global__ __launch_bounds__(kWaves * 64) void probe(const uint8_t* __restrict__ base, char* __restrict__ out,
                                                     int nbands, int strips, Geo g, int remap) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int blk = remap ? remap_xcd(blockIdx.x, gridDim.x) : blockIdx.x;
  const int unit = __builtin_amdgcn_readfirstlane(blk * kWaves + wave);
  const int per_img = nbands * strips;
  if (unit >= g.imgs * per_img) return;
  const int img = unit / per_img;
  const int rest = unit - img * per_img;
  const int band = rest / strips, strip = rest - band * strips;
  const uint8_t* p = base + (size_t)img * g.rows * g.stride;
  const Rsrc rs = __builtin_amdgcn_make_buffer_rsrc((void*)p, (short)0, g.rows * g.stride, 0x00020000);
  // strip window: an equal share of the footprint plus a 24-byte halo, 4-byte aligned
  const int share = (g.fw + strips - 1) / strips;
  const int b0 = (g.fb0 + strip * share - (strip ? 24 : 0)) & ~3;
  const int b1 = min(g.fb0 + g.fw, g.fb0 + (strip + 1) * share + 24);
  const int win = b1 - b0;
  int voff[NH];
#pragma unroll
  for (int h = 0; h < NH; h++) voff[h] = kInst * h + 12 * lane < win ? b0 + kInst * h + 12 * lane : kNoLoad;
  // whole-row prefetch offsets (PF): 4 instructions cover up to 3 KiB
  int pf[4];
#pragma unroll
  for (int h = 0; h < 4; h++) pf[h] = kInst * h + 12 * lane < g.fw ? (g.fb0 & ~3) + kInst * h + 12 * lane : kNoLoad;
  const bool do_pf = PF == 1 || (PF == 2 && strip == 0);
  lds_void* sink = (lds_void*)(smem + wave * kInst);
  const int oy0 = band * 224 / nbands, oy1 = (band + 1) * 224 / nbands;
  const int r0 = g.fy0 + (int)(oy0 * g.ratio), r1 = min(g.fy1, g.fy0 + (int)(oy1 * g.ratio) + 4);
  const int out_px = (224 + strips - 1) / strips;
  const int orow_bytes = 224 * 3 * g.out_elem;
  char* o = out + (size_t)img * 224 * orow_bytes + strip * out_px * 3 * g.out_elem;
  float acc[2][12 * NH];
#pragma unroll
  for (int s = 0; s < 2; s++)
#pragma unroll
    for (int i = 0; i < 12 * NH; i++) acc[s][i] = 0.0f;
  unsigned ring[D][3 * NH];
  auto issue = [&](int slot, int row) {
    row = min(row, r1 - 1);
#pragma unroll
    for (int h = 0; h < NH; h++) {
      const u32x3 v = __builtin_amdgcn_raw_buffer_load_b96(rs, voff[h], row * g.stride, 0);
      ring[slot][3 * h] = v.x, ring[slot][3 * h + 1] = v.y, ring[slot][3 * h + 2] = v.z;
    }
  };
  auto prefetch = [&](int row) {
    if (!do_pf || row >= r1) return;
#pragma unroll
    for (int h = 0; h < 4; h++)
      if (kInst * h < g.fw) __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, sink, 12, pf[h], row * g.stride, 0, 0);
  };
#pragma unroll
  for (int d = 0; d < D; d++) prefetch(r0 + d);
#pragma unroll
  for (int d = 0; d < D; d++) issue(d, r0 + d);
  int oy = oy0;
  for (int row = r0; row < r1; row += D) {
#pragma unroll
    for (int d = 0; d < D; d++) {
      float x[12 * NH];
#pragma unroll
      for (int i = 0; i < 12 * NH; i++) x[i] = (float)((ring[d][i >> 2] >> (8 * (i & 3))) & 0xffu);
      prefetch(row + d + 2 * D);
      issue(d, row + d + D);
#pragma unroll
      for (int i = 0; i < 12 * NH; i += 2) {
        f32x2 a = {acc[0][i], acc[0][i + 1]}, b = {acc[1][i], acc[1][i + 1]};
        a = __builtin_elementwise_fma(f32x2{0.25f, 0.25f}, f32x2{x[i], x[i + 1]}, a);
        b = __builtin_elementwise_fma(f32x2{0.125f, 0.125f}, f32x2{x[i], x[i + 1]}, b);
        acc[0][i] = a.x, acc[0][i + 1] = a.y, acc[1][i] = b.x, acc[1][i + 1] = b.y;
      }
      const int want = (int)((row + d - r0) / g.ratio) + oy0;
      if (want > oy && oy < oy1) {
        char* orow = o + (size_t)oy * orow_bytes;
        float sum[3] = {0.0f, 0.0f, 0.0f};
#pragma unroll
        for (int i = 0; i < 12 * NH; i++) sum[i % 3] += acc[0][i];
        for (int px = lane; px < out_px; px += 64) {
          if (g.out_elem == 4) {
            __builtin_nontemporal_store(f32x3{sum[0] + px, sum[1], sum[2]}, reinterpret_cast<f32x3*>(orow + 12 * px));
          } else {
            orow[3 * px] = (char)sum[0], orow[3 * px + 1] = (char)sum[1], orow[3 * px + 2] = (char)(sum[2] + px);
          }
        }
#pragma unroll
        for (int i = 0; i < 12 * NH; i++) acc[0][i] = acc[1][i], acc[1][i] = 0.0f;
        oy++;
      }
    }
  }
  float t = 0.0f;
#pragma unroll
  for (int i = 0; i < 12 * NH; i++) t += acc[1][i];
  if (t == -1.0f) out[lane] = (char)t;
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
  printf("%-64s %8.1f us  %7.1f GB/s\n", name, us, bytes / (us * 1e-6) / 1e9);
  fflush(stdout);
  return us;
}

// rounds: band count multiplied so the units fill that many occupancy rounds
// (shorter bands, more of them: the "sweep" form, where the dispatcher starts
// each XCD's next units in address order as earlier ones finish).
template <int NH, int D, int PF>
void run(const uint8_t* const* srcs, char* const* outs, const Geo& g, int strips, int cus, int rounds = 1,
         int remap = 0) {
  auto k = probe<NH, D, PF>;
  const int lds = kWaves * kInst;
  int occ = 0;
  CHECK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, reinterpret_cast<const void*>(k), kWaves * 64, lds));
  // units fill one round of the resident waves (the product planner's rule)
  const int waves = occ * kWaves * cus;
  const int nbands = rounds * (waves / (g.imgs * strips) > 0 ? waves / (g.imgs * strips) : 1);
  const int units = g.imgs * strips * nbands;
  char name[160];
  snprintf(name, sizeof name, "%-6s strips=%d NH=%d D=%d PF=%d R=%d X=%d (%2d waves/CU, bands %d)", g.name, strips, NH,
           D, PF, rounds, remap, occ * kWaves, nbands);
  timeit(name, g.bytes, [&] {
    hipLaunchKernelGGL(k, dim3((units + kWaves - 1) / kWaves), dim3(kWaves * 64), lds, 0, srcs[g_iter & 1],
                       outs[g_iter & 1], nbands, strips, g, remap);
  });
}

int main() {
  // C2: 256 x 1280x960 -> 341x256 -> 224 f32 (footprint 844 rows x 2532 B)
  const Geo c2{"c2", 256, 960, 3840, 56, 900, 640, 2532, 3.768f, 4, 256.0 * (844.0 * 844 * 3 + 224.0 * 224 * 12)};
  // C3's 480p: 512 x 640x480 -> 341x256 -> 224 u8 (footprint ~424 rows x 1272 B)
  const Geo p480{"480p", 512, 480, 1920, 28, 452, 324, 1272, 1.875f, 1, 512.0 * (424.0 * 424 * 3 + 224.0 * 224 * 3)};
  // C3's 720p: 512 x 1280x720 -> 455x256 -> 224 u8 (footprint ~633 rows x 1899 B)
  const Geo p720{"720p", 512, 720, 3840, 43, 676, 1050, 1899, 2.812f, 1,
                 512.0 * (633.0 * 633 * 3 + 224.0 * 224 * 3)};
  const size_t sbytes = (size_t)512 * 720 * 3840, obytes = (size_t)256 * 224 * 224 * 12;
  uint8_t *s0, *s1;
  char *o0, *o1;
  CHECK(hipMalloc(&s0, sbytes));
  CHECK(hipMalloc(&s1, sbytes));
  CHECK(hipMalloc(&o0, obytes));
  CHECK(hipMalloc(&o1, obytes));
  CHECK(hipMemset(s0, 1, sbytes));
  CHECK(hipMemset(s1, 2, sbytes));
  int cus = 0;
  CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  const uint8_t* srcs[2] = {s0, s1};
  char* outs[2] = {o0, o1};
  printf("# %d CUs\n", cus);
  // Round 5: the sweep and sibling forms against the
  // one-round band layout, C2 and 480p.
  for (int rep = 0; rep < 2; rep++) {
    run<2, 4, 0>(srcs, outs, c2, 2, cus);
    run<2, 4, 0>(srcs, outs, c2, 2, cus, 1, 1);
    run<2, 4, 0>(srcs, outs, c2, 2, cus, 2, 1);
    run<2, 4, 0>(srcs, outs, c2, 2, cus, 4, 1);
    run<2, 4, 0>(srcs, outs, c2, 2, cus, 8, 1);
    run<2, 4, 0>(srcs, outs, c2, 2, cus, 4, 0);
    run<1, 4, 0>(srcs, outs, c2, 8, cus);        // sibling: a workgroup's 8 waves = the 8 strips of one band
    run<1, 4, 0>(srcs, outs, c2, 8, cus, 1, 1);
    run<1, 4, 0>(srcs, outs, c2, 8, cus, 4, 1);
    run<1, 4, 0>(srcs, outs, c2, 4, cus, 1, 1);
    run<1, 4, 0>(srcs, outs, p480, 2, cus);
    run<1, 4, 0>(srcs, outs, p480, 2, cus, 1, 1);
    run<1, 4, 0>(srcs, outs, p480, 2, cus, 4, 1);
    run<1, 4, 0>(srcs, outs, p480, 2, cus, 8, 1);
    run<1, 4, 0>(srcs, outs, p480, 4, cus, 1, 1);
  }
  return 0;
}
