// tools/membench.hip -- read-bandwidth probe for the resample kernels' source
// access pattern (diagnostic, not part of the product).
//
// 256 images of 960 rows x 3840 B in HBM.  Each wave streams `rows` consecutive
// rows of one image, reading a window of `win` bytes per row (win/256 dword
// loads per lane, lanes 4 B apart, like wave.hip), keeping `depth` rows of
// loads in flight, and sums the words (so the loads are live).  Variants:
//   win = 1024 with 3 windows per row (the strip layout), 2048, 3072 (a full
//   footprint row per wave); depth 2..16.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#define CHECK(x)                                                                       \
  do {                                                                                 \
    hipError_t e = (x);                                                                \
    if (e != hipSuccess) {                                                             \
      fprintf(stderr, "%s failed: %s\n", #x, hipGetErrorString(e));                    \
      exit(1);                                                                         \
    }                                                                                  \
  } while (0)

constexpr int kImgRows = 960, kStride = 3840, kImgs = 256;

template <int NW, int DEPTH>
__global__ __launch_bounds__(256) void stream_rows(const uint8_t* base, int rows_per_unit, int windows_per_row,
                                                   int win_step, int nunits, unsigned* out) {
  const int lane = threadIdx.x & 63;
  const int unit = __builtin_amdgcn_readfirstlane(blockIdx.x * 4 + (threadIdx.x >> 6));
  if (unit >= nunits) return;
  const int units_per_img = (kImgRows / rows_per_unit) * windows_per_row;
  const int img = unit / units_per_img;
  const int rest = unit - img * units_per_img;
  const int band = rest / windows_per_row;
  const int win = rest - band * windows_per_row;
  const uint8_t* p = base + (size_t)img * kImgRows * kStride;
  const __amdgpu_buffer_rsrc_t r =
      __builtin_amdgcn_make_buffer_rsrc((void*)p, (short)0, kImgRows * kStride, 0x00020000);
  const int off = win * win_step + 4 * lane;
  const int r0 = band * rows_per_unit;
  unsigned ring[DEPTH][NW];
#pragma unroll
  for (int d = 0; d < DEPTH; d++)
#pragma unroll
    for (int j = 0; j < NW; j++) ring[d][j] = __builtin_amdgcn_raw_buffer_load_b32(r, off + 256 * j, (r0 + d) * kStride, 0);
  unsigned acc = 0;
  for (int row = r0; row < r0 + rows_per_unit; row += DEPTH) {
#pragma unroll
    for (int d = 0; d < DEPTH; d++) {
#pragma unroll
      for (int j = 0; j < NW; j++) {
        acc += ring[d][j];
        ring[d][j] = __builtin_amdgcn_raw_buffer_load_b32(r, off + 256 * j, (row + d + DEPTH) * kStride, 0);
      }
    }
  }
#pragma unroll
  for (int d = 0; d < DEPTH; d++)
#pragma unroll
    for (int j = 0; j < NW; j++) acc += ring[d][j];
  if (acc == 0x12345678u) out[0] = acc;
}

template <int NW, int DEPTH>
double run(const uint8_t* d, unsigned* out, int rows_per_unit, int windows_per_row, int win_step, int lds = 0) {
  const int nunits = kImgs * (kImgRows / rows_per_unit) * windows_per_row;
  const int blocks = (nunits + 3) / 4;
  hipEvent_t a, b;
  CHECK(hipEventCreate(&a));
  CHECK(hipEventCreate(&b));
  for (int w = 0; w < 3; w++)
    hipLaunchKernelGGL((stream_rows<NW, DEPTH>), dim3(blocks), dim3(256), lds, 0, d, rows_per_unit, windows_per_row,
                       win_step, nunits, out);
  CHECK(hipEventRecord(a));
  const int iters = 20;
  for (int i = 0; i < iters; i++)
    hipLaunchKernelGGL((stream_rows<NW, DEPTH>), dim3(blocks), dim3(256), lds, 0, d, rows_per_unit, windows_per_row,
                       win_step, nunits, out);
  CHECK(hipEventRecord(b));
  CHECK(hipEventSynchronize(b));
  float ms;
  CHECK(hipEventElapsedTime(&ms, a, b));
  const double bytes = (double)nunits * rows_per_unit * NW * 256;
  const double gbs = bytes / (ms / iters * 1e-3) / 1e9;
  printf("win=%4dB windows/row=%d step=%4d rows/unit=%3d depth=%2d units=%6d lds=%6d: %8.1f us  %7.1f GB/s\n",
         NW * 256, windows_per_row, win_step, rows_per_unit, DEPTH, nunits, lds, ms / iters * 1e3, gbs);
  return gbs;
}


// Reads like stream_rows (windows of `need` bytes, lanes past it masked) and,
// every 4th row, writes 1 KiB (16 B per lane) to the unit's own contiguous
// output region: about the read/write mix of the C2 kernel (155 MB / 568 MB).
template <int DEPTH, bool WRITE>
__global__ __launch_bounds__(256) void stream_rows_w(const uint8_t* base, float4* outbuf, int rows_per_unit,
                                                     int windows_per_row, int win_step, int need, int nunits) {
  const int lane = threadIdx.x & 63;
  const int unit = __builtin_amdgcn_readfirstlane(blockIdx.x * 4 + (threadIdx.x >> 6));
  if (unit >= nunits) return;
  const int units_per_img = (kImgRows / rows_per_unit) * windows_per_row;
  const int img = unit / units_per_img;
  const int rest = unit - img * units_per_img;
  const int band = rest / windows_per_row;
  const int win = rest - band * windows_per_row;
  const uint8_t* p = base + (size_t)img * kImgRows * kStride;
  const __amdgpu_buffer_rsrc_t r =
      __builtin_amdgcn_make_buffer_rsrc((void*)p, (short)0, kImgRows * kStride, 0x00020000);
  int off[4];
#pragma unroll
  for (int j = 0; j < 4; j++) off[j] = 4 * lane + 256 * j < need ? win * win_step + 4 * lane + 256 * j : 0x7ffffff0;
  const int r0 = band * rows_per_unit;
  float4* o = outbuf + (size_t)unit * (rows_per_unit / 4) * 64 + lane;
  unsigned ring[DEPTH][4];
#pragma unroll
  for (int d = 0; d < DEPTH; d++)
#pragma unroll
    for (int j = 0; j < 4; j++) ring[d][j] = __builtin_amdgcn_raw_buffer_load_b32(r, off[j], (r0 + d) * kStride, 0);
  unsigned acc = 0;
  for (int row = r0; row < r0 + rows_per_unit; row += DEPTH) {
#pragma unroll
    for (int d = 0; d < DEPTH; d++) {
#pragma unroll
      for (int j = 0; j < 4; j++) {
        acc += ring[d][j];
        ring[d][j] = __builtin_amdgcn_raw_buffer_load_b32(r, off[j], (row + d + DEPTH) * kStride, 0);
      }
      if (WRITE && (d & 3) == 3) {
        *o = make_float4((float)acc, (float)(acc >> 8), (float)(acc >> 16), (float)row);
        o += 64;
      }
    }
  }
  if (acc == 0x12345678u) outbuf[0].x = 1.0f;
}

template <int DEPTH, bool WRITE>
void run_w(const uint8_t* d, float4* out, int rows_per_unit, int windows_per_row, int win_step, int need) {
  const int nunits = kImgs * (kImgRows / rows_per_unit) * windows_per_row;
  const int blocks = (nunits + 3) / 4;
  hipEvent_t a, b;
  CHECK(hipEventCreate(&a));
  CHECK(hipEventCreate(&b));
  for (int w = 0; w < 3; w++)
    hipLaunchKernelGGL((stream_rows_w<DEPTH, WRITE>), dim3(blocks), dim3(256), 0, 0, d, out, rows_per_unit,
                       windows_per_row, win_step, need, nunits);
  CHECK(hipEventRecord(a));
  const int iters = 20;
  for (int i = 0; i < iters; i++)
    hipLaunchKernelGGL((stream_rows_w<DEPTH, WRITE>), dim3(blocks), dim3(256), 0, 0, d, out, rows_per_unit,
                       windows_per_row, win_step, need, nunits);
  CHECK(hipEventRecord(b));
  CHECK(hipEventSynchronize(b));
  float ms;
  CHECK(hipEventElapsedTime(&ms, a, b));
  const double rd = (double)nunits * rows_per_unit * need;
  const double wr = WRITE ? (double)nunits * (rows_per_unit / 4) * 1024 : 0.0;
  const double us = ms / iters * 1e3;
  printf("need=%4d windows/row=%d rows/unit=%3d depth=%2d write=%d: %8.1f us  read %6.1f MB write %6.1f MB  %7.1f GB/s\n",
         need, windows_per_row, rows_per_unit, DEPTH, (int)WRITE, us, rd / 1e6, wr / 1e6, (rd + wr) / (us * 1e-6) / 1e9);
}

int main() {
  uint8_t* d;
  unsigned* out;
  const size_t bytes = (size_t)kImgs * kImgRows * kStride;
  CHECK(hipMalloc(&d, bytes));
  CHECK(hipMalloc(&out, 16));
  CHECK(hipMemset(d, 1, bytes));
  float4* wout;
  CHECK(hipMalloc(&wout, (size_t)kImgs * kImgRows / 4 * 3 * 1024 + 4096));
  // real windows (844 rows x 855 B x 3 per image ~ the C2 footprint), without and with writes
  run_w<8, false>(d, wout, 80, 3, 844, 855);
  run_w<8, true>(d, wout, 80, 3, 844, 855);
  run_w<12, true>(d, wout, 80, 3, 844, 855);
  run_w<8, true>(d, wout, 48, 3, 844, 855);
  // strip layout (3 windows of 1 KiB per row, 80-row bands) at several occupancies
  for (int lds : {0, 40960, 54000}) run<4, 8>(d, out, 80, 3, 855, lds);
  run<4, 16>(d, out, 80, 3, 855, 40960);
  // one wave per footprint row (3 KiB window), and whole rows (3840 B, sequential image)
  run<12, 4>(d, out, 80, 1, 0, 0);
  run<12, 4>(d, out, 80, 1, 0, 40960);
  run<15, 4>(d, out, 80, 1, 0, 0);
  run<15, 4>(d, out, 40, 1, 0, 0);
  // one 1 KiB window per row
  run<4, 8>(d, out, 80, 1, 0, 0);
  return 0;
}
