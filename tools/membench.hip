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

int main() {
  uint8_t* d;
  unsigned* out;
  const size_t bytes = (size_t)kImgs * kImgRows * kStride;
  CHECK(hipMalloc(&d, bytes));
  CHECK(hipMalloc(&out, 16));
  CHECK(hipMemset(d, 1, bytes));
  // occupancy: 160 KiB LDS / lds bytes per 4-wave block
  for (int lds : {0, 20480, 32768, 40960, 54000, 81920}) run<4, 8>(d, out, 80, 3, 855, lds);
  for (int lds : {32768, 40960, 54000}) run<4, 16>(d, out, 80, 3, 855, lds);
  for (int lds : {40960, 54000}) run<4, 4>(d, out, 80, 3, 855, lds);
  return 0;
}
