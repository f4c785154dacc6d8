// tools/nt_ceiling.hip -- HBM ceilings by cache policy (diagnostic, not product).
//
// the copy ceiling bench.py quotes (mxd_copy_bandwidth, a
// 16-B-per-thread streaming copy with default-policy loads and stores) next to
// the same forms with nontemporal (nt) / sc1 policies, a read-only stream, and
// an LDS-DMA read stream (buffer_load ... lds, 1 KiB per wave instruction) in
// both policies.  Buffers of 2 GiB (far past the 256 MiB Infinity Cache),
// 2 alternating buffer pairs, median of 7 timed runs of 5 launches each.
//
//   hipcc --offload-arch=gfx950 -O3 tools/nt_ceiling.hip -o tools/nt_ceiling && tools/nt_ceiling
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

typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
using Rsrc = __amdgpu_buffer_rsrc_t;
using lds_u8 = __attribute__((address_space(3))) unsigned char;

__device__ __forceinline__ Rsrc rsrc(void* p, unsigned bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(p, (short)0, (int)bytes, 0x00020000);
}

// copy: one 16-B buffer load + store per thread, one 4-KiB chunk per block
// (each block owns its own 4 KiB window; the resource starts at that window so
// 32-bit offsets suffice).
template <int LA, int SA>
__global__ __launch_bounds__(256) void copy_k(char* a, char* b) {
  const size_t base = (size_t)blockIdx.x * 4096;
  const Rsrc ra = rsrc(a + base, 4096), rb = rsrc(b + base, 4096);
  const u32x4 v = __builtin_amdgcn_raw_buffer_load_b128(ra, threadIdx.x * 16, 0, LA);
  __builtin_amdgcn_raw_buffer_store_b128(v, rb, threadIdx.x * 16, 0, SA);
}

// read: U 16-B loads per thread over a 4*U-KiB chunk per block.
template <int LA, int U>
__global__ __launch_bounds__(256) void read_k(char* a, unsigned* out) {
  const size_t base = (size_t)blockIdx.x * 4096 * U;
  const Rsrc ra = rsrc(a + base, 4096 * U);
  unsigned acc = 0;
  u32x4 v[U];
#pragma unroll
  for (int u = 0; u < U; u++) v[u] = __builtin_amdgcn_raw_buffer_load_b128(ra, u * 4096 + threadIdx.x * 16, 0, LA);
#pragma unroll
  for (int u = 0; u < U; u++) acc ^= v[u].x ^ v[u].y ^ v[u].z ^ v[u].w;
  if (acc == 0x9e3779b9u) out[threadIdx.x] = acc;
}

// LDS-DMA read: every wave streams U pieces of 1 KiB into LDS (16 B per lane).
template <int LA, int U>
__global__ __launch_bounds__(256) void ldsdma_k(char* a, unsigned* out) {
  __shared__ __attribute__((aligned(16))) unsigned char smem[4 * U * 1024];
  const size_t base = (size_t)blockIdx.x * 4096 * U;
  const Rsrc ra = __builtin_amdgcn_make_buffer_rsrc(a + base, (short)0, 4096 * U, 0x00020000);
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
#pragma unroll
  for (int u = 0; u < U; u++)
    __builtin_amdgcn_raw_ptr_buffer_load_lds(ra, (lds_u8*)(smem + (wave * U + u) * 1024), 16,
                                             (wave * U + u) * 1024 + lane * 16, 0, 0, LA);
  __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0)
  __syncthreads();
  const unsigned v = *reinterpret_cast<unsigned*>(smem + threadIdx.x * 4);
  if (v == 0x9e3779b9u) out[threadIdx.x] = v;
}

template <class F>
static float time_us(F&& launch, int iters = 5, int reps = 7) {
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  for (int i = 0; i < 3; i++) launch(i);
  std::vector<float> t;
  for (int r = 0; r < reps; r++) {
    CHECK(hipEventRecord(e0));
    for (int i = 0; i < iters; i++) launch(i);
    CHECK(hipEventRecord(e1));
    CHECK(hipEventSynchronize(e1));
    float ms;
    CHECK(hipEventElapsedTime(&ms, e0, e1));
    t.push_back(ms * 1000.0f / iters);
  }
  std::sort(t.begin(), t.end());
  CHECK(hipEventDestroy(e0));
  CHECK(hipEventDestroy(e1));
  return t[t.size() / 2];
}

int main() {
  const size_t N = (size_t)2 << 30;  // bytes per buffer
  char *a[2], *b[2];
  unsigned* out;
  for (int i = 0; i < 2; i++) {
    CHECK(hipMalloc(&a[i], N));
    CHECK(hipMalloc(&b[i], N));
    CHECK(hipMemset(a[i], i + 1, N));
    CHECK(hipMemset(b[i], 0, N));
  }
  CHECK(hipMalloc(&out, 4096));
  CHECK(hipDeviceSynchronize());
  auto report = [&](const char* name, double bytes, float us) {
    printf("{\"probe\": \"%s\", \"us\": %.1f, \"GBps\": %.1f}\n", name, us, bytes / (us * 1e-6) / 1e9);
    fflush(stdout);
  };
  const unsigned cblocks = (unsigned)(N / 4096);
#define COPY(LA, SA, NAME) \
  report(NAME, 2.0 * N, time_us([&](int i) { copy_k<LA, SA><<<cblocks, 256>>>(a[i & 1], b[i & 1]); }))
  for (int round = 0; round < 2; round++) {
    COPY(0, 0, "copy ld default / st default");
    COPY(2, 0, "copy ld nt / st default");
    COPY(0, 2, "copy ld default / st nt");
    COPY(2, 2, "copy ld nt / st nt");
    COPY(16, 2, "copy ld sc1 / st nt");
    COPY(18, 18, "copy ld nt sc1 / st nt sc1");
#define READ(LA, U, NAME) \
  report(NAME, (double)N, time_us([&](int i) { read_k<LA, U><<<(unsigned)(N / (4096 * U)), 256>>>(a[i & 1], out); }))
    READ(0, 4, "read U4 default");
    READ(2, 4, "read U4 nt");
    READ(0, 8, "read U8 default");
    READ(2, 8, "read U8 nt");
    READ(16, 8, "read U8 sc1");
#define DMA(LA, U, NAME) \
  report(NAME, (double)N, time_us([&](int i) { ldsdma_k<LA, U><<<(unsigned)(N / (4096 * U)), 256>>>(a[i & 1], out); }))
    DMA(0, 4, "ldsdma U4 default");
    DMA(2, 4, "ldsdma U4 nt");
    DMA(0, 8, "ldsdma U8 default");
    DMA(2, 8, "ldsdma U8 nt");
    DMA(0, 16, "ldsdma U16 default");
    DMA(2, 16, "ldsdma U16 nt");
  }
  CHECK(hipDeviceSynchronize());
  return 0;
}
