// jpegdev.hip -- device-side finish of a split JPEG decode (see jpegdev.h).
//
// jpeg_idct: one thread per 8x8 block: dequantise, jidctint.c ISLOW (13-bit
//   constants, PASS1_BITS 2, 64-bit intermediates like libjpeg-turbo's JLONG;
//   its all-zero-AC shortcuts are exact, so the plain transform gives the same
//   bytes), the output range limit of libjpeg-turbo's SIMD IDCTs (+128,
//   clamp; jpeg.cpp range_limit), eight 8-byte row stores into the
//   component's sample plane.
// jpeg_color: one thread per eight horizontal output pixels of one image:
//   each component's sample by jdsample.c's rule for its sampling factors
//   (fancy triangle upsampling h2v1 / h1v2 / h2v2 with jpeg.cpp's edge cases,
//   replication otherwise), jdcolor.c's 16-bit fixed-point YCbCr -> RGB (or
//   RGB / grey as is), three 8-byte stores; 4:2:0, 4:2:2, 4:4:4 and grey
//   read their samples as aligned dwords with static byte indices (round 5:
//   107 us per 128-file C4 batch before, four pixels per thread through a
//   per-pixel switch).
#include "jpegdev.h"
#include "jpegycc.h"

namespace mxd {
namespace {

using i64 = long long;

constexpr int kConstBits = 13;
constexpr int kPass1Bits = 2;
constexpr i64 F0298 = 2446, F0390 = 3196, F0541 = 4433, F0765 = 6270, F0899 = 7373, F1175 = 9633, F1501 = 12299,
              F1847 = 15137, F1961 = 16069, F2053 = 16819, F2562 = 20995, F3072 = 25172;


// Natural index -> zig-zag index (the inverse of jutils.c jpeg_natural_order),
// for blocks the device entropy decode stores in zig-zag order.
constexpr int kNatZigzag[64] = {0, 1, 5, 6, 14, 15, 27, 28, 2, 4, 7, 13, 16, 26, 29, 42, 3, 8, 12, 17, 25, 30, 41, 43, 9, 11, 18, 24, 31, 40, 44, 53, 10, 19, 23, 32, 39, 45, 52, 54, 20, 22, 33, 38, 46, 51, 55, 60, 21, 34, 37, 47, 50, 56, 59, 61, 35, 36, 48, 49, 57, 58, 62, 63};

__device__ __forceinline__ uint32_t range_limit(i64 x) {
  const i64 v = x + 128;
  return (uint32_t)(v < 0 ? 0 : v > 255 ? 255 : v);
}

// One 1-D pass over 8 values (even part from 0/2/4/6, odd part from 1/3/5/7),
// jidctint.c's arithmetic; outputs in natural order before descaling.  T =
// i64 is libjpeg-turbo's JLONG; T = int32_t gives the same values when every
// input is below 2^14 in magnitude (the largest intermediate is then below
// 2^30.7: products of an input sum < 2^16 and a 13-bit constant, sums of
// three such), which is every block of a well-formed file (dequantised DCT
// coefficients of 8-bit samples stay below 2^12).
// x * k: int32 values here are below 2^17 and constants below 2^15, so the
// 24-bit multiply (full rate; v_mul_lo_u32 is quarter rate) is exact
template <class T>
__device__ __forceinline__ T mulk(T x, int k) {
  return x * (T)k;
}
template <>
__device__ __forceinline__ int32_t mulk<int32_t>(int32_t x, int k) {
  return __mul24(x, k);
}

template <class T>
__device__ __forceinline__ void idct8(T d0, T d1, T d2, T d3, T d4, T d5, T d6, T d7, T* o) {
  const T z1e = mulk<T>(d2 + d6, F0541);
  const T t2 = z1e + mulk<T>(d6, -F1847);
  const T t3 = z1e + mulk<T>(d2, F0765);
  const T t0 = (d0 + d4) * (T)(1 << kConstBits);
  const T t1 = (d0 - d4) * (T)(1 << kConstBits);
  const T t10 = t0 + t3, t13 = t0 - t3, t11 = t1 + t2, t12 = t1 - t2;
  T a0 = d7, a1 = d5, a2 = d3, a3 = d1;
  T z1 = a0 + a3, z2 = a1 + a2, z3 = a0 + a2, z4 = a1 + a3;
  const T z5 = mulk<T>(z3 + z4, F1175);
  a0 = mulk<T>(a0, F0298);
  a1 = mulk<T>(a1, F2053);
  a2 = mulk<T>(a2, F3072);
  a3 = mulk<T>(a3, F1501);
  z1 = mulk<T>(z1, -F0899);
  z2 = mulk<T>(z2, -F2562);
  z3 = mulk<T>(z3, -F1961) + z5;
  z4 = mulk<T>(z4, -F0390) + z5;
  a0 += z1 + z3;
  a1 += z2 + z4;
  a2 += z2 + z3;
  a3 += z1 + z4;
  o[0] = t10 + a3;
  o[7] = t10 - a3;
  o[1] = t11 + a2;
  o[6] = t11 - a2;
  o[2] = t12 + a1;
  o[5] = t12 - a1;
  o[3] = t13 + a0;
  o[4] = t13 - a0;
}

template <class T>
__device__ __forceinline__ T descale_t(T x, int n) {
  return (x + ((T)1 << (n - 1))) >> n;
}

// The block with JLONG (64-bit) arithmetic, for blocks whose values leave
// the int32 range (corrupt data): out of line, one column / row at a time,
// so the common path's register allocation does not carry it.
__device__ __noinline__ void idct_block_wide(const int32_t* __restrict__ din, uint8_t* out, int stride) {
  int32_t ws[64];
#pragma unroll 1
  for (int c = 0; c < 8; c++) {
    i64 o[8];
    idct8<i64>(din[c], din[8 + c], din[16 + c], din[24 + c], din[32 + c], din[40 + c], din[48 + c], din[56 + c], o);
#pragma unroll
    for (int r = 0; r < 8; r++) ws[8 * r + c] = (int32_t)descale_t<i64>(o[r], kConstBits - kPass1Bits);
  }
#pragma unroll 1
  for (int r = 0; r < 8; r++) {
    const int32_t* w = ws + 8 * r;
    i64 o[8];
    idct8<i64>(w[0], w[1], w[2], w[3], w[4], w[5], w[6], w[7], o);
    uint32_t lo4 = 0, hi4 = 0;
#pragma unroll
    for (int c = 0; c < 4; c++) {
      lo4 |= range_limit(descale_t<i64>(o[c], kConstBits + kPass1Bits + 3)) << (8 * c);
      hi4 |= range_limit(descale_t<i64>(o[c + 4], kConstBits + kPass1Bits + 3)) << (8 * c);
    }
    *reinterpret_cast<uint2*>(out + (i64)r * stride) = make_uint2(lo4, hi4);
  }
}

// Whether every value of v is inside (-2^14, 2^14) (the int32 IDCT's range).
__device__ __forceinline__ bool small14(const int32_t* v) {
  uint32_t acc = 0;
#pragma unroll
  for (int i = 0; i < 64; i++) acc |= (uint32_t)(v[i] + 16384);
  return acc < 32768u;
}

__global__ __launch_bounds__(256) void jpeg_idct(const int16_t* __restrict__ coef, const uint16_t* __restrict__ qt,
                                                 const JpegPlaneDev* __restrict__ planes, int nplanes, i64 nblocks,
                                                 uint8_t* __restrict__ samples) {
  const i64 g = (i64)blockIdx.x * 256 + threadIdx.x;
  // every plane's blocks start at a multiple of 64 in this numbering (the
  // host pads them), so a wave lies in one plane: its record, quantisation
  // table and flags are scalar (s_load), not per-lane vector loads
  const i64 g0 = ((i64)__builtin_amdgcn_readfirstlane((int)(g >> 32)) << 32) |
                 (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)g);
  if (g0 >= nblocks) return;
  int lo = 0, hi = nplanes - 1;  // the last plane whose first block is <= g0
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (planes[mid].first_block <= g0) lo = mid;
    else hi = mid - 1;
  }
  lo = __builtin_amdgcn_readfirstlane(lo);
  const JpegPlaneDev p = planes[lo];
  const i64 b = g - p.first_block;
  const int rw = p.bx1 - p.bx0;
  if (b >= (i64)rw * (p.by1 - p.by0)) return;  // the plane's padding
  const int ry = (int)((uint32_t)b / (uint32_t)rw);  // (a plane holds < 2^31 blocks)
  const int by = p.by0 + ry, bx = p.bx0 + ((int)b - ry * rw);
  const int stride = p.bw * 8;
  uint8_t* out = samples + p.out + (i64)by * 8 * stride + bx * 8;
  if (!p.coded) {
#pragma unroll
    for (int r = 0; r < 8; r++) *reinterpret_cast<uint2*>(out + (i64)r * stride) = make_uint2(0, 0);
    return;
  }
  int32_t d[64];
  {
    const int4* cp = reinterpret_cast<const int4*>(coef + p.coef + ((i64)by * p.bw + bx) * 64);
    const uint16_t* q = qt + p.qtab;  // uniform: scalar loads
    const bool zz = p.zigzag != 0;
    int32_t cw[64];  // the block's 64 stored coefficients, in storage order
#pragma unroll
    for (int k = 0; k < 8; k++) {
      const int4 c = cp[k];
      const int32_t w4[4] = {c.x, c.y, c.z, c.w};
#pragma unroll
      for (int j = 0; j < 4; j++) {
        cw[8 * k + 2 * j] = (int32_t)(int16_t)(w4[j] & 0xffff);
        cw[8 * k + 2 * j + 1] = (int32_t)(int16_t)((uint32_t)w4[j] >> 16);
      }
    }
    // natural position n holds stored coefficient kNatZigzag[n] of a zig-zag
    // block: both candidates are compile-time register indices, the choice a
    // select (a runtime index would put the block in scratch memory)
#pragma unroll
    for (int n = 0; n < 64; n++) d[n] = __mul24(zz ? cw[kNatZigzag[n]] : cw[n], (int32_t)q[n]);  // 16 x 16 bits: exact
  }
  // pass 1: columns -> int workspace (descaled by CONST_BITS - PASS1_BITS),
  // in place (column c of d is read before it is written), in 32-bit
  // arithmetic when every input allows it (small14; a block of corrupt data
  // that does not takes the JLONG path, idct_block_wide); pass 2: rows ->
  // samples, likewise
  if (!small14(d)) {
    int32_t dw[64];  // a memory copy for the out-of-line path only
#pragma unroll
    for (int i = 0; i < 64; i++) dw[i] = d[i];
    idct_block_wide(dw, out, stride);
    return;
  }
  int32_t ws[64];
#pragma unroll
  for (int c = 0; c < 8; c++) {
    int32_t o[8];
    idct8<int32_t>(d[c], d[8 + c], d[16 + c], d[24 + c], d[32 + c], d[40 + c], d[48 + c], d[56 + c], o);
#pragma unroll
    for (int r = 0; r < 8; r++) ws[8 * r + c] = descale_t<int32_t>(o[r], kConstBits - kPass1Bits);
  }
  if (!small14(ws)) {
    int32_t dw[64];  // (pass 1's values were exact: the wide path recomputes them)
#pragma unroll
    for (int i = 0; i < 64; i++) dw[i] = d[i];
    idct_block_wide(dw, out, stride);
    return;
  }
#pragma unroll
  for (int r = 0; r < 8; r++) {
    const int32_t* w = ws + 8 * r;
    int32_t o[8];
    idct8<int32_t>(w[0], w[1], w[2], w[3], w[4], w[5], w[6], w[7], o);
    uint32_t lo4 = 0, hi4 = 0;
#pragma unroll
    for (int c = 0; c < 4; c++) {
      lo4 |= range_limit(descale_t<int32_t>(o[c], kConstBits + kPass1Bits + 3)) << (8 * c);
      hi4 |= range_limit(descale_t<int32_t>(o[c + 4], kConstBits + kPass1Bits + 3)) << (8 * c);
    }
    *reinterpret_cast<uint2*>(out + (i64)r * stride) = make_uint2(lo4, hi4);
  }
}

// Component k's sample at output (x, y) (jpeg.cpp upsample_row).
__device__ __forceinline__ int sample_at(const uint8_t* __restrict__ pl, const JpegImgDev& m, int k, int x, int y) {
  const int stride = m.stride[k];
  switch (m.mode[k]) {
    case kUpFull:
      return pl[(i64)y * stride + x];
    case kUpH2V1: {
      const uint8_t* in = pl + (i64)y * stride;
      const int i = x >> 1, dw = m.dw[k];
      const int v = in[i] * 3;
      if (x & 1) return i == dw - 1 ? in[i] : (v + in[i + 1] + 2) >> 2;
      return i == 0 ? in[0] : (v + in[i - 1] + 1) >> 2;
    }
    case kUpH1V2:
    case kUpH2V2: {
      const int iy = y >> 1, below = y & 1, dh = m.dh[k];
      const int ny = min(max(below ? iy + 1 : iy - 1, 0), dh - 1);
      const uint8_t* in0 = pl + (i64)min(iy, dh - 1) * stride;
      const uint8_t* in1 = pl + (i64)ny * stride;
      if (m.mode[k] == kUpH1V2) return (in0[x] * 3 + in1[x] + (below ? 2 : 1)) >> 2;
      const int i = x >> 1, dw = m.dw[k];
      const int cs = in0[i] * 3 + in1[i];
      if (x & 1) return i == dw - 1 ? (cs * 4 + 7) >> 4 : (cs * 3 + in0[i + 1] * 3 + in1[i + 1] + 7) >> 4;
      return i == 0 ? (cs * 4 + 8) >> 4 : (cs * 3 + in0[i - 1] * 3 + in1[i - 1] + 8) >> 4;
    }
    default:
      return pl[(i64)(y / m.vx[k]) * stride + x / m.hx[k]];
  }
}

// Eight output pixels x0..x0+7 of row y (x0 a multiple of 8).  Common
// layouts read their samples as aligned dwords and upsample with static byte
// indices: 4:2:0 (h2v2 fancy), 4:2:2 (h2v1 fancy), 4:4:4 and grey; any other
// (h1v2, replication, RGB, mixed factors) takes sample_at per pixel.  Pixels
// past the row end (the row's padding up to a multiple of 8, which no
// resample tap reads) are computed from the samples past it.
__device__ __forceinline__ uint32_t ld4(const uint8_t* p) { return *reinterpret_cast<const uint32_t*>(p); }

// the 12 bytes from dword-aligned index c - 4 of a sample row (row_bytes a
// multiple of 8; c a multiple of 4): b[e] = row[c - 4 + e]
__device__ __forceinline__ void load12(const uint8_t* row, int c, int row_bytes, uint32_t (&d)[3]) {
  d[0] = c >= 4 ? ld4(row + c - 4) : 0u;
  d[1] = ld4(row + min(c, row_bytes - 4));
  d[2] = ld4(row + min(c + 4, row_bytes - 4));
}
__device__ __forceinline__ int byte_at(const uint32_t (&d)[3], int e) { return (int)((d[e >> 2] >> (8 * (e & 3))) & 255u); }

__device__ __forceinline__ void ycc_to_rgb(int y, int cb, int cr, uint32_t* px) { jpeg_ycc_to_rgb(y, cb, cr, px); }

__global__ __launch_bounds__(256) void jpeg_color(const uint8_t* __restrict__ samples,
                                                  const JpegImgDev* __restrict__ imgs, uint8_t* __restrict__ rgb) {
  const JpegImgDev& m = imgs[blockIdx.y];
  if (m.skip) return;  // its resize reads the planes (ImgDev::ycc)
  const int octs = (m.width + 7) >> 3;
  const i64 t = (i64)blockIdx.x * 256 + threadIdx.x;
  if (t >= (i64)m.height * octs) return;
  const int y = (int)(t / octs);
  const int x0 = (int)(t - (i64)y * octs) * 8;
  uint32_t px[8][3];
  const bool ycc = m.ncomp == 3 && !m.rgb && m.mode[0] == kUpFull && m.mode[1] == m.mode[2];
  const uint8_t* yrow = samples + m.plane[0] + (i64)y * m.stride[0] + x0;
  if (m.ncomp == 1) {
    const uint32_t a = ld4(yrow), b = ld4(yrow + 4);
#pragma unroll
    for (int j = 0; j < 8; j++) px[j][0] = px[j][1] = px[j][2] = ((j < 4 ? a : b) >> (8 * (j & 3))) & 255u;
  } else if (ycc && m.mode[1] == kUpFull) {  // 4:4:4
    const uint8_t* r1 = samples + m.plane[1] + (i64)y * m.stride[1] + x0;
    const uint8_t* r2 = samples + m.plane[2] + (i64)y * m.stride[2] + x0;
    const uint32_t ya[2] = {ld4(yrow), ld4(yrow + 4)}, ba[2] = {ld4(r1), ld4(r1 + 4)}, ra[2] = {ld4(r2), ld4(r2 + 4)};
#pragma unroll
    for (int j = 0; j < 8; j++) {
      const int sh = 8 * (j & 3);
      ycc_to_rgb((int)((ya[j >> 2] >> sh) & 255u), (int)((ba[j >> 2] >> sh) & 255u), (int)((ra[j >> 2] >> sh) & 255u),
                 px[j]);
    }
  } else if (ycc && (m.mode[1] == kUpH2V2 || m.mode[1] == kUpH2V1)) {  // 4:2:0 / 4:2:2, fancy
    const bool v2 = m.mode[1] == kUpH2V2;
    const uint32_t ya[2] = {ld4(yrow), ld4(yrow + 4)};
    const int c = x0 >> 1;  // chroma sample of pixel x0 (a multiple of 4)
    int cv[2][6];           // per chroma component: samples c-1 .. c+4, vertically upsampled (h2v2: 3 near + far)
#pragma unroll
    for (int k = 1; k < 3; k++) {
      const int dh = m.dh[k], stride = m.stride[k];
      const uint8_t* pl = samples + m.plane[k];
      uint32_t d0[3], d1[3];
      if (v2) {
        const int iy = y >> 1;
        const int ny = min(max((y & 1) ? iy + 1 : iy - 1, 0), dh - 1);
        load12(pl + (i64)min(iy, dh - 1) * stride, c, stride, d0);
        load12(pl + (i64)ny * stride, c, stride, d1);
#pragma unroll
        for (int e = 0; e < 6; e++) cv[k - 1][e] = byte_at(d0, e + 3) * 3 + byte_at(d1, e + 3);
      } else {
        load12(pl + (i64)y * stride, c, stride, d0);
#pragma unroll
        for (int e = 0; e < 6; e++) cv[k - 1][e] = byte_at(d0, e + 3);
      }
    }
#pragma unroll
    for (int j = 0; j < 8; j++) {
      const int e = 1 + (j >> 1);  // sample i = c + j / 2 at cv index e
      const int i = c + (j >> 1);
      int ch[2];
#pragma unroll
      for (int k = 0; k < 2; k++) {
        const int dw = m.dw[k + 1];
        const int cs = cv[k][e];
        if (v2) {  // jpeg.cpp upsample_row h2v2
          ch[k] = (j & 1) ? (i == dw - 1 ? (cs * 4 + 7) >> 4 : (cs * 3 + cv[k][e + 1] + 7) >> 4)
                          : (i == 0 ? (cs * 4 + 8) >> 4 : (cs * 3 + cv[k][e - 1] + 8) >> 4);
        } else {   // h2v1
          ch[k] = (j & 1) ? (i == dw - 1 ? cs : (cs * 3 + cv[k][e + 1] + 2) >> 2)
                          : (i == 0 ? cs : (cs * 3 + cv[k][e - 1] + 1) >> 2);
        }
      }
      ycc_to_rgb((int)((ya[j >> 2] >> (8 * (j & 3))) & 255u), ch[0], ch[1], px[j]);
    }
  } else {
#pragma unroll
    for (int j = 0; j < 8; j++) {
      const int x = min(x0 + j, m.width - 1);  // pixels past the row end: a copy of the last
      const int c0 = sample_at(samples + m.plane[0], m, 0, x, y);
      const int c1 = sample_at(samples + m.plane[1], m, 1, x, y);
      const int c2 = sample_at(samples + m.plane[2], m, 2, x, y);
      if (m.rgb == 1) {
        px[j][0] = (uint32_t)c0;
        px[j][1] = (uint32_t)c1;
        px[j][2] = (uint32_t)c2;
      } else {
        ycc_to_rgb(c0, c1, c2, px[j]);
        if (m.rgb == 2) {  // YCCK: the C, M, Y libjpeg outputs are 255 - R, G, B
          px[j][0] = 255u - px[j][0];
          px[j][1] = 255u - px[j][1];
          px[j][2] = 255u - px[j][2];
        }
      }
    }
  }
  uint32_t w[6];
#pragma unroll
  for (int q = 0; q < 6; q++) {
    uint32_t v = 0;
#pragma unroll
    for (int b = 0; b < 4; b++) v |= px[(4 * q + b) / 3][(4 * q + b) % 3] << (8 * b);
    w[q] = v;
  }
  uint2* o = reinterpret_cast<uint2*>(rgb + m.out + (i64)y * m.pitch + (i64)x0 * 3);
  o[0] = make_uint2(w[0], w[1]);
  o[1] = make_uint2(w[2], w[3]);
  o[2] = make_uint2(w[4], w[5]);
}

}  // namespace

void launch_jpeg_idct(const int16_t* coef, const uint16_t* qtabs, const JpegPlaneDev* planes, int32_t nplanes,
                      int64_t nblocks, uint8_t* samples, hipStream_t stream) {
  if (nblocks <= 0 || nplanes <= 0) return;
  hipLaunchKernelGGL(jpeg_idct, dim3((unsigned)((nblocks + 255) / 256)), dim3(256), 0, stream, coef, qtabs, planes,
                     nplanes, (i64)nblocks, samples);
}

void launch_jpeg_color(const uint8_t* samples, const JpegImgDev* imgs, int32_t n, int64_t max_oct_rows, uint8_t* rgb,
                       hipStream_t stream) {
  if (n <= 0 || max_oct_rows <= 0) return;
  hipLaunchKernelGGL(jpeg_color, dim3((unsigned)((max_oct_rows + 255) / 256), (unsigned)n), dim3(256), 0, stream,
                     samples, imgs, rgb);
}

}  // namespace mxd
