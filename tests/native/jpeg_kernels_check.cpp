// Exactness of the decoder's vectorised inner kernels against their scalar
// statements (tests/test_jpeg.py pins the whole decoder to libjpeg-turbo on
// natural images; this covers the value ranges those images never reach):
//   idct_islow32 (int32 lanes, guarded)  vs  idct_islow (jidctint.c, 64-bit)
//   ycc_rgb_row (integer formula)        vs  jdcolor.c's table construction
//   h2v2_fancy_row (column sums)         vs  jdsample.c's loop-carried form
// Built and run by tests/test_jpeg_kernels.py (g++ on the CPU).
#include "../../mlx-data_amd/csrc/jpeg.cpp"

#include <cstdio>
#include <random>

using namespace mxd::jpeg;

int main() {
  std::mt19937 gen(7);
  int fails = 0, fast = 0;
  uint16_t q[64];
  int16_t blk[64];
  uint8_t a[8 * 8], b[8 * 8];
  for (int t = 0; t < 200000; t++) {
    // magnitudes from tiny to the int16 limit, sparse and dense blocks
    const int mag = 1 << (gen() % 16);
    const int dens = 1 + gen() % 64;
    for (int i = 0; i < 64; i++) {
      q[i] = (uint16_t)(1 + gen() % (t % 7 == 0 ? 255 : 16));
      blk[i] = (int16_t)((int)(gen() % 64) < dens ? (int)(gen() % (2 * mag + 1)) - mag : 0);
    }
    idct_islow(blk, q, a, 8);
    if (idct_islow32(blk, q, b, 8)) {
      fast++;
      if (std::memcmp(a, b, 64)) fails++;
    }
  }
  // colour conversion: every (Y, Cb, Cr) against the table form
  std::vector<uint8_t> Y(256), Cb(256), Cr(256), o(3 * 256);
  for (int cb = 0; cb < 256; cb++)
    for (int cr = 0; cr < 256; cr++) {
      for (int y = 0; y < 256; y++) {
        Y[y] = (uint8_t)y;
        Cb[y] = (uint8_t)cb;
        Cr[y] = (uint8_t)cr;
      }
      for (int inv = 0; inv < 2; inv++) {
        ycc_rgb_row(Y.data(), Cb.data(), Cr.data(), o.data(), 256, inv);
        const int32_t half = 1 << 15;
        auto fix = [](double x) { return (int32_t)(x * 65536 + 0.5); };
        const int xr = cr - 128, xb = cb - 128;
        const int crr = (int)((fix(1.40200) * xr + half) >> 16), cbb = (int)((fix(1.77200) * xb + half) >> 16);
        const int32_t crg = -fix(0.71414) * xr, cbg = -fix(0.34414) * xb + half;
        for (int y = 0; y < 256; y++) {
          int v[3] = {y + crr, y + (int)((cbg + crg) >> 16), y + cbb};
          for (int k = 0; k < 3; k++) {
            int w = inv ? 255 - v[k] : v[k];
            w = w < 0 ? 0 : w > 255 ? 255 : w;
            if (o[3 * y + k] != w) fails++;
          }
        }
      }
    }
  // h2v2 fancy upsampling rows
  for (int t = 0; t < 2000; t++) {
    const int dw = 3 + gen() % 300;
    std::vector<uint8_t> in0(dw), in1(dw), out(2 * dw + 2), ref(2 * dw + 2);
    std::vector<int16_t> cs(dw);
    for (int x = 0; x < dw; x++) in0[x] = (uint8_t)gen(), in1[x] = (uint8_t)gen();
    h2v2_fancy_row(in0.data(), in1.data(), dw, out.data(), cs.data());
    int thiscol = in0[0] * 3 + in1[0], nextcol = in0[1] * 3 + in1[1];
    ref[0] = (uint8_t)((thiscol * 4 + 8) >> 4);
    ref[1] = (uint8_t)((thiscol * 3 + nextcol + 7) >> 4);
    int lastcol = thiscol;
    thiscol = nextcol;
    for (int x = 1; x < dw - 1; x++) {
      nextcol = in0[x + 1] * 3 + in1[x + 1];
      ref[2 * x] = (uint8_t)((thiscol * 3 + lastcol + 8) >> 4);
      ref[2 * x + 1] = (uint8_t)((thiscol * 3 + nextcol + 7) >> 4);
      lastcol = thiscol;
      thiscol = nextcol;
    }
    ref[2 * dw - 2] = (uint8_t)((thiscol * 3 + lastcol + 8) >> 4);
    ref[2 * dw - 1] = (uint8_t)((thiscol * 4 + 7) >> 4);
    if (std::memcmp(out.data(), ref.data(), 2 * dw)) fails++;
  }
  std::printf("jpeg_kernels: %d failures, %d of 200000 blocks on the int32 path\n", fails, fast);
  return fails ? 1 : 0;
}
