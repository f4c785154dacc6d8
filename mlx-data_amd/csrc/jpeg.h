// jpeg.h -- from-scratch JPEG decoder (libjpeg ISLOW + fancy upsampling
// semantics; see jpeg.cpp) behind mxd_jpeg_info / mxd_jpeg_decode.
#pragma once

#include <cstddef>
#include <cstdint>
#include <string>

namespace mxd {
namespace jpeg {

// The reference's signature check (core/image/ImageJPEG.cpp:68-97): FF D8 FF.
bool is_jpeg(const uint8_t* data, size_t size);

// Image size and component count from the frame header.
bool info(const uint8_t* data, size_t size, int* width, int* height, int* components, std::string* err);

// Decodes to height rows of width*3 bytes (RGB; grey replicated; CMYK: the
// first three channels) at dst_stride.  false + *err on failure.
bool decode(const uint8_t* data, size_t size, uint8_t* dst, int64_t dst_stride, int width, int height,
            std::string* err);

// ---- split decode (the device-side finish, SURVEY.md §8f f1 "later a
// device-side decode"): the entropy decode runs on the host and keeps the
// quantised DCT coefficients; dequantisation + IDCT, upsampling and colour
// conversion run later, on the host (finish) or on the GPU (jpegdev.hip).
// Both give the bytes decode() gives.
struct Coefs;  // opaque

struct CoefPlane {
  int h, v;         // sampling factors
  int dw, dh;       // samples of the component proper
  int bw, bh;       // blocks per row / column (MCU-padded grid; rows of bw * 8 samples)
  bool coded;       // false: no scan carried it, its samples are 0
  int64_t off;      // first coefficient (blocks of 64, natural order, row-major)
  const uint16_t* q;  // quantisation table (natural order)
};

struct CoefInfo {
  int width, height, ncomp;
  int used;         // components the output reads (CMYK: 3)
  int color_space;  // 0 grey, 1 YCbCr, 2 RGB, 3 CMYK, 4 YCCK
  int max_h, max_v;
  const int16_t* coef;
  int64_t coef_count;
  CoefPlane comp[4];
  bool device_ok;   // grey, YCbCr or RGB: the device kernels can finish it
};

// Entropy decode (every error decode() reports, from here); nullptr + *err.
Coefs* decode_coefs(const uint8_t* data, size_t size, std::string* err);
void free_coefs(Coefs* c);
CoefInfo coef_info(const Coefs* c);
// Host finish into height rows of width*3 bytes at dst_stride (thread-safe).
bool finish(const Coefs* c, uint8_t* dst, int64_t dst_stride, std::string* err);

}  // namespace jpeg
}  // namespace mxd
