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

}  // namespace jpeg
}  // namespace mxd
