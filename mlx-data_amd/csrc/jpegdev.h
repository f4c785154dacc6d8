// jpegdev.h -- the device-side finish of a split JPEG decode (SURVEY.md §8f
// f1, "later a device-side decode"): the host entropy-decodes (jpeg.h
// decode_coefs) and the GPU runs dequantisation + ISLOW IDCT, chroma
// upsampling and colour conversion, writing packed RGB rows that the resize
// kernels then read in place.  Same integer arithmetic as jpeg.cpp's host
// finish, so the bytes are identical (tests/test_gpu_jpeg.py).
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

namespace mxd {

// One component plane of one image.
struct JpegPlaneDev {
  int64_t coef;         // first coefficient (elements of the chunk's int16 buffer; 16-byte aligned)
  int64_t out;          // first sample byte in the chunk's sample buffer (bw * 8 per row)
  int64_t first_block;  // blocks of the planes before this one (the launch's flat block index)
  int32_t bw, bh;       // blocks per row / column
  int32_t qtab;         // first entry of its quantisation table (uint16 elements)
  int32_t coded;        // 0: no scan carried it, its samples are 0
  int32_t zigzag;       // 1: each block's coefficients in zig-zag order (the device entropy decode's), 0: natural
  // the blocks the resize can read ([bx0, bx1) x [by0, by1): its source
  // footprint, widened by the upsampling's reach): jpeg_idct's threads cover
  // this rectangle only (first_block numbers them), the rest is never read
  int32_t bx0, bx1, by0, by1;
  int32_t pad;
};

// Upsampling of one component to the output grid (jdsample.c), as jpeg.cpp
// upsample_row chooses it.
enum JpegUp : int32_t {
  kUpFull = 0,  // full size
  kUpH2V1 = 1,  // h2v1 fancy (dw > 2)
  kUpH1V2 = 2,  // h1v2 fancy
  kUpH2V2 = 3,  // h2v2 fancy (dw > 2)
  kUpRep = 4,   // replication by (hx, vx)
};

// One image's colour pass.
struct JpegImgDev {
  int64_t plane[3];  // sample-buffer byte offset of each component plane
  int64_t out;       // first RGB byte in the chunk's image buffer
  int32_t stride[3];  // bytes per plane row (bw * 8)
  int32_t dw[3], dh[3];
  int32_t mode[3];   // JpegUp
  int32_t hx[3], vx[3];
  int32_t ncomp;     // 1 (grey, replicated) or 3 (a CMYK / YCCK file's first three)
  int32_t rgb;       // 0: YCbCr -> RGB; 1: the components as they are (RGB; CMYK's C, M, Y);
                     // 2: YCCK, YCbCr -> RGB inverted (libjpeg's C, M, Y)
  int32_t width, height;
  int32_t pitch;     // bytes per RGB row (a multiple of 64, >= 3 * round_up(width, 8))
  int32_t skip;      // 1: a wave kernel reads the planes itself (ImgDev::ycc): no RGB frame
};

// Dequantise + IDCT every block of `nplanes` planes (`nblocks` in total).
void launch_jpeg_idct(const int16_t* coef, const uint16_t* qtabs, const JpegPlaneDev* planes, int32_t nplanes,
                      int64_t nblocks, uint8_t* samples, hipStream_t stream);
// Upsample + colour-convert `n` images (max_oct_rows = max over images of
// height * ceil(width / 8), the grid's x extent).
void launch_jpeg_color(const uint8_t* samples, const JpegImgDev* imgs, int32_t n, int64_t max_oct_rows,
                       uint8_t* rgb, hipStream_t stream);

}  // namespace mxd
