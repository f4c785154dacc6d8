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
  const int16_t* coef;  // nullptr while the entropy decode is pending (decoded on the device)
  int64_t coef_count;
  CoefPlane comp[4];
  bool device_ok;   // grey, YCbCr, RGB, CMYK, YCCK (not lossless): the device kernels can finish it
  bool entropy_pending;  // the coefficients come from the device entropy decode (jpeghuff.h)
};

// Entropy decode (every error decode() reports, from here); nullptr + *err.
Coefs* decode_coefs(const uint8_t* data, size_t size, std::string* err);
// Markers only when the file qualifies for the device entropy decode
// (device_entropy; jpeghuff.h): baseline / extended sequential, one scan
// carrying every component (grey, YCbCr or RGB), DC tables with categories
// <= 15, entropy-coded data ending at a marker, restart markers in sequence.
// Any other file is entropy-decoded here as by decode_coefs.  The file is
// copied: `data` need not outlive the call.
Coefs* parse_coefs(const uint8_t* data, size_t size, bool device_entropy, std::string* err);
// parse_coefs of the file at `path`, read straight into the Coefs' own copy
// (one open, a read sized by fstat, no intermediate buffer).  nullptr and
// *not_jpeg when the file does not start with the JPEG signature; nullptr
// with *err on any other failure (open / read / parse, or not a regular
// file) -- callers needing the reference's exact messages rerun their general
// path then.
Coefs* load_coefs(const char* path, bool device_entropy, bool* not_jpeg, std::string* err);
void free_coefs(Coefs* c);
CoefInfo coef_info(const Coefs* c);
// Host finish into height rows of width*3 bytes at dst_stride (thread-safe);
// a pending entropy decode runs on the host first.
bool finish(const Coefs* c, uint8_t* dst, int64_t dst_stride, std::string* err);

// ---- device entropy decode (pending coefficients)
struct EntropyScan {
  int nseg;                      // entropy-coded segments (restart intervals)
  const int64_t* seg_begin;      // raw bytes of segment s: [seg_begin[s], seg_end[s]) of `data`
  const int64_t* seg_end;
  const int64_t* seg_bytes;      // its unstuffed bytes (what unstuff writes)
  const uint8_t* data;           // the file
  int64_t mcus;                  // MCUs of the scan
  int restart_interval;          // MCUs per segment (0: one segment)
  int interleaved;               // 0: one component, blocks in raster order of the component proper
  int mcux;                      // MCUs per row / blocks per row of the component (single component)
  int bpm;                       // blocks per MCU
  int blk_comp[10], blk_dx[10], blk_dy[10], blk_dc[10], blk_ac[10];  // per MCU block (tables: see ntables)
  int ntables;                   // distinct tables the scan uses (blk_dc / blk_ac index them)
  int table_class[8], table_id[8];  // 0 DC / 1 AC, DHT index
};
EntropyScan entropy_scan(const Coefs* c);
// The derived table `table_id` of class `cls` in the device layout (jpeghuff.h
// HuffDev) into huff_dev (nullptr: only made ready).  Returns its serial in a
// small per-thread cache of built tables: two calls on one thread that
// return the same serial gave the same table.
uint64_t device_table(const Coefs* c, int cls, int table_id, void* huff_dev);
// Unstuffed bytes of the raw segment [b, e) (0xFF 0x00 -> 0xFF, fill 0xFF
// bytes dropped) into dst (>= e - b bytes); returns their count.
int64_t unstuff(const uint8_t* b, const uint8_t* e, uint8_t* dst);

}  // namespace jpeg
}  // namespace mxd
