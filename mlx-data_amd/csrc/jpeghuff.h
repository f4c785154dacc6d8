// jpeghuff.h -- device-side entropy decode of baseline / extended-sequential
// JPEGs (jpeghuff.hip; SURVEY.md §8f f1, "later a device-side decode";
// VERDICT r3 missing 1).  Plain data shared by the host (jpeg.cpp builds the
// tables, hostpath.cpp stages the segments) and the kernel; no HIP headers.
//
// What runs where.  The host parses the markers (jpeg.cpp parse_coefs with
// device entropy), finds the entropy-coded segments of the file's one scan
// (one per restart interval) and, at batch time, copies them unstuffed
// (0xFF 0x00 -> 0xFF, fill bytes dropped) into the staging buffer.  The GPU
// then decodes the Huffman symbols in parallel: each segment is cut into
// subsequences of `sub_bits` bits, one thread each.  A subsequence's decoder
// state at its start (bit position of the first symbol that starts in it,
// block of the MCU, coefficient index) is known only for the first one of a
// segment; the others start from a guess and the states are propagated
// (thread i hands its exit state to thread i + 1) until none changes -- the
// self-synchronisation of Huffman codes makes that take one or two rounds in
// practice, and at most one round per subsequence in any case (Weissenberger
// & Schmidt, "Massively parallel Huffman decoding on GPUs", ICPP 2018, for
// the idea; restated here for JPEG's block / coefficient context).  Block
// counts per subsequence are then prefix-summed, a second decode writes every
// coefficient into the image's planes (the layout jpeg.cpp's host decode
// produces, which jpegdev.hip's IDCT reads), and the DC differences are
// turned into values by per-component prefix sums (reset at every restart).
// libjpeg's "insufficient data" rule is kept: bits past a segment's end read
// as zeros, and once a block has consumed bits past the end the segment's
// remaining MCUs stay zero.
#pragma once

#include <cstdint>

namespace mxd {

// Lookahead bits of the device symbol table (tuning builds: -DMXD_HUFF_LOOK=9,
// the host decoder's): at 11 a code longer than the lookahead -- the branch
// every wave takes when any of its lanes meets one -- is rare.
#ifndef MXD_HUFF_LOOK
#define MXD_HUFF_LOOK 11
#endif
constexpr int kHuffLook = MXD_HUFF_LOOK;
constexpr int kHuffFacLook = 9;  // lookahead of the combined AC table (the host decoder's)
constexpr int kHuffMaxBlocks = 10;  // blocks per MCU (JPEG's limit)
constexpr int kHuffThreads = 1024;  // subsequences per job (one workgroup)

// One derived Huffman table (jdhuff.c jpeg_make_d_derived_tbl), as jpeg.cpp
// builds it for the host decoder.
struct HuffDev {
  uint16_t look[1 << kHuffLook];  // (length << 8) | symbol; 0: code longer than kHuffLook
  int32_t maxcode[18];
  int32_t valoffset[18];
  uint8_t vals[256];
  // AC fast path: value (int16, bits 0..15), run (bits 16..23; 0xFF = end of
  // block, 15 = ZRL), bits to consume (24..31; 0 = take the general path)
  uint32_t fac[1 << kHuffFacLook];
  // The symbol step over the same kHuffLook bits, in this table's class:
  // bits 0..4 the bits a symbol consumes (code + value bits), 5..11 the
  // coefficient-index advance (DC 1; a coefficient run + 1; ZRL 16; EOB 64),
  // 12..15 the value bits; 0: code longer than kHuffLook.
  uint16_t step[1 << kHuffLook];
};
// A step entry from a code's length and symbol (constexpr: host and device).
constexpr uint16_t huff_step_entry(int cls, int len, int sym) {
  return (uint16_t)(((len + (cls ? (sym & 15) : sym)) & 31) |
                    ((cls ? ((sym & 15) != 0 || (sym >> 4) == 15 ? (sym >> 4) + 1 : 64) : 1) << 5) |
                    ((cls ? (sym & 15) : sym) << 12));
}
static_assert(sizeof(HuffDev) % 16 == 0, "HuffDev keeps 16-byte alignment");

// One image of a device entropy-decode launch.
struct HuffImgDev {
  int64_t coef;            // first coefficient of the image's planes (int16 elements of the coefficient buffer)
  int64_t plane[3];        // first coefficient of each component plane, relative to coef
  int32_t bw[3];           // blocks per plane row (MCU-padded grid)
  int32_t tables;          // first HuffDev of the image (index into the launch's table array)
  int32_t ntables;         // HuffDev the image uses (<= 8)
  int32_t bpm;             // blocks per MCU (1 for a single-component scan)
  int32_t mcux;            // MCUs per row (interleaved) / blocks per row of the component proper (single component)
  int32_t interleaved;
  int32_t rst_mcus;        // MCUs per segment (the restart interval; every MCU when 0 restarts)
  int64_t mcus;            // MCUs of the scan
  int8_t blk_comp[kHuffMaxBlocks];  // per MCU block: component (frame index)
  int8_t blk_dc[kHuffMaxBlocks];    // its DC / AC table (index among the image's tables)
  int8_t blk_ac[kHuffMaxBlocks];
  int8_t blk_dx[kHuffMaxBlocks];    // its block offset inside the MCU (component blocks)
  int8_t blk_dy[kHuffMaxBlocks];
  int8_t comp_h[3], comp_v[3];     // sampling factors (blocks per MCU per component)
  int8_t pad[7];
};

// One entropy-coded segment (restart interval) of one image.
struct HuffSegDev {
  int64_t word;     // first 32-bit word of its unstuffed bytes (index into the launch's word buffer)
  int32_t bits;     // data bits (8 x unstuffed bytes); words past ceil(bits / 32) read as zeros
  int32_t img;      // HuffImgDev index
  int64_t mcu0;     // its first MCU
  int32_t mcus;     // its MCUs
  int32_t sub_bits; // bits per subsequence
};

// One workgroup of the launch: segments [seg0, seg0 + nseg) of one image
// (one subsequence length), whose subsequences (ceil(bits / sub_bits) each,
// >= 1) number nsub <= kHuffThreads; their words are staged contiguously
// from segment seg0's first word, words16 x 16 bytes, and are read from LDS
// (lds != 0: they fit the launch's dynamic LDS) or from device memory.
struct HuffJobDev {
  int32_t seg0, nseg, nsub, words16;
  int32_t lds, pad[3];
};
static_assert(sizeof(HuffJobDev) == 32, "HuffJobDev layout");

// Shortest subsequence (bits): a decoder that starts mid-stream needs some
// symbols to fall into step; the launch uses longer ones when a segment
// would otherwise need more than kHuffThreads.
constexpr int kHuffMinBits = 512;

// Dynamic LDS a job needs (its tables and segment records, plus its words
// when they are read from LDS), and the most a job may use.
int64_t jpeg_huff_lds_bytes(int ntables, int nseg, int64_t words);
int64_t jpeg_huff_lds_budget();

// Enqueues the decode of `njobs` jobs (threads: the largest job's
// subsequences; lds_bytes: the largest job's dynamic LDS, its words included
// when it reads them from LDS); coefficient offsets in HuffImgDev are int16
// elements of `coef`, segment words index `words`.  Returns 0, or -1 if the
// launch failed.
int launch_jpeg_huff(const uint32_t* words, const HuffDev* tables, const HuffImgDev* imgs, const HuffSegDev* segs,
                     const HuffJobDev* jobs, int32_t njobs, int32_t threads, int64_t lds_bytes, int16_t* coef,
                     void* stream);

}  // namespace mxd
