// jpeghuff.h -- device-side entropy decode of baseline / extended-sequential
// JPEGs (jpeghuff.hip; SURVEY.md §8f f1, "later a device-side decode";
// VERDICT r3 missing 1, r4 next 2).  Plain data shared by the host (jpeg.cpp
// builds the tables, hostpath.cpp plans the jobs and stages the segments) and
// the kernel; no HIP headers.
//
// What runs where.  The host parses the markers (jpeg.cpp parse_coefs with
// device entropy), finds the entropy-coded segments of the file's one scan
// (one per restart interval) and, at batch time, copies them unstuffed
// (0xFF 0x00 -> 0xFF, fill bytes dropped) into the staging buffer.  The GPU
// then decodes the Huffman symbols in parallel: every segment is cut into
// subsequences of `sub_bits` bits, one thread each.  A subsequence's decoder
// state at its start (bit position of the first symbol that starts in it,
// block of the MCU, coefficient index) is known only for the first one of a
// segment; the others start from a guess and the states are propagated
// (thread i hands its exit state to thread i + 1) until none changes -- the
// self-synchronisation of Huffman codes (Weissenberger & Schmidt, "Massively
// parallel Huffman decoding on GPUs", ICPP 2018, for the idea; restated here
// for JPEG's block / coefficient context).  Block counts per subsequence are
// then prefix-summed, a second decode writes every coefficient into the
// image's planes (the layout jpeg.cpp's host decode produces, which
// jpegdev.hip's IDCT reads), and the DC differences are turned into values by
// per-component prefix sums (reset at every restart).  libjpeg's
// "insufficient data" rule is kept: bits past a segment's end read as zeros,
// and once a block has consumed bits past the end the segment's remaining
// MCUs stay zero.
//
// Jobs (round 5).  A workgroup decodes one JOB: a run of at most
// kHuffThreads consecutive subsequences of one image, across segment
// boundaries.  An image of more subsequences is cut into several jobs, so a
// large photo without restart markers spreads over as many workgroups (CUs)
// as its length asks for.  A job that starts inside a segment first decodes
// up to kHuffWarm of the subsequences before its own (its warm-up): starting
// from a guess there, its decoder falls into step with the data before it
// reaches its own subsequences, so its own start state is almost always the
// true one already.  The true one comes from the previous job of the segment
// (a decoupled look-back: jobs take their indices from a ticket counter in
// the order their workgroups start, and each publishes its exit state,
// block count and DC sums when it has them); a job whose own start state
// differs from it re-synchronises from the true state, so the result never
// depends on the warm-up having been long enough.
#pragma once

#include <cstdint>

namespace mxd {

constexpr int kHuffLook = 11;       // lookahead bits of the device step table
constexpr int kHuffLong = 1024;     // step entries for codes longer than kHuffLook (16-bit patterns)
constexpr int kHuffMaxBlocks = 10;  // blocks per MCU (JPEG's limit)
constexpr int kHuffThreads = 1024;  // subsequences per job (one workgroup)
constexpr int kHuffWarm = 24;       // warm-up subsequences of a job that starts inside a segment

// One derived Huffman table (jdhuff.c jpeg_make_d_derived_tbl) in the device
// layout, as jpeg.cpp device_table builds it: the symbol STEP of every bit
// pattern -- bits 0..4 the bits a symbol consumes (code + value bits), 5..11
// the coefficient-index advance (DC 1; a coefficient run + 1; ZRL 16; EOB
// 64), 12..15 the value bits -- over kHuffLook bits (0: a longer code), and
// for the longer codes over the top kHuffLong 16-bit patterns, indexed from
// 65536 - kHuffLong (the kernel's constant base) (canonical codes: every
// code longer than kHuffLook bits lies in the top range of 16-bit patterns,
// from `long_base` on; patterns no code starts map to "16 bits, symbol 0",
// the host decoder's corrupt-code rule).  A table whose long codes reach
// below the top kHuffLong patterns keeps long_base = 65536, an empty second
// table, and is searched (maxcode / valoffset / vals).  Bits 16..31 of an
// entry are the step of a PAIR: in an AC table's kHuffLook-bit entries, when
// the pattern holds two whole symbols, value bits included, the first of
// which is not an EOB, bits 16..20 the bits both consume, 21..27 the index
// advance of both, 28..31 the second's value bits; otherwise the single
// symbol's own bits and advance again (value bits 0), so the decoder takes
// "the pair" whenever the first symbol leaves its block open (jpeghuff.hip
// Dec::step).
struct HuffDev {
  uint32_t step[1 << kHuffLook];
  uint32_t step_long[kHuffLong];
  int32_t long_base;
  int32_t search;  // 1: the two lookups do not cover every pattern (the launch takes the searching kernel)
  int32_t maxcode[18];
  int32_t valoffset[18];
  uint8_t vals[256];
  int32_t pad1[2];
};
// A step entry from a code's length and symbol (constexpr: host and device).
constexpr uint16_t huff_step_entry(int cls, int len, int sym) {
  return (uint16_t)(((len + (cls ? (sym & 15) : sym)) & 31) |
                    ((cls ? ((sym & 15) != 0 || (sym >> 4) == 15 ? (sym >> 4) + 1 : 64) : 1) << 5) |
                    ((cls ? (sym & 15) : sym) << 12));
}
// The table entry of a single symbol (its bits and advance repeated as the pair's).
constexpr uint32_t huff_step_single(uint16_t e) { return e ? (uint32_t)e | (uint32_t)(e & 0xfff) << 16 : 0u; }
// The table entry of a pair (first: a single entry of a symbol other than EOB, second: the next one's).
constexpr uint32_t huff_step_pair(uint16_t first, uint16_t second) {
  return (uint32_t)first |
         (uint32_t)(((first & 31) + (second & 31)) | (((first >> 5) & 127) + ((second >> 5) & 127)) << 5 |
                    (second >> 12) << 12)
             << 16;
}
static_assert(sizeof(HuffDev) % 16 == 0, "HuffDev keeps 16-byte alignment");

// One image of a device entropy-decode launch.
struct HuffImgDev {
  int64_t coef;            // first coefficient of the image's planes (int16 elements of the coefficient buffer)
  int64_t plane[4];        // first coefficient of each component plane, relative to coef (4: CMYK / YCCK)
  int32_t bw[4];           // blocks per plane row (MCU-padded grid)
  int32_t tables;          // first HuffDev of the image (index into the launch's table array)
  int32_t ntables;         // HuffDev the image uses (<= 8)
  int32_t bpm;             // blocks per MCU (1 for a single-component scan)
  int32_t mcux;            // MCUs per row (interleaved) / blocks per row of the component proper (single component)
  int32_t interleaved;
  int32_t rst_mcus;        // MCUs per segment (the restart interval; every MCU when 0 restarts)
  int32_t sub_bits;        // bits per subsequence (a multiple of 32)
  int64_t mcus;            // MCUs of the scan
  int8_t blk_comp[kHuffMaxBlocks];  // per MCU block: component (frame index)
  int8_t blk_dc[kHuffMaxBlocks];    // its DC / AC table (index among the image's tables)
  int8_t blk_ac[kHuffMaxBlocks];
  int8_t blk_dx[kHuffMaxBlocks];    // its block offset inside the MCU (component blocks)
  int8_t blk_dy[kHuffMaxBlocks];
  int8_t comp_h[4], comp_v[4];     // sampling factors (blocks per MCU per component)
};

// One entropy-coded segment (restart interval) of one image.
struct HuffSegDev {
  int64_t word;     // first 32-bit word of its unstuffed bytes (index into the launch's word buffer)
  int32_t bits;     // data bits (8 x unstuffed bytes); words past ceil(bits / 32) read as zeros
  int32_t img;      // HuffImgDev index
  int64_t mcu0;     // its first MCU
  int32_t mcus;     // its MCUs
  int32_t nsub;     // its subsequences: max(1, ceil(bits / sub_bits))
};

// One job (workgroup): subsequences [sub0, ...) of segment seg0 onwards, nsub
// of them (the first `warm` of them its warm-up, inside seg0), across nseg
// segments.  Its words are staged contiguously from word0 (segment seg0's
// first word + sub0 * sub_bits / 32), words16 x 16 bytes, read from LDS (lds
// != 0) or from device memory.  pred != 0: its first own subsequence continues
// a segment the previous job (index - 1) decodes the start of.
struct HuffJobDev {
  int64_t word0;
  int32_t seg0, nseg, sub0, nsub, warm, words16;
  int32_t lds, pred;
};
static_assert(sizeof(HuffJobDev) == 40, "HuffJobDev layout");

// What a job publishes for the next one (device memory, zeroed before the
// launch): 64-bit words, each written once with bit 63 set (so every word
// is its own ready flag and no fence orders them): [0] its last own
// subsequence's exit state (bit position in bits 0..31, 3 x the block of
// the MCU in 32..39, coefficient index in 40..47), [1] the block index there, [2..4]
// the DC-difference sums of that segment up to there, per component.
#ifdef MXD_HUFF_STAMPS
constexpr int kHuffPubWords = 32;  // diagnostic build: words 8.. hold the job's phase stamps (jpeghuff.hip)
#else
constexpr int kHuffPubWords = 8;
#endif
struct HuffPubDev {
  uint64_t w[kHuffPubWords];
};
constexpr uint64_t kHuffValid = (uint64_t)1 << 63;
static_assert(sizeof(HuffPubDev) == 8 * kHuffPubWords, "HuffPubDev layout");

// Launch control (device memory, staged zero before the launch): the job
// ticket counter, an error word (1: a job gave up waiting for its
// predecessor) and, when not null, a page-locked host word the error is
// also written to (the host reads it after the launch with no copy back).
struct HuffCtlDev {
  int32_t ticket, error;
  int32_t* err_host;
};
static_assert(sizeof(HuffCtlDev) == 16, "HuffCtlDev layout");

// Shortest subsequence (bits): a decoder that starts mid-stream needs some
// symbols to fall into step.
constexpr int kHuffMinBits = 512;

// Dynamic LDS a job needs (its tables and segment records, plus its words
// when they are read from LDS), and the most a job may use.
int64_t jpeg_huff_lds_bytes(int ntables, int nseg, int64_t words);
int64_t jpeg_huff_lds_budget();

// Enqueues the decode of `njobs` jobs (threads: the largest job's
// subsequences; lds_bytes: the largest job's dynamic LDS, its words included
// when it reads them from LDS); coefficient offsets in HuffImgDev are int16
// elements of `coef`, segment words index `words`; pub (njobs records) and ctl
// must be zero; search: some table has HuffDev::search set.  Returns 0, or -1
// if the launch failed.
int launch_jpeg_huff(const uint32_t* words, const HuffDev* tables, const HuffImgDev* imgs, const HuffSegDev* segs,
                     const HuffJobDev* jobs, int32_t njobs, int32_t threads, int64_t lds_bytes, HuffPubDev* pub,
                     HuffCtlDev* ctl, int16_t* coef, bool search, void* stream);


}  // namespace mxd
