// band.h -- the row-stream ("band") kernel of the fused resize + crop stage.
//
// One 256-thread workgroup runs one UNIT = (image, band of output rows, strip
// of output columns).  The source rows the band's taps read are streamed into
// an LDS ring by LDS-DMA (buffer_load_dwordx4 ... lds, 1 KiB per wave
// instruction, no VGPR staging), several output rows ahead; the vertical pass
// reads them from LDS and scatters each converted row into the open output
// rows (f32 FMA, tap order), the finished vertical row goes back to LDS as
// f32, and the horizontal pass gives each thread one output pixel (C taps
// chains), rounds like stbir and stores it.  Arithmetic is identical to
// wave.hip's (vertical first, byte units, f32 FMA chains from 0 in tap order,
// stbir's encode, exact q/255).
//
// The ring works in GROUPS: group g brings the source rows that become new
// for output row g - P of the band (P prologue groups collect the first
// output row's taps), at most DB rows.  Group g's rows live in LDS area
// g mod (la + 1) until its vertical pass is done; the finished vertical row
// then overwrites that area as f32 (an area holds max(DB, 4) row slots of
// NQ KiB, i.e. NQ KiB of floats), and the horizontal pass reads it one step
// later.  Two workgroup barriers per output row; the LDS-DMA of group g + la
// is issued right after the second one.
#pragma once

#include <cstdint>

#include "resample.h"

namespace mxd {

// Geometry classes: the horizontal tap bucket T fixes the most new source
// rows per output row the kernel accepts (DB) and the accumulator slots S.
struct BandClass {
  int32_t taps, db, s;
};
constexpr BandClass kBandClasses[] = {{2, 1, 3}, {4, 2, 2}, {6, 3, 2}, {8, 4, 2},
                                      {10, 5, 2}, {12, 6, 2}, {17, 9, 2}, {25, 13, 2}};
constexpr int kBandMaxNq = 4;          // source window of a strip row <= 4 KiB
constexpr int kBandThreads = 256;      // threads per workgroup = output pixels per strip row (max)
constexpr int kBandChunk = 1024;       // bytes per LDS-DMA wave instruction
constexpr int kBandEntryWords = 4;     // schedule entry: source row, S <= 3 weights

struct BandCfg {
  int32_t channels, f32, nq, taps, s, db;
  int32_t la;  // groups loaded ahead (>= 1)
  int32_t nimgs, nunits;
  int32_t per_img;  // units of every image when all images have the same count, else 0
};

// LDS bytes of one workgroup of cfg (ring of la + 1 areas + 1 KiB sink).
int band_lds_bytes(const BandCfg& cfg);
bool band_has_kernel(const BandCfg& cfg);
// Workgroups of cfg the device runs at once (occupancy x CUs), 0 if unknown.
int band_capacity(const BandCfg& cfg, int device);
int launch_band(const BandCfg& cfg, const ImgDev* imgs, void* stream);

}  // namespace mxd
