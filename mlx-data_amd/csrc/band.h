// band.h -- the row-stream ("band") kernel of the fused resize + crop stage.
//
// A UNIT = (image, band of output rows, strip of output columns).  The kernel
// is persistent: a grid of as many 256-thread workgroups as the device holds
// at once, workgroup w running units w, w + G, w + 2G, ... (G = grid size)
// back to back as ONE stream of groups, so the units the device works on at
// any moment are neighbouring bands of a few images (their halo rows shared
// in one XCD's L2, few DRAM pages and TLB entries open), and a unit's start
// costs no pipeline refill: the next unit's rows are already in flight while
// the current one finishes.
//
// The source rows a unit's taps read are streamed into an LDS ring by LDS-DMA
// (buffer_load_dwordx4 ... lds, 1 KiB per wave instruction, no VGPR
// staging), la groups ahead; the vertical pass reads them from LDS and
// scatters each converted row into the open output rows (f32 FMA, tap order),
// a finished vertical row goes back to LDS as f32, and the horizontal pass
// gives each thread one output pixel (C taps chains), rounds like stbir and
// stores it.  Arithmetic is identical to wave.hip's (vertical first, byte
// units, f32 FMA chains from 0 in tap order, stbir's encode, exact q/255).
//
// GROUPS: a band's schedule (band_plan.h) lists groups of at most DB source
// rows; the rows new for an output row fill one or more consecutive groups,
// the last of which COMPLETES that row (flag), so any downscale ratio runs
// (a 16:1 ratio brings 16 new rows per output row: two groups of 8).  Group
// g's rows live in LDS area g mod (la + 1) until its vertical pass is done;
// a completed vertical row then overwrites that area as f32 (an area holds
// max(DB, 4) row slots of NQ KiB, i.e. NQ KiB of floats) and the horizontal
// pass reads it one step later.  Two workgroup barriers per group; the
// LDS-DMA of group g + la is issued right after the second one.
#pragma once

#include <cstdint>

#include "resample.h"

namespace mxd {

// Kernel classes: horizontal tap bucket T, source rows per group DB,
// accumulator slots S (open output rows a source row's weights reach).
struct BandClass {
  int32_t taps, db, s;
};
constexpr BandClass kBandClasses[] = {{2, 1, 3},  {4, 2, 2},  {6, 3, 2},  {8, 4, 2}, {10, 5, 2},
                                      {12, 6, 2}, {17, 5, 2}, {25, 6, 2}, {32, 8, 2}};
constexpr int kBandMaxNq = 4;          // source window of a strip row <= 4 KiB
constexpr int kBandThreads = 256;      // threads per workgroup = output pixels per strip row (max)
constexpr int kBandChunk = 1024;       // bytes per LDS-DMA wave instruction
constexpr int kBandEntryWords = 4;     // schedule entry: source row, S <= 3 weights; group header: flags
constexpr int kBandRowDone = 1;        // group header flag: the group completes the oldest open output row

struct BandCfg {
  int32_t channels, f32, nq, taps, s, db;
  int32_t la;  // groups loaded ahead (>= 1)
  int32_t nimgs, nunits;
  int32_t per_img;  // units of every image when all images have the same count, else 0
  int32_t grid;     // workgroups (<= nunits; each runs units w, w + grid, ...)
};

// LDS bytes of one workgroup of cfg (ring of la + 1 areas + 1 KiB sink).
int band_lds_bytes(const BandCfg& cfg);
bool band_has_kernel(const BandCfg& cfg);
// Workgroups of cfg the device runs at once (occupancy x CUs), 0 if unknown.
int band_capacity(const BandCfg& cfg, int device);
// unit_img: image index of every unit (nullptr when cfg.per_img > 0).
int launch_band(const BandCfg& cfg, const ImgDev* imgs, const int32_t* unit_img, void* stream);

}  // namespace mxd
