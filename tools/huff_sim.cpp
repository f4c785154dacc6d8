// tools/huff_sim.cpp -- diagnostic (not product): a sequential CPU model of
// the device entropy decode's synchronisation (csrc/jpeghuff.hip), used to
// design round 5's phase speculation before writing it in HIP.
//
// Per file: the markers are parsed the product's way (jpeg.cpp parse_coefs
// with device entropy), the segments unstuffed, the device step table built
// (device_table), then the subsequences are synchronised in rounds:
//   plain   every subsequence whose start state changed decodes to its end
//           and hands its exit state on (round 4's kernel);
//   spec    as plain, and while the round's decodes leave threads free, the
//           D subsequences after each changed one also decode every block
//           phase b of the MCU from their current start position and
//           coefficient index; the chain is then walked through those
//           variants as far as the positions and indices agree.
// The write pass decodes every subsequence from its final state; the
// coefficients are compared with the host decoder's (decode_coefs).
//
// Build: g++ -O2 -std=c++17 -Imlx-data_amd/csrc -Iinclude tools/huff_sim.cpp mlx-data_amd/csrc/jpeg.cpp -o tools/huff_sim
// Run:   tools/huff_sim [--sub BITS] [--threads N] [--dmax D] [--spec 0|1] FILE...
#include <algorithm>
#include <array>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <string>
#include <vector>

#include "jpeg.h"
#include "jpeghuff.h"

using namespace mxd;

namespace {

struct State {
  int64_t pos;
  int b, k;
  bool operator==(const State& o) const { return pos == o.pos && b == o.b && k == o.k; }
  bool operator!=(const State& o) const { return !(*this == o); }
};

struct Seg {
  std::vector<uint8_t> bytes;
  int64_t bits;
  int64_t mcu0, mcus;
};

struct Img {
  jpeg::EntropyScan es;
  std::vector<HuffDev> tab;
  std::vector<Seg> segs;
  int bpm;
};

// 64 bits of the segment from bit `pos` (zeros past its end).
uint64_t peek64(const Seg& s, int64_t pos) {
  const int64_t byte = pos >> 3, n = (int64_t)s.bytes.size();
  auto at = [&](int64_t q) -> uint64_t { return q < n ? s.bytes[q] : 0; };
  uint64_t v = 0;
  for (int i = 0; i < 8; i++) v = (v << 8) | at(byte + i);
  const int off = pos & 7;
  if (off) v = (v << off) | (at(byte + 8) >> (8 - off));
  return v;
}

int extend(uint32_t v, int s) { return s == 0 ? 0 : (int)v < (1 << (s - 1)) ? (int)v + ((-1) << s) + 1 : (int)v; }

void long_peek(const HuffDev& t, uint64_t buf, int& len, int& sym) {
  const uint32_t p16 = (uint32_t)(buf >> 48);
  int l = 17;
  for (int ll = 16; ll > kHuffLook; ll--)
    if ((int32_t)(p16 >> (16 - ll)) <= t.maxcode[ll]) l = ll;
  if (l > 16) {
    len = 16;
    sym = 0;
  } else {
    len = l;
    sym = t.vals[((int32_t)(p16 >> (16 - l)) + t.valoffset[l]) & 0xff];
  }
}

// One symbol (jpeghuff.hip Dec::step, the step-table form).  Returns true at
// a block's end; *kk / *v: the coefficient position and value stored.
bool step(const Img& im, const Seg& s, State& st, int* kk = nullptr, int* v = nullptr, int* advp = nullptr) {
  const bool dc = st.k == 0;
  const HuffDev& t = im.tab[dc ? im.es.blk_dc[st.b] : im.es.blk_ac[st.b]];
  const uint64_t buf = peek64(s, st.pos);
  int e = t.step[(uint32_t)(buf >> (64 - kHuffLook))] & 0xffff;  // one symbol a step (the kernel pairs some)
  {
    // code length histogram (diagnostics): the code's length is the step's consumed bits minus the value bits
    int len, sym;
    long_peek(t, buf, len, sym);
    if (e) len = (e & 31) - (e >> 12);
    extern int64_t g_len[18];
    g_len[std::min(len, 17)]++;
  }
  if (!e) {
    int len, sym;
    long_peek(t, buf, len, sym);
    e = huff_step_entry(dc ? 0 : 1, len, sym);
  }
  const int shift = e & 31, adv = (e >> 5) & 127, sz = e >> 12;
  const uint32_t hi = (uint32_t)(buf >> 32);
  const uint32_t raw = sz ? (hi >> (32 - shift)) & ((1u << sz) - 1u) : 0u;
  st.pos += shift;
  if (advp) *advp = adv;
  const int knew = st.k + adv;
  if (kk) *kk = std::min(knew - 1, 63);
  if (v) *v = extend(raw, sz);
  const bool end = knew >= 64;
  st.k = end ? 0 : knew;
  st.b = end ? (st.b + 1 == im.bpm ? 0 : st.b + 1) : st.b;
  return end;
}

struct Sub {
  int seg;
  int64_t start, end;  // end: INT64_MAX for a segment's last subsequence
  bool first, last;
};

// Decodes from `in` until the first symbol boundary at or past `end`; returns the exit, counts steps and blocks.
// *kmax: the largest entry coefficient index for which a decode from the same position and block gives the
// same exit (entries in [1, *kmax]): the first block ends at an EOB that every such index reaches below 64
// (the AC symbols before it advance them alike); -1 when only in.k itself is known to.
State run(const Img& im, const Sub& u, State in, int64_t* steps, int64_t* blocks, int* kmax = nullptr) {
  const Seg& s = im.segs[u.seg];
  State st = in;
  int A = 0;
  bool first = true;
  if (kmax) *kmax = -1;
  while (st.pos < u.end) {
    int adv = 0;
    const bool end = step(im, s, st, nullptr, nullptr, &adv);
    if (first) {
      if (end) {
        first = false;
        if (kmax && in.k >= 1 && adv == 64) *kmax = 63 - A;
      } else {
        A += adv;
      }
    }
    *blocks += end ? 1 : 0;
    ++*steps;
  }
  return st;
}

int64_t g_chg[3] = {0, 0, 0};
int64_t g_len[18] = {0};
int64_t g_pair[4][3] = {{0}};
int64_t g_multi[6][2] = {{0}};
int64_t g_walk[4] = {0, 0, 0, 0};  // walk steps into a variant follower: all, same pos, same k class, accepted  // changes after round 0: all, same position, same position and index

struct PhaseStats;
struct Opts {
  int sub_bits = 512;
  int threads = 1024;
  int dmax = 8;
  int spec = 1;
  int spec_from = 1;  // first round that may speculate
  int krange = 1;
  int phase = 0;      // 1: the anchor / phase-map design; 2: design B (overlap, variants, breaks)
  int overlap = 512;
  int jobs = 0;       // emulate the round-5 kernel's jobs
  int r0_overlap = 0; // rounds: round 0 starts each subsequence this many bits early  // design B: round 0 starts this many bits before each piece     // accept a variant for entry indices its first block's EOB makes equivalent
};

struct Stats {
  int rounds = 0;
  int64_t work_steps = 0;   // symbol steps over all decodes of the rounds
  int64_t crit_steps = 0;   // sum over rounds of the round's longest decode
  int64_t write_steps = 0;
  std::vector<int> heads;   // per round: changed subsequences decoded
  std::vector<int> items;   // per round: decodes (heads + variants)
};

// The synchronisation of one image; returns each subsequence's final start state and blocks before it.
bool sync(const Img& im, const Opts& o, std::vector<Sub>& subs, std::vector<State>& in, std::vector<int64_t>& done,
          Stats& st) {
  subs.clear();
  for (int g = 0; g < (int)im.segs.size(); g++) {
    const int64_t n = std::max<int64_t>(1, (im.segs[g].bits + o.sub_bits - 1) / o.sub_bits);
    for (int64_t j = 0; j < n; j++)
      subs.push_back(Sub{g, j * o.sub_bits, j == n - 1 ? INT64_MAX : (j + 1) * o.sub_bits, j == 0, j == n - 1});
  }
  const int n = (int)subs.size();
  in.assign(n, State{0, 0, 0});
  done.assign(n, 0);
  std::vector<State> out(n);
  for (int i = 0; i < n; i++) in[i].pos = subs[i].start;
  std::vector<char> need(n, 0);
  for (int i = 0; i < n; i++) need[i] = !subs[i].last;
  // round-0 overlap (--r0-overlap W): a subsequence's start state is the
  // state a decoder from a guess W bits earlier reaches at its start
  int64_t r0_extra = 0;
  if (o.r0_overlap > 0)
    for (int i = 0; i < n; i++) {
      if (subs[i].first) continue;
      Sub w = subs[i];
      w.end = subs[i].start;
      int64_t stp = 0, bl = 0;
      in[i] = run(im, w, State{std::max<int64_t>(0, subs[i].start - o.r0_overlap), 0, 0}, &stp, &bl);
      st.work_steps += stp;
      r0_extra = std::max(r0_extra, stp);
    }
  st.crit_steps += r0_extra;
  for (int round = 0;; round++) {
    std::vector<int> heads;
    for (int i = 0; i < n; i++)
      if (need[i]) heads.push_back(i);
    if (heads.empty()) break;
    st.rounds = round + 1;
    // speculation depth: every variant of D followers of each head fits the threads left
    int D = 0;
    if (o.spec && round >= o.spec_from) {
      const int free = o.threads - (int)heads.size();
      D = std::min(o.dmax, std::max(0, free / std::max<int>(1, (int)heads.size() * im.bpm)));
    }
    int64_t crit = 0;
    std::vector<char> decoded(n, 0);
    for (int i : heads) {
      int64_t s = 0, b = 0;
      out[i] = run(im, subs[i], in[i], &s, &b);
      done[i] = b;
      decoded[i] = 1;
      st.work_steps += s;
      crit = std::max(crit, s);
    }
    int items = (int)heads.size();
    // variants: for each head's followers f (not segment firsts, not past the segment's last), every b
    struct Var {
      State out;
      int64_t blocks;
      int kmax;
    };
    std::vector<std::vector<Var>> var(n);
    std::vector<char> is_var(n, 0);
    if (D > 0)
      for (int i : heads)
        for (int d = 1; d <= D && i + d < n; d++) {
          const int f = i + d;
          if (subs[f].first || subs[f].last || need[f] || is_var[f]) break;
          is_var[f] = 1;
          var[f].resize(im.bpm);
          for (int b = 0; b < im.bpm; b++) {
            int64_t s = 0, bl = 0;
            var[f][b].out = run(im, subs[f], State{in[f].pos, b, in[f].k}, &s, &bl, o.krange ? &var[f][b].kmax : nullptr);
            if (!o.krange) var[f][b].kmax = -1;
            var[f][b].blocks = bl;
            st.work_steps += s;
            crit = std::max(crit, s);
            items++;
          }
        }
    st.crit_steps += crit;
    st.heads.push_back((int)heads.size());
    st.items.push_back(items);
    // hand the exits on; walk through the variants
    std::fill(need.begin(), need.end(), 0);
    for (int i : heads) {
      State e = out[i];
      int t = i + 1;
      while (t < n && !subs[t].first) {
        if (is_var[t] && getenv("WALK")) {
          g_walk[0]++;
          if (e.pos == in[t].pos) g_walk[1]++;
          if (e.pos == in[t].pos && (e.k >= 1) == (in[t].k >= 1)) g_walk[2]++;
          if (e.pos == in[t].pos && (e.k == in[t].k || (e.k >= 1 && in[t].k >= 1 && e.k <= var[t][e.b].kmax))) g_walk[3]++;
        }
        if (is_var[t] && e.pos == in[t].pos &&
            (e.k == in[t].k || (e.k >= 1 && in[t].k >= 1 && e.k <= var[t][e.b].kmax))) {
          in[t] = e;
          done[t] = var[t][e.b].blocks;
          out[t] = var[t][e.b].out;
          e = out[t];
          t++;
          continue;
        }
        if (e != in[t]) {
          if (getenv("TRACE") && t == atoi(getenv("TRACE")))
            std::printf("round %d sub %d: (%lld,%d,%d) -> (%lld,%d,%d)  [from head %d, walked %d]\n", round, t,
                        (long long)in[t].pos, in[t].b, in[t].k, (long long)e.pos, e.b, e.k, i, t - i - 1);
          if (round > 0) {
            g_chg[0]++;
            if (e.pos == in[t].pos) g_chg[1]++;
            if (e.pos == in[t].pos && e.k == in[t].k) g_chg[2]++;
          }
          in[t] = e;
          need[t] = !subs[t].last;
        }
        break;
      }
    }
    if (round > 10000) return false;
  }
  return true;
}

// Round-5 design: block-boundary anchors and phase maps instead of rounds.
//   A  each fixed-length piece decodes from a guessed start (the first of a
//      segment from its exact start) past its end to the first block
//      boundary there: anchor P_{i+1} (a true block boundary once the decoder
//      has fallen into step, which ~512 bits give it);
//   B  every piece [P_i, P_{i+1}) decodes from (P_i, b, 0) for every block b
//      of the MCU: phi_i(b) = the block at P_{i+1} if the decode lands there
//      exactly at a block boundary, else none;
//   C  phases composed from the segment start (b = 0): b_{i+1} = phi_i(b_i);
//      a none on that path (P_{i+1} not a true boundary) is repaired by
//      decoding on from the true state to the next anchor that lands
//   D  the write pass (write_check) from (P_i, b_i, 0).
struct PhaseStats {
  int64_t pieces = 0, repairs = 0, repair_rounds = 0, a_steps = 0, b_steps = 0, b_crit = 0;
};

PhaseStats g_ps;

bool phase_sync(const Img& im, const Opts& o, std::vector<Sub>& subs, std::vector<State>& in,
                std::vector<int64_t>& done, Stats& st, PhaseStats& ps) {
  subs.clear();
  in.clear();
  done.clear();
  for (int g = 0; g < (int)im.segs.size(); g++) {
    const Seg& sg = im.segs[g];
    const int64_t n = std::max<int64_t>(1, (sg.bits + o.sub_bits - 1) / o.sub_bits);
    // A: anchors
    std::vector<int64_t> P{0};
    for (int64_t j = 0; j + 1 < n; j++) {
      State stt{j * o.sub_bits, 0, 0};
      const int64_t lim = (j + 1) * o.sub_bits;
      bool blk_end = false;
      while (stt.pos < lim || !blk_end) {
        blk_end = step(im, sg, stt);
        ps.a_steps++;
        if (stt.pos > sg.bits) break;
      }
      if (stt.pos < sg.bits && stt.pos > P.back()) P.push_back(stt.pos);
    }
    const int m = (int)P.size();
    if (getenv("CHECKP")) {
      // the true block boundaries (a sequential decode of the segment)
      std::vector<int64_t> tb;
      State t{0, 0, 0};
      int64_t blocks = 0;
      while (blocks < sg.mcus * im.bpm && t.pos <= sg.bits) {
        if (step(im, sg, t)) {
          blocks++;
          tb.push_back(t.pos);
        }
      }
      int bad = 0;
      for (int i = 1; i < m; i++) bad += !std::binary_search(tb.begin(), tb.end(), P[i]);
      std::printf("segment %d: anchors %d, not true boundaries %d\n", g, m - 1, bad);
    }
    // B: phase maps
    std::vector<std::vector<int>> phi(m, std::vector<int>(im.bpm, -1));
    std::vector<std::vector<int64_t>> blocks(m, std::vector<int64_t>(im.bpm, 0));
    for (int i = 0; i + 1 < m; i++) {
      int64_t crit = 0;
      for (int b = 0; b < im.bpm; b++) {
        State stt{P[i], b, 0};
        int64_t bl = 0, stp = 0;
        while (stt.pos < P[i + 1]) {
          bl += step(im, sg, stt) ? 1 : 0;
          stp++;
        }
        ps.b_steps += stp;
        crit = std::max(crit, stp);
        if (stt.pos == P[i + 1] && stt.k == 0) phi[i][b] = stt.b;
        blocks[i][b] = bl;
      }
      ps.b_crit = std::max(ps.b_crit, crit);
    }
    // C: compose from the segment start; repair breaks
    int b = 0;
    int64_t pos = 0;
    int rounds_here = 0, run_repairs = 0;
    for (int i = 0; i < m; i++) {
      const bool last = i + 1 == m;
      subs.push_back(Sub{g, pos, last ? INT64_MAX : P[i + 1], subs.empty() || subs.back().seg != g, last});
      in.push_back(State{pos, b, 0});
      if (last) {
        done.push_back(0);
        break;
      }
      if (pos == P[i] && phi[i][b] >= 0) {
        done.push_back(blocks[i][b]);
        b = phi[i][b];
        pos = P[i + 1];
        run_repairs = 0;
        continue;
      }
      // repair: the true decode from (pos, b, 0) on to the first block boundary at or past P[i+1]
      ps.repairs++;
      if (++run_repairs > rounds_here) rounds_here = run_repairs;
      State stt{pos, b, 0};
      int64_t bl = 0;
      bool blk_end = false;
      while (stt.pos < P[i + 1] || !blk_end) {
        blk_end = step(im, sg, stt);
        bl += blk_end ? 1 : 0;
        if (stt.pos > sg.bits + 64) break;
      }
      subs.back().end = stt.pos;
      done.push_back(bl);
      b = stt.b;
      pos = stt.pos;
      // the next piece starts at pos (past its anchor when it did not land on it)
      if (i + 1 < m && pos != P[i + 1]) {
        // skip anchors the repair passed
        while (i + 2 < m && P[i + 2] <= pos) {
          i++;
        }
        if (i + 1 < m && pos > P[i + 1]) P[i + 1] = pos;  // phi of piece i+1 no longer applies (pos != its P)
      }
    }
    ps.repair_rounds += rounds_here;
    ps.pieces += m;
  }
  st.rounds = 1;
  return true;
}

// Round-5 design B: round 0 decodes every piece from a guess W bits before
// its start (the decoder falls into step over the overlap); round 1 decodes
// every piece from round 0's exit position and coefficient index in every
// block phase b; the walk from each segment's start then follows the phase
// variants while positions and indices agree; where they do not (a break),
// the next round decodes that piece from its now known true entry and the
// walk goes on.  Rounds = 2 + the breaks one after another along a segment.
struct DesignB {
  int64_t pieces = 0, breaks = 0, max_breaks = 0, r0_steps = 0, r1_steps = 0, r1_crit = 0, brk_steps = 0;
} g_db;

bool design_b(const Img& im, const Opts& o, std::vector<Sub>& subs, std::vector<State>& in,
              std::vector<int64_t>& done, Stats& st) {
  subs.clear();
  in.clear();
  done.clear();
  int64_t file_breaks = 0;
  for (int g = 0; g < (int)im.segs.size(); g++) {
    const Seg& sg = im.segs[g];
    const int64_t n = std::max<int64_t>(1, (sg.bits + o.sub_bits - 1) / o.sub_bits);
    std::vector<Sub> S;
    for (int64_t j = 0; j < n; j++)
      S.push_back(Sub{g, j * o.sub_bits, j == n - 1 ? INT64_MAX : (j + 1) * o.sub_bits, j == 0, j == n - 1});
    // round 0: exits from a guess W bits early (the first piece from the exact start)
    std::vector<State> X(n);
    for (int64_t j = 0; j + 1 < n; j++) {
      State t{j == 0 ? 0 : std::max<int64_t>(0, S[j].start - o.overlap), 0, 0};
      int64_t stp = 0, bl = 0;
      X[j] = run(im, S[j], t, &stp, &bl);
      g_db.r0_steps += stp;
    }
    // round 1: variants of every piece j >= 1 from (X[j-1].pos, b, X[j-1].k)
    struct Var {
      State out;
      int64_t blocks;
      int kmax;
    };
    std::vector<std::vector<Var>> V(n);
    for (int64_t j = 1; j + 1 < n; j++) {
      V[j].resize(im.bpm);
      int64_t crit = 0;
      for (int b = 0; b < im.bpm; b++) {
        int64_t stp = 0, bl = 0;
        V[j][b].out = run(im, S[j], State{X[j - 1].pos, b, X[j - 1].k}, &stp, &bl, &V[j][b].kmax);
        V[j][b].blocks = bl;
        g_db.r1_steps += stp;
        crit = std::max(crit, stp);
      }
      g_db.r1_crit = std::max(g_db.r1_crit, crit);
    }
    // the walk, with a break round wherever a piece's true entry is not among its variants
    State e{0, 0, 0};
    int64_t brk = 0;
    for (int64_t j = 0; j < n; j++) {
      subs.push_back(S[j]);
      in.push_back(e);
      if (S[j].last) {
        done.push_back(0);
        break;
      }
      const bool var_ok = j >= 1 && e.pos == X[j - 1].pos &&
                          (e.k == X[j - 1].k || (e.k >= 1 && X[j - 1].k >= 1 && e.k <= V[j][e.b].kmax));
      if (var_ok) {
        done.push_back(V[j][e.b].blocks);
        e = V[j][e.b].out;
        continue;
      }
      int64_t stp = 0, bl = 0;
      State x = run(im, S[j], e, &stp, &bl);
      done.push_back(bl);
      if (j >= 1) {
        brk++;
        g_db.brk_steps += stp;
      }
      e = x;
    }
    g_db.breaks += brk;
    file_breaks = std::max(file_breaks, brk);
    g_db.pieces += n;
  }
  g_db.max_breaks = std::max(g_db.max_breaks, file_breaks);
  st.rounds = 2 + (int)file_breaks;
  return true;
}

// Round-5 kernel emulation (--jobs 1): hostpath.cpp's job planning and
// jpeghuff.hip decode_job, job after job (the look-back sees the previous
// job's publication), each job's rounds as the workgroup runs them.  Checks
// the kernel's logic on the CPU; returns false on a mismatch.
int kZigzagNat2(int z) {
  static const int nat[64] = {0,  1,  8,  16, 9,  2,  3,  10, 17, 24, 32, 25, 18, 11, 4,  5,  12, 19, 26, 33, 40, 48,
                              41, 34, 27, 20, 13, 6,  7,  14, 21, 28, 35, 42, 49, 56, 57, 50, 43, 36, 29, 22, 15, 23,
                              30, 37, 44, 51, 58, 59, 52, 45, 38, 31, 39, 46, 53, 60, 61, 54, 47, 55, 62, 63};
  return nat[z];
}

struct JobStats {
  int64_t jobs = 0, fixes = 0, max_rounds = 0;
} g_js;

bool emulate_jobs(const Img& im, const Opts& o, const std::vector<int16_t>& host, const jpeg::CoefInfo& hinfo) {
  const int sb = o.sub_bits;
  const int nseg = (int)im.segs.size();
  std::vector<int64_t> nsub(nseg), sub_first;
  int64_t N = 0;
  for (int g = 0; g < nseg; g++) {
    nsub[g] = std::max<int64_t>(1, (im.segs[g].bits + sb - 1) / sb);
    sub_first.push_back(N);
    N += nsub[g];
  }
  sub_first.push_back(N);
  const int64_t cap = kHuffThreads - kHuffWarm;
  const int64_t njob = (N + cap - 1) / cap;
  std::vector<int64_t> cuts{0};
  for (int64_t q = 1; q < njob; q++) {
    int64_t cut = q * N / njob;
    const int64_t sgi = std::upper_bound(sub_first.begin(), sub_first.end(), cut) - sub_first.begin() - 1;
    if (cut - sub_first[sgi] <= 32 && sub_first[sgi] > cuts.back()) cut = sub_first[sgi];
    cuts.push_back(cut);
  }
  cuts.push_back(N);
  std::vector<int16_t> coef(host.size(), 0);
  struct Pub {
    State st;
    int64_t blocks;
    int dc[3];
  } pub{};
  for (size_t q = 0; q + 1 < cuts.size(); q++) {
    g_js.jobs++;
    const int64_t a0 = cuts[q], b0 = cuts[q + 1];
    const int64_t sa = std::upper_bound(sub_first.begin(), sub_first.end(), a0) - sub_first.begin() - 1;
    const int64_t ja = a0 - sub_first[sa];
    const int warm = (int)std::min<int64_t>(kHuffWarm, ja);
    const bool pred = ja > 0;
    const int n = (int)(b0 - a0 + warm);
    // job-local subsequences
    struct L {
      int seg;
      int64_t j;
      bool first, seg_last, own, job_last;
      int64_t start, end;
    };
    std::vector<L> sub(n);
    for (int t = 0; t < n; t++) {
      const int64_t gidx = a0 - warm + t;
      const int sg = (int)(std::upper_bound(sub_first.begin(), sub_first.end(), gidx) - sub_first.begin() - 1);
      L& l = sub[t];
      l.seg = sg;
      l.j = gidx - sub_first[sg];
      l.first = l.j == 0;
      l.seg_last = l.j == nsub[sg] - 1;
      l.own = t >= warm;
      l.job_last = t == n - 1;
      l.start = l.j * sb;
      l.end = l.seg_last ? INT64_MAX : l.start + sb;
    }
    std::vector<State> in(n), out(n);
    std::vector<int64_t> done(n, 0);
    for (int t = 0; t < n; t++) in[t] = State{sub[t].start, 0, 0};
    auto rounds = [&](std::vector<char> need, int fixed) {
      int r = 0;
      for (;; r++) {
        bool any = false;
        for (int t = 0; t < n; t++)
          if (need[t]) {
            any = true;
            int64_t stp = 0, bl = 0;
            Sub u{sub[t].seg, sub[t].start, sub[t].end, sub[t].first, sub[t].seg_last};
            out[t] = run(im, u, in[t], &stp, &bl);
            done[t] = bl;
          }
        if (!any) break;
        std::vector<char> nn(n, 0);
        for (int t = 1; t < n; t++) {
          if (sub[t].first || t == fixed) continue;
          if (out[t - 1] != in[t]) {
            in[t] = out[t - 1];
            nn[t] = !sub[t].seg_last;
          }
        }
        need = nn;
      }
      g_js.max_rounds = std::max<int64_t>(g_js.max_rounds, r);
    };
    std::vector<char> need(n);
    for (int t = 0; t < n; t++) need[t] = !sub[t].seg_last;
    rounds(need, -1);
    if (pred) {
      if (pub.st != in[warm]) {
        g_js.fixes++;
        in[warm] = pub.st;
        std::vector<char> nd(n, 0);
        nd[warm] = !sub[warm].seg_last;
        rounds(nd, warm);
      }
    }
    // blocks and write pass, DC
    std::vector<int64_t> g(n, 0);
    std::vector<std::array<int, 3>> dcs(n, {0, 0, 0});
    int64_t acc = 0;
    int cur_seg = -1;
    for (int t = warm; t < n; t++) {
      if (sub[t].seg != cur_seg) {
        cur_seg = sub[t].seg;
        acc = (pred && sub[t].seg == sub[warm].seg) ? pub.blocks : im.segs[cur_seg].mcu0 * im.bpm;
      }
      g[t] = acc;
      if (!sub[t].seg_last) acc += done[t];
      if (t == n - 1 && !sub[t].seg_last) {
        // publication: exit, block index (dc below)
      }
    }
    Pub np{};
    if (!sub[n - 1].seg_last) {
      np.st = out[n - 1];
      np.blocks = g[n - 1] + done[n - 1];
    }
    // write pass
    std::vector<std::array<int64_t, 2>> dcr(n, {-1, -1});
    for (int t = warm; t < n; t++) {
      const Seg& sg = im.segs[sub[t].seg];
      State st = in[t];
      int64_t gg = g[t];
      const int64_t g1 = (sg.mcu0 + sg.mcus) * im.bpm;
      while (!(st.pos >= sub[t].end || gg >= g1 || (st.b == 0 && st.k == 0 && st.pos > sg.bits))) {
        const int bj = (int)(gg % im.bpm);
        const int ci = im.es.blk_comp[bj];
        const jpeg::CoefPlane& cp = hinfo.comp[ci];
        int64_t m = gg / im.bpm, bx, by;
        if (im.es.interleaved) {
          by = (m / im.es.mcux) * cp.v + im.es.blk_dy[bj];
          bx = (m % im.es.mcux) * cp.h + im.es.blk_dx[bj];
        } else {
          by = gg / im.es.mcux;
          bx = gg % im.es.mcux;
        }
        int16_t* blk = coef.data() + cp.off + (by * cp.bw + bx) * 64;
        const bool dc = st.k == 0;
        int kk, v;
        const bool fin = step(im, sg, st, &kk, &v);
        if (dc) {
          dcs[t][ci] += v;
          if (dcr[t][0] < 0) dcr[t][0] = gg;
          dcr[t][1] = gg + 1;
          blk[0] = (int16_t)v;
        } else {
          blk[kZigzagNat2(kk)] = (int16_t)v;
        }
        if (fin) gg++;
      }
    }
    // DC prefix per segment, fix-up
    std::array<int, 3> base{0, 0, 0};
    cur_seg = -1;
    for (int t = warm; t < n; t++) {
      if (sub[t].seg != cur_seg) {
        cur_seg = sub[t].seg;
        for (int c = 0; c < 3; c++) base[c] = (pred && sub[t].seg == sub[warm].seg) ? pub.dc[c] : 0;
      }
      std::array<int, 3> pr = base;
      if (dcr[t][0] >= 0)
        for (int64_t b = dcr[t][0]; b < dcr[t][1]; b++) {
          const int bj = (int)(b % im.bpm);
          const int ci = im.es.blk_comp[bj];
          const jpeg::CoefPlane& cp = hinfo.comp[ci];
          int64_t m = b / im.bpm, bx, by;
          if (im.es.interleaved) {
            by = (m / im.es.mcux) * cp.v + im.es.blk_dy[bj];
            bx = (m % im.es.mcux) * cp.h + im.es.blk_dx[bj];
          } else {
            by = b / im.es.mcux;
            bx = b % im.es.mcux;
          }
          int16_t* d = coef.data() + cp.off + (by * cp.bw + bx) * 64;
          pr[ci] += d[0];
          d[0] = (int16_t)pr[ci];
        }
      for (int c = 0; c < 3; c++) base[c] += dcs[t][c];
    }
    for (int c = 0; c < 3; c++) np.dc[c] = base[c];
    pub = np;
  }
  return coef == host;
}

bool load(const char* path, Img& im, std::vector<int16_t>& host_coef, std::vector<int64_t>& plane_off,
          jpeg::CoefInfo& hinfo) {
  std::ifstream f(path, std::ios::binary);
  std::vector<uint8_t> data((std::istreambuf_iterator<char>(f)), std::istreambuf_iterator<char>());
  std::string err;
  jpeg::Coefs* c = jpeg::parse_coefs(data.data(), data.size(), true, &err);
  if (!c) return false;
  const jpeg::CoefInfo info = jpeg::coef_info(c);
  if (!info.entropy_pending) {
    jpeg::free_coefs(c);
    return false;
  }
  im.es = jpeg::entropy_scan(c);
  im.bpm = im.es.bpm;
  im.tab.resize(im.es.ntables);
  for (int t = 0; t < im.es.ntables; t++) jpeg::device_table(c, im.es.table_class[t], im.es.table_id[t], &im.tab[t]);
  im.segs.resize(im.es.nseg);
  const int64_t rst = im.es.restart_interval > 0 ? im.es.restart_interval : im.es.mcus;
  for (int g = 0; g < im.es.nseg; g++) {
    Seg& s = im.segs[g];
    s.bytes.resize(im.es.seg_end[g] - im.es.seg_begin[g] + 16);
    const int64_t nb = jpeg::unstuff(im.es.data + im.es.seg_begin[g], im.es.data + im.es.seg_end[g], s.bytes.data());
    s.bytes.resize(nb);
    s.bits = 8 * nb;
    s.mcu0 = g * rst;
    s.mcus = std::min(rst, im.es.mcus - s.mcu0);
  }
  jpeg::Coefs* h = jpeg::decode_coefs(data.data(), data.size(), &err);
  hinfo = jpeg::coef_info(h);
  host_coef.assign(hinfo.coef, hinfo.coef + hinfo.coef_count);
  plane_off.clear();
  for (int k = 0; k < hinfo.ncomp; k++) plane_off.push_back(hinfo.comp[k].off);
  jpeg::free_coefs(h);
  jpeg::free_coefs(c);
  return true;
}

constexpr int kZigzagNat[64] = {0,  1,  8,  16, 9,  2,  3,  10, 17, 24, 32, 25, 18, 11, 4,  5,  12, 19, 26, 33, 40, 48,
                                41, 34, 27, 20, 13, 6,  7,  14, 21, 28, 35, 42, 49, 56, 57, 50, 43, 36, 29, 22, 15, 23,
                                30, 37, 44, 51, 58, 59, 52, 45, 38, 31, 39, 46, 53, 60, 61, 54, 47, 55, 62, 63};

// Write pass from the synchronised states; compares with the host decoder.
bool write_check(const Img& im, const std::vector<Sub>& subs, const std::vector<State>& in,
                 const std::vector<int64_t>& done, const std::vector<int16_t>& host, const jpeg::CoefInfo& hinfo,
                 Stats& st) {
  std::vector<int16_t> coef(host.size(), 0);
  std::vector<int> pred(3, 0);
  int64_t g_before = 0;
  int last_seg = -1;
  for (size_t i = 0; i < subs.size(); i++) {
    const Sub& u = subs[i];
    const Seg& s = im.segs[u.seg];
    if (u.seg != last_seg) {
      g_before = 0;
      last_seg = u.seg;
      std::fill(pred.begin(), pred.end(), 0);
    }
    int64_t g = s.mcu0 * im.bpm + g_before;
    const int64_t g1 = (s.mcu0 + s.mcus) * im.bpm;
    State stt = in[i];
    bool ins = true;
    while (stt.pos < u.end && g < g1 && !(stt.b == 0 && stt.k == 0 && stt.pos > s.bits)) {
      const int bj = (int)(g % im.bpm);
      const int ci = im.es.blk_comp[bj];
      int64_t m = g / im.bpm, bx, by;
      const jpeg::CoefPlane& cp = hinfo.comp[ci];
      if (im.es.interleaved) {
        by = (m / im.es.mcux) * cp.v + im.es.blk_dy[bj];
        bx = (m % im.es.mcux) * cp.h + im.es.blk_dx[bj];
      } else {
        by = g / im.es.mcux;
        bx = g % im.es.mcux;
      }
      int16_t* blk = coef.data() + cp.off + (by * cp.bw + bx) * 64;
      const bool dc = stt.k == 0;
      int kk, v;
      const int64_t p0 = stt.pos;
      const bool fin = step(im, s, stt, &kk, &v);
      st.write_steps++;
      {
        // multi-symbol model: greedy steps of up to M symbols of one block whose bits fit W
        extern int64_t g_multi[6][2];
        static int acc_bits[6] = {0}, acc_n[6] = {0};
        static const int Wv[6] = {11, 12, 12, 13, 14, 16}, Mv[6] = {2, 2, 3, 3, 3, 4};
        const int len = (int)(stt.pos - p0);
        for (int m = 0; m < 6; m++) {
          // does this symbol join the open step?
          if (acc_n[m] > 0 && !dc && acc_bits[m] + len <= Wv[m] && acc_n[m] < Mv[m]) {
            acc_bits[m] += len;
            acc_n[m]++;
          } else {
            g_multi[m][0]++;  // a new step
            acc_bits[m] = len <= Wv[m] ? len : 99;
            acc_n[m] = 1;
          }
          if (fin || dc) acc_n[m] = dc && !fin ? acc_n[m] : 0;  // a block's end closes the step
          if (dc) acc_n[m] = 0;  // DC tables hold single symbols
          g_multi[m][1]++;
        }
      }
      {
        // pairing model (--pairs): greedy pairs of consecutive symbols of one block whose bits fit L
        extern int64_t g_pair[4][3];
        static int prev_len = -1, prev_dc = 0;
        const int len = (int)(stt.pos - p0);
        for (int L = 0; L < 4; L++) (void)L;
        if (prev_len >= 0) {
          // the previous symbol waits for a partner: this one (same block: the previous did not end it)
          for (int L = 0; L < 4; L++) {
            const int win = 10 + L;
            if (prev_len + len <= win) g_pair[L][prev_dc ? 1 : 0]++;
          }
          prev_len = -1;
        } else if (!fin) {
          prev_len = len;
          prev_dc = dc;
        }
        if (fin) prev_len = -1;
        g_pair[0][2]++;
      }
      if (dc) {
        pred[ci] += v;
        blk[0] = (int16_t)pred[ci];
      } else {
        blk[kZigzagNat[kk]] = (int16_t)v;
      }
      if (fin) g++;
    }
    (void)ins;
    if (i < done.size()) g_before += u.last ? 0 : done[i];
  }
  return coef == host;
}

}  // namespace

int main(int argc, char** argv) {
  Opts o;
  std::vector<const char*> files;
  for (int i = 1; i < argc; i++) {
    if (!std::strcmp(argv[i], "--sub")) o.sub_bits = std::atoi(argv[++i]);
    else if (!std::strcmp(argv[i], "--threads")) o.threads = std::atoi(argv[++i]);
    else if (!std::strcmp(argv[i], "--dmax")) o.dmax = std::atoi(argv[++i]);
    else if (!std::strcmp(argv[i], "--spec")) o.spec = std::atoi(argv[++i]);
    else if (!std::strcmp(argv[i], "--spec-from")) o.spec_from = std::atoi(argv[++i]);
    else if (!std::strcmp(argv[i], "--krange")) o.krange = std::atoi(argv[++i]);
    else if (!std::strcmp(argv[i], "--phase")) o.phase = std::atoi(argv[++i]);
    else if (!std::strcmp(argv[i], "--overlap")) o.overlap = std::atoi(argv[++i]);
    else if (!std::strcmp(argv[i], "--jobs")) o.jobs = std::atoi(argv[++i]);
    else if (!std::strcmp(argv[i], "--r0-overlap")) o.r0_overlap = std::atoi(argv[++i]);
    else files.push_back(argv[i]);
  }
  int nf = 0, bad = 0, maxr = 0;
  double rounds = 0, work = 0, crit = 0, write = 0, subs_total = 0;
  std::vector<double> heads_sum(64, 0), items_sum(64, 0);
  for (const char* p : files) {
    Img im;
    std::vector<int16_t> host;
    std::vector<int64_t> poff;
    jpeg::CoefInfo hinfo;
    if (!load(p, im, host, poff, hinfo)) continue;
    std::vector<Sub> subs;
    std::vector<State> in;
    std::vector<int64_t> done;
    Stats st;
    if (o.jobs) {
      const bool ok = emulate_jobs(im, o, host, hinfo);
      if (!ok) {
        std::printf("%s: JOBS MISMATCH\n", p);
        bad++;
      }
      nf++;
      continue;
    }
    PhaseStats ps;
    const bool ok_sync = o.phase == 2   ? design_b(im, o, subs, in, done, st)
                         : o.phase == 1 ? phase_sync(im, o, subs, in, done, st, ps)
                                        : sync(im, o, subs, in, done, st);
    g_ps.pieces += ps.pieces;
    g_ps.repairs += ps.repairs;
    g_ps.repair_rounds = std::max(g_ps.repair_rounds, ps.repair_rounds);
    g_ps.a_steps += ps.a_steps;
    g_ps.b_steps += ps.b_steps;
    g_ps.b_crit = std::max(g_ps.b_crit, ps.b_crit);
    if (!ok_sync) {
      std::printf("%s: no convergence\n", p);
      bad++;
      continue;
    }
    const bool ok = write_check(im, subs, in, done, host, hinfo, st);
    if (!ok) {
      std::printf("%s: MISMATCH\n", p);
      bad++;
    }
    nf++;
    rounds += st.rounds;
    maxr = std::max(maxr, st.rounds);
    work += st.work_steps;
    crit += st.crit_steps;
    write += st.write_steps;
    subs_total += subs.size();
    for (size_t r = 0; r < st.heads.size() && r < 64; r++) {
      heads_sum[r] += st.heads[r];
      items_sum[r] += st.items[r];
    }
  }
  if (!nf) return 1;
  if (o.jobs) {
    std::printf("jobs emulation: files %d bad %d, jobs %lld, predecessor fixes %lld, most rounds %lld\n", nf, bad,
                (long long)g_js.jobs, (long long)g_js.fixes, (long long)g_js.max_rounds);
    return bad ? 2 : 0;
  }
  if (o.phase == 2)
    std::printf("design B: pieces/file %.0f, breaks/file %.2f, most breaks in a file %lld, round 0 %.2f passes, "
                "round 1 %.2f passes (longest variant decode %lld steps), break decodes %.3f passes\n",
                (double)g_db.pieces / nf, (double)g_db.breaks / nf, (long long)g_db.max_breaks, g_db.r0_steps / write,
                g_db.r1_steps / write, (long long)g_db.r1_crit, g_db.brk_steps / write);
  if (o.phase == 1)
    std::printf("phase design: pieces/file %.0f, repairs/file %.2f (longest run %lld), A steps %.2f passes, B steps "
                "%.2f passes, longest B piece decode %lld steps\n",
                (double)g_ps.pieces / nf, (double)g_ps.repairs / nf, (long long)g_ps.repair_rounds,
                (double)g_ps.a_steps / write, (double)g_ps.b_steps / write, (long long)g_ps.b_crit);
  std::printf("files %d bad %d | subs/file %.0f | rounds avg %.2f max %d | work/write %.2f passes | critical "
              "steps/file %.0f (write pass %.0f per sub)\n",
              nf, bad, subs_total / nf, rounds / nf, maxr, work / write, crit / nf, write / subs_total);
  std::printf("changes after round 0: %lld, same pos %.1f %%, same pos+k %.1f %%\n", (long long)g_chg[0],
              100.0 * g_chg[1] / std::max<int64_t>(1, g_chg[0]), 100.0 * g_chg[2] / std::max<int64_t>(1, g_chg[0]));
  {
    int64_t tot = 0, over[4] = {0, 0, 0, 0};
    for (int l = 0; l < 18; l++) {
      tot += g_len[l];
      for (int q = 0; q < 4; q++) over[q] += l > 9 + q ? g_len[l] : 0;
    }
    std::printf("codes longer than 9/10/11/12 bits: %.3f / %.3f / %.3f / %.3f %% of symbols\n", 100.0 * over[0] / tot,
                100.0 * over[1] / tot, 100.0 * over[2] / tot, 100.0 * over[3] / tot);
  }
  if (g_walk[0])
    std::printf("walk: %lld steps, same pos %.1f %%, same k class %.1f %%, accepted %.1f %%\n", (long long)g_walk[0],
                100.0 * g_walk[1] / g_walk[0], 100.0 * g_walk[2] / g_walk[0], 100.0 * g_walk[3] / g_walk[0]);
  for (int L = 0; L < 4; L++)
    std::printf("pairs in %d bits: AC-AC %.1f %%, DC-AC %.1f %% of symbols paired\n", 10 + L,
                200.0 * g_pair[L][0] / g_pair[0][2], 200.0 * g_pair[L][1] / g_pair[0][2]);
  {
    static const int Wv[6] = {11, 12, 12, 13, 14, 16}, Mv[6] = {2, 2, 3, 3, 3, 4};
    for (int m = 0; m < 6; m++)
      std::printf("steps per symbol, <= %d symbols in %d bits: %.3f\n", Mv[m], Wv[m],
                  (double)g_multi[m][0] / g_multi[m][1]);
  }
  std::printf("heads per round:");
  for (int r = 0; r < 20 && heads_sum[r] > 0; r++) std::printf(" %.0f/%.0f", heads_sum[r] / nf, items_sum[r] / nf);
  std::printf("\n");
  return bad ? 2 : 0;
}
