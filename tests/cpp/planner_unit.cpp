// planner_unit.cpp -- CPU unit tests of the fused stage's host planning
// (mlx-data_amd/csrc/plan.cpp, band_plan.cpp) through capi_internal.h, linked
// against the in-tree libmxd_amd.so; no device call.  Built and run by
// tests/test_planner_unit.py.  Prints "ok <n>" or the first failure.
#include <cmath>
#include <cstdio>
#include <cstdlib>

#include "capi_internal.h"

using namespace mxd::capi;

static int g_checks = 0;
#define CHECK(c)                                                     \
  do {                                                               \
    g_checks++;                                                      \
    if (!(c)) {                                                      \
      std::printf("FAIL %s:%d: %s\n", __FILE__, __LINE__, #c);       \
      std::exit(1);                                                  \
    }                                                                \
  } while (0)

static mxd_image center(int sw, int sh, int size, int crop, bool f32) {
  mxd_image m{};
  int64_t rw = 0, rh = 0, cx = 0, cy = 0;
  mxd_resize_smallest_side_dims(sw, sh, size, &rw, &rh);
  mxd_center_crop_origin(rw, rh, crop, crop, &cx, &cy);
  static uint8_t dummy[64];
  m.src = dummy;
  m.src_stride = ((int64_t)sw * 3 + 15) / 16 * 16;
  m.src_w = sw;
  m.src_h = sh;
  m.channels = 3;
  m.resize_w = (int32_t)rw;
  m.resize_h = (int32_t)rh;
  m.crop_x = (int32_t)cx;
  m.crop_y = (int32_t)cy;
  m.crop_w = crop;
  m.crop_h = crop;
  m.dst = reinterpret_cast<void*>(uintptr_t(1) << 20);
  m.dst_stride = (int64_t)crop * 3 * (f32 ? 4 : 1);
  return m;
}

static ImgPlan plan(const mxd_image& m) {
  ImgPlan p;
  CHECK(host_tables().get(0, m.src_w, m.resize_w, &p.xt) == MXD_OK);
  CHECK(host_tables().get(0, m.src_h, m.resize_h, &p.yt) == MXD_OK);
  return p;
}

// band_rows: the fewest "rounds" of `capacity` units whose band height stays
// within the cap, units never above rounds * capacity, at least one row.
static void test_band_rows() {
  auto units = [](const std::vector<std::pair<int32_t, int32_t>>& s, int32_t ty) {
    int64_t u = 0;
    for (auto& x : s) u += (int64_t)x.first * ((x.second + std::min(ty, x.second) - 1) / std::min(ty, x.second));
    return u;
  };
  const std::vector<std::pair<int32_t, int32_t>> c2(256, {1, 224});
  CHECK(band_rows(c2, 1024, 64) == 56);  // one round: 4 bands x 256 images
  CHECK(units(c2, 56) == 1024);
  CHECK(band_rows(c2, 1024, 16) == 14);  // 4 rounds of 16 bands
  CHECK(units(c2, 14) == 4096);
  for (int cap : {1, 7, 100, 1024, 4096})
    for (int mx : {8, 16, 64, 128}) {
      std::vector<std::pair<int32_t, int32_t>> mixed;
      for (int i = 0; i < 37; i++) mixed.push_back({1 + i % 3, 1 + (i * 53) % 400});
      const int32_t ty = band_rows(mixed, cap, mx);
      CHECK(ty >= 1);
      const int64_t u = units(mixed, ty);
      const int64_t rounds = (u + cap - 1) / cap;
      CHECK(ty <= std::max(mx, 8) || ty >= 400);
      // no smaller height fits the same rounds
      if (ty > 8) CHECK(units(mixed, ty - 1) > rounds * cap || ty - 1 < 8);
    }
}

// plan_wave: C2 takes a scatter wave kernel; a 12 MP photo takes the 24-tap
// bucket with a depth-12 schedule, a 48 MP one (31:1) none.
static void test_plan_wave() {
  const mxd_image c2 = center(1280, 960, 256, 224, true);
  ImgPlan p = plan(c2);
  plan_wave(c2, whole(c2), 1, MXD_F32_DIV255, p);
  CHECK(p.wave);
  CHECK(p.kind == 2);  // scatter
  CHECK(p.s == 2 && p.dmax == 4);
  CHECK(p.nstrips >= 1 && p.tx * p.nstrips >= 224);
  const mxd_image big = center(4032, 3024, 256, 224, true);
  ImgPlan q = plan(big);
  plan_wave(big, whole(big), 1, MXD_F32_DIV255, q);
  CHECK(q.wave && q.kind == 2 && q.bucket == 24 && q.dmax == 12 && q.s == 2);
  const mxd_image huge = center(8000, 6000, 256, 224, true);
  ImgPlan h = plan(huge);
  plan_wave(huge, whole(huge), 1, MXD_F32_DIV255, h);
  CHECK(!h.wave);
  // an odd row stride leaves the wave kernels (4-byte aligned rows only)
  mxd_image odd = c2;
  odd.src_stride = 1280 * 3 + 1;
  ImgPlan r = plan(odd);
  plan_wave(odd, whole(odd), 1, MXD_F32_DIV255, r);
  CHECK(!r.wave);
}

// plan_band + band_schedule: class, strips, and a schedule whose groups bring
// every tap row of every output row exactly once per band, complete the rows
// in order, and carry each row's weights.
static void test_band_schedule(int sw, int sh, int ty) {
  const mxd_image m = center(sw, sh, 256, 224, true);
  ImgPlan p = plan(m);
  plan_band(m, whole(m), 1, p);
  CHECK(p.band);
  const mxd::AxisView yv = axis_view(*p.yt);
  std::vector<int32_t> w;
  int32_t bw = 0;
  const int32_t min_groups = p.bp.la + 2;
  CHECK(mxd::band_schedule(yv, m.crop_y, m.crop_h, ty, p.bp.db, p.bp.s, min_groups, &w, &bw));
  const int E = mxd::kBandEntryWords, gw = (1 + p.bp.db) * E;
  const int nb = (m.crop_h + ty - 1) / ty;
  CHECK((int64_t)w.size() == (int64_t)nb * bw);
  for (int b = 0; b < nb; b++) {
    const int32_t* band = w.data() + (size_t)b * bw;
    const int ng = band[0];
    CHECK(ng >= min_groups && E + ng * gw <= bw);
    const int y0 = b * ty, n = std::min(ty, m.crop_h - y0);
    std::vector<double> sum(n, 0.0);
    std::vector<int> seen(n, 0);
    int done = 0;
    for (int g = 0; g < ng; g++) {
      const int32_t* gr = band + E + g * gw;
      for (int j = 0; j < p.bp.db; j++) {
        const int32_t* e = gr + (1 + j) * E;
        if (e[0] < 0) continue;
        for (int s = 0; s < p.bp.s; s++) {
          float wt;
          std::memcpy(&wt, &e[1 + s], 4);
          if (wt == 0.0f) continue;
          const int u = done + s;
          CHECK(u < n);
          const int r = e[0], f = yv.first[m.crop_y + y0 + u];
          CHECK(r >= f && r < f + yv.count[m.crop_y + y0 + u]);
          CHECK(wt == yv.w[(size_t)(m.crop_y + y0 + u) * yv.width + (r - f)]);
          sum[u] += wt;
          seen[u]++;
        }
      }
      if (gr[0] & mxd::kBandRowDone) done++;
    }
    CHECK(done == n);
    for (int u = 0; u < n; u++) {
      // nonzero taps of the row, each once
      int nz = 0;
      for (int k = 0; k < yv.count[m.crop_y + y0 + u]; k++)
        nz += yv.w[(size_t)(m.crop_y + y0 + u) * yv.width + k] != 0.0f;
      CHECK(seen[u] == nz);
      CHECK(std::fabs(sum[u] - 1.0) < 1e-4);
    }
  }
}

int main() {
  test_band_rows();
  test_plan_wave();
  for (int ty : {1, 3, 8, 14, 16, 224}) {
    test_band_schedule(1280, 960, ty);   // 3.75:1, one group per row
    test_band_schedule(4032, 3024, ty);  // 11.8:1, two groups per row
    test_band_schedule(6000, 4000, ty);  // 15.6:1
    test_band_schedule(300, 200, ty);    // upsampling, rows with no new source row
  }
  std::printf("ok %d\n", g_checks);
  return 0;
}
