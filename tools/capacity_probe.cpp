// capacity_probe.cpp -- what the occupancy API reports for the wave kernel
// each workload's first image plans (blocks per CU, VGPRs, LDS per block),
// and the capacity the planner derives from it.  Built and run by
// tools/r03_capacity.sh on the GPU box.
#include <cstdio>

#include "capi_internal.h"

using namespace mxd::capi;

int main() {
  struct W { const char* name; int sw, sh, size, crop; bool f32; } ws[] = {
      {"c2", 1280, 960, 256, 224, true}, {"c4", 500, 375, 256, 224, true}, {"c5", 3840, 2160, 512, 448, false},
      {"c6", 4032, 3024, 256, 224, true}, {"c7", 6000, 4000, 256, 224, true}, {"c3_480p", 640, 480, 256, 224, false}};
  static uint8_t dummy[64];
  for (const W& w : ws) {
    mxd_image m{};
    int64_t rw = 0, rh = 0, cx = 0, cy = 0;
    mxd_resize_smallest_side_dims(w.sw, w.sh, w.size, &rw, &rh);
    mxd_center_crop_origin(rw, rh, w.crop, w.crop, &cx, &cy);
    m.src = dummy;
    m.src_stride = ((int64_t)w.sw * 3 + 15) / 16 * 16;
    m.src_w = w.sw;
    m.src_h = w.sh;
    m.channels = 3;
    m.resize_w = (int32_t)rw;
    m.resize_h = (int32_t)rh;
    m.crop_x = (int32_t)cx;
    m.crop_y = (int32_t)cy;
    m.crop_w = m.crop_h = w.crop;
    m.dst = reinterpret_cast<void*>(uintptr_t(1) << 20);
    m.dst_stride = (int64_t)w.crop * 3 * (w.f32 ? 4 : 1);
    ImgPlan p;
    tables().get(0, m.src_w, m.resize_w, &p.xt);
    tables().get(0, m.src_h, m.resize_h, &p.yt);
    plan_wave(m, whole(m), w.f32 ? 1 : 0, w.f32 ? MXD_F32_DIV255 : MXD_U8, p);
    const mxd::WaveCfg cfg{3, w.f32 ? 1 : 0, p.bucket, 0, 0, p.kind, p.s, p.dmax, p.q, p.shift, p.pp};
    int blocks = -1, vgprs = -1, lds = -1;
    const int wpb = mxd::wave_kernel_info(cfg, 0, &blocks, &vgprs, &lds);
    std::printf("{\"workload\": \"%s\", \"waves_per_block\": %d, \"api_blocks_per_cu\": %d, \"vgprs\": %d, "
                "\"lds_per_block\": %d, \"capacity\": %d}\n",
                w.name, wpb, blocks, vgprs, lds, mxd::wave_capacity(cfg, 0));
  }
  return 0;
}
