/*
 * oracle/stbir_oracle.c -- TEST INFRASTRUCTURE ONLY.
 *
 * CPU restatement of the mlx-data image hot path used as the parity checker
 * for the HIP kernels.  Only tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline leg may load this library; the product path never does.
 *
 * What is restated (reference = /root/reference, mlx-data 0.2.0):
 *   - core::image::scale             mlx/data/core/image/ImageTransform.cpp:33-39
 *   - ImageResizeSmallestSide        mlx/data/op/ImageTransform.cpp:78-94
 *   - core::image::resize            mlx/data/core/image/ImageTransform.cpp:41-62
 *       -> stbir_resize_uint8_linear (stb_image_resize2.h, nothings/stb@f0569113,
 *          pinned at CMakeLists.txt:19-26; NOT vendored, NOT present here) with
 *          STBIR_FILTER_TRIANGLE forced for up- and down-sampling
 *          (ImageTransform.cpp:7-9), STBIR_EDGE_CLAMP, uint8 linear.
 *   - ImageCenterCrop / core::image::crop / array::sub
 *                                    op/ImageTransform.cpp:115-126,
 *                                    core/image/ImageTransform.cpp:64-73,
 *                                    Array.cpp:544-583
 *   - core::image::hflip             core/image/ImageTransform.cpp:123-140
 *   - array::batch (fill pad + copy) Array.cpp:465-498
 *   - x.astype("float32") / 255      benchmarks/comparative/caltech101/mlx_data.py:46
 *   - core::image::rotate / affine   core/image/ImageTransform.cpp:75-121
 *   - core::image::channel_reduction core/image/ImageTransform.cpp:142-180
 *       (+ op::ImageChannelReduction presets, op/ImageTransform.cpp:362-392)
 *
 * Parity status: crop / hflip / batch / normalize are pinned bit-exact against
 * the reference's own Array.cpp compiled by oracle/Makefile (oracle/_ref).
 * The resize ARITHMETIC is "parity unpinned" by the reference: stb_image_resize2
 * is a FetchContent dependency absent from this container and the reference has
 * no image tests.  It restates stbir 2.x semantics and is
 * cross-checked against two independent implementations of the same filter
 * (torch antialiased bilinear in f32, Pillow BILINEAR) in tests/test_oracle.py.
 *
 * Arithmetic follows stbir: decode p*(1/255), f32 weights, f32 accumulation
 * (mul then add, no FMA: build with -ffp-contract=off), horizontal pass first,
 * encode (uint8)trunc(clamp(v*255+0.5)).
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

/* stbir__small_float: 2^-120, used to kill denormal weights. */
#define ORC_SMALL ((float)1 / (1 << 20) / (1 << 20) / (1 << 20) / (1 << 20) / (1 << 20) / (1 << 20))

static float orc_tri(float x) {
  if (x < 0.0f) x = -x;
  if (x <= 1.0f) return 1.0f - x;
  return 0.0f;
}

static int orc_gcd(int a, int b) {
  while (b) {
    int t = a % b;
    a = b;
    b = t;
  }
  return a;
}

/* stbir__insert_coeff restated: accumulate a folded (edge-clamped) tap. */
static void orc_insert(int* n0, int* n1, float* c, int px, float v, int cw) {
  if (px <= *n1) {
    if (px < *n0) {
      if (*n1 - px + 1 <= cw) {
        int o = *n0 - px, j;
        for (j = *n1 - *n0; j >= 0; j--) c[j + o] = c[j];
        for (j = 1; j < o; j++) c[j] = 0.0f;
        c[0] = v;
        *n0 = px;
      }
    } else {
      c[px - *n0] += v;
    }
  } else if (px - *n0 + 1 <= cw) {
    int j, e = px - *n0;
    for (j = *n1 - *n0 + 1; j < e; j++) c[j] = 0.0f;
    c[e] = v;
    *n1 = px;
  }
}

static int orc_clamp_px(int n, int size) {
  if (n < 0) return 0;
  if (n >= size) return size - 1;
  return n;
}

/*
 * Per-axis coefficient table, output pixels 0..out_size-1.
 * coeffs is out_size x cw floats (row per output); n0/n1 are inclusive input
 * ranges after edge folding.  Returns 0, or -1 if cw is too small.
 */
int orc_axis_coeffs(int in_size, int out_size, int cw, int* n0, int* n1, float* coeffs) {
  if (in_size <= 0 || out_size <= 0 || cw <= 0) return -1;
  memset(coeffs, 0, sizeof(float) * (size_t)out_size * (size_t)cw);
  if (in_size == out_size) { /* stbir picks point sampling: identity */
    for (int i = 0; i < out_size; i++) {
      n0[i] = n1[i] = i;
      coeffs[(size_t)i * cw] = 1.0f;
    }
    return 0;
  }
  const double scale_d = (double)out_size / (double)in_size;
  const float scale = (float)scale_d;
  const float inv_scale = (float)(1.0 / scale_d);
  const int g = orc_gcd(out_size, in_size);
  const int num = out_size / g, den = in_size / g;
  const int polyphase = num < out_size;
  const int end = polyphase ? num : out_size;

  if (scale >= 1.0f) {
    /* gather upsample: stbir__calculate_coefficients_for_gather_upsample */
    const float radius = 1.0f * scale;
    for (int n = 0; n < end; n++) {
      float* c = coeffs + (size_t)n * cw;
      float out_center = (float)n + 0.5f;
      float in_center_of_out = out_center * inv_scale;
      float in_lo = (out_center - radius) * inv_scale;
      float in_hi = (out_center + radius) * inv_scale;
      int first = (int)floorf(in_lo + 0.5f);
      int last = (int)floorf(in_hi - 0.5f);
      if (last < first) last = first;
      if (last - first + 1 > cw) last = first + cw - 1;
      int lnz = -1;
      for (int i = 0; i <= last - first; i++) {
        float in_px_center = (float)(i + first) + 0.5f;
        float v = orc_tri(in_center_of_out - in_px_center);
        if (v < ORC_SMALL && v > -ORC_SMALL) {
          if (i == 0) {
            ++first;
            i--;
            continue;
          }
          v = 0.0f;
        } else {
          lnz = i;
        }
        c[i] = v;
      }
      n0[n] = first;
      n1[n] = lnz + first;
    }
  } else {
    /* gather downsample: stbir__calculate_coefficients_for_gather_downsample */
    const float in_radius = 1.0f * inv_scale;
    const int margin = ((int)ceilf(1.0f * 2.0f / scale)) / 2;
    int first_out_inited = -1;
    for (int in_px = -margin; in_px < in_size + margin; in_px++) {
      float in_center = (float)in_px + 0.5f;
      float out_center_of_in = in_center * scale;
      float out_lo = (in_center - in_radius) * scale;
      float out_hi = (in_center + in_radius) * scale;
      int of = (int)floorf(out_lo + 0.5f);
      int ol = (int)floorf(out_hi - 0.5f);
      if (of < 0) of = 0;
      if (ol >= out_size) ol = out_size - 1;
      if (of > ol) continue;
      if (polyphase) {
        if (of == num) break;
        if (ol >= num) ol = num - 1;
      }
      for (int i = 0; i <= ol - of; i++) {
        float out_px_center = (float)(i + of) + 0.5f;
        float v = orc_tri(out_px_center - out_center_of_in) * scale;
        if (v < ORC_SMALL && v > -ORC_SMALL) v = 0.0f;
        int o = i + of;
        float* c = coeffs + (size_t)o * cw;
        if (o > first_out_inited) {
          first_out_inited = o;
          n0[o] = n1[o] = in_px;
          c[0] = v;
        } else {
          if (c[0] == 0.0f) n0[o] = in_px;
          n1[o] = in_px;
          if (in_px - n0[o] >= cw) return -1;
          c[in_px - n0[o]] = v;
        }
      }
    }
  }

  /* normalise each output's weights to sum to 1 (stbir cleanup / normalize) */
  for (int n = 0; n < end; n++) {
    float* c = coeffs + (size_t)n * cw;
    int e = n1[n] - n0[n];
    float total = 0.0f;
    for (int i = 0; i <= e; i++) total += c[i];
    if (total < ORC_SMALL && total > -ORC_SMALL) {
      n1[n] = n0[n];
      c[0] = 0.0f;
    } else if (total < 1.0f - ORC_SMALL || total > 1.0f + ORC_SMALL) {
      float fs = 1.0f / total;
      for (int i = 0; i <= e; i++) c[i] *= fs;
    }
  }

  /* polyphase: outputs repeat every `num` with the input shifted by `den` */
  if (polyphase) {
    for (int n = num; n < out_size; n++) {
      n0[n] = n0[n - num] + den;
      n1[n] = n1[n - num] + den;
      memcpy(coeffs + (size_t)n * cw, coeffs + (size_t)(n - num) * cw, sizeof(float) * (size_t)cw);
    }
  }

  /* clamp edges: fold out-of-range taps onto pixel 0 / in_size-1 */
  for (int n = 0; n < out_size; n++) {
    float* c = coeffs + (size_t)n * cw;
    if (n0[n] < 0) {
      float* src = c - (n0[n] + 1);
      for (int i = -1; i > n0[n]; i--) orc_insert(&n0[n], &n1[n], c, orc_clamp_px(i, in_size), *src--, cw);
      int save_n0 = n0[n];
      float save_c = src[0];
      n0[n] = 0;
      for (int i = 0; i <= n1[n]; i++) c[i] = c[i - save_n0];
      for (int i = n1[n] + 1; i < cw; i++) c[i] = 0.0f;
      orc_insert(&n0[n], &n1[n], c, orc_clamp_px(save_n0, in_size), save_c, cw);
    }
    if (n1[n] > in_size - 1) {
      int start = n0[n], endi = n1[n];
      n1[n] = in_size - 1;
      for (int i = in_size; i <= endi; i++) orc_insert(&n0[n], &n1[n], c, orc_clamp_px(i, in_size), c[i - start], cw);
      for (int i = n1[n] - n0[n] + 1; i < cw; i++) c[i] = 0.0f;
    }
    /* trim zero weights at both ends */
    while (n1[n] > n0[n] && c[0] == 0.0f) {
      memmove(c, c + 1, sizeof(float) * (size_t)(n1[n] - n0[n]));
      c[n1[n] - n0[n]] = 0.0f;
      n0[n]++;
    }
    while (n1[n] > n0[n] && c[n1[n] - n0[n]] == 0.0f) n1[n]--;
  }
  return 0;
}

/* Width of the coefficient rows orc_axis_coeffs needs for (in -> out). */
int orc_axis_width(int in_size, int out_size) {
  if (in_size <= 0 || out_size <= 0) return -1;
  if (in_size == out_size) return 1;
  double s = (double)out_size / (double)in_size;
  int w = (s >= 1.0) ? 4 : (int)ceil(2.0 / s) + 3;
  return w;
}

/* core::image::scale + ImageResizeSmallestSide: target dims (lround, double). */
int orc_resize_smallest_side_dims(int64_t w, int64_t h, int64_t size, int64_t* tw, int64_t* th) {
  if (size <= 0) return -1;
  double scale = (h > w) ? (double)size / (double)w : (double)size / (double)h;
  *tw = lround(scale * (double)w);
  *th = lround(scale * (double)h);
  return 0;
}

/*
 * stbir_resize_uint8_linear restated (triangle filter, clamp edges, packed
 * strides).  channels 1..4; with rgba_weighted (c = 4, the STBIR_RGBA layout
 * core::image::resize passes, ImageTransform.cpp:49-58) colours are
 * multiplied by their alpha after decode and divided by the filtered alpha
 * before encode (left as they are when that alpha is below stbir's tiny
 * float) -- SURVEY.md Appendix A item 9, a restatement (stb is absent):
 * parity unpinned.  Horizontal pass first into an f32 intermediate, then
 * vertical.
 */
int orc_resize_u8_layout(const uint8_t* src, int w, int h, int c, uint8_t* dst, int dw, int dh, int rgba_weighted) {
  if (w <= 0 || h <= 0 || dw <= 0 || dh <= 0 || c < 1 || c > 4) return -1;
  const int alpha = c == 4 && rgba_weighted;
  const int cwx = orc_axis_width(w, dw), cwy = orc_axis_width(h, dh);
  int* x0 = (int*)malloc(sizeof(int) * (size_t)dw * 2);
  int* y0 = (int*)malloc(sizeof(int) * (size_t)dh * 2);
  float* wx = (float*)malloc(sizeof(float) * (size_t)dw * cwx);
  float* wy = (float*)malloc(sizeof(float) * (size_t)dh * cwy);
  float* dec = (float*)malloc(sizeof(float) * (size_t)w * c);
  float* hbuf = (float*)malloc(sizeof(float) * (size_t)h * dw * c);
  float* vrow = (float*)malloc(sizeof(float) * (size_t)dw * c);
  int rc = -1;
  if (!x0 || !y0 || !wx || !wy || !dec || !hbuf || !vrow) goto out;
  if (orc_axis_coeffs(w, dw, cwx, x0, x0 + dw, wx)) goto out;
  if (orc_axis_coeffs(h, dh, cwy, y0, y0 + dh, wy)) goto out;
  const float inv255 = 1.0f / 255.0f;
  for (int r = 0; r < h; r++) {
    const uint8_t* s = src + (size_t)r * w * c;
    for (int i = 0; i < w * c; i++) dec[i] = (float)s[i] * inv255;
    if (alpha)
      for (int i = 0; i < w; i++)
        for (int k = 0; k < 3; k++) dec[4 * i + k] *= dec[4 * i + 3];
    float* hr = hbuf + (size_t)r * dw * c;
    for (int ox = 0; ox < dw; ox++) {
      const int a = x0[ox], b = x0[dw + ox];
      const float* cf = wx + (size_t)ox * cwx;
      for (int ch = 0; ch < c; ch++) {
        float acc = cf[0] * dec[a * c + ch];
        for (int k = 1; k <= b - a; k++) acc = acc + cf[k] * dec[(a + k) * c + ch];
        hr[ox * c + ch] = acc;
      }
    }
  }
  for (int oy = 0; oy < dh; oy++) {
    const int a = y0[oy], b = y0[dh + oy];
    const float* cf = wy + (size_t)oy * cwy;
    for (int i = 0; i < dw * c; i++) {
      float acc = cf[0] * hbuf[(size_t)a * dw * c + i];
      for (int k = 1; k <= b - a; k++) acc = acc + cf[k] * hbuf[(size_t)(a + k) * dw * c + i];
      vrow[i] = acc;
    }
    if (alpha)
      for (int i = 0; i < dw; i++) {
        const float a = vrow[4 * i + 3];
        if (a >= 7.52316384526264e-37f) { /* stbir's small float, 1 / 2^120 */
          const float ia = 1.0f / a;
          for (int k = 0; k < 3; k++) vrow[4 * i + k] *= ia;
        }
      }
    uint8_t* d = dst + (size_t)oy * dw * c;
    for (int i = 0; i < dw * c; i++) {
      float f = vrow[i] * 255.0f + 0.5f;
      if (f < 0.0f) f = 0.0f;
      if (f > 255.0f) f = 255.0f;
      d[i] = (uint8_t)f;
    }
  }
  rc = 0;
out:
  free(x0);
  free(y0);
  free(wx);
  free(wy);
  free(dec);
  free(hbuf);
  free(vrow);
  return rc;
}

int orc_resize_u8(const uint8_t* src, int w, int h, int c, uint8_t* dst, int dw, int dh) {
  return orc_resize_u8_layout(src, w, h, c, dst, dw, dh, c == 4);
}

/*
 * Kernel-order restatement of resize -> crop -> hflip (SURVEY.md §8(c)2's
 * "bit-exact when coefficient tables are shared" gate): the SAME tap tables as
 * orc_resize_u8 (orc_axis_coeffs), but vertical pass first, in byte units
 * (no decode to [0,1]), each sum an fmaf chain in tap order starting from 0,
 * then the horizontal pass the same way, then stbir's encode
 * (uint8)trunc(clamp(v + 0.5, 0, 255)).  This is the order the HIP kernels
 * sum in (mlx-data_amd/csrc/band.hip, wave.hip), so they must match it bit for
 * bit; it differs from the stbir-order restatement above only by f32
 * rounding (+-1).  channels 1..4 (no alpha weighting; the STBIR_RGBA form is
 * orc_resize_crop_vfirst_rgba below).  Writes the crop
 * window (cx, cy, cw, ch) of the (dw x dh) resize of the (w x h, row stride
 * `stride` bytes) source, mirrored when flip, as ch x cw x c bytes.
 */
int orc_resize_crop_vfirst(const uint8_t* src, int w, int h, int c, int64_t stride, uint8_t* dst, int dw, int dh,
                           int cx, int cy, int cw, int ch, int flip) {
  if (w <= 0 || h <= 0 || dw <= 0 || dh <= 0 || c < 1 || c > 4) return -1;
  if (cx < 0 || cy < 0 || cw <= 0 || ch <= 0 || cx + cw > dw || cy + ch > dh) return -1;
  const int cwx = orc_axis_width(w, dw), cwy = orc_axis_width(h, dh);
  int* x0 = (int*)malloc(sizeof(int) * (size_t)dw * 2);
  int* y0 = (int*)malloc(sizeof(int) * (size_t)dh * 2);
  float* wx = (float*)malloc(sizeof(float) * (size_t)dw * cwx);
  float* wy = (float*)malloc(sizeof(float) * (size_t)dh * cwy);
  float* vrow = (float*)malloc(sizeof(float) * (size_t)w * c);
  int rc = -1;
  if (!x0 || !y0 || !wx || !wy || !vrow) goto out;
  if (orc_axis_coeffs(w, dw, cwx, x0, x0 + dw, wx)) goto out;
  if (orc_axis_coeffs(h, dh, cwy, y0, y0 + dh, wy)) goto out;
  /* only the source columns the window's horizontal taps read */
  int xlo = x0[cx], xhi = x0[dw + cx];
  for (int ox = cx; ox < cx + cw; ox++) {
    if (x0[ox] < xlo) xlo = x0[ox];
    if (x0[dw + ox] > xhi) xhi = x0[dw + ox];
  }
  for (int r = 0; r < ch; r++) {
    const int oy = cy + r;
    const int a = y0[oy], b = y0[dh + oy];
    const float* cf = wy + (size_t)oy * cwy;
    for (int i = xlo * c; i < (xhi + 1) * c; i++) {
      float v = 0.0f;
      for (int k = 0; k <= b - a; k++) v = fmaf(cf[k], (float)src[(size_t)(a + k) * stride + i], v);
      vrow[i] = v;
    }
    uint8_t* d = dst + (size_t)r * cw * c;
    for (int x = 0; x < cw; x++) {
      const int ox = cx + (flip ? cw - 1 - x : x);
      const int xa = x0[ox], xb = x0[dw + ox];
      const float* cfx = wx + (size_t)ox * cwx;
      for (int k2 = 0; k2 < c; k2++) {
        float hsum = 0.0f;
        for (int k = 0; k <= xb - xa; k++) hsum = fmaf(cfx[k], vrow[(xa + k) * c + k2], hsum);
        float f = hsum + 0.5f;
        if (f < 0.0f) f = 0.0f;
        if (f > 255.0f) f = 255.0f;
        d[x * c + k2] = (uint8_t)f;
      }
    }
  }
  rc = 0;
out:
  free(x0);
  free(y0);
  free(wx);
  free(wy);
  free(vrow);
  return rc;
}

/*
 * Kernel-order restatement of the STBIR_RGBA (alpha-weighted, c = 4) resize ->
 * crop -> hflip, in stbir's float operations (a
 * restatement: parity unpinned): every byte decoded as b * (1/255), colours
 * multiplied by their decoded alpha, the vertical pass then the horizontal pass
 * (fmaf chains in tap order from 0, shared tap tables), colours multiplied by
 * 1 / filtered alpha unless it is below stbir's small float, encoded as
 * (uint8)trunc(clamp(v * 255 + 0.5)) with the multiply and add unfused (this
 * file is built with -ffp-contract=off).  The order of the general HIP kernel
 * (mlx-data_amd/csrc/resample.hip, ALPHA), which must match it bit for bit; it
 * differs from orc_resize_u8_layout (stbir's horizontal-first order) only by f32
 * rounding.
 */
int orc_resize_crop_vfirst_rgba(const uint8_t* src, int w, int h, int64_t stride, uint8_t* dst, int dw, int dh, int cx,
                                int cy, int cw, int ch, int flip) {
  const int c = 4;
  if (w <= 0 || h <= 0 || dw <= 0 || dh <= 0) return -1;
  if (cx < 0 || cy < 0 || cw <= 0 || ch <= 0 || cx + cw > dw || cy + ch > dh) return -1;
  const int cwx = orc_axis_width(w, dw), cwy = orc_axis_width(h, dh);
  int* x0 = (int*)malloc(sizeof(int) * (size_t)dw * 2);
  int* y0 = (int*)malloc(sizeof(int) * (size_t)dh * 2);
  float* wx = (float*)malloc(sizeof(float) * (size_t)dw * cwx);
  float* wy = (float*)malloc(sizeof(float) * (size_t)dh * cwy);
  float* vrow = (float*)malloc(sizeof(float) * (size_t)w * c);
  int rc = -1;
  if (!x0 || !y0 || !wx || !wy || !vrow) goto out;
  if (orc_axis_coeffs(w, dw, cwx, x0, x0 + dw, wx)) goto out;
  if (orc_axis_coeffs(h, dh, cwy, y0, y0 + dh, wy)) goto out;
  const float inv255 = 1.0f / 255.0f;
  int xlo = x0[cx], xhi = x0[dw + cx];
  for (int ox = cx; ox < cx + cw; ox++) {
    if (x0[ox] < xlo) xlo = x0[ox];
    if (x0[dw + ox] > xhi) xhi = x0[dw + ox];
  }
  for (int r = 0; r < ch; r++) {
    const int oy = cy + r;
    const int a = y0[oy], b = y0[dh + oy];
    const float* cf = wy + (size_t)oy * cwy;
    for (int px = xlo; px <= xhi; px++)
      for (int k2 = 0; k2 < c; k2++) {
        float v = 0.0f;
        for (int k = 0; k <= b - a; k++) {
          const uint8_t* p = src + (size_t)(a + k) * stride + (size_t)px * c;
          const float al = (float)p[3] * inv255;
          const float x = k2 < 3 ? (float)p[k2] * inv255 * al : al;
          v = fmaf(cf[k], x, v);
        }
        vrow[px * c + k2] = v;
      }
    uint8_t* d = dst + (size_t)r * cw * c;
    for (int x = 0; x < cw; x++) {
      const int ox = cx + (flip ? cw - 1 - x : x);
      const int xa = x0[ox], xb = x0[dw + ox];
      const float* cfx = wx + (size_t)ox * cwx;
      float px4[4];
      for (int k2 = 0; k2 < c; k2++) {
        float hsum = 0.0f;
        for (int k = 0; k <= xb - xa; k++) hsum = fmaf(cfx[k], vrow[(xa + k) * c + k2], hsum);
        px4[k2] = hsum;
      }
      if (px4[3] >= 7.52316384526264e-37f) { /* stbir's small float, 1 / 2^120 */
        const float ia = 1.0f / px4[3];
        for (int k2 = 0; k2 < 3; k2++) px4[k2] = px4[k2] * ia;
      }
      for (int k2 = 0; k2 < c; k2++) {
        float f = px4[k2] * 255.0f;
        f = f + 0.5f;
        if (f < 0.0f) f = 0.0f;
        if (f > 255.0f) f = 255.0f;
        d[x * c + k2] = (uint8_t)f;
      }
    }
  }
  rc = 0;
out:
  free(x0);
  free(y0);
  free(wx);
  free(wy);
  free(vrow);
  return rc;
}

/* ImageCenterCrop::apply_image offsets (integer floor). */
int orc_center_crop_origin(int64_t w, int64_t h, int64_t cw, int64_t ch, int64_t* x, int64_t* y) {
  if (ch > h || cw > w) return -1;
  *x = (w - cw) / 2;
  *y = (h - ch) / 2;
  return 0;
}

/* core::image::crop via array::sub: h row memcpys of w*c bytes. */
int orc_crop_u8(const uint8_t* src, int w, int h, int c, int x, int y, int cw, int ch, uint8_t* dst) {
  if (cw <= 0 || ch <= 0 || x < 0 || y < 0 || x >= w || y >= h || x + cw > w || y + ch > h) return -1;
  for (int r = 0; r < ch; r++) memcpy(dst + (size_t)r * cw * c, src + ((size_t)(y + r) * w + x) * c, (size_t)cw * c);
  return 0;
}

/* core::image::hflip */
int orc_hflip_u8(const uint8_t* src, int w, int h, int c, uint8_t* dst) {
  for (int r = 0; r < h; r++)
    for (int x = 0; x < w; x++)
      for (int k = 0; k < c; k++) dst[((size_t)r * w + x) * c + k] = src[((size_t)r * w + (w - x - 1)) * c + k];
  return 0;
}

/* x.astype("float32") / 255: correctly rounded f32 division. */
void orc_normalize_u8(const uint8_t* q, size_t n, float* out) {
  for (size_t i = 0; i < n; i++) out[i] = (float)q[i] / 255.0f;
}

/*
 * The composed per-sample hot path: resize_smallest_side(size) then
 * center_crop(cw, ch); writes ch x cw x c bytes.  Returns 0 or -1.
 */
int orc_resize_smallest_side_center_crop(const uint8_t* src, int w, int h, int c, int size, int cw, int ch,
                                         uint8_t* dst) {
  int64_t tw, th, x, y;
  if (orc_resize_smallest_side_dims(w, h, size, &tw, &th)) return -1;
  if (orc_center_crop_origin(tw, th, cw, ch, &x, &y)) return -1;
  uint8_t* tmp = (uint8_t*)malloc((size_t)tw * th * c);
  if (!tmp) return -1;
  int rc = orc_resize_u8(src, w, h, c, tmp, (int)tw, (int)th);
  if (!rc) rc = orc_crop_u8(tmp, (int)tw, (int)th, c, (int)x, (int)y, cw, ch, dst);
  free(tmp);
  return rc;
}

/* ---- rotate / affine (core/image/ImageTransform.cpp:75-121) -------------
 * Parity status: the reference file needs stb_image_resize2.h and is not
 * buildable here, so this is a line-by-line restatement of its integer /
 * float arithmetic (pinned by tests/golden/pixmap.npz, generated from this
 * file, and by the GPU kernels agreeing bit for bit).  fabs is taken in
 * float (the <cmath> float overload). */
int orc_rotate_geometry(int64_t w, int64_t h, double angle, int crop, float* mx, int64_t* tw, int64_t* th) {
  const float pi = (float)(atan(1.0) * 4);
  const float rangle = (float)(angle * (double)pi / 180.);
  const float c = cosf(rangle);
  const float s = sinf(rangle);
  mx[0] = c; mx[1] = s; mx[2] = 0; mx[3] = -s; mx[4] = c; mx[5] = 0;
  *tw = w;
  *th = h;
  if (!crop) {
    *tw = (int64_t)((float)w * fabsf(mx[0]) + (float)h * fabsf(mx[1]));
    *th = (int64_t)((float)h * fabsf(mx[3]) + (float)w * fabsf(mx[4]));
  }
  return (*tw <= 0 || *th <= 0) ? 1 : 0;
}

void orc_affine_u8(const uint8_t* src, int64_t w, int64_t h, int64_t c, const float* mx, int64_t tw, int64_t th,
                   uint8_t* dst) {
  const float twh = (float)(tw / 2.0);
  const float thh = (float)(th / 2.0);
  const float wh = (float)(w / 2.0);
  const float hh = (float)(h / 2.0);
  for (int64_t ty = 0; ty < th; ty++) {
    for (int64_t tx = 0; tx < tw; tx++) {
      const float fx = (float)tx - twh, fy = (float)ty - thh;
      const float sx = mx[0] * fx + mx[1] * fy + mx[2];
      const float sy = mx[3] * fx + mx[4] * fy + mx[5];
      const int64_t x = (int64_t)((double)sx + 0.5 + (double)wh);
      const int64_t y = (int64_t)((double)sy + 0.5 + (double)hh);
      uint8_t* o = dst + (ty * tw + tx) * c;
      if (x < 0 || y < 0 || x >= w || y >= h)
        memset(o, 0, (size_t)c);
      else
        memcpy(o, src + (y * w + x) * c, (size_t)c);
    }
  }
}

/* ---- channel reduction (core/image/ImageTransform.cpp:142-180) ---------- */
void orc_channel_reduction_u8(const uint8_t* src, int64_t w, int64_t h, float bias, const float* mult, uint8_t* dst) {
  const int scale = 256 * 256;
  const int ib = (int)(bias * (float)scale);
  int m[3];
  for (int i = 0; i < 3; i++) m[i] = (int)(mult[i] * (float)scale);
  for (int64_t i = 0; i < w * h; i++) {
    int v = (src[3 * i] * m[0] + src[3 * i + 1] * m[1] + src[3 * i + 2] * m[2] + ib) / scale;
    v = v <= 255 ? v : 255;
    v = v >= 0 ? v : 0;
    dst[i] = (uint8_t)v;
  }
}
