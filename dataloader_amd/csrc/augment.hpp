// augment.hpp — per-pixel building blocks of the per-view op chain
// (reference cpu.py:255-267), shared by the HIP kernels and the host emulator.
//
// Data layout of one view while it is being built (LDS on the GPU): three u8
// planes of S*S (R, G, B), row-major, already flipped.  Resize coefficient
// tables (per view, per axis) are int32: bounds[S][2] = (min, count), then
// taps[S][ksize].
#pragma once

#include "pixel_ops.hpp"
#include "resize.hpp"

namespace dino {

// Accessor for a u8 source region: the decoded RGB image (HWC, offset to the crop
// origin: px = 3, cs = 1) or the horizontally-resampled rows (planar: px = 1,
// cs = rows * S).
struct SrcView {
  const uint8_t* base;
  int64_t pitch;  // bytes per row
  int32_t px;     // bytes per pixel step
  int64_t cs;     // bytes per channel step
};

struct CoefView {
  const int32_t* bounds;  // [n][2]
  const int32_t* taps;    // [n][ksize]
  int32_t ksize;
};

DHD uint8_t hresize_at(const SrcView& s, const CoefView& cv, int row, int x, int ch) {
  int xmin = cv.bounds[2 * x], xcnt = cv.bounds[2 * x + 1];
  const int32_t* k = cv.taps + (int64_t)x * cv.ksize;
  const uint8_t* p = s.base + (int64_t)row * s.pitch + (int64_t)xmin * s.px + ch * s.cs;
  int32_t acc = 1 << (kPrecisionBits - 1);
  for (int t = 0; t < xcnt; ++t) acc += (int32_t)p[t * s.px] * k[t];
  return clip8_acc(acc);
}

DHD uint8_t vresize_at(const SrcView& s, const CoefView& cv, int y, int x, int ch) {
  int ymin = cv.bounds[2 * y], ycnt = cv.bounds[2 * y + 1];
  const int32_t* k = cv.taps + (int64_t)y * cv.ksize;
  const uint8_t* p = s.base + (int64_t)ymin * s.pitch + (int64_t)x * s.px + ch * s.cs;
  int32_t acc = 1 << (kPrecisionBits - 1);
  for (int t = 0; t < ycnt; ++t) acc += (int32_t)p[(int64_t)t * s.pitch] * k[t];
  return clip8_acc(acc);
}

// The jitter op chain is split at the contrast op (its degenerate image needs the
// mean of the whole crop as it stands right before it).  stage 0 = ops before
// contrast, stage 1 = contrast and the ops after it (+ grayscale).
struct JitterPlan {
  int32_t n_pre;        // ops in stage 0
  int32_t has_contrast; // contrast op present (then it is the first op of stage 1)
  int32_t n_post;       // ops after contrast
  uint32_t pre, post;   // op codes, one per byte (packed so that lanes keep them in registers)
  // Optional 256-entry tables of the view's brightness and contrast blends (LDS on the
  // GPU, jitter_tables): both ops are one function of the channel value per view, so a
  // lookup replaces the float blend (same values: the table holds blend_u8 itself).
  const uint8_t* tb;
  const uint8_t* tc;
};

DHD JitterPlan make_jitter_plan(const dino_view_params& p) {
  JitterPlan j;
  j.n_pre = j.n_post = j.has_contrast = 0;
  j.pre = j.post = 0;
  j.tb = j.tc = nullptr;
  if (!p.jitter) return j;
  const uint32_t ord = (uint32_t)p.order[0] | ((uint32_t)p.order[1] << 8) | ((uint32_t)p.order[2] << 16) |
                       ((uint32_t)p.order[3] << 24);
  int k = 0;
  for (; k < 4 && ((ord >> (8 * k)) & 0xFF) != 1; ++k) j.pre |= ((ord >> (8 * k)) & 0xFF) << (8 * j.n_pre++);
  if (k < 4) {
    j.has_contrast = 1;
    for (++k; k < 4; ++k) j.post |= ((ord >> (8 * k)) & 0xFF) << (8 * j.n_post++);
  }
  return j;
}

// One ColorJitter op on one pixel (torchvision ColorJitter.forward -> Pillow).
DHD void jitter_op(int op, int& r, int& g, int& b, const dino_view_params& p, int contrast_mean, int hue_d,
                   const uint8_t* tb = nullptr, const uint8_t* tc = nullptr) {
  switch (op) {
    case 0: {  // brightness: blend(black, img, f)
      if (tb) {
        r = tb[r], g = tb[g], b = tb[b];
        break;
      }
      r = blend_u8(0, r, p.brightness);
      g = blend_u8(0, g, p.brightness);
      b = blend_u8(0, b, p.brightness);
      break;
    }
    case 1: {  // contrast: blend(mean(L) grey, img, f)
      if (tc) {
        r = tc[r], g = tc[g], b = tc[b];
        break;
      }
      r = blend_u8(contrast_mean, r, p.contrast);
      g = blend_u8(contrast_mean, g, p.contrast);
      b = blend_u8(contrast_mean, b, p.contrast);
      break;
    }
    case 2: {  // saturation: blend(L->RGB, img, f)
      int l = rgb_to_l(r, g, b);
      r = blend_u8(l, r, p.saturation);
      g = blend_u8(l, g, p.saturation);
      b = blend_u8(l, b, p.saturation);
      break;
    }
    default:
      hue_shift(r, g, b, hue_d);
      break;
  }
}

DHD void jitter_stage0(const JitterPlan& j, int& r, int& g, int& b, const dino_view_params& p, int hue_d) {
  for (int k = 0; k < j.n_pre; ++k) jitter_op((j.pre >> (8 * k)) & 0xFF, r, g, b, p, 0, hue_d, j.tb, nullptr);
}

// Contrast (if any), later ops, then grayscale.
DHD void jitter_stage1(const JitterPlan& j, int& r, int& g, int& b, const dino_view_params& p, int contrast_mean,
                       int hue_d) {
  if (j.has_contrast) jitter_op(1, r, g, b, p, contrast_mean, hue_d, j.tb, j.tc);
  for (int k = 0; k < j.n_post; ++k) jitter_op((j.post >> (8 * k)) & 0xFF, r, g, b, p, contrast_mean, hue_d, j.tb, j.tc);
  if (p.gray) {
    int l = rgb_to_l(r, g, b);
    r = g = b = l;
  }
}

// ImageEnhance.Contrast: int(ImageStat.Stat(L).mean[0] + 0.5), sum exact in double.
DHD int contrast_mean_from_sum(uint64_t lsum, int64_t n) { return (int)((double)lsum / (double)n + 0.5); }

// torchvision _get_gaussian_kernel1d in float32 (exp evaluated in double, then rounded).
DHD void gaussian_kernel1d(int ksize, double sigma, float* k) {
  float half = (float)(ksize - 1) * 0.5f;
  float s = (float)sigma;
  float sum = 0.0f;
  for (int i = 0; i < ksize; ++i) {
    float x = -half + (float)i;
    float t = x / s;
    float e = (float)exp((double)(-0.5f * (t * t)));
    k[i] = e;
    sum += e;
  }
  for (int i = 0; i < ksize; ++i) k[i] = k[i] / sum;
}

DHD int reflect_idx(int i, int n) {
  if (i < 0) return -i;
  if (i >= n) return 2 * (n - 1) - i;
  return i;
}

// Blur of plane `pl` (S*S u8) at (y, x) with the 2-D kernel k2[ks*ks] (float32 products
// of the 1-D kernel, as torch.mm builds it), reflect padding, round-half-even.
DHD int blur_at(const uint8_t* pl, int S, int y, int x, const float* k2, int ks) {
  int p = ks >> 1;
  float acc = 0.0f;
  for (int a = 0; a < ks; ++a) {
    const uint8_t* row = pl + (int64_t)reflect_idx(y + a - p, S) * S;
    for (int bb = 0; bb < ks; ++bb) acc = fmaf(k2[a * ks + bb], (float)row[reflect_idx(x + bb - p, S)], acc);
  }
  float r = rintf(acc);
  return r <= 0.0f ? 0 : (r >= 255.0f ? 255 : (int)r);
}

}  // namespace dino
