// resize.hpp — Pillow's separable BICUBIC resampling (libImaging/Resample.c:
// bicubic_filter a = -0.5, precompute_coeffs, normalize_coeffs_8bpc with
// PRECISION_BITS = 22, ImagingResampleHorizontal/Vertical_8bpc with clip8).
// torchvision's RandomResizedCrop PIL path (reference cpu.py:172-183) is
// img.crop(box).resize((S, S), BICUBIC): the resample runs on the *cropped*
// image, so taps are clamped to the crop, box = (0, 0, w, h).
//
// Coefficients are computed in double exactly as Pillow does (no FMA
// contraction: the library is built with -ffp-contract=off) and quantised to
// the same int32 fixed point, so the uint8 result is bit-identical.
#pragma once

#include "common.hpp"

namespace dino {

constexpr int kPrecisionBits = 32 - 8 - 2;

DHD double bicubic_filter(double x) {
  const double a = -0.5;
  if (x < 0.0) x = -x;
  if (x < 1.0) return ((a + 2.0) * x - (a + 3.0)) * x * x + 1;
  if (x < 2.0) return (((x - 5) * x + 8) * x - 4) * a;
  return 0.0;
}

// Pillow's ksize for resampling in_size -> out_size (support 2 for bicubic).
DHD int resample_ksize(int in_size, int out_size) {
  double scale = (double)(float)in_size / out_size;
  double fs = scale < 1.0 ? 1.0 : scale;
  double support = 2.0 * fs;
  return (int)ceil(support) * 2 + 1;
}

// Coefficients of output index xx for in_size -> out_size with box (0, in_size).
// Writes bounds (xmin, xmax) and ksize int32 taps (zero padded).  Mirrors
// precompute_coeffs + normalize_coeffs_8bpc for one output position.
DHD void resample_coeffs_one(int in_size, int out_size, int xx, int ksize, int32_t* xmin_out, int32_t* xmax_out,
                             int32_t* k_out) {
  double in0 = 0.0, in1 = (double)(float)in_size;
  double scale = (in1 - in0) / out_size;
  double filterscale = scale < 1.0 ? 1.0 : scale;
  double support = 2.0 * filterscale;
  double center = in0 + (xx + 0.5) * scale;
  double ss = 1.0 / filterscale;
  int xmin = (int)(center - support + 0.5);
  if (xmin < 0) xmin = 0;
  int xmax = (int)(center + support + 0.5);
  if (xmax > in_size) xmax = in_size;
  xmax -= xmin;
  double ww = 0.0;
  // first pass: weights (Pillow stores them in the double kk buffer)
  for (int x = 0; x < xmax; ++x) {
    double w = bicubic_filter((x + xmin - center + 0.5) * ss);
    ww += w;
  }
  for (int x = 0; x < ksize; ++x) {
    int32_t q = 0;
    if (x < xmax) {
      double w = bicubic_filter((x + xmin - center + 0.5) * ss);
      if (ww != 0.0) w /= ww;
      q = w < 0 ? (int32_t)(-0.5 + w * (1 << kPrecisionBits)) : (int32_t)(0.5 + w * (1 << kPrecisionBits));
    }
    k_out[x] = q;
  }
  *xmin_out = xmin;
  *xmax_out = xmax;
}

// clip8 of the fixed-point accumulator (Resample.c).
DHD uint8_t clip8_acc(int32_t in) {
  if (in >= (1 << kPrecisionBits << 8)) return 255;
  if (in <= 0) return 0;
  return (uint8_t)(in >> kPrecisionBits);
}

}  // namespace dino
