// pixel_ops.hpp — the uint8 per-pixel operators of the reference op chain
// (cpu.py:256-267) with Pillow's C semantics, plus the normalize/cast epilogue
// (cpu.py:223-232) with torch's float32 semantics.
//
//  * blend_u8      libImaging/Blend.c ImagingBlend (float alpha, truncating cast,
//                  clipped extrapolation) — ImageEnhance.Brightness/Contrast/Color.enhance
//  * rgb_to_l      libImaging/Convert.c rgb2l (L24 fixed point) — convert("L")
//  * rgb_to_hsv / hsv_to_rgb   Convert.c rgb2hsv_row / hsv2rgb (float/double mix
//                  exactly as the C source promotes) — torchvision adjust_hue PIL path
//  * solarize_u8   ImageOps.solarize(threshold=128)
//  * normalize     to_tensor (x/255) + normalize ((x-m)/s) in float32, then bf16 RNE
//  * fp8           c10 fp8e4m3fn_from_fp32_value (Stage-5 cast)
#pragma once

#include <math.h>

#include "common.hpp"

namespace dino {

DHD uint8_t blend_u8(int in1, int in2, float alpha) {
  float temp = (float)in1 + alpha * (float)(in2 - in1);
  if (temp <= 0.0f) return 0;
  if (temp >= 255.0f) return 255;
  return (uint8_t)temp;  // C float->uchar conversion truncates toward zero
}

DHD int rgb_to_l(int r, int g, int b) { return (r * 19595 + g * 38470 + b * 7471 + 0x8000) >> 16; }

DHD int clip8i(int v) { return v <= 0 ? 0 : (v >= 255 ? 255 : v); }

// 1/d (d = 1..255) as correctly rounded doubles.  For integers 0 <= n <= d <= 255,
// (float)(n * (1/d)) equals the float quotient n / d: the double product is within
// 2^-52 (relative) of n/d, and a quotient with a denominator <= 255 that is not exact
// in float lies >= 2^-32 (relative) away from every float rounding midpoint.  The
// same holds for the rationals k/255 below.  (The exhaustive test of both
// conversions against Pillow over all 2^24 inputs, tests/test_emu_cpu.py, checks it.)
struct RcpU8 {
  double v[256];
  constexpr RcpU8() : v() {
    for (int d = 1; d < 256; ++d) v[d] = 1.0 / (double)d;
  }
};
inline constexpr RcpU8 kRcpU8{};
constexpr double kRcp255 = 1.0 / 255.0;

DHD void rgb_to_hsv(int r, int g, int b, int* oh, int* os, int* ov) {
  int maxc = r > g ? (r > b ? r : b) : (g > b ? g : b);
  int minc = r < g ? (r < b ? r : b) : (g < b ? g : b);
  *ov = maxc;
  if (minc == maxc) {
    *oh = 0;
    *os = 0;
    return;
  }
  // Convert.c rgb2hsv_row: float quotients (via the exact reciprocal products above)
  const int cri = maxc - minc;
  const double rcr = kRcpU8.v[cri];
  float s = (float)((double)cri * kRcpU8.v[maxc]);
  float rc = (float)((double)(maxc - r) * rcr);
  float gc = (float)((double)(maxc - g) * rcr);
  float bc = (float)((double)(maxc - b) * rcr);
  float h;
  if (r == maxc) {
    h = bc - gc;
  } else if (g == maxc) {
    h = (float)(2.0 + (double)rc - (double)bc);
  } else {
    h = (float)(4.0 + (double)gc - (double)rc);
  }
  // fmod(h / 6.0 + 1.0, 1.0): h is in [-1, 5], so the argument is in (0, 2) and the
  // remainder is the argument minus 1 when >= 1 (exact)
  const double x = (double)h / 6.0 + 1.0;
  h = (float)(x >= 1.0 ? x - 1.0 : x);
  *oh = clip8i((int)((double)h * 255.0));
  *os = clip8i((int)((double)s * 255.0));
}

DHD void hsv_to_rgb(int h, int s, int v, int* r, int* g, int* b) {
  if (s == 0) {
    *r = *g = *b = v;
    return;
  }
  // Convert.c hsv2rgb: i = floor(h * 6 / 255), f = its fraction (0 exactly when h * 6
  // is a multiple of 255), fs = s / 255 — the same values without double divisions
  const int h6 = h * 6;
  const int i = h6 / 255;
  float f = h6 - 255 * i == 0 ? 0.0f : (float)((double)h6 * kRcp255 - (double)i);
  float fs = (float)((double)s * kRcp255);
  int p = (int)round((double)(float)v * (1.0 - (double)fs));
  int q = (int)round((double)(float)v * (1.0 - (double)(fs * f)));  // fs * f is a float product in C
  int t = (int)round((double)(float)v * (1.0 - (double)fs * (1.0 - (double)f)));
  int up = clip8i(p), uq = clip8i(q), ut = clip8i(t);
  switch (i % 6) {
    case 0: *r = v;  *g = ut; *b = up; break;
    case 1: *r = uq; *g = v;  *b = up; break;
    case 2: *r = up; *g = v;  *b = ut; break;
    case 3: *r = up; *g = uq; *b = v;  break;
    case 4: *r = ut; *g = up; *b = v;  break;
    default: *r = v; *g = up; *b = uq; break;
  }
}

// torchvision adjust_hue on one pixel: RGB -> HSV, H += delta (uint8 wrap), -> RGB.
DHD void hue_shift(int& r, int& g, int& b, int delta) {
  int h, s, v;
  rgb_to_hsv(r, g, b, &h, &s, &v);
  h = (h + delta) & 255;
  hsv_to_rgb(h, s, v, &r, &g, &b);
}

// np.int8(hue_factor * 255).view(np.uint8)
DHD int hue_delta(float hue_factor) { return ((int)((double)hue_factor * 255.0)) & 255; }

DHD uint8_t solarize_u8(int p) { return (uint8_t)(p >= 128 ? 255 - p : p); }

DHD float u8_normalize(int p, float mean, float std) {
  float x = (float)p / 255.0f;
  x = x - mean;
  return x / std;
}

DHD uint32_t f32_bits(float f) {
  union { float f; uint32_t u; } c;
  c.f = f;
  return c.u;
}
DHD float bits_f32(uint32_t u) {
  union { float f; uint32_t u; } c;
  c.u = u;
  return c.f;
}

// float -> bfloat16 round-to-nearest-even (inputs here are finite).
DHD uint16_t f32_to_bf16(float f) {
  uint32_t u = f32_bits(f);
  u += 0x7FFFu + ((u >> 16) & 1u);
  return (uint16_t)(u >> 16);
}

DHD float bf16_to_f32(uint16_t h) { return bits_f32((uint32_t)h << 16); }

// c10::detail::fp8e4m3fn_from_fp32_value.
DHD uint8_t f32_to_fp8e4m3(float f) {
  const uint32_t fp8_max = 1087u << 20;
  const uint32_t denorm_mask = 141u << 23;
  uint32_t fb = f32_bits(f);
  uint8_t result;
  const uint32_t sign = fb & 0x80000000u;
  fb ^= sign;
  if (fb >= fp8_max) {
    result = 0x7f;
  } else if (fb < (121u << 23)) {
    fb = f32_bits(bits_f32(fb) + bits_f32(denorm_mask));
    result = (uint8_t)(fb - denorm_mask);
  } else {
    uint8_t mant_odd = (fb >> 20) & 1;
    fb += ((uint32_t)(7 - 127) << 23) + 0x7FFFFu;
    fb += mant_odd;
    result = (uint8_t)(fb >> 20);
  }
  return (uint8_t)(result | (uint8_t)(sign >> 24));
}

}  // namespace dino
