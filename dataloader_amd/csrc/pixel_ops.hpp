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

constexpr double kRcp255 = 1.0 / 255.0;

// 1/d in double: on the GPU the hardware reciprocal (a seed of roughly single
// precision) refined by one Newton step (relative error ~2^-44), on the host the
// division.  Used only as n * (1/d) -> float with n <= d <= 255: such a
// quotient is either exact in float or >= 2^-32 (relative) away from every float
// rounding midpoint, so both give the correctly rounded float quotient (and the GPU
// test of all 2^24 inputs against Pillow, tests/test_gpu_round5.py, checks it).
DHD double rcp_f64(double d) {
#if defined(__HIP_DEVICE_COMPILE__)
  const double y = __builtin_amdgcn_rcp(d);
  return fma(y, fma(-d, y, 1.0), y);
#else
  return 1.0 / d;
#endif
}

// Convert.c rgb2hsv_row for one pixel, restated without per-pixel divisions (checked
// over all 2^24 colours against Pillow, on the host by tests/test_emu_cpu.py and on the
// GPU by tests/test_gpu_round5.py):
//  * s = cri / maxc and the channel quotients are float quotients (C's
//    `cr / (float)maxc` etc.), from the reciprocal above;
//  * of the three quotients (maxc - x) / cri, the max channel's is 0 and the min
//    channel's 1 exactly, so h is `a + sign * qm` with qm the middle channel's quotient
//    and (a, sign) given by the case -- one rounding, as C's float / double expression;
//  * fmod(h / 6.0 + 1.0, 1.0): h in [-1, 5], so it is h / 6 for h >= 0 and 1 + h / 6
//    below; h / 6 as a double product with the rounded 1/6 gives the same float.
DHD void rgb_to_hsv(int r, int g, int b, int* oh, int* os, int* ov) {
  const int maxc = r > g ? (r > b ? r : b) : (g > b ? g : b);
  const int minc = r < g ? (r < b ? r : b) : (g < b ? g : b);
  *ov = maxc;
  const int cri = maxc - minc;
  const float s = (float)((double)cri * rcp_f64((double)(maxc > 0 ? maxc : 1)));
  const int mid = r + g + b - maxc - minc;
  const float qm = (float)((double)(maxc - mid) * rcp_f64((double)(cri > 0 ? cri : 1)));
  // r max: g min -> bc - gc = qm - 1, b min -> 1 - qm;  g max: r min -> 2 + 1 - qm,
  // b min -> 2 + qm - 1;  b max: r min -> 4 + qm - 1, g min -> 4 + 1 - qm
  float a, sg;
  if (r == maxc) {
    a = g == minc ? -1.0f : 1.0f;
    sg = g == minc ? 1.0f : -1.0f;
  } else if (g == maxc) {
    a = r == minc ? 3.0f : 1.0f;
    sg = r == minc ? -1.0f : 1.0f;
  } else {
    a = r == minc ? 3.0f : 5.0f;
    sg = r == minc ? 1.0f : -1.0f;
  }
  const float h = fmaf(sg, qm, a);
  const double y = (double)h * (1.0 / 6.0);
  const float hf = (float)(h >= 0.0f ? y : y + 1.0);
  *oh = cri == 0 ? 0 : clip8i((int)((double)hf * 255.0));
  *os = cri == 0 ? 0 : clip8i((int)((double)s * 255.0));
}

// Convert.c hsv2rgb: i = floor(h * 6 / 255), f its fraction, fs = s / 255, and the
// rounded values of v * (1 - fs), v * (1 - fs * f) and v * (1 - fs * (1 - f)), here as
// floor(v + 0.5 - v * x) by one float fma each (checked over all 2^24 inputs against
// Pillow, host and GPU).
DHD void hsv_to_rgb(int h, int s, int v, int* r, int* g, int* b) {
  const int h6 = h * 6;
  const int i = h6 / 255;
  const float f = (float)((double)(h6 - 255 * i) * kRcp255);
  const float fs = (float)((double)s * kRcp255);
  const float vf = (float)v, vh = vf + 0.5f;
  const int up = clip8i((int)floorf(fmaf(-vf, fs, vh)));
  const int uq = clip8i((int)floorf(fmaf(-vf, fs * f, vh)));
  const int ut = clip8i((int)floorf(fmaf(-vf, fmaf(-fs, f, fs), vh)));
  const int k = i == 6 ? 0 : i;  // i % 6
  int rr = k == 0 || k == 5 ? v : (k == 1 ? uq : (k == 4 ? ut : up));
  int gg = k == 1 || k == 2 ? v : (k == 0 ? ut : (k == 3 ? uq : up));
  int bb = k == 3 || k == 4 ? v : (k == 2 ? ut : (k == 5 ? uq : up));
  if (s == 0) rr = gg = bb = v;
  *r = rr;
  *g = gg;
  *b = bb;
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
