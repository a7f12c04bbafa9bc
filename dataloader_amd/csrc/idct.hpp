// idct.hpp — libjpeg-turbo jidctint.c jpeg_idct_islow (CONST_BITS 13,
// PASS1_BITS 2) with libjpeg's post-IDCT range-limit table semantics.  This is
// the DCT method Pillow's decoder uses (default JDCT_ISLOW).  libjpeg-turbo's SIMD
// versions (the code Pillow runs on x86) equal this C formulation for every block
// of valid 8-bit data; for the out-of-range coefficients of damaged streams they
// differ, and the SIMD arithmetic is restated below (idct_simd_*), used for blocks
// outside the bounds where the two provably agree (idct_col_safe / idct_row_safe).
#pragma once

#include "common.hpp"

namespace dino {

constexpr int kConstBits = 13;
constexpr int kPass1Bits = 2;
constexpr int32_t F0_298 = 2446, F0_390 = 3196, F0_541 = 4433, F0_765 = 6270, F0_899 = 7373,
                  F1_175 = 9633, F1_501 = 12299, F1_847 = 15137, F1_961 = 16069, F2_053 = 16819,
                  F2_562 = 20995, F3_072 = 25172;

template <typename T>
DHD int32_t descale(T x, int n) { return (int32_t)((x + ((T)1 << (n - 1))) >> n); }

// IDCT_range_limit(cinfo)[x & RANGE_MASK] for 8-bit samples (jdmaster.c prepare_range_limit_table).
DHD uint8_t range_limit_idct(int32_t x) {
  int32_t i = x & 1023;
  if (i < 128) return (uint8_t)(i + 128);
  if (i < 512) return 255;
  if (i < 896) return 0;
  return (uint8_t)(i - 896);
}

// One 1-D pass of the islow butterfly on 8 inputs.  d0..d7 are the (dequantized
// in pass 1) coefficients of one column/row; writes 8 results before descale.
// T = int64_t reproduces libjpeg's JLONG arithmetic for any input; T = int32_t is
// exact whenever every input magnitude is <= kIslow32Bound (worst-case sum of the
// butterfly's constants is 178219, and 178219 * 11000 + 2^17 < 2^31).
constexpr int32_t kIslow32Bound = 11000;

template <typename T>
struct Islow8 {
  T t10, t11, t12, t13, t0, t1, t2, t3;
};

template <typename T>
DHD Islow8<T> islow_core(T d0, T d1, T d2, T d3, T d4, T d5, T d6, T d7) {
  Islow8<T> r;
  // even part
  T z2 = d2, z3 = d6;
  T z1 = (z2 + z3) * F0_541;
  T tmp2 = z1 + z3 * (-F1_847);
  T tmp3 = z1 + z2 * F0_765;
  T tmp0 = (d0 + d4) * (1 << kConstBits);
  T tmp1 = (d0 - d4) * (1 << kConstBits);
  r.t10 = tmp0 + tmp3;
  r.t13 = tmp0 - tmp3;
  r.t11 = tmp1 + tmp2;
  r.t12 = tmp1 - tmp2;
  // odd part
  tmp0 = d7;
  tmp1 = d5;
  tmp2 = d3;
  tmp3 = d1;
  z1 = tmp0 + tmp3;
  z2 = tmp1 + tmp2;
  z3 = tmp0 + tmp2;
  T z4 = tmp1 + tmp3;
  T z5 = (z3 + z4) * F1_175;
  tmp0 = tmp0 * F0_298;
  tmp1 = tmp1 * F2_053;
  tmp2 = tmp2 * F3_072;
  tmp3 = tmp3 * F1_501;
  z1 = z1 * (-F0_899);
  z2 = z2 * (-F2_562);
  z3 = z3 * (-F1_961);
  z4 = z4 * (-F0_390);
  z3 += z5;
  z4 += z5;
  r.t0 = tmp0 + z1 + z3;
  r.t1 = tmp1 + z2 + z4;
  r.t2 = tmp2 + z2 + z3;
  r.t3 = tmp3 + z1 + z4;
  return r;
}

// coef: 64 quantized coefficients (natural order, int16); q: quant table (natural
// order, read as ISLOW_MULT_TYPE = short like jddctmgr.c).  out: 8x8 samples, row pitch `pitch`.
template <typename T, typename OutT>
DHD void idct_islow_t(const int16_t* coef, const uint16_t* q, OutT* out, int64_t pitch) {
  int32_t ws[64];
  for (int c = 0; c < 8; ++c) {
    T d[8];
    for (int r = 0; r < 8; ++r) d[r] = (T)((int32_t)coef[r * 8 + c] * (int32_t)(int16_t)q[r * 8 + c]);
    Islow8<T> t = islow_core<T>(d[0], d[1], d[2], d[3], d[4], d[5], d[6], d[7]);
    const int sh = kConstBits - kPass1Bits;
    ws[0 * 8 + c] = descale(t.t10 + t.t3, sh);
    ws[7 * 8 + c] = descale(t.t10 - t.t3, sh);
    ws[1 * 8 + c] = descale(t.t11 + t.t2, sh);
    ws[6 * 8 + c] = descale(t.t11 - t.t2, sh);
    ws[2 * 8 + c] = descale(t.t12 + t.t1, sh);
    ws[5 * 8 + c] = descale(t.t12 - t.t1, sh);
    ws[3 * 8 + c] = descale(t.t13 + t.t0, sh);
    ws[4 * 8 + c] = descale(t.t13 - t.t0, sh);
  }
  for (int r = 0; r < 8; ++r) {
    const int32_t* w = ws + r * 8;
    Islow8<T> t = islow_core<T>(w[0], w[1], w[2], w[3], w[4], w[5], w[6], w[7]);
    const int sh = kConstBits + kPass1Bits + 3;
    OutT* o = out + r * pitch;
    o[0] = range_limit_idct(descale(t.t10 + t.t3, sh));
    o[7] = range_limit_idct(descale(t.t10 - t.t3, sh));
    o[1] = range_limit_idct(descale(t.t11 + t.t2, sh));
    o[6] = range_limit_idct(descale(t.t11 - t.t2, sh));
    o[2] = range_limit_idct(descale(t.t12 + t.t1, sh));
    o[5] = range_limit_idct(descale(t.t12 - t.t1, sh));
    o[3] = range_limit_idct(descale(t.t13 + t.t0, sh));
    o[4] = range_limit_idct(descale(t.t13 - t.t0, sh));
  }
}

// Exact for all inputs: 64-bit reference arithmetic.
template <typename OutT>
DHD void idct_islow(const int16_t* coef, const uint16_t* q, OutT* out, int64_t pitch) {
  idct_islow_t<int64_t>(coef, q, out, pitch);
}

DHD int32_t iabs32(int32_t x) { return x < 0 ? -x : x; }

DHD int32_t max_abs8(const int32_t* v) {
  int32_t m = 0;
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const int32_t a = iabs32(v[i]);
    m = a > m ? a : m;
  }
  return m;
}

// 1-D passes of idct_islow, each in int32 when its own 8 inputs are within
// kIslow32Bound (always, for valid 8-bit JPEG data) and in int64 otherwise, so
// the result equals libjpeg's JLONG arithmetic for any input.
// Pass 1: one column of dequantized coefficients d[0..7] (rows) -> workspace column.
template <typename T>
DHD void idct_pass1_t(const int32_t* d, int32_t* w) {
  const Islow8<T> t = islow_core<T>(d[0], d[1], d[2], d[3], d[4], d[5], d[6], d[7]);
  const int sh = kConstBits - kPass1Bits;
  w[0] = descale(t.t10 + t.t3, sh);
  w[7] = descale(t.t10 - t.t3, sh);
  w[1] = descale(t.t11 + t.t2, sh);
  w[6] = descale(t.t11 - t.t2, sh);
  w[2] = descale(t.t12 + t.t1, sh);
  w[5] = descale(t.t12 - t.t1, sh);
  w[3] = descale(t.t13 + t.t0, sh);
  w[4] = descale(t.t13 - t.t0, sh);
}

DHD void idct_pass1(const int32_t* d, int32_t* w) {
  if (max_abs8(d) <= kIslow32Bound)
    idct_pass1_t<int32_t>(d, w);
  else
    idct_pass1_t<int64_t>(d, w);
}

// Pass 2: one workspace row w[0..7] -> 8 output samples.
template <typename T>
DHD void idct_pass2_t(const int32_t* w, uint8_t* o) {
  const Islow8<T> t = islow_core<T>(w[0], w[1], w[2], w[3], w[4], w[5], w[6], w[7]);
  const int sh = kConstBits + kPass1Bits + 3;
  o[0] = range_limit_idct(descale(t.t10 + t.t3, sh));
  o[7] = range_limit_idct(descale(t.t10 - t.t3, sh));
  o[1] = range_limit_idct(descale(t.t11 + t.t2, sh));
  o[6] = range_limit_idct(descale(t.t11 - t.t2, sh));
  o[2] = range_limit_idct(descale(t.t12 + t.t1, sh));
  o[5] = range_limit_idct(descale(t.t12 - t.t1, sh));
  o[3] = range_limit_idct(descale(t.t13 + t.t0, sh));
  o[4] = range_limit_idct(descale(t.t13 - t.t0, sh));
}

DHD void idct_pass2(const int32_t* w, uint8_t* o) {
  if (max_abs8(w) <= kIslow32Bound)
    idct_pass2_t<int32_t>(w, o);
  else
    idct_pass2_t<int64_t>(w, o);
}

// ---- libjpeg-turbo SIMD islow (simd/x86_64/jidctint-sse2.asm, -avx2.asm) -------------
// The same butterfly on 16-bit lanes: dequantisation keeps the low 16 bits of the
// product (pmullw); in0 +/- in4, in7 + in3 and in5 + in1 are 16-bit sums (paddw/psubw);
// the rotations are pmaddwd pairs with the constants pre-combined (z1 folded into
// both of its products) and the 32-bit sums wrap; pass 1 saturates to int16
// (packssdw), pass 2 to [-128, 127] (packssdw, packsswb) before adding 128.  A block
// whose rows 1..7 are all zero takes pass 1 as (dc * q) << 2 in 16 bits (psllw).
DHD int32_t wrap16(int32_t x) { return (int32_t)(int16_t)x; }
DHD int32_t clamp_i32(int32_t x, int32_t lo, int32_t hi) { return x < lo ? lo : (x > hi ? hi : x); }
DHD int32_t add_w32(int32_t a, int32_t b) { return (int32_t)((uint32_t)a + (uint32_t)b); }
DHD int32_t sub_w32(int32_t a, int32_t b) { return (int32_t)((uint32_t)a - (uint32_t)b); }
DHD int32_t pmaddwd(int32_t a, int32_t ca, int32_t b, int32_t cb) {
  return (int32_t)(uint32_t)((int64_t)a * ca + (int64_t)b * cb);
}

// One 1-D pass on eight int16 inputs; o[0..7] = the output sums before the descale.
DHD void idct_simd_core(const int32_t* in, int32_t* o) {
  const int32_t tmp3 = pmaddwd(in[2], F0_541 + F0_765, in[6], F0_541);
  const int32_t tmp2 = pmaddwd(in[2], F0_541, in[6], F0_541 - F1_847);
  const int32_t tmp0 = wrap16(in[0] + in[4]) * (1 << kConstBits);
  const int32_t tmp1 = wrap16(in[0] - in[4]) * (1 << kConstBits);
  const int32_t t10 = add_w32(tmp0, tmp3), t13 = sub_w32(tmp0, tmp3);
  const int32_t t11 = add_w32(tmp1, tmp2), t12 = sub_w32(tmp1, tmp2);
  const int32_t z3s = wrap16(in[7] + in[3]), z4s = wrap16(in[5] + in[1]);
  const int32_t z3 = pmaddwd(z3s, F1_175 - F1_961, z4s, F1_175);
  const int32_t z4 = pmaddwd(z3s, F1_175, z4s, F1_175 - F0_390);
  const int32_t u0 = add_w32(pmaddwd(in[7], F0_298 - F0_899, in[1], -F0_899), z3);
  const int32_t u3 = add_w32(pmaddwd(in[7], -F0_899, in[1], F1_501 - F0_899), z4);
  const int32_t u1 = add_w32(pmaddwd(in[5], F2_053 - F2_562, in[3], -F2_562), z4);
  const int32_t u2 = add_w32(pmaddwd(in[5], -F2_562, in[3], F3_072 - F2_562), z3);
  o[0] = add_w32(t10, u3);
  o[7] = sub_w32(t10, u3);
  o[1] = add_w32(t11, u2);
  o[6] = sub_w32(t11, u2);
  o[2] = add_w32(t12, u1);
  o[5] = sub_w32(t12, u1);
  o[3] = add_w32(t13, u0);
  o[4] = sub_w32(t13, u0);
}

DHD int32_t simd_descale(int32_t x, int n) { return add_w32(x, 1 << (n - 1)) >> n; }

// Pass 1 of one column: raw coefficients c[0..7] (rows) and their quant values;
// dc_only = rows 1..7 of the whole block are zero.  w: int16 workspace column.
DHD void idct_simd_pass1(const int32_t* c, const int32_t* q, bool dc_only, int32_t* w) {
  int32_t in[8];
#pragma unroll
  for (int r = 0; r < 8; ++r) in[r] = wrap16(c[r] * q[r]);
  if (dc_only) {
    const int32_t v = wrap16(in[0] * (1 << kPass1Bits));
#pragma unroll
    for (int r = 0; r < 8; ++r) w[r] = v;
    return;
  }
  int32_t o[8];
  idct_simd_core(in, o);
#pragma unroll
  for (int r = 0; r < 8; ++r) w[r] = clamp_i32(simd_descale(o[r], kConstBits - kPass1Bits), -32768, 32767);
}

// Pass 2 of one row of int16 workspace values -> 8 samples.
DHD void idct_simd_pass2(const int32_t* w, uint8_t* out) {
  int32_t o[8];
  idct_simd_core(w, o);
#pragma unroll
  for (int k = 0; k < 8; ++k) out[k] = (uint8_t)(clamp_i32(simd_descale(o[k], kConstBits + kPass1Bits + 3), -128, 127) + 128);
}

// Bounds under which the C and the SIMD formulation give the same result.  Pass 1 of
// a column of dequantised values d: every 1-D output is d0 + sum_k d_k sqrt2 cos(.)
// times 4 (PASS1_BITS), so |d0| + 1.4143 sum_{k>=1} |d_k| <= 8190 keeps it inside
// int16 (no saturation), keeps every product and 16-bit sum from wrapping, and makes
// the DC-only shortcut equal to the general path.  Pass 2 of a row w: sum |w| <= 11500
// keeps the 16-bit sums and bounds the output by 11500 * 1.4143 / 32 + 0.5 < 512,
// the range where the C range-limit table clamps instead of wrapping.
// Cheap sufficient forms: |d0| <= 2047 with every other |d_k| <= 600 (2047 + 1.4143 *
// 7 * 600 < 8190); every |w| <= 1437 (8 * 1437 <= 11500).
DHD bool idct_col_safe_fast(const int32_t* d) {
  int32_t m = 0;
#pragma unroll
  for (int r = 1; r < 8; ++r) {
    const int32_t a = iabs32(d[r]);
    m = a > m ? a : m;
  }
  return iabs32(d[0]) <= 2047 && m <= 600;
}
DHD bool idct_col_safe(const int32_t* d) {
  int32_t s = 0;
#pragma unroll
  for (int r = 1; r < 8; ++r) {
    const int32_t a = iabs32(d[r]);
    s += a > 8190 ? 8191 : a;
  }
  const int32_t a0 = iabs32(d[0]);
  return a0 <= 8190 && 10000 * a0 + 14143 * s <= 81900000;
}
DHD bool idct_row_safe(const int32_t* w) {
  int32_t s = 0;
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    const int32_t a = iabs32(w[k]);
    s += a > 11500 ? 11501 : a;
  }
  return s <= 11500;
}

// Whole block through the two passes as the kernel runs them (host emulator; k_idct
// runs one pass per lane): the C passes when every column is within its bound, else
// the SIMD pass 1 for the block; per row, the C pass 2 within its bound, else SIMD.
DHD void idct_islow_fast(const int16_t* coef, const uint16_t* q, uint8_t* out, int64_t pitch) {
  int32_t ws[64];
  bool safe = true, dc_only = true;
  for (int c = 0; c < 8; ++c) {
    int32_t d[8];
    for (int r = 0; r < 8; ++r) d[r] = (int32_t)coef[r * 8 + c] * (int32_t)(int16_t)q[r * 8 + c];
    safe = safe && idct_col_safe(d);
    for (int r = 1; r < 8; ++r) dc_only = dc_only && coef[r * 8 + c] == 0;
  }
  for (int c = 0; c < 8; ++c) {
    int32_t d[8], w[8];
    if (safe) {
      for (int r = 0; r < 8; ++r) d[r] = (int32_t)coef[r * 8 + c] * (int32_t)(int16_t)q[r * 8 + c];
      idct_pass1(d, w);
    } else {
      int32_t cc[8], qq[8];
      for (int r = 0; r < 8; ++r) {
        cc[r] = coef[r * 8 + c];
        qq[r] = (int32_t)(int16_t)q[r * 8 + c];
      }
      idct_simd_pass1(cc, qq, dc_only, w);
    }
    for (int r = 0; r < 8; ++r) ws[r * 8 + c] = w[r];
  }
  for (int r = 0; r < 8; ++r) {
    if (idct_row_safe(ws + r * 8)) idct_pass2(ws + r * 8, out + r * pitch);
    else idct_simd_pass2(ws + r * 8, out + r * pitch);
  }
}

}  // namespace dino
