// idct.hpp — the islow inverse DCT as Pillow runs it on x86: libjpeg-turbo's SIMD
// implementation (simd/x86_64/jidctint-sse2.asm, jidctint-avx2.asm) of jidctint.c
// jpeg_idct_islow (CONST_BITS 13, PASS1_BITS 2).  For every block of valid 8-bit
// data it equals the C formulation; for the out-of-range coefficients of damaged
// streams it differs (16-bit dequantisation and sums, saturation instead of the C
// range-limit table's wrap-around), and Pillow's output follows this one
// (tests/test_idct_simd_cpu.py pins it against Pillow with crafted coefficients).
//
// The butterfly on 16-bit lanes: dequantisation keeps the low 16 bits of the
// product (pmullw); in0 +/- in4, in7 + in3 and in5 + in1 are 16-bit sums
// (paddw/psubw); the rotations are pmaddwd pairs with the constants pre-combined
// (z1 folded into both of its products) and the 32-bit sums wrap; pass 1 saturates
// to int16 (packssdw), pass 2 to [-128, 127] (packssdw, packsswb) before adding 128.
// A block whose rows 1..7 are all zero takes pass 1 as (dc * q) << 2 in 16 bits (psllw).
#pragma once

#include "common.hpp"

namespace dino {

constexpr int kConstBits = 13;
constexpr int kPass1Bits = 2;
constexpr int32_t F0_298 = 2446, F0_390 = 3196, F0_541 = 4433, F0_765 = 6270, F0_899 = 7373,
                  F1_175 = 9633, F1_501 = 12299, F1_847 = 15137, F1_961 = 16069, F2_053 = 16819,
                  F2_562 = 20995, F3_072 = 25172;

DHD int32_t wrap16(int32_t x) { return (int32_t)(int16_t)x; }
DHD int32_t clamp_i32(int32_t x, int32_t lo, int32_t hi) { return x < lo ? lo : (x > hi ? hi : x); }
DHD int32_t add_w32(int32_t a, int32_t b) { return (int32_t)((uint32_t)a + (uint32_t)b); }
DHD int32_t sub_w32(int32_t a, int32_t b) { return (int32_t)((uint32_t)a - (uint32_t)b); }
// pmaddwd on int16 operands: |a c_a + b c_b| < 2 * 32768 * 25172 < 2^31, exact in int32
DHD int32_t pmaddwd(int32_t a, int32_t ca, int32_t b, int32_t cb) { return a * ca + b * cb; }

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

// Pass 1 of one column: raw coefficients c[0..7] (rows, int16 values) and their
// quant values q (as int16); dc_only = rows 1..7 of the whole block are zero.
// w: the int16 workspace column.
DHD void idct_pass1(const int32_t* c, const int32_t* q, bool dc_only, int32_t* w) {
  int32_t in[8], o[8];
#pragma unroll
  for (int r = 0; r < 8; ++r) in[r] = wrap16(c[r] * q[r]);
  idct_simd_core(in, o);
  const int32_t dcv = wrap16(in[0] * (1 << kPass1Bits));
#pragma unroll
  for (int r = 0; r < 8; ++r) w[r] = dc_only ? dcv : clamp_i32(simd_descale(o[r], kConstBits - kPass1Bits), -32768, 32767);
}

// Pass 2 of one row of int16 workspace values -> 8 samples.
DHD void idct_pass2(const int32_t* w, uint8_t* out) {
  int32_t o[8];
  idct_simd_core(w, o);
#pragma unroll
  for (int k = 0; k < 8; ++k) out[k] = (uint8_t)(clamp_i32(simd_descale(o[k], kConstBits + kPass1Bits + 3), -128, 127) + 128);
}

// Whole block (host emulator; k_idct runs one column / row per lane).  coef: 64
// quantized coefficients (natural order); q: quant table (natural order, read as
// ISLOW_MULT_TYPE = short, as jddctmgr.c does in a SIMD build); out: 8x8 samples.
DHD void idct_block(const int16_t* coef, const uint16_t* q, uint8_t* out, int64_t pitch) {
  bool dc_only = true;
  for (int k = 8; k < 64; ++k) dc_only = dc_only && coef[k] == 0;
  int32_t ws[64];
  for (int c = 0; c < 8; ++c) {
    int32_t cc[8], qq[8], w[8];
    for (int r = 0; r < 8; ++r) {
      cc[r] = coef[r * 8 + c];
      qq[r] = (int32_t)(int16_t)q[r * 8 + c];
    }
    idct_pass1(cc, qq, dc_only, w);
    for (int r = 0; r < 8; ++r) ws[r * 8 + c] = w[r];
  }
  for (int r = 0; r < 8; ++r) idct_pass2(ws + r * 8, out + r * pitch);
}

}  // namespace dino
