// color.hpp — chroma upsampling (libjpeg-turbo jdsample.c, do_fancy_upsampling =
// TRUE, which is Pillow's setting) and colour conversion (jdcolor.c
// ycc_rgb_convert, fixed point with SCALEBITS 16), evaluated per output pixel.
//
// libjpeg's row/column context rules become index clamps: the row above the
// first row is row 0 (jdmainct.c make_funny_pointers), rows past the last real
// sample row repeat it (set_bottom_pointers), and the first/last column cases
// of the fancy upsamplers equal a clamp of the neighbour column.
#pragma once

#include "common.hpp"

namespace dino {

enum UpMethod : int32_t { kUpFull = 0, kUpH2V1Fancy, kUpH2V1Box, kUpH1V2Fancy, kUpH2V2Fancy, kUpH2V2Box, kUpInt };

// jinit_upsampler method choice for one component.
DHD int upsample_method(int hf, int vf, int dw) {
  if (hf == 1 && vf == 1) return kUpFull;
  if (hf == 2 && vf == 1) return dw > 2 ? kUpH2V1Fancy : kUpH2V1Box;
  if (hf == 1 && vf == 2) return kUpH1V2Fancy;
  if (hf == 2 && vf == 2) return dw > 2 ? kUpH2V2Fancy : kUpH2V2Box;
  return kUpInt;
}

struct PlaneView {
  const uint8_t* p;
  int32_t pitch;   // bytes per row
  int32_t dw, dh;  // valid samples
  int32_t hf, vf;  // max_h / h, max_v / v
  int32_t method;
};

DHD int clampi(int x, int lo, int hi) { return x < lo ? lo : (x > hi ? hi : x); }

DHD int pv_at(const PlaneView& v, int x, int y) { return v.p[(int64_t)y * v.pitch + x]; }

// Component sample at full-resolution pixel (x, y).
DHD int upsample_at(const PlaneView& v, int x, int y) {
  switch (v.method) {
    case kUpFull:
      return pv_at(v, x, y);
    case kUpH2V1Fancy: {
      int c = x >> 1;
      int n = (x & 1) ? clampi(c + 1, 0, v.dw - 1) : clampi(c - 1, 0, v.dw - 1);
      int bias = (x & 1) ? 2 : 1;
      return (pv_at(v, c, y) * 3 + pv_at(v, n, y) + bias) >> 2;
    }
    case kUpH1V2Fancy: {
      int r = y >> 1;
      int n = (y & 1) ? clampi(r + 1, 0, v.dh - 1) : clampi(r - 1, 0, v.dh - 1);
      int bias = (y & 1) ? 2 : 1;
      return (pv_at(v, x, r) * 3 + pv_at(v, x, n) + bias) >> 2;
    }
    case kUpH2V2Fancy: {
      int r = y >> 1, c = x >> 1;
      int rn = (y & 1) ? clampi(r + 1, 0, v.dh - 1) : clampi(r - 1, 0, v.dh - 1);
      int cn = (x & 1) ? clampi(c + 1, 0, v.dw - 1) : clampi(c - 1, 0, v.dw - 1);
      int cs_this = pv_at(v, c, r) * 3 + pv_at(v, c, rn);
      int cs_next = pv_at(v, cn, r) * 3 + pv_at(v, cn, rn);
      return (x & 1) ? (cs_this * 3 + cs_next + 7) >> 4 : (cs_this * 3 + cs_next + 8) >> 4;
    }
    default:  // box replication (h2v1_upsample, h2v2_upsample, int_upsample)
      return pv_at(v, x / v.hf, y / v.vf);
  }
}

DHD uint8_t clamp255(int x) { return (uint8_t)(x < 0 ? 0 : (x > 255 ? 255 : x)); }

// jdcolor.c build_ycc_rgb_table + ycc_rgb_convert.
DHD void ycc_to_rgb(int y, int cb, int cr, uint8_t* rgb) {
  const int32_t kHalf = 1 << 15;
  int xcr = cr - 128, xcb = cb - 128;
  int r_add = (91881 * xcr + kHalf) >> 16;            // FIX(1.40200)
  int b_add = (116130 * xcb + kHalf) >> 16;           // FIX(1.77200)
  int g_add = ((-46802) * xcr + (-22554) * xcb + kHalf) >> 16;  // FIX(0.71414), FIX(0.34414)
  rgb[0] = clamp255(y + r_add);
  rgb[1] = clamp255(y + g_add);
  rgb[2] = clamp255(y + b_add);
}

}  // namespace dino
