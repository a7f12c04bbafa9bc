// Host emulator of the HIP kernels' per-lane logic — TEST INFRASTRUCTURE ONLY.
//
// Compiles the very same __host__ __device__ functions the kernels use
// (dataloader_amd/csrc/*.hpp) for the CPU, and drives them with plain loops
// that mimic the kernels' lane/phase structure, so the CPU test suite can
// check the device algorithms against Pillow without a GPU.  The product
// library never links this file.
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <vector>

#include "../../dataloader_amd/csrc/color.hpp"
#include "../../dataloader_amd/csrc/huffman.hpp"
#include "../../dataloader_amd/csrc/idct.hpp"
#include "../../dataloader_amd/csrc/jpeg_parse.hpp"
#include "../../dataloader_amd/csrc/pixel_ops.hpp"
#include "../../dataloader_amd/csrc/resize.hpp"
#include "../../dataloader_amd/csrc/augment.hpp"
#include "../../dataloader_amd/csrc/mask.hpp"
#include "models.hpp"
#include "../../dataloader_amd/csrc/sampler.hpp"

using namespace dino;

extern "C" {

// ---- exhaustive pixel-op tables --------------------------------------------
void emu_rgb_to_hsv_all(uint8_t* out) {
  for (int r = 0; r < 256; ++r)
    for (int g = 0; g < 256; ++g)
      for (int b = 0; b < 256; ++b) {
        int h, s, v;
        rgb_to_hsv(r, g, b, &h, &s, &v);
        size_t i = (((size_t)r << 16) | (g << 8) | b) * 3;
        out[i] = (uint8_t)h;
        out[i + 1] = (uint8_t)s;
        out[i + 2] = (uint8_t)v;
      }
}

void emu_hsv_to_rgb_all(uint8_t* out) {
  for (int h = 0; h < 256; ++h)
    for (int s = 0; s < 256; ++s)
      for (int v = 0; v < 256; ++v) {
        int r, g, b;
        hsv_to_rgb(h, s, v, &r, &g, &b);
        size_t i = (((size_t)h << 16) | (s << 8) | v) * 3;
        out[i] = (uint8_t)r;
        out[i + 1] = (uint8_t)g;
        out[i + 2] = (uint8_t)b;
      }
}

void emu_rgb_to_l_all(uint8_t* out) {
  for (int r = 0; r < 256; ++r)
    for (int g = 0; g < 256; ++g)
      for (int b = 0; b < 256; ++b) out[((size_t)r << 16) | (g << 8) | b] = (uint8_t)rgb_to_l(r, g, b);
}

// out[a*256+b] = blend(a, b, alpha)
void emu_blend_table(float alpha, uint8_t* out) {
  for (int a = 0; a < 256; ++a)
    for (int b = 0; b < 256; ++b) out[a * 256 + b] = blend_u8(a, b, alpha);
}

void emu_normalize(const uint8_t* in, int64_t n, float mean, float std, uint16_t* bf16_out, float* f32_out) {
  for (int64_t i = 0; i < n; ++i) {
    float v = u8_normalize(in[i], mean, std);
    f32_out[i] = v;
    bf16_out[i] = f32_to_bf16(v);
  }
}

void emu_fp8(const float* in, int64_t n, uint8_t* out) {
  for (int64_t i = 0; i < n; ++i) out[i] = f32_to_fp8e4m3(in[i]);
}

// ---- JPEG -------------------------------------------------------------------
int emu_parse(const uint8_t* p, int64_t len, int32_t* info /* status,w,h,ncomp,color,bpm,ri,scan_off */) {
  ImgDesc d;
  parse_jpeg(p, len, 1 << 16, &d);
  info[0] = d.status;
  info[1] = d.width;
  info[2] = d.height;
  info[3] = d.ncomp;
  info[4] = d.color;
  info[5] = d.blocks_per_mcu;
  info[6] = d.restart_interval;
  info[7] = d.scan_off;
  return d.status;
}

// Full decode through the kernel-model pipeline.  mode 0: sequential Huffman,
// mode 1: speculative parallel Huffman with `lanes` lanes.  out_rgb: w*h*3.
// stats (nullable): int32[4] = {sync rounds, redecoded subsequences, lanes used, 0}
int emu_decode(const uint8_t* p, int64_t len, int mode, int lanes, uint8_t* out_rgb, int32_t* stats) {
  return host_model_decode(p, len, mode, lanes, out_rgb, stats);
}

// Stage outputs of the decode model (for GPU debugging): sizes returned in sizes[3].
int emu_decode_stages(const uint8_t* p, int64_t len, int mode, int lanes, uint8_t* rgb, uint8_t* ent, int64_t ent_cap,
                      int16_t* coef, int64_t coef_cap, uint8_t* planes, int64_t plane_cap, int64_t* sizes) {
  StageCapture cap;
  int r = host_model_decode(p, len, mode, lanes, rgb, nullptr, &cap);
  sizes[0] = (int64_t)cap.ent.size();
  sizes[1] = (int64_t)cap.coef.size() * 2;
  sizes[2] = (int64_t)cap.planes.size();
  if (ent) memcpy(ent, cap.ent.data(), std::min<int64_t>(ent_cap, sizes[0]));
  if (coef) memcpy(coef, cap.coef.data(), std::min<int64_t>(coef_cap, sizes[1]));
  if (planes) memcpy(planes, cap.planes.data(), std::min<int64_t>(plane_cap, sizes[2]));
  return r;
}

// Per-scan symbol counts of a multi-scan image (analysis aid): out[i] = symbols of scan
// i, levels[i] = its dependency level; returns the number of scans (< 0: status).
int emu_prog_scan_stats(const uint8_t* p, int64_t len, int64_t* out, int32_t* levels, int32_t cap) {
  ImgDesc d;
  if (parse_jpeg(p, len, 1 << 16, &d) != DINO_IMG_OK || d.kind != 1) return -1;
  std::vector<ScanRec> scans(kMaxScans);
  HostMarkerFinder find;
  if (prog_walk(p, len, &d, scans.data(), find) != DINO_IMG_OK) return d.status;
  std::vector<int16_t> coef(d.coef_bytes / 2, 0);
  std::vector<ProgTable> tabs(8);
  for (int i = 0; i < d.n_scans && i < cap; ++i) {
    const ScanRec& sr = scans[i];
    ScanTables tb;
    for (int k = 0; k < 4; ++k) {
      tb.dc[k] = tb.ac[k] = &tabs[0];
      if (sr.dc_tab[k] >= 0 && prog_build_table(p + sr.dc_tab[k], true, &tabs[k])) tb.dc[k] = &tabs[k];
      if (sr.ac_tab[k] >= 0 && prog_build_table(p + sr.ac_tab[k], false, &tabs[4 + k])) tb.ac[k] = &tabs[4 + k];
    }
    const long before = g_prog_host_symbols;
    prog_decode_scan(p, len, d, sr, tb, coef.data(), kNaturalOrder);
    out[i] = g_prog_host_symbols - before;
    levels[i] = sr.level;
  }
  return d.n_scans;
}

// ---- resize + augment ---------------------------------------------------------
// Full per-view augment: src RGB (HWC), params, -> out (3*S*S) of dtype out_dtype.
int emu_augment_view(const uint8_t* rgb, int W, int H, const dino_view_params* vp, const float* mean,
                     const float* stdv, int out_dtype, void* out) {
  return host_model_augment(rgb, W, H, *vp, mean, stdv, out_dtype, out);
}

// Stage checkpoint: resized+flipped uint8 crop (HWC) only.
int emu_resized_crop(const uint8_t* rgb, int W, int H, const dino_view_params* vp, uint8_t* out) {
  return host_model_resized_crop(rgb, W, H, *vp, out);
}

// ---- masks ----------------------------------------------------------------------
int emu_masks(int H, int W, int target, int minp, int maxp, double la0, double la1, int n, uint32_t* py_state,
              uint32_t* np_state, uint8_t* out) {
  MaskParams mp{H, W, target, minp, maxp, la0, la1};
  MtState py, np;
  mt_load(py, py_state);
  mt_load(np, np_state);
  std::vector<uint8_t> scratch((size_t)H * W * 4 + 16);
  for (int i = 0; i < n; ++i) gen_mask(mp, py, np, out + (size_t)i * H * W, (int32_t*)scratch.data());
  mt_store(py, py_state);
  mt_store(np, np_state);
  return 0;
}

// ---- sampler ----------------------------------------------------------------------
int emu_sample_params(const dino_aug_config* cfg, uint64_t seed, uint64_t batch_index, int sample, int W,
                      int H, int ok, dino_view_params* out) {
  int nv = cfg->n_global + cfg->n_local;
  for (int v = 0; v < nv; ++v) sample_view(*cfg, seed, batch_index, sample, v, W, H, ok, &out[v]);
  return nv;
}

}  // extern "C"
