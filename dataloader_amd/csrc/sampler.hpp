// sampler.hpp — device-side draw of every random decision of one (sample, view),
// with the reference's distributions (cpu.py:172-267, torchvision
// RandomResizedCrop.get_params / ColorJitter.get_params) but a counter-based
// Philox4x32-10 stream keyed by (seed, batch_index, sample, view).  Unlike the
// reference (process-global RNGs consumed by up to 16 threads in arbitrary
// order) the result is independent of scheduling, and the drawn
// record is exported so the CPU oracle can replay it exactly.
#pragma once

#include <math.h>

#include "common.hpp"

namespace dino {

struct Philox {
  uint32_t ctr[4];
  uint32_t key[2];
  uint32_t out[4];
  int idx;
};

DHD void philox_round(uint32_t* c, const uint32_t* k) {
  const uint32_t M0 = 0xD2511F53u, M1 = 0xCD9E8D57u;
  uint64_t p0 = (uint64_t)M0 * c[0];
  uint64_t p1 = (uint64_t)M1 * c[2];
  uint32_t hi0 = (uint32_t)(p0 >> 32), lo0 = (uint32_t)p0;
  uint32_t hi1 = (uint32_t)(p1 >> 32), lo1 = (uint32_t)p1;
  uint32_t n0 = hi1 ^ c[1] ^ k[0];
  uint32_t n1 = lo1;
  uint32_t n2 = hi0 ^ c[3] ^ k[1];
  uint32_t n3 = lo0;
  c[0] = n0;
  c[1] = n1;
  c[2] = n2;
  c[3] = n3;
}

DHD void philox_block(const uint32_t* ctr, const uint32_t* key, uint32_t* out) {
  uint32_t c[4] = {ctr[0], ctr[1], ctr[2], ctr[3]};
  uint32_t k[2] = {key[0], key[1]};
  for (int r = 0; r < 10; ++r) {
    philox_round(c, k);
    k[0] += 0x9E3779B9u;
    k[1] += 0xBB67AE85u;
  }
  out[0] = c[0];
  out[1] = c[1];
  out[2] = c[2];
  out[3] = c[3];
}

DHD void philox_init(Philox& g, uint64_t seed, uint64_t batch_index, uint32_t sample, uint32_t view) {
  g.key[0] = (uint32_t)seed;
  g.key[1] = (uint32_t)(seed >> 32);
  g.ctr[0] = 0;
  g.ctr[1] = view;
  g.ctr[2] = sample;
  g.ctr[3] = (uint32_t)batch_index ^ (uint32_t)(batch_index >> 32) * 0x9E3779B9u;
  g.idx = 4;
}

DHD uint32_t philox_next(Philox& g) {
  if (g.idx == 4) {
    philox_block(g.ctr, g.key, g.out);
    g.ctr[0]++;
    g.idx = 0;
  }
  return g.out[g.idx++];
}

// float32 in [0, 1) with 24 random bits (torch's uniform_ resolution for float).
DHD float u01f(Philox& g) { return (float)(philox_next(g) >> 8) * (1.0f / 16777216.0f); }
// double in [0, 1) with 53 bits (Python random.random resolution).
DHD double u01d(Philox& g) {
  uint32_t a = philox_next(g) >> 5, b = philox_next(g) >> 6;
  return ((double)a * 67108864.0 + (double)b) * (1.0 / 9007199254740992.0);
}
// integer in [0, n) (n >= 1), Lemire multiply-shift.
DHD int32_t randbelow(Philox& g, int32_t n) { return (int32_t)(((uint64_t)philox_next(g) * (uint32_t)n) >> 32); }

DHD float uniform_f(Philox& g, float lo, float hi) { return lo + (hi - lo) * u01f(g); }

// Python round() on a double (half to even).
DHD double py_round(double x) { return rint(x); }

DHD void sample_view(const dino_aug_config& cfg, uint64_t seed, uint64_t batch_index, int sample, int view, int W,
                     int H, int ok, dino_view_params* out) {
  Philox g;
  philox_init(g, seed, batch_index, (uint32_t)sample, (uint32_t)view);
  dino_view_params p;
  const bool global = view < cfg.n_global;
  p.out_size = global ? cfg.global_size : cfg.local_size;
  const float* sc = global ? cfg.global_scale : cfg.local_scale;
  float blur_p = global ? (view == 0 ? cfg.blur_prob_global1 : cfg.blur_prob_global2) : cfg.blur_prob_local;
  float sol_p = (global && view == 1) ? cfg.solarize_prob : 0.0f;
  // ---- RandomResizedCrop.get_params (10 tries, then central crop) ----
  if (W < 1) W = 1;
  if (H < 1) H = 1;
  const double area = (double)H * (double)W;
  const float lr0 = (float)log(3.0 / 4.0), lr1 = (float)log(4.0 / 3.0);  // torch.log(tensor(ratio)) in f32
  int ci = -1, cj = 0, ch = 0, cw = 0;
  for (int t = 0; t < 10; ++t) {
    double target_area = area * (double)uniform_f(g, sc[0], sc[1]);
    double aspect = (double)(float)exp((double)uniform_f(g, lr0, lr1));
    int w = (int)py_round(sqrt(target_area * aspect));
    int h = (int)py_round(sqrt(target_area / aspect));
    uint32_t ri = philox_next(g), rj = philox_next(g);
    if (0 < w && w <= W && 0 < h && h <= H) {
      ch = h;
      cw = w;
      ci = (int)(((uint64_t)ri * (uint32_t)(H - h + 1)) >> 32);
      cj = (int)(((uint64_t)rj * (uint32_t)(W - w + 1)) >> 32);
      break;
    }
  }
  if (ci < 0) {
    double in_ratio = (double)W / (double)H;
    if (in_ratio < 3.0 / 4.0) {
      cw = W;
      ch = (int)py_round((double)cw / (3.0 / 4.0));
    } else if (in_ratio > 4.0 / 3.0) {
      ch = H;
      cw = (int)py_round((double)ch * (4.0 / 3.0));
    } else {
      cw = W;
      ch = H;
    }
    ci = (H - ch) / 2;
    cj = (W - cw) / 2;
  }
  p.crop_top = ci;
  p.crop_left = cj;
  p.crop_h = ch;
  p.crop_w = cw;
  // ---- flip, ColorJitter, grayscale, blur, solarize (cpu.py:256-266) ----
  p.flip = u01d(g) < (double)cfg.flip_prob;
  p.jitter = !(u01d(g) > (double)cfg.color_jitter_prob);
  uint8_t ord[4] = {0, 1, 2, 3};
  for (int i = 3; i > 0; --i) {  // uniform permutation (torch.randperm(4))
    int j = randbelow(g, i + 1);
    uint8_t tmp = ord[i];
    ord[i] = ord[j];
    ord[j] = tmp;
  }
  float bl = 1.0f - cfg.brightness, cl = 1.0f - cfg.contrast, sl = 1.0f - cfg.saturation;
  p.brightness = uniform_f(g, bl > 0.0f ? bl : 0.0f, 1.0f + cfg.brightness);
  p.contrast = uniform_f(g, cl > 0.0f ? cl : 0.0f, 1.0f + cfg.contrast);
  p.saturation = uniform_f(g, sl > 0.0f ? sl : 0.0f, 1.0f + cfg.saturation);
  p.hue = uniform_f(g, -cfg.hue, cfg.hue);
  for (int i = 0; i < 4; ++i) p.order[i] = ord[i];
  p.gray = u01d(g) < (double)cfg.grayscale_prob;
  p.blur = !(u01d(g) > (double)blur_p);
  double sig = (double)cfg.blur_sigma_min + ((double)cfg.blur_sigma_max - (double)cfg.blur_sigma_min) * u01d(g);
  p.sigma = p.blur ? sig : 1.0;
  int ks = ((int)(p.sigma * 4 + 1)) | 1;
  p.ksize = ks > 3 ? ks : 3;
  double su = u01d(g);
  p.solarize = (sol_p > 0.0f) && su < (double)sol_p;
  p.pad0[0] = p.pad0[1] = p.pad0[2] = 0;
  p.pad1 = ok ? 0 : 1;
  p.resize_w = p.resize_h = 0;
  p.out_x = p.out_y = 0;
  if (cfg.recipe == DINO_RECIPE_LEJEPA) {
    // CPULeJEPAPipeline (cpu.py:447-459): the context view keeps RRC + ColorJitter (with
    // probability color_jitter_prob) + flip; targets are RRC only; no grayscale, blur, solarize
    p.gray = 0;
    p.blur = 0;
    p.sigma = 1.0;
    p.ksize = 3;
    p.solarize = 0;
    if (!global) {
      p.flip = 0;
      p.jitter = 0;
    }
  } else if (cfg.recipe == DINO_RECIPE_EVAL) {
    // CPUEvalPipeline (cpu.py:400-411): Resize(int(S * 256 / 224)) of the shorter side, then
    // CenterCrop(S); deterministic.  The crop box is the whole image, resampled to the
    // torchvision output size, and the view is the centred window of it.
    const int S = p.out_size;
    const int size = (int)((double)S * 256.0 / 224.0);
    int nw, nh;
    if (W <= H) {
      nw = size;
      nh = (int)((double)size * (double)H / (double)W);
    } else {
      nw = (int)((double)size * (double)W / (double)H);
      nh = size;
    }
    p.flip = p.jitter = p.gray = p.blur = p.solarize = 0;
    p.sigma = 1.0;
    p.ksize = 3;
    p.crop_top = p.crop_left = 0;
    p.crop_w = W;
    p.crop_h = H;
    p.resize_w = nw;
    p.resize_h = nh;
    p.out_x = (int)py_round((double)(nw - S) / 2.0);
    p.out_y = (int)py_round((double)(nh - S) / 2.0);
    // an axis that is not resampled is a plain crop: fold its window into the crop box
    if (nw == W) {
      p.crop_left = p.out_x;
      p.crop_w = S;
      p.resize_w = S;
      p.out_x = 0;
    }
    if (nh == H) {
      p.crop_top = p.out_y;
      p.crop_h = S;
      p.resize_h = S;
      p.out_y = 0;
    }
  }
  if (!p.jitter) {
    p.brightness = p.contrast = p.saturation = 1.0f;
    p.hue = 0.0f;
    for (int i = 0; i < 4; ++i) p.order[i] = (uint8_t)i;
  }
  *out = p;
}

}  // namespace dino
