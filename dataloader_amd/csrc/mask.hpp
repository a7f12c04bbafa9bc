// mask.hpp — iBOT block-mask generation, bit-exact with reference
// MaskingGenerator (masking.py:148-269) driven by CPython's `random` and NumPy's
// legacy RandomState.  Both are MT19937; the state layout is the one
// random.getstate() / RandomState.get_state() expose (624 words + index), so
// the Python wrapper can seed exactly like `random.seed(s); np.random.seed(s)`.
//
// CPython algorithms (Lib/random.py, Modules/_randommodule.c):
//   random()      = (a*2^26 + b) / 2^53, a = next>>5, b = next>>6
//   uniform(a,b)  = a + (b-a)*random()
//   randint(a,b)  = a + _randbelow(b-a+1); _randbelow(n): k = n.bit_length(),
//                   r = getrandbits(k) until r < n; getrandbits(k<=32) = next >> (32-k)
// NumPy legacy (numpy/random/_legacy + distributions.c):
//   choice(a, k, replace=False) = a[permutation(len(a))[:k]]
//   permutation(n) = shuffle(arange(n)): for i = n-1..1: j = random_interval(i), swap
//   random_interval(max) = smallest all-ones mask >= max; next32 & mask until <= max
#pragma once

#include <math.h>

#include "common.hpp"

namespace dino {

struct MtState {
  uint32_t mt[624];
  int32_t idx;
};

DHD void mt_load(MtState& s, const uint32_t* w) {
  for (int i = 0; i < 624; ++i) s.mt[i] = w[i];
  s.idx = (int32_t)w[624];
}
DHD void mt_store(const MtState& s, uint32_t* w) {
  for (int i = 0; i < 624; ++i) w[i] = s.mt[i];
  w[624] = (uint32_t)s.idx;
}

DHD void mt_twist(MtState& s) {
  const uint32_t UPPER = 0x80000000u, LOWER = 0x7fffffffu, MATA = 0x9908b0dfu;
  int kk = 0;
  for (; kk < 624 - 397; ++kk) {
    uint32_t y = (s.mt[kk] & UPPER) | (s.mt[kk + 1] & LOWER);
    s.mt[kk] = s.mt[kk + 397] ^ (y >> 1) ^ ((y & 1u) ? MATA : 0u);
  }
  for (; kk < 623; ++kk) {
    uint32_t y = (s.mt[kk] & UPPER) | (s.mt[kk + 1] & LOWER);
    s.mt[kk] = s.mt[kk + (397 - 624)] ^ (y >> 1) ^ ((y & 1u) ? MATA : 0u);
  }
  uint32_t y = (s.mt[623] & UPPER) | (s.mt[0] & LOWER);
  s.mt[623] = s.mt[396] ^ (y >> 1) ^ ((y & 1u) ? MATA : 0u);
  s.idx = 0;
}

DHD uint32_t mt_next(MtState& s) {
  if (s.idx >= 624) mt_twist(s);
  uint32_t y = s.mt[s.idx++];
  y ^= (y >> 11);
  y ^= (y << 7) & 0x9d2c5680u;
  y ^= (y << 15) & 0xefc60000u;
  y ^= (y >> 18);
  return y;
}

DHD double py_random(MtState& s) {
  uint32_t a = mt_next(s) >> 5, b = mt_next(s) >> 6;
  return ((double)a * 67108864.0 + (double)b) * (1.0 / 9007199254740992.0);
}

DHD double py_uniform(MtState& s, double a, double b) { return a + (b - a) * py_random(s); }

DHD int bit_length(uint32_t n) {
  int k = 0;
  while (n) {
    ++k;
    n >>= 1;
  }
  return k;
}

DHD int py_randbelow(MtState& s, uint32_t n) {
  int k = bit_length(n);  // n >= 1 here
  uint32_t r = mt_next(s) >> (32 - k);
  while (r >= n) r = mt_next(s) >> (32 - k);
  return (int)r;
}

DHD int py_randint(MtState& s, int a, int b) { return a + py_randbelow(s, (uint32_t)(b - a + 1)); }

DHD uint32_t np_random_interval(MtState& s, uint32_t max) {
  if (max == 0) return 0;
  uint32_t mask = max;
  mask |= mask >> 1;
  mask |= mask >> 2;
  mask |= mask >> 4;
  mask |= mask >> 8;
  mask |= mask >> 16;
  uint32_t v;
  while ((v = (mt_next(s) & mask)) > max) {
  }
  return v;
}

struct MaskParams {
  int32_t H, W, target, min_patches, max_patches;
  double log_aspect0, log_aspect1;
};

// One mask (flat, H*W bytes 0/1).  scratch: >= H*W int32.
DHD void gen_mask(const MaskParams& mp, MtState& py, MtState& np, uint8_t* mask, int32_t* scratch) {
  const int H = mp.H, W = mp.W;
  for (int i = 0; i < H * W; ++i) mask[i] = 0;
  int count = 0;
  while (count < mp.target) {
    int remaining = mp.target - count;
    int cap = remaining < mp.max_patches ? remaining : mp.max_patches;
    int delta = 0;
    for (int attempt = 0; attempt < 10; ++attempt) {  // _place_block
      double target_area = py_uniform(py, (double)mp.min_patches, (double)cap);
      double aspect = exp(py_uniform(py, mp.log_aspect0, mp.log_aspect1));
      int h = (int)rint(sqrt(target_area * aspect));
      int w = (int)rint(sqrt(target_area / aspect));
      if (w >= W || h >= H) continue;
      int top = py_randint(py, 0, H - h);
      int left = py_randint(py, 0, W - w);
      int already = 0;
      for (int y = top; y < top + h; ++y)
        for (int x = left; x < left + w; ++x) already += mask[y * W + x];
      int nw = h * w - already;
      if (0 < nw && nw <= cap) {
        for (int y = top; y < top + h; ++y)
          for (int x = left; x < left + w; ++x) mask[y * W + x] = 1;
        delta = nw;
        break;
      }
    }
    if (delta == 0) break;
    count += delta;
  }
  // _complete_randomly
  int cur = 0;
  for (int i = 0; i < H * W; ++i) cur += mask[i];
  int shortfall = mp.target - cur;
  if (shortfall <= 0) return;
  int n = 0;
  for (int i = 0; i < H * W; ++i)
    if (!mask[i]) scratch[n++] = i;  // unmasked flat indices, ascending
  if (shortfall > n) shortfall = n;
  // permutation(n): shuffle arange(n), then take unmasked[perm[k]] for k < shortfall.
  // Shuffle the index array directly: unmasked[perm] == shuffle applied to unmasked.
  for (int i = n - 1; i > 0; --i) {
    int j = (int)np_random_interval(np, (uint32_t)i);
    int32_t t = scratch[i];
    scratch[i] = scratch[j];
    scratch[j] = t;
  }
  for (int k = 0; k < shortfall; ++k) mask[scratch[k]] = 1;
}

}  // namespace dino
