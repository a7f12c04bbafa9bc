// Wave-level step mix of k_huff1's first decode on one image (analysis tool, host only).
// Each of 256 lanes decodes its range from a guessed state; lanes advance one step per
// wave iteration, 64 to a wave.  Counts, per wave iteration, how often ANY lane of the
// wave takes the long-code path (AC > kLookBits / DC > kDcLookBits bits), is at a block
// boundary (checkpoint branch), or decodes a DC vs AC symbol, and the per-symbol rates.
// usage: step_study FILE.jpg [lookbits_for_report]
#include <stdio.h>
#include <stdlib.h>
#include <algorithm>
#include <vector>
#include "tests/emu/models.hpp"
using namespace dino;

struct Flags {
  uint8_t slow_ac, slow_dc, dc, boundary;
  uint8_t len;  // code length
};

int main(int argc, char** argv) {
  const int lanes = 256;
  FILE* f = fopen(argv[1], "rb");
  std::vector<uint8_t> buf(1 << 24);
  size_t n = fread(buf.data(), 1, buf.size(), f);
  fclose(f);
  ImgDesc d;
  parse_jpeg(buf.data(), n, 1 << 16, &d);
  Destuffed ds = model_destuff(buf.data() + d.scan_off, (int)(n - d.scan_off));
  HuffTables* tabs = new HuffTables;
  HuffImage im;
  model_tables(buf.data(), d, tabs, im);
  const BitReader br{(const uint32_t*)ds.bytes.data(), (uint32_t)ds.len};
  const uint32_t nbits = ds.len * 8;
  uint32_t sub = ((nbits + lanes - 1) / lanes + 31) & ~31u;
  int nl = std::min(lanes, (int)((nbits + sub - 1) / sub));
  std::vector<std::vector<Flags>> steps(nl);
  long slow_len[18] = {0};
  long nsym = 0, nslow_ac = 0, nslow_dc = 0, ndc = 0, len_hist[18] = {0};
  for (int i = 0; i < nl; ++i) {
    uint32_t end = i == nl - 1 ? nbits : (i + 1) * sub;
    BitCursor cur;
    bc_init<kSrcPadded>(cur, br, i * sub);
    int32_t blk = 0, z = 0;
    while (cur.pos < end) {
      bc_fill<kSrcPadded>(cur, br);
      Flags fl{};
      const bool dc = z == 0;
      const int comp = hi_comp(im, blk);
      const HuffTable* t = dc ? reinterpret_cast<const HuffTable*>(im.tabs->dc + comp) : im.tabs->ac + comp;
      const uint32_t hi32 = (uint32_t)(cur.buf >> 32);
      const uint32_t e = t->look[hi32 >> (dc ? 32 - kDcLookBits : 32 - kLookBits)];
      fl.dc = dc;
      fl.boundary = dc;
      if (!e) {
        (dc ? fl.slow_dc : fl.slow_ac) = 1;
        int sym, len;
        if (dc) huff_slow(cur, im.tabs->dc + comp, &sym, &len);
        else huff_slow(cur, im.tabs->ac + comp, &sym, &len);
        slow_len[len < 18 ? len : 17]++;
      }
      huff_step<kSrcPadded>(cur, br, im, blk, z);
      steps[i].push_back(fl);
      ++nsym;
      nslow_ac += fl.slow_ac;
      nslow_dc += fl.slow_dc;
      ndc += dc;
      if (e) len_hist[e & 31]++;
    }
  }
  long iters = 0, any_slow_ac = 0, any_slow_dc = 0, any_dc = 0, all_dc = 0, active_lane_steps = 0;
  for (int w = 0; w * 64 < nl; ++w) {
    size_t mx = 0;
    for (int l = w * 64; l < std::min(nl, w * 64 + 64); ++l) mx = std::max(mx, steps[l].size());
    for (size_t k = 0; k < mx; ++k) {
      int sa = 0, sd = 0, dcn = 0, act = 0;
      for (int l = w * 64; l < std::min(nl, w * 64 + 64); ++l) {
        if (k >= steps[l].size()) continue;
        ++act;
        sa |= steps[l][k].slow_ac;
        sd |= steps[l][k].slow_dc;
        dcn += steps[l][k].dc;
      }
      ++iters;
      any_slow_ac += sa;
      any_slow_dc += sd;
      any_dc += dcn > 0;
      all_dc += dcn == act;
      active_lane_steps += act;
    }
  }
  printf("bits %u lanes %d sub %u symbols %ld (%.2f bits/sym) dc %.3f slow_ac/sym %.4f slow_dc/sym %.4f\n", nbits, nl,
         sub, nsym, (double)nbits / nsym, (double)ndc / nsym, (double)nslow_ac / nsym, (double)nslow_dc / nsym);
  printf("wave iters %ld (lane util %.3f): any slow_ac %.3f any slow_dc %.3f any dc %.3f all dc %.3f\n", iters,
         (double)active_lane_steps / (iters * 64.0), (double)any_slow_ac / iters, (double)any_slow_dc / iters,
         (double)any_dc / iters, (double)all_dc / iters);
  printf("code length hist (fast path):");
  for (int l = 1; l <= 16; ++l) printf(" %d:%ld", l, len_hist[l]);
  printf("\nslow code lengths:");
  for (int l = 1; l <= 17; ++l) if (slow_len[l]) printf(" %d:%ld", l, slow_len[l]);
  printf("\n");
  return 0;
}
