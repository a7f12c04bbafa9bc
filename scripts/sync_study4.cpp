// Multi-hypothesis start study of the speculative Huffman decode (analysis tool, host only).
// Each lane starts at its range start with every block-in-MCU phase c (z = 0) as a separate
// hypothesis.  Hypotheses advance in bit order; one that lands on a state another has
// visited at the same bit is merged into it, one that decodes an impossible symbol (zigzag
// past 63, a DC / AC category beyond 8-bit baseline) is dropped.  Reports, per lane: the
// bits until a single hypothesis remains, and whether that survivor is on the true path
// (and after how many bits the true decode joins it).
// build: g++ -O2 -std=c++17 -I. scripts/sync_study4.cpp -o /tmp/sync_study4
#include <stdio.h>
#include <stdlib.h>
#include <algorithm>
#include <map>
#include <unordered_map>
#include <vector>
#include "tests/emu/models.hpp"
using namespace dino;

int main(int argc, char** argv) {
  const int lanes = argc > 2 ? atoi(argv[2]) : 256;
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
  std::unordered_map<uint32_t, uint32_t> truth;  // pos -> (c << 8) | z
  {
    BitCursor cur;
    bc_init<kSrcPadded>(cur, br, 0);
    int32_t blk = 0, z = 0, nb = 0;
    while (cur.pos < nbits && nb < d.total_blocks) {
      truth[cur.pos] = ((uint32_t)blk << 8) | (uint32_t)z;
      StepOut o = huff_step<kSrcPadded>(cur, br, im, blk, z);
      nb += o.block_done;
    }
  }
  const int P = im.blocks_per_mcu;
  uint32_t sub = ((nbits + lanes - 1) / lanes + 31) & ~31u;
  long n_one = 0, n_true = 0, n_lanes = 0, n_never = 0, bits_one = 0, steps_all = 0, bits_join = 0;
  std::vector<long> hist(14, 0);
  for (int i = 1; i < lanes && i * sub < nbits; ++i) {
    const uint32_t start = i * sub, end = std::min(nbits, (i + 1) * sub);
    struct H { BitCursor cur; int32_t blk, z; bool alive; };
    std::vector<H> hs(P);
    for (int c = 0; c < P; ++c) {
      bc_init<kSrcPadded>(hs[c].cur, br, start);
      hs[c].blk = c; hs[c].z = 0; hs[c].alive = true;
    }
    std::multimap<uint32_t, std::pair<uint32_t, int>> seen;  // pos -> (state, hyp)
    int alive = P, steps = 0;
    uint32_t single_at = 0;
    while (alive > 1) {
      int h = -1;
      for (int c = 0; c < P; ++c)
        if (hs[c].alive && (h < 0 || hs[c].cur.pos < hs[h].cur.pos)) h = c;
      if (hs[h].cur.pos >= end + 4096) break;
      const uint32_t st = ((uint32_t)hs[h].blk << 8) | (uint32_t)hs[h].z;
      bool merged = false;
      auto rg = seen.equal_range(hs[h].cur.pos);
      for (auto it = rg.first; it != rg.second; ++it)
        if (it->second.first == st && it->second.second != h && hs[it->second.second].alive) merged = true;
      if (merged) { hs[h].alive = false; --alive; continue; }
      seen.emplace(hs[h].cur.pos, std::make_pair(st, h));
      const int zb = hs[h].z;
      StepOut o = huff_step<kSrcPadded>(hs[h].cur, br, im, hs[h].blk, hs[h].z);
      ++steps;
      const bool bad = (o.kind == 1 && o.zz > 63) || (o.kind == 0 && (o.value > 2047 || o.value < -2047)) ||
                       (o.kind == 1 && (o.value > 1023 || o.value < -1023));
      (void)zb;
      if (bad && alive > 1) { hs[h].alive = false; --alive; }
    }
    ++n_lanes;
    steps_all += steps;
    if (alive != 1) { ++n_never; continue; }
    int h = 0;
    while (!hs[h].alive) ++h;
    single_at = hs[h].cur.pos;
    ++n_one;
    bits_one += single_at - start;
    int b = 0;
    while ((1u << b) <= single_at - start && b < 13) ++b;
    hist[b]++;
    // does the survivor follow the true path?  walk it to the end of the range
    BitCursor cur = hs[h].cur;
    int32_t blk = hs[h].blk, z = hs[h].z;
    bool on = false;
    while (cur.pos < end + 2048) {
      auto it = truth.find(cur.pos);
      if (it != truth.end() && it->second == (((uint32_t)blk << 8) | (uint32_t)z)) { on = true; break; }
      huff_step<kSrcPadded>(cur, br, im, blk, z);
    }
    if (on) { ++n_true; bits_join += cur.pos - start; }
  }
  printf("%s lanes %d sub %u: %ld lanes, single survivor %ld (never %ld), survivor on the true path %ld; "
         "mean bits to one survivor %.0f, mean bits to true %.0f, hyp steps per lane %.0f; log2 bits hist:",
         argv[1], lanes, sub, n_lanes, n_one, n_never, n_true, n_one ? (double)bits_one / n_one : 0.0,
         n_true ? (double)bits_join / n_true : 0.0, (double)steps_all / std::max(1L, n_lanes));
  for (int b = 0; b < 14; ++b) printf(" %ld", hist[b]);
  printf("\n");
  return 0;
}
