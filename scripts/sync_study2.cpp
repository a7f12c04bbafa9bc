// Sync distance (bits from the lane start to the first true state) per start phase c
// for every lane of a one-segment image: distribution of the best of subsets of
// phases.  Analysis tool, host only.
#include <stdio.h>
#include <stdlib.h>
#include <algorithm>
#include <unordered_map>
#include <vector>
#include "tests/emu/models.hpp"
using namespace dino;

int main(int argc, char** argv) {
  int lanes = argc > 2 ? atoi(argv[2]) : 256;
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
  std::unordered_map<uint32_t, uint32_t> truth;
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
  const int bpm = im.blocks_per_mcu;
  uint32_t sub = (nbits + lanes - 1) / lanes;
  const uint32_t cap = 40000;
  std::vector<std::vector<uint32_t>> D(bpm);
  for (int i = 1; i < lanes; ++i) {
    const uint32_t start = i * sub;
    if (start >= nbits) break;
    for (int c0 = 0; c0 < bpm; ++c0) {
      BitCursor cur;
      bc_init<kSrcPadded>(cur, br, start);
      int32_t blk = c0, z = 0;
      uint32_t dist = cap;
      while (cur.pos < nbits && cur.pos - start < cap) {
        auto it = truth.find(cur.pos);
        if (it != truth.end() && it->second == (((uint32_t)blk << 8) | (uint32_t)z)) {
          dist = cur.pos - start;
          break;
        }
        huff_step<kSrcPadded>(cur, br, im, blk, z);
      }
      D[c0].push_back(dist);
    }
  }
  const int m = (int)D[0].size();
  auto report = [&](const char* name, std::vector<int> phases) {
    std::vector<uint32_t> best(m);
    for (int k = 0; k < m; ++k) {
      uint32_t b = cap;
      for (int c : phases) b = std::min(b, D[c][k]);
      best[k] = b;
    }
    std::sort(best.begin(), best.end());
    double mean = 0;
    for (auto v : best) mean += v;
    printf("  %-12s mean %7.0f  p50 %6u p90 %6u p99 %6u max %6u  P(>2600) %.3f P(>5200) %.3f\n", name, mean / m,
           best[m / 2], best[m * 9 / 10], best[m * 99 / 100], best[m - 1],
           (double)(std::upper_bound(best.begin(), best.end(), 2600u) - best.begin() < m ? m - (std::upper_bound(best.begin(), best.end(), 2600u) - best.begin()) : 0) / m,
           (double)(m - (std::upper_bound(best.begin(), best.end(), 5200u) - best.begin())) / m);
  };
  printf("%s bpm %d lanes %d sub %u\n", argv[1], bpm, m, sub);
  report("c=0", {0});
  report("c=4", {4});
  report("c=0,4", {0, 4});
  report("c=0,2,4", {0, 2, 4});
  report("c=0,1,4,5", {0, 1, 4, 5});
  std::vector<int> all;
  for (int c = 0; c < bpm; ++c) all.push_back(c);
  report("all", all);
  return 0;
}
