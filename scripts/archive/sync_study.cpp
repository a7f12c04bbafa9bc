// Sync-distance study of the speculative Huffman decode (analysis tool, host only).
// For each lane of a one-segment image: decode from the guessed state {i*sub, c, 0}
// and report after how many steps the decode first stands on a true step boundary
// (bit-aligned) and on the true state (pos, c, z), and whether that happens in range.
// build: g++ -O2 -std=c++17 -I. scripts/sync_study.cpp -o /tmp/sync_study
#include <stdio.h>
#include <stdlib.h>
#include <unordered_map>
#include <vector>
#include "tests/emu/models.hpp"
using namespace dino;

int main(int argc, char** argv) {
  int lanes = argc > 2 ? atoi(argv[2]) : 256;
  const int heur = argc > 3 ? atoi(argv[3]) : 0;
  long jumps_total = 0;
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
  // true decode: state at every step start
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
  uint32_t sub = (nbits + lanes - 1) / lanes;
  sub = (sub + 31) & ~31u;
  int never = 0, aligned_wrong = 0;
  long steps_sync = 0, steps_range = 0, n_sync = 0;
  std::vector<int> hist(12, 0);
  long fa_steps = 0, n_fa = 0, fa_c = 0, fa_z = 0, fa_bothdc = 0;
  for (int i = 1; i < lanes; ++i) {
    const uint32_t start = i * sub, end = std::min(nbits, (i + 1) * sub);
    BitCursor cur;
    bc_init<kSrcPadded>(cur, br, start);
    int32_t blk = 0, z = 0;
    int steps = 0, first_align = -1, sync = -1, blocks = 0, njump = 0;
    uint32_t bpos = start;
    int bc = 0;
    while (cur.pos < end) {
      auto it = truth.find(cur.pos);
      if (it != truth.end()) {
        if (first_align < 0) {
          first_align = steps;
          fa_steps += steps;
          ++n_fa;
          const uint32_t tc = it->second >> 8, tz = it->second & 255;
          if ((int)tc == blk) ++fa_c;
          if ((int)tz == z) ++fa_z;
          if (z == 0 && tz == 0) ++fa_bothdc;
        }
        if (it->second == (((uint32_t)blk << 8) | (uint32_t)z)) {
          sync = steps;
          break;
        }
      }
      const int zb = z;
      if (z == 0) {
        bpos = cur.pos;
        bc = blk;
      }
      StepOut o = huff_step<kSrcPadded>(cur, br, im, blk, z);
      const bool bad = (o.kind == 1 && o.zz > 63) || (o.kind == 2 && o.block_done && zb + 16 > 64 && zb != 0 && z == 0 && false) ||
                       (o.kind == 0 && (o.value > 2047 || o.value < -2047)) || (o.kind == 1 && (o.value > 1023 || o.value < -1023));
      blocks += o.block_done;
      ++steps;
      if (heur && bad && njump < heur) {
        ++njump;
        ++jumps_total;
        bc_init<kSrcPadded>(cur, br, bpos);
        blk = (bc + 1) % im.blocks_per_mcu;
        bc = blk;
        z = 0;
      }
    }
    int total = steps;
    if (sync < 0) {
      ++never;
      if (first_align >= 0) ++aligned_wrong;
    } else {
      steps_sync += sync;
      ++n_sync;
      int b = 0;
      while ((1 << b) <= blocks && b < 11) ++b;
      hist[b]++;
    }
    steps_range += total;
  }
  printf("%s lanes %d sub %u: never-sync %d (%.1f%%, %d of them bit-aligned at some point), mean sync steps %.1f, "
         "blocks-to-sync log2 hist:", argv[1], lanes, sub, never, 100.0 * never / (lanes - 1), aligned_wrong,
         n_sync ? (double)steps_sync / n_sync : 0.0);
  for (int b = 0; b < 12; ++b) printf(" %d", hist[b]);
  printf(" jumps %ld", jumps_total);
  printf("\n  first bit alignment after %.1f steps (n=%ld); there c right %ld, z right %ld, both at DC %ld\n",
         n_fa ? (double)fa_steps / n_fa : 0.0, n_fa, fa_c, fa_z, fa_bothdc);
  return 0;
}
