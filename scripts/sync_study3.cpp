// Step-level simulation of k_huff1's sync phase on one image (analysis tool, host only):
// (a) synchronous rounds: each round costs the longest re-decode (in steps) of the
//     workgroup's lanes; (b) barrier-free polling: waves of 64 lanes advance in lockstep,
//     an iteration costs `budget` steps when any lane of the wave works, finality per
//     wave prefix.  Prints the sync-phase length in steps for both, and the first decode.
#include <stdio.h>
#include <stdlib.h>
#include <algorithm>
#include <vector>
#include "tests/emu/models.hpp"
using namespace dino;

struct Lane {
  HState S;
  RangeOut R, R1;
  int ncp;
  std::vector<Checkpoint> cps;
  uint32_t start, end;
};

// steps of a re-decode from st (same walk as decode_range_sync)
static int redo_steps(const BitReader& br, const HuffImage& im, const Lane& L, HState st, RangeOut* out) {
  RedoState r;
  redo_begin<kSrcPadded>(r, br, im, st);
  int steps = 0;
  while (!redo_run<kSrcPadded>(r, br, im, L.end, L.cps.data(), 1, L.ncp, L.R1, 1, out)) ++steps;
  return steps;
}

int main(int argc, char** argv) {
  const int lanes = 256, budget = argc > 2 ? atoi(argv[2]) : 8;
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
  std::vector<Lane> L(nl);
  int first_max = 0;
  for (int i = 0; i < nl; ++i) {
    L[i].start = i * sub;
    L[i].end = i == nl - 1 ? nbits : (i + 1) * sub;
    L[i].cps.resize(kHuffCheckpoints);
    L[i].S = HState{L[i].start, 0, 0};
    L[i].R = L[i].R1 = decode_range<kSrcPadded>(br, im, L[i].S, L[i].end, L[i].cps.data(), 1, kHuffCheckpoints, &L[i].ncp);
    // first-decode steps
    BitCursor cur;
    bc_init<kSrcPadded>(cur, br, L[i].start);
    int32_t blk = 0, z = 0, st = 0;
    while (cur.pos < L[i].end) { huff_step<kSrcPadded>(cur, br, im, blk, z); ++st; }
    first_max = std::max(first_max, st);
  }
  // (a) rounds
  std::vector<Lane> A = L;
  long rounds_steps = 0;
  int rounds = 0;
  for (;;) {
    std::vector<HState> want(nl);
    std::vector<char> redo(nl, 0);
    bool any = false;
    for (int i = 1; i < nl; ++i) {
      want[i] = A[i - 1].R.end;
      redo[i] = !hstate_eq(want[i], A[i].S);
      any |= redo[i];
    }
    ++rounds;
    if (!any) break;
    int mx = 0;
    for (int i = 1; i < nl; ++i)
      if (redo[i]) {
        A[i].S = want[i];
        mx = std::max(mx, redo_steps(br, im, A[i], want[i], &A[i].R));
      }
    rounds_steps += mx;
  }
  // (b) barrier-free, waves in lockstep (all waves advance one iteration per tick)
  std::vector<Lane> B = L;
  std::vector<uint64_t> E(nl);
  std::vector<char> fin(nl), working(nl, 0);
  std::vector<RedoState> rd(nl);
  std::vector<int> left(nl, 0);
  for (int i = 0; i < nl; ++i) {
    fin[i] = i == 0;
    E[i] = pack_end(B[i].R1.end) | (fin[i] ? kEndFinal : 0ull);
  }
  const int nw = (nl + 63) / 64;
  long ticks_steps = 0;
  int ticks = 0;
  for (;;) {
    bool all = true;
    for (char x : fin) all = all && x;
    if (all) break;
    ++ticks;
    std::vector<uint64_t> seen(nl);
    for (int i = 0; i < nl; ++i) seen[i] = i ? E[i - 1] : 0;
    int tick_cost = 1;  // an idle poll
    for (int w = 0; w < nw; ++w) {
      const int w0 = w * 64, w1 = std::min(nl, w0 + 64);
      uint64_t F = 0, N = 0, idle = 0, pf = 0;
      int wave_steps = 0;
      bool wave_fin = true;
      for (int i = w0; i < w1; ++i) wave_fin = wave_fin && fin[i];
      if (wave_fin) continue;
      for (int i = w0; i < w1; ++i) {
        const int wl = i - w0;
        if (!fin[i]) {
          const uint64_t v = seen[i];
          const HState pe = unpack_end(v);
          if (v & kEndFinal) pf |= 1ull << wl;
          if (!hstate_eq(pe, B[i].S)) {
            B[i].S = pe;
            redo_begin<kSrcPadded>(rd[i], br, im, pe);
            working[i] = 1;
          }
          if (working[i]) {
            int s = 0;
            bool done = false;
            while (s < budget) {
              ++s;
              if (redo_run<kSrcPadded>(rd[i], br, im, B[i].end, B[i].cps.data(), 1, B[i].ncp, B[i].R1, 1, &B[i].R)) {
                done = true;
                break;
              }
            }
            wave_steps = std::max(wave_steps, s);
            if (done) {
              working[i] = 0;
              N |= 1ull << wl;
              E[i] = pack_end(B[i].R.end);
            }
          }
        }
        if (fin[i]) F |= 1ull << wl;
        if (!working[i]) idle |= 1ull << wl;
      }
      for (int wl = w1 - w0; wl < 64; ++wl) F |= 1ull << wl;
      uint64_t P = F | (idle & ~(N << 1));
      if (!(F & 1ull) && !(pf & 1ull)) P &= ~1ull;
      const uint64_t run = ~P == 0ull ? ~0ull : (((~P) & (P + 1ull)) - 1ull);
      for (int i = w0; i < w1; ++i)
        if (!fin[i] && ((run >> (i - w0)) & 1ull)) {
          fin[i] = 1;
          E[i] = pack_end(B[i].R.end) | kEndFinal;
        }
      tick_cost = std::max(tick_cost, wave_steps);
    }
    ticks_steps += tick_cost;
  }
  bool same = true;
  for (int i = 0; i < nl; ++i) same = same && hstate_eq(A[i].S, B[i].S);
  printf("%s lanes %d: first decode %d steps; rounds %d -> %ld steps; barrier-free %d ticks -> %ld steps (budget %d)%s\n",
         argv[1], nl, first_max, rounds, rounds_steps, ticks, ticks_steps, budget, same ? "" : " MISMATCH");
  return 0;
}
