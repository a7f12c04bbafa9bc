// pscan.hpp — the coefficient-buffer scan decoder (progressive SOF2 files and
// sequential files whose components arrive in several scans), round 3.
//
// Semantics are progressive.hpp's (libjpeg-turbo 3.1 jdphuff.c decode_mcu_DC_first /
// decode_mcu_AC_first / decode_mcu_DC_refine / decode_mcu_AC_refine, jdhuff.c
// decode_mcu and jpeg_fill_bit_buffer, jdmarker.c read_restart_marker +
// jpeg_resync_to_restart); what changes is the machine it is written for.
//
// Device mapping (kernels.hip k_pwalk / k_pscan): one wave per *scan*.  The serial
// part of a scan — the bit reader, the Huffman lookups, the run/EOB bookkeeping — is
// wave-uniform code: every value it touches comes from kernel arguments or from
// loads through address-space-4 (constant) pointers, so the compiler keeps it in
// SGPRs and runs it on the scalar ALU, reading the stream bytes and the decoder
// tables through the scalar cache.  The lanes do the parallel part next to it: a
// coefficient sink that collects up to 64 (element, value) stores in lane registers
// (a select per entry) and writes them with one vector store; for AC refinement scans the
// lanes hold the 64 coefficients of a block (lane k = zigzag k), one ballot gives
// the block's non-zero mask for the scalar decoder, and the corrections it returns
// are applied and stored lane-parallel.  A 16-block group of coefficients is
// prefetched while the previous group is decoded.
//
// The round-2 k_prog ran a scan per lane of one wave per image: scans of a level
// diverged against each other, and every bit-reader refill and coefficient access
// was a dependent vector-memory or LDS round trip on that lane (~2000 cycles per
// symbol measured, scripts/prog_phases.py, profiles/r03_prog_phases_k_prog.txt).
//
// The host emulator runs the same functions with plain memory (HostCoefSink).
#pragma once

#include "progressive.hpp"

namespace dino {

#if defined(__HIP_DEVICE_COMPILE__)
#define DINO_CONST __attribute__((address_space(4)))
#else
#define DINO_CONST
#endif

// The aligned 32-bit word at absolute address a (device: s_load_dword).
DHD uint32_t pw32(uintptr_t a) { return *(const DINO_CONST uint32_t*)a; }

// ---------------------------------------------------------------------------
// Decoder tables in global memory (built once per image by k_pwalk)
// ---------------------------------------------------------------------------
constexpr int kPLookBits = 9;
struct PTab {
  uint16_t look[1 << kPLookBits];  // (symbol << 4) | code length; 0: code longer than kPLookBits
  int32_t maxcode[18];
  int32_t valoffset[18];
  uint32_t huffval[64];            // the 256 symbol bytes, packed little-endian
  uint32_t pad[284];
};
static_assert(sizeof(PTab) == 2560, "PTab layout");

// Fill a PTab from a derived table (huff_build_derived) of the same code.
template <typename Src>
DHD void ptab_fill_derived(const Src* t, PTab* o) {
  for (int l = 0; l < 18; ++l) {
    o->maxcode[l] = t->maxcode[l];
    o->valoffset[l] = t->valoffset[l];
  }
  for (int i = 0; i < 64; ++i)
    o->huffval[i] = (uint32_t)t->huffval[4 * i] | (uint32_t)t->huffval[4 * i + 1] << 8 |
                    (uint32_t)t->huffval[4 * i + 2] << 16 | (uint32_t)t->huffval[4 * i + 3] << 24;
  for (int i = 0; i < 284; ++i) o->pad[i] = 0;
}
template <typename Src>
DHD uint16_t ptab_look_entry(const Src* t, int idx) {
  for (int l = 1; l <= kPLookBits; ++l) {
    const int code = idx >> (kPLookBits - l);
    if (code <= t->maxcode[l]) return (uint16_t)((uint32_t)t->huffval[(code + t->valoffset[l]) & 255] << 4 | (uint32_t)l);
  }
  return 0;
}

// Codes longer than the lookahead: the canonical-code search over the lengths
// kPLookBits + 1 .. 16, libjpeg's l = 17 fake zero when none matches.  p: the next 32 bits.
DHD void ptab_slow(const DINO_CONST PTab* t, uint32_t p, int* sym, int* len) {
  const uint32_t p17 = p >> 15;
  int32_t mc[16 - kPLookBits], vo[16 - kPLookBits];  // loaded together (one scalar-cache wait)
#pragma unroll
  for (int q = 0; q < 16 - kPLookBits; ++q) {
    mc[q] = t->maxcode[kPLookBits + 1 + q];
    vo[q] = t->valoffset[kPLookBits + 1 + q];
  }
  int l = 17, off = 0;
#pragma unroll
  for (int q = 16 - kPLookBits - 1; q >= 0; --q) {  // the shortest matching length wins
    if ((int32_t)(p17 >> (17 - (kPLookBits + 1 + q))) <= mc[q]) {
      l = kPLookBits + 1 + q;
      off = vo[q];
    }
  }
  *len = l;
  if (l > 16) {
    *sym = 0;  // JWRN_HUFF_BAD_CODE
    return;
  }
  const int ix = ((int)(p17 >> (17 - l)) + off) & 255;
  *sym = (int)((t->huffval[ix >> 2] >> (8 * (ix & 3))) & 0xFFu);
}

// ---------------------------------------------------------------------------
// Per-image scan list (k_pwalk -> k_pscan), in the image's htab region:
//   PHdr | PScan[kMaxScans] (sorted by dependency level, stable) | PTab[ntab]
// ---------------------------------------------------------------------------
// Dependency-level order of the scans (stable): rank of scan i.
DHD int prog_level_rank(const ScanRec* scans, int n, int i) {
  int r = 0;
  for (int j = 0; j < n; ++j)
    r += scans[j].level < scans[i].level || (scans[j].level == scans[i].level && j < i);
  return r;
}

struct PScan {
  ScanRec sr;
  int32_t dlen;     // lane images: the scan's destuffed bytes (k_pwalk)
  uint64_t tslots;  // byte k: table slot of DC table k (k < 4) / AC table k - 4; 0xFF none
  uint64_t deps;    // pipelined scans: byte k = sorted index of an earlier scan it reads after, 0xFF none
  int32_t pipe;     // 1: follows its dependencies block by block (prog_pipelined), 0: waits for its level
  int32_t slot;     // lane images: the refinement slot it records into (lane_plan), -1 none
};
static_assert(sizeof(PScan) == 112, "PScan layout");
struct PHdr {
  int32_t n_scans, n_levels;
  int32_t cnt[kMaxScans];   // scans per level
  int32_t done[kMaxScans];  // scans of each level completed (k_pscan)
  int32_t prog[kMaxScans];  // blocks each scan (sorted index) has finished and published
  int32_t lane;             // 1: decoded by k_plscan + k_papply (lscan.hpp), 0: by k_pscan
  uint32_t lane_nac, lane_ndc, lane_al_dc;  // lane_pack
  uint64_t lane_al_ac;
  uint64_t lane_band[3];
  int32_t pad[2];
};
static_assert(sizeof(PHdr) == 832, "PHdr layout");

// Scans whose coefficient sets intersect (a shared component and overlapping write ranges,
// scan_write_end; AC scans only, which are progressive).
DHD bool scans_overlap(const ScanRec& a, const ScanRec& b) {
  if (scan_write_end(a, true) < b.ss || scan_write_end(b, true) < a.ss) return false;
  for (int i = 0; i < a.ns && i < 4; ++i)
    for (int j = 0; j < b.ns && j < 4; ++j)
      if (a.comp[i] == b.comp[j]) return true;
  return false;
}
// A scan k_pscan decodes on its block-streaming AC path (one component, destuffed reader).
DHD bool scan_streams(const ScanRec& a, bool progressive) {
  return progressive && a.ss > 0 && a.ns == 1 && a.restart_interval == 0;
}
// Block pipelining: scan i may follow the earlier scans that wrote its coefficients block by
// block (instead of waiting for their whole level) when it and all of them stream the same
// component's blocks in the same raster order.  deps: their sorted indices (rank).
DHD bool prog_pipelined(const ScanRec* scans, int n, int i, bool progressive, uint64_t* deps) {
  *deps = ~0ull;
  if (!scan_streams(scans[i], progressive)) return false;
  int nd = 0;
  for (int j = 0; j < i; ++j) {
    if (!scans_overlap(scans[j], scans[i])) continue;
    if (nd == 8 || !scan_streams(scans[j], progressive) || scans[j].comp[0] != scans[i].comp[0]) {
      *deps = ~0ull;
      return false;
    }
    const uint64_t r = (uint64_t)prog_level_rank(scans, n, j);
    *deps = (*deps & ~(0xFFull << (8 * nd))) | (r << (8 * nd));
    ++nd;
  }
  return true;
}
constexpr int64_t kPScanOff = sizeof(PHdr);
constexpr int64_t kPTabOff = kPScanOff + (int64_t)kMaxScans * sizeof(PScan);
constexpr int kPMaxTabs = 32;  // distinct DHT tables an image's scans may use (more: host decode)
constexpr int64_t kPRegionBytes = kPTabOff + (int64_t)kPMaxTabs * sizeof(PTab);
DHD int ptab_capacity(int64_t region_bytes) {
  const int64_t n = (region_bytes - kPTabOff) / (int64_t)sizeof(PTab);
  return n < 0 ? 0 : (n > kPMaxTabs ? kPMaxTabs : (int)n);
}

// Table slots: every distinct table definition (BITS offset) the scans use gets a
// slot.  Returns the slot count, or -1 when more than `cap` are needed.
DHD int prog_table_slots(const ScanRec* scans, int n, int32_t* slot_off, uint8_t* slot_dc, uint64_t* tslots,
                         int cap) {
  int ns = 0;
  for (int i = 0; i < n; ++i) {
    uint64_t ts = ~0ull;
    for (int k = 0; k < 8; ++k) {
      const int32_t off = k < 4 ? scans[i].dc_tab[k] : scans[i].ac_tab[k - 4];
      if (off < 0) continue;
      int s = 0;
      while (s < ns && slot_off[s] != off) ++s;
      if (s == ns) {
        if (ns >= cap) return -1;
        slot_off[ns] = off;
        slot_dc[ns] = k < 4;
        ++ns;
      }
      ts = (ts & ~(0xFFull << (8 * k))) | ((uint64_t)s << (8 * k));
    }
    tslots[i] = ts;
  }
  return ns;
}


// ---------------------------------------------------------------------------
// Scalar bit reader over the raw (stuffed) scan bytes: RawBits' semantics, bytes
// fetched as aligned words (never a word that holds no byte of the image)
// ---------------------------------------------------------------------------
struct PBits {
  uintptr_t base;    // absolute address of image byte 0
  int64_t len;
  int64_t bp;        // next raw byte
  uint64_t buf;      // MSB aligned
  int32_t nbits, real, unread, insufficient;
};

DHD int pb_byte(const PBits& r, int64_t k) {
  const uintptr_t a = r.base + (uintptr_t)k;
  return (int)((pw32(a & ~(uintptr_t)3) >> (8 * (a & 3))) & 0xFFu);
}
// Bytes k..k+3 as a big-endian word (k + 8 <= len).
DHD uint32_t pb_be32(const PBits& r, int64_t k) {
  const uintptr_t a = r.base + (uintptr_t)k, A = a & ~(uintptr_t)3;
  const uint64_t x = ((uint64_t)pw32(A + 4) << 32 | pw32(A)) >> (8 * (a & 3));
  return bswap32((uint32_t)x);
}

DHD void pb_init(PBits& r, uintptr_t base, int64_t len, int64_t pos) {
  r.base = base;
  r.len = len;
  r.bp = pos;
  r.buf = 0;
  r.nbits = r.real = r.unread = r.insufficient = 0;
}

DHD void pb_fill(PBits& r) {
  while (r.nbits <= 32) {
    if (!r.unread) {
      if (r.bp + 8 <= r.len) {
        const uint32_t w = pb_be32(r, r.bp);
        const uint32_t t = ~w;  // a byte of w is 0xFF <=> that byte of t is 0
        if (!((t - 0x01010101u) & ~t & 0x80808080u)) {
          r.buf |= (uint64_t)w << (32 - r.nbits);
          r.nbits += 32;
          r.real += 32;
          r.bp += 4;
          continue;
        }
      }
      if (r.bp < r.len) {
        const int c = pb_byte(r, r.bp);
        if (c != 0xFF) {
          r.buf |= (uint64_t)c << (56 - r.nbits);
          r.nbits += 8;
          r.real += 8;
          r.bp += 1;
          continue;
        }
        int64_t k = r.bp + 1;
        while (k < r.len && pb_byte(r, k) == 0xFF) ++k;
        if (k < r.len && pb_byte(r, k) == 0) {  // stuffed FF
          r.buf |= (uint64_t)0xFF << (56 - r.nbits);
          r.nbits += 8;
          r.real += 8;
          r.bp = k + 1;
          continue;
        }
        r.unread = k < r.len ? pb_byte(r, k) : 0xD9;
        r.bp = k + 1;
      } else {
        r.unread = 0xD9;
      }
    }
    r.nbits += 32;  // zero fill
  }
}

DHD void pb_skip(PBits& r, int n) {
  r.buf <<= n;
  r.nbits -= n;
  r.real -= n;
  if (r.real < 0) {
    r.insufficient = 1;  // JWRN_HIT_MARKER
    r.real = 0;
  }
}

DHD uint32_t pb_bits(PBits& r, int n) {  // GET_BITS(n), 0 <= n <= 16
  pb_fill(r);
  const uint32_t v = n ? (uint32_t)(r.buf >> 32) >> (32 - n) : 0u;
  pb_skip(r, n);
  return v;
}

// next_marker_at on the scalar reader.
DHD int pb_next_marker(const PBits& r, int64_t pos, int64_t* after) {
  for (;;) {
    while (pos < r.len && pb_byte(r, pos) != 0xFF) ++pos;
    if (pos >= r.len) return -1;
    while (pos < r.len && pb_byte(r, pos) == 0xFF) ++pos;
    if (pos >= r.len) return -1;
    const int c = pb_byte(r, pos++);
    if (c != 0) {
      *after = pos;
      return c;
    }
  }
}

// process_restart: read_restart_marker + jpeg_resync_to_restart (rb_restart).
DHD void pb_restart(PBits& r, int* next_restart_num) {
  r.buf = 0;
  r.nbits = 0;
  r.real = 0;
  const int desired = *next_restart_num;
  if (!r.unread) {
    int64_t after = 0;
    const int c = pb_next_marker(r, r.bp, &after);
    r.unread = c < 0 ? 0xD9 : c;
    r.bp = c < 0 ? r.len : after;
  }
  if (r.unread == 0xD0 + desired) {
    r.unread = 0;
  } else {
    for (;;) {
      const int marker = r.unread;
      int action;
      if (marker < 0xC0)
        action = 2;
      else if (marker < 0xD0 || marker > 0xD7)
        action = 3;
      else if (marker == 0xD0 + ((desired + 1) & 7) || marker == 0xD0 + ((desired + 2) & 7))
        action = 3;
      else if (marker == 0xD0 + ((desired - 1) & 7) || marker == 0xD0 + ((desired - 2) & 7))
        action = 2;
      else
        action = 1;
      if (action == 1) {
        r.unread = 0;
        break;
      }
      if (action == 3) break;
      int64_t after = 0;
      const int c = pb_next_marker(r, r.bp, &after);
      r.unread = c < 0 ? 0xD9 : c;
      r.bp = c < 0 ? r.len : after;
    }
  }
  *next_restart_num = (desired + 1) & 7;
  if (!r.unread) r.insufficient = 0;
}


// ---------------------------------------------------------------------------
// Readers.  A reader gives the next 32 bits (peek), consumes bits (skip), reports
// libjpeg's insufficient_data flag and processes restart markers:
//   RawReader    the stuffed bytes (PBits: FF00, markers, restart resync)
//   HostClean /  the scan's entropy bytes destuffed first (FF00 -> FF, fill FFs
//   device       dropped, ended at the first other marker), then read as a plain bit
//   CleanReader  string; insufficient_data <=> more bits consumed than the string holds.
//                Used for scans without restart intervals.
// ---------------------------------------------------------------------------
struct RawReader {
  PBits b;
  DHD uint32_t peek() {
    pb_fill(b);
    return (uint32_t)(b.buf >> 32);
  }
  DHD void skip(int n) { pb_skip(b, n); }
  DHD bool insuff() const { return b.insufficient != 0; }
  DHD void restart(int* next_rst) { pb_restart(b, next_rst); }
};

// Destuffing rule of RawBits' fill: a byte other than FF is data, except a 00 right
// after an FF; an FF followed by 00 is a data FF; an FF followed by FF is fill; an FF
// followed by anything else (or by the end of the image) ends the data.
// Host form: the data bytes of [from, len) of p.
inline int64_t host_destuff(const uint8_t* p, int64_t len, int64_t from, uint8_t* out) {
  int64_t n = 0;
  for (int64_t i = from; i < len; ++i) {
    const int b = p[i];
    const int nx = i + 1 < len ? p[i + 1] : -1;
    if (b == 0xFF) {
      if (nx == 0x00) out[n++] = 0xFF;
      else if (nx != 0xFF) break;
    } else if (!(b == 0x00 && i > from && p[i - 1] == 0xFF)) {
      out[n++] = (uint8_t)b;
    }
  }
  return n;
}

struct HostClean {
  const uint8_t* s;   // destuffed bytes, >= 8 zero bytes of padding after n
  int64_t n;          // data bytes
  uint64_t pos = 0;   // bits consumed
  uint32_t peek() const {
    const uint64_t byte = pos >> 3;
    uint64_t x = 0;
    for (int k = 0; k < 5; ++k) x = x << 8 | (byte + k < (uint64_t)n ? s[byte + k] : 0u);
    return (uint32_t)((x << (24 + (pos & 7))) >> 32);
  }
  void skip(int k) { pos += (uint64_t)k; }
  bool insuff() const { return pos > (uint64_t)n * 8; }
  void restart(int*) {}
};

// GET_BITS(n), 0 <= n <= 16.
template <class R>
DHD uint32_t rbits(R& r, int n) {
  const uint32_t v = n ? r.peek() >> (32 - n) : 0u;
  r.skip(n);
  return v;
}

// Extra bits of a symbol from the same peek: the s bits after the len-bit code.
DHD uint32_t peek_extra(uint32_t p, int len, int s) { return s ? (p << len) >> (32 - s) : 0u; }

// Read one correction bit per set bit of c (increasing k) into corr.
template <class R>
DHD void r_corrections(R& r, uint64_t c, uint64_t* corr) {
  int n = __builtin_popcountll(c);
  while (n > 0) {
    const int take = n > 16 ? 16 : n;
    uint32_t bits = rbits(r, take) << (32 - take);
    for (int j = 0; j < take; ++j) {
      const uint64_t lowest = c & (~c + 1ull);
      if (bits & 0x80000000u) *corr |= lowest;
      bits <<= 1;
      c &= c - 1ull;
    }
    n -= take;
  }
}

// decode_mcu_AC_refine of one block on zigzag masks (ac_refine_block): nzz = the
// block's non-zero coefficients before the scan; returns corrections read as 1, new
// coefficients and their signs.
template <class R, class T>
DHD void r_refine_block(R& r, const T& t, int ss, int se, uint64_t nzz, int32_t* eobrun, uint64_t* corr_out,
                        uint64_t* new_out, uint64_t* neg_out) {
  uint64_t corr = 0, nzn = 0, neg = 0;
  int k = ss;
  const uint64_t band = (uint64_t)low_bits(se + 1) & ~(uint64_t)low_bits(ss);
  if (*eobrun == 0) {
    while (k <= se) {
      const uint32_t p = r.peek();
      int sym, len;
      t.lookup(4, p, &sym, &len);
      const int rr = sym >> 4, s = sym & 15;
      bool negative = false;
      if (s) {
        negative = peek_extra(p, len, 1) == 0;  // (a size other than 1 is a warning; the bit is read regardless)
        r.skip(len + 1);
      } else if (rr != 15) {
        *eobrun = (1 << rr) + (int32_t)peek_extra(p, len, rr);
        r.skip(len + rr);
        break;
      } else {
        r.skip(len);
      }
      // the (rr+1)-th not-yet-non-zero position at or after k (se + 1 when there is none)
      uint64_t z = ~nzz & band & ~(uint64_t)low_bits(k);
      for (int j = 0; j < rr && z; ++j) z &= z - 1ull;
      const int stop = z ? __builtin_ctzll(z) : se + 1;
      r_corrections(r, nzz & band & (uint64_t)low_bits(stop) & ~(uint64_t)low_bits(k), &corr);
      k = stop;
      if (s) {  // the new coefficient (k may be se + 1 on a corrupt stream: libjpeg's safety entries)
        const uint64_t bit = k < 64 ? 1ull << k : 1ull << 63;
        nzn |= bit;
        if (negative) neg |= bit;
        else neg &= ~bit;
      }
      ++k;
    }
  }
  if (*eobrun > 0) {
    if (k <= se) r_corrections(r, nzz & band & ~(uint64_t)low_bits(k), &corr);
    (*eobrun)--;
  }
  *corr_out = corr;
  *new_out = nzn;
  *neg_out = neg;
}

// Byte k of a packed word of bytes (constant-index selection, no private array).
DHD int pbyte64(uint64_t w, int k) { return (int)((w >> (8 * k)) & 0xFFu); }

// MCU geometry of a scan on an image descriptor reached through pointer type D
// (device: address space 4).  Per block of an interleaved MCU: component, x / y
// offsets and scan component index in 2-bit fields (scan_geom's layout).
template <typename D>
DHD ScanGeom pscan_geom(D d, const ScanRec& sr) {
  ScanGeom g;
  g.comp = g.bx = g.by = g.kk = 0;
  const int ncomp = d->ncomp;
#pragma unroll
  for (int c = 0; c < kMaxComp; ++c) {
    const int cc = c < ncomp ? c : 0;
    g.ch[c] = d->comp[cc].h;
    g.cv[c] = d->comp[cc].v;
    g.plane[c] = d->comp[cc].coef_off / 2;
    g.bw[c] = d->comp[cc].bw;
  }
  if (sr.ns == 1) {
    const int ci = sr.comp[0];
    g.mcus_x = ceil_div(d->comp[ci].dw, 8);
    g.mcus_y = ceil_div(d->comp[ci].dh, 8);
    g.bpm = 1;
    g.comp = (uint32_t)ci;
  } else {
    g.mcus_x = d->mcus_x;
    g.mcus_y = d->mcus_y;
    int b = 0;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      if (k >= sr.ns) break;
      const int ci = k == 0 ? sr.comp[0] : (k == 1 ? sr.comp[1] : (k == 2 ? sr.comp[2] : sr.comp[3]));
      const int h = sel3(g.ch, ci), v = sel3(g.cv, ci);
      for (int y = 0; y < v; ++y)
        for (int x = 0; x < h; ++x) {
          g.comp |= (uint32_t)ci << (2 * b);
          g.bx |= (uint32_t)x << (2 * b);
          g.by |= (uint32_t)y << (2 * b);
          g.kk |= (uint32_t)k << (2 * b);
          ++b;
        }
    }
    g.bpm = b;
  }
  return g;
}

// Coefficient element (int16 index from the image's coefficient base) of block blk of
// the MCU at (mx, my).
DHD int64_t pscan_block_elem(const ScanRec& sr, const ScanGeom& g, int mx, int my, int blk) {
  const int cc = sg_field(g.comp, blk);
  int bx = mx, by = my;
  if (sr.ns != 1) {
    bx = mx * sel3(g.ch, cc) + sg_field(g.bx, blk);
    by = my * sel3(g.cv, cc) + sg_field(g.by, blk);
  }
  return sel3(g.plane, cc) + ((int64_t)by * sel3(g.bw, cc) + bx) * 64;
}

// One whole scan.  T: lookup(k, p, &sym, &len) for table position k of the scan (DC
// table of scan component k < 4, AC table k - 4) and nat(k) (jpeg_natural_order with its
// safety entries).  Sink: set(elem, v) / orw(elem, v) for the sequential, DC and AC first
// scans and the DC refinement; rbegin / rnz / rapply for AC refinement (the block's
// zigzag non-zero mask before the scan, and the corrections to apply); flush() at the end.
template <typename R, typename T, typename D, typename Sink>
DHD void pscan_decode(R& r, const T& t, D d, const ScanRec& sr, bool prog, Sink& sink) {
  const ScanGeom g = pscan_geom(d, sr);
  const int ri = sr.restart_interval, al = sr.al, ss = sr.ss, se = sr.se;
  int rtg = ri, next_rst = 0;
  DcPred last_dc{0, 0, 0, 0};
  int32_t eobrun = 0;
  const bool ac_refine = prog && ss > 0 && sr.ah > 0;
  const bool ac_first = prog && ss > 0 && sr.ah == 0;
  const bool dc_refine = prog && ss == 0 && sr.ah > 0;
  if (ac_refine) sink.rbegin(sel3(g.plane, (int)g.comp), sel3(g.bw, (int)g.comp), g.mcus_x, g.mcus_y);
  int64_t m = 0;
  for (int my = 0; my < g.mcus_y; ++my) {
    for (int mx = 0; mx < g.mcus_x; ++mx, ++m) {
      if (ri) {
        if (rtg == 0) {
          r.restart(&next_rst);
          last_dc = DcPred{0, 0, 0, 0};
          eobrun = 0;
          rtg = ri;
        }
      }
      if (ac_refine) {
        const uint64_t nzz = sink.rnz(m);
        if (!r.insuff()) {
          uint64_t corr, nzn, neg;
          r_refine_block(r, t, ss, se, nzz, &eobrun, &corr, &nzn, &neg);
          sink.rapply(corr, nzn, neg, al);
        }
      } else if (!r.insuff()) {
        if (ac_first) {  // decode_mcu_AC_first (one block per MCU)
          if (eobrun > 0) {
            eobrun--;
          } else {
            const int64_t e0 = pscan_block_elem(sr, g, mx, my, 0);
            for (int k = ss; k <= se; k++) {
              const uint32_t p = r.peek();
              int sym, len;
              t.lookup(4, p, &sym, &len);
              const int rr = sym >> 4, s = sym & 15;
              if (s) {
                k += rr;
                const int v = huff_extend((int)peek_extra(p, len, s), s);
                r.skip(len + s);
                sink.set(e0 + t.nat(k), (int32_t)((uint32_t)v << al));
              } else if (rr == 15) {
                r.skip(len);
                k += 15;
              } else {
                eobrun = (1 << rr) + (int32_t)peek_extra(p, len, rr) - 1;
                r.skip(len + rr);
                break;
              }
            }
          }
        } else {
          for (int blk = 0; blk < g.bpm; ++blk) {
            const int64_t e0 = pscan_block_elem(sr, g, mx, my, blk);
            const int kk = sg_field(g.kk, blk);
            if (dc_refine) {  // decode_mcu_DC_refine
              if (rbits(r, 1)) sink.orw(e0, 1 << al);
              continue;
            }
            // DC symbol (decode_mcu_DC_first / decode_mcu)
            const uint32_t p = r.peek();
            int s, len;
            t.lookup(kk, p, &s, &len);
            const int dv = s ? huff_extend((int)peek_extra(p, len, s), s) : 0;
            r.skip(len + s);
            if (prog) {
              sink.set(e0, (int32_t)((uint32_t)last_dc.add(kk, dv) << al));
              continue;
            }
            sink.set(e0, last_dc.add(kk, dv));
            for (int k = 1; k < 64; k++) {  // jdhuff decode_mcu AC coefficients
              const uint32_t q = r.peek();
              int sym, ln;
              t.lookup(4 + kk, q, &sym, &ln);
              const int rr = sym >> 4, sv = sym & 15;
              if (sv) {
                k += rr;
                const int v = huff_extend((int)peek_extra(q, ln, sv), sv);
                r.skip(ln + sv);
                sink.set(e0 + t.nat(k), v);
              } else {
                r.skip(ln);
                if (rr != 15) break;
                k += 15;
              }
            }
          }
        }
      }
      if (ri) rtg--;
    }
  }
  sink.flush();
}

// Host tables: PTab array + the scan's slot word.
struct HostTabs {
  const PTab* tabs;
  uint64_t ts;
  void lookup(int k, uint32_t p, int* sym, int* len) const {
    const PTab* t = tabs + pbyte64(ts, k);
    const uint32_t e = t->look[p >> (32 - kPLookBits)];
    if (e) {
      *sym = (int)(e >> 4);
      *len = (int)(e & 15u);
    } else {
      ptab_slow((const DINO_CONST PTab*)t, p, sym, len);
    }
  }
  int nat(int k) const { return kNaturalOrder[k]; }
};

// Host sink: plain memory (the emulator and its tests).
struct HostCoefSink {
  int16_t* coef;
  int64_t plane = 0, cur = 0;
  int32_t bw = 0, mx = 1;
  void set(int64_t e, int32_t v) { coef[e] = (int16_t)v; }
  void orw(int64_t e, int32_t v) { coef[e] = (int16_t)(coef[e] | v); }
  void rbegin(int64_t pl, int32_t w, int32_t mcus_x, int32_t) {
    plane = pl;
    bw = w;
    mx = mcus_x;
  }
  uint64_t rnz(int64_t m) {
    const int64_t by = m / mx, bx = m - by * mx;
    cur = plane + (by * bw + bx) * 64;
    return block_nz_zz(coef + cur);
  }
  void rapply(uint64_t corr, uint64_t nzn, uint64_t neg, int al) {
    for (uint64_t mm = corr | nzn; mm; mm &= mm - 1) {
      const int k = __builtin_ctzll(mm);
      const int pos = kNaturalOrder[k];
      coef[cur + pos] = ac_refine_value(coef[cur + pos], (corr >> k) & 1u, (nzn >> k) & 1u, (neg >> k) & 1u, al);
    }
  }
  void flush() {}
};

}  // namespace dino
