// progressive.hpp — multi-scan JPEG decoding (progressive SOF2, and sequential
// SOF0/SOF1 files whose components arrive in several scans), restated from
// libjpeg-turbo 3.1 (inside Pillow, the decoder the reference calls at
// cpu.py:251):
//   jdmarker.c   read_markers / get_sos / get_dht / get_dri / next_marker /
//                read_restart_marker, jdmarker.c jpeg_resync_to_restart
//   jdinput.c    per_scan_setup (MCU geometry of interleaved and non-interleaved
//                scans), latch_quant_tables
//   jdphuff.c    start_pass_phuff_decoder (scan validation, coef_bits), decode_mcu_DC_first,
//                decode_mcu_AC_first, decode_mcu_DC_refine, decode_mcu_AC_refine,
//                process_restart
//   jdhuff.c     decode_mcu (sequential scans of a multi-scan file), jpeg_fill_bit_buffer
//                (the zero fill and `insufficient_data` after a marker)
//   jdcoefct.c   smoothing_ok (block smoothing: images that would be smoothed are
//                reported DINO_IMG_UNSUPPORTED and decoded by the host fallback)
//
// The coefficients of such an image live in a dense int16 buffer (natural order,
// component planes of bw x bh blocks, CompDesc::coef_off), zeroed before the first
// scan; k_idct then transforms it like the baseline path's sparse entries.
//
// Device mapping (kernels.hip k_prog): one wave per image.  The wave walks the
// marker segments together (prog_walk, uniform control flow; the search for the
// end of each scan's entropy data is wave-cooperative), builds the scan table and
// a dependency level per scan; then scan i is decoded by lane i, level by level
// (scans of one level touch disjoint coefficients: different components or
// spectral bands).  The host emulator runs the same functions serially.
#pragma once

#include <cstring>

#include "huffman.hpp"

namespace dino {

constexpr int kMaxScans = DINO_MAX_SCANS;
constexpr int kProgLookBits = 9;
using ProgTable = HuffTableT<kProgLookBits>;

// LDS data of k_prog (tables, byte ring, refinement block, natural order) is reached
// through address-space-3 pointers on the device, so its accesses are ds_* (LDS
// counter only); through generic pointers they would be flat accesses, which also
// wait on the lane's outstanding global loads and stores.  Empty on the host.
#if defined(__HIP_DEVICE_COMPILE__)
#define DINO_LDS __attribute__((address_space(3)))
#define DINO_GLOBAL __attribute__((address_space(1)))
#else
#define DINO_LDS
#define DINO_GLOBAL
#endif
using LdsTable = const DINO_LDS ProgTable*;
// global coefficient / byte pointers for the device's loads and stores (global_* rather
// than flat_*: a flat access counts against the LDS counter too, so every LDS wait
// would also wait for the lane's outstanding global loads and stores)
template <typename T>
DHD DINO_GLOBAL T* gmem(T* p) { return (DINO_GLOBAL T*)p; }
template <typename T>
DHD const DINO_GLOBAL T* gmem(const T* p) { return (const DINO_GLOBAL T*)p; }

// One scan of a multi-scan image (image-relative byte offsets).
struct ScanRec {
  int32_t data_off;          // first entropy-coded byte
  int32_t data_end;          // the FF of the marker that ends the scan's entropy data
  int32_t ns, ss, se, ah, al;
  int32_t restart_interval;
  int32_t level;             // dependency level (scans of one level are independent)
  int32_t comp[4];           // frame component index of each scan component
  int32_t dc_tab[4];         // offset of the BITS[16] of the DC table in effect, -1 if not needed
  int32_t ac_tab[4];         // same for the AC table
};

// libjpeg-turbo jpeg_natural_order with the 16 safety entries (jutils.c) is
// kNaturalOrder (jpeg_parse.hpp).

// ---------------------------------------------------------------------------
// Marker walk over the scans (read_markers from the first SOS to EOI)
// ---------------------------------------------------------------------------

// Host finder: the FF of the first marker at or after `from` that ends entropy-coded
// data (FF followed by a byte other than 00, FF, D0..D7), or -1.
struct HostMarkerFinder {  // (memchr: the probe walks every scan of a progressive file, 56 -> 10.5 us per 640x480 image)
  int64_t operator()(const uint8_t* p, int64_t from, int64_t len) const {
    for (int64_t k = from; k + 1 < len; ++k) {
      const void* f = memchr(p + k, 0xFF, (size_t)(len - 1 - k));
      if (!f) return -1;
      k = (const uint8_t*)f - p;
      const int c = p[k + 1];
      if (c == 0x00 || c == 0xFF || (c >= 0xD0 && c <= 0xD7)) continue;
      return k;
    }
    return -1;
  }
};

// libjpeg next_marker(): from pos, skip garbage up to an FF, then fill FFs; an FF00
// pair is garbage too.  Returns the marker code and sets *after to the byte after it,
// or -1 at the end of the data.
DHD int next_marker_at(const uint8_t* p, int64_t len, int64_t pos, int64_t* after) {
  for (;;) {
    while (pos < len && p[pos] != 0xFF) ++pos;
    if (pos >= len) return -1;
    while (pos < len && p[pos] == 0xFF) ++pos;
    if (pos >= len) return -1;
    const int c = p[pos++];
    if (c != 0) {
      *after = pos;
      return c;
    }
  }
}

// The last coefficient (zigzag index) a scan may write.  On a corrupt stream an AC first
// scan's run moves k up to se + 15 before the store and an AC refinement puts a new
// coefficient at se + 1 (libjpeg's natural-order safety entries map k > 63 to 63), so
// scans of adjacent bands of one component can write the same coefficient; ordering them
// by these ranges keeps libjpeg's file order for every stream, not only valid ones.
DHD int scan_write_end(const ScanRec& sr, bool progressive) {
  if (!progressive) return 63;
  if (sr.ss == 0) return sr.se;
  const int e = sr.se + (sr.ah == 0 ? 15 : 1);
  return e < 63 ? e : 63;
}

// Walk the scans of a kind-1 image (d->first_sos is the FF of its first SOS), filling
// scans[0..n) and d->n_scans; updates d->status on error.  Every lane of a wave may
// run it (all values are wave-uniform); `find` is the entropy-data end finder.
// coef_bits tracking follows start_pass_phuff_decoder; smoothing_ok decides whether
// libjpeg would smooth the output (-> DINO_IMG_UNSUPPORTED, decoded by the host).
template <typename Finder>
DHD int prog_walk(const uint8_t* p, int64_t len, ImgDesc* d, ScanRec* scans, Finder& find) {
  int32_t dht[8];
  for (int i = 0; i < 8; ++i) dht[i] = d->huff_off[i];
  int32_t ri = d->restart_interval;
  int8_t coef_bits[kMaxComp][10];     // coefficients 0..9 (what smoothing_ok reads), -1 = never coded
  int8_t level_of[kMaxComp][64];      // last level that wrote (component, coefficient)
  for (int c = 0; c < kMaxComp; ++c) {
    for (int k = 0; k < 10; ++k) coef_bits[c][k] = -1;
    for (int k = 0; k < 64; ++k) level_of[c][k] = -1;
  }
  bool latched[kMaxComp] = {false, false, false};
  bool qt_redefined[4] = {false, false, false, false};
  int n = 0;
  int64_t pos = d->first_sos + 2;  // after the SOS marker code
  int m = 0xDA;
  for (;;) {
    // pos: first byte of the segment of marker m (its length field)
    if (m == 0xD9) break;  // EOI
    if (m == 0x01 || (m >= 0xD0 && m <= 0xD7) || m == 0xD8) {
      // parameterless (TEM, RSTn outside a scan); a second SOI: libjpeg JERR_SOI_DUPLICATE
      if (m == 0xD8) return (d->status = DINO_IMG_CORRUPT);
      int64_t after;
      m = next_marker_at(p, len, pos, &after);
      if (m < 0) return (d->status = DINO_IMG_TRUNCATED);
      pos = after;
      continue;
    }
    if (pos + 2 > len) return (d->status = DINO_IMG_TRUNCATED);
    const int seglen = rd16(p + pos);
    if (seglen < 2 || pos + seglen > len) return (d->status = seglen < 2 ? DINO_IMG_CORRUPT : DINO_IMG_TRUNCATED);
    const uint8_t* s = p + pos + 2;
    const int sn = seglen - 2;
    int64_t next_pos = pos + seglen;
    if (m == 0xDA) {  // SOS (get_sos)
      if (sn < 1) return (d->status = DINO_IMG_CORRUPT);
      const int ns = s[0];
      if (sn != 4 + 2 * ns || ns < 1 || ns > 4) return (d->status = DINO_IMG_CORRUPT);  // JERR_BAD_LENGTH
      if (n >= kMaxScans) return (d->status = DINO_IMG_UNSUPPORTED);
      ScanRec sr;
      sr.ns = ns;
      int used = 0;
      for (int k = 0; k < 4; ++k) sr.comp[k] = 0, sr.dc_tab[k] = sr.ac_tab[k] = -1;
      int tds[4] = {0, 0, 0, 0}, tas[4] = {0, 0, 0, 0};
      for (int k = 0; k < ns; ++k) {
        // get_sos: the first frame component with this id whose cur_comp_info slot (indexed
        // by FRAME position) is still empty, i.e. frame index >= k; none -> JERR_BAD_COMPONENT_ID
        const int cs = s[1 + 2 * k];
        int ci = -1;
        for (int c = k; c < d->ncomp; ++c)
          if (d->comp[c].id == cs) {
            ci = c;
            break;
          }
        if (ci < 0) return (d->status = DINO_IMG_CORRUPT);
        if (used & (1 << ci)) return (d->status = DINO_IMG_UNSUPPORTED);  // a component twice in one scan
        used |= 1 << ci;
        sr.comp[k] = ci;
        tds[k] = s[2 + 2 * k] >> 4;
        tas[k] = s[2 + 2 * k] & 15;
      }
      sr.ss = s[1 + 2 * ns];
      sr.se = s[2 + 2 * ns];
      sr.ah = s[3 + 2 * ns] >> 4;
      sr.al = s[3 + 2 * ns] & 15;
      sr.restart_interval = ri;
      if (d->progressive) {
        // start_pass_phuff_decoder validation (JERR_BAD_PROGRESSION)
        const bool dc_band = sr.ss == 0;
        bool bad = false;
        if (dc_band) {
          if (sr.se != 0) bad = true;
        } else {
          if (sr.ss > sr.se || sr.se > 63) bad = true;
          if (ns != 1) bad = true;
        }
        if (sr.ah != 0 && sr.al != sr.ah - 1) bad = true;
        if (sr.al > 13) bad = true;
        if (bad) return (d->status = DINO_IMG_CORRUPT);
        for (int k = 0; k < ns; ++k) {
          const int ci = sr.comp[k];
          for (int cf = sr.ss; cf <= sr.se && cf < 10; ++cf) coef_bits[ci][cf] = (int8_t)sr.al;
        }
        // derived tables (jpeg_make_d_derived_tbl): DC first scans need the DC table of
        // each component, AC scans (first and refine) the AC table; DC refine none
        for (int k = 0; k < ns; ++k) {
          if (dc_band) {
            if (sr.ah == 0) {
              if (tds[k] > 3 || dht[tds[k]] < 0) return (d->status = DINO_IMG_CORRUPT);
              sr.dc_tab[k] = dht[tds[k]];
            }
          } else {
            if (tas[k] > 3 || dht[4 + tas[k]] < 0) return (d->status = DINO_IMG_CORRUPT);
            sr.ac_tab[k] = dht[4 + tas[k]];
          }
        }
      } else {
        // sequential (jdhuff start_pass_huff_decoder): Ss/Se/Ah/Al are ignored (a warning)
        sr.ss = 0;
        sr.se = 63;
        sr.ah = sr.al = 0;
        for (int k = 0; k < ns; ++k) {
          if (tds[k] > 3 || tas[k] > 3 || dht[tds[k]] < 0 || dht[4 + tas[k]] < 0)
            return (d->status = DINO_IMG_CORRUPT);  // JERR_NO_HUFF_TABLE
          sr.dc_tab[k] = dht[tds[k]];
          sr.ac_tab[k] = dht[4 + tas[k]];
        }
        for (int k = 0; k < ns; ++k)
          for (int cf = 0; cf < 10; ++cf) coef_bits[sr.comp[k]][cf] = 0;
      }
      // per_scan_setup: blocks in an interleaved MCU (JERR_BAD_MCU_SIZE)
      if (ns > 1) {
        int bpm = 0;
        for (int k = 0; k < ns; ++k) bpm += d->comp[sr.comp[k]].h * d->comp[sr.comp[k]].v;
        if (bpm > kMaxBlocksPerMcu) return (d->status = DINO_IMG_BADDATA);
      }
      // latch_quant_tables: a component's table is copied at its first scan
      for (int k = 0; k < ns; ++k) {
        const int ci = sr.comp[k];
        if (!latched[ci]) {
          const int tq = d->comp[ci].tq;
          if (!((d->qt_seen_mask >> tq) & 1)) return (d->status = DINO_IMG_CORRUPT);  // JERR_NO_QUANT_TABLE
          if (qt_redefined[tq]) return (d->status = DINO_IMG_UNSUPPORTED);  // latched after a DQT between scans
          latched[ci] = true;
        }
      }
      // dependency level: after every earlier scan that wrote (or, on a corrupt stream, may
      // have written) one of the coefficients it may write
      const int wend = scan_write_end(sr, d->progressive != 0);
      int lv = -1;
      for (int k = 0; k < ns; ++k)
        for (int cf = sr.ss; cf <= wend; ++cf) lv = level_of[sr.comp[k]][cf] > lv ? level_of[sr.comp[k]][cf] : lv;
      sr.level = lv + 1;
      for (int k = 0; k < ns; ++k)
        for (int cf = sr.ss; cf <= wend; ++cf) level_of[sr.comp[k]][cf] = (int8_t)sr.level;
      // entropy data: up to the first marker that is not RSTn
      sr.data_off = (int32_t)next_pos;
      const int64_t e = find(p, next_pos, len);
      if (e < 0) return (d->status = DINO_IMG_TRUNCATED);  // no EOI: Pillow reports a truncated file
      sr.data_end = (int32_t)e;
      scans[n++] = sr;
      int64_t after;
      m = next_marker_at(p, len, e, &after);
      if (m < 0) return (d->status = DINO_IMG_TRUNCATED);
      pos = after;
      continue;
    }
    switch (m) {
      case 0xC4: {  // DHT
        int q = 0;
        while (q < sn) {
          if (q + 17 > sn) return (d->status = DINO_IMG_CORRUPT);
          const int tc = s[q] >> 4, th = s[q] & 15;
          int cnt = 0;
          for (int i = 1; i <= 16; ++i) cnt += s[q + i];
          if (cnt > 256 || q + 17 + cnt > sn || tc > 1 || th > 3) return (d->status = DINO_IMG_CORRUPT);
          dht[tc * 4 + th] = (int32_t)(pos + 2 + q + 1);
          q += 17 + cnt;
        }
        break;
      }
      case 0xDB: {  // DQT between scans: fine unless a component still to be latched uses it
        int q = 0;
        while (q < sn) {
          const int pq = s[q] >> 4, tq = s[q] & 15;
          if (tq > 3 || pq > 1) return (d->status = DINO_IMG_CORRUPT);
          const int need = pq ? 128 : 64;
          if (q + 1 + need > sn) return (d->status = DINO_IMG_CORRUPT);
          qt_redefined[tq] = true;
          q += 1 + need;
        }
        break;
      }
      case 0xDD:  // DRI
        if (sn != 2) return (d->status = DINO_IMG_CORRUPT);
        ri = rd16(s);
        break;
      case 0xC0: case 0xC1: case 0xC2: case 0xC3: case 0xC5: case 0xC6: case 0xC7:
      case 0xC9: case 0xCA: case 0xCB: case 0xCD: case 0xCE: case 0xCF:
        return (d->status = DINO_IMG_CORRUPT);  // JERR_SOF_DUPLICATE
      case 0xCC:                                // DAC
        return (d->status = DINO_IMG_UNSUPPORTED);
      default:
        break;  // APPn, COM, DNL, ...: skipped
    }
    int64_t after;
    m = next_marker_at(p, len, next_pos, &after);
    if (m < 0) return (d->status = DINO_IMG_TRUNCATED);
    pos = after;
  }
  d->n_scans = n;
  if (n == 0) return (d->status = DINO_IMG_CORRUPT);
  // smoothing_ok (jdcoefct.c, SAVED_COEFS = 10)
  if (d->progressive) {
    bool useful = false, possible = true;
    for (int c = 0; c < d->ncomp; ++c) {
      if (!latched[c]) {
        possible = false;
        break;
      }
      const uint16_t* q = d->qt[d->comp[c].tq];
      if (!q[0] || !q[1] || !q[8] || !q[16] || !q[9] || !q[2] || !q[3] || !q[10] || !q[17] || !q[24]) {
        possible = false;
        break;
      }
      if (coef_bits[c][0] < 0) {
        possible = false;
        break;
      }
      for (int k = 1; k < 10; ++k) useful = useful || coef_bits[c][k] != 0;
    }
    if (possible && useful) return (d->status = DINO_IMG_UNSUPPORTED);
  }
  return d->status;
}

// ---------------------------------------------------------------------------
// Bit reader over the raw (stuffed) entropy bytes with libjpeg's marker rules
// ---------------------------------------------------------------------------
// Raw bytes come through rb_byte: on the host straight from memory; on the device
// from a 64-byte LDS ring per lane holding the bytes of absolute addresses
// [hi - 64, hi), staged 32 aligned bytes at a time (two 16-byte loads and one wait
// per 32 bytes instead of a dependent load per byte or word; the lane's decode is a
// serial chain, so every exposed load latency adds to it).
struct RawBits {
  const uint8_t* p;
  int64_t len;       // image bytes (hard bound)
  int64_t bp;        // next raw byte
  uint64_t buf;      // MSB aligned
  int32_t nbits;     // valid bits in buf (real + zero fill)
  int32_t real;      // real (not zero-fill) bits among them; < 0: bits were needed past a marker
  int32_t unread;    // marker code the reader stopped at (0: none)
  int32_t insufficient;
  DINO_LDS uint8_t* ring;  // device: 64 bytes of LDS (16-byte aligned); nullptr: read memory directly
  uintptr_t hi;      // device: end (absolute address) of the staged bytes
  uintptr_t bend;    // device: end of the readable buffer (the batch's packed bytes)
};

DHD void rb_init(RawBits& r, const uint8_t* p, int64_t len, int64_t pos, DINO_LDS uint8_t* ring = nullptr,
                 const uint8_t* bend = nullptr) {
  r.p = p;
  r.len = len;
  r.bp = pos;
  r.buf = 0;
  r.nbits = 0;
  r.real = 0;
  r.unread = 0;
  r.insufficient = 0;
  r.ring = ring;
  r.hi = 0;
  r.bend = (uintptr_t)bend;
}

// Stage the 32 bytes from the 16-byte-aligned address at or before `a` (continuing
// from hi when a lies in the next 16 bytes) into the ring.
DHD void rb_stage(RawBits& r, uintptr_t a) {
  const uintptr_t A = (a >= r.hi && a < r.hi + 16 && r.hi) ? r.hi : (a & ~(uintptr_t)15);
  DINO_LDS uint4* dst0 = (DINO_LDS uint4*)(r.ring + (A & 63));
  DINO_LDS uint4* dst1 = (DINO_LDS uint4*)(r.ring + ((A + 16) & 63));
  if (A + 32 <= r.bend) {
    const uint4 c0 = *gmem((const uint4*)A), c1 = *gmem((const uint4*)(A + 16));
    *dst0 = c0;
    *dst1 = c1;
  } else {  // the end of the batch buffer: bytewise, zeros past it
    for (int j = 0; j < 32; ++j) r.ring[(A + j) & 63] = A + j < r.bend ? *gmem((const uint8_t*)(A + j)) : 0;
  }
  r.hi = A + 32;
}

DHD int rb_byte(RawBits& r, int64_t k) {
  if (!r.ring) return r.p[k];
  const uintptr_t a = (uintptr_t)(r.p + k);
  if (a >= r.hi || a + 48 < r.hi) rb_stage(r, a);
  return r.ring[a & 63];
}

// jpeg_fill_bit_buffer: bytes until >= 33 bits; an FF00 is a data FF; any other
// marker stops the reader (unread = its code, bp after it) and zeros follow.
DHD void rb_fill(RawBits& r) {
  while (r.nbits <= 32) {
    if (!r.unread) {
      // four plain bytes at once when none of them is 0xFF
      if (r.bp + 4 <= r.len) {
        const uint32_t w = (uint32_t)rb_byte(r, r.bp) << 24 | (uint32_t)rb_byte(r, r.bp + 1) << 16 |
                           (uint32_t)rb_byte(r, r.bp + 2) << 8 | (uint32_t)rb_byte(r, r.bp + 3);
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
        int c = rb_byte(r, r.bp);
        if (c != 0xFF) {
          r.buf |= (uint64_t)c << (56 - r.nbits);
          r.nbits += 8;
          r.real += 8;
          r.bp += 1;
          continue;
        }
        int64_t k = r.bp + 1;
        while (k < r.len && rb_byte(r, k) == 0xFF) ++k;
        if (k < r.len && rb_byte(r, k) == 0) {  // stuffed FF
          r.buf |= (uint64_t)0xFF << (56 - r.nbits);
          r.nbits += 8;
          r.real += 8;
          r.bp = k + 1;
          continue;
        }
        r.unread = k < r.len ? rb_byte(r, k) : 0xD9;  // (the walk guarantees a marker before the end)
        r.bp = k + 1;
      } else {
        r.unread = 0xD9;
      }
    }
    r.nbits += 32;  // zero fill (buf already holds zeros below its valid bits)
  }
}

DHD uint32_t rb_peek32(const RawBits& r) { return (uint32_t)(r.buf >> 32); }

DHD void rb_skip(RawBits& r, int n) {
  r.buf <<= n;
  r.nbits -= n;
  r.real -= n;
  if (r.real < 0) {
    r.insufficient = 1;  // JWRN_HIT_MARKER: bits needed past the marker
    r.real = 0;
  }
}

DHD uint32_t rb_bits(RawBits& r, int n) {  // GET_BITS(n), 0 <= n <= 16
  rb_fill(r);
  const uint32_t v = n ? rb_peek32(r) >> (32 - n) : 0u;
  rb_skip(r, n);
  return v;
}

// HUFF_DECODE: one symbol (lookahead, else the bit-serial path incl. the l = 17 fake zero).
inline long g_prog_host_symbols = 0;  // host model statistics (symbols decoded by rb_huff; never on the device)

template <typename TabPtr>
DHD int rb_huff(RawBits& r, TabPtr t) {
  constexpr int LB = kProgLookBits;
#if !defined(__HIP_DEVICE_COMPILE__)
  ++g_prog_host_symbols;
#endif
  rb_fill(r);
  const uint32_t hi = rb_peek32(r);
  const uint32_t e = t->look[hi >> (32 - LB)];
  int sym, len;
  if (e) {
    sym = (int)(e >> 5);
    len = (int)(e & 31u);
  } else {
    huff_slow_bits<LB>(hi >> 15, t, &sym, &len);
  }
  rb_skip(r, len);
  return sym;
}

// ---------------------------------------------------------------------------
// Restart processing (jdphuff/jdhuff process_restart + read_restart_marker +
// jpeg_resync_to_restart)
// ---------------------------------------------------------------------------
DHD void rb_restart(RawBits& r, int* next_restart_num) {
  r.buf = 0;
  r.nbits = 0;
  r.real = 0;
  const int desired = *next_restart_num;
  if (!r.unread) {
    int64_t after;
    const int c = next_marker_at(r.p, r.len, r.bp, &after);
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
      int64_t after;
      const int c = next_marker_at(r.p, r.len, r.bp, &after);
      r.unread = c < 0 ? 0xD9 : c;
      r.bp = c < 0 ? r.len : after;
    }
  }
  *next_restart_num = (desired + 1) & 7;
  if (!r.unread) r.insufficient = 0;
}

// ---------------------------------------------------------------------------
// Scan decoders.  `coef` is the image's dense int16 coefficient buffer; blocks are
// addressed by (component, bx, by).  The coefficient access policy is a template
// argument so that the device version can use atomics / LDS staging where scans of
// the same level share memory words.
// ---------------------------------------------------------------------------
DHD int16_t* coef_block(int16_t* coef, const ImgDesc& d, int c, int bx, int by) {
  const CompDesc& cd = d.comp[c];
  return coef + cd.coef_off / 2 + ((int64_t)by * cd.bw + bx) * 64;
}

// OR v into the int16 at p.  Other lanes may write the other half of its 32-bit word
// at the same time (scans of one level): the device uses a word atomic.
template <typename P>
DHD void coef_or16(P p, int v) {
#if defined(__HIP_DEVICE_COMPILE__)
  DINO_GLOBAL uint32_t* w = gmem((uint32_t*)((uintptr_t)p & ~(uintptr_t)3));
  const uint32_t sh = ((uintptr_t)p & 2) ? 16u : 0u;
  __hip_atomic_fetch_or(w, ((uint32_t)(uint16_t)v) << sh, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
#else
  *p = (int16_t)(*p | v);
#endif
}

struct ScanTables {
  LdsTable dc[4];
  LdsTable ac[4];
};
// Table of scan component k (constant indices only; see ScanGeom).
DHD LdsTable sel4(const LdsTable* t, int k) { return k == 0 ? t[0] : (k == 1 ? t[1] : (k == 2 ? t[2] : t[3])); }

// Geometry of the scan's MCUs (jdinput.c per_scan_setup).  Per block of the MCU a
// 2-bit field each of component, x and y offset and scan component index (bits
// [2b, 2b + 2); <= 10 blocks): a lane never indexes a private array at run time
// (that would live in scratch memory, one global-latency access per use).
struct ScanGeom {
  int32_t mcus_x, mcus_y, bpm;
  uint32_t comp, bx, by, kk;
  int32_t ch[kMaxComp], cv[kMaxComp];  // sampling factors, read with constant indices
  int64_t plane[kMaxComp];             // coefficient plane offset (int16 units) and blocks per row
  int32_t bw[kMaxComp];
};
DHD int sg_field(uint32_t f, int b) { return (int)((f >> (2 * b)) & 3u); }
template <typename T>
DHD T sel3(const T* a, int c) { return c == 0 ? a[0] : (c == 1 ? a[1] : a[2]); }

DHD ScanGeom scan_geom(const ImgDesc& d, const ScanRec& sr) {
  ScanGeom g;
  g.comp = g.bx = g.by = g.kk = 0;
  for (int c = 0; c < kMaxComp; ++c) {
    const CompDesc& cd = d.comp[c < d.ncomp ? c : 0];
    g.ch[c] = cd.h;
    g.cv[c] = cd.v;
    g.plane[c] = cd.coef_off / 2;
    g.bw[c] = cd.bw;
  }
  if (sr.ns == 1) {
    const CompDesc& cd = d.comp[sr.comp[0]];
    g.mcus_x = ceil_div(cd.dw, 8);
    g.mcus_y = ceil_div(cd.dh, 8);
    g.bpm = 1;
    g.comp = (uint32_t)sr.comp[0];
  } else {
    g.mcus_x = d.mcus_x;
    g.mcus_y = d.mcus_y;
    int b = 0;
#pragma unroll
    for (int k = 0; k < 4; ++k) {  // constant indices into sr (no private array indexed at run time)
      if (k >= sr.ns) break;
      const int ci = sr.comp[k];
      const CompDesc& cd = d.comp[ci];
      for (int y = 0; y < cd.v; ++y)
        for (int x = 0; x < cd.h; ++x) {
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

// Coefficient block (int16 pointer) of block `blk` of MCU m, and its component.
DHD int16_t* scan_block(int16_t* coef, const ScanRec& sr, const ScanGeom& g, int64_t m, int blk, int* c) {
  const int my = (int)(m / g.mcus_x), mx = (int)(m - (int64_t)my * g.mcus_x);
  const int cc = sg_field(g.comp, blk);
  *c = cc;
  int bx = mx, by = my;
  if (sr.ns != 1) {
    bx = mx * sel3(g.ch, cc) + sg_field(g.bx, blk);
    by = my * sel3(g.cv, cc) + sg_field(g.by, blk);
  }
  return coef + sel3(g.plane, cc) + ((int64_t)by * sel3(g.bw, cc) + bx) * 64;
}

// AC refinement of one block (decode_mcu_AC_refine), on masks in zigzag order.
// nzz: the block's coefficients that were non-zero before the scan (bit k = zigzag
// index k).  Returned (also zigzag): corr = correction bits read as 1, nzn = new
// coefficients, neg = their sign.  libjpeg walks k one position at a time; here a
// symbol's run and the correction bits it passes are found with bit operations and
// the correction bits are read together (the bits and their order are the same).
DHD int64_t low_bits(int n) { return n >= 64 ? -1ll : (int64_t)((1ull << n) - 1ull); }

// Read one correction bit per set bit of c (increasing k) into corr.
DHD void refine_corrections(RawBits& r, uint64_t c, uint64_t* corr) {
  int n = __builtin_popcountll(c);
  while (n > 0) {
    const int take = n > 16 ? 16 : n;
    uint32_t bits = rb_bits(r, take) << (32 - take);  // MSB first, in increasing k
    for (int j = 0; j < take; ++j) {
      const uint64_t lowest = c & (~c + 1ull);
      if (bits & 0x80000000u) *corr |= lowest;
      bits <<= 1;
      c &= c - 1ull;
    }
    n -= take;
  }
}

DHD void ac_refine_block(RawBits& r, LdsTable tbl, const ScanRec& sr, uint64_t nzz, int32_t* eobrun,
                         uint64_t* corr_out, uint64_t* new_out, uint64_t* neg_out) {
  uint64_t corr = 0, nzn = 0, neg = 0;
  int k = sr.ss;
  const int se = sr.se;
  const uint64_t band = (uint64_t)low_bits(se + 1) & ~(uint64_t)low_bits(sr.ss);
  if (*eobrun == 0) {
    while (k <= se) {
      const int sym = rb_huff(r, tbl);
      int rr = sym >> 4, s = sym & 15;
      bool negative = false;
      if (s) {
        // (a size other than 1 is a warning; the sign bit is read regardless)
        negative = rb_bits(r, 1) == 0;
      } else if (rr != 15) {
        *eobrun = 1 << rr;
        if (rr) *eobrun += (int32_t)rb_bits(r, rr);
        break;
      }
      // the (rr+1)-th not-yet-non-zero position at or after k (se + 1 when there is none)
      uint64_t z = ~nzz & band & ~(uint64_t)low_bits(k);
      for (int j = 0; j < rr && z; ++j) z &= z - 1ull;
      const int stop = z ? __builtin_ctzll(z) : se + 1;
      // correction bits of the non-zero coefficients passed on the way
      refine_corrections(r, nzz & band & (uint64_t)low_bits(stop) & ~(uint64_t)low_bits(k), &corr);
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
    if (k <= se) refine_corrections(r, nzz & band & ~(uint64_t)low_bits(k), &corr);
    (*eobrun)--;
  }
  *corr_out = corr;
  *new_out = nzn;
  *neg_out = neg;
}

// New value of a refined coefficient (v: its value before the scan).
DHD int16_t ac_refine_value(int16_t v, bool corr, bool is_new, bool negative, int al) {
  const int p1 = 1 << al, m1 = (int)(~0u << al);
  int x = v;
  if (corr && (x & p1) == 0) x += x >= 0 ? p1 : m1;
  if (is_new) x = negative ? m1 : p1;
  return (int16_t)x;
}

// Decode one whole scan.  Block stores go through `Store` (host: plain memory; device:
// the lane's policy).  Returns 0.
struct PlainCoefIO {
  DHD void load_block(const int16_t* b, int16_t* out) const {
    for (int i = 0; i < 64; ++i) out[i] = b[i];
  }
};

// The scan's DC predictors, one per scan component (constant indices only).
struct DcPred {
  int32_t v0, v1, v2, v3;
  DHD int32_t add(int k, int32_t s) {  // last_dc_val[ci] += s, returned (unsigned wrap as libjpeg-turbo)
    const int32_t cur = k == 0 ? v0 : (k == 1 ? v1 : (k == 2 ? v2 : v3));
    const int32_t r = (int32_t)((uint32_t)cur + (uint32_t)s);
    if (k == 0) v0 = r;
    else if (k == 1) v1 = r;
    else if (k == 2) v2 = r;
    else v3 = r;
    return r;
  }
};

// Non-zero mask of a block's coefficients in zigzag order (bit k = coefficient
// natural_order[k]): the refinement works on zigzag masks.
template <typename P>
DHD uint64_t block_nz_zz(P b) {
  uint64_t nzz = 0;
#if defined(__HIP_DEVICE_COMPILE__)
  const DINO_GLOBAL uint4* b4 = gmem((const uint4*)b);  // blocks are 128-byte aligned
  uint32_t w[32];
#pragma unroll
  for (int q = 0; q < 8; ++q) {
    const uint4 v = b4[q];
    w[4 * q] = v.x;
    w[4 * q + 1] = v.y;
    w[4 * q + 2] = v.z;
    w[4 * q + 3] = v.w;
  }
#pragma unroll
  for (int k = 0; k < 64; ++k) {  // constant indices: registers only
    const int pos = kNaturalOrder[k];
    nzz |= (uint64_t)(((w[pos >> 1] >> (16 * (pos & 1))) & 0xFFFFu) != 0) << k;
  }
#else
  for (int k = 0; k < 64; ++k) nzz |= (uint64_t)(b[kNaturalOrder[k]] != 0) << k;
#endif
  return nzz;
}

// `nat`: jpeg_natural_order with its 16 safety entries (kNaturalOrder; the device
// passes an LDS copy); `ring` / `bend`: the device's byte staging (see RawBits).
// AC refinement scan (single component: one block per MCU), device form: block m is
// staged in the lane's LDS buffer `blkbuf` (64 int16) from registers loaded one
// block ahead, corrections are applied there, and only the changed coefficients are
// stored (other scans of the level may be writing other coefficients of the block).
DHD void prog_refine_scan_staged(RawBits& r, const ScanRec& sr, const ScanGeom& g, int64_t nmcu, LdsTable ac0,
                                 int16_t* coef, const DINO_LDS uint8_t* nat, DINO_LDS int16_t* blkbuf) {
  const int ri = sr.restart_interval, al = sr.al;
  int rtg = ri, next_rst = 0;
  int32_t eobrun = 0;
  int c;
  uint4 nxt[8];
  {
    const DINO_GLOBAL uint4* b4 = gmem((const uint4*)scan_block(coef, sr, g, 0, 0, &c));
#pragma unroll
    for (int q = 0; q < 8; ++q) nxt[q] = b4[q];
  }
  DINO_LDS uint4* lb = (DINO_LDS uint4*)blkbuf;
  for (int64_t m = 0; m < nmcu; ++m) {
    if (ri) {
      if (rtg == 0) {
        rb_restart(r, &next_rst);
        eobrun = 0;
        rtg = ri;
      }
    }
    DINO_GLOBAL int16_t* b = gmem(scan_block(coef, sr, g, m, 0, &c));
    // this block (loaded one block ago) -> LDS and its zigzag non-zero mask; the next one is loaded meanwhile
    uint64_t nzz = 0;
    {
      uint32_t w[32];
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        lb[q] = nxt[q];
        w[4 * q] = nxt[q].x;
        w[4 * q + 1] = nxt[q].y;
        w[4 * q + 2] = nxt[q].z;
        w[4 * q + 3] = nxt[q].w;
      }
#pragma unroll
      for (int k = 0; k < 64; ++k) {
        const int pos = kNaturalOrder[k];
        nzz |= (uint64_t)(((w[pos >> 1] >> (16 * (pos & 1))) & 0xFFFFu) != 0) << k;
      }
    }
    if (m + 1 < nmcu) {
      const DINO_GLOBAL uint4* b4 = gmem((const uint4*)scan_block(coef, sr, g, m + 1, 0, &c));
#pragma unroll
      for (int q = 0; q < 8; ++q) nxt[q] = b4[q];
    }
    if (!r.insufficient) {
      uint64_t corr, nzn, neg;
      ac_refine_block(r, ac0, sr, nzz, &eobrun, &corr, &nzn, &neg);
      for (uint64_t mm = corr | nzn; mm; mm &= mm - 1) {
        const int k = __builtin_ctzll(mm);
        const int pos = nat[k];
        const int16_t v = ac_refine_value(blkbuf[pos], (corr >> k) & 1u, (nzn >> k) & 1u, (neg >> k) & 1u, al);
        blkbuf[pos] = v;
        b[pos] = v;
      }
    }
    if (ri) rtg--;
  }
}

DHD void prog_decode_scan(const uint8_t* p, int64_t len, const ImgDesc& d, const ScanRec& sr, const ScanTables& tb,
                          int16_t* coef, const DINO_LDS uint8_t* nat, DINO_LDS uint8_t* ring = nullptr,
                          const uint8_t* bend = nullptr, DINO_LDS int16_t* blkbuf = nullptr) {
  RawBits r;
  rb_init(r, p, len, sr.data_off, ring, bend);
  const ScanGeom g = scan_geom(d, sr);
  const int64_t nmcu = (int64_t)g.mcus_x * g.mcus_y;
  const int ri = sr.restart_interval;
  int rtg = ri, next_rst = 0;
  DcPred last_dc{0, 0, 0, 0};
  int32_t eobrun = 0;
  const bool prog = d.progressive != 0;
  const int al = sr.al;
  const LdsTable ac0 = tb.ac[0];
  if (blkbuf && prog && sr.ss > 0 && sr.ah > 0) {  // AC refinement, device
    prog_refine_scan_staged(r, sr, g, nmcu, ac0, coef, nat, blkbuf);
    return;
  }
  for (int64_t m = 0; m < nmcu; ++m) {
    if (ri) {
      if (rtg == 0) {
        rb_restart(r, &next_rst);
        last_dc = DcPred{0, 0, 0, 0};
        eobrun = 0;
        rtg = ri;
      }
    }
    if (!r.insufficient) {
      for (int blk = 0; blk < g.bpm; ++blk) {
        int c;
        DINO_GLOBAL int16_t* b = gmem(scan_block(coef, sr, g, m, blk, &c));
        const int kk = sg_field(g.kk, blk);
        if (!prog) {  // jdhuff decode_mcu (sequential scan of a multi-scan file)
          int s = rb_huff(r, sel4(tb.dc, kk));
          if (s) s = huff_extend((int)rb_bits(r, s), s);
          b[0] = (int16_t)last_dc.add(kk, s);
          const LdsTable act = sel4(tb.ac, kk);
          for (int k = 1; k < 64; k++) {
            const int sym = rb_huff(r, act);
            const int rr = sym >> 4, ss = sym & 15;
            if (ss) {
              k += rr;
              const int v = huff_extend((int)rb_bits(r, ss), ss);
              b[nat[k]] = (int16_t)v;
            } else {
              if (rr != 15) break;
              k += 15;
            }
          }
        } else if (sr.ss == 0) {
          if (sr.ah == 0) {  // decode_mcu_DC_first
            int s = rb_huff(r, sel4(tb.dc, kk));
            if (s) s = huff_extend((int)rb_bits(r, s), s);
            b[0] = (int16_t)((uint32_t)last_dc.add(kk, s) << al);
          } else {  // decode_mcu_DC_refine
            if (rb_bits(r, 1)) coef_or16(b, 1 << al);
          }
        } else if (sr.ah == 0) {  // decode_mcu_AC_first
          if (eobrun > 0) {
            eobrun--;
          } else {
            for (int k = sr.ss; k <= sr.se; k++) {
              const int sym = rb_huff(r, ac0);
              const int rr = sym >> 4, ss = sym & 15;
              if (ss) {
                k += rr;
                const int v = huff_extend((int)rb_bits(r, ss), ss);
                b[nat[k]] = (int16_t)((uint32_t)v << al);
              } else if (rr == 15) {
                k += 15;
              } else {
                eobrun = 1 << rr;
                if (rr) eobrun += (int32_t)rb_bits(r, rr);
                eobrun--;
                break;
              }
            }
          }
        } else {  // decode_mcu_AC_refine
          const uint64_t nzz = block_nz_zz(b);
          uint64_t corr, nzn, neg;
          ac_refine_block(r, ac0, sr, nzz, &eobrun, &corr, &nzn, &neg);
          for (uint64_t mm = corr | nzn; mm; mm &= mm - 1) {
            const int k = __builtin_ctzll(mm);
            const int pos = nat[k];
            b[pos] = ac_refine_value(b[pos], (corr >> k) & 1u, (nzn >> k) & 1u, (neg >> k) & 1u, al);
          }
        }
      }
    }
    if (ri) rtg--;
  }
}

// Build the derived table + lookahead of one DHT table (host/serial form).
DHD bool prog_build_table(const uint8_t* bits16, bool is_dc, ProgTable* t) {
  if (!huff_build_derived(bits16, is_dc, t)) return false;
  for (int i = 0; i < (1 << kProgLookBits); ++i) t->look[i] = huff_look_entry(t, i);
  return true;
}

}  // namespace dino
