// huffman.hpp — baseline Huffman entropy decoding, restated from libjpeg-turbo
// jdhuff.c (jpeg_make_d_derived_tbl, jpeg_huff_decode, decode_mcu_slow) in a
// form that a GPU lane can run from an arbitrary bit position.
//
// The decoder works on the *destuffed* entropy stream (0xFF00 -> 0xFF, RSTn
// removed; see k_destuff), big-endian bit order, zero padded at the end — the
// same zero fill libjpeg inserts after it hits a marker (jdhuff.c
// jpeg_fill_bit_buffer).
//
// Decoding is expressed as "steps": one step = one Huffman symbol plus its
// extra bits (a DC difference, an AC run/level, a ZRL or an EOB).  The state
// between steps is (bit position, block-in-MCU index c, zigzag index z).  That
// state is all a lane needs to resume decoding, which is what makes the
// speculative self-synchronising parallel decode in k_huffman possible.
#pragma once

#include "jpeg_parse.hpp"

namespace dino {

// Derived decoding table for one Huffman table (jpeg_make_d_derived_tbl), what the
// long-code path reads, and the same with its LB-bit lookahead (the progressive
// decoder's tables).  Lookahead entry for each LB-bit prefix: (symbol << 5) | code
// length, 0 when the code is longer than LB.  AC tables look ahead kLookBits = 11
// bits; DC tables kDcLookBits = 9 (the standard DC codes are <= 9 bits for luma and
// only the rare categories >= 10 of chroma need the slow path).
constexpr int kDcLookBits = 9;
struct HuffDerived {
  int32_t maxcode[18];     // maxcode[l], -1 if no codes of length l; [17] sentinel
  int32_t valoffset[18];
  uint8_t huffval[256];
};
template <int LB>
struct HuffTableT {
  int32_t maxcode[18];
  int32_t valoffset[18];
  uint8_t huffval[256];
  uint16_t look[1 << LB];
};

// Skip entries of the state-only decodes (look-back, first decode, sync re-decodes):
// what a step does to the decoder state without its coefficient value, indexed like
// `look`: bits consumed (code + extra bits) | zigzag advance << 5 (DC 1; AC: r + 1,
// ZRL 16, EOB 64), 0 when the code is longer than the lookahead.  An AC entry whose
// second symbol's code also lies inside the lookahead carries that symbol too: its
// bits << 12 | its advance << 17 | 1 << 24 (skip_step takes both while the first leaves
// the block open): ~1.7 symbols per lookup on the bench streams instead of 1.
struct HuffSkip {
  uint32_t ac[3][1 << kLookBits];
  uint32_t dc[3][1 << kDcLookBits];
};
constexpr uint32_t kSkipPair = 1u << 24;

// The tables of an image (AC of components 0..2, DC of components 0..2): derived
// tables, value lookaheads, skip entries.  The lookaheads and the skip entries are
// separate arrays so that k_huff1 can hold only the skip entries while it runs the
// state-only decodes and load the lookaheads over them for its write pass.
struct HuffTables {
  HuffDerived ac[3];
  HuffDerived dc[3];
  uint32_t ac_look[3][1 << kLookBits];   // value lookahead with the second symbol (look_pair_entry)
  uint16_t dc_look[3][1 << kDcLookBits];
  HuffSkip skip;
};
static_assert(sizeof(HuffTables) % 16 == 0, "HuffTables is copied in 16-byte words");
static_assert(offsetof(HuffTables, ac_look) % 16 == 0 && offsetof(HuffTables, skip) % 16 == 0, "16-byte parts");
constexpr int kHuffLookBytes = (int)(offsetof(HuffTables, skip) - offsetof(HuffTables, ac_look));

// Build maxcode/valoffset/huffval (not the lookahead) from BITS[16] + HUFFVAL.
// Returns false on an invalid table (libjpeg JERR_BAD_HUFF_TABLE).
template <typename T>
DHD bool huff_build_derived(const uint8_t* bits16, bool is_dc, T* t) {
  int p = 0;
  int code = 0;
  for (int l = 1; l <= 16; ++l) {
    int cnt = bits16[l - 1];
    if (p + cnt > 256) return false;
    if (cnt) {
      t->valoffset[l] = p - code;
      p += cnt;
      code += cnt;
      t->maxcode[l] = code - 1;
    } else {
      t->maxcode[l] = -1;
      t->valoffset[l] = 0;
    }
    // Figure C.2: codes of length l must fit in l bits (no all-ones code)
    if (code > (1 << l)) return false;
    if (code == (1 << l) && cnt) {
      // the last code of this length is all ones: libjpeg rejects code >= 1<<si
      return false;
    }
    code <<= 1;
  }
  t->maxcode[0] = -1;
  t->valoffset[0] = 0;
  t->maxcode[17] = 0xFFFFF;
  t->valoffset[17] = 0;
  const uint8_t* vals = bits16 + 16;
  for (int i = 0; i < p; ++i) {
    t->huffval[i] = vals[i];
    if (is_dc && vals[i] > 15) return false;
  }
  for (int i = p; i < 256; ++i) t->huffval[i] = 0;
  return true;
}

DHD int huff_extend(int x, int s) { return x < (1 << (s - 1)) ? x + (int)(((unsigned)-1) << s) + 1 : x; }

// Lookahead entry for the LB-bit prefix `idx` (computable independently per entry).
template <int LB, typename T>
DHD uint16_t look_entry_of(const T* t, int idx) {
  for (int l = 1; l <= LB; ++l) {
    const int code = idx >> (LB - l);
    if (code <= t->maxcode[l]) {  // canonical code: first length whose maxcode covers the prefix
      const int sym = t->huffval[(code + t->valoffset[l]) & 255];
      return (uint16_t)((sym << 5) | l);
    }
  }
  return 0;
}
template <int LB>
DHD uint16_t huff_look_entry(const HuffTableT<LB>* t, int idx) {
  return look_entry_of<LB>(t, idx);
}

// AC value lookahead entry of index idx: the single-symbol entry (symbol << 5 | code
// length, bits 0-12) and, when the next symbol's code is decided by the index's remaining
// bits after the first symbol's code and extra bits, that symbol too: its code length
// << 13 | its symbol << 17 | kLookPair.  decode_write then takes two coefficients per
// step (the write pass of the speculative decode: ~1.7 symbols per lookup on the bench
// streams).
constexpr uint32_t kLookPair = 1u << 25;
// look: the table's single-symbol entries (bits 0-12 of each word; any pair bits above
// are ignored, so the entries can be completed in place, each by its own thread).
template <int LB>
DHD uint32_t look_pair_entry(const uint32_t* look, int idx) {
  const uint32_t e = look[idx] & 0x1FFFu;
  if (!e) return 0u;
  const int used = (int)(e & 31u) + (int)((e >> 5) & 15u);
  if (used >= LB) return e;
  const uint32_t l2 = look[(idx << used) & ((1 << LB) - 1)] & 0x1FFFu;
  if (!l2 || (int)(l2 & 31u) > LB - used) return e;
  return e | ((l2 & 31u) << 13) | ((l2 >> 5) << 17) | kLookPair;
}

// Skip entry of a decoded symbol (see HuffSkip); len 17 is libjpeg's fake zero.
DHD uint32_t skip_from_sym(int sym, int len, bool dc) {
  const int s = dc ? sym : sym & 15, r = dc ? 0 : sym >> 4;
  const int zinc = dc ? 1 : (s ? r + 1 : (r == 15 ? 16 : 64));
  return (uint32_t)(len + s) | ((uint32_t)zinc << 5);
}

// Skip entry for a lookahead entry (0 stays 0: the long-code path).
DHD uint32_t skip_entry(uint32_t look, bool dc) {
  return look ? skip_from_sym((int)(look >> 5), (int)(look & 31u), dc) : 0u;
}

// AC skip entry of lookahead index idx (look: the table's LB-bit value lookahead, its
// single-symbol part) with the second symbol when its code is decided by the index's
// remaining bits and both symbols fit the 32 bits a step may consume.
template <int LB>
DHD uint32_t skip_pair_entry(const uint32_t* look, int idx) {
  const uint32_t e = skip_entry(look[idx] & 0x1FFFu, false);
  const int len1 = (int)(e & 31u);
  if (!e || len1 >= LB) return e;
  const uint32_t l2 = look[(idx << len1) & ((1 << LB) - 1)] & 0x1FFFu;
  if (!l2 || (int)(l2 & 31u) > LB - len1) return e;
  const uint32_t e2 = skip_entry(l2, false);
  if (len1 + (int)(e2 & 31u) > 32) return e;
  return e | ((e2 & 31u) << 12) | ((e2 >> 5) << 17) | kSkipPair;
}

// Bit reader over a destuffed, zero-padded big-endian byte stream.
struct BitReader {
  const uint32_t* words;   // 4-byte aligned base of the stream (byte-swapped on read)
  uint32_t nbytes;         // readable bytes; later bytes read as 0 (libjpeg's zero fill)
};

DHD uint32_t bswap32(uint32_t x) {
  return (x >> 24) | ((x >> 8) & 0xFF00u) | ((x << 8) & 0xFF0000u) | (x << 24);
}

DHD uint32_t br_word(const BitReader& br, uint32_t i) {
  uint32_t b = i * 4;
  if (b + 4 <= br.nbytes) return bswap32(br.words[i]);
  if (b >= br.nbytes) return 0u;
  uint32_t w = bswap32(br.words[i]);
  return w & (0xFFFFFFFFu << (8 * (b + 4 - br.nbytes)));  // keep the first (nbytes-b) bytes
}

// 32 bits starting at absolute bit position pos (MSB first).
DHD uint32_t br_peek32(const BitReader& br, uint32_t pos) {
  uint32_t w = pos >> 5, sh = pos & 31;
  uint64_t v = ((uint64_t)br_word(br, w) << 32) | br_word(br, w + 1);
  return (uint32_t)(v >> (32 - sh));
}

// A lane's cached view of the stream: 64-bit window, left aligned, plus the next
// kPrefetchWords stream words in flight.  The words are kept raw (as loaded) and only
// byte-swapped / end-masked when they enter the window, so a load is waited on
// kPrefetchWords refills (~32 bits each) after it is issued: the speculative decode
// kernels keep one stream line per lane live, ~L2-sized in all, so a refill often comes
// from the Infinity Cache or HBM rather than L2.
constexpr int kPrefetchWords = 1;
struct BitCursor {
  uint64_t buf;        // next bits, MSB first
  int32_t nbits;       // valid bits in buf
  uint32_t pos;        // absolute bit position of the next unread bit
  uint32_t next_word;  // index of the word held (raw) in pf[0]
  uint32_t pf[kPrefetchWords];
};

// Stream sources (template argument kWin of the routines below):
//   kSrcGlobal (false)  destuffed bytes in global memory, exact end: the word holding
//                       br.nbytes keeps only its first bytes, later words read as 0
//                       (restart intervals, whose data is followed by the next one);
//   kSrcWin (true)      a copy staged as big-endian-swapped words, zero beyond nbytes;
//   kSrcPadded          destuffed bytes in global memory followed by >= 8 zero bytes
//                       (k_destuff's pad): a read past the end is clamped to the first
//                       all-zero word, so no masking is needed on the hot path.
// A load past the end is clamped (never out of bounds, no branch around the load).
// (Reading the padded stream as 16-byte chunks fetched a chunk ahead was measured and
// dropped: k_huff1 +20 %; the refill is not what the decode waits on.)
enum : int { kSrcGlobal = 0, kSrcWin = 1, kSrcPadded = 2 };

// Source of the speculative decode kernels (k_huff1/2/3) and of their emulator.
constexpr int kHuffSrc = kSrcPadded;

template <int kWin>
DHD uint32_t src_raw(const BitReader& br, uint32_t i) {
  if (kWin == kSrcPadded) {
    const uint32_t zw = (br.nbytes + 3) >> 2;  // first word wholly inside the zero pad
    return br.words[i < zw ? i : zw];
  }
  const uint32_t last = br.nbytes > 0 ? (br.nbytes - 1) >> 2 : 0u;
  return br.words[i < last ? i : last];
}

template <int kWin>
DHD uint32_t src_cook(const BitReader& br, uint32_t raw, uint32_t i) {
  const uint32_t w = kWin == kSrcWin ? raw : bswap32(raw);
  if (kWin == kSrcPadded) return w;
  const uint32_t b = i * 4;
  if (b + 4 <= br.nbytes) return w;
  if (b >= br.nbytes) return 0u;
  return w & (0xFFFFFFFFu << (8 * (b + 4 - br.nbytes)));  // keep the first (nbytes-b) bytes
}

template <int kWin>
DHD uint32_t src_word(const BitReader& br, uint32_t i) {
  return src_cook<kWin>(br, src_raw<kWin>(br, i), i);
}

DHD uint32_t win_word(const BitReader& br, uint32_t i) { return src_word<kSrcWin>(br, i); }

// Ensure >= 32 valid bits.
template <int kWin>
DHD void bc_fill(BitCursor& c, const BitReader& br) {
  if (c.nbits < 32) {
    c.buf |= (uint64_t)src_cook<kWin>(br, c.pf[0], c.next_word) << (32 - c.nbits);
    c.nbits += 32;
#pragma unroll
    for (int k = 0; k + 1 < kPrefetchWords; ++k) c.pf[k] = c.pf[k + 1];
    c.pf[kPrefetchWords - 1] = src_raw<kWin>(br, c.next_word + kPrefetchWords);
    c.next_word++;
  }
}

template <int kWin>
DHD void bc_init(BitCursor& c, const BitReader& br, uint32_t pos) {
  c.pos = pos;
  uint32_t w = pos >> 5, sh = pos & 31;
  c.buf = (((uint64_t)src_word<kWin>(br, w) << 32) | src_word<kWin>(br, w + 1)) << sh;
  c.nbits = 64 - (int)sh;
  c.next_word = w + 2;
#pragma unroll
  for (int k = 0; k < kPrefetchWords; ++k) c.pf[k] = src_raw<kWin>(br, w + 2 + k);
}

DHD uint32_t bc_peek(const BitCursor& c, int n) { return (uint32_t)(c.buf >> (64 - n)); }

DHD void bc_skip(BitCursor& c, int n) {
  c.buf <<= n;
  c.nbits -= n;
  c.pos += n;
}

// Symbol whose code is longer than LB bits (jpeg_huff_decode's bit-serial loop,
// incl. the l = 17 "fake zero").  The maxcode values are read up front and the
// length found by comparisons, so the lane waits on LDS once, not per bit.
// p17: the next 17 bits of the stream (code of up to 16 bits + sentinel).
template <int LB, typename TabPtr>
DHD void huff_slow_bits(uint32_t p17, TabPtr t, int* sym, int* len) {
  int32_t mc[17 - LB], vo[17 - LB];
#pragma unroll
  for (int k = 0; k < 17 - LB; ++k) {
    mc[k] = t->maxcode[LB + 1 + k];
    vo[k] = t->valoffset[LB + 1 + k];
  }
  int l = 17, off = 0;
#pragma unroll
  for (int k = 16 - LB; k >= 0; --k) {
    if ((int32_t)(p17 >> (16 - LB - k)) <= mc[k]) {
      l = LB + 1 + k;
      off = vo[k];
    }
  }
  if (l > 16) {  // JWRN_HUFF_BAD_CODE: libjpeg fakes a zero after 17 bits
    *sym = 0;
    *len = 17;
    return;
  }
  const int code = (int)(p17 >> (17 - l));
  *sym = t->huffval[(code + off) & 255];
  *len = l;
}

template <int LB, typename T>
DHD void huff_slow(const BitCursor& c, const T* t, int* sym, int* len) {
  huff_slow_bits<LB>(bc_peek(c, 17), t, sym, len);
}

// Decoder state between steps.
struct HState {
  uint32_t pos;   // bit position of the next step
  int32_t c;      // block index within the MCU
  int32_t z;      // next zigzag index; 0 = expecting the DC symbol
};

DHD bool hstate_eq(const HState& a, const HState& b) { return a.pos == b.pos && a.c == b.c && a.z == b.z; }

// Tables of one image as the decoder sees them (pointers into LDS on the GPU).
// Everything a lane indexes per step is a base pointer or a packed word, so that
// no per-lane array is dynamically indexed (which would spill it to scratch).
struct HuffImage {
  const HuffTables* tabs;      // derived tables and value lookaheads as in HuffTables
  uint32_t skip_off;           // byte offset of the HuffSkip entries from tabs
  uint32_t mcu_comp;           // component of block b of the MCU in bits [2b, 2b+2)
  int32_t blocks_per_mcu;
};

DHD const uint32_t* hi_skip(const HuffImage& im) {
  return reinterpret_cast<const uint32_t*>(reinterpret_cast<const uint8_t*>(im.tabs) + im.skip_off);
}

DHD void hi_init(HuffImage& im, const HuffTables* tabs, const uint8_t* mcu_comp, int blocks_per_mcu) {
  im.tabs = tabs;
  im.skip_off = (uint32_t)offsetof(HuffTables, skip);
  im.mcu_comp = 0;
  for (int i = 0; i < blocks_per_mcu && i < kMaxBlocksPerMcu; ++i) im.mcu_comp |= (uint32_t)(mcu_comp[i] & 3) << (2 * i);
  im.blocks_per_mcu = blocks_per_mcu;
}

DHD int hi_comp(const HuffImage& im, int blk) { return (int)((im.mcu_comp >> (2 * blk)) & 3u); }

// a[c] += v for a 3-vector kept in registers.
DHD void add3(int32_t* a, int c, int32_t v) {
  if (c == 0)
    a[0] += v;
  else if (c == 1)
    a[1] += v;
  else
    a[2] += v;
}

DHD int32_t get3(const int32_t* a, int c) { return c == 0 ? a[0] : (c == 1 ? a[1] : a[2]); }

// Result of one step.
struct StepOut {
  int32_t kind;    // 0 = DC (value = diff), 1 = AC coefficient (value, zz index), 2 = no coefficient
  int32_t value;
  int32_t zz;
  int32_t ac2;     // a second AC coefficient in the same step (value2, zz2)
  int32_t value2;
  int32_t zz2;
  int32_t block_done;
};

// Bits [off, off + width) (LSB = bit 0) of x; width 0 gives 0.
DHD uint32_t ubfe(uint32_t x, uint32_t off, uint32_t width) {
#if defined(__HIP_DEVICE_COMPILE__)
  return __builtin_amdgcn_ubfe(x, off, width);
#else
  return width ? (x >> off) & (0xFFFFFFFFu >> (32 - width)) : 0u;
#endif
}

// Execute one step from cursor c / state (c, z).  Updates state.  One lookahead
// read gives the symbol and code length of every code of <= kLookBits bits; the
// extra bits are then extracted from the same 32-bit view of the window, so
// short and long (code + extra) steps take one branch-free path and the lanes of
// a wave only diverge for codes longer than kLookBits.  An AC entry carrying a second
// symbol (look_pair_entry) completes it in the same step while the first leaves the
// block open (ac2 = 1: a second coefficient; a second ZRL or EOB only moves z).
template <int kWin>
DHD StepOut huff_step(BitCursor& cur, const BitReader& br, const HuffImage& im, int32_t& blk, int32_t& z) {
  StepOut o;
  o.block_done = 0;
  o.ac2 = 0;
  bc_fill<kWin>(cur, br);
  const int comp = hi_comp(im, blk);
  const bool dc = z == 0;
  const uint32_t hi32 = (uint32_t)(cur.buf >> 32);  // >= 32 valid bits after bc_fill
  const uint32_t e = dc ? (uint32_t)im.tabs->dc_look[comp][hi32 >> (32 - kDcLookBits)]
                        : im.tabs->ac_look[comp][hi32 >> (32 - kLookBits)];
  int sym, len;
  if (e) {
    sym = (int)((e >> 5) & 255u);
    len = (int)(e & 31u);
  } else if (dc) {
    huff_slow<kDcLookBits>(cur, im.tabs->dc + comp, &sym, &len);
  } else {
    huff_slow<kLookBits>(cur, im.tabs->ac + comp, &sym, &len);
  }
  const int s = dc ? sym : sym & 15;  // s <= 15 (DC tables are validated), len <= 17: len + s < 32
  const int r = dc ? 0 : sym >> 4;
  const uint32_t x = ubfe(hi32, (uint32_t)(32 - len - s), (uint32_t)s);
  const int v = s ? huff_extend((int)x, s) : 0;
  int used = len + s;
  if (dc) {
    o.kind = 0;
    o.value = v;
    o.zz = 0;
    z = 1;
  } else if (s) {  // = (v != 0): an extended value of s >= 1 bits is never 0; the
                   // state update then does not wait on the value (dead in the skip decodes)
    z += r;
    o.kind = 1;
    o.value = v;
    o.zz = z > 79 ? 79 : z;
    z += 1;
  } else {
    o.kind = 2;
    o.value = 0;
    o.zz = 0;
    if (r == 15)
      z += 16;
    else
      z = 64;  // EOB
  }
  if ((e & kLookPair) && z < 64) {  // (AC entries only) the second symbol, inside the same 32-bit view
    const int len2 = (int)((e >> 13) & 15u), sym2 = (int)((e >> 17) & 255u);
    const int s2 = sym2 & 15, r2 = sym2 >> 4;
    const uint32_t x2 = ubfe(hi32, (uint32_t)(32 - used - len2 - s2), (uint32_t)s2);
    used += len2 + s2;
    if (s2) {
      z += r2;
      o.ac2 = 1;
      o.value2 = huff_extend((int)x2, s2);
      o.zz2 = z > 79 ? 79 : z;
      z += 1;
    } else if (r2 == 15) {
      z += 16;
    } else {
      z = 64;
    }
  }
  bc_skip(cur, used);
  if (z >= 64) {
    z = 0;
    blk = blk + 1 == im.blocks_per_mcu ? 0 : blk + 1;
    o.block_done = 1;
  }
  return o;
}

// huff_step's effect on the state (c, z, bit position) alone, for the decodes that
// only look for block boundaries and end states: one HuffSkip lookup gives the bits
// and the zigzag advance, so no extra-bit value is extracted.  Same state sequence as
// huff_step (checked by the emulator tests, which run both on the same streams).
// With a two-symbol entry both are taken when the first leaves the block open and ends
// before `lim`: the decodes stop at the first step boundary >= their end, which must
// stay a boundary they visit (the sync rounds compare end and start states), and
// block boundaries (checkpoints) are never stepped over.
template <int kWin>
DHD void skip_step(BitCursor& cur, const BitReader& br, const HuffImage& im, int32_t& blk, int32_t& z, uint32_t lim) {
  bc_fill<kWin>(cur, br);
  const int comp = hi_comp(im, blk);
  const bool dc = z == 0;
  const uint32_t hi32 = (uint32_t)(cur.buf >> 32);
  const uint32_t* tab = hi_skip(im) + (dc ? 3 * (1 << kLookBits) + comp * (1 << kDcLookBits) : comp * (1 << kLookBits));
  uint32_t e = tab[hi32 >> (dc ? 32 - kDcLookBits : 32 - kLookBits)];
  if (!e) {
    int sym, len;
    if (dc)
      huff_slow<kDcLookBits>(cur, im.tabs->dc + comp, &sym, &len);
    else
      huff_slow<kLookBits>(cur, im.tabs->ac + comp, &sym, &len);
    e = skip_from_sym(sym, len, dc);
  }
  uint32_t len = e & 31u;
  int32_t zi = (int32_t)((e >> 5) & 127u);
  if ((e & kSkipPair) && z + zi < 64 && cur.pos + len < lim) {
    len += (e >> 12) & 31u;
    zi += (int32_t)((e >> 17) & 127u);
  }
  bc_skip(cur, (int)len);
  z += zi;
  if (z >= 64) {
    z = 0;
    blk = blk + 1 == im.blocks_per_mcu ? 0 : blk + 1;
  }
}

// ---------------------------------------------------------------------------
// Lane-level routines of the self-synchronising parallel decode (k_huffman).
// ---------------------------------------------------------------------------

// The step of the state-only decodes (skip_step; huff_step there measured slower).
template <int kWin>
DHD void state_step(BitCursor& cur, const BitReader& br, const HuffImage& im, int32_t& blk, int32_t& z, uint32_t lim) {
  skip_step<kWin>(cur, br, im, blk, z, lim);
}

// A guessed start state for the range starting at bit `to`: decode state-only from an
// earlier bit `from` (block-in-MCU 0, zigzag 0 guessed there) up to the first step
// boundary >= to.  By then the decode has usually fallen into the true codeword and
// MCU-phase sequence (the sync distance), so the range's first decode starts from the
// true state more often and the sync rounds redo fewer ranges.
template <int kWin>
DHD HState decode_lookback(const BitReader& br, const HuffImage& im, uint32_t from, uint32_t to) {
  BitCursor cur;
  bc_init<kWin>(cur, br, from);
  int32_t blk = 0, z = 0;
  while (cur.pos < to) state_step<kWin>(cur, br, im, blk, z, to);
  return HState{cur.pos, blk, z};
}

// What a lane learns by decoding the steps that start in [st.pos, end).
struct RangeOut {
  HState end;      // state at the first step boundary >= end
  int32_t nblk;    // blocks whose DC step starts in the range
};

constexpr int kHuffCheckpoints = 16;  // block boundaries recorded per lane by the first decode
constexpr int kHuffCpDense = 4;    // leading blocks that all get a checkpoint
constexpr int kHuffCpStride = 8;  // then every kHuffCpStride-th block (power of 2)

// A block boundary (state before a DC step) seen by a lane's first decode:
// bit position, block-in-MCU index c and the blocks started before it.
struct Checkpoint {
  uint32_t pos;
  uint32_t cn;  // (blocks before << 4) | c
};

// A state is only ever produced by the decoder itself; clamp anyway so that no
// index derived from it can leave the MCU tables.
DHD HState sanitize(HState st, int bpm) {
  if (st.c < 0 || st.c >= bpm) st.c = 0;
  if (st.z < 0 || st.z > 63) st.z = 0;
  return st;
}

// First (speculative) decode of a range; records up to kmax block boundaries at
// cps[0], cps[cstride], ... (the kernels interleave the lanes' checkpoints, so that
// the lanes of a wave recording their n-th checkpoint write neighbouring words).
template <int kWin>
DHD RangeOut decode_range(const BitReader& br, const HuffImage& im, HState st, uint32_t end, Checkpoint* cps,
                          int cstride, int kmax, int32_t* ncp) {
  st = sanitize(st, im.blocks_per_mcu);
  RangeOut r;
  r.nblk = 0;
  int n = 0;
  BitCursor cur;
  bc_init<kWin>(cur, br, st.pos);
  int32_t blk = st.c, z = st.z;
  while (cur.pos < end) {
    if (z == 0) {
      // every block boundary at first (where a re-decode from a corrected state
      // usually meets the first decode), then every kHuffCpStride-th: fewer stores
      if (n < kmax && (r.nblk < kHuffCpDense || (r.nblk & (kHuffCpStride - 1)) == 0))
        cps[(n++) * cstride] = Checkpoint{cur.pos, ((uint32_t)r.nblk << 4) | (uint32_t)blk};
      r.nblk++;
    }
    state_step<kWin>(cur, br, im, blk, z, end);
  }
  r.end.pos = cur.pos;
  r.end.c = blk;
  r.end.z = z;
  *ncp = n;
  return r;
}

// Re-decode of a range from a corrected start state.  As soon as the decode
// reaches a block boundary the first decode also passed through (same bit
// position, same block-in-MCU index), everything after it is what the first
// decode already found: its end state and remaining block count are reused.
template <int kWin>
DHD RangeOut decode_range_sync(const BitReader& br, const HuffImage& im, HState st, uint32_t end,
                               const Checkpoint* cps, int cstride, int ncp, RangeOut first) {
  st = sanitize(st, im.blocks_per_mcu);
  int32_t nblk = 0;
  int j = 0;
  BitCursor cur;
  bc_init<kWin>(cur, br, st.pos);
  int32_t blk = st.c, z = st.z;
  // the next checkpoint at or after the position, kept in registers: memory is only
  // read when the decode passes one (every kHuffCpStride blocks), not at every block
  Checkpoint cp = ncp > 0 ? cps[0] : Checkpoint{0xFFFFFFFFu, 0u};
  while (cur.pos < end) {
    if (z == 0) {
      while (cp.pos < cur.pos) cp = ++j < ncp ? cps[j * cstride] : Checkpoint{0xFFFFFFFFu, 0u};
      if (cp.pos == cur.pos && (int32_t)(cp.cn & 15u) == blk) {
        RangeOut r = first;
        r.nblk = nblk + first.nblk - (int32_t)(cp.cn >> 4);
        return r;
      }
      nblk++;
    }
    state_step<kWin>(cur, br, im, blk, z, end);
  }
  RangeOut r;
  r.end.pos = cur.pos;
  r.end.c = blk;
  r.end.z = z;
  r.nblk = nblk;
  return r;
}

// Block sink interface (duck-typed): begin(absolute_block) opens a block,
// ac(zigzag_index, int16) receives one non-zero AC coefficient (zigzag indices are
// strictly increasing within a block; an index > 63 only comes from a corrupt
// stream and is the block's last, mapped to natural position 63 as libjpeg's
// jpeg_natural_order does), dc(int16) the block's DC, end() closes the block;
// zero(absolute_block) records an all-zero block whose DC is an absolute 0.
// Decode from `st` (a true state) and emit every block whose DC step starts before
// `end`, finishing the last one past `end`; the leading partial block (st.z != 0)
// belongs to the previous lane and is decoded without being emitted.  Stops at
// `total_blocks`.  DC: with `pred` the sink gets the absolute value (DC predictors
// carried by the caller); without, the difference (summed later by the DC prefix
// pass, k_dcscan).  A difference fits int16: DC categories are <= 15.
// `avail`: bits of entropy data before the terminating marker.  libjpeg
// (jdhuff.c jpeg_fill_bit_buffer / decode_mcu) zero-fills a step that needs bits
// past it, sets insufficient_data and finishes that MCU from zero bits; every later
// MCU of the segment is left all zero (DC 0, not predicted).  So an MCU that starts
// past `avail` and everything after it become zero blocks.  Only the lane whose
// range runs to the end of the segment reaches them (any other stops at its range
// end first).  Returns the bit position.
template <int kWin, typename Sink>
DHD uint32_t decode_write(const BitReader& br, const HuffImage& im, HState st, uint32_t end, int32_t first_block,
                          int32_t total_blocks, int32_t* pred, uint32_t avail, Sink& sink) {
  st = sanitize(st, im.blocks_per_mcu);
  BitCursor cur;
  bc_init<kWin>(cur, br, st.pos);
  int32_t blk = st.c, z = st.z;
  while (z != 0) {  // skip the tail of the previous lane's block
    huff_step<kWin>(cur, br, im, blk, z);
  }
  int32_t b = first_block;
  if (!(b < total_blocks && cur.pos < end)) return cur.pos;
  // one step per iteration, blocks opened and closed inside the loop: a loop per block
  // would keep a wave in each block until its longest lane finished that block
  bool open = false;
  int comp = 0;
  for (;;) {
    if (!open) {
      if (blk == 0 && cur.pos > avail) {  // insufficient_data before this MCU: the rest stays zero
        for (; b < total_blocks; ++b) sink.zero(b);
        break;
      }
      sink.begin(b);
      comp = hi_comp(im, blk);
      open = true;
    }
    const StepOut o = huff_step<kWin>(cur, br, im, blk, z);
    if (o.kind == 0) {
      if (pred) add3(pred, comp, o.value);
      sink.dc((int16_t)(pred ? get3(pred, comp) : o.value));
    } else if (o.kind == 1) {
      sink.ac(o.zz, (int16_t)o.value);
    }
    if (o.ac2) sink.ac(o.zz2, (int16_t)o.value2);
    if (o.block_done) {
      sink.end();
      ++b;
      open = false;
      if (!(b < total_blocks && cur.pos < end)) break;
    }
  }
  return cur.pos;
}

// Element offset (int16 units) of absolute block b inside the image's coefficient area.
DHD int64_t coef_block_offset(const ImgDesc& d, int32_t b) {
  const int bpm = d.blocks_per_mcu;
  const int m = b / bpm, c = b - m * bpm;
  const CompDesc& cd = d.comp[d.mcu_comp[c]];
  const int one = d.ncomp == 1;
  const int bx = (m % d.mcus_x) * (one ? 1 : cd.h) + d.mcu_bx[c];
  const int by = (m / d.mcus_x) * (one ? 1 : cd.v) + d.mcu_by[c];
  return cd.coef_off / 2 + ((int64_t)by * cd.bw + bx) * 64;
}

}  // namespace dino
