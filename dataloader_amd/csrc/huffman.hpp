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

// Derived decoding table for one Huffman table (jpeg_make_d_derived_tbl).
struct HuffTable {
  int32_t maxcode[18];     // maxcode[l], -1 if no codes of length l; [17] sentinel
  int32_t valoffset[18];
  uint8_t huffval[256];
  uint16_t look[1 << kLookBits];  // (len << 8) | symbol for codes <= kLookBits bits, 0 = slow path
};

// Build maxcode/valoffset/huffval (not the lookahead) from BITS[16] + HUFFVAL.
// Returns false on an invalid table (libjpeg JERR_BAD_HUFF_TABLE).
DHD bool huff_build_derived(const uint8_t* bits16, bool is_dc, HuffTable* t) {
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

// Lookahead entry for the kLookBits-bit prefix `idx` (computable independently per entry).
DHD uint16_t huff_look_entry(const HuffTable* t, int idx) {
  for (int l = 1; l <= kLookBits; ++l) {
    int code = idx >> (kLookBits - l);
    if (code <= t->maxcode[l]) {  // canonical code: first length whose maxcode covers the prefix
      int sym = t->huffval[(code + t->valoffset[l]) & 255];
      return (uint16_t)((l << 8) | sym);
    }
  }
  return 0;
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

// A lane's cached view of the stream: 64-bit window, left aligned.
struct BitCursor {
  uint64_t buf;   // next bits, MSB first
  int32_t nbits;  // valid bits in buf
  uint32_t pos;   // absolute bit position of the next unread bit
  uint32_t next_word;
};

DHD void bc_init(BitCursor& c, const BitReader& br, uint32_t pos) {
  c.pos = pos;
  uint32_t w = pos >> 5, sh = pos & 31;
  c.buf = (((uint64_t)br_word(br, w) << 32) | br_word(br, w + 1)) << sh;
  c.nbits = 64 - (int)sh;
  c.next_word = w + 2;
}

// Ensure >= 32 valid bits.
DHD void bc_fill(BitCursor& c, const BitReader& br) {
  if (c.nbits < 32) {
    c.buf |= (uint64_t)br_word(br, c.next_word) << (32 - c.nbits);
    c.nbits += 32;
    c.next_word++;
  }
}

DHD uint32_t bc_peek(const BitCursor& c, int n) { return (uint32_t)(c.buf >> (64 - n)); }

DHD void bc_skip(BitCursor& c, int n) {
  c.buf <<= n;
  c.nbits -= n;
  c.pos += n;
}

// Decode one Huffman symbol (jpeg_huff_decode semantics incl. the l=17 "fake zero").
// Requires >= 17 valid bits in the cursor.
DHD int huff_decode_sym(BitCursor& c, const HuffTable* t) {
  uint32_t look = bc_peek(c, kLookBits);
  uint16_t e = t->look[look];
  if (e) {
    bc_skip(c, e >> 8);
    return e & 0xFF;
  }
  uint32_t p16 = bc_peek(c, 17);  // 17 bits: code of up to 16 bits + sentinel
  int l = kLookBits + 1;
  int code = (int)(p16 >> (17 - l));
  while (code > t->maxcode[l]) {
    ++l;
    code = (int)(p16 >> (17 - l));
    if (l == 17) break;
  }
  if (l > 16) {
    bc_skip(c, 17);
    return 0;  // JWRN_HUFF_BAD_CODE: libjpeg fakes a zero
  }
  bc_skip(c, l);
  return t->huffval[(code + t->valoffset[l]) & 255];
}

DHD int huff_extend(int x, int s) { return x < (1 << (s - 1)) ? x + (int)(((unsigned)-1) << s) + 1 : x; }

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
  const HuffTable* tabs;   // [6]: DC tables of components 0..2, then AC tables 0..2
  uint32_t mcu_comp;       // component of block b of the MCU in bits [2b, 2b+2)
  int32_t blocks_per_mcu;
};

DHD void hi_init(HuffImage& im, const HuffTable* tabs, const uint8_t* mcu_comp, int blocks_per_mcu) {
  im.tabs = tabs;
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
  int32_t block_done;
};

// Execute one step from cursor c / state (c, z).  Updates state.
DHD StepOut huff_step(BitCursor& cur, const BitReader& br, const HuffImage& im, int32_t& blk, int32_t& z) {
  StepOut o;
  o.block_done = 0;
  bc_fill(cur, br);
  int comp = hi_comp(im, blk);
  if (z == 0) {
    int s = huff_decode_sym(cur, im.tabs + comp);
    int diff = 0;
    if (s) {  // >= 15 bits remain after a <= 17-bit code (bc_fill guaranteed >= 32)
      uint32_t r = bc_peek(cur, s);
      bc_skip(cur, s);
      diff = huff_extend((int)r, s);
    }
    o.kind = 0;
    o.value = diff;
    o.zz = 0;
    z = 1;
  } else {
    int rs = huff_decode_sym(cur, im.tabs + 3 + comp);
    int r = rs >> 4, s = rs & 15;
    if (s) {
      z += r;
      uint32_t v = bc_peek(cur, s);
      bc_skip(cur, s);
      o.kind = 1;
      o.value = huff_extend((int)v, s);
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
  }
  if (z >= 64) {
    z = 0;
    blk = blk + 1 == im.blocks_per_mcu ? 0 : blk + 1;
    o.block_done = 1;
  }
  return o;
}

// ---------------------------------------------------------------------------
// Lane-level routines of the self-synchronising parallel decode (k_huffman).
// ---------------------------------------------------------------------------

// What a lane learns by decoding the steps that start in [st.pos, end).
struct RangeOut {
  HState end;          // state at the first step boundary >= end
  int32_t nblk;        // blocks whose DC step starts in the range
  int32_t dcsum[kMaxComp];
};

// A state is only ever produced by the decoder itself; clamp anyway so that no
// index derived from it can leave the MCU tables.
DHD HState sanitize(HState st, int bpm) {
  if (st.c < 0 || st.c >= bpm) st.c = 0;
  if (st.z < 0 || st.z > 63) st.z = 0;
  return st;
}

DHD RangeOut decode_range(const BitReader& br, const HuffImage& im, HState st, uint32_t end) {
  st = sanitize(st, im.blocks_per_mcu);
  RangeOut r;
  r.nblk = 0;
  r.dcsum[0] = r.dcsum[1] = r.dcsum[2] = 0;
  BitCursor cur;
  bc_init(cur, br, st.pos);
  int32_t blk = st.c, z = st.z;
  while (cur.pos < end) {
    if (z == 0) r.nblk++;
    int comp = hi_comp(im, blk);
    StepOut o = huff_step(cur, br, im, blk, z);
    if (o.kind == 0) add3(r.dcsum, comp, o.value);
  }
  r.end.pos = cur.pos;
  r.end.c = blk;
  r.end.z = z;
  return r;
}

// Block sink interface (duck-typed): zero(), set(natural_index, int16), flush(absolute_block).
// Decode from `st` (a true state, with DC predictors `pred`) and emit every block whose DC
// step starts before `end`, finishing the last one past `end`; the leading partial block
// (st.z != 0) belongs to the previous lane and is decoded without being emitted.  Stops at
// `total_blocks`.  Returns the bit position reached.
template <typename Sink>
DHD uint32_t decode_write(const BitReader& br, const HuffImage& im, HState st, uint32_t end, int32_t first_block,
                          int32_t total_blocks, int32_t* pred, Sink& sink) {
  st = sanitize(st, im.blocks_per_mcu);
  BitCursor cur;
  bc_init(cur, br, st.pos);
  int32_t blk = st.c, z = st.z;
  while (z != 0) {  // skip the tail of the previous lane's block
    huff_step(cur, br, im, blk, z);
  }
  int32_t b = first_block;
  while (b < total_blocks && cur.pos < end) {
    sink.zero();
    int comp = hi_comp(im, blk);
    for (;;) {
      StepOut o = huff_step(cur, br, im, blk, z);
      if (o.kind == 0) {
        add3(pred, comp, o.value);
        sink.set(0, (int16_t)get3(pred, comp));
      } else if (o.kind == 1) {
        sink.set(kNaturalOrder[o.zz], (int16_t)o.value);
      }
      if (o.block_done) break;
    }
    sink.flush(b);
    ++b;
  }
  return cur.pos;
}

}  // namespace dino
