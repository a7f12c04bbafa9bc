// lscan.hpp — progressive JPEGs decoded many at once: one LANE per scan (round 6).
//
// Semantics are pscan.hpp's (libjpeg-turbo 3.1 jdphuff.c decode_mcu_DC_first /
// decode_mcu_AC_first / decode_mcu_DC_refine / decode_mcu_AC_refine, jdhuff.c
// jpeg_fill_bit_buffer's zero fill and insufficient_data); what changes is the mapping.
//
// k_pscan (pscan.hpp) decodes a scan per wave as wave-uniform scalar code.  Its throughput
// is bounded by the scalar ALU, which the four SIMDs of a CU share: ~2 scan waves per CU
// saturate it, and the batch kernels running next to the side decode need it too (side
// pools of 512 progressive images took 50-120 ms of GPU time each under a running C2
// pipeline, 5.6k progressive images/s, profiles/r06_prog_side_*).  Here a wave decodes the
// same scan index of 64 images, one per lane, as ordinary vector code: the work moves to
// the VALU (64 lanes per instruction, 4 SIMDs per CU), so a 512-image pool needs 8 waves
// per scan index instead of 512, while a lane's symbol latency stays close to a scan
// wave's.
//
// What a lane must not do is wait on memory inside its serial chain, so the scan's state
// lives where a lane reaches it cheaply:
//   * the scan's entropy bytes are destuffed beforehand (k_pwalk) and read through a
//     4-dword register window with two dwords loaded ahead (LaneReader);
//   * the lookahead table of the scan's main Huffman table (8 bits, 256 entries) sits in
//     the lane's row of the workgroup's LDS; other tables and longer codes go to the PTab
//     in global memory (LaneTabs);
//   * AC refinement needs, per block, which coefficients earlier scans made non-zero, not
//     their values.  That "history" is kept as a zigzag bit mask per block (side record,
//     below), set by the AC first scans and the refinements' new coefficients with
//     fire-and-forget atomic ORs (scans of one level may share a mask word, never a bit).
//     The refinement itself (corrections, new coefficients, signs) is recorded per block
//     and scan as three masks, and k_papply applies all of them, in scan order, after the
//     last scan — data-parallel, a lane per coefficient.  DC refinement bits are deferred
//     the same way (one byte per block and scan).
//
// Deferring is exact when every coefficient's first scan precedes its refinements (the
// rule of every valid progression; lane_plan checks it, with the slot capacities below).
// Other images — restart intervals, bogus progressions, sequential multi-scan files — keep
// the wave decoder (k_pscan), which applies everything in place.
//
// The host emulator (tests/emu) runs lane_plan / lane_scan_decode / lane_apply_block with
// plain memory.
#pragma once

#include "pscan.hpp"

namespace dino {

// Side record of a block (kind-1 images, the image's binfo area; block b = coefficient
// element >> 6 of the dense buffer): the zigzag non-zero mask, the AC refinement triples
// {corrections, new, negative} of up to kLMaxAcSlots scans of its component, then one
// byte per DC refinement scan.
constexpr int kLSideBytes = 128;
constexpr int kLMaxAcSlots = 4;
constexpr int kLMaxDcSlots = 8;
constexpr int kLTripleOff = 8;
constexpr int kLDcOff = kLTripleOff + 24 * kLMaxAcSlots;
static_assert(kLDcOff + kLMaxDcSlots <= kLSideBytes, "side record layout");

// Which refinement slot each scan writes and the slots' approximation bits.  Packed (4 bits
// per field) into the image's PHdr by k_pwalk.
struct LanePlan {
  int32_t ok;
  int32_t nac[kMaxComp];                 // AC refinement slots per component
  int32_t al_ac[kMaxComp][kLMaxAcSlots];
  int32_t band_ac[kMaxComp][kLMaxAcSlots];  // ss | se << 6
  int32_t ndc;                           // DC refinement slots (scans)
  int32_t al_dc[kLMaxDcSlots];
};

// lane_plan: slot[i] = the refinement slot of scan i (file order; -1 for first scans).
// Returns whether the image may take the lane decoder.
DHD bool lane_plan(const ScanRec* scans, int n, bool progressive, int32_t* slot, LanePlan* lp) {
  lp->ok = 0;
  lp->ndc = 0;
  for (int c = 0; c < kMaxComp; ++c) {
    lp->nac[c] = 0;
    for (int s = 0; s < kLMaxAcSlots; ++s) lp->al_ac[c][s] = lp->band_ac[c][s] = 0;
  }
  for (int s = 0; s < kLMaxDcSlots; ++s) lp->al_dc[s] = 0;
  if (!progressive || n <= 0) return false;
  uint64_t first[kMaxComp] = {0, 0, 0}, refined[kMaxComp] = {0, 0, 0};  // coefficient bit masks
  for (int i = 0; i < n; ++i) {
    const ScanRec& sr = scans[i];
    slot[i] = -1;
    if (sr.restart_interval != 0) return false;
    const uint64_t band = (uint64_t)low_bits(sr.se + 1) & ~(uint64_t)low_bits(sr.ss);
    for (int k = 0; k < sr.ns && k < 4; ++k) {
      const int c = sr.comp[k];
      if (c < 0 || c >= kMaxComp) return false;
      if (sr.ah == 0) {  // a first scan: never after a first or a refinement of the same coefficient
        if ((first[c] | refined[c]) & band) return false;
        first[c] |= band;
      } else {
        refined[c] |= band;
      }
    }
    if (sr.ah == 0) continue;
    if (sr.ss == 0) {
      if (lp->ndc >= kLMaxDcSlots) return false;
      slot[i] = lp->ndc;
      lp->al_dc[lp->ndc++] = sr.al;
    } else {
      const int c = sr.comp[0];
      if (lp->nac[c] >= kLMaxAcSlots) return false;
      slot[i] = lp->nac[c];
      lp->band_ac[c][lp->nac[c]] = sr.ss | sr.se << 6;
      lp->al_ac[c][lp->nac[c]++] = sr.al;
    }
  }
  lp->ok = 1;
  return true;
}

// Packed form (PHdr::lane_*): nac 4 bits per component; AC slot al's 4 bits each, component c
// at bits [16 c, 16 c + 16) of a 64-bit word; AC slot bands 12 bits each (ss | se << 6), one
// 64-bit word per component; DC al's 4 bits each.
DHD void lane_pack(const LanePlan& lp, uint32_t* nac, uint64_t* al_ac, uint64_t* band_ac, uint32_t* ndc,
                   uint32_t* al_dc) {
  *nac = 0;
  *al_ac = 0;
  for (int c = 0; c < kMaxComp; ++c) {
    *nac |= (uint32_t)lp.nac[c] << (4 * c);
    band_ac[c] = 0;
    for (int s = 0; s < kLMaxAcSlots; ++s) {
      *al_ac |= (uint64_t)(lp.al_ac[c][s] & 15) << (16 * c + 4 * s);
      band_ac[c] |= (uint64_t)(lp.band_ac[c][s] & 0xFFF) << (12 * s);
    }
  }
  *ndc = (uint32_t)lp.ndc;
  *al_dc = 0;
  for (int s = 0; s < kLMaxDcSlots; ++s) *al_dc |= (uint32_t)(lp.al_dc[s] & 15) << (4 * s);
}

// Index of set bit number r (0-based, increasing) of z, or 64 when z has <= r set bits:
// branch-free (a lane-divergent loop costs every lane of the wave its longest trip).
DHD int select64(uint64_t z, int r) {
  uint32_t x = (uint32_t)z;
  int pos = 0, c = __builtin_popcount(x);
  bool up = r >= c;
  x = up ? (uint32_t)(z >> 32) : x;
  r -= up ? c : 0;
  pos += up ? 32 : 0;
#pragma unroll
  for (int w = 16; w >= 1; w >>= 1) {
    c = __builtin_popcount(x & ((1u << w) - 1u));
    up = r >= c;
    x = up ? x >> w : x;
    r -= up ? c : 0;
    pos += up ? w : 0;
  }
  return (r == 0 && (x & 1u)) ? pos : 64;
}

// decode_mcu_AC_refine of one block (r_refine_block's bookkeeping) that returns the
// correction bits as read — in stream order, MSB first, one per coefficient of the band
// that was non-zero before the scan (every one of them gets exactly one) — instead of
// distributing them: k_papply (lane_apply_block) matches them with those coefficients.
template <class R, class T>
DHD void r_refine_block_seq(R& r, const T& t, int ss, int se, uint64_t nzz, int32_t* eobrun, uint64_t* seq_out,
                            uint64_t* new_out, uint64_t* neg_out) {
  uint64_t seq = 0, nzn = 0, neg = 0;
  int nseq = 0;
  int k = ss;
  const uint64_t band = (uint64_t)low_bits(se + 1) & ~(uint64_t)low_bits(ss);
  auto take = [&](int n) {  // n correction bits, <= 63 in all
    while (n > 0) {
      const int m = n > 32 ? 32 : n;
      const uint32_t v = r.peek() >> (32 - m);
      r.skip(m);
      seq |= ((uint64_t)v << (64 - m)) >> nseq;
      nseq += m;
      n -= m;
    }
  };
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
      const int z = select64(~nzz & band & ~(uint64_t)low_bits(k), rr);
      const int stop = z < 64 ? z : se + 1;
      take(__builtin_popcountll(nzz & band & (uint64_t)low_bits(stop) & ~(uint64_t)low_bits(k)));
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
    if (k <= se) take(__builtin_popcountll(nzz & band & ~(uint64_t)low_bits(k)));
    (*eobrun)--;
  }
  *seq_out = seq;
  *new_out = nzn;
  *neg_out = neg;
}

// One progressive scan on one lane.  R: peek / skip / insuff, maintain() once per step;
// T: lookup(k, p, &sym, &len) (DC scans), lookup_ac(p, &sym, &len), nat(k); Out: set(elem, v)
// (a coefficient), begin_ac(first block, blocks per row, blocks per scan row, blocks, refine)
// then mask(m) (the history of the scan's m-th block) and maintain(m) once per step,
// mask_or(b, bits), ac_ops(b, seq, nzn, neg), dc_op(b).
//
// The AC scans run as a step machine: a step is one symbol of the current block, or a
// block that needs none (EOB run, insufficient data), so the lanes of a wave, each on its
// own image, advance independently instead of in lock step per block (where every block
// would cost the wave its busiest lane's symbols).
template <typename R, typename T, typename D, typename Out>
DHD void lane_scan_decode(R& r, const T& t, D d, const ScanRec& sr, Out& o) {
  const ScanGeom g = pscan_geom(d, sr);
  const int al = sr.al, ss = sr.ss, se = sr.se;
  int32_t eobrun = 0;
  if (ss > 0) {  // AC scans: one component, one block per MCU (start_pass_phuff_decoder)
    const int ci = (int)g.comp;
    const int64_t plane = sel3(g.plane, ci);
    const int32_t bw = sel3(g.bw, ci), mcx = g.mcus_x, mcy = g.mcus_y;
    const uint64_t band = (uint64_t)low_bits(se + 1) & ~(uint64_t)low_bits(ss);
    const bool refine = sr.ah > 0;
    const int32_t nblk = mcx * mcy;
    o.begin_ac(plane >> 6, bw, mcx, nblk, refine);
    int32_t m = 0, mx = 0, my = 0;
    bool in_blk = false;
    int k = ss;
    uint64_t nzz = 0, seq = 0, nzn = 0, neg = 0, bits = 0;
    int nseq = 0;
    auto take = [&](int n) {  // n correction bits (<= 63 in a block), appended MSB first
      while (n > 0) {
        const int q = n > 32 ? 32 : n;
        const uint32_t v = r.peek() >> (32 - q);
        r.skip(q);
        seq |= ((uint64_t)v << (64 - q)) >> nseq;
        nseq += q;
        n -= q;
      }
    };
    while (m < nblk) {
      r.maintain();
      o.maintain(m);
      const int64_t e0 = plane + ((int64_t)my * bw + mx) * 64;
      const int64_t b = e0 >> 6;
      bool done = false;  // the block is finished after this step
      if (!in_blk) {
        if (refine) nzz = o.mask(m) & band;
        if (r.insuff()) {  // (libjpeg: the block is skipped, the EOB run kept)
          done = true;
        } else if (eobrun > 0) {
          if (refine) take(__builtin_popcountll(nzz));  // a correction bit per non-zero coefficient
          eobrun--;
          done = true;
        } else {
          in_blk = true;
          k = ss;
          seq = nzn = neg = bits = 0;
          nseq = 0;
        }
      }
      if (in_blk) {  // one symbol
        const uint32_t p = r.peek();
        int sym, len;
        t.lookup_ac(p, &sym, &len);
        const int rr = sym >> 4, s = sym & 15;
        if (refine) {  // decode_mcu_AC_refine (see r_refine_block)
          bool negative = false;
          bool eob = false;
          if (s) {
            negative = peek_extra(p, len, 1) == 0;  // (a size other than 1 is a warning; the bit is read regardless)
            r.skip(len + 1);
          } else if (rr != 15) {
            eobrun = (1 << rr) + (int32_t)peek_extra(p, len, rr);
            r.skip(len + rr);
            eob = true;
          } else {
            r.skip(len);
          }
          if (eob) {
            if (k <= se) take(__builtin_popcountll(nzz & ~(uint64_t)low_bits(k)));
            eobrun--;
            done = true;
          } else {
            // the (rr+1)-th not-yet-non-zero position at or after k (se + 1 when there is none)
            const int z = select64(~nzz & band & ~(uint64_t)low_bits(k), rr);
            const int stop = z < 64 ? z : se + 1;
            take(__builtin_popcountll(nzz & (uint64_t)low_bits(stop) & ~(uint64_t)low_bits(k)));
            k = stop;
            if (s) {  // the new coefficient (k may be se + 1 on a corrupt stream: libjpeg's safety entries)
              const uint64_t bit = k < 64 ? 1ull << k : 1ull << 63;
              nzn |= bit;
              if (negative) neg |= bit;
              else neg &= ~bit;
            }
            done = ++k > se;
          }
        } else {  // decode_mcu_AC_first
          if (s) {
            k += rr;
            const int v = huff_extend((int)peek_extra(p, len, s), s);
            r.skip(len + s);
            const int16_t x = (int16_t)((uint32_t)v << al);
            o.set(e0 + t.nat(k), x);
            bits |= (uint64_t)(x != 0) << (k < 64 ? k : 63);
            done = ++k > se;
          } else if (rr == 15) {
            r.skip(len);
            k += 15;
            done = ++k > se;
          } else {
            eobrun = (1 << rr) + (int32_t)peek_extra(p, len, rr) - 1;
            r.skip(len + rr);
            done = true;
          }
        }
      }
      if (done) {
        if (refine) {
          if (seq | nzn) o.ac_ops(b, seq, nzn, neg);
          if (nzn) o.mask_or(b, nzn);
        } else if (bits) {
          o.mask_or(b, bits);
        }
        seq = nzn = neg = bits = 0;
        nseq = 0;
        in_blk = false;
        ++m;
        if (++mx == mcx) {
          mx = 0;
          ++my;
        }
      }
    }
    return;
  }
  // DC scans (interleaved when ns > 1)
  DcPred last_dc{0, 0, 0, 0};
  const bool refine = sr.ah > 0;
  for (int my = 0; my < g.mcus_y; ++my) {
    for (int mx = 0; mx < g.mcus_x; ++mx) {
      r.maintain();
      if (r.insuff()) continue;
      for (int blk = 0; blk < g.bpm; ++blk) {
        const int64_t e0 = pscan_block_elem(sr, g, mx, my, blk);
        if (refine) {  // decode_mcu_DC_refine
          if (rbits(r, 1)) o.dc_op(e0 >> 6);
          continue;
        }
        const int kk = sg_field(g.kk, blk);  // decode_mcu_DC_first
        const uint32_t p = r.peek();
        int s, len;
        t.lookup(kk, p, &s, &len);
        const int dv = s ? huff_extend((int)peek_extra(p, len, s), s) : 0;
        r.skip(len + s);
        o.set(e0, (int16_t)((uint32_t)last_dc.add(kk, dv) << al));
      }
    }
  }
}

// The deferred refinements of one block, in scan order (k_papply's host form): slot s's
// correction sequence goes, bit j, to the j-th coefficient of its band that is non-zero
// once the slots before it are applied (the history its decode saw).  blk: the
// block's 64 coefficients (natural order), side: its side record, c: its component.
DHD void lane_apply_block(int16_t* blk, const uint8_t* side, int c, uint32_t nac, uint64_t al_ac,
                          const uint64_t* band_ac, uint32_t ndc, uint32_t al_dc) {
  const int na = (int)((nac >> (4 * c)) & 15u);
  for (int s = 0; s < na; ++s) {
    const uint64_t* tr = (const uint64_t*)(side + kLTripleOff + 24 * s);
    const uint64_t seq = tr[0], nzn = tr[1], neg = tr[2];
    const int al = (int)((al_ac >> (16 * c + 4 * s)) & 15u);
    const int bd = (int)((band_ac[c] >> (12 * s)) & 0xFFFu), ss = bd & 63, se = bd >> 6;
    uint64_t corr = 0;  // the sequence's bits on the band's coefficients non-zero before the scan
    int j = 0;
    for (int k = ss; k <= se; ++k)
      if (blk[kNaturalOrder[k]] != 0) corr |= (uint64_t)((seq >> (63 - j++)) & 1u) << k;
    for (uint64_t mm = corr | nzn; mm; mm &= mm - 1) {
      const int k = __builtin_ctzll(mm);
      const int pos = kNaturalOrder[k];
      blk[pos] = ac_refine_value(blk[pos], (corr >> k) & 1u, (nzn >> k) & 1u, (neg >> k) & 1u, al);
    }
  }
  for (int s = 0; s < (int)ndc; ++s)
    if (side[kLDcOff + s]) blk[0] = (int16_t)(blk[0] | (1 << ((al_dc >> (4 * s)) & 15u)));
}

// Host forms of the lane decoder's reader / tables (the emulator): no prefetching to maintain.
struct HostLaneClean : HostClean {
  void maintain() {}
};
struct HostLaneTabs : HostTabs {
  void lookup_ac(uint32_t p, int* sym, int* len) const { lookup(4, p, sym, len); }
};

}  // namespace dino
