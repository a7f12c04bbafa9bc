// Host models of the kernels' phase structure — TEST INFRASTRUCTURE ONLY.
// Each function below mirrors one kernel of dataloader_amd/csrc/kernels.hip with
// plain loops over lanes / threads, calling the same per-lane device functions.
#pragma once

#include <string.h>

#include <algorithm>
#include <vector>

#include "../../dataloader_amd/csrc/augment.hpp"
#include "../../dataloader_amd/csrc/color.hpp"
#include "../../dataloader_amd/csrc/huffman.hpp"
#include "../../dataloader_amd/csrc/idct.hpp"
#include "../../dataloader_amd/csrc/jpeg_parse.hpp"
#include "../../dataloader_amd/csrc/progressive.hpp"
#include "../../dataloader_amd/csrc/pscan.hpp"
#include "../../dataloader_amd/csrc/lscan.hpp"

namespace dino {

// ---- k_destuff (sequential statement of the same classification) ----------
struct Destuffed {
  std::vector<uint8_t> bytes;   // padded with zeros to a multiple of 16 + 64 (k_destuff's pad)
  std::vector<int32_t> rst;     // destuffed byte offset where each restart segment starts
  int32_t len = 0;
  int32_t terminated = 0;
  int32_t rst_bad = 0;  // an RST out of sequence (k_destuff_write)
};

inline Destuffed model_destuff(const uint8_t* r, int n) {
  Destuffed d;
  int E = n;
  for (int k = 0; k < n; ++k) {
    if (r[k] != 0xFF) continue;
    int nx = k + 1 < n ? r[k + 1] : -1;
    if (nx == 0x00 || (nx >= 0xD0 && nx <= 0xD7) || nx == 0xFF) continue;
    E = k;
    d.terminated = nx >= 0;
    break;
  }
  for (int k = 0; k < E; ++k) {
    if (r[k] == 0xFF) {
      int nx = k + 1 < n ? r[k + 1] : -1;
      if (nx == 0x00) d.bytes.push_back(0xFF);
      else if (nx >= 0xD0 && nx <= 0xD7) {
        if ((nx & 7) != (int)(d.rst.size() & 7)) d.rst_bad = 1;
        d.rst.push_back((int32_t)d.bytes.size());
      }
      // fill byte: dropped
    } else if (k > 0 && r[k - 1] == 0xFF) {
      // second byte of FF00 / FFDx: dropped
    } else {
      d.bytes.push_back(r[k]);
    }
  }
  d.len = (int32_t)d.bytes.size();
  while (d.bytes.size() % 16) d.bytes.push_back(0);
  for (int i = 0; i < 64; ++i) d.bytes.push_back(0);
  return d;
}

constexpr int32_t kDcAbsZero = INT32_MIN;  // dcd marker: an absolute DC of 0 (insufficient data)

struct CoefSink {
  const ImgDesc* d;
  int16_t* coef;            // image coefficient area
  int32_t* dcd = nullptr;   // set: DC differences per block (speculative mode), else absolute DC
  int16_t* blk = nullptr;
  int32_t b = 0;
  void begin(int32_t blk_index) {
    b = blk_index;
    blk = coef + coef_block_offset(*d, b);
    memset(blk, 0, 128);
  }
  void ac(int zz, int16_t v) { blk[kNaturalOrder[zz]] = v; }
  void dc(int16_t v) {
    if (dcd)
      dcd[b] = v;
    else
      blk[0] = v;
  }
  void end() {}
  void zero(int32_t blk_index) {
    begin(blk_index);
    if (dcd) dcd[b] = kDcAbsZero;
  }
};

// k_dcscan: running DC sums per component over the blocks in decode order.
inline void model_dcscan(const ImgDesc& d, const HuffImage& im, const int32_t* dcd, int16_t* coef) {
  int32_t p[kMaxComp] = {0, 0, 0};
  for (int32_t b = 0; b < d.total_blocks; ++b) {
    const int c = hi_comp(im, b % d.blocks_per_mcu);
    if (dcd[b] == kDcAbsZero) {
      coef[coef_block_offset(d, b)] = 0;
      continue;
    }
    add3(p, c, dcd[b]);
    coef[coef_block_offset(d, b)] = (int16_t)get3(p, c);
  }
}

inline bool model_tables(const uint8_t* p, const ImgDesc& d, HuffTables* tabs, HuffImage& im) {
  for (int c = 0; c < d.ncomp; ++c) {
    if (!huff_build_derived(p + d.huff_off[d.comp[c].td], true, &tabs->dc[c])) return false;
    if (!huff_build_derived(p + d.huff_off[4 + d.comp[c].ta], false, &tabs->ac[c])) return false;
    for (int i = 0; i < (1 << kDcLookBits); ++i) tabs->dc_look[c][i] = look_entry_of<kDcLookBits>(&tabs->dc[c], i);
    for (int i = 0; i < (1 << kLookBits); ++i) tabs->ac_look[c][i] = look_entry_of<kLookBits>(&tabs->ac[c], i);
    for (int i = 0; i < (1 << kDcLookBits); ++i) tabs->skip.dc[c][i] = skip_entry(tabs->dc_look[c][i], true);
    for (int i = 0; i < (1 << kLookBits); ++i) tabs->skip.ac[c][i] = skip_pair_entry<kLookBits>(tabs->ac_look[c], i);
    for (int i = 0; i < (1 << kLookBits); ++i) tabs->ac_look[c][i] = look_pair_entry<kLookBits>(tabs->ac_look[c], i);
  }
  hi_init(im, tabs, d.mcu_comp, d.blocks_per_mcu);
  return true;
}

// ---- k_huffman, speculative mode over `lanes` lanes in segments of `seg` lanes ----
// k_huff1: every range decoded from a guessed state recording checkpoints, then
// rounds inside each segment re-decode the ranges whose start state changed
// (stopping at the first checkpoint match; a segment's first lane keeps its
// guess).  k_huff2: the same rounds across the whole image, then the block scan.
// k_huff3: blocks written (DC as differences); then k_dcscan.
template <int kWin>
inline void model_huffman_spec(const BitReader& br, const HuffImage& im, const ImgDesc& d, uint32_t nbits, int lanes,
                               int seg, CoefSink& sink, int32_t* dcd, int32_t* stats) {
  const int total_blocks = d.total_blocks;
  int n = lanes;
  uint32_t sub = (nbits + n - 1) / n;
  sub = (sub + 31) & ~31u;
  if (sub == 0) sub = 32;
  n = std::max(1, std::min(n, (int)((nbits + sub - 1) / sub)));  // as k_htab's h_lanes: no range starts past the data
  if (seg <= 0) seg = n;
  std::vector<HState> S(n);
  std::vector<RangeOut> R(n), R1(n);
  std::vector<Checkpoint> cps((size_t)n * kHuffCheckpoints);
  std::vector<int32_t> ncp(n);
  auto rend = [&](int i) -> uint32_t { return i == n - 1 ? nbits : (uint32_t)(i + 1) * sub; };
  auto wend = [&](int i) -> uint32_t { return i == n - 1 ? 0xFFFFFFFFu : (uint32_t)(i + 1) * sub; };
  for (int i = 0; i < n; ++i) {
    S[i] = HState{(uint32_t)i * sub, 0, 0};
    R[i] = R1[i] = decode_range<kWin>(br, im, S[i], rend(i), &cps[(size_t)i * kHuffCheckpoints], 1, kHuffCheckpoints, &ncp[i]);
  }
  int rounds = 0, redone = 0;
  for (int pass = 0; pass < 2; ++pass) {  // 0: inside segments (k_huff1), 1: whole image (k_huff2)
    for (;;) {
      std::vector<HState> want(n);
      std::vector<char> redo(n, 0);
      for (int i = 1; i < n; ++i) {
        if (pass == 0 && i % seg == 0) continue;
        want[i] = R[i - 1].end;
        redo[i] = !hstate_eq(want[i], S[i]);
      }
      bool any = false;
      for (int i = 1; i < n; ++i) {
        if (!redo[i]) continue;
        S[i] = want[i];
        R[i] = decode_range_sync<kWin>(br, im, S[i], rend(i), &cps[(size_t)i * kHuffCheckpoints], 1, ncp[i], R1[i]);
        any = true;
        ++redone;
      }
      ++rounds;
      if (!any) break;
    }
  }
  int32_t blk0 = 0;
  sink.dcd = dcd;
  for (int i = 0; i < n; ++i) {
    decode_write<kWin>(br, im, S[i], wend(i), blk0, total_blocks, (int32_t*)nullptr, nbits, sink);
    blk0 += R[i].nblk;
  }
  sink.dcd = nullptr;
  model_dcscan(d, im, dcd, sink.coef);
  if (stats) {
    stats[0] = rounds;
    stats[1] = redone;
    stats[2] = n;
  }
}

struct StageCapture {
  std::vector<uint8_t> ent;
  std::vector<int16_t> coef;
  std::vector<uint8_t> planes;
  ImgDesc desc;
};

inline int model_idct_color(const ImgDesc& d, const std::vector<int16_t>& coef, uint8_t* out_rgb, StageCapture* cap);

// k_pwalk + k_pscan: the marker walk, the table slots, then every scan in file order
// (the kernels' level order gives the same coefficients: scans of one level touch
// disjoint coefficients), each through pscan_decode with plain-memory stores.
inline int host_model_decode_multiscan(const uint8_t* p, int64_t len, ImgDesc& d, uint8_t* out_rgb, int32_t* stats,
                                       StageCapture* cap) {
  std::vector<ScanRec> scans(kMaxScans);
  HostMarkerFinder find;
  if (prog_walk(p, len, &d, scans.data(), find) != DINO_IMG_OK) return d.status;
  std::vector<int32_t> slot_off(kPMaxTabs);
  std::vector<uint8_t> slot_dc(kPMaxTabs);
  std::vector<uint64_t> ts(kMaxScans);
  const int ntab = prog_table_slots(scans.data(), d.n_scans, slot_off.data(), slot_dc.data(), ts.data(), kPMaxTabs);
  if (ntab < 0) return DINO_IMG_UNSUPPORTED;
  std::vector<PTab> tabs(ntab > 0 ? ntab : 1);
  for (int s = 0; s < ntab; ++s) {
    ProgTable t;
    if (!huff_build_derived(p + slot_off[s], slot_dc[s] != 0, &t)) return DINO_IMG_CORRUPT;
    ptab_fill_derived(&t, &tabs[s]);
    for (int i = 0; i < (1 << kPLookBits); ++i) tabs[s].look[i] = ptab_look_entry(&t, i);
  }
  std::vector<int16_t> coef(d.coef_bytes / 2, 0);
  std::vector<uint8_t> clean(len + 16, 0);
  for (int i = 0; i < d.n_scans; ++i) {
    const ScanRec& sr = scans[i];
    HostCoefSink sink{coef.data()};
    const HostTabs tb{tabs.data(), ts[i]};
    if (sr.restart_interval == 0) {  // k_pscan's destuffed reader
      HostClean r{clean.data(), host_destuff(p, len, sr.data_off, clean.data())};
      pscan_decode(r, tb, &d, sr, d.progressive != 0, sink);
      std::fill(clean.begin(), clean.end(), 0);
    } else {
      RawReader r;
      pb_init(r.b, (uintptr_t)p, len, sr.data_off);
      pscan_decode(r, tb, &d, sr, d.progressive != 0, sink);
    }
  }
  if (stats) {
    stats[0] = d.n_scans;
    int mx = 0;
    for (int i = 0; i < d.n_scans; ++i) mx = std::max(mx, scans[i].level);
    stats[1] = mx + 1;
  }
  if (cap) {
    cap->desc = d;
    cap->coef = coef;
  }
  return model_idct_color(d, coef, out_rgb, cap);
}

// k_pwalk + k_plscan + k_papply (lscan.hpp): every scan through lane_scan_decode with the
// refinements deferred to side records, then applied block by block in scan order.
// Returns 1 (not decoded) when lane_plan leaves the image to the wave decoder.
struct HostLaneOut {
  int16_t* coef;
  uint8_t* side;
  int slot;
  int64_t blk0 = 0;
  int32_t bw = 0, mcx = 1;
  void set(int64_t e, int16_t v) { coef[e] = v; }
  void begin_ac(int64_t b0, int32_t w, int32_t mx, int32_t, bool) {
    blk0 = b0;
    bw = w;
    mcx = mx;
  }
  void maintain(int32_t) {}
  uint64_t mask(int32_t m) const {
    const int64_t b = blk0 + (int64_t)(m / mcx) * bw + m % mcx;
    return *(const uint64_t*)(side + b * kLSideBytes);
  }
  void mask_or(int64_t b, uint64_t bits) { *(uint64_t*)(side + b * kLSideBytes) |= bits; }
  void ac_ops(int64_t b, uint64_t seq, uint64_t nzn, uint64_t neg) {
    uint64_t* tr = (uint64_t*)(side + b * kLSideBytes + kLTripleOff + 24 * slot);
    tr[0] = seq;
    tr[1] = nzn;
    tr[2] = neg;
  }
  void dc_op(int64_t b) { side[b * kLSideBytes + kLDcOff + slot] = 1; }
};

inline int host_model_decode_lane(const uint8_t* p, int64_t len, ImgDesc& d, uint8_t* out_rgb, int32_t* stats,
                                  StageCapture* cap) {
  std::vector<ScanRec> scans(kMaxScans);
  HostMarkerFinder find;
  if (prog_walk(p, len, &d, scans.data(), find) != DINO_IMG_OK) return d.status;
  std::vector<int32_t> slot(kMaxScans, -1);
  LanePlan lp;
  if (!lane_plan(scans.data(), d.n_scans, d.progressive != 0, slot.data(), &lp)) return 1;
  std::vector<int32_t> slot_off(kPMaxTabs);
  std::vector<uint8_t> slot_dc(kPMaxTabs);
  std::vector<uint64_t> ts(kMaxScans);
  const int ntab = prog_table_slots(scans.data(), d.n_scans, slot_off.data(), slot_dc.data(), ts.data(), kPMaxTabs);
  if (ntab < 0) return DINO_IMG_UNSUPPORTED;
  std::vector<PTab> tabs(ntab > 0 ? ntab : 1);
  for (int s = 0; s < ntab; ++s) {
    ProgTable t;
    if (!huff_build_derived(p + slot_off[s], slot_dc[s] != 0, &t)) return DINO_IMG_CORRUPT;
    ptab_fill_derived(&t, &tabs[s]);
    for (int i = 0; i < (1 << kPLookBits); ++i) tabs[s].look[i] = ptab_look_entry(&t, i);
  }
  const int64_t nblk = d.coef_bytes / 128;
  std::vector<int16_t> coef(d.coef_bytes / 2, 0);
  std::vector<uint8_t> side((size_t)nblk * kLSideBytes, 0);
  std::vector<uint8_t> clean(len + 16, 0);
  // the kernels run the scans level by level; file order gives the same result (a scan only
  // reads the history of earlier levels, which file order has finished too)
  for (int i = 0; i < d.n_scans; ++i) {
    const ScanRec& sr = scans[i];
    HostLaneOut o{coef.data(), side.data(), slot[i]};
    HostLaneTabs tb;
    tb.tabs = tabs.data();
    tb.ts = ts[i];
    HostLaneClean r;
    r.s = clean.data();
    r.n = host_destuff(p, len, sr.data_off, clean.data());
    lane_scan_decode(r, tb, &d, sr, o);
    std::fill(clean.begin(), clean.end(), 0);
  }
  uint32_t nac, ndc, al_dc;
  uint64_t al_ac, band_ac[kMaxComp];
  lane_pack(lp, &nac, &al_ac, band_ac, &ndc, &al_dc);
  for (int c = 0; c < d.ncomp; ++c) {
    const int64_t b0 = d.comp[c].coef_off / 128, nb = (int64_t)d.comp[c].bw * d.comp[c].bh;
    for (int64_t b = b0; b < b0 + nb; ++b)
      lane_apply_block(coef.data() + b * 64, side.data() + b * kLSideBytes, c, nac, al_ac, band_ac, ndc, al_dc);
  }
  if (stats) {
    stats[0] = d.n_scans;
    stats[1] = lp.ndc;
  }
  if (cap) {
    cap->desc = d;
    cap->coef = coef;
  }
  return model_idct_color(d, coef, out_rgb, cap);
}

inline int host_model_decode(const uint8_t* p, int64_t len, int mode, int lanes, uint8_t* out_rgb, int32_t* stats,
                             StageCapture* cap = nullptr) {
  ImgDesc d;
  if (parse_jpeg(p, len, 1 << 16, &d) != DINO_IMG_OK) return d.status;
  if (d.kind == 2) {
    memcpy(out_rgb, p + 16, (size_t)d.width * d.height * 3);
    return DINO_IMG_OK;
  }
  if (d.kind == 1 && mode == 4) return host_model_decode_lane(p, len, d, out_rgb, stats, cap);
  if (d.kind == 1) return host_model_decode_multiscan(p, len, d, out_rgb, stats, cap);
  Destuffed ds = model_destuff(p + d.scan_off, d.scan_len);
  if (cap) {
    cap->desc = d;
    cap->ent.assign(ds.bytes.begin(), ds.bytes.begin() + ds.len);
  }
  if (!ds.terminated) return DINO_IMG_TRUNCATED;
  if (d.restart_interval > 0 && ((int)ds.rst.size() < d.n_rst_max - 1 || ds.rst_bad)) {
    d.kind = 1;  // k_htab: resync semantics on the coefficient-buffer path
    return host_model_decode_multiscan(p, len, d, out_rgb, stats, cap);
  }
  HuffTables tabs;
  HuffImage im;
  if (!model_tables(p, d, &tabs, im)) return DINO_IMG_CORRUPT;
  std::vector<int16_t> coef(d.coef_bytes / 2, 0);
  CoefSink sink;
  sink.d = &d;
  sink.coef = coef.data();
  BitReader br{(const uint32_t*)ds.bytes.data(), (uint32_t)ds.len};
  // mode 2: the stream as k_huffman stages it in LDS (big-endian-swapped words + zero pad)
  std::vector<uint32_t> win((ds.len + 64 + 3) / 4, 0u);
  for (size_t i = 0; i < win.size(); ++i) win[i] = br_word(br, (uint32_t)i);
  if (d.restart_interval > 0) {
    int nseg = d.n_rst_max;
    if ((int)ds.rst.size() < nseg - 1) return DINO_IMG_BADDATA;
    int per = d.restart_interval * d.blocks_per_mcu;
    for (int k = 0; k < nseg; ++k) {
      uint32_t start = k == 0 ? 0 : (uint32_t)ds.rst[k - 1] * 8;
      BitReader sb{br.words, k + 1 < nseg ? (uint32_t)ds.rst[k] : (uint32_t)ds.len};
      int32_t pred[kMaxComp] = {0, 0, 0};
      int first = k * per, last = std::min(first + per, d.total_blocks);
      if (mode == 2) {  // segments read from the staged (swapped) words, as k_huffman's LDS window
        BitReader sw{win.data(), k + 1 < nseg ? (uint32_t)ds.rst[k] : (uint32_t)ds.len};
        decode_write<true>(sw, im, HState{start, 0, 0}, 0xFFFFFFFFu, first, last, pred, sw.nbytes * 8u, sink);
      } else {
        decode_write<false>(sb, im, HState{start, 0, 0}, 0xFFFFFFFFu, first, last, pred, sb.nbytes * 8u, sink);
      }
    }
  } else if (mode == 0) {
    int32_t pred[kMaxComp] = {0, 0, 0};
    decode_write<false>(br, im, HState{0, 0, 0}, 0xFFFFFFFFu, 0, d.total_blocks, pred, br.nbytes * 8u, sink);
  } else {
    std::vector<int32_t> dcd(d.total_blocks, 0);
    if (mode == 2) {
      BitReader bw{win.data(), (uint32_t)win.size() * 4};
      model_huffman_spec<true>(bw, im, d, (uint32_t)ds.len * 8, lanes, 0, sink, dcd.data(), stats);
    } else {
      model_huffman_spec<kHuffSrc>(br, im, d, (uint32_t)ds.len * 8, lanes, mode == 3 ? 16 : 0, sink, dcd.data(),
                                stats);
    }
  }
  if (cap) cap->coef = coef;
  return model_idct_color(d, coef, out_rgb, cap);
}

// k_idct + k_color of the decode model (dense coefficients).
inline int model_idct_color(const ImgDesc& d, const std::vector<int16_t>& coef, uint8_t* out_rgb, StageCapture* cap) {
  // k_idct
  std::vector<uint8_t> planes;
  int64_t psz = 0;
  for (int c = 0; c < d.ncomp; ++c) psz += (int64_t)d.comp[c].bw * d.comp[c].bh * 64;
  planes.resize(psz);
  for (int c = 0; c < d.ncomp; ++c) {
    const CompDesc& cd = d.comp[c];
    int pitch = cd.bw * 8;
    for (int by = 0; by < cd.bh; ++by)
      for (int bx = 0; bx < cd.bw; ++bx)
        idct_block(coef.data() + cd.coef_off / 2 + ((int64_t)by * cd.bw + bx) * 64, d.qt[cd.tq],
                   planes.data() + cd.plane_off + (int64_t)by * 8 * pitch + bx * 8, pitch);
  }
  if (cap) cap->planes = planes;
  // k_color
  PlaneView pv[kMaxComp];
  for (int c = 0; c < d.ncomp; ++c) {
    const CompDesc& cd = d.comp[c];
    pv[c].p = planes.data() + cd.plane_off;
    pv[c].pitch = cd.bw * 8;
    pv[c].dw = cd.dw;
    pv[c].dh = cd.dh;
    pv[c].hf = d.max_h / cd.h;
    pv[c].vf = d.max_v / cd.v;
    pv[c].method = upsample_method(pv[c].hf, pv[c].vf, cd.dw);
  }
  for (int y = 0; y < d.height; ++y)
    for (int x = 0; x < d.width; ++x) {
      uint8_t* o = out_rgb + ((int64_t)y * d.width + x) * 3;
      if (d.ncomp == 1) {
        o[0] = o[1] = o[2] = (uint8_t)upsample_at(pv[0], x, y);
      } else {
        int a = upsample_at(pv[0], x, y), b = upsample_at(pv[1], x, y), c = upsample_at(pv[2], x, y);
        if (d.color == kYCbCr) {
          ycc_to_rgb(a, b, c, o);
        } else {
          o[0] = (uint8_t)a;
          o[1] = (uint8_t)b;
          o[2] = (uint8_t)c;
        }
      }
    }
  return DINO_IMG_OK;
}

// ---- k_rcoeffs + k_hresize + k_augment for one view ---------------------------
struct ViewModel {
  std::vector<int32_t> hb, ht, vb, vt;
  int kh = 0, kv = 0;
  std::vector<uint8_t> tmp;  // horizontal pass output, crop_h x S x 3
};

inline void model_coeffs(int in_size, int S, std::vector<int32_t>& b, std::vector<int32_t>& t, int& k) {
  k = resample_ksize(in_size, S);
  b.assign(2 * S, 0);
  t.assign((size_t)S * k, 0);
  for (int x = 0; x < S; ++x) resample_coeffs_one(in_size, S, x, k, &b[2 * x], &b[2 * x + 1], &t[(size_t)x * k]);
}

// Resized + flipped crop, planar u8 [3][S][S].
inline void model_resize_planar(const uint8_t* rgb, int W, int H, const dino_view_params& p, uint8_t* planes) {
  const int S = p.out_size;
  const bool need_h = p.crop_w != S, need_v = p.crop_h != S;
  SrcView src{rgb + ((int64_t)p.crop_top * W + p.crop_left) * 3, (int64_t)W * 3, 3, 1};
  ViewModel vm;
  if (need_h) {
    model_coeffs(p.crop_w, S, vm.hb, vm.ht, vm.kh);
    CoefView cv{vm.hb.data(), vm.ht.data(), vm.kh};
    vm.tmp.assign((size_t)p.crop_h * S * 3, 0);
    for (int r = 0; r < p.crop_h; ++r)
      for (int x = 0; x < S; ++x)
        for (int ch = 0; ch < 3; ++ch)
          vm.tmp[(size_t)ch * p.crop_h * S + (size_t)r * S + x] = hresize_at(src, cv, r, x, ch);
    src = SrcView{vm.tmp.data(), (int64_t)S, 1, (int64_t)p.crop_h * S};  // planar, as k_hresize writes it
  }
  if (need_v) model_coeffs(p.crop_h, S, vm.vb, vm.vt, vm.kv);
  CoefView cvv{vm.vb.data(), vm.vt.data(), vm.kv};
  for (int y = 0; y < S; ++y)
    for (int x = 0; x < S; ++x) {
      int xo = p.flip ? S - 1 - x : x;
      for (int ch = 0; ch < 3; ++ch) {
        uint8_t v = need_v ? vresize_at(src, cvv, y, x, ch)
                           : src.base[(int64_t)y * src.pitch + (int64_t)x * src.px + ch * src.cs];
        planes[(size_t)ch * S * S + (size_t)y * S + xo] = v;
      }
    }
}

inline int host_model_resized_crop(const uint8_t* rgb, int W, int H, const dino_view_params& p, uint8_t* out_hwc) {
  const int S = p.out_size;
  std::vector<uint8_t> pl((size_t)3 * S * S);
  model_resize_planar(rgb, W, H, p, pl.data());
  for (int i = 0; i < S * S; ++i)
    for (int ch = 0; ch < 3; ++ch) out_hwc[(size_t)i * 3 + ch] = pl[(size_t)ch * S * S + i];
  return 0;
}

inline int host_model_augment(const uint8_t* rgb, int W, int H, const dino_view_params& p, const float* mean,
                              const float* stdv, int out_dtype, void* out) {
  const int S = p.out_size;
  const int64_t N = (int64_t)S * S;
  std::vector<uint8_t> pl((size_t)3 * N);
  model_resize_planar(rgb, W, H, p, pl.data());
  uint8_t *R = pl.data(), *G = R + N, *B = G + N;
  JitterPlan jp = make_jitter_plan(p);
  int hd = hue_delta(p.hue);
  uint64_t lsum = 0;
  for (int64_t i = 0; i < N; ++i) {  // pass A: ops before contrast + L sum
    int r = R[i], g = G[i], b = B[i];
    jitter_stage0(jp, r, g, b, p, hd);
    R[i] = (uint8_t)r;
    G[i] = (uint8_t)g;
    B[i] = (uint8_t)b;
    lsum += (uint64_t)rgb_to_l(r, g, b);
  }
  int cmean = contrast_mean_from_sum(lsum, N);
  for (int64_t i = 0; i < N; ++i) {  // pass B: contrast, later ops, grayscale
    int r = R[i], g = G[i], b = B[i];
    jitter_stage1(jp, r, g, b, p, cmean, hd);
    R[i] = (uint8_t)r;
    G[i] = (uint8_t)g;
    B[i] = (uint8_t)b;
  }
  float k1[16], k2[256];
  int ks = p.ksize;
  if (p.blur) {
    gaussian_kernel1d(ks, p.sigma, k1);
    for (int a = 0; a < ks; ++a)
      for (int b = 0; b < ks; ++b) k2[a * ks + b] = k1[a] * k1[b];
  }
  for (int ch = 0; ch < 3; ++ch)
    for (int y = 0; y < S; ++y)
      for (int x = 0; x < S; ++x) {
        const uint8_t* plane = pl.data() + (size_t)ch * N;
        int v = p.blur ? blur_at(plane, S, y, x, k2, ks) : plane[(size_t)y * S + x];
        if (p.solarize) v = solarize_u8(v);
        float f = u8_normalize(v, mean[ch], stdv[ch]);
        size_t o = (size_t)ch * N + (size_t)y * S + x;
        if (out_dtype == DINO_OUT_BF16) ((uint16_t*)out)[o] = f32_to_bf16(f);
        else if (out_dtype == DINO_OUT_FP32) ((float*)out)[o] = f;
        else ((uint8_t*)out)[o] = f32_to_fp8e4m3(bf16_to_f32(f32_to_bf16(f)));
      }
  return 0;
}

}  // namespace dino
