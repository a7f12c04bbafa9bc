// plan.hpp — workspace planning shared by k_plan / k_vplan (device) and the host
// probe dino_probe (capi.hip), so that the host computes exactly the bytes the
// kernels will ask for and can grow the workspaces before launching a batch.
#pragma once

#include "kernels.hpp"
#include "progressive.hpp"
#include "pscan.hpp"
#include "lscan.hpp"
#include "resize.hpp"

namespace dino {

// Per-lane state of the speculative decode (global, k_huff1 -> k_huff2 -> k_huff3).
struct LaneRec {
  HState S;       // start state used by the lane's current decode
  RangeOut R;     // its result
  RangeOut R1;    // result of the first (guessed-state) decode, for checkpoint syncs
  int32_t ncp;    // checkpoints recorded by the first decode
  int32_t blk0;   // first block the lane emits (k_huff2 scan)
  HState W;       // k_huff2 scratch: wanted start state
  int32_t pad;
};
static_assert(sizeof(LaneRec) == 68, "LaneRec layout");

// Lanes reserved for the speculative Huffman decode (restart images decode per interval).
DHD int32_t huff_lanes_cap(const ImgDesc& d) {
  if (d.restart_interval > 0 || d.kind != 0) return 0;
  const int64_t nbits = ((int64_t)d.scan_len + 64) * 8;  // >= the destuffed stream
  const int64_t seg = nbits <= kHuffSegBits ? 1 : (nbits + kHuffSegBits - 1) / kHuffSegBits;
  return (int32_t)(seg * kHuffThreads);
}

// Sparse entry capacity per block (see SparseSink): 63 u32 entries + 1 alignment halfword.
constexpr int kEntHalfwordsPerBlock = 128;

// Byte sizes of an image's workspace regions, in chunk order: destuffed entropy
// bytes, restart offsets, coefficients (baseline: sparse entries, 128 halfwords of
// capacity per block, see SparseSink; kind 1: the dense int16 buffer), block info
// (uint2 per block), component planes, RGB, speculative checkpoints, Huffman
// tables, lane records, destuff part counts.
struct ChunkSizes {
  int64_t ent, rst, coef, binfo, plane, rgb, cps, htab, hlane, dspart, tail;
  DHD int64_t sum() const { return ent + rst + coef + binfo + plane + rgb + cps + htab + hlane + dspart; }
  DHD int64_t total() const { return sum() + tail; }
};

// Image areas start 256-byte aligned (tail pads each image), and so does the sparse entry
// area (rst pads ent + rst): a lane's entry region starts at a multiple of 256 bytes in
// memory too (SparseSink stores groups of up to 64 bytes aligned to their size).
DHD int64_t align256(int64_t x) { return (x + 255) & ~(int64_t)255; }
DHD ChunkSizes chunk_finish(ChunkSizes z) {
  z.tail = align256(z.sum()) - z.sum();
  return z;
}

// Destuff work items of an image: 32 KiB parts of its scan (>= 1, so that the
// descriptor is always completed by k_destuff_write); none for kinds 1 and 2.
constexpr int kDsPartBytes = 32 * 1024;
DHD int ds_parts(const ImgDesc& d) {
  if (d.status != DINO_IMG_OK || d.kind != 0) return 0;
  const int n = (d.scan_len + 16 + kDsPartBytes - 1) / kDsPartBytes;
  return n > 1 ? n : 1;
}

DHD ChunkSizes image_chunk_bytes(const ImgDesc& d) {
  ChunkSizes z{};
  if (d.status != DINO_IMG_OK) return z;
  z.rgb = align16((int64_t)d.width * d.height * 3 + 16);
  if (d.kind == 2) return chunk_finish(z);
  int64_t p = 0;
  for (int c = 0; c < d.ncomp; ++c) p += (int64_t)d.comp[c].bw * d.comp[c].bh * 64;
  z.plane = align16(p);
  if (d.kind == 1) {
    z.ent = align16((int64_t)d.scan_len + 64);  // each scan's destuffed bytes (k_pscan)
    z.coef = align16(d.coef_bytes);
    z.binfo = (d.coef_bytes / 128) * kLSideBytes;  // side records of the lane decoder (lscan.hpp)
    z.htab = kPRegionBytes;  // scan list + decoder tables (k_pwalk -> k_pscan)
    return chunk_finish(z);
  }
  z.ent = align16((int64_t)d.scan_len + 64);
  z.rst = align256(z.ent + 4 * ((int64_t)d.n_rst_max + 1)) - z.ent;
  z.coef = (int64_t)d.total_blocks * kEntHalfwordsPerBlock * 2;
  z.binfo = align16((int64_t)d.total_blocks * 8);
  const int64_t lanes = huff_lanes_cap(d);
  z.cps = lanes * kHuffCheckpoints * (int64_t)sizeof(Checkpoint);
  z.htab = align16((int64_t)sizeof(HuffTables));
  z.hlane = align16(lanes * (int64_t)sizeof(LaneRec));
  z.dspart = 16 * (int64_t)ds_parts(d);
  return chunk_finish(z);
}

// A restart image that k_htab moves to the coefficient-buffer path keeps its baseline
// table area: its one scan needs at most 4 DC + 4 AC tables there.
static_assert(((int64_t)sizeof(HuffTables) - kPTabOff) / (int64_t)sizeof(PTab) >= 8, "switched restart images");

// Horizontal taps in the signed-dot4 layout (k_hresize): per output x an int4
// {xmin, groups, corr, 0}, then groups of 4 taps as signed base-256 digit planes.
DHD int64_t hdot_table_bytes(int S, int kh) { return kh ? (int64_t)S * 16 * (1 + (kh + 3) / 4) : 0; }

// Augment scratch of one view: horizontal-pass rows + resize coefficient tables.
DHD int64_t view_scratch_bytes(int S, int crop_w, int crop_h, int kh, int kv) {
  const int64_t htmp = kh ? align16((int64_t)crop_h * S * 3) : 0;
  return htmp + align16((int64_t)S * (4 + kh + kv) * 4) + hdot_table_bytes(S, kh);
}

// Upper bound of a view's scratch over every crop of a W x H image (crop sides <= the
// image's; the tap count grows with the crop side).
DHD int64_t view_scratch_bound(int S, int W, int H) {
  const int kh = resample_ksize(W > S ? W : S, S), kv = resample_ksize(H > S ? H : S, S);
  return view_scratch_bytes(S, W, H, kh, kv);
}

}  // namespace dino
