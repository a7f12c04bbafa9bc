// common.hpp — internal types shared by the host+device code of the ingest path.
//
// Every function in the *.hpp files of this directory is __host__ __device__:
// the HIP kernels (kernels.hip) call them per lane, and the test-only host
// emulator (tests/emu/emu.cpp) calls the very same code to check it against
// Pillow on the CPU.  Arithmetic that must match Pillow/libjpeg bit for bit is
// written without FMA contraction (the library is built with -ffp-contract=off).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/dino_ingest.h"

#define DHD __host__ __device__ __forceinline__

namespace dino {

constexpr int kMaxComp = 3;
constexpr int kMaxBlocksPerMcu = 10;   // libjpeg D_MAX_BLOCKS_IN_MCU
constexpr int kLookBits = 11;          // Huffman lookahead table bits

enum ColorSpace : int32_t { kGray = 0, kYCbCr = 1, kRGB = 2 };

struct CompDesc {
  int32_t id, h, v, tq, td, ta;
  int32_t bw, bh;        // coefficient block grid actually coded (incl. MCU padding)
  int32_t dw, dh;        // libjpeg downsampled_width / downsampled_height
  int64_t coef_off;      // byte offset of block (0,0) inside the image's coefficient area
  int64_t plane_off;     // byte offset of the sample plane (pitch bw*8) inside the plane area
};

// Per-image descriptor written by k_parse / k_plan, read by every later stage.
struct ImgDesc {
  int32_t status;
  int32_t width, height, ncomp, color;
  int32_t max_h, max_v;
  int32_t mcus_x, mcus_y, blocks_per_mcu;
  int32_t restart_interval;
  int32_t scan_off;        // entropy-coded data start, relative to the image's first byte
  int32_t scan_len;        // raw bytes from scan_off to the end of the image buffer
  int32_t n_rst_max;       // restart markers expected for a well-formed stream
  int32_t huff_off[8];     // DC 0-3, AC 0-3: offset of the 16 BITS bytes (HUFFVAL follows), -1 absent
  uint8_t mcu_comp[kMaxBlocksPerMcu];
  uint8_t mcu_bx[kMaxBlocksPerMcu];
  uint8_t mcu_by[kMaxBlocksPerMcu];
  uint8_t pad0[2];
  uint16_t qt[4][64];      // quant tables, natural order
  CompDesc comp[kMaxComp];
  int32_t total_blocks;    // MCUs * blocks_per_mcu
  // filled by k_plan (byte offsets into the ctx workspace)
  int64_t base;            // start of this image's chunk
  int64_t ent_off, rst_off, plane_off, rgb_off;
  int64_t coef_off;        // sparse AC entries (u32, 64 per block of capacity; k_huffman SparseSink)
  int64_t cps_off;         // k_huffman checkpoints (speculative decode), kHuffThreads x kHuffCheckpoints
  int64_t reserved0;
  int64_t binfo_off;       // uint2 per block (decode order): first sparse entry, (int16 DC << 16) | entry count
  int64_t coef_bytes;      // dense int16 coefficient bytes (host emulator layout)
  int64_t htab_off;        // Huffman decoder tables (6 x HuffTable), built once per image by k_htab
  int64_t hlane_off;       // per-lane records of the speculative decode (LaneRec x h_lanes_cap)
  int32_t h_lanes_cap;     // lanes reserved by k_plan (from the raw scan length)
  int32_t h_lanes;         // active lanes (restart images: restart intervals)
  int32_t h_sub;           // bits per lane range
  int32_t h_items;         // Huffman work items (kHuffThreads lanes each)
  int32_t h_item_base;     // first work item of the image in the batch (k_hseg)
  int32_t ds_items;        // destuff work items (32 KiB parts of the scan, k_plan)
  int32_t ds_item_base;    // first destuff work item of the image in the batch (k_plan)
  int32_t pad2;
  int64_t dspart_off;      // per-part counts of k_destuff_count (16 bytes per part)
  // filled by k_destuff
  int32_t ent_len;         // destuffed entropy bytes
  int32_t n_rst;           // RST markers found
  int32_t terminated;      // a terminating marker (EOI/other) was found
  int32_t rst_bad;         // an RST marker out of sequence (k_destuff_write)
  // decode path (k_parse): 0 baseline single scan (speculative Huffman kernels),
  // 1 coefficient buffer (progressive or multi-scan sequential, k_prog),
  // 2 pre-decoded RGB container (DINO_RAW_MAGIC, copied by k_color)
  int32_t kind;
  int32_t progressive;     // SOF2
  int32_t first_sos;       // the FF of the first SOS marker (image-relative; k_prog's walk starts there)
  int32_t n_scans;         // kind 1: scans (k_prog)
  int32_t qt_seen_mask;    // DQT slots defined before the first SOS
  int32_t aug_status;      // DINO_IMG_NO_SPACE when k_vplan could not place one of its views
};

// Bytes of resize-coefficient scratch reserved per view: bounds + int32 taps, both axes.
DHD int64_t rcoef_stride_bytes(int out_size, int max_dim) {
  // ksize = 2*ceil(support*scale)+1 with support 2 and scale <= max_dim/out
  int k = 2 * ((2 * max_dim + out_size - 1) / out_size) + 3;
  return (int64_t)2 * out_size * (k + 2) * 4;
}

DHD int ceil_div(int a, int b) { return (a + b - 1) / b; }

}  // namespace dino
