// kernels.hip — the gfx950 kernels of the DINO Stage-3 ingest path.
//
// Decode half (one JPEG per workgroup where the work is serial per image):
//   k_parse     1 lane / image      marker parse -> ImgDesc
//   k_plan      1 workgroup         per-image workspace offsets (prefix sum), capacity check
//   k_destuff   256 lanes / image   0xFF00 unstuffing + RSTn removal (block compaction)
//   k_htab .. k_huff3                self-synchronising speculative Huffman decode in
//                                   work items of 256 lanes (see the Huffman section)
//   k_idct      lanes over blocks   islow IDCT (int32 fast path, int64 exact fallback)
//   k_color     lanes over pixels   fancy upsampling + YCbCr->RGB
// Augment half (per view):
//   k_params    1 lane / view       Philox draw of the view record (optional)
//   k_vplan     1 workgroup         per-view scratch offsets
//   k_rcoeffs   lanes over outputs  Pillow bicubic coefficient tables (both axes)
//   k_hresize   lanes over pixels   horizontal pass (crop rows -> S columns, u8)
//   k_augment   1 workgroup / view  vertical pass -> LDS planes -> jitter -> gray
//                                   -> blur + solarize + normalize -> NCHW output
// Plus k_masks (iBOT) and k_bf16_to_fp8 (Stage 5).
#include "augment.hpp"
#include "color.hpp"
#include "huffman.hpp"
#include "idct.hpp"
#include "jpeg_parse.hpp"
#include "kernels.hpp"
#include "lscan.hpp"
#include "mask.hpp"
#include "plan.hpp"
#include "progressive.hpp"
#include "pscan.hpp"
#include "sampler.hpp"

#include <stdio.h>
#include <stdlib.h>

namespace dino {

// Workgroup coordinates of a (x, y = image, z) grid.  (An XCD-aware renumbering, each XCD
// owning whole images so that one image's workgroups share one L2, was measured and dropped:
// the per-image kernels' working sets are small against the 4 MiB L2s.)
struct BlkIdx {
  int x, y, z;
};
// Issue priority of the batch kernels' waves (s_setprio): above the progressive side
// decode's scan waves (k_pscan keeps the default 0), so that a SIMD running both issues the
// batch's instruction first when both are ready (measured: side route 95.6k -> 97.3k img/s).
__device__ __forceinline__ void main_prio() { __builtin_amdgcn_s_setprio(3); }
__device__ __forceinline__ BlkIdx xcd_blk() {
  main_prio();
  const uint32_t X = gridDim.x, Y = gridDim.y, Z = gridDim.z;
  uint32_t L = blockIdx.x + X * (blockIdx.y + Y * blockIdx.z);
  (void)Z;
  BlkIdx b;
  b.x = (int)(L % X);
  L /= X;
  b.y = (int)(L % Y);
  b.z = (int)(L / Y);
  return b;
}

// ---------------------------------------------------------------------------
// k_parse
// ---------------------------------------------------------------------------
// One wave per image: the wave copies the file's first kParsePrefix bytes into LDS with
// wide loads, then lane 0 walks the markers there (the walk is a chain of dependent byte
// reads: LDS latency instead of global latency).  The parse depends on the length only
// through bounds checks and scan_len = len - scan_off, so a walk that reaches SOS inside
// the prefix is the walk over the whole file with scan_len corrected; one that does not
// (a header longer than the prefix, a raw container) is redone on the global bytes.
constexpr int kParsePrefix = 4096;
__global__ void __launch_bounds__(64) k_parse(const uint8_t* __restrict__ bytes, const int64_t* __restrict__ offsets,
                                              const int64_t* __restrict__ lengths,
                                              const uint8_t* __restrict__ raw_mask, int B, int max_dim,
                                              ImgDesc* __restrict__ desc) {
  __shared__ __attribute__((aligned(16))) uint8_t s_raw[kParsePrefix + 16];
  const int i = blockIdx.x;
  const int64_t off = offsets[i], len = lengths ? lengths[i] : offsets[i + 1] - off;
  const int64_t n = len < kParsePrefix ? len : kParsePrefix;
  const uint8_t* src = bytes + off;
  // aligned 16-byte chunks from the chunk holding src (the copy starts `lead` bytes into
  // s_raw); a chunk that would pass the end of the caller's buffer is copied bytewise
  const int lead = (int)((uintptr_t)src & 15);
  const uint4* base = (const uint4*)(src - lead);
  const uint8_t* buf_end = bytes + offsets[B];
  const int nchunks = (int)((lead + n + 15) >> 4);
  for (int c = threadIdx.x; c < nchunks; c += 64) {
    if ((const uint8_t*)(base + c + 1) <= buf_end) {
      *(uint4*)(s_raw + 16 * c) = base[c];
    } else {
      for (int j = 0; j < 16; ++j) {
        const int64_t k = 16 * (int64_t)c + j - lead;
        if (k >= 0 && k < n) s_raw[16 * c + j] = src[k];
      }
    }
  }
  __syncthreads();
  const uint8_t* s_head = s_raw + lead;
  if (threadIdx.x != 0) return;
  ImgDesc d;
  if (len <= 0) {
    d.status = DINO_IMG_CORRUPT;
    d.width = d.height = d.ncomp = 0;
    d.kind = 0;
    d.aug_status = 0;
  } else {
    const bool raw = raw_mask != nullptr && raw_mask[i] != 0;
    parse_jpeg(s_head, n, max_dim, &d, raw);
    if (n < len) {
      if (d.status == DINO_IMG_OK && !raw) d.scan_len = (int32_t)(len - d.scan_off);
      else parse_jpeg(src, len, max_dim, &d, raw);
    }
  }
  desc[i] = d;
}

// ---------------------------------------------------------------------------
// k_plan: exclusive scan of per-image chunk sizes (single workgroup of 1024)
// ---------------------------------------------------------------------------
// Places the image at `base` (or marks it DINO_IMG_NO_SPACE).
__device__ void plan_place(ImgDesc& d, const ChunkSizes& z, int64_t base, int64_t ws_size) {
  const int64_t sz = z.total();
  if (sz == 0) return;
  if (base < 0 || base + sz > ws_size) {
    d.status = DINO_IMG_NO_SPACE;
    return;
  }
  d.base = base;
  d.ent_off = base;
  d.rst_off = d.ent_off + z.ent;
  d.coef_off = d.rst_off + z.rst;
  d.binfo_off = d.coef_off + z.coef;
  d.plane_off = d.binfo_off + z.binfo;
  d.rgb_off = d.plane_off + z.plane;
  d.cps_off = d.rgb_off + z.rgb;
  d.htab_off = d.cps_off + z.cps;
  d.hlane_off = d.htab_off + z.htab;
  d.dspart_off = d.hlane_off + z.hlane;
  d.h_lanes_cap = huff_lanes_cap(d);
}

// Exclusive scan of the images' chunk sizes.  When the batch does not fit the
// workspace, images are accepted greedily in batch order instead (one lane), so
// that an image that does not fit leaves its bytes to the later ones: only images
// that cannot be placed get DINO_IMG_NO_SPACE (the host probe, dino_probe, sizes
// the workspace so that this does not happen on the product path).
__global__ void __launch_bounds__(1024) k_plan(ImgDesc* __restrict__ desc, int B, int64_t ws_size,
                                              PCtl* __restrict__ pctl) {
  __shared__ int64_t part[1024];
  __shared__ int32_t dpart[1024];
  const int t = threadIdx.x;
  if (t == 0) {  // the batch's coefficient-buffer registry (k_pwalk, k_pscan, k_plscan)
    pctl->ticket = 0;
    pctl->nprog = 0;
    pctl->max_scans = 0;
    pctl->cap = (uint32_t)B;
    pctl->lticket = 0;
    pctl->nlane = 0;
    pctl->lmax_scans = 0;
  }
  const int per = (B + 1023) / 1024;
  int64_t local = 0;
  int32_t dlocal = 0;
  for (int k = 0; k < per; ++k) {
    int i = t * per + k;
    if (i < B) {
      local += image_chunk_bytes(desc[i]).total();
      dlocal += ds_parts(desc[i]);
    }
  }
  part[t] = local;
  dpart[t] = dlocal;
  __syncthreads();
  for (int s = 1; s < 1024; s <<= 1) {  // Hillis-Steele inclusive scans
    int64_t v = t >= s ? part[t - s] : 0;
    int32_t dv = t >= s ? dpart[t - s] : 0;
    __syncthreads();
    part[t] += v;
    dpart[t] += dv;
    __syncthreads();
  }
  const bool fits = part[1023] <= ws_size;
  int64_t base = part[t] - local;
  int32_t dbase = dpart[t] - dlocal;
  for (int k = 0; k < per; ++k) {
    int i = t * per + k;
    if (i >= B) continue;
    ImgDesc& d = desc[i];
    d.ds_item_base = dbase;
    d.ds_items = ds_parts(d);  // as counted by the scan above (the kernels skip images not OK)
    dbase += d.ds_items;
    const ChunkSizes z = image_chunk_bytes(d);
    if (fits) plan_place(d, z, base, ws_size);
    base += z.total();
  }
  if (!fits) {
    __syncthreads();
    if (t == 0) {
      int64_t b = 0;
      for (int i = 0; i < B; ++i) {
        ImgDesc& d = desc[i];
        const ChunkSizes z = image_chunk_bytes(d);
        const int64_t sz = z.total();
        if (sz == 0) continue;
        if (b + sz <= ws_size) {
          plan_place(d, z, b, ws_size);
          b += sz;
        } else {
          d.status = DINO_IMG_NO_SPACE;
        }
      }
    }
  }
}

// ---------------------------------------------------------------------------
// k_destuff: one workgroup (256 lanes) per image
// ---------------------------------------------------------------------------
constexpr int kDestuffThreads = 256;

__device__ __forceinline__ int classify_ff(const uint8_t* r, int n, int k) {
  // for r[k] == 0xFF: 0 keep (FF00), 1 RST, 2 fill (FFFF), 3 terminating marker, 4 truncated (last byte)
  if (k + 1 >= n) return 4;
  int nx = r[k + 1];
  if (nx == 0x00) return 0;
  if (nx >= 0xD0 && nx <= 0xD7) return 1;
  if (nx == 0xFF) return 2;
  return 3;
}

// One pass over the scan in tiles of 256 lanes x 16 bytes: each lane loads one
// aligned 16-byte chunk (plus the bytes either side for the 0xFF rules),
// classifies it, and the workgroup scans (kept bytes, RST markers) packed in one
// word to place the lane's output.  The first terminating marker ends the scan.
template <int NT>
__device__ __forceinline__ uint32_t block_excl_scan(uint32_t v, uint32_t* s_wave, uint32_t* total) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  uint32_t x = v;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const uint32_t y = __shfl_up(x, o);
    if (lane >= o) x += y;
  }
  if (lane == 63) s_wave[w] = x;
  __syncthreads();
  uint32_t before = 0, all = 0;
#pragma unroll
  for (int k = 0; k < NT / 64; ++k) {
    const uint32_t t = s_wave[k];
    before += k < w ? t : 0u;
    all += t;
  }
  __syncthreads();
  *total = all;
  return before + x - v;
}

// A lane's 16-byte chunk c of the scan, classified: bit j of keep = byte kept,
// of rstm = an RSTn marker starts there; term = scan index of the first
// terminating marker in the chunk (n if none).
struct DsChunk {
  uint32_t wv[4];
  uint32_t keep, rstm;
  int term;
};

__device__ __forceinline__ DsChunk ds_classify(const uint8_t* r, int n, const uint4* base, int lead, int nchunks,
                                               const uint8_t* buf_end, int c) {
  DsChunk o;
  o.wv[0] = o.wv[1] = o.wv[2] = o.wv[3] = 0u;
  o.keep = o.rstm = 0u;
  o.term = n;
  const int k0 = 16 * c - lead;  // scan index of byte 0 of this chunk
  int prevb = -1, nextb = -1;
  if (c >= nchunks) return o;
  if ((const uint8_t*)(base + c + 1) <= buf_end) {
    const uint4 u = base[c];
    o.wv[0] = u.x;
    o.wv[1] = u.y;
    o.wv[2] = u.z;
    o.wv[3] = u.w;
  } else {
#pragma unroll
    for (int j = 0; j < 16; ++j)
      if (k0 + j >= 0 && k0 + j < n) o.wv[j >> 2] |= (uint32_t)r[k0 + j] << (8 * (j & 3));
  }
  if (k0 - 1 >= 0 && k0 - 1 < n) prevb = r[k0 - 1];
  if (k0 + 16 >= 0 && k0 + 16 < n) nextb = r[k0 + 16];
  // branch-free per byte; the first terminating marker clips the chunk afterwards
  uint32_t termm = 0u;
#pragma unroll
  for (int j = 0; j < 16; ++j) {
    const int k = k0 + j;
    const bool valid = k >= 0 && k < n;
    const int v = (o.wv[j >> 2] >> (8 * (j & 3))) & 255;
    const int pv = j > 0 ? (int)((o.wv[(j - 1) >> 2] >> (8 * ((j - 1) & 3))) & 255) : prevb;
    const int nx = j < 15 ? (k + 1 < n ? (int)((o.wv[(j + 1) >> 2] >> (8 * ((j + 1) & 3))) & 255) : -1) : nextb;
    // for 0xFF: 0 keep (FF00), 1 RST, 2 fill (FFFF), 3 terminating marker, 4 truncated (last byte)
    const int cls = nx < 0 ? 4 : (nx == 0x00 ? 0 : ((nx >= 0xD0 && nx <= 0xD7) ? 1 : (nx == 0xFF ? 2 : 3)));
    const bool ff = v == 0xFF;
    const bool kept = ff ? cls == 0 : !(k > 0 && pv == 0xFF);
    o.keep |= (uint32_t)(valid && kept) << j;
    o.rstm |= (uint32_t)(valid && ff && cls == 1) << j;
    termm |= (uint32_t)(valid && ff && cls >= 3) << j;
  }
  if (termm) {
    const int f = __ffs(termm) - 1;
    const uint32_t low = (1u << f) - 1u;
    o.keep &= low;
    o.rstm &= low;
    o.term = k0 + f;
  }
  return o;
}

// Drop a chunk's bytes at or after scan index E.
__device__ __forceinline__ void ds_clip(DsChunk& ch, int k0, int E) {
  const int lim = E - k0;
  const uint32_t mask = lim <= 0 ? 0u : (lim >= 16 ? 0xFFFFu : ((1u << lim) - 1u));
  ch.keep &= mask;
  ch.rstm &= mask;
}

// Geometry of an image's scan in 16-byte chunks (aligned loads; chunk c covers
// scan bytes [16c - lead, 16c - lead + 16)) and parts of kDsPartChunks chunks.
constexpr int kDsTiles = 8;
constexpr int kDsPartChunks = kDestuffThreads * kDsTiles;  // 32 KiB of scan per work item
struct DsGeom {
  const uint8_t* r;
  int n, lead, nchunks;
  const uint4* base;
  const uint8_t* buf_end;
};

__device__ __forceinline__ DsGeom ds_geom(const uint8_t* bytes, const int64_t* offsets, int B, const ImgDesc& d,
                                          int img) {
  DsGeom g;
  g.r = bytes + offsets[img] + d.scan_off;
  g.n = d.scan_len;
  g.lead = (int)((uintptr_t)g.r & 15);
  g.base = (const uint4*)(g.r - g.lead);
  g.nchunks = (g.lead + g.n + 15) >> 4;
  g.buf_end = bytes + offsets[B];  // a whole-chunk load must not pass the caller's buffer
  return g;
}

// Work item -> (image, part) over desc[].ds_item_base (k_plan); -1 past the end.
__device__ int ds_item_image(const ImgDesc* desc, int B, int item) {
  const ImgDesc& last = desc[B - 1];
  if (item >= last.ds_item_base + last.ds_items) return -1;
  int lo = 0, hi = B - 1;
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (desc[mid].ds_item_base <= item) lo = mid;
    else hi = mid - 1;
  }
  while (lo > 0 && desc[lo].ds_items == 0) --lo;
  return lo;
}

// Per-part results of k_destuff_count: kept bytes, RST markers, first terminator.
struct DsPart {
  int32_t kept, nrst, term, pad;
};

// k_destuff_count: persistent over (image, part) items; counts the part's kept
// bytes and RST markers and finds its first terminating marker.
__global__ void __launch_bounds__(kDestuffThreads) k_destuff_count(const uint8_t* __restrict__ bytes,
                                                                   const int64_t* __restrict__ offsets, int B,
                                                                   const ImgDesc* __restrict__ desc,
                                                                   uint8_t* __restrict__ ws) {
  main_prio();
  __shared__ uint32_t s_wave[kDestuffThreads / 64];
  __shared__ int s_img;
  __shared__ int s_term;
  const int t = threadIdx.x;
  for (int item = blockIdx.x;; item += gridDim.x) {
    if (t == 0) {
      s_img = ds_item_image(desc, B, item);
      s_term = 0x7FFFFFFF;
    }
    __syncthreads();
    const int img = s_img;
    if (img < 0) return;
    const ImgDesc& d = desc[img];
    if (d.status != DINO_IMG_OK) {
      __syncthreads();
      continue;
    }
    const DsGeom g = ds_geom(bytes, offsets, B, d, img);
    const int part = item - d.ds_item_base;
    uint32_t kept = 0, nrst = 0;
    int term = g.n;
#pragma unroll 1
    for (int tile = 0; tile < kDsTiles; ++tile) {
      const int c = part * kDsPartChunks + tile * kDestuffThreads + t;
      DsChunk ch = ds_classify(g.r, g.n, g.base, g.lead, g.nchunks, g.buf_end, c);
      if (ch.term < g.n) ds_clip(ch, 16 * c - g.lead, ch.term);
      term = min(term, ch.term);
      kept += __popc(ch.keep);
      nrst += __popc(ch.rstm);
    }
    if (term < g.n) atomicMin(&s_term, term);
    uint32_t tot;
    (void)block_excl_scan<kDestuffThreads>(kept | (nrst << 16), s_wave, &tot);  // nrst per part < 65536
    if (t == 0) {
      // bytes after the part's own first terminator were not counted past it in each
      // lane, but a later lane of the same part may have counted bytes after an earlier
      // lane's terminator: k_destuff_write recounts exactly; here only the totals of parts
      // wholly before the image's first terminator are used
      DsPart* dp = (DsPart*)(ws + d.dspart_off) + part;
      dp->kept = (int32_t)(tot & 0xFFFFu) + (int32_t)0;
      dp->nrst = (int32_t)(tot >> 16);
      dp->term = s_term == 0x7FFFFFFF ? g.n : s_term;
      dp->pad = 0;
    }
    __syncthreads();
  }
}

// k_destuff_write: persistent over the same items.  The part's output offset is
// the kept bytes of the image's earlier parts (all before the first terminator E);
// bytes at or after E are dropped; the part holding E (or the image's last part)
// zero-pads the stream and fills the descriptor.
__global__ void __launch_bounds__(kDestuffThreads) k_destuff_write(const uint8_t* __restrict__ bytes,
                                                                   const int64_t* __restrict__ offsets, int B,
                                                                   ImgDesc* __restrict__ desc,
                                                                   uint8_t* __restrict__ ws) {
  main_prio();
  __shared__ uint32_t s_wave[kDestuffThreads / 64];
  __shared__ int s_img;
  __shared__ int s_E;
  __shared__ uint32_t s_o0, s_r0;
  __shared__ __attribute__((aligned(16))) uint8_t s_buf[kDestuffThreads * 16 + 16];  // a tile's output + alignment
  const int t = threadIdx.x;
  for (int item = blockIdx.x;; item += gridDim.x) {
    if (t == 0) s_img = ds_item_image(desc, B, item);
    __syncthreads();
    const int img = s_img;
    if (img < 0) return;
    ImgDesc* d = &desc[img];
    if (d->status != DINO_IMG_OK) {
      __syncthreads();
      continue;
    }
    const DsGeom g = ds_geom(bytes, offsets, B, *d, img);
    const int part = item - d->ds_item_base;
    const DsPart* dp = (const DsPart*)(ws + d->dspart_off);
    if (t == 0) {  // first terminator of the image, output offset of this part
      int E = g.n;
      uint32_t o0 = 0, r0 = 0;
      for (int p = 0; p < d->ds_items; ++p) {
        if (p < part && E == g.n) {
          o0 += (uint32_t)dp[p].kept;
          r0 += (uint32_t)dp[p].nrst;
        }
        if (dp[p].term < g.n) {
          E = dp[p].term;
          break;
        }
      }
      s_E = E;
      s_o0 = o0;
      s_r0 = r0;
    }
    __syncthreads();
    const int E = s_E;
    const int part_k0 = part * kDsPartChunks * 16 - g.lead;
    if (part_k0 < E || (part == 0)) {
      uint8_t* out = ws + d->ent_off;
      int32_t* rst = (int32_t*)(ws + d->rst_off);
      const int nrst_cap = d->n_rst_max + 1;
      uint32_t o_run = s_o0, rc_run = s_r0;
#pragma unroll 1
      for (int tile = 0; tile < kDsTiles; ++tile) {
        const int c = part * kDsPartChunks + tile * kDestuffThreads + t;
        DsChunk ch = ds_classify(g.r, g.n, g.base, g.lead, g.nchunks, g.buf_end, c);
        if (E < g.n) ds_clip(ch, 16 * c - g.lead, E);
        uint32_t tot;
        const uint32_t ex = block_excl_scan<kDestuffThreads>((uint32_t)__popc(ch.keep) | ((uint32_t)__popc(ch.rstm) << 16),
                                                             s_wave, &tot);
        // the tile's kept bytes are compacted in LDS (byte j of the lane at its rank among
        // the lane's kept bytes), then stored as aligned words: per-byte global stores in a
        // loop over the kept bits would run 16 trips in every wave
        const uint32_t lead = o_run & 3u, lo = lead + (ex & 0xFFFFu);
#pragma unroll
        for (int j = 0; j < 16; ++j)
          if (ch.keep & (1u << j))
            s_buf[lo + __popc(ch.keep & ((1u << j) - 1u))] = (uint8_t)((ch.wv[j >> 2] >> (8 * (j & 3))) & 255);
        if (ch.rstm) {  // restart markers: their output offsets and sequence check
          uint32_t ro = rc_run + (ex >> 16);
          for (uint32_t m = ch.rstm; m; m &= m - 1) {
            const int j = __ffs(m) - 1;
            const uint32_t o = o_run + (ex & 0xFFFFu) + __popc(ch.keep & ((1u << j) - 1u));
            if ((int)ro < nrst_cap) rst[ro] = (int32_t)o;
            // RSTn must count 0..7 in order; otherwise libjpeg's read_restart_marker
            // resyncs (jdmarker.c jpeg_resync_to_restart), which k_prog restates
            if ((g.r[16 * c - g.lead + j + 1] & 7u) != (ro & 7u)) atomicOr(&d->rst_bad, 1);
            ++ro;
          }
        }
        __syncthreads();
        {
          const uint32_t n = tot & 0xFFFFu, nw = (lead + n + 3) >> 2;
          uint32_t* ow = (uint32_t*)(out + (o_run - lead));  // 4-byte aligned (ent_off is 16-aligned)
          for (uint32_t w = t; w < nw; w += kDestuffThreads) {
            const uint32_t b0 = 4 * w, b1 = b0 + 4;  // LDS bytes [b0, b1) = output bytes o_run - lead + b0 ...
            const uint32_t v = *(const uint32_t*)(s_buf + b0);
            if (b0 >= lead && b1 <= lead + n) {
              ow[w] = v;
            } else {  // a word shared with the previous or the next tile: its own bytes only
              for (uint32_t k = b0; k < b1; ++k)
                if (k >= lead && k < lead + n) out[o_run - lead + k] = (uint8_t)(v >> (8 * (k - b0)));
            }
          }
        }
        __syncthreads();
        o_run += tot & 0xFFFFu;
        rc_run += tot >> 16;
      }
      // the part that ends the stream: holds E, or is the image's last part
      const int part_k1 = part_k0 + kDsPartChunks * 16;
      const bool last = (E < g.n) ? (E >= part_k0 && E < part_k1) : (part == d->ds_items - 1);
      if (last) {
        const int total = (int)o_run;
        for (int k = total + t; k < total + 64 && k < g.n + 64; k += kDestuffThreads) out[k] = 0;
        if (t == 0) {
          const int term = (E < g.n) && (E + 1 < g.n);  // a marker (not a trailing lone 0xFF) ended the scan
          d->ent_len = total;
          d->n_rst = (int32_t)rc_run;
          d->terminated = term;
          if (!term) {
            d->status = DINO_IMG_TRUNCATED;
          }
        }
      }
    }
    __syncthreads();
  }
}

// ---------------------------------------------------------------------------
// Huffman stage: self-synchronising speculative decode, split in work items of
// kHuffThreads lanes so that a large image spreads over many workgroups.
//
// An image's destuffed stream (nbits) is cut into lane ranges of `h_sub` bits;
// kHuffThreads consecutive ranges form one work item (a "segment").  Segments
// target kHuffSegBits bits, so work per workgroup is about the same for a
// 640x480 and a 1600x2133 image, and a batch of mixed sizes balances over the
// chip instead of waiting on its largest image.
//   k_htab   1 WG / image   decoder tables -> global (once per image), segment plan
//   k_hseg   1 WG           exclusive scan of work items over the batch
//   k_huff1  persistent     per segment: first decode of every range from a guessed
//                           state (block-in-MCU 0, zigzag 0) recording checkpoints,
//                           then sync rounds inside the segment (lane 0's guess kept)
//   k_huff2  1 WG / image   sync rounds across the whole image (fixes each segment's
//                           first lane and anything it cascades into), then the
//                           exclusive scan of block counts -> each lane's first block
//   k_huff3  persistent     per segment: each lane re-decodes its range from its true
//                           state and appends its blocks (SparseSink); images with
//                           restart intervals decode one interval per lane here
// ---------------------------------------------------------------------------
constexpr int kMinSubBits = 1024;  // shortest lane range of a one-segment image


// Work items (segments) an image needs for a stream of `nbits` bits, and the
// lanes reserved for it at plan time (from the raw scan length, >= the destuffed one).
__device__ __forceinline__ int huff_segments(int64_t nbits) {
  return nbits <= kHuffSegBits ? 1 : (int)((nbits + kHuffSegBits - 1) / kHuffSegBits);
}

// Entry words a lane buffers in LDS before it stores them as one aligned group: 32-byte
// groups in k_huff1 (its buffers borrow the skip tables' LDS), 64-byte groups in k_huff3.
// Word w of lane t sits at [w][t], so the lanes' halfword writes never share a bank.
// (Measured and dropped, DESIGN.md §5: a register shift register instead of LDS, block
// records buffered and stored in pairs or groups, 64-byte groups in k_huff1.)
constexpr int kSinkLds = 8;
constexpr int kSinkLds3 = 8;  // (16: 64-byte groups, but 47 KiB of LDS per item with the pair lookaheads: slower)

// k_huff1's tables in LDS: a HuffTables up to its lookaheads (the derived tables), then
// one region that holds the skip entries and the lanes' range results R during the
// state-only decodes and the value lookaheads + the SparseSink buffers (kSinkLds words per
// lane) during the write pass of a single-segment image (loaded over the skip entries
// once the rounds are done and R is read; the next item reloads its skip entries).
// 39 KiB in all: 4 items per CU.
constexpr int kHuffLookOff = (int)offsetof(HuffTables, ac_look);
constexpr int kHuffSinkOff = kHuffLookOff + kHuffLookBytes;
constexpr int kHuffROff = kHuffLookOff + (int)sizeof(HuffSkip);
constexpr int kHuffSkipPhaseBytes = (int)sizeof(HuffSkip) + (int)sizeof(RangeOut) * kHuffThreads;
constexpr int kHuffWritePhaseBytes = kHuffLookBytes + kSinkLds * 4 * kHuffThreads;
constexpr int kHuff1TabBytes =
    kHuffLookOff + (kHuffSkipPhaseBytes > kHuffWritePhaseBytes ? kHuffSkipPhaseBytes : kHuffWritePhaseBytes);
struct HuffLds {     // k_huff1
  ImgDesc sd;
  alignas(16) uint8_t tab[kHuff1TabBytes];
  uint32_t wave[kHuffThreads / 64];
  int32_t img, item;
};
static_assert(sizeof(HuffLds) <= 40 * 1024, "4 k_huff1 items per CU");
// k_huff3 writes coefficients (huff_step): the skip entries stay in global memory
constexpr int kHuffTabBytesNoSkip = (int)offsetof(HuffTables, skip);
static_assert(kHuffTabBytesNoSkip % 16 == 0, "HuffTables::skip is 16-byte aligned");
struct HuffLds3 {    // k_huff3 (no lane exchange)
  ImgDesc sd;
  alignas(16) uint8_t tab[kHuffTabBytesNoSkip];  // a HuffTables without its skip member
  int32_t img, item;
  uint32_t sink[kSinkLds3 * kHuffThreads];  // SparseSink buffers
};

static_assert(sizeof(ImgDesc) % 16 == 8 || sizeof(ImgDesc) % 16 == 0, "ImgDesc layout");
constexpr int kHuffLdsBytes = (int)((sizeof(HuffLds) + 15) & ~(size_t)15);
constexpr int kHuff3LdsBytes = (int)((sizeof(HuffLds3) + 15) & ~(size_t)15);

// Block record flag: the DC field is an absolute value (k_dcscan keeps it).
constexpr uint32_t kBinfoAbsDc = 1u << 15;

// Sparse coefficient output.  A lane appends its blocks' non-zero AC coefficients
// to a private region of the image's entry area that starts at 128 halfwords per
// block before its first block (a block needs at most 127, so regions never
// overlap), buffered in LDS (W words per lane) and stored as aligned W-word groups, so
// that each lane writes whole contiguous lines instead of scattered 2-byte coefficients
// into a dense block.  A coefficient takes one halfword, zigzag index | (int10 value << 6),
// while its value fits 10 bits; from the block's first coefficient that does not,
// the rest of the block is written as u32 entries (zigzag | int16 value << 16) at the
// next even halfword.  binfo[b] = {first halfword, n16 | n32 << 7 | (int16 DC << 16)}:
// one 8-byte record per block carries the DC too (a difference until k_dcscan sums
// it in place; absolute with restart intervals).  k_idct scatters the entries into
// its LDS block.
template <int W>  // entry words buffered per lane in LDS
struct SparseSinkT {
  static_assert(W % 4 == 0 && W > 0, "whole 16-byte chunks");
  uint32_t* ent;   // image entry area
  uint2* binfo;    // image block info
  uint32_t n;      // halfwords in stored groups (relative to the image entry area), multiple of 2 W
  uint32_t k;      // halfwords buffered in LDS
  uint32_t bstart, dcw, n16, n32;
  bool wide;       // the open block has switched to u32 entries
  int32_t b;
  uint32_t* lb;    // this lane's buffer column in LDS (word w at lb[w * kHuffThreads])
  __device__ void lds_flush(uint32_t words) {  // the buffer's first `words` words -> entries at n
    uint4* dst = (uint4*)(ent + (n >> 1));
#pragma unroll
    for (int q = 0; q < W / 4; ++q)
      if ((uint32_t)(4 * q) < words)
        dst[q] = make_uint4(lb[(4 * q) * kHuffThreads], lb[(4 * q + 1) * kHuffThreads], lb[(4 * q + 2) * kHuffThreads],
                            lb[(4 * q + 3) * kHuffThreads]);
  }
  __device__ void open(int32_t first_block) {
    n = (uint32_t)first_block * kEntHalfwordsPerBlock;
    k = 0;
  }
  __device__ void begin(int32_t blk) {
    b = blk;
    bstart = n + k;
    dcw = 0;
    n16 = n32 = 0;
    wide = false;
  }
  // a lane's region starts 256-byte aligned, so a group of W words is aligned too
  __device__ void put(uint32_t h) {
    ((uint16_t*)(lb + (k >> 1) * kHuffThreads))[k & 1] = (uint16_t)h;
    if (++k == 2 * W) {
      lds_flush(W);
      n += 2 * W;
      k = 0;
    }
  }
  __device__ void ac(int zz, int16_t v) {
    const uint32_t z = (uint32_t)(zz > 63 ? 63 : zz);  // 64..79 (corrupt streams) share natural position 63
    if (!wide && v >= -512 && v <= 511) {
      put(z | ((uint32_t)(v & 0x3FF) << 6));
      ++n16;
      return;
    }
    if (!wide) {
      wide = true;
      if ((n + k) & 1u) put(0u);  // u32 entries start at an even halfword
    }
    put(z);
    put((uint32_t)(uint16_t)v);
    ++n32;
  }
  __device__ void dc(int16_t v) { dcw = (uint32_t)(uint16_t)v << 16; }
  __device__ void record(int32_t blk, uint2 r) { binfo[blk] = r; }
  __device__ void end() { record(b, make_uint2(bstart, n16 | (n32 << 7) | dcw)); }
  // an all-zero block with absolute DC 0 (kBinfoAbsDc: k_dcscan does not add it up)
  __device__ void zero(int32_t blk) { record(blk, make_uint2(n + k, kBinfoAbsDc)); }
  __device__ void close() {  // the region is a multiple of 8 halfwords: a whole-chunk tail store stays inside it
    if (k) {
      if (k & 1) ((uint16_t*)(lb + (k >> 1) * kHuffThreads))[1] = 0;
      const uint32_t used = (k + 1) >> 1, words = (used + 3) & ~3u;
      for (uint32_t w = used; w < words; ++w) lb[w * kHuffThreads] = 0u;
      lds_flush(words);
    }
  }
};
using SparseSink = SparseSinkT<kSinkLds>;

// Lane geometry of a non-restart image: range [i*sub, end) of every active lane.
__device__ __forceinline__ uint32_t lane_range_end(const ImgDesc& d, int i, uint32_t nbits) {
  return i == d.h_lanes - 1 ? nbits : (uint32_t)(i + 1) * (uint32_t)d.h_sub;
}
__device__ __forceinline__ uint32_t lane_write_end(const ImgDesc& d, int i) {
  return i == d.h_lanes - 1 ? 0xFFFFFFFFu : (uint32_t)(i + 1) * (uint32_t)d.h_sub;
}

// ---------------------------------------------------------------------------
// k_htab: one workgroup per image.  Builds the decoder tables (derived tables of the
// DC/AC table of every component, then the kLookBits lookahead) in LDS and copies
// them to the image's table area; plans the image's segments.
// ---------------------------------------------------------------------------
__global__ void __launch_bounds__(kHuffThreads) k_htab(const uint8_t* __restrict__ bytes,
                                                       const int64_t* __restrict__ offsets,
                                                       ImgDesc* __restrict__ desc, uint8_t* __restrict__ ws) {
  main_prio();
  __shared__ HuffTables s_tab;
  __shared__ int32_t s_bad;
  ImgDesc& d = desc[blockIdx.x];
  const int t = threadIdx.x;
  if (d.status != DINO_IMG_OK || d.kind != 0) return;
  if (d.restart_interval > 0 && (d.n_rst < d.n_rst_max - 1 || d.rst_bad)) {
    // missing or out-of-sequence restart markers (counted by k_destuff_write, which
    // has completed): libjpeg resyncs (jdmarker.c jpeg_resync_to_restart) and decodes
    // what it finds, empty segments once the data has ended; the coefficient-buffer
    // path restates that walk, and its dense buffer fits in the sparse entry area
    if (t == 0) {
      if (align16(d.coef_bytes) <= (int64_t)d.total_blocks * kEntHalfwordsPerBlock * 2) d.kind = 1;
      else d.status = DINO_IMG_BADDATA;
    }
    return;
  }
  const uint8_t* p = bytes + offsets[blockIdx.x];
  if (t == 0) s_bad = 0;
  __syncthreads();
  if (t < 2 * d.ncomp) {
    const int c = t >> 1, ac = t & 1;
    const bool ok = ac ? huff_build_derived(p + d.huff_off[4 + d.comp[c].ta], false, &s_tab.ac[c])
                       : huff_build_derived(p + d.huff_off[d.comp[c].td], true, &s_tab.dc[c]);
    if (!ok) atomicOr(&s_bad, 1);
  }
  __syncthreads();
  if (s_bad) {
    if (t == 0) d.status = DINO_IMG_CORRUPT;
    return;
  }
  for (int e = t; e < 3 * (1 << kLookBits); e += kHuffThreads) {
    const int c = e >> kLookBits, idx = e & ((1 << kLookBits) - 1);
    if (c < d.ncomp) s_tab.ac_look[c][idx] = look_entry_of<kLookBits>(&s_tab.ac[c], idx);
  }
  for (int e = t; e < 3 * (1 << kDcLookBits); e += kHuffThreads) {
    const int c = e >> kDcLookBits, idx = e & ((1 << kDcLookBits) - 1);
    if (c < d.ncomp) s_tab.dc_look[c][idx] = look_entry_of<kDcLookBits>(&s_tab.dc[c], idx);
  }
  __syncthreads();
  for (int e = t; e < 3 * (1 << kLookBits); e += kHuffThreads) {
    const int c = e >> kLookBits, idx = e & ((1 << kLookBits) - 1);
    if (c < d.ncomp) {  // (both read only the entries' single-symbol bits, which stay as they are)
      s_tab.skip.ac[c][idx] = skip_pair_entry<kLookBits>(s_tab.ac_look[c], idx);
      s_tab.ac_look[c][idx] = look_pair_entry<kLookBits>(s_tab.ac_look[c], idx);
    }
  }
  for (int e = t; e < 3 * (1 << kDcLookBits); e += kHuffThreads) {
    const int c = e >> kDcLookBits, idx = e & ((1 << kDcLookBits) - 1);
    if (c < d.ncomp) s_tab.skip.dc[c][idx] = skip_entry(s_tab.dc_look[c][idx], true);
  }
  __syncthreads();
  uint4* dst = (uint4*)(ws + d.htab_off);
  const uint4* src = (const uint4*)&s_tab;
  for (int k = t; k < (int)(sizeof(HuffTables) / 16); k += kHuffThreads) dst[k] = src[k];
  if (t == 0) {
    const int64_t nbits = (int64_t)d.ent_len * 8;
    if (d.restart_interval > 0) {
      d.h_items = (d.n_rst_max + kHuffThreads - 1) / kHuffThreads;
      d.h_sub = 0;
      d.h_lanes = d.n_rst_max;
    } else {
      const int nseg = min(huff_segments(nbits), d.h_lanes_cap / kHuffThreads);
      int n = nseg * kHuffThreads;
      if (nseg == 1) n = (int)max((int64_t)1, min((int64_t)kHuffThreads, (nbits + kMinSubBits - 1) / kMinSubBits));
      uint32_t sub = (uint32_t)((nbits + n - 1) / n);
      sub = max(32u, (sub + 31u) & ~31u);
      d.h_sub = (int32_t)sub;
      d.h_lanes = (int32_t)max((int64_t)1, (nbits + sub - 1) / sub);
      d.h_items = (d.h_lanes + kHuffThreads - 1) / kHuffThreads;
    }
  }
}

// k_hseg: first work item of every image (exclusive scan over the batch, one WG of 1024).
__global__ void __launch_bounds__(1024) k_hseg(ImgDesc* __restrict__ desc, int B) {
  __shared__ int32_t part[1024];
  const int t = threadIdx.x;
  const int per = (B + 1023) / 1024;
  int32_t local = 0;
  for (int k = 0; k < per; ++k) {
    const int i = t * per + k;
    if (i < B && desc[i].status == DINO_IMG_OK && desc[i].kind == 0) local += desc[i].h_items;
  }
  part[t] = local;
  __syncthreads();
  for (int s = 1; s < 1024; s <<= 1) {
    const int32_t v = t >= s ? part[t - s] : 0;
    __syncthreads();
    part[t] += v;
    __syncthreads();
  }
  int32_t base = part[t] - local;
  for (int k = 0; k < per; ++k) {
    const int i = t * per + k;
    if (i >= B) continue;
    ImgDesc& d = desc[i];
    d.h_item_base = base;
    if (d.status == DINO_IMG_OK && d.kind == 0) base += d.h_items;
    else d.h_items = 0;
  }
}

// Image owning work item `item` (binary search over h_item_base); -1 past the end.
__device__ int huff_item_image(const ImgDesc* desc, int B, int item) {
  const ImgDesc& last = desc[B - 1];
  if (item >= last.h_item_base + last.h_items) return -1;
  int lo = 0, hi = B - 1;
  while (lo < hi) {  // last image with h_item_base <= item and h_items > 0
    const int mid = (lo + hi + 1) >> 1;
    if (desc[mid].h_item_base <= item) lo = mid;
    else hi = mid - 1;
  }
  while (lo > 0 && desc[lo].h_items == 0) --lo;
  return lo;
}

// An image of one segment without restart intervals and with short lane ranges is
// decoded completely by k_huff1 (its lanes' start states are final after the
// in-segment rounds).  Long ranges stay with k_huff3: in k_huff1 their second
// decode would double the longest serial chain of the launch.
__device__ __forceinline__ bool huff_single_segment(const ImgDesc& d) {
  return d.restart_interval == 0 && d.h_items == 1 && d.h_sub <= 3072;
}

// Loads work item `item`'s image descriptor and tables into LDS; false past the end.
// With skip_single, the tables of a single-segment image are not loaded (L.img = -2).
template <typename LdsT>
__device__ bool huff_load_item(LdsT& L, const ImgDesc* desc, int B, const uint8_t* ws, int item, bool skip_single = false,
                               int tab_bytes = (int)sizeof(HuffTables)) {
  if (threadIdx.x == 0) {
    L.img = huff_item_image(desc, B, item);
    if (L.img >= 0) {
      L.sd = desc[L.img];
      if (skip_single && huff_single_segment(L.sd)) L.img = -2;
    }
  }
  __syncthreads();
  if (L.img == -1) return false;
  if (L.img == -2) return true;
  const uint4* src = (const uint4*)(ws + L.sd.htab_off);
  uint4* dst = (uint4*)&L.tab;
  if (tab_bytes < 0) {  // k_huff1: the derived tables, then the skip entries at the lookaheads' offset
#pragma unroll 1
    for (int k = threadIdx.x; k < kHuffLookOff / 16; k += kHuffThreads) dst[k] = src[k];
    const uint4* ss = (const uint4*)(ws + L.sd.htab_off + offsetof(HuffTables, skip));
    uint4* sd = (uint4*)((uint8_t*)&L.tab + kHuffLookOff);
#pragma unroll 1
    for (int k = threadIdx.x; k < (int)(sizeof(HuffSkip) / 16); k += kHuffThreads) sd[k] = ss[k];
  } else {
#pragma unroll 1
    for (int k = threadIdx.x; k < tab_bytes / 16; k += kHuffThreads) dst[k] = src[k];
  }
  __syncthreads();
  return true;
}

#ifdef DINO_HUFF_PHASES
// Phase timestamps of k_huff1 work items (instrumented builds only, scripts/huff_phases.py):
// [item][0..4] = start, after the first decode, after the sync rounds, end; [item][4] = rounds.
constexpr int kPhaseItems = 8192;
__device__ uint64_t g_huff_phase[kPhaseItems][5];
#define HUFF_PHASE(k, v)                                              \
  do {                                                               \
    if (threadIdx.x == 0 && item < kPhaseItems) g_huff_phase[item][k] = (v); \
  } while (0)
#else
#define HUFF_PHASE(k, v) \
  do {                   \
  } while (0)
#endif

constexpr int kHuffLookback = 2048;  // bits a lane decodes before its range to guess its start state

__global__ void __launch_bounds__(kHuffThreads) k_huff1(const ImgDesc* __restrict__ desc, int B,
                                                        uint8_t* __restrict__ ws) {
  main_prio();
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  HuffLds& L = *reinterpret_cast<HuffLds*>(smem);
  const int t = threadIdx.x;
  for (int item = blockIdx.x;; item += gridDim.x) {
    if (!huff_load_item(L, desc, B, ws, item, false, -1)) return;
    const ImgDesc& sd = L.sd;
    if (sd.restart_interval > 0) {
      __syncthreads();
      continue;
    }
    HuffImage im;
    hi_init(im, reinterpret_cast<const HuffTables*>(L.tab), sd.mcu_comp, sd.blocks_per_mcu);
    im.skip_off = (uint32_t)kHuffLookOff;  // the skip entries sit where the value lookaheads come later
    RangeOut* const R = reinterpret_cast<RangeOut*>(L.tab + kHuffROff);  // lane results (skip phase)
    const BitReader br{(const uint32_t*)(ws + sd.ent_off), (uint32_t)sd.ent_len};
    const uint32_t nbits = (uint32_t)sd.ent_len * 8u;
    const int i = (item - sd.h_item_base) * kHuffThreads + t;  // lane index within the image
    const bool active = i < sd.h_lanes;
    const uint32_t rend = lane_range_end(sd, i, nbits);
    LaneRec* lr = (LaneRec*)(ws + sd.hlane_off);
    // checkpoint k of lane i at [k][lane]: a wave's lanes write neighbouring words
    Checkpoint* cps = (Checkpoint*)(ws + sd.cps_off) + i;
    const int cstride = sd.h_lanes_cap;
    int32_t ncp = 0;
    HState myS{(uint32_t)i * (uint32_t)sd.h_sub, 0, 0};  // this lane's start state and first-decode
    RangeOut myR1{};                                      // result stay in registers; only R is shared
    HUFF_PHASE(0, wall_clock64());
    if (kHuffLookback > 0 && active && i > 0) {  // guess the start state from kHuffLookback bits earlier
      const uint32_t to = myS.pos, from = to > (uint32_t)kHuffLookback ? to - (uint32_t)kHuffLookback : 0u;
      myS = decode_lookback<kHuffSrc>(br, im, from, to);
    }
    if (active) {
      myR1 = decode_range<kHuffSrc>(br, im, myS, rend, cps, cstride, kHuffCheckpoints, &ncp);
      R[t] = myR1;
    }
    __syncthreads();  // lane t-1's first decode (another wave) is visible before round 0
    HUFF_PHASE(1, wall_clock64());
    int round = 0;
    for (; round < kHuffThreads + 1; ++round) {
      HState want;
      bool redo = false;
      if (active && t >= 1) {
        want = R[t - 1].end;
        redo = !hstate_eq(want, myS);
      }
      __syncthreads();
      if (redo) {
        myS = want;
        R[t] = decode_range_sync<kHuffSrc>(br, im, want, rend, cps, cstride, ncp, myR1);
      }
      if (!__syncthreads_or(redo ? 1 : 0)) break;
    }
    const RangeOut res = R[t];
    HUFF_PHASE(2, wall_clock64());
    HUFF_PHASE(4, (uint64_t)round | ((uint64_t)(huff_single_segment(sd) ? 1 : 0) << 32));
    if (huff_single_segment(sd)) {
      // the whole image is this segment: its start states are final, so the blocks
      // are written here while the stream is still in cache (k_huff2 and k_huff3 skip it);
      // the value lookaheads replace the skip entries (no lane reads those any more)
      {
        const uint4* ls = (const uint4*)(ws + sd.htab_off + kHuffLookOff);
        uint4* ld = (uint4*)(L.tab + kHuffLookOff);
#pragma unroll 1
        for (int k = t; k < kHuffLookBytes / 16; k += kHuffThreads) ld[k] = ls[k];
      }
      __syncthreads();
      uint32_t tot;
      const uint32_t blk0 = block_excl_scan<kHuffThreads>(active ? (uint32_t)res.nblk : 0u, L.wave, &tot);
      if (active) {
        SparseSink sink;
        sink.ent = (uint32_t*)(ws + sd.coef_off);
        sink.binfo = (uint2*)(ws + sd.binfo_off);
        sink.lb = reinterpret_cast<uint32_t*>(L.tab + kHuffSinkOff) + t;
        sink.open((int32_t)blk0);
        decode_write<kHuffSrc>(br, im, myS, lane_write_end(sd, i), (int32_t)blk0, sd.total_blocks, (int32_t*)nullptr,
                                 nbits, sink);
        sink.close();
      }
    } else if (active) {
      LaneRec& o = lr[i];
      o.S = myS;
      o.R = res;
      o.R1 = myR1;
      o.ncp = ncp;
    }
    __syncthreads();
    HUFF_PHASE(3, wall_clock64());
  }
}

// k_huff2: one workgroup per image.  Rounds over all the image's lanes: a lane whose
// start state differs from its predecessor's end re-decodes (stopping at the first
// checkpoint the first decode also passed).  Then blk0 = exclusive scan of nblk.
constexpr int kHuff2Threads = 256;

__global__ void __launch_bounds__(kHuff2Threads) k_huff2(const ImgDesc* __restrict__ desc, uint8_t* __restrict__ ws) {
  main_prio();
  __shared__ HuffTables s_tab;
  __shared__ uint32_t s_wave[kHuff2Threads / 64];
  const ImgDesc& d = desc[blockIdx.x];
  const int t = threadIdx.x;
  if (d.status != DINO_IMG_OK || d.kind != 0 || d.restart_interval > 0 || huff_single_segment(d)) return;
  const int n = d.h_lanes;
  LaneRec* lr = (LaneRec*)(ws + d.hlane_off);
  if (n > kHuffThreads) {  // several segments: their first lanes started from guesses
    {
      const uint4* src = (const uint4*)(ws + d.htab_off);
      uint4* dst = (uint4*)&s_tab;
      for (int k = t; k < (int)(sizeof(HuffTables) / 16); k += kHuff2Threads) dst[k] = src[k];
    }
    __syncthreads();
    HuffImage im;
    hi_init(im, &s_tab, d.mcu_comp, d.blocks_per_mcu);
    const BitReader br{(const uint32_t*)(ws + d.ent_off), (uint32_t)d.ent_len};
    const uint32_t nbits = (uint32_t)d.ent_len * 8u;
    const Checkpoint* cps = (const Checkpoint*)(ws + d.cps_off);
    for (int round = 0; round <= n; ++round) {
      int any = 0;
      for (int i = 1 + t; i < n; i += kHuff2Threads) {
        const HState want = lr[i - 1].R.end;
        const bool redo = !hstate_eq(want, lr[i].S);
        lr[i].W = want;
        lr[i].pad = redo;
        any |= redo;
      }
      if (!__syncthreads_or(any)) break;
      for (int i = 1 + t; i < n; i += kHuff2Threads) {
        if (lr[i].pad) {
          const HState want = lr[i].W;
          lr[i].S = want;
          lr[i].R = decode_range_sync<kHuffSrc>(br, im, want, lane_range_end(d, i, nbits),
                                             cps + i, d.h_lanes_cap, lr[i].ncp, lr[i].R1);
        }
      }
      __syncthreads();
    }
  }
  // blk0: contiguous chunk of lanes per thread, block scan of the chunk sums
  const int per = (n + kHuff2Threads - 1) / kHuff2Threads;
  const int i0 = min(n, t * per), i1 = min(n, i0 + per);
  uint32_t sum = 0;
  for (int i = i0; i < i1; ++i) sum += (uint32_t)lr[i].R.nblk;
  uint32_t tot;
  uint32_t run = block_excl_scan<kHuff2Threads>(sum, s_wave, &tot);
  for (int i = i0; i < i1; ++i) {
    lr[i].blk0 = (int32_t)run;
    run += (uint32_t)lr[i].R.nblk;
  }
}

__global__ void __launch_bounds__(kHuffThreads) k_huff3(const ImgDesc* __restrict__ desc, int B,
                                                        uint8_t* __restrict__ ws) {
  main_prio();
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  HuffLds3& L = *reinterpret_cast<HuffLds3*>(smem);
  const int t = threadIdx.x;
  for (int item = blockIdx.x;; item += gridDim.x) {
    if (!huff_load_item(L, desc, B, ws, item, true, kHuffTabBytesNoSkip)) return;
    if (L.img == -2) {  // decoded by k_huff1
      __syncthreads();
      continue;
    }
    const ImgDesc& sd = L.sd;
    HuffImage im;
    hi_init(im, reinterpret_cast<const HuffTables*>(L.tab), sd.mcu_comp, sd.blocks_per_mcu);
    const uint32_t* words = (const uint32_t*)(ws + sd.ent_off);
    SparseSinkT<kSinkLds3> sink;
    sink.ent = (uint32_t*)(ws + sd.coef_off);
    sink.binfo = (uint2*)(ws + sd.binfo_off);
    sink.lb = L.sink + t;
    const int i = (item - sd.h_item_base) * kHuffThreads + t;
    if (sd.restart_interval > 0) {
      // restart intervals are independent: one lane per interval, absolute DC
      const int nseg = sd.n_rst_max;
      if (i < nseg) {
        const int32_t* rst = (const int32_t*)(ws + sd.rst_off);
        const int per = sd.restart_interval * sd.blocks_per_mcu;
        const uint32_t start = i == 0 ? 0u : (uint32_t)rst[i - 1] * 8u;
        const BitReader sb{words, i + 1 < nseg ? (uint32_t)rst[i] : (uint32_t)sd.ent_len};
        int32_t pred[kMaxComp] = {0, 0, 0};
        const int first = i * per, last = min(first + per, sd.total_blocks);
        if (first < last) {
          sink.open(first);
          decode_write<false>(sb, im, HState{start, 0, 0}, 0xFFFFFFFFu, first, last, pred, sb.nbytes * 8u, sink);
          sink.close();
        }
      }
    } else if (i < sd.h_lanes) {
      const LaneRec& r = ((const LaneRec*)(ws + sd.hlane_off))[i];
      const BitReader br{words, (uint32_t)sd.ent_len};
      sink.open(r.blk0);
      decode_write<kHuffSrc>(br, im, r.S, lane_write_end(sd, i), r.blk0, sd.total_blocks, (int32_t*)nullptr,
                               br.nbytes * 8u, sink);
      sink.close();
    }
    __syncthreads();
  }
}

// ---------------------------------------------------------------------------
// Coefficient-buffer images (kind 1: progressive, multi-scan sequential, restart
// images with missing / out-of-sequence markers), pscan.hpp:
//   k_pwalk  one workgroup per image: the marker walk (wave 0), the scan list in
//            dependency-level order, every decoder table the scans use (global
//            PTab, read through the scalar cache), the zeroed coefficient buffer,
//            and the image's registration in the batch's PCtl
//   k_pscan  persistent waves taking scan tickets; one wave decodes one scan, its
//            serial part wave-uniform (scalar ALU + scalar cache), its coefficient
//            stores lane-parallel; a scan waits for the previous level's scans of
//            its image (only ever scans with earlier tickets: no deadlock)
// ---------------------------------------------------------------------------
#ifdef DINO_PROG_PHASES
// per image (first kProgPhaseImgs of the batch) and scan (level order): start, end
// (wall_clock64) and the scan's level / band / approximation (instrumented builds only)
constexpr int kProgPhaseImgs = 64;
__device__ uint64_t g_prog_phase[kProgPhaseImgs][64][3];
hipError_t copy_prog_phases(uint64_t* host) {
  hipError_t e = hipDeviceSynchronize();
  if (e != hipSuccess) return e;
  return hipMemcpyFromSymbol(host, HIP_SYMBOL(g_prog_phase), sizeof(g_prog_phase));
}
#endif

// Wave-cooperative search for the end of a scan's entropy data (see HostMarkerFinder):
// each lane classifies 16 bytes per step, the first lane with a marker wins.
struct WaveMarkerFinder {
  __device__ int64_t operator()(const uint8_t* p, int64_t from, int64_t len) const {
    const int lane = threadIdx.x & 63;
    for (int64_t base = from; base + 1 < len; base += 64 * 16) {
      const int64_t k0 = base + lane * 16;
      uint32_t b[17];
#pragma unroll
      for (int j = 0; j < 17; ++j) b[j] = k0 + j < len ? p[k0 + j] : 0u;
      int hit = 16;
#pragma unroll
      for (int j = 15; j >= 0; --j) {
        const uint32_t c = b[j + 1];
        if (k0 + j + 1 < len && b[j] == 0xFFu && c != 0x00u && c != 0xFFu && !(c >= 0xD0u && c <= 0xD7u)) hit = j;
      }
      const uint64_t m = __ballot(hit < 16);
      if (m) {
        const int first = __ffsll((long long)m) - 1;
        return base + first * 16 + __shfl(hit, first);
      }
    }
    return -1;
  }
};

constexpr int kPWalkThreads = 256;
struct PWalkLds {
  ImgDesc d;
  ScanRec scans[kMaxScans];
  uint64_t ts[kMaxScans];
  int32_t slot_off[kPMaxTabs];
  uint8_t slot_dc[kPMaxTabs];
  ProgTable tab[kPMaxTabs];
  int32_t ntab, bad;
  int32_t lslot[kMaxScans];  // lane_plan
  LanePlan lp;
  int32_t lane;
};
__device__ __forceinline__ uint32_t wave_destuff(const uint8_t* img, int64_t len, int64_t from, uint8_t* dst, int lane);

__global__ void __launch_bounds__(kPWalkThreads) k_pwalk(const uint8_t* __restrict__ bytes,
                                                         const int64_t* __restrict__ offsets,
                                                         const int64_t* __restrict__ lengths,
                                                         ImgDesc* __restrict__ desc, uint8_t* __restrict__ ws,
                                                         PCtl* __restrict__ pctl, int lane_ok) {
  __shared__ PWalkLds L;
  const int img = blockIdx.x, t = threadIdx.x;
  if (desc[img].status != DINO_IMG_OK || desc[img].kind != 1) return;
  const uint8_t* p = bytes + offsets[img];
  const int64_t len = lengths ? lengths[img] : offsets[img + 1] - offsets[img];
  if (t == 0) L.d = desc[img];
  __syncthreads();
  if (t < 64) {  // wave 0: every lane runs the walk on the LDS descriptor (identical values, identical writes)
    WaveMarkerFinder find;
    prog_walk(p, len, &L.d, L.scans, find);
  }
  __syncthreads();
  const ImgDesc& dl = L.d;
  uint8_t* region = ws + dl.htab_off;
  if (t == 0 && dl.status == DINO_IMG_OK) {
    // the region k_plan placed (kind 1: kPRegionBytes; a restart image switched by k_htab: its table area)
    L.ntab = prog_table_slots(L.scans, dl.n_scans, L.slot_off, L.slot_dc, L.ts,
                              ptab_capacity(dl.hlane_off - dl.htab_off));
    L.bad = 0;
    // the lane decoder (lscan.hpp) when the script allows deferring the refinements and the
    // side records were planned (kind 1 from the parse: a restart image k_htab switched is not)
    L.lane = lane_plan(L.scans, dl.n_scans, dl.progressive != 0, L.lslot, &L.lp) &&
             dl.plane_off - dl.binfo_off >= (dl.coef_bytes / 128) * kLSideBytes && lane_ok;
  }
  __syncthreads();
  if (dl.status != DINO_IMG_OK || L.ntab < 0) {
    if (t == 0) desc[img].status = dl.status != DINO_IMG_OK ? dl.status : DINO_IMG_UNSUPPORTED;
    return;
  }
  const int n = dl.n_scans, ntab = L.ntab;
  if (t < ntab && !huff_build_derived(p + L.slot_off[t], L.slot_dc[t] != 0, &L.tab[t])) atomicOr(&L.bad, 1);
  __syncthreads();
  if (L.bad) {  // JERR_BAD_HUFF_TABLE (libjpeg raises when the scan using it starts: the image fails either way)
    if (t == 0) desc[img].status = DINO_IMG_CORRUPT;
    return;
  }
  PTab* tabs = (PTab*)(region + kPTabOff);
  for (int e = t; e < ntab << kPLookBits; e += kPWalkThreads)
    tabs[e >> kPLookBits].look[e & ((1 << kPLookBits) - 1)] = ptab_look_entry(&L.tab[e >> kPLookBits], e & ((1 << kPLookBits) - 1));
  if (t < ntab) ptab_fill_derived(&L.tab[t], &tabs[t]);
  PHdr* hd = (PHdr*)region;
  PScan* ps = (PScan*)(region + kPScanOff);
  if (t < n) {
    PScan o;
    o.sr = L.scans[t];
    o.tslots = L.ts[t];
    o.pipe = prog_pipelined(L.scans, n, t, dl.progressive != 0, &o.deps) ? 1 : 0;
    o.dlen = 0;
    o.slot = L.lane ? L.lslot[t] : -1;
    ps[prog_level_rank(L.scans, n, t)] = o;
  }
  int nlev = 0;
  for (int i = 0; i < n; ++i) nlev = L.scans[i].level + 1 > nlev ? L.scans[i].level + 1 : nlev;
  if (t < kMaxScans) {
    int c = 0;
    for (int i = 0; i < n; ++i) c += L.scans[i].level == t;
    hd->cnt[t] = c;
    hd->done[t] = 0;
    hd->prog[t] = 0;
  }
  if (t == 0) {
    hd->n_scans = n;
    hd->n_levels = nlev;
    hd->lane = L.lane;
    lane_pack(L.lp, &hd->lane_nac, &hd->lane_al_ac, hd->lane_band, &hd->lane_ndc, &hd->lane_al_dc);
  }
  // libjpeg's zeroed coefficient arrays (+ the lane decoder's side records)
  {
    uint4* c4 = (uint4*)(ws + dl.coef_off);
    const int64_t nq = dl.coef_bytes >> 4;
    for (int64_t q = t; q < nq; q += kPWalkThreads) c4[q] = make_uint4(0u, 0u, 0u, 0u);
    if (L.lane) {
      uint4* s4 = (uint4*)(ws + dl.binfo_off);
      const int64_t ns = (dl.coef_bytes / 128) * (kLSideBytes / 16);
      for (int64_t q = t; q < ns; q += kPWalkThreads) s4[q] = make_uint4(0u, 0u, 0u, 0u);
    }
  }
  if (L.lane) {  // every scan destuffed here, a wave per scan (k_pscan does it per scan wave)
    __syncthreads();  // the PScan records (dlen) are complete
    const int w = t >> 6, ln = t & 63;
    for (int i = w; i < n; i += kPWalkThreads / 64) {
      const ScanRec& sr = L.scans[i];
      uint8_t* clean = ws + dl.ent_off + ((sr.data_off - dl.scan_off + 3) & ~3);
      const uint32_t dlen = wave_destuff(p, len, sr.data_off, clean, ln);
      if (ln == 0) ps[prog_level_rank(L.scans, n, i)].dlen = (int32_t)dlen;
    }
  }
  if (t == 0) {
    desc[img].n_scans = n;
    if (L.lane) {
      const uint32_t k = atomicAdd(&pctl->nlane, 1u);
      pctl->pimg[pctl->cap - 1 - k] = img;
      atomicMax(&pctl->lmax_scans, (uint32_t)n);
    } else {
      const uint32_t k = atomicAdd(&pctl->nprog, 1u);
      pctl->pimg[k] = img;
      atomicMax(&pctl->max_scans, (uint32_t)n);
    }
  }
}

// Lane-conditional stores of the scan waves go to this dummy slot instead of branching
// around the store: a divergent branch inside the decode loops makes the compiler's
// uniformity analysis treat the loops' scalar state (bit position, EOB run, masks) as
// divergent at the join, which moves the whole serial decode from SGPRs to VGPRs
// (measured: 250 instructions per symbol instead of ~50).
// Stores go through buffer resources whose range check drops the disabled lanes' stores
// (offset kNoStore is out of range): no branch, and no lane writes anything it should not
// (a shared dummy address would be written by every wave at once).  The OR entries of the
// DC refinement (atomics) keep a dummy word, one per lane and wave slot.
constexpr uint32_t kNoStore = 0x80000000u;
__device__ __forceinline__ __amdgpu_buffer_rsrc_t store_rsrc(void* base) {
  return __builtin_amdgcn_make_buffer_rsrc(base, (short)0, 0x7FFFFFFF, 0x00020000);
}
__device__ __forceinline__ void store16_if(__amdgpu_buffer_rsrc_t r, bool c, int64_t elem, int16_t v) {
  __builtin_amdgcn_raw_buffer_store_b16((unsigned short)v, r, c ? (int)(uint32_t)(elem * 2) : (int)kNoStore, 0, 0);
}
__device__ __forceinline__ void store8_if(__amdgpu_buffer_rsrc_t r, bool c, uint32_t off, uint8_t v) {
  __builtin_amdgcn_raw_buffer_store_b8(v, r, c ? (int)off : (int)kNoStore, 0, 0);
}
__device__ uint32_t g_pscan_dummy[1024 * 64];

// The lanes' half of a scan (see pscan.hpp): pending (element, value) stores in lane
// registers, and for AC refinement the 16-block groups of coefficients (lane k holds
// zigzag coefficient k of each block of the group).
struct WaveCoefSink {
  int16_t* coef;
  DINO_LDS int16_t* stage;  // [16][64]: the staged group's coefficients
  int lane, natk;
  int32_t n;                // pending entries (uniform)
  int32_t eidx, eval;       // lane n's entry: element, value (| 1 << 16: OR into the coefficient)
  // AC refinement
  int64_t plane;
  int32_t bw, mcx, nblk;
  int32_t grp, nxgrp, g;
  int32_t cbx, cby;         // block (x, y) of the next rnz
  int64_t cur;              // element of the current block
  uint32_t mlo, mhi;        // lane j: zigzag non-zero mask of block j of the staged group
  int32_t nx[16];           // the next group's coefficients (prefetched)

  __device__ __forceinline__ void flush() {  // (branch-free: see g_pscan_dummy)
    const bool act = lane < n, isor = (eval & 0x10000) != 0;
    uint32_t* w = (act & isor) ? (uint32_t*)(coef + (eidx & ~1)) : &g_pscan_dummy[((blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6)) & 1023) * 64 + lane];
    __hip_atomic_fetch_or(w, isor ? (uint32_t)(eval & 0xFFFF) << (16 * (eidx & 1)) : 0u, __ATOMIC_RELAXED,
                          __HIP_MEMORY_SCOPE_AGENT);
    store16_if(store_rsrc(coef), act & !isor, eidx, (int16_t)eval);
    n = 0;
  }
  __device__ __forceinline__ void put(int64_t e, int32_t v) {
    eidx = lane == n ? (int32_t)e : eidx;
    eval = lane == n ? v : eval;
    if (++n == 64) flush();
  }
  __device__ __forceinline__ void set(int64_t e, int32_t v) { put(e, v & 0xFFFF); }
  __device__ __forceinline__ void orw(int64_t e, int32_t v) { put(e, (v & 0xFFFF) | 0x10000); }

  __device__ __forceinline__ void load_group(int32_t G) {
    const int32_t m0 = G * 16;
    int32_t by = m0 / mcx, bx = m0 - by * mcx;
#pragma unroll
    for (int j = 0; j < 16; ++j) {
      const int64_t e = plane + ((int64_t)by * bw + bx) * 64;
      nx[j] = m0 + j < nblk ? (int32_t)coef[e + natk] : 0;
      if (++bx == mcx) {
        bx = 0;
        ++by;
      }
    }
    nxgrp = G;
  }
  __device__ __forceinline__ void rbegin(int64_t pl, int32_t w, int32_t mcus_x, int32_t mcus_y) {
    plane = pl;
    bw = w;
    mcx = mcus_x;
    nblk = mcus_x * mcus_y;
    grp = -1;
    cbx = cby = 0;
    load_group(0);
  }
  // rnz is called for m = 0, 1, 2, ... in order
  __device__ __forceinline__ uint64_t rnz(int64_t m) {
    const int32_t G = (int32_t)(m >> 4);
    if (G != grp) {
      if (nxgrp != G) load_group(G);
#pragma unroll
      for (int j = 0; j < 16; ++j) {
        stage[j * 64 + lane] = (int16_t)nx[j];
        const uint64_t b = __ballot(nx[j] != 0);
        mlo = lane == j ? (uint32_t)b : mlo;
        mhi = lane == j ? (uint32_t)(b >> 32) : mhi;
      }
      grp = G;
      if ((G + 1) * 16 < nblk) load_group(G + 1);  // prefetched while this group decodes
    }
    g = (int32_t)(m & 15);
    cur = plane + ((int64_t)cby * bw + cbx) * 64;
    if (++cbx == mcx) {
      cbx = 0;
      ++cby;
    }
    return (uint64_t)(uint32_t)__builtin_amdgcn_readlane((int32_t)mhi, g) << 32 |
           (uint32_t)__builtin_amdgcn_readlane((int32_t)mlo, g);
  }
  __device__ __forceinline__ void rapply(uint64_t corr, uint64_t nzn, uint64_t neg, int al) {
    const bool c = (corr >> lane) & 1u, nw = (nzn >> lane) & 1u;
    const int16_t v = stage[g * 64 + lane];
    const int16_t x = ac_refine_value(v, c, nw, (neg >> lane) & 1u, al);
    store16_if(store_rsrc(coef), x != v, cur + natk, x);  // (branch-free: see g_pscan_dummy)
  }
};

// The scan's decoder tables in VGPRs: 8 table positions (DC of scan component k < 4,
// AC k - 4) x 512 lookahead entries of 16 bits; entry i of position k is half (i & 1) of
// lane ((k * 512 + i) >> 1) & 63 of register (k * 512 + i) >> 7.  A lookup is one
// indexed register move + one readlane: no memory access on the decode chain.  Codes
// longer than the lookahead search the PTab (scalar cache).  Lane k also holds
// jpeg_natural_order[k].
typedef uint32_t u32x32 __attribute__((ext_vector_type(32)));
struct VTab {
  u32x32 v;
  const DINO_CONST PTab* tabs;
  uint64_t ts;
  uint32_t natv;
  uint32_t hv4, mv4;  // AC table (position 4): huffval dwords; lanes 0-6 maxcode[10..16], 8-14 valoffset[10..16]
  __device__ __forceinline__ void load(const PTab* tb, uint64_t slots, int lane) {
    tabs = (const DINO_CONST PTab*)tb;
    ts = slots;
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const int s = pbyte64(slots, k);
      const uint32_t* src = (const uint32_t*)tb[s < 0xFF ? s : 0].look;
#pragma unroll
      for (int j = 0; j < 4; ++j) v[4 * k + j] = s < 0xFF ? src[64 * j + lane] : 0u;
    }
    natv = kNaturalOrder[lane];
    const int s4 = pbyte64(slots, 4);
    const PTab* t4 = tb + (s4 < 0xFF ? s4 : 0);
    hv4 = t4->huffval[lane];
    const int q = lane & 7;
    mv4 = q < 7 && lane < 16 ? (uint32_t)(lane < 8 ? t4->maxcode[kPLookBits + 1 + q] : t4->valoffset[kPLookBits + 1 + q]) : 0u;
  }
  __device__ __forceinline__ void lookup(int k, uint32_t p, int* sym, int* len) const {
    // (uniform, but the compiler may compute it on the VALU: without the readfirstlane the
    // indexed move would become a waterfall loop)
    const uint32_t h = (uint32_t)__builtin_amdgcn_readfirstlane((int32_t)((uint32_t)k * 512u + (p >> (32 - kPLookBits))));
    const uint32_t x = (uint32_t)__builtin_amdgcn_readlane((int32_t)v[h >> 7], (h >> 1) & 63);
    const uint32_t e = (h & 1) ? x >> 16 : x & 0xFFFFu;
    if (e) {
      *sym = (int)(e >> 4);
      *len = (int)(e & 15u);
    } else if (k == 4) {  // the AC table's long codes from lane registers (no scalar-cache round trip)
      const uint32_t p17 = p >> 15;
      int l = 17, off = 0;
#pragma unroll
      for (int q = 16 - kPLookBits - 1; q >= 0; --q) {
        if ((int32_t)(p17 >> (17 - (kPLookBits + 1 + q))) <= __builtin_amdgcn_readlane((int32_t)mv4, q)) {
          l = kPLookBits + 1 + q;
          off = __builtin_amdgcn_readlane((int32_t)mv4, 8 + q);
        }
      }
      *len = l;
      const int ix = ((int)(p17 >> (17 - (l > 16 ? 16 : l))) + off) & 255;
      *sym = l > 16 ? 0 : (int)(((uint32_t)__builtin_amdgcn_readlane((int32_t)hv4, ix >> 2) >> (8 * (ix & 3))) & 0xFFu);
    } else {
      ptab_slow(tabs + pbyte64(ts, k), p, sym, len);
    }
  }
  __device__ __forceinline__ int nat(int k) const { return __builtin_amdgcn_readlane((int32_t)natv, k < 64 ? k : 63); }
};

// The destuffed scan as a bit string, read through two 256-byte windows of lane
// registers (A: dwords 64 wa .. 64 wa + 63, B: the next 64, loaded when A is entered, so
// the load has a whole window of decoding to land).  Bytes past the data read as zeros.
struct CleanReader {
  const uint32_t* src;  // destuffed bytes (4-byte aligned; the last dword zero padded)
  uint32_t nw;          // dwords holding data
  uint32_t pos, nbits;  // bits consumed, data bits
  int32_t wa;
  uint32_t A, B, Braw;  // Braw: the next-but-one window as loaded (swapped when it becomes B)
  int lane;
  __device__ __forceinline__ uint32_t rawload(int32_t gi) const {
    const uint32_t w = (uint32_t)gi * 64u + (uint32_t)lane;
    return src[w < nw ? w : 0u];  // (always loaded: no branch, see g_pscan_dummy)
  }
  __device__ __forceinline__ uint32_t swapw(int32_t gi, uint32_t x) const {
    return (uint32_t)gi * 64u + (uint32_t)lane < nw ? __builtin_bswap32(x) : 0u;
  }
  __device__ __forceinline__ uint32_t loadw(int32_t gi) const { return swapw(gi, rawload(gi)); }
  __device__ __forceinline__ void init(const uint32_t* s, uint32_t nbytes, int ln) {
    src = s;
    nw = (nbytes + 3) >> 2;
    nbits = nbytes * 8;
    pos = 0;
    lane = ln;
    wa = 0;
    A = loadw(0);
    B = loadw(1);
    Braw = rawload(2);
  }
  __device__ __forceinline__ uint32_t peek() const {
    const uint32_t ps = pos;
    const int32_t wu = wa;
    const uint32_t w = ps >> 5, sh = ps & 31;
    // dwords w and w + 1: both in A, or w in A and w + 1 the first of B (w < 64 (wa + 1))
    const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int32_t)A, w & 63);
    const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int32_t)((int32_t)((w + 1) >> 6) == wu ? A : B), (w + 1) & 63);
    const uint64_t x = (uint64_t)hi << 32 | lo;
    return (uint32_t)((x << sh) >> 32);
  }
  __device__ __forceinline__ void skip(int n) {
    pos += (uint32_t)n;
    if ((int32_t)(pos >> 11) > wa) {  // the load of the new B was issued a window ago: no wait here
      A = B;
      ++wa;
      B = swapw(wa + 1, Braw);
      Braw = rawload(wa + 2);
    }
  }
  __device__ __forceinline__ bool insuff() const { return pos > nbits; }
  __device__ __forceinline__ void restart(int*) {}
};

// Destuff [from, ...) of the image into dst (4-byte aligned) with host_destuff's rule,
// 256 bytes per step (one aligned dword per lane, neighbours by shuffles); returns the
// data bytes.  The bytes after them up to the next dword boundary are zeroed.
__device__ __forceinline__ uint32_t wave_destuff(const uint8_t* img, int64_t len, int64_t from, uint8_t* dst, int lane) {
  const uintptr_t beg = (uintptr_t)(img + from), end = (uintptr_t)(img + len);
  uint32_t out = 0, carry = 0;  // carry: the byte before this step's first dword
  const __amdgpu_buffer_rsrc_t dr = store_rsrc(dst);
  const uint64_t lt = lane ? ~0ull >> (64 - lane) : 0ull;  // lanes below this one
  for (uintptr_t c = beg & ~(uintptr_t)3; c < end; c += 256) {
    const uintptr_t wa = c + 4u * (uint32_t)lane;
    // (loads clamped to the first word instead of branched around: see g_pscan_dummy)
    const uintptr_t w0 = beg & ~(uintptr_t)3;
    const uint32_t wl = *(const uint32_t*)(wa < end ? wa : w0);
    const uint32_t w = wa < end ? wl : 0u;
    // (every lane runs both shuffles: a lane reading an inactive lane would get nothing)
    const uint32_t dn = (uint32_t)__shfl_down((int)w, 1);
    const uint32_t up = (uint32_t)__shfl_up((int)w, 1);
    const bool nxt = (lane == 63) & (wa + 4 < end);
    const uint32_t wl4 = *(const uint32_t*)(nxt ? wa + 4 : w0);
    const uint32_t wn = lane == 63 ? (nxt ? wl4 : 0u) : dn;
    const uint32_t wp = lane ? up : carry << 24;
    uint32_t keep = 0, term = 0;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const uintptr_t a = wa + i;
      const uint32_t b = (w >> (8 * i)) & 255u;
      const uint32_t nx = i < 3 ? (w >> (8 * i + 8)) & 255u : wn & 255u;
      const uint32_t pv = i > 0 ? (w >> (8 * i - 8)) & 255u : wp >> 24;
      const bool valid = (a >= beg) & (a < end), nxv = a + 1 < end, pvv = a > beg;
      // (bitwise, branch-free: see g_pscan_dummy)
      const bool isff = b == 0xFFu;
      const bool kff = isff & nxv & (nx == 0u);
      const bool tff = isff & !kff & (!nxv | (nx != 0xFFu));
      const bool knon = !isff & !((b == 0u) & pvv & (pv == 0xFFu));
      keep |= (uint32_t)(valid & (kff | knon)) << i;
      term |= (uint32_t)(valid & tff) << i;
    }
    const uint64_t tl = __ballot(term != 0);
    if (tl) {
      const int f = __ffsll((long long)tl) - 1;
      const int fi = __shfl(term ? __builtin_ctz(term) : 0, f);
      keep = lane > f ? 0u : (lane == f ? keep & ((1u << fi) - 1u) : keep);
    }
    const uint32_t cnt = __builtin_popcount(keep);
    const uint64_t b0 = __ballot(cnt & 1u), b1 = __ballot(cnt & 2u), b2 = __ballot(cnt & 4u);
    uint32_t o = out + (uint32_t)(__builtin_popcountll(b0 & lt) + 2 * __builtin_popcountll(b1 & lt) +
                                  4 * __builtin_popcountll(b2 & lt));
#pragma unroll
    for (int i = 0; i < 4; ++i) {  // (branch-free: see g_pscan_dummy)
      const bool k = (keep >> i) & 1u;
      store8_if(dr, k, o, (uint8_t)(w >> (8 * i)));
      o += k;
    }
    out += (uint32_t)(__builtin_popcountll(b0) + 2 * __builtin_popcountll(b1) + 4 * __builtin_popcountll(b2));
    if (tl) break;
    carry = (uint32_t)__builtin_amdgcn_readlane((int32_t)w, 63) >> 24;
  }
  store8_if(dr, (uint32_t)lane < ((4u - (out & 3u)) & 3u), out + lane, 0);
  __threadfence();  // this wave reads the bytes back (CleanReader)
  return out;
}

// Specialised loops for the AC scans of progressive files (the bulk of their symbols:
// ~85 % of a libjpeg-default progressive 640x480 file, profiles/r03_prog_phases_*):
// one component, the AC table at table position 4, the destuffed reader, no restart
// intervals.  A wave issues at most one instruction per cycle and a dependent chain
// far fewer, so these loops keep the per-symbol path short: the bit-mask searches of
// the refinement (the run's stop position, the correction bits) are one lane-parallel
// rank (v_mbcnt) + ballot each instead of a loop over bits, and the AC-first values
// collect in lane k = zigzag k of the block (one masked store per block).
__device__ __forceinline__ uint32_t lane_rank(uint64_t mask) {  // set bits of mask below this lane
  return __builtin_amdgcn_mbcnt_hi((uint32_t)(mask >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)mask, 0u));
}
__device__ __forceinline__ uint64_t ubal(bool b) { return __ballot(b); }

// Correction bits (one per set bit of c, increasing k, MSB first), read as a bit mask.
__device__ __forceinline__ uint64_t fast_corrections(CleanReader& r, uint64_t c, int lane) {
  int n = __builtin_popcountll(c);
  if (!n) return 0;
  const uint32_t rank = lane_rank(c);
  const bool in = (c >> lane) & 1u;
  uint64_t corr = 0;
  int base = 0;
  while (n > 0) {
    const int take = n > 32 ? 32 : n;
    const uint32_t bits = r.peek();
    const int32_t q = (int32_t)rank - base;
    // (bitwise &: a short-circuit && on lane values is a divergent branch, see g_pscan_dummy)
    corr |= ubal(in & (q >= 0) & (q < take) & (((bits >> ((31 - q) & 31)) & 1u) != 0u));
    r.skip(take);
    base += take;
    n -= take;
  }
  return corr;
}
// The same when the caller already holds the next pav bits (pw, MSB first): no new peek
// when they suffice (a refinement symbol's code + sign leave >= 14 of its 32-bit peek).
__device__ __forceinline__ uint64_t fast_corrections_p(CleanReader& r, uint64_t c, int lane, uint32_t pw, int pav) {
  const int n = __builtin_popcountll(c);
  if (!n) return 0;
  if (n > pav) return fast_corrections(r, c, lane);
  const uint32_t rank = lane_rank(c);  // < n <= 32 on the lanes of c
  const uint64_t corr = ubal((((c >> lane) & 1u) != 0u) & (((pw >> ((31 - rank) & 31)) & 1u) != 0u));
  r.skip(n);
  return corr;
}

// Block pipelining between the AC scans of one component (prog_pipelined): a scan
// publishes how many of its blocks are stored every kPipeBlocks blocks (release: the
// wave's stores are complete and written back first), and a scan that reads what
// earlier scans wrote waits, before it loads a group of coefficients, until every one of
// them has published past that group (acquire).  Its dependencies hold earlier tickets,
// so they are running or done.
constexpr int kPipeBlocks = 128;
struct ScanPipe {
  int32_t* prog;      // PHdr::prog
  int32_t self;       // this scan's sorted index (publishes prog[self])
  uint64_t deps;      // sorted indices of the scans it follows (0xFF: none)
  int32_t avail;      // blocks every dependency has published (as last seen)
  __device__ __forceinline__ void publish(int32_t nb) {
    __hip_atomic_store(&prog[self], nb, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
  }
  __device__ __forceinline__ void need(int32_t nb) {  // wait until every dependency passed block nb
    while (avail < nb) {
      int32_t m = 0x7FFFFFFF;
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        const int dj = pbyte64(deps, k);
        if (dj != 0xFF) {
          const int32_t v = __builtin_amdgcn_readfirstlane(__hip_atomic_load(&prog[dj], __ATOMIC_ACQUIRE,
                                                                             __HIP_MEMORY_SCOPE_AGENT));
          m = v < m ? v : m;
        }
      }
      avail = m;
      if (avail < nb) __builtin_amdgcn_s_sleep(8);
    }
  }
};

// decode_mcu_AC_refine over the whole scan (see r_refine_block for the bookkeeping).
__device__ __forceinline__ void fast_ac_refine(CleanReader& r, const VTab& t, const ScanRec& sr, int64_t plane, int32_t bw,
                               int32_t mcx, int32_t mcy, WaveCoefSink& sink, int lane, ScanPipe& pp) {
  const int ss = sr.ss, se = sr.se, al = sr.al;
  const uint64_t band = (uint64_t)low_bits(se + 1) & ~(uint64_t)low_bits(ss);
  int32_t eobrun = 0;
  const int32_t nblk = mcx * mcy;
  pp.need(min(32, nblk));  // rbegin loads the first group, rnz the next one ahead
  sink.rbegin(plane, bw, mcx, mcy);
  for (int32_t m = 0; m < nblk; ++m) {
    if ((m & 15) == 0) pp.need(min(m + 32, nblk));
    const uint64_t nzz = sink.rnz(m) & band;
    if (r.insuff()) continue;
    uint64_t corr = 0, nzn = 0, neg = 0;
    int k = ss;
    if (eobrun == 0) {
      while (k <= se) {
        const uint32_t p = r.peek();
        int sym, len;
        t.lookup(4, p, &sym, &len);
        const int rr = sym >> 4, s = sym & 15;
        bool negative = false;
        int used;
        if (s) {
          negative = ((p << len) >> 31) == 0u;
          used = len + 1;
        } else if (rr != 15) {
          eobrun = (1 << rr) + (int32_t)peek_extra(p, len, rr);
          r.skip(len + rr);
          break;
        } else {
          used = len;
        }
        r.skip(used);
        // stop: the (rr+1)-th position at or after k that was zero before the scan (rr = 0: the first)
        const uint64_t z = ~nzz & band & ~(uint64_t)low_bits(k);
        uint64_t hit = z;
        if (rr) hit = ubal((((z >> lane) & 1u) != 0u) & (lane_rank(z) == (uint32_t)rr));
        const int stop = hit ? __builtin_ctzll(hit) : se + 1;
        corr |= fast_corrections_p(r, nzz & (uint64_t)low_bits(stop) & ~(uint64_t)low_bits(k), lane,
                                   used < 32 ? p << used : 0u, 32 - used);
        k = stop;
        if (s) {
          const uint64_t bit = k < 64 ? 1ull << k : 1ull << 63;
          nzn |= bit;
          if (negative) neg |= bit;
          else neg &= ~bit;
        }
        ++k;
      }
    }
    if (eobrun > 0) {
      if (k <= se) corr |= fast_corrections(r, nzz & ~(uint64_t)low_bits(k), lane);
      --eobrun;
    }
    sink.rapply(corr, nzn, neg, al);
    if (((m + 1) & (kPipeBlocks - 1)) == 0) pp.publish(m + 1);
  }
  pp.publish(nblk);
}

// decode_mcu_AC_first over the whole scan: values gather in lane k (zigzag k) of the
// block and leave with one masked store.
__device__ __forceinline__ void fast_ac_first(CleanReader& r, const VTab& t, const ScanRec& sr, int16_t* coef, int64_t plane,
                              int32_t bw, int32_t mcx, int32_t mcy, int lane, int natk, ScanPipe& pp) {
  const int ss = sr.ss, se = sr.se, al = sr.al;
  const __amdgpu_buffer_rsrc_t cr = store_rsrc(coef);
  int32_t eobrun = 0;
  int32_t bx = 0;
  int64_t rowe = plane;  // element of block (0, by)
  for (int32_t by = 0; by < mcy; ++by, rowe += (int64_t)bw * 64) {
    // an AC first scan follows the earlier scans that may write its coefficients (a corrupt
    // neighbour band's run, progressive.hpp scan_write_end) row by row
    pp.need((by + 1) * mcx);
    for (bx = 0; bx < mcx; ++bx) {
      if (eobrun > 0) {
        --eobrun;
        continue;
      }
      if (r.insuff()) continue;
      int32_t val = 0;
      uint64_t have = 0;
      for (int k = ss; k <= se; k++) {
        const uint32_t p = r.peek();
        int sym, len;
        t.lookup(4, p, &sym, &len);
        const int rr = sym >> 4, s = sym & 15;
        if (s) {
          k += rr;
          const int v = huff_extend((int)peek_extra(p, len, s), s);
          r.skip(len + s);
          const int kk = k < 64 ? k : 63;  // (libjpeg's safety entries map k > 63 to 63)
          val = lane == kk ? (int32_t)((uint32_t)v << al) : val;
          have |= 1ull << kk;
        } else if (rr == 15) {
          r.skip(len);
          k += 15;
        } else {
          eobrun = (1 << rr) + (int32_t)peek_extra(p, len, rr) - 1;
          r.skip(len + rr);
          break;
        }
      }
      store16_if(cr, (have >> lane) & 1u, rowe + (int64_t)bx * 64 + natk, (int16_t)val);
    }
    const int32_t done = (by + 1) * mcx;  // (published when it crosses a multiple of kPipeBlocks)
    if (done / kPipeBlocks != (done - mcx) / kPipeBlocks) pp.publish(done);
  }
  pp.publish(mcx * mcy);
}

// Scan waves per workgroup: each wave takes its own tickets; the waves of one workgroup
// sit on different SIMDs of the CU (4, measured in profiles/r03_prog_*).
constexpr int kPScanThreads = 64 * 4;
__global__ void __launch_bounds__(kPScanThreads) k_pscan(const uint8_t* __restrict__ bytes,
                                                         const int64_t* __restrict__ offsets,
                                                         const int64_t* __restrict__ lengths,
                                                         const ImgDesc* __restrict__ desc, uint8_t* __restrict__ ws,
                                                         PCtl* __restrict__ pctl, int prio) {
  __shared__ int16_t s_stage[4][16 * 64];
  if (prio) __builtin_amdgcn_s_setprio(3);
  const int lane = threadIdx.x & 63;
  const DINO_CONST PCtl* cc = (const DINO_CONST PCtl*)pctl;
  const uint32_t nprog = cc->nprog;
  const uint32_t total = nprog * cc->max_scans;
  const DINO_CONST int64_t* offs = (const DINO_CONST int64_t*)offsets;
  const DINO_CONST int64_t* lens = (const DINO_CONST int64_t*)lengths;
  for (;;) {
    uint32_t tk = 0;
    if (lane == 0) tk = atomicAdd(&pctl->ticket, 1u);
    tk = (uint32_t)__builtin_amdgcn_readfirstlane((int32_t)__shfl(tk, 0));
    if (tk >= total) break;
    const uint32_t j = tk / nprog;
    const int img = cc->pimg[tk - j * nprog];
    const DINO_CONST ImgDesc* d = (const DINO_CONST ImgDesc*)(desc + img);
    uint8_t* region = ws + d->htab_off;
    const DINO_CONST PHdr* hd = (const DINO_CONST PHdr*)region;
    if ((int)j >= hd->n_scans) continue;
    const DINO_CONST PScan* ps = (const DINO_CONST PScan*)(region + kPScanOff) + j;
    const ScanRec sr = ps->sr;
    const int64_t off = offs[img];
    const int64_t len = lengths ? lens[img] : offs[img + 1] - off;
    const uint8_t* p = bytes + off;
    // the scan's bytes destuffed and its tables in registers before waiting for its level
    VTab tb;
    tb.load((const PTab*)(region + kPTabOff), ps->tslots, lane);
    uint32_t* clean = (uint32_t*)(ws + d->ent_off + ((sr.data_off - d->scan_off + 3) & ~3));
    const uint32_t dlen = sr.restart_interval == 0 ? wave_destuff(p, len, sr.data_off, (uint8_t*)clean, lane) : 0u;
    const bool pipe = ps->pipe != 0;
    if (sr.level > 0 && !pipe) {  // the previous level's scans of this image (earlier tickets, running or done)
      int32_t* dn = &((PHdr*)region)->done[sr.level - 1];
      const int32_t need = hd->cnt[sr.level - 1];
      for (;;) {
        const int32_t v = __builtin_amdgcn_readfirstlane(__hip_atomic_load(dn, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT));
        if (v >= need) break;
        __builtin_amdgcn_s_sleep(4);
      }
    }
#ifdef DINO_PROG_PHASES
    const uint64_t t0 = wall_clock64();
#endif
    WaveCoefSink sink;
    sink.coef = (int16_t*)(ws + d->coef_off);
    sink.stage = (DINO_LDS int16_t*)s_stage[threadIdx.x >> 6];
    sink.lane = lane;
    sink.natk = kNaturalOrder[lane];
    sink.n = 0;
    sink.eidx = sink.eval = 0;
    sink.mlo = sink.mhi = 0;
    sink.grp = sink.nxgrp = -1;
    const bool prog = d->progressive != 0;
    if (sr.restart_interval == 0) {
      CleanReader r;
      r.init(clean, dlen, lane);
      if (prog && sr.ss > 0) {  // AC scans: one component (start_pass_phuff_decoder)
        const int ci = sr.comp[0];
        const int64_t plane = d->comp[ci].coef_off / 2;
        const int32_t bw = d->comp[ci].bw, mcx = ceil_div(d->comp[ci].dw, 8), mcy = ceil_div(d->comp[ci].dh, 8);
        ScanPipe pp{&((PHdr*)region)->prog[0], (int32_t)j, pipe ? ps->deps : ~0ull, pipe ? 0 : 0x7FFFFFFF};
        if (sr.ah > 0) fast_ac_refine(r, tb, sr, plane, bw, mcx, mcy, sink, lane, pp);
        else fast_ac_first(r, tb, sr, sink.coef, plane, bw, mcx, mcy, lane, sink.natk, pp);
      } else {
        pscan_decode(r, tb, d, sr, prog, sink);
      }
    } else {
      RawReader r;
      pb_init(r.b, (uintptr_t)p, len, sr.data_off);
      pscan_decode(r, tb, d, sr, prog, sink);
    }
#ifdef DINO_PROG_PHASES
    if (img < kProgPhaseImgs && lane == 0) {
      g_prog_phase[img][j][0] = t0;
      g_prog_phase[img][j][1] = wall_clock64();
      g_prog_phase[img][j][2] = (uint64_t)sr.level | ((uint64_t)sr.ss << 8) | ((uint64_t)sr.se << 16) |
                                ((uint64_t)sr.ah << 24) | ((uint64_t)sr.al << 28) | ((uint64_t)sr.ns << 32);
    }
#endif
    __threadfence();  // this scan's coefficient stores before its completion count
    if (lane == 0) __hip_atomic_fetch_add(&((PHdr*)region)->done[sr.level], 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
  }
}

// ---------------------------------------------------------------------------
// k_plscan + k_papply: the lane decoder of progressive images (lscan.hpp).  A one-wave
// workgroup takes tickets (scan index j, group of 64 lane images): lane i decodes scan j
// of image i of the group once every lane's image has finished the scans of the level
// before (earlier tickets, so no wait is ever on a later one).  k_papply then applies the
// deferred refinements, a lane per coefficient.
// ---------------------------------------------------------------------------
constexpr int kLLookBits = 8;                               // LDS lookahead of the scan's main table
// A lane's LDS table row: the lookahead (u16 entries), maxcode / valoffset of the lengths
// kLLookBits + 1 .. 16 and the 256 symbol bytes (the slow path of the same table); 16-byte
// aligned rows of 212 words (212 mod 64 = 20: the 64 rows start on different banks).
constexpr int kLSlowLens = 16 - kLLookBits;
constexpr int kLRowMc = (1 << kLLookBits) / 2;
constexpr int kLRowVo = kLRowMc + kLSlowLens;
constexpr int kLRowHv = kLRowVo + kLSlowLens;
constexpr int kLLookWords = 212;
static_assert(kLRowHv + 64 <= kLLookWords && kLSlowLens == 8, "lane table row");
// Per lane, in LDS as [entry][lane] (conflict-free): a ring of the scan's destuffed dwords
// and a ring of the next blocks' history masks.  Rings are refilled in wave-wide phases
// (all lanes that have room load a chunk at once, one memory wait per phase), so the decode
// steps themselves never wait on global memory: on gfx9 a load's wait also waits for every
// store issued before it, and the lanes' triggers would otherwise never line up.
#ifdef DINO_LANE_SMALL_RINGS  // (A/B: half-size rings, 79 KiB of LDS per wave instead of 103.5)
constexpr int kLRing = 64, kLChunk = 16, kLLow = 16;
constexpr int kLMRing = 16, kLMChunk = 8, kLMLow = 4;
#else
constexpr int kLRing = 128, kLChunk = 32, kLLow = 16;   // dwords (kLLow: > a DC MCU's 10 blocks x 32 bits)
constexpr int kLMRing = 32, kLMChunk = 16, kLMLow = 4;  // masks
#endif
constexpr int kPLscanLds = 64 * kLLookWords * 4 + kLRing * 64 * 4 + kLMRing * 64 * 8 + 80;

struct LaneReader {
  const DINO_GLOBAL uint32_t* src;
  DINO_LDS uint32_t* ring;  // this lane's column: dword i at ring[(i % kLRing) * 64]
  uint32_t nw, nbits, pos, wi, tail;
  uint32_t a0, a1, a2;      // dwords wi, wi + 1, wi + 2
  __device__ __forceinline__ void fill_chunk() {
    uint32_t v[kLChunk];
#pragma unroll
    for (int q = 0; q < kLChunk; ++q) v[q] = src[tail + q < nw ? tail + q : 0u];  // (always a valid address)
#pragma unroll
    for (int q = 0; q < kLChunk; ++q)
      ring[((tail + q) % kLRing) * 64] = tail + q < nw ? __builtin_bswap32(v[q]) : 0u;
    tail += kLChunk;
  }
  __device__ __forceinline__ void init(const uint32_t* s, uint32_t nbytes, DINO_LDS uint32_t* rg) {
    src = gmem(s);
    ring = rg;
    nw = (nbytes + 3) >> 2;
    nbits = nbytes * 8;
    pos = wi = tail = 0;
    fill_chunk();
    fill_chunk();
    a0 = ring[0];
    a1 = ring[64];
    a2 = ring[128];
  }
  __device__ __forceinline__ void maintain() {
    if (__ballot(tail - wi < (uint32_t)kLLow)) {  // a refill phase (the wave's active lanes)
      if (kLRing - (tail - wi) >= (uint32_t)kLChunk) fill_chunk();
    }
  }
  __device__ __forceinline__ uint32_t peek() const {
    const uint64_t x = ((uint64_t)a0 << 32 | a1) << (pos & 31);
    return (uint32_t)(x >> 32);
  }
  __device__ __forceinline__ void skip(int n) {  // n <= 32: at most one dword boundary
    pos += (uint32_t)n;
    if ((pos >> 5) != wi) {
      ++wi;
      a0 = a1;
      a1 = a2;
      a2 = ring[((wi + 2) % kLRing) * 64];
    }
  }
  __device__ __forceinline__ bool insuff() const { return pos > nbits; }
};

// Codes longer than the lookahead: the canonical-code search over lengths from .. 16 in
// the image's PTab (global), libjpeg's l = 17 fake zero when none matches.
__device__ __forceinline__ void lane_slow(const DINO_GLOBAL PTab* t, uint32_t p, int from, int* sym, int* len) {
  const uint32_t p17 = p >> 15;
  int32_t mc[8], vo[8];
#pragma unroll
  for (int q = 0; q < 8; ++q) {  // lengths 9 .. 16, loaded together
    mc[q] = t->maxcode[9 + q];
    vo[q] = t->valoffset[9 + q];
  }
  int l = 17, off = 0;
#pragma unroll
  for (int q = 7; q >= 0; --q) {  // the shortest matching length wins
    if (9 + q >= from && (int32_t)(p17 >> (17 - (9 + q))) <= mc[q]) {
      l = 9 + q;
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

// The same on the lane's LDS row (its main table's codes longer than the lookahead).
__device__ __forceinline__ void lane_slow_lds(const DINO_LDS uint32_t* row, uint32_t p, int* sym, int* len) {
  const DINO_LDS uint4* r4 = (const DINO_LDS uint4*)(row + kLRowMc);
  const uint4 m0 = r4[0], m1 = r4[1], v0 = r4[2], v1 = r4[3];  // loaded together
  const int32_t mc[8] = {(int32_t)m0.x, (int32_t)m0.y, (int32_t)m0.z, (int32_t)m0.w,
                         (int32_t)m1.x, (int32_t)m1.y, (int32_t)m1.z, (int32_t)m1.w};
  const int32_t vo[8] = {(int32_t)v0.x, (int32_t)v0.y, (int32_t)v0.z, (int32_t)v0.w,
                         (int32_t)v1.x, (int32_t)v1.y, (int32_t)v1.z, (int32_t)v1.w};
  const uint32_t p17 = p >> 15;
  int l = 17, off = 0;
#pragma unroll
  for (int q = kLSlowLens - 1; q >= 0; --q) {  // the shortest matching length wins
    if ((int32_t)(p17 >> (17 - (kLLookBits + 1 + q))) <= mc[q]) {
      l = kLLookBits + 1 + q;
      off = vo[q];
    }
  }
  *len = l;
  const int ix = ((int)(p17 >> (17 - (l > 16 ? 16 : l))) + off) & 255;
  const uint32_t h = (row[kLRowHv + (ix >> 2)] >> (8 * (ix & 3))) & 0xFFu;
  *sym = l > 16 ? 0 : (int)h;  // (l = 17: JWRN_HUFF_BAD_CODE)
}

struct LaneTabs {
  const DINO_LDS uint32_t* look;  // this lane's row: the main table (lpos) and its slow path
  int lpos;
  const PTab* tabs;
  uint64_t ts;
  const DINO_LDS uint8_t* natl;
  __device__ __forceinline__ void lookup_ac(uint32_t p, int* sym, int* len) const {  // position 4, always the row
    const uint32_t i = p >> (32 - kLLookBits);
    const uint32_t w = look[i >> 1];
    const uint32_t e = (i & 1) ? w >> 16 : w & 0xFFFFu;
    if (e) {
      *sym = (int)(e >> 4);
      *len = (int)(e & 15u);
    } else {
      lane_slow_lds(look, p, sym, len);
    }
  }
  __device__ __forceinline__ void lookup(int k, uint32_t p, int* sym, int* len) const {
    if (k == lpos) {
      lookup_ac(p, sym, len);
      return;
    }
    const DINO_GLOBAL PTab* t = gmem(tabs + pbyte64(ts, k));
    const uint32_t e = t->look[p >> (32 - kPLookBits)];
    if (e) {
      *sym = (int)(e >> 4);
      *len = (int)(e & 15u);
    } else {
      lane_slow(t, p, kPLookBits + 1, sym, len);
    }
  }
  __device__ __forceinline__ int nat(int k) const { return natl[k < 79 ? k : 79]; }
};

// Stores of a lane's scan: coefficients (first scans), the history masks (fire-and-forget
// atomic ORs), the deferred refinements (side records).  A refinement reads the next blocks'
// histories from its LDS ring.
struct LaneOut {
  DINO_GLOBAL int16_t* coef;
  uint8_t* side;
  int32_t slot;
  DINO_LDS uint2* mring;  // this lane's column: mask of block m at mring[(m % kLMRing) * 64]
  int64_t blk0;
  int32_t bw, mcx, nblk, mtail, mtx, mty;
  bool refine;
  __device__ __forceinline__ void set(int64_t e, int16_t v) { coef[e] = v; }
  __device__ __forceinline__ void fill_masks() {
    uint2 v[kLMChunk];
    int32_t x = mtx, y = mty;
#pragma unroll
    for (int q = 0; q < kLMChunk; ++q) {
      const int64_t b = mtail + q < nblk ? blk0 + (int64_t)y * bw + x : blk0;  // (always a valid address)
      v[q] = *gmem((const uint2*)(side + b * kLSideBytes));
      if (++x == mcx) {
        x = 0;
        ++y;
      }
    }
#pragma unroll
    for (int q = 0; q < kLMChunk; ++q) mring[((mtail + q) % kLMRing) * 64] = v[q];
    mtx = x;
    mty = y;
    mtail += kLMChunk;
  }
  __device__ __forceinline__ void begin_ac(int64_t b0, int32_t w, int32_t mx, int32_t n, bool ref) {
    blk0 = b0;
    bw = w;
    mcx = mx;
    nblk = n;
    refine = ref;
    mtail = mtx = mty = 0;
    if (refine) {
      fill_masks();
      fill_masks();
    }
  }
  __device__ __forceinline__ void maintain(int32_t m) {
    const bool low = refine && mtail < nblk && mtail - m < kLMLow;
    if (__ballot(low)) {  // a refill phase
      if (refine && mtail < nblk && kLMRing - (mtail - m) >= kLMChunk) fill_masks();
    }
  }
  __device__ __forceinline__ uint64_t mask(int32_t m) const {
    const uint2 v = mring[(m % kLMRing) * 64];
    return (uint64_t)v.y << 32 | v.x;
  }
  __device__ __forceinline__ void mask_or(int64_t b, uint64_t bits) {
    __hip_atomic_fetch_or((uint64_t*)(side + b * kLSideBytes), bits, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  __device__ __forceinline__ void ac_ops(int64_t b, uint64_t seq, uint64_t nzn, uint64_t neg) {
    DINO_GLOBAL uint64_t* tr = gmem((uint64_t*)(side + b * kLSideBytes + kLTripleOff + 24 * slot));
    tr[0] = seq;
    tr[1] = nzn;
    tr[2] = neg;
  }
  __device__ __forceinline__ void dc_op(int64_t b) { *gmem(side + b * kLSideBytes + kLDcOff + slot) = 1; }
};

__global__ void __launch_bounds__(64) k_plscan(const ImgDesc* __restrict__ desc, uint8_t* __restrict__ ws,
                                               PCtl* __restrict__ pctl, int prio) {
  if (prio) __builtin_amdgcn_s_setprio(3);
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  DINO_LDS uint32_t* s_look = (DINO_LDS uint32_t*)smem;
  DINO_LDS uint32_t* s_ring = s_look + 64 * kLLookWords;
  DINO_LDS uint2* s_mring = (DINO_LDS uint2*)(s_ring + kLRing * 64);
  DINO_LDS uint8_t* s_nat = (DINO_LDS uint8_t*)(s_mring + kLMRing * 64);
  const int lane = threadIdx.x;
  for (int i = lane; i < 80; i += 64) s_nat[i] = kNaturalOrder[i];
  __syncthreads();
  const uint32_t nlane = pctl->nlane, cap = pctl->cap;
  if (nlane == 0) return;
  const uint32_t ngroups = (nlane + 63) / 64;
  const uint32_t total = ngroups * pctl->lmax_scans;
  DINO_LDS uint32_t* row = s_look + lane * kLLookWords;
  for (;;) {
    uint32_t tk = 0;
    if (lane == 0) tk = atomicAdd(&pctl->lticket, 1u);
    tk = (uint32_t)__builtin_amdgcn_readfirstlane((int32_t)__shfl(tk, 0));
    if (tk >= total) break;
    const uint32_t j = tk / ngroups, g = tk - j * ngroups;
    const uint32_t li = g * 64 + (uint32_t)lane;
    const int img = li < nlane ? pctl->pimg[cap - 1 - li] : -1;
    const ImgDesc* d = desc + (img >= 0 ? img : 0);
    uint8_t* region = ws + d->htab_off;
    PHdr* hd = (PHdr*)region;
    const bool act = img >= 0 && (int)j < hd->n_scans;
    PScan ps;
    if (act) ps = ((const PScan*)(region + kPScanOff))[j];
    const ScanRec& sr = ps.sr;
    const PTab* tabs = (const PTab*)(region + kPTabOff);
    // the scan's main table (AC: position 4, DC: position 0) into the lane's LDS row, as
    // kLLookBits-bit entries (codes of <= kLLookBits bits, else 0) + its slow-path arrays
    const int lpos = act && sr.ss > 0 ? 4 : 0;
    const int tsl = act ? pbyte64(ps.tslots, lpos) : 0xFF;
    if (tsl != 0xFF) {
      const DINO_GLOBAL uint4* src = gmem((const uint4*)tabs[tsl].look);
#pragma unroll 8
      for (int q = 0; q < (1 << kPLookBits) / 8; ++q) {  // 8 entries of the 9-bit table -> 4 of ours
        const uint4 v = src[q];
        uint32_t e[4] = {v.x & 0xFFFFu, v.y & 0xFFFFu, v.z & 0xFFFFu, v.w & 0xFFFFu};
#pragma unroll
        for (int k = 0; k < 4; ++k) e[k] = (e[k] & 15u) <= (uint32_t)kLLookBits ? e[k] : 0u;
        row[2 * q] = e[0] | e[1] << 16;
        row[2 * q + 1] = e[2] | e[3] << 16;
      }
      const DINO_GLOBAL PTab* tg = gmem(tabs + tsl);
#pragma unroll
      for (int q = 0; q < kLSlowLens; ++q) {
        row[kLRowMc + q] = (uint32_t)tg->maxcode[kLLookBits + 1 + q];
        row[kLRowVo + q] = (uint32_t)tg->valoffset[kLLookBits + 1 + q];
      }
#pragma unroll 8
      for (int q = 0; q < 64; ++q) row[kLRowHv + q] = tg->huffval[q];
    }
    // wait for the previous level of every lane's image (earlier tickets)
    for (;;) {
      bool ready = true;
      if (act && sr.level > 0)
        ready = __hip_atomic_load(&hd->done[sr.level - 1], __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT) >=
                hd->cnt[sr.level - 1];
      if (!__ballot(!ready)) break;
      __builtin_amdgcn_s_sleep(8);
    }
#ifdef DINO_PROG_PHASES
    const uint64_t t0 = wall_clock64();
#endif
    if (act) {
      LaneReader r;
      r.init((const uint32_t*)(ws + d->ent_off + ((sr.data_off - d->scan_off + 3) & ~3)), (uint32_t)ps.dlen,
             s_ring + lane);
      LaneTabs t{(const DINO_LDS uint32_t*)row, tsl != 0xFF ? lpos : -1, tabs, ps.tslots,
                 (const DINO_LDS uint8_t*)s_nat};
      LaneOut o;
      o.coef = gmem((int16_t*)(ws + d->coef_off));
      o.side = ws + d->binfo_off;
      o.slot = ps.slot;
      o.mring = s_mring + lane;
      o.refine = false;
      lane_scan_decode(r, t, d, sr, o);
#ifdef DINO_PROG_PHASES
      if (img < kProgPhaseImgs) {
        g_prog_phase[img][j][0] = t0;
        g_prog_phase[img][j][1] = wall_clock64();
        g_prog_phase[img][j][2] = (uint64_t)sr.level | ((uint64_t)sr.ss << 8) | ((uint64_t)sr.se << 16) |
                                  ((uint64_t)sr.ah << 24) | ((uint64_t)sr.al << 28) | ((uint64_t)sr.ns << 32);
      }
#endif
      __threadfence();  // this scan's stores before its completion count
      __hip_atomic_fetch_add(&hd->done[sr.level], 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
}

// The deferred refinements (lane_apply_block), data-parallel: a wave per block, lane k =
// zigzag coefficient k.  Grid (x, lane image).
constexpr int kPApplyWgs = 16;
__global__ void __launch_bounds__(256) k_papply(const ImgDesc* __restrict__ desc, uint8_t* __restrict__ ws,
                                                const PCtl* __restrict__ pctl) {
  const uint32_t k = blockIdx.y;
  if (k >= pctl->nlane) return;
  const int img = pctl->pimg[pctl->cap - 1 - k];
  const ImgDesc& d = desc[img];
  const PHdr* hd = (const PHdr*)(ws + d.htab_off);
  const uint32_t nac = hd->lane_nac, ndc = hd->lane_ndc, al_dc = hd->lane_al_dc;
  const uint64_t al_ac = hd->lane_al_ac;
  const uint64_t band_ac[3] = {hd->lane_band[0], hd->lane_band[1], hd->lane_band[2]};
  if (nac == 0 && ndc == 0) return;
  const int lane = threadIdx.x & 63;
  const int pos = kNaturalOrder[lane];
  const int64_t nb0 = (int64_t)d.comp[0].bw * d.comp[0].bh;
  const int64_t nb1 = d.ncomp > 1 ? (int64_t)d.comp[1].bw * d.comp[1].bh : 0;
  const int64_t nblk = d.coef_bytes / 128;
  int16_t* coef = (int16_t*)(ws + d.coef_off);
  const uint8_t* side = ws + d.binfo_off;
  const int64_t step = (int64_t)gridDim.x * (blockDim.x >> 6);
  for (int64_t b = (int64_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6); b < nblk; b += step) {
    const int c = b < nb0 ? 0 : (b < nb0 + nb1 ? 1 : 2);
    const int na = (int)((nac >> (4 * c)) & 15u);
    const uint8_t* sd = side + b * kLSideBytes;
    const int16_t v0 = coef[b * 64 + pos];
    int16_t v = v0;
    const uint64_t bw = c == 0 ? band_ac[0] : (c == 1 ? band_ac[1] : band_ac[2]);
    for (int s = 0; s < na; ++s) {
      const uint64_t* tr = (const uint64_t*)(sd + kLTripleOff + 24 * s);
      const uint64_t seq = tr[0], nzn = tr[1], neg = tr[2];
      const int bd = (int)((bw >> (12 * s)) & 0xFFFu), ss = bd & 63, se = bd >> 6;
      // correction bit j of the sequence -> the band's j-th coefficient non-zero so far
      const bool hist = v != 0 && lane >= ss && lane <= se;
      const uint64_t hm = __ballot(hist);
      const uint32_t j = lane_rank(hm);
      const bool corr = hist && ((seq >> ((63 - j) & 63)) & 1u);
      v = ac_refine_value(v, corr, (nzn >> lane) & 1u, (neg >> lane) & 1u, (int)((al_ac >> (16 * c + 4 * s)) & 15u));
    }
    if (lane == 0)
      for (int s = 0; s < (int)ndc; ++s)
        if (sd[kLDcOff + s]) v = (int16_t)(v | (1 << ((al_dc >> (4 * s)) & 15u)));
    if (v != v0) coef[b * 64 + pos] = v;
  }
}

// ---------------------------------------------------------------------------
// k_dcscan: DC predictors of a speculatively decoded image (no restart
// intervals): per-component running sums of the DC differences k_huffman left
// in decode order (the high half of each block record), replaced in place by the
// absolute (int16) DC values.  One workgroup per image, tiles of 2048 blocks.
// ---------------------------------------------------------------------------
constexpr int kDcScanThreads = 256;

__global__ void __launch_bounds__(kDcScanThreads) k_dcscan(const ImgDesc* __restrict__ desc, uint8_t* __restrict__ ws) {
  main_prio();
  constexpr int K = 8;  // blocks per lane per tile: a wave covers 512 consecutive blocks
  __shared__ uint32_t s_wave[kDcScanThreads / 64];
  const ImgDesc& d = desc[blockIdx.x];
  if (d.status != DINO_IMG_OK || d.kind != 0 || d.restart_interval > 0) return;
  const int T = d.total_blocks, bpm = d.blocks_per_mcu;
  uint32_t mc = 0;
  for (int i = 0; i < bpm && i < kMaxBlocksPerMcu; ++i) mc |= (uint32_t)(d.mcu_comp[i] & 3) << (2 * i);
  // the .y word of each block's record: (int16 DC << 16) | entry count
  uint32_t* info = (uint32_t*)(ws + d.binfo_off) + 1;
  int32_t carry[kMaxComp] = {0, 0, 0};
  for (int t0 = 0; t0 < T; t0 += kDcScanThreads * K) {
    // a tile: lane t owns K consecutive blocks, so each lane's loads and stores fill
    // its own 64-byte span at once (no partially written lines left behind)
    const int b0 = t0 + (int)threadIdx.x * K;
    uint32_t y[K];
#pragma unroll
    for (int j = 0; j < K; ++j) y[j] = b0 + j < T ? info[2 * (int64_t)(b0 + j)] : 0u;
    const int pos0 = b0 % bpm;
    int32_t s[kMaxComp] = {0, 0, 0};
    int pos = pos0;
#pragma unroll
    for (int j = 0; j < K; ++j) {
      add3(s, (int)((mc >> (2 * pos)) & 3u), (int32_t)y[j] >> 16);
      pos = pos + 1 == bpm ? 0 : pos + 1;
    }
    uint32_t tot[kMaxComp];
    int32_t pfx[kMaxComp];
#pragma unroll
    for (int c = 0; c < kMaxComp; ++c)
      pfx[c] = carry[c] + (int32_t)block_excl_scan<kDcScanThreads>((uint32_t)s[c], s_wave, &tot[c]);
    pos = pos0;
#pragma unroll
    for (int j = 0; j < K; ++j) {
      const int c = (int)((mc >> (2 * pos)) & 3u);
      add3(pfx, c, (int32_t)y[j] >> 16);
      // in place: JCOEF (int16) DC, as libjpeg stores it; a zero block after the data
      // ran out (kBinfoAbsDc, always the image's tail) keeps its absolute 0
      if (b0 + j < T && !(y[j] & kBinfoAbsDc)) info[2 * (int64_t)(b0 + j)] = (y[j] & 0xFFFFu) | ((uint32_t)get3(pfx, c) << 16);
      pos = pos + 1 == bpm ? 0 : pos + 1;
    }
#pragma unroll
    for (int c = 0; c < kMaxComp; ++c) carry[c] += (int32_t)tot[c];
  }
}

// ---------------------------------------------------------------------------
// k_idct: grid (gx, B); lanes over the 8x8 blocks of one image
// ---------------------------------------------------------------------------
// 8 lanes per 8x8 block, blocks in component-plane raster order (so that a wave's
// output rows are 8 blocks = 64 contiguous bytes of a plane row).  The group reads
// the block's decode-order index, its sparse entries (binfo, see SparseSink) and
// DC, zeroes the LDS block and scatters the entries (lane l takes entries l, l+8,
// ...), then lane l dequantizes + runs pass 1 on column l and pass 2 on row l, and
// stores output row l as one 8-byte word.
constexpr int kIdctBlocksPerWg = 32;

// A wave's 8 blocks live only in its own 8 LDS slots, so the steps of one block need
// no workgroup barrier: a wave's LDS operations execute in issue order, and the
// wavefront-scope fences keep the compiler from moving LDS accesses across this point.
__device__ __forceinline__ void wave_lds_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

#ifndef DINO_IDCT_WGS
#define DINO_IDCT_WGS 32
#endif
constexpr int kIdctWgs = DINO_IDCT_WGS;  // workgroups per image (grid-stride over its blocks)

// The steps of one 8-lane group's block (k_idct).  sb: the group's LDS block,
// rows of 9 words, all zero on entry.
// Dense coefficients (kind 1): lane l loads row l of the block (8 int16 = one 16-byte load).
__device__ __forceinline__ void idct_group_dense(int32_t* sb, int l, const uint8_t* blk) {
  const uint4 q = *(const uint4*)(blk + l * 16);
  const uint32_t w4[4] = {q.x, q.y, q.z, q.w};
#pragma unroll
  for (int j = 0; j < 8; ++j) sb[l * 9 + j] = (int32_t)(int16_t)(w4[j >> 1] >> (16 * (j & 1)));
}
// Sparse entries (kind 0): the block record bi and the block's halfword entries
// l, l + 8, .. (kIdctPre of them) already loaded into pre[]; halfword entries
// (zigzag | int10 value << 6), then u32 entries from the next even halfword (see
// SparseSink); the DC is int16 (absolute after k_dcscan).
#ifndef DINO_IDCT_PRE
#define DINO_IDCT_PRE 4
#endif
constexpr int kIdctPre = DINO_IDCT_PRE;  // halfword entries per lane loaded a block ahead (8 lanes: 8 kIdctPre)
__device__ __forceinline__ void idct_load_pre(uint32_t* pre, int l, uint2 bi, const uint16_t* ent16) {
  const uint32_t c = bi.y & 0x7Fu;
#pragma unroll
  for (int m = 0; m < kIdctPre; ++m) pre[m] = l + 8 * m < (int)c ? ent16[bi.x + l + 8 * m] : 0u;
}
__device__ __forceinline__ void idct_group_sparse(int32_t* sb, int l, const uint8_t* s_nat, uint2 bi, const uint32_t* pre,
                                                  const uint16_t* ent16, const uint32_t* ent) {
  if (l == 0) sb[0] = (int32_t)bi.y >> 16;
  const uint32_t c16 = bi.y & 0x7Fu, c32 = (bi.y >> 7) & 0x7Fu;
#pragma unroll
  for (int m = 0; m < kIdctPre; ++m)
    if (l + 8 * m < (int)c16) sb[s_nat[pre[m] & 63u]] = (int32_t)(int16_t)pre[m] >> 6;
  for (uint32_t j = l + 8 * kIdctPre; j < c16; j += 8) {
    const uint32_t h = ent16[bi.x + j];
    sb[s_nat[h & 63u]] = (int32_t)(int16_t)h >> 6;
  }
  const uint32_t* e32 = ent + ((bi.x + c16 + 1) >> 1);
  for (uint32_t j = l; j < c32; j += 8) {
    const uint32_t e = e32[j];
    sb[s_nat[e & 63u]] = (int32_t)(int16_t)(e >> 16);
  }
}
// Dequantize + pass 1 on column l (reads and writes only this lane's column).
__device__ __forceinline__ void idct_group_pass1(int32_t* sb, int l, const uint16_t* q) {
  int32_t raw[8], qq[8], wcol[8];
  bool acz = true;  // rows 1..7 of this column are zero
#pragma unroll
  for (int r = 0; r < 8; ++r) {
    raw[r] = sb[r * 9 + l];
    qq[r] = (int32_t)(int16_t)q[r * 8 + l];
    if (r) acz = acz && raw[r] == 0;
  }
  // libjpeg-turbo's SIMD pass 1 decides its DC-only shortcut for the whole block
  const int gsh = threadIdx.x & 56;  // this group's first lane within the wave
  idct_pass1(raw, qq, ((__ballot(acz) >> gsh) & 0xFFu) == 0xFFu, wcol);
#pragma unroll
  for (int r = 0; r < 8; ++r) sb[r * 9 + l] = wcol[r];
}
// Pass 2 on row l: returns output row l (8 samples); the row is cleared for the next block.
__device__ __forceinline__ uint64_t idct_group_pass2(int32_t* sb, int l) {
  int32_t row[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) row[j] = sb[l * 9 + j];
#pragma unroll
  for (int j = 0; j < 8; ++j) sb[l * 9 + j] = 0;
  union {
    uint8_t b[8];
    uint64_t u;
  } o;
  idct_pass2(row, o.b);
  return o.u;
}

__global__ void __launch_bounds__(256) k_idct(const ImgDesc* __restrict__ desc, uint8_t* __restrict__ ws) {
  const BlkIdx bk = xcd_blk();
  // rows of 9 words, blocks 72 words apart: both the column (pass 1) and the row
  // (pass 2) accesses of a wave's 8 groups x 8 lanes hit 64 distinct banks
  __shared__ int32_t s_blk[kIdctBlocksPerWg][72];
  __shared__ uint8_t s_nat[80];
  const ImgDesc& d = desc[bk.y];
  if (d.status != DINO_IMG_OK || d.kind == 2) return;
  // kind 1 (progressive / multi-scan): dense int16 coefficients in natural order,
  // component planes of bw x bh blocks (k_prog); kind 0: sparse entries + block records
  const bool dense = d.kind == 1;
  if (threadIdx.x < 80) s_nat[threadIdx.x] = (uint8_t)((kNaturalOrder[threadIdx.x] >> 3) * 9 + (kNaturalOrder[threadIdx.x] & 7));
  const int ncomp = d.ncomp;
  const int64_t nb0 = (int64_t)d.comp[0].bw * d.comp[0].bh;
  const int64_t nb1 = ncomp > 1 ? (int64_t)d.comp[1].bw * d.comp[1].bh : 0;
  const int64_t nb2 = ncomp > 2 ? (int64_t)d.comp[2].bw * d.comp[2].bh : 0;
  const int64_t tot = nb0 + nb1 + nb2;
  const uint32_t* ent = (const uint32_t*)(ws + d.coef_off);
  const uint2* binfo = (const uint2*)(ws + d.binfo_off);
  uint8_t* planes = ws + d.plane_off;
  // first position of each component inside the MCU (interleaved scans)
  int moff[kMaxComp] = {0, 0, 0};
  for (int i = d.blocks_per_mcu - 1; i >= 0; --i) {
    const int c = d.mcu_comp[i];
    if (c == 0) moff[0] = i;
    else if (c == 1) moff[1] = i;
    else moff[2] = i;
  }
  const int grp = threadIdx.x >> 3, l = threadIdx.x & 7;
  int32_t* sb = s_blk[grp];
  // plane block g -> component, position and decode-order index (32-bit: a plane has < 2^31 blocks);
  // a plane block no MCU covers has b = -1 and stays all zero
  struct Blk {
    int c, bx, by, b;
  };
  auto locate = [&](int g) {
    Blk r;
    r.c = g < nb0 ? 0 : (g < nb0 + nb1 ? 1 : 2);
    const int k = g - (r.c == 0 ? 0 : (r.c == 1 ? (int)nb0 : (int)(nb0 + nb1)));
    const CompDesc& cd = d.comp[r.c];
    r.by = k / cd.bw;
    r.bx = k - r.by * cd.bw;
    if (ncomp == 1) {
      r.b = r.bx < d.mcus_x ? r.by * d.mcus_x + r.bx : -1;
    } else {
      const int mo = r.c == 0 ? moff[0] : (r.c == 1 ? moff[1] : moff[2]);
      const int my = r.by / cd.v, mx = r.bx / cd.h;
      r.b = (my * d.mcus_x + mx) * d.blocks_per_mcu + mo + (r.by - my * cd.v) * cd.h + (r.bx - mx * cd.h);
    }
    return r;
  };
  const int T = (int)tot, step = gridDim.x * kIdctBlocksPerWg;
  // The next block's record is loaded one iteration ahead, and its first 16 entries
  // at the end of the current iteration (once the record has arrived), so the
  // scatter at the top of an iteration normally waits on nothing.
  int gn = bk.x * kIdctBlocksPerWg + grp;
  Blk nx = locate(gn < T ? gn : 0);
  uint2 bin = make_uint2(0u, 0u);
  if (!dense && gn < T && nx.b >= 0 && nx.b < d.total_blocks) bin = binfo[nx.b];
  const uint16_t* ent16 = (const uint16_t*)ent;
  uint32_t pre[kIdctPre] = {};  // the next block's first halfword entries (l, l + 8, ..)
  auto first_entries = [&]() {
    if (!dense) idct_load_pre(pre, l, bin, ent16);
  };
  if (gn < T) first_entries();
#pragma unroll
  for (int j = 0; j < 8; ++j) sb[l * 9 + j] = 0;
  __syncthreads();
  for (int g0 = bk.x * kIdctBlocksPerWg; g0 < T; g0 += step) {
    const bool valid = gn < T;
    const Blk cur = nx;
    const uint2 bi = bin;
    gn += step;
    if (gn < T) {  // prefetch the next block's record while this one is transformed
      nx = locate(gn);
      bin = make_uint2(0u, 0u);
      if (!dense && nx.b >= 0 && nx.b < d.total_blocks) bin = binfo[nx.b];
    }
    if (valid && dense) {
      const CompDesc& cc = d.comp[cur.c];
      idct_group_dense(sb, l, ws + d.coef_off + cc.coef_off + ((int64_t)cur.by * cc.bw + cur.bx) * 128);
    } else if (valid) {
      idct_group_sparse(sb, l, s_nat, bi, pre, ent16, ent);
    }
    wave_lds_sync();
    const CompDesc& cd = d.comp[cur.c];
    if (valid) idct_group_pass1(sb, l, d.qt[cd.tq]);
    wave_lds_sync();
    if (valid) {
      const int pitch = cd.bw * 8;
      *(uint64_t*)(planes + cd.plane_off + ((int64_t)cur.by * 8 + l) * pitch + cur.bx * 8) = idct_group_pass2(sb, l);
    }
    if (gn < T) first_entries();
    wave_lds_sync();
  }
}

// ---------------------------------------------------------------------------
// k_color: grid (gx, B); lanes over output pixels
// ---------------------------------------------------------------------------
__device__ __forceinline__ PlaneView make_plane_view(const ImgDesc& d, const uint8_t* ws, int c) {
  const CompDesc& cd = d.comp[c];
  PlaneView v;
  v.p = ws + d.plane_off + cd.plane_off;
  v.pitch = cd.bw * 8;
  v.dw = cd.dw;
  v.dh = cd.dh;
  v.hf = d.max_h / cd.h;
  v.vf = d.max_v / cd.v;
  v.method = upsample_method(v.hf, v.vf, cd.dw);
  return v;
}

// (k_color reads 4 bytes at row[s] as two aligned words + v_alignbyte: the second word
// may lie past the row, planes are followed by more workspace, never unmapped.)

// h2v2 fancy upsampling of one chroma plane for the 4 pixels x0..x0+3 of row y,
// given the samples [c0-1, c0+2] of the nearer row (n) and the farther row (f).
// edge: bit 0 column c0-1 is left of the plane, bits 1 / 2 columns c0+1 / c0+2 are
// right of it; such a column is the clamp of its neighbour (jdsample.c's first and
// last column formulas), whatever bytes were loaded for it.
__device__ __forceinline__ void h2v2_quad(uint32_t n, uint32_t f, int x0, uint32_t edge, int* out) {
  int cs[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) cs[j] = 3 * (int)((n >> (8 * j)) & 255u) + (int)((f >> (8 * j)) & 255u);
  if (edge & 1u) cs[0] = cs[1];
  if (edge & 2u) cs[2] = cs[1];
  if (edge & 4u) cs[3] = cs[2];
  // an even pixel x blends column x/2 with its left neighbour ((3a + b + 8) >> 4), an odd
  // one with its right neighbour ((3a + b + 7) >> 4); with cs[1] = column x0/2 the four
  // pixels use fixed columns for each parity of x0 (no dynamically indexed cs)
  const int e0 = (cs[1] * 3 + cs[0] + 8) >> 4, e1 = (cs[1] * 3 + cs[2] + 7) >> 4;
  const int e2 = (cs[2] * 3 + cs[1] + 8) >> 4, e3 = (cs[2] * 3 + cs[3] + 7) >> 4;
  const int o3 = (cs[3] * 3 + cs[2] + 8) >> 4;
  const bool odd = x0 & 1;
  out[0] = odd ? e1 : e0;
  out[1] = odd ? e2 : e1;
  out[2] = odd ? e3 : e2;
  out[3] = odd ? o3 : e3;
}

#ifndef DINO_COLOR_WGS
#define DINO_COLOR_WGS 16
#endif
constexpr int kColorWgs = DINO_COLOR_WGS;  // workgroups per image
#ifndef DINO_COLOR_BATCH
#define DINO_COLOR_BATCH 1
#endif
constexpr int kColorBatch = DINO_COLOR_BATCH;  // quads whose loads a lane issues together (measured: 4 and 8 slower)

// Four consecutive pixels per lane (12 output bytes = three aligned dword stores;
// the RGB area is padded by 16 bytes, so the last partial quad may store whole words).
// 4:2:0 interior quads (the common case) take a vectorised path: one word of Y and
// two words per chroma row instead of per-pixel byte loads; edges, quads that wrap
// a row and other samplings use the per-pixel path (same arithmetic).
__global__ void __launch_bounds__(256) k_color(const uint8_t* __restrict__ bytes, const int64_t* __restrict__ offsets,
                                               const ImgDesc* __restrict__ desc, uint8_t* __restrict__ ws) {
  const BlkIdx bk = xcd_blk();
  const ImgDesc& d = desc[bk.y];
  if (d.status != DINO_IMG_OK) return;
  if (d.kind == 2) {  // pre-decoded RGB container: copy the pixels into the workspace
    const uint8_t* src = bytes + offsets[bk.y] + d.scan_off;
    uint32_t* dst = (uint32_t*)(ws + d.rgb_off);
    const int64_t n = (int64_t)d.width * d.height * 3, nw = (n + 3) >> 2;
    for (int64_t q = (int64_t)bk.x * blockDim.x + threadIdx.x; q < nw; q += (int64_t)gridDim.x * blockDim.x) {
      uint32_t w = 0;
#pragma unroll
      for (int j = 0; j < 4; ++j)
        if (4 * q + j < n) w |= (uint32_t)src[4 * q + j] << (8 * j);
      dst[q] = w;
    }
    return;
  }
  const int nc = d.ncomp;
  const PlaneView p0 = make_plane_view(d, ws, 0);
  const PlaneView p1 = nc > 1 ? make_plane_view(d, ws, 1) : p0;
  const PlaneView p2 = nc > 1 ? make_plane_view(d, ws, 2) : p0;
  const bool ycc = nc > 1 && d.color == kYCbCr;
  const bool fast420 = ycc && p0.method == kUpFull && p1.method == kUpH2V2Fancy && p2.method == kUpH2V2Fancy &&
                       p1.dw == p2.dw && p1.dh == p2.dh;
  uint32_t* rgb = (uint32_t*)(ws + d.rgb_off);
  const int W = d.width;
  const int64_t npx = (int64_t)W * d.height;
  const int64_t nq = (npx + 3) >> 2;  // npx < 2^31 (max_image_dim <= 16384 is enforced by k_parse limits)
  // (y, x) of the lane's first quad by one division; later quads advance by the
  // stride (dy rows + dx pixels) without dividing again.
#ifdef DINO_COLOR_STRIDED
  // grid-strided: workgroup x takes every gridDim.x-th run of 256 quads
  const int64_t q0 = (int64_t)bk.x * blockDim.x + threadIdx.x, qs = (int64_t)gridDim.x * blockDim.x;
  const int64_t qend = nq;
#else
  // one contiguous band of rows per workgroup: the chroma rows an output row pair shares
  // with its neighbours are read by the same workgroup (one XCD's L2) instead of by up to
  // five workgroups on different XCDs, each fetching them again
  const int64_t band = ((nq + gridDim.x - 1) / gridDim.x + blockDim.x - 1) / blockDim.x * blockDim.x;
  const int64_t q0 = (int64_t)bk.x * band + threadIdx.x, qs = blockDim.x;
  const int64_t qend = min(nq, (int64_t)(bk.x + 1) * band);
#endif
  const uint32_t pstride = (uint32_t)(qs * 4);
  const int dy = (int)(pstride / (uint32_t)W), dx = (int)(pstride - (uint32_t)dy * (uint32_t)W);
  int yq = (int)((uint32_t)(q0 * 4) / (uint32_t)W), xq = (int)((uint32_t)(q0 * 4) - (uint32_t)yq * (uint32_t)W);
  // kColorBatch quads per lane per iteration: every load of the batch is issued before
  // any of its quads is converted (the RGB stores may alias the planes for the compiler,
  // so it would not move the next quad's loads above this quad's stores by itself)
  for (int64_t qb = q0; qb < qend; qb += kColorBatch * qs) {
    int ys[kColorBatch], xs[kColorBatch];
    bool fast[kColorBatch];
    uint32_t yw0[kColorBatch], yw1[kColorBatch], cw[kColorBatch][8];
#pragma unroll
    for (int k = 0; k < kColorBatch; ++k) {
      const int y = yq, x = xq;
      ys[k] = y;
      xs[k] = x;
      xq += dx;
      yq += dy;
      if (xq >= W) {
        xq -= W;
        ++yq;
      }
      // every 4:2:0 quad inside one row (row edges included: the fancy upsampler's edge
      // columns are clamps, applied to the loaded samples below) takes the vector path;
      // a lane on the generic per-pixel path would make its whole wave run that too
      fast[k] = fast420 && qb + k * qs < qend && x + 3 < W;
      if (fast[k]) {  // raw words: Y at x, Cb / Cr at column x/2 - 1 of the nearer and the farther row
        const int r = y >> 1;
        const int rf = (y & 1) ? min(r + 1, p1.dh - 1) : max(r - 1, 0);
        const int cc = (x >> 1) - 1;
        const uint32_t* yp = (const uint32_t*)(p0.p + (int64_t)y * p0.pitch + (x & ~3));
        yw0[k] = yp[0];
        yw1[k] = yp[1];
        const uint32_t* cp[4] = {(const uint32_t*)(p1.p + (int64_t)r * p1.pitch + (cc & ~3)),
                                 (const uint32_t*)(p1.p + (int64_t)rf * p1.pitch + (cc & ~3)),
                                 (const uint32_t*)(p2.p + (int64_t)r * p2.pitch + (cc & ~3)),
                                 (const uint32_t*)(p2.p + (int64_t)rf * p2.pitch + (cc & ~3))};
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          cw[k][2 * j] = cp[j][0];
          cw[k][2 * j + 1] = cp[j][1];
        }
      }
    }
#pragma unroll
    for (int k = 0; k < kColorBatch; ++k) {
      const int64_t q = qb + k * qs;
      if (q >= qend) break;
      int y = ys[k], x = xs[k];
      const int64_t i0 = q * 4;
      union {
        uint8_t b[12];
        uint32_t w[3];
      } o;
      if (fast[k]) {
        const int c0 = x >> 1;
        const uint32_t csh = (uint32_t)((c0 - 1) & 3);
        const uint32_t yw = __builtin_amdgcn_alignbyte(yw1[k], yw0[k], (uint32_t)(x & 3));
        const uint32_t edge = (c0 == 0 ? 1u : 0u) | (c0 + 1 >= p1.dw ? 2u : 0u) | (c0 + 2 >= p1.dw ? 4u : 0u);
        int cb[4], cr[4];
        h2v2_quad(__builtin_amdgcn_alignbyte(cw[k][1], cw[k][0], csh), __builtin_amdgcn_alignbyte(cw[k][3], cw[k][2], csh),
                  x, edge, cb);
        h2v2_quad(__builtin_amdgcn_alignbyte(cw[k][5], cw[k][4], csh), __builtin_amdgcn_alignbyte(cw[k][7], cw[k][6], csh),
                  x, edge, cr);
#pragma unroll
        for (int j = 0; j < 4; ++j) ycc_to_rgb((int)((yw >> (8 * j)) & 255u), cb[j], cr[j], o.b + 3 * j);
      } else if (fast420) {  // a 4:2:0 quad that wraps a row: per pixel, same arithmetic
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          if (i0 + j < npx) {
            const int r = y >> 1, c = x >> 1;
            const int rn = (y & 1) ? min(r + 1, p1.dh - 1) : max(r - 1, 0);
            const int cn = (x & 1) ? min(c + 1, p1.dw - 1) : max(c - 1, 0);
            const int bias = (x & 1) ? 7 : 8;
            const int tb = pv_at(p1, c, r) * 3 + pv_at(p1, c, rn), nb = pv_at(p1, cn, r) * 3 + pv_at(p1, cn, rn);
            const int tr = pv_at(p2, c, r) * 3 + pv_at(p2, c, rn), nr = pv_at(p2, cn, r) * 3 + pv_at(p2, cn, rn);
            ycc_to_rgb(pv_at(p0, x, y), (tb * 3 + nb + bias) >> 4, (tr * 3 + nr + bias) >> 4, o.b + 3 * j);
          } else {
            o.b[3 * j] = o.b[3 * j + 1] = o.b[3 * j + 2] = 0;
          }
          if (++x == W) {
            x = 0;
            ++y;
          }
        }
      } else {
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          if (i0 + j < npx) {
            if (nc == 1) {
              const uint8_t v = (uint8_t)upsample_at(p0, x, y);
              o.b[3 * j] = o.b[3 * j + 1] = o.b[3 * j + 2] = v;
            } else {
              const int a = upsample_at(p0, x, y), b = upsample_at(p1, x, y), c = upsample_at(p2, x, y);
              if (ycc) {
                ycc_to_rgb(a, b, c, o.b + 3 * j);
              } else {
                o.b[3 * j] = (uint8_t)a;
                o.b[3 * j + 1] = (uint8_t)b;
                o.b[3 * j + 2] = (uint8_t)c;
              }
            }
          } else {
            o.b[3 * j] = o.b[3 * j + 1] = o.b[3 * j + 2] = 0;
          }
          if (++x == W) {
            x = 0;
            ++y;
          }
        }
      }
      rgb[3 * q] = o.w[0];
      rgb[3 * q + 1] = o.w[1];
      rgb[3 * q + 2] = o.w[2];
    }
  }
}

// ---------------------------------------------------------------------------
// Augment half
// ---------------------------------------------------------------------------
__global__ void k_params(const ImgDesc* __restrict__ desc, int B, dino_aug_config cfg, uint64_t seed,
                         uint64_t batch_index, dino_view_params* __restrict__ out) {
  const int nv = cfg.n_global + cfg.n_local;
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= B * nv) return;
  int b = i / nv, v = i - b * nv;
  const ImgDesc& d = desc[b];
  int ok = d.status == DINO_IMG_OK;
  if (!ok && d.status < 0 && cfg.recipe == DINO_RECIPE_LEJEPA) {
    // CPULeJEPAPipeline (cpu.py:446-448) crops an undecodable image's views from a black
    // 224 x 224 canvas: the draws are those of that canvas (k_final writes its values)
    sample_view(cfg, seed, batch_index, b, v, 224, 224, 1, &out[i]);
    return;
  }
  sample_view(cfg, seed, batch_index, b, v, ok ? d.width : 1, ok ? d.height : 1, ok, &out[i]);
}

// Resample target of a view's crop box (0 in the record means the view size S).
__device__ __forceinline__ int view_rw(const dino_view_params& p) { return p.resize_w > 0 ? p.resize_w : p.out_size; }
__device__ __forceinline__ int view_rh(const dino_view_params& p) { return p.resize_h > 0 ? p.resize_h : p.out_size; }

// Scratch of one view (plan.hpp view_scratch_bytes); 0 when the view is not rendered.
__device__ void view_sizes(const dino_view_params& p, int ok, int64_t* bytes, int32_t* kh, int32_t* kv) {
  *kh = ok && p.crop_w != view_rw(p) ? resample_ksize(p.crop_w, view_rw(p)) : 0;
  *kv = ok && p.crop_h != view_rh(p) ? resample_ksize(p.crop_h, view_rh(p)) : 0;
  *bytes = ok ? view_scratch_bytes(p.out_size, p.crop_w, p.crop_h, *kh, *kv) : 0;
}

// Host-supplied records are validated before any kernel indexes memory with them.
__device__ bool params_valid(const dino_view_params& p, const ImgDesc& d, int S) {
  if (p.out_size != S) return false;
  if (p.crop_top < 0 || p.crop_left < 0 || p.crop_h < 1 || p.crop_w < 1) return false;
  if ((int64_t)p.crop_top + p.crop_h > d.height || (int64_t)p.crop_left + p.crop_w > d.width) return false;
  if (p.blur && (p.ksize < 1 || p.ksize > 15 || (p.ksize & 1) == 0 || !(p.sigma > 0.0) || p.ksize / 2 >= S))
    return false;  // torch reflect padding needs pad < S
  for (int k = 0; k < 4; ++k)
    if (p.order[k] > 3) return false;
  // window of the resampled box: inside it, and an axis that is not resampled has no window
  const int rw = view_rw(p), rh = view_rh(p);
  if (rw < S || rh < S || rw > 65536 || rh > 65536 || p.out_x < 0 || p.out_y < 0) return false;
  if (p.out_x + S > rw || p.out_y + S > rh) return false;
  if (p.crop_w == rw && (rw != S || p.out_x != 0)) return false;
  if (p.crop_h == rh && (rh != S || p.out_y != 0)) return false;
  return true;
}

__device__ int hr_view_chunks(int S, int cw, int ch, int kh);

// k_vsizes: one lane per view: validity and scratch bytes into plan[i] (htmp_off holds
// the size and rcoef_off the offset of the coefficient tables inside it until k_vplan
// places the view), so that the single-workgroup scan only reads packed records.
__global__ void __launch_bounds__(256) k_vsizes(const ImgDesc* __restrict__ desc, const dino_view_params* __restrict__ prm,
                                                int B, int nv, int n_global, int gsize, int lsize,
                                                ViewPlan* __restrict__ plan) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= B * nv) return;
  const ImgDesc& d = desc[i / nv];
  const int S = (i % nv) < n_global ? gsize : lsize;
  const int ok = d.status == DINO_IMG_OK && params_valid(prm[i], d, S);
  int64_t a;
  int32_t kh, kv;
  view_sizes(prm[i], ok, &a, &kh, &kv);
  ViewPlan vp;
  vp.ok = ok;
  vp.lsum = 0;
  vp.kh = kh;
  vp.kv = kv;
  vp.htmp_off = a;
  vp.rcoef_off = kh ? align16((int64_t)prm[i].crop_h * S * 3) : 0;
  vp.hr_chunks = ok && kh ? hr_view_chunks(S, prm[i].crop_w, prm[i].crop_h, kh) : 0;
  vp.hr_base = 0;
  plan[i] = vp;
}

// Per-view scratch offsets: exclusive scan of the views' scratch sizes, or (when the
// batch's views do not fit the augment workspace) greedy placement in batch order by
// one lane.  A view that cannot be placed is not rendered and its image is marked
// DINO_IMG_NO_SPACE (reported by dino_batch_info; the host sizes the workspace with
// dino_probe + dino_reserve so that this does not happen on the product path).
__global__ void __launch_bounds__(1024) k_vplan(ImgDesc* __restrict__ desc, const dino_view_params* __restrict__ prm,
                                                int B, int nv, int n_global, int gsize, int lsize, int64_t aws_size,
                                                ViewPlan* __restrict__ plan) {
  __shared__ int64_t part[1024];
  __shared__ int2 hpart[1024];
  const int t = threadIdx.x, N = B * nv;
  for (int b = t; b < B; b += 1024) desc[b].aug_status = 0;
  if (t == 0) plan[N] = ViewPlan{};  // k_hresize's work-item counters (global, local views): hr_chunks, hr_base
  const int per = (N + 1023) / 1024;
  int64_t local = 0;
  int2 hl = make_int2(0, 0);  // k_hresize work items of this thread's global / local views
  for (int k = 0; k < per; ++k) {
    int i = t * per + k;
    if (i < N) {
      local += plan[i].htmp_off;  // k_vsizes: the view's scratch bytes
      if ((i % nv) < n_global) hl.x += plan[i].hr_chunks;
      else hl.y += plan[i].hr_chunks;
    }
  }
  part[t] = local;
  hpart[t] = hl;
  __syncthreads();
  for (int s = 1; s < 1024; s <<= 1) {
    int64_t v = t >= s ? part[t - s] : 0;
    int2 hv = t >= s ? hpart[t - s] : make_int2(0, 0);
    __syncthreads();
    part[t] += v;
    hpart[t].x += hv.x;
    hpart[t].y += hv.y;
    __syncthreads();
  }
  const bool fits = part[1023] <= aws_size;
  int64_t base = part[t] - local;
  int2 hb = make_int2(hpart[t].x - hl.x, hpart[t].y - hl.y);
  for (int k = 0; k < per; ++k) {
    int i = t * per + k;
    if (i >= N) continue;
    ViewPlan vp = plan[i];
    const int64_t a = vp.htmp_off;
    vp.ok = vp.ok && fits;
    vp.htmp_off = base;
    vp.rcoef_off += base;
    if ((i % nv) < n_global) {
      vp.hr_base = hb.x;
      hb.x += vp.hr_chunks;
    } else {
      vp.hr_base = hb.y;
      hb.y += vp.hr_chunks;
    }
    plan[i] = vp;
    base += a;
  }
  if (!fits) {
    __syncthreads();
    if (t == 0) {
      int64_t b = 0;
      for (int i = 0; i < N; ++i) {
        ViewPlan& vp = plan[i];
        const ImgDesc& d = desc[i / nv];
        int S = (i % nv) < n_global ? gsize : lsize;
        if (!(d.status == DINO_IMG_OK && params_valid(prm[i], d, S))) continue;
        int64_t a;
        int32_t kh, kv;
        view_sizes(prm[i], 1, &a, &kh, &kv);
        if (b + a <= aws_size) {
          vp.ok = 1;
          vp.htmp_off = b;
          vp.rcoef_off = b + (kh ? align16((int64_t)prm[i].crop_h * S * 3) : 0);
          b += a;
        } else {
          desc[i / nv].aug_status = DINO_IMG_NO_SPACE;
        }
      }
    }
  }
}

__global__ void __launch_bounds__(256) k_rcoeffs(const dino_view_params* __restrict__ prm, const ViewPlan* __restrict__ plan,
                                                 int nv, int v0, uint8_t* __restrict__ aws) {
  const int i = blockIdx.y * nv + v0 + blockIdx.x;
  const ViewPlan vp = plan[i];
  if (!vp.ok) return;
  const dino_view_params p = prm[i];
  const int S = p.out_size;
  int32_t* base = (int32_t*)(aws + vp.rcoef_off);
  int32_t* hb = base;                 // [S][2]
  int32_t* vb = base + 2 * S;         // [S][2]
  int32_t* ht = base + 4 * S;         // [S][kh]
  int32_t* vt = ht + (int64_t)S * vp.kh;
  int4* hx = (int4*)(aws + vp.rcoef_off + align16((int64_t)S * (4 + vp.kh + vp.kv) * 4));
  uint4* hg = (uint4*)(hx + S);
  for (int x = threadIdx.x; x < S; x += blockDim.x) {
    if (vp.kh) {
      int32_t* k = ht + (int64_t)x * vp.kh;
      resample_coeffs_one(p.crop_w, view_rw(p), p.out_x + x, vp.kh, &hb[2 * x], &hb[2 * x + 1], k);
      // sum_t p_t k_t = sum_t (p_t - 128) k_t + 128 sum_t k_t, and k_t = D0 + 256 D1 + 65536 D2
      // with signed digits D in [-128, 127] (exact for |k| < 2^23 - 2^15; normalised bicubic
      // taps stay below 1.1 x 2^22): three v_dot4 products per 4 taps
      const int cnt = hb[2 * x + 1], ng = (cnt + 3) / 4;
      int32_t ksum = 0;
      for (int g = 0; g < ng; ++g) {
        uint32_t dp[3] = {0u, 0u, 0u};
        for (int j = 0; j < 4; ++j) {
          const int t = 4 * g + j;
          const int32_t kt = t < cnt ? k[t] : 0;
          ksum += kt;
          const int32_t d0 = (int32_t)(int8_t)(uint8_t)(kt & 0xFF);
          const int32_t r1 = (kt - d0) >> 8;
          const int32_t d1 = (int32_t)(int8_t)(uint8_t)(r1 & 0xFF);
          const int32_t d2 = (r1 - d1) >> 8;
          dp[0] |= (uint32_t)(uint8_t)d0 << (8 * j);
          dp[1] |= (uint32_t)(uint8_t)d1 << (8 * j);
          dp[2] |= (uint32_t)(uint8_t)d2 << (8 * j);
        }
        hg[(int64_t)g * S + x] = make_uint4(dp[0], dp[1], dp[2], 0u);
      }
      // k_hresize runs the view's ng_max groups for every output: zero taps past this one's
      for (int g = ng; g < (vp.kh + 3) / 4; ++g) hg[(int64_t)g * S + x] = make_uint4(0u, 0u, 0u, 0u);
      hx[x] = make_int4(hb[2 * x], ng, 128 * ksum + (1 << (kPrecisionBits - 1)), 0);
    }
    if (vp.kv)
      resample_coeffs_one(p.crop_h, view_rh(p), p.out_y + x, vp.kv, &vb[2 * x], &vb[2 * x + 1], vt + (int64_t)x * vp.kv);
  }
}

// Horizontal pass.  A workgroup owns bands of R source rows of one view.  The
// crop's pixels for those rows are staged in LDS as RGBX words (each lane turns
// 12 source bytes = 4 pixels into one 16-byte LDS store); the view's taps are
// staged in LDS too when they fit.  Each lane then resamples one (row, x) with
// one LDS word per tap and writes the three channels to planar temp rows
// [3][crop_h][S].  Crops too wide for LDS take a direct (global) path.
constexpr int kHresizeMinRows = 8;  // rows per band the slice width is chosen for
constexpr int kHrBandsPerItem = 8;  // row bands of one slice per work item
constexpr int kHrDirectItems = 4;  // work items of a direct-path view
constexpr int kHrStageUnroll = 4;  // staging loads in flight per lane (2: 168.0k, 8: 168.8k, 4: 170.2k img/s C2)

// Tile shape of a view's horizontal pass: the widest slice of outputs (all of S,
// else a multiple of 8) whose taps (16 bytes per output + 16 per output and group
// of 4 taps) and kHresizeMinRows staged rows fit kHresizeLds; then as many rows per
// band as fit (<= 16).  R = 0: even 8 outputs do not fit (direct path).
struct HrTile {
  int sw, pitch, R, R3p;
};
__device__ __forceinline__ int hresize_pitch(int S, int cw, int kh, int sw) {
  // widest source span of a slice (+ 4 for the word alignment of its first column)
  const int span = min(cw, (int)(((int64_t)sw * cw + S - 1) / S) + kh + 2) + 4;
  return ((span + 3) & ~3) + 8;  // + slack for the last group's upper word
}
// Words per staged source group: 3 R row-channel words + 2, rounded to 2 mod 4.  Even, so
// a row pair's six words are one 8-byte-aligned run; 2 mod 4, so the row pairs that the
// lanes of a ds_read_b64 group read at distinct source groups k fall on distinct bank
// pairs (k R3p mod 64): with R = 10 or 14 (R3p 32 / 44) up to 16-way conflicts, 52 % of
// the kernel's LDS cycles (SQ_LDS_BANK_CONFLICT, profiles/r05_c2_lds.txt).
__host__ __device__ __forceinline__ int hresize_r3p(int R) {
  const int r = 3 * R + 2;
  return (r & 3) == 0 ? r + 2 : r;
}
// LDS bytes of a band of R rows: (pitch / 4) source words x R3p row-channel words,
// plus room for the over-read of the last output's zero-tap groups (ng_max words).
__device__ __forceinline__ int hresize_rows_bytes(int pitch, int R, int ng_max) {
  return (pitch / 4 + ng_max + 1) * hresize_r3p(R) * 4;
}
__device__ __forceinline__ HrTile hresize_tile(int S, int cw, int kh) {
  const int ng_max = (kh + 3) / 4;
  const int tap_bytes = 16 * (1 + (ng_max | 1));
  HrTile t{0, 0, 0, 0};
  int sw = S;
  while (tap_bytes * sw + hresize_rows_bytes(hresize_pitch(S, cw, kh, sw), kHresizeMinRows, ng_max) > kHresizeLds) {
    sw = sw == S ? ((S - 1) & ~7) : sw - 8;
    if (sw < 8) return t;
  }
  t.sw = sw;
  t.pitch = hresize_pitch(S, cw, kh, sw);
  int R = 16;
  while (R > kHresizeMinRows && tap_bytes * sw + hresize_rows_bytes(t.pitch, R, ng_max) > kHresizeLds) R -= 2;
  t.R = R;
  t.R3p = hresize_r3p(R);
  return t;
}

// Work items of a view's horizontal pass (k_vsizes): kHrBandsPerItem row bands of one
// slice each, so that a batch of mixed crop sizes spreads over the persistent grid in
// pieces of similar size (a large crop's view is many items, a small one's few).
__device__ int hr_view_chunks(int S, int cw, int ch, int kh) {
  const HrTile t = hresize_tile(S, cw, kh);
  if (t.R < 1) return kHrDirectItems;
  const int nsl = (S + t.sw - 1) / t.sw, nbands = (ch + t.R - 1) / t.R;
  return nsl * ((nbands + kHrBandsPerItem - 1) / kHrBandsPerItem);
}

// The view of work item c among the nc class views (b, v0 + j), j = view index mod nvc:
// the last view whose first item is <= c (views without items share their successor's
// first item).  64-ary search by each wave: two rounds of loads for 4096 views.
__device__ __forceinline__ int hr_find_view(const ViewPlan* __restrict__ plan, int nv, int v0, int nvc, int nc, int c) {
  int lo = 0, len = nc;
  const int lane = threadIdx.x & 63;
  while (len > 1) {
    const int step = (len + 63) >> 6;
    const int cand = lo + lane * step;
    bool le = false;
    if (cand < lo + len) {
      const int b = cand / nvc;
      le = plan[b * nv + v0 + (cand - b * nvc)].hr_base <= c;
    }
    const uint64_t m = __ballot(le);  // bit 0 set: plan[lo].hr_base <= c holds throughout
    const int last = 63 - __builtin_clzll(m);
    lo += last * step;
    len = min(step, len - last * step);
  }
  return lo;
}

// One tile: nr staged rows x the outputs [x0, x0 + sw) of a slice.  Lane (row pair, x)
// accumulates three signed-dot4 digit products per row, channel and group of 4 taps.
// Rows are staged with the sign bit flipped (p - 128 as int8) from source column c0,
// word-interleaved: word (gw, r, c) = 4 pixels gw of row r, channel c at gw * R3p + 3 r + c
// (R3p = hresize_r3p(R): even, so a row pair's six words are one 8-byte-aligned run: three
// ds_read_b64 per group and one address for all of them).  The taps' pixels start at xmin,
// so each group's 4 pixels are one v_alignbyte of a word and the next group's (carried).
// The group loop runs the view's ng_max groups for every lane (taps past an output's own
// count are zero digits, k_rcoeffs), a wave-uniform trip count the compiler unrolls for
// NG <= 8.  Exact: the int32 sum equals Pillow's.
template <int NG>
__device__ __forceinline__ void hresize_tile_dot(const uint32_t* __restrict__ rows, int R3p, int nr, int r0, int x0,
                                                 int sw, int c0, int S, int ng, int ngp, const int4* __restrict__ hx,
                                                 const uint4* __restrict__ hg, uint8_t* __restrict__ tmp, int64_t cpl) {
  if (NG) ng = NG;
  const int npair = (nr + 1) >> 1;
  const int qs = R3p >> 1;  // uint2 stride per source group
  // lane task (row pair rp, output xl), advanced by the block size without dividing again
  const int dq = (int)blockDim.x / sw, dr = (int)blockDim.x - dq * sw;
  int rp = (int)threadIdx.x / sw, xl = (int)threadIdx.x - rp * sw;
  for (; rp < npair; rp += dq, xl += dr, (xl >= sw ? (xl -= sw, ++rp) : 0)) {
    const int ra = 2 * rp;  // rows ra, ra + 1 (a band's odd last row pairs with an unstored row: not written)
    const int4 h = hx[xl];
    const int lo = h.x - c0;
    const uint32_t sh = (uint32_t)(lo & 3);
    const uint2* q = (const uint2*)(rows + __umul24((uint32_t)(lo >> 2), (uint32_t)R3p) + 3 * ra);
    uint32_t lw[6];
    {
      const uint2 a0 = q[0], a1 = q[1], a2 = q[2];
      lw[0] = a0.x, lw[1] = a0.y, lw[2] = a1.x, lw[3] = a1.y, lw[4] = a2.x, lw[5] = a2.y;
    }
    int32_t acc[6][3];  // digit 0 starts at the rounding + sign-flip correction h.z
#pragma unroll
    for (int k = 0; k < 6; ++k) acc[k][0] = h.z, acc[k][1] = acc[k][2] = 0;
    const uint4* dgp = hg + xl * ngp;  // this output's taps: ngp consecutive groups (immediate offsets)
#pragma unroll
    for (int g = 0; g < ng; ++g) {
      const uint4 dg = dgp[g];
      const uint2* qn = q + (g + 1) * qs;
      const uint2 b0 = qn[0], b1 = qn[1], b2 = qn[2];
      const uint32_t uw[6] = {b0.x, b0.y, b1.x, b1.y, b2.x, b2.y};
#pragma unroll
      for (int k = 0; k < 6; ++k) {
        const int32_t pa = (int32_t)__builtin_amdgcn_alignbyte(uw[k], lw[k], sh);
        acc[k][0] = __builtin_amdgcn_sdot4(pa, (int32_t)dg.x, acc[k][0], false);
        acc[k][1] = __builtin_amdgcn_sdot4(pa, (int32_t)dg.y, acc[k][1], false);
        acc[k][2] = __builtin_amdgcn_sdot4(pa, (int32_t)dg.z, acc[k][2], false);
        lw[k] = uw[k];
      }
    }
    // int32 wrap-around is harmless: the true sum (Pillow's int32 ss) fits in int32
    // (clip8_acc as one med3: the sum is < 2^30 unless it clips to 255, and <= 0 clips to 0;
    // 32-bit offsets: a view's planes hold < 3 x 2^20 x 1024 bytes)
    const uint32_t ob = (uint32_t)((r0 + ra) * S + x0 + xl);
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      if (ra + i >= nr) break;
#pragma unroll
      for (int c = 0; c < 3; ++c) {
        const int k = 3 * i + c;
        const uint32_t so = (uint32_t)__builtin_amdgcn_readfirstlane((int)((uint32_t)(i * S) + (uint32_t)c * (uint32_t)cpl));
        const int32_t sum = (int32_t)((uint32_t)acc[k][0] + ((uint32_t)acc[k][1] << 8) + ((uint32_t)acc[k][2] << 16));
        tmp[ob + so] = (uint8_t)min(max(sum >> kPrecisionBits, 0), 255);
      }
    }
  }
}

// Horizontal pass in tiles of (slice of outputs) x (band of rows), shaped by
// hresize_tile: the slice's taps always come from LDS, and the band stages only the
// source columns the slice reads [xmin(x0), xmin(x1-1) + xcnt(x1-1)), so wide crops
// take narrower slices to keep >= kHresizeMinRows rows per band.  A persistent grid
// takes the class's work items (kHrBandsPerItem bands of one slice, hr_view_chunks) in
// turn: with mixed crop sizes (C3) a fixed number of workgroups per view left the
// largest views' workgroups running alone at the end of the launch.
__device__ __forceinline__ void hresize_item(const ImgDesc* __restrict__ desc, const dino_view_params* __restrict__ prm,
                                             const ViewPlan* __restrict__ plan, int nv, int v0, int nvc, int nc, int c,
                                             const uint8_t* __restrict__ ws, uint8_t* __restrict__ aws, uint8_t* smem);

#ifndef DINO_HRESIZE_WAVES  // (A/B: minimum waves per SIMD the register allocation must allow)
#define DINO_HRESIZE_WAVES 1
#endif
__global__ void __launch_bounds__(256, DINO_HRESIZE_WAVES) k_hresize(const ImgDesc* __restrict__ desc, const dino_view_params* __restrict__ prm,
                                                 ViewPlan* __restrict__ plan, int nv, int v0, int nvc, int B,
                                                 const uint8_t* __restrict__ ws, uint8_t* __restrict__ aws) {
  main_prio();
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  __shared__ int s_item[2];
  const int nc = B * nvc;
  // persistent grid over the class's work items (k_vplan's per-class prefix), taken in turn
  // from the class's counter (zeroed by k_vplan), the next one fetched while this one runs
  const ViewPlan vl = plan[(B - 1) * nv + v0 + nvc - 1];
  const int nitems_all = vl.hr_base + vl.hr_chunks;
  int* ctr = v0 == 0 ? &plan[B * nv].hr_chunks : &plan[B * nv].hr_base;
  if (threadIdx.x == 0) s_item[0] = atomicAdd(ctr, 1);
  __syncthreads();
  for (int it = 0, c = s_item[0]; c < nitems_all; ++it) {
    if (threadIdx.x == 0) s_item[(it + 1) & 1] = atomicAdd(ctr, 1);
    hresize_item(desc, prm, plan, nv, v0, nvc, nc, c, ws, aws, smem);
    __syncthreads();
    c = s_item[(it + 1) & 1];
  }
}

__device__ __forceinline__ void hresize_item(const ImgDesc* __restrict__ desc, const dino_view_params* __restrict__ prm,
                                             const ViewPlan* __restrict__ plan, int nv, int v0, int nvc, int nc, int c,
                                             const uint8_t* __restrict__ ws, uint8_t* __restrict__ aws, uint8_t* smem) {
  {
    const int j = hr_find_view(plan, nv, v0, nvc, nc, c);
    const int b = j / nvc;
    const int i = b * nv + v0 + (j - b * nvc);
    const ViewPlan vp = plan[i];
    if (!vp.ok || !vp.kh) return;  // (no items: not reached)
    const int item = c - vp.hr_base;
    const dino_view_params p = prm[i];
    const ImgDesc& d = desc[b];
    const int S = p.out_size, W = d.width, cw = p.crop_w, kh = vp.kh;
    const int32_t* gb = (const int32_t*)(aws + vp.rcoef_off);
    const int32_t* gt = gb + 4 * S;
    const int4* ghx = (const int4*)(aws + vp.rcoef_off + align16((int64_t)S * (4 + vp.kh + vp.kv) * 4));
    const uint4* ghg = (const uint4*)(ghx + S);
    const uint8_t* rgb = ws + d.rgb_off;
    uint8_t* tmp = aws + vp.htmp_off;
    const int64_t cpl = (int64_t)p.crop_h * S;
    const int ng_max = (kh + 3) / 4;
    const int ngp = ng_max | 1;  // tap groups per output in LDS: odd, so 16 lanes' b128 reads hit distinct banks
    const HrTile tl = hresize_tile(S, cw, kh);
    const int sw = tl.sw, pitch = tl.pitch, R = tl.R, R3p = tl.R3p;
    if (R < 1) {  // direct path: taps and pixels from global memory (crops too wide for LDS)
      const SrcView src{rgb + ((int64_t)p.crop_top * W + p.crop_left) * 3, (int64_t)W * 3, 3, 1};
      const CoefView cv{gb, gt, kh};
      for (int64_t e = (int64_t)item * blockDim.x + threadIdx.x; e < cpl; e += (int64_t)kHrDirectItems * blockDim.x) {
        const int r = (int)(e / S), x = (int)(e - (int64_t)r * S);
        for (int ch = 0; ch < 3; ++ch) tmp[ch * cpl + e] = hresize_at(src, cv, r, x, ch);
      }
      return;
    }
    // LDS: the staged rows first (an edge output's zero-tap over-read stays inside the rows'
    // pad), then the slice's taps
    uint32_t* rows = (uint32_t*)smem;
    int4* lx = (int4*)(smem + ((hresize_rows_bytes(pitch, R, ng_max) + 15) & ~15));
    uint4* lg = (uint4*)(lx + sw);
    const int nbands = (p.crop_h + R - 1) / R;
    const int nbg = (nbands + kHrBandsPerItem - 1) / kHrBandsPerItem;
    // the item: slice sl (outputs [x0, x0 + swn)), bands [band0, band1)
    const int sl = item / nbg;
    const int band0 = (item - sl * nbg) * kHrBandsPerItem, band1 = min(nbands, band0 + kHrBandsPerItem);
    const int x0 = sl * sw, swn = min(sw, S - x0);
    const int c0 = ghx[x0].x & ~3;  // first source column staged (4-aligned within the crop)
    const int c1 = min(cw, ghx[x0 + swn - 1].x + gb[2 * (x0 + swn - 1) + 1]);
    const int ngroups = (c1 - c0 + 3) >> 2;  // staged groups of 4 pixels per row
    // taps of the slice -> LDS (the previous item ended with a barrier)
    for (int k = threadIdx.x; k < swn; k += blockDim.x) lx[k] = ghx[x0 + k];
    for (int k = threadIdx.x; k < swn * ng_max; k += blockDim.x) {
      const int g = k / swn, xl = k - g * swn;
      lg[xl * ngp + g] = ghg[(int64_t)g * S + x0 + xl];
    }
    // staging item e of a band: row e / ngroups, group e % ngroups (12 source bytes = 4
    // pixels -> one word per channel, de-interleaved by v_perm byte selects, sign bit
    // flipped).  kHrStageUnroll items per lane in flight: their 16-byte loads are issued
    // together and waited on once (one item at a time waited a full memory latency per
    // item: k_hresize 0.95 -> 0.85 ms per C2 step).  (Issuing the next band's first chunk
    // before this band's dot products, registers held across them, measured slower: 114-147
    // VGPRs, 3-4 waves per SIMD instead of 5.)
    const int64_t spitch = (int64_t)W * 3;
    const int dr = (int)blockDim.x / ngroups, dg = (int)blockDim.x - dr * ngroups;
    struct Stage {
      const uint8_t* base;
      int nst, e, sr, sg;
    };
    auto stage_begin = [&](int band) {
      const int r0 = band * R;
      Stage st;
      st.base = rgb + ((int64_t)(p.crop_top + r0) * W + p.crop_left + c0) * 3;
      st.nst = min(R, p.crop_h - r0) * ngroups;
      st.e = (int)threadIdx.x;
      st.sr = (int)threadIdx.x / ngroups;
      st.sg = (int)threadIdx.x - st.sr * ngroups;
      return st;
    };
    uint4 wv[kHrStageUnroll];
    uint32_t shv[kHrStageUnroll], dov[kHrStageUnroll];
    auto stage_issue = [&](Stage& st) {  // loads of the chunk at st.e (none past the band)
#pragma unroll
      for (int u = 0; u < kHrStageUnroll; ++u) {
        const bool ok = st.e + u * (int)blockDim.x < st.nst;
        // past the band: load the band's first words again (in bounds), nothing is stored
        const uint8_t* src = ok ? st.base + st.sr * spitch + 12 * st.sg : st.base;
        const uint32_t mis = (uint32_t)((uintptr_t)src & 3);
        wv[u] = *(const uint4*)(src - mis);
        shv[u] = ok ? 8u * mis : 0xFFFFFFFFu;
        dov[u] = (uint32_t)(st.sg * R3p + 3 * st.sr);
        st.sr += dr;
        st.sg += dg;
        if (st.sg >= ngroups) st.sg -= ngroups, ++st.sr;
      }
      st.e += kHrStageUnroll * (int)blockDim.x;
    };
    auto stage_commit = [&]() {
#pragma unroll
      for (int u = 0; u < kHrStageUnroll; ++u) {
        if (shv[u] == 0xFFFFFFFFu) break;
        const uint32_t sh = shv[u];
        const uint32_t q0 = (uint32_t)((((uint64_t)wv[u].y << 32) | wv[u].x) >> sh);  // R0 G0 B0 R1
        const uint32_t q1 = (uint32_t)((((uint64_t)wv[u].z << 32) | wv[u].y) >> sh);  // G1 B1 R2 G2
        const uint32_t q2 = (uint32_t)((((uint64_t)wv[u].w << 32) | wv[u].z) >> sh);  // B2 R3 G3 B3
        const uint32_t cr = __builtin_amdgcn_perm(q2, __builtin_amdgcn_perm(q1, q0, 0x0C060300u), 0x05020100u);
        const uint32_t cg = __builtin_amdgcn_perm(q2, __builtin_amdgcn_perm(q1, q0, 0x0C070401u), 0x06020100u);
        const uint32_t cb = __builtin_amdgcn_perm(q2, __builtin_amdgcn_perm(q1, q0, 0x0C0C0502u), 0x07040100u);
        uint32_t* dst = rows + dov[u];
        dst[0] = cr ^ 0x80808080u;
        dst[1] = cg ^ 0x80808080u;
        dst[2] = cb ^ 0x80808080u;
      }
    };
    for (int band = band0; band < band1; ++band) {
      const int r0 = band * R, nr = min(R, p.crop_h - r0);
      Stage st = stage_begin(band);
      while (st.e < st.nst) {
        stage_issue(st);
        stage_commit();
      }
      __syncthreads();
      switch (ng_max) {
#define DINO_HR_CASE(N) \
  case N: \
    hresize_tile_dot<N>(rows, R3p, nr, r0, x0, swn, c0, S, ng_max, ngp, lx, lg, tmp, cpl); \
    break;
        DINO_HR_CASE(1)
        DINO_HR_CASE(2)
        DINO_HR_CASE(3)
        DINO_HR_CASE(4)
        DINO_HR_CASE(5)
        DINO_HR_CASE(6)
        DINO_HR_CASE(7)
        DINO_HR_CASE(8)
#undef DINO_HR_CASE
        default:
          hresize_tile_dot<0>(rows, R3p, nr, r0, x0, swn, c0, S, ng_max, ngp, lx, lg, tmp, cpl);
      }
      __syncthreads();
    }
  }
}

// Per-view slot of the u8 crop planes [3][S][S] (global views first, then local views).
__device__ __forceinline__ int64_t crop_slot(const dino_aug_config& cfg, int B, int b, int v) {
  const int64_t g3 = 3ll * cfg.global_size * cfg.global_size, l3 = 3ll * cfg.local_size * cfg.local_size;
  if (v < cfg.n_global) return ((int64_t)b * cfg.n_global + v) * g3;
  return (int64_t)B * cfg.n_global * g3 + ((int64_t)b * cfg.n_local + (v - cfg.n_global)) * l3;
}

// Division of non-negative ints by a workgroup-uniform divisor d by one 64-bit
// multiply: exact whenever e * d < 2^32 (the rounding of m = ceil(2^32 / d) stays
// below 1/d over that range; here e * d < 2^26 for any view size <= 1024, the
// dino_ctx_create limit).
struct FastDiv {
  uint64_t m;
  __device__ explicit FastDiv(uint32_t d) : m(((1ull << 32) + d - 1) / d) {}
  __device__ uint32_t div(uint32_t e) const { return (uint32_t)(((uint64_t)e * m) >> 32); }
};

// Vertical pass (+ flip) and the ColorJitter ops that precede contrast, over a
// band of vert_rows(S) output rows; adds the band's L sum to the view's counter.
// Fast path (planar temp rows, S % 4 == 0): a lane produces 4 adjacent pixels
// from one 4-byte load per channel and tap and stores one word per plane.
constexpr int kVertRows = 8;
// rows per workgroup: 16 for the small (local) views, whose 8-row bands are short
__host__ __device__ __forceinline__ int vert_rows(int S) { return S > 128 ? kVertRows : 2 * kVertRows; }

// Rows [y0, y0 + nr) of a view through the vertical pass (+ flip) and the stage-0
// ColorJitter ops; every result goes out through put4(y, xo, w0, w1, w2) (four
// adjacent output pixels starting at column xo, one byte per pixel and plane, in
// output order) or put1(y, xo, r, g, b).  Returns the lane's sum of L over its
// pixels (used only when the view has a contrast op).
template <typename Put4, typename Put1>
__device__ __forceinline__ uint32_t vert_apply(const ImgDesc& d, const dino_view_params& p, const ViewPlan& vp,
                                               const uint8_t* __restrict__ ws, const uint8_t* __restrict__ aws, int S,
                                               int y0, int nr, const JitterPlan& jp, int hd, Put4 put4, Put1 put1) {
  const int W = d.width;
  const bool need_h = vp.kh != 0, need_v = vp.kv != 0;
  const int32_t* cbase = (const int32_t*)(aws + vp.rcoef_off);
  const CoefView cvv{cbase + 2 * S, cbase + 4 * S + (int64_t)S * vp.kh, vp.kv};
  const int64_t cpl = (int64_t)p.crop_h * S;
  const uint8_t* htmp = aws + vp.htmp_off;
  uint32_t lsum = 0;
  if (need_h && (S & 3) == 0) {
    const int nq = S >> 2;
    const FastDiv dq((uint32_t)nq);
    for (int e = threadIdx.x; e < nr * nq; e += blockDim.x) {
      const int yl = (int)dq.div((uint32_t)e);
      const int y = y0 + yl, xq = e - yl * nq;
      uint32_t w[3];
      if (need_v) {
        const int ymin = cvv.bounds[2 * y], ycnt = cvv.bounds[2 * y + 1];
        const int32_t* k = cvv.taps + (int64_t)y * cvv.ksize;
        // taps outer, channels inner: one tap load serves the three planes, whose
        // three row loads are independent (exact int32 sums: the order is free)
        const uint8_t* q = htmp + (int64_t)ymin * S + 4 * xq;
        int32_t a[3][4];
#pragma unroll
        for (int c = 0; c < 3; ++c) a[c][0] = a[c][1] = a[c][2] = a[c][3] = 1 << (kPrecisionBits - 1);
#pragma unroll 2
        for (int t = 0; t < ycnt; ++t) {
          const int32_t kk = k[t];
#pragma unroll
          for (int c = 0; c < 3; ++c) {
            const uint32_t u = *(const uint32_t*)(q + c * cpl + (int64_t)t * S);
            a[c][0] += (int32_t)(u & 255u) * kk;
            a[c][1] += (int32_t)((u >> 8) & 255u) * kk;
            a[c][2] += (int32_t)((u >> 16) & 255u) * kk;
            a[c][3] += (int32_t)(u >> 24) * kk;
          }
        }
#pragma unroll
        for (int c = 0; c < 3; ++c)
          w[c] = (uint32_t)clip8_acc(a[c][0]) | ((uint32_t)clip8_acc(a[c][1]) << 8) |
                 ((uint32_t)clip8_acc(a[c][2]) << 16) | ((uint32_t)clip8_acc(a[c][3]) << 24);
      } else {
#pragma unroll
        for (int c = 0; c < 3; ++c) w[c] = *(const uint32_t*)(htmp + c * cpl + (int64_t)y * S + 4 * xq);
      }
      uint32_t o[3] = {0u, 0u, 0u};
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        int r = (w[0] >> (8 * j)) & 255, g = (w[1] >> (8 * j)) & 255, bb = (w[2] >> (8 * j)) & 255;
        jitter_stage0(jp, r, g, bb, p, hd);
        if (jp.has_contrast) lsum += (uint32_t)rgb_to_l(r, g, bb);
        o[0] |= (uint32_t)r << (8 * j);
        o[1] |= (uint32_t)g << (8 * j);
        o[2] |= (uint32_t)bb << (8 * j);
      }
      if (p.flip) put4(y, S - 4 - 4 * xq, __builtin_bswap32(o[0]), __builtin_bswap32(o[1]), __builtin_bswap32(o[2]));
      else put4(y, 4 * xq, o[0], o[1], o[2]);
    }
  } else {
    const SrcView src = need_h ? SrcView{htmp, (int64_t)S, 1, cpl}
                               : SrcView{ws + d.rgb_off + ((int64_t)p.crop_top * W + p.crop_left) * 3, (int64_t)W * 3,
                                         3, 1};
    for (int e = threadIdx.x; e < nr * S; e += blockDim.x) {
      const int y = y0 + e / S, x = e % S;
      int r, g, bb;
      if (need_v) {
        r = vresize_at(src, cvv, y, x, 0);
        g = vresize_at(src, cvv, y, x, 1);
        bb = vresize_at(src, cvv, y, x, 2);
      } else {
        const uint8_t* q = src.base + (int64_t)y * src.pitch + (int64_t)x * src.px;
        r = q[0];
        g = q[src.cs];
        bb = q[2 * src.cs];
      }
      jitter_stage0(jp, r, g, bb, p, hd);
      put1(y, p.flip ? S - 1 - x : x, r, g, bb);
      if (jp.has_contrast) lsum += (uint32_t)rgb_to_l(r, g, bb);
    }
  }
  return lsum;
}

// Sum of a value over the workgroup (up to 1024 lanes, s_part holds one word per
// wave); every lane gets the total.
__device__ __forceinline__ uint32_t wg_sum(uint32_t v, uint32_t* s_part) {
  for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off);
  if ((threadIdx.x & 63) == 0) s_part[threadIdx.x >> 6] = v;
  __syncthreads();
  uint32_t t = 0;
  for (int w = 0; w < (int)(blockDim.x >> 6); ++w) t += s_part[w];
  __syncthreads();
  return t;
}

// The view's brightness / contrast blends as 256-entry LDS tables (JitterPlan::tb / tc):
// filled by the workgroup's first 256 lanes, read after the caller's next barrier
// (brightness, contrast and saturation together were 4.6 % of a C2 step, diagnosis build
// without them: 175.8k -> 183.8k img/s; the tables: k_final 0.345 -> 0.324 ms).
// stages: bit 0 = stage 0 (the ops before contrast), bit 1 = stage 1 (contrast and after);
// a table is made only when a stage the caller runs holds its op.
__device__ __forceinline__ bool jitter_has(uint32_t ops, int n, int op) {
  bool f = false;
  for (int k = 0; k < n; ++k) f |= (int)((ops >> (8 * k)) & 0xFFu) == op;
  return f;
}
__device__ __forceinline__ void jitter_tables(JitterPlan& jp, const dino_view_params& p, uint8_t* tb, uint8_t* tc,
                                              int contrast_mean, int stages) {
  if (!p.jitter) return;
  const bool b = ((stages & 1) && jitter_has(jp.pre, jp.n_pre, 0)) || ((stages & 2) && jitter_has(jp.post, jp.n_post, 0));
  const bool c = tc && (stages & 2) && jp.has_contrast;
  if (threadIdx.x < 256) {
    if (b) tb[threadIdx.x] = blend_u8(0, (int)threadIdx.x, p.brightness);
    if (c) tc[threadIdx.x] = blend_u8(contrast_mean, (int)threadIdx.x, p.contrast);
  }
  if (b) jp.tb = tb;
  if (c) jp.tc = tc;
}

__global__ void __launch_bounds__(256) k_vert(const ImgDesc* __restrict__ desc, const dino_view_params* __restrict__ prm,
                                              ViewPlan* __restrict__ plan, int nv, int v0, int B,
                                              const uint8_t* __restrict__ ws, const uint8_t* __restrict__ aws,
                                              uint8_t* __restrict__ gcrop, dino_aug_config cfg, int S) {
  const BlkIdx bk = xcd_blk();
  __shared__ uint32_t s_part[4];
  const int b = bk.z, v = v0 + bk.y;
  const int i = b * nv + v;
  const ViewPlan vp = plan[i];
  if (!vp.ok) return;
  const dino_view_params p = prm[i];
  const int64_t N = (int64_t)S * S;
  uint8_t* crop = gcrop + crop_slot(cfg, B, b, v);  // (256 lanes: s_part holds 4 waves)
  // (no blend tables here: a band of 8 rows is too short to repay making one, k_vert 0.272
  // -> 0.288 ms per C2 step with them)
  const JitterPlan jp = make_jitter_plan(p);
  const int y0 = bk.x * vert_rows(S);
  const int nr = min(vert_rows(S), S - y0);
  const uint32_t lsum = vert_apply(
      desc[b], p, vp, ws, aws, S, y0, nr, jp, hue_delta(p.hue),
      [&](int y, int xo, uint32_t w0, uint32_t w1, uint32_t w2) {
        const int64_t off = (int64_t)y * S + xo;
        *(uint32_t*)(crop + off) = w0;
        *(uint32_t*)(crop + N + off) = w1;
        *(uint32_t*)(crop + 2 * N + off) = w2;
      },
      [&](int y, int xo, int r, int g, int bb) {
        const int64_t o = (int64_t)y * S + xo;
        crop[o] = (uint8_t)r;
        crop[N + o] = (uint8_t)g;
        crop[2 * N + o] = (uint8_t)bb;
      });
  if (jp.has_contrast) {
    const uint32_t tot = wg_sum(lsum, s_part);
    if (threadIdx.x == 0) atomicAdd(&plan[i].lsum, tot);
  }
}

// The normalize + cast epilogue of one u8 value (to_tensor / 255, (x - mean) / std in
// float32, then the output type); k_final tabulates it per channel.
template <typename OutT>
__device__ __forceinline__ OutT out_cast(float f);
template <>
__device__ __forceinline__ uint16_t out_cast<uint16_t>(float f) {
  return f32_to_bf16(f);
}
template <>
__device__ __forceinline__ float out_cast<float>(float f) {
  return f;
}
template <>
__device__ __forceinline__ uint8_t out_cast<uint8_t>(float f) {
  return f32_to_fp8e4m3(bf16_to_f32(f32_to_bf16(f)));
}

// Four adjacent output values; one vector store when all four are in the row and aligned.
template <typename OutT>
__device__ __forceinline__ void store_vals4(OutT* out, int64_t o, const OutT* v, int n, bool vec) {
  if (vec) {
    if (sizeof(OutT) == 2) {
      *(uint2*)(out + o) = make_uint2((uint32_t)(uint16_t)v[0] | ((uint32_t)(uint16_t)v[1] << 16),
                                      (uint32_t)(uint16_t)v[2] | ((uint32_t)(uint16_t)v[3] << 16));
    } else if (sizeof(OutT) == 4) {
      *(float4*)(out + o) = make_float4((float)v[0], (float)v[1], (float)v[2], (float)v[3]);
    } else {
      *(uint32_t*)(out + o) = (uint32_t)(uint8_t)v[0] | ((uint32_t)(uint8_t)v[1] << 8) |
                              ((uint32_t)(uint8_t)v[2] << 16) | ((uint32_t)(uint8_t)v[3] << 24);
    }
  } else {
    for (int j = 0; j < n; ++j) out[o + j] = v[j];
  }
}

// Contrast (with the view's mean) and later ColorJitter ops, grayscale, then blur
// + solarize + normalize + cast over a band of final_rows(S) output rows.  The band
// and its blur halo (rows and columns, reflected as torch's reflect padding) are
// staged in LDS after the stage-1 jitter, so the blur reads a plain window.  A
// lane produces 4 adjacent outputs of one channel; the kernel size is a template
// parameter for the sizes the DINO sigma range yields (3..9).
constexpr int kFinalRows = 32;
// rows per workgroup: 16 for the large (global) views keeps their LDS tile small
// enough for 7 workgroups per CU
__host__ __device__ __forceinline__ int final_rows(int S) { return S > 128 ? 16 : kFinalRows; }
constexpr int kMaxBlurPad = 7;

struct FinalLds {
  float k1[16];
  float k2[256];
};

__host__ __device__ __forceinline__ int final_tile_pitch(int S, int pad) { return (((S + 3) & ~3) + 2 * pad + 3) & ~3; }
// LDS reserved for the tile (the largest blur halo)
__host__ __device__ __forceinline__ int final_tile_bytes(int S) {
  return 3 * (final_rows(S) + 2 * kMaxBlurPad) * final_tile_pitch(S, kMaxBlurPad);
}

constexpr int kBlurRegKs = 7;  // blur kernels up to this size keep their weights in registers
template <int KS, typename OutT>
__device__ __forceinline__ void final_compute(const uint8_t* __restrict__ tile, int tp, int64_t tplane, int nr, int y0,
                                              int S, int ks_rt, const float* __restrict__ k2, bool solarize,
                                              const OutT* __restrict__ ntab, OutT* __restrict__ out) {
  const int ks = KS > 0 ? KS : ks_rt;
  // the 2-D blur weights of a small kernel in registers: the tap loop then reads only
  // the pixel rows from LDS (same products, same fma order)
  float wreg[(KS > 0 && KS <= kBlurRegKs) ? KS * KS : 1];
  if (KS > 0 && KS <= kBlurRegKs) {
#pragma unroll
    for (int k = 0; k < (KS > 0 && KS <= kBlurRegKs ? KS * KS : 0); ++k) wreg[k] = k2[k];
  }
  const int nq = (S + 3) >> 2;
  const int64_t N = (int64_t)S * S;
  const bool vec_ok = (S & 3) == 0;
  const FastDiv dplane((uint32_t)(nr * nq)), drow((uint32_t)nq);
  for (int e = threadIdx.x; e < 3 * nr * nq; e += blockDim.x) {
    const int ch = (int)dplane.div((uint32_t)e), rem = e - ch * nr * nq;
    const int y = (int)drow.div((uint32_t)rem), x0 = 4 * (rem - y * nq);
    const uint8_t* pl = tile + ch * tplane;
    int val[4];
    if (KS == 1) {
      const uint32_t u = *(const uint32_t*)(pl + y * tp + x0);
#pragma unroll
      for (int j = 0; j < 4; ++j) val[j] = (u >> (8 * j)) & 255;
    } else {
      float acc[4] = {0.0f, 0.0f, 0.0f, 0.0f};
      if (KS > 0 && KS <= kBlurRegKs) {  // weights held in registers (loaded once per workgroup)
        constexpr int NW = (KS + 3 + 3) / 4;
#pragma unroll
        for (int a = 0; a < KS; ++a) {
          const uint32_t* row = (const uint32_t*)(pl + (y + a) * tp + x0);
          uint32_t wv[NW];
#pragma unroll
          for (int q = 0; q < NW; ++q) wv[q] = row[q];
#pragma unroll
          for (int c = 0; c < KS; ++c) {
            const float kk = wreg[a * KS + c];
#pragma unroll
            for (int j = 0; j < 4; ++j) {
              const int bi = c + j;
              acc[j] = fmaf(kk, (float)((wv[bi >> 2] >> (8 * (bi & 3))) & 255u), acc[j]);
            }
          }
        }
      } else if (KS > 0) {
        constexpr int NW = (KS + 3 + 3) / 4;
#pragma unroll 1
        for (int a = 0; a < KS; ++a) {
          const uint32_t* row = (const uint32_t*)(pl + (y + a) * tp + x0);
          uint32_t wv[NW];
#pragma unroll
          for (int q = 0; q < NW; ++q) wv[q] = row[q];
#pragma unroll
          for (int c = 0; c < KS; ++c) {
            const float kk = k2[a * KS + c];
#pragma unroll
            for (int j = 0; j < 4; ++j) {
              const int bi = c + j;
              acc[j] = fmaf(kk, (float)((wv[bi >> 2] >> (8 * (bi & 3))) & 255u), acc[j]);
            }
          }
        }
      } else {
        for (int a = 0; a < ks; ++a) {
          const uint8_t* row = pl + (y + a) * tp + x0;
          for (int c = 0; c < ks; ++c) {
            const float kk = k2[a * ks + c];
#pragma unroll
            for (int j = 0; j < 4; ++j) acc[j] = fmaf(kk, (float)row[c + j], acc[j]);
          }
        }
      }
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const float rr = rintf(acc[j]);
        val[j] = rr <= 0.0f ? 0 : (rr >= 255.0f ? 255 : (int)rr);
      }
    }
    const OutT* tb = ntab + 256 * ch;
    OutT o4[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) o4[j] = tb[solarize ? solarize_u8(val[j]) : val[j]];
    const int n = min(4, S - x0);
    store_vals4<OutT>(out, ch * N + (int64_t)(y0 + y) * S + x0, o4, n, vec_ok);
  }
}

// Separable form of the same blur for the kernel sizes the DINO sigma range yields: a
// lane takes 4 columns x kBlurStrip rows of one channel, convolves each tile row it
// needs once with the 1-D kernel (float fma chain over the taps), then the strip's
// columns with the 1-D kernel again.  The 2-D kernel of torchvision is the outer
// product of the same 1-D weights, so the two forms differ only in float rounding
// (the parity tests hold blurred views to one level on <= 0.5 % of pixels, as for the
// 2-D form against torch's conv2d); per output it takes 2 KS (KS + kBlurStrip - 1) /
// kBlurStrip fmas instead of KS^2.  k_final (the large views' bands) takes it: 0.378 ->
// 0.358 ms per C2 step; k_vfinal keeps the 2-D form, whose registers leave it 7 waves per
// SIMD instead of 5 (0.466 vs 0.494 ms).
constexpr int kBlurStrip = 4;
template <int KS, typename OutT>
__device__ __forceinline__ void final_compute_sep(const uint8_t* __restrict__ tile, int tp, int64_t tplane, int nr,
                                                  int y0, int S, const float* __restrict__ k1, bool solarize,
                                                  const OutT* __restrict__ ntab, OutT* __restrict__ out) {
  constexpr int R = kBlurStrip, NW = (KS + 3 + 3) / 4, TR = R + KS - 1;
  float w[KS];
#pragma unroll
  for (int k = 0; k < KS; ++k) w[k] = k1[k];
  const int nq = (S + 3) >> 2, ng = (nr + R - 1) / R;
  const int last_row = nr + KS - 2;  // the tile's last row (band + halo)
  const int64_t N = (int64_t)S * S;
  const bool vec_ok = (S & 3) == 0;
  const FastDiv dplane((uint32_t)(ng * nq)), dgrp((uint32_t)nq);
  for (int e = threadIdx.x; e < 3 * ng * nq; e += blockDim.x) {
    const int ch = (int)dplane.div((uint32_t)e), rem = e - ch * ng * nq;
    const int gy = (int)dgrp.div((uint32_t)rem), x0 = 4 * (rem - gy * nq);
    const int ys = gy * R;
    const uint8_t* pl = tile + ch * tplane + x0;
    float acc[R][4];
#pragma unroll
    for (int r = 0; r < R; ++r)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[r][j] = 0.0f;
#pragma unroll
    for (int a = 0; a < TR; ++a) {
      // rows past the band's last only feed outputs past it, which are not stored
      const uint32_t* row = (const uint32_t*)(pl + min(ys + a, last_row) * tp);
      uint32_t wv[NW];
#pragma unroll
      for (int q = 0; q < NW; ++q) wv[q] = row[q];
      float h[4] = {0.0f, 0.0f, 0.0f, 0.0f};
#pragma unroll
      for (int c = 0; c < KS; ++c)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int bi = c + j;
          h[j] = fmaf(w[c], (float)((wv[bi >> 2] >> (8 * (bi & 3))) & 255u), h[j]);
        }
#pragma unroll
      for (int r = 0; r < R; ++r) {
        if (a - r < 0 || a - r >= KS) continue;
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[r][j] = fmaf(w[a - r], h[j], acc[r][j]);
      }
    }
    const OutT* tb = ntab + 256 * ch;
    const int n = min(4, S - x0);
#pragma unroll
    for (int r = 0; r < R; ++r) {
      if (ys + r >= nr) break;
      OutT o4[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const float rr = rintf(acc[r][j]);
        const int v = rr <= 0.0f ? 0 : (rr >= 255.0f ? 255 : (int)rr);
        o4[j] = tb[solarize ? solarize_u8(v) : v];
      }
      store_vals4<OutT>(out, ch * N + (int64_t)(y0 + ys + r) * S + x0, o4, n, vec_ok);
    }
  }
}

template <typename OutT>
__global__ void __launch_bounds__(256) k_final(const ImgDesc* __restrict__ desc, const dino_view_params* __restrict__ prm,
                                               const ViewPlan* __restrict__ plan, int nv, int v0, int B,
                                               const uint8_t* __restrict__ gcrop, ViewPtrs views, dino_aug_config cfg,
                                               int S, const float* __restrict__ norm) {
  const BlkIdx bk = xcd_blk();
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  FinalLds& H = *reinterpret_cast<FinalLds*>(smem);
  uint8_t* tile = smem + sizeof(FinalLds);
  const int b = bk.z, v = v0 + bk.y;
  const int i = b * nv + v;
  const ViewPlan vp = plan[i];
  const int64_t N = (int64_t)S * S;
  const int y0 = bk.x * final_rows(S);
  const int nr = min(final_rows(S), S - y0);
  OutT* out = (OutT*)views.p[v] + (int64_t)b * 3 * N;
  const float* nb = norm ? norm + (int64_t)b * 6 : nullptr;
  if (!vp.ok) {
    // reference cpu.py:253: undecodable -> zeros; LeJEPA (cpu.py:446-448) crops a black
    // canvas instead, whose every op (crop, resize, jitter, flip) keeps it black, so its
    // views are the normalised value of 0
    const bool canvas = cfg.recipe == DINO_RECIPE_LEJEPA && desc[b].status < 0;
    for (int e = threadIdx.x; e < 3 * nr * S; e += blockDim.x) {
      const int ch = e / (nr * S), rem = e - ch * nr * S;
      out[(int64_t)ch * N + (int64_t)y0 * S + rem] =
          canvas ? out_cast<OutT>(u8_normalize(0, nb ? nb[ch] : cfg.mean[ch], nb ? nb[3 + ch] : cfg.std[ch])) : (OutT)0;
    }
    return;
  }
  const dino_view_params p = prm[i];
  const uint8_t* crop = gcrop + crop_slot(cfg, B, b, v);
  const int ks = p.blur ? p.ksize : 1;
  const int pad = ks >> 1;
  const int tr = nr + 2 * pad;                 // tile rows (band + reflected halo)
  const int tw = S + 2 * pad;                  // tile columns (row + reflected halo)
  const int tp = final_tile_pitch(S, pad);
  const int64_t tplane = (int64_t)tr * tp;
  if (p.blur && threadIdx.x == 0) gaussian_kernel1d(ks, p.sigma, H.k1);
  // the epilogue of each u8 value per channel (global or per-image statistics), after
  // the largest tile the launch reserves
  OutT* ntab = reinterpret_cast<OutT*>(tile + final_tile_bytes(S));
  for (int e = threadIdx.x; e < 3 * 256; e += blockDim.x) {
    const int c = e >> 8;
    ntab[e] = out_cast<OutT>(u8_normalize(e & 255, nb ? nb[c] : cfg.mean[c], nb ? nb[3 + c] : cfg.std[c]));
  }
  JitterPlan jp = make_jitter_plan(p);
  const int hd = hue_delta(p.hue);
  const int cmean = contrast_mean_from_sum(vp.lsum, N);
  __shared__ uint8_t s_tb[256], s_tc[256];
  jitter_tables(jp, p, s_tb, s_tc, cmean, 2);
  if (jp.tb || jp.tc) __syncthreads();
  auto stage_px = [&](int lr, int tc, int r, int g, int bb) {
    jitter_stage1(jp, r, g, bb, p, cmean, hd);
    const int to = lr * tp + tc;
    tile[to] = (uint8_t)r;
    tile[tplane + to] = (uint8_t)g;
    tile[2 * tplane + to] = (uint8_t)bb;
  };
  if ((S & 3) == 0) {
    // the band's rows four source pixels per lane (one word per plane), then the
    // reflected halo columns: 4x fewer dependent global loads than one pixel per lane
    const int nq = S >> 2;
    const FastDiv dq((uint32_t)nq);
    for (int e = threadIdx.x; e < tr * nq; e += blockDim.x) {
      const int lr = (int)dq.div((uint32_t)e), q = e - lr * nq;
      const int64_t so = (int64_t)reflect_idx(y0 - pad + lr, S) * S + 4 * q;
      const uint32_t wr = *(const uint32_t*)(crop + so), wg = *(const uint32_t*)(crop + N + so),
                     wb = *(const uint32_t*)(crop + 2 * N + so);
#pragma unroll
      for (int j = 0; j < 4; ++j)
        stage_px(lr, pad + 4 * q + j, (int)((wr >> (8 * j)) & 255u), (int)((wg >> (8 * j)) & 255u),
                 (int)((wb >> (8 * j)) & 255u));
    }
    if (pad > 0) {
      const FastDiv dh((uint32_t)(2 * pad));
      for (int e = threadIdx.x; e < tr * 2 * pad; e += blockDim.x) {
        const int lr = (int)dh.div((uint32_t)e), h = e - lr * 2 * pad;
        const int tc = h < pad ? h : S + h;  // columns [0, pad) and [S + pad, S + 2 pad)
        const int64_t so = (int64_t)reflect_idx(y0 - pad + lr, S) * S + reflect_idx(tc - pad, S);
        stage_px(lr, tc, crop[so], crop[N + so], crop[2 * N + so]);
      }
    }
  } else {
    const FastDiv dtw((uint32_t)tw);
    for (int e = threadIdx.x; e < tr * tw; e += blockDim.x) {
      const int lr = (int)dtw.div((uint32_t)e), tc = e - lr * tw;
      const int64_t so = (int64_t)reflect_idx(y0 - pad + lr, S) * S + reflect_idx(tc - pad, S);
      stage_px(lr, tc, crop[so], crop[N + so], crop[2 * N + so]);
    }
  }
  __syncthreads();
  if (p.blur && threadIdx.x < ks * ks) H.k2[threadIdx.x] = H.k1[threadIdx.x / ks] * H.k1[threadIdx.x % ks];
  __syncthreads();
  const bool sol = p.solarize != 0;
  switch (ks) {
    case 1: final_compute<1, OutT>(tile, tp, tplane, nr, y0, S, ks, H.k2, sol, ntab, out); break;
    case 3: final_compute_sep<3, OutT>(tile, tp, tplane, nr, y0, S, H.k1, sol, ntab, out); break;
    case 5: final_compute_sep<5, OutT>(tile, tp, tplane, nr, y0, S, H.k1, sol, ntab, out); break;
    case 7: final_compute_sep<7, OutT>(tile, tp, tplane, nr, y0, S, H.k1, sol, ntab, out); break;
    case 9: final_compute_sep<9, OutT>(tile, tp, tplane, nr, y0, S, H.k1, sol, ntab, out); break;
    default: final_compute<0, OutT>(tile, tp, tplane, nr, y0, S, ks, H.k2, sol, ntab, out); break;
  }
}

// k_vert + k_final for small views in one workgroup per view: the vertical pass and
// the stage-0 jitter write the view into an LDS tile, the workgroup reduces the
// contrast mean, applies the later ops in place, reflects the blur halo and runs the
// same blur/solarize/normalise epilogue -- the view never goes through HBM.
// Tile: S + 2 pad rows; columns from -pad (the window base, word-aligned) to S + pad.
__host__ __device__ __forceinline__ int vfinal_tile_bytes(int S) {
  return 3 * (S + 2 * kMaxBlurPad) * final_tile_pitch(S, kMaxBlurPad) + 16;
}
constexpr int kVFinalMaxS = 128;  // views up to this size take the fused kernel
constexpr int kVFinalThreads = 512;  // 8 waves per view: the vertical pass is load-latency bound

template <typename OutT>
__global__ void __launch_bounds__(kVFinalThreads) k_vfinal(const ImgDesc* __restrict__ desc, const dino_view_params* __restrict__ prm,
                                                const ViewPlan* __restrict__ plan, int nv, int v0, const uint8_t* __restrict__ ws,
                                                const uint8_t* __restrict__ aws, ViewPtrs views, dino_aug_config cfg, int S,
                                                const float* __restrict__ norm) {
  const BlkIdx bk = xcd_blk();
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  __shared__ uint32_t s_part[kVFinalThreads / 64];
  FinalLds& H = *reinterpret_cast<FinalLds*>(smem);
  uint8_t* tile = smem + sizeof(FinalLds);
  const int b = bk.y, v = v0 + bk.x;
  const int i = b * nv + v;
  const ViewPlan vp = plan[i];
  const int64_t N = (int64_t)S * S;
  OutT* out = (OutT*)views.p[v] + (int64_t)b * 3 * N;
  const float* nb = norm ? norm + (int64_t)b * 6 : nullptr;
  if (!vp.ok) {  // as k_final: zeros, or LeJEPA's black canvas normalised
    const bool canvas = cfg.recipe == DINO_RECIPE_LEJEPA && desc[b].status < 0;
    for (int e = threadIdx.x; e < 3 * S * S; e += blockDim.x) {
      const int ch = e / (S * S);
      out[e] = canvas ? out_cast<OutT>(u8_normalize(0, nb ? nb[ch] : cfg.mean[ch], nb ? nb[3 + ch] : cfg.std[ch])) : (OutT)0;
    }
    return;
  }
  const dino_view_params p = prm[i];
  const int ks = p.blur ? p.ksize : 1;
  const int pad = ks >> 1;
  const int tp = final_tile_pitch(S, pad);
  const int64_t tplane = (int64_t)(S + 2 * pad) * tp;
  OutT* ntab = reinterpret_cast<OutT*>(tile + vfinal_tile_bytes(S));
  if (p.blur && threadIdx.x == 0) gaussian_kernel1d(ks, p.sigma, H.k1);
  for (int e = threadIdx.x; e < 3 * 256; e += blockDim.x) {
    const int c = e >> 8;
    ntab[e] = out_cast<OutT>(u8_normalize(e & 255, nb ? nb[c] : cfg.mean[c], nb ? nb[3 + c] : cfg.std[c]));
  }
  JitterPlan jp = make_jitter_plan(p);
  const int hd = hue_delta(p.hue);
  __shared__ uint8_t s_tb[256], s_tc[256];
  jitter_tables(jp, p, s_tb, nullptr, 0, 3);  // the contrast table once the view's mean is known
  if (jp.tb) __syncthreads();
  uint8_t* in0 = tile + (int64_t)pad * tp + pad;  // interior (0, 0)
  const uint32_t lsum = vert_apply(
      desc[b], p, vp, ws, aws, S, 0, S, jp, hd,
      [&](int y, int xo, uint32_t w0, uint32_t w1, uint32_t w2) {
        uint8_t* q = in0 + y * tp + xo;  // byte stores: the interior starts at column pad
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          q[j] = (uint8_t)(w0 >> (8 * j));
          q[tplane + j] = (uint8_t)(w1 >> (8 * j));
          q[2 * tplane + j] = (uint8_t)(w2 >> (8 * j));
        }
      },
      [&](int y, int xo, int r, int g, int bb) {
        uint8_t* q = in0 + y * tp + xo;
        q[0] = (uint8_t)r;
        q[tplane] = (uint8_t)g;
        q[2 * tplane] = (uint8_t)bb;
      });
  __syncthreads();
  const int cmean = jp.has_contrast ? contrast_mean_from_sum(wg_sum(lsum, s_part), N) : 0;
  if (jp.has_contrast) {
    jitter_tables(jp, p, s_tb, s_tc, cmean, 2);
    __syncthreads();
  }
  // the ops after contrast, in place on the interior (none: no jitter and no grayscale)
  const FastDiv ds((uint32_t)S);
  const bool stage1 = jp.has_contrast || jp.n_post > 0 || p.gray;
  for (int e = threadIdx.x; stage1 && e < S * S; e += blockDim.x) {
    const int y = (int)ds.div((uint32_t)e), x = e - y * S;
    uint8_t* q = in0 + y * tp + x;
    int r = q[0], g = q[tplane], bb = q[2 * tplane];
    jitter_stage1(jp, r, g, bb, p, cmean, hd);
    q[0] = (uint8_t)r;
    q[tplane] = (uint8_t)g;
    q[2 * tplane] = (uint8_t)bb;
  }
  if (pad > 0) {
    __syncthreads();
    // blur halo: torch's reflect padding of the jittered view
    // over the halo only: 2 pad full rows above and below, then 2 pad columns of the interior rows
    const int tw = S + 2 * pad, nrow = 2 * pad * tw;
    const FastDiv dtw((uint32_t)tw), dh((uint32_t)(2 * pad));
    for (int e = threadIdx.x; e < nrow + S * 2 * pad; e += blockDim.x) {
      int r, c;
      if (e < nrow) {
        const int k = (int)dtw.div((uint32_t)e);
        c = e - k * tw;
        r = k < pad ? k : S + k;  // rows [0, pad) and [S + pad, S + 2 pad)
      } else {
        const int f = e - nrow, k = (int)dh.div((uint32_t)f), h = f - k * 2 * pad;
        r = pad + k;
        c = h < pad ? h : S + h;
      }
      const int sr = reflect_idx(r - pad, S), sc = reflect_idx(c - pad, S);
      const uint8_t* src = in0 + sr * tp + sc;
      uint8_t* dst = tile + r * tp + c;
      dst[0] = src[0];
      dst[tplane] = src[tplane];
      dst[2 * tplane] = src[2 * tplane];
    }
  }
  __syncthreads();
  if (p.blur && threadIdx.x < ks * ks) H.k2[threadIdx.x] = H.k1[threadIdx.x / ks] * H.k1[threadIdx.x % ks];
  __syncthreads();
  const bool sol = p.solarize != 0;
  switch (ks) {
    case 1: final_compute<1, OutT>(tile, tp, tplane, S, 0, S, ks, H.k2, sol, ntab, out); break;
    case 3: final_compute<3, OutT>(tile, tp, tplane, S, 0, S, ks, H.k2, sol, ntab, out); break;
    case 5: final_compute<5, OutT>(tile, tp, tplane, S, 0, S, ks, H.k2, sol, ntab, out); break;
    case 7: final_compute<7, OutT>(tile, tp, tplane, S, 0, S, ks, H.k2, sol, ntab, out); break;
    case 9: final_compute<9, OutT>(tile, tp, tplane, S, 0, S, ks, H.k2, sol, ntab, out); break;
    default: final_compute<0, OutT>(tile, tp, tplane, S, 0, S, ks, H.k2, sol, ntab, out); break;
  }
}

// ---------------------------------------------------------------------------
// Decode-only recipe (reference CPUUserAugPipeline, cpu.py:484-500; DALI
// _build_decode_only_pipeline, pipeline.py:693-756): every image of the batch
// resampled whole (Pillow BICUBIC, horizontal pass then vertical, each only when
// that axis changes size) to ow x oh, normalised and cast, NCHW.  Scratch per
// image (k_dplan, the ViewPlan slot of view 0): coefficient tables of both axes +
// the horizontal pass's rows (planar u8 [3][H][ow]).
// ---------------------------------------------------------------------------
__device__ void dec_sizes(const ImgDesc& d, int ow, int oh, int64_t* bytes, int32_t* kh, int32_t* kv) {
  const bool ok = d.status == DINO_IMG_OK;
  *kh = ok && d.width != ow ? resample_ksize(d.width, ow) : 0;
  *kv = ok && d.height != oh ? resample_ksize(d.height, oh) : 0;
  *bytes = ok ? align16((int64_t)ow * (2 + *kh) * 4) + align16((int64_t)oh * (2 + *kv) * 4) +
                    (*kh ? align16((int64_t)d.height * ow * 3) : 0)
              : 0;
}

__global__ void __launch_bounds__(1024) k_dplan(ImgDesc* __restrict__ desc, int B, int ow, int oh, int64_t aws_size,
                                                ViewPlan* __restrict__ plan) {
  __shared__ int64_t part[1024];
  const int t = threadIdx.x;
  const int per = (B + 1023) / 1024;
  int64_t local = 0;
  for (int k = 0; k < per; ++k) {
    const int i = t * per + k;
    if (i < B) {
      desc[i].aug_status = 0;
      int64_t a;
      int32_t kh, kv;
      dec_sizes(desc[i], ow, oh, &a, &kh, &kv);
      local += a;
    }
  }
  part[t] = local;
  __syncthreads();
  for (int s = 1; s < 1024; s <<= 1) {
    const int64_t v = t >= s ? part[t - s] : 0;
    __syncthreads();
    part[t] += v;
    __syncthreads();
  }
  const bool fits = part[1023] <= aws_size;
  int64_t base = part[t] - local;
  for (int k = 0; k < per; ++k) {
    const int i = t * per + k;
    if (i >= B) continue;
    int64_t a;
    int32_t kh, kv;
    dec_sizes(desc[i], ow, oh, &a, &kh, &kv);
    ViewPlan vp;
    vp.ok = desc[i].status == DINO_IMG_OK && fits;
    vp.kh = kh;
    vp.kv = kv;
    vp.lsum = 0;
    vp.rcoef_off = base;
    vp.htmp_off = base + align16((int64_t)ow * (2 + kh) * 4) + align16((int64_t)oh * (2 + kv) * 4);
    plan[i] = vp;
    base += a;
  }
  if (!fits) {
    __syncthreads();
    if (t == 0) {
      int64_t b = 0;
      for (int i = 0; i < B; ++i) {
        if (desc[i].status != DINO_IMG_OK) continue;
        int64_t a;
        int32_t kh, kv;
        dec_sizes(desc[i], ow, oh, &a, &kh, &kv);
        if (b + a <= aws_size) {
          plan[i].ok = 1;
          plan[i].rcoef_off = b;
          plan[i].htmp_off = b + align16((int64_t)ow * (2 + kh) * 4) + align16((int64_t)oh * (2 + kv) * 4);
          b += a;
        } else {
          desc[i].aug_status = DINO_IMG_NO_SPACE;
        }
      }
    }
  }
}

__global__ void __launch_bounds__(256) k_dcoeffs(const ImgDesc* __restrict__ desc, const ViewPlan* __restrict__ plan,
                                                 int ow, int oh, uint8_t* __restrict__ aws) {
  const int b = blockIdx.x;
  const ViewPlan vp = plan[b];
  if (!vp.ok) return;
  const ImgDesc& d = desc[b];
  int32_t* hb = (int32_t*)(aws + vp.rcoef_off);
  int32_t* ht = hb + 2 * ow;
  int32_t* vb = (int32_t*)(aws + vp.rcoef_off + align16((int64_t)ow * (2 + vp.kh) * 4));
  int32_t* vt = vb + 2 * oh;
  if (vp.kh)
    for (int x = threadIdx.x; x < ow; x += blockDim.x)
      resample_coeffs_one(d.width, ow, x, vp.kh, &hb[2 * x], &hb[2 * x + 1], ht + (int64_t)x * vp.kh);
  if (vp.kv)
    for (int y = threadIdx.x; y < oh; y += blockDim.x)
      resample_coeffs_one(d.height, oh, y, vp.kv, &vb[2 * y], &vb[2 * y + 1], vt + (int64_t)y * vp.kv);
}

__global__ void __launch_bounds__(256) k_dhpass(const ImgDesc* __restrict__ desc, const ViewPlan* __restrict__ plan,
                                                int ow, const uint8_t* __restrict__ ws, uint8_t* __restrict__ aws) {
  const int b = blockIdx.y;
  const ViewPlan vp = plan[b];
  if (!vp.ok || !vp.kh) return;
  const ImgDesc& d = desc[b];
  const int32_t* hb = (const int32_t*)(aws + vp.rcoef_off);
  const CoefView cv{hb, hb + 2 * ow, vp.kh};
  const SrcView src{ws + d.rgb_off, (int64_t)d.width * 3, 3, 1};
  uint8_t* tmp = aws + vp.htmp_off;
  const int64_t n = (int64_t)d.height * ow, plane = n;
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < n; e += (int64_t)gridDim.x * blockDim.x) {
    const int y = (int)(e / ow), x = (int)(e - (int64_t)y * ow);
#pragma unroll
    for (int c = 0; c < 3; ++c) tmp[c * plane + e] = hresize_at(src, cv, y, x, c);
  }
}

template <typename OutT>
__global__ void __launch_bounds__(256) k_dvpass(const ImgDesc* __restrict__ desc, const ViewPlan* __restrict__ plan,
                                                int ow, int oh, const uint8_t* __restrict__ ws,
                                                const uint8_t* __restrict__ aws, OutT* __restrict__ out, float m0,
                                                float m1, float m2, float s0, float s1, float s2,
                                                const float* __restrict__ norm) {
  const int b = blockIdx.y;
  const ViewPlan vp = plan[b];
  const ImgDesc& d = desc[b];
  const int64_t n = (int64_t)oh * ow;
  OutT* o = out + (int64_t)b * 3 * n;
  const float* nb = norm ? norm + (int64_t)b * 6 : nullptr;
  const float mean[3] = {nb ? nb[0] : m0, nb ? nb[1] : m1, nb ? nb[2] : m2};
  const float stdv[3] = {nb ? nb[3] : s0, nb ? nb[4] : s1, nb ? nb[5] : s2};
  if (!vp.ok) {  // undecodable (cpu.py:496-497) or not placed: zeros
    for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < 3 * n; e += (int64_t)gridDim.x * blockDim.x)
      o[e] = (OutT)0;
    return;
  }
  const int32_t* vb = (const int32_t*)(aws + vp.rcoef_off + align16((int64_t)ow * (2 + vp.kh) * 4));
  const CoefView cv{vb, vb + 2 * oh, vp.kv};
  const SrcView src = vp.kh ? SrcView{aws + vp.htmp_off, (int64_t)ow, 1, (int64_t)d.height * ow}
                            : SrcView{ws + d.rgb_off, (int64_t)d.width * 3, 3, 1};
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < n; e += (int64_t)gridDim.x * blockDim.x) {
    const int y = (int)(e / ow), x = (int)(e - (int64_t)y * ow);
#pragma unroll
    for (int c = 0; c < 3; ++c) {
      const int v = vp.kv ? vresize_at(src, cv, y, x, c)
                          : src.base[(int64_t)y * src.pitch + (int64_t)x * src.px + c * src.cs];
      o[c * n + e] = out_cast<OutT>(u8_normalize(v, mean[c], stdv[c]));
    }
  }
}

template <typename OutT>
static hipError_t launch_dec_out(const DecodeOnlyArgs& a, hipStream_t s) {
  const int gx = 64;
  k_dvpass<OutT><<<dim3(gx, a.batch), 256, 0, s>>>(a.desc, a.plan, a.ow, a.oh, a.ws, a.aws, (OutT*)a.out, a.mean[0],
                                                   a.mean[1], a.mean[2], a.std[0], a.std[1], a.std[2], a.norm);
  return hipGetLastError();
}

hipError_t launch_decode_only(const DecodeOnlyArgs& a, hipStream_t s) {
  if (a.batch <= 0) return hipSuccess;
  k_dplan<<<1, 1024, 0, s>>>(a.desc, a.batch, a.ow, a.oh, a.aws_size, a.plan);
  k_dcoeffs<<<a.batch, 256, 0, s>>>(a.desc, a.plan, a.ow, a.oh, a.aws);
  k_dhpass<<<dim3(64, a.batch), 256, 0, s>>>(a.desc, a.plan, a.ow, a.ws, a.aws);
  switch (a.out_dtype) {
    case DINO_OUT_FP32: return launch_dec_out<float>(a, s);
    case DINO_OUT_FP8_E4M3: return launch_dec_out<uint8_t>(a, s);
    default: return launch_dec_out<uint16_t>(a, s);
  }
}

// ---------------------------------------------------------------------------
// iBOT masks: one lane runs the (inherently sequential) generator; the mask and
// the completion scratch live in LDS (dynamic, 5 bytes per patch), the MT states too.
// ---------------------------------------------------------------------------
constexpr int kMaskLdsMaxPatches = 8192;  // 40 KiB of dynamic LDS (grids up to 90 x 90)

__global__ void k_masks(MaskParams mp, int n, uint32_t* __restrict__ py_state, uint32_t* __restrict__ np_state,
                        uint8_t* __restrict__ out) {
  __shared__ MtState py, np;
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  const int hw = mp.H * mp.W;
  int32_t* scratch = reinterpret_cast<int32_t*>(smem);
  uint8_t* mask = smem + 4 * hw;
  if (threadIdx.x == 0) {
    mt_load(py, py_state);
    mt_load(np, np_state);
  }
  __syncthreads();
  for (int k = 0; k < n; ++k) {
    if (threadIdx.x == 0) gen_mask(mp, py, np, mask, scratch);
    __syncthreads();
    for (int i = threadIdx.x; i < hw; i += blockDim.x) out[(int64_t)k * hw + i] = mask[i];
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    mt_store(py, py_state);
    mt_store(np, np_state);
  }
}

__global__ void k_bf16_to_fp8(const uint16_t* __restrict__ in, uint8_t* __restrict__ out, int64_t n) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    out[i] = f32_to_fp8e4m3(bf16_to_f32(in[i]));
}

// copy of one decoded image out of the workspace (tests / debug)
__global__ void k_copy_rgb(const ImgDesc* __restrict__ desc, int idx, const uint8_t* __restrict__ ws,
                           uint8_t* __restrict__ dst) {
  const ImgDesc& d = desc[idx];
  if (d.status != DINO_IMG_OK) return;
  const int64_t n = (int64_t)d.width * d.height * 3;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    dst[i] = ws[d.rgb_off + i];
}

// Decoded images -> raw containers (the side decoder): image idx[k]'s RGB to base + off[k]
// (base null: off[k] is the destination's device address), grid (x, n).  16-byte copies when
// source and destination are both 16-byte aligned (the workspace's RGB areas are; the
// containers' data starts 16 bytes into a 16-byte aligned slice), the tail and unaligned
// cases bytewise.  With `header`, the 16 bytes before the data get the container header
// {DINO_RAW_MAGIC, width, height, 0} (little-endian words).
__global__ void k_copy_rgb_packed(const ImgDesc* __restrict__ desc, int B, const int32_t* __restrict__ idx,
                                  const int64_t* __restrict__ off, const uint8_t* __restrict__ ws,
                                  uint8_t* __restrict__ base, int header) {
  const int k = blockIdx.y, i = idx[k];
  if (i < 0 || i >= B) return;
  const ImgDesc& d = desc[i];
  if (d.status != DINO_IMG_OK) return;
  const int64_t n = (int64_t)d.width * d.height * 3;
  const uint8_t* src = ws + d.rgb_off;
  uint8_t* dst = base ? base + off[k] : reinterpret_cast<uint8_t*>(static_cast<uintptr_t>(off[k]));
  if (header && blockIdx.x == 0 && threadIdx.x < 16) {
    const uint32_t w[4] = {DINO_RAW_MAGIC, (uint32_t)d.width, (uint32_t)d.height, 0u};
    const int j = threadIdx.x;
    dst[j - 16] = (uint8_t)(w[j >> 2] >> (8 * (j & 3)));
  }
  const int64_t t0 = (int64_t)blockIdx.x * blockDim.x + threadIdx.x, ts = (int64_t)gridDim.x * blockDim.x;
  int64_t head = 0;
  if ((((uintptr_t)src | (uintptr_t)dst) & 15) == 0) {
    const int64_t n16 = n >> 4;
    for (int64_t q = t0; q < n16; q += ts) ((uint4*)dst)[q] = ((const uint4*)src)[q];
    head = n16 << 4;
  }
  for (int64_t q = head + t0; q < n; q += ts) dst[q] = src[q];
}

__global__ void k_info(const ImgDesc* __restrict__ desc, int B, int32_t* __restrict__ info) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= B) return;
  const ImgDesc& d = desc[i];
  info[4 * i + 0] = d.status != DINO_IMG_OK ? d.status : d.aug_status;
  info[4 * i + 1] = d.width;
  info[4 * i + 2] = d.height;
  info[4 * i + 3] = d.ncomp;
}


}  // namespace dino

// ===========================================================================
// Launchers
// ===========================================================================
namespace dino {

void KernelTimer::begin(int k, hipStream_t s) {
  if (!enabled) return;
  if (!created) {
    for (int i = 0; i < kMaxPending; ++i) {
      (void)hipEventCreate(&ev[i][0]);
      (void)hipEventCreate(&ev[i][1]);
    }
    created = true;
    reset();
  }
  if (n >= kMaxPending) collect();
  id[n] = k;
  (void)hipEventRecord(ev[n][0], s);
}

void KernelTimer::end(hipStream_t s) {
  if (!enabled || !created) return;
  (void)hipEventRecord(ev[n][1], s);
  ++n;
}

void KernelTimer::collect() {
  for (int i = 0; i < n; ++i) {
    float ms = 0.f;
    (void)hipEventSynchronize(ev[i][1]);
    if (hipEventElapsedTime(&ms, ev[i][0], ev[i][1]) == hipSuccess) {
      total_ms[id[i]] += ms;
      count[id[i]] += 1;
    }
  }
  n = 0;
}

void KernelTimer::reset() {
  n = 0;
  for (int i = 0; i < kKNumKernels; ++i) {
    total_ms[i] = 0.0;
    count[i] = 0;
  }
}

void KernelTimer::destroy() {
  if (!created) return;
  for (int i = 0; i < kMaxPending; ++i) {
    (void)hipEventDestroy(ev[i][0]);
    (void)hipEventDestroy(ev[i][1]);
  }
  created = false;
}

// DINO_SYNC_CHECK=1: synchronise after every kernel and report which one failed
// (debugging aid; pinpoints a faulting kernel instead of a later sync point).
static const bool g_sync_check = [] {
  const char* v = getenv("DINO_SYNC_CHECK");
  return v && v[0] == '1';
}();
static const char* const kKernelNames[kKNumKernels] = {"k_parse", "k_plan", "k_destuff", "k_huff1", "k_idct",
                                                       "k_color", "k_params", "k_vplan", "k_rcoeffs", "k_hresize",
                                                       "k_final_global", "k_final_local", "k_vert_global",
                                                       "k_vert_local", "k_dcscan", "k_htab", "k_hseg", "k_huff2",
                                                       "k_huff3", "k_prog", "k_pwalk", "k_plscan",
                                                       "k_papply"};
const char* g_failed_kernel = "";

#define TIMED(tm, kid, s, launch)                          \
  do {                                                     \
    if (tm) (tm)->begin(kid, s);                           \
    launch;                                                \
    if (tm) (tm)->end(s);                                  \
    if (g_sync_check) {                                    \
      hipError_t se_ = hipStreamSynchronize(s);            \
      if (se_ == hipSuccess) se_ = hipGetLastError();      \
      if (se_ != hipSuccess) {                             \
        g_failed_kernel = kKernelNames[kid];               \
        fprintf(stderr, "[dino] %s failed: %s\n", kKernelNames[kid], hipGetErrorString(se_)); \
        return se_;                                        \
      }                                                    \
    }                                                      \
  } while (0)

// Persistent grids of the segment kernels: as many workgroups as can be resident
// on the device at once (occupancy query x CUs); items beyond them come in later turns.
static int persistent_grid(const void* fn, int lds, int cus) {
  int per = 4;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, fn, kHuffThreads, lds) != hipSuccess || per < 1) per = 4;
  return per * cus;
}

// Per-device launch geometry (called by dino_ctx_create with `device` current).
hipError_t init_launch_geom(int device, LaunchGeom* g) {
  int cus = 256;
  hipError_t e = hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device);
  if (e != hipSuccess) return e;
  if ((e = hipFuncSetAttribute(reinterpret_cast<const void*>(&k_huff1), hipFuncAttributeMaxDynamicSharedMemorySize,
                               kHuffLdsBytes)) != hipSuccess)
    return e;
  if ((e = hipFuncSetAttribute(reinterpret_cast<const void*>(&k_huff3), hipFuncAttributeMaxDynamicSharedMemorySize,
                               kHuff3LdsBytes)) != hipSuccess)
    return e;
  g->grid_ds = 4 * cus;
  g->grid3 = persistent_grid(reinterpret_cast<const void*>(&k_huff3), kHuff3LdsBytes, cus);
  g->grid1 = persistent_grid(reinterpret_cast<const void*>(&k_huff1), kHuffLdsBytes, cus);
  if ((e = hipFuncSetAttribute(reinterpret_cast<const void*>(&k_hresize), hipFuncAttributeMaxDynamicSharedMemorySize,
                               kHresizeLds)) != hipSuccess)
    return e;
  g->grid_hr = persistent_grid(reinterpret_cast<const void*>(&k_hresize), kHresizeLds, cus);
  if ((e = hipFuncSetAttribute(reinterpret_cast<const void*>(&k_plscan), hipFuncAttributeMaxDynamicSharedMemorySize,
                               kPLscanLds)) != hipSuccess)
    return e;
  // scan waves: one per CU by default.  A scan's serial decode runs on the CU's one scalar
  // unit, which the CU's waves share: two scan waves on a CU each run at about half speed
  // (DINO_PSCAN_PER_CU: waves per CU, measured in profiles/r03_prog_*).
  const char* pc = getenv("DINO_PSCAN_PER_CU");
  const int per_cu = pc && atoi(pc) > 0 ? atoi(pc) : 1;
  g->grid_ps = per_cu * cus;
  // lane scan waves: one ticket each (a 512-image pool of libjpeg-default files: 80); the rest exit
  const char* ls = getenv("DINO_PLSCAN_WAVES");
  g->grid_ls = ls && atoi(ls) > 0 ? atoi(ls) : 2 * cus;
  // the scan waves' issue priority: 0 below the batch kernels (s_setprio 3, main_prio), 1 level
  const char* sp = getenv("DINO_SCAN_PRIO");
  g->scan_prio = sp ? atoi(sp) : 0;
  // the lane decoder is opt-in (DINO_PROG_LANE=1): its throughput is higher but a scan's latency
  // is ~3x a scan wave's, more than the side route's look-ahead covers
  const char* pl = getenv("DINO_PROG_LANE");
  g->prog_lane = pl ? (atoi(pl) != 0) : 0;
  return hipSuccess;
}

hipError_t launch_decode(const DecodeArgs& a, hipStream_t s, KernelTimer* tm) {
  const int B = a.batch;
  if (B <= 0) return hipSuccess;
  TIMED(tm, kKParse, s, (k_parse<<<B, 64, 0, s>>>(a.bytes, a.offsets, a.lengths, a.raw_mask, B, a.max_dim, a.desc)));
  TIMED(tm, kKPlan, s, (k_plan<<<1, 1024, 0, s>>>(a.desc, B, a.ws_size, a.pctl)));
  const int grid_ds = a.geom.grid_ds, grid1 = a.geom.grid1, grid3 = a.geom.grid3;
  TIMED(tm, kKDestuff, s, (k_destuff_count<<<grid_ds, kDestuffThreads, 0, s>>>(a.bytes, a.offsets, B, a.desc, a.ws)));
  TIMED(tm, kKDestuff, s, (k_destuff_write<<<grid_ds, kDestuffThreads, 0, s>>>(a.bytes, a.offsets, B, a.desc, a.ws)));
  TIMED(tm, kKHtab, s, (k_htab<<<B, kHuffThreads, 0, s>>>(a.bytes, a.offsets, a.desc, a.ws)));
  // after k_htab's kind switch
  TIMED(tm, kKPwalk, s, (k_pwalk<<<B, kPWalkThreads, 0, s>>>(a.bytes, a.offsets, a.lengths, a.desc, a.ws, a.pctl,
                                                               a.geom.prog_lane)));
  TIMED(tm, kKProg, s, (k_pscan<<<a.geom.grid_ps, kPScanThreads, 0, s>>>(a.bytes, a.offsets, a.lengths, a.desc, a.ws, a.pctl,
                                                                             a.geom.scan_prio)));
  if (a.geom.prog_lane) {  // the lane decoder (opt-in): k_pwalk registers no lane image otherwise
    TIMED(tm, kKPlscan, s, (k_plscan<<<a.geom.grid_ls, 64, kPLscanLds, s>>>(a.desc, a.ws, a.pctl, a.geom.scan_prio)));
    TIMED(tm, kKPapply, s, (k_papply<<<dim3(kPApplyWgs, B), 256, 0, s>>>(a.desc, a.ws, a.pctl)));
  }
  TIMED(tm, kKHseg, s, (k_hseg<<<1, 1024, 0, s>>>(a.desc, B)));
  TIMED(tm, kKHuff1, s, (k_huff1<<<grid1, kHuffThreads, kHuffLdsBytes, s>>>(a.desc, B, a.ws)));
  TIMED(tm, kKHuff2, s, (k_huff2<<<B, kHuff2Threads, 0, s>>>(a.desc, a.ws)));
  TIMED(tm, kKHuff3, s, (k_huff3<<<grid3, kHuffThreads, kHuff3LdsBytes, s>>>(a.desc, B, a.ws)));
  TIMED(tm, kKDcscan, s, (k_dcscan<<<B, kDcScanThreads, 0, s>>>(a.desc, a.ws)));
  TIMED(tm, kKIdct, s, (k_idct<<<dim3(kIdctWgs, B), 256, 0, s>>>(a.desc, a.ws)));
  TIMED(tm, kKColor, s, (k_color<<<dim3(kColorWgs, B), 256, 0, s>>>(a.bytes, a.offsets, a.desc, a.ws)));
  return hipGetLastError();
}

hipError_t launch_params(const ImgDesc* desc, int batch, const dino_aug_config& cfg, uint64_t seed,
                         uint64_t batch_index, dino_view_params* out, hipStream_t s, KernelTimer* tm) {
  const int n = batch * (cfg.n_global + cfg.n_local);
  if (n <= 0) return hipSuccess;
  TIMED(tm, kKParams, s, (k_params<<<(n + 63) / 64, 64, 0, s>>>(desc, batch, cfg, seed, batch_index, out)));
  return hipGetLastError();
}

template <typename OutT>
static hipError_t launch_augment_class(const AugmentArgs& a, int v0, int nvc, int S, hipStream_t s, KernelTimer* tm) {
  const int B = a.batch, nv = a.cfg.n_global + a.cfg.n_local;
  if (nvc <= 0) return hipSuccess;
  const int kfin = v0 == 0 ? kKFinalGlobal : kKFinalLocal;
  const int kvert = v0 == 0 ? kKVertGlobal : kKVertLocal;
  const int rc_threads = S < 256 ? (S + 63) / 64 * 64 : 256;  // one lane per output column
  TIMED(tm, kKRcoeffs, s, (k_rcoeffs<<<dim3(nvc, B), rc_threads, 0, s>>>(a.params, a.plan, nv, v0, a.aws)));
  TIMED(tm, kKHresize, s,
        (k_hresize<<<a.grid_hr, 256, kHresizeLds, s>>>(a.desc, a.params, a.plan, nv, v0, nvc, B, a.ws, a.aws)));
  if (S <= kVFinalMaxS) {  // small views: vertical pass and epilogue fused, the view stays in LDS
    const int lds = (int)sizeof(FinalLds) + vfinal_tile_bytes(S) + 3 * 256 * (int)sizeof(OutT);
    TIMED(tm, kfin, s,
          (k_vfinal<OutT><<<dim3(nvc, B), kVFinalThreads, lds, s>>>(a.desc, a.params, a.plan, nv, v0, a.ws, a.aws, a.views, a.cfg,
                                                         S, a.norm)));
    return hipGetLastError();
  }
  TIMED(tm, kvert, s,
        (k_vert<<<dim3((S + vert_rows(S) - 1) / vert_rows(S), nvc, B), 256, 0, s>>>(a.desc, a.params, a.plan, nv, v0, B,
                                                                             a.ws, a.aws, a.gcrop, a.cfg, S)));
  const int lds = (int)sizeof(FinalLds) + final_tile_bytes(S) + 3 * 256 * (int)sizeof(OutT);
  TIMED(tm, kfin, s,
        (k_final<OutT><<<dim3((S + final_rows(S) - 1) / final_rows(S), nvc, B), 256, lds, s>>>(
            a.desc, a.params, a.plan, nv, v0, B, a.gcrop, a.views, a.cfg, S, a.norm)));
  return hipGetLastError();
}

template <typename OutT>
static hipError_t launch_augment_t(const AugmentArgs& a, hipStream_t s, KernelTimer* tm) {
  hipError_t e = launch_augment_class<OutT>(a, 0, a.cfg.n_global, a.cfg.global_size, s, tm);
  if (e != hipSuccess) return e;
  return launch_augment_class<OutT>(a, a.cfg.n_global, a.cfg.n_local, a.cfg.local_size, s, tm);
}

hipError_t launch_augment(const AugmentArgs& a, hipStream_t s, KernelTimer* tm) {
  const int B = a.batch, nv = a.cfg.n_global + a.cfg.n_local;
  if (B <= 0 || nv <= 0) return hipSuccess;
  TIMED(tm, kKVplan, s, (k_vsizes<<<(B * nv + 255) / 256, 256, 0, s>>>(a.desc, a.params, B, nv, a.cfg.n_global,
                                                                       a.cfg.global_size, a.cfg.local_size, a.plan)));
  TIMED(tm, kKVplan, s, (k_vplan<<<1, 1024, 0, s>>>(a.desc, a.params, B, nv, a.cfg.n_global, a.cfg.global_size,
                                                     a.cfg.local_size, a.aws_size, a.plan)));
  switch (a.cfg.out_dtype) {
    case DINO_OUT_FP32:
      return launch_augment_t<float>(a, s, tm);
    case DINO_OUT_FP8_E4M3:
      return launch_augment_t<uint8_t>(a, s, tm);
    default:
      return launch_augment_t<uint16_t>(a, s, tm);
  }
}

hipError_t launch_info(const ImgDesc* desc, int batch, int32_t* info, hipStream_t s) {
  if (batch <= 0) return hipSuccess;
  k_info<<<(batch + 63) / 64, 64, 0, s>>>(desc, batch, info);
  return hipGetLastError();
}

// The per-pixel colour operators over all 2^24 inputs (index = a << 16 | b << 8 | c):
// op 0 RGB -> HSV, op 1 HSV -> RGB, op 2 hue_shift by `param` (the ColorJitter hue op);
// out[3 * index + k].  For the exhaustive device-side checks against Pillow.
__global__ void __launch_bounds__(256) k_pixel_ops(int op, int param, uint8_t* __restrict__ out) {
  const int idx = blockIdx.x * 256 + threadIdx.x;
  int x = (idx >> 16) & 255, y = (idx >> 8) & 255, z = idx & 255;
  if (op == 0) {
    int h, sv, v;
    rgb_to_hsv(x, y, z, &h, &sv, &v);
    x = h, y = sv, z = v;
  } else if (op == 1) {
    hsv_to_rgb(x, y, z, &x, &y, &z);
  } else {
    hue_shift(x, y, z, param);
  }
  out[3 * (int64_t)idx] = (uint8_t)x;
  out[3 * (int64_t)idx + 1] = (uint8_t)y;
  out[3 * (int64_t)idx + 2] = (uint8_t)z;
}

hipError_t launch_pixel_ops(int op, int param, uint8_t* out, hipStream_t s) {
  k_pixel_ops<<<(1 << 24) / 256, 256, 0, s>>>(op, param, out);
  return hipGetLastError();
}

hipError_t launch_copy_rgb(const ImgDesc* desc, int idx, const uint8_t* ws, uint8_t* dst, hipStream_t s) {
  k_copy_rgb<<<256, 256, 0, s>>>(desc, idx, ws, dst);
  return hipGetLastError();
}

hipError_t launch_copy_rgb_packed(const ImgDesc* desc, int B, int n, const int32_t* idx, const int64_t* off,
                                  const uint8_t* ws, uint8_t* base, int header, hipStream_t s) {
  if (n <= 0) return hipSuccess;
  k_copy_rgb_packed<<<dim3(16, n), 256, 0, s>>>(desc, B, idx, off, ws, base, header);
  return hipGetLastError();
}

hipError_t launch_masks(int H, int W, int target, int minp, int maxp, double la0, double la1, int n, uint32_t* py,
                        uint32_t* np, uint8_t* out, hipStream_t s) {
  MaskParams mp{H, W, target, minp, maxp, la0, la1};
  if ((int64_t)H * W > kMaskLdsMaxPatches) return hipErrorInvalidValue;
  k_masks<<<1, 64, 5 * H * W + 16, s>>>(mp, n, py, np, out);
  return hipGetLastError();
}

#ifdef DINO_HUFF_PHASES
hipError_t copy_huff_phases(uint64_t* host, int64_t n_items) {
  hipError_t e = hipDeviceSynchronize();
  if (e != hipSuccess) return e;
  const int64_t n = n_items < kPhaseItems ? n_items : kPhaseItems;
  return hipMemcpyFromSymbol(host, HIP_SYMBOL(g_huff_phase), sizeof(uint64_t) * 5 * n);
}
#endif

hipError_t launch_bf16_to_fp8(const uint16_t* in, uint8_t* out, int64_t n, hipStream_t s) {
  if (n <= 0) return hipSuccess;
  int64_t blocks = (n + 255) / 256;
  if (blocks > 4096) blocks = 4096;
  k_bf16_to_fp8<<<(unsigned)blocks, 256, 0, s>>>(in, out, n);
  return hipGetLastError();
}

}  // namespace dino
