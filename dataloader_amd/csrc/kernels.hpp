// kernels.hpp — launch interface between the C ABI (capi.hip) and kernels.hip.
#pragma once

#include "common.hpp"

namespace dino {

// Per-(image, view) scratch placement, written by k_vplan.
// Lanes of k_huffman (one workgroup per image).
constexpr int kHuffThreads = 256;
// Bits of entropy-coded stream per Huffman work item (kHuffThreads lanes); an image
// larger than this is decoded by several workgroups (k_huff1 / k_huff3).
#ifndef DINO_HUFF_SEG_KBITS
#define DINO_HUFF_SEG_KBITS 2048
#endif
constexpr int64_t kHuffSegBits = (int64_t)DINO_HUFF_SEG_KBITS * 1024;

// LDS of k_hresize: taps (when they fit in kHresizeTapLds) + planar rows of one band.
constexpr int kHresizeLds = 26 * 1024;

struct ViewPlan {
  int64_t htmp_off;   // horizontal-pass rows (crop_h x S x 3 u8) in the augment workspace
  int64_t rcoef_off;  // resize coefficient tables
  int32_t kh, kv;     // taps per output of the horizontal / vertical pass (0 = pass skipped)
  int32_t ok;         // image decoded and scratch available
  uint32_t lsum;      // sum of L over the crop before the contrast op (k_vert atomics)
  int32_t hr_chunks;  // k_hresize work items of the view (k_vsizes)
  int32_t hr_base;    // its first work item among its class's views (global / local, k_vplan)
};


// Optional per-kernel HIP-event timing (bench / profiling).  Events are recorded on
// the launch stream around each kernel; elapsed times are summed on demand.
enum KernelId : int {
  kKParse = 0, kKPlan, kKDestuff, kKHuff1, kKIdct, kKColor, kKParams, kKVplan, kKRcoeffs, kKHresize,
  kKFinalGlobal, kKFinalLocal, kKVertGlobal, kKVertLocal, kKDcscan, kKHtab, kKHseg, kKHuff2, kKHuff3, kKProg,
  kKPwalk, kKPlscan, kKPapply, kKNumKernels
};

struct KernelTimer {
  static constexpr int kMaxPending = 4096;
  hipEvent_t ev[kMaxPending][2];
  int id[kMaxPending];
  int n = 0;
  bool enabled = false;
  bool created = false;
  double total_ms[kKNumKernels];
  int64_t count[kKNumKernels];
  void begin(int k, hipStream_t s);
  void end(hipStream_t s);
  void collect();  // synchronises the recorded events, accumulates, resets the pending list
  void reset();
  void destroy();
};

// Launch geometry of one device (computed per ctx by dino_ctx_create).
struct LaunchGeom {
  int32_t grid_ds;   // persistent destuff grid
  int32_t grid1;     // persistent k_huff1 grid (occupancy x CUs)
  int32_t grid3;     // persistent k_huff3 grid
  int32_t grid_ps;   // persistent k_pscan grid (waves)
  int32_t grid_ls;   // persistent k_plscan grid (one-wave workgroups)
  int32_t prog_lane; // 1: eligible progressive images take k_plscan (DINO_PROG_LANE=0: all k_pscan)
  int32_t scan_prio; // 1: scan waves at the batch kernels' issue priority (DINO_SCAN_PRIO)
  int32_t grid_hr;   // persistent k_hresize grid (occupancy x CUs)
};

// Coefficient-buffer images of a batch (k_plan zeroes, k_pwalk registers, k_pscan
// takes tickets): ticket t = scan t / nprog of image pimg[t % nprog] (each image's scans
// in dependency-level order, so a scan only ever waits for scans with earlier tickets).
// Lane images (k_plscan, lscan.hpp) register from the other end: limg(k) = pimg[cap - 1 - k];
// lticket t = scan t / ngroups of the 64-image group t % ngroups.
struct PCtl {
  uint32_t ticket, nprog, max_scans, cap;
  uint32_t lticket, nlane, lmax_scans, pad;
  int32_t pimg[1];  // [max_batch]
};
DHD int64_t pctl_bytes(int max_batch) { return 32 + 4 * (int64_t)(max_batch > 0 ? max_batch : 1); }
hipError_t init_launch_geom(int device, LaunchGeom* g);

struct DecodeArgs {
  const uint8_t* bytes;
  const int64_t* offsets;
  const int64_t* lengths;   // per image byte count (nullable: offsets[i+1] - offsets[i]); spans input
  const uint8_t* raw_mask;  // per image: 1 = pre-decoded RGB container (nullable: none)
  int32_t batch;
  int32_t max_dim;
  ImgDesc* desc;
  uint8_t* ws;
  int64_t ws_size;
  LaunchGeom geom;
  PCtl* pctl;
};

// Output pointers travel as a kernel argument (no host->device copy whose source
// could die before an asynchronous copy reads it).
constexpr int kMaxViews = 32;
struct ViewPtrs {
  void* p[kMaxViews];
};

struct AugmentArgs {
  ImgDesc* desc;
  int32_t batch;
  const dino_view_params* params;
  ViewPlan* plan;
  const uint8_t* ws;
  uint8_t* aws;
  int64_t aws_size;
  uint8_t* gcrop;          // u8 crop planes of every view (k_vert -> k_final)
  ViewPtrs views;          // n_views output pointers (device memory)
  dino_aug_config cfg;
  const float* norm;       // per-image {mean[3], std[3]} ([0, 1] scale), nullable -> cfg.mean / cfg.std
  int32_t grid_hr;         // LaunchGeom::grid_hr
};

// Decode-only recipe (dino_resize_batch).
struct DecodeOnlyArgs {
  ImgDesc* desc;
  int32_t batch, ow, oh, out_dtype;
  ViewPlan* plan;
  const uint8_t* ws;
  uint8_t* aws;
  int64_t aws_size;
  float mean[3], std[3];
  const float* norm;
  void* out;
};

hipError_t launch_decode(const DecodeArgs& a, hipStream_t s, KernelTimer* tm = nullptr);
hipError_t launch_decode_only(const DecodeOnlyArgs& a, hipStream_t s);
hipError_t launch_params(const ImgDesc* desc, int batch, const dino_aug_config& cfg, uint64_t seed,
                         uint64_t batch_index, dino_view_params* out, hipStream_t s, KernelTimer* tm = nullptr);
hipError_t launch_augment(const AugmentArgs& a, hipStream_t s, KernelTimer* tm = nullptr);
hipError_t launch_info(const ImgDesc* desc, int batch, int32_t* info, hipStream_t s);
hipError_t launch_copy_rgb(const ImgDesc* desc, int idx, const uint8_t* ws, uint8_t* dst, hipStream_t s);
hipError_t launch_copy_rgb_packed(const ImgDesc* desc, int B, int n, const int32_t* idx, const int64_t* off,
                                  const uint8_t* ws, uint8_t* base, int header, hipStream_t s);
hipError_t launch_pixel_ops(int op, int param, uint8_t* out, hipStream_t s);
hipError_t launch_masks(int H, int W, int target, int minp, int maxp, double la0, double la1, int n, uint32_t* py,
                        uint32_t* np, uint8_t* out, hipStream_t s);
#ifdef DINO_HUFF_PHASES
hipError_t copy_huff_phases(uint64_t* host, int64_t n_items);
#endif
#ifdef DINO_PROG_PHASES
hipError_t copy_prog_phases(uint64_t* host);
#endif
hipError_t launch_bf16_to_fp8(const uint16_t* in, uint8_t* out, int64_t n, hipStream_t s);

}  // namespace dino
