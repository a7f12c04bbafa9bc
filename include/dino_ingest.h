/*
 * dino_ingest.h — C ABI of the MI355X-native DINO Stage-3 ingest backend.
 *
 * This is the drop-in boundary for the reference's CPU hot path: everything
 * that ``CPUBackend``'s ``CPUAugPipeline.run_one_batch`` does per batch
 * (reference src/dino_loader/backends/cpu.py:309-367 — decode, random-resized
 * crop x N views, colour jitter, grayscale, gaussian blur, solarize,
 * normalize+cast) plus the iBOT mask generator (reference
 * src/dino_loader/masking.py:148-172) and the Stage-5 FP8 cast (reference
 * src/dino_loader/memory.py:193-214), as plain-pointer entry points.
 *
 * Conventions
 *  - Every entry point returns int status: DINO_OK (0) or a negative DINO_E*;
 *    dino_last_error() gives a thread-local message.  No C++ exception crosses
 *    the ABI.
 *  - Pointers named d_* are device (HBM) pointers; "stream" is a hipStream_t
 *    passed as void*.  All work is enqueued on that stream; nothing blocks the
 *    host unless stated.
 *  - One dino_ctx per device; a ctx is not thread-safe (callers serialise),
 *    several ctx may run concurrently on different devices/streams.
 *  - Per-image status codes (d_info[i][0]): 0 ok, <0 the reference would have
 *    raised inside Image.open/convert (cpu.py:250-253) -> zero-filled output
 *    (the reference's own semantics), >0 the reference decodes the image but this
 *    call did not (a flavour the GPU decoder does not implement, or workspace
 *    capacity) -> zero-filled output and the caller is expected to recover: the
 *    Python layer pre-screens host batches with dino_probe, grows the workspaces
 *    with dino_reserve and hands flavours it cannot decode over as pre-decoded
 *    RGB images (DINO_RAW_MAGIC below), so the product path never zero-fills an
 *    image the reference would have decoded (status > 0 left after a hand-over is
 *    counted per batch by the Python layer and raised as a RuntimeWarning).
 *  - Input images are JPEG byte strings, or pre-decoded RGB images in the raw
 *    container: 16-byte header {uint32 DINO_RAW_MAGIC, uint32 width, uint32
 *    height, uint32 0} followed by width*height*3 bytes of HWC RGB.  A container
 *    is only accepted where the caller marks it in the raw mask (uint8 per image,
 *    nullable = no containers): the magic is never trusted inside user data.
 *  - ABI 3 (from 2): raw masks on dino_decode / dino_run_batch / dino_probe, a
 *    stream on dino_reserve (stream-ordered growth, no device-wide sync), and
 *    max_image_dim 0 = no side limit (65535).
 *  - ABI 4 (from 3, additive): "spans" input (dino_decode_spans, dino_run_batch_spans,
 *    dino_probe_spans) so that a batch can be copied to HBM as the contiguous byte
 *    ranges of mapped tar shards it lies in, tar headers and sidecars included, with no
 *    host gather; dino_host_register / dino_host_unregister / dino_copy_h2d to page-lock
 *    those mappings and DMA from them; dino_gather_probe (pack + probe in one threaded
 *    pass); the native shard feed dino_feed_* (the host half of a batch off the Python
 *    interpreter).  Round 6, still additive within ABI 4: dino_tar_index_fd (header-only
 *    tar index over a file descriptor), dino_ctx_set_prog_decoder (wave / lane decoder of
 *    progressive images per context), dino_copy_rgb_packed (a pool's images into one
 *    buffer in one launch).
 */
#ifndef DINO_INGEST_H
#define DINO_INGEST_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define DINO_ABI_VERSION 4

/* return codes */
#define DINO_OK 0
#define DINO_EINVAL (-1)
#define DINO_ENOMEM (-2)
#define DINO_EHIP (-3)
#define DINO_ECAPACITY (-4)
#define DINO_EFORMAT (-5)            /* input is not in the expected format (e.g. not a tar) */
#define DINO_ERANGE (-6)             /* caller-provided output capacity too small */
/* positive warnings of dino_tar_index (the samples before the fault are reported) */
#define DINO_TAR_TRUNCATED 1         /* a member's data runs past the buffer (tarfile ReadError) */
#define DINO_TAR_BAD_HEADER 2        /* invalid header after offset 0 (tarfile stops iterating) */

/* per-image status codes */
#define DINO_IMG_OK 0
#define DINO_IMG_CORRUPT (-1)        /* not a JPEG / malformed header / bad table */
#define DINO_IMG_TRUNCATED (-2)      /* entropy data ends before the last MCU, no EOI */
#define DINO_IMG_BADDATA (-3)        /* libjpeg would error (bad sampling, MCU too large) */
#define DINO_IMG_TOO_LARGE (-4)      /* > 2 x PIL.Image.MAX_IMAGE_PIXELS: Pillow raises DecompressionBombError */
#define DINO_IMG_UNSUPPORTED 1       /* arithmetic / lossless / hierarchical / >8-bit / CMYK / 2-component,
                                        progressive needing libjpeg block smoothing, > DINO_MAX_SCANS scans */
#define DINO_IMG_MULTISCAN 2         /* (ABI v1; no longer produced: multi-scan files are decoded) */
#define DINO_IMG_NO_SPACE 3          /* the ctx workspace could not hold the image or one of its views
                                        (dino_reserve more and run again) */
#define DINO_IMG_LIMIT 4             /* JPEG width or height above a caller-chosen max_image_dim (the
                                        default has no side limit; the Python layer hands these to Pillow) */

/* raw pre-decoded RGB container ("DRGB" little-endian) */
#define DINO_RAW_MAGIC 0x42475244u
/* scans of one progressive / multi-scan image the device decoder accepts */
#define DINO_MAX_SCANS 64

/* output dtypes */
#define DINO_OUT_BF16 0
#define DINO_OUT_FP32 1
#define DINO_OUT_FP8_E4M3 2

typedef struct dino_ctx dino_ctx;

/* Pre-allocation ceilings (reference config.py:236-237 max_*_crop_size). */
typedef struct dino_limits {
  int32_t max_batch;           /* images per call */
  int32_t max_views;           /* views per image (n_global + n_local) */
  int32_t max_crop_size;       /* largest S of any view (<= 1024) */
  int32_t max_image_dim;       /* largest JPEG width or height accepted; 0 (default) -> 65535, i.e. no
                                  side limit (only Pillow's decompression-bomb pixel count applies) */
  int64_t workspace_bytes;     /* decode workspace (HBM); 0 -> default */
} dino_limits;

/* Augmentation hyper-parameters (reference DINOAugConfig, config.py:243-272). */
typedef struct dino_aug_config {
  int32_t n_global, n_local;
  int32_t global_size, local_size;
  float global_scale[2], local_scale[2];
  float blur_prob_global1, blur_prob_global2, blur_prob_local;
  float solarize_prob, color_jitter_prob, grayscale_prob, flip_prob;
  float blur_sigma_min, blur_sigma_max;
  float brightness, contrast, saturation, hue;
  float mean[3], std[3];
  int32_t out_dtype;           /* DINO_OUT_* */
  int32_t recipe;              /* DINO_RECIPE_*: how dino_sample_params draws the views */
} dino_aug_config;

/* View recipes of dino_sample_params (reference backends/cpu.py):
 *  DINOV2  n_global + n_local multi-crop (CPUAugPipeline, cpu.py:309-367);
 *  LEJEPA  view 0 = context: RandomResizedCrop(global_size, global_scale), ColorJitter with
 *          probability color_jitter_prob, flip with probability flip_prob; views 1.. =
 *          targets: RandomResizedCrop(local_size, local_scale) only (CPULeJEPAPipeline,
 *          cpu.py:421-461);
 *  EVAL    one view: Resize(shorter side -> int(global_size * 256 / 224), BICUBIC) then
 *          CenterCrop(global_size) (CPUEvalPipeline, cpu.py:380-413). */
#define DINO_RECIPE_DINOV2 0
#define DINO_RECIPE_LEJEPA 1
#define DINO_RECIPE_EVAL 2

/* Every random decision of one (sample, view) — reference cpu.py:172-267.
 * 80 bytes, layout shared with dataloader_amd/params.py (numpy dtype).
 * Geometry: the view is the window [out_x, out_x + S) x [out_y, out_y + S) of the
 * crop box resized (Pillow BICUBIC) to resize_w x resize_h; resize_w/h = 0 mean S
 * (RandomResizedCrop), a window needs the crop box itself to be resampled. */
typedef struct dino_view_params {
  int32_t crop_top, crop_left, crop_h, crop_w;   /* RandomResizedCrop (i, j, h, w) */
  int32_t out_size;                              /* S */
  uint8_t flip, jitter, gray, blur;
  uint8_t solarize, pad0[3];
  uint8_t order[4];                              /* ColorJitter op order 0=B 1=C 2=S 3=H */
  float brightness, contrast, saturation, hue;   /* ColorJitter factors */
  double sigma;                                  /* blur sigma */
  int32_t ksize;                                 /* blur kernel size */
  int32_t pad1;
  int32_t resize_w, resize_h;                    /* resample target of the crop box (0 -> S) */
  int32_t out_x, out_y;                          /* view window inside the resampled box */
} dino_view_params;

/* Library / context */
int dino_abi_version(void);
const char* dino_last_error(void);
int dino_ctx_create(int device, const dino_limits* limits, dino_ctx** out);
int dino_ctx_destroy(dino_ctx* ctx);

/* Stage 3, decode half: JPEG bytes -> RGB planes kept in the ctx workspace.
 * d_bytes: packed JPEG bytes, d_offsets: int64[batch+1] byte offsets.
 * d_raw_mask (nullable): uint8[batch], 1 where the image is a raw RGB container.
 * d_info (nullable): int32[batch][4] = {status, width, height, components}. */
int dino_decode(dino_ctx* ctx, const uint8_t* d_bytes, const int64_t* d_offsets, const uint8_t* d_raw_mask,
                int32_t batch, int32_t* d_info, void* stream);

/* Spans form of dino_decode: image i is d_bytes[d_offsets[i], d_offsets[i] + d_lengths[i])
 * (d_lengths nullable: d_offsets[i+1] - d_offsets[i]); d_offsets[batch] is the size of the
 * d_bytes buffer (bytes between and after images are ignored: e.g. the tar headers and
 * sidecars of a shard range copied as a whole).  Replaces the per-sample bytes(mv)
 * copies of reference hpc_source.py:360 / shard_reader.py:346-376 on the device feed. */
int dino_decode_spans(dino_ctx* ctx, const uint8_t* d_bytes, const int64_t* d_offsets, const int64_t* d_lengths,
                      const uint8_t* d_raw_mask, int32_t batch, int32_t* d_info, void* stream);

/* Copy decoded image i (HWC uint8 RGB, pitch = width*3) to d_rgb (debug / tests). */
int dino_copy_rgb(dino_ctx* ctx, int32_t index, uint8_t* d_rgb, void* stream);

/* Copy n decoded images at once (round 6, the side decoder's raw containers): image
 * d_index[k] of the last call (device int32[n]) to d_base + d_offset[k] (device int64[n]),
 * one launch for the whole pool; with d_base NULL, d_offset[k] is the destination's device
 * address.  flags DINO_COPY_HEADER: the 16 bytes before each destination get the raw
 * container header {DINO_RAW_MAGIC, width, height, 0}.  Images that did not decode, and
 * indices outside the last call's batch, are skipped.  n <= 65535. */
#define DINO_COPY_HEADER 1
int dino_copy_rgb_packed(dino_ctx* ctx, int32_t n, const int32_t* d_index, const int64_t* d_offset, uint8_t* d_base,
                         int32_t flags, void* stream);

/* The per-pixel colour operators of the ColorJitter hue op over all 2^24 inputs
 * (index = a << 16 | b << 8 | c; d_out: 3 * 2^24 bytes, out[3 * index + k]): op 0 RGB -> HSV
 * (Pillow convert("HSV")), op 1 HSV -> RGB (convert("RGB")), op 2 the hue shift by
 * `param` (torchvision adjust_hue's PIL path).  Tests / verification only. */
int dino_pixel_ops_all(int32_t op, int32_t param, uint8_t* d_out, void* stream);

/* Sample view params on device (counter-based Philox keyed by seed, batch_index,
 * sample, view) for the last decoded batch; writes batch*n_views records. */
int dino_sample_params(dino_ctx* ctx, const dino_aug_config* cfg, uint64_t seed, uint64_t batch_index,
                       dino_view_params* d_params, void* stream);

/* Stage 3, augment half: for every image of the last decoded batch and every view v,
 * write views[v] = [batch, 3, S_v, S_v] (dtype cfg->out_dtype, NCHW contiguous).
 * views: HOST array of n_views DEVICE pointers (copied into the ctx before return).
 * d_params: batch*n_views records (sample-major). Zero-fills images with status != 0. */
int dino_augment(dino_ctx* ctx, const dino_aug_config* cfg, const dino_view_params* d_params,
                 void* const* views, void* stream);

/* One call = decode + sample params + augment (CPUAugPipeline.run_one_batch).
 * d_params_out (nullable) receives the sampled records. */
int dino_run_batch(dino_ctx* ctx, const uint8_t* d_bytes, const int64_t* d_offsets, const uint8_t* d_raw_mask,
                   int32_t batch, const dino_aug_config* cfg, uint64_t seed, uint64_t batch_index,
                   dino_view_params* d_params_out, void* const* views, int32_t* d_info,
                   void* stream);

/* dino_run_batch on the spans form of dino_decode_spans. */
int dino_run_batch_spans(dino_ctx* ctx, const uint8_t* d_bytes, const int64_t* d_offsets, const int64_t* d_lengths,
                         const uint8_t* d_raw_mask, int32_t batch, const dino_aug_config* cfg, uint64_t seed,
                         uint64_t batch_index, dino_view_params* d_params_out, void* const* d_views,
                         int32_t* d_info, void* stream);

/* Decode-only recipe (reference CPUUserAugPipeline.run_one_batch, cpu.py:484-500, and the
 * DALI decode-only graph, pipeline.py:693-756): every image of the last decoded batch
 * resampled whole (Pillow BICUBIC) to out_w x out_h, normalised ((p / 255 - mean) / std,
 * or the dino_set_norm statistics) and cast into d_out = [batch, 3, out_h, out_w] NCHW.
 * Images with status != 0 are zero-filled.  The caller applies UserAugSpec.aug_fn to the
 * result (the reference stacks per-image tensors, so all images of a batch must resize
 * to the same shape; the Python layer checks that before calling). */
int dino_resize_batch(dino_ctx* ctx, int32_t out_w, int32_t out_h, const float* mean, const float* std,
                      int32_t out_dtype, void* d_out, void* stream);

/* Per-image status of the last batch after augmentation (the decode status, or
 * DINO_IMG_NO_SPACE when one of the image's views did not fit the augment workspace):
 * d_info: int32[batch][4] as dino_decode's. */
int dino_batch_info(dino_ctx* ctx, int32_t* d_info, void* stream);

/* Host pre-screen of a batch held in HOST memory (same packing as dino_decode): runs
 * the device parser (and, for progressive / multi-scan files, its marker walk) on
 * the CPU.  info (nullable): int32[batch][4] = {status the device decode will report,
 * width, height, kind (0 baseline, 1 multi-scan, 2 raw RGB, -1 failed)}.  ws_need:
 * decode workspace bytes the batch needs; aws_need: an upper bound of the augment
 * workspace for cfg's views (0 when cfg is NULL).  Images with status > 0 are the
 * ones the caller should decode itself and pass as raw RGB (DINO_RAW_MAGIC).
 * raw_mask (nullable, HOST): as dino_decode's.
 * Replaces nothing in the reference (its decode cannot fail for capacity). */
int dino_probe(const uint8_t* bytes, const int64_t* offsets, const uint8_t* raw_mask, int32_t batch,
               int32_t max_image_dim, const dino_aug_config* cfg, int32_t* info, int64_t* ws_need,
               int64_t* aws_need);

/* dino_probe over images given as absolute HOST addresses + lengths (e.g. JPEG members
 * of mapped tar shards, as dino_gather's input), so a batch can be screened where it
 * lies without packing it. */
int dino_probe_spans(const uint64_t* ptrs, const int64_t* lens, const uint8_t* raw_mask, int32_t batch,
                     int32_t max_image_dim, const dino_aug_config* cfg, int32_t* info, int64_t* ws_need,
                     int64_t* aws_need);

/* dino_gather + dino_probe in one pass: nthreads copier threads pack the images (absolute
 * HOST addresses + lengths) into dst (streaming stores; dst_offsets[n+1] as dino_gather's)
 * and parse each image's header right after copying it (info / ws_need / aws_need as
 * dino_probe's, no raw containers).  The host half of a feed batch in one native call. */
int dino_gather_probe(const uint64_t* src_ptrs, const int64_t* lens, int32_t n, uint8_t* dst, int64_t dst_cap,
                      int64_t* dst_offsets, int32_t nthreads, int32_t max_image_dim, const dino_aug_config* cfg,
                      int32_t* info, int64_t* ws_need, int64_t* aws_need);

/* Page-lock a host range (e.g. a mapped /dev/shm shard, reference shard_cache.py:584-609)
 * for DMA: hipHostRegister, read-only where the runtime supports it.  Unregister only
 * after every copy from the range has retired. */
int dino_host_register(void* host, int64_t nbytes);
int dino_host_unregister(void* host);
/* Asynchronous host -> device copy on `stream` (a DMA when host lies in registered or
 * pinned memory). */
int dino_copy_h2d(void* d_dst, const void* host_src, int64_t nbytes, void* stream);

/* A stream on its own hardware queue (a CU-masked stream: the runtime never shares
 * its queue with other streams), for work that must not queue behind, or hold up,
 * the batch streams: the progressive side decode (dataloader_amd/progside.py).
 * cu_count == 0 or >= the device's CUs: every CU; else cu_count CUs spread evenly.
 * cu_count < 0: instead a non-blocking stream of the least priority (HIP keeps a pool of
 * GPU_MAX_HW_QUEUES queues per priority; torch's streams use the normal and high pools),
 * used once at creation so that streams made in a row take different queues: the
 * pipeline's batch slots and its H2D copy stream (DINO_ROLE_STREAMS=low). */
int dino_stream_create(int device, int32_t cu_count, void** stream);
int dino_stream_destroy(void* stream);

/* Grow the ctx's decode / augment workspaces to at least the given sizes (never
 * shrinks), stream-ordered on `stream` (the stream the ctx's batches run on): the old
 * buffers are released after the work already enqueued there, nothing else on the
 * device waits (switching to another stream first synchronises the previous one).
 * Growing the decode workspace invalidates the last decoded batch; growing only the
 * augment workspace keeps it (dino_augment may run on it again, e.g. at new crop sizes). */
int dino_reserve(dino_ctx* ctx, int64_t ws_bytes, int64_t aws_bytes, void* stream);

/* Augment-workspace bound of a probed batch for cfg's views: info is dino_probe's
 * int32[batch][4] (HOST), aws_need as dino_probe's.  Lets a caller re-augment a decoded
 * batch at other crop sizes (a resolution change with batches in flight) after growing
 * the augment workspace, without the batch's bytes. */
int dino_augment_need(const int32_t* info, int32_t batch, const dino_aug_config* cfg, int64_t* aws_need);
int dino_workspace_sizes(dino_ctx* ctx, int64_t* ws_bytes, int64_t* aws_bytes);

/* iBOT block masks (reference MaskingGenerator.__call__, masking.py:148-172).
 * d_py_state: uint32[625] = CPython random.getstate() words + index;
 * d_np_state: uint32[625] = numpy RandomState MT19937 key + pos.
 * Both are advanced in place, exactly as n_masks sequential gen() calls would.
 * d_out: bool/uint8 [n_masks, height*width]. */
int dino_masks(int32_t height, int32_t width, int32_t num_masking_patches, int32_t min_num_patches,
               int32_t max_num_patches, double log_aspect_min, double log_aspect_max, int32_t n_masks,
               uint32_t* d_py_state, uint32_t* d_np_state, uint8_t* d_out, void* stream);
/* The same generator on the host (HOST pointers; no GPU involved): the reference-API
 * MaskingGenerator.__call__ uses it so that no batch synchronises a device stream.
 * dino_masks (device) accepts grids of up to 8192 patches, the host version any. */
int dino_masks_host(int32_t height, int32_t width, int32_t num_masking_patches, int32_t min_num_patches,
                    int32_t max_num_patches, double log_aspect_min, double log_aspect_max, int32_t n_masks,
                    uint32_t* py_state, uint32_t* np_state, uint8_t* out);

/* Decoder of this ctx's coefficient-buffer (progressive / multi-scan) images, from the next
 * call on (round 6): DINO_PROG_WAVE (the default, or DINO_PROG_LANE=1 in the environment at
 * dino_ctx_create) decodes one scan per wave (k_pscan, ~28 ms per libjpeg-default 640x480
 * file); DINO_PROG_LANES decodes scan j of 64 images in the lanes of one wave (k_plscan +
 * k_papply) where the image's scan script allows it (else the wave decoder): lower GPU cost
 * per image, several times the latency, so it pays for large pools decoded well ahead of
 * their batches (the side route's look-ahead).  Results are identical.  No reference
 * counterpart: Pillow decodes one image at a time on a CPU thread (cpu.py:251). */
#define DINO_PROG_WAVE 0
#define DINO_PROG_LANES 1
int dino_ctx_set_prog_decoder(dino_ctx* ctx, int32_t decoder);

/* Per-kernel HIP-event timing of this ctx's launches (bench / profiling).
 * Kernel ids: 0 parse, 1 plan, 2 destuff, 3 huff1, 4 idct, 5 color, 6 params,
 * 7 vplan, 8 rcoeffs, 9 hresize, 10 final(global views), 11 final(local views),
 * 12 vert(global views), 13 vert(local views), 14 dcscan, 15 htab, 16 hseg,
 * 17 huff2, 18 huff3, 19 prog (progressive / multi-scan decode).
 * dino_kernel_times synchronises the recorded events, returns the sums since the
 * last call (ms, launches) and resets them. */
int dino_set_timing(dino_ctx* ctx, int32_t enable);
int dino_kernel_times(dino_ctx* ctx, double* total_ms, int64_t* counts, int32_t n);

/* Debug / test introspection of the last decoded batch: copy image `index`'s
 * region (0 descriptor, 1 destuffed entropy bytes, 2 sparse DCT coefficient entries + block info,
 * 3 component planes, 4 RGB, 5 speculative Huffman lane records: 68 bytes per lane =
 * start state, range result, first-decode result, checkpoints, first block, 6 the scan-list
 * header of a kind-1 image: 832 bytes, int32 at byte 776 = 1 when the lane decoder took it)
 * into d_dst (<= max_bytes).  Synchronises the stream. */
int dino_debug_region(dino_ctx* ctx, int32_t index, int32_t region, void* d_dst, int64_t max_bytes, void* stream);

/* Per-dataset normalisation (reference NormSource, pipeline.py:109-180, and
 * build_norm_arrays, norm_utils.py:51-88 — DALI-only in the reference): d_norm is a
 * device array of n records {mean[3], std[3]} in [0, 1] scale, one per image of the
 * batch, used by every later dino_augment / dino_run_batch on this ctx instead of
 * cfg->mean / cfg->std (x = (p / 255 - mean) / std, as the CPU path computes).  NULL
 * restores the global statistics.  The array must stay valid while those calls run. */
int dino_set_norm(dino_ctx* ctx, const float* d_norm, int32_t n);

/* Stage-5 cast (reference FP8Formatter.quantise, memory.py:193-214, scale 1):
 * bf16 -> OCP float8_e4m3fn, round-to-nearest-even, bit-identical to torch's
 * .to(torch.float8_e4m3fn) (c10 fp8e4m3fn_from_fp32_value: |x| >= 480 -> NaN).
 * The reference's TE cast_to_fp8 saturates to +-448 instead; the two agree on
 * every normalised pixel value (|x| < 3), which is all this path produces. */
int dino_bf16_to_fp8(const uint16_t* d_in, uint8_t* d_out, int64_t n, void* stream);

/* ---- Host-side shard ingest (tario.cpp) ---------------- */

/* One WebDataset sample of a tar shard: byte ranges inside the tar buffer (-1 when
 * the member is absent) and its key (into the caller's key buffer, -1 if it did
 * not fit; key_len is always the full length). */
typedef struct dino_tar_sample {
  int64_t img_off, img_len;    /* .jpg / .jpeg member */
  int64_t meta_off, meta_len;  /* .json sidecar */
  int64_t key_off;
  int32_t key_len;
  int32_t reserved;
} dino_tar_sample;

/* Index a tar shard held in memory (e.g. the mmap of a /dev/shm shard-cache file
 * past its 16-byte header, reference shard_cache.py:83-85, 584-609): members are
 * grouped into samples by WebDataset key; samples without an image are skipped.
 * Replaces the tar walk of dino_loader.datasets.utils._extract_jpegs_with_meta
 * (absent dependency; called at reference hpc_source.py:461-467).  Returns DINO_OK,
 * a positive DINO_TAR_* warning (samples before the fault are valid), or < 0. */
int dino_tar_index(const uint8_t* tar, int64_t len, dino_tar_sample* out, int64_t cap, char* keys, int64_t keys_cap,
                   int64_t* n_samples, int64_t* n_members);
/* The same walk over a file (the shard-cache file's fd, tar bytes [base, base + len)): only
 * the 512-byte headers and pax / long-name records are read (pread), so indexing a shard
 * never faults its members' data in (the native feed's openers). */
int dino_tar_index_fd(int32_t fd, int64_t base, int64_t len, dino_tar_sample* out, int64_t cap, char* keys,
                      int64_t keys_cap, int64_t* n_samples, int64_t* n_members);
const char* dino_tar_last_error(void);

/* Pack n byte ranges (absolute host addresses, e.g. JPEG members of mapped shards)
 * into dst (pinned host memory) back to back; dst_offsets[n+1] receives the int64
 * offsets dino_run_batch reads.  nthreads copier threads (1 below 1 MiB).  Replaces
 * the per-sample bytes(mv) copies of reference hpc_source.py:360 and the batch
 * assembly of shard_reader.py:346-376. */
int dino_gather(const uint64_t* src_ptrs, const int64_t* lens, int64_t n, uint8_t* dst, int64_t dst_cap,
                int64_t* dst_offsets, int32_t nthreads);

/* ---- Native shard feed (feed.hip): the host half of a batch without Python -------
 * An opener thread maps shard-cache files ([data_len:u64][magic:u64] + tar, reference
 * shard_cache.py:83-85), faults them in and indexes them (dino_tar_index) a few shards
 * ahead; a packer thread packs each batch of `batch` consecutive samples (straddling
 * shards; the last partial batch of an epoch is dropped, dali_backend.py:187) into a
 * pinned slot with `nthreads` copier threads, probing every image right after its copy.
 * Replaces ShardIterator / MixingSource's per-sample extraction + bytes(mv) copies
 * (reference hpc_source.py:329-385, :405-478) and _ReaderAdapter.__call__
 * (shard_reader.py:346-376) for the device backend.  Shard I/O errors are reported once
 * (DINO_FEED_SHARD_ERROR) and the shard is skipped (hpc_source.py:358-366). */
typedef struct dino_feed dino_feed;
typedef struct dino_feed_batch {
  int32_t slot;                /* pass to dino_feed_copy / dino_feed_release */
  int32_t n;                   /* images (= batch) */
  int64_t nbytes;              /* packed bytes */
  const uint8_t* host;         /* pinned packed bytes (valid until the slot's copy retires / release) */
  const int64_t* offsets;      /* int64[n+1], pinned */
  const int32_t* info;         /* int32[n][4] as dino_probe's */
  int64_t ws_need, aws_need;   /* as dino_probe's (aws for the feed's cfg) */
  int64_t seq;                 /* batch number since the feed was created */
} dino_feed_batch;
#define DINO_FEED_END 1            /* dino_feed_next: the epoch has no more batches */
#define DINO_FEED_TIMEOUT 2        /* dino_feed_next: nothing ready within timeout_ms */
#define DINO_FEED_SHARD_ERROR 3    /* dino_feed_next: a shard could not be read (skipped; dino_feed_last_error) */
int dino_feed_create(int32_t batch, int32_t nthreads, int32_t nslots, int32_t lookahead, int32_t max_image_dim,
                     const dino_aug_config* cfg, dino_feed** out);
int dino_feed_destroy(dino_feed* feed);
int dino_feed_push(dino_feed* feed, const char* shard_cache_path);
int dino_feed_end_epoch(dino_feed* feed);
int dino_feed_set_cfg(dino_feed* feed, const dino_aug_config* cfg);
/* Non-master ranks: wait up to timeout_ms for a pushed shard-cache file the node master has
 * not written yet (reference NodeSharedShardCache.get_view -> _inotify_wait,
 * shard_cache.py:596-603, :373-449: inotify on the cache directory, stat-poll fallback);
 * a shard still missing then is reported as DINO_FEED_SHARD_ERROR ("Timed out ...") and
 * skipped (hpc_source.py:358-366).  0 (default): a shard must be ready when opened. */
int dino_feed_set_shard_wait(dino_feed* feed, int32_t timeout_ms);
/* enable != 0: each shard's samples are taken in a seeded random order keyed by (seed, epoch,
 * shard path) (the extraction step's shuffle buffer, hpc_source.py:461-467). */
int dino_feed_set_shuffle(dino_feed* feed, int32_t enable, uint64_t seed);
/* The epoch that keys the shuffle of the shards opened from now on (default: epochs since create,
 * i.e. dino_feed_reset calls), so that a job resumed at epoch k gets epoch k's sample order
 * (reference ShardIterator.reset_epoch, hpc_source.py:242-273). */
int dino_feed_set_epoch(dino_feed* feed, uint64_t epoch);
/* Next packed batch in order (blocks up to timeout_ms; < 0: forever). */
int dino_feed_next(dino_feed* feed, int32_t timeout_ms, dino_feed_batch* out);
/* H2D copies of a handed-out slot (bytes, offsets) on `stream`; the slot is reused after they retire. */
int dino_feed_copy(dino_feed* feed, int32_t slot, uint8_t* d_bytes, int64_t* d_offsets, void* stream);
/* Hand a slot back without copying it (the caller copied what it needed). */
int dino_feed_release(dino_feed* feed, int32_t slot);
/* New epoch: drops pushed shards and packed batches not handed out. */
int dino_feed_reset(dino_feed* feed);
/* seconds[4] = open+fault+index, pack+probe, waiting for a free slot, waiting for samples;
 * counts[3] = batches packed, shards consumed, shards failed. */
int dino_feed_stats(dino_feed* feed, double* seconds, int64_t* counts);
const char* dino_feed_last_error(void);

#ifdef __cplusplus
}
#endif
#endif /* DINO_INGEST_H */
