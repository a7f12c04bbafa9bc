// capi.hip — the C ABI declared in include/dino_ingest.h.
//
// A dino_ctx owns the device-side descriptors and two workspaces sized once
// from dino_limits (the pre-allocation ceilings of reference config.py:236-237):
// the decode workspace (destuffed entropy bytes, DCT coefficients, component
// planes, RGB images) and the augment workspace (horizontal-pass rows and
// resize coefficient tables).  Nothing is allocated per call and no call
// blocks the host: every entry point only enqueues work on the given stream.
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <string>
#include <thread>
#include <vector>

#include <hip/hip_ext.h>

#include "hostcopy.hpp"
#include "jpeg_parse.hpp"
#include "kernels.hpp"
#include "mask.hpp"
#include "plan.hpp"
#include "probe.hpp"
#include "progressive.hpp"

using namespace dino;

namespace {
thread_local std::string g_err;

int fail(int code, const char* fmt, const char* a = "", long long b = 0) {
  char buf[512];
  snprintf(buf, sizeof(buf), fmt, a, b);
  g_err = buf;
  return code;
}

int hip_fail(hipError_t e, const char* where) {
  char buf[512];
  snprintf(buf, sizeof(buf), "%s: %s", where, hipGetErrorString(e));
  g_err = buf;
  return DINO_EHIP;
}
}  // namespace

struct dino_ctx {
  int device = 0;
  dino_limits lim{};
  ImgDesc* d_desc = nullptr;
  uint8_t* d_ws = nullptr;
  int64_t ws_size = 0;
  uint8_t* d_aws = nullptr;
  int64_t aws_size = 0;
  ViewPlan* d_plan = nullptr;
  dino_view_params* d_params = nullptr;
  uint8_t* d_gcrop = nullptr;
  PCtl* d_pctl = nullptr;         // the batch's coefficient-buffer registry (k_plan / k_pwalk / k_pscan)
  const float* d_norm = nullptr;  // per-image normalisation (dino_set_norm), nullable
  int32_t norm_n = 0;
  int32_t last_batch = -1;
  hipStream_t ws_stream = nullptr;  // stream of the last dino_reserve (the workspaces' release order)
  LaunchGeom geom{};
  KernelTimer* timer = nullptr;
  KernelTimer* tm() { return timer && timer->enabled ? timer : nullptr; }
};

extern "C" {

int dino_abi_version(void) { return DINO_ABI_VERSION; }

const char* dino_last_error(void) { return g_err.c_str(); }

int dino_ctx_create(int device, const dino_limits* limits, dino_ctx** out) {
  if (!out || !limits) return fail(DINO_EINVAL, "dino_ctx_create: null argument%s%lld");
  *out = nullptr;
  dino_limits L = *limits;
  if (L.max_batch <= 0 || L.max_views <= 0 || L.max_crop_size <= 0)
    return fail(DINO_EINVAL, "dino_ctx_create: max_batch/max_views/max_crop_size must be > 0%s%lld");
  if (L.max_crop_size > 1024)  // k_final's LDS tile and its 32-bit index arithmetic are sized for S <= 1024
    return fail(DINO_EINVAL, "dino_ctx_create: max_crop_size %s%lld > 1024", "", L.max_crop_size);
  // JPEG sides are 16-bit: 0 (or anything above) means no side limit (the bomb limit of
  // jpeg_parse.hpp check_dims bounds every pixel index)
  if (L.max_image_dim <= 0 || L.max_image_dim > kMaxImageDim) L.max_image_dim = kMaxImageDim;
  hipError_t e = hipSetDevice(device);
  if (e != hipSuccess) return hip_fail(e, "hipSetDevice");
  dino_ctx* c = new dino_ctx();
  c->device = device;
  c->lim = L;
  if ((e = init_launch_geom(device, &c->geom)) != hipSuccess) {
    delete c;
    return hip_fail(e, "dino_ctx_create: launch geometry");
  }
  // decode workspace: default 16 MiB per image of the batch (a 1600x2133 JPEG needs ~26 MiB,
  // a 640x480 one ~2.4 MiB; images that do not fit are reported DINO_IMG_TOO_LARGE)
  c->ws_size = L.workspace_bytes > 0 ? L.workspace_bytes : (int64_t)L.max_batch * (16ll << 20);
  c->aws_size = (int64_t)L.max_batch * L.max_views * ((int64_t)L.max_crop_size * 3 * 1024 + (256ll << 10));
  const int64_t nrec = (int64_t)L.max_batch * L.max_views;
  // the two growable workspaces come from the stream-ordered allocator, so that dino_reserve
  // can retire them on the ctx's stream instead of synchronising the device
  if ((e = hipMalloc(&c->d_desc, sizeof(ImgDesc) * L.max_batch)) != hipSuccess ||
      (e = hipMallocAsync((void**)&c->d_ws, c->ws_size, nullptr)) != hipSuccess ||
      (e = hipMallocAsync((void**)&c->d_aws, c->aws_size, nullptr)) != hipSuccess ||
      (e = hipStreamSynchronize(nullptr)) != hipSuccess ||
      (e = hipMalloc(&c->d_plan, sizeof(ViewPlan) * (nrec + 1))) != hipSuccess ||  // + k_hresize's item counters
      (e = hipMalloc(&c->d_params, sizeof(dino_view_params) * nrec)) != hipSuccess ||
      (e = hipMalloc((void**)&c->d_pctl, pctl_bytes(L.max_batch))) != hipSuccess) {
    dino_ctx_destroy(c);
    return hip_fail(e, "dino_ctx_create: hipMalloc");
  }
  {  // u8 crop planes of every view between the vertical and final passes
    int64_t gb = (int64_t)L.max_batch * L.max_views * 3 * L.max_crop_size * L.max_crop_size;
    if ((e = hipMalloc(&c->d_gcrop, gb)) != hipSuccess) {
      dino_ctx_destroy(c);
      return hip_fail(e, "dino_ctx_create: hipMalloc(gcrop)");
    }
  }
  *out = c;
  return DINO_OK;
}

int dino_ctx_destroy(dino_ctx* c) {
  if (!c) return DINO_OK;
  (void)hipFree(c->d_desc);
  // (callers synchronise the ctx's streams before destroying it: the null stream suffices)
  if (c->d_ws) (void)hipFreeAsync(c->d_ws, nullptr);
  if (c->d_aws) (void)hipFreeAsync(c->d_aws, nullptr);
  (void)hipStreamSynchronize(nullptr);
  (void)hipFree(c->d_plan);
  (void)hipFree(c->d_params);
  (void)hipFree(c->d_gcrop);
  (void)hipFree(c->d_pctl);
  if (c->timer) {
    c->timer->destroy();
    delete c->timer;
  }
  delete c;
  return DINO_OK;
}

int dino_decode_spans(dino_ctx* c, const uint8_t* d_bytes, const int64_t* d_offsets, const int64_t* d_lengths,
                      const uint8_t* d_raw_mask, int32_t batch, int32_t* d_info, void* stream) {
  if (!c || !d_bytes || !d_offsets) return fail(DINO_EINVAL, "dino_decode: null argument%s%lld");
  if (batch < 0 || batch > c->lim.max_batch)
    return fail(DINO_EINVAL, "dino_decode: batch %s%lld exceeds ctx max_batch", "", batch);
  hipStream_t s = (hipStream_t)stream;
  DecodeArgs a{d_bytes, d_offsets, d_lengths, d_raw_mask, batch, c->lim.max_image_dim, c->d_desc, c->d_ws,
               c->ws_size, c->geom, c->d_pctl};
  hipError_t e = launch_decode(a, s, c->tm());
  if (e != hipSuccess) return hip_fail(e, "dino_decode");
  if (d_info && (e = launch_info(c->d_desc, batch, d_info, s)) != hipSuccess) return hip_fail(e, "dino_decode(info)");
  c->last_batch = batch;
  return DINO_OK;
}

int dino_decode(dino_ctx* c, const uint8_t* d_bytes, const int64_t* d_offsets, const uint8_t* d_raw_mask,
                int32_t batch, int32_t* d_info, void* stream) {
  return dino_decode_spans(c, d_bytes, d_offsets, nullptr, d_raw_mask, batch, d_info, stream);
}

int dino_copy_rgb(dino_ctx* c, int32_t index, uint8_t* d_rgb, void* stream) {
  if (!c || !d_rgb || index < 0 || index >= c->last_batch) return fail(DINO_EINVAL, "dino_copy_rgb: bad index%s%lld");
  hipError_t e = launch_copy_rgb(c->d_desc, index, c->d_ws, d_rgb, (hipStream_t)stream);
  return e == hipSuccess ? DINO_OK : hip_fail(e, "dino_copy_rgb");
}

int dino_copy_rgb_packed(dino_ctx* c, int32_t n, const int32_t* d_index, const int64_t* d_offset, uint8_t* d_base,
                         int32_t flags, void* stream) {
  if (!c || n < 0 || (n > 0 && (!d_index || !d_offset)) || (flags & ~DINO_COPY_HEADER))
    return fail(DINO_EINVAL, "dino_copy_rgb_packed: bad arguments%s%lld");
  if (n > 65535) return fail(DINO_EINVAL, "dino_copy_rgb_packed: n %s%lld > 65535", "", (long long)n);
  hipError_t e = launch_copy_rgb_packed(c->d_desc, c->last_batch, n, d_index, d_offset, c->d_ws, d_base,
                                        (flags & DINO_COPY_HEADER) != 0, (hipStream_t)stream);
  return e == hipSuccess ? DINO_OK : hip_fail(e, "dino_copy_rgb_packed");
}

int dino_pixel_ops_all(int32_t op, int32_t param, uint8_t* d_out, void* stream) {
  if (!d_out || op < 0 || op > 2) return fail(DINO_EINVAL, "dino_pixel_ops_all: bad args%s%lld");
  hipError_t e = launch_pixel_ops(op, param & 255, d_out, (hipStream_t)stream);
  return e == hipSuccess ? DINO_OK : hip_fail(e, "dino_pixel_ops_all");
}

static int check_cfg(const dino_ctx* c, const dino_aug_config* cfg) {
  if (!cfg) return fail(DINO_EINVAL, "null dino_aug_config%s%lld");
  const int nv = cfg->n_global + cfg->n_local;
  if (cfg->n_global < 0 || cfg->n_local < 0 || nv <= 0 || nv > c->lim.max_views)
    return fail(DINO_EINVAL, "view count %s%lld outside [1, max_views]", "", nv);
  if (cfg->global_size <= 4 || cfg->local_size <= 4 || cfg->global_size > c->lim.max_crop_size ||
      cfg->local_size > c->lim.max_crop_size)
    return fail(DINO_EINVAL, "crop size outside (4, max_crop_size]%s%lld");
  if (cfg->out_dtype < DINO_OUT_BF16 || cfg->out_dtype > DINO_OUT_FP8_E4M3)
    return fail(DINO_EINVAL, "unknown out_dtype %s%lld", "", cfg->out_dtype);
  if (cfg->recipe < DINO_RECIPE_DINOV2 || cfg->recipe > DINO_RECIPE_EVAL)
    return fail(DINO_EINVAL, "unknown recipe %s%lld", "", cfg->recipe);
  return DINO_OK;
}

int dino_sample_params(dino_ctx* c, const dino_aug_config* cfg, uint64_t seed, uint64_t batch_index,
                       dino_view_params* d_params, void* stream) {
  if (!c || !d_params) return fail(DINO_EINVAL, "dino_sample_params: null argument%s%lld");
  if (c->last_batch < 0) return fail(DINO_EINVAL, "dino_sample_params: no decoded batch%s%lld");
  int r = check_cfg(c, cfg);
  if (r) return r;
  hipError_t e = launch_params(c->d_desc, c->last_batch, *cfg, seed, batch_index, d_params, (hipStream_t)stream,
                                c->tm());
  return e == hipSuccess ? DINO_OK : hip_fail(e, "dino_sample_params");
}

int dino_augment(dino_ctx* c, const dino_aug_config* cfg, const dino_view_params* d_params, void* const* d_views,
                 void* stream) {
  if (!c || !d_params || !d_views) return fail(DINO_EINVAL, "dino_augment: null argument%s%lld");
  if (c->last_batch < 0) return fail(DINO_EINVAL, "dino_augment: no decoded batch%s%lld");
  int r = check_cfg(c, cfg);
  if (r) return r;
  const int nv = cfg->n_global + cfg->n_local;
  if (nv > kMaxViews) return fail(DINO_EINVAL, "dino_augment: more than %s%lld views", "", kMaxViews);
  if (c->d_norm && c->norm_n < c->last_batch)
    return fail(DINO_EINVAL, "dino_augment: dino_set_norm covers %s%lld images, fewer than the batch", "", c->norm_n);
  hipStream_t s = (hipStream_t)stream;
  AugmentArgs a{c->d_desc, c->last_batch, d_params, c->d_plan, c->d_ws, c->d_aws, c->aws_size, c->d_gcrop, {}, *cfg,
                c->d_norm, c->geom.grid_hr};
  for (int v = 0; v < nv; ++v) {
    if (!d_views[v]) return fail(DINO_EINVAL, "dino_augment: null output pointer for view %s%lld", "", v);
    a.views.p[v] = d_views[v];
  }
  hipError_t e = launch_augment(a, s, c->tm());
  return e == hipSuccess ? DINO_OK : hip_fail(e, "dino_augment");
}

int dino_set_norm(dino_ctx* c, const float* d_norm, int32_t n) {
  if (!c) return fail(DINO_EINVAL, "dino_set_norm: null ctx%s%lld");
  if (d_norm && n < 1) return fail(DINO_EINVAL, "dino_set_norm: %s%lld entries", "", n);
  c->d_norm = d_norm;
  c->norm_n = d_norm ? n : 0;
  return DINO_OK;
}

int dino_run_batch_spans(dino_ctx* c, const uint8_t* d_bytes, const int64_t* d_offsets, const int64_t* d_lengths,
                         const uint8_t* d_raw_mask, int32_t batch, const dino_aug_config* cfg, uint64_t seed,
                         uint64_t batch_index, dino_view_params* d_params_out, void* const* d_views, int32_t* d_info,
                         void* stream) {
  if (!c) return fail(DINO_EINVAL, "dino_run_batch: null ctx%s%lld");
  int r = check_cfg(c, cfg);
  if (r) return r;
  if ((r = dino_decode_spans(c, d_bytes, d_offsets, d_lengths, d_raw_mask, batch, nullptr, stream))) return r;
  dino_view_params* prm = d_params_out ? d_params_out : c->d_params;
  if ((r = dino_sample_params(c, cfg, seed, batch_index, prm, stream))) return r;
  if ((r = dino_augment(c, cfg, prm, d_views, stream))) return r;
  return d_info ? dino_batch_info(c, d_info, stream) : DINO_OK;
}

int dino_run_batch(dino_ctx* c, const uint8_t* d_bytes, const int64_t* d_offsets, const uint8_t* d_raw_mask,
                   int32_t batch, const dino_aug_config* cfg, uint64_t seed, uint64_t batch_index,
                   dino_view_params* d_params_out, void* const* d_views, int32_t* d_info, void* stream) {
  return dino_run_batch_spans(c, d_bytes, d_offsets, nullptr, d_raw_mask, batch, cfg, seed, batch_index,
                              d_params_out, d_views, d_info, stream);
}

int dino_resize_batch(dino_ctx* c, int32_t out_w, int32_t out_h, const float* mean, const float* stdv,
                      int32_t out_dtype, void* d_out, void* stream) {
  if (!c || !mean || !stdv || !d_out) return fail(DINO_EINVAL, "dino_resize_batch: null argument%s%lld");
  if (c->last_batch < 0) return fail(DINO_EINVAL, "dino_resize_batch: no decoded batch%s%lld");
  if (out_w < 1 || out_h < 1 || out_w > 65535 || out_h > 65535)
    return fail(DINO_EINVAL, "dino_resize_batch: output size %s%lld out of range", "", (long long)out_w * out_h);
  if (out_dtype < DINO_OUT_BF16 || out_dtype > DINO_OUT_FP8_E4M3)
    return fail(DINO_EINVAL, "dino_resize_batch: unknown out_dtype %s%lld", "", out_dtype);
  if (c->d_norm && c->norm_n < c->last_batch)
    return fail(DINO_EINVAL, "dino_resize_batch: dino_set_norm covers %s%lld images, fewer than the batch", "",
                c->norm_n);
  DecodeOnlyArgs a{c->d_desc, c->last_batch, out_w, out_h, out_dtype, c->d_plan, c->d_ws, c->d_aws, c->aws_size,
                   {mean[0], mean[1], mean[2]}, {stdv[0], stdv[1], stdv[2]}, c->d_norm, d_out};
  hipError_t e = launch_decode_only(a, (hipStream_t)stream);
  return e == hipSuccess ? DINO_OK : hip_fail(e, "dino_resize_batch");
}

int dino_batch_info(dino_ctx* c, int32_t* d_info, void* stream) {
  if (!c || !d_info) return fail(DINO_EINVAL, "dino_batch_info: null argument%s%lld");
  if (c->last_batch < 0) return fail(DINO_EINVAL, "dino_batch_info: no decoded batch%s%lld");
  hipError_t e = launch_info(c->d_desc, c->last_batch, d_info, (hipStream_t)stream);
  return e == hipSuccess ? DINO_OK : hip_fail(e, "dino_batch_info");
}

int dino_reserve(dino_ctx* c, int64_t ws_bytes, int64_t aws_bytes, void* stream) {
  if (!c || ws_bytes < 0 || aws_bytes < 0) return fail(DINO_EINVAL, "dino_reserve: bad arguments%s%lld");
  if (ws_bytes <= c->ws_size && aws_bytes <= c->aws_size) return DINO_OK;
  // Stream-ordered: the old buffers are released after the work already enqueued on
  // `stream` (the only stream this ctx's batches run on) and the new ones are usable by
  // everything enqueued after this call; no other stream of the device waits.
  hipStream_t s = (hipStream_t)stream;
  hipError_t e = hipSetDevice(c->device);
  if (e != hipSuccess) return hip_fail(e, "dino_reserve: hipSetDevice");
  if (s != c->ws_stream) {  // the previous owner stream's work on the old buffers must finish first
    if ((e = hipStreamSynchronize(c->ws_stream)) != hipSuccess) return hip_fail(e, "dino_reserve: synchronize");
    c->ws_stream = s;
  }
  if (ws_bytes > c->ws_size) {
    const int64_t n = ws_bytes + ws_bytes / 8;  // headroom: fewer regrowths
    c->last_batch = -1;  // the decoded batch (if any) lived in the old workspace
    (void)hipFreeAsync(c->d_ws, s);
    c->d_ws = nullptr;
    c->ws_size = 0;
    if ((e = hipMallocAsync((void**)&c->d_ws, n, s)) != hipSuccess)
      return hip_fail(e, "dino_reserve: hipMallocAsync(workspace)");
    c->ws_size = n;
  }
  if (aws_bytes > c->aws_size) {
    const int64_t n = aws_bytes + aws_bytes / 8;
    (void)hipFreeAsync(c->d_aws, s);
    c->d_aws = nullptr;
    c->aws_size = 0;
    if ((e = hipMallocAsync((void**)&c->d_aws, n, s)) != hipSuccess)
      return hip_fail(e, "dino_reserve: hipMallocAsync(augment workspace)");
    c->aws_size = n;
  }
  return DINO_OK;
}

int dino_augment_need(const int32_t* info, int32_t batch, const dino_aug_config* cfg, int64_t* aws_need) {
  if (!info || batch < 0 || !cfg || !aws_need) return fail(DINO_EINVAL, "dino_augment_need: bad arguments%s%lld");
  int64_t aws = 0;
  for (int32_t i = 0; i < batch; ++i) {
    if (info[4 * i] != DINO_IMG_OK) continue;
    for (int v = 0; v < cfg->n_global + cfg->n_local; ++v)
      aws += view_scratch_bound(v < cfg->n_global ? cfg->global_size : cfg->local_size, info[4 * i + 1],
                                info[4 * i + 2]);
  }
  *aws_need = aws;
  return DINO_OK;
}

int dino_workspace_sizes(dino_ctx* c, int64_t* ws_bytes, int64_t* aws_bytes) {
  if (!c || !ws_bytes || !aws_bytes) return fail(DINO_EINVAL, "dino_workspace_sizes: null argument%s%lld");
  *ws_bytes = c->ws_size;
  *aws_bytes = c->aws_size;
  return DINO_OK;
}

}  // extern "C"

namespace {
template <class Src>
int probe_impl(Src src, const uint8_t* raw_mask, int32_t batch, int32_t max_image_dim, const dino_aug_config* cfg,
               int32_t* info, int64_t* ws_need, int64_t* aws_need) {
  if (max_image_dim <= 0 || max_image_dim > kMaxImageDim) max_image_dim = kMaxImageDim;
  int64_t ws = 0, aws = 0;
  std::vector<ScanRec> scans(kMaxScans);
  for (int32_t i = 0; i < batch; ++i) {
    const uint8_t* p;
    int64_t len;
    src(i, &p, &len);
    probe_one(p, len, raw_mask != nullptr && raw_mask[i] != 0, max_image_dim, cfg, scans.data(),
              info ? info + 4 * i : nullptr, &ws, &aws);
  }
  *ws_need = ws;
  *aws_need = aws;
  return DINO_OK;
}
}  // namespace

extern "C" {

int dino_probe(const uint8_t* bytes, const int64_t* offsets, const uint8_t* raw_mask, int32_t batch,
               int32_t max_image_dim, const dino_aug_config* cfg, int32_t* info, int64_t* ws_need, int64_t* aws_need) {
  if ((!bytes && batch > 0) || !offsets || batch < 0 || !ws_need || !aws_need)
    return fail(DINO_EINVAL, "dino_probe: bad arguments%s%lld");
  return probe_impl(
      [&](int32_t i, const uint8_t** p, int64_t* len) {
        *p = bytes + offsets[i];
        *len = offsets[i + 1] - offsets[i];
      },
      raw_mask, batch, max_image_dim, cfg, info, ws_need, aws_need);
}

int dino_probe_spans(const uint64_t* ptrs, const int64_t* lens, const uint8_t* raw_mask, int32_t batch,
                     int32_t max_image_dim, const dino_aug_config* cfg, int32_t* info, int64_t* ws_need,
                     int64_t* aws_need) {
  if (((!ptrs || !lens) && batch > 0) || batch < 0 || !ws_need || !aws_need)
    return fail(DINO_EINVAL, "dino_probe_spans: bad arguments%s%lld");
  return probe_impl(
      [&](int32_t i, const uint8_t** p, int64_t* len) {
        *p = (const uint8_t*)(uintptr_t)ptrs[i];
        *len = lens[i];
      },
      raw_mask, batch, max_image_dim, cfg, info, ws_need, aws_need);
}

int dino_gather_probe(const uint64_t* src_ptrs, const int64_t* lens, int32_t n, uint8_t* dst, int64_t dst_cap,
                      int64_t* dst_offsets, int32_t nthreads, int32_t max_image_dim, const dino_aug_config* cfg,
                      int32_t* info, int64_t* ws_need, int64_t* aws_need) {
  if (n < 0 || (n > 0 && (!src_ptrs || !lens || !dst)) || !dst_offsets || !ws_need || !aws_need)
    return fail(DINO_EINVAL, "dino_gather_probe: bad arguments%s%lld");
  if (max_image_dim <= 0 || max_image_dim > kMaxImageDim) max_image_dim = kMaxImageDim;
  dst_offsets[0] = 0;
  for (int32_t i = 0; i < n; ++i) {
    if (lens[i] < 0) return fail(DINO_EINVAL, "dino_gather_probe: negative length%s%lld");
    dst_offsets[i + 1] = dst_offsets[i] + lens[i];
  }
  if (dst_offsets[n] > dst_cap) return fail(DINO_ERANGE, "dino_gather_probe: destination too small%s%lld");
  const int64_t total = dst_offsets[n];
  int nt = nthreads > 0 ? nthreads : 1;
  nt = (int)std::min<int64_t>(nt, std::max<int32_t>(n, 1));
  std::vector<int64_t> ws(nt, 0), aws(nt, 0);
  // thread k copies, then probes, images [first(k), first(k+1)): first(k) is the first image
  // starting at or after byte k*total/nt (the header is still in cache when its parse runs)
  auto first = [&](int k) -> int32_t {
    if (k <= 0) return 0;
    if (k >= nt) return n;
    return (int32_t)(std::lower_bound(dst_offsets, dst_offsets + n, total * k / nt) - dst_offsets);
  };
  auto work = [&](int k) {
    std::vector<ScanRec> scans(kMaxScans);
    for (int32_t i = first(k), e = first(k + 1); i < e; ++i) {
      const uint8_t* src = (const uint8_t*)(uintptr_t)src_ptrs[i];
      if (lens[i]) stream_copy(dst + dst_offsets[i], src, lens[i]);
      probe_one(src, lens[i], false, max_image_dim, cfg, scans.data(), info ? info + 4 * i : nullptr, &ws[k],
                &aws[k]);
    }
    stream_fence();
  };
  if (nt == 1) {
    work(0);
  } else {
    std::vector<std::thread> th;
    th.reserve(nt - 1);
    for (int k = 1; k < nt; ++k) th.emplace_back(work, k);
    work(0);
    for (auto& t : th) t.join();
  }
  int64_t w = 0, a = 0;
  for (int k = 0; k < nt; ++k) {
    w += ws[k];
    a += aws[k];
  }
  *ws_need = w;
  *aws_need = a;
  return DINO_OK;
}

int dino_stream_create(int device, int32_t cu_count, void** stream) {
  if (!stream) return fail(DINO_EINVAL, "dino_stream_create: null argument%s%lld");
  *stream = nullptr;
  hipError_t e = hipSetDevice(device);
  if (e != hipSuccess) return hip_fail(e, "hipSetDevice");
  if (cu_count < 0) {  // a non-blocking stream from the least priority's pool of hardware queues
    int least = 0, greatest = 0;
    hipStream_t s = nullptr;
    hipEvent_t ev = nullptr;
    if ((e = hipDeviceGetStreamPriorityRange(&least, &greatest)) == hipSuccess &&
        (e = hipStreamCreateWithPriority(&s, hipStreamNonBlocking, least)) == hipSuccess &&
        (e = hipEventCreateWithFlags(&ev, hipEventDisableTiming)) == hipSuccess &&
        (e = hipEventRecord(ev, s)) == hipSuccess)  // first use: HIP picks the stream's queue now
      e = hipEventSynchronize(ev);
    if (ev) (void)hipEventDestroy(ev);
    if (e != hipSuccess) {
      if (s) (void)hipStreamDestroy(s);
      return hip_fail(e, "dino_stream_create");
    }
    *stream = (void*)s;
    return DINO_OK;
  }
  int n = 0;
  if ((e = hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, device)) != hipSuccess)
    return hip_fail(e, "dino_stream_create");
  const int k = cu_count <= 0 || cu_count >= n ? n : cu_count;
  std::vector<uint32_t> mask((n + 31) / 32, 0u);
  for (int i = 0; i < k; ++i) {
    const int cu = (int)((int64_t)i * n / k);
    mask[cu >> 5] |= 1u << (cu & 31);
  }
  hipStream_t s = nullptr;
  if ((e = hipExtStreamCreateWithCUMask(&s, (uint32_t)mask.size(), mask.data())) != hipSuccess)
    return hip_fail(e, "hipExtStreamCreateWithCUMask");
  *stream = (void*)s;
  return DINO_OK;
}

int dino_stream_destroy(void* stream) {
  if (!stream) return DINO_OK;
  hipError_t e = hipStreamDestroy((hipStream_t)stream);
  return e == hipSuccess ? DINO_OK : hip_fail(e, "hipStreamDestroy");
}

int dino_host_register(void* host, int64_t nbytes) {
  if (!host || nbytes <= 0) return fail(DINO_EINVAL, "dino_host_register: bad arguments%s%lld");
  // read-only page-locking first (shard mappings are PROT_READ), then the default flags
  hipError_t e = hipHostRegister(host, (size_t)nbytes, hipHostRegisterReadOnly);
  if (e != hipSuccess) {
    (void)hipGetLastError();
    e = hipHostRegister(host, (size_t)nbytes, hipHostRegisterDefault);
  }
  return e == hipSuccess ? DINO_OK : hip_fail(e, "dino_host_register");
}

int dino_host_unregister(void* host) {
  if (!host) return fail(DINO_EINVAL, "dino_host_unregister: null pointer%s%lld");
  hipError_t e = hipHostUnregister(host);
  return e == hipSuccess ? DINO_OK : hip_fail(e, "dino_host_unregister");
}

int dino_copy_h2d(void* d_dst, const void* host_src, int64_t nbytes, void* stream) {
  if ((!d_dst || !host_src) && nbytes > 0) return fail(DINO_EINVAL, "dino_copy_h2d: null argument%s%lld");
  if (nbytes <= 0) return DINO_OK;
  hipError_t e = hipMemcpyAsync(d_dst, host_src, (size_t)nbytes, hipMemcpyHostToDevice, (hipStream_t)stream);
  return e == hipSuccess ? DINO_OK : hip_fail(e, "dino_copy_h2d");
}

int dino_masks(int32_t height, int32_t width, int32_t num_masking_patches, int32_t min_num_patches,
               int32_t max_num_patches, double log_aspect_min, double log_aspect_max, int32_t n_masks,
               uint32_t* d_py_state, uint32_t* d_np_state, uint8_t* d_out, void* stream) {
  if (height <= 0 || width <= 0 || n_masks < 0 || !d_py_state || !d_np_state || (!d_out && n_masks))
    return fail(DINO_EINVAL, "dino_masks: bad arguments%s%lld");
  if (num_masking_patches < 0 || num_masking_patches > height * width)
    return fail(DINO_EINVAL, "dino_masks: num_masking_patches %s%lld out of range", "", num_masking_patches);
  if (n_masks == 0) return DINO_OK;
  if ((int64_t)height * width > 8192)
    return fail(DINO_EINVAL, "dino_masks: grid of %s%lld patches (> 8192; use dino_masks_host)", "",
                (long long)height * width);
  hipError_t e = launch_masks(height, width, num_masking_patches, min_num_patches, max_num_patches, log_aspect_min,
                              log_aspect_max, n_masks, d_py_state, d_np_state, d_out, (hipStream_t)stream);
  return e == hipSuccess ? DINO_OK : hip_fail(e, "dino_masks");
}

int dino_masks_host(int32_t height, int32_t width, int32_t num_masking_patches, int32_t min_num_patches,
                    int32_t max_num_patches, double log_aspect_min, double log_aspect_max, int32_t n_masks,
                    uint32_t* py_state, uint32_t* np_state, uint8_t* out) {
  if (height <= 0 || width <= 0 || n_masks < 0 || !py_state || !np_state || (!out && n_masks))
    return fail(DINO_EINVAL, "dino_masks_host: bad arguments%s%lld");
  if (num_masking_patches < 0 || num_masking_patches > height * width)
    return fail(DINO_EINVAL, "dino_masks_host: num_masking_patches %s%lld out of range", "", num_masking_patches);
  MaskParams mp{height, width, num_masking_patches, min_num_patches, max_num_patches, log_aspect_min, log_aspect_max};
  MtState py, np;
  mt_load(py, py_state);
  mt_load(np, np_state);
  std::vector<int32_t> scratch((size_t)height * width);
  for (int32_t k = 0; k < n_masks; ++k) gen_mask(mp, py, np, out + (int64_t)k * height * width, scratch.data());
  mt_store(py, py_state);
  mt_store(np, np_state);
  return DINO_OK;
}

int dino_ctx_set_prog_decoder(dino_ctx* c, int32_t decoder) {
  if (!c) return fail(DINO_EINVAL, "dino_ctx_set_prog_decoder: null ctx%s%lld");
  if (decoder != DINO_PROG_WAVE && decoder != DINO_PROG_LANES)
    return fail(DINO_EINVAL, "dino_ctx_set_prog_decoder: unknown decoder%s %lld", "", (long long)decoder);
  c->geom.prog_lane = decoder == DINO_PROG_LANES;  // read at each launch (launch_decode)
  return DINO_OK;
}

int dino_set_timing(dino_ctx* c, int32_t enable) {
  if (!c) return fail(DINO_EINVAL, "dino_set_timing: null ctx%s%lld");
  if (!c->timer) c->timer = new KernelTimer();
  c->timer->enabled = enable != 0;
  if (c->timer->created) c->timer->reset();
  return DINO_OK;
}

int dino_kernel_times(dino_ctx* c, double* total_ms, int64_t* counts, int32_t n) {
  if (!c || !total_ms || !counts) return fail(DINO_EINVAL, "dino_kernel_times: null argument%s%lld");
  for (int i = 0; i < n; ++i) {
    total_ms[i] = 0.0;
    counts[i] = 0;
  }
  if (!c->timer || !c->timer->created) return DINO_OK;
  c->timer->collect();
  for (int i = 0; i < n && i < kKNumKernels; ++i) {
    total_ms[i] = c->timer->total_ms[i];
    counts[i] = c->timer->count[i];
  }
  c->timer->reset();
  return DINO_OK;
}

int dino_debug_region(dino_ctx* c, int32_t index, int32_t region, void* d_dst, int64_t max_bytes, void* stream) {
  if (!c || !d_dst || index < 0 || index >= c->last_batch) return fail(DINO_EINVAL, "dino_debug_region: bad args%s%lld");
  hipStream_t s = (hipStream_t)stream;
  ImgDesc d;
  hipError_t e = hipMemcpyAsync(&d, c->d_desc + index, sizeof(ImgDesc), hipMemcpyDeviceToHost, s);
  if (e == hipSuccess) e = hipStreamSynchronize(s);
  if (e != hipSuccess) return hip_fail(e, "dino_debug_region");
  const void* src = nullptr;
  int64_t n = 0;
  switch (region) {
    case 0: src = c->d_desc + index; n = sizeof(ImgDesc); break;
    case 1: src = c->d_ws + d.ent_off; n = d.ent_len; break;
    case 2: src = c->d_ws + d.coef_off; n = d.plane_off - d.coef_off; break;  // sparse entries + block info
    case 3: src = c->d_ws + d.plane_off; n = d.rgb_off - d.plane_off; break;
    case 4: src = c->d_ws + d.rgb_off; n = (int64_t)d.width * d.height * 3; break;
    case 5:  // speculative-decode lane records (68 bytes each, restart images: none)
      src = c->d_ws + d.hlane_off;
      n = d.restart_interval > 0 ? 0 : (int64_t)d.h_lanes * 68;
      break;
    case 6:  // kind 1: the scan list header (PHdr: levels, lane-decoder flag and slots)
      src = c->d_ws + d.htab_off;
      n = d.kind == 1 ? (int64_t)sizeof(PHdr) : 0;
      break;
    default: return fail(DINO_EINVAL, "dino_debug_region: region %s%lld", "", region);
  }
  if (d.status != 0 && region != 0) return fail(DINO_EINVAL, "dino_debug_region: image status %s%lld", "", d.status);
  if (n > max_bytes) n = max_bytes;
  e = hipMemcpyAsync(d_dst, src, n, hipMemcpyDeviceToDevice, s);
  return e == hipSuccess ? (int)0 : hip_fail(e, "dino_debug_region");
}

#ifdef DINO_HUFF_PHASES
// Instrumented builds only: copy the k_huff1 phase timestamps of the last launch.
int dino_debug_huff_phases(uint64_t* host_out, int64_t n_items) {
  hipError_t e = copy_huff_phases(host_out, n_items);
  return e == hipSuccess ? DINO_OK : hip_fail(e, "dino_debug_huff_phases");
}
#endif

#ifdef DINO_PROG_PHASES
// Instrumented builds only: per-scan timestamps of k_prog ([64 images][64 scans][3]).
int dino_debug_prog_phases(uint64_t* host_out) {
  hipError_t e = copy_prog_phases(host_out);
  return e == hipSuccess ? DINO_OK : hip_fail(e, "dino_debug_prog_phases");
}
#endif

int dino_bf16_to_fp8(const uint16_t* d_in, uint8_t* d_out, int64_t n, void* stream) {
  if ((!d_in || !d_out) && n > 0) return fail(DINO_EINVAL, "dino_bf16_to_fp8: null argument%s%lld");
  hipError_t e = launch_bf16_to_fp8(d_in, d_out, n, (hipStream_t)stream);
  return e == hipSuccess ? DINO_OK : hip_fail(e, "dino_bf16_to_fp8");
}

}  // extern "C"
