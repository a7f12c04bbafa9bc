"""Device-side engine: one ``dino_ctx`` per GPU plus torch-owned I/O buffers.

``IngestEngine`` is the thin Python layer over the C ABI.  torch provides the
device memory for inputs/outputs and the stream; every heavy step runs in the
HIP kernels of ``libdino_ingest.so``.
"""

from __future__ import annotations

import contextlib
import ctypes

import numpy as np
import torch

from . import _lib
from .params import OUT_BF16, OUT_FP8_E4M3, OUT_FP32, VIEW_PARAMS_DTYPE, DinoLimits

_TORCH_OUT = {OUT_BF16: torch.bfloat16, OUT_FP32: torch.float32, OUT_FP8_E4M3: torch.float8_e4m3fn}


def _ptr(t: torch.Tensor) -> ctypes.c_void_p:
    return ctypes.c_void_p(t.data_ptr())


def _optr(t: torch.Tensor | None) -> ctypes.c_void_p:
    return ctypes.c_void_p(t.data_ptr() if t is not None else 0)


def _stream_handle(device: torch.device, stream: torch.cuda.Stream | None = None) -> ctypes.c_void_p:
    s = stream if stream is not None else torch.cuda.current_stream(device)
    return ctypes.c_void_p(s.cuda_stream)


def pack_jpegs(jpegs, pin: bool = True) -> tuple[torch.Tensor, torch.Tensor]:
    """Pack a list of JPEG byte strings / uint8 arrays into one host buffer + int64 offsets[B+1]."""
    lens = np.fromiter((len(j) for j in jpegs), dtype=np.int64, count=len(jpegs))
    offsets = np.zeros(len(jpegs) + 1, dtype=np.int64)
    np.cumsum(lens, out=offsets[1:])
    total = int(offsets[-1])
    buf = torch.empty(max(total, 1) + 16, dtype=torch.uint8, pin_memory=pin)
    view = buf.numpy()
    for j, o, n in zip(jpegs, offsets[:-1], lens):
        view[o:o + n] = np.frombuffer(j, dtype=np.uint8) if isinstance(j, (bytes, bytearray, memoryview)) else j
    return buf, torch.from_numpy(offsets)


class IngestEngine:
    """Owns a ``dino_ctx`` (decode + augment workspaces sized from the limits)."""

    def __init__(self, device: int | torch.device = 0, max_batch: int = 512, max_views: int = 10,
                 max_crop_size: int = 224, max_image_dim: int = 0, workspace_bytes: int = 0,
                 stream: torch.cuda.Stream | None = None):
        self.lib = _lib.load()
        if not torch.cuda.is_available():
            raise _lib.DinoError("IngestEngine needs a ROCm GPU (torch.cuda.is_available() is False); "
                                 "there is no CPU fallback")
        self.device = torch.device("cuda", device) if isinstance(device, int) else torch.device(device)
        self.limits = DinoLimits(max_batch, max_views, max_crop_size, max_image_dim, workspace_bytes)
        self._ctx = ctypes.c_void_p()
        with torch.cuda.device(self.device):
            _lib.check(self.lib.dino_ctx_create(self.device.index or 0, ctypes.byref(self.limits),
                                                ctypes.byref(self._ctx)), "dino_ctx_create")
        self.last_batch = 0
        self.stream = stream  # None: launch on torch's current stream
        self.prog_lanes: bool | None = None  # set_prog_decoder's choice (None: the library default)

    def _s(self) -> ctypes.c_void_p:
        return _stream_handle(self.device, self.stream)

    def on_stream(self):
        """Context in which torch allocations/ops are ordered with this engine's launches."""
        return torch.cuda.stream(self.stream) if self.stream is not None else contextlib.nullcontext()

    # ------------------------------------------------------------------ decode
    def decode(self, d_bytes: torch.Tensor, d_offsets: torch.Tensor, batch: int,
               info: torch.Tensor | None = None, raw_mask: torch.Tensor | None = None,
               lengths: torch.Tensor | None = None) -> torch.Tensor:
        """``raw_mask``: device uint8[batch], 1 where the image is a raw RGB container (hand-over);
        ``lengths``: device int64[batch], the spans form (``dino_decode_spans``)."""
        if info is None:
            with self.on_stream():
                info = torch.empty(batch, 4, dtype=torch.int32, device=self.device)
        _lib.check(self.lib.dino_decode_spans(self._ctx, _ptr(d_bytes), _ptr(d_offsets), _optr(lengths),
                                              _optr(raw_mask), batch, _ptr(info), self._s()), "dino_decode")
        self.last_batch = batch
        return info

    def copy_from_host(self, d_dst: torch.Tensor, dst_off: int, host_addr: int, nbytes: int,
                       stream: torch.cuda.Stream | None = None) -> None:
        """Asynchronous DMA of ``nbytes`` at host address ``host_addr`` (page-locked) into
        ``d_dst[dst_off:]`` on ``stream`` (default: this engine's stream; ``dino_copy_h2d``)."""
        assert 0 <= dst_off and dst_off + nbytes <= d_dst.numel() * d_dst.element_size()
        s = ctypes.c_void_p(stream.cuda_stream) if stream is not None else self._s()
        _lib.check(self.lib.dino_copy_h2d(ctypes.c_void_p(d_dst.data_ptr() + dst_off), ctypes.c_void_p(host_addr),
                                          int(nbytes), s), "dino_copy_h2d")

    def _to_current(self) -> None:
        """Order torch's current stream after this engine's launches, so that a tensor the
        engine just filled on its own stream can be used (``.cpu()``, ops) on the current one."""
        if self.stream is not None:
            torch.cuda.current_stream(self.device).wait_stream(self.stream)

    def copy_rgb(self, index: int, width: int, height: int) -> torch.Tensor:
        with self.on_stream():
            out = torch.zeros(height, width, 3, dtype=torch.uint8, device=self.device)
        _lib.check(self.lib.dino_copy_rgb(self._ctx, index, _ptr(out), self._s()),
                   "dino_copy_rgb")
        self._to_current()
        return out

    def debug_region(self, index: int, region: int, nbytes: int) -> torch.Tensor:
        with self.on_stream():
            out = torch.zeros(nbytes, dtype=torch.uint8, device=self.device)
        _lib.check(self.lib.dino_debug_region(self._ctx, index, region, _ptr(out), nbytes,
                                              self._s()), "dino_debug_region")
        self._to_current()
        return out

    KERNEL_NAMES = ["k_parse", "k_plan", "k_destuff", "k_huff1", "k_idct", "k_color", "k_params", "k_vplan",
                    "k_rcoeffs", "k_hresize", "k_final_global", "k_final_local", "k_vert_global", "k_vert_local",
                    "k_dcscan", "k_htab", "k_hseg", "k_huff2", "k_huff3", "k_prog", "k_pwalk", "k_plscan",
                    "k_papply"]

    def set_prog_decoder(self, lanes: bool) -> None:
        """Decode this context's coefficient-buffer images with the lane decoder (``True``:
        64 images per wave, for large pools decoded well ahead) or the wave decoder."""
        _lib.check(self.lib.dino_ctx_set_prog_decoder(self._ctx, int(bool(lanes))), "dino_ctx_set_prog_decoder")
        self.prog_lanes = bool(lanes)

    def set_timing(self, enable: bool) -> None:
        _lib.check(self.lib.dino_set_timing(self._ctx, int(enable)), "dino_set_timing")

    def kernel_times(self) -> dict[str, tuple[float, int]]:
        """{kernel: (total ms, launches)} since the last call (HIP events on the launch stream)."""
        n = len(self.KERNEL_NAMES)
        ms = (ctypes.c_double * n)()
        cnt = (ctypes.c_int64 * n)()
        _lib.check(self.lib.dino_kernel_times(self._ctx, ms, cnt, n), "dino_kernel_times")
        return {k: (ms[i], cnt[i]) for i, k in enumerate(self.KERNEL_NAMES)}

    # ----------------------------------------------------------------- augment
    def sample_params(self, cfg, seed: int, batch_index: int, out: torch.Tensor | None = None) -> torch.Tensor:
        n = self.last_batch * (cfg.n_global + cfg.n_local)
        if out is None:
            with self.on_stream():
                out = torch.empty(n * VIEW_PARAMS_DTYPE.itemsize, dtype=torch.uint8, device=self.device)
        _lib.check(self.lib.dino_sample_params(self._ctx, ctypes.byref(cfg), seed & (2**64 - 1), batch_index,
                                               _ptr(out), self._s()), "dino_sample_params")
        return out

    def alloc_views(self, cfg, batch: int) -> list[torch.Tensor]:
        dt = _TORCH_OUT[cfg.out_dtype]
        sizes = [cfg.global_size] * cfg.n_global + [cfg.local_size] * cfg.n_local
        with self.on_stream():
            return [torch.empty(batch, 3, s, s, dtype=dt, device=self.device) for s in sizes]

    def augment(self, cfg, params: torch.Tensor, views: list[torch.Tensor] | None = None) -> list[torch.Tensor]:
        if views is None:
            views = self.alloc_views(cfg, self.last_batch)
        ptrs = (ctypes.c_void_p * len(views))(*[v.data_ptr() for v in views])
        _lib.check(self.lib.dino_augment(self._ctx, ctypes.byref(cfg), _ptr(params), ptrs,
                                         self._s()), "dino_augment")
        return views

    def run_batch(self, d_bytes, d_offsets, batch: int, cfg, seed: int, batch_index: int,
                  views: list[torch.Tensor] | None = None, params_out: torch.Tensor | None = None,
                  info: torch.Tensor | None = None, raw_mask: torch.Tensor | None = None,
                  lengths: torch.Tensor | None = None):
        """``lengths`` (device int64[batch], optional): the spans form (``dino_run_batch_spans``):
        image i is d_bytes[d_offsets[i] : d_offsets[i] + lengths[i]]."""
        if views is None:
            views = self.alloc_views(cfg, batch)
        if info is None:
            with self.on_stream():
                info = torch.empty(batch, 4, dtype=torch.int32, device=self.device)
        ptrs = (ctypes.c_void_p * len(views))(*[v.data_ptr() for v in views])
        pp = _ptr(params_out) if params_out is not None else ctypes.c_void_p(0)
        _lib.check(self.lib.dino_run_batch_spans(self._ctx, _ptr(d_bytes), _ptr(d_offsets), _optr(lengths),
                                                 _optr(raw_mask), batch, ctypes.byref(cfg),
                                                 seed & (2**64 - 1), batch_index, pp, ptrs, _ptr(info),
                                                 self._s()), "dino_run_batch")
        self.last_batch = batch
        return views, info

    def resize_batch(self, out_w: int, out_h: int, mean, std, out_dtype: int, batch: int | None = None,
                     out: torch.Tensor | None = None) -> torch.Tensor:
        """Decode-only recipe on the last decoded batch (``dino_resize_batch``): [B, 3, out_h, out_w]."""
        batch = self.last_batch if batch is None else batch
        if out is None:
            with self.on_stream():
                out = torch.empty(batch, 3, out_h, out_w, dtype=_TORCH_OUT[out_dtype], device=self.device)
        m = (ctypes.c_float * 3)(*[float(x) for x in mean])
        sd = (ctypes.c_float * 3)(*[float(x) for x in std])
        _lib.check(self.lib.dino_resize_batch(self._ctx, out_w, out_h, m, sd, out_dtype, _ptr(out), self._s()),
                   "dino_resize_batch")
        return out

    def batch_info(self, info: torch.Tensor) -> torch.Tensor:
        """Per-image status after augmentation (``dino_batch_info``) into ``info`` [B, 4] int32."""
        _lib.check(self.lib.dino_batch_info(self._ctx, _ptr(info), self._s()), "dino_batch_info")
        return info

    def workspace_sizes(self) -> tuple[int, int]:
        ws, aws = ctypes.c_int64(0), ctypes.c_int64(0)
        _lib.check(self.lib.dino_workspace_sizes(self._ctx, ctypes.byref(ws), ctypes.byref(aws)),
                   "dino_workspace_sizes")
        return int(ws.value), int(aws.value)

    def reserve(self, ws_bytes: int, aws_bytes: int) -> bool:
        """Grow the decode / augment workspaces to at least these sizes (``dino_reserve``),
        stream-ordered on this engine's stream (no other stream of the device waits).
        Returns True when it had to reallocate."""
        cur_ws, cur_aws = self.workspace_sizes()
        if ws_bytes <= cur_ws and aws_bytes <= cur_aws:
            return False
        with torch.cuda.device(self.device):
            _lib.check(self.lib.dino_reserve(self._ctx, int(ws_bytes), int(aws_bytes), self._s()), "dino_reserve")
        return True

    def set_norm(self, d_norm: torch.Tensor | None) -> None:
        """Per-image {mean[3], std[3]} ([0, 1] scale) for the next batches (``dino_set_norm``);
        None restores the global statistics.  The tensor must outlive the batches using it."""
        if d_norm is None:
            _lib.check(self.lib.dino_set_norm(self._ctx, ctypes.c_void_p(0), 0), "dino_set_norm")
            return
        assert d_norm.dtype == torch.float32 and d_norm.is_contiguous() and d_norm.shape[-1] == 6
        _lib.check(self.lib.dino_set_norm(self._ctx, _ptr(d_norm), int(d_norm.shape[0])), "dino_set_norm")

    def close(self) -> None:
        if self._ctx:
            torch.cuda.synchronize(self.device)
            self.lib.dino_ctx_destroy(self._ctx)
            self._ctx = ctypes.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:  # noqa: BLE001
            pass


def params_from_device(t: torch.Tensor) -> np.ndarray:
    """Device param buffer -> numpy structured array of dino_view_params."""
    return t.cpu().numpy().view(VIEW_PARAMS_DTYPE)


def params_to_device(arr: np.ndarray, device) -> torch.Tensor:
    raw = np.ascontiguousarray(arr, dtype=VIEW_PARAMS_DTYPE).view(np.uint8)
    return torch.from_numpy(raw.copy()).to(device)
