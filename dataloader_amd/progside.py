"""Progressive / multi-scan JPEGs decoded ahead of their batch, on the device.

``k_prog`` (the coefficient-buffer decoder) runs one wave per image with the scans of a
dependency level on its lanes; an AC-refinement scan is inherently serial (how many
correction bits a symbol carries depends on which coefficients of *its* block earlier
scans made non-zero), so one image takes ~15-100 ms of latency (``scripts/prog_phases.py``)
while a whole baseline batch takes ~3.4 ms.  Decoded inside its batch, a single
progressive image stalls the pipeline (the "progressive cliff").

The side path takes that latency off the batch: when a batch is prepared — many batches
before its launch (``MI355XAugPipeline(side_ahead=N)``; the reference's own prefetch
queue, pipeline.py:317) — its progressive images are decoded as a mini-batch by one of a
pool of small contexts on their own HIP streams, each image's RGB copied into a device
buffer in the raw container layout (``DINO_RAW_MAGIC`` header + HWC bytes).  At launch
the batch's input points those images at their containers (spans ABI, raw mask) and its
stream waits for the side decode's event, so the batch's own kernels treat them like any
other decoded image.  Same decoder, same bytes: the views are bit-identical to the
in-batch device route (``tests/test_gpu_round3.py``).
"""

from __future__ import annotations

import struct
from collections import deque

import numpy as np
import torch

from . import _lib, fallback
from .engine import IngestEngine, pack_jpegs


class SideJob:
    """One mini-batch on the side path: device containers by batch index, ready after ``event``."""

    __slots__ = ("containers", "event", "engine", "status", "order")

    def __init__(self, containers: dict, event: torch.cuda.Event, engine, status: torch.Tensor, order: list):
        self.containers = containers
        self.event = event
        self.engine = engine
        self.status = status      # pinned int32[n][4]: the side decode's per-image outcome
        self.order = order        # batch index of each mini-batch row

    def ready(self) -> dict:
        """The containers of images the side decode finished (waits for it; normally long done).
        An image the device decoder failed on is left out: its batch decodes it again and
        reaches the same outcome (zero-filled views where Pillow raises)."""
        self.event.synchronize()
        st = self.status.numpy()[:, 0]
        return {i: c for i, c in self.containers.items() if st[self.order.index(i)] == 0}


class _SideEngine:
    def __init__(self, device: torch.device, max_images: int, max_image_dim: int):
        self.stream = torch.cuda.Stream(device=device)
        self.eng = IngestEngine(device, max_batch=max_images, max_views=1, max_crop_size=8,
                                max_image_dim=max_image_dim, workspace_bytes=64 << 20, stream=self.stream)
        self.max_images = max_images
        self.last: torch.cuda.Event | None = None   # the engine's workspace is free once this completes
        self.keep = None                             # host / device inputs of the job in flight

    def idle(self) -> bool:
        return self.last is None or self.last.query()


class DeviceSideDecoder:
    """A pool of ``engines`` side contexts (created on demand up to the cap); ``submit``
    blocks only when every context still has a job in flight (backpressure)."""

    def __init__(self, device: torch.device, max_images: int = 64, engines: int = 48, max_image_dim: int = 0):
        self.device = device
        self.max_images = int(max_images)
        self.cap = max(1, int(engines))
        self.max_image_dim = int(max_image_dim)
        self._engines: list[_SideEngine] = []
        self._rr = 0
        self.jobs = 0
        self.images = 0

    def _engine(self) -> _SideEngine:
        for e in self._engines:
            if e.idle():
                return e
        if len(self._engines) < self.cap:
            e = _SideEngine(self.device, self.max_images, self.max_image_dim)
            self._engines.append(e)
            return e
        e = self._engines[self._rr % len(self._engines)]
        self._rr += 1
        e.last.synchronize()
        return e

    def submit(self, jpegs: dict) -> SideJob | None:
        """Decode ``{batch index: JPEG bytes}`` (at most ``max_images``) on a side context;
        images the decoder fails on are left out (their batch decodes them itself and
        reaches the same failure)."""
        idx = sorted(jpegs)[: self.max_images]
        if not idx:
            return None
        se = self._engine()
        items = [jpegs[i] for i in idx]
        hb, off = pack_jpegs(items, pin=True)
        info, ws, _ = fallback.probe(hb.data_ptr(), off.numpy(), len(items), self.max_image_dim)
        eng = se.eng
        eng.reserve(ws, 0)
        conts = {}
        heads = []
        with eng.on_stream():
            d_bytes = hb.to(self.device, non_blocking=True)
            d_off = off.to(self.device, non_blocking=True)
            d_info = eng.decode(d_bytes, d_off, len(items))
            status = torch.empty((len(items), 4), dtype=torch.int32, pin_memory=True)
            status.copy_(d_info, non_blocking=True)
            for k, i in enumerate(idx):
                st, w, h = int(info[k, 0]), int(info[k, 1]), int(info[k, 2])
                if st != 0 or int(info[k, 3]) == 2:
                    continue
                c = torch.empty(16 + w * h * 3, dtype=torch.uint8, device=self.device)
                hdr = torch.frombuffer(bytearray(struct.pack("<IIII", _lib.RAW_MAGIC, w, h, 0)),
                                       dtype=torch.uint8).pin_memory()
                heads.append(hdr)
                c[:16].copy_(hdr, non_blocking=True)
                _lib.check(eng.lib.dino_copy_rgb(eng._ctx, k, _rgb_ptr(c), eng._s()), "dino_copy_rgb")
                conts[i] = c
            ev = torch.cuda.Event()
            ev.record(se.stream)
        # decode failures found on the device (the probe passed): that image stays in its batch
        se.last = ev
        se.keep = (hb, off, d_bytes, d_off, heads)
        self.jobs += 1
        self.images += len(conts)
        return SideJob(conts, ev, se, status, idx) if conts else None

    def close(self) -> None:
        for e in self._engines:
            if e.last is not None:
                e.last.synchronize()
            e.eng.close()
        self._engines.clear()


def _rgb_ptr(c: torch.Tensor):
    import ctypes
    return ctypes.c_void_p(c.data_ptr() + 16)


def side_mask(info: np.ndarray) -> np.ndarray:
    """Images of a probed batch the side path takes: decodable coefficient-buffer images
    (``info[:, 3] == 1``: progressive, multi-scan sequential, damaged restart intervals)."""
    return (info[:, 0] == 0) & (info[:, 3] == 1)
