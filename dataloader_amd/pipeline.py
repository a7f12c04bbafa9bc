"""MI355X multi-crop pipeline — the device counterpart of ``CPUAugPipeline``.

Mirrors reference ``src/dino_loader/backends/cpu.py``:

* ``MI355XAugPipeline.run_one_batch``  <- ``CPUAugPipeline.run_one_batch`` :309-367
  (reads (G, L) from the resolution source, pulls exactly ``batch_size`` JPEGs
  from the source, returns ``{"view_i": Tensor[B,3,S,S]}``), but the JPEG
  bytes are packed once, copied to HBM in one transfer and decoded ONCE per
  image (the reference decodes per view, cpu.py:251) by the HIP kernels.
* ``close()`` semantics :369-377 (idempotent; run after close -> RuntimeError).
* ``MI355XPipelineIterator`` <- ``CPUPipelineIterator`` :506-527.

Randomness: every (sample, view) record comes from a counter-based Philox
stream keyed by (seed, batch index, sample, view) on the device, so the
output does not depend on thread scheduling; ``last_params()`` exports the
records so the CPU oracle can replay a batch exactly.

Failures are never silent: every host batch is pre-screened (``fallback.py``:
``dino_probe``, Pillow hand-over of the JPEG flavours the GPU decoder does not
implement, ``dino_reserve``), and every batch's per-image status is read back
asynchronously and accounted in ``stats``; an image that the reference would
have decoded but that came back zero-filled raises a ``RuntimeWarning``.
"""

from __future__ import annotations

import atexit
import ctypes
import itertools
import os
import queue
import sys
import threading
import time
import warnings
import weakref
from collections import Counter, deque
from typing import Any

import numpy as np
import torch

from . import fallback
from .engine import IngestEngine, pack_jpegs, params_from_device
from .params import OUT_BF16, OUT_FP8_E4M3, OUT_FP32, RECORD_BYTES, make_aug_config

_DTYPES = {"bf16": OUT_BF16, "fp32": OUT_FP32, "fp8": OUT_FP8_E4M3}


def _out_code(out_dtype) -> int:
    if isinstance(out_dtype, int):
        return out_dtype
    if isinstance(out_dtype, torch.dtype):
        return {torch.bfloat16: OUT_BF16, torch.float32: OUT_FP32, torch.float8_e4m3fn: OUT_FP8_E4M3}[out_dtype]
    return _DTYPES.get(out_dtype, OUT_BF16)


def _refcounts(views) -> list[int]:
    """``sys.getrefcount`` of each tensor of ``views``, every one taken through this same
    code path (the loop variable and getrefcount's argument included), so that the counts
    compare with ``_REFS_PIPELINE_ONLY``, measured through it at import: how many references
    an interpreter version adds on this path is then never assumed (CPython 3.11
    moved a call's argument reference into the callee's frame)."""
    out = []
    for t in views:
        out.append(sys.getrefcount(t))
    return out


def _calibrate_refs() -> int:
    """The count ``_refcounts`` reports for a tensor that only a slot holds: its view-cache
    list and its outputs dict (the probe holds one more reference, its local ``t``)."""
    t = torch.empty(0)
    cache, outputs = [t], {"view_0": t}
    n = _refcounts(cache)[0] - 1
    del outputs
    return n


_REFS_PIPELINE_ONLY = _calibrate_refs()


def _all_unshared(views, in_dicts: list[int]) -> bool:
    """Nothing outside the pipeline holds any tensor of ``views`` or its memory: each tensor
    object is referenced only by the output ring's list and the ``in_dicts[i]`` slot outputs
    dicts that hold it (one reference each), and its storage only by the tensor (a view,
    slice or chunk the caller kept shares the storage and raises its use count)."""
    if any(n > _REFS_PIPELINE_ONLY - 1 + k for n, k in zip(_refcounts(views), in_dicts)):
        return False
    use_count = getattr(torch._C, "_storage_Use_Count", None)
    if use_count is None:  # no way to see views: never reuse
        return False
    return all(use_count(t.untyped_storage()._cdata) <= 2 for t in views)  # t + the temporary storage object


class _Slot:
    """One in-flight batch: an engine (ctx + stream) and the batch's small buffers."""

    def __init__(self, engine: IngestEngine):
        self.engine = engine
        self.params: torch.Tensor | None = None
        self.info: torch.Tensor | None = None
        self.event: torch.cuda.Event | None = None
        self.inflight = None
        self.outputs: dict[str, torch.Tensor] | None = None
        self.norm: torch.Tensor | None = None         # per-image normalisation records of the batch
        self.batch_id = -1
        self.batch_index = -1                          # the batch's RNG key (seed, batch_index)
        self.sizes: tuple[int, int] | None = None     # (G, L) the views were made at
        self.probe: np.ndarray | None = None          # dino_probe info of the batch (host batches)
        self.d_in: torch.Tensor | None = None         # HBM copy of the batch's bytes (spans feed)
        # native feed: two HBM input buffers (bytes, offsets) used alternately, so the copy of a
        # batch runs on the copy stream while the slot's previous batch still decodes
        self.d_ins: list = [None, None]
        self.d_offs: list = [None, None]
        self.buf_done: list = [None, None]            # event after the last batch that read each buffer
        self.buf_next = 0
        self.view_set = -1                            # the output set (pipeline ring) of the slot's batch


class _Staging:
    """A pinned host buffer the batch's JPEG bytes (+ int64 offsets + raw mask) are packed
    into before the H2D copy.  Owned by the host half while it is being filled and until the
    launch that copies it out has retired (``released`` event)."""

    def __init__(self):
        self.buf: torch.Tensor | None = None
        self.off: torch.Tensor | None = None
        self.lens: torch.Tensor | None = None
        self.mask: torch.Tensor | None = None
        self.released: torch.cuda.Event | None = None
        self.busy = False

    def fit(self, nbytes: int, n: int) -> None:
        if nbytes > 0 and (self.buf is None or self.buf.numel() < nbytes):
            self.buf = torch.empty(max(nbytes, 1) * 5 // 4 + 64, dtype=torch.uint8, pin_memory=True)
        if self.off is None or self.off.numel() < n + 1:
            self.off = torch.empty(n + 1, dtype=torch.int64, pin_memory=True)
            self.lens = torch.empty(n, dtype=torch.int64, pin_memory=True)
            self.mask = torch.empty(n, dtype=torch.uint8, pin_memory=True)


class _StagingRing:
    """Round-robin staging buffers shared by the host half (fills) and the launch (frees)."""

    def __init__(self, n: int):
        self._bufs = [_Staging() for _ in range(max(2, n))]
        self._next = 0
        self._cv = threading.Condition()
        self._closed = False

    def close(self) -> None:
        with self._cv:
            self._closed = True
            self._cv.notify_all()

    def acquire(self) -> _Staging:
        with self._cv:
            st = self._bufs[self._next]
            self._next = (self._next + 1) % len(self._bufs)
            while st.busy and not self._closed:  # still waiting to be launched (rare: the ring is sized for it)
                self._cv.wait()
            if self._closed:
                raise RuntimeError("MI355XAugPipeline closed")
            st.busy = True
        if st.released is not None:
            st.released.synchronize()  # the H2D copy of its previous batch retired
            st.released = None
        return st

    def release(self, st: _Staging, event: torch.cuda.Event | None) -> None:
        with self._cv:
            st.released = event
            st.busy = False
            self._cv.notify_all()


class _Prepared:
    """A pulled, packed and probed host batch whose host-routed images are decoding in the pool."""

    def __init__(self, staging: _Staging, jpegs, offsets: np.ndarray, info: np.ndarray, ws: int, aws: int,
                 sizes: tuple[int, int], futures: dict, spans=None, feed=None):
        self.staging = staging        # None: no Python staging (native feed slot, or not yet needed)
        self.spans = spans            # tario.BatchSpans: the batch stays in its page-locked shard ranges
        self.feed = feed              # tario.FeedBatch: the batch is packed in a native feed slot
        self.side = None              # progside.SideJob: its coefficient-buffer images, decoded ahead
        self.room: dict = {}          # batch index -> offset of room for its container in the HBM copy
        self.side_submitted = False   # _side_submit ran (on the prefetch thread, or at the pull)
        self.jpegs = jpegs            # the source's list (None for the native feed)
        self.offsets = offsets
        self.info = info
        self.ws, self.aws = ws, aws
        self.sizes = sizes            # (G, L) the augment-workspace bound was computed for
        self.futures = futures
        # side look-ahead: the batch's input copied to HBM when it entered the look-ahead (its
        # pinned staging / feed slot / shard ranges are free again); ready after `copied`
        self.dev = None               # (d_bytes, d_offsets, d_lens or None)
        self.lens = None              # host image lengths of a spans batch staged on the device
        self.copied: torch.cuda.Event | None = None


_END = object()
# open pipelines, closed at interpreter exit before torch tears down: a prefetch thread must
# not hold pinned tensors while the interpreter finalises them
_LIVE: "weakref.WeakSet[MI355XAugPipeline]" = weakref.WeakSet()

# One torch stream per (device, role, index) for the life of the process: every pipeline
# reuses the streams of the first one.  HIP multiplexes streams onto a few hardware queues
# (GPU_MAX_HW_QUEUES, 4 by default) in creation order, so fresh streams for each pipeline
# land on other queues than the first pipeline's did, and a second side-route pipeline in
# a process ran at 68-70k img/s against 101k for the first (profiles/r04_side_repeat_*).
# The first request on a device takes the usual roles' streams in one fixed order (the
# order a feed-driven side-route pipeline asks for them), so the mapping does not depend
# on which kind of pipeline a process builds first.
#
# A set of role streams belongs to one live pipeline at a time: pipelines alive
# together (train + val loaders) take different sets, so one's kernels never queue behind the
# other's on a shared stream; a set is handed to the next pipeline once its owner closes.
_ROLE_STREAMS: dict = {}
_ROLE_LOCK = threading.Lock()
_ROLE_ORDER = (("copy", 0), ("slot", 0), ("slot", 1), ("slot", 2), ("side_copy", 0), ("side_copy", 1))
_SETS_BUSY: dict = {}   # device index -> stream-set ids held by live pipelines


def _dev_index(device) -> int:
    dev = torch.device("cuda", device) if isinstance(device, int) else torch.device(device)
    return dev.index if dev.index is not None else torch.cuda.current_device()


def acquire_stream_set(device) -> int:
    """The lowest stream-set id no live pipeline on ``device`` holds (released by ``close``)."""
    idx = _dev_index(device)
    with _ROLE_LOCK:
        busy = _SETS_BUSY.setdefault(idx, set())
        s = 0
        while s in busy:
            s += 1
        busy.add(s)
        return s


def release_stream_set(device, s: int) -> None:
    with _ROLE_LOCK:
        _SETS_BUSY.get(_dev_index(device), set()).discard(s)


_RAW_ROLE_STREAMS: list = []  # (device, handle) of the role streams dino_stream_create made


def _new_role_stream(idx: int, role: str) -> torch.cuda.Stream:
    """A role's stream.  The batch slots and the copy stream come from the least priority's
    pool of hardware queues (``dino_stream_create(-1)``), the other roles from torch's pool
    (DINO_ROLE_STREAMS=torch: all of them).  HIP multiplexes streams onto GPU_MAX_HW_QUEUES
    = 4 queues per priority; from torch's pool two of the three slots shared one and ran one
    after the other (their batches queue in one FIFO: 128 of 198 e2e batches started on the
    other slot's end), e2e 156.3k img/s; on queues of their own 172.9k (C2 177.2k,
    ``scripts/rolestream_study.sh``).  The streams live as long as the process, as torch's
    pool streams do."""
    if role in ("slot", "copy") and os.environ.get("DINO_ROLE_STREAMS", "low") == "low":
        from . import _lib
        h = ctypes.c_void_p()
        _lib.check(_lib.load().dino_stream_create(idx, -1, ctypes.byref(h)), "dino_stream_create")
        _RAW_ROLE_STREAMS.append((idx, h.value))
        return torch.cuda.ExternalStream(h.value, device=torch.device("cuda", idx))
    return torch.cuda.Stream(device=idx)


def role_stream(device, role: str, k: int = 0, stream_set: int = 0) -> torch.cuda.Stream:
    idx = _dev_index(device)
    with _ROLE_LOCK:
        if not any(key[:2] == (idx, stream_set) for key in _ROLE_STREAMS):
            for r, j in _ROLE_ORDER:
                _ROLE_STREAMS[(idx, stream_set, r, j)] = _new_role_stream(idx, r)
        st = _ROLE_STREAMS.get((idx, stream_set, role, k))
        if st is None:
            st = _ROLE_STREAMS[(idx, stream_set, role, k)] = _new_role_stream(idx, role)
        return st


@atexit.register
def _close_live() -> None:
    """At interpreter exit, before any library is finalized: close the open pipelines, then
    destroy the role streams this module created with dino_stream_create (after the device is
    idle and torch's allocator has retired its blocks' stream events), so that no stream of
    ours is still alive when the HIP runtime and a profiler's tool library tear down (VERDICT r5
    weak #6: an intermittent SIGSEGV in __cxa_finalize after a rocprofv3 run printed its line)."""
    for p in list(_LIVE):
        try:
            p.close()
        except Exception:  # noqa: BLE001
            pass
    release_role_streams()


def release_role_streams() -> None:
    """Destroy every role stream made by dino_stream_create (process exit; no pipeline may be
    open).  Later role_stream() calls make new ones."""
    if not _RAW_ROLE_STREAMS or _LIVE:
        return
    try:
        from . import _lib
        lib = _lib.load()
        for dev in {d for d, _ in _RAW_ROLE_STREAMS}:
            torch.cuda.synchronize(dev)
        torch.cuda.empty_cache()
        with _ROLE_LOCK:
            for key in [k for k, st in _ROLE_STREAMS.items() if isinstance(st, torch.cuda.ExternalStream)]:
                del _ROLE_STREAMS[key]
            while _RAW_ROLE_STREAMS:
                _, h = _RAW_ROLE_STREAMS.pop()
                lib.dino_stream_destroy(ctypes.c_void_p(h))
    except Exception:  # noqa: BLE001 - exit path: never raise
        pass


RAW_AHEAD = 2  # pulled, not yet packed batches the prefetcher's puller thread holds (list sources)
# pack threads of a list source's prefetcher (DINO_PACK_THREADS): two measured no faster than
# one on c2_prog (the packs then contend for the job's CPU share, profiles/r06_side_plan/r6x)
PACK_THREADS = 1


class _Prefetcher:
    """The host half of the pipeline on worker threads (DALI's prefetch queue, reference
    pipeline.py:317 ``prefetch_queue_depth``): pull the next batch from the source, pack it
    into pinned staging (``dino_gather``), ``dino_probe`` it and submit its Pillow
    hand-overs, up to ``ahead`` batches ahead of the launches.  The GIL is released inside
    the native calls, so this overlaps the launch thread and the GPU.

    For a source that hands over JPEG lists (the reference's ``_ReaderAdapter``) the pull
    runs on a thread of its own, up to ``RAW_AHEAD`` batches ahead, and ``PACK_THREADS``
    threads pack the pulled batches: the source's Python call and the native pack overlap
    instead of adding up (c2_prog: ~0.8 ms pull + 1.2-3 ms pack per batch).
    Batches are handed out in the source's order (sequence numbers, a reorder buffer of at
    most ``ahead`` batches); the source's end and its errors arrive in place."""

    def __init__(self, pipe: "MI355XAugPipeline", ahead: int):
        self._pipe = pipe
        self._ahead = max(1, ahead)
        self._stop = threading.Event()
        self.finished = False       # the source raised StopIteration (the END marker is queued)
        self._cv = threading.Condition()
        self._out: dict = {}        # sequence number -> _Prepared, _END or an exception
        self._next = 0              # sequence number get() hands out next
        self._raw: queue.Queue | None = None
        self._threads: list[threading.Thread] = []
        if not pipe._spans_feed and not pipe._native:
            self._raw = queue.Queue(maxsize=RAW_AHEAD)
            n = max(1, int(os.environ.get("DINO_PACK_THREADS", PACK_THREADS)))
            self._threads.append(threading.Thread(target=self._pull_loop, name="dino-pull", daemon=True))
            self._threads += [threading.Thread(target=self._pack_loop, name=f"dino-prefetch-{k}", daemon=True)
                              for k in range(n)]
        else:
            self._threads.append(threading.Thread(target=self._run, name="dino-prefetch", daemon=True))
        for t in self._threads:
            t.start()

    # ---- producers
    def _emit(self, seq: int, item) -> bool:
        """Place item `seq` in the reorder buffer once it is within `ahead` of the next hand-out."""
        with self._cv:
            while seq - self._next >= self._ahead and not self._stop.is_set():
                self._cv.wait(0.1)
            if self._stop.is_set():
                return False
            self._out[seq] = item
            self._cv.notify_all()
            return True

    def _settle(self, seq: int, item) -> bool:
        """Emit a prepared batch, or drop it if the prefetcher is closing."""
        if isinstance(item, _Prepared) and not self._emit(seq, item):
            self._pipe._drop(item)
            return False
        return isinstance(item, _Prepared) or self._emit(seq, item)

    def _run(self) -> None:  # one thread pulls and packs (spans / native sources)
        seq = 0
        try:
            while not self._stop.is_set():
                pb = self._pipe._prepare_next()
                self._pipe._stage_early(pb)
                if not self._settle(seq, pb):
                    return
                seq += 1
        except StopIteration:
            self.finished = True
            self._emit(seq, _END)
        except BaseException as e:  # noqa: BLE001 - handed to the launch thread
            self._emit(seq, e)

    def _put_raw(self, item) -> bool:
        while not self._stop.is_set():
            try:
                self._raw.put(item, timeout=0.1)
                return True
            except queue.Full:
                continue
        return False

    def _pull_loop(self) -> None:
        seq = 0
        try:
            while not self._stop.is_set():
                if not self._put_raw((seq, self._pipe._pull_raw())):
                    return
                seq += 1
        except StopIteration:
            self._put_raw((seq, _END))
        except BaseException as e:  # noqa: BLE001 - handed to a pack thread, then the launch thread
            self._put_raw((seq, e))

    def _pack_loop(self) -> None:
        while not self._stop.is_set():
            try:
                seq, raw = self._raw.get(timeout=0.1)
            except queue.Empty:
                continue
            if raw is _END or isinstance(raw, BaseException):
                if raw is _END:
                    self.finished = True
                self._put_raw((seq, raw))  # the other pack threads see the end too
                self._emit(seq, raw)
                return
            try:
                pb = self._pipe._pack_raw(raw)
                self._pipe._stage_early(pb)
            except BaseException as e:  # noqa: BLE001 - handed to the launch thread in place
                self._emit(seq, e)
                continue
            if not self._settle(seq, pb):
                return

    # ---- consumer
    def get(self, block: bool = True) -> _Prepared | None:
        with self._cv:
            while self._next not in self._out:
                if not block or self._stop.is_set():
                    return None
                self._cv.wait(0.1)
            item = self._out[self._next]
            if item is not _END and not isinstance(item, BaseException):
                del self._out[self._next]
                self._next += 1
                self._cv.notify_all()
        if item is _END:
            raise StopIteration
        if isinstance(item, BaseException):
            raise item
        return item

    def close(self) -> None:
        self._stop.set()
        with self._cv:
            self._cv.notify_all()
        for t in self._threads:
            t.join(timeout=5.0)
        with self._cv:  # free staging of batches never launched
            items, self._out = list(self._out.values()), {}
        for item in items:
            if isinstance(item, _Prepared):
                self._pipe._drop(item)
        while self._raw is not None:
            try:
                self._raw.get_nowait()
            except queue.Empty:
                break


SIDE_URGENT_SHORT = 8  # side look-ahead batches flushed at once while the look-ahead is short (_pull_side)


class MI355XAugPipeline:
    """``depth`` > 1 keeps that many batches in flight: each slot owns a ctx and a
    HIP stream, consecutive batches alternate slots, so one batch's entropy
    decode (latency bound) overlaps another's resize/jitter kernels.

    ``prefetch`` (default: 1 when depth > 1) runs the host half — pull, pack into pinned
    staging, probe, Pillow hand-overs — that many batches ahead on a worker thread, so the
    calling thread only launches (H2D copy + kernels) and hands over."""

    def __init__(self, source: Any, aug_cfg, batch_size: int, resolution_src=None, seed: int = 0,
                 out_dtype="bf16", device: int = 0, max_image_dim: int = 0, workspace_bytes: int = 0,
                 engine: IngestEngine | None = None, depth: int = 1, norm=None,
                 view_names: list[str] | None = None, host_fallback: bool = True,
                 multiscan_route: str = "auto", host_workers: int | None = None,
                 multiscan_host_max: int | None = None, prefetch: int | None = None,
                 start_host_pool: bool = False, side_ahead: int = 64):
        self._source = source
        self._aug_cfg = aug_cfg
        self._batch_size = int(batch_size)
        self._resolution_src = resolution_src
        self._out = _out_code(out_dtype)
        self._seed = int(seed)
        self._norm = norm  # NormTable (per-dataset statistics) or None: global mean/std
        self._names = list(view_names) if view_names else [f"view_{i}" for i in range(aug_cfg.n_views)]
        self._batch_index = 0
        self._max_image_dim = int(max_image_dim)
        self._host_fallback = bool(host_fallback)
        if multiscan_route not in ("auto", "device", "host", "side"):
            raise ValueError(f"multiscan_route must be 'auto', 'device', 'host' or 'side', not {multiscan_route!r}")
        self._multiscan_route = multiscan_route
        # "side": coefficient-buffer images decoded on the device ahead of their batch (progside.py),
        # side_ahead batches before it is launched
        self._side_ahead = max(1, int(side_ahead)) if multiscan_route == "side" else 0
        self._route = "device" if multiscan_route == "side" else multiscan_route  # what route_mask sees
        self._side = None
        self._ahead: deque = deque()   # prepared batches waiting for launch (side path)
        self._side_hot = 0             # batches the look-ahead stays engaged for (see _pull_side)
        self._source_end = False
        workers = int(host_workers) if host_workers else min(8, os.cpu_count() or 1)
        self._host = fallback.HostDecoder(workers)
        if start_host_pool:
            self._host.start()
        # "auto": the host takes a batch's coefficient-buffer images while its workers finish
        # them in about the time k_prog needs for any number of them (~100 ms vs ~6 ms/image)
        self._host_max = int(multiscan_host_max) if multiscan_host_max is not None else 8 * workers
        # per-image outcome of every batch handed over (status code -> images), images the
        # GPU decoder left to Pillow, and workspace regrowths
        self.stats = {"batches": 0, "images": 0, "status": Counter(), "host_decoded": 0, "reserves": 0,
                      "side_decoded": 0}
        # host-side seconds per phase: pull / pack / probe (host half), wait (launch thread
        # waiting for the host half), launch (H2D copies + kernel enqueue)
        self.host_seconds = {"pull": 0.0, "pack": 0.0, "probe": 0.0, "wait": 0.0, "launch": 0.0}
        self._pending: deque = deque()   # (pinned status copy, its event, batch id, images) per launched batch
        self._info_pool: list = []       # pinned status buffers of accounted batches
        self.depth = max(1, int(depth))
        self.prefetch_ahead = (1 if self.depth > 1 else 0) if prefetch is None else max(0, int(prefetch))
        if self._side_ahead:
            self.prefetch_ahead = max(1, self.prefetch_ahead)
        self._prefetcher: _Prefetcher | None = None
        # the side look-ahead holds its batches in HBM (``_stage_on_device``), not in staging
        # (+ PACK_THREADS: a pack thread holds a buffer while the batch the launch waits for is
        # still being packed by another)
        self._ring = _StagingRing(self.depth + self.prefetch_ahead + (4 if self._side_ahead else 0) + 2 + PACK_THREADS)
        # copier threads of the host half's pack (dino_gather_probe): the source's own count
        # (the native feeds) or DINO_GATHER_THREADS (default 8)
        self._gather_threads = int(getattr(source, "nthreads", 0) or os.environ.get("DINO_GATHER_THREADS", 8))
        self._native = hasattr(source, "next_spans")
        # the feed can hand batches over where they lie (page-locked shard ranges, DMA'd as they are)
        self._spans_feed = hasattr(source, "next_batch_spans")
        # the native feed (tario.NativeShardFeed): batches arrive packed + probed by C++ threads
        self._feed = hasattr(source, "next_prepared")
        self._held: deque = deque()   # the feed's next batch, prepared one ahead (Pillow hand-overs start early)
        # H2D copies of the native feed's batches, off the slots' streams (DINO_COPY_STREAM=0: on them)
        self._copy_stream = None
        self._device_arg = device
        self._closed = True  # until the end of __init__: close() must not run on a half-built pipeline
        self._slots: list[_Slot] = []
        self._stream_set = acquire_stream_set(device)
        try:
            self._init_device(aug_cfg, device, depth, engine, max_image_dim, workspace_bytes)
        except BaseException:  # a failed construction hands its stream set back
            for sl in self._slots:
                if sl.engine is not engine:
                    sl.engine.close()
            self._host.close()
            release_stream_set(device, self._stream_set)
            raise

    def _init_device(self, aug_cfg, device, depth, engine, max_image_dim, workspace_bytes) -> None:
        if (self._feed and depth > 1 and os.environ.get("DINO_COPY_STREAM", "1") != "0") or self._side_ahead:
            self._copy_stream = role_stream(device, "copy", 0, self._stream_set)
        max_crop = max(int(aug_cfg.max_global_crop_size or aug_cfg.global_crop_size),
                       int(aug_cfg.max_local_crop_size or aug_cfg.local_crop_size),
                       aug_cfg.global_crop_size, aug_cfg.local_crop_size)
        for k in range(self.depth):
            if k == 0 and engine is not None:
                eng = engine
            else:
                stream = role_stream(device, "slot", k, self._stream_set) if self.depth > 1 else None
                eng = IngestEngine(device, max_batch=self._batch_size, max_views=aug_cfg.n_views,
                                   max_crop_size=max_crop, max_image_dim=max_image_dim,
                                   workspace_bytes=workspace_bytes, stream=stream)
            self._slots.append(_Slot(eng))
        self._last: _Slot = self._slots[0]          # the last launched batch
        # output sets (shape key, tensors, consumer stream), batch n -> set n % (depth + 1)
        self._view_ring: list = [None] * (self.depth + 1)
        self._handed: _Slot | None = None            # the last batch handed over (iterator / run_one_batch)
        # study hook (DINO_TIMELINE=1): per batch, host stamps and timing events on the copy and
        # slot streams (``timeline()``); off, nothing is recorded
        self._timeline: list | None = [] if os.environ.get("DINO_TIMELINE") == "1" else None
        if self._feed:
            sizes = self._sizes()
            self._feed_sizes = sizes
            self._source.configure(max_image_dim=self._max_image_dim, cfg=self._cfg(*sizes))
        self._closed = False
        _LIVE.add(self)

    @staticmethod
    def side_queue(prefetch_ahead: int, side_ahead: int) -> int:
        """The prefetch thread's queue length on the side route (see ``_pull_one``)."""
        return prefetch_ahead + min(side_ahead, 4)

    @staticmethod
    def pulled_bound(depth: int, prefetch_ahead: int, side_ahead: int) -> int:
        """Most batches pulled from the source and not yet handed over, on the side route: the
        look-ahead, the prefetch queue, the batches being packed (one per pack thread), the
        puller's queue and the batch it holds, and the batches in flight.  A source whose metadata FIFO
        pairs each pulled batch with its hand-over (reference _ReaderAdapter._meta_queue,
        shard_reader.py:98, 357-375) must hold this many."""
        return (side_ahead + MI355XAugPipeline.side_queue(prefetch_ahead, side_ahead) + PACK_THREADS + RAW_AHEAD + 1 +
                depth)

    @property
    def engine(self) -> IngestEngine:
        return self._slots[0].engine

    @property
    def device(self) -> torch.device:
        return self.engine.device

    def set_timing(self, enable: bool) -> None:
        for sl in self._slots:
            sl.engine.set_timing(enable)

    def kernel_times(self) -> dict[str, tuple[float, int]]:
        """Per-kernel (ms, launches) summed over the slots (HIP events on each slot's stream)."""
        tot: dict[str, tuple[float, int]] = {}
        for sl in self._slots:
            for k, (ms, n) in sl.engine.kernel_times().items():
                a, b = tot.get(k, (0.0, 0))
                tot[k] = (a + ms, b + n)
        return tot

    def _sizes(self) -> tuple[int, int]:
        if self._resolution_src is None:
            return self._aug_cfg.global_crop_size, self._aug_cfg.local_crop_size
        g, l = self._resolution_src()
        return int(g), int(l)

    def _cfg(self, g: int, l: int):
        return make_aug_config(self._aug_cfg, g, l, self._out)

    def _next_slot(self) -> _Slot:
        return self._slots[self._batch_index % self.depth]

    def run_device_batch(self, d_bytes: torch.Tensor, d_offsets: torch.Tensor, batch: int | None = None,
                         views: list[torch.Tensor] | None = None,
                         raw_mask: torch.Tensor | None = None) -> dict[str, torch.Tensor]:
        """Stage 3 on JPEG bytes already resident in HBM (the benchmark's device-resident path).

        With depth > 1 the work is enqueued on the slot's stream after the caller's
        stream (which produced d_bytes); the caller's stream is NOT made to wait for
        the outputs — call ``wait()`` (or synchronise) before reading them."""
        if self._closed:
            raise RuntimeError("MI355XAugPipeline.run_one_batch() called after close()")
        sl = self._next_slot()
        if sl.engine.stream is not None:
            sl.engine.stream.wait_stream(torch.cuda.current_stream(self.device))
        return self._launch(sl, d_bytes, d_offsets, batch, views, raw_mask=raw_mask)

    def _launch(self, sl: _Slot, d_bytes, d_offsets, batch, views, cfg=None, account: bool = False,
                raw_mask: torch.Tensor | None = None, sizes=None, probe: np.ndarray | None = None,
                lengths: torch.Tensor | None = None):
        batch = self._batch_size if batch is None else int(batch)
        if cfg is None:
            sizes = self._sizes()
            cfg = self._cfg(*sizes)
        sl.sizes, sl.probe, sl.batch_index = sizes, probe, self._batch_index
        eng = sl.engine
        if sl.params is None or sl.params.numel() < batch * self._aug_cfg.n_views * RECORD_BYTES:
            with eng.on_stream():
                sl.params = torch.empty(batch * self._aug_cfg.n_views * RECORD_BYTES, dtype=torch.uint8,
                                        device=self.device)
        if self._norm is not None:  # per-dataset statistics of this batch's images (DALI NormSource)
            recs = torch.from_numpy(self._norm.batch_records(batch)).pin_memory()
            with eng.on_stream():
                sl.norm = recs.to(self.device, non_blocking=True)
            eng.set_norm(sl.norm)
        if views is None:
            views = self._views_for(sl, cfg, batch)
        else:
            sl.view_set = -1  # the caller's own tensors, not a set of the ring
        views, info = eng.run_batch(d_bytes, d_offsets, batch, cfg, self._seed, self._batch_index,
                                    views=views, params_out=sl.params, raw_mask=raw_mask, lengths=lengths)
        sl.info = info
        sl.outputs = {self._names[i]: v for i, v in enumerate(views)}
        if account:  # per-image status back to the host asynchronously (accounted at a later hand-over)
            # each pending batch owns a pinned status buffer from a small pool, so launching never
            # waits for an earlier batch of the slot to finish
            host = self._info_pool.pop() if self._info_pool else None
            if host is None or host.shape[0] < batch:
                host = torch.empty((batch, 4), dtype=torch.int32, pin_memory=True)
            with eng.on_stream():
                host[:batch].copy_(info, non_blocking=True)
            done = torch.cuda.Event()
            done.record(eng.stream if eng.stream is not None else torch.cuda.current_stream(self.device))
            sl.batch_id = self._batch_index
            self._pending.append((host, done, sl.batch_id, batch))
        if eng.stream is not None:
            sl.event = torch.cuda.Event()
            sl.event.record(eng.stream)
            if sl.view_set >= 0 and self._view_ring[sl.view_set] is not None:
                self._view_ring[sl.view_set][3] = sl.event  # a later batch reusing the set waits for it
        self._last = sl
        self._handed = None
        self._batch_index += 1
        return sl.outputs

    def _views_for(self, sl: _Slot, cfg, batch: int) -> list[torch.Tensor]:
        """Output tensors for the slot's next batch.  Batch n takes output set n % (depth + 1)
        of a ring: with ``depth`` batches in flight, the set's previous batch (n - depth - 1)
        is one the caller has replaced by a later one in ``for batch in loader`` (whose loop
        variable still holds batch n - depth while batch n launches, so a set per slot was
        never free then: every batch allocated its outputs anew, ~1.3 ms of the host thread
        per batch).  The set is reused when nothing but the pipeline references it, else new
        tensors are made; a reused set is written only after the work the caller had queued
        on its stream by now (the caching allocator's record_stream rule, applied at reuse)."""
        key = (batch, cfg.n_global, cfg.n_local, cfg.global_size, cfg.local_size, cfg.out_dtype)
        j = self._batch_index % len(self._view_ring)
        sl.view_set = j
        vc = self._view_ring[j]
        if vc is not None and vc[0] == key:
            in_dicts = [sum(1 for s in self._slots if s.outputs is not None and any(o is t for o in s.outputs.values()))
                        for t in vc[1]]
            if _all_unshared(vc[1], in_dicts):
                if sl.engine.stream is not None:
                    if vc[2] is not None:  # the caller's work on the set's last hand-over
                        ev = torch.cuda.Event()
                        ev.record(vc[2])
                        sl.engine.stream.wait_event(ev)
                    if vc[3] is not None:  # the set's last writer, a batch of another slot
                        sl.engine.stream.wait_event(vc[3])
                return vc[1]
        views = sl.engine.alloc_views(cfg, batch)
        # [shape key, tensors, consumer stream of the last hand-over, completion of the last writer]
        self._view_ring[j] = [key, views, None, None]
        return views

    # ------------------------------------------------------------------ host half
    def _prepare_next(self) -> _Prepared:
        """Pull the next batch from the source and make it ready to launch: pack it into a
        pinned staging buffer and probe it in one native pass (``dino_gather_probe``: the
        copier threads parse each image's header right after copying it: status, kind,
        workspace bytes for the current (G, L)), then submit the Pillow decodes of the images
        routed to the host (``fallback.route_mask``).  A page-locked spans feed batch that
        needs no hand-over is not packed at all (its shard ranges are DMA'd at launch).
        Runs on the prefetch thread (or inline at prefetch 0)."""
        return self._pack_raw(self._pull_raw())

    def _pull_raw(self) -> tuple:
        """The pull half of ``_prepare_next``: the source's next batch as (spans batch or None,
        JPEG list or None, pointers, lengths, references keeping the bytes alive)."""
        from .tario import spans_of
        t0 = time.perf_counter()
        bs = None
        jpegs = None
        keep = None
        if self._spans_feed:
            bs = self._source.next_batch_spans()  # may raise StopIteration (end of epoch)
            ptrs, lens = bs.ptrs, bs.lens
        elif self._native:
            ptrs, lens, _ = spans_of(self._source.next_spans())  # may raise StopIteration
        else:
            jpegs = self._source()  # may raise StopIteration (end of epoch)
            ptrs, lens, keep = spans_of(jpegs)
        self.host_seconds["pull"] += time.perf_counter() - t0
        return bs, jpegs, ptrs, lens, keep

    def _pack_raw(self, raw: tuple) -> _Prepared:
        """The pack half of ``_prepare_next`` (see there)."""
        bs, jpegs, ptrs, lens, _keep = raw
        B = self._batch_size
        hs = self.host_seconds
        try:
            if len(lens) != B:
                raise ValueError(f"source returned {len(lens)} samples, expected {B}")
            sizes = self._sizes()
            cfg = self._cfg(*sizes)
            t1 = time.perf_counter()
            if bs is not None and bs.registered:
                info, ws, aws = fallback.probe_spans(ptrs, lens, self._max_image_dim, cfg)
                if not fallback.route_mask(info, self._host_fallback, self._route, self._host_max).any():
                    st = self._ring.acquire()
                    st.fit(0, B)
                    st.off.numpy()[: B + 1] = bs.offsets
                    st.lens.numpy()[:B] = lens
                    hs["probe"] += time.perf_counter() - t1
                    return _Prepared(st, None, bs.offsets, info, ws, aws, sizes, {}, spans=bs)
            st = self._ring.acquire()
            hs["staging"] = hs.get("staging", 0.0) + time.perf_counter() - t1  # waiting for a free staging buffer
            try:
                st.fit(int(lens.sum()), B)
                off, info, ws, aws = fallback.gather_probe(ptrs, lens, st.buf, self._gather_threads,
                                                           self._max_image_dim, cfg)
                st.off.numpy()[: B + 1] = off
                hs["pack"] += time.perf_counter() - t1
                if bs is not None:  # packed: the shard ranges are no longer read
                    self._source.retire(bs, None)
                    bs = None
                mask = fallback.route_mask(info, self._host_fallback, self._route, self._host_max)
                futures = {}
                idx = np.flatnonzero(mask)
                if len(idx):
                    if jpegs is None:  # packed native feed: slice the images back out of the staging buffer
                        hb = st.buf.numpy()
                        jpegs = [bytes(hb[off[i]:off[i + 1]]) for i in range(B)]
                    futures = {int(i): self._host.submit(jpegs[i]) for i in idx}
                return _Prepared(st, jpegs, off, info, ws, aws, sizes, futures)
            except BaseException:
                self._ring.release(st, None)
                raise
        except BaseException:
            if bs is not None:
                self._source.retire(bs, None)
            raise

    def _drop(self, pb: _Prepared) -> None:
        """A prepared batch that will never launch: free its staging, retire its shard ranges,
        hand its feed slot back."""
        if pb.staging is not None:
            self._ring.release(pb.staging, None)
        if pb.spans is not None:
            self._source.retire(pb.spans, None)
        if pb.feed is not None:
            self._source.release(pb.feed)

    def _prepare_feed(self, block: bool) -> _Prepared | None:
        """The native feed's next batch as a ``_Prepared`` (None: not ready and ``block`` is
        False; StopIteration at the epoch end).  Images routed to Pillow are copied out of
        the slot and their decodes submitted; such a batch is re-packed at launch."""
        fb = self._source.next_prepared(timeout=None if block else 0.0)
        if fb is None:
            return None
        mask = fallback.route_mask(fb.info, self._host_fallback, self._route, self._host_max)
        if not mask.any():
            return _Prepared(None, None, fb.offsets, fb.info, fb.ws, fb.aws, self._feed_sizes, {}, feed=fb)
        try:
            jpegs = fb.jpegs()
        finally:
            self._source.release(fb)
        futures = {int(i): self._host.submit(jpegs[i]) for i in np.flatnonzero(mask)}
        return _Prepared(None, jpegs, fb.offsets, fb.info, fb.ws, fb.aws, self._feed_sizes, futures)

    def _pull_feed(self) -> _Prepared:
        t0 = time.perf_counter()
        try:
            pb = self._held.popleft() if self._held else self._prepare_feed(block=True)
            try:  # one batch ahead: its Pillow hand-overs (if any) run while this one is on the GPU
                nxt = self._prepare_feed(block=False)
                if nxt is not None:
                    self._held.append(nxt)
            except StopIteration:
                pass
            return pb
        finally:
            self.host_seconds["wait"] += time.perf_counter() - t0

    def _pull_one(self, block: bool) -> _Prepared | None:
        """The next prepared batch from the feed or the prefetch thread (None: none ready and
        not ``block``); StopIteration at the end of the epoch."""
        if self._feed:
            return self._prepare_feed(block)
        if self._prefetcher is None:
            # the side path's look-ahead fills from this queue, which _pull_side drains at every
            # launch: a queue longer than prefetch_ahead lets the look-ahead grow by up to 4
            # batches per launch (a queue of 1 would keep it where it starts) without pulling
            # many more batches from the source than the look-ahead holds
            self._prefetcher = _Prefetcher(self, self.side_queue(self.prefetch_ahead, self._side_ahead))
        return self._prefetcher.get(block)

    def _side_submit(self, pb: _Prepared) -> None:
        """Start the side decode of the batch's coefficient-buffer images (progside.py)."""
        from . import progside
        if pb.side_submitted:
            return
        pb.side_submitted = True
        m = progside.side_mask(pb.info)
        for i in pb.futures:
            m[i] = False
        idx = np.flatnonzero(m)
        if not len(idx):
            return
        if self._side is None:
            lanes, pool = progside.side_plan(self._side_ahead)
            self._side = progside.DeviceSideDecoder(self.device, max_images=pool, max_image_dim=self._max_image_dim,
                                                    stream_set=self._stream_set, lanes=lanes)
            self.stats["side_lanes"] = lanes
        if pb.jpegs is not None:
            imgs = {int(i): pb.jpegs[i] for i in idx}
        elif pb.feed is not None:
            o = pb.feed.offsets
            imgs = {int(i): ctypes.string_at(pb.feed.host + int(o[i]), int(o[i + 1] - o[i])) for i in idx}
        elif pb.spans is not None:  # a batch left where it lies (page-locked shard ranges): never packed
            imgs = {int(i): ctypes.string_at(int(pb.spans.ptrs[i]), int(pb.spans.lens[i])) for i in idx}
        else:
            hb, o = pb.staging.buf.numpy(), pb.offsets
            imgs = {int(i): hb[o[i]:o[i + 1]].tobytes() for i in idx}
        room = {}
        if pb.dev is not None and pb.room:
            room = {i: (pb.dev[0], pb.room[i]) for i in imgs if i in pb.room}
        pb.side = self._side.add(imgs, room, pb.copied if room else None)

    def _stage_early(self, pb: _Prepared) -> None:
        """On the prefetch thread: a batch bound for the side look-ahead (the route is engaged,
        or the batch carries coefficient-buffer images) goes to HBM right after its pack, so
        its staging buffer returns to the ring when the copy retires instead of when the
        launch thread pulls the batch (the prefetch thread waited ~1-2 ms per batch for a free
        staging buffer, c2_prog).  Only batches whose images the source handed over as a list
        (``pb.jpegs``, what the side decoder reads them from later)."""
        if not self._side_ahead or pb.jpegs is None or pb.futures or pb.dev is not None:
            return
        from . import progside
        if self._side_hot > 0 or progside.side_mask(pb.info).any():
            self._stage_on_device(pb)

    def _stage_on_device(self, pb: _Prepared) -> None:
        """Copy a batch that joins the side look-ahead to HBM now, on the copy stream, and free
        its host buffer (pinned staging, native feed slot, page-locked shard ranges) once the
        copy retires: the look-ahead is up to ``side_ahead`` batches deep, and holding them in
        host buffers would take that many pinned batches.  A batch waiting for Pillow
        hand-overs stays on the host (it is re-packed at launch)."""
        if pb.futures or pb.dev is not None:
            return
        cs = self._copy_stream
        B = len(pb.offsets) - 1
        d_lens = None
        with torch.cuda.stream(cs):
            if pb.feed is not None:
                fb = pb.feed
                d_bytes = torch.empty(max(fb.nbytes, 1) + 64, dtype=torch.uint8, device=self.device)
                d_off = torch.empty(B + 1, dtype=torch.int64, device=self.device)
                try:
                    self._source.copy(fb, d_bytes.data_ptr(), d_off.data_ptr(), cs.cuda_stream)
                except BaseException:
                    self._source.release(fb)
                    raise
                finally:
                    pb.feed = None  # the slot returns to the packer when this copy retires
            elif pb.spans is not None:
                nbytes = int(pb.spans.offsets[-1])
                d_bytes = torch.empty(max(nbytes, 1) + 64, dtype=torch.uint8, device=self.device)
                pos = 0
                eng = self._slots[0].engine
                for addr, n in pb.spans.parts:
                    eng.copy_from_host(d_bytes, pos, addr, n, stream=cs)
                    pos += n
                d_off = pb.staging.off[: B + 1].to(self.device, non_blocking=True)
                d_lens = pb.staging.lens[:B].to(self.device, non_blocking=True)
            else:
                st = pb.staging
                nbytes = int(pb.offsets[-1])
                # room after the batch's bytes for the raw containers of its coefficient-buffer
                # images: the side decoder writes them there, so the launch needs no merge copy
                from . import progside
                pos = (nbytes + 15) & ~15
                for i in np.flatnonzero(progside.side_mask(pb.info)):
                    if int(i) not in pb.futures:
                        pb.room[int(i)] = pos
                        pos += (16 + int(pb.info[i, 1]) * int(pb.info[i, 2]) * 3 + 15) & ~15
                d_bytes = torch.empty(max(pos, 1) + 64, dtype=torch.uint8, device=self.device)
                d_bytes[:max(nbytes, 1)].copy_(st.buf[:max(nbytes, 1)], non_blocking=True)
                d_off = st.off[: B + 1].to(self.device, non_blocking=True)
            ev = torch.cuda.Event()
            ev.record(cs)
        if pb.spans is not None:
            pb.lens = np.asarray(pb.spans.lens, np.int64).copy()
            self._source.retire(pb.spans, ev)
            pb.spans = None
        if pb.staging is not None:
            self._ring.release(pb.staging, ev)
            pb.staging = None
        pb.dev = (d_bytes, d_off, d_lens)
        pb.copied = ev

    def _pull_side(self) -> _Prepared:
        """The side path's look-ahead: keep up to side_ahead prepared batches, each with its
        side decode started as it arrives; hand out the oldest.

        The look-ahead is engaged only while coefficient-buffer images are about: a batch
        with one (re)arms it for the next ``side_ahead`` batches pulled.  Disengaged, the
        pipeline pulls one batch at a time and launches it from its own host buffer (feed
        slot / pinned staging) as the plain route does, so a stream of baseline JPEGs pays
        neither the HBM staging copy nor the look-ahead's extra buffers (with
        the look-ahead always on the e2e rate fell from 145.6k to 125.6k img/s)."""
        t0 = time.perf_counter()
        try:
            while not self._source_end and (not self._ahead or
                                            (self._side_hot > 0 and len(self._ahead) < self._side_ahead)):
                # a head batch whose side decode is still running waits for it behind further
                # batches (pulled blocking) rather than at its launch: when the host half is the
                # bottleneck the look-ahead never fills otherwise, every pool is flushed small and
                # late, and each launch waits out a whole side decode (~30 ms of k_pscan latency)
                head_busy = bool(self._ahead) and self._ahead[0].side is not None and not self._ahead[0].side.done()
                try:
                    pb = self._pull_one(block=not self._ahead or head_busy)
                except StopIteration:
                    self._source_end = True
                    break
                if pb is None:
                    break
                self._side_submit(pb)
                if pb.side is not None:
                    if self._side_hot == 0:  # engaging: the batches already ahead free their host buffers too
                        for q in self._ahead:
                            self._stage_on_device(q)
                    self._side_hot = self._side_ahead
                elif self._side_hot > 0:
                    self._side_hot -= 1
                if self._side_hot > 0:
                    self._stage_on_device(pb)
                self._ahead.append(pb)
            if not self._ahead:
                raise StopIteration
            # the pool launches when it holds min_images, or once its oldest batch is within
            # half the look-ahead of its own launch (a decode then has those batches' time to
            # finish; flushing at launch would make the batch wait for it).  With the lane
            # plan, while the look-ahead is shorter than that (the host half fell behind), only
            # the next SIDE_URGENT_SHORT batches are urgent: flushing every batch as it arrived
            # made pools of one batch's images, whose launches starved the batches and kept the
            # look-ahead short (c2_prog 50-78k img/s in that state, profiles/r06_side_plan/r6q)
            half = max(1, self._side_ahead // 2)
            short = self._side is not None and self._side.lanes and len(self._ahead) <= half
            urgent = min(len(self._ahead), SIDE_URGENT_SHORT if short else half)
            if self._side is not None and any(pb.side is not None and pb.side.pending
                                              for pb in itertools.islice(self._ahead, urgent)):
                self._side.flush()
                self.stats["side_urgent"] = self.stats.get("side_urgent", 0) + 1
            return self._ahead.popleft()
        finally:
            self.host_seconds["wait"] += time.perf_counter() - t0

    def _pull(self) -> _Prepared:
        if self._side_ahead:
            return self._pull_side()
        if self._feed:
            return self._pull_feed()
        if self.prefetch_ahead <= 0:
            return self._prepare_next()
        if self._prefetcher is None:
            self._prefetcher = _Prefetcher(self, self.prefetch_ahead)
        t0 = time.perf_counter()
        try:
            return self._prefetcher.get()
        finally:
            self.host_seconds["wait"] += time.perf_counter() - t0

    def _host_result(self, f, jpeg) -> bytes:
        try:
            return f.result()
        except Exception:  # noqa: BLE001 - a broken worker pool: decode here (same bytes)
            return fallback.pillow_container(jpeg)

    def _screen(self, sl: _Slot, pb: _Prepared, cfg, sizes) -> tuple[torch.Tensor, torch.Tensor, int, torch.Tensor | None]:
        """Collect a prepared batch's host decodes (re-packing the batch into its staging if
        there were any), re-probe only if that or the crop sizes changed what the probe saw,
        and grow the slot's workspaces (stream-ordered).  Returns the pinned buffer, pinned
        offsets, byte count and pinned raw mask (None when the batch has no container)."""
        B = len(pb.offsets) - 1
        raw = None
        ws, aws = pb.ws, pb.aws
        if pb.futures and pb.staging is None:  # a native feed batch with hand-overs: re-packed here
            pb.staging = self._ring.acquire()
        st = pb.staging
        if pb.futures:
            from .tario import gather
            jpegs = list(pb.jpegs)
            for i, f in pb.futures.items():
                jpegs[i] = self._host_result(f, jpegs[i])
            self.stats["host_decoded"] += len(pb.futures)
            rm = fallback.raw_mask_of(jpegs, pb.futures)
            st.fit(sum(len(j) for j in jpegs), B)
            off = gather(jpegs, st.buf, 8)
            st.off.numpy()[: B + 1] = off
            st.mask.numpy()[:B] = rm
            raw = st.mask[:B]
            pb.info, ws, aws = fallback.probe(st.buf.data_ptr(), off, B, self._max_image_dim, cfg, rm)
            nbytes = int(off[-1])
        else:
            nbytes = int(pb.offsets[-1])
            if tuple(sizes) != tuple(pb.sizes):
                aws = fallback.augment_need(pb.info, cfg)
        if sl.engine.reserve(ws, aws):
            self.stats["reserves"] += 1
        if st is None:  # native feed slot: copied by dino_feed_copy
            return None, None, nbytes, raw
        return st.buf, st.off[: B + 1], nbytes, raw

    def _account(self, block: bool = False) -> None:
        """Fold the per-image status of finished batches into ``stats`` (oldest first)."""
        while self._pending:
            host, done, bid, batch = self._pending[0]
            if not block and not done.query():
                break
            done.synchronize()
            self._pending.popleft()
            st = host[:batch, 0].numpy().copy()
            self._info_pool.append(host)
            self.stats["batches"] += 1
            self.stats["images"] += batch
            self.stats["status"].update(int(x) for x in st)
            bad = st[st > 0]
            if bad.size:
                from ._lib import IMG_STATUS
                kinds = ", ".join(f"{n} {IMG_STATUS.get(int(k), k)}" for k, n in Counter(bad.tolist()).items())
                warnings.warn(f"MI355XAugPipeline: batch {bid}: {bad.size} decodable image(s) returned zero-filled "
                              f"views ({kinds}); see MI355XAugPipeline.stats", RuntimeWarning, stacklevel=3)

    def _enqueue_one(self) -> _Slot:
        """Take the next prepared batch and enqueue it on the next slot: H2D copies of the
        staging on the slot's stream, then the kernels (``dino_run_batch``)."""
        if self._closed:
            raise RuntimeError("MI355XAugPipeline.run_one_batch() called after close()")
        self._tl_pull = time.perf_counter()
        return self._enqueue_prepared(self._pull())

    def _enqueue_prepared(self, pb: _Prepared) -> _Slot:
        if self._closed:
            self._drop(pb)
            raise RuntimeError("MI355XAugPipeline.run_one_batch() called after close()")
        st = pb.staging
        t0 = time.perf_counter()
        tl = {"t0": t0, "pull": getattr(self, "_tl_pull", t0)} if self._timeline is not None else None
        copied = None
        buf_j = None  # the native feed's input buffer of the slot this batch reads
        try:
            sl = self._next_slot()
            sizes = self._sizes()
            cfg = self._cfg(*sizes)
            host_buf, host_off, nbytes, raw = self._screen(sl, pb, cfg, sizes)
            B = len(pb.offsets) - 1
            d_lens = None
            with sl.engine.on_stream():
                if pb.dev is not None:  # copied to HBM when it joined the side look-ahead
                    cur = torch.cuda.current_stream(self.device)
                    cur.wait_event(pb.copied)
                    d_bytes, d_offsets, d_lens = pb.dev
                    for t in pb.dev:
                        if t is not None:
                            t.record_stream(cur)
                elif pb.feed is not None:  # the native feed's pinned slot: bytes + offsets in two DMAs
                    fb, pb.feed = pb.feed, None
                    j = sl.buf_next
                    sl.buf_next ^= 1
                    if sl.d_ins[j] is None or sl.d_ins[j].numel() < fb.nbytes + 64:
                        if sl.buf_done[j] is not None:  # the old buffer's last reader must finish first
                            sl.buf_done[j].synchronize()
                        sl.d_ins[j] = torch.empty(max(fb.nbytes, 1) * 9 // 8 + 64, dtype=torch.uint8,
                                                  device=self.device)
                    if sl.d_offs[j] is None or sl.d_offs[j].numel() < B + 1:
                        if sl.buf_done[j] is not None:
                            sl.buf_done[j].synchronize()
                        sl.d_offs[j] = torch.empty(B + 1, dtype=torch.int64, device=self.device)
                    cs = self._copy_stream if self._copy_stream is not None else sl.engine.stream
                    try:
                        if cs is not sl.engine.stream and sl.buf_done[j] is not None:
                            cs.wait_event(sl.buf_done[j])
                        if tl is not None:
                            tl["issue"] = time.perf_counter()
                            tl["c0"] = torch.cuda.Event(enable_timing=True)
                            tl["c0"].record(cs)
                        self._source.copy(fb, sl.d_ins[j].data_ptr(), sl.d_offs[j].data_ptr(),
                                          cs.cuda_stream if cs is not None else 0)
                        if tl is not None:
                            tl["c1"] = torch.cuda.Event(enable_timing=True)
                            tl["c1"].record(cs)
                    except BaseException:
                        self._source.release(fb)
                        raise
                    if cs is not sl.engine.stream:
                        arrived = torch.cuda.Event()
                        arrived.record(cs)
                        torch.cuda.current_stream(self.device).wait_event(arrived)
                    d_bytes, d_offsets = sl.d_ins[j], sl.d_offs[j][: B + 1]
                    buf_j = j
                elif pb.spans is not None:  # DMA the batch's shard ranges as they lie (no host copy)
                    nbytes = int(pb.spans.offsets[-1])
                    if sl.d_in is None or sl.d_in.numel() < nbytes:
                        sl.d_in = torch.empty(max(nbytes, 1) * 9 // 8 + 64, dtype=torch.uint8, device=self.device)
                    pos = 0
                    for addr, n in pb.spans.parts:
                        sl.engine.copy_from_host(sl.d_in, pos, addr, n)
                        pos += n
                    d_bytes = sl.d_in
                    d_lens = st.lens[:B].to(self.device, non_blocking=True)
                else:
                    d_bytes = host_buf[:max(nbytes, 1)].to(self.device, non_blocking=True)
                if host_off is not None and pb.dev is None:
                    d_offsets = host_off.to(self.device, non_blocking=True)
                d_raw = raw.to(self.device, non_blocking=True) if raw is not None else None
                side = None
                if pb.side is not None:  # coefficient-buffer images decoded ahead: their containers
                    if pb.side.pending:  # still in the side pool: decode it now
                        self._side.flush()
                    conts = pb.side.ready()
                    if conts:
                        tm = time.perf_counter()
                        base = host_off.numpy() if host_off is not None else pb.offsets
                        # image lengths: the spans form's own (its offsets point into shard
                        # ranges, the gaps hold tar headers and sidecars); packed: the gaps
                        base_lens = pb.spans.lens if pb.spans is not None else \
                            pb.lens if pb.lens is not None else np.diff(base[: B + 1])
                        d_bytes, d_offsets, d_lens, d_raw = self._merge_side(
                            pb.side, conts, d_bytes, int(base[B]), base, base_lens, raw, B)
                        side = conts
                        self.stats["side_decoded"] += len(conts)
                        self.host_seconds["merge"] = self.host_seconds.get("merge", 0.0) + time.perf_counter() - tm
                copied = torch.cuda.Event()
                copied.record()
            if tl is not None:
                tl["k0"] = torch.cuda.Event(enable_timing=True)
                tl["k0"].record(sl.engine.stream)
            self._launch(sl, d_bytes, d_offsets, B, None, cfg=cfg, account=True, raw_mask=d_raw, sizes=sizes,
                         probe=pb.info, lengths=d_lens)
            if tl is not None:
                tl["k1"] = torch.cuda.Event(enable_timing=True)
                tl["k1"].record(sl.engine.stream)
                tl["t1"] = time.perf_counter()
                tl["slot"] = self._slots.index(sl)
                self._timeline.append(tl)
            if buf_j is not None:
                sl.buf_done[buf_j] = sl.event
            sl.inflight = (d_bytes, d_offsets, d_raw, d_lens, side)  # device copies live until the slot's next batch
        except BaseException:
            if pb.staging is not None:
                self._ring.release(pb.staging, copied)
            if pb.spans is not None:
                self._source.retire(pb.spans, copied)
            if pb.feed is not None:
                self._source.release(pb.feed)
            raise
        if pb.staging is not None:
            self._ring.release(pb.staging, copied)
        if pb.spans is not None:
            self._source.retire(pb.spans, copied)
        self.host_seconds["launch"] += time.perf_counter() - t0
        return sl

    def _merge_side(self, job, conts: dict, d_bytes: torch.Tensor, nbytes: int, base_off: np.ndarray,
                    base_lens: np.ndarray, raw: torch.Tensor | None, B: int):
        """The batch's input with its side-decoded images swapped for their device containers
        (spans form: the batch bytes, then the containers; those images' offsets and lengths
        point at their containers and the raw mask marks them).  Runs on the slot's stream,
        after the side decode (stream wait)."""
        cur = torch.cuda.current_stream(self.device)
        cur.wait_event(job.event)
        off = np.asarray(base_off, np.int64)[: B + 1].copy()
        lens = np.asarray(base_lens, np.int64)[:B].copy()
        rawm = raw.cpu().numpy().astype(np.uint8) if raw is not None else np.zeros(B, np.uint8)
        base, cap = d_bytes.data_ptr(), d_bytes.numel()
        if all(base <= c.data_ptr() and c.data_ptr() + c.numel() <= base + cap for c in conts.values()):
            # every container was written into the room after the batch's bytes: no copy
            for i, c in conts.items():
                off[i], lens[i], rawm[i] = c.data_ptr() - base, int(c.numel()), 1
            off[B] = cap
            h_off = torch.from_numpy(off).pin_memory()
            h_len = torch.from_numpy(lens.astype(np.int64)).pin_memory()
            h_raw = torch.from_numpy(rawm).pin_memory()
            return (d_bytes, h_off.to(self.device, non_blocking=True), h_len.to(self.device, non_blocking=True),
                    h_raw.to(self.device, non_blocking=True))
        pos = (nbytes + 15) & ~15
        total = pos + sum((int(c.numel()) + 15) & ~15 for c in conts.values())
        merged = torch.empty(total + 64, dtype=torch.uint8, device=self.device)
        merged[:nbytes].copy_(d_bytes[:nbytes], non_blocking=True)
        for i, c in conts.items():
            n = int(c.numel())
            merged[pos:pos + n].copy_(c, non_blocking=True)
            c.record_stream(cur)
            off[i], lens[i], rawm[i] = pos, n, 1
            pos += (n + 15) & ~15
        off[B] = total
        h_off = torch.from_numpy(off).pin_memory()
        h_len = torch.from_numpy(lens.astype(np.int64)).pin_memory()
        h_raw = torch.from_numpy(rawm).pin_memory()
        return (merged, h_off.to(self.device, non_blocking=True), h_len.to(self.device, non_blocking=True),
                h_raw.to(self.device, non_blocking=True))

    def _refresh(self, sl: _Slot, sizes: tuple[int, int]) -> None:
        """The crop sizes changed (``ResolutionSource.set``, reference loader.py:280-308) after
        this batch was launched: make its views again at the new sizes from the decoded images
        still in the slot's workspace (same (seed, batch index) records), so that a resolution
        change takes effect on the next batch handed over (CPUBackend semantics, cpu.py:315-317)
        even with ``depth`` batches in flight."""
        cfg = self._cfg(*sizes)
        eng = sl.engine
        if eng.reserve(0, fallback.augment_need(sl.probe, cfg)):
            self.stats["reserves"] += 1
        eng.sample_params(cfg, self._seed, sl.batch_index, out=sl.params)
        views = eng.augment(cfg, sl.params)
        eng.batch_info(sl.info)
        sl.outputs = {self._names[i]: v for i, v in enumerate(views)}
        sl.sizes = sizes
        sl.view_set = -1  # fresh tensors at the new sizes: not a set of the ring
        if eng.stream is not None:
            sl.event = torch.cuda.Event()
            sl.event.record(eng.stream)

    def _hand_over(self, sl: _Slot) -> dict[str, torch.Tensor]:
        """Order the caller's stream after the slot's work and tie the outputs to it."""
        self._account()
        if self._resolution_src is not None and sl.probe is not None:
            sizes = self._sizes()
            if tuple(sizes) != tuple(sl.sizes):
                self._refresh(sl, sizes)
        if sl.event is not None:
            cur = torch.cuda.current_stream(self.device)
            cur.wait_event(sl.event)
            for t in sl.outputs.values():
                t.record_stream(cur)
            if sl.view_set >= 0 and self._view_ring[sl.view_set] is not None:
                self._view_ring[sl.view_set][2] = cur  # the stream the set was handed to
        self._handed = sl
        return dict(sl.outputs)  # the caller's own dict: its references keep the tensors from reuse

    def timeline(self) -> list[dict]:
        """The DINO_TIMELINE=1 records (after a synchronize): per batch, host seconds of the
        launch start / copy issue / launch end and device ms of copy start / end and kernel
        start / end, both relative to the first record."""
        if not self._timeline:
            return []
        torch.cuda.synchronize(self.device)
        ref = self._timeline[0]
        e0 = ref.get("c0") or ref["k0"]
        out = []
        for r in self._timeline:
            d = {"slot": r["slot"], "pull": r["pull"] - ref["t0"], "t0": r["t0"] - ref["t0"], "t1": r["t1"] - ref["t0"]}
            if "issue" in r:
                d["issue"] = r["issue"] - ref["t0"]
            for k in ("c0", "c1", "k0", "k1"):
                if k in r:
                    d[k] = e0.elapsed_time(r[k]) / 1e3
            out.append(d)
        return out

    def wait(self) -> None:
        """Make the caller's stream wait for the last enqueued batch."""
        self._hand_over(self._last)

    def run_one_batch(self) -> dict[str, torch.Tensor]:
        return self._hand_over(self._enqueue_one())

    def restart_epoch(self) -> None:
        """After the source's StopIteration and its reset: let the host half pull again."""
        while self._held:  # the native feed's look-ahead batch belongs to the finished epoch
            self._drop(self._held.popleft())
        while self._ahead:
            self._drop(self._ahead.popleft())
        self._source_end = False
        if self._prefetcher is not None and self._prefetcher.finished:
            self._prefetcher.close()
            self._prefetcher = None

    def _recent(self) -> _Slot:
        """The batch whose outputs the caller saw last: the last one handed over since the last
        launch (the iterator keeps later batches in flight), else the last one launched."""
        return self._handed if self._handed is not None else self._last

    def last_params(self) -> np.ndarray:
        """Records of the last batch (see ``_recent``), sample-major (``[b * n_views + v]``)."""
        sl = self._recent()
        if sl.event is not None:
            sl.event.synchronize()
        n = sl.engine.last_batch * self._aug_cfg.n_views
        return params_from_device(sl.params[: n * RECORD_BYTES])

    def last_status(self) -> np.ndarray:
        sl = self._recent()
        if sl.event is not None:
            sl.event.synchronize()
        return sl.info[:, 0].cpu().numpy() if sl.info is not None else np.zeros(0, np.int32)

    def flush_stats(self) -> dict:
        """Wait for every launched batch and fold its status into ``stats``."""
        self._account(block=True)
        return self.stats

    def close(self) -> None:
        if not self._closed:
            self._closed = True
            _LIVE.discard(self)
            try:
                self._ring.close()
                if self._prefetcher is not None:
                    self._prefetcher.close()
                    self._prefetcher = None
                while self._held:
                    self._drop(self._held.popleft())
                while self._ahead:
                    self._drop(self._ahead.popleft())
                self._account(block=True)
            finally:
                self._host.close()
                if self._side is not None:
                    self._side.close()
                for sl in self._slots:
                    sl.engine.close()
                release_stream_set(self._device_arg, self._stream_set)

    def __del__(self):
        try:
            self.close()
        except Exception:  # noqa: BLE001
            pass


class MI355XPipelineIterator:
    """DALIGenericIterator-shaped wrapper: ``next()`` -> ``[ {view_name: Tensor} ]``.

    Keeps ``pipeline.depth`` batches in flight (DALI's GPU prefetch queue): each
    ``next()`` tops the queue up, then hands over the oldest batch.  The pipeline's
    prefetch thread prepares the host half of the next batches (pull, pack, probe, Pillow
    hand-overs) while the GPU works."""

    def __init__(self, pipeline: MI355XAugPipeline, output_map: list[str], batch_size: int) -> None:
        self._pipe = pipeline
        self._output_map = list(output_map)
        self._exhausted = False
        self._queue: deque = deque()
        self._source_done = False

    def __iter__(self):
        return self

    def __next__(self) -> list[dict[str, torch.Tensor]]:
        if self._exhausted:
            raise StopIteration
        pipe = self._pipe
        while not self._source_done and len(self._queue) < pipe.depth:
            try:
                self._queue.append(pipe._enqueue_one())
            except StopIteration:
                self._source_done = True
        if not self._queue:
            self._exhausted = True
            raise StopIteration
        return [self._pipe._hand_over(self._queue.popleft())]

    def reset(self) -> None:
        self._exhausted = False
        self._source_done = False
        self._queue.clear()  # batches prepared but not launched are the source's next ones: kept
        self._pipe.restart_epoch()


class MI355XUserAugPipeline:
    """``UserAugSpec`` on the GPU: the reference's ``CPUUserAugPipeline.run_one_batch``
    (cpu.py:484-500) — decode, resize the shorter side to ``decode_size`` (Pillow BICUBIC,
    torchvision ``Resize`` geometry), normalise — as HIP kernels (``dino_resize_batch``),
    then ``aug_fn`` on the device tensor.  Like the reference (which ``torch.stack``s the
    per-image tensors) every image of a batch must resize to the same shape; an
    undecodable image contributes zeros of shape (3, decode_size, decode_size)."""

    def __init__(self, source: Any, spec, batch_size: int, out_dtype="bf16", device: int = 0,
                 max_image_dim: int = 0, workspace_bytes: int = 0, norm=None):
        self._source = source
        self._spec = spec
        self._batch_size = int(batch_size)
        self._out = _out_code(out_dtype)
        self._norm = norm
        self._max_image_dim = int(max_image_dim)
        self._engine = IngestEngine(device, max_batch=self._batch_size, max_views=1, max_crop_size=8,
                                    max_image_dim=max_image_dim, workspace_bytes=workspace_bytes)
        self.stats = {"batches": 0, "images": 0, "status": Counter(), "host_decoded": 0}
        self._pending_status: deque = deque()
        self._closed = False

    @property
    def device(self) -> torch.device:
        return self._engine.device

    def _fold_status(self, st: np.ndarray) -> None:
        self.stats["batches"] += 1
        self.stats["images"] += len(st)
        self.stats["status"].update(int(x) for x in st)
        if (st > 0).any():
            warnings.warn(f"MI355XUserAugPipeline: {int((st > 0).sum())} decodable image(s) returned zeros",
                          RuntimeWarning, stacklevel=3)

    def _drain_status(self, block: bool = False) -> None:
        while self._pending_status and (block or self._pending_status[0][1].query()):
            host, ev = self._pending_status.popleft()
            ev.synchronize()
            self._fold_status(host[:, 0].numpy())

    def flush_stats(self) -> dict:
        self._drain_status(block=True)
        return self.stats

    def run_one_batch(self) -> dict[str, torch.Tensor]:
        if self._closed:
            raise RuntimeError("MI355XUserAugPipeline.run_one_batch() called after close()")
        from .config import resize_shorter_size
        jpegs = self._source()
        assert len(jpegs) == self._batch_size
        host_buf, offsets = pack_jpegs(jpegs, pin=True)
        info, ws, _ = fallback.probe(host_buf.data_ptr(), offsets.numpy(), len(jpegs), self._max_image_dim)
        raw = None
        if np.isin(info[:, 0], (fallback.IMG_UNSUPPORTED, fallback.IMG_LIMIT)).any():
            jpegs, n, rm = fallback.hand_over(list(jpegs), info[:, 0])
            self.stats["host_decoded"] += n
            host_buf, offsets = pack_jpegs(jpegs, pin=True)
            info, ws, _ = fallback.probe(host_buf.data_ptr(), offsets.numpy(), len(jpegs), self._max_image_dim,
                                         raw_mask=rm)
            raw = torch.from_numpy(rm).pin_memory()
        ds = int(self._spec.decode_size)
        shapes = {resize_shorter_size(int(w), int(h), ds) if st == 0 else (ds, ds)
                  for st, w, h, _ in info.tolist()}
        if len(shapes) != 1:  # the reference's torch.stack raises on unequal shapes
            raise RuntimeError(f"stack expects each tensor to be equal size, got resized shapes {sorted(shapes)}")
        ow, oh = shapes.pop()
        aws = 0
        for st, w, h, _ in info.tolist():
            if st == 0:
                kh = 2 * (-(-2 * w // ow)) + 3
                kv = 2 * (-(-2 * h // oh)) + 3
                aws += ow * (2 + kh) * 4 + oh * (2 + kv) * 4 + h * ow * 3 + 64
        self._engine.reserve(ws, aws)
        eng = self._engine
        d_bytes = host_buf.to(self.device, non_blocking=True)
        d_off = offsets.to(self.device, non_blocking=True)
        d_raw = raw.to(self.device, non_blocking=True) if raw is not None else None
        if self._norm is not None:
            self._norm_dev = torch.from_numpy(self._norm.batch_records(len(jpegs))).to(self.device)
            eng.set_norm(self._norm_dev)
        d_info = eng.decode(d_bytes, d_off, len(jpegs), raw_mask=d_raw)
        out = eng.resize_batch(ow, oh, self._spec.mean, self._spec.std, self._out)
        eng.batch_info(d_info)
        self._inflight = (host_buf, d_bytes, d_off, d_raw)
        probe_ok = info[:, 0] == 0
        if (ow, oh) != (ds, ds) and probe_ok.any():
            # an image that probes fine but fails on the device (damaged entropy data) is the
            # reference's (ds, ds) zero tensor, which its torch.stack refuses next to (ow, oh):
            # only then does the batch need its device status before returning
            st = d_info[:, 0].cpu().numpy()
            if ((st != 0) & probe_ok).any():
                raise RuntimeError(f"stack expects each tensor to be equal size, got resized shapes "
                                   f"{sorted({(ow, oh), (ds, ds)})}")
            self._fold_status(st)
        else:  # shapes cannot disagree: the status is read back asynchronously
            host = torch.empty(d_info.shape, dtype=d_info.dtype, pin_memory=True)
            host.copy_(d_info, non_blocking=True)
            ev = torch.cuda.Event()
            ev.record()
            self._pending_status.append((host, ev))
            self._drain_status()
        return self._spec.aug_fn(out)

    def close(self) -> None:
        if not self._closed:
            self._closed = True
            self._drain_status(block=True)
            self._engine.close()

    def __del__(self):
        try:
            self.close()
        except Exception:  # noqa: BLE001
            pass


class MI355XUserAugIterator:
    """The DALIBackend's ``_UserAugIterator`` contract (dali_backend.py:27-56): ``next()`` ->
    ``[aug_fn(decoded)]``, with a ValueError when a view of ``output_map`` is missing."""

    def __init__(self, pipeline: MI355XUserAugPipeline, output_map: list[str]) -> None:
        self._pipe = pipeline
        self._map = list(output_map)

    def __iter__(self):
        return self

    def __next__(self) -> list[dict[str, torch.Tensor]]:
        augmented = self._pipe.run_one_batch()
        missing = [k for k in self._map if k not in augmented]
        if missing:
            raise ValueError(f"UserAugSpec.aug_fn did not return expected view(s): {missing}. "
                             f"Got keys: {list(augmented.keys())}")
        return [augmented]

    def reset(self) -> None:
        """Stateless between batches."""
