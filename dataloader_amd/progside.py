"""Progressive / multi-scan JPEGs decoded ahead of their batch, on the device.

``k_prog`` (the coefficient-buffer decoder) runs one wave per image with the scans of a
dependency level on its lanes; an AC-refinement scan is inherently serial (how many
correction bits a symbol carries depends on which coefficients of *its* block earlier
scans made non-zero), so one image takes ~15-100 ms of latency (``scripts/prog_phases.py``)
while a whole baseline batch takes ~3.4 ms.  Decoded inside its batch, a single
progressive image stalls the pipeline (the "progressive cliff").

The side path takes that latency off the batch.  When a batch is prepared — up to
``side_ahead`` batches before its launch (the reference's own prefetch queue,
pipeline.py:317) — its progressive images join a pending pool; the pool is decoded as one
mini-batch (one ``k_prog`` wave per image, all concurrent) once it holds ``min_images``
images or a batch that needs it is about to launch, by one of a few side contexts on
their own HIP streams.  Each image's RGB is copied into a device buffer in the raw
container layout (``DINO_RAW_MAGIC`` header + HWC bytes).  At launch the batch's input
points those images at their containers (spans ABI, raw mask) and its stream waits for
the side decode's event, so the batch's own kernels treat them like any other decoded
image.  Same decoder, same bytes: the views are bit-identical to the in-batch device
route (``tests/test_gpu_round3.py``).
"""

from __future__ import annotations

import ctypes
import queue
import threading
import time
import weakref

import numpy as np
import torch

from . import _lib, fallback
from .engine import IngestEngine
from .tario import gather


class SideJob:
    """One batch's share of the side path: device containers by batch index, ready after
    ``event`` (None until the pool holding its images is launched)."""

    __slots__ = ("containers", "event", "status", "rows", "pending", "launched", "error", "t_add", "t_launch",
                 "owner", "room", "room_ready")

    def __init__(self, room: dict | None = None, room_ready: torch.cuda.Event | None = None):
        self.room = room or {}                    # batch index -> (device buffer, offset): where its
        self.room_ready = room_ready              # container goes in the batch's own input buffer
        self.containers: dict = {}
        self.event: torch.cuda.Event | None = None
        self.status: torch.Tensor | None = None   # pinned int32[n][4] of the mini-batch
        self.rows: dict = {}                      # batch index -> mini-batch row
        self.pending = True                       # still in the pool (not handed to the launcher)
        self.launched = threading.Event()         # the launcher thread has enqueued its decode
        self.error: BaseException | None = None
        self.t_add = time.perf_counter()          # host clock: joined the pool / its decode enqueued
        self.t_launch = 0.0
        self.owner = None                         # the DeviceSideDecoder (lead-time statistics)

    def done(self) -> bool:
        """Its side decode has been launched and has finished (ready() would not wait)."""
        return self.launched.is_set() and (self.event is None or self.event.query())

    def ready(self) -> dict:
        """The containers of images the side decode finished (waits for its launch and for
        the decode; normally long done).  An image the device decoder failed on is left out:
        its batch decodes it again and reaches the same outcome (zero-filled views where
        Pillow raises)."""
        t0 = time.perf_counter()
        if self.pending and self.owner is not None:  # still in the pool: hand it to the launcher now
            self.owner.flush()
        self.launched.wait()
        if self.error is not None:
            raise RuntimeError("side decode launch failed") from self.error
        if self.event is None:
            return {}
        self.event.synchronize()
        if self.owner is not None:
            lt = self.owner.lead
            lt["jobs"] += 1
            lt["wait_s"] += time.perf_counter() - t0
            lt["since_add_s"] += t0 - self.t_add
            lt["since_launch_s"] += t0 - self.t_launch
        st = self.status.numpy()[:, 0]
        return {i: c for i, c in self.containers.items() if st[self.rows[i]] == 0}


class _RawStream:
    """A HIP stream torch never sees: only the library's launches run on it (``cuda_stream`` is
    all ``IngestEngine`` reads).  torch must not record anything on it (an ExternalStream
    would let the caching allocators record free-time events on it, so destroying it
    would leave them a dangling stream: the segfault at close, gpurun_out/ss2.err)."""

    __slots__ = ("cuda_stream", "device")

    def __init__(self, handle: int, device: int):
        self.cuda_stream = handle
        self.device = device


_LIVE_STREAMS = {"created": 0, "destroyed": 0}


def live_streams() -> int:
    """Dedicated side streams created and not yet destroyed (0 once every side decoder closed)."""
    return _LIVE_STREAMS["created"] - _LIVE_STREAMS["destroyed"]


def _create_stream(device: int, cu_count: int) -> _RawStream:
    h = ctypes.c_void_p()
    _lib.check(_lib.load().dino_stream_create(device, cu_count, ctypes.byref(h)), "dino_stream_create")
    _LIVE_STREAMS["created"] += 1
    return _RawStream(h.value, device)


class _SideEngine:
    """One side context on a stream with its own hardware queue (``dino_stream_create``):
    a side decode runs for milliseconds, and on a queue shared with a batch stream the
    batch's kernels would wait behind it (measured: pools of >= 32 images on shared
    queues fell to 2.4k img/s, profiles/r03_route_study.jsonl).  ``cu_count`` > 0 confines
    the side decode to that many CUs.

    Only the library's kernels run on the dedicated stream: every torch allocation, copy
    and scatter of a side launch runs on this context's torch stream ``copy``, ordered with
    the dedicated stream by events both ways, so the stream is destroyed at ``close``.
    Consecutive launches of a context are ordered by the dedicated stream itself."""

    def __init__(self, device: torch.device, max_images: int, max_image_dim: int, cu_count: int = 0,
                 dedicated: bool = True, index: int = 0, stream_set: int = 0, lanes: bool = False):
        from .pipeline import role_stream
        self.raw = _create_stream(device.index or 0, int(cu_count)) if dedicated else None
        self.stream = self.raw if dedicated else role_stream(device, "side", index, stream_set)
        self.eng = IngestEngine(device, max_batch=max_images, max_views=1, max_crop_size=8,
                                max_image_dim=max_image_dim, workspace_bytes=64 << 20, stream=self.stream)
        self.eng.set_prog_decoder(lanes)
        self.copy = role_stream(device, "side_copy", index, stream_set)  # this context's torch stream (allocations, copies)
        self.last: torch.cuda.Event | None = None   # the engine's workspace is free once this completes
        self.keep = None                             # host / device inputs of the mini-batch in flight
        self.hbuf: torch.Tensor | None = None        # pinned pack buffer, reused once `last` completes

    def idle(self) -> bool:
        return self.last is None or self.last.query()

    def close(self) -> None:
        if self.last is not None:
            self.last.synchronize()
        self.keep = None
        self.eng.close()
        if self.raw is not None:
            _lib.check(_lib.load().dino_stream_destroy(ctypes.c_void_p(self.raw.cuda_stream)), "dino_stream_destroy")
            _LIVE_STREAMS["destroyed"] += 1
            self.raw = None


# Side decoder plan by look-ahead (c2_prog: B = 512 C2 batches, one image in 16 progressive;
# RESULTS.md round 6, profiles/r06_side_plan/).  The wave decoder (k_pscan) finishes a pool
# sooner but costs the batches more GPU time per image; the lane decoder (k_plscan) costs
# little per image and its launch time barely grows with the pool (one 64-image group per
# wave), but a launch takes ~250-450 ms under a running pipeline.  So with a look-ahead
# that can hold two pools of 4096 images decoding at once (>= LANES_MIN_AHEAD batches) the
# lane decoder on large pools wins (lane, look-ahead 256, pools of 4096: 89-112k img/s;
# wave, look-ahead 48, pools of 512: 72k; wave, look-ahead 256, pools of 2048: 77k); a
# shorter look-ahead (a source whose metadata FIFO caps it, backend.side_look_ahead) keeps
# the wave decoder on pools of 512.
LANES_MIN_AHEAD = 128
LANE_POOL = 4096
WAVE_POOL = 512
# A pool flushed before it filled (the look-ahead ran short: the host half fell behind the
# batches) goes to the wave decoder when it is smaller than this: a lane-decoder launch takes
# ~120 ms even for a few images, and small lane pools launched back to back starved the
# batches (c2_prog 50k img/s with pools of 32-500 images, profiles/r06_side_plan/r6n).
LANE_MIN_POOL = 1024


def side_plan(side_ahead: int) -> tuple[bool, int]:
    """(lane decoder?, pool size in images) for a side look-ahead of ``side_ahead`` batches;
    ``DINO_SIDE_DECODER=wave|lanes`` and ``DINO_SIDE_MAX`` override."""
    import os
    want = os.environ.get("DINO_SIDE_DECODER", "")
    lanes = want == "lanes" if want in ("wave", "lanes") else int(side_ahead) >= LANES_MIN_AHEAD
    return lanes, int(os.environ.get("DINO_SIDE_MAX", LANE_POOL if lanes else WAVE_POOL))


class DeviceSideDecoder:
    """Pending pool + ``engines`` side contexts (created on demand).  ``add`` queues a
    batch's images and hands the pool to the launcher once it holds ``min_images``;
    ``flush`` hands it over now (a batch holding pending images is about to launch).
    The launches (pack, probe, H2D, the decode and container copies, ~30 ms of host time
    for a pool of 512 images, and the wait for a free context when every one still has a
    mini-batch in flight) run on a launcher thread of their own: on the pipeline's launch
    thread they cost the c2_prog leg ~3 ms per batch (``scripts/prof_leg.py``)."""

    def __init__(self, device: torch.device, max_images: int = WAVE_POOL, min_images: int | None = None,
                 engines: int | None = None, max_image_dim: int = 0, stream_set: int = 0, lanes: bool = False):
        import os
        # measured (scripts/route_study.py, 16 progressive per 256-image batch, dedicated queues,
        # look-ahead 64, profiles/r03_side_pools.jsonl): pools of 16 images on 2 contexts 11.2k img/s,
        # 64: 37.7k, 128: 53.2k, 256: 66.5k, 512: 74.3k.  One k_pscan launch of N progressive images
        # takes ~30 ms up to N = 64 and 45 ms at N = 512 (scripts/prog_scale.py), so the pool waits
        # for max_images, or until its oldest batch is half the look-ahead from its launch (pipeline.py)
        max_images = int(os.environ.get("DINO_SIDE_MAX", max_images))
        min_images = int(os.environ.get("DINO_SIDE_MIN", max_images)) if min_images is None else min_images
        engines = int(os.environ.get("DINO_SIDE_ENGINES", 2)) if engines is None else engines
        self.cu_count = int(os.environ.get("DINO_SIDE_CUS", 0))
        self.timing = os.environ.get("DINO_SIDE_TIMING", "0") == "1"  # per-launch GPU spans (analysis)
        self.spans: list = []
        self.dedicated = os.environ.get("DINO_SIDE_DEDICATED", "1") != "0"
        self.device = device
        self.max_images = int(max_images)
        self.min_images = max(1, min(int(min_images), self.max_images))
        self.cap = max(1, int(engines))
        self.max_image_dim = int(max_image_dim)
        self.stream_set = int(stream_set)  # the owning pipeline's role streams (pipeline.acquire_stream_set)
        self.lanes = bool(lanes)           # the side contexts' decoder (side_plan)
        self.lane_min = int(os.environ.get("DINO_SIDE_LANE_MIN", LANE_MIN_POOL))  # smaller pools: wave decoder
        self._engines: list[_SideEngine] = []
        self._rr = 0
        self._pool: list = []   # (job, batch index, JPEG bytes)
        self.launches = 0
        self.lane_launches = 0  # launches the lane decoder took (the rest: the wave decoder)
        self.images = 0
        self.host_seconds = 0.0   # spent in _launch (pack, probe, launches; waits for a free context)
        self.phase_seconds = {"engine": 0.0, "pack": 0.0, "probe": 0.0, "decode": 0.0, "containers": 0.0}
        # per batch handed out: waits in ready(), time since its images joined the pool and
        # since their decode was enqueued (host clock)
        self.lead = {"jobs": 0, "wait_s": 0.0, "since_add_s": 0.0, "since_launch_s": 0.0}
        # add (the prefetch thread) and flush (also the launch thread, for a batch about to launch)
        self._lock = threading.RLock()
        self._parts: "queue.Queue" = queue.Queue()   # pools handed to the launcher thread
        # the thread holds only a weak reference: a decoder nobody closes can still be collected
        self._launcher = threading.Thread(target=_launcher_loop, args=(weakref.ref(self), self._parts),
                                          name="dino-side-launcher", daemon=True)
        self._launcher.start()

    def __del__(self):
        if getattr(self, "_parts", None) is not None:
            self._parts.put(None)

    def add(self, imgs: dict, room: dict | None = None, room_ready=None) -> SideJob | None:
        """Queue a batch's images (batch index -> JPEG bytes).  ``room``: batch index -> (device
        tensor, offset) of space reserved for the image's container in the batch's own input
        buffer, usable once ``room_ready`` has completed; the others get containers of their own."""
        if not imgs:
            return None
        job = SideJob(room, room_ready)
        job.owner = self
        with self._lock:
            for i in sorted(imgs):
                self._pool.append((job, int(i), imgs[i]))
            if len(self._pool) >= self.min_images:
                self.flush()
        return job

    def _engine(self) -> _SideEngine:
        for e in self._engines:
            if e.idle():
                return e
        if len(self._engines) < self.cap:
            e = _SideEngine(self.device, self.max_images, self.max_image_dim, self.cu_count, self.dedicated,
                            index=len(self._engines), stream_set=self.stream_set, lanes=self.lanes)
            self._engines.append(e)
            return e
        e = self._engines[self._rr % len(self._engines)]
        self._rr += 1
        e.last.synchronize()
        return e

    def flush(self) -> None:
        """Hand the pending pool to the launcher now (in mini-batches of at most
        ``max_images``); returns at once."""
        with self._lock:
            while self._pool:
                part, self._pool = self._pool[: self.max_images], self._pool[self.max_images:]
                for job, _, _ in part:
                    job.pending = False
                self._parts.put(part)

    def _run_part(self, part: list) -> None:
        try:
            with torch.cuda.device(self.device):
                self._launch(part)
        except BaseException as e:  # noqa: BLE001 -- the batches waiting on it re-raise
            for job, _, _ in part:
                job.error = e
        finally:
            for job, _, _ in part:
                job.launched.set()

    def _launch(self, part: list) -> None:
        t_start = time.perf_counter()
        ph = self.phase_seconds
        se = self._engine()
        t1 = time.perf_counter()
        ph["engine"] += t1 - t_start
        eng = se.eng
        lanes = self.lanes and len(part) >= self.lane_min
        if eng.prog_lanes != lanes:
            eng.set_prog_decoder(lanes)
        self.lane_launches += int(lanes)
        items = [j for _, _, j in part]
        # the pool's bytes go into this context's own pinned buffer (reused: the context is idle,
        # so its last upload has completed) by the native gather's threads (no GIL): a fresh
        # pinned buffer per pool (pack_jpegs) cost a pinned allocation of the pool's size
        # (~350 MB for 4096 C2 images) and a Python-loop copy on this thread
        total = sum(len(j) for j in items)
        if se.hbuf is None or se.hbuf.numel() < total + 16:
            se.hbuf = torch.empty(total * 5 // 4 + 4096, dtype=torch.uint8, pin_memory=True)
        hb = se.hbuf
        off = torch.from_numpy(gather(items, hb, 4))
        t2 = time.perf_counter()
        ph["pack"] += t2 - t1
        info, ws, _ = fallback.probe(hb.data_ptr(), off.numpy(), len(items), self.max_image_dim)
        t3 = time.perf_counter()
        ph["probe"] += t3 - t2
        eng.reserve(ws, 0)
        heads = []
        cs = se.copy
        es = torch.cuda.ExternalStream(se.stream.cuda_stream, device=self.device) if se.raw is not None \
            else se.stream  # (only to enqueue event waits / records: torch never allocates on it)
        for k, (job, i, _) in enumerate(part):
            job.rows[i] = k
        keep = [(k, job, i, int(info[k, 1]), int(info[k, 2])) for k, (job, i, _) in enumerate(part)
                if int(info[k, 0]) == 0 and int(info[k, 3]) != 2]
        with torch.cuda.stream(cs):
            if self.timing:
                t0 = torch.cuda.Event(enable_timing=True)
                t0.record(es)
            d_bytes = hb[:max(total, 1) + 16].to(self.device, non_blocking=True)
            d_off = off.to(self.device, non_blocking=True)
            d_info = torch.empty((len(items), 4), dtype=torch.int32, device=self.device)
            # every decoded image's container: the room reserved for it in its batch's input
            # buffer when the batch has some (_stage_on_device), else a 16-byte aligned slice of
            # one pool buffer; one dino_copy_rgb_packed launch writes all their headers and pixels
            # at absolute addresses
            big = d_idx = d_dst = None
            if keep:
                own = [(job, i) for _, job, i, _, _ in keep if i not in job.room]
                sizes = {(id(job), i): (16 + w * h * 3 + 15) & ~15 for _, job, i, w, h in keep}
                if own:
                    big = torch.empty(sum(sizes[(id(j), i)] for j, i in own), dtype=torch.uint8, device=self.device)
                dst, conts, o = [], [], 0
                for k, job, i, w, h in keep:
                    if i in job.room:
                        buf, pos = job.room[i]
                        c = buf[pos:pos + 16 + w * h * 3]
                    else:
                        c = big[o:o + 16 + w * h * 3]
                        o += sizes[(id(job), i)]
                    conts.append(c)
                    dst.append(c.data_ptr() + 16)
                h_idx = torch.from_numpy(np.array([k for k, _, _, _, _ in keep], np.int32)).pin_memory()
                h_dst = torch.from_numpy(np.array(dst, np.int64)).pin_memory()
                heads.extend((h_idx, h_dst))
                d_idx = h_idx.to(self.device, non_blocking=True)
                d_dst = h_dst.to(self.device, non_blocking=True)
            # the library's kernels on the dedicated stream, after the inputs (and after any
            # earlier use of the memory the allocator just handed out, on this torch stream)
            ready = torch.cuda.Event()
            ready.record(cs)
            es.wait_event(ready)
            eng.decode(d_bytes, d_off, len(items), info=d_info)
            t4 = time.perf_counter()
            ph["decode"] += t4 - t3
            if keep:
                waited = set()
                for _, job, i, _, _ in keep:  # the batches' input buffers hold their bytes (and are ours)
                    if i in job.room and job.room_ready is not None and id(job) not in waited:
                        es.wait_event(job.room_ready)
                        waited.add(id(job))
                _lib.check(eng.lib.dino_copy_rgb_packed(eng._ctx, len(keep), ctypes.c_void_p(d_idx.data_ptr()),
                                                        ctypes.c_void_p(d_dst.data_ptr()), None, _lib.COPY_HEADER,
                                                        eng._s()), "dino_copy_rgb_packed")
                for (k, job, i, w, h), c in zip(keep, conts):
                    job.containers[i] = c
            # the status copy and the completion event on the decode's own stream: a torch stream
            # made to wait for the decode would hold its hardware queue (shared with other
            # streams, GPU_MAX_HW_QUEUES) for the whole decode -- the batches' H2D copies
            # queued behind it, their staging buffers stayed busy and the host half stalled
            # (c2_prog: 3.3 ms per batch waiting for staging)
            status = torch.empty((len(items), 4), dtype=torch.int32, pin_memory=True)
            with torch.cuda.stream(es):
                status.copy_(d_info, non_blocking=True)
            ph["containers"] += time.perf_counter() - t4
            ev = torch.cuda.Event(enable_timing=self.timing)
            ev.record(es)
            if self.timing:
                self.spans.append((t0, ev, len(part)))
        t_end = time.perf_counter()
        for job, _, _ in part:
            job.event, job.status, job.t_launch = ev, status, t_end
        se.last = ev
        se.keep = (hb, off, d_bytes, d_off, heads, d_info, big, d_idx, d_dst)
        self.launches += 1
        self.images += len(part)
        self.host_seconds += time.perf_counter() - t_start

    def launch_ms(self) -> list:
        """(GPU ms, images) of every timed launch (DINO_SIDE_TIMING=1)."""
        out = []
        for a, b, n in self.spans:
            b.synchronize()
            out.append((round(a.elapsed_time(b), 2), n))
        return out

    def close(self) -> None:
        with self._lock:  # jobs never handed to the launcher fail instead of waiting forever
            closed = RuntimeError("DeviceSideDecoder closed before the side decode was launched")
            for job, _, _ in self._pool:
                job.pending = False
                job.error = closed
                job.launched.set()
            self._pool.clear()
        if self._launcher.is_alive():  # the launcher finishes the parts queued before the sentinel
            self._parts.put(None)
            self._launcher.join()
        if self.timing:
            import sys
            print("side launches (ms, images):", self.launch_ms(), file=sys.stderr)
        with self._lock:
            for e in self._engines:
                e.close()
            self._engines.clear()


def _launcher_loop(ref, parts: "queue.Queue") -> None:
    """The side decoder's launcher thread: runs the pools handed over by ``flush`` until the
    sentinel, or until its decoder is gone."""
    while True:
        part = parts.get()
        dec = ref() if part is not None else None
        if dec is None:
            if part is not None:  # the decoder was collected with a pool queued: fail its jobs
                for job, _, _ in part:
                    job.error = RuntimeError("DeviceSideDecoder collected before the side decode was launched")
                    job.launched.set()
            return
        dec._run_part(part)
        del dec


def side_mask(info: np.ndarray) -> np.ndarray:
    """Images of a probed batch the side path takes: decodable coefficient-buffer images
    (``info[:, 3] == 1``: progressive, multi-scan sequential, damaged restart intervals)."""
    return (info[:, 0] == 0) & (info[:, 3] == 1)
