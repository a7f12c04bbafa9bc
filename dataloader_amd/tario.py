"""Host-side shard ingest: /dev/shm shard cache → native tar index → pinned batch.

This is the feed of the Stage-3 device path:

* :class:`ShmShardCache` — the read path of the reference's node-local
  ``NodeSharedShardCache`` (``shard_cache.py:476-712``): one file per shard in
  ``/dev/shm/<job_id>/<sha1(path)[:16]>`` laid out as ``[data_len:u64][magic:u64]``
  + tar bytes, magic ``0xDEADBEEFCAFEF00D`` written last (``:83-85, :689-703``),
  mmapped zero-copy (``get_view``, ``:584-609``).  The node master loads missing
  shards (``prefetch``: in the background, at most ``prefetch_window`` at once) and
  evicts LRU files over budget; the other ranks wait for its writes (inotify,
  ``:373-449``).  The heartbeat, orphan purge and signal handlers of the reference
  are control plane (out of scope).
* :func:`index_tar` — ``dino_tar_index`` (C++, ``csrc/tario.cpp``) over a mapped
  shard: WebDataset samples (key, .jpg range, .json range) without Python
  per-member work.
* :func:`extract_jpegs_with_meta` — the reference's extraction call
  (``hpc_source.py:461-467`` → the absent ``dino_datasets`` helper
  ``_extract_jpegs_with_meta``) restated on the native index: ``SampleRecord``s with
  JSON metadata, optional quality filter and shuffle buffer.  The helper itself is
  not in ``/root/reference``; its semantics here are restated from its call site
  (parity unpinned beyond the reference's fixture tars).
* :class:`ShardBatchFeeder` — B JPEGs per batch from mapped shards: either where
  they lie (page-locked shard ranges DMA'd to HBM as they are, decoded through the
  spans ABI: no host copy), or packed by ``dino_gather`` (threaded memcpy) into a
  pinned buffer + int64 offsets, the layout ``dino_run_batch`` reads after one H2D
  copy.
"""

from __future__ import annotations

import contextlib
import ctypes
import hashlib
import json
import mmap
import os
import struct
import threading
from collections import OrderedDict
from dataclasses import dataclass
from pathlib import Path
from typing import Any, Iterator, Sequence

import numpy as np

from . import _lib

HDR_FMT = "QQ"
HDR_SIZE = struct.calcsize(HDR_FMT)
READY_MAGIC = 0xDEAD_BEEF_CAFE_F00D
TAR_TRUNCATED, TAR_BAD_HEADER = 1, 2


class DinoTarSample(ctypes.Structure):
    _fields_ = [("img_off", ctypes.c_int64), ("img_len", ctypes.c_int64), ("meta_off", ctypes.c_int64),
                ("meta_len", ctypes.c_int64), ("key_off", ctypes.c_int64), ("key_len", ctypes.c_int32),
                ("reserved", ctypes.c_int32)]


SAMPLE_DTYPE = np.dtype([("img_off", "<i8"), ("img_len", "<i8"), ("meta_off", "<i8"), ("meta_len", "<i8"),
                         ("key_off", "<i8"), ("key_len", "<i4"), ("reserved", "<i4")])
assert SAMPLE_DTYPE.itemsize == ctypes.sizeof(DinoTarSample)


class SampleRecord:
    """Same contract as reference ``augmentation.SampleRecord`` (augmentation.py:67-90)."""

    __slots__ = ("jpeg", "key", "metadata")

    def __init__(self, jpeg, metadata: dict | None = None, key: str = "") -> None:
        self.jpeg = jpeg
        self.metadata = metadata
        self.key = key


def _addr(buf) -> tuple[int, int, Any]:
    """(address, length, keep-alive) of a bytes-like object without copying it."""
    if isinstance(buf, np.ndarray):
        a = np.ascontiguousarray(buf).view(np.uint8).reshape(-1)
        return a.ctypes.data, a.size, a
    if isinstance(buf, (bytes, bytearray, memoryview, mmap.mmap)):
        a = np.frombuffer(buf, dtype=np.uint8)
        return (a.ctypes.data if a.size else 0), a.size, a
    raise TypeError(f"unsupported buffer type {type(buf).__name__}")


@dataclass
class TarIndex:
    """Samples of one shard: byte ranges into the indexed buffer, keys, status."""

    samples: np.ndarray   # SAMPLE_DTYPE[n]
    keys: list[str]
    n_members: int
    status: int           # 0 ok, 1 truncated member, 2 bad header after offset 0

    def __len__(self) -> int:
        return len(self.samples)


def index_tar(buf) -> TarIndex:
    """Index a WebDataset tar held in memory (``dino_tar_index``)."""
    lib = _lib.load()
    addr, n, keep = _addr(buf)
    cap = max(16, n // 1024 + 16)           # a member takes >= 1024 bytes (header + data block)
    out = np.zeros(cap, SAMPLE_DTYPE)
    keys = np.zeros(max(256, cap * 64), np.uint8)
    ns, nm = ctypes.c_int64(), ctypes.c_int64()
    rc = lib.dino_tar_index(ctypes.c_void_p(addr), n, ctypes.c_void_p(out.ctypes.data), cap,
                            ctypes.c_void_p(keys.ctypes.data), keys.size, ctypes.byref(ns), ctypes.byref(nm))
    del keep
    return _index_result(lib, rc, out, keys, ns, nm)


def index_tar_fd(fd: int, base: int, length: int) -> TarIndex:
    """Index the tar bytes [base, base + length) of an open file by reading only its headers
    (``dino_tar_index_fd``: pread, the members' data is never read); offsets are relative to
    ``base``, as ``index_tar`` of those bytes reports them."""
    lib = _lib.load()
    cap = max(16, int(length) // 1024 + 16)
    out = np.zeros(cap, SAMPLE_DTYPE)
    keys = np.zeros(max(256, cap * 64), np.uint8)
    ns, nm = ctypes.c_int64(), ctypes.c_int64()
    rc = lib.dino_tar_index_fd(int(fd), int(base), int(length), ctypes.c_void_p(out.ctypes.data), cap,
                               ctypes.c_void_p(keys.ctypes.data), keys.size, ctypes.byref(ns), ctypes.byref(nm))
    return _index_result(lib, rc, out, keys, ns, nm)


def _index_result(lib, rc, out, keys, ns, nm) -> TarIndex:
    if rc < 0:
        raise _lib.DinoError(f"dino_tar_index failed ({rc}): {lib.dino_tar_last_error().decode(errors='replace')}")
    s = out[:ns.value].copy()
    kb = keys.tobytes()
    names = [kb[o:o + ln].decode("utf-8", errors="surrogateescape") if o >= 0 else "" for o, ln in
             zip(s["key_off"].tolist(), s["key_len"].tolist())]
    return TarIndex(s, names, int(nm.value), int(rc))


def extract_jpegs_with_meta(data, metadata_key: str | None = None, min_quality: float | None = None,
                            shuffle_buffer: int = 0, rng: np.random.Generator | None = None,
                            copy: bool = False) -> list[SampleRecord]:
    """Samples of one shard as ``SampleRecord`` (reference call site hpc_source.py:461-467).

    ``jpeg`` is a zero-copy ``memoryview`` into ``data`` unless ``copy``;
    ``metadata`` the parsed JSON sidecar (``metadata[metadata_key]`` when a key is
    given and present); samples whose ``quality_score`` is below ``min_quality``
    are dropped; ``shuffle_buffer > 1`` permutes the shard's samples with ``rng``.
    """
    idx = index_tar(data)
    mv = memoryview(data) if not isinstance(data, np.ndarray) else memoryview(np.ascontiguousarray(data))
    mv = mv.cast("B") if mv.format != "B" else mv
    recs: list[SampleRecord] = []
    for row, key in zip(idx.samples, idx.keys):
        meta = None
        if row["meta_off"] >= 0:
            try:
                meta = json.loads(bytes(mv[row["meta_off"]:row["meta_off"] + row["meta_len"]]))
            except (ValueError, UnicodeDecodeError):
                meta = None
        if metadata_key is not None and isinstance(meta, dict) and metadata_key in meta:
            meta = meta[metadata_key]
        if min_quality is not None and isinstance(meta, dict):
            q = meta.get("quality_score")
            if q is not None and q < min_quality:
                continue
        j = mv[row["img_off"]:row["img_off"] + row["img_len"]]
        recs.append(SampleRecord(bytes(j) if copy else j, meta, key))
    if shuffle_buffer > 1 and len(recs) > 1:
        rng = rng if rng is not None else np.random.default_rng()
        recs = [recs[i] for i in rng.permutation(len(recs))]
    return recs


def spans_of(srcs: Sequence) -> tuple[np.ndarray, np.ndarray, list]:
    """(uint64 addresses, int64 lengths, keep-alive list) of a sequence of (address, length)
    pairs or bytes-like objects."""
    keep = []
    n = len(srcs)
    ptrs = np.empty(n, np.uint64)
    lens = np.empty(n, np.int64)
    if n and isinstance(srcs[0], tuple):
        a = np.asarray(srcs, dtype=np.int64).reshape(n, 2)
        ptrs[:] = a[:, 0].astype(np.uint64)
        lens[:] = a[:, 1]
        return ptrs, lens, keep
    for i, s in enumerate(srcs):
        if isinstance(s, tuple):
            ptrs[i], lens[i] = s
        else:
            a, ln, k = _addr(s)
            keep.append(k)
            ptrs[i], lens[i] = a, ln
    return ptrs, lens, keep


def gather(srcs: Sequence, dst: "Any", nthreads: int = 8) -> np.ndarray:
    """Pack byte ranges back to back into ``dst`` (pinned torch uint8 tensor or ndarray).

    ``srcs``: sequence of (address, length) pairs or bytes-like objects.
    Returns int64 offsets[n+1] (``dino_gather``)."""
    lib = _lib.load()
    ptrs, lens, keep = spans_of(srcs)
    off = np.empty(len(srcs) + 1, np.int64)
    if hasattr(dst, "data_ptr"):
        daddr, dcap = dst.data_ptr(), dst.numel() * dst.element_size()
    else:
        daddr, dcap, _ = _addr(dst)
    rc = lib.dino_gather(ctypes.c_void_p(ptrs.ctypes.data), ctypes.c_void_p(lens.ctypes.data), len(srcs),
                         ctypes.c_void_p(daddr), dcap, ctypes.c_void_p(off.ctypes.data), nthreads)
    del keep
    if rc != 0:
        raise _lib.DinoError(f"dino_gather failed ({rc}): {lib.dino_tar_last_error().decode(errors='replace')}")
    return off


# ---------------------------------------------------------------------------
# /dev/shm shard cache (read path of reference NodeSharedShardCache)
# ---------------------------------------------------------------------------
class _Mapped:
    __slots__ = ("fd", "mm", "data_len", "refs", "arr")

    def __init__(self, path: Path) -> None:
        self.fd = os.open(str(path), os.O_RDONLY)
        try:
            self.mm = mmap.mmap(self.fd, 0, access=mmap.ACCESS_READ)
        except Exception:
            os.close(self.fd)
            raise
        data_len, magic = struct.unpack_from(HDR_FMT, self.mm, 0)
        if magic != READY_MAGIC:
            self.close()
            raise RuntimeError(f"Shard {path} has corrupt header (magic={magic:#x})")
        self.data_len = int(data_len)
        self.refs = 0
        self.arr = np.frombuffer(self.mm, np.uint8, count=self.data_len, offset=HDR_SIZE)

    def close(self) -> None:
        self.arr = None
        with contextlib.suppress(Exception):
            self.mm.close()
        with contextlib.suppress(Exception):
            os.close(self.fd)


def shm_path(base: Path, shard_path: str) -> Path:
    """``/dev/shm/<job>/<sha1(shard_path)[:16]>`` (reference shard_cache.py:619-622)."""
    return base / hashlib.sha1(shard_path.encode()).hexdigest()[:16]


def write_shm_shard(shm: Path, data) -> None:
    """Atomic shard write: header with magic 0, data, then the ready magic, rename
    (reference shard_cache.py:689-703)."""
    tmp = shm.with_suffix(".tmp")
    try:
        with open(tmp, "wb") as f:
            n = len(data) if not isinstance(data, np.ndarray) else data.nbytes
            f.write(struct.pack(HDR_FMT, n, 0))
            f.write(data)
            f.seek(0)
            f.write(struct.pack(HDR_FMT, n, READY_MAGIC))
        tmp.rename(shm)
    except Exception:
        with contextlib.suppress(Exception):
            tmp.unlink()
        raise


def is_ready(shm: Path) -> bool:
    """The file exists and carries the ready magic (reference ``_is_ready``, shard_cache.py:331-340)."""
    try:
        with open(shm, "rb") as f:
            hdr = f.read(HDR_SIZE)
        return len(hdr) == HDR_SIZE and struct.unpack(HDR_FMT, hdr)[1] == READY_MAGIC
    except OSError:
        return False


_IN_CLOSE_WRITE, _IN_MOVED_TO, _IN_NONBLOCK, _IN_CLOEXEC = 0x8, 0x80, 0o4000, 0o2000000


def wait_ready(shm: Path, timeout_s: float) -> None:
    """Block until the node master has written ``shm`` (reference ``_inotify_wait``,
    shard_cache.py:373-449): check, watch the cache directory for ``IN_CLOSE_WRITE |
    IN_MOVED_TO``, check again (closes the race with a rename between the first check and
    the watch), then wake on events; stat-polls every 50 ms where inotify is unavailable.
    Raises ``TimeoutError`` after ``timeout_s`` seconds, as the reference does."""
    import select
    import time
    shm = Path(shm)
    if is_ready(shm):
        return
    deadline = time.monotonic() + timeout_s
    ifd = wd = -1
    try:
        libc = ctypes.CDLL(None, use_errno=True)
        ifd = libc.inotify_init1(_IN_NONBLOCK | _IN_CLOEXEC)
        if ifd >= 0:
            wd = libc.inotify_add_watch(ifd, str(shm.parent).encode(), _IN_CLOSE_WRITE | _IN_MOVED_TO)
    except (OSError, AttributeError):
        ifd = wd = -1
    try:
        while not is_ready(shm):
            left = deadline - time.monotonic()
            if left <= 0:
                raise TimeoutError(f"Timed out ({timeout_s:.0f}s) waiting for shard: {shm}")
            if wd >= 0:
                r, _, _ = select.select([ifd], [], [], min(left, 1.0))
                if r:
                    with contextlib.suppress(OSError):
                        os.read(ifd, 4096)
            else:
                time.sleep(min(left, 0.05))
    finally:
        if wd >= 0:
            libc.inotify_rm_watch(ifd, wd)
        if ifd >= 0:
            os.close(ifd)


class ShmShardCache:
    """Node-local ``/dev/shm`` shard cache with zero-copy mapped reads.

    Same public surface as the reference cache (``prefetch``, ``get``, ``get_view``,
    ``utilisation``) plus ``get_array`` (a uint8 ndarray over the mapping, what
    :func:`index_tar` and :class:`ShardBatchFeeder` consume) and ``close``.
    """

    WARN_INTERVAL_S = 60.0  # reference _SHM_WARN_INTERVAL

    def __init__(self, job_id: str = "dino", node_master: bool = True, max_gb: float = 128.0,
                 base_dir: str | os.PathLike = "/dev/shm", max_mapped: int = 256,
                 shard_timeout_s: float = 300.0, prefetch_window: int = 4, warn_threshold: float = 0.85) -> None:
        self._base = Path(base_dir) / job_id
        self._base.mkdir(parents=True, exist_ok=True)
        self._node_master = node_master
        self.shard_timeout_s = float(shard_timeout_s)  # how long a non-master rank waits for a shard (reference :507)
        self._max_bytes = int(max_gb * (1 << 30))
        self._lru: OrderedDict[str, int] = OrderedDict()
        self._total = 0
        self._lock = threading.Lock()
        self._maps: OrderedDict[str, _Mapped] = OrderedDict()
        self._max_mapped = max_mapped
        # the node master's background loads (reference prefetch: at most prefetch_window
        # concurrent filesystem -> /dev/shm copies, shard_cache.py:548-559, 633)
        self._window = max(1, int(prefetch_window))
        self._pool = None
        self._in_flight: dict = {}
        self._warn_threshold = float(warn_threshold)
        self._last_warn = 0.0

    @property
    def base(self) -> Path:
        return self._base

    def _path(self, shard_path: str) -> Path:
        return shm_path(self._base, shard_path)

    @property
    def node_master(self) -> bool:
        return self._node_master

    def path_of(self, shard_path: str) -> Path:
        """The cache file of ``shard_path`` (it may not be written yet)."""
        return self._path(shard_path)

    def _ensure(self, shard_path: str) -> Path:
        """The ready cache file of ``shard_path``: the node master loads a missing shard; any
        other rank waits for the master's write (reference get_view, shard_cache.py:588-603)
        and raises ``TimeoutError`` after ``shard_timeout_s``."""
        shm = self._path(shard_path)
        if is_ready(shm):
            return shm
        if not self._node_master:
            wait_ready(shm, self.shard_timeout_s)
            return shm
        from concurrent.futures import Future
        with self._lock:
            fut = self._in_flight.get(shard_path)
            mine = fut is None and not is_ready(shm)
            if mine:  # a synchronous load registers like a background one: prefetch() and other
                fut = self._in_flight[shard_path] = Future()  # callers of this shard wait for it
        if fut is None:  # loaded between the first check and the lock
            return shm
        if not mine:  # a load of this shard is running: wait for it (reference get_view, :588-595)
            fut.result()
            return shm
        try:
            self._load(shard_path)
            fut.set_result(None)
        except BaseException as e:
            fut.set_exception(e)
            raise
        finally:
            with self._lock:
                self._in_flight.pop(shard_path, None)
        return shm

    def _load(self, shard_path: str) -> None:
        """Filesystem -> /dev/shm (node master; reference _load_one, shard_cache.py:624-688)."""
        with open(shard_path, "rb") as f:
            data = f.read()
        self.put(shard_path, data)

    def put(self, shard_path: str, data) -> Path:
        """Write shard bytes into the cache (node master), evicting LRU shards over budget.  A
        shard larger than the whole budget raises at once (reference [FIX-EVICT-EARLY], :648-655)."""
        n = len(data) if not isinstance(data, np.ndarray) else data.nbytes
        if n > self._max_bytes:
            raise RuntimeError(f"ShmShardCache: shard {shard_path!r} ({n >> 20} MB) exceeds the entire shm budget "
                               f"({self._max_bytes >> 30} GB). Increase node_shm_gb.")
        shm = self._path(shard_path)
        with self._lock:
            while self._lru and self._total + n > self._max_bytes:
                old, sz = self._lru.popitem(last=False)
                self._total -= sz
                self._drop(old)
        write_shm_shard(shm, data)
        with self._lock:
            self._total -= self._lru.pop(shard_path, 0)  # a rewrite replaces the size already counted
            self._lru[shard_path] = n
            self._total += n
        self._check_utilisation()
        return shm

    def _check_utilisation(self) -> None:
        """Warn (at most once a minute) when the cache is over ``warn_threshold`` of its budget
        (reference _update_utilisation_metric, shard_cache.py:738-753)."""
        import time
        import warnings
        util = self.utilisation
        now = time.monotonic()
        if util >= self._warn_threshold and now - self._last_warn >= self.WARN_INTERVAL_S:
            self._last_warn = now
            warnings.warn(f"/dev/shm utilisation is {util * 100:.1f}% (threshold {self._warn_threshold * 100:.0f}%). "
                          "Increase node_shm_gb or reduce shard_prefetch_window. Budget: "
                          f"{self._max_bytes / (1 << 30):.1f} GB, used: {self._total / (1 << 30):.1f} GB.",
                          RuntimeWarning, stacklevel=3)

    def _drop(self, shard_path: str) -> None:
        m = self._maps.get(shard_path)
        if m is not None and m.refs == 0:
            self._maps.pop(shard_path).close()
        with contextlib.suppress(OSError):
            self._path(shard_path).unlink()

    def prefetch(self, shard_path: str) -> None:
        """Schedule a shard for background loading (node master only; reference :548-559): at
        most ``prefetch_window`` loads run at once, a shard already cached or loading is skipped."""
        if not self._node_master:
            return
        if is_ready(self._path(shard_path)):
            return
        with self._lock:
            if shard_path in self._in_flight:
                return
            if self._pool is None:
                from concurrent.futures import ThreadPoolExecutor
                self._pool = ThreadPoolExecutor(max_workers=self._window, thread_name_prefix="shard-io")
            fut = self._pool.submit(self._load, shard_path)
            self._in_flight[shard_path] = fut

        def _done(_f, p=shard_path):
            with self._lock:
                self._in_flight.pop(p, None)
        fut.add_done_callback(_done)

    def _acquire(self, shard_path: str) -> _Mapped:
        shm = self._ensure(shard_path)
        with self._lock:
            m = self._maps.get(shard_path)
            if m is None:
                idle = [k for k, v in self._maps.items() if v.refs == 0]
                while idle and len(self._maps) >= self._max_mapped:
                    self._maps.pop(idle.pop(0)).close()
                m = _Mapped(shm)
                self._maps[shard_path] = m
            self._maps.move_to_end(shard_path)
            m.refs += 1
            if shard_path in self._lru:
                self._lru.move_to_end(shard_path)
            return m

    def _release(self, shard_path: str) -> None:
        with self._lock:
            m = self._maps.get(shard_path)
            if m is not None:
                m.refs = max(0, m.refs - 1)

    @contextlib.contextmanager
    def get_view(self, shard_path: str) -> Iterator[memoryview]:
        """Zero-copy view of the shard's tar bytes (reference shard_cache.py:584-609)."""
        m = self._acquire(shard_path)
        try:
            yield memoryview(m.mm)[HDR_SIZE:HDR_SIZE + m.data_len]
        finally:
            self._release(shard_path)

    def get_array(self, shard_path: str) -> np.ndarray:
        """uint8 array over the mapped tar bytes; the mapping stays open until close()."""
        m = self._acquire(shard_path)
        return m.arr

    def get(self, shard_path: str) -> bytes:
        with self.get_view(shard_path) as v:
            return bytes(v)

    @property
    def utilisation(self) -> float:
        if self._max_bytes == 0:
            return 0.0
        with self._lock:
            return self._total / self._max_bytes

    def close(self, remove: bool = False) -> None:
        pool, self._pool = self._pool, None
        if pool is not None:
            pool.shutdown(wait=True, cancel_futures=True)
        with self._lock:
            for m in self._maps.values():
                m.close()
            self._maps.clear()
            if remove and self._node_master:
                for k in list(self._lru):
                    with contextlib.suppress(OSError):
                        self._path(k).unlink()
                self._lru.clear()
                self._total = 0
                with contextlib.suppress(OSError):
                    self._base.rmdir()


@dataclass
class BatchSpans:
    """One batch as byte ranges of mapped shards (``ShardBatchFeeder.next_batch_spans``).

    ``ptrs``/``lens``: each sample's JPEG member (absolute host address, length).
    ``parts``: the contiguous shard ranges that hold the samples, in batch order
    (address, bytes): copied to HBM as they lie, tar headers and sidecars included.
    ``offsets``: int64[B+1], each sample's offset in the concatenated parts, and
    [B] = their total size (the spans form of ``dino_decode_spans``).
    ``registered``: every part lies in page-locked memory (a DMA source).
    ``shards``: feeder shard indices of the parts (retirement bookkeeping)."""

    ptrs: np.ndarray
    lens: np.ndarray
    parts: list
    offsets: np.ndarray
    registered: bool
    shards: list


class ShardBatchFeeder:
    """Batches of B JPEGs from mapped shards.

    Shard i of the list belongs to this rank when ``i % world == rank``
    (reference hpc_source.py:154-156).  Each shard is mapped, pre-faulted, indexed
    natively and (``register``) page-locked once, on a worker thread, when first
    reached; batches never straddle an epoch and the last partial batch is dropped
    (dali_backend.py:187).  Two ways out:

    * ``next_batch_spans()``: the batch where it lies (``BatchSpans``) — the
      pipeline DMAs the shard ranges straight to HBM (no host copy) and decodes
      with the spans ABI; ``retire(batch, event)`` hands back the event after which
      the copies have read the ranges, and a consumed shard is unregistered once
      every batch taken from it has retired;
    * ``next_spans()`` / ``next_into(dst)``: (address, length) pairs, packed by
      ``dino_gather`` into a pinned buffer (batches the pipeline must re-pack, e.g.
      with Pillow hand-overs)."""

    def __init__(self, cache: ShmShardCache, shard_paths: Sequence[str], batch_size: int, rank: int = 0,
                 world: int = 1, nthreads: int = 8, lookahead: int = 2, register: bool = False) -> None:
        from concurrent.futures import ThreadPoolExecutor
        self._cache = cache
        self._paths = [p for i, p in enumerate(shard_paths) if i % world == rank]
        self._B = batch_size
        self.nthreads = nthreads
        self._shard = 0
        self._row = 0
        self._cur: tuple[np.ndarray, TarIndex] | None = None
        self.index_seconds = 0.0   # time spent preparing shards (map + pre-fault + index + register), off the caller's thread
        self.wait_seconds = 0.0    # time the caller waited for a shard to be ready
        self._lookahead = max(0, int(lookahead))
        self._pool = ThreadPoolExecutor(max_workers=max(1, self._lookahead), thread_name_prefix="shard-index") \
            if self._lookahead else None
        self._futs: dict[int, Any] = {}
        self._register = bool(register)
        self.register_error: str | None = None
        self._reg_lock = threading.Lock()
        # shard index -> {"addr", "handed", "retired", "events", "consumed"} of page-locked shards
        self._reg: dict[int, dict] = {}

    def _prepare(self, k: int) -> tuple[np.ndarray, TarIndex]:
        """Map shard k, fault its pages in, index it and page-lock it (a worker thread;
        ctypes drops the GIL)."""
        import time
        t0 = time.perf_counter()
        arr = self._cache.get_array(self._paths[k])
        prefault(arr)
        idx = index_tar(arr)
        if self._register and arr.size:
            with self._reg_lock:
                ent = self._reg.get(k)
                if ent is not None:          # still locked from an earlier epoch
                    ent["consumed"] = False
                    need = False
                else:
                    need = True
            if need:
                rc = _lib.load().dino_host_register(ctypes.c_void_p(arr.ctypes.data), arr.nbytes)
                if rc == 0:
                    with self._reg_lock:
                        self._reg[k] = {"addr": arr.ctypes.data, "handed": 0, "retired": 0, "events": [],
                                        "consumed": False}
                else:  # no GPU runtime / the mapping cannot be locked: the gather path serves
                    self._register = False
                    self.register_error = _lib.load().dino_last_error().decode(errors="replace")
        self.index_seconds += time.perf_counter() - t0
        return arr, idx

    def _open(self, k: int) -> tuple[np.ndarray, TarIndex]:
        import time
        if self._pool is None:
            return self._prepare(k)
        for j in range(k, min(len(self._paths), k + 1 + self._lookahead)):
            if j not in self._futs:
                self._futs[j] = self._pool.submit(self._prepare, j)
        t0 = time.perf_counter()
        res = self._futs.pop(k).result()
        self.wait_seconds += time.perf_counter() - t0
        return res

    @property
    def _batch_size(self) -> int:
        """The source convention backends read (reference shard_reader.py:327-329, cpu.py:671)."""
        return self._B

    _resolution_src = None  # no per-batch crop sizes: the pipeline's configured sizes apply

    def _take(self) -> list[tuple[int, np.ndarray, np.ndarray]]:
        """The next batch as (shard index, shard array, index rows) runs; StopIteration at the epoch end."""
        runs = []
        got = 0
        while got < self._B:
            if self._cur is None:
                if self._shard >= len(self._paths):
                    raise StopIteration
                self._cur = self._open(self._shard)
                self._row = 0
            arr, idx = self._cur
            take = min(self._B - got, len(idx) - self._row)
            if take > 0:
                runs.append((self._shard, arr, idx.samples[self._row:self._row + take]))
                got += take
            self._row += take
            if self._row >= len(idx):
                self._consumed(self._shard)
                self._cur = None
                self._shard += 1
        return runs

    def next_spans(self) -> list[tuple[int, int]]:
        """(address, length) of the next batch's JPEGs; StopIteration at the epoch end."""
        spans: list[tuple[int, int]] = []
        for _, arr, rows in self._take():
            spans.extend(zip((arr.ctypes.data + rows["img_off"]).tolist(), rows["img_len"].tolist()))
        self._unregister_retired()
        return spans

    def next_batch_spans(self) -> BatchSpans:
        """The next batch where it lies (see ``BatchSpans``); StopIteration at the epoch end.
        The caller must ``retire`` it once its copies are enqueued (or dropped)."""
        runs = self._take()
        ptrs = np.empty(self._B, np.uint64)
        lens = np.empty(self._B, np.int64)
        offs = np.empty(self._B + 1, np.int64)
        parts, shards = [], []
        registered = True
        i = pos = 0
        for k, arr, rows in runs:
            io, il = rows["img_off"], rows["img_len"]
            lo, hi = int(io[0]), int(io[-1] + il[-1])
            n = len(rows)
            ptrs[i:i + n] = arr.ctypes.data + io
            lens[i:i + n] = il
            offs[i:i + n] = pos + (io - lo)
            parts.append((arr.ctypes.data + lo, hi - lo))
            shards.append(k)
            with self._reg_lock:
                ent = self._reg.get(k)
                if ent is None:
                    registered = False
                else:
                    ent["handed"] += 1
            pos += hi - lo
            i += n
        offs[self._B] = pos
        self._unregister_retired()
        return BatchSpans(ptrs, lens, parts, offs, registered, shards)

    def retire(self, batch: BatchSpans, event=None) -> None:
        """The copies out of ``batch``'s ranges are enqueued and complete with ``event``
        (an object with ``query()`` / ``synchronize()``, e.g. a torch.cuda.Event; None: no
        copy was made from them)."""
        with self._reg_lock:
            for k in batch.shards:
                ent = self._reg.get(k)
                if ent is not None:
                    ent["retired"] += 1
                    if event is not None:
                        ent["events"].append(event)
        self._unregister_retired()

    def _consumed(self, k: int) -> None:
        with self._reg_lock:
            ent = self._reg.get(k)
            if ent is not None:
                ent["consumed"] = True

    def _unregister_retired(self, block: bool = False) -> None:
        """Unlock every consumed shard whose batches have all retired and whose copies finished."""
        with self._reg_lock:
            done = []
            for k, ent in self._reg.items():
                if not block and (not ent["consumed"] or ent["retired"] < ent["handed"]):
                    continue
                ev = ent["events"]
                while ev and (block or ev[0].query()):
                    ev.pop(0).synchronize()
                if ev:
                    continue
                done.append(k)
            for k in done:
                ent = self._reg.pop(k)
                _lib.load().dino_host_unregister(ctypes.c_void_p(ent["addr"]))

    def next_into(self, dst) -> np.ndarray:
        return gather(self.next_spans(), dst, self.nthreads)

    def reset(self) -> None:
        self._shard, self._row, self._cur = 0, 0, None

    def close(self) -> None:
        if self._pool is not None:
            self._pool.shutdown(wait=True, cancel_futures=True)
            self._pool = None
        self._futs.clear()
        self._unregister_retired(block=True)


class FeedBatch:
    """A packed batch handed out by the native feed: it lives in a pinned slot until
    ``NativeShardFeed.copy`` retires or ``release`` is called."""

    __slots__ = ("slot", "n", "nbytes", "host", "offsets", "info", "ws", "aws", "seq")

    def __init__(self, b) -> None:
        self.slot, self.n, self.nbytes, self.seq = int(b.slot), int(b.n), int(b.nbytes), int(b.seq)
        self.host = int(b.host or 0)
        self.offsets = np.ctypeslib.as_array(ctypes.cast(b.offsets, ctypes.POINTER(ctypes.c_int64)),
                                             (self.n + 1,)).copy()
        self.info = np.ctypeslib.as_array(ctypes.cast(b.info, ctypes.POINTER(ctypes.c_int32)), (self.n, 4)).copy()
        self.ws, self.aws = int(b.ws_need), int(b.aws_need)

    def jpegs(self) -> list[bytes]:
        """Copies of the batch's images (for the Pillow hand-over path)."""
        o = self.offsets
        return [ctypes.string_at(self.host + int(o[i]), int(o[i + 1] - o[i])) for i in range(self.n)]


class NativeShardFeed:
    """The node-local shard feed run natively (``dino_feed_*``, csrc/feed.hip): an opener
    thread maps, pre-faults and indexes this rank's shard-cache files a few shards ahead;
    a packer thread packs every batch of B samples into a pinned slot with ``nthreads``
    copier threads and probes each image right after its copy.  No Python runs per batch
    on the host half, so it does not wait for the GIL behind the launch thread.

    Same source conventions as :class:`ShardBatchFeeder` (``_batch_size``,
    ``_resolution_src``; shard i belongs to rank ``i % world``, reference
    hpc_source.py:154-156; the last partial batch of an epoch is dropped,
    dali_backend.py:187; an unreadable shard is skipped with a warning,
    hpc_source.py:358-366).  ``MI355XAugPipeline`` consumes it through
    ``next_prepared`` / ``copy`` / ``release``."""

    def __init__(self, cache: ShmShardCache, shard_paths: Sequence[str], batch_size: int, rank: int = 0,
                 world: int = 1, nthreads: int = 8, slots: int = 6, lookahead: int = 2,
                 shuffle: bool = False, seed: int = 0) -> None:
        self._cache = cache
        self._paths = [p for i, p in enumerate(shard_paths) if i % world == rank]
        # shuffle: the reference's per-epoch shard order (ShardIterator._make_shard_cycle,
        # hpc_source.py:205, 263, 488-500: numpy default_rng(seed + rank [+ epoch * 997]).shuffle)
        # and a seeded in-shard sample order (the extraction shuffle buffer, :461-467)
        self._shuffle = bool(shuffle)
        self._seed = int(seed) + int(rank)
        self.epoch = 0
        self._B = int(batch_size)
        self.nthreads = int(nthreads)
        self._slots = max(2, int(slots))
        self._lookahead = max(1, int(os.environ.get("DINO_FEED_LOOKAHEAD", lookahead)))
        self._max_dim = 0
        self._cfg = None
        self._feed = ctypes.c_void_p()
        self._started = False
        self.shard_errors: list[str] = []

    @property
    def _batch_size(self) -> int:
        return self._B

    _resolution_src = None

    def configure(self, max_image_dim: int = 0, cfg=None) -> None:
        """Probe settings (the pipeline's ``max_image_dim`` and its view config for the
        augment-workspace bound); the native feed starts on the first ``next_prepared``."""
        self._max_dim = int(max_image_dim)
        self._cfg = cfg
        if self._feed:
            _lib.check(_lib.load().dino_feed_set_cfg(self._feed, ctypes.byref(cfg) if cfg is not None else None),
                       "dino_feed_set_cfg")

    def _check(self, rc: int, what: str) -> None:
        if rc != 0:
            raise _lib.DinoError(f"{what} failed ({rc}): {_lib.load().dino_feed_last_error().decode(errors='replace')}")

    def epoch_order(self, epoch: int | None = None) -> list[str]:
        """This rank's shard order for ``epoch`` (the reference's shard cycle)."""
        paths = list(self._paths)
        if self._shuffle:
            e = self.epoch if epoch is None else int(epoch)
            np.random.default_rng(self._seed + e * 997).shuffle(paths)
        return paths

    def _start(self) -> None:
        lib = _lib.load()
        if not self._feed:
            cfg = ctypes.byref(self._cfg) if self._cfg is not None else None
            self._check(lib.dino_feed_create(self._B, self.nthreads, self._slots, self._lookahead, self._max_dim, cfg,
                                             ctypes.byref(self._feed)), "dino_feed_create")
            if not self._cache.node_master:  # the opener waits for the node master's writes
                self._check(lib.dino_feed_set_shard_wait(self._feed, int(self._cache.shard_timeout_s * 1000)),
                            "dino_feed_set_shard_wait")
            self._check(lib.dino_feed_set_shuffle(self._feed, int(self._shuffle), self._seed & (2**64 - 1)),
                        "dino_feed_set_shuffle")
        # the in-shard order is keyed by this epoch, as the shard order is (a resumed
        # reset(epoch=k) on a fresh feed keyed the samples by the number of resets instead)
        self._check(lib.dino_feed_set_epoch(self._feed, int(self.epoch) & (2**64 - 1)), "dino_feed_set_epoch")
        for p in self.epoch_order():
            shm = self._cache._ensure(p) if self._cache.node_master else self._cache.path_of(p)
            self._check(lib.dino_feed_push(self._feed, str(shm).encode()), "dino_feed_push")
        self._check(lib.dino_feed_end_epoch(self._feed), "dino_feed_end_epoch")
        self._started = True

    def next_prepared(self, timeout: float | None = None) -> FeedBatch | None:
        """The next packed batch; None when ``timeout`` (seconds) passes first; StopIteration
        at the end of the epoch."""
        if not self._started:
            self._start()
        lib = _lib.load()
        out = _lib.DinoFeedBatch()
        ms = -1 if timeout is None else int(timeout * 1000)
        while True:
            rc = lib.dino_feed_next(self._feed, ms, ctypes.byref(out))
            if rc == _lib.FEED_SHARD_ERROR:
                msg = lib.dino_feed_last_error().decode(errors="replace")
                self.shard_errors.append(msg)
                import warnings
                warnings.warn(f"NativeShardFeed: skipped a shard: {msg}", RuntimeWarning, stacklevel=2)
                continue
            if rc == _lib.FEED_END:
                raise StopIteration
            if rc == _lib.FEED_TIMEOUT:
                return None
            self._check(rc, "dino_feed_next")
            return FeedBatch(out)

    def copy(self, batch: FeedBatch, d_bytes: int, d_offsets: int, stream: int) -> None:
        """H2D copies of ``batch`` (bytes, offsets) to device addresses on ``stream`` (a hipStream_t)."""
        self._check(_lib.load().dino_feed_copy(self._feed, batch.slot, ctypes.c_void_p(d_bytes),
                                               ctypes.c_void_p(d_offsets), ctypes.c_void_p(stream)), "dino_feed_copy")

    def release(self, batch: FeedBatch) -> None:
        if self._feed:
            _lib.load().dino_feed_release(self._feed, batch.slot)

    def stats(self) -> dict:
        if not self._feed:
            return {}
        sec = (ctypes.c_double * 4)()
        cnt = (ctypes.c_int64 * 3)()
        self._check(_lib.load().dino_feed_stats(self._feed, sec, cnt), "dino_feed_stats")
        return {"open_s": sec[0], "pack_s": sec[1], "slot_wait_s": sec[2], "sample_wait_s": sec[3],
                "batches": cnt[0], "shards_done": cnt[1], "shards_failed": cnt[2]}

    def reset(self, epoch: int | None = None) -> None:
        """New epoch (the pushed shards and packed batches not yet handed out are dropped);
        ``epoch`` defaults to the next one (reference ShardIterator.reset_epoch, :242-273)."""
        if self._feed:
            self._check(_lib.load().dino_feed_reset(self._feed), "dino_feed_reset")
        self.epoch = self.epoch + 1 if epoch is None else int(epoch)
        self._started = False

    def close(self) -> None:
        if self._feed:
            _lib.load().dino_feed_destroy(self._feed)
            self._feed = ctypes.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:  # noqa: BLE001
            pass


_MADV_POPULATE_READ = 22  # Linux >= 5.14


def prefault(arr: np.ndarray) -> None:
    """Populate the page tables of a mapped shard before the gather reads it
    (madvise(MADV_POPULATE_READ) on the mapping, else a one-byte-per-page read)."""
    base = getattr(arr, "base", None)
    if isinstance(base, memoryview):
        base = base.obj
    mm = base if isinstance(base, mmap.mmap) else None
    if mm is not None and hasattr(mm, "madvise"):
        try:
            mm.madvise(_MADV_POPULATE_READ)
            return
        except OSError:
            pass
    if arr.size:
        int(arr[::4096].sum())
