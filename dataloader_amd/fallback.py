"""Host pre-screen and hand-over of the JPEG flavours the GPU decoder does not implement.

The reference decodes every image with Pillow (``Image.open(BytesIO(b)).convert("RGB")``,
reference ``src/dino_loader/backends/cpu.py:251``).  The HIP decoder covers
baseline, extended-sequential, progressive and multi-scan Huffman JPEGs
(8-bit, 1 or 3 components); everything else it reports with a positive status
(``include/dino_ingest.h``).  So that no image the reference would decode comes
back as zeros, each host batch is screened *before* it is launched:

1. ``dino_probe`` runs the device's own parser (and its progressive marker walk)
   on the host bytes — a few microseconds per image — and reports every image's
   status, plus the exact decode-workspace bytes and an augment-workspace bound;
2. images with status ``DINO_IMG_UNSUPPORTED`` (CMYK/YCCK, arithmetic, lossless,
   progressive files libjpeg would block-smooth, > 64 scans) are decoded here by
   Pillow — the very call the reference makes — and travel to the GPU as
   pre-decoded RGB images (``DINO_RAW_MAGIC`` container); if Pillow raises, the
   image travels as zero bytes, which the device reports as corrupt and
   zero-fills, exactly as the reference does (cpu.py:252-253);
3. the engine grows its workspaces to the probe's numbers (``dino_reserve``), so
   ``DINO_IMG_NO_SPACE`` cannot occur for a screened batch.

The augmentation of a handed-over image still runs entirely in the HIP kernels.
The hand-over is counted (``MI355XAugPipeline.stats``).
"""

from __future__ import annotations

import ctypes
import io
import struct

import numpy as np

from . import _lib

IMG_UNSUPPORTED = 1
IMG_LIMIT = 4


def decode_with_pillow(jpeg) -> np.ndarray | None:
    """HWC uint8 RGB exactly as the reference decodes it (cpu.py:251), or None where it raises."""
    from PIL import Image
    try:
        return np.asarray(Image.open(io.BytesIO(bytes(jpeg))).convert("RGB"))
    except Exception:  # noqa: BLE001 - mirrors cpu.py:252
        return None


def raw_container(rgb: np.ndarray) -> bytes:
    """Pre-decoded RGB image in the ABI's raw container (16-byte header + HWC bytes)."""
    h, w, c = rgb.shape
    assert c == 3 and rgb.dtype == np.uint8
    return struct.pack("<IIII", _lib.RAW_MAGIC, w, h, 0) + np.ascontiguousarray(rgb).tobytes()


def probe(host_buf_ptr: int, offsets: np.ndarray, batch: int, max_image_dim: int, cfg=None,
          raw_mask: np.ndarray | None = None):
    """``dino_probe`` over a packed host batch -> (info[B,4] int32, ws_bytes, aws_bytes).
    ``raw_mask``: uint8[B], 1 where the image is a raw RGB container (a hand-over)."""
    lib = _lib.load()
    info = np.zeros((batch, 4), np.int32)
    ws, aws = ctypes.c_int64(0), ctypes.c_int64(0)
    offs = np.ascontiguousarray(offsets, np.int64)
    rm = None if raw_mask is None else np.ascontiguousarray(raw_mask, np.uint8)
    _lib.check(lib.dino_probe(ctypes.c_void_p(host_buf_ptr), offs.ctypes.data_as(ctypes.c_void_p),
                              rm.ctypes.data_as(ctypes.c_void_p) if rm is not None else None, batch,
                              max_image_dim, ctypes.byref(cfg) if cfg is not None else None,
                              info.ctypes.data_as(ctypes.c_void_p), ctypes.byref(ws), ctypes.byref(aws)),
               "dino_probe")
    return info, int(ws.value), int(aws.value)


def probe_spans(ptrs: np.ndarray, lens: np.ndarray, max_image_dim: int, cfg=None):
    """``dino_probe_spans`` over images where they lie (absolute host addresses + lengths,
    e.g. JPEG members of mapped shards) -> (info[B,4] int32, ws_bytes, aws_bytes)."""
    lib = _lib.load()
    p = np.ascontiguousarray(ptrs, np.uint64)
    n = np.ascontiguousarray(lens, np.int64)
    batch = len(p)
    info = np.zeros((batch, 4), np.int32)
    ws, aws = ctypes.c_int64(0), ctypes.c_int64(0)
    _lib.check(lib.dino_probe_spans(p.ctypes.data_as(ctypes.c_void_p), n.ctypes.data_as(ctypes.c_void_p), None,
                                    batch, max_image_dim, ctypes.byref(cfg) if cfg is not None else None,
                                    info.ctypes.data_as(ctypes.c_void_p), ctypes.byref(ws), ctypes.byref(aws)),
               "dino_probe_spans")
    return info, int(ws.value), int(aws.value)


def gather_probe(ptrs: np.ndarray, lens: np.ndarray, dst, nthreads: int, max_image_dim: int, cfg=None):
    """``dino_gather_probe``: pack the images (absolute host addresses + lengths) into the
    pinned tensor ``dst`` and probe each right after its copy, on ``nthreads`` threads ->
    (int64 offsets[B+1], info[B,4] int32, ws_bytes, aws_bytes)."""
    lib = _lib.load()
    p = np.ascontiguousarray(ptrs, np.uint64)
    n = np.ascontiguousarray(lens, np.int64)
    batch = len(p)
    off = np.empty(batch + 1, np.int64)
    info = np.zeros((batch, 4), np.int32)
    ws, aws = ctypes.c_int64(0), ctypes.c_int64(0)
    _lib.check(lib.dino_gather_probe(p.ctypes.data_as(ctypes.c_void_p), n.ctypes.data_as(ctypes.c_void_p), batch,
                                     ctypes.c_void_p(dst.data_ptr()), dst.numel() * dst.element_size(),
                                     off.ctypes.data_as(ctypes.c_void_p), int(nthreads), max_image_dim,
                                     ctypes.byref(cfg) if cfg is not None else None,
                                     info.ctypes.data_as(ctypes.c_void_p), ctypes.byref(ws), ctypes.byref(aws)),
               "dino_gather_probe")
    return off, info, int(ws.value), int(aws.value)


def augment_need(info: np.ndarray, cfg) -> int:
    """``dino_augment_need``: augment-workspace bytes of a probed batch for ``cfg``'s views."""
    lib = _lib.load()
    inf = np.ascontiguousarray(info, np.int32)
    aws = ctypes.c_int64(0)
    _lib.check(lib.dino_augment_need(inf.ctypes.data_as(ctypes.c_void_p), len(inf), ctypes.byref(cfg),
                                     ctypes.byref(aws)), "dino_augment_need")
    return int(aws.value)


def pillow_container(jpeg) -> bytes:
    """One hand-over: the Pillow decode as a raw container, or b"" where Pillow raises."""
    rgb = decode_with_pillow(jpeg)
    return raw_container(rgb) if rgb is not None else b""


def hand_over(jpegs: list, status: np.ndarray, mask: np.ndarray | None = None,
              pool: "HostDecoder | None" = None) -> tuple[list, int, np.ndarray]:
    """Replace the images the GPU decoder does not decode (``status`` ``IMG_UNSUPPORTED`` or
    ``IMG_LIMIT``, or ``mask`` when given) by Pillow-decoded raw RGB containers (zero bytes
    where Pillow raises), in ``pool``'s worker processes when given.  Returns (new list,
    images handed over, raw mask: uint8[B], 1 where the new entry is a container — the
    mask dino_probe / dino_decode need to accept it)."""
    idx = np.flatnonzero(np.isin(status, (IMG_UNSUPPORTED, IMG_LIMIT)) if mask is None else mask)
    out = list(jpegs)
    if pool is not None and len(idx) > 1:
        for i, f in zip(idx, [pool.submit(jpegs[i]) for i in idx]):
            out[i] = f.result()
    else:
        for i in idx:
            out[i] = pillow_container(jpegs[i])
    return out, len(idx), raw_mask_of(out, idx)


def raw_mask_of(images: list, handed) -> np.ndarray:
    """uint8[B]: 1 for the handed-over entries that hold a container (Pillow did not raise)."""
    m = np.zeros(len(images), np.uint8)
    for i in handed:
        m[int(i)] = len(images[int(i)]) > 0
    return m


def route_mask(info: np.ndarray, host_fallback: bool, multiscan_route: str, host_max: int) -> np.ndarray:
    """Images of a probed batch to decode with Pillow on the host.

    * ``DINO_IMG_UNSUPPORTED`` images and JPEGs over a caller-chosen ``max_image_dim``
      (``DINO_IMG_LIMIT``), always (when ``host_fallback``);
    * coefficient-buffer images (``info[:, 3] == 1``: progressive, multi-scan sequential,
      damaged restart intervals), which ``k_prog`` decodes one image per workgroup with
      every scan serial — about 100 ms of latency for a batch holding any — so that
      a batch with a few of them would wait on the slowest: ``"host"`` sends them all to
      Pillow, ``"device"`` none, ``"auto"`` all of them when the batch has at most
      ``host_max`` (the host decodes ~6 ms per 640x480 image per worker, off the
      critical path when prepared one batch ahead), else none."""
    mask = np.isin(info[:, 0], (IMG_UNSUPPORTED, IMG_LIMIT)) if host_fallback else np.zeros(len(info), bool)
    ms = (info[:, 0] == 0) & (info[:, 3] == 1)
    if multiscan_route == "host" or (multiscan_route == "auto" and 0 < ms.sum() <= host_max):
        mask |= ms
    return mask


class HostDecoder:
    """A pool of worker processes for the Pillow hand-over.  Pillow's decode of one JPEG
    holds the GIL for most of its run (threads give no speed-up), so the workers are
    processes, started with ``spawn`` (a fork of a process that has initialised HIP is not
    safe).  ``start()`` starts them eagerly (the backend-built pipeline does, so that a
    script whose spawned children cannot start — no ``if __name__ == "__main__":`` guard
    around the training loop — fails at construction, not at the first CMYK file
    mid-epoch); otherwise they start with the first submitted image.  If the pool cannot
    start or breaks, the hand-over continues in this process (same bytes, slower) with a
    ``RuntimeWarning``."""

    def __init__(self, workers: int):
        self.workers = max(1, int(workers))
        self._pool = None
        self._inline = False

    def start(self) -> None:
        """Start the workers now and wait until each has imported Pillow."""
        if self._pool is not None or self._inline:
            return
        import multiprocessing as mp
        from concurrent.futures import ProcessPoolExecutor
        try:
            self._pool = ProcessPoolExecutor(self.workers, mp_context=mp.get_context("spawn"))
            # the executor starts a process per submit that finds no idle one: start them all
            # now (each imports Pillow on its no-op decode) rather than one per later batch
            warm = [self._pool.submit(decode_with_pillow, b"") for _ in range(self.workers)]
            for f in warm:
                f.result(timeout=120)
        except Exception as e:  # noqa: BLE001 - BrokenProcessPool, spawn bootstrap errors, timeouts
            self._fall_back(e)

    def _fall_back(self, err: BaseException) -> None:
        import warnings
        warnings.warn(f"HostDecoder: the Pillow worker pool is unavailable ({type(err).__name__}: {err}); "
                      "handing images over in-process (a spawned worker re-imports __main__: guard the "
                      "training script with `if __name__ == '__main__':`)", RuntimeWarning, stacklevel=3)
        if self._pool is not None:
            self._pool.shutdown(wait=False, cancel_futures=True)
            self._pool = None
        self._inline = True

    def submit(self, jpeg):
        from concurrent.futures import Future
        if self._pool is None and not self._inline:
            self.start()
        if not self._inline:
            try:
                return self._pool.submit(pillow_container, bytes(jpeg))
            except Exception as e:  # noqa: BLE001 - the pool broke after it started
                self._fall_back(e)
        f = Future()
        f.set_result(pillow_container(jpeg))
        return f

    def close(self) -> None:
        if self._pool is not None:
            self._pool.shutdown(wait=True, cancel_futures=True)
            self._pool = None
