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


def probe(host_buf_ptr: int, offsets: np.ndarray, batch: int, max_image_dim: int, cfg=None):
    """``dino_probe`` over a packed host batch -> (info[B,4] int32, ws_bytes, aws_bytes)."""
    lib = _lib.load()
    info = np.zeros((batch, 4), np.int32)
    ws, aws = ctypes.c_int64(0), ctypes.c_int64(0)
    offs = np.ascontiguousarray(offsets, np.int64)
    _lib.check(lib.dino_probe(ctypes.c_void_p(host_buf_ptr), offs.ctypes.data_as(ctypes.c_void_p), batch,
                              max_image_dim, ctypes.byref(cfg) if cfg is not None else None,
                              info.ctypes.data_as(ctypes.c_void_p), ctypes.byref(ws), ctypes.byref(aws)),
               "dino_probe")
    return info, int(ws.value), int(aws.value)


def hand_over(jpegs: list, status: np.ndarray) -> tuple[list, int]:
    """Replace the images the GPU decoder does not implement by Pillow-decoded raw RGB
    containers (zero bytes where Pillow raises).  Returns (new list, images handed over)."""
    out = list(jpegs)
    n = 0
    for i in np.flatnonzero(status == IMG_UNSUPPORTED):
        rgb = decode_with_pillow(jpegs[i])
        out[i] = raw_container(rgb) if rgb is not None else b""
        n += 1
    return out, n
