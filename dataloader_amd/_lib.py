"""ctypes binding of ``libdino_ingest.so`` (the C ABI of ``include/dino_ingest.h``).

The library is built in-tree by ``__graft_entry__.build()`` (hipcc, gfx950).
There is no fallback: if it is missing or a GPU is absent, every call raises.
"""

from __future__ import annotations

import ctypes
import os
from pathlib import Path

from .params import DinoAugConfig, DinoLimits

_PKG = Path(__file__).resolve().parent
LIB_PATH = _PKG / "libdino_ingest.so"

DINO_OK = 0
IMG_STATUS = {0: "ok", -1: "corrupt", -2: "truncated", -3: "bad-data", -4: "too-large (Pillow bomb check)",
              1: "unsupported", 2: "multi-scan", 3: "no-space", 4: "over max_image_dim (handed to Pillow)"}
ABI_VERSION = 4
RAW_MAGIC = 0x42475244  # "DRGB": pre-decoded RGB container (include/dino_ingest.h)
COPY_HEADER = 1  # dino_copy_rgb_packed flags: write the container header in front of each image

_lib = None
FEED_END, FEED_TIMEOUT, FEED_SHARD_ERROR = 1, 2, 3


class DinoError(RuntimeError):
    pass


class DinoFeedBatch(ctypes.Structure):
    """``dino_feed_batch`` (include/dino_ingest.h)."""

    _fields_ = [("slot", ctypes.c_int32), ("n", ctypes.c_int32), ("nbytes", ctypes.c_int64),
                ("host", ctypes.c_void_p), ("offsets", ctypes.c_void_p), ("info", ctypes.c_void_p),
                ("ws_need", ctypes.c_int64), ("aws_need", ctypes.c_int64), ("seq", ctypes.c_int64)]


def load() -> ctypes.CDLL:
    """Load the HIP library; raise loudly when it is not built."""
    global _lib
    if _lib is not None:
        return _lib
    path = Path(os.environ.get("DINO_INGEST_LIB", LIB_PATH))  # experiments may point at a variant build
    if not path.exists():
        raise DinoError(f"{path} not found: run `python -c 'import __graft_entry__ as g; g.build()'` "
                        "(hipcc --offload-arch=gfx950). There is no CPU fallback.")
    lib = ctypes.CDLL(str(path), mode=os.RTLD_NOW | os.RTLD_GLOBAL)
    vp, i32, i64, u64, dbl = ctypes.c_void_p, ctypes.c_int32, ctypes.c_int64, ctypes.c_uint64, ctypes.c_double
    sig = {
        "dino_abi_version": (i32, []),
        "dino_last_error": (ctypes.c_char_p, []),
        "dino_ctx_create": (i32, [ctypes.c_int, ctypes.POINTER(DinoLimits), ctypes.POINTER(vp)]),
        "dino_ctx_destroy": (i32, [vp]),
        "dino_decode": (i32, [vp, vp, vp, vp, i32, vp, vp]),
        "dino_decode_spans": (i32, [vp, vp, vp, vp, vp, i32, vp, vp]),
        "dino_run_batch_spans": (i32, [vp, vp, vp, vp, vp, i32, ctypes.POINTER(DinoAugConfig), u64, u64, vp,
                                       ctypes.POINTER(vp), vp, vp]),
        "dino_probe_spans": (i32, [vp, vp, vp, i32, i32, ctypes.POINTER(DinoAugConfig), vp, ctypes.POINTER(i64),
                                   ctypes.POINTER(i64)]),
        "dino_gather_probe": (i32, [vp, vp, i32, vp, i64, vp, i32, i32, ctypes.POINTER(DinoAugConfig), vp,
                                    ctypes.POINTER(i64), ctypes.POINTER(i64)]),
        "dino_feed_create": (i32, [i32, i32, i32, i32, i32, ctypes.POINTER(DinoAugConfig), ctypes.POINTER(vp)]),
        "dino_feed_destroy": (i32, [vp]),
        "dino_feed_push": (i32, [vp, ctypes.c_char_p]),
        "dino_feed_end_epoch": (i32, [vp]),
        "dino_feed_set_cfg": (i32, [vp, ctypes.POINTER(DinoAugConfig)]),
        "dino_feed_set_shard_wait": (i32, [vp, i32]),
        "dino_feed_set_shuffle": (i32, [vp, i32, ctypes.c_uint64]),
        "dino_feed_set_epoch": (i32, [vp, ctypes.c_uint64]),
        "dino_feed_next": (i32, [vp, i32, ctypes.POINTER(DinoFeedBatch)]),
        "dino_feed_copy": (i32, [vp, i32, vp, vp, vp]),
        "dino_feed_release": (i32, [vp, i32]),
        "dino_feed_reset": (i32, [vp]),
        "dino_feed_stats": (i32, [vp, vp, vp]),
        "dino_feed_last_error": (ctypes.c_char_p, []),
        "dino_host_register": (i32, [vp, i64]),
        "dino_host_unregister": (i32, [vp]),
        "dino_copy_h2d": (i32, [vp, vp, i64, vp]),
        "dino_stream_create": (i32, [i32, i32, ctypes.POINTER(vp)]),
        "dino_stream_destroy": (i32, [vp]),
        "dino_copy_rgb": (i32, [vp, i32, vp, vp]),
        "dino_copy_rgb_packed": (i32, [vp, i32, vp, vp, vp, i32, vp]),
        "dino_pixel_ops_all": (i32, [i32, i32, vp, vp]),
        "dino_sample_params": (i32, [vp, ctypes.POINTER(DinoAugConfig), u64, u64, vp, vp]),
        "dino_augment": (i32, [vp, ctypes.POINTER(DinoAugConfig), vp, ctypes.POINTER(vp), vp]),
        "dino_run_batch": (i32, [vp, vp, vp, vp, i32, ctypes.POINTER(DinoAugConfig), u64, u64, vp,
                                 ctypes.POINTER(vp), vp, vp]),
        "dino_masks": (i32, [i32, i32, i32, i32, i32, dbl, dbl, i32, vp, vp, vp, vp]),
        "dino_bf16_to_fp8": (i32, [vp, vp, i64, vp]),
        "dino_debug_region": (i32, [vp, i32, i32, vp, i64, vp]),
        "dino_set_timing": (i32, [vp, i32]),
        "dino_ctx_set_prog_decoder": (i32, [vp, i32]),
        "dino_kernel_times": (i32, [vp, vp, vp, i32]),
        "dino_tar_index": (i32, [vp, i64, vp, i64, vp, i64, ctypes.POINTER(i64), ctypes.POINTER(i64)]),
        "dino_tar_index_fd": (i32, [i32, i64, i64, vp, i64, vp, i64, ctypes.POINTER(i64), ctypes.POINTER(i64)]),
        "dino_tar_last_error": (ctypes.c_char_p, []),
        "dino_gather": (i32, [vp, vp, i64, vp, i64, vp, i32]),
        "dino_set_norm": (i32, [vp, vp, i32]),
        "dino_batch_info": (i32, [vp, vp, vp]),
        "dino_probe": (i32, [vp, vp, vp, i32, i32, ctypes.POINTER(DinoAugConfig), vp, ctypes.POINTER(i64),
                             ctypes.POINTER(i64)]),
        "dino_reserve": (i32, [vp, i64, i64, vp]),
        "dino_augment_need": (i32, [vp, i32, ctypes.POINTER(DinoAugConfig), ctypes.POINTER(i64)]),
        "dino_workspace_sizes": (i32, [vp, ctypes.POINTER(i64), ctypes.POINTER(i64)]),
        "dino_masks_host": (i32, [i32, i32, i32, i32, i32, dbl, dbl, i32, vp, vp, vp]),
        "dino_resize_batch": (i32, [vp, i32, i32, vp, vp, i32, vp, vp]),
    }
    for name, (res, args) in sig.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    _lib = lib
    return lib


def check(rc: int, what: str) -> None:
    if rc != DINO_OK:
        msg = load().dino_last_error().decode(errors="replace")
        raise DinoError(f"{what} failed ({rc}): {msg}")


def exported_symbols() -> list[str]:
    return ["dino_abi_version", "dino_last_error", "dino_ctx_create", "dino_ctx_destroy", "dino_decode",
            "dino_copy_rgb", "dino_pixel_ops_all", "dino_sample_params", "dino_augment", "dino_run_batch", "dino_masks",
            "dino_bf16_to_fp8", "dino_debug_region", "dino_set_timing", "dino_kernel_times",
            "dino_ctx_set_prog_decoder", "dino_copy_rgb_packed", "dino_tar_index", "dino_tar_index_fd", "dino_tar_last_error", "dino_gather", "dino_set_norm", "dino_batch_info",
            "dino_probe", "dino_reserve", "dino_workspace_sizes", "dino_masks_host", "dino_resize_batch",
            "dino_augment_need", "dino_decode_spans", "dino_run_batch_spans", "dino_probe_spans",
            "dino_host_register", "dino_host_unregister", "dino_copy_h2d", "dino_gather_probe",
            "dino_feed_create", "dino_feed_destroy", "dino_feed_push", "dino_feed_end_epoch", "dino_feed_set_cfg",
            "dino_feed_set_shard_wait", "dino_feed_set_shuffle", "dino_feed_set_epoch",
            "dino_feed_next", "dino_feed_copy", "dino_feed_release", "dino_feed_reset", "dino_feed_stats",
            "dino_feed_last_error", "dino_stream_create", "dino_stream_destroy"]
