"""Host mirrors of the C ABI structs in ``include/dino_ingest.h``.

``VIEW_PARAMS_DTYPE`` is the numpy layout of ``dino_view_params`` (80 bytes):
every random decision ``_augment_one`` makes for one (sample, view)
(reference ``src/dino_loader/backends/cpu.py:172-267``).  Records are stored
sample-major: ``params[b * n_views + v]``.
"""

from __future__ import annotations

import ctypes

import numpy as np

VIEW_PARAMS_DTYPE = np.dtype([
    ("crop_top", "<i4"), ("crop_left", "<i4"), ("crop_h", "<i4"), ("crop_w", "<i4"),
    ("out_size", "<i4"),
    ("flip", "u1"), ("jitter", "u1"), ("gray", "u1"), ("blur", "u1"),
    ("solarize", "u1"), ("pad0", "u1", (3,)),
    ("order", "u1", (4,)),
    ("brightness", "<f4"), ("contrast", "<f4"), ("saturation", "<f4"), ("hue", "<f4"),
    ("sigma", "<f8"),
    ("ksize", "<i4"), ("pad1", "<i4"),
    ("resize_w", "<i4"), ("resize_h", "<i4"), ("out_x", "<i4"), ("out_y", "<i4"),
])
assert VIEW_PARAMS_DTYPE.itemsize == 80
RECORD_BYTES = VIEW_PARAMS_DTYPE.itemsize
RECIPE_DINOV2, RECIPE_LEJEPA, RECIPE_EVAL = 0, 1, 2

OUT_BF16, OUT_FP32, OUT_FP8_E4M3 = 0, 1, 2


class DinoLimits(ctypes.Structure):
    _fields_ = [
        ("max_batch", ctypes.c_int32),
        ("max_views", ctypes.c_int32),
        ("max_crop_size", ctypes.c_int32),
        ("max_image_dim", ctypes.c_int32),
        ("workspace_bytes", ctypes.c_int64),
    ]


class DinoAugConfig(ctypes.Structure):
    _fields_ = [
        ("n_global", ctypes.c_int32), ("n_local", ctypes.c_int32),
        ("global_size", ctypes.c_int32), ("local_size", ctypes.c_int32),
        ("global_scale", ctypes.c_float * 2), ("local_scale", ctypes.c_float * 2),
        ("blur_prob_global1", ctypes.c_float), ("blur_prob_global2", ctypes.c_float),
        ("blur_prob_local", ctypes.c_float),
        ("solarize_prob", ctypes.c_float), ("color_jitter_prob", ctypes.c_float),
        ("grayscale_prob", ctypes.c_float), ("flip_prob", ctypes.c_float),
        ("blur_sigma_min", ctypes.c_float), ("blur_sigma_max", ctypes.c_float),
        ("brightness", ctypes.c_float), ("contrast", ctypes.c_float),
        ("saturation", ctypes.c_float), ("hue", ctypes.c_float),
        ("mean", ctypes.c_float * 3), ("std", ctypes.c_float * 3),
        ("out_dtype", ctypes.c_int32), ("recipe", ctypes.c_int32),
    ]


def make_aug_config(aug_cfg, global_size: int, local_size: int, out_dtype: int) -> DinoAugConfig:
    """Build the C struct from a ``DINOAugConfig``-shaped object (reference config.py:243-272);
    ``aug_cfg.recipe`` (default DINOv2) selects the view recipe (``DINO_RECIPE_*``)."""
    c = DinoAugConfig()
    c.recipe = int(getattr(aug_cfg, "recipe", RECIPE_DINOV2))
    c.n_global = int(aug_cfg.n_global_crops)
    c.n_local = int(aug_cfg.n_local_crops)
    c.global_size = int(global_size)
    c.local_size = int(local_size)
    c.global_scale[:] = [float(x) for x in aug_cfg.global_crops_scale]
    c.local_scale[:] = [float(x) for x in aug_cfg.local_crops_scale]
    c.blur_prob_global1 = aug_cfg.blur_prob_global1
    c.blur_prob_global2 = aug_cfg.blur_prob_global2
    c.blur_prob_local = aug_cfg.blur_prob_local
    c.solarize_prob = aug_cfg.solarize_prob
    c.color_jitter_prob = aug_cfg.color_jitter_prob
    c.grayscale_prob = aug_cfg.grayscale_prob
    c.flip_prob = aug_cfg.flip_prob
    c.blur_sigma_min = aug_cfg.blur_sigma_min
    c.blur_sigma_max = aug_cfg.blur_sigma_max
    c.brightness = aug_cfg.brightness
    c.contrast = aug_cfg.contrast
    c.saturation = aug_cfg.saturation
    c.hue = aug_cfg.hue
    c.mean[:] = [float(x) for x in aug_cfg.mean]
    c.std[:] = [float(x) for x in aug_cfg.std]
    c.out_dtype = int(out_dtype)
    return c
