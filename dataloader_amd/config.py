"""Configuration objects the hot path reads, mirroring the reference's API.

Field names, defaults and meaning follow reference ``src/dino_loader/config.py``
(``NormStats`` :32-98, ``PipelineConfig`` :146-208, ``DINOAugConfig`` :216-313)
and ``augmentation.py`` (``DinoV2AugSpec`` :245-286), so objects built for the
reference loader can be handed to :class:`~dataloader_amd.backend.MI355XBackend`
unchanged (the backend only duck-types the attributes below).
"""

from __future__ import annotations

import threading
from dataclasses import dataclass, field
from typing import Any

import numpy as np


@dataclass(frozen=True)
class NormStats:
    mean: tuple = (0.485, 0.456, 0.406)
    std: tuple = (0.229, 0.224, 0.225)

    def __post_init__(self):
        if any(s <= 0.0 for s in self.std):
            raise ValueError(f"NormStats.std must be strictly positive, got {self.std}.")


@dataclass(frozen=True)
class PipelineConfig:
    num_threads: int = 8
    device_id: int = 0
    hw_decoder_load: float = 0.90
    cpu_queue: int = 16
    gpu_queue: int = 6
    seed: int = 0
    fuse_normalization: bool = True
    dali_fp8_output: bool = False
    output_dtype: str = "bf16"


@dataclass
class DINOAugConfig:
    global_crop_size: int = 224
    local_crop_size: int = 96
    n_global_crops: int = 2
    n_local_crops: int = 8
    global_crops_scale: tuple = (0.32, 1.0)
    local_crops_scale: tuple = (0.05, 0.32)
    blur_prob_global1: float = 1.0
    blur_prob_global2: float = 0.1
    blur_prob_local: float = 0.5
    solarize_prob: float = 0.2
    color_jitter_prob: float = 0.8
    grayscale_prob: float = 0.2
    blur_sigma_min: float = 0.1
    blur_sigma_max: float = 2.0
    brightness: float = 0.8
    contrast: float = 0.8
    saturation: float = 0.8
    hue: float = 0.2
    flip_prob: float = 0.5
    preserve_aspect_ratio: bool = True
    resolution_schedule: list = field(default_factory=list)
    max_global_crop_size: int = 0
    max_local_crop_size: int = 0
    mean: tuple = (0.485, 0.456, 0.406)
    std: tuple = (0.229, 0.224, 0.225)

    def __post_init__(self):
        if self.max_global_crop_size == 0:
            self.max_global_crop_size = self.global_crop_size
        if self.max_local_crop_size == 0:
            self.max_local_crop_size = self.local_crop_size
        if self.resolution_schedule:
            self.resolution_schedule = sorted(self.resolution_schedule, key=lambda x: x[0])
            if any(e < 0 for e, _ in self.resolution_schedule):
                raise ValueError("DINOAugConfig: resolution_schedule epochs must be >= 0")

    @property
    def n_views(self) -> int:
        return self.n_global_crops + self.n_local_crops

    @property
    def norm_stats(self) -> NormStats:
        return NormStats(mean=self.mean, std=self.std)

    def crop_size_at_epoch(self, epoch: int) -> int:
        size = self.global_crop_size
        for e, s in self.resolution_schedule:
            if epoch >= e:
                size = s
        return size


@dataclass
class DinoV2AugSpec:
    aug_cfg: DINOAugConfig = field(default_factory=DINOAugConfig)
    fuse_normalization: bool = True
    fp8_output: bool = False

    @property
    def output_map(self) -> list[str]:
        return [f"view_{i}" for i in range(self.aug_cfg.n_views)]

    @property
    def norm_stats(self) -> NormStats:
        return self.aug_cfg.norm_stats

    @property
    def initial_global_size(self) -> int:
        return self.aug_cfg.global_crop_size

    @property
    def initial_local_size(self) -> int:
        return self.aug_cfg.local_crop_size

    @property
    def supports_masking(self) -> bool:
        return True

    @property
    def n_views(self) -> int:
        return self.aug_cfg.n_views

    def split_views(self, views: list[Any]) -> tuple[list[Any], list[Any]]:
        n = self.aug_cfg.n_global_crops
        return views[:n], views[n:]


class ResolutionSource:
    """Thread-safe (global, local) crop size holder (reference sources/resolution.py:23-71)."""

    def __init__(self, global_size: int, local_size: int) -> None:
        self._g, self._l = global_size, local_size
        self._lock = threading.Lock()

    def set(self, global_size: int, local_size: int) -> None:
        with self._lock:
            self._g, self._l = global_size, local_size

    def __call__(self):
        with self._lock:
            return np.array(self._g, dtype=np.int32), np.array(self._l, dtype=np.int32)


@dataclass
class EvalAugSpec:
    """Reference ``EvalAugSpec`` (augmentation.py:290-334): resize shorter side + centre crop."""

    crop_size: int = 224
    mean: tuple = (0.485, 0.456, 0.406)
    std: tuple = (0.229, 0.224, 0.225)
    interpolation: str = "bicubic"

    @property
    def output_map(self) -> list[str]:
        return ["view_0"]

    @property
    def norm_stats(self) -> NormStats:
        return NormStats(mean=self.mean, std=self.std)

    @property
    def initial_global_size(self) -> int:
        return self.crop_size

    @property
    def initial_local_size(self) -> int:
        return self.crop_size

    @property
    def supports_masking(self) -> bool:
        return False


@dataclass
class LeJEPAAugSpec:
    """Reference ``LeJEPAAugSpec`` (augmentation.py:336-399): one context crop + N target crops."""

    context_crop_size: int = 224
    target_crop_size: int = 96
    n_target_views: int = 4
    context_scale: tuple = (0.85, 1.0)
    target_scale: tuple = (0.15, 0.30)
    mean: tuple = (0.485, 0.456, 0.406)
    std: tuple = (0.229, 0.224, 0.225)

    @property
    def output_map(self) -> list[str]:
        return ["context", *[f"target_{i}" for i in range(self.n_target_views)]]

    @property
    def norm_stats(self) -> NormStats:
        return NormStats(mean=self.mean, std=self.std)

    @property
    def initial_global_size(self) -> int:
        return self.context_crop_size

    @property
    def initial_local_size(self) -> int:
        return self.target_crop_size

    @property
    def supports_masking(self) -> bool:
        return False


@dataclass
class UserAugSpec:
    """Reference ``UserAugSpec`` (augmentation.py:400-473): decode + resize the shorter side to
    ``decode_size`` + normalise, then ``aug_fn(Tensor[B,C,H,W]) -> dict[str, Tensor]``."""

    aug_fn: Any
    _output_map: list
    decode_size: int = 256
    mean: tuple = (0.485, 0.456, 0.406)
    std: tuple = (0.229, 0.224, 0.225)
    warn_not_dali: bool = True

    @property
    def uses_dali(self) -> bool:
        return False

    @property
    def output_map(self) -> list[str]:
        return self._output_map

    @property
    def n_views(self) -> int:
        return len(self.output_map)

    @property
    def norm_stats(self) -> NormStats:
        return NormStats(mean=self.mean, std=self.std)

    @property
    def initial_global_size(self) -> int:
        return self.decode_size

    @property
    def initial_local_size(self) -> int:
        return self.decode_size

    def split_views(self, views: list) -> tuple[list, list]:
        mid = max(1, len(views) // 2)
        return views[:mid], views[mid:]

    def __post_init__(self) -> None:
        if not callable(self.aug_fn):
            raise TypeError("UserAugSpec.aug_fn must be callable.")
        if not self.output_map:
            raise ValueError("UserAugSpec.output_map must be a non-empty list of view names.")
        if self.decode_size < 1:
            raise ValueError(f"UserAugSpec.decode_size must be >= 1, got {self.decode_size}.")
        if self.warn_not_dali:  # reference augmentation.py:464-473 (same category and text)
            import warnings
            warnings.warn(
                "UserAugSpec: aug_fn runs outside the DALI computation graph. "
                "JPEG decoding still uses the nvjpeg hardware pipeline, but "
                "augmentation ops cannot be fused with decode. "
                "Expect ~10–20% throughput reduction vs. a native DALI pipeline. "
                "Suppress with warn_not_dali=False once acknowledged.",
                UserWarning,
                stacklevel=3,
            )


def resize_shorter_size(width: int, height: int, size: int) -> tuple[int, int]:
    """torchvision ``Resize(size)`` output (w, h) for an int size (``_compute_resized_output_size``):
    the shorter side becomes ``size``, the longer ``int(size * long / short)`` (reference cpu.py:190-191)."""
    if width <= height:
        return size, int(size * height / width)
    return int(size * width / height), size


def recipe_aug_config(spec: Any) -> DINOAugConfig:
    """The view recipe of an Eval / LeJEPA spec as a ``DINOAugConfig`` + ``recipe`` code
    (``DINO_RECIPE_*``), so that the same kernels and sampler serve every spec:

    * LeJEPA (reference cpu.py:447-459): view 0 = context, RandomResizedCrop(context_crop_size,
      context_scale) + ``_color_jitter(ctx, 0.8, 0.8, 0.8, 0.2, 0.8)`` + flip(0.5); views 1..N =
      RandomResizedCrop(target_crop_size, target_scale) only;
    * Eval (reference cpu.py:400-411): one view, resize shorter side to int(S * 256 / 224)
      (BICUBIC) then centre crop S.
    """
    from .params import RECIPE_EVAL, RECIPE_LEJEPA
    kind = type(spec).__name__
    if kind == "LeJEPAAugSpec":
        cfg = DINOAugConfig(global_crop_size=spec.context_crop_size, local_crop_size=spec.target_crop_size,
                            n_global_crops=1, n_local_crops=spec.n_target_views,
                            global_crops_scale=tuple(spec.context_scale), local_crops_scale=tuple(spec.target_scale),
                            blur_prob_global1=0.0, blur_prob_global2=0.0, blur_prob_local=0.0, solarize_prob=0.0,
                            color_jitter_prob=0.8, grayscale_prob=0.0, brightness=0.8, contrast=0.8, saturation=0.8,
                            hue=0.2, flip_prob=0.5, mean=tuple(spec.mean), std=tuple(spec.std))
        cfg.recipe = RECIPE_LEJEPA
        return cfg
    if kind == "EvalAugSpec":
        cfg = DINOAugConfig(global_crop_size=spec.crop_size, local_crop_size=spec.crop_size, n_global_crops=1,
                            n_local_crops=0, blur_prob_global1=0.0, blur_prob_global2=0.0, blur_prob_local=0.0,
                            solarize_prob=0.0, color_jitter_prob=0.0, grayscale_prob=0.0, flip_prob=0.0,
                            mean=tuple(spec.mean), std=tuple(spec.std))
        cfg.recipe = RECIPE_EVAL
        return cfg
    raise TypeError(f"no view recipe for {kind}")
