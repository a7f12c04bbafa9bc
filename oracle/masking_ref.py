"""Transcription of reference ``MaskingGenerator`` (TEST INFRASTRUCTURE ONLY).

Follows reference ``src/dino_loader/masking.py``:
``__init__`` :87-142, ``__call__`` :148-172, ``_place_block`` :193-230,
``_complete_randomly`` :232-269.

The reference draws from the process-global ``random`` and legacy
``numpy.random`` states.  Here the two generators are explicit objects
(``random.Random`` / ``numpy.random.RandomState``), which is bit-identical to
``random.seed(s); np.random.seed(s)`` on the globals (test_masking.py:252-263)
because both module-level APIs are thin wrappers around one such instance.
"""

from __future__ import annotations

import math
import random

import numpy as np

MAX_ATTEMPTS_PER_BLOCK = 10   # masking.py:57


class RefMaskingGenerator:
    def __init__(self, input_size, num_masking_patches=None, min_num_patches=4,
                 max_num_patches=None, min_aspect=0.3, max_aspect=None,
                 py_rng: random.Random | None = None, np_rng: np.random.RandomState | None = None):
        if isinstance(input_size, int):
            input_size = (input_size, input_size)
        self.height, self.width = input_size
        self.num_patches = self.height * self.width
        if num_masking_patches is None:
            num_masking_patches = self.num_patches // 2
        self.num_masking_patches = num_masking_patches
        if self.num_masking_patches > self.num_patches or self.num_masking_patches < 0:
            raise ValueError("num_masking_patches out of range")
        self.min_num_patches = min_num_patches
        self.max_num_patches = num_masking_patches if max_num_patches is None else max_num_patches
        if self.num_masking_patches > 0 and self.min_num_patches > self.max_num_patches:
            raise ValueError("min_num_patches > max_num_patches")
        max_aspect = max_aspect if max_aspect is not None else 1.0 / min_aspect
        self.log_aspect_ratio = (math.log(min_aspect), math.log(max_aspect))
        self.rnd = py_rng if py_rng is not None else random.Random(0)
        self.nprnd = np_rng if np_rng is not None else np.random.RandomState(0)

    def __call__(self, flat: bool = False) -> np.ndarray:
        mask = np.zeros((self.height, self.width), dtype=bool)
        count = 0
        while count < self.num_masking_patches:
            remaining = self.num_masking_patches - count
            cap = min(remaining, self.max_num_patches)
            delta = self._place_block(mask, cap)
            if delta == 0:
                break
            count += delta
        mask = self._complete_randomly(mask, self.num_masking_patches)
        return mask.ravel() if flat else mask

    def _place_block(self, mask, max_patches):
        for _ in range(MAX_ATTEMPTS_PER_BLOCK):
            target_area = self.rnd.uniform(self.min_num_patches, max_patches)
            aspect = math.exp(self.rnd.uniform(*self.log_aspect_ratio))
            h = int(round(math.sqrt(target_area * aspect)))
            w = int(round(math.sqrt(target_area / aspect)))
            if w >= self.width or h >= self.height:
                continue
            top = self.rnd.randint(0, self.height - h)
            left = self.rnd.randint(0, self.width - w)
            new = h * w - int(mask[top:top + h, left:left + w].sum())
            if 0 < new <= max_patches:
                mask[top:top + h, left:left + w] = True
                return new
        return 0

    def _complete_randomly(self, mask, target):
        shortfall = target - int(mask.sum())
        if shortfall <= 0:
            return mask
        unmasked = np.where(~mask.ravel())[0]
        shortfall = min(shortfall, len(unmasked))
        chosen = self.nprnd.choice(unmasked, size=shortfall, replace=False)
        mask.flat[chosen] = True
        return mask
