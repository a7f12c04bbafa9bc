"""GPU-backed drop-in for reference ``MaskingGenerator`` (masking.py:60-269).

Same constructor, validation, ``__call__(flat=False)``, ``get_shape()`` and
``__repr__`` as the reference.  The block placement and random completion run
in the HIP kernel ``k_masks`` on CPython-``random`` / legacy-NumPy MT19937
states, so the bits are identical to the reference's.

Two ways to drive it:

* ``gen(flat=...)`` — exact reference semantics including side effects: the
  process-global ``random`` and ``numpy.random`` states are read, advanced by the
  C++ host twin of the kernel (``dino_masks_host``, no GPU stream involved), and
  written back (as the reference consumes them, masking.py:208-262).
* ``gen.generate(n)`` — device-resident fast path: ``n`` masks as a
  ``[n, H*W]`` bool tensor on the GPU from the generator's own state
  (``seed(s)`` == ``random.seed(s); np.random.seed(s)``), no host round trip.
"""

from __future__ import annotations

import ctypes
import math
import random

import numpy as np
import torch

from . import _lib


def _py_state_words(state) -> np.ndarray:
    ver, words, _gauss = state
    return np.asarray(words, dtype=np.uint32)  # 624 + index


def _np_state_words(state) -> np.ndarray:
    _name, key, pos, _hg, _cg = state
    return np.concatenate([np.asarray(key, np.uint32), np.asarray([pos], np.uint32)])


class MaskingGenerator:
    def __init__(self, input_size, num_masking_patches=None, min_num_patches: int = 4,
                 max_num_patches=None, min_aspect: float = 0.3, max_aspect=None, device=None) -> None:
        if isinstance(input_size, int):
            input_size = (input_size, input_size)
        self.height, self.width = input_size
        self.num_patches = self.height * self.width
        if num_masking_patches is None:
            num_masking_patches = self.num_patches // 2
        self.num_masking_patches = num_masking_patches
        if self.num_masking_patches > self.num_patches:
            raise ValueError(f"MaskingGenerator: num_masking_patches={num_masking_patches} exceeds grid size "
                             f"({self.height}x{self.width}={self.num_patches}).")
        if self.num_masking_patches < 0:
            raise ValueError(f"MaskingGenerator: num_masking_patches must be >= 0, got {num_masking_patches}.")
        self.min_num_patches = min_num_patches
        self.max_num_patches = num_masking_patches if max_num_patches is None else max_num_patches
        if self.num_masking_patches > 0 and self.min_num_patches > self.max_num_patches:
            raise ValueError(f"MaskingGenerator: min_num_patches={min_num_patches} > "
                             f"max_num_patches={self.max_num_patches}.")
        eff_max = max_aspect if max_aspect is not None else 1.0 / min_aspect
        self.log_aspect_ratio = (math.log(min_aspect), math.log(eff_max))
        self._device = torch.device(device) if device is not None else None
        self._py = None
        self._np = None

    # --------------------------------------------------------------- helpers
    @property
    def device(self) -> torch.device:
        if self._device is None:
            self._device = torch.device("cuda", torch.cuda.current_device())
        return self._device

    def _run(self, n: int, py: torch.Tensor, npst: torch.Tensor) -> torch.Tensor:
        lib = _lib.load()
        out = torch.empty(max(n, 1), self.height * self.width, dtype=torch.bool, device=self.device)
        stream = ctypes.c_void_p(torch.cuda.current_stream(self.device).cuda_stream)
        _lib.check(lib.dino_masks(self.height, self.width, self.num_masking_patches, self.min_num_patches,
                                  self.max_num_patches, self.log_aspect_ratio[0], self.log_aspect_ratio[1], n,
                                  ctypes.c_void_p(py.data_ptr()), ctypes.c_void_p(npst.data_ptr()),
                                  ctypes.c_void_p(out.data_ptr()), stream), "dino_masks")
        return out[:n]

    def seed(self, s: int) -> None:
        """Own state == ``random.seed(s); np.random.seed(s)``."""
        self._py = torch.from_numpy(_py_state_words(random.Random(s).getstate()).copy()).to(self.device)
        self._np = torch.from_numpy(_np_state_words(np.random.RandomState(s).get_state()).copy()).to(self.device)

    def generate(self, n: int) -> torch.Tensor:
        """``n`` consecutive masks from the generator's own device-resident state."""
        if self._py is None:
            self.seed(0)
        return self._run(n, self._py, self._np)

    # ------------------------------------------------------------ reference API
    def __call__(self, flat: bool = False) -> np.ndarray:
        """Reference ``MaskingGenerator.__call__`` (masking.py:148-172): one mask from the
        process-global ``random`` / ``numpy.random`` states, advanced exactly as the
        reference advances them.  Runs the C++ host twin of ``k_masks``
        (``dino_masks_host``): no GPU stream is touched or synchronised."""
        py_state = random.getstate()
        np_state = np.random.get_state()
        pyw = _py_state_words(py_state).copy()
        npw = _np_state_words(np_state).copy()
        mask = np.empty(self.height * self.width, np.bool_)
        lib = _lib.load()
        vp = ctypes.c_void_p
        _lib.check(lib.dino_masks_host(self.height, self.width, self.num_masking_patches, self.min_num_patches,
                                       self.max_num_patches, self.log_aspect_ratio[0], self.log_aspect_ratio[1], 1,
                                       pyw.ctypes.data_as(vp), npw.ctypes.data_as(vp), mask.ctypes.data_as(vp)),
                   "dino_masks_host")
        random.setstate((py_state[0], tuple(int(x) for x in pyw), py_state[2]))
        np.random.set_state((np_state[0], npw[:624].astype(np.uint32), int(npw[624]), np_state[3], np_state[4]))
        mask = mask.reshape(self.height, self.width)
        return mask.ravel() if flat else mask

    @staticmethod
    def _complete_randomly(mask: np.ndarray, target: int) -> np.ndarray:
        """Reference ``_complete_randomly`` (masking.py:232-269): fill up to ``target`` masked
        patches at random positions drawn with ``np.random.choice`` (legacy global state),
        in place, also on non-contiguous arrays."""
        shortfall = target - int(mask.sum())
        if shortfall <= 0:
            return mask
        unmasked = np.flatnonzero(~mask.ravel())  # C order, like the reference's ravel
        shortfall = min(shortfall, unmasked.size)
        chosen = np.random.choice(unmasked, size=shortfall, replace=False)
        mask.flat[chosen] = True  # in place whatever the memory layout
        return mask

    def get_shape(self) -> tuple[int, int]:
        return self.height, self.width

    def __repr__(self) -> str:
        return (f"MaskingGenerator({self.height}x{self.width} -> [{self.min_num_patches}~{self.max_num_patches}] "
                f"target={self.num_masking_patches}, log_aspect=[{self.log_aspect_ratio[0]:.3f}, "
                f"{self.log_aspect_ratio[1]:.3f}])")
