"""Per-dataset normalisation (reference ``NormSource``, ``pipeline.py:109-180``, and
``build_norm_arrays``, ``norm_utils.py:51-88``).

In the reference this is DALI-only: the CPU backend normalises every sample with
the global ``DINOAugConfig.mean/std``.  Here it is a device epilogue option of the
same kernels: each image of a batch gets the {mean, std} of its source dataset,
looked up from the dataset indices the mixing source reports through
``register_dataset_index_callback`` (``shard_reader.py:386-395``).
"""

from __future__ import annotations

import threading
from typing import Any, Sequence

import numpy as np

from .config import NormStats


def _stats(mean, std, fallback: NormStats) -> NormStats:
    """``NormStats.from_config``: a dataset without its own stats uses the global ones."""
    if mean is None or std is None:
        return fallback
    return NormStats(tuple(float(x) for x in mean), tuple(float(x) for x in std))


class NormTable:
    """Lookup of per-dataset stats + the current batch's dataset indices (thread-safe,
    copy-on-write like the reference's ``set_dataset_indices``)."""

    def __init__(self, aug_cfg: Any, specs: Sequence[Any]) -> None:
        self.fallback = NormStats(tuple(aug_cfg.mean), tuple(aug_cfg.std))
        self.table = [_stats(getattr(s, "mean", None), getattr(s, "std", None), self.fallback) for s in specs]
        self._indices: list[int] = [0]
        self._lock = threading.Lock()

    def set_dataset_indices(self, indices: Sequence[int]) -> None:
        new = [int(i) for i in indices]
        with self._lock:
            self._indices = new

    def batch_records(self, batch: int) -> np.ndarray:
        """float32 [batch, 6] = mean[3], std[3] in [0, 1] scale, one row per image."""
        with self._lock:
            idx = list(self._indices)
        if not idx:
            idx = [0]
        n = len(self.table)
        out = np.empty((batch, 6), np.float32)
        for b in range(batch):
            i = idx[b] if b < len(idx) else idx[-1]
            st = self.table[min(max(i, 0), n - 1)] if n else self.fallback
            out[b, :3] = st.mean
            out[b, 3:] = st.std
        return out


def build_norm_arrays(indices: Sequence[int], norm_table: Sequence[NormStats],
                      fallback: NormStats) -> tuple[np.ndarray, np.ndarray]:
    """Reference ``build_norm_arrays`` (norm_utils.py:51-88): per-sample (means, stds),
    float32 (B, 3), in [0, 255] scale; empty indices -> one row of the fallback;
    an index past the table uses its last entry."""
    if not indices:
        m = np.asarray(fallback.mean, np.float32)[None] * 255.0
        s = np.asarray(fallback.std, np.float32)[None] * 255.0
        return m.astype(np.float32), s.astype(np.float32)
    n = len(norm_table)
    means = np.stack([np.asarray(norm_table[min(i, n - 1)].mean, np.float32) * np.float32(255.0) for i in indices])
    stds = np.stack([np.asarray(norm_table[min(i, n - 1)].std, np.float32) * np.float32(255.0) for i in indices])
    return means, stds
