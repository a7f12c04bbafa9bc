"""Per-dataset normalisation tables on CPU (reference NormSource pipeline.py:109-180,
build_norm_arrays norm_utils.py:51-88) and the dino_set_norm argument checks."""

from __future__ import annotations

import numpy as np

from dataloader_amd.config import DINOAugConfig, NormStats
from dataloader_amd.norm import NormTable, build_norm_arrays


class _Spec:
    def __init__(self, mean=None, std=None):
        self.mean, self.std = mean, std


def test_norm_table_lookup_and_fallback():
    cfg = DINOAugConfig()
    t = NormTable(cfg, [_Spec(), _Spec((0.5, 0.5, 0.5), (0.25, 0.25, 0.25))])
    t.set_dataset_indices([1, 0, 5])
    r = t.batch_records(4)  # short index list: the last index repeats
    assert r.dtype == np.float32 and r.shape == (4, 6)
    np.testing.assert_array_equal(r[0], np.float32([0.5, 0.5, 0.5, 0.25, 0.25, 0.25]))
    np.testing.assert_array_equal(r[1], np.float32(list(cfg.mean) + list(cfg.std)))
    np.testing.assert_array_equal(r[2], r[0])  # index past the table -> last entry
    np.testing.assert_array_equal(r[3], r[2])


def test_build_norm_arrays_matches_reference_rules():
    fb = NormStats()
    table = [NormStats((0.1, 0.2, 0.3), (0.4, 0.5, 0.6)), NormStats((0.7, 0.8, 0.9), (0.3, 0.2, 0.1))]
    m, s = build_norm_arrays([], table, fb)
    assert m.shape == (1, 3) and m.dtype == np.float32
    np.testing.assert_array_equal(m[0], np.array(fb.mean, np.float32) * np.float32(255.0))
    m, s = build_norm_arrays([0, 1, 9], table, fb)
    np.testing.assert_array_equal(m[2], np.array(table[1].mean, np.float32) * np.float32(255.0))
    np.testing.assert_array_equal(s[0], np.array(table[0].std, np.float32) * np.float32(255.0))


def test_set_norm_rejects_bad_arguments():
    import ctypes

    from dataloader_amd import _lib
    lib = _lib.load()
    assert lib.dino_set_norm(None, None, 0) == -1
    assert b"null ctx" in lib.dino_last_error()
