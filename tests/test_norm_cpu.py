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


def test_eval_geometry_follows_torchvision_rules():
    from oracle.cpu_ref import eval_geometry
    # Resize(256) of the shorter side, long side int(256 * long / short); CenterCrop offsets
    # int(round((dim - 224) / 2.0)) with Python's half-to-even round
    assert eval_geometry(640, 480, 224) == (341, 256, 58, 16)
    assert eval_geometry(480, 640, 224) == (256, 341, 16, 58)
    assert eval_geometry(256, 256, 224) == (256, 256, 16, 16)
    assert eval_geometry(300, 257, 224) == (298, 256, 37, 16)


def test_recipe_configs_and_spec_dispatch():
    import pytest

    from dataloader_amd.backend import MI355XBackend
    from dataloader_amd.config import EvalAugSpec, LeJEPAAugSpec, PipelineConfig, recipe_aug_config
    from dataloader_amd.params import RECIPE_EVAL, RECIPE_LEJEPA, make_aug_config
    c = recipe_aug_config(LeJEPAAugSpec(n_target_views=5))
    assert (c.n_global_crops, c.n_local_crops, c.global_crop_size, c.local_crop_size) == (1, 5, 224, 96)
    k = make_aug_config(c, 224, 96, 0)
    assert k.recipe == RECIPE_LEJEPA and k.color_jitter_prob == pytest.approx(0.8) and k.blur_prob_local == 0
    e = make_aug_config(recipe_aug_config(EvalAugSpec(crop_size=192)), 192, 192, 0)
    assert e.recipe == RECIPE_EVAL and (e.n_global, e.n_local, e.global_size) == (1, 0, 192)

    class SomeOtherSpec:  # not a recipe the backend knows: TypeError, as cpu.py:708-709
        pass

    with pytest.raises(TypeError):
        MI355XBackend().build_pipeline(None, SomeOtherSpec(), PipelineConfig(), None)
