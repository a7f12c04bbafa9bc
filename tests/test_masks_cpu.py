"""The drop-in ``MaskingGenerator`` on the host path (``dino_masks_host``, the C++ twin of
``k_masks``) — no GPU needed.

* bit-exact against the transcription of reference masking.py:148-269
  (oracle/masking_ref.py) for square and non-square grids and edge targets, and
  against the committed golden masks;
* the reference's own pinned assertions, restated from reference
  tests/test_masking.py:137-297 (shape, dtype, exact count, 0 / all / 1x1 targets,
  non-square grids, non-contiguous completion, determinism under
  ``random.seed`` + ``np.random.seed``).
"""

from __future__ import annotations

import random
from pathlib import Path

import numpy as np
import pytest

from dataloader_amd.masking import MaskingGenerator
from oracle.masking_ref import RefMaskingGenerator

GOLD = Path(__file__).resolve().parent / "golden"


def _ref_and_ours(grid, seed, **kw):
    ref = RefMaskingGenerator(grid, py_rng=random.Random(seed), np_rng=np.random.RandomState(seed), **kw)
    ours = MaskingGenerator(grid, **kw)
    random.seed(seed)
    np.random.seed(seed)
    return ref, ours


@pytest.mark.parametrize("grid,kw", [
    ((14, 14), {}), ((16, 16), {}), ((37, 37), {}), ((10, 12), {"num_masking_patches": 40}),
    ((10, 16), {"num_masking_patches": 75}), ((12, 10), {"num_masking_patches": 60, "min_aspect": 0.5}),
    ((8, 8), {"num_masking_patches": 0}), ((4, 4), {"num_masking_patches": 16}),
    ((1, 1), {"num_masking_patches": 1, "min_num_patches": 1}),
    ((2, 2), {"num_masking_patches": 2, "min_num_patches": 1}),
    ((16, 16), {"num_masking_patches": 128, "max_num_patches": 20, "min_num_patches": 8}),
])
def test_host_twin_bit_exact_with_global_side_effects(grid, kw):
    ref, ours = _ref_and_ours(grid, 7, **kw)
    for _ in range(12):
        np.testing.assert_array_equal(ours(flat=True), ref(flat=True))
    # the process-global states advanced exactly as the reference's calls advance them
    assert random.random() == ref.rnd.random()
    assert np.random.randint(1 << 30) == ref.nprnd.randint(1 << 30)


def test_golden_masks():
    g = np.load(GOLD / "masks.npz")
    for key in g.files:  # seed{s}_grid{n}: the first masks after random.seed(s); np.random.seed(s)
        seed, grid = (int(x) for x in key.replace("seed", "").split("_grid"))
        gen = MaskingGenerator((grid, grid))
        random.seed(seed)
        np.random.seed(seed)
        for k in range(g[key].shape[0]):
            np.testing.assert_array_equal(gen(flat=True), g[key][k], err_msg=f"{key}[{k}]")


# ---- reference tests/test_masking.py:137-297, restated ----------------------------
def test_output_shape_and_dtype():
    gen = MaskingGenerator(input_size=(14, 14), num_masking_patches=75)
    assert gen().shape == (14, 14)
    assert gen(flat=True).shape == (196,)
    assert MaskingGenerator(input_size=(8, 8), num_masking_patches=20)().dtype == bool


def test_exact_count():
    gen = MaskingGenerator(input_size=(14, 14), num_masking_patches=75)
    assert all(int(gen().sum()) == 75 for _ in range(50))
    gen = MaskingGenerator(input_size=(8, 8), num_masking_patches=30)
    assert all(int(gen(flat=True).sum()) == 30 for _ in range(10))


def test_edge_targets():
    assert int(MaskingGenerator(input_size=(8, 8), num_masking_patches=0)().sum()) == 0
    assert int(MaskingGenerator(input_size=(4, 4), num_masking_patches=16)().sum()) == 16
    assert int(MaskingGenerator(input_size=(1, 1), num_masking_patches=1, min_num_patches=1)().sum()) == 1


def test_non_square_no_out_of_bounds():
    gen = MaskingGenerator(input_size=(10, 12), num_masking_patches=40)
    for _ in range(20):
        m = gen()
        assert m.shape == (10, 12) and m.dtype == bool and int(m.sum()) == 40


def test_complete_randomly_non_contiguous():
    gen = MaskingGenerator(input_size=(8, 8), num_masking_patches=30)
    mask = np.zeros((8, 8), dtype=bool, order="F")
    assert int(gen._complete_randomly(mask, target=30).sum()) == 30
    base = np.zeros((8, 8), dtype=bool)
    view = base[::2, ::2]
    assert int(MaskingGenerator._complete_randomly(view, target=8).sum()) == 8
    full = np.ones((4, 4), dtype=bool)
    assert int(gen._complete_randomly(full, target=4).sum()) == 16
    small = np.zeros((2, 2), dtype=bool)
    assert int(gen._complete_randomly(small, target=6).sum()) <= 4


def test_determinism_under_global_seeds():
    gen = MaskingGenerator(input_size=(14, 14), num_masking_patches=75)
    np.random.seed(42)
    random.seed(42)
    m1 = gen()
    np.random.seed(42)
    random.seed(42)
    assert np.array_equal(m1, gen())
    masks = [gen() for _ in range(10)]
    assert any(not np.array_equal(a, b) for a, b in zip(masks, masks[1:]))


def test_validation_and_repr():
    with pytest.raises(ValueError):
        MaskingGenerator(input_size=(4, 4), num_masking_patches=17)
    with pytest.raises(ValueError):
        MaskingGenerator(input_size=(4, 4), num_masking_patches=-1)
    with pytest.raises(ValueError):
        MaskingGenerator(input_size=(4, 4), num_masking_patches=8, min_num_patches=9)
    g = MaskingGenerator(16)
    assert g.get_shape() == (16, 16) and "16x16" in repr(g)
