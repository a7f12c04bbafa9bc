"""The CPU oracle against the committed golden vectors and against Pillow itself.

Pins the oracle: the golden fixtures (tests/golden/, made by make_golden.py)
hold Pillow's decode of each JPEG and the oracle's bf16 views for parameter
records drawn in CPUBackend's order.  If Pillow / torch change underneath, these
tests say so before any GPU comparison is trusted.
"""

from __future__ import annotations

import json
import random
from pathlib import Path

import numpy as np
import pytest
import torch
from PIL import Image, ImageEnhance, ImageOps

from oracle import cpu_ref
from oracle.masking_ref import RefMaskingGenerator
from tests.helpers import record_to_params

GOLD = Path(__file__).resolve().parent / "golden"
META = json.loads((GOLD / "meta.json").read_text())


def test_decode_matches_golden():
    for name in META["jpegs"]:
        data = (GOLD / f"{name}.jpg").read_bytes()
        ref = np.load(GOLD / f"{name}.rgb.npy")
        np.testing.assert_array_equal(np.asarray(cpu_ref.decode_rgb(data)), ref, err_msg=name)


def test_views_match_golden():
    recs = np.load(GOLD / "views.params.npy")
    views = np.load(GOLD / "views.bf16.npz")
    nv = META["views_per_image"]
    k = 0
    for name in META["jpegs"]:
        data = (GOLD / f"{name}.jpg").read_bytes()
        img = cpu_ref.decode_rgb(data)
        for v in range(nv):
            p = record_to_params(recs[k])
            got = cpu_ref.augment_one(data, p, decoded=img).view(torch.int16).numpy().reshape(-1)
            np.testing.assert_array_equal(got, views[f"arr_{k}"], err_msg=f"{name} view {v}")
            k += 1


def test_golden_param_draws_reproduce():
    """draw_params_like_cpubackend replays the committed records from the same seeds."""
    cfg = cpu_ref.AugCfg(global_crop_size=32, local_crop_size=16, n_local_crops=2)
    gen = torch.Generator().manual_seed(0)
    rnd = random.Random(0)
    recs = np.load(GOLD / "views.params.npy")
    k = 0
    for name in META["jpegs"]:
        w, h = cpu_ref.decode_rgb((GOLD / f"{name}.jpg").read_bytes()).size
        for spec in cpu_ref.view_table(cfg):
            p = cpu_ref.draw_params_like_cpubackend(w, h, spec, cfg, gen, rnd)
            assert p == record_to_params(recs[k]), (name, k)
            k += 1


def test_masks_match_golden():
    m = np.load(GOLD / "masks.npz")
    for seed in (0, 1, 42):
        for grid in (14, 16, 37):
            g = RefMaskingGenerator(grid, py_rng=random.Random(seed), np_rng=np.random.RandomState(seed))
            got = np.stack([g(flat=True) for _ in range(4)])
            np.testing.assert_array_equal(got, m[f"seed{seed}_grid{grid}"])


def test_ref_masks_use_global_rng_like_reference():
    """random.seed + np.random.seed on the globals == explicit generator objects (test_masking.py:252-263)."""
    random.seed(42)
    np.random.seed(42)
    a = RefMaskingGenerator(14, py_rng=random, np_rng=np.random.mtrand._rand)(flat=True)
    b = RefMaskingGenerator(14, py_rng=random.Random(42), np_rng=np.random.RandomState(42))(flat=True)
    np.testing.assert_array_equal(a, b)


@pytest.mark.parametrize("grid,target,minp", [(14, 75, 4), (16, 128, 4), (37, 684, 4), (8, 0, 4), (4, 16, 4),
                                             (1, 1, 1)])
def test_ref_mask_exact_count(grid, target, minp):
    g = RefMaskingGenerator(grid, num_masking_patches=target, min_num_patches=minp, py_rng=random.Random(3),
                            np_rng=np.random.RandomState(3))
    for _ in range(3):
        m = g(flat=True)
        assert m.dtype == bool and m.shape == (grid * grid,) and int(m.sum()) == target


def test_oracle_ops_are_pillow_ops():
    """The oracle's jitter ops are literally Pillow's enhancers (torchvision PIL path)."""
    rng = np.random.default_rng(0)
    img = Image.fromarray(rng.integers(0, 256, (20, 30, 3), dtype=np.uint8))
    np.testing.assert_array_equal(np.asarray(cpu_ref.adjust_brightness(img, 1.3)),
                                  np.asarray(ImageEnhance.Brightness(img).enhance(1.3)))
    np.testing.assert_array_equal(np.asarray(cpu_ref.adjust_contrast(img, 0.4)),
                                  np.asarray(ImageEnhance.Contrast(img).enhance(0.4)))
    sol = ImageOps.solarize(img, 128)
    a = np.asarray(img).astype(int)
    np.testing.assert_array_equal(np.asarray(sol), np.where(a >= 128, 255 - a, a))


def test_hue_delta_matches_int8_view():
    for h in np.linspace(-0.5, 0.5, 101, dtype=np.float32):
        assert (int(float(h) * 255) & 0xFF) == int(np.int8(float(h) * 255).view(np.uint8))


def test_gaussian_blur_reflect_semantics():
    """Constant image stays constant; reflect padding, kernel normalised."""
    img = Image.new("RGB", (12, 10), (77, 150, 3))
    out = cpu_ref.gaussian_blur(img, 9, 1.7)
    np.testing.assert_array_equal(np.asarray(out), np.asarray(img))
    k = cpu_ref.gaussian_kernel1d(7, 1.2)
    assert abs(float(k.sum()) - 1.0) < 1e-6 and torch.allclose(k, k.flip(0))


def test_rrc_params_in_bounds():
    gen = torch.Generator().manual_seed(1)
    for w, h in [(640, 480), (50, 400), (400, 50), (1, 1), (3, 2)]:
        for scale in [(0.32, 1.0), (0.05, 0.32)]:
            for _ in range(50):
                i, j, hh, ww = cpu_ref.rrc_get_params(w, h, scale, (3 / 4, 4 / 3), gen)
                assert 0 <= i and 0 <= j and 0 < hh <= h and 0 < ww <= w and i + hh <= h and j + ww <= w


def test_corrupt_jpeg_gives_zeros():
    p = cpu_ref.ViewParams(out_size=32)
    t = cpu_ref.augment_one(b"not a valid jpeg", p)
    assert t.shape == (3, 32, 32) and torch.count_nonzero(t) == 0


def test_r2_decodes_match_golden_hashes(emu):
    """Round-2 fixtures (odd/large sizes, progressive files): Pillow and the kernel model
    (emulator, incl. the progressive k_prog path) both give the committed decode hash."""
    import hashlib

    from tests.helpers import emu_decode
    for name, m in META["jpegs_r2"].items():
        data = (GOLD / f"{name}.jpg").read_bytes()
        ref = np.asarray(cpu_ref.decode_rgb(data), dtype=np.uint8)
        assert ref.shape == (m["height"], m["width"], 3)
        assert hashlib.sha256(ref.tobytes()).hexdigest() == m["rgb_sha256"], name
        r, out, _ = emu_decode(emu, data, 0, 1)
        assert r == 0 and hashlib.sha256(out.tobytes()).hexdigest() == m["rgb_sha256"], name


def test_views224_match_golden():
    """Full DINOAugConfig (2 x 224 + 8 x 96) records and views reproduce from the oracle."""
    g = META["views224"]
    recs = np.load(GOLD / "views224.params.npy")
    views = np.load(GOLD / "views224.bf16.npz")
    cfg = cpu_ref.AugCfg()
    gen = torch.Generator().manual_seed(1)
    rnd = random.Random(1)
    k = 0
    for name in g["jpegs"]:
        data = (GOLD / f"{name}.jpg").read_bytes()
        img = cpu_ref.decode_rgb(data)
        for spec in cpu_ref.view_table(cfg):
            p = cpu_ref.draw_params_like_cpubackend(img.size[0], img.size[1], spec, cfg, gen, rnd)
            assert p == record_to_params(recs[k]), (name, k)
            got = cpu_ref.augment_one(data, p, decoded=img).view(torch.int16).numpy().reshape(-1)
            np.testing.assert_array_equal(got, views[f"arr_{k}"], err_msg=f"{name} view {k}")
            k += 1
