"""Generate the committed golden fixtures (run from the repo root).

    python tests/golden/make_golden.py

Inputs are synthetic JPEGs encoded here with Pillow (no reference code is
involved: the reference cannot be imported).  Expected outputs:
  * decoded RGB from Pillow/libjpeg-turbo (``Image.open(...).convert("RGB")``,
    reference cpu.py:251) — the decoder known-answer vectors;
  * per-view parameter records drawn in CPUBackend's order from
    torch.Generator(0) + random.Random(0), and the bf16 view tensors the oracle
    computes from them (reference cpu.py:235-267, small_aug_cfg of the
    reference's tests/conftest.py:71-84: 32/16 px, 2 + 2 views);
  * iBOT masks from MaskingGenerator's algorithm with random.seed(s) +
    np.random.seed(s) (reference test_masking.py:252-263), seeds {0, 1, 42} x
    grids {14, 16, 37}, first 4 masks;
  * round 2 (SURVEY §8c list): odd and large sizes (225x333, 1601x1203) and
    progressive files (4:2:0 / 4:4:4 / gray / with restart intervals) with the
    SHA-256 of Pillow's decode (large RGB arrays are not committed), and records
    + bf16 views at the reference's full DINOAugConfig (2 x 224 + 8 x 96, drawn in
    CPUBackend's order from torch.Generator(1) + random.Random(1)).
Environment recorded in meta.json (Python / numpy / Pillow / libjpeg-turbo / torch).
"""

from __future__ import annotations

import hashlib
import json
import random
import sys
from pathlib import Path

import numpy as np
import torch

ROOT = Path(__file__).resolve().parents[2]
sys.path.insert(0, str(ROOT))

from dataloader_amd.synthetic import encode_jpeg, textured_rgb  # noqa: E402
from oracle import cpu_ref  # noqa: E402
from oracle.masking_ref import RefMaskingGenerator  # noqa: E402
from tests.helpers import params_to_record  # noqa: E402

OUT = Path(__file__).resolve().parent


def jpeg_cases():
    rng = np.random.default_rng(2024)
    cases = [
        ("s420_64x48", encode_jpeg(textured_rgb(64, 48, rng), quality=85, subsampling=2)),
        ("s422_33x17", encode_jpeg(textured_rgb(33, 17, rng), quality=85, subsampling=1)),
        ("s444_40x40", encode_jpeg(textured_rgb(40, 40, rng), quality=85, subsampling=0)),
        ("q50_71x53", encode_jpeg(textured_rgb(71, 53, rng), quality=50)),
        ("q95_48x64", encode_jpeg(textured_rgb(48, 64, rng), quality=95)),
        ("gray_50x30", encode_jpeg(textured_rgb(50, 30, rng), gray=True)),
        ("dri_96x64", encode_jpeg(textured_rgb(96, 64, rng), restart_mcus=3)),
        ("odd_17x9", encode_jpeg(textured_rgb(17, 9, rng))),
        ("one_1x1", encode_jpeg(textured_rgb(1, 1, rng))),
        ("wide_160x40", encode_jpeg(textured_rgb(160, 40, rng))),
    ]
    return cases


def jpeg_cases_r2():
    """Round-2 additions: larger / odd sizes and progressive files (SHA-256 of the decode)."""
    rng = np.random.default_rng(2025)
    return [
        ("odd_225x333", encode_jpeg(textured_rgb(225, 333, rng), quality=85)),
        ("big_1601x1203", encode_jpeg(textured_rgb(1601, 1203, rng), quality=75)),
        ("prog_640x480", encode_jpeg(textured_rgb(640, 480, rng), quality=85, progressive=True)),
        ("prog444_96x96", encode_jpeg(textured_rgb(96, 96, rng), quality=90, subsampling=0, progressive=True)),
        ("prog_gray_200x150", encode_jpeg(textured_rgb(200, 150, rng), progressive=True, gray=True)),
        ("prog_rst_321x123", encode_jpeg(textured_rgb(321, 123, rng), progressive=True, restart_mcus=5)),
    ]


def views_224(meta):
    """Records + bf16 views at the full DINOAugConfig for two of the round-2 images."""
    cfg = cpu_ref.AugCfg()  # 2 x 224 + 8 x 96, reference defaults (config.py:243-272)
    table = cpu_ref.view_table(cfg)
    gen = torch.Generator().manual_seed(1)
    rnd = random.Random(1)
    names, recs, views = ["odd_225x333", "prog_640x480"], [], []
    for name in names:
        data = (OUT / f"{name}.jpg").read_bytes()
        img = cpu_ref.decode_rgb(data)
        for spec in table:
            p = cpu_ref.draw_params_like_cpubackend(img.size[0], img.size[1], spec, cfg, gen, rnd)
            recs.append(params_to_record(p))
            views.append(cpu_ref.augment_one(data, p, decoded=img).view(torch.int16).numpy().reshape(-1))
    np.save(OUT / "views224.params.npy", np.stack(recs))
    np.savez_compressed(OUT / "views224.bf16.npz", *views)
    meta["views224"] = {"jpegs": names, "views_per_image": len(table), "view_sizes": [s.crop_size for s in table]}


def main():
    meta = {"python": sys.version.split()[0], "numpy": np.__version__, "torch": torch.__version__}
    from PIL import __version__ as pil_version, features
    meta["pillow"] = pil_version
    meta["libjpeg_turbo"] = features.version("libjpeg_turbo")
    cases = jpeg_cases()
    cfg = cpu_ref.AugCfg(global_crop_size=32, local_crop_size=16, n_local_crops=2)
    table = cpu_ref.view_table(cfg)
    gen = torch.Generator().manual_seed(0)
    rnd = random.Random(0)
    names, recs, views = [], [], []
    for name, data in cases:
        (OUT / f"{name}.jpg").write_bytes(data)
        img = cpu_ref.decode_rgb(data)
        np.save(OUT / f"{name}.rgb.npy", np.asarray(img, dtype=np.uint8))
        names.append(name)
        for spec in table:
            p = cpu_ref.draw_params_like_cpubackend(img.size[0], img.size[1], spec, cfg, gen, rnd)
            recs.append(params_to_record(p))
            views.append(cpu_ref.augment_one(data, p, decoded=img).view(torch.int16).numpy().reshape(-1))
    np.save(OUT / "views.params.npy", np.stack(recs))
    np.savez_compressed(OUT / "views.bf16.npz", *views)
    masks = {}
    for seed in (0, 1, 42):
        for grid in (14, 16, 37):
            g = RefMaskingGenerator(grid, py_rng=random.Random(seed), np_rng=np.random.RandomState(seed))
            masks[f"seed{seed}_grid{grid}"] = np.stack([g(flat=True) for _ in range(4)])
    np.savez_compressed(OUT / "masks.npz", **masks)
    meta["jpegs"] = names
    meta["views_per_image"] = len(table)
    meta["view_sizes"] = [s.crop_size for s in table]
    r2 = {}
    for name, data in jpeg_cases_r2():
        (OUT / f"{name}.jpg").write_bytes(data)
        img = np.asarray(cpu_ref.decode_rgb(data), dtype=np.uint8)
        r2[name] = {"width": int(img.shape[1]), "height": int(img.shape[0]),
                    "rgb_sha256": hashlib.sha256(img.tobytes()).hexdigest()}
    meta["jpegs_r2"] = r2
    views_224(meta)
    (OUT / "meta.json").write_text(json.dumps(meta, indent=1))
    print("golden written:", len(names), "jpegs,", len(views), "views,", len(masks), "mask sets")


if __name__ == "__main__":
    main()
