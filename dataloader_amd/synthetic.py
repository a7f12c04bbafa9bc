"""Synthetic textured JPEG generation for tests and benchmarks.

The reference fixtures encode *solid-colour* JPEGs (reference
``tests/fixtures/__init__.py:54-64``), ~5 KB at 640x480, which make Huffman
decoding trivial.  These images are textured (a smooth random colour field,
a few hard-edged shapes and pixel noise) so that q85 4:2:0 lands around
1.5-2.5 bits/pixel, like natural photographs.

Also writes WebDataset-style tar shards (``sample_%06d.jpg`` + ``.json``) in the
layout of the reference fixtures (``tests/fixtures/__init__.py:80-139``).
"""

from __future__ import annotations

import io
import json
import tarfile

import numpy as np
from PIL import Image


def textured_rgb(width: int, height: int, rng: np.random.Generator, noise: float = 10.0) -> np.ndarray:
    gw, gh = max(2, width // 24), max(2, height // 24)
    field = rng.integers(0, 256, size=(gh, gw, 3), dtype=np.uint8)
    base = np.asarray(Image.fromarray(field, "RGB").resize((width, height), Image.BILINEAR), dtype=np.float32)
    # a few hard-edged rectangles / discs for high-frequency structure
    yy, xx = np.mgrid[0:height, 0:width]
    for _ in range(int(rng.integers(3, 8))):
        col = rng.integers(0, 256, size=3).astype(np.float32)
        cx, cy = rng.integers(0, width), rng.integers(0, height)
        r = rng.integers(max(4, min(width, height) // 16), max(8, min(width, height) // 4))
        if rng.random() < 0.5:
            m = (xx - cx) ** 2 + (yy - cy) ** 2 < r * r
        else:
            m = (abs(xx - cx) < r) & (abs(yy - cy) < r // 2 + 1)
        base[m] = 0.35 * base[m] + 0.65 * col
    base += rng.normal(0.0, noise, size=base.shape).astype(np.float32)
    return np.clip(base + 0.5, 0, 255).astype(np.uint8)


def encode_jpeg(rgb: np.ndarray, quality: int = 85, subsampling: int | str = -1,
                restart_mcus: int = 0, progressive: bool = False, gray: bool = False) -> bytes:
    img = Image.fromarray(rgb, "RGB")
    if gray:
        img = img.convert("L")
    buf = io.BytesIO()
    kw = dict(format="JPEG", quality=quality, progressive=progressive)
    if not gray and subsampling != -1:
        kw["subsampling"] = subsampling
    if restart_mcus:
        kw["restart_marker_blocks"] = restart_mcus
    img.save(buf, **kw)
    return buf.getvalue()


def make_jpeg(width: int, height: int, seed: int, quality: int = 85, **kw) -> bytes:
    rng = np.random.default_rng(seed)
    return encode_jpeg(textured_rgb(width, height, rng), quality=quality, **kw)


def make_dataset(n: int, width: int = 640, height: int = 480, seed: int = 0, quality: int = 85,
                 mixed: bool = False, min_short: int = 224, max_short: int = 1600) -> list[bytes]:
    """``n`` textured JPEGs.  ``mixed``: short side ~ U{min_short..max_short}, aspect U[3/4,4/3]."""
    rng = np.random.default_rng(seed)
    out = []
    for k in range(n):
        if mixed:
            short = int(rng.integers(min_short, max_short + 1))
            aspect = float(rng.uniform(0.75, 4.0 / 3.0))
            long_ = max(short, int(round(short * max(aspect, 1.0 / aspect))))
            w, h = (long_, short) if rng.random() < 0.5 else (short, long_)
        else:
            w, h = width, height
        out.append(encode_jpeg(textured_rgb(w, h, np.random.default_rng([seed, k])), quality=quality))
    return out


def write_shard_tar(path: str, jpegs: list[bytes], with_metadata: bool = True) -> None:
    with tarfile.open(path, "w") as tf:
        for i, data in enumerate(jpegs):
            key = f"sample_{i:06d}"
            ti = tarfile.TarInfo(f"{key}.jpg")
            ti.size = len(data)
            tf.addfile(ti, io.BytesIO(data))
            if with_metadata:
                meta = json.dumps({"quality_score": 1.0, "caption": f"synthetic {i}"}).encode()
                tj = tarfile.TarInfo(f"{key}.json")
                tj.size = len(meta)
                tf.addfile(tj, io.BytesIO(meta))
