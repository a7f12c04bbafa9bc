#!/usr/bin/env python
"""Decode a batch of 64 progressive 640x480 JPEGs a few times (profiling target for k_prog)."""
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))


def main():
    import torch

    from dataloader_amd.engine import IngestEngine, pack_jpegs
    from dataloader_amd.synthetic import encode_jpeg, textured_rgb
    rng = np.random.default_rng(0)
    jpegs = [encode_jpeg(textured_rgb(640, 480, rng), quality=85, progressive=True) for _ in range(64)]
    dev = torch.device("cuda", 0)
    hb, off = pack_jpegs(jpegs, pin=True)
    d_bytes, d_off = hb.to(dev), off.to(dev)
    eng = IngestEngine(dev, max_batch=64, max_views=10, max_crop_size=224)
    for _ in range(3):
        eng.decode(d_bytes, d_off, 64)
    torch.cuda.synchronize()
    eng.close()
    print("done")


if __name__ == "__main__":
    main()
