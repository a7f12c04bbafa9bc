#!/usr/bin/env python
"""Host packing throughput of dino_gather_probe (512 C2 JPEGs, ~43 MB, into a pinned staging
buffer) by copier-thread count: the c2_prog leg's prefetch thread packs every batch."""
import sys
import time
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[2]))
import torch  # noqa: E402

import bench  # noqa: E402
from dataloader_amd import fallback  # noqa: E402
from dataloader_amd.config import DINOAugConfig  # noqa: E402
from dataloader_amd.pipeline import make_aug_config  # noqa: E402
from dataloader_amd.tario import spans_of  # noqa: E402

if __name__ == "__main__":
    uniq = bench.make_unique(256, 640, 480, 1, False, 8)
    B = 512
    cfg = make_aug_config(DINOAugConfig(), 224, 96, 0)
    for pin in (False, True):
        buf = torch.empty(64 << 20, dtype=torch.uint8, pin_memory=pin)
        for nt in (1, 2, 4, 8, 16):
            ts = []
            for r in range(8):
                jp = [uniq[(r * 131 + i * 7) % len(uniq)] for i in range(B)]
                ptrs, lens, keep = spans_of(jp)
                t = time.perf_counter()
                fallback.gather_probe(ptrs, lens, buf, nt, 0, cfg)
                ts.append(time.perf_counter() - t)
            ts.sort()
            print(f"pinned={pin} threads={nt:2d} median {ts[4] * 1e3:.2f} ms  best {ts[0] * 1e3:.2f} ms  "
                  f"{lens.sum() / ts[4] / 1e9:.1f} GB/s", flush=True)
