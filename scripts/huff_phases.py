#!/usr/bin/env python
"""k_huff1 phase split from an instrumented build (DINO_HUFF_PHASES).

usage: python scripts/huff_phases.py [--mixed]   (builds build/lib_phases.so if missing)
Runs a few device-resident batches of the bench workload, then prints per work item the
mean / max duration of: first decode, sync rounds, write (single-segment items), and
the round counts.
"""
import ctypes
import os
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
LIB = Path(os.environ.get("DINO_PHASE_LIB", ROOT / "build" / "lib_phases.so"))


def main():
    mixed = "--mixed" in sys.argv
    if not LIB.exists():
        from dataloader_amd import build as b
        LIB.parent.mkdir(exist_ok=True)
        b.build(force=True, out=LIB, defines=("DINO_HUFF_PHASES",))
    os.environ["DINO_INGEST_LIB"] = str(LIB)
    import bench
    uniq = bench.make_unique(512, 640, 480, 1, mixed, 0)
    import torch

    from dataloader_amd import _lib
    from dataloader_amd.config import DINOAugConfig
    from dataloader_amd.engine import pack_jpegs
    from dataloader_amd.pipeline import MI355XAugPipeline
    lib = _lib.load()
    lib.dino_debug_huff_phases.argtypes = [ctypes.c_void_p, ctypes.c_int64]
    buf, off = pack_jpegs(uniq, pin=True)
    d_bytes, d_off = buf.to("cuda"), off.to("cuda")
    pipe = MI355XAugPipeline(None, DINOAugConfig(), 512, seed=1, depth=1,
                             workspace_bytes=512 * (40 << 20) if mixed else 0)
    ph = np.zeros((8192, 12), np.uint64)
    for _ in range(2):
        pipe.run_device_batch(d_bytes, d_off, 512)
    torch.cuda.synchronize()
    _lib.check(lib.dino_debug_huff_phases(ph.ctypes.data, 8192), "phases")  # (and zero them)
    pipe.run_device_batch(d_bytes, d_off, 512)
    torch.cuda.synchronize()
    _lib.check(lib.dino_debug_huff_phases(ph.ctypes.data, 8192), "phases")
    used = ph[:, 4] > 0
    ph = ph[used].astype(np.int64)
    t0 = ph[:, 0].min()
    us = lambda a, b: (ph[:, b] - ph[:, a]) / 100.0  # wall_clock64: 100 MHz -> us
    rounds = (ph[:, 5] & 0xFFFFFFFF)
    single = (ph[:, 5] >> 32) & 1
    print(f"items {len(ph)}  single-segment {int(single.sum())}  span {(ph[:, 4].max() - t0) / 100.0:.1f} us")
    for name, d in (("look-back", us(0, 1)), ("first decode", us(1, 2)), ("sync rounds", us(2, 3)),
                    ("write/store", us(3, 4)), ("item", us(0, 4))):
        print(f"  {name:13s} mean {d.mean():8.1f} us  p50 {np.median(d):8.1f}  max {d.max():8.1f}")
    print(f"  rounds mean {rounds.mean():.2f} max {rounds.max()}  hist {np.bincount(rounds)[:8].tolist()}")
    redone = ph[:, 6]
    matched = redone - ph[:, 9]
    print(f"  lanes re-decoded per item mean {redone.mean():.1f} (of 256) max {redone.max()}; unmatched mean "
          f"{ph[:, 9].mean():.2f}; prefix bits mean {ph[:, 7].sum() / max(1, matched.sum()):.0f} "
          f"max-per-item mean {ph[:, 8].mean():.0f} max {ph[:, 8].max()}; emission full {ph[:, 10].mean():.2f}, "
          f"rewritten whole {ph[:, 11].mean():.2f} lanes per item")
    pipe.close()


if __name__ == "__main__":
    main()
