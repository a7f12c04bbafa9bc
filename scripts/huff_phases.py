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
    for _ in range(3):
        pipe.run_device_batch(d_bytes, d_off, 512)
    torch.cuda.synchronize()
    ph = np.zeros((8192, 5), np.uint64)
    _lib.check(lib.dino_debug_huff_phases(ph.ctypes.data, 8192), "phases")
    used = ph[:, 3] > 0
    ph = ph[used].astype(np.int64)
    t0 = ph[:, 0].min()
    d1 = (ph[:, 1] - ph[:, 0]) / 100.0  # wall_clock64: 100 MHz -> us
    d2 = (ph[:, 2] - ph[:, 1]) / 100.0
    d3 = (ph[:, 3] - ph[:, 2]) / 100.0
    rounds = (ph[:, 4] & 0xFFFFFFFF)
    single = (ph[:, 4] >> 32) & 1
    print(f"items {len(ph)}  single-segment {int(single.sum())}  span {(ph[:, 3].max() - t0) / 100.0:.1f} us")
    for name, d in (("first decode", d1), ("sync rounds", d2), ("write/store", d3)):
        print(f"  {name:13s} mean {d.mean():8.1f} us  p50 {np.median(d):8.1f}  max {d.max():8.1f}")
    print(f"  rounds mean {rounds.mean():.2f} max {rounds.max()}  hist {np.bincount(rounds)[:8].tolist()}")
    pipe.close()


if __name__ == "__main__":
    main()
