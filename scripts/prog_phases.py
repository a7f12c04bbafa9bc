#!/usr/bin/env python
"""k_prog per-scan timing from an instrumented build (DINO_PROG_PHASES), analysis aid.

usage: python scripts/prog_phases.py   (builds build/lib_progph.so if missing)
Decodes a batch of 64 progressive 640x480 JPEGs and prints, per scan of the first
image, its level, band, duration (us) and the host model's symbol count, then the
per-level critical path (max over the batch) and the cycles per symbol."""
import ctypes
import os
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
LIB = Path(os.environ.get("DINO_PROGPH_LIB", str(ROOT / "build" / "lib_progph.so")))


def main():
    if not LIB.exists():
        from dataloader_amd import build as b
        LIB.parent.mkdir(exist_ok=True)
        b.build(force=True, out=LIB, defines=("DINO_PROG_PHASES",))
    os.environ["DINO_INGEST_LIB"] = str(LIB)
    import torch

    from dataloader_amd import _lib
    from dataloader_amd.engine import IngestEngine, pack_jpegs
    from dataloader_amd.synthetic import encode_jpeg, textured_rgb
    from tests.helpers import build_emu
    rng = np.random.default_rng(0)
    jpegs = [encode_jpeg(textured_rgb(640, 480, rng), quality=85, progressive=True) for _ in range(64)]
    emu = build_emu()
    buf = np.frombuffer(jpegs[0], np.uint8)
    sym = np.zeros(64, np.int64)
    lv = np.zeros(64, np.int32)
    P = ctypes.c_void_p
    n = emu.emu_prog_scan_stats(buf.ctypes.data_as(P), ctypes.c_int64(len(jpegs[0])), sym.ctypes.data_as(P),
                                lv.ctypes.data_as(P), 64)
    lib = _lib.load()
    lib.dino_debug_prog_phases.argtypes = [ctypes.c_void_p]
    dev = torch.device("cuda", 0)
    hb, off = pack_jpegs(jpegs, pin=True)
    d_bytes, d_off = hb.to(dev), off.to(dev)
    eng = IngestEngine(dev, max_batch=64, max_views=10, max_crop_size=224)
    for _ in range(2):
        eng.decode(d_bytes, d_off, 64)
    torch.cuda.synchronize()
    ph = np.zeros((64, 64, 3), np.uint64)
    _lib.check(lib.dino_debug_prog_phases(ph.ctypes.data), "phases")
    dur = (ph[:, :, 1].astype(np.int64) - ph[:, :, 0].astype(np.int64)) / 100.0  # 100 MHz -> us
    print(f"scans {n}")
    for i in range(n):
        meta = int(ph[0, i, 2])
        ss, se, ah, al = (meta >> 8) & 255, (meta >> 16) & 255, (meta >> 24) & 15, (meta >> 28) & 15
        cyc = dur[:, i].max() * 2400 / max(sym[i], 1)
        print(f"  scan {i}: level {meta & 255} band {ss}-{se} ah {ah} al {al}  {dur[0, i]:8.1f} us (max {dur[:, i].max():8.1f})"
              f"  symbols {sym[i]:6d}  ~{cyc:6.0f} cycles/symbol")
    for level in range(int(lv[:n].max()) + 1):
        idx = [i for i in range(n) if lv[i] == level]
        print(f"  level {level}: max scan {dur[:, idx].max():8.1f} us")
    # per image: first scan start -> last scan end (the scans' critical path, with pipelining)
    st, en = ph[:, :n, 0].astype(np.int64), ph[:, :n, 1].astype(np.int64)
    span = (en.max(axis=1) - st.min(axis=1)) / 100.0
    print(f"  image makespan (first scan start -> last scan end): mean {span.mean():8.1f} us, max {span.max():8.1f} us")
    eng.close()


if __name__ == "__main__":
    main()
