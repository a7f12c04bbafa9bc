"""Debug aid: decode progressive JPEGs on the GPU and compare the coefficient buffer of
each with the host model's (tests/emu): first differing block per component and the
zigzag positions that differ.  usage: python scripts/gpu_debug_prog.py [jpeg ...]"""
import ctypes
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))


def main():
    import torch

    from dataloader_amd.engine import IngestEngine, pack_jpegs
    from tests.helpers import build_emu
    files = sys.argv[1:] or [str(ROOT / "tests" / "golden" / "prog_640x480.jpg")]
    jpegs = [Path(f).read_bytes() for f in files]
    emu = build_emu()
    dev = torch.device("cuda", 0)
    hb, off = pack_jpegs(jpegs, pin=True)
    eng = IngestEngine(dev, max_batch=len(jpegs), max_views=1, max_crop_size=8)
    info = eng.decode(hb.to(dev), off.to(dev), len(jpegs)).cpu().numpy()
    print("info", info.tolist())
    P = ctypes.c_void_p
    for i, j in enumerate(jpegs):
        buf = np.frombuffer(j, np.uint8)
        cap = 64 << 20
        coef = np.zeros(cap // 2, np.int16)
        sizes = np.zeros(3, np.int64)
        rgb = np.zeros(16384 * 16384 * 3 // 64, np.uint8)
        r = emu.emu_decode_stages(buf.ctypes.data_as(P), ctypes.c_int64(len(j)), 0, 1, rgb.ctypes.data_as(P), None,
                                  ctypes.c_int64(0), coef.ctypes.data_as(P), ctypes.c_int64(cap), None,
                                  ctypes.c_int64(0), sizes.ctypes.data_as(P))
        n = int(sizes[1])
        ref = coef[: n // 2]
        got = eng.debug_region(i, 2, n).cpu().numpy().view(np.int16)[: n // 2]
        bad = np.flatnonzero(ref != got)
        print(f"image {i}: emu status {r}, {n // 128} blocks, {len(bad)} coefficients differ")
        if len(bad):
            blocks = np.unique(bad // 64)
            print("  first blocks", blocks[:10].tolist(), "count", len(blocks))
            b = blocks[0]
            print("  positions", (bad[bad // 64 == b] % 64).tolist())
            print("  ref", ref[b * 64:(b + 1) * 64].tolist())
            print("  got", got[b * 64:(b + 1) * 64].tolist())
    eng.close()


if __name__ == "__main__":
    main()
