#!/usr/bin/env python
"""Lane decoder debugging aid: decode the damaged progressive cases of
tests/test_gpu_round6.py on the GPU (lane path) and through the host lane model
(tests/emu), and report the first differing coefficient per failing image."""
import ctypes
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[2]
sys.path.insert(0, str(ROOT))


def main():
    import torch

    from dataloader_amd import fallback
    from dataloader_amd.engine import IngestEngine, pack_jpegs
    from dataloader_amd.synthetic import encode_jpeg, textured_rgb
    from oracle import cpu_ref
    from tests.helpers import build_emu
    emu = build_emu()
    P = ctypes.c_void_p
    rng = np.random.default_rng(602)
    jpegs = []
    for t in range(70):
        j = bytearray(encode_jpeg(textured_rgb(160 + t, 120, rng), quality=90, progressive=True))
        pos = int(len(j) * (0.15 + 0.8 * (t % 10) / 10))
        for k in range(pos, min(pos + 30 + t, len(j) - 4)):
            if j[k] != 0xFF and j[k - 1] != 0xFF:
                j[k] = (j[k] * 37 + 11 + t) & 0x7F
        jpegs.append(bytes(j))
    dev = torch.device("cuda", 0)
    eng = IngestEngine(dev, max_batch=len(jpegs), max_views=1, max_crop_size=8)
    hb, off = pack_jpegs(jpegs, pin=True)
    info, ws, _ = fallback.probe(hb.data_ptr(), off.numpy(), len(jpegs), 0)
    eng.reserve(ws, 0)
    st = eng.decode(hb.to(dev), off.to(dev), len(jpegs)).cpu().numpy()
    for i in [int(x) for x in (sys.argv[1:] or ["10", "20"])]:
        j = jpegs[i]
        ref = cpu_ref.decode_rgb(j)
        got = eng.copy_rgb(i, int(st[i, 1]), int(st[i, 2])).cpu().numpy()
        print(f"image {i}: status {st[i, 0]}, pixels differing {int((got != np.asarray(ref)).sum())}")
        d = eng.debug_region(i, 0, 1024).cpu().numpy()
        hdr = eng.debug_region(i, 6, 832).cpu().numpy()
        print("  lane flag", int(hdr[776:780].view(np.int32)[0]))
        buf = np.frombuffer(j, np.uint8)
        sizes = np.zeros(3, np.int64)
        cap = 1 << 24
        coef = np.zeros(cap // 2, np.int16)
        rgb = np.zeros(int(st[i, 1]) * int(st[i, 2]) * 3, np.uint8)
        emu.emu_decode_stages(buf.ctypes.data_as(P), ctypes.c_int64(len(j)), 4, 1, rgb.ctypes.data_as(P), None,
                              ctypes.c_int64(0), coef.ctypes.data_as(P), ctypes.c_int64(cap), None, ctypes.c_int64(0),
                              sizes.ctypes.data_as(P))
        n = int(sizes[1])
        host = coef[: n // 2]
        dev_coef = eng.debug_region(i, 2, n).cpu().numpy().view(np.int16)[: n // 2]
        diff = np.nonzero(host != dev_coef)[0]
        print(f"  coef bytes {n}, differing coefficients {len(diff)}")
        if len(diff):
            blk = diff // 64
            print("  first blocks", sorted(set(blk.tolist()))[:12], "positions", (diff[:12] % 64).tolist())
            b0 = int(blk[0])
            print("  host", host[b0 * 64:b0 * 64 + 64].tolist())
            print("  dev ", dev_coef[b0 * 64:b0 * 64 + 64].tolist())
    eng.close()


if __name__ == "__main__":
    main()
