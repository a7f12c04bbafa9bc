#!/usr/bin/env python
"""Progressive-only decode capacity (analysis aid): one ``decode`` launch of N progressive
640x480 JPEGs, N = 16 .. 512, and N concurrent launches of 16 on separate streams.

usage: python scripts/prog_scale.py [--ns 16,64,256,512] [--reps 5]
Prints one JSON line per case: images per launch, ms per launch, progressive img/s.  The
mixed-batch bound follows: with k progressive per 256-image batch, a route can reach at
most prog_img_s * 256 / k img/s."""
import argparse
import json
import sys
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ns", default="16,64,256,512")
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--streams", default="4,16")
    a = ap.parse_args()
    import torch

    from dataloader_amd import fallback
    from dataloader_amd.engine import IngestEngine, pack_jpegs
    from dataloader_amd.synthetic import encode_jpeg, textured_rgb
    rng = np.random.default_rng(0)
    base = [encode_jpeg(textured_rgb(640, 480, rng), quality=85, progressive=True) for _ in range(32)]
    dev = torch.device("cuda", 0)
    nmax = max(int(x) for x in a.ns.split(","))
    jpegs = [base[i % len(base)] for i in range(nmax)]
    for n in [int(x) for x in a.ns.split(",")]:
        hb, off = pack_jpegs(jpegs[:n], pin=True)
        d_bytes, d_off = hb.to(dev), off.to(dev)
        eng = IngestEngine(dev, max_batch=n, max_views=1, max_crop_size=8)
        eng.reserve(fallback.probe(hb.data_ptr(), off.numpy(), n, 0)[1], 0)
        info = eng.decode(d_bytes, d_off, n)
        torch.cuda.synchronize()
        assert int((info[:, 0] != 0).sum()) == 0, info[:, 0]
        t0 = time.perf_counter()
        for _ in range(a.reps):
            eng.decode(d_bytes, d_off, n)
        torch.cuda.synchronize()
        ms = (time.perf_counter() - t0) * 1e3 / a.reps
        print(json.dumps({"case": "one_launch", "images": n, "ms_per_launch": round(ms, 2),
                          "prog_img_s": round(n * 1e3 / ms, 1)}), flush=True)
        eng.close()
    # concurrent launches of 16 images on separate streams (the side path's shape)
    hb, off = pack_jpegs(jpegs[:16], pin=True)
    d_bytes, d_off = hb.to(dev), off.to(dev)
    for ns in [int(x) for x in a.streams.split(",")]:
        streams = [torch.cuda.Stream(device=dev) for _ in range(ns)]
        engs = [IngestEngine(dev, max_batch=16, max_views=1, max_crop_size=8, stream=s) for s in streams]
        ws = fallback.probe(hb.data_ptr(), off.numpy(), 16, 0)[1]
        for e in engs:
            e.reserve(ws, 0)
            e.decode(d_bytes, d_off, 16)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(a.reps):
            for e in engs:
                e.decode(d_bytes, d_off, 16)
        torch.cuda.synchronize()
        ms = (time.perf_counter() - t0) * 1e3 / a.reps
        print(json.dumps({"case": "streams", "streams": ns, "images": 16 * ns, "ms_per_round": round(ms, 2),
                          "prog_img_s": round(16 * ns * 1e3 / ms, 1)}), flush=True)
        for e in engs:
            e.close()


if __name__ == "__main__":
    main()
