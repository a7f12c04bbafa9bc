"""Huffman phase profile (debug aid): k_huffman wall-clock stamps per image.

usage: DINO_HUFF_PROFILE=1 [DINO_INGEST_LIB=...] python scripts/exp_huff.py [batch]
"""
import ctypes
import os
import sys

sys.path.insert(0, os.getcwd())
import bench  # noqa: E402

if __name__ == "__main__":
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 512
    uniq = bench.make_unique(256, 640, 480, 1, False, 0)
    import numpy as np
    import torch
    from dataloader_amd.engine import IngestEngine, pack_jpegs
    dev = torch.device("cuda", 0)
    jpegs = [uniq[i % len(uniq)] for i in range(B)]
    hb, off = pack_jpegs(jpegs, pin=True)
    d_bytes, d_off = hb.to(dev), off.to(dev)
    eng = IngestEngine(dev, max_batch=B, max_views=10, max_crop_size=224, max_image_dim=2048)
    eng.set_timing(True)
    for _ in range(3):
        eng.decode(d_bytes, d_off, B)
    torch.cuda.synchronize()
    eng.kernel_times()
    for _ in range(5):
        eng.decode(d_bytes, d_off, B)
    kt = eng.kernel_times()
    prof = torch.zeros(B, 8, dtype=torch.int64, device=dev)
    for i in range(B):
        rc = eng.lib.dino_debug_region(eng._ctx, i, 5, ctypes.c_void_p(prof[i].data_ptr()), 64,
                                       ctypes.c_void_p(torch.cuda.current_stream(dev).cuda_stream))
        assert rc == 0, eng.lib.dino_last_error()
    torch.cuda.synchronize()
    p = prof.cpu().numpy().astype(np.float64)
    us = lambda a, b: (p[:, b] - p[:, a]) / 100.0  # 100 MHz wall clock -> us
    print(f"lib={os.environ.get('DINO_INGEST_LIB', 'default')} batch={B}")
    for name, (a, b) in {"tables": (0, 1), "phase1": (1, 2), "sync": (2, 3), "write": (3, 4), "total": (0, 4)}.items():
        v = us(a, b)
        print(f"  {name:7s} mean {v.mean():8.1f} us  max {v.max():8.1f} us")
    print(f"  rounds mean {p[:, 5].mean():.2f} max {p[:, 5].max():.0f}; lanes {p[:, 6].mean():.0f}")
    span = (p[:, 4].max() - p[:, 0].min()) / 100.0
    print(f"  kernel span (first start -> last end) {span:.1f} us")
    for k in ("k_destuff", "k_huffman", "k_dcscan", "k_idct", "k_color"):
        ms, n = kt[k]
        print(f"  {k:10s} {ms / max(n, 1):.4f} ms/launch")
    eng.close()
