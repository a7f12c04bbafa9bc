"""Diagnosis: which decode path / batch size / depth gives RGB that differs from Pillow."""
import sys
from pathlib import Path

import numpy as np
import torch

ROOT = Path(__file__).resolve().parents[2]
sys.path.insert(0, str(ROOT))
import bench  # noqa: E402
from dataloader_amd.config import DINOAugConfig  # noqa: E402
from dataloader_amd.engine import IngestEngine, pack_jpegs  # noqa: E402
from dataloader_amd.pipeline import MI355XAugPipeline  # noqa: E402
from oracle import cpu_ref  # noqa: E402

uniq = bench.make_unique(1024, 640, 480, 1, False, 16)
refs = {}


def ref(i):
    if i not in refs:
        refs[i] = np.asarray(cpu_ref.decode_rgb(uniq[i]))
    return refs[i]


def check(eng, idx, label, limit=64):
    bad = []
    for b, i in enumerate(idx[:limit]):
        r = ref(i)
        got = eng.copy_rgb(b, r.shape[1], r.shape[0]).cpu().numpy()
        if not np.array_equal(got, r):
            bad.append(b)
    print(f"{label}: {len(bad)} of {min(limit, len(idx))} differ; first {bad[:12]}", flush=True)


dev = torch.device("cuda", 0)
for B in (2, 3, 16, 64, 512):
    idx = list(range(512, 512 + B))
    hb, off = pack_jpegs([uniq[i] for i in idx], pin=True)
    eng = IngestEngine(dev, max_batch=B, max_views=10, max_crop_size=224)
    info = eng.decode(hb.to(dev), off.to(dev), B).cpu().numpy()
    assert (info[:, 0] == 0).all()
    check(eng, idx, f"engine.decode B={B}")
    eng.close()
# the pipeline, device-resident, depth 1 and 3
for depth in (1, 3):
    B = 512
    jp = [uniq[i % 1024] for i in range(6 * B)]
    hb, off = pack_jpegs(jp, pin=True)
    d_bytes, d_off = hb.to(dev), off.to(dev)
    pipe = MI355XAugPipeline(None, DINOAugConfig(), B, seed=1234, device=0, depth=depth)
    for k in range(6):
        pipe.run_device_batch(d_bytes, d_off[k * B:(k + 1) * B + 1], B)
    torch.cuda.synchronize()
    sl = pipe._slots[5 % depth]
    check(sl.engine, [(5 * B + b) % 1024 for b in range(B)], f"pipeline depth={depth} batch 5")
    pipe.close()
