"""Dump per-stage decode outputs of the GPU for a few test images (debug aid)."""
import sys
import numpy as np
import torch
sys.path.insert(0, '.')
from dataloader_amd.engine import IngestEngine, pack_jpegs
from tests.test_gpu_parity import _jpeg_zoo

jpegs = _jpeg_zoo()
dev = torch.device('cuda', 0)
eng = IngestEngine(dev, max_batch=len(jpegs), max_views=10, max_crop_size=224)
buf, off = pack_jpegs(jpegs, pin=False)
info = eng.decode(buf.to(dev), off.to(dev), len(jpegs)).cpu().numpy()
out = {'info': info}
for i in [0, 9, 12, 15, 24]:
    for r in range(5):
        try:
            out[f'img{i}_r{r}'] = eng.debug_region(i, r, 64 << 20).cpu().numpy()
        except Exception as e:
            print('region', i, r, e)
np.savez_compressed('gpurun_out/dbg_decode.npz', **out)
print('saved', info[:5])
