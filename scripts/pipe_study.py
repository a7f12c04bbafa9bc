"""Pipelined ms per C2 step of the decode half, the augment half and the whole step, at
several depths (batches in flight, one ctx + stream each).  Analysis aid:
    python scripts/pipe_study.py [steps] [depths e.g. 1,2,3,4]
"""
import os
import sys
import time

sys.path.insert(0, os.getcwd())
import bench  # noqa: E402

if __name__ == "__main__":
    steps = int(sys.argv[1]) if len(sys.argv) > 1 else 30
    depths = [int(x) for x in (sys.argv[2] if len(sys.argv) > 2 else "1,2,3,4").split(",")]
    B = 512
    uniq = bench.make_unique(1024, 640, 480, 1, False, 16)
    import torch
    from dataloader_amd.config import DINOAugConfig
    from dataloader_amd.engine import IngestEngine, pack_jpegs
    from dataloader_amd.params import make_aug_config
    dev = torch.device("cuda", 0)
    jpegs = [uniq[i % len(uniq)] for i in range(4 * B)]
    hb, off = pack_jpegs(jpegs, pin=True)
    d_bytes, d_off = hb.to(dev), off.to(dev)
    cfg = make_aug_config(DINOAugConfig(), 224, 96, 0)
    maxd = max(depths)
    engs = [IngestEngine(dev, max_batch=B, max_views=10, max_crop_size=224, max_image_dim=2048,
                         stream=torch.cuda.Stream(dev)) for _ in range(maxd)]
    views = [e.alloc_views(cfg, B) for e in engs]
    params = []
    for k, e in enumerate(engs):  # decode once so that augment-only has images to work on
        s = (k % 4) * B
        _, _ = e.run_batch(d_bytes, d_off[s:s + B + 1], B, cfg, 1, k, views=views[k])
        params.append(e.sample_params(cfg, 1, k))
    torch.cuda.synchronize()

    def run(kind, depth):
        def one(k):
            e = engs[k % depth]
            s = (k % 4) * B
            if kind == "decode":
                e.decode(d_bytes, d_off[s:s + B + 1], B)
            elif kind == "augment":
                e.augment(cfg, params[k % depth], views=views[k % depth])
            else:
                e.run_batch(d_bytes, d_off[s:s + B + 1], B, cfg, 1, k, views=views[k % depth])
        for k in range(2 * depth):
            one(k)
        torch.cuda.synchronize()
        t = time.perf_counter()
        for k in range(steps):
            one(k)
        torch.cuda.synchronize()
        return (time.perf_counter() - t) / steps * 1e3

    # split: per slot a high-priority decode stream and a normal augment stream, so that
    # the next batch's decode is dispatched ahead of this batch's augment workgroups
    lo, hi = torch.cuda.Stream.priority_range()
    orig = [e.stream for e in engs]
    dstreams = [torch.cuda.Stream(dev, priority=hi) for _ in range(maxd)]
    astreams = [torch.cuda.Stream(dev, priority=lo) for _ in range(maxd)]

    def run_split(depth, prio=True):
        def one(k):
            j = k % depth
            e = engs[j]
            s = (k % 4) * B
            ds = dstreams[j] if prio else orig[j]
            as_ = astreams[j]
            ds.wait_stream(as_)  # the ctx's workspaces: the slot's previous augment is done
            e.stream = ds
            e.decode(d_bytes, d_off[s:s + B + 1], B)
            e.sample_params(cfg, 1, k, out=params[j])
            as_.wait_stream(ds)
            e.stream = as_
            e.augment(cfg, params[j], views=views[j])
        for k in range(2 * depth):
            one(k)
        torch.cuda.synchronize()
        t = time.perf_counter()
        for k in range(steps):
            one(k)
        torch.cuda.synchronize()
        ms = (time.perf_counter() - t) / steps * 1e3
        for j, e in enumerate(engs):
            e.stream = orig[j]
        return ms

    print("priority range", lo, hi, flush=True)
    for d in depths:
        r = {kind: round(run(kind, d), 3) for kind in ("decode", "augment", "full")}
        r["split_prio"] = round(run_split(d, True), 3)
        r["split_noprio"] = round(run_split(d, False), 3)
        print(f"depth {d}: ms/step {r}", flush=True)
