"""What slows the e2e feed's host half down?  The prefetch-thread work (next_batch_spans +
dino_gather_probe into pinned staging) timed alone and next to each kind of main-thread
load: a Python busy loop (GIL), a loop of 43 MB pinned H2D copies (host memory / DMA), and
the device-resident Stage-3 loop (launch thread + GPU).
usage: python scripts/e2e_study.py [--batches 100] [--threads 8]
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import threading
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--batches", type=int, default=100)
    ap.add_argument("--batch", type=int, default=512)
    ap.add_argument("--unique", type=int, default=512)
    ap.add_argument("--threads", default="4,8,12")
    args = ap.parse_args()
    import bench
    B = args.batch
    uniq = bench.make_unique(args.unique, 640, 480, 1, False, 8)
    import numpy as np
    import torch

    from dataloader_amd import fallback
    from dataloader_amd.config import DINOAugConfig
    from dataloader_amd.params import OUT_BF16, make_aug_config
    from dataloader_amd.pipeline import MI355XAugPipeline
    from dataloader_amd.tario import ShardBatchFeeder, ShmShardCache
    cfg = make_aug_config(DINOAugConfig(), 224, 96, OUT_BF16)
    n = (args.batches + 4) * B
    jpegs = [uniq[i % len(uniq)] for i in range(n)]
    shards = bench.make_shards(jpegs, 1000)
    cache = ShmShardCache(job_id=f"e2e_study_{os.getpid()}", base_dir="/dev/shm", max_gb=64.0)
    dev = torch.device("cuda", 0)
    res = {}
    try:
        paths = [f"/synthetic/shard-{k:05d}.tar" for k in range(len(shards))]
        for p, t in zip(paths, shards):
            cache.put(p, t)
        del shards
        pinned = [torch.empty(60 << 20, dtype=torch.uint8, pin_memory=True) for _ in range(2)]
        # main-thread loads
        from dataloader_amd.engine import pack_jpegs
        hb, off = pack_jpegs(uniq[:B], pin=True)
        d_bytes, d_off = hb.to(dev), off.to(dev)
        pipe = MI355XAugPipeline(None, DINOAugConfig(), B, seed=1, depth=3)
        views = [sl.engine.alloc_views(pipe._cfg(224, 96), B) for sl in pipe._slots]
        d_sink = torch.empty(60 << 20, dtype=torch.uint8, device=dev)
        torch.cuda.synchronize()

        def load_none(stop):
            stop.wait()

        def load_gil(stop):
            x = 0
            while not stop.is_set():
                x += 1

        def load_h2d(stop):
            s = torch.cuda.Stream()
            with torch.cuda.stream(s):
                while not stop.is_set():
                    d_sink[: 43 << 20].copy_(pinned[1][: 43 << 20], non_blocking=True)
                    s.synchronize()

        def load_stage3(stop):
            k = 0
            while not stop.is_set():
                pipe.run_device_batch(d_bytes, d_off, B, views=views[k % 3])
                k += 1
                if k % 3 == 0:
                    torch.cuda.synchronize()
            torch.cuda.synchronize()

        def load_both(stop):
            t = threading.Thread(target=load_h2d, args=(stop,))
            t.start()
            load_stage3(stop)
            t.join()

        for nt in [int(x) for x in args.threads.split(",")]:
            for name, fn in (("idle", load_none), ("gil", load_gil), ("h2d", load_h2d), ("stage3", load_stage3),
                             ("stage3+h2d", load_both)):
                feeder = ShardBatchFeeder(cache, paths, B, nthreads=nt)
                feeder.next_batch_spans()  # first shard ready
                stop = threading.Event()
                th = threading.Thread(target=fn, args=(stop,))
                th.start()
                time.sleep(0.05)
                t_pull = t_pack = 0.0
                nb = 0
                t_all = time.perf_counter()
                for k in range(args.batches):
                    t0 = time.perf_counter()
                    bs = feeder.next_batch_spans()
                    t1 = time.perf_counter()
                    fallback.gather_probe(bs.ptrs, bs.lens, pinned[0], nt, 0, cfg)
                    t2 = time.perf_counter()
                    feeder.retire(bs, None)
                    t_pull += t1 - t0
                    t_pack += t2 - t1
                    nb += 1
                t_all = time.perf_counter() - t_all
                stop.set()
                th.join()
                feeder.close()
                r = {"pull_ms": round(t_pull / nb * 1e3, 3), "pack_probe_ms": round(t_pack / nb * 1e3, 3),
                     "batch_ms": round(t_all / nb * 1e3, 3)}
                res[f"t{nt}_{name}"] = r
                print(json.dumps({f"t{nt}_{name}": r}), flush=True)
        pipe.close()
    finally:
        cache.close(remove=True)
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
