#!/usr/bin/env python
"""Host half at N ranks on one node (analysis aid): N NativeShardFeed instances
(one per rank, shards i % N == rank of one shared /dev/shm cache) run at once, each in its own
process with `--threads` copier threads; rank 0 optionally drives the full GPU pipeline
(MI355XBackend.build_pipeline + iterator, the e2e leg's path) while the others consume their
batches on the host only.  Prints one JSON line: per-rank images/s and /dev/shm read GB/s,
the aggregate, and the host's CPU count / model.

usage: python scripts/host_feed_study.py [--ranks 8] [--threads 2] [--seconds 8] [--gpu-rank]
"""
from __future__ import annotations

import argparse
import json
import multiprocessing as mp
import os
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))


def _rank(rank: int, world: int, job: str, paths: list, B: int, threads: int, seconds: float, gpu: bool, q,
          lookahead: int = 2) -> None:
    from dataloader_amd import tario
    cache = tario.ShmShardCache(job_id=job, node_master=False, shard_timeout_s=60.0)
    feed = tario.NativeShardFeed(cache, paths, B, rank=rank, world=world, nthreads=threads, slots=6,
                                 lookahead=lookahead)
    n_img = n_bytes = 0
    t_end = None
    if gpu:
        import torch

        from dataloader_amd.backend import MI355XBackend
        from dataloader_amd.config import DINOAugConfig, DinoV2AugSpec, PipelineConfig
        spec = DinoV2AugSpec(aug_cfg=DINOAugConfig())
        be = MI355XBackend()
        pipe = be.build_pipeline(feed, spec, PipelineConfig(device_id=0, seed=rank, gpu_queue=6), None)
        it = be.build_pipeline_iterator(pipe, spec, spec.output_map, B)
        for _ in range(4):  # warm-up
            next(it)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        while time.perf_counter() - t0 < seconds:
            try:
                next(it)
            except StopIteration:
                feed.reset()
                it.reset()
                continue
            n_img += B
        torch.cuda.synchronize()
        t_end = time.perf_counter() - t0
        st = pipe.flush_stats()
        pipe.close()
        extra = {"statuses": {str(k): v for k, v in st["status"].items()}}
    else:
        t0 = time.perf_counter()
        while time.perf_counter() - t0 < seconds:
            try:
                fb = feed.next_prepared(timeout=30.0)
            except StopIteration:
                feed.reset()
                continue
            n_img += fb.n
            n_bytes += fb.nbytes
            feed.release(fb)
        t_end = time.perf_counter() - t0
        extra = {}
    fs = feed.stats()
    feed.close()
    q.put(dict(rank=rank, gpu=gpu, images_per_s=round(n_img / t_end, 1), seconds=round(t_end, 2),
               shm_read_GBs=round(n_bytes / t_end / 1e9, 2) if n_bytes else None,
               feed={k: (round(v, 3) if isinstance(v, float) else v) for k, v in fs.items()}, **extra))


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--ranks", type=int, default=8)
    ap.add_argument("--threads", type=int, default=2)
    ap.add_argument("--seconds", type=float, default=8.0)
    ap.add_argument("--batch", type=int, default=512)
    ap.add_argument("--per-rank", type=int, default=4000, help="images per rank (one epoch)")
    ap.add_argument("--shard", type=int, default=500)
    ap.add_argument("--gpu-rank", action="store_true", help="rank 0 runs the GPU pipeline")
    ap.add_argument("--lookahead", type=int, default=2, help="shards opened ahead per feed (= opener threads, <= 4)")
    a = ap.parse_args()
    from bench import _cpu_model, make_shards, make_unique
    from dataloader_amd import tario
    uniq = make_unique(512, 640, 480, 5, False, 16)
    total = a.ranks * a.per_rank
    jpegs = [uniq[i % len(uniq)] for i in range(total)]
    shards = make_shards(jpegs, a.shard)
    job = f"host_feed_{os.getpid()}"
    master = tario.ShmShardCache(job_id=job, node_master=True, max_gb=64.0)
    paths = [f"/synthetic/shard-{k:05d}.tar" for k in range(len(shards))]
    for p, t in zip(paths, shards):
        master.put(p, t)
    shard_bytes = sum(len(t) for t in shards)
    del shards, jpegs
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_rank, args=(r, a.ranks, job, paths, a.batch, a.threads, a.seconds,
                                             a.gpu_rank and r == 0, q, a.lookahead)) for r in range(a.ranks)]
    try:
        for p in procs:
            p.start()
        res = sorted((q.get(timeout=600) for _ in procs), key=lambda r: r["rank"])
    finally:
        for p in procs:
            p.join(timeout=60)
            if p.is_alive():
                p.kill()
        master.close(remove=True)
    host = [r for r in res if not r["gpu"]]
    print(json.dumps({
        "ranks": a.ranks, "threads_per_feed": a.threads, "lookahead": a.lookahead, "batch": a.batch,
        "seconds": a.seconds,
        "cpu_count": os.cpu_count(), "affinity": len(os.sched_getaffinity(0)), "cpu_model": _cpu_model(),
        "mean_jpeg_bytes": round(shard_bytes / total),
        "per_rank": res,
        "host_feeds_images_per_s_min": min((r["images_per_s"] for r in host), default=None),
        "host_feeds_images_per_s_sum": round(sum(r["images_per_s"] for r in host), 1),
        "host_feeds_shm_read_GBs_sum": round(sum(r["shm_read_GBs"] or 0 for r in host), 2),
    }), flush=True)


if __name__ == "__main__":
    main()
