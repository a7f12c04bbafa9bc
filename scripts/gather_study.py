"""Host half of the e2e feed, piece by piece (where do the ~5 ms per 512-image batch go?).

Times, per batch of B C2 JPEGs from /dev/shm tar shards: next_spans (Python), dino_gather
into a pinned torch buffer vs a plain numpy buffer at 1/2/4/8/16 threads, dino_probe, and a
hipHostRegister'ed-shard H2D (no host gather) if the runtime accepts the mapping.
usage: python scripts/gather_study.py [--batches 20]
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--batches", type=int, default=20)
    ap.add_argument("--batch", type=int, default=512)
    ap.add_argument("--unique", type=int, default=512)
    args = ap.parse_args()
    import bench
    B = args.batch
    uniq = bench.make_unique(args.unique, 640, 480, 1, False, 8)
    import numpy as np
    import torch

    from dataloader_amd import fallback
    from dataloader_amd.tario import ShardBatchFeeder, ShmShardCache, gather
    n = (args.batches + 2) * B
    jpegs = [uniq[i % len(uniq)] for i in range(n)]
    shards = bench.make_shards(jpegs, 1000)
    cache = ShmShardCache(job_id=f"gather_study_{os.getpid()}", base_dir="/dev/shm", max_gb=64.0)
    res = {"cpu_affinity": len(os.sched_getaffinity(0)), "cpu_count": os.cpu_count()}
    try:
        paths = [f"/synthetic/shard-{k:05d}.tar" for k in range(len(shards))]
        for p, t in zip(paths, shards):
            cache.put(p, t)
        del shards
        need = 0
        pinned = torch.empty(200 << 20, dtype=torch.uint8, pin_memory=True)
        plain = np.empty(200 << 20, np.uint8)
        plain[::4096] = 0
        for nt in (1, 2, 4, 8, 16):
            for dst_name, dst in (("pinned", pinned), ("numpy", plain)):
                feeder = ShardBatchFeeder(cache, paths, B, nthreads=nt)
                t_sp = t_g = 0.0
                nbytes = 0
                for k in range(args.batches):
                    t0 = time.perf_counter()
                    sp = feeder.next_spans()
                    t1 = time.perf_counter()
                    off = gather(sp, dst, nt)
                    t2 = time.perf_counter()
                    if k:
                        t_sp += t1 - t0
                        t_g += t2 - t1
                        nbytes += int(off[-1])
                feeder.close()
                m = args.batches - 1
                res[f"gather_{dst_name}_t{nt}"] = {"ms_per_batch": round(t_g / m * 1e3, 3),
                                                   "GBs": round(nbytes / t_g / 1e9, 2),
                                                   "spans_ms": round(t_sp / m * 1e3, 3)}
                need = nbytes // m
                print(json.dumps({f"t{nt}_{dst_name}": res[f"gather_{dst_name}_t{nt}"]}), flush=True)
        # probe
        feeder = ShardBatchFeeder(cache, paths, B, nthreads=8)
        off = gather(feeder.next_spans(), pinned, 8)
        t0 = time.perf_counter()
        for _ in range(10):
            fallback.probe(pinned.data_ptr(), off, B, 0, None)
        res["probe_ms"] = round((time.perf_counter() - t0) / 10 * 1e3, 3)
        # H2D of a pinned batch
        dev = torch.device("cuda", 0)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(10):
            d = pinned[:need].to(dev, non_blocking=True)
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t0) / 10
        res["h2d_pinned"] = {"ms": round(dt * 1e3, 3), "GBs": round(need / dt / 1e9, 2)}
        # H2D straight from a registered shard mapping (no host gather)
        arr = cache.get_array(paths[0])
        cr = torch.cuda.cudart()
        try:
            rc = cr.cudaHostRegister(arr.ctypes.data, arr.nbytes, 0)
            res["host_register_rc"] = int(rc) if not isinstance(rc, tuple) else [int(x) for x in rc]
            t = torch.from_numpy(arr)
            res["registered_is_pinned"] = bool(t.is_pinned())
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(10):
                d = t[:need].to(dev, non_blocking=True)
            torch.cuda.synchronize()
            dt = (time.perf_counter() - t0) / 10
            res["h2d_registered"] = {"ms": round(dt * 1e3, 3), "GBs": round(need / dt / 1e9, 2)}
            cr.cudaHostUnregister(arr.ctypes.data)
        except Exception as e:  # noqa: BLE001
            res["host_register_error"] = repr(e)
        t0 = time.perf_counter()
        for _ in range(3):
            d = torch.from_numpy(arr[:need]).to(dev)
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t0) / 3
        res["h2d_pageable"] = {"ms": round(dt * 1e3, 3), "GBs": round(need / dt / 1e9, 2)}
        feeder.close()
    finally:
        cache.close(remove=True)
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
