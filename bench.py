#!/usr/bin/env python
"""Stage-3 throughput benchmark (BASELINE.json metric).

One step = the full Stage-3 hot path over one batch of ``--batch`` JPEGs whose
bytes are already resident in HBM: decode (parse, destuff, Huffman, IDCT,
upsample+colour) + 10 views (2x224^2 + 8x96^2: random-resized crop, flip,
colour jitter, grayscale, blur, solarize, normalize -> bf16 NCHW) — reference
``CPUAugPipeline.run_one_batch`` (cpu.py:309-367).

Workload (BASELINE.json configs[1]): per GPU, a 50 000-image dataset of
synthetic textured 640x480 q85 4:2:0 JPEGs resident in HBM (``--unique``
distinct encodes tiled to ``--images``), batch 512.  Multi-GPU: one process per
GPU (torchrun), each rank with its own images and seed (seed + rank), no
collective on the data path; a barrier + MAX over ranks brackets the timed
region (weak scaling).

Prints ONE JSON line on rank 0 (see DESIGN.md §Measurement for every field).
"""

from __future__ import annotations

import argparse
import json
import os
import random
import sys
import time
from concurrent.futures import ThreadPoolExecutor
from multiprocessing import get_context
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent
sys.path.insert(0, str(ROOT))

METRIC = "images/sec decode+10-crop, device-resident (JPEG bytes in HBM), 1/2/4/8 GPU"
PEAK_HBM_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md chip table)


def _gen_one(args):
    w, h, seed, mixed = args
    from dataloader_amd.synthetic import encode_jpeg, textured_rgb
    rng = np.random.default_rng(seed)
    if mixed:
        short = int(rng.integers(224, 1601))
        aspect = float(rng.uniform(0.75, 4.0 / 3.0))
        long_ = max(short, int(round(short * max(aspect, 1.0 / aspect))))
        w, h = (long_, short) if rng.random() < 0.5 else (short, long_)
    return encode_jpeg(textured_rgb(w, h, rng), quality=85)


def make_unique(n: int, w: int, h: int, base_seed: int, mixed: bool, procs: int) -> list[bytes]:
    # 'spawn': never fork a process that may already hold a HIP context
    jobs = [(w, h, base_seed * 100003 + k, mixed) for k in range(n)]
    if procs <= 1:  # in-process (profiler runs: no worker processes to tear down)
        return [_gen_one(j) for j in jobs]
    pool = get_context("spawn").Pool(procs)
    try:
        return pool.map(_gen_one, jobs, chunksize=4)
    finally:
        pool.close()  # let workers exit on their own (no SIGTERM under rocprofv3)
        pool.join()


def jpeg_meta(j: bytes):
    import io

    from PIL import Image
    im = Image.open(io.BytesIO(j))
    return im.size


def algorithmic_bytes(jpegs, g: int, l: int, n_g: int, n_l: int, out_bytes: int, recs=None) -> dict:
    """Per-image algorithmic bytes of the path and of each kernel's interface.

    ``recs`` (the last batch's view records) sizes the resize kernels' interfaces
    from the crops actually drawn: k_hresize reads crop_h*crop_w*3 and writes
    crop_h*S*3; k_vert reads that and writes the 3*S^2 u8 crop; k_final reads the
    crop and writes the normalised view.
    """
    s_jpeg = float(np.mean([len(j) for j in jpegs]))
    dims = [jpeg_meta(j) for j in jpegs]
    px = float(np.mean([w * h for w, h in dims]))
    # 4:2:0 coefficient count: luma + 2 quarter-size chroma, padded to 16x16 MCUs
    nblk = [((w + 15) // 16) * ((h + 15) // 16) * 6 for w, h in dims]
    blocks = float(np.mean(nblk))
    # images k_huff1 finishes itself (one 2 Mbit segment, lane ranges <= 3072 bits,
    # kernels.hip huff_single_segment); the others are written by k_huff3
    def fused(nbytes):
        nbits = nbytes * 8
        if nbits > 2048 * 1024:
            return False
        n = max(1, min(256, -(-nbits // 1024)))
        sub = max(32, (-(-nbits // n) + 31) // 32 * 32)
        return sub <= 3072
    fz = [fused(len(j)) for j in jpegs]
    blk_fused = float(np.mean([b if f else 0 for b, f in zip(nblk, fz)]))
    s_unfused = float(np.mean([len(j) if not f else 0 for j, f in zip(jpegs, fz)]))
    out = out_bytes * 3 * (n_g * g * g + n_l * l * l)
    ab = {
        "path": s_jpeg + out,                       # S_jpeg + 1 044 480 B (bf16)
        "k_destuff": s_jpeg,                         # per launch: count pass reads, write pass reads + writes
        # first (speculative) decode reads the entropy stream; for the images it finishes
        # itself it also writes their coefficients (dense int16 equivalent)
        "k_huff1": s_jpeg + blk_fused * 128,
        # re-decode of the other images: entropy bytes in, coefficients out
        "k_huff3": s_unfused + (blocks - blk_fused) * 128,
        "k_idct": blocks * 128 + blocks * 64,
        "k_color": blocks * 64 + px * 3,
        "k_final_global": (3 + out_bytes * 3) * n_g * g * g,
        "k_final_local": (3 + out_bytes * 3) * n_l * l * l,
        "s_jpeg": s_jpeg,
        "pixels": px,
    }
    if recs is not None and len(recs):
        nv = n_g + n_l
        r = recs.reshape(-1, nv)
        hr = (r["crop_h"].astype(np.float64) * 3 * (r["crop_w"] + r["out_size"])).sum(1).mean()
        ab["k_hresize"] = float(hr)
        for name, sl, S in (("k_vert_global", slice(0, n_g), g), ("k_vert_local", slice(n_g, nv), l)):
            rr = r[:, sl]
            ab[name] = float((rr["crop_h"].astype(np.float64) * 3 * S + 3 * S * S).sum(1).mean())
    return ab


def cpu_baseline(jpegs, seconds: float, batch: int = 32) -> dict:
    """Reference-faithful CPUBackend restatement timed on this host's cores (oracle, kind 'port')."""
    import torch

    from oracle import cpu_ref
    torch.set_num_threads(1)
    workers = min(batch, os.cpu_count() or 4, 16)             # cpu.py:286, 303-306
    cfg = cpu_ref.AugCfg()
    table = cpu_ref.view_table(cfg)
    gen = torch.Generator().manual_seed(0)
    rnd = random.Random(0)

    def sample(j):
        img = cpu_ref.decode_rgb(j)
        w, h = img.size
        outs = []
        for spec in table:                                     # decode per view, as cpu.py:251
            p = cpu_ref.draw_params_like_cpubackend(w, h, spec, cfg, gen, rnd)
            outs.append(cpu_ref.augment_one(j, p))
        return outs

    done = 0
    t0 = time.perf_counter()
    with ThreadPoolExecutor(max_workers=workers) as ex:
        k = 0
        while True:
            b = [jpegs[(k * batch + i) % len(jpegs)] for i in range(batch)]
            res = list(ex.map(sample, b))
            _ = [torch.stack([r[v] for r in res]) for v in range(len(table))]
            done += batch
            k += 1
            if time.perf_counter() - t0 >= seconds:
                break
    dt = time.perf_counter() - t0
    return {"value": done / dt, "unit": "images/s", "cores": workers, "kind": "port",
            "sample": f"{done} images ({batch}/batch) of the same synthetic JPEG pool, CPUBackend restatement "
                      f"(PIL+torch), decode per view, ThreadPoolExecutor({workers}), {dt:.1f}s"}


def make_shards(jpegs, shard_size: int) -> list[bytes]:
    """WebDataset tar shards shaped like the reference fixtures (sample_%06d.jpg + .json)."""
    import io
    import tarfile
    shards = []
    for s0 in range(0, len(jpegs), shard_size):
        buf = io.BytesIO()
        with tarfile.open(fileobj=buf, mode="w") as tf:
            for i in range(s0, min(len(jpegs), s0 + shard_size)):
                for name, data in ((f"sample_{i:06d}.jpg", jpegs[i]),
                                   (f"sample_{i:06d}.json", json.dumps({"quality_score": 1.0}).encode())):
                    ti = tarfile.TarInfo(name)
                    ti.size = len(data)
                    tf.addfile(ti, io.BytesIO(data))
        shards.append(buf.getvalue())
    return shards


def run_e2e(args, uniq, rank: int, world: int, dev, cfg, B: int) -> dict:
    """C5 end-to-end: shards in /dev/shm (reference cache file format) -> dino_tar_index ->
    dino_gather into pinned staging -> H2D -> Stage 3, batches in flight as the main run."""
    import torch
    import torch.distributed as dist

    from dataloader_amd.pipeline import MI355XAugPipeline
    from dataloader_amd.sharding import rank_seed
    from dataloader_amd.tario import ShardBatchFeeder, ShmShardCache

    n = (args.warmup + args.steps + 1) * B
    jpegs = [uniq[i % len(uniq)] for i in range(n)]
    shards = make_shards(jpegs, args.shard_size)
    cache = ShmShardCache(job_id=f"dino_bench_{os.getpid()}", base_dir="/dev/shm", max_gb=64.0)
    try:
        paths = [f"/synthetic/rank{rank}/shard-{k:05d}.tar" for k in range(len(shards))]
        for p, t in zip(paths, shards):
            cache.put(p, t)  # Stage 1 (filesystem -> /dev/shm) is outside the timed region
        del shards
        feeder = ShardBatchFeeder(cache, paths, B, nthreads=args.gather_threads)
        pipe = MI355XAugPipeline(feeder, cfg, B, seed=rank_seed(1234, rank), out_dtype=args.dtype,
                                 device=dev.index, max_image_dim=4096 if args.mixed else 2048, depth=args.depth)
        for _ in range(args.warmup):
            pipe._enqueue_one()
        pipe.wait()
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        feeder.index_seconds = 0.0
        t0 = time.perf_counter()
        for _ in range(args.steps):
            pipe._enqueue_one()
        pipe.wait()
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        dt = time.perf_counter() - t0
        st = pipe.last_status()
        if (st != 0).any():
            raise RuntimeError(f"e2e decode failures: {np.unique(st, return_counts=True)}")
        shards_opened = feeder._shard
        feeder.close()
        pipe.close()
        if world > 1:
            t = torch.tensor([dt], device=dev, dtype=torch.float64)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            dt = float(t.item())
        return {"e2e_images_per_s": round(world * args.steps * B / dt, 1),
                "e2e_ms_per_step": round(dt / args.steps * 1e3, 3),
                "e2e_shard_prepare_ms_total": round(feeder.index_seconds * 1e3, 3),
                "e2e_shard_wait_ms_total": round(feeder.wait_seconds * 1e3, 3),
                "e2e_shards": shards_opened, "e2e_gather_threads": args.gather_threads,
                "e2e_path": "/dev/shm tar shards (shard_cache file format) -> dino_tar_index -> dino_gather "
                            "(pinned) -> H2D -> Stage 3"}
    finally:
        cache.close(remove=True)


def load_traffic(kernel: str):
    f = ROOT / "profiles" / "pmc_traffic.json"
    if not f.exists():
        return None
    try:
        d = json.loads(f.read_text())
        return d.get(kernel, {}).get("hbm_bytes_per_launch")
    except Exception:  # noqa: BLE001
        return None


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--batch", type=int, default=512)
    ap.add_argument("--images", type=int, default=50000)
    ap.add_argument("--unique", type=int, default=256)
    ap.add_argument("--procs", type=int, default=-1, help="JPEG encoder processes (0: in-process)")
    ap.add_argument("--depth", type=int, default=3, help="batches in flight (slots with their own ctx + stream)")
    ap.add_argument("--width", type=int, default=640)
    ap.add_argument("--height", type=int, default=480)
    ap.add_argument("--mixed", action="store_true", help="C3: short side U{224..1600} (+ iBOT masks)")
    ap.add_argument("--masks", action="store_true", help="iBOT masks per batch (default with --mixed)")
    ap.add_argument("--dtype", default="bf16", choices=["bf16", "fp8", "fp32"])
    ap.add_argument("--cpu-seconds", type=float, default=20.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--h2d", action="store_true", help="also time the H2D-inclusive rate (pinned host bytes)")
    ap.add_argument("--kernel-json", default="", help="write per-kernel times here (rank 0)")
    ap.add_argument("--e2e", action="store_true",
                    help="C5: also time tar shards in /dev/shm -> native index -> pinned gather -> H2D -> kernels")
    ap.add_argument("--shard-size", type=int, default=1000, help="samples per synthetic tar shard (--e2e)")
    ap.add_argument("--gather-threads", type=int, default=8, help="dino_gather copier threads (--e2e)")
    args = ap.parse_args()

    rank = int(os.environ.get("RANK", 0))
    world = int(os.environ.get("WORLD_SIZE", 1))
    local_rank = int(os.environ.get("LOCAL_RANK", 0))
    # synthetic data first, before anything initialises the GPU in this process
    procs = args.procs if args.procs >= 0 else min(16, os.cpu_count() or 4)
    uniq = make_unique(args.unique, args.width, args.height, 1 + rank, args.mixed, procs)

    import torch
    import torch.distributed as dist

    torch.cuda.set_device(local_rank)
    dev = torch.device("cuda", local_rank)
    if world > 1:
        dist.init_process_group("nccl", device_id=dev)

    from dataloader_amd.config import DINOAugConfig
    from dataloader_amd.engine import pack_jpegs
    from dataloader_amd.pipeline import MI355XAugPipeline
    from dataloader_amd.sharding import rank_seed

    n_img = args.images
    jpegs = [uniq[i % len(uniq)] for i in range(n_img)]
    host_buf, offsets = pack_jpegs(jpegs, pin=True)
    d_bytes = host_buf.to(dev)
    d_off = offsets.to(dev)
    torch.cuda.synchronize()

    cfg = DINOAugConfig()
    B = args.batch
    pipe = MI355XAugPipeline(None, cfg, B, seed=rank_seed(1234, rank), out_dtype=args.dtype, device=local_rank,
                             max_image_dim=4096 if args.mixed else 2048, depth=args.depth,
                             workspace_bytes=B * (40 << 20) if args.mixed else 0)
    ccfg = pipe._cfg(cfg.global_crop_size, cfg.local_crop_size)
    views = [sl.engine.alloc_views(ccfg, B) for sl in pipe._slots]  # one output set per in-flight slot
    n_batches = n_img // B
    masks_on = args.masks or args.mixed
    maskgen = None
    if masks_on:
        from dataloader_amd.masking import MaskingGenerator
        grid = cfg.global_crop_size // 14                     # patch 14: 16x16 at 224
        maskgen = MaskingGenerator((grid, grid), num_masking_patches=grid * grid // 2, device=dev)
        maskgen.seed(rank_seed(1234, rank))

    def step(k: int):
        s = (k % n_batches) * B
        pipe.run_device_batch(d_bytes, d_off[s:s + B + 1], B, views=views[k % pipe.depth])
        if maskgen is not None:  # one mask per batch, broadcast to [B, H*W] (loader.py:585-590)
            maskgen.generate(1).expand(B, -1)

    for k in range(args.warmup):
        step(k)
    torch.cuda.synchronize()
    st = pipe.last_status()
    if (st != 0).any():
        raise RuntimeError(f"decode failures in warmup batch: {np.unique(st, return_counts=True)}")
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for k in range(args.steps):
        step(args.warmup + k)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    dt = time.perf_counter() - t0
    # per-kernel HIP-event times: a separate pass with the batches serialised, so that a
    # kernel's events do not also span the other slot's concurrently running kernels
    pipe.set_timing(True)
    pipe.kernel_times()
    t_ser = time.perf_counter()
    for k in range(args.steps):
        step(args.warmup + args.steps + k)
        torch.cuda.synchronize()
    t_ser = time.perf_counter() - t_ser
    ktimes = pipe.kernel_times()
    pipe.set_timing(False)
    if world > 1:
        t = torch.tensor([dt], device=dev, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())

    h2d_rate = None
    if args.h2d:
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        for k in range(args.steps):
            s = (k % n_batches) * B
            base = int(offsets[s])
            nbytes = int(offsets[s + B]) - base
            hb = host_buf[base:base + nbytes].to(dev, non_blocking=True)
            ho = (offsets[s:s + B + 1] - base).to(dev, non_blocking=True)
            pipe.run_device_batch(hb, ho, B, views=views[k % pipe.depth])
        torch.cuda.synchronize()
        h2d_rate = args.steps * B / (time.perf_counter() - t1)

    e2e = run_e2e(args, uniq, rank, world, dev, cfg, B) if args.e2e else None

    value = world * args.steps * B / dt
    out_bytes = {"bf16": 2, "fp8": 1, "fp32": 4}[args.dtype]
    ab = algorithmic_bytes(uniq, cfg.global_crop_size, cfg.local_crop_size, cfg.n_global_crops,
                           cfg.n_local_crops, out_bytes, recs=pipe.last_params())
    per_kernel = {k: {"avg_ms": (ms / n if n else 0.0), "launches": n, "total_ms": ms} for k, (ms, n) in ktimes.items()}
    dom = max(per_kernel, key=lambda k: per_kernel[k]["total_ms"])
    dom_bytes = ab.get(dom)
    roof = None
    if dom_bytes:
        bytes_launch = dom_bytes * B
        achieved = bytes_launch / (per_kernel[dom]["avg_ms"] * 1e-3) / 1e9
        traffic = load_traffic(dom)
        roof = {"bound": "hbm", "achieved": round(achieved, 2), "peak": PEAK_HBM_GBS, "unit": "GB/s",
                "frac": round(achieved / PEAK_HBM_GBS, 5), "traffic": traffic, "kernel": dom,
                "algorithmic_bytes_per_launch": int(bytes_launch)}
    # the same figure for every timed kernel whose interface bytes are defined
    roof_all = {}
    for k, v in per_kernel.items():
        if ab.get(k) and v["avg_ms"] > 0:
            gbs = ab[k] * B / (v["avg_ms"] * 1e-3) / 1e9
            roof_all[k] = {"achieved_GBs": round(gbs, 1), "frac": round(gbs / PEAK_HBM_GBS, 4),
                           "avg_ms": round(v["avg_ms"], 4)}
    ms_step = dt / args.steps * 1e3
    path_gbs = ab["path"] * B * world / (dt / args.steps) / 1e9
    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cpu = cpu_baseline(uniq, args.cpu_seconds)
    if rank == 0:
        line = {
            "metric": METRIC, "value": round(value, 1), "unit": "images/s", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(ms_step, 3),
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "u8",
            "data": "synthetic",
            "config": {"workload": ("C3 mixed short side 224-1600, iBOT masks 16x16" if args.mixed else
                                    f"C2 {args.images} synthetic {args.width}x{args.height} q85 4:2:0 JPEGs "
                                    "resident in HBM") + f", 2x224^2+8x96^2 views, {args.dtype} out",
                       "global_batch": B * world, "batch_per_gpu": B, "parallelism": f"dp{world}",
                       "batches_in_flight": pipe.depth, "masks": masks_on,
                       "mean_jpeg_bytes": round(ab["s_jpeg"]), "out_dtype": args.dtype},
            "roofline": roof,
            "roofline_kernels": roof_all,
            "path_roofline": {"algorithmic_bytes_per_image": int(ab["path"]), "achieved_GBs": round(path_gbs, 2),
                              "frac": round(path_gbs / PEAK_HBM_GBS / max(world, 1), 5)},
            "kernels_ms_per_step": {k: round(v["total_ms"] / args.steps, 4) for k, v in per_kernel.items()},
            "serialized_ms_per_step": round(t_ser / args.steps * 1e3, 3),
            "cpu_baseline": cpu,
        }
        if h2d_rate is not None:
            line["h2d_inclusive_images_per_s"] = round(h2d_rate, 1)
        if e2e is not None:
            line["e2e"] = e2e
        print(json.dumps(line), flush=True)
        if args.kernel_json:
            Path(args.kernel_json).write_text(json.dumps(per_kernel, indent=1))
    pipe.close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
