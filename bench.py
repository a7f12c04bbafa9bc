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
    w, h, seed, mixed, prog = args
    from dataloader_amd.synthetic import encode_jpeg, textured_rgb
    rng = np.random.default_rng(seed)
    if mixed:
        short = int(rng.integers(224, 1601))
        aspect = float(rng.uniform(0.75, 4.0 / 3.0))
        long_ = max(short, int(round(short * max(aspect, 1.0 / aspect))))
        w, h = (long_, short) if rng.random() < 0.5 else (short, long_)
    return encode_jpeg(textured_rgb(w, h, rng), quality=85, progressive=prog)


def make_unique(n: int, w: int, h: int, base_seed: int, mixed: bool, procs: int, prog_frac: float = 0.0) -> list[bytes]:
    # 'spawn': never fork a process that may already hold a HIP context
    # every round(1 / prog_frac)-th encode is progressive (libjpeg's simple progression)
    step = int(round(1.0 / prog_frac)) if prog_frac > 0 else 0
    jobs = [(w, h, base_seed * 100003 + k, mixed, bool(step) and k % step == step - 1) for k in range(n)]
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


def sparse_entry_bytes(pipe, dims_420: list[bytes]) -> tuple[float, float]:
    """Mean bytes of the sparse coefficient entries k_huff1 / k_huff3 wrote per block, read
    back from the block records of the last decoded batch (dino_debug_region 2): a block
    record {first halfword, n16 | n32 << 7 | DC << 16} gives n16 halfword entries + n32
    u32 entries (+ 1 alignment halfword); 8 bytes of record per block on top."""
    eng = pipe._last.engine
    tot_e = tot_b = 0.0
    for i in range(min(eng.last_batch, 16, len(dims_420))):
        if b"\xff\xc2" in dims_420[i][:4096]:  # progressive (k_prog's dense buffer, not entries)
            continue
        w, h = jpeg_meta(dims_420[i])
        nblk = ((w + 15) // 16) * ((h + 15) // 16) * 6
        reg = eng.debug_region(i, 2, nblk * 256 + nblk * 8).cpu().numpy()
        y = reg[nblk * 256:nblk * 256 + nblk * 8].view(np.uint32)[1::2]
        n16 = (y & 0x7F).astype(np.int64)
        n32 = ((y >> 7) & 0x7F).astype(np.int64)
        tot_e += float((2 * n16 + 4 * n32 + 2 * (n32 > 0)).sum())
        tot_b += nblk
    return (tot_e / tot_b if tot_b else 0.0), 8.0


def algorithmic_bytes(jpegs, g: int, l: int, n_g: int, n_l: int, out_bytes: int, recs=None,
                      entry_bytes_per_block: float = 20.0) -> dict:
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
    per_blk = entry_bytes_per_block + 8.0       # sparse entries + the 8-byte block record
    ab = {
        "path": s_jpeg + out,                       # S_jpeg + 1 044 480 B (bf16)
        "k_destuff": s_jpeg,                         # per launch: count pass reads, write pass reads + writes
        # first (speculative) decode reads the entropy stream; for the images it finishes
        # itself it also writes their sparse coefficient entries + block records (measured)
        "k_huff1": s_jpeg + blk_fused * per_blk,
        # re-decode of the other images: entropy bytes in, sparse entries + records out
        "k_huff3": s_unfused + (blocks - blk_fused) * per_blk,
        "k_idct": blocks * per_blk + blocks * 64,
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
        if l <= VFINAL_MAX_S:  # local views: k_vfinal (timed as k_final_local) reads the h-pass rows, writes the view
            rr = r[:, n_g:nv]
            ab["k_final_local"] = float((rr["crop_h"].astype(np.float64) * 3 * l).sum(1).mean()) + out_bytes * 3 * n_l * l * l
            ab.pop("k_vert_local")
    return ab


VFINAL_MAX_S = 128  # kernels.hip kVFinalMaxS: views up to this size run k_vfinal (vertical pass + epilogue fused)


def _measure(fn, warmup: int, iters: int, budget_s: float) -> dict:
    """scripts/benchmark.py:161-190 of the reference: warm-up, then per-iteration wall times ->
    mean/std/p50/p95 (ms).  ``iters`` is capped so that the timed part stays within ``budget_s``."""
    import statistics
    for _ in range(warmup):
        fn()
    times = []
    t_start = time.perf_counter()
    for _ in range(iters):
        t0 = time.perf_counter()
        fn()
        times.append((time.perf_counter() - t0) * 1e3)
        if time.perf_counter() - t_start > budget_s and len(times) >= 5:
            break
    st = sorted(times)
    return {"mean_ms": statistics.mean(times), "std_ms": statistics.stdev(times) if len(times) > 1 else 0.0,
            "p50_ms": statistics.median(times), "p95_ms": st[min(len(st) - 1, int(0.95 * len(st)))],
            "iters": len(times)}


def _cpu_model() -> str:
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def _ref_faithful_runner(jpegs, batch: int, workers: int):
    """CPUAugPipeline.run_one_batch restated (cpu.py:309-367): a ThreadPoolExecutor of
    min(B, cpu_count, 16) workers created once (cpu.py:286, 303-306), every view re-decoding
    the JPEG (cpu.py:251), per-view draws from the torch + Python RNGs, torch.stack per view."""
    import torch

    from oracle import cpu_ref
    cfg = cpu_ref.AugCfg()
    table = cpu_ref.view_table(cfg)
    gen = torch.Generator().manual_seed(0)
    rnd = random.Random(0)

    def sample(j):
        img = cpu_ref.decode_rgb(j)
        w, h = img.size
        outs = []
        for spec in table:
            p = cpu_ref.draw_params_like_cpubackend(w, h, spec, cfg, gen, rnd)
            outs.append(cpu_ref.augment_one(j, p))
        return outs

    ex = ThreadPoolExecutor(max_workers=workers)
    state = {"k": 0}

    def run():
        k = state["k"]
        state["k"] += 1
        b = [jpegs[(k * batch + i) % len(jpegs)] for i in range(batch)]
        res = list(ex.map(sample, b))
        return [torch.stack([r[v] for r in res]) for v in range(len(table))]
    return run, ex


def _best_cpu_chunk(args):
    """One process of the 'best CPU' pool: decode ONCE per image, then the 10 views."""
    jpegs, seed = args
    import torch

    from oracle import cpu_ref
    torch.set_num_threads(1)
    cfg = cpu_ref.AugCfg()
    table = cpu_ref.view_table(cfg)
    gen = torch.Generator().manual_seed(seed)
    rnd = random.Random(seed)
    n = 0
    for j in jpegs:
        img = cpu_ref.decode_rgb(j)
        for spec in table:
            p = cpu_ref.draw_params_like_cpubackend(img.size[0], img.size[1], spec, cfg, gen, rnd)
            cpu_ref.augment_one(j, p, decoded=img)
        n += 1
    return n


def cpu_baseline(c2_jpegs, c1_jpegs, budget_s: float = 10.0, procs: int = 16) -> dict:
    """SURVEY §8(d) CPU baseline, timed on this host (oracle restatement, kind 'port'):

    * value: the reference-faithful CPUBackend on the C2 images (640x480), B = 32;
    * c1: the same on BASELINE configs[0] (one tar shard of 256 x 256^2 JPEGs, B = 32);
    * best_cpu: a process pool over the box's CPU share, decoding once per image.
    Per-batch timing as reference scripts/benchmark.py:161-190 (mean/std/p50/p95)."""
    import torch
    from multiprocessing import get_context
    torch.set_num_threads(1)
    B = 32
    workers = min(B, os.cpu_count() or 4, 16)                    # cpu.py:286
    out = {"unit": "images/s", "cores": workers, "kind": "port", "batch": B,
           "cpu_count": os.cpu_count(), "cpu_model": _cpu_model()}
    run, ex = _ref_faithful_runner(c2_jpegs, B, workers)
    m = _measure(run, 2, 30, budget_s)
    out.update({"value": round(B / (m["mean_ms"] / 1e3), 2), "per_batch_ms": {k: round(v, 2) for k, v in m.items()},
                "sample": f"C2: {m['iters']} timed batches of {B} synthetic 640x480 q85 JPEGs (after 2 warm-up), "
                          f"CPUBackend restatement (Pillow + torch), decode per view, ThreadPoolExecutor({workers})"})
    ex.shutdown()
    run, ex = _ref_faithful_runner(c1_jpegs, B, workers)
    m = _measure(run, 2, 30, budget_s / 2)
    out["c1"] = {"images_per_s": round(B / (m["mean_ms"] / 1e3), 2), "per_batch_ms": {k: round(v, 2) for k, v in m.items()},
                 "workload": "BASELINE configs[0]: 256 synthetic 256x256 JPEGs (one tar shard), B = 32, "
                             "DINOAugConfig(n_local_crops=8), reference-faithful"}
    ex.shutdown()
    # best CPU: one process per core of the box's share, decode once per image
    nb = 16 * procs
    pool = get_context("spawn").Pool(procs)
    try:
        chunks = [([c2_jpegs[(i * 16 + k) % len(c2_jpegs)] for k in range(16)], i) for i in range(procs)]
        pool.map(_best_cpu_chunk, chunks)                        # warm-up: imports, first decode
        t0 = time.perf_counter()
        done = sum(pool.map(_best_cpu_chunk, chunks))
        dt = time.perf_counter() - t0
    finally:
        pool.close()
        pool.join()
    out["best_cpu"] = {"images_per_s": round(done / dt, 2), "processes": procs, "images": nb,
                       "mode": "process pool, decode once per image, C2 images"}
    return out


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
            t = torch.tensor([dt], dtype=torch.float64)
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


PMC_FILES = ("r02_pmc_traffic.json", "r01_s7_pmc_traffic.json")


def load_traffic() -> tuple[dict, str | None]:
    """Per-launch HBM bytes per kernel from the newest committed PMC summary (FETCH_SIZE and
    WRITE_SIZE passes of this bench under rocprofv3, scripts/gpu_pmc.sh; corrections of
    MI355X_MICROARCH.md §HBM): {kernel: bytes}, file name."""
    for name in PMC_FILES:
        f = ROOT / "profiles" / name
        if f.exists():
            try:
                d = json.loads(f.read_text())
                return {k: v.get("hbm_bytes_per_launch") for k, v in d.items() if not k.startswith("_")}, name
            except Exception:  # noqa: BLE001
                pass
    return {}, None


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=98, help="timed steps (98 x 512 covers the 50k set once)")
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--batch", type=int, default=512)
    ap.add_argument("--images", type=int, default=50000)
    ap.add_argument("--unique", type=int, default=2048, help="distinct JPEG encodes tiled to --images")
    ap.add_argument("--procs", type=int, default=-1, help="JPEG encoder processes (0: in-process)")
    ap.add_argument("--depth", type=int, default=3, help="batches in flight (slots with their own ctx + stream)")
    ap.add_argument("--width", type=int, default=640)
    ap.add_argument("--height", type=int, default=480)
    ap.add_argument("--mixed", action="store_true", help="C3: short side U{224..1600} (+ iBOT masks)")
    ap.add_argument("--progressive-frac", type=float, default=0.0,
                    help="share of progressive encodes (web datasets hold some; decoded by k_prog)")
    ap.add_argument("--masks", action="store_true", help="iBOT masks per batch (default with --mixed)")
    ap.add_argument("--dtype", default="bf16", choices=["bf16", "fp8", "fp32"])
    ap.add_argument("--cpu-seconds", type=float, default=10.0, help="time budget of each CPU-baseline leg")
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
    uniq = make_unique(args.unique, args.width, args.height, 1 + rank, args.mixed, procs, args.progressive_frac)

    import torch
    import torch.distributed as dist

    # one GPU per rank; more ranks than GPUs (a rehearsal of the N-rank path on a smaller
    # box) share them round-robin
    ndev = max(1, torch.cuda.device_count())
    local_rank = local_rank % ndev
    torch.cuda.set_device(local_rank)
    dev = torch.device("cuda", local_rank)
    if world > 1:
        # barrier + MAX of the elapsed time only: a CPU (gloo) group, no RCCL on this path
        dist.init_process_group("gloo")

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
    k_last = args.warmup + 2 * args.steps - 1  # the batch the last slot still holds
    s_last = (k_last % n_batches) * B
    ent_b, _ = sparse_entry_bytes(pipe, jpegs[s_last:s_last + 16])
    if world > 1:
        t = torch.tensor([dt], dtype=torch.float64)
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
                           cfg.n_local_crops, out_bytes, recs=pipe.last_params(), entry_bytes_per_block=ent_b)
    per_kernel = {k: {"avg_ms": (ms / n if n else 0.0), "launches": n, "total_ms": ms} for k, (ms, n) in ktimes.items()}
    dom = max(per_kernel, key=lambda k: per_kernel[k]["total_ms"])
    traffic, traffic_src = load_traffic()
    # algorithmic bytes per image = S_jpeg + sum over views of 3 S^2 x out bytes;
    # one launch of any Stage-3 kernel processes the batch of B images
    bytes_launch = ab["path"] * B
    achieved = bytes_launch / (per_kernel[dom]["avg_ms"] * 1e-3) / 1e9
    roof = {"bound": "hbm", "achieved": round(achieved, 2), "peak": PEAK_HBM_GBS, "unit": "GB/s",
            "frac": round(achieved / PEAK_HBM_GBS, 5), "traffic": traffic.get(dom), "kernel": dom,
            "algorithmic_bytes_per_launch": int(bytes_launch), "avg_launch_ms": round(per_kernel[dom]["avg_ms"], 4),
            "definition": "SURVEY 8(d) bytes per image (S_jpeg + 3*sum(S_v^2)*out_bytes) x batch / dominant kernel's "
                          "mean launch time (HIP events on its stream, serialized pass after the timed region)",
            "traffic_source": f"profiles/{traffic_src}" if traffic_src else None}
    # each kernel on its own interface bytes (what it must read + write; huffman entries measured)
    roof_all = {}
    for k, v in per_kernel.items():
        if ab.get(k) and v["avg_ms"] > 0:
            gbs = ab[k] * B / (v["avg_ms"] * 1e-3) / 1e9
            roof_all[k] = {"achieved_GBs": round(gbs, 1), "frac": round(gbs / PEAK_HBM_GBS, 4),
                           "avg_ms": round(v["avg_ms"], 4), "interface_bytes_per_launch": int(ab[k] * B),
                           "traffic_bytes_per_launch": traffic.get(k)}
    ms_step = dt / args.steps * 1e3
    path_gbs = ab["path"] * B * world / (dt / args.steps) / 1e9
    step_traffic = None
    if traffic:
        step_traffic = sum((traffic.get(k) or 0) * v["launches"] / max(args.steps, 1) for k, v in per_kernel.items())
    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        c1 = make_unique(256, 256, 256, 7, False, procs)
        cpu = cpu_baseline(uniq, c1, args.cpu_seconds)
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
                       "mean_jpeg_bytes": round(ab["s_jpeg"]), "out_dtype": args.dtype,
                       "progressive_frac": args.progressive_frac},
            "roofline": roof,
            "roofline_kernels": roof_all,
            "path_roofline": {"algorithmic_bytes_per_image": int(ab["path"]), "achieved_GBs": round(path_gbs, 2),
                              "frac": round(path_gbs / PEAK_HBM_GBS / max(world, 1), 5),
                              "pmc_traffic_bytes_per_step": int(step_traffic) if step_traffic else None,
                              "algorithmic_bytes_per_step": int(ab["path"] * B),
                              "sparse_entry_bytes_per_block": round(ent_b, 2)},
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
