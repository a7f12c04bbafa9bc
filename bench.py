#!/usr/bin/env python
"""Stage-3 throughput benchmark (BASELINE.json metric).

One step = the full Stage-3 hot path over one batch of ``--batch`` JPEGs whose
bytes are already resident in HBM: decode (parse, destuff, Huffman, IDCT,
upsample+colour) + 10 views (2x224^2 + 8x96^2: random-resized crop, flip,
colour jitter, grayscale, blur, solarize, normalize -> bf16 NCHW) — reference
``CPUAugPipeline.run_one_batch`` (cpu.py:309-367).

Workload (BASELINE.json configs[1]): per GPU, a 50 000-image dataset of
synthetic textured 640x480 q85 4:2:0 JPEGs resident in HBM (``--unique``
distinct encodes tiled to ``--images``), batch 512.

Multi-GPU (configs[3], weak scaling): one process per GPU, each rank with its
own images and seed (seed + rank, reference config.py:204; shard ``i % world ==
rank``, hpc_source.py:154-156), no collective on the data path.  Either the
driver starts the ranks (torchrun: RANK/WORLD_SIZE/LOCAL_RANK in the env), or
``bench.py --gpus N`` starts them itself, before anything touches a GPU.  Every
rank needs a device of its own: with fewer visible GPUs than ranks the bench
refuses, unless ``--rehearsal`` (ranks then share devices round-robin and the
line says so: ``"rehearsal": true``, ``n_gpus`` = distinct devices).  A gloo
barrier + MAX of the per-rank elapsed times brackets the timed region.

At N = 1 the line also carries the other BASELINE configs, each timed the same
way in this process: ``c3`` (configs[2]: mixed resolution + iBOT masks),
``fp8`` (configs[4]: E4M3 epilogue), ``c2_dri`` (C2 with restart markers,
SURVEY §8(d)) and ``e2e`` (configs[4]: /dev/shm tar shards through
``MI355XBackend.build_pipeline`` + ``build_pipeline_iterator``, the drop-in
path), plus the CPU baseline.

Prints ONE JSON line on rank 0 (see DESIGN.md §Measurement for every field).
"""

from __future__ import annotations

import argparse
import json
import os
import random
import socket
import subprocess
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
VFINAL_MAX_S = 128  # kernels.hip kVFinalMaxS: views up to this size run k_vfinal (vertical pass + epilogue fused)


# ----------------------------------------------------------------------------- synthetic data
def _gen_one(args):
    w, h, seed, mixed, prog, rst = args
    from dataloader_amd.synthetic import encode_jpeg, textured_rgb
    rng = np.random.default_rng(seed)
    if mixed:
        short = int(rng.integers(224, 1601))
        aspect = float(rng.uniform(0.75, 4.0 / 3.0))
        long_ = max(short, int(round(short * max(aspect, 1.0 / aspect))))
        w, h = (long_, short) if rng.random() < 0.5 else (short, long_)
    return encode_jpeg(textured_rgb(w, h, rng), quality=85, progressive=prog, restart_mcus=rst)


def make_unique(n: int, w: int, h: int, base_seed: int, mixed: bool, procs: int, prog_frac: float = 0.0,
                restart_mcus: int = 0) -> list[bytes]:
    """``n`` distinct textured JPEGs (every round(1 / prog_frac)-th one progressive, libjpeg's
    simple progression; ``restart_mcus`` > 0: a DRI marker with that interval)."""
    step = int(round(1.0 / prog_frac)) if prog_frac > 0 else 0
    jobs = [(w, h, base_seed * 100003 + k, mixed, bool(step) and k % step == step - 1, restart_mcus)
            for k in range(n)]
    if procs <= 1:  # in-process (profiler runs: no worker processes to tear down)
        return [_gen_one(j) for j in jobs]
    # 'spawn': never fork a process that may already hold a HIP context
    pool = get_context("spawn").Pool(procs)
    try:
        return pool.map(_gen_one, jobs, chunksize=4)
    finally:
        pool.close()  # let workers exit on their own (no SIGTERM under rocprofv3)
        pool.join()


def jpeg_meta(j: bytes):
    import io

    from PIL import Image
    return Image.open(io.BytesIO(j)).size


# ----------------------------------------------------------------------------- algorithmic bytes
def sparse_entry_bytes(pipe, jpegs: list[bytes]) -> float:
    """Mean bytes of the sparse coefficient entries k_huff1 / k_huff3 wrote per block, read
    back from the block records of the last decoded batch (dino_debug_region 2): a block
    record {first halfword, n16 | n32 << 7 | DC << 16} gives n16 halfword entries + n32
    u32 entries (+ 1 alignment halfword); 8 bytes of record per block on top."""
    eng = pipe._last.engine
    tot_e = tot_b = 0.0
    for i in range(min(eng.last_batch, 16, len(jpegs))):
        if b"\xff\xc2" in jpegs[i][:4096]:  # progressive (k_prog's dense buffer, not entries)
            continue
        w, h = jpeg_meta(jpegs[i])
        nblk = ((w + 15) // 16) * ((h + 15) // 16) * 6
        reg = eng.debug_region(i, 2, nblk * 256 + nblk * 8).cpu().numpy()
        y = reg[nblk * 256:nblk * 256 + nblk * 8].view(np.uint32)[1::2]
        n16 = (y & 0x7F).astype(np.int64)
        n32 = ((y >> 7) & 0x7F).astype(np.int64)
        tot_e += float((2 * n16 + 4 * n32 + 2 * (n32 > 0)).sum())
        tot_b += nblk
    return tot_e / tot_b if tot_b else 0.0


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
    def fused(j):
        if b"\xff\xdd" in j[:2048]:  # restart intervals: k_huff3 decodes one interval per lane
            return False
        nbits = len(j) * 8
        if nbits > 2048 * 1024:
            return False
        n = max(1, min(256, -(-nbits // 1024)))
        sub = max(32, (-(-nbits // n) + 31) // 32 * 32)
        return sub <= 3072
    fz = [fused(j) for j in jpegs]
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
        # entries + records in, planes out; planes in, RGB out
        "k_idct": blocks * (per_blk + 64),
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


# ----------------------------------------------------------------------------- CPU baseline
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


# ----------------------------------------------------------------------------- rank launcher
def _free_port() -> int:
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def visible_devices() -> int:
    """GPUs this process may use.  ``torch.cuda.device_count()`` does not initialise a
    device on this image, so the launcher may still start rank processes afterwards."""
    import torch
    return int(torch.cuda.device_count())


_VIS_VARS = ("HIP_VISIBLE_DEVICES", "ROCR_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES")


def physical_device(device: int) -> str:
    """A name of the GPU behind local device index ``device`` that is comparable across
    ranks: the visible-devices entry when a launcher isolates ranks that way, else the index."""
    for var in _VIS_VARS:
        v = os.environ.get(var)
        if v:
            ids = [x.strip() for x in v.split(",") if x.strip()]
            return f"{var}:{ids[device]}" if device < len(ids) else f"{var}:?{device}"
    return str(device)


def check_devices(world: int, devices: int, rehearsal: bool) -> None:
    """One GPU per rank, or an explicit rehearsal (ranks share devices round-robin).  With
    per-rank visible-device isolation each rank sees one device: the distinct-device check
    then runs over the gathered physical names (``check_distinct``)."""
    if devices < 1:
        raise SystemExit(f"bench.py: no GPU visible (need {world}); nothing to measure")
    isolated = any(os.environ.get(v) for v in _VIS_VARS) and "DINO_BENCH_LAUNCHED" not in os.environ
    if world > devices and not rehearsal and not isolated:
        raise SystemExit(f"bench.py: {world} ranks but only {devices} GPU(s) visible; every rank needs a GPU of "
                         f"its own (pass --rehearsal to let ranks share devices; the line then says so)")


def check_distinct(per_rank: list, rehearsal: bool) -> int:
    """Distinct physical GPUs over the ranks; refuse sharing unless it is a rehearsal."""
    names = [r["physical"] for r in per_rank]
    distinct = len(set(names))
    if distinct < len(names) and not rehearsal:
        raise SystemExit(f"bench.py: {len(names)} ranks share {distinct} GPU(s) ({names}); pass --rehearsal "
                         "to allow it (the line then says so)")
    return distinct


def launch_ranks(n: int, argv: list[str], devices: int, rehearsal: bool = False,
                 cmd: list[str] | None = None, extra_env: dict | None = None) -> int:
    """``bench.py --gpus N`` without a launcher env: start N rank processes (this script
    again, or ``cmd``) with RANK / WORLD_SIZE / LOCAL_RANK / LOCAL_WORLD_SIZE /
    MASTER_ADDR=127.0.0.1 / MASTER_PORT set, wait for all of them and return the first
    non-zero exit code (the others are terminated).  Nothing here touches a GPU."""
    check_devices(n, devices, rehearsal)
    port = _free_port()
    cmd = cmd or [sys.executable, "-u", str(Path(__file__).resolve()), *argv]
    procs = []
    for r in range(n):
        env = dict(os.environ)
        env.update({"RANK": str(r), "WORLD_SIZE": str(n), "LOCAL_RANK": str(r), "LOCAL_WORLD_SIZE": str(n),
                    "MASTER_ADDR": "127.0.0.1", "MASTER_PORT": str(port), "DINO_BENCH_LAUNCHED": "1"})
        env.update(extra_env or {})
        procs.append(subprocess.Popen(cmd, env=env))
    rc = 0
    try:
        pending = list(procs)
        while pending:
            for p in list(pending):
                r = p.poll()
                if r is None:
                    continue
                pending.remove(p)
                if r != 0 and rc == 0:
                    rc = r
                    for q in pending:  # one rank failed: the others would wait at a barrier forever
                        q.terminate()
            time.sleep(0.05)
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
                p.wait()
    return rc


# ----------------------------------------------------------------------------- timing
def run_leg(pipe, d_bytes, d_off, n_img: int, B: int, steps: int, warmup: int, world: int, dist,
            maskgen=None, serial: bool = True) -> dict:
    """Time exactly ``steps`` device-resident batches (after ``warmup``), bracketed by a
    barrier + synchronize; then (``serial``) the same number of batches one at a time with
    the library's HIP-event timer (a kernel's events must not also span the other slots'
    concurrently running kernels)."""
    import torch
    ccfg = pipe._cfg(*pipe._sizes())
    views = [sl.engine.alloc_views(ccfg, B) for sl in pipe._slots]  # one output set per in-flight slot
    n_batches = max(1, n_img // B)

    def step(k: int):
        s = (k % n_batches) * B
        pipe.run_device_batch(d_bytes, d_off[s:s + B + 1], B, views=views[k % pipe.depth])
        if maskgen is not None:  # one mask per batch, broadcast to [B, H*W] (loader.py:585-590)
            maskgen.generate(1).expand(B, -1)

    # every batch's per-image status ([B, 4] int32 from the batch's own kernels) goes to a pinned
    # row asynchronously on the batch's stream, inside the timed region (an 8 KiB copy per
    # batch); all of them are checked afterwards: a timed batch with a zero-filled image
    # (anything but the reference's own corrupt -> zeros, cpu.py:250-253, none of which the
    # synthetic sets hold) fails the leg instead of raising its rate unseen
    n_rows = warmup + 2 * steps
    status = torch.zeros((n_rows, B, 4), dtype=torch.int32, pin_memory=True)

    def record_status(k: int):
        sl = pipe._last
        with sl.engine.on_stream():
            status[k].copy_(sl.info, non_blocking=True)

    for k in range(warmup):
        step(k)
        record_status(k)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for k in range(steps):
        step(warmup + k)
        record_status(warmup + k)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    dt = time.perf_counter() - t0
    out = {"dt": dt, "ktimes": {}, "t_ser": None, "last_batch": None}
    if serial:
        pipe.set_timing(True)
        pipe.kernel_times()
        t_ser = time.perf_counter()
        for k in range(steps):
            step(warmup + steps + k)
            record_status(warmup + steps + k)
            torch.cuda.synchronize()
        out["t_ser"] = time.perf_counter() - t_ser
        out["ktimes"] = pipe.kernel_times()
        pipe.set_timing(False)
        k_last = warmup + 2 * steps - 1  # the batch the last slot still holds
        out["last_batch"] = (k_last % n_batches) * B
    rows = warmup + steps * (2 if serial else 1)
    st = status[:rows, :, 0].numpy()
    if (st != 0).any():
        codes, counts = np.unique(st[st != 0], return_counts=True)
        bad_rows = sorted(set(np.nonzero(st)[0].tolist()))
        raise RuntimeError(f"bench: {int((st != 0).sum())} image(s) not decoded in batches {bad_rows[:8]} "
                           f"(status codes {dict(zip(codes.tolist(), counts.tolist()))})")
    out["statuses_checked"] = int(steps * B)            # the timed batches' images, all status 0
    out["statuses_checked_total"] = int(rows * B)        # + warm-up + serialized pass
    out["recs"] = pipe.last_params()
    return out


def load_traffic(tag: str) -> tuple[dict, str | None]:
    """Per-launch HBM bytes per kernel from the newest committed PMC summary of this
    workload (``profiles/r*_pmc_<tag>.json``: FETCH_SIZE and WRITE_SIZE passes of this bench
    under rocprofv3, scripts/gpu_pmc.sh; corrections of MI355X_MICROARCH.md §HBM)."""
    cands = sorted((ROOT / "profiles").glob(f"r*_pmc_{tag}.json"), reverse=True)
    if tag == "c2":
        cands.append(ROOT / "profiles" / "r02_pmc_traffic.json")
    for f in cands:
        if f.exists():
            try:
                d = json.loads(f.read_text())
                return {k: v.get("hbm_bytes_per_launch") for k, v in d.items() if not k.startswith("_")}, f.name
            except Exception:  # noqa: BLE001
                pass
    return {}, None


def summarize(leg: dict, ab: dict, B: int, steps: int, world: int, tag: str) -> dict:
    """value / ms per step / per-kernel times / the dominant kernel's roofline for one leg."""
    dt = leg["dt"]
    per_kernel = {k: {"avg_ms": (ms / n if n else 0.0), "launches": n, "total_ms": ms}
                  for k, (ms, n) in leg["ktimes"].items()}
    traffic, traffic_src = load_traffic(tag)
    out = {"value": round(world * steps * B / dt, 1), "ms_per_step": round(dt / steps * 1e3, 3),
           "mean_jpeg_bytes": round(ab["s_jpeg"]), "mean_pixels": round(ab["pixels"]),
           "statuses_checked": leg.get("statuses_checked"), "statuses_checked_total": leg.get("statuses_checked_total")}
    if per_kernel:
        # per step: a kernel launched once per view class (k_hresize, k_rcoeffs: twice per step)
        # is charged all its launches of the step, never one launch
        lps = {k: v["launches"] / max(steps, 1) for k, v in per_kernel.items()}
        step_ms = {k: v["total_ms"] / max(steps, 1) for k, v in per_kernel.items()}
        dom = max(per_kernel, key=lambda k: step_ms[k])
        # algorithmic bytes per image = S_jpeg + sum over views of 3 S^2 x out bytes;
        # a step processes the batch of B images, its launches of the dominant kernel share them
        bytes_step = ab["path"] * B
        bytes_launch = bytes_step / max(lps[dom], 1e-9)
        achieved = bytes_step / (step_ms[dom] * 1e-3) / 1e9
        dom_traffic = traffic.get(dom)
        dom_iface = ab.get(dom, 0.0) * B / max(lps[dom], 1e-9)   # the kernel's own interface bytes per launch
        path_gbs = ab["path"] * B * world / (dt / steps) / 1e9
        path_frac = round(path_gbs / PEAK_HBM_GBS / max(world, 1), 5)
        out["roofline"] = {
            "bound": "hbm", "achieved": round(achieved, 2), "peak": PEAK_HBM_GBS, "unit": "GB/s",
            "frac": round(achieved / PEAK_HBM_GBS, 5), "traffic": dom_traffic, "kernel": dom,
            "algorithmic_bytes_per_launch": int(bytes_launch), "avg_launch_ms": round(per_kernel[dom]["avg_ms"], 4),
            "launches_per_step": round(lps[dom], 3), "kernel_ms_per_step": round(step_ms[dom], 4),
            "interface_bytes_per_launch": int(dom_iface) if dom_iface else None,
            "traffic_over_interface": round(dom_traffic / dom_iface, 3) if dom_traffic and dom_iface else None,
            "path_frac": path_frac,
            "definition": "SURVEY 8(d) bytes per image (S_jpeg + 3*sum(S_v^2)*out_bytes) x batch (bytes of a "
                          "step) / the dominant kernel's time per step (sum of its launches' HIP-event times on "
                          "its stream, serialized pass after the timed region); per launch: bytes / launches "
                          "per step over the mean launch time (the same ratio). path_frac: the whole timed step "
                          "against the same bytes. traffic: PMC HBM bytes per launch (rocprofv3, "
                          "traffic_source); traffic_over_interface: that over the kernel's own interface bytes",
            "traffic_source": f"profiles/{traffic_src}" if traffic_src else None,
            "ceiling_note": "SURVEY 8(d): the algorithmic bytes (JPEG in + views out, ~1.1 MB per C2 image) "
                            "put the whole path at ~1-3 % of HBM even at ~200k img/s; it is bound by serial "
                            "entropy decode and per-pixel integer work, so a 70 % HBM-roofline target is out "
                            "of reach by this definition (SURVEY 8(d) 'Honest expectation'). frac and "
                            "path_frac are reported as measured, not rescaled"}
        roof_all = {}
        for k, v in per_kernel.items():
            if ab.get(k) and v["avg_ms"] > 0:
                gbs = ab[k] * B / (step_ms[k] * 1e-3) / 1e9
                iface_launch = ab[k] * B / max(lps[k], 1e-9)
                tr = traffic.get(k)
                roof_all[k] = {"achieved_GBs": round(gbs, 1), "frac": round(gbs / PEAK_HBM_GBS, 4),
                               "avg_ms": round(v["avg_ms"], 4), "launches_per_step": round(lps[k], 3),
                               "ms_per_step": round(step_ms[k], 4),
                               "interface_bytes_per_step": int(ab[k] * B),
                               "interface_bytes_per_launch": int(iface_launch),
                               "traffic_bytes_per_launch": tr,
                               "traffic_over_interface": round(tr / iface_launch, 3) if tr else None}
        out["roofline_kernels"] = roof_all
        out["kernels_ms_per_step"] = {k: round(v["total_ms"] / steps, 4) for k, v in per_kernel.items() if v["launches"]}
        step_traffic = sum((traffic.get(k) or 0) * v["launches"] / max(steps, 1) for k, v in per_kernel.items()) \
            if traffic else None
        out["path_roofline"] = {"algorithmic_bytes_per_image": int(ab["path"]), "achieved_GBs": round(path_gbs, 2),
                                "frac": path_frac,
                                "pmc_traffic_bytes_per_step": int(step_traffic) if step_traffic else None,
                                "algorithmic_bytes_per_step": int(ab["path"] * B)}
    if leg.get("t_ser") is not None:
        out["serialized_ms_per_step"] = round(leg["t_ser"] / steps * 1e3, 3)
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


class _GilSampler:
    """Study tool (DINO_GIL_SAMPLER=1): a thread that wakes every 0.5 ms and charges the time
    it took to get the GIL back to the line each other thread was on when it got it (the
    line that held the GIL, or the one that just dropped it)."""

    def __init__(self):
        import threading
        from collections import Counter
        self._stop = threading.Event()
        self.hist: dict = {}
        self._C = Counter
        self._t = threading.Thread(target=self._run, daemon=True)
        self._t.start()

    def _run(self):
        import threading
        me = threading.get_ident()
        names = {}
        while not self._stop.is_set():
            t = time.perf_counter()
            time.sleep(0.0005)
            late = time.perf_counter() - t - 0.0005
            for tid, fr in sys._current_frames().items():
                if tid == me:
                    continue
                if tid not in names:
                    names[tid] = next((th.name for th in threading.enumerate() if th.ident == tid), str(tid))
                f = fr
                key = f"{Path(f.f_code.co_filename).name}:{f.f_lineno}:{f.f_code.co_name}"
                h = self.hist.setdefault(names[tid], self._C())
                h[key] += late

    def stop(self) -> dict:
        self._stop.set()
        self._t.join()
        return {n: [(k, round(v * 1e3, 2)) for k, v in h.most_common(8)] for n, h in self.hist.items()}


def run_e2e(args, uniq, rank: int, world: int, cfg, B: int, dist) -> dict:
    """C5 end-to-end, through the drop-in path: tar shards in /dev/shm (reference cache file
    format) -> ShardBatchFeeder (native tar index) -> ``MI355XBackend.build_pipeline`` (prefetch
    thread: dino_gather into pinned staging + dino_probe) + ``build_pipeline_iterator``
    (``PipelineConfig.gpu_queue`` batches in flight) -> H2D -> Stage 3; ``next()`` hands each
    batch's views to the caller's stream as DINODataLoader consumes them (dali_node.py:110)."""
    import torch

    from dataloader_amd.backend import MI355XBackend
    from dataloader_amd.config import DinoV2AugSpec, PipelineConfig
    from dataloader_amd.tario import NativeShardFeed, ShardBatchFeeder, ShmShardCache

    if os.environ.get("DINO_SWITCH_INTERVAL"):  # study knob: the GIL hand-off interval
        sys.setswitchinterval(float(os.environ["DINO_SWITCH_INTERVAL"]))
    pcfg = PipelineConfig(device_id=torch.cuda.current_device(), seed=1234 + rank, gpu_queue=args.gpu_queue,
                          output_dtype=args.dtype if args.dtype != "fp8" else "bf16",
                          dali_fp8_output=args.dtype == "fp8")
    backend = MI355XBackend(max_in_flight=args.e2e_in_flight)
    depth = backend.queue_depth(pcfg, B)
    # steady state: a timed window of e2e_steps batches after e2e_warmup, over a
    # set of at least 4 x the side look-ahead (the look-ahead then never spans the set)
    steps, warm = args.e2e_steps, max(args.warmup, args.e2e_warmup)
    look = backend.side_look_ahead(pcfg, None, depth)
    n_batches = max(warm + steps + depth + 8, 4 * look)
    n = n_batches * B
    # distinct shard files (Stage 1's output); their contents repeat a few tars of the distinct
    # encodes so that the bench holds only those in memory
    per = args.shard_size
    n_shards = -(-n // per)
    blobs = [make_shards([uniq[(k * 7919 + i) % len(uniq)] for i in range(per)], per)[0]
             for k in range(min(n_shards, 8))]
    cache = ShmShardCache(job_id=f"dino_bench_{os.getpid()}", base_dir="/dev/shm", max_gb=64.0)
    try:
        paths = [f"/synthetic/rank{rank}/shard-{k:05d}.tar" for k in range(n_shards)]
        for k, p in enumerate(paths):
            cache.put(p, blobs[k % len(blobs)])  # Stage 1 (filesystem -> /dev/shm) is outside the timed region
        del blobs
        if args.e2e_feed == "native":
            # seeded per-epoch shard order + in-shard sample order (hpc_source.py:263, 461-467)
            feeder = NativeShardFeed(cache, paths, B, nthreads=args.gather_threads, slots=depth + 3,
                                     shuffle=True, seed=1234 + rank, rank=0, world=1)  # per-rank path set
        else:
            feeder = ShardBatchFeeder(cache, paths, B, nthreads=args.gather_threads)
        spec = DinoV2AugSpec(aug_cfg=cfg)
        pipe = backend.build_pipeline(feeder, spec, pcfg, None)
        it = backend.build_pipeline_iterator(pipe, spec, spec.output_map, B)
        for _ in range(warm):
            out = next(it)
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        sampler = _GilSampler() if os.environ.get("DINO_GIL_SAMPLER") else None
        t0 = time.perf_counter()
        for _ in range(steps):
            out = next(it)
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        dt = time.perf_counter() - t0
        if sampler is not None:
            print(json.dumps({"gil_sampler": sampler.stop()}), file=sys.stderr, flush=True)
        assert len(out) == 1 and len(out[0]) == cfg.n_views
        st = pipe.flush_stats()
        if os.environ.get("DINO_TIMELINE") == "1":  # study: per-batch host / device timeline
            Path("gpurun_out").mkdir(exist_ok=True)
            Path("gpurun_out/timeline_e2e.json").write_text(json.dumps(pipe.timeline()))
        bad = {k: v for k, v in st["status"].items() if k != 0}
        if bad:
            raise RuntimeError(f"e2e decode failures: {bad}")
        res = {"e2e_images_per_s": round(world * steps * B / dt, 1),
               "statuses_checked": int(st["images"]), "batches_accounted": int(st["batches"]),
               "e2e_ms_per_step": round(dt / steps * 1e3, 3),
               "e2e_steps": steps, "e2e_warmup": warm, "e2e_set_batches": n_batches, "e2e_shards": n_shards,
               "e2e_shuffle": args.e2e_feed == "native", "e2e_side_look_ahead": look,
               "e2e_shard_prepare_ms_total": round(getattr(feeder, "index_seconds", 0.0) * 1e3, 3),
               "e2e_shard_wait_ms_total": round(getattr(feeder, "wait_seconds", 0.0) * 1e3, 3),
               "e2e_gather_threads": args.gather_threads, "e2e_batches_in_flight": pipe.depth,
               "e2e_host_ms_per_batch": {k: round(v * 1e3 / max(1, warm + steps), 3)
                                         for k, v in pipe.host_seconds.items()},
               "e2e_prefetch_ahead": pipe.prefetch_ahead,
               "e2e_feed": args.e2e_feed,
               "e2e_path": ("/dev/shm tar shards (shard_cache file format) -> NativeShardFeed (C++ opener + packer "
                            "threads: mmap, pre-fault, tar index, pack + probe into pinned slots) -> "
                            "MI355XBackend.build_pipeline + build_pipeline_iterator -> H2D -> Stage 3")
                           if args.e2e_feed == "native" else
                           ("/dev/shm tar shards (shard_cache file format) -> ShardBatchFeeder -> "
                            "MI355XBackend.build_pipeline (prefetch thread: dino_gather_probe into pinned staging) "
                            "+ build_pipeline_iterator -> H2D -> Stage 3")}
        if hasattr(feeder, "stats"):
            res["e2e_feed_stats"] = {k: (round(v, 4) if isinstance(v, float) else v) for k, v in feeder.stats().items()}
        feeder.close()
        pipe.close()
        return res
    finally:
        cache.close(remove=True)


class _ProgMixSource:
    """A callable source with the reference's conventions (``_batch_size``, ``_resolution_src``;
    _ReaderAdapter.__call__, shard_reader.py:346-376): batch k holds the C2 images with one
    image in every ``1 / prog_frac`` replaced by a progressive encode (a different set each batch)."""

    def __init__(self, base, prog, B: int, prog_frac: float, n_batches: int):
        self._base, self._prog, self._B = base, prog, B
        self._every = max(1, int(round(1.0 / prog_frac)))
        self._n = n_batches
        self._k = 0
        self._batch_size = B
        self._resolution_src = None
        self.progressive_pulled = 0

    def __call__(self):
        if self._k >= self._n:
            raise StopIteration
        k, B = self._k, self._B
        self._k += 1
        out = [self._base[(k * B + i) % len(self._base)] for i in range(B)]
        t = 0
        for i in range(k % self._every, B, self._every):
            out[i] = self._prog[(k * 61 + t) % len(self._prog)]
            t += 1
        self.progressive_pulled += t
        return out


def _side_stats(pipe) -> dict | None:
    """The side decoder's launches: pools, images, host seconds per phase on its launcher
    thread, and (DINO_SIDE_TIMING=1) each launch's GPU span."""
    sd = getattr(pipe, "_side", None)
    if sd is None:
        return None
    out = {"launches": sd.launches, "lane_launches": sd.lane_launches, "images": sd.images,
           "urgent_flushes": pipe.stats.get("side_urgent", 0),
           "launcher_s": {k: round(v, 3) for k, v in sd.phase_seconds.items()},
           "per_batch_ms": {k: round(v * 1e3 / max(1, sd.lead["jobs"]), 2) for k, v in sd.lead.items() if k != "jobs"}}
    if sd.timing:
        ms = sd.launch_ms()
        out["gpu_ms_per_launch"] = [m for m, _ in ms][:64]
        out["images_per_launch"] = [n for _, n in ms][:64]
    return out


def run_prog_leg(args, uniq, uniq_prog, rank: int, world: int, cfg, B: int, dist) -> dict:
    """Progressive mix through the drop-in path: ``MI355XBackend.build_pipeline``
    + ``build_pipeline_iterator`` with the backend's default routing, on C2 batches in which one
    image in 16 is a progressive JPEG (16 per 256; web datasets hold such files, the GPU peer
    decodes them on the device, reference pipeline.py:429-434).  Host-fed (the source returns
    JPEG byte lists, as _ReaderAdapter does); the warm-up fills the side look-ahead first."""
    import torch

    from dataloader_amd.backend import MI355XBackend
    from dataloader_amd.config import DinoV2AugSpec, PipelineConfig

    pcfg = PipelineConfig(device_id=torch.cuda.current_device(), seed=4321 + rank, gpu_queue=args.gpu_queue)
    backend = MI355XBackend()
    # the warm-up fills the side look-ahead; the timed window spans several side pools
    ahead = backend.side_look_ahead(pcfg, None, 3)
    warm = max(args.warmup, ahead + 16)
    steps = max(args.steps, 96, 2 * ahead)
    src = _ProgMixSource(uniq, uniq_prog, B, args.prog_mix, warm + steps + 64)
    spec = DinoV2AugSpec(aug_cfg=cfg)
    pipe = backend.build_pipeline(src, spec, pcfg, None)
    it = backend.build_pipeline_iterator(pipe, spec, spec.output_map, B)
    try:
        for _ in range(warm):
            out = next(it)
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        t0 = time.perf_counter()
        for _ in range(steps):
            out = next(it)
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        dt = time.perf_counter() - t0
        assert len(out) == 1 and len(out[0]) == cfg.n_views
        st = pipe.flush_stats()
        bad = {k: v for k, v in st["status"].items() if k != 0}
        if bad:
            raise RuntimeError(f"c2_prog decode failures: {bad}")
        handed = warm + steps
        prog_handed = sum(len(range(k % src._every, B, src._every)) for k in range(handed))
        return {"value": round(world * steps * B / dt, 1), "ms_per_step": round(dt / steps * 1e3, 3),
                "steps": steps, "warmup": warm, "progressive_per_batch": len(range(0, B, src._every)),
                "progressive_frac": round(1.0 / src._every, 5),
                "route": pipe._multiscan_route, "side_ahead": pipe._side_ahead, "batches_in_flight": pipe.depth,
                "statuses_checked": int(st["images"]), "batches_accounted": int(st["batches"]),
                "side_decoded": int(st["side_decoded"]), "host_decoded": int(st["host_decoded"]),
                "progressive_handed_over": prog_handed,
                "host_ms_per_batch": {k: round(v * 1e3 / max(1, handed), 3) for k, v in pipe.host_seconds.items()},
                "side": _side_stats(pipe),
                "workload": f"C2 (640x480 q85, B = {B}) with one image in {src._every} a progressive encode "
                            f"({len(uniq_prog)} distinct), host-fed through MI355XBackend.build_pipeline "
                            "(default route) + build_pipeline_iterator"}
    finally:
        pipe.close()


# ----------------------------------------------------------------------------- main
def build_parser() -> argparse.ArgumentParser:
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=None,
                    help="ranks (one GPU each); without a launcher env bench.py starts them itself")
    ap.add_argument("--rehearsal", action="store_true",
                    help="allow more ranks than GPUs (round-robin sharing; the line is marked as a rehearsal)")
    ap.add_argument("--dry-run", action="store_true",
                    help="launcher + rank aggregation only, no GPU work (CPU tests of the N-rank path)")
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
    ap.add_argument("--restart-mcus", type=int, default=0,
                    help="restart interval (MCUs) of the encodes: the DRI variant of SURVEY 8(d)")
    ap.add_argument("--masks", action="store_true", help="iBOT masks per batch (default with --mixed)")
    ap.add_argument("--dtype", default="bf16", choices=["bf16", "fp8", "fp32"])
    ap.add_argument("--cpu-seconds", type=float, default=10.0, help="time budget of each CPU-baseline leg")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-extras", action="store_true",
                    help="N = 1: skip the c3 / fp8 / c2_dri / e2e legs (profiling runs)")
    ap.add_argument("--extra-unique", type=int, default=1024, help="distinct encodes of the c3 / c2_dri legs")
    ap.add_argument("--h2d", action="store_true", help="also time the H2D-inclusive rate (pinned host bytes)")
    ap.add_argument("--kernel-json", default="", help="write per-kernel times here (rank 0)")
    ap.add_argument("--e2e", action="store_true", help="C5 end-to-end leg even with --no-extras or N > 1")
    ap.add_argument("--gpu-queue", type=int, default=6, help="PipelineConfig.gpu_queue of the e2e leg")
    ap.add_argument("--shard-size", type=int, default=1000, help="samples per synthetic tar shard (e2e)")
    ap.add_argument("--e2e-steps", type=int, default=200, help="timed batches of the e2e leg (steady state)")
    ap.add_argument("--e2e-warmup", type=int, default=16, help="untimed batches of the e2e leg (at least --warmup)")
    ap.add_argument("--gather-threads", type=int, default=8, help="copier threads of the e2e feed")
    ap.add_argument("--e2e-in-flight", type=int, default=3, help="MI355XBackend(max_in_flight) of the e2e leg")
    ap.add_argument("--e2e-feed", default="native", choices=["native", "python"],
                    help="e2e host half: the native shard feed (C++ threads) or the Python prefetch thread")
    ap.add_argument("--legs", default="fp8,c3,c2_dri,c2_prog,e2e",
                    help="extra legs to run (comma list; the default line runs all)")
    ap.add_argument("--only-leg", default="", choices=["", "c2_prog", "e2e"],
                    help="internal: run this leg alone and print its JSON (the c2_prog and, at N = 1, e2e "
                         "legs run in child processes)")
    ap.add_argument("--prog-mix", type=float, default=1.0 / 16,
                    help="c2_prog leg: share of progressive images per batch (0: skip the leg)")
    return ap


def _procs(args, world: int) -> int:
    if args.procs >= 0:
        return args.procs
    try:
        share = len(os.sched_getaffinity(0))
    except AttributeError:
        share = os.cpu_count() or 4
    return max(2, min(16, share // max(1, world)))


def _maps_at_exit(path: str) -> None:
    """Study hook (DINO_EXIT_MAPS=path): the process's library map written at interpreter exit,
    to resolve the PCs of a crash during library finalization."""
    import atexit

    def dump():
        try:
            Path(path).write_text(Path("/proc/self/maps").read_text())
        except OSError:
            pass
    atexit.register(dump)


if os.environ.get("DINO_EXIT_MAPS"):  # every process of the run, spawn workers included ({pid})
    _maps_at_exit(os.environ["DINO_EXIT_MAPS"].replace("{pid}", str(os.getpid())))


def main(argv: list[str] | None = None) -> int:
    argv = list(sys.argv[1:] if argv is None else argv)
    args = build_parser().parse_args(argv)
    launched = "WORLD_SIZE" in os.environ
    if not launched and (args.gpus or 1) > 1:
        devices = int(os.environ.get("DINO_BENCH_DEVICES", args.gpus)) if args.dry_run else visible_devices()
        return launch_ranks(args.gpus, argv, devices, args.rehearsal)
    rank = int(os.environ.get("RANK", 0))
    world = int(os.environ.get("WORLD_SIZE", 1))
    local_rank = int(os.environ.get("LOCAL_RANK", 0))
    if args.gpus is not None and args.gpus != world:
        raise SystemExit(f"bench.py: --gpus {args.gpus} but the launcher started {world} rank(s)")
    if args.dry_run:
        return dry_run(args, rank, world, local_rank)
    if args.only_leg:
        return run_leg_only(args)
    return run_rank(args, rank, world, local_rank)


def run_leg_only(args) -> int:
    """One host-fed leg in a process of its own (what a training job has: one loader
    pipeline per process).  After the other legs in their process the c2_prog leg measured
    57-70k img/s against 95-110k in a fresh one, and the e2e leg 95-127k against 135-142k
    (state left by earlier pipelines)."""
    procs = _procs(args, 1)
    uniq = make_unique(args.unique, args.width, args.height, 1, args.mixed, procs, args.progressive_frac,
                       args.restart_mcus)
    uniq_prog = make_unique(64, args.width, args.height, 31, False, procs, 1.0) if args.only_leg == "c2_prog" else None
    import torch
    torch.cuda.set_device(0)
    from dataloader_amd.config import DINOAugConfig
    if args.only_leg == "c2_prog":
        res = run_prog_leg(args, uniq, uniq_prog, 0, 1, DINOAugConfig(), args.batch, None)
    else:
        res = run_e2e(args, uniq, 0, 1, DINOAugConfig(), args.batch, None)
    print(json.dumps(res), flush=True)
    return 0


def run_leg_child(args, leg: str) -> dict:
    """Start ``bench.py --only-leg <leg>`` as a child process (same data seeds and sizes)
    and return its leg record."""
    import subprocess
    cmd = [sys.executable, str(Path(__file__).resolve()), "--only-leg", leg, "--steps", str(args.steps),
           "--warmup", str(args.warmup), "--batch", str(args.batch), "--unique", str(args.unique),
           "--procs", str(args.procs), "--width", str(args.width), "--height", str(args.height),
           "--prog-mix", str(args.prog_mix), "--gpu-queue", str(args.gpu_queue),
           "--progressive-frac", str(args.progressive_frac), "--restart-mcus", str(args.restart_mcus),
           "--shard-size", str(args.shard_size), "--gather-threads", str(args.gather_threads),
           "--e2e-steps", str(args.e2e_steps), "--e2e-warmup", str(args.e2e_warmup),
           "--e2e-in-flight", str(args.e2e_in_flight), "--e2e-feed", args.e2e_feed]
    if args.mixed:
        cmd.append("--mixed")
    env = {k: v for k, v in os.environ.items() if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK")}
    out = subprocess.run(cmd, capture_output=True, text=True, timeout=900, env=env)
    if out.returncode != 0:
        raise RuntimeError(f"{leg} child failed ({out.returncode}): {out.stderr[-2000:]}")
    res = json.loads(out.stdout.strip().splitlines()[-1])
    res["process"] = "child (a fresh process, as a training job's loader)"
    return res


def _init_group(world: int):
    import torch.distributed as dist
    if world > 1:
        # barrier + MAX / gather of the per-rank times only: a CPU (gloo) group, no RCCL on this path
        dist.init_process_group("gloo")
    return dist


def _rank_report(dist, world: int, rank: int, device: int, dt: float, steps: int, B: int) -> tuple[float, list]:
    """MAX of the per-rank elapsed times and every rank's own rate (gloo)."""
    mine = {"rank": rank, "device": device, "physical": physical_device(device),
            "ms_per_step": round(dt / steps * 1e3, 3), "images_per_s": round(steps * B / dt, 1)}
    if world == 1:
        return dt, [mine]
    allr = [None] * world
    dist.all_gather_object(allr, mine)
    return max(r["ms_per_step"] for r in allr) * steps / 1e3, allr


def dry_run(args, rank: int, world: int, local_rank: int) -> int:
    """The N-rank plumbing without a GPU: env, gloo group, per-rank report, the rank-0 line."""
    dist = _init_group(world)
    devices = int(os.environ.get("DINO_BENCH_DEVICES", world))
    check_devices(world, devices, args.rehearsal)
    B, steps = args.batch, args.steps
    dt = 0.001 * steps * (1 + 0.1 * rank)  # a fake, rank-dependent elapsed time
    if world > 1:
        dist.barrier()
    dt_max, per_rank = _rank_report(dist, world, rank, local_rank % devices, dt, steps, B)
    distinct = check_distinct(per_rank, args.rehearsal)
    if rank == 0:
        line = {"metric": METRIC, "value": round(world * steps * B / dt_max, 1), "unit": "images/s",
                "n_gpus": distinct, "ranks": world, "steps": steps, "warmup": args.warmup,
                "ms_per_step": round(dt_max / steps * 1e3, 3), "dry_run": True, "per_rank": per_rank,
                "env": {"RANK": os.environ.get("RANK"), "WORLD_SIZE": os.environ.get("WORLD_SIZE"),
                        "LOCAL_RANK": os.environ.get("LOCAL_RANK"), "MASTER_ADDR": os.environ.get("MASTER_ADDR")}}
        if world > distinct:
            line["rehearsal"] = True
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()
    return 0


def run_rank(args, rank: int, world: int, local_rank: int) -> int:
    extras = world == 1 and not args.no_extras
    legs_on = set(args.legs.split(","))
    procs = _procs(args, world)
    # synthetic data first, before anything initialises the GPU in this process
    uniq = make_unique(args.unique, args.width, args.height, 1 + rank, args.mixed, procs, args.progressive_frac,
                       args.restart_mcus)
    if extras:
        print(f"bench: rank {rank}: synthesising the c3 / c2_dri sets", file=sys.stderr, flush=True)
        uniq_c3 = make_unique(args.extra_unique, 0, 0, 11 + rank, True, procs) \
            if not args.mixed and "c3" in legs_on else None
        uniq_dri = make_unique(args.extra_unique, args.width, args.height, 21 + rank, False, procs, 0.0, 4) \
            if not args.restart_mcus and "c2_dri" in legs_on else None
        # (the c2_prog leg synthesises its own sets in its child process)
        prog_on = args.prog_mix > 0 and not args.mixed and "c2_prog" in legs_on

    import torch
    devices = visible_devices()
    check_devices(world, devices, args.rehearsal)
    device = local_rank % devices  # distinct per rank unless --rehearsal
    torch.cuda.set_device(device)
    dev = torch.device("cuda", device)
    dist = _init_group(world)

    from dataloader_amd.config import DINOAugConfig
    from dataloader_amd.engine import pack_jpegs
    from dataloader_amd.masking import MaskingGenerator
    from dataloader_amd.pipeline import MI355XAugPipeline
    from dataloader_amd.sharding import rank_seed

    cfg = DINOAugConfig()
    B = args.batch
    out_bytes = {"bf16": 2, "fp8": 1, "fp32": 4}[args.dtype]

    def to_device(u, n_img):
        jp = [u[i % len(u)] for i in range(n_img)]
        hb, off = pack_jpegs(jp, pin=True)
        return jp, hb, off, hb.to(dev), off.to(dev)

    def make_maskgen():
        grid = cfg.global_crop_size // 14                     # patch 14: 16x16 at 224
        mg = MaskingGenerator((grid, grid), num_masking_patches=grid * grid // 2, device=dev)
        mg.seed(rank_seed(1234, rank))
        return mg

    def leg(u, n_img, mixed: bool, dtype: str, masks: bool, tag: str, steps: int, warmup: int, serial=True):
        jp, hb, off, d_bytes, d_off = to_device(u, n_img)
        torch.cuda.synchronize()
        pipe = MI355XAugPipeline(None, cfg, B, seed=rank_seed(1234, rank), out_dtype=dtype, device=device,
                                 max_image_dim=0, depth=args.depth,
                                 workspace_bytes=B * (40 << 20) if mixed else 0)
        try:
            res = run_leg(pipe, d_bytes, d_off, n_img, B, steps, warmup, world, dist,
                          maskgen=make_maskgen() if masks else None, serial=serial)
            ent_b = 0.0
            if res["last_batch"] is not None:
                s_last = res["last_batch"]
                ent_b = sparse_entry_bytes(pipe, jp[s_last:s_last + 16])
            ob = {"bf16": 2, "fp8": 1, "fp32": 4}[dtype]
            ab = algorithmic_bytes(u, cfg.global_crop_size, cfg.local_crop_size, cfg.n_global_crops,
                                   cfg.n_local_crops, ob, recs=res["recs"], entry_bytes_per_block=ent_b or 20.0)
            summ = summarize(res, ab, B, steps, world, tag)
            if "path_roofline" in summ:
                summ["path_roofline"]["sparse_entry_bytes_per_block"] = round(ent_b, 2)
            return res, summ, (pipe, hb, off)
        except BaseException:
            pipe.close()
            raise

    masks_on = args.masks or args.mixed
    main_tag = "c3" if args.mixed else ("fp8" if args.dtype == "fp8" else ("dri" if args.restart_mcus else "c2"))
    res, summ, (pipe, host_buf, offsets) = leg(uniq, args.images, args.mixed, args.dtype, masks_on, main_tag,
                                               args.steps, args.warmup)
    dt, per_rank = _rank_report(dist, world, rank, device, res["dt"], args.steps, B)
    distinct = check_distinct(per_rank, args.rehearsal)

    h2d_rate = None
    if args.h2d:
        ccfg = pipe._cfg(*pipe._sizes())
        views = [sl.engine.alloc_views(ccfg, B) for sl in pipe._slots]
        n_batches = args.images // B
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
    pipe.close()
    del host_buf, offsets
    torch.cuda.empty_cache()

    legs = {}
    if extras:
        n_extra = max(args.batch * (args.steps + args.warmup), 8 * B)
        if args.dtype == "bf16" and not args.mixed and not args.restart_mcus and "fp8" in legs_on:
            print("bench: fp8 leg", file=sys.stderr, flush=True)
            _, s_fp8, (p, _, _) = leg(uniq, args.images, False, "fp8", False, "fp8", args.steps, args.warmup)
            p.close()
            legs["fp8"] = dict(s_fp8, workload="C5 epilogue: C2 with FP8-E4M3 output (fused cast, scale 1)")
        if uniq_c3 is not None:
            print("bench: c3 leg", file=sys.stderr, flush=True)
            torch.cuda.empty_cache()
            _, s_c3, (p, _, _) = leg(uniq_c3, min(n_extra, 8192), True, args.dtype, True, "c3", args.steps,
                                     args.warmup)
            p.close()
            legs["c3"] = dict(s_c3, workload=f"C3: {args.extra_unique} distinct mixed-resolution JPEGs (short side "
                                             f"224-1600, aspect 3/4-4/3), B = {B}, iBOT masks 16x16, {args.dtype} out")
            torch.cuda.empty_cache()
        if uniq_dri is not None:
            print("bench: c2_dri leg", file=sys.stderr, flush=True)
            _, s_dri, (p, _, _) = leg(uniq_dri, n_extra, False, args.dtype, False, "dri", args.steps, args.warmup)
            p.close()
            legs["c2_dri"] = dict(s_dri, workload=f"C2 with restart markers every 4 MCUs (DRI), "
                                                  f"{args.extra_unique} distinct encodes, {args.dtype} out")
        if prog_on:
            print("bench: c2_prog leg", file=sys.stderr, flush=True)
            torch.cuda.empty_cache()
            legs["c2_prog"] = run_leg_child(args, "c2_prog")
            legs["c2_prog"]["vs_c2"] = round(legs["c2_prog"]["value"] / (world * args.steps * B / dt), 4)
    e2e = None
    if args.e2e or (extras and "e2e" in legs_on):
        print("bench: e2e leg", file=sys.stderr, flush=True)
        # N = 1: in a child process, as c2_prog (N > 1: in the ranks, for their barriers)
        e2e = run_leg_child(args, "e2e") if world == 1 else run_e2e(args, uniq, rank, world, cfg, B, dist)

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        print("bench: cpu baseline", file=sys.stderr, flush=True)
        c1 = make_unique(256, 256, 256, 7, False, procs)
        cpu = cpu_baseline(uniq if not args.mixed else uniq[:256], c1, args.cpu_seconds)
    if rank == 0:
        ms_step = dt / args.steps * 1e3
        line = {
            "metric": METRIC, "value": round(world * args.steps * B / dt, 1), "unit": "images/s",
            "n_gpus": distinct, "ranks": world,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(ms_step, 3),
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "u8",
            "data": "synthetic",
            "config": {"workload": ("C3 mixed short side 224-1600, iBOT masks 16x16" if args.mixed else
                                    f"C2 {args.images} synthetic {args.width}x{args.height} q85 4:2:0 JPEGs "
                                    "resident in HBM") + (f", DRI every {args.restart_mcus} MCUs" if args.restart_mcus
                                                          else "") + f", 2x224^2+8x96^2 views, {args.dtype} out",
                       "global_batch": B * world, "batch_per_gpu": B, "parallelism": f"dp{world}",
                       "batches_in_flight": args.depth, "masks": masks_on,
                       "mean_jpeg_bytes": summ["mean_jpeg_bytes"], "out_dtype": args.dtype,
                       "progressive_frac": args.progressive_frac},
            "per_rank": per_rank,
            "roofline": summ.get("roofline"),
            "roofline_kernels": summ.get("roofline_kernels"),
            "path_roofline": summ.get("path_roofline"),
            "kernels_ms_per_step": summ.get("kernels_ms_per_step"),
            "statuses_checked": summ.get("statuses_checked"),
            "serialized_ms_per_step": summ.get("serialized_ms_per_step"),
            "cpu_baseline": cpu,
        }
        if world > distinct:
            line["rehearsal"] = True
            line["note"] = f"{world} ranks shared {distinct} device(s): not a scaling measurement"
        line.update(legs)
        if h2d_rate is not None:
            line["h2d_inclusive_images_per_s"] = round(h2d_rate, 1)
        if e2e is not None:
            line["e2e"] = e2e
        print(json.dumps(line), flush=True)
        if args.kernel_json:
            Path(args.kernel_json).write_text(json.dumps(res["ktimes"], indent=1))
    if world > 1:
        dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())
