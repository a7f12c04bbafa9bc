"""Multi-rank path on CPU: world_size 2 over gloo (the GPU run uses one process per GPU).

The hot path has no collective: each rank owns shards i % world == rank and
seeds with seed + rank.  The benchmark's only cross-rank ops are a barrier and
a MAX reduction of the elapsed time; both are exercised here over gloo.
"""

from __future__ import annotations

import os
import socket

import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank: int, world: int, port: int, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from dataloader_amd.sharding import RankInfo, rank_seed, rank_shards
    info = RankInfo.from_env()
    shards = [f"shard-{i:06d}.tar" for i in range(11)]
    mine = rank_shards(shards, info.rank, info.world_size)
    gathered = [None] * world
    dist.all_gather_object(gathered, mine)
    dist.barrier()
    elapsed = torch.tensor([0.5 + rank], dtype=torch.float64)
    dist.all_reduce(elapsed, op=dist.ReduceOp.MAX)
    if rank == 0:
        q.put((gathered, float(elapsed), [rank_seed(7, r) for r in range(world)], info.world_size))
    dist.destroy_process_group()


def test_two_rank_partition_and_timing():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    gathered, elapsed, seeds, world = q.get(timeout=120)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert world == 2
    a, b = gathered
    assert set(a).isdisjoint(b) and len(a) + len(b) == 11 and a[0] == "shard-000000.tar" and b[0] == "shard-000001.tar"
    assert elapsed == 1.5          # MAX over ranks, as bench.py reports
    assert seeds == [7, 8]         # seed + rank (reference config.py:204)


def _feed_worker(rank: int, world: int, port: int, base_dir: str, paths: list, q):
    """One rank of the real feed: its shards (i % world == rank) from the node cache written by
    the node master, native tar index + pinned gather per batch, the host pre-screen of each
    batch, and its seed (seed + rank).  Reports what it would hand to its GPU."""
    import hashlib

    import numpy as np
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from dataloader_amd import fallback
    from dataloader_amd.sharding import RankInfo, rank_seed
    from dataloader_amd.tario import ShardBatchFeeder, ShmShardCache, gather
    info = RankInfo.from_env()
    cache = ShmShardCache(job_id="dist", base_dir=base_dir, node_master=False)
    feeder = ShardBatchFeeder(cache, paths, 8, rank=info.rank, world=info.world_size, nthreads=2)
    staging = torch.empty(1 << 20, dtype=torch.uint8)
    batches = []
    while True:
        try:
            spans = feeder.next_spans()
        except StopIteration:
            break
        off = np.asarray(gather(spans, staging, 2), np.int64)
        st, ws, _ = fallback.probe(staging.data_ptr(), off, len(spans), 16384)
        blobs = [staging.numpy()[off[i]:off[i + 1]].tobytes() for i in range(len(spans))]
        batches.append(([hashlib.sha1(b).hexdigest() for b in blobs], st[:, 0].tolist(), ws))
    feeder.close()
    gathered = [None] * world
    dist.all_gather_object(gathered, (batches, rank_seed(1234, info.rank)))
    dist.barrier()
    if rank == 0:
        q.put(gathered)
    dist.destroy_process_group()


def test_two_rank_native_feed(tmp_path):
    """World size 2 over gloo through the real per-rank feed: disjoint samples whose union is
    every full batch of each rank's shards, identical results when re-run, per-rank seeds."""
    import hashlib
    import io
    import tarfile

    from dataloader_amd.synthetic import make_jpeg
    from dataloader_amd.tario import ShmShardCache
    jpegs = [make_jpeg(48 + 8 * (i % 5), 40, i) for i in range(70)]
    cache = ShmShardCache(job_id="dist", base_dir=tmp_path)
    paths, per_shard = [], []
    for s0 in range(0, 70, 10):  # 7 shards of 10 samples
        buf = io.BytesIO()
        with tarfile.open(fileobj=buf, mode="w") as tf:
            for i in range(s0, s0 + 10):
                ti = tarfile.TarInfo(f"sample_{i:06d}.jpg")
                ti.size = len(jpegs[i])
                tf.addfile(ti, io.BytesIO(jpegs[i]))
        paths.append(f"/node/shard-{s0 // 10:03d}.tar")
        cache.put(paths[-1], buf.getvalue())
        per_shard.append([hashlib.sha1(jpegs[i]).hexdigest() for i in range(s0, s0 + 10)])

    def run():
        ctx = mp.get_context("spawn")
        q = ctx.Queue()
        port = _free_port()
        procs = [ctx.Process(target=_feed_worker, args=(r, 2, port, str(tmp_path), paths, q)) for r in range(2)]
        for p in procs:
            p.start()
        out = q.get(timeout=180)
        for p in procs:
            p.join(timeout=60)
            assert p.exitcode == 0
        return out

    first, again = run(), run()
    assert first == again  # deterministic per rank
    (b0, s0), (b1, s1) = first
    assert (s0, s1) == (1234, 1235)
    seen = [[h for hs, _, _ in b for h in hs] for b in (b0, b1)]
    assert set(seen[0]).isdisjoint(seen[1])
    for r, seen_r in enumerate(seen):
        mine = [h for i, hs in enumerate(per_shard) if i % 2 == r for h in hs]
        assert seen_r == mine[: len(mine) // 8 * 8]  # shard order, last partial batch dropped
    assert all(st == [0] * 8 and ws > 0 for b in (b0, b1) for _, st, ws in b)
    cache.close(remove=True)
