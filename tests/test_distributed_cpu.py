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
