"""Per-rank work partition for multi-GPU runs (no collective on the data path).

Mirrors the reference's data-parallel rules: shard ``i`` belongs to rank
``i % world_size`` (reference sources/hpc_source.py:154-156,
sources/wds_source.py:141-144) and every rank offsets its RNG seed by its rank
(reference config.py:204, ``seed = cfg.seed + rank``).  Each GPU process runs
its own ``dino_ctx`` on its own stream over its own shards; the only
cross-rank operations are the benchmark's barrier and MAX-of-elapsed.
"""

from __future__ import annotations

import os
from dataclasses import dataclass


@dataclass(frozen=True)
class RankInfo:
    rank: int = 0
    world_size: int = 1
    local_rank: int = 0

    @classmethod
    def from_env(cls) -> "RankInfo":
        """RANK/WORLD_SIZE/LOCAL_RANK (torchrun) with SLURM fallbacks (reference loader.py:648-674)."""
        def _get(*names, default=0):
            for n in names:
                v = os.environ.get(n)
                if v is not None:
                    return int(v)
            return default
        return cls(rank=_get("RANK", "SLURM_PROCID"), world_size=_get("WORLD_SIZE", "SLURM_NTASKS", default=1),
                   local_rank=_get("LOCAL_RANK", "SLURM_LOCALID"))


def rank_shards(shards: list, rank: int, world_size: int) -> list:
    """Shards owned by ``rank``: ``i % world_size == rank``."""
    if not 0 <= rank < world_size:
        raise ValueError(f"rank {rank} outside [0, {world_size})")
    return [s for i, s in enumerate(shards) if i % world_size == rank]


def rank_seed(seed: int, rank: int) -> int:
    """Per-rank pipeline seed (``PipelineConfig.from_loader_config``: seed + rank)."""
    return int(seed) + int(rank)
