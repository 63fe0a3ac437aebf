"""Multi-GPU layout for the env step: envs shard trivially — one process per GPU,
contiguous env blocks, seed = base + rank (reference train.py:125-132), no collective on the data
path. Only the benchmark's timing uses a collective (max over ranks)."""
from __future__ import annotations

import os
from dataclasses import dataclass


@dataclass
class Shard:
    rank: int
    world: int
    local_rank: int
    envs_per_rank: int
    seed: int

    @property
    def env_offset(self) -> int:
        return self.rank * self.envs_per_rank

    @property
    def total_envs(self) -> int:
        return self.world * self.envs_per_rank


def shard_from_env(envs_per_rank: int, base_seed: int = 42) -> Shard:
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", str(rank)))
    return Shard(rank, world, local, envs_per_rank, base_seed + rank)


def max_over_ranks(value: float, device=None) -> float:
    """Max of a host scalar over all ranks (no-op without an initialised process group)."""
    import torch
    import torch.distributed as dist
    if not (dist.is_available() and dist.is_initialized()):
        return float(value)
    t = torch.tensor([float(value)], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())
