"""Multi-GPU sharding of env instances (one process per GPU).

Env instances are independent, so the step path needs no collective: rank r
of a world of size G owns global env ids [r*E_local, (r+1)*E_local) and seeds
each with ``base_seed + global_id`` -- exactly the seed VectorizedEnv would
give that env in a single process (MAPPO/env_vectorized.py:8-9), so every
env's stream is identical for any G.  The only collectives are outside the
timed step loop: a barrier and a MAX over per-rank wall times (throughput is
then total agent-steps / slowest rank), and an optional all-gather of
rollout tensors for a single learner.
"""
from __future__ import annotations

import os

import torch
import torch.distributed as dist


def world():
    """(rank, world_size, local_rank) from the torchrun environment."""
    return (int(os.environ.get("RANK", "0")), int(os.environ.get("WORLD_SIZE", "1")),
            int(os.environ.get("LOCAL_RANK", "0")))


def shard(envs_per_rank: int, rank: int, base_seed: int):
    """Global env ids and seeds of this rank (weak scaling: fixed envs per rank)."""
    first = rank * envs_per_rank
    ids = list(range(first, first + envs_per_rank))
    return ids, [base_seed + i for i in ids]


def shard_strong(total_envs: int, rank: int, world_size: int, base_seed: int):
    """Global env ids and seeds of this rank when a fixed total is split (strong scaling)."""
    per, rem = divmod(total_envs, world_size)
    first = rank * per + min(rank, rem)
    n = per + (1 if rank < rem else 0)
    ids = list(range(first, first + n))
    return ids, [base_seed + i for i in ids]


def max_over_ranks(values, device=None):
    """Element-wise MAX of a list of floats over all ranks (identity without a group)."""
    if not (dist.is_available() and dist.is_initialized()):
        return [float(v) for v in values]
    t = torch.tensor([float(v) for v in values], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return [float(x) for x in t.tolist()]


def sum_over_ranks(values, device=None):
    if not (dist.is_available() and dist.is_initialized()):
        return [float(v) for v in values]
    t = torch.tensor([float(v) for v in values], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.SUM)
    return [float(x) for x in t.tolist()]


def gather_rollout(t: torch.Tensor):
    """All-gather a per-rank rollout tensor along dim 0 (collation for one learner)."""
    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size() == 1:
        return t
    parts = [torch.empty_like(t) for _ in range(dist.get_world_size())]
    dist.all_gather(parts, t.contiguous())
    return torch.cat(parts, 0)
