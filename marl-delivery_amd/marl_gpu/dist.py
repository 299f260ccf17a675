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

import bisect
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


def map_group_sizes(total_envs: int, n_maps: int):
    """Envs per map of a mixed-map batch laid out as contiguous map groups, the first groups
    taking the remainder: 65536 envs over map1..map5 -> 13108, 13107, 13107, 13107, 13107
    (SURVEY.md §8(d) config 4)."""
    per, rem = divmod(int(total_envs), int(n_maps))
    return [per + (1 if m < rem else 0) for m in range(n_maps)]


def shard_mixed(total_envs: int, n_maps: int, rank: int, world_size: int, base_seed: int):
    """This rank's part of a mixed-map batch (config 4).

    The global batch is the map groups back to back (``map_group_sizes``); global env g
    runs map ``env_map[g]`` with seed ``base_seed + g`` -- what one VectorizedEnv-style process
    would give it (MAPPO/env_vectorized.py:8-9) -- and rank r owns the contiguous global ids
    ``shard_strong`` deals it, so the map groups are dealt to ranks in contiguous blocks and a
    rank holds at most a few same-map runs.  Returns (global ids, seeds, local env -> map index,
    [(map index, first local env, n envs)] of the rank's runs)."""
    sizes = map_group_sizes(total_envs, n_maps)
    ids, seeds = shard_strong(total_envs, rank, world_size, base_seed)
    bounds = [0]
    for s in sizes:
        bounds.append(bounds[-1] + s)
    env_map, runs = [], []
    for local, g in enumerate(ids):
        m = bisect.bisect_right(bounds, g) - 1
        env_map.append(m)
        if runs and runs[-1][0] == m:
            runs[-1][2] += 1
        else:
            runs.append([m, local, 1])
    return ids, seeds, env_map, [tuple(r) for r in runs]


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


def gather_rollout(t: torch.Tensor, group=None):
    """All-gather a per-rank rollout tensor along dim 0, in rank order: the collation of every
    env's buffers for one learner (the reference's trainer stacks its per-env buffers on one host,
    MAPPO/trainer.py:172-286).  Shards may differ in their leading size (``shard_strong`` gives the
    lower ranks the remainder): the sizes are all-gathered first, every rank's part is padded to
    the largest, and the padding is dropped from the result.  The trailing dims must agree.  On
    RCCL the collective runs on the device tensors (one all_gather_into_tensor over xGMI); gloo
    has no device all-gather, so a CUDA tensor goes through host memory there (rehearsal only).
    Off the step path: one call per rollout, not per step."""
    if not (dist.is_available() and dist.is_initialized()):
        return t
    ws = dist.get_world_size(group)
    if ws == 1:
        return t
    t = t.contiguous()
    host = dist.get_backend(group) == "gloo" and t.is_cuda
    dev = torch.device("cpu") if host else t.device
    n = torch.tensor([t.shape[0]], dtype=torch.int64, device=dev)
    ns = [torch.zeros_like(n) for _ in range(ws)]
    dist.all_gather(ns, n, group=group)
    sizes = [int(x.item()) for x in ns]
    mx = max(sizes)
    src = t.to(dev) if host else t
    if t.shape[0] < mx:   # pad this rank's part to the common size
        pad = torch.zeros((mx - t.shape[0],) + tuple(t.shape[1:]), dtype=t.dtype, device=dev)
        src = torch.cat([src, pad], 0)
    if host:
        parts = [torch.empty_like(src) for _ in range(ws)]
        dist.all_gather(parts, src, group=group)
        flat = torch.cat(parts, 0)
    else:
        flat = torch.empty((ws * mx,) + tuple(t.shape[1:]), dtype=t.dtype, device=dev)
        dist.all_gather_into_tensor(flat, src, group=group)
    if min(sizes) < mx:
        flat = torch.cat([flat[r * mx:r * mx + sizes[r]] for r in range(ws)], 0)
    return flat.to(t.device) if host else flat
