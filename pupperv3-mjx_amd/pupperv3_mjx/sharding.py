"""Env sharding across GPUs (one process per GPU) and the optional learner gather.

SURVEY.md 8(e): envs are independent, so a global batch of G envs is cut into contiguous
per-rank shards with no collective inside the step.  Env i of the global batch gets the same
PRNG key (``jax.random.split(PRNGKey(seed), G)[i]``) whatever the world size, so a sharded run
reproduces the single-GPU run env-for-env.  The only collective is the optional per-step
gather of ``obs | reward | done`` to every rank (RCCL all_gather over xGMI on GPUs; gloo on CPU
in tests), sized for uneven shards by padding to the largest shard.
"""
from __future__ import annotations

from typing import Tuple

import numpy as np

from . import rng


def shard_bounds(global_envs: int, world: int, rank: int) -> Tuple[int, int]:
    """(first env id, env count) of `rank`'s contiguous shard; the remainder goes to low ranks."""
    if world < 1 or not 0 <= rank < world:
        raise ValueError(f"bad rank {rank} for world {world}")
    if global_envs < world:
        raise ValueError(f"{global_envs} envs cannot be sharded over {world} ranks")
    base, rem = divmod(global_envs, world)
    count = base + (1 if rank < rem else 0)
    start = rank * base + min(rank, rem)
    return start, count


def shard_keys(seed: int, global_envs: int, world: int, rank: int, partitionable: bool = True) -> np.ndarray:
    """Reset keys of this rank's shard: rows [start, start+count) of split(PRNGKey(seed), G)."""
    start, count = shard_bounds(global_envs, world, rank)
    keys = rng.split(rng.PRNGKey(seed), global_envs, partitionable=partitionable)
    return np.ascontiguousarray(keys[start:start + count])


def gather_batch(obs, reward, done, global_envs: int, group=None):
    """All-gather this rank's (obs [n, D], reward [n], done [n]) torch tensors into global
    [G, D] / [G] / [G] tensors on every rank (torch.distributed; RCCL or gloo)."""
    import torch
    import torch.distributed as dist

    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    start, n = shard_bounds(global_envs, world, rank)
    nmax = shard_bounds(global_envs, world, 0)[1]
    D = obs.shape[1]
    local = torch.zeros((nmax, D + 2), dtype=torch.float32, device=obs.device)
    local[:n, :D] = obs
    local[:n, D] = reward
    local[:n, D + 1] = done
    full = torch.empty((world * nmax, D + 2), dtype=torch.float32, device=obs.device)
    dist.all_gather_into_tensor(full, local, group=group)
    rows = [full[r * nmax:r * nmax + shard_bounds(global_envs, world, r)[1]] for r in range(world)]
    out = torch.cat(rows, 0)
    return out[:, :D], out[:, D], out[:, D + 1]
