"""Env-batch sharding over one process per GPU.

Envs are independent units: rank r owns the contiguous global range
[offset_r, offset_r + count_r) and steps it with no per-step collective.  The
global env index is part of every Philox key, so a trajectory does not depend
on how the batch is sharded.  The only collective is the optional
`gather_rollout`, an all-gather of per-env rollout scalars (reward f32, done /
is_goal bytes) — over RCCL (`backend="nccl"` on ROCm, xGMI) for GPU ranks,
gloo for CPU tests.  Observation planes are never gathered.
"""
from __future__ import annotations

import os
from typing import Dict, Optional, Tuple

import torch
import torch.distributed as dist


def shard_range(total: int, world: int, rank: int) -> Tuple[int, int]:
    """(offset, count) of `rank`'s contiguous share; the first total % world ranks get one more."""
    if world <= 0 or not 0 <= rank < world or total < 0:
        raise ValueError("bad shard request")
    base, extra = divmod(total, world)
    count = base + (1 if rank < extra else 0)
    offset = rank * base + min(rank, extra)
    return offset, count


def env_ranks() -> Tuple[int, int, int]:
    """(rank, world_size, local_rank) from the torchrun environment (defaults 0, 1, 0)."""
    return (int(os.environ.get("RANK", "0")), int(os.environ.get("WORLD_SIZE", "1")),
            int(os.environ.get("LOCAL_RANK", "0")))


def init(backend: Optional[str] = None, device: Optional[torch.device] = None) -> Tuple[int, int, int]:
    """Initialise the default process group if WORLD_SIZE > 1 (nccl == RCCL for GPU ranks)."""
    rank, world, local = env_ranks()
    if world > 1 and not dist.is_initialized():
        if backend is None:
            backend = "nccl" if torch.cuda.is_available() else "gloo"
        kw = {"device_id": device} if (backend == "nccl" and device is not None) else {}
        dist.init_process_group(backend, **kw)
    return rank, world, local


def _all_gather(t: torch.Tensor, group=None) -> torch.Tensor:
    world = dist.get_world_size(group)
    if t.is_cuda and dist.get_backend(group) != "gloo":  # RCCL: one all_gather_into_tensor
        out = torch.empty((world * t.shape[0],) + tuple(t.shape[1:]), dtype=t.dtype, device=t.device)
        dist.all_gather_into_tensor(out, t.contiguous(), group=group)
        return out
    # gloo (CPU tests, or several ranks rehearsed on one GPU): through host memory
    src = t.detach().cpu().contiguous()
    parts = [torch.empty_like(src) for _ in range(world)]
    dist.all_gather(parts, src, group=group)
    return torch.cat(parts).to(t.device)


def gather_env_rows(x: torch.Tensor, total: Optional[int] = None, group=None) -> torch.Tensor:
    """All-gather a per-env tensor (n_local, ...) of every rank into global env order
    (total, ...) — one collective.  Shards may differ in size by one (shard_range): each is padded
    to the largest for the collective and unpadded afterwards.  `total`: the global env count
    (default world * n_local)."""
    world = dist.get_world_size(group)
    n = x.shape[0]
    if total is None:
        total = n * world
    cap = -(-total // world)
    padded = torch.zeros((cap,) + tuple(x.shape[1:]), dtype=x.dtype, device=x.device)
    padded[:n] = x
    allp = _all_gather(padded, group).view((world, cap) + tuple(x.shape[1:]))
    return torch.cat([allp[r, :shard_range(total, world, r)[1]] for r in range(world)])


def gather_rollout(reward: torch.Tensor, done: torch.Tensor, is_goal: torch.Tensor,
                   total: Optional[int] = None, group=None) -> Dict[str, torch.Tensor]:
    """All-gather per-env rollout scalars into global env order (one collective per call):
    reward f32 and the done / is_goal flags packed into one (n, 2) float32 row per env."""
    packed = torch.stack([reward.float(), done.to(torch.float32) + 2.0 * is_goal.to(torch.float32)], 1)
    g = gather_env_rows(packed, total, group)
    flags = g[:, 1].to(torch.int32)
    return {"reward": g[:, 0].contiguous(), "done": (flags & 1).bool(), "is_goal": (flags & 2).bool()}
