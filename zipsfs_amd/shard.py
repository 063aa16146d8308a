"""Round-robin buffer sharding across GPUs and the single results exchange.

Buffers are independent, so the batch shards with no data-path collective:
global buffer i is owned by rank i mod world.  The only
exchange is one all-gather of the 32-bit CRCs (RCCL over xGMI with the
"nccl" backend; gloo works for CPU tests).  Rank r's k-th local result is
global buffer r + world*k.
"""
from __future__ import annotations

import numpy as np


def shard_indices(n_total: int, rank: int, world: int) -> np.ndarray:
    """Global buffer indices owned by `rank`."""
    if not 0 <= rank < world:
        raise ValueError("rank out of range")
    return np.arange(rank, n_total, world, dtype=np.int64)


def local_count(n_total: int, rank: int, world: int) -> int:
    return max(0, (n_total - rank + world - 1) // world)


def gather_crcs(local, n_total: int, group=None):
    """All-gather every rank's local CRCs and return them in global order.

    `local` is an int32 tensor (device or CPU) with local_count(...) entries.
    Collective: every rank must call it.  Returns an int32 tensor of n_total
    on the same device as `local` (CPU staging when the backend is gloo).
    """
    import torch
    import torch.distributed as dist
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    if local.numel() != local_count(n_total, rank, world):
        raise ValueError("local result count does not match the shard")
    per = (n_total + world - 1) // world
    backend = dist.get_backend(group)
    dev = local.device if backend != "gloo" else torch.device("cpu")
    pad = torch.zeros(per, dtype=torch.int32, device=dev)
    pad[: local.numel()].copy_(local)
    allv = torch.empty(world * per, dtype=torch.int32, device=dev)
    dist.all_gather_into_tensor(allv, pad, group=group)
    # [world, per] -> global: index r + world*k  <-  allv[r, k]
    out = allv.view(world, per).t().reshape(-1)[:n_total]
    return out.to(local.device)
