"""Multi-GPU layout: one process per GPU, batches of independent ciphertexts
sharded contiguously across ranks, key material replicated by ONE broadcast per key (RCCL over
xGMI on MI355X; gloo in the CPU tests).  The PBS hot loop has no collective.
"""
from __future__ import annotations

import os

import numpy as np


def env_rank_world():
    return int(os.environ.get("RANK", 0)), int(os.environ.get("WORLD_SIZE", 1)), int(os.environ.get("LOCAL_RANK", 0))


def shard_range(total: int, rank: int, world: int) -> tuple[int, int]:
    """Contiguous shard [lo, hi) of `total` items for `rank` (sizes differ by at most one)."""
    base, extra = divmod(total, world)
    lo = rank * base + min(rank, extra)
    hi = lo + base + (1 if rank < extra else 0)
    return lo, hi


def broadcast_u64(array: np.ndarray | None, numel: int, src: int, device):
    """Broadcast a u64 key (numel words) from `src` to every rank; returns a tensor on `device`.

    On GPU ranks this is a single RCCL broadcast of the device buffer (xGMI point-to-point links);
    with the gloo backend the tensor stays on the CPU."""
    import torch
    import torch.distributed as dist

    if array is not None:
        t = torch.from_numpy(np.ascontiguousarray(array, dtype=np.uint64).view(np.int64)).to(device)
    else:
        t = torch.empty(numel, dtype=torch.int64, device=device)
    if dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1:
        dist.broadcast(t, src=src)
    return t


def gather_u64(local: np.ndarray, total_rows: int, device):
    """All-gather of per-rank row shards (optional replicated result)."""
    import torch
    import torch.distributed as dist

    world = dist.get_world_size()
    rank = dist.get_rank()
    lo, hi = shard_range(total_rows, rank, world)
    assert local.shape[0] == hi - lo
    width = local.shape[1]
    maxrows = -(-total_rows // world)
    buf = torch.zeros((maxrows, width), dtype=torch.int64, device=device)
    buf[: hi - lo] = torch.from_numpy(np.ascontiguousarray(local).view(np.int64)).to(device)
    outs = [torch.empty_like(buf) for _ in range(world)]
    dist.all_gather(outs, buf)
    rows = []
    for r in range(world):
        a, b = shard_range(total_rows, r, world)
        rows.append(outs[r][: b - a].cpu().numpy().view(np.uint64))
    return np.concatenate(rows, axis=0)
