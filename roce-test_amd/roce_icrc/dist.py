"""Multi-GPU sharding of ICRC batches: one process per GPU, RCCL all-gather.

Packets are independent, so a batch shards with no data-path exchange
(SURVEY.md §8e): rank r owns a contiguous range of packets, computes their
ICRCs with its own GPU, and the only collective is one all-gather of the
4-byte results so that every rank ends with the whole result vector in
packet order (torch.distributed "nccl" = RCCL over xGMI on MI355X; "gloo" on
CPU for the tests).  The reference has no multi-device code of its own; its
scale-out is N endpoints behind one switch (switchd/vswitchd.hpp:150-154).
"""
from __future__ import annotations

import numpy as np


def shard_range(total: int, world: int, rank: int) -> tuple[int, int]:
    """Contiguous, balanced [lo, hi) of ``total`` packets for ``rank``."""
    if world <= 0 or not 0 <= rank < world:
        raise ValueError("bad world/rank")
    base, extra = divmod(total, world)
    lo = rank * base + min(rank, extra)
    return lo, lo + base + (1 if rank < extra else 0)


def byte_balanced_cuts(lengths, world: int) -> list[int]:
    """Packet-index cuts splitting a ragged batch into ``world`` shards of
    about equal bytes (prefix sum of lengths; SURVEY.md §8e "mixed")."""
    lengths = np.asarray(lengths, dtype=np.uint64)
    csum = np.cumsum(lengths, dtype=np.uint64)
    total = int(csum[-1]) if len(csum) else 0
    cuts = [0]
    for k in range(1, world):
        target = total * k // world
        cuts.append(int(np.searchsorted(csum, target, side="left")) + (1 if len(csum) else 0))
        cuts[-1] = min(max(cuts[-1], cuts[-2]), len(lengths))
    cuts.append(len(lengths))
    return cuts


def all_gather_icrc(local, world: int, group=None):
    """All-gather per-rank uint32 ICRC vectors (as int32 tensors) of possibly
    unequal length into the global vector, on every rank.  Equal lengths take
    one all_gather_into_tensor (one RCCL call); unequal ones are padded to the
    longest shard first."""
    import torch
    import torch.distributed as dist

    n = torch.tensor([local.numel()], dtype=torch.int64, device=local.device)
    sizes = [torch.zeros_like(n) for _ in range(world)]
    dist.all_gather(sizes, n, group=group)
    sizes = [int(s.item()) for s in sizes]
    m = max(sizes)
    buf = local if local.numel() == m else torch.cat(
        [local, torch.zeros(m - local.numel(), dtype=local.dtype, device=local.device)])
    out = torch.empty(world * m, dtype=local.dtype, device=local.device)
    dist.all_gather_into_tensor(out, buf.contiguous(), group=group)
    if all(s == m for s in sizes):
        return out
    return torch.cat([out[r * m: r * m + sizes[r]] for r in range(world)])
