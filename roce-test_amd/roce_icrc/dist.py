"""Multi-GPU sharding of ICRC batches: one process per GPU, RCCL all-gather.

Packets are independent, so a batch shards with no data-path exchange
(SURVEY.md §8e): rank r owns a contiguous range of packets, computes their
ICRCs with its own GPU, and the only collective is one all-gather of the
4-byte results so that every rank ends with the whole result vector in
packet order (torch.distributed "nccl" = RCCL over xGMI on MI355X; "gloo" on
CPU for the tests).  The reference has no multi-device code of its own; its
scale-out is N endpoints behind one switch (switchd/vswitchd.hpp:150-154).

Shards are cut either by packet count (fixed-size batches, :func:`shard_range`)
or at equal bytes (mixed-MTU batches, :func:`byte_balanced_cuts`), so shard
sizes may differ by rank.  :class:`IcrcGather` all-gathers such unequal shards
with ONE ``all_gather_into_tensor`` per step: every rank computes into a
buffer padded to the longest shard (the padding is never read back), and the
global vector is the concatenation of each rank's first ``sizes[r]`` entries.
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


def cuts_to_sizes(cuts) -> list[int]:
    return [int(cuts[r + 1] - cuts[r]) for r in range(len(cuts) - 1)]


class IcrcGather:
    """All-gather of per-rank ICRC vectors whose lengths ``sizes`` are known up
    front (they follow from the cuts every rank computes identically), so a
    step costs exactly one collective and no host synchronisation.

    ``local_buffer()`` gives a rank's compute buffer (int32, padded to
    ``max(sizes)``); ``start(local, out)`` launches the all-gather into an
    ``out`` of ``world * max(sizes)`` entries (async handle, or None when
    ``async_op`` is false); ``compact(out)`` returns the global vector in
    packet order."""

    def __init__(self, sizes, group=None):
        self.sizes = [int(s) for s in sizes]
        self.world = len(self.sizes)
        self.m = max(self.sizes) if self.sizes else 0
        self.group = group
        self.equal = all(s == self.m for s in self.sizes)

    def local_buffer(self, device):
        import torch

        return torch.zeros(self.m, dtype=torch.int32, device=device)

    def gathered_buffer(self, device):
        import torch

        return torch.empty(self.world * self.m, dtype=torch.int32, device=device)

    def start(self, local, out, async_op: bool = False):
        import torch.distributed as dist

        if local.numel() != self.m or out.numel() != self.world * self.m:
            raise ValueError("IcrcGather: buffers must be padded to max(sizes)")
        return dist.all_gather_into_tensor(out, local, group=self.group, async_op=async_op)

    def compact(self, out):
        import torch

        if self.equal:
            return out
        return torch.cat([out[r * self.m: r * self.m + self.sizes[r]] for r in range(self.world)])

    def shard_of(self, out, rank: int):
        """Rank ``rank``'s ICRCs inside a gathered buffer."""
        return out[rank * self.m: rank * self.m + self.sizes[rank]]


def all_gather_icrc(local, world: int, group=None, sizes=None):
    """All-gather per-rank uint32 ICRC vectors (as int32 tensors) of possibly
    unequal length into the global vector, on every rank.  ``sizes`` (every
    rank's length) saves the size exchange when the caller knows them; one
    ``all_gather_into_tensor`` moves the (padded) results."""
    import torch
    import torch.distributed as dist

    if sizes is None:
        n = torch.tensor([local.numel()], dtype=torch.int64, device=local.device)
        got = [torch.zeros_like(n) for _ in range(world)]
        dist.all_gather(got, n, group=group)
        sizes = [int(s.item()) for s in got]
    if len(sizes) != world or sizes[dist.get_rank(group)] != local.numel():
        raise ValueError("all_gather_icrc: sizes do not match the group / the local shard")
    g = IcrcGather(sizes, group=group)
    buf = local if local.numel() == g.m else torch.cat(
        [local, torch.zeros(g.m - local.numel(), dtype=local.dtype, device=local.device)])
    out = g.gathered_buffer(local.device)
    g.start(buf.contiguous(), out)
    return g.compact(out)
