"""CPU: the N > 1 path (sharding + all-gather of results) with world_size-2 gloo.

Each rank computes the ICRCs of its shard (here with the CPU oracle: this
container has no GPU; tests/test_gpu_dist.py runs the same sharding and
gather with the HIP kernels over an nccl group), all-gathers them with the
helpers bench.py uses over RCCL (IcrcGather: one all_gather_into_tensor of
padded shards; all_gather_icrc), and every rank must end with exactly the
single-process result vector, for equal and unequal (byte-balanced) shards."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from roce_icrc.dist import IcrcGather, all_gather_icrc, byte_balanced_cuts, cuts_to_sizes, shard_range


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, count, n, q):
    import oracle_c

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        lo, hi = shard_range(count, world, rank)
        local = oracle_c.synth_batch(0x1CEC0DE, lo, hi - lo, n)
        mine = oracle_c.icrc_batch(local, stride=n)
        got = all_gather_icrc(torch.from_numpy(mine.view(np.int32).copy()), world)
        q.put((rank, got.numpy().view(np.uint32).copy()))
    finally:
        dist.destroy_process_group()


def _mix_worker(rank, world, port, count, q):
    import oracle_c

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        lens_g = np.random.default_rng(11).choice(np.array([64, 256, 1024, 4096], np.uint32), size=count)
        cuts = byte_balanced_cuts(lens_g, world)
        g = IcrcGather(cuts_to_sizes(cuts))
        lo, hi = cuts[rank], cuts[rank + 1]
        buf, offs = oracle_c.synth_ragged(0x1CEC0DE, lo, lens_g[lo:hi])
        mine = oracle_c.icrc_batch(buf, offsets=offs, lengths=lens_g[lo:hi])
        local = g.local_buffer("cpu")
        local[: hi - lo] = torch.from_numpy(mine.view(np.int32).copy())
        out = g.gathered_buffer("cpu")
        g.start(local, out, async_op=True).wait()
        assert torch.equal(g.shard_of(out, rank), local[: hi - lo])
        q.put((rank, g.compact(out).numpy().view(np.uint32).copy(), g.equal))
    finally:
        dist.destroy_process_group()


def test_gloo_world2_byte_balanced_mix_unequal_shards():
    """C4's split: one global mixed-MTU batch cut at equal bytes (unequal packet
    counts), every rank generates its shard from the global index, one padded
    all_gather_into_tensor, compacted == the single-process result."""
    import oracle_c

    world, count = 2, 3001
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_mix_worker, args=(r, world, port, count, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = {}
    for _ in range(world):
        r, v, eq = q.get(timeout=120)
        res[r] = v
    for p in procs:
        p.join(60)
        assert p.exitcode == 0
    lens_g = np.random.default_rng(11).choice(np.array([64, 256, 1024, 4096], np.uint32), size=count)
    assert not eq  # the byte cut gives the ranks different packet counts
    buf, offs = oracle_c.synth_ragged(0x1CEC0DE, 0, lens_g)
    want = oracle_c.icrc_batch(buf, offsets=offs, lengths=lens_g)
    for r in range(world):
        np.testing.assert_array_equal(res[r], want)


def test_synth_ragged_restatement_matches_fixed():
    """Packet contents depend only on (seed, global index, length): the ragged
    generator agrees with the fixed-size one packet by packet."""
    import oracle_c

    lens = np.array([64, 1024, 256, 4096, 64], np.uint32)
    buf, offs = oracle_c.synth_ragged(7, 100, lens)
    for k, (o, n) in enumerate(zip(offs, lens)):
        np.testing.assert_array_equal(buf[int(o): int(o) + int(n)], oracle_c.synth_batch(7, 100 + k, 1, int(n))[0])


@pytest.mark.parametrize("count,n", [(1000, 1024), (777, 64)])
def test_gloo_world2_gather_matches_single_process(count, n):
    import oracle_c

    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, count, n, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(60)
        assert p.exitcode == 0
    want = oracle_c.icrc_batch(oracle_c.synth_batch(0x1CEC0DE, 0, count, n), stride=n)
    for r in range(world):
        np.testing.assert_array_equal(res[r], want)


def test_shard_range_covers_exactly():
    for total in (0, 1, 7, 1 << 20):
        for world in (1, 2, 3, 8):
            spans = [shard_range(total, world, r) for r in range(world)]
            assert spans[0][0] == 0 and spans[-1][1] == total
            assert all(spans[i][1] == spans[i + 1][0] for i in range(world - 1))
            sizes = [h - l for l, h in spans]
            assert max(sizes) - min(sizes) <= 1


def test_byte_balanced_cuts_mixed_mtu():
    rng = np.random.default_rng(4)
    lens = rng.choice([64, 256, 1024, 4096], size=40000)
    for world in (2, 4, 8):
        cuts = byte_balanced_cuts(lens, world)
        assert cuts[0] == 0 and cuts[-1] == len(lens) and cuts == sorted(cuts)
        shard_bytes = [int(lens[cuts[i]:cuts[i + 1]].sum()) for i in range(world)]
        assert max(shard_bytes) - min(shard_bytes) <= 2 * 4096


def _simulate_plan(counts, ops):
    """Execute an all-gather plan on host buffers with RCCL's semantics:
    in-place all-gather, and grouped send/recv matched in issue order per
    (sender, receiver) pair.  Returns every device's buffer."""
    n, total = len(counts), int(sum(counts))
    at = np.concatenate([[0], np.cumsum(counts)]).astype(np.int64)
    bufs = [np.full(total, -1, np.int64) for _ in range(n)]
    for k in range(n):
        bufs[k][at[k]:at[k + 1]] = np.arange(at[k], at[k + 1])  # shard k computed on device k
    ag = [x for x in ops if x[1] == 0]
    if ag:
        assert len(ag) == n and {x[0] for x in ag} == set(range(n))
        c = ag[0][4]
        for dev, _, peer, off, cnt in ag:  # in place: sendbuff == recvbuff + rank * count
            assert cnt == c and off == dev * c and peer == -1
        full = np.concatenate([bufs[k][k * c:(k + 1) * c] for k in range(n)])
        bufs = [full.copy() for _ in range(n)]
        return bufs
    sends = {}
    for dev, kind, peer, off, cnt in ops:
        assert peer != dev and cnt > 0
        if kind == 1:
            sends.setdefault((dev, peer), []).append(bufs[dev][off:off + cnt].copy())
    for dev, kind, peer, off, cnt in ops:
        if kind == 2:
            data = sends[(peer, dev)].pop(0)
            assert len(data) == cnt
            bufs[dev][off:off + cnt] = data
    assert all(not v for v in sends.values())  # every send matched by exactly one receive
    return bufs


@pytest.mark.parametrize("counts", [[5, 5, 5], [7, 0, 3], [1, 1000, 2, 9], [4, 4], [0, 0], [3]])
def test_allgather_plan_every_device_ends_with_every_shard(counts):
    """ricrc_allgather_plan (the plan ricrc_batch_device_all issues through
    RCCL, pure host code): simulated with RCCL's semantics, every device's
    buffer ends with all shards in shard order -- equal counts through the
    in-place all-gather, unequal (byte-balanced) counts through matched
    send/recv pairs, zero-length shards moving nothing."""
    import roce_icrc

    ops = roce_icrc.allgather_plan(counts)
    if len(counts) == 1 or sum(counts) == 0:
        assert ops == [] or all(x[4] == 0 for x in ops)
    bufs = _simulate_plan(counts, ops)
    for b in bufs:
        np.testing.assert_array_equal(b, np.arange(sum(counts)))
    if len(set(counts)) > 1:
        n = len(counts)
        nz = sum(1 for c in counts if c)
        assert len(ops) == 2 * nz * (n - 1)  # each non-empty shard sent to and received by every peer
