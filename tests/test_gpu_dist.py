"""GPU: the multi-GPU path through the product, on one MI355X.

* bench.py's multi-process form: a world-size-1 ``nccl`` (RCCL) group, a C3
  shard (shard_range of the 4 M x 4 KiB batch over 8 ranks) computed by
  ricrc_batch_device and all-gathered by IcrcGather, bit-exact vs the oracle;
  the same for a byte-balanced C4 (mixed-MTU) shard.
* The single-process C ABI form: ricrc_comm_init (ncclCommInitAll over the
  context's devices) + ricrc_batch_device_all / ricrc_allgather on a
  one-device context.  (The 8-device runs are the driver's.)
* ricrc_synth_ragged_device against its host restatement, ricrc_prime.
* ricrc_batch_host's error path: a failure forced after chunk 2 leaves
  nothing in flight, and the next call on the same context is bit-exact.
"""
import os
import socket
import time

import numpy as np
import pytest

torch = pytest.importorskip("torch")

import oracle_c  # noqa: E402

from roce_icrc.dist import IcrcGather, byte_balanced_cuts, cuts_to_sizes, shard_range  # noqa: E402

pytestmark = pytest.mark.gpu
SEED = 0x1CEC0DE


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.fixture(scope="module")
def nccl_group():
    import torch.distributed as dist

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_free_port()))
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
    yield dist
    dist.destroy_process_group()


def test_c3_shard_through_rccl_group(ctx, nccl_group):
    """Rank 3 of 8's shard of C3 (524288 x 4096 B = 2 GiB), generated from the
    global packet index, computed by the HIP kernel, gathered over RCCL."""
    T, world, r, n = 4 << 20, 8, 3, 4096
    lo, hi = shard_range(T, world, r)
    count = hi - lo
    buf = torch.empty(count * n, dtype=torch.uint8, device="cuda")
    st = torch.cuda.current_stream()
    ctx.synth_device(buf, SEED, lo, count, n, stream=st)
    g = IcrcGather([count])
    local, out = g.local_buffer("cuda"), g.gathered_buffer("cuda")
    ctx.batch_device(buf, count, local, stride=n, stream=st)
    g.start(local, out, async_op=True).wait()
    torch.cuda.synchronize()
    got = g.compact(out).cpu().numpy().view(np.uint32)
    want = oracle_c.icrc_batch(buf.cpu().numpy(), stride=n, threads=16)
    np.testing.assert_array_equal(got, want)
    # the bytes are the generator's for the GLOBAL index (shard-independent)
    for k in (0, 1, count // 2, count - 1):
        np.testing.assert_array_equal(buf[k * n:(k + 1) * n].cpu().numpy(),
                                      oracle_c.synth_batch(SEED, lo + k, 1, n)[0])


def test_c4_byte_balanced_shard_through_rccl_group(ctx, nccl_group):
    """Rank 5 of 8 of a 1 M-packet mixed-MTU batch cut at equal bytes."""
    lens_g = np.random.default_rng(SEED).choice(np.array([64, 256, 1024, 4096], np.uint32), size=1 << 20)
    cuts = byte_balanced_cuts(lens_g, 8)
    lo, hi = cuts[5], cuts[6]
    lens = np.ascontiguousarray(lens_g[lo:hi])
    offs = np.zeros(len(lens), np.uint64)
    offs[1:] = np.cumsum(lens[:-1], dtype=np.uint64)
    nbytes = int(lens.sum(dtype=np.uint64))
    buf = torch.zeros(nbytes, dtype=torch.uint8, device="cuda")
    d_offs = torch.from_numpy(offs.view(np.int64)).cuda()
    d_lens = torch.from_numpy(lens.view(np.int32)).cuda()
    st = torch.cuda.current_stream()
    ctx.synth_ragged_device(buf, SEED, lo, len(lens), d_offs, d_lens, stream=st)
    g = IcrcGather([len(lens)])
    local, out = g.local_buffer("cuda"), g.gathered_buffer("cuda")
    ctx.batch_device(buf, len(lens), local, offsets=d_offs, lengths=d_lens, stream=st)
    g.start(local, out)  # synchronous form (--in-stream-gather)
    torch.cuda.synchronize()
    got = g.compact(out).cpu().numpy().view(np.uint32)
    hbuf, _ = oracle_c.synth_ragged(SEED, lo, lens)
    np.testing.assert_array_equal(buf.cpu().numpy(), hbuf)  # device generator == its restatement
    want = oracle_c.icrc_batch(hbuf, offsets=offs, lengths=lens, threads=16)
    np.testing.assert_array_equal(got, want)


@pytest.mark.parametrize("ragged", [False, True])
def test_batch_device_all_one_device_context(ragged):
    """ricrc_comm_init + ricrc_batch_device_all on a one-device context (the
    C ABI's single-process multi-GPU entry; RCCL loaded at run time)."""
    import roce_icrc

    c = roce_icrc.Context(devices=[0])
    try:
        c.comm_init()
        c.comm_init()  # idempotent
        st = c.stream(0)
        if ragged:
            lens = np.random.default_rng(3).choice(np.array([64, 256, 1024, 4096], np.uint32), size=50000)
            hbuf, offs = oracle_c.synth_ragged(SEED, 0, lens)
            d = torch.from_numpy(hbuf).cuda()
            d_offs = torch.from_numpy(offs.view(np.int64)).cuda()
            d_lens = torch.from_numpy(lens.view(np.int32)).cuda()
            torch.cuda.synchronize()
            out = torch.empty(len(lens), dtype=torch.int32, device="cuda")
            c.batch_device_all([d], [len(lens)], [out], offsets=[d_offs], lengths=[d_lens])
            want = oracle_c.icrc_batch(hbuf, offsets=offs, lengths=lens, threads=8)
        else:
            n, count = 4096, 100000
            d = torch.empty(n * count, dtype=torch.uint8, device="cuda")
            c.synth_device(d, SEED, 0, count, n, stream=st)
            c.sync()
            out = torch.empty(count, dtype=torch.int32, device="cuda")
            c.batch_device_all([d], [count], [out], stride=n)
            want = oracle_c.icrc_batch(d.cpu().numpy(), stride=n, threads=8)
        c.sync()
        c.allgather([len(want)], [out])  # one device: in place, a no-op
        c.sync()
        np.testing.assert_array_equal(out.cpu().numpy().view(np.uint32), want)
    finally:
        c.close()


def test_batch_device_all_needs_comm_init():
    import roce_icrc

    c = roce_icrc.Context(devices=[0])
    try:
        out = torch.empty(1, dtype=torch.int32, device="cuda")
        with pytest.raises(roce_icrc.ICRCError) as e:
            c.batch_device_all([out], [1], [out], stride=64)
        assert e.value.rc == -22
    finally:
        c.close()


def test_prime_runs_for_the_requested_time(ctx):
    t0 = time.perf_counter()
    ctx.prime(20000)
    dt = time.perf_counter() - t0
    assert 0.019 < dt < 2.0
    ctx.prime(0)


def test_batch_host_failure_leaves_nothing_in_flight(ctx_env):
    """RICRC_FAIL_CHUNK=2 (read by ricrc_create, fires once): the call fails
    with -EIO after queueing chunk 2 of 4 (1 M packets per chunk); the next
    call on the same context -- reusing the same staging slots and streams --
    is bit-exact."""
    import roce_icrc

    n, count = 64, (3 << 20) + 12345
    host = oracle_c.synth_batch(SEED, 0, count, n)
    want = oracle_c.icrc_batch(host, stride=n, threads=16)
    ctx = ctx_env(RICRC_FAIL_CHUNK=2)
    with pytest.raises(roce_icrc.ICRCError) as e:
        ctx.batch_host(host, stride=n)
    assert e.value.rc == -5
    np.testing.assert_array_equal(ctx.batch_host(host, stride=n), want)
    lens = np.full(count, n, np.uint32)
    offs = np.arange(count, dtype=np.uint64) * n
    ctx = ctx_env(RICRC_FAIL_CHUNK=0)
    with pytest.raises(roce_icrc.ICRCError):
        ctx.batch_host(host, offs, lens)
    np.testing.assert_array_equal(ctx.batch_host(host, offs, lens), want)
