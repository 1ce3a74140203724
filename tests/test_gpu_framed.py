"""GPU parity: framed NIC rings through the strided-chain kernel (SURVEY 8(a)
row a4).

A NIC receive ring of 1, 2 or 4 KiB slots with the L3 packet at l3_offset
(14: Ethernet, 18: one VLAN tag, 22: two) running to the slot's end takes
icrc_sck_kernel's framed instantiation (FR, icrc_sck.hip): the kernel folds
the whole slot from a zero register with the bytes before the L3 start
zeroed, which leaves the register at zero up to the L3 start, and seeds and
masks L3 bytes 0..32 in line 0.  Every ICRC is compared bit-exactly with the
C oracle on the same bytes and with the ragged pipeline the same rings took
before (RICRC_NO_FRAMED)."""
import numpy as np
import pytest

torch = pytest.importorskip("torch")

import oracle_c  # noqa: E402
import roce_icrc  # noqa: E402

pytestmark = pytest.mark.gpu

SEED = 0xF2A3ED


def _dev(a):
    return torch.from_numpy(np.ascontiguousarray(a)).to("cuda")


def _out(count):
    return torch.full((count,), -1, dtype=torch.int32, device="cuda")


def _host_u32(t):
    torch.cuda.synchronize()
    return t.cpu().numpy().view(np.uint32)


@pytest.mark.parametrize("stride", [1024, 2048, 4096])
@pytest.mark.parametrize("l3", [1, 2, 14, 18, 22, 64, 92])
def test_framed_ring_matches_oracle(ctx, stride, l3):
    rng = np.random.default_rng(stride * 131 + l3)
    count = 3001 if stride < 4096 else 1501
    frames = rng.integers(0, 256, size=count * stride, dtype=np.uint8)
    d = _dev(frames)
    assert roce_icrc.kernel_path(d, count, stride=stride, l3_offset=l3, ctx=ctx) == "icrc_sck_kernel"
    out = _out(count)
    ctx.batch_device(d, count, out, stride=stride, l3_offset=l3)
    want = oracle_c.icrc_batch(frames, stride=stride, count=count, l3_offset=l3, threads=8)
    np.testing.assert_array_equal(_host_u32(out), want)


@pytest.mark.parametrize("count", [1, 7, 8, 9, 63, 64, 65, 8 * 16 * 3 + 5, 70001])
def test_framed_ring_tails(ctx, count):
    """Partial groups (8 slots; 32 for 1 KiB super-groups), partial rounds
    of result slots, a few groups per wave."""
    for stride in (1024, 4096):
        rng = np.random.default_rng(count + stride)
        frames = rng.integers(0, 256, size=count * stride, dtype=np.uint8)
        out = _out(count)
        ctx.batch_device(_dev(frames), count, out, stride=stride, l3_offset=14)
        np.testing.assert_array_equal(_host_u32(out), oracle_c.icrc_batch(frames, stride=stride, count=count,
                                                                           l3_offset=14, threads=8))


def test_framed_ring_same_as_ragged_pipeline(ctx, ctx_env):
    """RICRC_NO_FRAMED sends the ring to the ragged pipeline (the round-4
    path): the same ICRCs."""
    count, stride = 20000, 2048
    frames = np.random.default_rng(5).integers(0, 256, size=count * stride, dtype=np.uint8)
    d = _dev(frames)
    rag = ctx_env(RICRC_NO_FRAMED=1)
    assert roce_icrc.kernel_path(d, count, stride=stride, l3_offset=18, ctx=rag).startswith(("rsck_bucket", "icrc_rswg_kernel"))
    a, b = _out(count), _out(count)
    ctx.batch_device(d, count, a, stride=stride, l3_offset=18)
    rag.batch_device(d, count, b, stride=stride, l3_offset=18)
    np.testing.assert_array_equal(_host_u32(a), _host_u32(b))


def test_framed_ring_not_taken(ctx):
    """Rings the framed kernel does not fold: another slot size, an L3 offset
    past line 0's masks, a misaligned base, per-slot lengths (the ragged
    pipeline: a strided-chain variant that stopped each lane at its packet's
    end measured no faster, profiles/r05/NOTES.md)."""
    d = torch.zeros(4096 * 8 + 16, dtype=torch.uint8, device="cuda")
    path = lambda **kw: roce_icrc.kernel_path(kw.pop("base", d), 8, ctx=ctx, **kw)  # noqa: E731
    assert path(stride=4096, l3_offset=14) == "icrc_sck_kernel"
    assert path(stride=1536, l3_offset=14).startswith(("rsck_bucket", "icrc_rswg_kernel"))
    assert path(stride=4096, l3_offset=93).startswith(("rsck_bucket", "icrc_rswg_kernel"))
    assert path(base=d[2:], stride=4096, l3_offset=14).startswith(("rsck_bucket", "icrc_rswg_kernel"))
    lens = torch.full((8,), 1000, dtype=torch.int32, device="cuda")
    assert path(stride=4096, l3_offset=14, lengths=lens).startswith(("rsck_bucket", "icrc_rswg_kernel"))


def test_framed_ring_verify_mode(ctx):
    """Stamp every slot's trailer with the oracle, corrupt some, verify."""
    count, stride, l3 = 5000, 4096, 14
    rng = np.random.default_rng(77)
    frames = rng.integers(0, 256, size=(count, stride), dtype=np.uint8)
    icrcs = oracle_c.icrc_batch(frames, stride=stride, count=count, l3_offset=l3, threads=8)
    frames[:, stride - 4:] = icrcs.view(np.uint8).reshape(count, 4)
    bad = rng.choice(count, size=97, replace=False)
    frames[bad, l3 + 40] ^= 0x5A
    out = _out(count)
    ctx.batch_device(_dev(frames), count, out, stride=stride, l3_offset=l3, verify=True)
    ok = np.ones(count, np.uint32)
    ok[bad] = 0
    np.testing.assert_array_equal(_host_u32(out), ok)


@pytest.mark.parametrize("family", ["v6", "auto"])
def test_framed_ring_other_families(ctx, family):
    """IPv6 / AUTO: the framed kernel's IPv4 masks, then the linear fix-up."""
    count, stride, l3 = 4000, 1024, 14
    rng = np.random.default_rng(91)
    frames = rng.integers(0, 256, size=(count, stride), dtype=np.uint8)
    frames[: count // 2, l3] = 0x60 | (frames[: count // 2, l3] & 15)  # version 6 for half of them
    frames[count // 2:, l3] = 0x45
    out = _out(count)
    d = _dev(frames)
    assert roce_icrc.kernel_path(d, count, stride=stride, l3_offset=l3, ctx=ctx, family=family) == \
        "icrc_sck_kernel+family_fix_kernel"
    ctx.batch_device(d, count, out, stride=stride, l3_offset=l3, family=family)
    want = oracle_c.icrc_batch(frames, stride=stride, count=count, l3_offset=l3, threads=8, family=family)
    np.testing.assert_array_equal(_host_u32(out), want)


@pytest.mark.slow
def test_framed_ring_full_size_bit_exact(ctx):
    """1,048,576 slots of 4 KiB, L3 at 14 (4082-byte packets, bench.py
    --l3-offset 14 --stride 4096), slots generated on the device, every ICRC
    compared with the C oracle on the very same bytes; then every trailer
    stamped and verified."""
    count, stride, l3 = 1 << 20, 4096, 14
    d = torch.empty(count * stride, dtype=torch.uint8, device="cuda")
    ctx.synth_device(d, SEED, 0, count, stride)
    out = _out(count)
    ctx.batch_device(d, count, out, stride=stride, l3_offset=l3)
    got = _host_u32(out)
    host = d.cpu().numpy()
    np.testing.assert_array_equal(got, oracle_c.icrc_batch(host, stride=stride, count=count, l3_offset=l3,
                                                           threads=16))
    host.reshape(count, stride)[:, stride - 4:] = got.view(np.uint8).reshape(count, 4)
    d.copy_(torch.from_numpy(host))
    ctx.batch_device(d, count, out, stride=stride, l3_offset=l3, verify=True)
    assert int(_host_u32(out).sum()) == count


# ---- rings with a length per slot (a NIC's completion byte counts) ----------
# These take the ragged pipeline (bucketed by line count, so groups of equal
# length fold without waste).

def _slot_lens(rng, count, stride, l3, odd=True):
    """Mostly packets inside their slot; with `odd`, a sprinkling of every
    odd case: 4 <= n < 44 (computed by the gather), n < 4 and n > 65535 (0),
    packets running past their slot (their bytes are read where they lie)."""
    lens = rng.integers(44, stride - l3 + 1, size=count).astype(np.uint32)
    lens[rng.random(count) < 0.2] = stride - l3  # full slots
    if odd:
        k = max(count // 40, 1)
        idx = rng.choice(count, size=4 * k, replace=False)
        lens[idx[:k]] = rng.integers(4, 44, size=k)
        lens[idx[k:2 * k]] = rng.integers(0, 4, size=k)
        lens[idx[2 * k:3 * k]] = 70000
        lens[idx[3 * k:]] = rng.integers(stride - l3 + 1, stride - l3 + 300, size=k)
    return lens


def _want_slots(frames, lens, stride, count, l3, family="v4"):
    want = oracle_c.icrc_batch(frames, lengths=np.where(lens > 65535, 0, lens).astype(np.uint32), stride=stride,
                               count=count, l3_offset=l3, threads=8, family=family)  # (n < 4: 0)
    return want


@pytest.mark.parametrize("stride", [1024, 2048, 4096])
@pytest.mark.parametrize("l3", [0, 14, 18, 92])
def test_slot_lengths_match_oracle(ctx, ctx_env, stride, l3):
    """Slots with per-slot lengths, every odd length case, against the oracle;
    RICRC_NO_FRAMED changes nothing for them."""
    rng = np.random.default_rng(stride + 7 * l3)
    count = 3001
    frames = rng.integers(0, 256, size=count * stride + 4096, dtype=np.uint8)  # slack: packets past the last slot
    lens = _slot_lens(rng, count, stride, l3)
    d, d_len = _dev(frames), _dev(lens)
    assert roce_icrc.kernel_path(d, count, stride=stride, lengths=d_len, l3_offset=l3, ctx=ctx).startswith(("rsck_bucket", "icrc_rswg_kernel"))
    want = _want_slots(frames, lens, stride, count, l3)
    out = _out(count)
    ctx.batch_device(d, count, out, stride=stride, lengths=d_len, l3_offset=l3)
    np.testing.assert_array_equal(_host_u32(out), want)
    rag = ctx_env(RICRC_NO_FRAMED=1)
    assert roce_icrc.kernel_path(d, count, stride=stride, lengths=d_len, l3_offset=l3, ctx=rag).startswith(("rsck_bucket", "icrc_rswg_kernel"))
    out2 = _out(count)
    rag.batch_device(d, count, out2, stride=stride, lengths=d_len, l3_offset=l3)
    np.testing.assert_array_equal(_host_u32(out2), want)


@pytest.mark.parametrize("count", [1, 7, 9, 65, 8 * 16 * 3 + 5, 70001])
def test_slot_lengths_tails(ctx, count):
    for stride in (1024, 2048, 4096):
        rng = np.random.default_rng(count * 3 + stride)
        frames = rng.integers(0, 256, size=count * stride + 4096, dtype=np.uint8)
        lens = _slot_lens(rng, count, stride, 14, odd=count > 8)
        out = _out(count)
        ctx.batch_device(_dev(frames), count, out, stride=stride, lengths=_dev(lens), l3_offset=14)
        np.testing.assert_array_equal(_host_u32(out), _want_slots(frames, lens, stride, count, 14))


def test_slot_lengths_verify_mode(ctx):
    count, stride, l3 = 6000, 2048, 14
    rng = np.random.default_rng(123)
    frames = rng.integers(0, 256, size=(count, stride), dtype=np.uint8)
    lens = rng.integers(20, stride - l3 + 1, size=count).astype(np.uint32)  # short ones included
    icrcs = oracle_c.icrc_batch(frames, lengths=lens, stride=stride, count=count, l3_offset=l3, threads=8)
    for i in range(count):
        e = l3 + int(lens[i])
        frames[i, e - 4:e] = np.frombuffer(int(icrcs[i]).to_bytes(4, "little"), np.uint8)
    bad = rng.choice(count, size=101, replace=False)
    frames[bad, l3 + 9] ^= 0x21  # the IP protocol byte: not masked
    out = _out(count)
    ctx.batch_device(_dev(frames), count, out, stride=stride, lengths=_dev(lens), l3_offset=l3, verify=True)
    ok = np.ones(count, np.uint32)
    ok[bad] = 0
    np.testing.assert_array_equal(_host_u32(out), ok)


@pytest.mark.parametrize("family", ["v6", "auto"])
def test_slot_lengths_other_families(ctx, family):
    count, stride, l3 = 3000, 4096, 14
    rng = np.random.default_rng(5150)
    frames = rng.integers(0, 256, size=(count, stride), dtype=np.uint8)
    frames[: count // 2, l3] = 0x60 | (frames[: count // 2, l3] & 15)
    frames[count // 2:, l3] = 0x45
    lens = _slot_lens(rng, count, stride, l3, odd=False)
    out = _out(count)
    d, d_len = _dev(frames), _dev(lens)
    assert roce_icrc.kernel_path(d, count, stride=stride, lengths=d_len, l3_offset=l3, ctx=ctx,
                                 family=family).endswith("+family_fix_kernel")
    ctx.batch_device(d, count, out, stride=stride, lengths=d_len, l3_offset=l3, family=family)
    np.testing.assert_array_equal(_host_u32(out), _want_slots(frames, lens, stride, count, l3, family))


def test_slot_lengths_status_and_framelen(ctx):
    """The status call over such a ring (strict, frame lengths from the IP
    header)."""
    import icrc_oracle as O

    count, stride, l3 = 2000, 2048, 14
    rng = np.random.default_rng(77)
    frames = rng.integers(0, 256, size=(count, stride), dtype=np.uint8)
    lens = rng.integers(60, stride - l3 + 1, size=count).astype(np.uint32)
    for i in range(count):  # IPv4 headers whose total_len is the packet, padded frames beyond it
        n = int(lens[i]) - (4 if i % 3 == 0 else 0)
        frames[i, 12:14] = (0x08, 0x00)
        frames[i, l3] = 0x45
        frames[i, l3 + 2:l3 + 4] = (n >> 8, n & 255)
        frames[i, l3 + 9] = 17
        frames[i, l3 + 22:l3 + 24] = (0x12, 0xB7)  # UDP dport 4791
    out = torch.full((count,), -1, dtype=torch.int32, device="cuda")
    st = torch.full((count,), 255, dtype=torch.uint8, device="cuda")
    ctx.batch_device_st(_dev(frames), count, out, st, stride=stride, lengths=_dev(lens), l3_offset=l3,
                        strict=True, framelen=True)
    torch.cuda.synchronize()
    w_out, w_st = O.status_batch(frames.reshape(-1), stride=stride, lengths=lens, count=count, l3_offset=l3,
                                 strict=True, framelen=True)
    np.testing.assert_array_equal(st.cpu().numpy(), np.asarray(w_st, np.uint8))
    np.testing.assert_array_equal(out.cpu().numpy().view(np.uint32), np.asarray(w_out, np.uint32))


@pytest.mark.slow
def test_slot_lengths_full_size_bit_exact(ctx):
    """1,048,576 slots of 2 KiB holding 1500-byte packets behind a 14-byte
    Ethernet header (MTU-sized traffic in a NIC's 2 KiB receive buffers),
    every ICRC against the C oracle on the same device-generated bytes."""
    count, stride, l3 = 1 << 20, 2048, 14
    d = torch.empty(count * stride, dtype=torch.uint8, device="cuda")
    ctx.synth_device(d, SEED ^ 5, 0, count, stride)
    lens = np.full(count, 1500, np.uint32)
    out = _out(count)
    ctx.batch_device(d, count, out, stride=stride, lengths=_dev(lens), l3_offset=l3)
    np.testing.assert_array_equal(_host_u32(out), oracle_c.icrc_batch(d.cpu().numpy(), lengths=lens, stride=stride,
                                                                      count=count, l3_offset=l3, threads=16))


@pytest.mark.slow
@pytest.mark.parametrize("lo,hi", [(64, 1010), (200, 200), (450, 450)])
def test_slot_lengths_1k_full_size_bit_exact(ctx, lo, hi):
    """1,048,576 slots of 1 KiB behind a 14-byte Ethernet header with a
    completion length per slot (the NIC receive ring of
    small buffers; uniform 64-1010 B, and single lengths of two and four
    lines), every ICRC against the C oracle on the same device-generated
    bytes, then every trailer stamped and verified."""
    count, stride, l3 = 1 << 20, 1024, 14
    lens = np.random.default_rng(lo * 7 + hi).integers(lo, hi + 1, size=count).astype(np.uint32)
    d = torch.zeros(count * stride, dtype=torch.uint8, device="cuda")
    offs = np.arange(count, dtype=np.uint64) * stride + l3
    ctx.synth_ragged_device(d, SEED ^ 9, 0, count, _dev(offs), _dev(lens))
    d_len = _dev(lens)
    out = _out(count)
    ctx.batch_device(d, count, out, stride=stride, lengths=d_len, l3_offset=l3)
    got = _host_u32(out)
    host = d.cpu().numpy()
    np.testing.assert_array_equal(got, oracle_c.icrc_batch(host, lengths=lens, stride=stride, count=count,
                                                           l3_offset=l3, threads=16))
    tail = (offs + lens.astype(np.uint64) - 4).astype(np.int64)
    host[(tail[:, None] + np.arange(4, dtype=np.int64)[None, :]).reshape(-1)] = got.view(np.uint8)
    d.copy_(torch.from_numpy(host))
    ctx.batch_device(d, count, out, stride=stride, lengths=d_len, l3_offset=l3, verify=True)
    assert int(_host_u32(out).astype(np.uint64).sum()) == count
