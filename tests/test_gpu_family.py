"""GPU: RoCEv2 over IPv6 and per-packet AUTO family on the batch paths
(ricrc_batch_device_ex / ricrc_verify_device_ex / ricrc_batch_host_ex)
against the CPU oracle's IPv6 restatement (oracle/icrc_oracle.c, rxe masks).

The reference is IPv4-only (header.p4:42-53, shuffle_ingress_parser.p4:16-19);
IPv6 is SURVEY.md §8f-3, so these cases are "parity unpinned" by reference
fixtures and pinned by the oracle's own IPv6 tests (tests/test_ipv6_repair.py).
Bit-exact, integer arithmetic.
"""
import numpy as np
import pytest

torch = pytest.importorskip("torch")

import oracle_c  # noqa: E402

pytestmark = pytest.mark.gpu

SEED = 0x6F6


def _dev(a):
    return torch.from_numpy(np.ascontiguousarray(a)).to("cuda")


def _u32(t):
    torch.cuda.synchronize()
    return t.cpu().numpy().view(np.uint32)


def _out(count):
    return torch.empty(count, dtype=torch.int32, device="cuda")


def _v6_rows(rng, count, n, stride=None):
    """Random IPv6 RoCEv2-shaped packets (version 6, next header UDP, payload
    length n-40, dport 4791); masked fields random."""
    stride = stride or n
    rows = rng.integers(0, 256, (count, stride), dtype=np.uint8)
    rows[:, 0] = 0x60 | (rows[:, 0] & 0x0F)
    rows[:, 4] = (n - 40) >> 8
    rows[:, 5] = (n - 40) & 0xFF
    rows[:, 6] = 17
    rows[:, 42], rows[:, 43] = 0x12, 0xB7
    return rows


def _want(buf, family, **kw):
    return oracle_c.icrc_batch(buf, family=family, threads=8, **kw)


@pytest.mark.parametrize("n", [64, 128, 256, 1024, 2048, 4096, 1500])
def test_v6_fixed_stride(ctx, n):
    """Every fixed-size kernel (SCK 1/2/4 KiB, TSK 64-512 B, direct 1500 B)
    followed by the family fix-up."""
    rng = np.random.default_rng(SEED + n)
    count = 2000
    stride = (n + 15) // 16 * 16
    rows = _v6_rows(rng, count, n, stride)
    out = _out(count)
    if stride == n:
        ctx.batch_device(_dev(rows), count, out, stride=n, family="v6")
        np.testing.assert_array_equal(_u32(out), _want(rows, "v6", stride=n))
    else:
        offs = np.arange(count, dtype=np.uint64) * stride
        lens = np.full(count, n, np.uint32)
        ctx.batch_device(_dev(rows), count, out, offsets=_dev(offs), lengths=_dev(lens), family="v6")
        np.testing.assert_array_equal(_u32(out), _want(rows, "v6", offsets=offs, lengths=lens))


def test_auto_mixed_fixed(ctx):
    count, n = 4096, 1024
    rng = np.random.default_rng(SEED)
    v4 = oracle_c.synth_batch(SEED, 0, count, n)
    v6 = _v6_rows(rng, count, n)
    rows = np.where((np.arange(count) % 3 == 0)[:, None], v6, v4)
    out = _out(count)
    ctx.batch_device(_dev(rows), count, out, stride=n, family="auto")
    np.testing.assert_array_equal(_u32(out), _want(rows, "auto", stride=n))
    ctx.batch_device(_dev(rows), count, out, stride=n, family="v4")  # v4 masks on everything
    np.testing.assert_array_equal(_u32(out), _want(rows, "v4", stride=n))


def test_auto_ragged_mix_ethernet_offset(ctx):
    """C4-style mix of lengths, odd gaps, Ethernet l3_offset, both families,
    plus lengths below the minimum and an invalid one (0)."""
    rng = np.random.default_rng(SEED + 1)
    count, l3 = 3000, 14
    lens = rng.choice([64, 256, 1024, 4096, 61, 77, 333], count).astype(np.uint32)
    lens[5], lens[17], lens[29] = 0, 10, 60
    gaps = rng.integers(0, 24, count).astype(np.uint64)
    offs = np.zeros(count, np.uint64)
    offs[1:] = np.cumsum(lens[:-1].astype(np.uint64) + l3 + gaps[:-1])
    buf = rng.integers(0, 256, int(offs[-1]) + l3 + int(lens[-1]) + 16, dtype=np.uint8)
    for i in range(count):
        buf[int(offs[i]) + l3] = 0x60 if i % 2 else 0x45
    out = _out(count)
    ctx.batch_device(_dev(buf), count, out, offsets=_dev(offs), lengths=_dev(lens), l3_offset=l3, family="auto")
    want = _want(buf, "auto", offsets=offs, lengths=lens, l3_offset=l3)
    want[lens < 4] = 0
    np.testing.assert_array_equal(_u32(out), want)


@pytest.mark.parametrize("family", ["v6", "auto"])
def test_verify_v6(ctx, family):
    count, n = 2000, 256
    rng = np.random.default_rng(SEED + 2)
    rows = _v6_rows(rng, count, n)
    if family == "auto":
        rows[::2] = oracle_c.synth_batch(SEED, 0, count, n)[::2]
    rows[:, n - 4:] = _want(rows, family, stride=n).view(np.uint8).reshape(count, 4)
    bad = np.arange(1, count, 9)
    rows[bad, 60 + bad % 150] ^= 0x01
    # masked IPv6 fields (flow label, hop limit) change freely on the good packets
    v6rows = np.flatnonzero(rows[:, 0] >> 4 == 6)
    rows[v6rows, 2] ^= 0x5A
    rows[v6rows, 7] ^= 0xFF
    out = _out(count)
    ctx.batch_device(_dev(rows), count, out, stride=n, verify=True, family=family)
    want = np.ones(count, np.uint32)
    want[bad] = 0
    np.testing.assert_array_equal(_u32(out), want)


def test_batch_host_v6(ctx):
    count, n = 5000, 1024
    rows = _v6_rows(np.random.default_rng(SEED + 3), count, n)
    got = ctx.batch_host(rows, stride=n, family="v6")
    np.testing.assert_array_equal(got, _want(rows, "v6", stride=n))


def test_bad_family_flags(ctx):
    import roce_icrc
    out = _out(1)
    d = torch.zeros(64, dtype=torch.uint8, device="cuda")
    rc = roce_icrc.lib.ricrc_batch_device_ex(ctx.handle, 0, d.data_ptr(), None, None, 64, 1, 0,
                                             out.data_ptr(), None, 7)
    assert rc < 0


@pytest.mark.parametrize("n", [1024, 2048, 4096])
@pytest.mark.parametrize("family", ["v6", "auto"])
@pytest.mark.parametrize("grid", [None, "1"])
def test_sck_native_family_compute_and_verify(ctx, ctx_env, n, family, grid):
    """The strided-chain kernel applies the IPv6 / per-packet AUTO masks itself
    (no fix-up pass): every lane slot's mask words, the version nibble
    broadcast across a packet's 8 lanes, partial last groups, one workgroup
    walking many groups (RICRC_SCK_GRID=1), verify mode with corruptions."""
    if grid:
        ctx = ctx_env(RICRC_SCK_GRID=grid)
    count = 8 * 16 * 5 + 3
    rng = np.random.default_rng(SEED + n)
    rows = _v6_rows(rng, count, n)
    if family == "auto":
        v4 = oracle_c.synth_batch(SEED, 0, count, n)
        pick = rng.random(count) < 0.5
        rows[pick] = v4[pick]
    want = _want(rows, family, stride=n)
    out = _out(count)
    ctx.batch_device(_dev(rows), count, out, stride=n, family=family)
    np.testing.assert_array_equal(_u32(out), want)
    rows[:, n - 4:] = want.view(np.uint8).reshape(count, 4)
    bad = np.arange(2, count, 7)
    rows[bad, 40 + bad % (n - 48)] ^= 0x10
    ok6 = np.flatnonzero((rows[:, 0] >> 4 == 6) & (np.arange(count) % 7 != 2))
    rows[ok6, 1] ^= 0xA5   # flow label / traffic class: masked for IPv6
    rows[ok6, 7] ^= 0x3C   # hop limit
    rows[ok6, 52] ^= 0xFF  # BTH byte 4
    ctx.batch_device(_dev(rows), count, out, stride=n, verify=True, family=family)
    w = np.ones(count, np.uint32)
    w[bad] = 0
    np.testing.assert_array_equal(_u32(out), w)


@pytest.mark.slow
def test_headline_ipv6_native(ctx):
    """1 M x 4096 B IPv6 packets through the native-mask SCK, bit-exact."""
    count, n = 1 << 20, 4096
    rows = _v6_rows(np.random.default_rng(SEED + 9), count, n)
    out = _out(count)
    ctx.batch_device(_dev(rows), count, out, stride=n, family="v6")
    np.testing.assert_array_equal(_u32(out), oracle_c.icrc_batch(rows, stride=n, family="v6", threads=16))
