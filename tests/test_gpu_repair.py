"""GPU: batch incremental repair (ricrc_repair_device) against the CPU oracle.

The switch's egress rewrites PSN / MSN / opcode of packets that already carry
an ICRC (shuffle_egress.p4:635-671).  Each test stamps a batch with the
oracle's ICRCs, rewrites a byte range, repairs on the GPU from the old bytes
and the old trailer, and compares with the oracle recomputed over the
rewritten bytes -- bit-exact, integer arithmetic.  The full-size case checks
the size-independent property repair == recompute and verify == 1 everywhere.
"""
import numpy as np
import pytest

torch = pytest.importorskip("torch")

import oracle_c  # noqa: E402
import roce_icrc  # noqa: E402

pytestmark = pytest.mark.gpu

SEED = 0x2E9A1


def _dev(a):
    return torch.from_numpy(np.ascontiguousarray(a)).to("cuda")


def _host(t):
    torch.cuda.synchronize()
    return t.cpu().numpy()


def _stamp(host_rows, icrcs, n):
    host_rows[:, n - 4:n] = icrcs.view(np.uint8).reshape(-1, 4)


@pytest.mark.parametrize("n", [64, 1024, 4096])
@pytest.mark.parametrize("off,ln", [(37, 3), (36, 4), (8, 4), (0, 44), (28, 12), (40, 16)])
def test_repair_fixed_stride(ctx, n, off, ln):
    """Fixed-stride batches; ranges over the PSN (37..39), masked IPv4 bytes
    (ttl/proto/csum 8..11), the whole header, and the first payload bytes."""
    count = 3000
    if off + ln > n - 4:
        pytest.skip("range past the covered bytes")
    host = oracle_c.synth_batch(SEED, 0, count, n)
    _stamp(host, oracle_c.icrc_batch(host, stride=n), n)
    old = host[:, off:off + ln].copy()
    rng = np.random.default_rng(SEED + off)
    host[:, off:off + ln] = rng.integers(0, 256, (count, ln), dtype=np.uint8)
    if off == 0:
        host[:, 0] = 0x45  # keep the IP version (the family is per packet)
    want = oracle_c.icrc_batch(host, stride=n)
    d = _dev(host)
    out = torch.empty(count, dtype=torch.int32, device="cuda")
    ctx.repair_device(d, count, off, _dev(old), out=out, stride=n, stamp=True)
    np.testing.assert_array_equal(_host(out).view(np.uint32), want)
    got_rows = _host(d).reshape(count, n)
    np.testing.assert_array_equal(got_rows[:, n - 4:].copy().view(np.uint32).ravel(), want)
    np.testing.assert_array_equal(got_rows[:, :n - 4], host[:, :n - 4])  # only trailers written


def test_repair_ragged_misaligned_with_invalid(ctx):
    """Offsets + lengths, odd alignments, an Ethernet l3_offset, lengths too
    short for the range (out 0, trailer untouched), out-only mode."""
    rng = np.random.default_rng(SEED)
    count, l3 = 2500, 14
    lens = rng.choice([44, 45, 60, 64, 255, 256, 1023, 1024, 4096, 9000], count).astype(np.uint32)
    lens[::97] = 30  # shorter than the rewritten range
    gaps = rng.integers(0, 40, count)
    offs = np.zeros(count, np.uint64)
    offs[1:] = np.cumsum(lens[:-1].astype(np.uint64) + l3 + gaps[:-1].astype(np.uint64))
    buf = rng.integers(0, 256, int(offs[-1]) + l3 + int(lens[-1]) + 64, dtype=np.uint8)
    for i in range(count):
        buf[int(offs[i]) + l3] = 0x45
    want_old = oracle_c.icrc_batch(buf, offsets=offs, lengths=lens, l3_offset=l3)
    for i in range(count):
        s = int(offs[i]) + l3 + int(lens[i]) - 4
        if lens[i] >= 44:
            buf[s:s + 4] = np.frombuffer(int(want_old[i]).to_bytes(4, "little"), np.uint8)
    off, ln = 33, 7  # DestQP + AckReq/PSN
    old = np.stack([buf[int(o) + l3 + off:int(o) + l3 + off + ln] for o in offs])
    before = buf.copy()
    for i in range(count):
        b = int(offs[i]) + l3 + off
        buf[b:b + ln] = rng.integers(0, 256, ln, dtype=np.uint8)
    want = oracle_c.icrc_batch(buf, offsets=offs, lengths=lens, l3_offset=l3)
    valid = lens >= off + ln + 4
    want[~valid] = 0
    d = _dev(buf)
    out = torch.empty(count, dtype=torch.int32, device="cuda")
    ctx.repair_device(d, count, off, _dev(old), out=out, offsets=_dev(offs), lengths=_dev(lens),
                      l3_offset=l3, stamp=False)
    np.testing.assert_array_equal(_host(out).view(np.uint32), want)
    np.testing.assert_array_equal(_host(d), buf)  # stamp=False: nothing written
    ctx.repair_device(d, count, off, _dev(old), out=None, offsets=_dev(offs), lengths=_dev(lens),
                      l3_offset=l3, stamp=True)
    got = _host(d)
    for i in np.flatnonzero(valid)[:400]:
        s = int(offs[i]) + l3 + int(lens[i]) - 4
        assert int.from_bytes(bytes(got[s:s + 4]), "little") == want[i]
    for i in np.flatnonzero(~valid):
        s = int(offs[i]) + l3
        assert np.array_equal(got[s:s + int(lens[i])], buf[s:s + int(lens[i])])
    del before


@pytest.mark.parametrize("off,ln", [(1, 60), (0, 8), (44, 12), (52, 4)])
@pytest.mark.parametrize("family", ["v6", "auto"])
def test_repair_ipv6_and_auto(ctx, family, off, ln):
    """RoCEv2 over IPv6: flow label / traffic class / hop limit are masked, so
    rewriting them must leave the ICRC alone; a PSN rewrite must not."""
    rng = np.random.default_rng(SEED + 6)
    count, n = 1500, 256
    host = rng.integers(0, 256, (count, n), dtype=np.uint8)
    host[:, 0] = 0x60 | (host[:, 0] & 0x0F)
    if family == "auto":
        host[::2, 0] = 0x45  # half IPv4
    fam_of = np.where(host[:, 0] >> 4 == 6, "v6", "v4")
    icrcs = np.array([oracle_c.icrc_one(bytes(r), family=f) for r, f in zip(host, fam_of)], np.uint32)
    _stamp(host, icrcs, n)
    # (1, 60): traffic class/flow label ... BTH PSN; (0, 8): the partly masked
    # version/traffic-class byte and the hop limit; (44, 12): UDP csum + BTH;
    # (52, 4): the IPv6 FECN/BECN byte (for IPv4 packets: payload)
    old = host[:, off:off + ln].copy()
    version = host[:, 0] & 0xF0
    host[:, off:off + ln] = rng.integers(0, 256, (count, ln), dtype=np.uint8)
    host[:, 0] = version | (host[:, 0] & 0x0F)  # the family stays (a version change is refused)
    want = np.array([oracle_c.icrc_one(bytes(r), family=f) for r, f in zip(host, fam_of)], np.uint32)
    out = torch.empty(count, dtype=torch.int32, device="cuda")
    ctx.repair_device(_dev(host), count, off, _dev(old), out=out, stride=n, family=family, stamp=False)
    np.testing.assert_array_equal(_host(out).view(np.uint32), want)


def test_repair_auto_version_change_is_refused_per_packet(ctx):
    count, n = 256, 128
    host = oracle_c.synth_batch(SEED, 0, count, n)
    _stamp(host, oracle_c.icrc_batch(host, stride=n), n)
    old = host[:, 0:2].copy()
    host[::3, 0] = 0x60  # version change on every third packet
    want = oracle_c.icrc_batch(host, stride=n)
    want[::3] = 0
    out = torch.empty(count, dtype=torch.int32, device="cuda")
    d = _dev(host)
    ctx.repair_device(d, count, 0, _dev(old), out=out, stride=n, family="auto", stamp=True)
    np.testing.assert_array_equal(_host(out).view(np.uint32), want)
    rows = _host(d).reshape(count, n)
    np.testing.assert_array_equal(rows[::3], host[::3])  # refused packets untouched


def test_repair_errors(ctx):
    d = torch.zeros(4096, dtype=torch.uint8, device="cuda")
    old = torch.zeros(300, dtype=torch.uint8, device="cuda")
    out = torch.empty(1, dtype=torch.int32, device="cuda")
    with pytest.raises(roce_icrc.ICRCError):
        ctx.repair_device(d, 1, 0, old.view(1, 300), out=out, stride=4096)   # len > RICRC_REPAIR_MAX
    with pytest.raises(roce_icrc.ICRCError):
        ctx.repair_device(d, 1, 37, old[:3].view(1, 3), out=None, stride=4096, stamp=False)  # nowhere to write
    with pytest.raises(ValueError):
        ctx.repair_device(d, 1, 37, old[:3].view(1, 3), out=out, stride=4096, family="v5")
    ctx.repair_device(d, 0, 37, old[:3].view(1, 3), out=out, stride=4096)  # empty batch: no-op


@pytest.mark.slow
def test_repair_headline_size_property(ctx):
    """1 M x 4096 B (the BASELINE headline batch): stamp on the GPU, rewrite every
    PSN, repair in place; the repaired ICRCs equal a full recompute and every
    trailer verifies."""
    count, n = 1 << 20, 4096
    buf = torch.empty(count * n, dtype=torch.uint8, device="cuda")
    ctx.synth_device(buf, SEED, 0, count, n)
    icrc = torch.empty(count, dtype=torch.int32, device="cuda")
    ctx.batch_device(buf, count, icrc, stride=n)
    rows = buf.view(count, n)
    rows[:, n - 4:] = icrc.view(torch.uint8).view(count, 4)
    off, ln = 37, 3
    old = rows[:, off:off + ln].clone()
    g = torch.Generator(device="cuda").manual_seed(SEED)
    rows[:, off:off + ln] = torch.randint(0, 256, (count, ln), dtype=torch.uint8, device="cuda", generator=g)
    rep = torch.empty(count, dtype=torch.int32, device="cuda")
    ctx.repair_device(buf, count, off, old, out=rep, stride=n, stamp=True)
    full = torch.empty(count, dtype=torch.int32, device="cuda")
    ctx.batch_device(buf, count, full, stride=n)
    ver = torch.empty(count, dtype=torch.int32, device="cuda")
    ctx.batch_device(buf, count, ver, stride=n, verify=True)
    torch.cuda.synchronize()
    assert torch.equal(rep, full)
    assert int(ver.sum()) == count
    assert int((rep != icrc).sum()) > count * 0.99  # the PSNs really changed the ICRCs
    # spot-check against the oracle on a host copy of the first packets
    host = rows[:2048].cpu().numpy()
    np.testing.assert_array_equal(rep[:2048].cpu().numpy().view(np.uint32),
                                  oracle_c.icrc_batch(host, stride=n))
