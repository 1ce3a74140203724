"""RoCEv2 over IPv6 masks and incremental ICRC repair after
header rewrites (§8f-2), on the CPU.

IPv6 parity: the reference is IPv4-only (header.p4:42-53), so the IPv6 masks
follow IBTA Annex A17 as the Linux rxe driver applies them (rxe_icrc.c) --
"parity unpinned" by the reference; pinned here by the oracle's independent
formulations agreeing, the CRC-32 residue, and mask invariance exactly on the
rxe field set (and on nothing else).  Repair is checked against a full
recomputation of the rewritten packet."""
import random
import types
import zlib

import numpy as np
import pytest

import icrc_oracle as o
import oracle_c
import roce_icrc
from roce_icrc import wire

V6_MASKED = {0: 0x0F, 1: 0xFF, 2: 0xFF, 3: 0xFF, 7: 0xFF, 46: 0xFF, 47: 0xFF, 52: 0xFF}


def v6_packet(rng, n, tclass=None, flow=None):
    """A RoCEv2-over-IPv6 SEND_ONLY of n bytes from the wire adapter (payload random)."""
    p = types.SimpleNamespace(opcode="SEND_ONLY", smac=rng.randrange(4), dmac=-1, psn=rng.randrange(1 << 24),
                              dqpn=rng.randrange(1 << 24), ackreq=1, addr=0, len=0, msn=0, si=0, data=[])
    pkt = wire.encode(p, ipv6=True, tclass=rng.randrange(256) if tclass is None else tclass,
                      flow=rng.randrange(1 << 20) if flow is None else flow, hop=rng.randrange(256))
    pay = n - len(pkt)
    assert pay >= 0 and pay % 4 == 0
    body = bytearray(pkt[:-4]) + bytes(rng.randrange(256) for _ in range(pay)) + b"\0\0\0\0"
    # fix the IPv6 payload length / UDP length for the grown packet
    body[4:6] = (n - 40).to_bytes(2, "big")
    body[44:46] = (n - 40).to_bytes(2, "big")
    return body


def test_oracle_formulations_agree_ipv6():
    rng = random.Random(6)
    for n in (64, 68, 100, 256, 1024, 4096):
        pkt = v6_packet(rng, n)
        want = o.icrc(pkt, "v6")
        assert o.icrc_bitwise(pkt, "v6") == o.icrc_rxe(pkt, "v6") == want
        for kind in ("bitwise", "bytewise", "fast"):
            assert oracle_c.icrc_one(pkt, kind, "v6") == want
        assert o.residue_ok(o.stamp(pkt, "v6"), "v6")
        assert o.icrc(pkt, "auto") == want and (pkt[0] >> 4) == 6


def test_ipv6_mask_invariance_is_exactly_the_rxe_field_set():
    rng = random.Random(7)
    pkt = v6_packet(rng, 256)
    base = roce_icrc.icrc(pkt, "v6")
    for i in range(60):
        for bit in range(8):
            q = bytearray(pkt)
            q[i] ^= 1 << bit
            masked = (V6_MASKED.get(i, 0) >> bit) & 1
            assert (roce_icrc.icrc(q, "v6") == base) == bool(masked), (i, bit)


def test_library_matches_oracle_ipv6_and_auto():
    rng = random.Random(8)
    for _ in range(300):
        n = rng.choice([64, 68, 72, 96, 128, 500, 1024, 1500, 4096])
        pkt = v6_packet(rng, n)
        assert roce_icrc.icrc(pkt, "v6") == o.icrc(pkt, "v6")
        assert roce_icrc.icrc(pkt, "auto") == o.icrc(pkt, "v6")
        raw = bytes(rng.randrange(256) for _ in range(rng.randrange(4, 300)))
        assert roce_icrc.icrc(raw, "v6") == o.icrc(raw, "v6")
        assert roce_icrc.icrc(raw, "auto") == o.icrc(raw, "auto")
        assert roce_icrc.icrc(raw) == o.icrc(raw)  # the plain call keeps the reference's IPv4 masks
    stamped = roce_icrc.stamp(bytearray(v6_packet(rng, 512)), "v6")
    assert roce_icrc.verify(stamped, "v6") and roce_icrc.verify(stamped, "auto")
    assert o.residue_ok(bytes(stamped), "v6")
    with pytest.raises(ValueError):
        roce_icrc.icrc(stamped, "v5")


def test_classify_v4_v6():
    rng = random.Random(9)
    p = types.SimpleNamespace(opcode="ACK", smac=-1, dmac=0, psn=5, dqpn=0x11, ackreq=0, addr=0, len=0,
                              msn=1, si=0, data=[])
    assert roce_icrc.classify(wire.encode(p)) == 4
    assert roce_icrc.classify(wire.encode(p, ipv6=True)) == 6
    v6 = v6_packet(rng, 300)
    assert roce_icrc.classify(v6) == 6
    bad = bytearray(v6)
    bad[6] = 6  # next header TCP
    assert roce_icrc.classify(bad) == 0
    assert roce_icrc.classify(b"\x00" * 64) == 0


@pytest.mark.parametrize("family", ["v4", "v6", "auto"])
def test_repair_equals_recompute(family):
    rng = random.Random(hash(family) & 0xFFFF)
    for _ in range(400):
        n = rng.choice([44, 48, 60, 64, 100, 256, 1024, 4096, 9000])
        if family == "v4":
            pkt = bytearray(rng.randrange(256) for _ in range(n))
            pkt[0] = 0x45
        else:
            pkt = v6_packet(rng, max(64, n - n % 4)) if n >= 64 else bytearray(rng.randrange(256) for _ in range(n))
            if n < 64:
                pkt[0] = 0x60
        n = len(pkt)
        old_icrc = roce_icrc.icrc(pkt, family)
        m = n - 4
        off = rng.randrange(1 if family != "v4" else 0, m + 1) if m else 0  # keep the version byte
        ln = rng.randrange(0, min(64, m - off) + 1)
        old = bytes(pkt[off:off + ln])
        for i in range(off, off + ln):  # the rewrite (PSN / MSN / opcode / anything in range)
            pkt[i] = rng.randrange(256)
        assert roce_icrc.repair(pkt, off, old, old_icrc, family) == roce_icrc.icrc(pkt, family)


def test_repair_psn_patch_like_the_switch():
    """The switch's egress PSN patch (shuffle_egress.p4:635-671): BTH PSN bytes
    37..39 of an ACK rewritten; repair in O(3 bytes)."""
    p = types.SimpleNamespace(opcode="ACK", smac=-1, dmac=0, psn=5, dqpn=0x11, ackreq=0, addr=0, len=0,
                              msn=1, si=0, data=[])
    for ipv6 in (False, True):
        fam = "v6" if ipv6 else "v4"
        pkt = roce_icrc.stamp(wire.encode(p, ipv6=ipv6), fam)
        old_icrc = wire.trailer(pkt)
        psn_off = (40 if ipv6 else 20) + 8 + 9
        old = bytes(pkt[psn_off:psn_off + 3])
        pkt[psn_off:psn_off + 3] = (0xABCDEF).to_bytes(3, "big")
        new = roce_icrc.repair(pkt, psn_off, old, old_icrc, fam)
        assert new == roce_icrc.icrc(pkt, fam) == o.icrc(bytes(pkt), fam)
        pkt[-4:] = new.to_bytes(4, "little")
        assert roce_icrc.verify(pkt, fam)


def test_repair_errors():
    pkt = bytearray(100)
    pkt[0] = 0x45
    with pytest.raises(roce_icrc.ICRCError):
        roce_icrc.repair(pkt, 90, b"\0" * 8, 0)          # range past n-4
    v6 = bytearray(100)
    v6[0] = 0x60
    with pytest.raises(roce_icrc.ICRCError):
        roce_icrc.repair(v6, 0, b"\x45", 0, "auto")      # AUTO rewrite changing the IP version
    assert roce_icrc.repair(pkt, 10, b"", 0x1234) == 0x1234  # empty range: unchanged
