"""GPU: per-packet status and RoCEv2 classification of batches (NIC rings
carrying more than RoCE), against the oracle's restatement of the reference's
ingress accept path (shuffle_ingress_parser.p4:12-36: EtherType 0x0800 ->
IPv4 protocol 17 -> UDP dport 4791) and the product's CPU ricrc_classify.

The ring mixes RoCEv2/IPv4, RoCEv2/IPv6, ARP, TCP, UDP to another port,
IPv4 with options, a total_len that disagrees with the descriptor, RoCE
headers behind the wrong EtherType, and descriptor lengths outside
[RICRC_MIN_LEN, RICRC_MAX_LEN]."""
import numpy as np
import pytest

torch = pytest.importorskip("torch")

import icrc_oracle as O  # noqa: E402
import oracle_c  # noqa: E402
import roce_icrc  # noqa: E402

pytestmark = pytest.mark.gpu

KINDS = ("roce4", "roce6", "arp", "tcp", "udp53", "ihl6", "badtotal", "roce4_as_v6", "roce6_as_v4", "badlen")


def _l3(kind, n, rng, i):
    """(L3 bytes, EtherType) of one frame of the given kind, n bytes of L3."""
    if kind in ("roce4", "tcp", "udp53", "ihl6", "badtotal", "roce4_as_v6"):
        p = bytearray(oracle_c.synth_batch(0xA11 + i, i, 1, n)[0].tobytes())  # SEND_ONLY template
        if kind == "tcp":
            p[9] = 6
        elif kind == "udp53":
            p[22:24] = (53).to_bytes(2, "big")
        elif kind == "ihl6":
            p[0] = 0x46
        elif kind == "badtotal":
            p[2:4] = (n + 4).to_bytes(2, "big")
        p[-4:] = O.icrc(bytes(p)).to_bytes(4, "little")
        return bytes(p), (0x86DD if kind == "roce4_as_v6" else 0x0800)
    if kind in ("roce6", "roce6_as_v4"):
        p = bytearray(rng.integers(0, 256, n, dtype=np.uint8).tobytes())
        p[0] = 0x60 | (p[0] & 0x0F)
        p[4:6] = (n - 40).to_bytes(2, "big")
        p[6] = 17
        p[42:44] = (4791).to_bytes(2, "big")
        p[-4:] = O.icrc(bytes(p), "v6").to_bytes(4, "little")
        return bytes(p), (0x0800 if kind == "roce6_as_v4" else 0x86DD)
    if kind == "arp":
        p = bytearray(rng.integers(0, 256, n, dtype=np.uint8).tobytes())
        p[0:8] = bytes.fromhex("0001080006040001")
        return bytes(p), 0x0806
    raise ValueError(kind)


# RICRC_F_FRAMELEN rings: Ethernet frames whose descriptor length is the
# frame's extent past L3 -- a 44-byte SEND_ONLY (no payload) padded to the
# 60-byte minimum frame (2 bytes of padding), frames that keep their 4-byte
# FCS, both at once, and RoCEv2/IPv6 with an FCS.
FRAME_KINDS = ("pad44", "fcs", "pad44_fcs", "roce6_fcs")


def mixed_ring(count, seed, framed=True, frame_kinds=False):
    """Frames back to back with small gaps: (buf, offsets, lengths, kinds,
    EtherTypes).  Offsets point at the frame; L3 starts 14 bytes later when
    framed (else at the offset, no Ethernet header).  frame_kinds: a quarter
    of the frames carry Ethernet padding and / or an FCS after the datagram
    (FRAME_KINDS), their descriptor length covering it."""
    rng = np.random.default_rng(seed)
    sizes = np.array([64, 100, 256, 1024, 1500, 4096], np.uint32)
    kinds = [KINDS[k] for k in rng.choice(len(KINDS), size=count, p=[.35, .15, .05, .08, .07, .05, .05, .05, .05, .10])]
    if frame_kinds:
        fk = rng.choice(len(FRAME_KINDS), size=count)
        kinds = [FRAME_KINDS[f] if rng.random() < 0.25 else k for k, f in zip(kinds, fk)]
    parts, offs, lens, ets, pos = [], [], [], [], 0
    for i, kind in enumerate(kinds):
        gap = int(rng.integers(0, 12))
        parts.append(np.zeros(gap, np.uint8))
        pos += gap
        if kind == "badlen":
            n_desc = int(rng.choice([0, 3, 20, 43, 70000, 0xFFFFFFFF]))
            body, et = _l3("roce4", 64, rng, i)
        elif kind in FRAME_KINDS:
            n = 44 if kind.startswith("pad44") else int(rng.choice(sizes))
            body, et = _l3("roce6" if kind == "roce6_fcs" else "roce4", max(n, 64) if kind == "roce6_fcs" else n,
                           rng, i)
            tail = (bytes(2) if kind.startswith("pad44") else b"") + \
                (rng.integers(0, 256, 4, dtype=np.uint8).tobytes() if kind.endswith("fcs") else b"")
            body += tail
            n_desc = len(body)
        else:
            n = int(rng.choice(sizes[sizes >= (64 if "roce6" in kind else 46)]))
            body, et = _l3(kind, n, rng, i)
            n_desc = n
        hdr = bytes(range(1, 13)) + et.to_bytes(2, "big") if framed else b""
        frame = np.frombuffer(hdr + body, np.uint8)
        parts.append(frame)
        offs.append(pos)
        lens.append(n_desc)
        ets.append(et)
        pos += frame.size
    parts.append(np.zeros(128, np.uint8))
    return (np.concatenate(parts), np.array(offs, np.uint64), np.array(lens, np.uint32), kinds, ets)


def _dev(a):
    return torch.from_numpy(np.ascontiguousarray(a)).cuda()


def _want_class(buf, offs, lens, l3, ets):
    """Oracle classification per packet, and the product's CPU classifier."""
    o_cls, p_cls = [], []
    for o, n, et in zip(offs.tolist(), lens.tolist(), ets):
        if n < roce_icrc.MIN_LEN or n > roce_icrc.MAX_LEN:
            o_cls.append(0)
            p_cls.append(0)
            continue
        pkt = buf[o + l3:o + l3 + n].tobytes()
        o_cls.append(O.classify(pkt, et if l3 >= 14 else None))
        c = roce_icrc.classify(pkt)
        if l3 >= 14 and c and et != (0x0800 if c == 4 else 0x86DD):
            c = 0
        p_cls.append(c)
    return np.array(o_cls, np.uint8), np.array(p_cls, np.uint8)


@pytest.mark.parametrize("framed", [True, False])
def test_classify_device_matches_oracle_and_cpu_classifier(ctx, framed):
    buf, offs, lens, kinds, ets = mixed_ring(3000, 1 + framed, framed)
    l3 = 14 if framed else 0
    o_cls, p_cls = _want_class(buf, offs, lens, l3, ets)
    np.testing.assert_array_equal(o_cls, p_cls)
    cls = torch.empty(len(lens), dtype=torch.uint8, device="cuda")
    ctx.classify_device(_dev(buf), len(lens), cls, offsets=_dev(offs), lengths=_dev(lens), l3_offset=l3,
                        stream=torch.cuda.current_stream())
    torch.cuda.synchronize()
    got = cls.cpu().numpy()
    np.testing.assert_array_equal(got, o_cls)
    k = np.array(kinds)
    assert set(got[k == "roce4"]) == {4} and set(got[k == "roce6"]) == {6}
    for bad in ("arp", "tcp", "udp53", "ihl6", "badtotal", "badlen"):
        assert not got[k == bad].any(), bad
    if framed:  # RoCE headers behind the other family's EtherType
        assert not got[k == "roce4_as_v6"].any() and not got[k == "roce6_as_v4"].any()


@pytest.mark.parametrize("family,strict,verify", [("auto", True, False), ("v4", True, False), ("v6", True, False),
                                                  ("auto", False, False), ("auto", True, True),
                                                  ("v4", False, True)])
@pytest.mark.parametrize("framed", [True, False])
def test_status_batch_device_and_host(ctx, family, strict, verify, framed):
    """Per packet: status and out (ICRC, or 1/0 in verify mode) equal the
    oracle's status_batch; out = 0 wherever status != OK -- so an ICRC of 0
    and a rejected / bad packet are told apart by the status, not the value."""
    buf, offs, lens, kinds, ets = mixed_ring(2500, 7 + framed, framed)
    l3 = 14 if framed else 0
    if verify:  # corrupt the payload of every 9th packet (stamped ones fail verify)
        for i in range(0, len(lens), 9):
            if roce_icrc.MIN_LEN <= lens[i] <= roce_icrc.MAX_LEN:
                buf[int(offs[i]) + l3 + int(lens[i]) - 5] ^= 0x08
    w_out, w_st = O.status_batch(buf, offsets=offs, lengths=lens, l3_offset=l3, family=family, strict=strict,
                                 verify=verify)
    assert (w_st == O.ST_BADLEN).sum() > 100 and (w_st == O.ST_OK).sum() > 300
    if strict:
        assert (w_st == O.ST_NOTROCE).sum() > 300
    else:
        assert not (w_st == O.ST_NOTROCE).any()
    count = len(lens)
    out = torch.full((count,), -1, dtype=torch.int32, device="cuda")
    st = torch.full((count,), 0xEE, dtype=torch.uint8, device="cuda")
    ctx.batch_device_st(_dev(buf), count, out, st, offsets=_dev(offs), lengths=_dev(lens), l3_offset=l3,
                        family=family, strict=strict, verify=verify, stream=torch.cuda.current_stream())
    torch.cuda.synchronize()
    np.testing.assert_array_equal(st.cpu().numpy(), w_st)
    np.testing.assert_array_equal(out.cpu().numpy().view(np.uint32), w_out)
    h_out, h_st = ctx.batch_host_st(buf, offs, lens, l3_offset=l3, family=family, strict=strict, verify=verify)
    np.testing.assert_array_equal(h_st, w_st)
    np.testing.assert_array_equal(h_out, w_out)
    perm = np.random.default_rng(2).permutation(count)  # the host path's gather route
    h_out, h_st = ctx.batch_host_st(buf, offs[perm], lens[perm], l3_offset=l3, family=family, strict=strict,
                                    verify=verify)
    np.testing.assert_array_equal(h_st, w_st[perm])
    np.testing.assert_array_equal(h_out, w_out[perm])


@pytest.mark.parametrize("n,stride", [(4096, 4096), (1024, 1024), (64, 64), (1500, 1536)])
def test_status_fixed_stride_batches(ctx, n, stride):
    """Fixed-length batches through the strided-chain / streaming kernels with
    a status: all OK without strict (no header read); with strict, packets
    whose UDP port was rewritten are NOTROCE and read 0."""
    count = 3001
    host = oracle_c.synth_batch(0x57A7, 0, count, n, stride)
    want = oracle_c.icrc_batch(host, stride=stride, count=count) if n == stride else \
        oracle_c.icrc_batch(host, offsets=np.arange(count, dtype=np.uint64) * stride,
                            lengths=np.full(count, n, np.uint32))
    out = torch.empty(count, dtype=torch.int32, device="cuda")
    st = torch.empty(count, dtype=torch.uint8, device="cuda")
    d = _dev(host)
    ctx.batch_device_st(d, count, out, st, stride=stride, stream=torch.cuda.current_stream()) if n == stride else \
        ctx.batch_device_st(d, count, out, st, offsets=_dev(np.arange(count, dtype=np.uint64) * stride),
                            lengths=_dev(np.full(count, n, np.uint32)), stream=torch.cuda.current_stream())
    torch.cuda.synchronize()
    assert not st.cpu().numpy().any()
    np.testing.assert_array_equal(out.cpu().numpy().view(np.uint32), want)
    if n != stride:
        return
    host[::7, 23] ^= 1  # dport 4791 -> 4790: not RoCE
    want_st = np.zeros(count, np.uint8)
    want_st[::7] = roce_icrc.ST_NOTROCE
    ctx.batch_device_st(_dev(host), count, out, st, stride=stride, strict=True, stream=torch.cuda.current_stream())
    torch.cuda.synchronize()
    np.testing.assert_array_equal(st.cpu().numpy(), want_st)
    got = out.cpu().numpy().view(np.uint32)
    assert not got[::7].any()
    keep = want_st == 0
    np.testing.assert_array_equal(got[keep], want[keep])


def test_status_call_errors(ctx):
    import errno

    d = torch.zeros(4096, dtype=torch.uint8, device="cuda")
    out = torch.empty(1, dtype=torch.int32, device="cuda")
    st = torch.empty(1, dtype=torch.uint8, device="cuda")
    with pytest.raises(roce_icrc.ICRCError) as e:  # the batch's one length out of range: a call error
        ctx.batch_device_st(d, 1, out, st, stride=40)
    assert e.value.rc == -errno.EINVAL
    with pytest.raises(roce_icrc.ICRCError):  # no status array
        ctx.batch_device_st(d, 1, out, None, stride=64)
    rc = ctx._lib.ricrc_batch_device_st(ctx.handle, 0, d.data_ptr(), None, None, 64, 1, 0, out.data_ptr(),
                                        st.data_ptr(), None, 0x800)
    assert rc == -errno.EINVAL  # unknown flag bit


@pytest.mark.parametrize("family,strict,verify", [("v4", True, False), ("auto", True, False), ("auto", False, False),
                                                  ("auto", True, True)])
def test_framelen_padded_and_fcs_frames(ctx, family, strict, verify):
    """RICRC_F_FRAMELEN on an Ethernet NIC ring whose descriptor lengths are
    frame extents: 44-byte SEND_ONLY packets padded to the 60-byte minimum
    frame, frames that keep their FCS, both, RoCEv2/IPv6 with an FCS, next to
    every reject case of the mixed ring.  The packet's length comes from its IP
    header (the reference's parser never uses a descriptor length,
    shuffle_ingress_parser.p4:12-36; total_len at header.p4:45); status and out
    equal the oracle's status_batch(framelen=True) on the device and on both
    host routes (span, gather)."""
    buf, offs, lens, kinds, ets = mixed_ring(3000, 41, True, frame_kinds=True)
    l3 = 14
    k = np.array(kinds)
    for kind in FRAME_KINDS:
        assert (k == kind).sum() > 50, kind
    if verify:  # corrupt one covered byte of every 9th packet: the IP length decides where the trailer is
        for i in range(0, len(lens), 9):
            if roce_icrc.MIN_LEN <= lens[i] <= roce_icrc.MAX_LEN:
                buf[int(offs[i]) + l3 + 40] ^= 0x08
    w_out, w_st = O.status_batch(buf, offsets=offs, lengths=lens, l3_offset=l3, family=family, strict=strict,
                                 verify=verify, framelen=True)
    fr = np.isin(k, FRAME_KINDS) & ~((k == "roce6_fcs") & strict & (family == "v4"))
    assert (w_st[fr] == O.ST_OK).all()  # every padded / FCS frame (of an accepted family) is accepted and computed
    if not verify:
        for i in np.flatnonzero(fr)[:200]:  # over the datagram only: the IP length, not the descriptor's
            o, n = int(offs[i]) + l3, int(lens[i])
            pkt = buf[o:o + n].tobytes()
            m = O.frame_l3_len(pkt)
            assert m < n and w_out[i] == O.icrc(pkt[:m], family)
    if strict:  # without the flag the same frames are rejected (total_len != descriptor length)
        _, st0 = O.status_batch(buf, offsets=offs, lengths=lens, l3_offset=l3, family=family, strict=True)
        assert (st0[fr] == O.ST_NOTROCE).all()
        assert (w_st == O.ST_NOTROCE).sum() > 300
    count = len(lens)
    out = torch.full((count,), -1, dtype=torch.int32, device="cuda")
    st = torch.full((count,), 0xEE, dtype=torch.uint8, device="cuda")
    ctx.batch_device_st(_dev(buf), count, out, st, offsets=_dev(offs), lengths=_dev(lens), l3_offset=l3,
                        family=family, strict=strict, verify=verify, framelen=True, stream=torch.cuda.current_stream())
    torch.cuda.synchronize()
    np.testing.assert_array_equal(st.cpu().numpy(), w_st)
    np.testing.assert_array_equal(out.cpu().numpy().view(np.uint32), w_out)
    h_out, h_st = ctx.batch_host_st(buf, offs, lens, l3_offset=l3, family=family, strict=strict, verify=verify,
                                    framelen=True)
    np.testing.assert_array_equal(h_st, w_st)
    np.testing.assert_array_equal(h_out, w_out)
    perm = np.random.default_rng(3).permutation(count)  # the gather route
    h_out, h_st = ctx.batch_host_st(buf, offs[perm], lens[perm], l3_offset=l3, family=family, strict=strict,
                                    verify=verify, framelen=True)
    np.testing.assert_array_equal(h_st, w_st[perm])
    np.testing.assert_array_equal(h_out, w_out[perm])


def test_framelen_fixed_stride_ring(ctx):
    """A fixed-slot ring (no per-packet lengths: every descriptor is the slot)
    of 44..1500-byte packets under RICRC_F_FRAMELEN: the device pre-pass gives
    each packet its IP length, so the batch runs as a ragged one."""
    rng = np.random.default_rng(5)
    count, slot, l3 = 2048, 1536, 14
    buf = rng.integers(0, 256, count * slot + 64, dtype=np.uint8)
    for i in range(count):
        n = int(rng.choice([44, 60, 256, 1000, 1500 - l3]))
        body, et = _l3("roce4", n, rng, i)
        o = i * slot
        buf[o + 12:o + 14] = np.frombuffer(et.to_bytes(2, "big"), np.uint8)
        buf[o + l3:o + l3 + n] = np.frombuffer(body, np.uint8)
    w_out, w_st = O.status_batch(buf, stride=slot, count=count, l3_offset=l3, strict=True, framelen=True)
    assert (w_st == O.ST_OK).all()
    out = torch.empty(count, dtype=torch.int32, device="cuda")
    st = torch.empty(count, dtype=torch.uint8, device="cuda")
    ctx.batch_device_st(_dev(buf), count, out, st, stride=slot, l3_offset=l3, strict=True, framelen=True,
                        stream=torch.cuda.current_stream())
    torch.cuda.synchronize()
    np.testing.assert_array_equal(st.cpu().numpy(), w_st)
    np.testing.assert_array_equal(out.cpu().numpy().view(np.uint32), w_out)
    h_out, h_st = ctx.batch_host_st(buf, stride=slot, count=count, l3_offset=l3, strict=True, framelen=True)
    np.testing.assert_array_equal(h_st, w_st)
    np.testing.assert_array_equal(h_out, w_out)
