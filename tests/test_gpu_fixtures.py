"""GPU replay of the committed reference-derived fixtures, checked against the
ICRC values STORED in the fixtures (not a fresh oracle call).

* tests/golden/sim_stream.{bin,json}: every transmission of the unchanged
  reference simulator (python/simulator.py:49-55, 59-82) for seeds 1-3 --
  2,256 packets: 48-byte ACKs, READ / WRITE / LOOPBACK(REPL) packets of odd
  lengths, serialised by roce_icrc.wire (captured by gen_sim_stream.py).
* tests/golden/icrc_golden.{bin,json}: 60 vectors, among them the known
  answer built from the reference's own P4 ACK template
  (shuffle_ingress.p4:514-560, :717-724) -> ICRC 0x22791F6C, the READ / WRITE
  templates, every opcode, and raw byte strings of 4..43 bytes.

Each fixture goes through the HIP kernels as ONE ragged batch: device
offsets + lengths (back to back, odd alignments), Ethernet-framed
(l3_offset = 14), the host-buffer path (span and gather routes), verify mode
on the stamped bytes, the per-packet status path with the RoCEv2 classifier,
and a second stream (the ragged path's per-stream workspaces)."""
import json
import os

import numpy as np
import pytest

torch = pytest.importorskip("torch")

import roce_icrc  # noqa: E402

pytestmark = pytest.mark.gpu

HERE = os.path.join(os.path.dirname(__file__), "golden")


def _load(name):
    meta = json.load(open(os.path.join(HERE, name + ".json")))
    blob = np.frombuffer(open(os.path.join(HERE, name + ".bin"), "rb").read(), np.uint8)
    return meta, blob


def sim_stream():
    """(blob, offsets, lengths, stored ICRCs) of all seeds' transmissions."""
    meta, blob = _load("sim_stream")
    recs = [r for s in meta["seeds"].values() for r in s["packets"]]
    offs = np.array([r["offset"] for r in recs], np.uint64)
    lens = np.array([r["len"] for r in recs], np.uint32)
    icrc = np.array([r["icrc"] for r in recs], np.uint32)
    return blob, offs, lens, icrc


def golden():
    meta, blob = _load("icrc_golden")
    cases = meta["cases"]
    offs = np.array([c["offset"] for c in cases], np.uint64)
    lens = np.array([c["len"] for c in cases], np.uint32)
    icrc = np.array([c["icrc"] for c in cases], np.uint32)
    assert int(icrc[0]) == meta["ack_kat"]["icrc"] == 0x22791F6C
    return blob, offs, lens, icrc


FIXTURES = {"sim_stream": sim_stream, "golden": golden}


def _packed(blob, offs, lens, gap_rng=None, l3_offset=0, ethertype=0x0800):
    """The fixture's packets re-packed into one buffer: optional Ethernet
    header in front of each (l3_offset = 14) and random gaps (odd starts)."""
    parts, new_offs, pos = [], [], 0
    for o, n in zip(offs.tolist(), lens.tolist()):
        gap = int(gap_rng.integers(0, 19)) if gap_rng is not None else 0
        parts.append(np.zeros(gap, np.uint8))
        pos += gap
        new_offs.append(pos)
        if l3_offset:
            eth = np.zeros(l3_offset, np.uint8)
            eth[:12] = np.arange(12, dtype=np.uint8) + 1  # dmac | smac
            eth[12:14] = (ethertype >> 8, ethertype & 0xFF)
            parts.append(eth)
        parts.append(blob[o:o + n])
        pos += l3_offset + n
    parts.append(np.zeros(64, np.uint8))
    return np.concatenate(parts), np.array(new_offs, np.uint64)


def _dev(a):
    return torch.from_numpy(np.ascontiguousarray(a)).cuda()


def _u32(t):
    torch.cuda.synchronize()
    return t.cpu().numpy().view(np.uint32)


@pytest.mark.parametrize("name", sorted(FIXTURES))
@pytest.mark.parametrize("layout", ["as_captured", "gaps", "ethernet"])
def test_fixture_device_batch_matches_stored_icrc(ctx, name, layout):
    blob, offs, lens, stored = FIXTURES[name]()
    l3 = 14 if layout == "ethernet" else 0
    if layout == "as_captured":
        buf, o = np.concatenate([blob, np.zeros(64, np.uint8)]), offs
    else:
        buf, o = _packed(blob, offs, lens, np.random.default_rng(len(lens)), l3_offset=l3)
    out = torch.empty(len(lens), dtype=torch.int32, device="cuda")
    ctx.batch_device(_dev(buf), len(lens), out, offsets=_dev(o), lengths=_dev(lens), l3_offset=l3,
                     stream=torch.cuda.current_stream())
    np.testing.assert_array_equal(_u32(out), stored)


@pytest.mark.parametrize("name", sorted(FIXTURES))
def test_fixture_on_a_second_stream(ctx, name):
    blob, offs, lens, stored = FIXTURES[name]()
    buf, o = _packed(blob, offs, lens, np.random.default_rng(3))
    st = torch.cuda.Stream()
    with torch.cuda.stream(st):
        out = torch.empty(len(lens), dtype=torch.int32, device="cuda")
        ctx.batch_device(_dev(buf), len(lens), out, offsets=_dev(o), lengths=_dev(lens), stream=st)
    st.synchronize()
    np.testing.assert_array_equal(out.cpu().numpy().view(np.uint32), stored)


@pytest.mark.parametrize("name", sorted(FIXTURES))
def test_fixture_host_batch_span_and_gather(ctx, name):
    """ricrc_batch_host: the ascending ring takes the span route, the shuffled
    descriptors the gather route.  Packets under RICRC_MIN_LEN (the golden
    raw_* strings) are an -EINVAL for this call, so they are left out here
    and checked through the status call below."""
    blob, offs, lens, stored = FIXTURES[name]()
    keep = lens >= roce_icrc.MIN_LEN
    buf, o = _packed(blob, offs[keep], lens[keep], np.random.default_rng(5), l3_offset=14)
    np.testing.assert_array_equal(ctx.batch_host(buf, o, lens[keep], l3_offset=14), stored[keep])
    perm = np.random.default_rng(6).permutation(int(keep.sum()))
    np.testing.assert_array_equal(ctx.batch_host(buf, o[perm], lens[keep][perm], l3_offset=14), stored[keep][perm])


@pytest.mark.parametrize("name", sorted(FIXTURES))
def test_fixture_verify_mode_on_stamped_bytes(ctx, name):
    """The fixture packets stamped with their STORED ICRCs verify on the GPU;
    every 5th with one unmasked covered byte flipped fails."""
    blob, offs, lens, stored = FIXTURES[name]()
    buf, o = _packed(blob, offs, lens, np.random.default_rng(7))
    for i, (p, n) in enumerate(zip(o.tolist(), lens.tolist())):
        buf[p + n - 4:p + n] = np.frombuffer(int(stored[i]).to_bytes(4, "little"), np.uint8)
    bad = np.arange(0, len(lens), 5)
    for i in bad:  # byte n-5: the last covered byte, never a masked offset for n >= 44
        p, n = int(o[i]), int(lens[i])
        buf[p + max(n - 5, 0)] ^= 0x20
    out = torch.empty(len(lens), dtype=torch.int32, device="cuda")
    ctx.batch_device(_dev(buf), len(lens), out, offsets=_dev(o), lengths=_dev(lens), verify=True,
                     stream=torch.cuda.current_stream())
    want = np.ones(len(lens), np.uint32)
    want[bad] = 0
    got = _u32(out)
    short = lens < 5  # a 4-byte packet covers no byte: the flip hit its trailer, still a mismatch
    np.testing.assert_array_equal(got[~short], want[~short])


@pytest.mark.parametrize("name", sorted(FIXTURES))
def test_fixture_status_path_strict(ctx, name):
    """ricrc_batch_device_st / ricrc_batch_host_st, strict (the ingress
    parser's accept path) on Ethernet frames with EtherType 0x0800: every
    simulator packet is RoCEv2/IPv4 and keeps its stored ICRC; golden vectors
    under RICRC_MIN_LEN are RICRC_ST_BADLEN; golden vectors that are not
    RoCEv2 (raw bytes) are RICRC_ST_NOTROCE with out = 0."""
    blob, offs, lens, stored = FIXTURES[name]()
    buf, o = _packed(blob, offs, lens, np.random.default_rng(9), l3_offset=14)
    cls = np.array([roce_icrc.classify(blob[int(a):int(a) + int(n)].tobytes()) for a, n in zip(offs, lens)])
    want_st = np.where(lens < roce_icrc.MIN_LEN, roce_icrc.ST_BADLEN,
                       np.where(cls == 4, roce_icrc.ST_OK, roce_icrc.ST_NOTROCE)).astype(np.uint8)
    want_out = np.where(want_st == roce_icrc.ST_OK, stored, 0).astype(np.uint32)
    if name == "sim_stream":
        assert (want_st == roce_icrc.ST_OK).all()
    out = torch.empty(len(lens), dtype=torch.int32, device="cuda")
    st = torch.empty(len(lens), dtype=torch.uint8, device="cuda")
    ctx.batch_device_st(_dev(buf), len(lens), out, st, offsets=_dev(o), lengths=_dev(lens), l3_offset=14,
                        strict=True, stream=torch.cuda.current_stream())
    np.testing.assert_array_equal(_u32(out), want_out)
    np.testing.assert_array_equal(st.cpu().numpy(), want_st)
    h_out, h_st = ctx.batch_host_st(buf, o, lens, l3_offset=14, strict=True)
    np.testing.assert_array_equal(h_out, want_out)
    np.testing.assert_array_equal(h_st, want_st)
