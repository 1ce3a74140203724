"""CPU: pin the oracle before trusting it (no GPU).

The reference has no ICRC vectors, so the oracle is pinned by (1) the CRC-32
check value of the parameter set Tofino's HashAlgorithm_t.CRC32 names
(shuffle_egress.p4:461), (2) the hand-derived ACK known answer built from the
reference's P4 templates, (3) three independent formulations agreeing, (4) the
CRC-32 residue, (5) mask invariance exactly on the fields calc_icrc() forces
to 0xFF (shuffle_egress.p4:467-485), and (6) the committed golden vectors.
"""
import json
import os
import random
import struct
import zlib

import numpy as np
import pytest

import icrc_oracle as O
import oracle_c

GOLDEN = os.path.join(os.path.dirname(__file__), "golden")


def golden():
    meta = json.load(open(os.path.join(GOLDEN, "icrc_golden.json")))
    blob = open(os.path.join(GOLDEN, "icrc_golden.bin"), "rb").read()
    return meta, [(c["desc"], blob[c["offset"]: c["offset"] + c["len"]], c["icrc"]) for c in meta["cases"]]


def test_crc32_parameter_set_kat():
    assert zlib.crc32(b"123456789") == 0xCBF43926
    assert O._crc32_bitwise(b"123456789") ^ 0xFFFFFFFF == 0xCBF43926


def test_ack_known_answer():
    pkt = bytes.fromhex("450200301234400040110000c0a80164c0a80101457b12b7001c00001140ffff"
                        "0000001100000005000000016c1f7922")
    assert O.icrc(pkt) == 0x22791F6C
    assert pkt[-4:] == struct.pack("<I", 0x22791F6C)  # little-endian trailer (shuffle_egress.p4:493)
    assert O.residue_ok(pkt)


def test_prefix_register_is_rxe_seed():
    assert zlib.crc32(O.PREFIX) ^ 0xFFFFFFFF == O.REGISTER_AFTER_PREFIX == 0xDEBB20E3


def test_golden_vectors_all_formulations():
    meta, cases = golden()
    assert meta["crc32_check_123456789"] == 0xCBF43926
    assert len(cases) >= 50
    for desc, pkt, want in cases:
        assert O.icrc(pkt) == want, desc
        assert O.icrc_bitwise(pkt) == want, desc
        assert O.icrc_rxe(pkt) == want, desc
        for kind in ("bitwise", "bytewise", "fast"):
            assert oracle_c.icrc_one(pkt, kind) == want, (desc, kind)
        assert O.residue_ok(O.stamp(pkt)), desc


@pytest.mark.parametrize("n", [44, 64, 1024, 4096])
def test_mask_invariance(n):
    rng = random.Random(n)
    pkt = bytearray(rng.getrandbits(8) for _ in range(n))
    base = O.icrc(bytes(pkt))
    for off in O.MASK_OFFSETS:  # masked: any value, same ICRC
        q = bytearray(pkt)
        q[off] ^= 0xA5
        assert O.icrc(bytes(q)) == base, off
    for off in [o for o in (0, 2, 9, 12, 20, 28, 33, 39, 40, n - 5) if o < n - 4]:  # covered: must change
        q = bytearray(pkt)
        q[off] ^= 0x01
        assert O.icrc(bytes(q)) != base, off
    q = bytearray(pkt)
    q[-1] ^= 0xFF  # the trailer itself is not covered
    assert O.icrc(bytes(q)) == base


def test_batch_oracles_agree_and_threads():
    buf = oracle_c.synth_batch(11, 0, 300, 1024)
    a = oracle_c.icrc_batch(buf, stride=1024, threads=1, kind="bytewise")
    b = oracle_c.icrc_batch(buf, stride=1024, threads=4, kind="fast")
    c = O.icrc_batch(buf, stride=1024)
    np.testing.assert_array_equal(a, b)
    np.testing.assert_array_equal(a, c)


def test_synth_generator_header_template():
    """Synthetic packets are RoCEv2 SEND_ONLY per the reference templates."""
    buf = oracle_c.synth_batch(5, 1000, 8, 4096)
    for k, pkt in enumerate(buf):
        i = 1000 + k
        assert pkt[0] == 0x45 and pkt[9] == 17
        assert struct.unpack(">H", pkt[2:4].tobytes())[0] == 4096
        assert struct.unpack(">H", pkt[22:24].tobytes())[0] == 4791
        assert pkt[28] == 0x04 and pkt[29] == 0x40
        assert struct.unpack(">I", b"\0" + pkt[37:40].tobytes())[0] == i & 0xFFFFFF
    # masked fields are random across packets
    assert len({int(p[1]) for p in oracle_c.synth_batch(5, 0, 64, 64)}) > 8


def test_gf_helpers_against_bruteforce():
    rng = random.Random(3)
    for _ in range(20):
        r, n = rng.getrandbits(32), rng.randrange(0, 300)
        x8n = O.crc_shift(0x80000000, n)
        assert O.gf_mul(r, x8n) == O.crc_shift(r, n)


def test_ack_matches_calc_icrc_field_list():
    """For the packet calc_icrc() was written for -- the switch's write ACK,
    IPv4 || UDP || BTH || AETH || ICRC (48 B, shuffle_ingress.p4:514-560) --
    the oracle's "0xFF x 8 || masked L3[0, n-4)" hashes exactly the P4 field
    list of shuffle_egress.p4:464-491, concatenated in order (network byte
    order), through the CRC32 preset (= zlib.crc32).  Everything beyond that
    shape is the deliberate IBTA generalisation (icrc_oracle.py header)."""
    import struct
    import zlib

    rng = random.Random(17)
    for _ in range(200):
        f = dict(ver_ihl=0x45, diffserv=rng.getrandbits(8), total_len=48, ident=rng.getrandbits(16),
                 flag_offset=rng.getrandbits(16), ttl=rng.getrandbits(8), proto=17, csum=rng.getrandbits(16),
                 src=rng.getrandbits(32), dst=rng.getrandbits(32), sport=rng.getrandbits(16), dport=4791,
                 ulen=28, ucsum=rng.getrandbits(16), opcode=0x11, se=rng.getrandbits(8), pkey=rng.getrandbits(16),
                 fbr=rng.getrandbits(8), dqpn=rng.getrandbits(24), psn=rng.getrandbits(32),
                 syndrome=rng.getrandbits(8), msn=rng.getrandbits(24))
        l3 = (struct.pack(">BBHHHBBHII", f["ver_ihl"], f["diffserv"], f["total_len"], f["ident"], f["flag_offset"],
                          f["ttl"], f["proto"], f["csum"], f["src"], f["dst"])
              + struct.pack(">HHHH", f["sport"], f["dport"], f["ulen"], f["ucsum"])
              + struct.pack(">BBHB", f["opcode"], f["se"], f["pkey"], f["fbr"]) + f["dqpn"].to_bytes(3, "big")
              + struct.pack(">I", f["psn"]) + struct.pack(">B", f["syndrome"]) + f["msn"].to_bytes(3, "big")
              + b"\0\0\0\0")
        assert len(l3) == 48
        fields = (b"\xff" * 8                                                      # :465
                  + struct.pack(">B", f["ver_ihl"]) + b"\xff"                       # :466-467
                  + struct.pack(">HHH", f["total_len"], f["ident"], f["flag_offset"])  # :468-470
                  + b"\xff" + struct.pack(">B", f["proto"]) + b"\xff\xff"           # :471-473
                  + struct.pack(">II", f["src"], f["dst"])                          # :474-475
                  + struct.pack(">HHH", f["sport"], f["dport"], f["ulen"]) + b"\xff\xff"  # :477-480
                  + struct.pack(">BBH", f["opcode"], f["se"], f["pkey"]) + b"\xff"  # :482-485
                  + f["dqpn"].to_bytes(3, "big") + struct.pack(">I", f["psn"])     # :486-487
                  + struct.pack(">B", f["syndrome"]) + f["msn"].to_bytes(3, "big"))  # :489-490
        assert len(fields) == 52
        assert O.icrc(l3) == zlib.crc32(fields)


def test_classify_restatement_matches_product_classifier():
    """oracle.classify (the ingress parser's accept path restated,
    shuffle_ingress_parser.p4:12-36) against the product's CPU ricrc_classify
    on RoCEv2 packets of both families and on every single-field violation:
    version/IHL, protocol, total_len / payload length, UDP dport, lengths at
    and beyond the bounds -- and the EtherType rule for framed packets."""
    import random

    import roce_icrc

    rng = random.Random(12)
    ack = bytes.fromhex("450200301234400040110000c0a80164c0a80101457b12b7001c00001140ffff"
                        "0000001100000005000000016c1f7922")
    assert O.classify(ack) == roce_icrc.classify(ack) == 4
    assert O.classify(ack, 0x0800) == 4 and O.classify(ack, 0x86DD) == 0 and O.classify(ack, 0x0806) == 0

    def v6(n):
        p = bytearray(rng.getrandbits(8) for _ in range(n))
        p[0] = 0x60 | (p[0] & 15)
        p[4:6] = (n - 40).to_bytes(2, "big")
        p[6] = 17
        p[42:44] = (4791).to_bytes(2, "big")
        return p

    def v4(n):
        p = bytearray(rng.getrandbits(8) for _ in range(n))
        p[0], p[9] = 0x45, 17
        p[2:4] = n.to_bytes(2, "big")
        p[22:24] = (4791).to_bytes(2, "big")
        return p

    cases = []
    for n in (44, 45, 63, 64, 65, 100, 1024, 4096, 9000):
        cases += [v4(n)] + ([v6(n)] if n >= 64 else [])
        for off, val in ((0, 0x46), (0, 0x55), (9, 6), (2, 0), (23, 0xB8), (22, 0)):
            p = v4(n)
            p[off] = val
            cases.append(p)
        if n >= 64:
            for off, val in ((0, 0x50), (6, 6), (4, 0xFF), (43, 0xB8)):
                p = v6(n)
                p[off] = val
                cases.append(p)
    cases += [v4(44)[:43], bytes(43), bytes(64)]
    for p in cases:
        p = bytes(p)
        assert O.classify(p) == roce_icrc.classify(p), p[:8].hex()
    assert sum(O.classify(bytes(p)) == 4 for p in cases) >= 9
    assert sum(O.classify(bytes(p)) == 6 for p in cases) >= 6


def test_status_batch_restatement_on_a_small_ring():
    """oracle.status_batch on a hand-built ring: bad lengths, a non-RoCE frame
    under strict, framed EtherType checks, verify mode."""
    ack = bytearray.fromhex("450200301234400040110000c0a80164c0a80101457b12b7001c00001140ffff"
                            "0000001100000005000000016c1f7922")
    tcp = bytearray(ack)
    tcp[9] = 6
    frames = [b"\x01" * 12 + b"\x08\x00" + ack, b"\x01" * 12 + b"\x08\x00" + tcp,
              b"\x01" * 12 + b"\x86\xdd" + ack, b"\x01" * 12 + b"\x08\x00" + ack]
    buf = np.frombuffer(b"".join(frames), np.uint8)
    offs = np.array([0, 62, 124, 186], np.uint64)
    lens = np.array([48, 48, 48, 40], np.uint32)
    out, st = O.status_batch(buf, offs, lens, l3_offset=14, strict=True)
    assert st.tolist() == [O.ST_OK, O.ST_NOTROCE, O.ST_NOTROCE, O.ST_BADLEN]
    assert out.tolist() == [0x22791F6C, 0, 0, 0]
    out, st = O.status_batch(buf, offs, lens, l3_offset=14)
    assert st.tolist() == [O.ST_OK, O.ST_OK, O.ST_OK, O.ST_BADLEN] and out[1] == O.icrc(bytes(tcp))
    out, st = O.status_batch(buf, offs, lens, l3_offset=14, strict=True, verify=True)
    assert out.tolist() == [1, 0, 0, 0]
