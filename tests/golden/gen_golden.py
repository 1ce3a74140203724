#!/usr/bin/env python3
"""Generate the committed ICRC golden vectors (tests/golden/icrc_golden.{bin,json}).

Parity status: the reference holds NO ICRC vectors (its only ICRC is the
disabled Tofino action p4/shuffle/shuffle_egress.p4:461-494), so these are
build-derived: inputs are RoCEv2 packets shaped after the reference's own
header templates and opcodes, expected values come from the oracle
(oracle/icrc_oracle.py, zlib) and are cross-checked against the independent
bitwise formulation and the CRC-32 residue before being written.

Contents (all little-endian JSON ints, packets concatenated in the .bin):
* ACK from the P4 template (shuffle_ingress.p4:514-560 + IPv4 fields of
  :717-724), the hand-derived known answer 0x22791F6C;
* READ request template (shuffle_ingress.p4:694-743, total_len 60) and a
  WRITE_ONLY built from it (:758-812);
* REPL (0x15, shuffle_header.p4:12,105-118) with 1..4 shuffle items;
* SEND_ONLY packets at the BASELINE sizes (64/256/1024/4096) and ragged
  sizes (44..9000), random masked fields and payloads;
* every opcode of header.p4:16-34 with its extension header;
* the CRC-32 check string "123456789" (KAT 0xCBF43926 of the underlying CRC).

Run:  python tests/golden/gen_golden.py   (deterministic; seed fixed below)
"""
import json
import os
import random
import struct
import sys
import zlib

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "..", "oracle"))
import icrc_oracle as O  # noqa: E402

SEED = 0x601DE11


def ipv4(total_len, tos=0x02, ident=0x1234, flags=0x4000, ttl=64, csum=0, src=(192, 168, 1, 100),
         dst=(192, 168, 1, 1)):
    return struct.pack(">BBHHHBBH4B4B", 0x45, tos, total_len, ident, flags, ttl, 17, csum, *src, *dst)


def udp(length, sport=0x457B, csum=0):
    return struct.pack(">HHHH", sport, 4791, length, csum)


def bth(opcode, dqpn, psn, ackreq=0, pad=0, fb=0, pkey=0xFFFF):
    return struct.pack(">BBHB", opcode, 0x40 | (pad << 4), pkey, fb) + dqpn.to_bytes(3, "big") + \
        struct.pack(">I", ((0x80 if ackreq else 0) << 24) | (psn & 0xFFFFFF))


def build(opcode, ext, payload, rnd=None, **kw):
    pad = (-len(payload)) % 4
    payload = payload + b"\0" * pad
    n = 20 + 8 + 12 + len(ext) + len(payload) + 4
    ipk = dict(tos=kw.get("tos", 0x02), ttl=kw.get("ttl", 64), csum=kw.get("csum", 0))
    pkt = ipv4(n, **ipk) + udp(n - 20, csum=kw.get("ucsum", 0)) + \
        bth(opcode, kw.get("dqpn", 0x11), kw.get("psn", 0), kw.get("ackreq", 0), pad, kw.get("fb", 0)) + \
        ext + payload
    return pkt + (kw.get("trailer") or b"\0\0\0\0")


def main():
    rng = random.Random(SEED)
    cases = []

    def add(desc, pkt):
        cases.append((desc, bytes(pkt)))

    # Known answer: ACK from the P4 template, psn 5, AETH syndrome 0 / msn 1.
    ack = build(0x11, struct.pack(">I", 1), b"", dqpn=0x11, psn=5)
    add("ack_p4_template_kat", ack)
    add("read_req_p4_template", build(0x0C, struct.pack(">QII", 0x7F0000001000, 0x1234, 1024), b"",
                                      dqpn=0x93589, psn=7))
    add("write_only_p4_template", build(0x0A, struct.pack(">QII", 0x7F0000002000, 0x42, 16),
                                        bytes(range(16)), dqpn=0xD13CB, psn=9, ackreq=1))
    for items in range(1, 5):
        body = b"".join(struct.pack(">HHIQ", i, 4, 4 * (items - 1 - i), 0x7F0000003000 + 4 * i) for i in range(items))
        add(f"repl_{items}_items", build(0x15, struct.pack(">BBH", 0, items, 3), body, psn=items))
    # Every opcode with its extension header (shuffle_ingress_parser.p4:39-64).
    for op in list(range(0x00, 0x12)) + [0x15]:
        ext = b""
        if op in (0x06, 0x0A, 0x0C):
            ext = struct.pack(">QII", rng.getrandbits(64), rng.getrandbits(32), rng.getrandbits(32))
        elif op in (0x0D, 0x0F, 0x10, 0x11):
            ext = struct.pack(">I", rng.getrandbits(32))
        elif op in (0x03, 0x05, 0x09, 0x0B):
            ext = struct.pack(">I", rng.getrandbits(32))  # ImmDt
        payload = bytes(rng.getrandbits(8) for _ in range(rng.randrange(0, 200)))
        add(f"opcode_{op:#04x}", build(op, ext, payload, dqpn=rng.getrandbits(24), psn=rng.getrandbits(24),
                                       tos=rng.getrandbits(8), ttl=rng.getrandbits(8),
                                       csum=rng.getrandbits(16), ucsum=rng.getrandbits(16),
                                       fb=rng.getrandbits(8)))
    # SEND_ONLY at BASELINE sizes and ragged sizes, masked fields random.
    for n in [64, 256, 1024, 4096] * 3 + [44, 45, 48, 52, 60, 61, 63, 65, 100, 1500, 2048, 4100, 8192, 9000]:
        payload = bytes(rng.getrandbits(8) for _ in range(max(0, n - 44)))
        pkt = bytearray(build(0x04, b"", payload, dqpn=rng.getrandbits(24), psn=rng.getrandbits(24),
                              tos=rng.getrandbits(8), ttl=rng.getrandbits(8), csum=rng.getrandbits(16),
                              ucsum=rng.getrandbits(16), fb=rng.getrandbits(8),
                              trailer=bytes(rng.getrandbits(8) for _ in range(4))))
        if len(pkt) != n:  # odd sizes: trim / pad the payload so total_len == n
            pkt = pkt[:n] if len(pkt) > n else pkt + bytes(n - len(pkt))
            pkt[2:4] = struct.pack(">H", n)
        add(f"send_only_{n}", pkt)
    # Raw short buffers (masks beyond the end are skipped).
    for n in (4, 5, 8, 12, 33, 36, 40, 43):
        add(f"raw_{n}", bytes(rng.getrandbits(8) for _ in range(n)))

    blob = bytearray()
    index = []
    for desc, pkt in cases:
        v = O.icrc(pkt)
        assert v == O.icrc_bitwise(pkt), desc
        stamped = O.stamp(pkt)
        assert O.residue_ok(stamped), desc
        index.append({"desc": desc, "offset": len(blob), "len": len(pkt), "icrc": v,
                      "wire": struct.pack("<I", v).hex()})
        blob += pkt
    kat = O.icrc(ack)
    assert kat == 0x22791F6C, hex(kat)
    meta = {
        "generator": "tests/golden/gen_golden.py", "seed": SEED,
        "oracle": "oracle/icrc_oracle.py (zlib.crc32 over 0xFF*8 || masked L3[0,n-4)), "
                  "cross-checked bitwise + residue",
        "crc32_check_123456789": zlib.crc32(b"123456789"),
        "ack_kat": {"hex": ack[:-4].hex() + struct.pack("<I", kat).hex(), "icrc": kat},
        "cases": index,
    }
    with open(os.path.join(HERE, "icrc_golden.bin"), "wb") as f:
        f.write(blob)
    with open(os.path.join(HERE, "icrc_golden.json"), "w") as f:
        json.dump(meta, f, indent=1)
    print(f"{len(index)} vectors, {len(blob)} bytes")


if __name__ == "__main__":
    main()
