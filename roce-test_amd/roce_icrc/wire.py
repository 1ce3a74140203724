"""RoCEv2 wire format for the reference's abstract ``Packet`` objects.

The reference's Python model (python/rdma.py:5-54) carries packets as field
bags with no byte representation, so "stamp the ICRC at the wire crossing"
(python/simulator.py:49-55, 59-82) first needs bytes.  This module is that
adapter: it serialises a ``Packet`` (duck-typed -- any object with the same
attribute names works, the reference class itself included) into an L3
RoCEv2 packet laid out per p4/common/header.p4:42-112 and
p4/shuffle/shuffle_header.p4:105-118, with the trailer left for the ICRC.

Field mapping (all multi-byte fields big-endian, as on the wire):
* opcode names -> BTH opcodes (header.p4:16-34); "READ" is READ_REQ (0x0c),
  "READ_RESPONSE" READ_RES_ONLY (0x10), "NAK" an ACK whose AETH syndrome is
  0x60 (NAK, PSN sequence error), "LOOPBACK" the shuffle REPL opcode 0x15
  (shuffle_header.p4:12) carrying repl_h + item_h entries.
* smac/dmac endpoint ids -> IPv4 192.168.1.(id+1), the switch (-1) ->
  192.168.1.100 (switchd/vswitchd.hpp:52-56, shuffle_drv.hpp:15).
* dqpn -1 / -2 (the switch's virtual request / write QPs, python/endpoint.py:
  37,50) -> vir_qp_info.req_qpn / dst_qpn (switchd/shuffle_drv.hpp:25-30).
* IPv4 template of shuffle_ingress.p4:717-724 (tos 0x02, id 0x1234, DF, ttl
  64, proto 17), BTH se/m/pad/tver 0x40 | pad<<4 and P_Key 0xffff
  (shuffle_ingress.p4:734-735), UDP sport 0x457b for switch-originated packets
  (shuffle_drv.hpp:16).
* payload ``data`` elements: int (or None) -> 4-byte word; 4-tuple
  (dmac, len, wb_off, dst_addr) -> 16-byte shuffle_request / item_h
  (common/types.h:86-91, big-endian as endpoint/shuffle_endpoint.cpp:23-26).
"""
from __future__ import annotations

import struct

# header.p4:16-34 and shuffle_header.p4:12
OPCODES = {
    "SEND_FIRST": 0x00, "SEND_MIDDLE": 0x01, "SEND_LAST": 0x02, "SEND_ONLY": 0x04,
    "WRITE_FIRST": 0x06, "WRITE_MIDDLE": 0x07, "WRITE_LAST": 0x08, "WRITE_ONLY": 0x0A,
    "READ": 0x0C, "READ_RES_FIRST": 0x0D, "READ_RES_MIDDLE": 0x0E, "READ_RES_LAST": 0x0F,
    "READ_RESPONSE": 0x10, "ACK": 0x11, "NAK": 0x11, "LOOPBACK": 0x15,
}
RETH_OPS = {0x06, 0x0A, 0x0C}              # shuffle_ingress_parser.p4:39-64
AETH_OPS = {0x0D, 0x0F, 0x10, 0x11}
ROCE_PORT = 4791                            # header.p4:14
VIR_UDP_PORT = 0x457B                       # shuffle_drv.hpp:16
VIR_REQ_QPN, VIR_DST_QPN = 0x93589, 0xD13CB  # shuffle_drv.hpp:25-30
SWITCH_IP = bytes([192, 168, 1, 100])       # vswitchd.hpp:56


def ip_of(mac: int) -> bytes:
    return SWITCH_IP if mac is None or mac < 0 else bytes([192, 168, 1, (mac + 1) & 0xFF])


def qpn_of(dqpn: int) -> int:
    if dqpn == -1:
        return VIR_REQ_QPN
    if dqpn == -2:
        return VIR_DST_QPN
    return dqpn & 0xFFFFFF


def _i(v) -> int:
    """Plain Python int of a field (the reference mixes ints and numpy scalars)."""
    return int(v) if v is not None else 0


def _element(e) -> bytes:
    if e is None:
        return b"\x00" * 4
    if isinstance(e, (tuple, list)):
        dmac, ln, wb_off, dst_addr = (_i(x) for x in e)
        return struct.pack(">HHIQ", dmac & 0xFFFF, ln & 0xFFFF, wb_off & 0xFFFFFFFF,
                           dst_addr & 0xFFFFFFFFFFFFFFFF)
    return struct.pack(">I", _i(e) & 0xFFFFFFFF)


def ipv4_checksum(hdr: bytes) -> int:
    s = sum(struct.unpack(">10H", hdr))
    while s >> 16:
        s = (s & 0xFFFF) + (s >> 16)
    return (~s) & 0xFFFF


def ip6_of(mac: int) -> bytes:
    """IPv6 address of an endpoint for the IPv6 variant: fd00::192.168.1.x
    (unique-local prefix + the IPv4 address of :func:`ip_of`)."""
    return bytes([0xFD] + [0] * 11) + ip_of(mac)


def encode(p, ipv6: bool = False, tclass: int = 0x02, flow: int = 0, hop: int = 64) -> bytearray:
    """Serialise a reference ``Packet`` into an L3 RoCEv2 packet (trailer zeroed).

    ``ipv6=True`` builds RoCEv2 over IPv6 instead (not in the IPv4-only
    reference): a 40-byte IPv6 header (version 6, ``tclass``, ``flow``,
    payload length, next header 17, ``hop``) in place of IPv4, then the same
    UDP / BTH / extension / payload bytes."""
    opname = getattr(p, "opcode", "")
    if opname not in OPCODES:
        raise ValueError(f"unknown opcode {opname!r}")
    op = OPCODES[opname]
    data = list(getattr(p, "data", []) or [])
    ext = b""
    if op == 0x15:  # REPL: repl_h {flag, item_cnt, item_id} + items
        items = b"".join(_element(e) for e in data)
        ext = struct.pack(">BBH", 0, len(data) & 0xFF, _i(getattr(p, "si", 0)) & 0xFFFF)
        payload = items
    else:
        if op in RETH_OPS:
            ext += struct.pack(">QII", _i(getattr(p, "addr", 0)) & 0xFFFFFFFFFFFFFFFF, 0,
                               _i(getattr(p, "len", 0)) & 0xFFFFFFFF)
        if op in AETH_OPS:
            syndrome = 0x60 if opname == "NAK" else 0x00
            ext += struct.pack(">I", (syndrome << 24) | (_i(getattr(p, "msn", 0)) & 0xFFFFFF))
        payload = b"".join(_element(e) for e in data)
    pad = (-len(payload)) % 4
    payload += b"\x00" * pad
    iph = 40 if ipv6 else 20
    n = iph + 8 + 12 + len(ext) + len(payload) + 4
    smac, dmac = _i(getattr(p, "smac", 0)), _i(getattr(p, "dmac", 0))
    if ipv6:
        vtf = (6 << 28) | ((tclass & 0xFF) << 20) | (flow & 0xFFFFF)
        ip = bytearray(struct.pack(">IHBB16s16s", vtf, n - 40, 17, hop & 0xFF, ip6_of(smac), ip6_of(dmac)))
    else:
        ip = bytearray(struct.pack(">BBHHHBBH4s4s", 0x45, 0x02, n, 0x1234, 0x4000, 64, 17, 0,
                                   ip_of(smac), ip_of(dmac)))
        ip[10:12] = struct.pack(">H", ipv4_checksum(bytes(ip)))
    sport = VIR_UDP_PORT if (smac is None or smac < 0) else (0xC000 | (smac & 0x3FFF))
    udp = struct.pack(">HHHH", sport, ROCE_PORT, n - iph, 0)
    psn = _i(getattr(p, "psn", 0)) & 0xFFFFFF
    ackreq = 0x80 if getattr(p, "ackreq", 0) else 0
    bth = struct.pack(">BBHI", op, 0x40 | (pad << 4), 0xFFFF, qpn_of(_i(getattr(p, "dqpn", 0)))) + \
        struct.pack(">I", (ackreq << 24) | psn)
    return bytearray(ip + udp + bth + ext + payload + b"\x00\x00\x00\x00")


def trailer(pkt) -> int:
    """The 32-bit value held in the trailer (little-endian, shuffle_egress.p4:493)."""
    return struct.unpack("<I", bytes(pkt[-4:]))[0]
