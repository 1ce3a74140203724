"""CPU oracle for the RoCEv2 Invariant CRC (ICRC) -- TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import
this module, and only as a checker.  The product path (libroceicrc + HIP
kernels) never routes through it.

Parity status: the reference's own tests pin nothing at this boundary (it has
no tests and its only ICRC is a disabled Tofino action), so the oracle is a
spec restatement cross-checked three ways (zlib.crc32, a bitwise CRC-32, the
CRC-32 residue) plus build-derived golden vectors and one hand-derived
known-answer packet built from the reference's P4 header templates.
-> "parity unpinned" in the sense of the task contract; see DESIGN.md §Oracle.

Spec followed (all citations relative to the reference root):

* ``p4/shuffle/shuffle_egress.p4:461``  ``Hash<bit<32>>(HashAlgorithm_t.CRC32)``:
  CRC-32/IEEE, reflected poly 0xEDB88320, init 0xFFFFFFFF, xorout 0xFFFFFFFF
  (Tofino's CRC32 preset; the SDE is not vendored -> restated, = zlib.crc32).
* ``shuffle_egress.p4:465`` the 64-bit 0xFF..FF prefix (the masked LRH/GRH
  stand-in of IBTA Annex A17 for RoCEv2).
* ``shuffle_egress.p4:466-475`` IPv4: ver_ihl kept, diffserv -> 0xFF (:467),
  total_len/id/flags kept, ttl -> 0xFF (:471), protocol kept, hdr_checksum ->
  0xFFFF (:473), src/dst kept.
* ``shuffle_egress.p4:477-480`` UDP: ports/length kept, checksum -> 0xFFFF.
* ``shuffle_egress.p4:482-487`` BTH: opcode, se/m/pad/tver, pkey kept,
  FECN/BECN/resv byte -> 0xFF (:485), dqpn and ackreq/psn kept.
* ``shuffle_egress.p4:489-490`` the AETH (syndrome, MSN), unmasked.  That is
  where the reference's field list ENDS: calc_icrc() is written for the
  switch-generated write ACKs only (its one call site, :669, commented out),
  whose L3 packet is IPv4 ‖ UDP ‖ BTH ‖ AETH ‖ ICRC (48 bytes,
  shuffle_ingress.p4:539,550).  DELIBERATE GENERALISATION: for any other
  packet this oracle covers every byte after BTH up to the trailer
  (extension headers, payload, pad), unmasked -- IBTA Annex A17's ICRC,
  which the Linux rxe driver computes the same way and which NICs check.
  For the reference's ACK shape both definitions are the same bytes
  (tests/test_oracle.py::test_ack_matches_calc_icrc_field_list).
* ``shuffle_egress.p4:493`` the 32-bit value is emitted byte-swapped, i.e. the
  trailer holds the CRC little-endian.
* Header layout offsets: ``p4/common/header.p4:42-53`` (ipv4_h, 20 B),
  ``:67-72`` (udp_h, 8 B), ``:75-85`` (bth_h, 12 B).
"""
from __future__ import annotations

import struct
import zlib

import numpy as np

# L3 byte offsets forced to 0xFF before the CRC (shuffle_egress.p4:467,471,473,480,485)
MASK_OFFSETS = (1, 8, 10, 11, 26, 27, 32)
# RoCEv2 over IPv6 -- not in the IPv4-only reference (header.p4:42-53).  Spec:
# IBTA Annex A17 ICRC invariant fields, as the Linux rxe driver applies them
# (drivers/infiniband/sw/rxe/rxe_icrc.c: ip6h->priority = 0xf (byte 0 low
# nibble), ip6h->flow_lbl[0..2] = 0xff (bytes 1-3), ip6h->hop_limit = 0xff
# (byte 7), udph->check = 0xffff (bytes 40+6, 40+7), bth->qpn |= ~QPN_MASK
# (BTH byte 4 at 48+4)).  OR-values per L3 offset.
MASKS_V6 = ((0, 0x0F), (1, 0xFF), (2, 0xFF), (3, 0xFF), (7, 0xFF), (46, 0xFF), (47, 0xFF), (52, 0xFF))
MASKS_V4 = tuple((o, 0xFF) for o in MASK_OFFSETS)
PREFIX = b"\xff" * 8                      # shuffle_egress.p4:465
POLY_REFLECTED = 0xEDB88320
CRC32_RESIDUE = 0x2144DF1C                # crc32(msg || LE32(crc32(msg))), any msg
REGISTER_AFTER_PREFIX = 0xDEBB20E3        # ~crc32(8*0xFF): the rxe seed
ROCE_UDP_PORT = 4791                      # header.p4:14
MIN_PKT = 20 + 8 + 12 + 4                 # IPv4 + UDP + BTH + ICRC


def family_of(l3: bytes, family: str = "v4") -> str:
    """'v4' / 'v6', or for 'auto' the IP version nibble (6 -> 'v6', else 'v4')."""
    if family == "auto":
        return "v6" if len(l3) and (l3[0] >> 4) == 6 else "v4"
    if family not in ("v4", "v6"):
        raise ValueError(family)
    return family


def masked_body(l3: bytes, family: str = "v4") -> bytes:
    """The L3 bytes the ICRC covers, [0, n-4), with the invariant masks applied."""
    n = len(l3)
    if n < 4:
        raise ValueError("packet shorter than the ICRC trailer")
    b = bytearray(l3[: n - 4])
    for o, v in (MASKS_V6 if family_of(l3, family) == "v6" else MASKS_V4):
        if o < len(b):
            b[o] |= v
    return bytes(b)


def icrc(l3: bytes, family: str = "v4") -> int:
    """ICRC value of one L3 RoCEv2 packet (trailer bytes = LE32 of the result).

    Restates calc_icrc() (shuffle_egress.p4:463-494) with zlib's CRC-32, which
    is the same parameter set as Tofino's HashAlgorithm_t.CRC32.
    """
    return zlib.crc32(PREFIX + masked_body(l3, family)) & 0xFFFFFFFF


_BIT_TABLE = None


def _crc32_bitwise(data: bytes, crc: int = 0xFFFFFFFF) -> int:
    """Independent bit-at-a-time reflected CRC-32 register update (no table)."""
    for byte in data:
        crc ^= byte
        for _ in range(8):
            crc = (crc >> 1) ^ (POLY_REFLECTED if crc & 1 else 0)
    return crc


def icrc_bitwise(l3: bytes, family: str = "v4") -> int:
    """Second, table-free formulation used to cross-check :func:`icrc`."""
    return _crc32_bitwise(PREFIX + masked_body(l3, family)) ^ 0xFFFFFFFF


def icrc_rxe(l3: bytes, family: str = "v4") -> int:
    """Third formulation: Linux-rxe style seed 0xDEBB20E3 at IP byte 0."""
    return _crc32_bitwise(masked_body(l3, family), REGISTER_AFTER_PREFIX) ^ 0xFFFFFFFF


def residue_ok(l3: bytes, family: str = "v4") -> bool:
    """CRC-32 over prefix||masked||trailer equals the CRC-32 residue 0x2144DF1C
    (register 0xDEBB20E3 before xorout) iff the trailer (little-endian,
    shuffle_egress.p4:493) holds the right ICRC."""
    return (zlib.crc32(PREFIX + masked_body(l3, family) + bytes(l3[-4:])) & 0xFFFFFFFF) == CRC32_RESIDUE


def stamp(l3: bytes, family: str = "v4") -> bytes:
    """Return ``l3`` with its trailer replaced by the correct ICRC (LE32)."""
    return bytes(l3[:-4]) + struct.pack("<I", icrc(l3, family))


def icrc_batch(buf: np.ndarray, offsets=None, lengths=None, stride: int = 0,
               count: int | None = None, l3_offset: int = 0, family: str = "v4") -> np.ndarray:
    """Per-packet loop over a packed batch (same addressing as ricrc_batch_*)."""
    mv = memoryview(np.ascontiguousarray(buf).reshape(-1).view(np.uint8))
    if count is None:
        count = len(offsets) if offsets is not None else len(mv) // stride
    out = np.empty(count, dtype=np.uint32)
    for i in range(count):
        o = int(offsets[i]) if offsets is not None else i * stride
        n = int(lengths[i]) if lengths is not None else stride - l3_offset
        s = o + l3_offset
        out[i] = icrc(mv[s: s + n].tobytes(), family)
    return out


# --------------------------------------------------------------------------
# GF(2) helpers (reflected representation: bit 31 = x^0) used by tests to
# check the product's combine/shift helpers independently of the product.
# --------------------------------------------------------------------------
def gf_mul(a: int, b: int) -> int:
    p = 0
    for i in range(31, -1, -1):
        if (a >> i) & 1:
            p ^= b
        b = (b >> 1) ^ (POLY_REFLECTED if b & 1 else 0)
    return p


def crc_shift(reg: int, nbytes: int) -> int:
    """Register advanced over ``nbytes`` zero bytes (brute force)."""
    for _ in range(nbytes):
        for _ in range(8):
            reg = (reg >> 1) ^ (POLY_REFLECTED if reg & 1 else 0)
    return reg


# --------------------------------------------------------------------------
# RoCEv2 classification: the ingress parser's accept path
# (p4/shuffle/shuffle_ingress_parser.p4:12-36) -- Ethernet ether_type
# ETHERTYPE_IPV4 0x0800 (header.p4:8) -> parse_ipv4 -> protocol
# IP_PROTOCOLS_UDP 17 (header.p4:11) -> parse_udp -> dst_port UDP_PORT_ROCE
# 4791 (header.p4:14) -> parse_bth.  Every other frame falls through to
# `accept` without a BTH: not RoCE, no ICRC.  The ipv4_h of header.p4:42-53
# has no options (IHL 5), and the packet is the IPv4 datagram (total_len = n).
# IPv6 (not in the reference): IBTA Annex A17's RoCEv2 over IPv6 -- version 6,
# next header 17, payload length n - 40, UDP dst_port 4791.
# --------------------------------------------------------------------------
ETHERTYPE_IPV4 = 0x0800                   # header.p4:8
ETHERTYPE_IPV6 = 0x86DD
IP_PROTOCOLS_UDP = 17                     # header.p4:11
MAX_PKT = 65535                           # IPv4 total_len is 16 bits (header.p4:45)


def classify(l3: bytes, ethertype: int | None = None) -> int:
    """4 (RoCEv2 over IPv4), 6 (over IPv6) or 0.  ``ethertype``: the frame's
    EtherType when the packet came in an Ethernet frame (it must be the
    family's), None for a bare L3 packet."""
    n = len(l3)
    if n < MIN_PKT or n > MAX_PKT:
        return 0
    be16 = lambda o: (l3[o] << 8) | l3[o + 1]  # noqa: E731
    c = 0
    if l3[0] == 0x45 and l3[9] == IP_PROTOCOLS_UDP and be16(2) == n and be16(22) == ROCE_UDP_PORT:
        c = 4
    elif (l3[0] >> 4) == 6 and n >= 40 + 8 + 12 + 4 and l3[6] == IP_PROTOCOLS_UDP and be16(4) == n - 40 \
            and be16(42) == ROCE_UDP_PORT:
        c = 6
    if c and ethertype is not None and ethertype != (ETHERTYPE_IPV4 if c == 4 else ETHERTYPE_IPV6):
        c = 0
    return c


ST_OK, ST_BADLEN, ST_NOTROCE = 0, 1, 2


def frame_l3_len(frame: bytes) -> int:
    """RICRC_F_FRAMELEN: the L3 length of a packet given the bytes from its L3
    header to the end of its frame, which on an Ethernet NIC ring may carry
    minimum-frame padding and the FCS after the datagram.  The reference's
    parser keys only on EtherType / protocol / dport
    (shuffle_ingress_parser.p4:12-36) and never uses a descriptor length; the
    datagram's own extent is ipv4_h.total_len (header.p4:45), or, for IPv6,
    payload length + 40.  That length is taken whenever it lies in
    [MIN_PKT, len(frame)]; otherwise the frame length stands (and a strict
    classification then rejects the packet).  A frame extent outside
    [MIN_PKT, MAX_PKT] is a bad length whatever its header says."""
    n = len(frame)
    if n < MIN_PKT or n > MAX_PKT:
        return n
    v = frame[0] >> 4
    t = ((frame[2] << 8) | frame[3]) if v == 4 else (((frame[4] << 8) | frame[5]) + 40 if v == 6 else 0)
    return t if MIN_PKT <= t <= n else n


def status_batch(buf: np.ndarray, offsets=None, lengths=None, stride: int = 0, count: int | None = None,
                 l3_offset: int = 0, family: str = "v4", strict: bool = False, verify: bool = False,
                 framelen: bool = False):
    """(out, status) of ricrc_batch_*_st on a packed batch: per packet
    ST_BADLEN for a length outside [MIN_PKT, MAX_PKT], ST_NOTROCE under
    ``strict`` for a packet :func:`classify` rejects (EtherType checked when
    l3_offset >= 14) or of a family not asked for, else ST_OK with the ICRC
    (``verify``: 1/0 trailer check); out = 0 where status != ST_OK.
    ``framelen`` (RICRC_F_FRAMELEN): the descriptor length is the frame's
    extent past L3 and the packet's is :func:`frame_l3_len` of it."""
    mv = memoryview(np.ascontiguousarray(buf).reshape(-1).view(np.uint8))
    if count is None:
        count = len(offsets) if offsets is not None else len(mv) // stride
    out = np.zeros(count, dtype=np.uint32)
    st = np.zeros(count, dtype=np.uint8)
    accept = {"v4": (4,), "v6": (6,), "auto": (4, 6)}[family]
    for i in range(count):
        o = int(offsets[i]) if offsets is not None else i * stride
        n = int(lengths[i]) if lengths is not None else stride - l3_offset
        if framelen and MIN_PKT <= n <= MAX_PKT:
            n = frame_l3_len(mv[o + l3_offset: o + l3_offset + n].tobytes())
        if n < MIN_PKT or n > MAX_PKT:
            st[i] = ST_BADLEN
            continue
        s = o + l3_offset
        pkt = mv[s: s + n].tobytes()
        if strict:
            et = (mv[s - 2] << 8 | mv[s - 1]) if l3_offset >= 14 else None
            if classify(pkt, et) not in accept:
                st[i] = ST_NOTROCE
                continue
        v = icrc(pkt, family)
        out[i] = (1 if struct.unpack("<I", pkt[-4:])[0] == v else 0) if verify else v
    return out, st
