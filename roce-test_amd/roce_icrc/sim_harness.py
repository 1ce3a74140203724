"""Drop-in harness: ICRC stamping/verification around the reference simulator.

`python/simulator.py` (the reference's caller, kept unchanged) moves abstract
`Packet` objects through `queue.Queue`s.  A packet's life is: the sender puts
it on its tx queue (rdma.py:165 `QP.tx_once`, switch.py `tx_queue.put`), the
simulator's tick loop takes it off (the wire crossing, simulator.py:49-55 for
QP->switch, 59-82 for switch->QP and loopback), may lose it (simulator.py:
51-53, 61-71), and puts it on the receiver's rx queue.

`WireTap` replaces `queue.Queue` while the simulator builds its QPs/switch
and models the two NICs of that crossing with the product's per-packet entry
points (libroceicrc_cpu.so via ctypes):

* **transmit** (a packet put on a queue that is not on the wire yet): the
  packet is serialised to RoCEv2 bytes (`wire.encode`) and its ICRC stamped
  (`ricrc_stamp_one`) -- including packets the switch rewrote, which is
  exactly the stale-ICRC case the reference hides by turning NIC checking off
  (scripts/icrc/disable-icrc.sh:13,30);
* **receive** (the simulator putting a packet that is on the wire onto the
  receiver's queue): the receiving NIC checks the ICRC (`ricrc_verify_one`)
  and **drops** the packet when it fails, so it never reaches the receiver,
  and the reference's own loss recovery -- the retry timer and go-back-N
  (simulator.py:35-43, rdma.py:244-247) -- retransmits it, exactly as for
  the simulator's random loss.

Corruption injection (`flip_prob > 0`, next to the simulator's 1/101 loss):
a bit of the wire image outside the trailer is flipped after stamping; the
receiving NIC must catch and drop every such packet.
"""
from __future__ import annotations

import contextlib
import io
import queue
import random
import runpy

from . import icrc, stamp, verify, wire

_RealQueue = queue.Queue
# L3 offsets calc_icrc() forces to 0xFF (shuffle_egress.p4:467,471,473,480,485):
# a bit flip there does not change the ICRC, so the check rightly accepts it.
INVARIANT_MASKED = frozenset((1, 8, 10, 11, 26, 27, 32))


def packet_fields(p) -> list:
    """JSON-able field tuple of a reference Packet (python/rdma.py:5-37)."""
    def i(v):
        return int(v) if v is not None else None

    data = []
    for e in getattr(p, "data", []) or []:
        data.append([i(x) for x in e] if isinstance(e, tuple) else i(e))
    return [p.opcode] + [i(getattr(p, f)) for f in ("smac", "dmac", "psn", "dqpn", "ackreq", "addr", "len",
                                                       "msn", "si")] + [data]


def _is_packet(item) -> bool:
    return hasattr(item, "opcode") and hasattr(item, "dqpn")  # a Packet, not a WR on a CQ


class WireTap:
    def __init__(self, flip_prob: float = 0.0, rng: random.Random | None = None, record: bool = True,
                 flip_at=()):
        self.flip_prob = flip_prob
        self.flip_at = frozenset(flip_at)  # transmission numbers (0-based) to corrupt deterministically
        self.rng = rng or random.Random(0)
        self.record = record
        self.records = []        # (event, fields, wire hex, icrc) per transmission
        self.stamped = 0         # transmissions (ICRC stamped by the sending NIC)
        self.verified = 0        # arrivals that passed the receiving NIC's check
        self.corrupted = 0       # transmissions with an injected bit flip
        self.caught = 0          # corrupted arrivals the check rejected
        self.dropped = 0         # arrivals dropped by the check (== caught unless a clean packet failed)
        self.benign = 0          # corrupted arrivals accepted: the flip hit an invariant-masked field
        self.missed = 0          # corrupted arrivals accepted although a covered byte flipped (must stay 0)

    def _transmit(self, item):
        raw = stamp(wire.encode(item))
        k = self.stamped
        self.stamped += 1
        if self.record:
            self.records.append(("tx", packet_fields(item), raw.hex(), icrc(raw)))
        item._icrc_corrupt = False
        if k in self.flip_at or (self.flip_prob and self.rng.random() < self.flip_prob):
            pos = self.rng.randrange(40, len(raw) - 4) if k in self.flip_at else self.rng.randrange(0, len(raw) - 4)
            raw[pos] ^= 1 << self.rng.randrange(8)
            item._icrc_corrupt = True
            item._flip_pos = pos
            self.corrupted += 1
        item._wire = raw
        item._on_wire = True

    def _receive(self, item) -> bool:
        """The receiving NIC's check; False = drop."""
        item._on_wire = False
        ok = verify(item._wire)
        if item._icrc_corrupt:
            # A flip can hit an invariant-masked field (tos, ttl, checksums,
            # FECN/BECN): the ICRC does not cover those, so the packet is
            # still valid as far as the check goes.
            if not ok:
                self.caught += 1
            elif item._flip_pos in INVARIANT_MASKED:
                self.benign += 1
            else:
                self.missed += 1
            item._icrc_corrupt = False
        if not ok:
            self.dropped += 1
            return False
        self.verified += 1
        return True

    def _queue_class(self):
        tap = self

        class NicQueue(_RealQueue):
            def put(self, item, *a, **k):
                if _is_packet(item):
                    if getattr(item, "_on_wire", False):
                        if not tap._receive(item):
                            return  # dropped by the receiving NIC: the sender's retry recovers it
                    else:
                        tap._transmit(item)
                super().put(item, *a, **k)

        return NicQueue

    @contextlib.contextmanager
    def installed(self):
        queue.Queue = self._queue_class()
        try:
            yield self
        finally:
            queue.Queue = _RealQueue


def run_simulator(simulator_py: str, seed: int, tap: WireTap | None = None) -> tuple:
    """Run the reference simulator as __main__ with a fixed seed under a tap.
    Returns (tap, captured stdout) -- the prints are the reference's own
    tracing (retries, losses) and its end-state report."""
    tap = tap or WireTap()
    random.seed(seed)
    buf = io.StringIO()
    with tap.installed(), contextlib.redirect_stdout(buf):
        runpy.run_path(simulator_py, run_name="__main__")
    return tap, buf.getvalue()
