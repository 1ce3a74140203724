"""Drop-in harness: ICRC stamping/verification around the reference simulator.

`python/simulator.py` (the reference's caller, kept unchanged) moves abstract
`Packet` objects through `queue.Queue`s at its two wire crossings
(simulator.py:49-55 QP->switch, 59-82 switch->QP/loopback).  `WireTap`
replaces `queue.Queue` while the simulator builds its QPs/switch, so every
packet put on a queue is serialised to RoCEv2 bytes (`wire.encode`) and
stamped with its ICRC (`ricrc_one` via ctypes), and every packet taken off a
queue is checked the way a receiving NIC checks it (`ricrc_verify_one`) --
the check the reference disables with scripts/icrc/disable-icrc.sh.

Optional corruption injection (next to the simulator's own 1/101 loss,
simulator.py:51,61): with `flip_prob > 0` a bit of the wire image is flipped
after stamping and the receiver's verify must catch it.
"""
from __future__ import annotations

import contextlib
import io
import queue
import random
import runpy

from . import icrc, stamp, verify, wire

_RealQueue = queue.Queue


def packet_fields(p) -> list:
    """JSON-able field tuple of a reference Packet (python/rdma.py:5-37)."""
    def i(v):
        return int(v) if v is not None else None

    data = []
    for e in getattr(p, "data", []) or []:
        data.append([i(x) for x in e] if isinstance(e, tuple) else i(e))
    return [p.opcode] + [i(getattr(p, f)) for f in ("smac", "dmac", "psn", "dqpn", "ackreq", "addr", "len",
                                                       "msn", "si")] + [data]


class WireTap:
    def __init__(self, flip_prob: float = 0.0, rng: random.Random | None = None, record: bool = True):
        self.flip_prob = flip_prob
        self.rng = rng or random.Random(0)
        self.record = record
        self.records = []        # (event, fields, wire hex, icrc)
        self.stamped = 0
        self.verified = 0
        self.corrupted = 0
        self.caught = 0

    def _queue_class(self):
        tap = self

        class StampingQueue(_RealQueue):
            def put(self, item, *a, **k):
                if hasattr(item, "opcode") and hasattr(item, "dqpn"):  # a Packet, not a WR on a CQ
                    raw = stamp(wire.encode(item))
                    tap.stamped += 1
                    if tap.record:
                        tap.records.append(("tx", packet_fields(item), raw.hex(), icrc(raw)))
                    if tap.flip_prob and tap.rng.random() < tap.flip_prob:
                        pos = tap.rng.randrange(40, len(raw) - 4) if len(raw) > 44 else 0
                        raw[pos] ^= 1 << tap.rng.randrange(8)
                        item._icrc_corrupt = True
                        tap.corrupted += 1
                    item._wire = raw
                super().put(item, *a, **k)

            def get(self, *a, **k):
                item = super().get(*a, **k)
                raw = getattr(item, "_wire", None)
                if raw is not None:
                    ok = verify(raw)
                    if getattr(item, "_icrc_corrupt", False):
                        assert not ok, "corrupted packet passed the ICRC check"
                        tap.caught += 1
                        item._icrc_corrupt = False
                        item._wire = stamp(wire.encode(item))  # retransmitted clean
                    else:
                        assert ok, "ICRC mismatch on a clean packet"
                        tap.verified += 1
                return item

        return StampingQueue

    @contextlib.contextmanager
    def installed(self):
        queue.Queue = self._queue_class()
        try:
            yield self
        finally:
            queue.Queue = _RealQueue


def run_simulator(simulator_py: str, seed: int, tap: WireTap | None = None) -> WireTap:
    """Run the reference simulator as __main__ with a fixed seed under a tap.
    Its prints are captured (they are the reference's own tracing)."""
    tap = tap or WireTap()
    random.seed(seed)
    with tap.installed(), contextlib.redirect_stdout(io.StringIO()):
        runpy.run_path(simulator_py, run_name="__main__")
    return tap
