"""BASELINE configs[0]: the reference simulator's packets, per-packet ICRC on CPU.

The fixture (tests/golden/sim_stream.*) is the packet stream of the unchanged
reference python/simulator.py for seeds 1-3, captured by
tests/golden/gen_sim_stream.py with ICRCs from the oracle.  Here: the adapter
re-serialises every Packet to the same bytes, ricrc_one (ctypes) reproduces
every ICRC, the verify path accepts them and corruption is caught.  The GPU
replay of the same fixture -- the whole stream as one ragged batch through the
HIP kernels, host path, verify and status modes, against the ICRCs stored in
the fixture -- is tests/test_gpu_fixtures.py."""
import json
import os
import queue
import random
import types

import numpy as np
import pytest

import roce_icrc
from roce_icrc import sim_harness, wire

HERE = os.path.join(os.path.dirname(__file__), "golden")


def stream():
    meta = json.load(open(os.path.join(HERE, "sim_stream.json")))
    blob = open(os.path.join(HERE, "sim_stream.bin"), "rb").read()
    return meta, blob


def as_packet(fields):
    keys = ("opcode", "smac", "dmac", "psn", "dqpn", "ackreq", "addr", "len", "msn", "si", "data")
    p = types.SimpleNamespace(**dict(zip(keys, fields)))
    p.data = [tuple(e) if isinstance(e, list) else e for e in p.data]
    return p


def test_stream_fixture_sizes():
    """One record per transmission; every transmitted packet either arrived and
    passed the receiving NIC's check or was lost by the simulator's own loss
    model (simulator.py:51-53, 61-71) -- no ICRC failures without injection."""
    meta, _ = stream()
    for seed, s in meta["seeds"].items():
        assert s["stamped"] == len(s["packets"]) > 600
        assert s["verified"] + s["lost_by_simulator"] == s["stamped"] and 0 < s["lost_by_simulator"] < 20
        ops = {p["fields"][0] for p in s["packets"]}
        assert {"WRITE_FIRST", "LOOPBACK", "READ", "READ_RESPONSE", "WRITE_ONLY", "ACK"} <= ops


def test_adapter_and_per_packet_icrc_match_fixture():
    meta, blob = stream()
    for s in meta["seeds"].values():
        for rec in s["packets"]:
            raw = blob[rec["offset"]: rec["offset"] + rec["len"]]
            enc = wire.encode(as_packet(rec["fields"]))
            assert bytes(enc[:-4]) == raw[:-4], rec["fields"][:2]
            assert roce_icrc.icrc(raw) == rec["icrc"]
            assert wire.trailer(raw) == rec["icrc"]
            assert roce_icrc.verify(raw)
            assert roce_icrc.is_rocev2(raw)


def test_wiretap_drops_corrupted_packets():
    """Replay the fixture's packets across one tapped wire crossing (tx queue ->
    get -> rx queue put, as simulator.py:49-55 does) with bit flips: every flip
    of a covered byte is caught and the packet never reaches the receiver."""
    meta, _ = stream()
    pkts = [as_packet(r["fields"]) for r in meta["seeds"]["1"]["packets"][:300]]
    tap = sim_harness.WireTap(flip_prob=0.5, rng=random.Random(3))
    with tap.installed():
        tx, rx = queue.Queue(), queue.Queue()
        for p in pkts:
            tx.put(p)
        while not tx.empty():
            rx.put(tx.get())
        arrived = rx.qsize()
    assert tap.stamped == 300 and tap.corrupted > 100
    assert tap.missed == 0 and tap.caught + tap.benign == tap.corrupted and tap.caught > 100
    assert tap.dropped == tap.caught and arrived == tap.verified == 300 - tap.caught
    assert queue.Queue is sim_harness._RealQueue


REF_SIM = "/root/reference/python/simulator.py"


@pytest.mark.skipif(not os.path.exists(REF_SIM), reason="the reference is only present in the build container")
@pytest.mark.parametrize("seed,at", [(1, 20), (1, 100), (1, 200), (7, 50), (7, 150)])
def test_reference_simulator_recovers_from_icrc_drops(seed, at):
    """The unchanged reference simulator under the tap, one packet corrupted on
    the wire (transmission number `at`): the receiving NIC drops it, the
    simulator's own retry / go-back-N (simulator.py:35-43, rdma.py:244-247)
    retransmits -- one more retry than the clean run of the same seed -- and
    its end-state check (simulator.py:151-161) passes.  (The reference allows
    5 retries per work request for ALL losses of a run, its own random ones
    included (simulator.py:41-43), so one injected drop per run is what
    every seed survives; seeds 1 and 7 have 3 retries of their own.)"""
    import sys

    sys.path.insert(0, os.path.dirname(REF_SIM))
    _, clean = sim_harness.run_simulator(REF_SIM, seed, sim_harness.WireTap(record=False))
    tap = sim_harness.WireTap(record=False, flip_at=[at], rng=random.Random(seed))
    tap, log = sim_harness.run_simulator(REF_SIM, seed, tap)
    for text in (clean, log):
        assert "Wrong result" not in text and "Too many retries" not in text and "Traceback" not in text
    assert tap.corrupted == tap.caught == tap.dropped == 1 and tap.missed == 0
    assert log.count("Retry (") >= clean.count("Retry (")
    assert "Endpoint 0" in log  # the end-state report ran after simulate() returned
