"""BASELINE configs[0]: the reference simulator's packets, per-packet ICRC on CPU.

The fixture (tests/golden/sim_stream.*) is the packet stream of the unchanged
reference python/simulator.py for seeds 1-3, captured by
tests/golden/gen_sim_stream.py with ICRCs from the oracle.  Here: the adapter
re-serialises every Packet to the same bytes, ricrc_one (ctypes) reproduces
every ICRC, the verify path accepts them, corruption is caught, and (GPU) the
whole stream as one ragged batch through the ragged kernel matches."""
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
    meta, _ = stream()
    for seed, s in meta["seeds"].items():
        assert s["stamped"] == s["verified"] == len(s["packets"]) > 1000
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


def test_wiretap_catches_corruption():
    meta, _ = stream()
    pkts = [as_packet(r["fields"]) for r in meta["seeds"]["1"]["packets"][:300]]
    tap = sim_harness.WireTap(flip_prob=0.5, rng=random.Random(3))
    with tap.installed():
        q = queue.Queue()
        for p in pkts:
            q.put(p)
        while not q.empty():
            q.get()
    assert tap.stamped == 300 and tap.corrupted > 100
    assert tap.caught == tap.corrupted and tap.verified == 300 - tap.corrupted
    assert queue.Queue is sim_harness._RealQueue


@pytest.mark.gpu
def test_sim_stream_as_ragged_gpu_batch(ctx):
    torch = pytest.importorskip("torch")
    meta, blob = stream()
    recs = [r for s in meta["seeds"].values() for r in s["packets"]]
    buf = np.frombuffer(blob, np.uint8).copy()
    offs = np.array([r["offset"] for r in recs], np.uint64)
    lens = np.array([r["len"] for r in recs], np.uint32)
    want = np.array([r["icrc"] for r in recs], np.uint32)
    out = torch.empty(len(recs), dtype=torch.int32, device="cuda")
    d = lambda a: torch.from_numpy(a).to("cuda")  # noqa: E731
    ctx.batch_device(d(buf), len(recs), out, offsets=d(offs), lengths=d(lens),
                     stream=torch.cuda.current_stream())
    torch.cuda.synchronize()
    np.testing.assert_array_equal(out.cpu().numpy().view(np.uint32), want)
    np.testing.assert_array_equal(ctx.batch_host(buf, offs, lens), want)
