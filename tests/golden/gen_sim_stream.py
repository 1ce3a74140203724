#!/usr/bin/env python3
"""Capture the reference simulator's packet stream as a fixture (run HERE only).

Runs the reference's unchanged python/simulator.py (BASELINE configs[0]:
per-packet ICRC on the CPU at the simulator's wire crossings) under
roce_icrc.sim_harness.WireTap for fixed seeds, and records for every packet
transmission (a packet put on a tx queue: the sending NIC) its Packet fields (python/rdma.py:5-37), the RoCEv2 bytes the
adapter produced (roce_icrc.wire) with the ICRC stamped, and the ICRC as
computed by the ORACLE (not the product).  The reference itself never leaves
this container: tests and the GPU box only read the JSON/BIN written here.

    python tests/golden/gen_sim_stream.py /root/reference/python
"""
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path[:0] = [os.path.join(ROOT, "roce-test_amd"), os.path.join(ROOT, "oracle")]

import icrc_oracle as O  # noqa: E402
from roce_icrc import sim_harness  # noqa: E402

SEEDS = (1, 2, 3)


def main(refpy):
    sys.path.insert(0, refpy)
    sim = os.path.join(refpy, "simulator.py")
    out = {"generator": "tests/golden/gen_sim_stream.py", "simulator": "python/simulator.py (unchanged)",
           "seeds": {}}
    blob = bytearray()
    for seed in SEEDS:
        tap, log = sim_harness.run_simulator(sim, seed)
        assert "Wrong result" not in log and "Too many retries" not in log
        recs = []
        for ev, fields, wire_hex, v in tap.records:
            raw = bytes.fromhex(wire_hex)
            assert O.icrc(raw) == v and O.residue_ok(raw), fields
            recs.append({"fields": fields, "offset": len(blob), "len": len(raw), "icrc": v})
            blob += raw
        out["seeds"][str(seed)] = {"stamped": tap.stamped, "verified": tap.verified,
                                   "lost_by_simulator": tap.stamped - tap.verified - tap.dropped, "packets": recs}
        print(f"seed {seed}: {tap.stamped} packets stamped, {tap.verified} verified")
    with open(os.path.join(HERE, "sim_stream.bin"), "wb") as f:
        f.write(blob)
    with open(os.path.join(HERE, "sim_stream.json"), "w") as f:
        json.dump(out, f, separators=(",", ":"))


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "/root/reference/python")
