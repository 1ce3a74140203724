#!/usr/bin/env python3
"""BASELINE configs[0] / north_star "reference path timed": the reference's
python/simulator.py (unchanged) per run, alone and under the WireTap harness
that stamps and verifies the ICRC of every packet at its wire crossings with
libroceicrc_cpu.so (ricrc_stamp_one / ricrc_verify_one via ctypes).

The reference never leaves the build container, so this runs HERE only; the
result is committed as profiles/r02/sim_plumbing.json and quoted in DESIGN.md
labelled "container".

    python tools/sim_plumbing.py [/root/reference/python] > profiles/r02/sim_plumbing.json
"""
import contextlib
import io
import json
import os
import platform
import random
import runpy
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "roce-test_amd"))

from roce_icrc import sim_harness  # noqa: E402


def cpu_model():
    with open("/proc/cpuinfo") as f:
        for line in f:
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    return platform.processor()


def main(refpy):
    sys.path.insert(0, refpy)
    sim = os.path.join(refpy, "simulator.py")
    seeds = list(range(1, 11))
    plain, tapped, pkts = [], [], []
    for s in seeds:
        random.seed(s)
        t0 = time.perf_counter()
        with contextlib.redirect_stdout(io.StringIO()):
            runpy.run_path(sim, run_name="__main__")
        plain.append(time.perf_counter() - t0)
        t0 = time.perf_counter()
        tap, _ = sim_harness.run_simulator(sim, s, sim_harness.WireTap(record=False))
        tapped.append(time.perf_counter() - t0)
        pkts.append(tap.stamped)
    mp, mt = sum(plain) / len(plain), sum(tapped) / len(tapped)
    n = sum(pkts) / len(pkts)
    print(json.dumps({
        "where": "build container (the reference does not travel to the GPU box)",
        "cpu_model": cpu_model(), "cores_used": 1, "seeds": seeds,
        "simulator_ms_per_run": round(mp * 1e3, 2),
        "simulator_with_icrc_ms_per_run": round(mt * 1e3, 2),
        "packets_per_run": round(n, 1),
        "icrc_overhead_us_per_packet": round((mt - mp) / n * 1e6, 2),
        "note": "overhead per transmitted packet = wire.encode + ricrc_stamp_one at the sender + "
                "ricrc_verify_one at the receiver (Python adapter included)",
    }))


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "/root/reference/python")
