#!/usr/bin/env python3
"""Framed NIC rings on one GPU, device-resident (numbers quoted in DESIGN.md).

A receive ring of `slot`-byte slots, the L3 packet at `--l3` (14: Ethernet) in
each, its length per slot from a lengths array (the completion's byte count)
or, `full`, the slot's end (no lengths array).  Slots are filled with random
bytes on the device; every ICRC of the first 64 K slots is checked against
the C oracle.  Kernel time from HIP events around `--reps` back-to-back
batches after a 100 ms warm phase; algorithmic bytes = the packets' bytes + 4
written (+ 4 read from the lengths array) per slot.  One JSON line per case.

    python tools/ring_bench.py [--count N] [--reps R] [--cases 1024:64-1010,1024:200]
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "roce-test_amd"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))

CASES = (  # (slot bytes, lengths: "full" | (lo, hi) uniform | n fixed)
    (4096, "full"), (4096, (2048, 4082)), (4096, (64, 4082)), (4096, 4082),
    (2048, "full"), (2048, 1500), (2048, (64, 2034)), (1024, (64, 1010)),
)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--count", type=int, default=1 << 20)
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--l3", type=int, default=14)
    ap.add_argument("--cases", default="",
                    help="comma-separated slot:lengths cases, lengths 'full', 'lo-hi' or n (default: CASES)")
    a = ap.parse_args()
    import numpy as np
    import torch

    import oracle_c
    import roce_icrc

    ctx = roce_icrc.Context(devices=[0])
    dev = torch.device("cuda", 0)
    s = torch.cuda.current_stream()
    rng = np.random.default_rng(0x1CEC0DE)
    cases = CASES
    if a.cases:
        cases = []
        for c in a.cases.split(","):
            slot, spec = c.split(":")
            if spec != "full":
                spec = tuple(int(x) for x in spec.split("-")) if "-" in spec else int(spec)
            cases.append((int(slot), spec))
    for slot, spec in cases:
        n_slots = a.count
        buf = torch.empty(n_slots * slot, dtype=torch.uint8, device=dev)
        ctx.synth_device(buf, 7, 0, n_slots, slot, stream=s)  # random-looking bytes in every slot
        if spec == "full":
            lens, d_len, kw = None, None, {}
            nbytes = n_slots * (slot - a.l3)
        else:
            if isinstance(spec, tuple):
                lens = rng.integers(spec[0], spec[1] + 1, size=n_slots).astype(np.uint32)
            else:
                lens = np.full(n_slots, spec, np.uint32)
            d_len = torch.from_numpy(lens.view(np.int32)).to(dev)
            kw = {"lengths": d_len}
            nbytes = int(lens.sum(dtype=np.uint64))
        out = torch.empty(n_slots, dtype=torch.int32, device=dev)
        path = roce_icrc.kernel_path(buf, n_slots, stride=slot, l3_offset=a.l3, ctx=ctx, **kw)
        run = lambda: ctx.batch_device(buf, n_slots, out, stride=slot, l3_offset=a.l3, stream=s, **kw)  # noqa: E731
        t_end = time.time() + 0.1
        while time.time() < t_end:
            run()
            torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(s)
        for _ in range(a.reps):
            run()
        e1.record(s)
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / a.reps
        k = min(n_slots, 65536)
        host = buf[:k * slot].cpu().numpy()
        want = oracle_c.icrc_batch(host, lengths=None if lens is None else lens[:k], stride=slot, count=k,
                                   l3_offset=a.l3, threads=16)
        got = out[:k].cpu().numpy().view(np.uint32)
        if not np.array_equal(got, want):
            raise SystemExit(f"slot {slot} {spec}: mismatch at {int(np.flatnonzero(got != want)[0])}")
        alg = nbytes + 4 * n_slots + (4 * n_slots if lens is not None else 0)
        print(json.dumps({"slot": slot, "lengths": spec if not isinstance(spec, tuple) else f"{spec[0]}-{spec[1]}",
                          "l3_offset": a.l3, "slots": n_slots, "kernels": path, "ms": round(ms, 4),
                          "GiB_s": round(nbytes / ms / 1e6 / 1.073741824, 1),
                          "frac": round(alg / ms / 1e9 / 8.0, 4), "checked": k}), flush=True)
        del buf, out, d_len
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
