#!/usr/bin/env python3
"""Incremental repair vs full recompute on one GPU (numbers quoted in DESIGN.md).

The switch egress's PSN patch (shuffle_egress.p4:635-671) on device-resident
batches: every packet's BTH PSN (L3 bytes 37..39) rewritten, then either
ricrc_repair_device (old bytes + old trailer -> new ICRC, stamped in place)
or ricrc_batch_device over the whole packet.  HIP-event kernel time on the
stream both kernels run on; each measured repair is checked against the full
recompute (device) and a sample against the C oracle.  One JSON line per case.

    python tools/repair_bench.py [--quick]
"""
from __future__ import annotations

import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "roce-test_amd"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--quick", action="store_true")
    ap.add_argument("--reps", type=int, default=50)
    args = ap.parse_args()
    import numpy as np
    import torch

    import oracle_c
    import roce_icrc

    ctx = roce_icrc.Context(devices=[0])
    s = torch.cuda.current_stream()
    cases = [(1 << 20, 64), (1 << 20, 1024), (1 << 20, 4096)]
    if args.quick:
        cases = [(1 << 16, 4096)]
    off, ln = 37, 3
    for count, n in cases:
        buf = torch.empty(count * n, dtype=torch.uint8, device="cuda")
        ctx.synth_device(buf, 0x1CEC0DE, 0, count, n, stream=s)
        icrc = torch.empty(count, dtype=torch.int32, device="cuda")
        ctx.batch_device(buf, count, icrc, stride=n, stream=s)
        rows = buf.view(count, n)
        rows[:, n - 4:] = icrc.view(torch.uint8).view(count, 4)
        old = rows[:, off:off + ln].clone()
        g = torch.Generator(device="cuda").manual_seed(7)
        rows[:, off:off + ln] = torch.randint(0, 256, (count, ln), dtype=torch.uint8, device="cuda", generator=g)
        stamped = rows[:, n - 4:].clone()
        rep = torch.empty(count, dtype=torch.int32, device="cuda")
        full = torch.empty(count, dtype=torch.int32, device="cuda")

        def run_repair():
            ctx.repair_device(buf, count, off, old, out=rep, stride=n, stamp=True, stream=s)

        def run_repair_out():
            ctx.repair_device(buf, count, off, old, out=rep, stride=n, stamp=False, stream=s)

        def run_full():
            ctx.batch_device(buf, count, full, stride=n, stream=s)

        res = {}
        for name, fn in (("repair_out", run_repair_out), ("repair", run_repair), ("recompute", run_full)):
            times = []
            for r in range(args.reps + 10):
                if name == "repair":
                    rows[:, n - 4:] = stamped  # the old trailers again (repair is not idempotent)
                a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                a.record(s)
                fn()
                b.record(s)
                if r >= 10:
                    times.append((a, b))
            torch.cuda.synchronize()
            res[name] = sorted(x.elapsed_time(y) for x, y in times)[len(times) // 2]
        torch.cuda.synchronize()
        if not torch.equal(rep, full):
            raise SystemExit(f"{count} x {n}: repair != recompute")
        host = rows[:512].cpu().numpy()
        if not np.array_equal(rep[:512].cpu().numpy().view(np.uint32), oracle_c.icrc_batch(host, stride=n)):
            raise SystemExit(f"{count} x {n}: repair != oracle")
        alg = count * (2 * ln + 4 + 4 + 4)  # new + old range bytes, old trailer, new trailer, out
        print(json.dumps({
            "case": f"{count} x {n} B, PSN rewrite (L3 bytes {off}..{off + ln - 1})",
            "repair_ms": round(res["repair"], 4), "repair_no_stamp_ms": round(res["repair_out"], 4), "recompute_ms": round(res["recompute"], 4),
            "speedup": round(res["recompute"] / res["repair"], 2),
            "repair_Mpkt_s": round(count / res["repair"] / 1e3, 1),
            "repair_alg_GBps": round(alg / res["repair"] / 1e6, 1),
            "bit_exact": True}), flush=True)
    # IPv6 family on the batch path: the IPv4-mask kernel + the header fix-up pass.
    count, n = (1 << 16, 4096) if args.quick else (1 << 20, 4096)
    buf = torch.empty(count * n, dtype=torch.uint8, device="cuda")
    ctx.synth_device(buf, 0x1CEC0DE, 0, count, n, stream=s)
    buf.view(count, n)[:, 0] = 0x60
    out = torch.empty(count, dtype=torch.int32, device="cuda")
    res = {}
    for fam in ("v4", "v6", "auto"):
        times = []
        for r in range(args.reps + 10):
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record(s)
            ctx.batch_device(buf, count, out, stride=n, stream=s, family=fam)
            b.record(s)
            if r >= 10:
                times.append((a, b))
        torch.cuda.synchronize()
        res[fam] = sorted(x.elapsed_time(y) for x, y in times)[len(times) // 2]
        host = buf.view(count, n)[:512].cpu().numpy()
        if not np.array_equal(out[:512].cpu().numpy().view(np.uint32),
                              oracle_c.icrc_batch(host, stride=n, family=fam)):
            raise SystemExit(f"family {fam}: mismatch vs oracle")
    print(json.dumps({
        "case": f"{count} x {n} B IPv6 packets, batch ICRC by family",
        "v4_masks_ms": round(res["v4"], 4), "v6_ms": round(res["v6"], 4), "auto_ms": round(res["auto"], 4),
        "v6_GiBps": round(count * n / res["v6"] / 1e-3 / 2**30, 1),
        "v6_overhead": round(res["v6"] / res["v4"] - 1, 3), "bit_exact_sample": True}), flush=True)
    ctx.close()


if __name__ == "__main__":
    main()
