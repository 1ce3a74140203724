#!/usr/bin/env python3
"""Per-launch fixed cost of the fixed-size kernels: HIP-event time of one
ricrc_batch_device launch over batches of 2^k packets of one size, after
ricrc_prime and a warmup; prints a JSON line per size and the least-squares
intercept (fixed us per launch) and slope (GB/s of the streaming part).

    python tools/size_sweep.py [--size 4096] [--counts 262144,524288,...]
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "roce-test_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--size", type=int, default=4096)
    ap.add_argument("--counts", default="131072,262144,524288,1048576,2097152,4194304")
    ap.add_argument("--reps", type=int, default=20)
    a = ap.parse_args()
    import numpy as np
    import torch

    import roce_icrc

    ctx = roce_icrc.Context(devices=[0])
    st = torch.cuda.current_stream()
    counts = [int(c) for c in a.counts.split(",")]
    big = torch.empty(max(counts) * a.size, dtype=torch.uint8, device="cuda")
    ctx.synth_device(big, 0x1CEC0DE, 0, max(counts), a.size, stream=st)
    out = torch.empty(max(counts), dtype=torch.int32, device="cuda")
    xs, ys = [], []
    for c in counts:
        ctx.prime(25000)
        for _ in range(5):
            ctx.batch_device(big, c, out, stride=a.size, stream=st)
        evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(a.reps)]
        for e0, e1 in evs:
            e0.record(st)
            ctx.batch_device(big, c, out, stride=a.size, stream=st)
            e1.record(st)
        torch.cuda.synchronize()
        us = sorted(e0.elapsed_time(e1) * 1e3 for e0, e1 in evs)
        med = us[len(us) // 2]
        xs.append(c * a.size)
        ys.append(med)
        print(json.dumps({"size": a.size, "count": c, "bytes": c * a.size, "us_median": round(med, 2),
                          "us_min": round(us[0], 2), "GBps": round(c * a.size / med / 1e3, 1)}), flush=True)
    A = np.vstack([np.array(xs, float), np.ones(len(xs))]).T
    slope, icpt = np.linalg.lstsq(A, np.array(ys), rcond=None)[0]
    print(json.dumps({"fit": "us = bytes / (GBps * 1e3) + intercept", "GBps": round(1 / slope / 1e3, 1),
                      "intercept_us": round(icpt, 2)}), flush=True)
    ctx.close()


if __name__ == "__main__":
    main()
