#!/usr/bin/env python3
"""Timing probe of the ragged path on uniform and mixed batches (device-resident,
HIP-event time of one batch_device call incl. its pre/post passes).

    python tools/rsck_probe.py [--sizes 64,256,1024,4096] [--total-mib 1024]
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "roce-test_amd"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--sizes", default="64,256,1024,4096")
    ap.add_argument("--total-mib", type=int, default=1024)
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--rsck-only", action="store_true")
    args = ap.parse_args()
    import numpy as np
    import torch

    import oracle_c
    import roce_icrc

    ctx = roce_icrc.Context(devices=[0])
    dev = torch.device("cuda", 0)
    s = torch.cuda.current_stream()
    for n in [int(x) for x in args.sizes.split(",")]:
        count = (args.total_mib << 20) // n
        pk = torch.empty(count * n, dtype=torch.uint8, device=dev)
        ctx.synth_device(pk, 0x5EED, 0, count, n, stream=s)
        offs = torch.arange(count, dtype=torch.int64, device=dev) * n
        lens = torch.full((count,), n, dtype=torch.int32, device=dev)
        out = torch.empty(count, dtype=torch.int32, device=dev)
        for knob in ((None,) if args.rsck_only else (None, "RICRC_NO_RSCK")):
            if knob:
                os.environ[knob] = "1"
            for _ in range(3):
                ctx.batch_device(pk, count, out, offsets=offs, lengths=lens, stream=s)
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record(s)
            for _ in range(args.reps):
                ctx.batch_device(pk, count, out, offsets=offs, lengths=lens, stream=s)
            b.record(s)
            torch.cuda.synchronize()
            ms = a.elapsed_time(b) / args.reps
            if knob:
                os.environ.pop(knob)
            ns = min(count, 4096)
            want = oracle_c.icrc_batch(pk[: ns * n].cpu().numpy(), stride=n)
            ok = bool(np.array_equal(out[:ns].cpu().numpy().view(np.uint32), want))
            print(json.dumps({"n": n, "count": count, "path": "piece" if knob else "rsck", "ms": round(ms, 4),
                              "gib_s": round(count * n / (ms * 1e-3) / 2**30, 1), "ok": ok}), flush=True)
        del pk, offs, lens, out
        torch.cuda.empty_cache()
    ctx.close()


if __name__ == "__main__":
    main()
