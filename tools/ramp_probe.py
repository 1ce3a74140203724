#!/usr/bin/env python3
"""Where does the first-launches slowdown of the headline kernel come from?

Per-launch HIP-event durations of the 1 M x 4096 B batch through
ricrc_batch_device, in phases separated by host-side idle gaps:

  fresh   : the first launches after the synthetic fill (a fresh process)
  idle_X  : after X ms of GPU idle (a clock ramp shows up again; a one-time
            per-process cost does not)
  primed  : after a ~20 ms busy pre-pass of other GPU work (the synthetic
            generator re-run over the batch)

    python tools/ramp_probe.py [--n 40] > gpurun_out/ramp.jsonl
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "roce-test_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=40)
    ap.add_argument("--count", type=int, default=1 << 20)
    ap.add_argument("--size", type=int, default=4096)
    a = ap.parse_args()
    import torch

    import roce_icrc

    dev = torch.device("cuda", 0)
    ctx = roce_icrc.Context(devices=[0])
    st = torch.cuda.current_stream()
    pk = torch.empty(a.count * a.size, dtype=torch.uint8, device=dev)
    out = torch.empty(a.count, dtype=torch.int32, device=dev)
    ctx.synth_device(pk, 0x1CEC0DE, 0, a.count, a.size, stream=st)
    torch.cuda.synchronize()

    def phase(name, n):
        evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(n)]
        t0 = time.perf_counter()
        for e0, e1 in evs:
            e0.record(st)
            ctx.batch_device(pk, a.count, out, stride=a.size, stream=st)
            e1.record(st)
        torch.cuda.synchronize()
        wall = (time.perf_counter() - t0) * 1e3 / n
        us = [round(e0.elapsed_time(e1) * 1e3, 1) for e0, e1 in evs]
        print(json.dumps({"phase": name, "wall_ms_per_launch": round(wall, 4), "us": us}), flush=True)

    phase("fresh", a.n)
    for gap in (2, 20, 200, 1000):
        time.sleep(gap / 1e3)
        phase(f"idle_{gap}ms", a.n)
    time.sleep(0.2)
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < 0.02:
        ctx.synth_device(pk, 0x1CEC0DE, 0, a.count, a.size, stream=st)
        torch.cuda.synchronize()
    phase("primed_synth_20ms", a.n)
    time.sleep(0.2)
    # a priming pass of the ICRC kernel itself on a small slice: ~2 ms busy
    for _ in range(3):
        ctx.batch_device(pk, a.count, out, stride=a.size, stream=st)
    phase("after_3_launches_idle200", a.n)
    ctx.close()


if __name__ == "__main__":
    main()
