#!/usr/bin/env python3
"""Headline benchmark: device-resident RoCEv2 ICRC GiB/s (BASELINE.json metric).

One step = one pass of the ICRC hot path (libroceicrc's streaming kernel on
gfx950) over one resident batch of synthetic RoCEv2 SEND_ONLY packets:
1,048,576 x 4096 B per GPU (BASELINE headline config; weak scaling at N > 1,
where every rank also all-gathers the 4-byte results over RCCL, as the
north_star's multi-GPU design asks).

    python bench.py [--gpus N --steps K --warmup W]
    python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N

Prints ONE JSON line on rank 0 (the task's bench contract) with a
``roofline`` block (kernel bytes / HIP-event kernel time vs 8 TB/s HBM) and,
at N = 1, a ``cpu_baseline`` block (the C oracle port timed on this host's
cores over a bounded sample of the same packets; the sample's GPU results are
also checked bit-exact against it).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "roce-test_amd"))

METRIC = "device-resident ICRC GiB/s on 1M×4096B RoCE packets; bit-exact vs reference"
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec, /opt/skills/guides/MI355X_MICROARCH.md
SEED = 0x1CEC0DE


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=100)
    # The first ~20 launches of a fresh process run ~10 % slower (clock / TLB
    # ramp measured in tools/microbench/abl.hip); 40 untimed steps cover it.
    ap.add_argument("--warmup", type=int, default=40)
    ap.add_argument("--count", type=int, default=1 << 20, help="packets per GPU")
    ap.add_argument("--size", type=int, default=4096, help="L3 packet bytes (IPv4 total_len)")
    ap.add_argument("--no-gather", action="store_true", help="skip the RCCL all-gather at N>1")
    ap.add_argument("--in-stream-gather", dest="overlap_gather", action="store_false",
                    help="order step i's all-gather after its kernel on the compute stream "
                         "(default: async on RCCL's stream, overlapping step i+1's kernel)")
    ap.add_argument("--cpu-seconds", type=float, default=6.0, help="wall budget of the CPU baseline")
    ap.add_argument("--no-cpu", action="store_true")
    return ap.parse_args()


def kernel_source_hash():
    """sha256 of the headline kernel's sources: PMC traffic measured on other code is stale."""
    import hashlib

    h = hashlib.sha256()
    for name in ("icrc_kernels.hip", "icrc_device.h", "icrc_math.h", "icrc_kernels.h"):
        with open(os.path.join(ROOT, "roce-test_amd", "csrc", name), "rb") as f:
            h.update(f.read())
    return h.hexdigest()[:16]


def load_traffic(size, count):
    """HBM bytes per launch measured by a separate rocprofv3 --pmc pass
    (profiles/pmc_traffic.json, produced by tools/pmc_traffic.py) on this very
    kernel source, or None."""
    p = os.path.join(ROOT, "profiles", "pmc_traffic.json")  # from tools/pmc_traffic.py
    try:
        with open(p) as f:
            d = json.load(f)
        if d.get("size") == size and d.get("count") == count and d.get("kernel_src") == kernel_source_hash():
            return d.get("hbm_bytes_per_launch")
    except (OSError, ValueError):
        pass
    return None


def kernel_label(size):
    """The kernel libroceicrc's dispatch picks for back-to-back packets of `size` bytes."""
    if size in (1024, 2048, 4096):
        return "strided-chain ICRC kernel (icrc_sck_kernel)"
    if 128 <= size <= 4096 and size & (size - 1) == 0:
        return "transposed streaming ICRC kernel (icrc_tsk_kernel)"
    return "streaming ICRC kernel"


def cpu_baseline(sample_host, got_sample, size, budget_s):
    """Time the C oracle (slice-by-8, pthreads over the host's cores)."""
    import numpy as np

    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle_c

    threads = max(1, min(16, len(os.sched_getaffinity(0))))
    want = oracle_c.icrc_batch(sample_host, stride=size, threads=threads)
    if not np.array_equal(want, got_sample):
        raise SystemExit("bench: GPU ICRCs differ from the oracle on the CPU-baseline sample")
    reps, t0 = 0, time.perf_counter()
    while True:
        oracle_c.icrc_batch(sample_host, stride=size, threads=threads)
        reps += 1
        dt = time.perf_counter() - t0
        if dt >= budget_s:
            break
    nbytes = sample_host.size * reps
    return {
        "value": nbytes / dt / 2**30,
        "unit": "GiB/s",
        "cores": threads,
        "kind": "port",
        "sample": f"{sample_host.shape[0]} x {size} B packets of the same synthetic batch, "
                  f"{reps} passes in {dt:.1f} s; oracle/icrc_oracle.c slice-by-8, {threads} threads",
    }


def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))

    import numpy as np
    import torch
    import torch.distributed as dist

    import roce_icrc

    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    distributed = "MASTER_ADDR" in os.environ  # launched by torch.distributed.run
    if distributed:
        dist.init_process_group("nccl", device_id=dev)
    ctx = roce_icrc.Context(devices=[local])

    count, size = args.count, args.size
    stream = torch.cuda.current_stream()
    pk = torch.empty(count * size, dtype=torch.uint8, device=dev)
    # Rank r owns global packets [r*count, (r+1)*count) (dist.shard_range of
    # world*count): generated on its own device from the global index.
    ctx.synth_device(pk, SEED, rank * count, count, size, stream=stream)
    do_gather = distributed and not args.no_gather
    # Double-buffered results.  Default: step i's all-gather runs async on
    # RCCL's stream, overlapping step i+1's kernel, and a buffer is reused only
    # after the gather that read it has been waited for.  --in-stream-gather:
    # the gather is ordered after the kernel on the compute stream.  (Each ICRC
    # workgroup fills a whole CU, so the kernel's blocks on CUs that RCCL holds
    # start late: measured +3-6 % kernel time with 16-32 CUs held for
    # 100-150 us, against a fully exposed gather in-stream)
    outs = [torch.empty(count, dtype=torch.int32, device=dev) for _ in range(2)]
    gathered = [torch.empty(world * count, dtype=torch.int32, device=dev) for _ in range(2)] if do_gather else None
    pending = [None, None]

    def step(i, ev=None):
        b = i & 1
        if pending[b] is not None:
            pending[b].wait()  # the current stream waits for the gather that read outs[b]
            pending[b] = None
        if ev is not None:
            ev[0].record(stream)
        ctx.batch_device(pk, count, outs[b], stride=size, stream=stream)
        if ev is not None:
            ev[1].record(stream)
        if do_gather:
            if args.overlap_gather:
                pending[b] = dist.all_gather_into_tensor(gathered[b], outs[b], async_op=True)
            else:
                dist.all_gather_into_tensor(gathered[b], outs[b])

    def drain():
        for b in range(2):
            if pending[b] is not None:
                pending[b].wait()
                pending[b] = None

    for i in range(args.warmup):
        step(i)
    drain()
    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
           for _ in range(args.steps)]
    torch.cuda.synchronize()
    if distributed:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(args.steps):
        step(i, evs[i])
    drain()
    torch.cuda.synchronize()
    if distributed:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    kern_ms = sum(a.elapsed_time(b) for a, b in evs) / args.steps
    out = outs[(args.steps - 1) & 1]
    if do_gather:  # every rank holds all world*count ICRCs in packet order
        g = gathered[(args.steps - 1) & 1]
        if not torch.equal(g[rank * count:(rank + 1) * count], out):
            raise SystemExit("bench: all-gathered ICRCs do not contain this rank's shard")

    if distributed:
        t = torch.tensor([elapsed, kern_ms], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed, kern_ms = float(t[0]), float(t[1])

    total_bytes = world * count * size * args.steps
    value = total_bytes / elapsed / 2**30
    alg_bytes = count * size + 4 * count  # per launch: packets read + ICRCs written
    achieved = alg_bytes / (kern_ms * 1e-3) / 1e9
    traffic = load_traffic(size, count)

    result = {
        "metric": METRIC,
        "value": round(value, 2),
        "unit": "GiB/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(elapsed * 1e3 / args.steps, 4),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u8",
        "data": "synthetic (device-generated RoCEv2 SEND_ONLY packets, seeded; reference P4 header template)",
        "config": {"workload": f"{count} x {size} B RoCEv2 packets per GPU, device-resident, "
                               + kernel_label(size) + (" + RCCL all-gather of ICRCs" + (" (overlapped)" if args.overlap_gather else "")
                                                           if do_gather else ""),
                   "packets_per_gpu": count, "packet_bytes": size,
                   "parallelism": f"dp{world}" + (" (all-gather u32 results)" if do_gather else "")},
        "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic,
                     "kernel_ms": round(kern_ms, 4), "alg_bytes_per_launch": alg_bytes},
    }

    if world == 1 and not args.no_cpu:
        ns = min(count, 32768)
        torch.cuda.synchronize()
        sample = pk[: ns * size].cpu().numpy().reshape(ns, size)
        got = out[:ns].cpu().numpy().view(np.uint32)
        result["cpu_baseline"] = cpu_baseline(sample, got, size, args.cpu_seconds)

    if rank == 0:
        print(json.dumps(result), flush=True)
    ctx.close()
    if distributed:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
