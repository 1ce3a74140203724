#!/usr/bin/env python3
"""Headline benchmark: device-resident RoCEv2 ICRC GiB/s (BASELINE.json metric).

One step = one pass of the ICRC hot path (libroceicrc's streaming kernel on
gfx950) over one resident batch of synthetic RoCEv2 SEND_ONLY packets:
1,048,576 x 4096 B per GPU (BASELINE headline config; weak scaling at N > 1,
where every rank also all-gathers the 4-byte results over RCCL, as the
north_star's multi-GPU design asks).

    python bench.py [--gpus N --steps K --warmup W]
    python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N
    python bench.py --mix        # BASELINE configs[4]: 4 M mixed-MTU packets per GPU

--mix runs the C4 workload instead of the headline: 4,194,304 packets per GPU
with lengths uniform over {64, 256, 1024, 4096}, packed back to back and
addressed by uint64 offsets + uint32 lengths (the ragged path: bucketing
passes + strided-chain fold + piece kernel + gather), its own metric name.

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
MIX_METRIC = "device-resident ICRC GiB/s on mixed-MTU (64/256/1024/4096 B) RoCE packets; bit-exact vs reference"
MIX_SIZES = (64, 256, 1024, 4096)
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec, /opt/skills/guides/MI355X_MICROARCH.md
SEED = 0x1CEC0DE


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=100)
    # The first ~20 launches of a fresh process run ~10 % slower (clock / TLB
    # ramp measured in tools/microbench/abl.hip); 40 untimed steps cover it.
    ap.add_argument("--warmup", type=int, default=40)
    ap.add_argument("--count", type=int, default=None, help="packets per GPU (default 1 M; 4 M with --mix)")
    ap.add_argument("--size", "--mtu", dest="size", type=int, default=4096, help="L3 packet bytes (IPv4 total_len)")
    ap.add_argument("--mix", action="store_true",
                    help="C4: lengths uniform over 64/256/1024/4096 B, offsets + lengths (ragged path)")
    ap.add_argument("--seed", type=int, default=SEED)
    ap.add_argument("--no-gather", action="store_true", help="skip the RCCL all-gather at N>1")
    ap.add_argument("--in-stream-gather", dest="overlap_gather", action="store_false",
                    help="order step i's all-gather after its kernel on the compute stream "
                         "(default: async on RCCL's stream, overlapping step i+1's kernel)")
    ap.add_argument("--cpu-seconds", type=float, default=6.0, help="wall budget of the CPU baseline")
    ap.add_argument("--no-cpu", action="store_true")
    a = ap.parse_args()
    if a.count is None:
        a.count = (4 << 20) if a.mix else (1 << 20)
    return a


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


def cpu_baseline(sample_host, got_sample, size, budget_s, offsets=None, lengths=None):
    """Time the C oracle (slice-by-8, pthreads over the host's cores)."""
    import numpy as np

    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle_c

    threads = max(1, min(16, len(os.sched_getaffinity(0))))
    kw = dict(offsets=offsets, lengths=lengths) if offsets is not None else dict(stride=size)
    want = oracle_c.icrc_batch(sample_host, threads=threads, **kw)
    if not np.array_equal(want, got_sample):
        raise SystemExit("bench: GPU ICRCs differ from the oracle on the CPU-baseline sample")
    reps, t0 = 0, time.perf_counter()
    while True:
        oracle_c.icrc_batch(sample_host, threads=threads, **kw)
        reps += 1
        dt = time.perf_counter() - t0
        if dt >= budget_s:
            break
    nbytes = (int(lengths.sum(dtype=np.uint64)) if lengths is not None else sample_host.size) * reps
    what = (f"{len(lengths)} mixed-MTU packets ({int(lengths.sum(dtype=np.uint64))} B)" if lengths is not None
            else f"{sample_host.shape[0]} x {size} B packets")
    return {
        "value": nbytes / dt / 2**30,
        "unit": "GiB/s",
        "cores": threads,
        "kind": "port",
        "sample": f"{what} of the same synthetic batch, "
                  f"{reps} passes in {dt:.1f} s; oracle/icrc_oracle.c slice-by-8, {threads} threads",
    }


def build_mix(torch, np, ctx, dev, stream, seed, rank, count):
    """C4 batch on `dev`: lengths uniform over MIX_SIZES (numpy PCG64 keyed on
    (seed, rank), so every rank holds its own shard), packets packed back to
    back; packet contents from the device generator of its size class,
    scattered into place.  Returns (buf, offsets, lengths, d_offsets, d_lengths)."""
    rng = np.random.default_rng([seed, rank])
    lens = rng.choice(np.array(MIX_SIZES, np.uint32), size=count)
    offs = np.zeros(count, np.uint64)
    offs[1:] = np.cumsum(lens[:-1], dtype=np.uint64)
    nbytes = int(lens.sum(dtype=np.uint64))
    buf = torch.empty(nbytes, dtype=torch.uint8, device=dev)
    for n in MIX_SIZES:
        idx = np.flatnonzero(lens == n)
        if len(idx) == 0:
            continue
        tmp = torch.empty(len(idx) * n, dtype=torch.uint8, device=dev)
        ctx.synth_device(tmp, seed, rank * count, len(idx), n, stream=stream)
        rows = tmp.view(len(idx), n)
        starts = torch.from_numpy(offs[idx].view(np.int64)).to(dev)
        cols = torch.arange(n, device=dev)
        step = max(1, (64 << 20) // n)
        for c in range(0, len(idx), step):
            ix = (starts[c:c + step, None] + cols[None, :]).reshape(-1)
            buf[ix] = rows[c:c + step].reshape(-1)
        del tmp, rows, starts
    d_offs = torch.from_numpy(offs.view(np.int64)).to(dev)
    d_lens = torch.from_numpy(lens.view(np.int32)).to(dev)
    return buf, offs, lens, d_offs, d_lens


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
    if args.mix:
        pk, h_offs, h_lens, d_offs, d_lens = build_mix(torch, np, ctx, dev, stream, args.seed, rank, count)
        rank_bytes = int(h_lens.sum(dtype=np.uint64))
    else:
        pk = torch.empty(count * size, dtype=torch.uint8, device=dev)
        # Rank r owns global packets [r*count, (r+1)*count) (dist.shard_range of
        # world*count): generated on its own device from the global index.
        ctx.synth_device(pk, args.seed, rank * count, count, size, stream=stream)
        d_offs = d_lens = None
        rank_bytes = count * size
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
        if args.mix:
            ctx.batch_device(pk, count, outs[b], offsets=d_offs, lengths=d_lens, stream=stream)
        else:
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

    all_bytes = rank_bytes
    if distributed:
        t = torch.tensor([elapsed, kern_ms], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed, kern_ms = float(t[0]), float(t[1])
        nb = torch.tensor([rank_bytes], dtype=torch.int64, device=dev)
        dist.all_reduce(nb, op=dist.ReduceOp.SUM)
        all_bytes = int(nb[0])

    total_bytes = all_bytes * args.steps
    value = total_bytes / elapsed / 2**30
    # per launch: packets read + ICRCs written (+ 12 B of offset/length descriptors per packet, ragged)
    alg_bytes = rank_bytes + 4 * count + (12 * count if args.mix else 0)
    achieved = alg_bytes / (kern_ms * 1e-3) / 1e9
    traffic = None if args.mix else load_traffic(size, count)

    if args.mix:
        workload = (f"{count} RoCEv2 packets per GPU, lengths uniform over 64/256/1024/4096 B "
                    f"({rank_bytes} B on rank 0), packed, uint64 offsets + uint32 lengths, device-resident, "
                    "ragged strided-chain path (bucketing passes + icrc_rsck_kernel + piece kernel + gather)")
    else:
        workload = f"{count} x {size} B RoCEv2 packets per GPU, device-resident, " + kernel_label(size)
    if do_gather:
        workload += " + RCCL all-gather of ICRCs" + (" (overlapped)" if args.overlap_gather else "")
    result = {
        "metric": MIX_METRIC if args.mix else METRIC,
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
        "config": {"workload": workload,
                   "packets_per_gpu": count, "packet_bytes": "mix 64/256/1024/4096" if args.mix else size,
                   "parallelism": f"dp{world}" + (" (all-gather u32 results)" if do_gather else "")},
        "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic,
                     "kernel_ms": round(kern_ms, 4), "alg_bytes_per_launch": alg_bytes},
    }

    if world == 1 and not args.no_cpu:
        ns = min(count, 32768)
        torch.cuda.synchronize()
        got = out[:ns].cpu().numpy().view(np.uint32)
        if args.mix:
            span = int(h_offs[ns - 1]) + int(h_lens[ns - 1])
            sample = pk[:span].cpu().numpy()
            result["cpu_baseline"] = cpu_baseline(sample, got, size, args.cpu_seconds,
                                                  offsets=h_offs[:ns].copy(), lengths=h_lens[:ns].copy())
        else:
            sample = pk[: ns * size].cpu().numpy().reshape(ns, size)
            result["cpu_baseline"] = cpu_baseline(sample, got, size, args.cpu_seconds)

    if rank == 0:
        print(json.dumps(result), flush=True)
    ctx.close()
    if distributed:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
