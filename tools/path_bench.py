#!/usr/bin/env python3
"""Secondary-path throughput on one GPU (numbers quoted in DESIGN.md).

Device-resident (HIP-event kernel time, inputs already in HBM):
  * fixed-size batches at the BASELINE configs' MTUs (C1 64 B, 256 B, C2 1024 B,
    headline 4096 B) through the default dispatch (SCK for 1/2/4 KiB, TSK for
    smaller powers of two) and, for comparison, with RICRC_NO_SCK=1 (TSK) and
    with RICRC_NO_SCK=1 RICRC_NO_TSK=1 (the stride/offset streaming kernel);
  * the C4 ragged mix (N uniform over {64,256,1024,4096}, packed, uint64
    offsets + uint32 lengths) through the ragged kernel.
Host-resident (ricrc_batch_host: host in, host out; PCIe-inclusive):
  * 1 M x 4096 B from pageable numpy input, pinned (ricrc_host_alloc) input,
    registered (ricrc_host_register) input;
  * the C4 mix (packed, offsets + lengths) pageable, pinned and registered;
  * an Ethernet-framed NIC ring of 4 KiB slots (14-byte L2 header, RoCEv2
    frames of 64..4096 B, some padded / with FCS) through ricrc_batch_host_st
    with RICRC_F_STRICT (+ RICRC_F_FRAMELEN): the per-packet status route
    (gather with the EtherType bytes).

Every measured batch is also checked: the device results against a CPU
recomputation on a sample (C oracle).  Prints one JSON object per line.

    python tools/path_bench.py [--quick]
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

SEED = 0x1CEC0DE


def emit(**kw):
    print(json.dumps(kw), flush=True)


def check_sample(np, oracle_c, host_bytes, offs, lens, got, what, stride=0):
    want = oracle_c.icrc_batch(host_bytes, offsets=offs, lengths=lens, stride=stride, threads=16)
    if not np.array_equal(want, got):
        bad = int(np.flatnonzero(want != got)[0])
        raise SystemExit(f"{what}: mismatch at packet {bad}: got {got[bad]:#x} want {want[bad]:#x}")


def time_device(torch, ctx, fn, reps, warm):
    s = torch.cuda.current_stream()
    for _ in range(warm):
        fn(s)
    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(reps)]
    for a, b in evs:
        a.record(s)
        fn(s)
        b.record(s)
    torch.cuda.synchronize()
    return sum(a.elapsed_time(b) for a, b in evs) / reps


def ring_bench(args, np, ctx, oracle_c):
    # -- Ethernet-framed NIC ring through the status route -----------------
    # 4 KiB slots: 12 bytes of MACs, EtherType 0x0800, then a RoCEv2 packet of
    # 64..4096-14 B (a quarter carry 2 bytes of padding + a 4-byte FCS inside
    # the descriptor length: RICRC_F_FRAMELEN takes the IP length).
    import icrc_oracle as O

    slot, l3 = 4096, 14
    ring_n = (1 << 18) if args.quick else (1 << 20)
    sizes = np.random.default_rng(5).choice(np.array([64, 256, 1024, slot - l3 - 6], np.uint32), size=ring_n)
    extra = np.where(np.random.default_rng(6).random(ring_n) < 0.25, 6, 0).astype(np.uint32)
    ring = np.zeros(ring_n * slot, np.uint8)
    tmpl = {n: oracle_c.synth_batch(SEED, 0, 4096, int(n)) for n in np.unique(sizes)}
    for n in np.unique(sizes):
        idx = np.flatnonzero(sizes == n)
        rows = ring.reshape(ring_n, slot)
        rows[idx, 12] = 0x08
        rows[idx, l3:l3 + n] = tmpl[n][np.arange(len(idx)) % 4096]
    descr = sizes + extra
    offs = np.arange(ring_n, dtype=np.uint64) * slot
    ns = 4096
    w_out, w_st = O.status_batch(ring[: ns * slot], offsets=offs[:ns], lengths=descr[:ns], l3_offset=l3,
                                 strict=True, framelen=True)
    for label, kw in (("strict", dict(strict=True)), ("strict+framelen", dict(strict=True, framelen=True))):
        if "framelen" not in kw:  # the descriptor lengths are the datagrams' here
            lens_k = sizes
        else:
            lens_k = descr
        got, st = ctx.batch_host_st(ring, offs, lens_k, l3_offset=l3, **kw)  # warm
        if "framelen" in kw and not (np.array_equal(st[:ns], w_st) and np.array_equal(got[:ns], w_out)):
            raise SystemExit("host ring status route: mismatch against the oracle")
        if (st != 0).any():
            raise SystemExit(f"host ring {label}: {int((st != 0).sum())} packets rejected")
        t0 = time.perf_counter()
        for _ in range(3):
            ctx.batch_host_st(ring, offs, lens_k, l3_offset=l3, **kw)
        dt = (time.perf_counter() - t0) / 3
        nb = int(sizes.sum(dtype=np.uint64))
        emit(path="host", input=f"Ethernet NIC ring, 4 KiB slots, ricrc_batch_host_st {label}", packets=ring_n,
             bytes=nb, ring_bytes=ring.size, ms=round(dt * 1e3, 2), gib_s=round(nb / dt / 2**30, 2))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--quick", action="store_true")
    ap.add_argument("--skip-host", action="store_true")
    ap.add_argument("--only-ragged", action="store_true", help="only the C4 ragged device measurement")
    ap.add_argument("--only-ring", action="store_true", help="only the Ethernet-framed NIC ring (status route)")
    ap.add_argument("--ragged-paths", default="rsck", help="which ragged paths to time (rsck)")
    args = ap.parse_args()
    import numpy as np
    import torch

    import oracle_c
    import roce_icrc

    ctx = roce_icrc.Context(devices=[0])
    if args.only_ring:
        ring_bench(args, np, ctx, oracle_c)
        ctx.close()
        return
    dev = torch.device("cuda", 0)
    reps, warm = (10, 5) if args.quick else (50, 20)
    total = 1 << 30 if args.quick else 4 << 30

    # -- fixed-size device-resident -------------------------------------
    for n in (() if args.only_ragged else (64, 256, 1024, 4096)):
        count = total // n if n >= 1024 else min(total // n, 1 << 24)
        if n == 64:
            count = 1 << 20  # C1: 1 M x 64 B
        pk = torch.empty(count * n, dtype=torch.uint8, device=dev)
        out = torch.empty(count, dtype=torch.int32, device=dev)
        ctx.synth_device(pk, SEED, 0, count, n, stream=torch.cuda.current_stream())
        for mode in ("default", "tsk", "stream"):
            knobs = {"default": [], "tsk": ["RICRC_NO_SCK"], "stream": ["RICRC_NO_SCK", "RICRC_NO_TSK"]}[mode]
            if mode == "tsk" and n not in (1024, 2048, 4096):
                continue  # TSK is already the default there
            for k in knobs:
                os.environ[k] = "1"
            try:
                ms = time_device(torch, ctx, lambda s: ctx.batch_device(pk, count, out, stride=n, stream=s),
                                 reps, warm)
            finally:
                for k in knobs:
                    os.environ.pop(k, None)
            ns = min(count, 8192)
            check_sample(np, oracle_c, pk[: ns * n].cpu().numpy(), None, None,
                         out[:ns].cpu().numpy().view(np.uint32), f"{n}B/{mode}", stride=n)
            alg = count * n + 4 * count
            emit(path="device", kernel=mode, packet_bytes=n, packets=count, kernel_ms=round(ms, 4),
                 gib_s=round(count * n / (ms * 1e-3) / 2**30, 1),
                 hbm_frac=round(alg / (ms * 1e-3) / 8e12, 4))
        del pk, out
        torch.cuda.empty_cache()

    # -- C4 ragged mix ----------------------------------------------------
    rng = np.random.default_rng(SEED)
    count = (1 << 20) if args.quick else (4 << 20)
    lens = rng.choice(np.array([64, 256, 1024, 4096], np.uint32), size=count)
    offs = np.zeros(count, np.uint64)
    offs[1:] = np.cumsum(lens[:-1], dtype=np.uint64)
    nbytes = int(lens.sum(dtype=np.uint64))
    # Build the packed buffer on the device from per-size synthetic packets:
    # packet i of size n is synth(seed, i, n) (same generator as the bench).
    buf = torch.empty(nbytes, dtype=torch.uint8, device=dev)
    d_offs = torch.from_numpy(offs.view(np.int64)).to(dev)
    d_lens = torch.from_numpy(lens.view(np.int32)).to(dev)
    s = torch.cuda.current_stream()
    for n in (64, 256, 1024, 4096):
        idx = np.flatnonzero(lens == n)
        tmp = torch.empty(len(idx) * n, dtype=torch.uint8, device=dev)
        ctx.synth_device(tmp, SEED, 0, len(idx), n, stream=s)
        # scatter the rows into the packed buffer, in chunks (int64 index)
        rows = tmp.view(len(idx), n)
        starts = torch.from_numpy(offs[idx].view(np.int64)).to(dev)
        cols = torch.arange(n, device=dev)
        step = max(1, (64 << 20) // n)
        for c in range(0, len(idx), step):
            ix = (starts[c:c + step, None] + cols[None, :]).reshape(-1)
            buf[ix] = rows[c:c + step].reshape(-1)
        del tmp, rows, starts
    out = torch.empty(count, dtype=torch.int32, device=dev)
    kp = roce_icrc.kernel_path(buf, count, offsets=d_offs, lengths=d_lens, ctx=ctx)
    paths = [(lbl, knob) for key, lbl, knob in (("rsck", f"ragged, C4 mix ({kp})", None),)
             if key in args.ragged_paths.split(",")]
    for label, knob in paths:
        if knob:
            os.environ[knob] = "1"
        try:
            ms = time_device(torch, ctx, lambda s: ctx.batch_device(buf, count, out, offsets=d_offs,
                                                                     lengths=d_lens, stream=s), reps, warm)
        finally:
            if knob:
                os.environ.pop(knob, None)
        ns = 8192
        span = int(offs[ns - 1] + lens[ns - 1])
        check_sample(np, oracle_c, buf[:span].cpu().numpy(), offs[:ns], lens[:ns],
                     out[:ns].cpu().numpy().view(np.uint32), label)
        alg = nbytes + 16 * count
        emit(path="device", kernel=label, packets=count, bytes=nbytes, kernel_ms=round(ms, 4),
             gib_s=round(nbytes / (ms * 1e-3) / 2**30, 1), hbm_frac=round(alg / (ms * 1e-3) / 8e12, 4))
    host_ragged = (buf.cpu().numpy(), offs, lens, out.cpu().numpy().view(np.uint32).copy())
    del buf, out, d_offs, d_lens
    torch.cuda.empty_cache()

    if args.skip_host or args.only_ragged:
        ctx.close()
        return

    # -- host path (PCIe-inclusive) ------------------------------------------
    n = 4096
    count = total // n
    pk = torch.empty(count * n, dtype=torch.uint8, device=dev)
    want_dev = torch.empty(count, dtype=torch.int32, device=dev)
    ctx.synth_device(pk, SEED, 0, count, n, stream=torch.cuda.current_stream())
    ctx.batch_device(pk, count, want_dev, stride=n, stream=torch.cuda.current_stream())
    torch.cuda.synchronize()
    want = want_dev.cpu().numpy().view(np.uint32).copy()
    pageable = pk.cpu().numpy()
    del pk, want_dev
    torch.cuda.empty_cache()

    def host_run(label, arr, reps_h):
        got = ctx.batch_host(arr, stride=n)  # warm (allocates staging)
        if not np.array_equal(got, want):
            raise SystemExit(f"host {label}: mismatch")
        t0 = time.perf_counter()
        for _ in range(reps_h):
            ctx.batch_host(arr, stride=n)
        dt = (time.perf_counter() - t0) / reps_h
        emit(path="host", input=label, packet_bytes=n, packets=count, ms=round(dt * 1e3, 2),
             gib_s=round(count * n / dt / 2**30, 2))

    host_run("pageable", pageable, 3)
    pinned = ctx.host_alloc(pageable.size)
    pinned[:] = pageable
    host_run("pinned (ricrc_host_alloc)", pinned, 3)
    ctx.host_free(pinned)
    if hasattr(ctx, "host_register"):
        ctx.host_register(pageable)
        host_run("registered (ricrc_host_register)", pageable, 3)
        ctx.host_unregister(pageable)

    del pageable
    hb, ho, hl, hw = host_ragged
    rb = int(hl.sum(dtype=np.uint64))

    def host_ragged_run(label, arr, reps_h):
        got = ctx.batch_host(arr, ho, hl)  # warm
        if not np.array_equal(got, hw):
            raise SystemExit(f"host ragged {label}: mismatch")
        t0 = time.perf_counter()
        for _ in range(reps_h):
            ctx.batch_host(arr, ho, hl)
        dt = (time.perf_counter() - t0) / reps_h
        emit(path="host", input=f"{label} ragged C4 mix", packets=len(hl), bytes=rb, ms=round(dt * 1e3, 2),
             gib_s=round(rb / dt / 2**30, 2))

    host_ragged_run("pageable", hb, 3)
    pinned = ctx.host_alloc(hb.size)
    pinned[:] = hb
    host_ragged_run("pinned", pinned, 3)
    ctx.host_free(pinned)
    ctx.host_register(hb)
    host_ragged_run("registered", hb, 3)
    ctx.host_unregister(hb)
    del hb

    ring_bench(args, np, ctx, oracle_c)
    ctx.close()


if __name__ == "__main__":
    main()
