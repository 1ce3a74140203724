#!/usr/bin/env python3
"""Headline benchmark: device-resident RoCEv2 ICRC GiB/s (BASELINE.json metric).

One step = one pass of the ICRC hot path (libroceicrc's gfx950 kernels) over
one resident batch of synthetic RoCEv2 SEND_ONLY packets, plus, at N > 1, the
RCCL all-gather of the 4-byte results over xGMI (the north_star's multi-GPU
design; overlapped with the next step's kernel by default).

    python bench.py [--gpus N --steps K --warmup W]     N > 1: self-launches torchrun
    python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N
    python bench.py --global-count 4194304               C3: a fixed 4 M x 4 KiB batch
    python bench.py --mix                                C4: mixed-MTU ragged batch

Workloads (the packet batch is one global batch of T packets,
cut into contiguous per-rank shards by roce_icrc.dist, each rank generating
its shard on its own device from the global packet index):
  default       T = 1,048,576 x 4096 B per GPU (BASELINE headline; weak scaling)
  --global-count T   T packets in all, shard_range split (strong scaling; C3)
  --mix         lengths uniform over {64, 256, 1024, 4096}, packed back to
                back, uint64 offsets + uint32 lengths (the ragged path); T =
                4 M per GPU (weak) or --global-count; shards cut at equal bytes
                (byte_balanced_cuts), so shard sizes differ and the gather is
                the unequal-shard IcrcGather (one all_gather_into_tensor).

Prints ONE JSON line on rank 0 (the task's bench contract) with a
``roofline`` block (rank 0's kernel bytes / HIP-event kernel time vs 8 TB/s)
and, at N = 1, a ``cpu_baseline`` block (the product's own CPU batch path,
ricrc_batch_cpu, on this host's CPU share over a bounded sample of the same
packets; the C oracle port's figure beside it), the C0 per-packet CPU latency
of the product's ricrc_one, and ``e2e``: the headline batch through
ricrc_batch_host from pinned host memory (host in, host out, PCIe included).  Every rank checks a sample of EVERY
rank's gathered ICRCs against the oracle restatement of the generator (after
the timed region), so "bit-exact" holds at every N.
"""
from __future__ import annotations

import argparse
import json
import os
import socket
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "roce-test_amd"))

METRIC = "device-resident ICRC GiB/s on 1M×4096B RoCE packets; bit-exact vs reference"
MIX_METRIC = "device-resident ICRC GiB/s on mixed-MTU (64/256/1024/4096 B) RoCE packets; bit-exact vs reference"
MIX_SIZES = (64, 256, 1024, 4096)
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec, /opt/skills/guides/MI355X_MICROARCH.md
SEED = 0x1CEC0DE
# Headline kernel's sources: PMC traffic (profiles/pmc_traffic.json) is only
# reported for the exact sources it was measured on -- the kernel's own and
# icrc_api.cpp, which picks its launch configuration (grids, pass sizes).
SCK_SOURCES = ("icrc_sck.hip", "icrc_sck.h", "icrc_device.h", "icrc_math.h", "icrc_api.cpp")
# The ragged pipeline's (C4, --mix): passes, fold, one-line kernel, gather.
RAGGED_SOURCES = ("icrc_rsck.hip", "icrc_kernels.h", "icrc_sck.h", "icrc_device.h", "icrc_math.h", "icrc_api.cpp")
# The quad kernel's (C1: back-to-back 64-byte packets).
QUAD_SOURCES = ("icrc_kernels.hip", "icrc_kernels.h", "icrc_device.h", "icrc_math.h", "icrc_api.cpp")


RAGGED_KERNELS = ("rsck_bucket", "icrc_rsck_kernel", "icrc_rsmall_kernel", "rsck_gather", "icrc_rswg_kernel")


def traffic_record(mix, size, count=None, l3_offset=0, stride=None, slot_lengths=None):
    """(profiles/ file, kernel sources, kernel names) of the PMC traffic
    record for a workload of `count` packets on this rank (tools/pmc_traffic.py
    writes it), or None.  The BASELINE counts (1 M fixed-size packets, 4 M
    mixed) keep their round-3 names; other counts (C3's 16 GiB batch, the
    8-GPU shard stand-ins) carry the count in the name; framed rings their
    slot and L3 offset."""
    std = (4 << 20) if mix else (1 << 20)
    tag = "" if count in (None, std) else f"_{count}"
    if slot_lengths is not None:  # a ring with a length per slot: the ragged pipeline
        lo, hi = slot_lengths
        return f"pmc_traffic_ring{l3_offset}_{stride or size}_len{lo}-{hi}{tag}.json", RAGGED_SOURCES, RAGGED_KERNELS
    if l3_offset:  # 1, 2 and 4 KiB slots with the L3 start in line 0: the SCK's framed variant
        name = f"pmc_traffic_ring{l3_offset}_{stride or size}{tag}.json"
        if (stride or size) in (1024, 2048, 4096) and l3_offset <= 92:
            return name, SCK_SOURCES, ("icrc_sck_kernel",)
        return name, RAGGED_SOURCES, RAGGED_KERNELS
    if mix:
        return f"pmc_traffic_mix{tag}.json", RAGGED_SOURCES, RAGGED_KERNELS
    if size == 4096:
        return (f"pmc_traffic_4096{tag}.json" if tag else "pmc_traffic.json"), SCK_SOURCES, ("icrc_sck_kernel",)
    if size in (1024, 2048):
        return f"pmc_traffic_{size}{tag}.json", SCK_SOURCES, ("icrc_sck_kernel",)
    if size == 64:
        return f"pmc_traffic_64{tag}.json", QUAD_SOURCES, ("icrc_quad_kernel",)
    return None


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--warmup", type=int, default=40)
    ap.add_argument("--count", type=int, default=None, help="packets per GPU (default 1 M; 4 M with --mix)")
    ap.add_argument("--global-count", type=int, default=None,
                    help="packets in the whole batch, split over the ranks (strong scaling; C3 = 4194304)")
    ap.add_argument("--size", "--mtu", dest="size", type=int, default=4096, help="L3 packet bytes (IPv4 total_len)")
    ap.add_argument("--mix", action="store_true",
                    help="C4: lengths uniform over 64/256/1024/4096 B, offsets + lengths (ragged path)")
    ap.add_argument("--seed", type=int, default=SEED)
    ap.add_argument("--family", choices=("v4", "v6", "auto"), default="v4",
                    help="address-family masks (v4 = the reference's; v6/auto: SURVEY §8f-3)")
    ap.add_argument("--no-gather", action="store_true", help="skip the RCCL all-gather at N>1")
    ap.add_argument("--in-stream-gather", dest="overlap_gather", action="store_false",
                    help="order step i's all-gather after its kernel on the compute stream "
                         "(default: async on RCCL's stream, overlapping step i+1's kernel)")
    # After >= 20 ms of GPU idle the first ~12 launches run up to 15 % slower
    # (profiles/r02/ramp_probe.jsonl); ricrc_prime keeps the device busy this
    # long right before the warmup (untimed).
    ap.add_argument("--prime-ms", type=float, default=25.0)
    # ... and the board's power ramps over tens of ms of sustained load: the
    # workload's own steps (kernels only, untimed) for this long before the
    # warmup steps (profiles/r04/s23_*).
    ap.add_argument("--warm-ms", type=float, default=100.0)
    # HIP events bracket the K timed steps as a whole (kernel_ms = their span
    # / K, inter-kernel gaps included: a conservative launch duration); with
    # --step-events every step's kernel(s) get their own pair -- two event
    # records between consecutive kernels cost ~5 us of GPU time per step
    # (each is a release to system scope), which the wall-clock value pays.
    ap.add_argument("--step-events", action="store_true")
    ap.add_argument("--cpu-seconds", type=float, default=10.0, help="wall budget of the CPU baseline")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--pass-times", action="store_true",
                    help="diagnostics (--mix): HIP events between the ragged pipeline's passes (RICRC_PASS_TIMES; "
                         "a few us per step) -> pass_ms, and the GPU's clocks / power around the timed steps")
    ap.add_argument("--no-gpu-state", action="store_true",
                    help="with --pass-times: skip the amd-smi readings around the timed steps")
    ap.add_argument("--gpu-state-delay", type=float, default=0.0,
                    help="with --pass-times: seconds to wait after the first amd-smi reading (diagnostics)")
    ap.add_argument("--plan-only", action="store_true",
                    help="print the shard plan every rank would run (gloo, no GPU) and exit")
    # Ethernet-framed NIC rings (common/huge_malloc.h:12-22):
    # slots of --stride bytes (default --size), the L3 packet at --l3-offset
    # in each, stride - l3_offset bytes long.
    ap.add_argument("--l3-offset", type=int, default=0, help="L3 start inside each slot (14: Ethernet framing)")
    ap.add_argument("--stride", type=int, default=None, help="slot bytes of a framed ring (default --size)")
    # ... with a completion length per slot (a NIC receive ring): the packet
    # lengths uniform over [lo, hi] (PCG64 on the seed), a uint32 lengths array
    # beside the ring (the ragged pipeline).
    ap.add_argument("--slot-lengths", default=None, metavar="LO:HI",
                    help="framed ring with per-slot packet lengths uniform over [LO, HI] (needs --stride)")
    # The other BASELINE configs, measured by the same command after the
    # headline: N = 1 adds c1 (1 M x 64 B), c2 (1 M x
    # 1 KiB) and c4 (the 4 M mix); N > 1 adds c3_strong (4 M x 4 KiB in all)
    # and c4_strong (the 4 M mix in all, byte-balanced).
    ap.add_argument("--no-side", action="store_true", help="the main workload only")
    ap.add_argument("--side-count", type=int, default=None,
                    help="packets of every side config (tests; default: the BASELINE counts)")
    a = ap.parse_args(argv)
    if a.count is None:
        a.count = (4 << 20) if a.mix else (1 << 20)
    if a.stride is None:
        a.stride = a.size
    if a.mix and (a.l3_offset or a.stride != a.size):
        ap.error("--l3-offset / --stride describe fixed-slot rings, not --mix")
    if not 0 <= a.l3_offset < a.stride:
        ap.error("--l3-offset must lie inside the slot")
    a.pkt = a.stride - a.l3_offset  # L3 bytes per packet (the largest, with --slot-lengths)
    if a.slot_lengths is not None:
        try:
            lo, hi = (int(x) for x in a.slot_lengths.split(":"))
        except ValueError:
            ap.error("--slot-lengths takes LO:HI")
        if a.mix or not 44 <= lo <= hi <= a.pkt:
            ap.error(f"--slot-lengths: need 44 <= LO <= HI <= stride - l3_offset = {a.pkt} (and no --mix)")
        a.slot_lengths = (lo, hi)
    return a


def launcher_argv(argv, gpus, port):
    """The torch.distributed.run command that re-runs this script on `gpus` ranks."""
    return [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={gpus}",
            "--master-addr=127.0.0.1", f"--master-port={port}", os.path.abspath(__file__)] + list(argv)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def check_world(args, env=os.environ):
    """None when this process runs the bench as it is; (0, "relaunch") for
    --gpus N > 1 outside torchrun (re-run on N ranks); (2, message) when
    WORLD_SIZE disagrees with --gpus (never report a mislabelled run)."""
    ws = env.get("WORLD_SIZE")
    if ws is None:
        return None if args.gpus == 1 else (0, "relaunch")
    if int(ws) != args.gpus:
        return (2, f"bench: --gpus {args.gpus} but WORLD_SIZE={ws}; refusing to report a mislabelled run")
    return None


def kernel_source_hash(sources=None):
    """sha256 of a kernel's sources (default: the headline kernel's, SCK_SOURCES)."""
    import hashlib

    h = hashlib.sha256()
    for name in sources or SCK_SOURCES:
        with open(os.path.join(ROOT, "roce-test_amd", "csrc", name), "rb") as f:
            h.update(f.read())
    return h.hexdigest()[:16]


def load_traffic(args, count):
    """HBM bytes per launch measured by separate rocprofv3 --pmc passes
    (profiles/pmc_traffic*.json, from tools/pmc_traffic.py) on this very
    workload and kernel source, or None."""
    rec = traffic_record(args.mix, args.size, count, args.l3_offset, args.stride, args.slot_lengths)
    if args.family != "v4" or rec is None:
        return None
    name, srcs, _ = rec
    p = os.path.join(ROOT, "profiles", name)
    try:
        with open(p) as f:
            d = json.load(f)
        same = d.get("count") == count and d.get("kernel_src") == kernel_source_hash(srcs)
        same = same and (d.get("size") == "mix" if args.mix else d.get("size") == args.size)
        same = same and d.get("l3_offset", 0) == args.l3_offset and d.get("stride", args.size) == args.stride
        same = same and d.get("slot_lengths") == (list(args.slot_lengths) if args.slot_lengths else None)
        if same:
            return d.get("hbm_bytes_per_launch")
    except (OSError, ValueError):
        pass
    return None


# What each kernel of the dispatch is, for the workload string.
KERNEL_ROLES = {
    "icrc_sck_kernel": "strided-chain ICRC kernel",
    "icrc_quad_kernel": "quad ICRC kernel (64-byte packets, lane-quad transposes)",
    "icrc_tsk_kernel": "transposed streaming ICRC kernel",
    "icrc_stream_kernel": "direct streaming ICRC kernel",
    "rsck_bucket": "bucket pass",
    "icrc_rsck_kernel": "strided-chain fold (8 packets of >= 2 lines a group; one-line packets one a lane)",
    "icrc_rsmall_kernel": "one-line packets",
    "rsck_gather": "gather",
    "icrc_rswg_kernel": "workgroup-local ragged kernel (classify, fold, write in one launch)",
    "family_fix_kernel": "address-family fix-up",
}


def kernel_path(args, base=0x100000, count=1):
    """The kernels libroceicrc's dispatch launches for this workload, straight
    from the library (ricrc_kernel_path: the same code that launches them),
    with ``base`` the batch's device address (only its alignment matters)."""
    import roce_icrc

    if args.mix:
        return roce_icrc.kernel_path(base, count, offsets=8, lengths=8, family=args.family)
    return roce_icrc.kernel_path(base, count, stride=args.stride, l3_offset=args.l3_offset, family=args.family,
                                 lengths=8 if args.slot_lengths else None)


def kernel_label(args, base=0x100000, count=1):
    """Human-readable label of kernel_path: 'role (kernel) -> role (kernel)'."""
    ks = kernel_path(args, base, count).split("+")
    return " -> ".join(f"{KERNEL_ROLES.get(k, k)} ({k})" for k in ks)


def rccl_version():
    """RCCL's version as torch reports it ("nccl" is RCCL on ROCm), or None."""
    try:
        import torch

        v = torch.cuda.nccl.version()
        return ".".join(map(str, v)) if isinstance(v, tuple) else str(v)
    except Exception:
        return None


def gpu_state(dev):
    """Clock / power / temperature readings of GPU `dev` right now (amd-smi,
    else rocm-smi; JSON as the tool prints it), or an error string."""
    for cmd in (["amd-smi", "metric", "-g", str(dev), "-c", "-p", "-t", "--json"],
                ["rocm-smi", "-d", str(dev), "--showclocks", "--showpower", "--showtemp", "--json"]):
        try:
            r = subprocess.run(cmd, capture_output=True, text=True, timeout=20)
            if r.returncode == 0 and r.stdout.strip():
                return {"tool": cmd[0], "t": round(time.time(), 3), "data": json.loads(r.stdout)}
        except (OSError, subprocess.SubprocessError, ValueError):
            continue
    return "unavailable"


def cpu_share():
    """Host threads this process may use: its affinity, capped by the CPU share
    the box grants one GPU (OMP_NUM_THREADS, 16 on the GPU pool)."""
    n = len(os.sched_getaffinity(0))
    share = os.environ.get("OMP_NUM_THREADS")
    if share and share.isdigit() and int(share) > 0:
        n = min(n, int(share))
    return max(1, n)


def cpu_model():
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


# ----------------------------------------------------- cpu_baseline leg (oracle)
def _oracle():
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import icrc_oracle
    import oracle_c

    return oracle_c, icrc_oracle


def oracle_check(gathered, sizes, cuts, args, lens_global=None, per_rank=256):
    """Checker (untimed): regenerate a sample of every rank's packets on the
    host from the generator's restatement and compare the gathered ICRCs."""
    import numpy as np

    oracle_c, _ = _oracle()
    bad = 0
    for r in range(len(sizes)):
        lo, n = cuts[r], sizes[r]
        if n == 0:
            continue
        idx = np.unique(np.concatenate([np.arange(min(per_rank, n)),
                                        np.linspace(0, n - 1, num=min(per_rank, n)).astype(np.int64)]))
        if lens_global is None:
            pk = np.concatenate([oracle_c.synth_batch(args.seed, lo + int(k), 1, args.pkt) for k in idx])
            want = oracle_c.icrc_batch(pk.reshape(-1), stride=args.pkt, family=args.family)
        else:
            lens = lens_global[lo + idx]
            bufs = [oracle_c.synth_ragged(args.seed, lo + int(k), lens[j:j + 1])[0] for j, k in enumerate(idx)]
            offs = np.zeros(len(idx), np.uint64)
            offs[1:] = np.cumsum(lens[:-1], dtype=np.uint64)
            want = oracle_c.icrc_batch(np.concatenate(bufs), offsets=offs, lengths=lens, family=args.family)
        got = gathered[lo + idx]
        bad += int((got != want).sum())
    return bad


def product_cpu(sample_host, got_sample, size, budget_s, threads, offsets=None, lengths=None, family="v4"):
    """The product's own CPU batch path (ricrc_batch_cpu in libroceicrc_cpu.so:
    the slice-by-16 fold of ricrc_one, icrc_cpu.cpp) on the same sample and
    threads: GiB/s, or an error string if its ICRCs differ from the GPU's."""
    import numpy as np

    import roce_icrc

    kw = dict(offsets=offsets, lengths=lengths) if offsets is not None else dict(stride=size)
    if not np.array_equal(roce_icrc.icrc_batch_cpu(sample_host, threads=threads, family=family, **kw), got_sample):
        return "mismatch"
    reps, t0 = 0, time.perf_counter()
    while True:
        roce_icrc.icrc_batch_cpu(sample_host, threads=threads, family=family, **kw)
        reps += 1
        dt = time.perf_counter() - t0
        if dt >= budget_s:
            break
    nbytes = int(lengths.sum(dtype=np.uint64)) if lengths is not None else sample_host.size
    return nbytes * reps / dt / 2**30


def cpu_baseline(sample_host, got_sample, size, budget_s, offsets=None, lengths=None, family="v4"):
    """The cpu_baseline block: ``value`` is the product's own CPU batch path
    (ricrc_batch_cpu, slice-by-16, pthreads over this host's CPU share; SURVEY
    §8(d)(3)) on a sample of the batch.  The C oracle (slice-by-8, same
    threads) checks the GPU's ICRCs on the sample first and is timed beside it
    (``oracle_port_GiBs``), with a 1-core zlib figure (the Python oracle,
    zlib.crc32 per packet)."""
    import numpy as np

    oracle_c, icrc_oracle = _oracle()
    threads = cpu_share()
    kw = dict(offsets=offsets, lengths=lengths) if offsets is not None else dict(stride=size)
    kw["family"] = family
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
    sample_bytes = int(lengths.sum(dtype=np.uint64)) if lengths is not None else sample_host.size
    what = (f"{len(lengths)} mixed-MTU packets ({sample_bytes} B)" if lengths is not None
            else f"{sample_host.shape[0]} x {size} B packets")
    # 1 core, zlib.crc32 per packet (icrc_oracle.icrc), ~2 s
    flat = sample_host.reshape(-1)
    pk = ([bytes(flat[int(o): int(o) + int(n)]) for o, n in zip(offsets, lengths)] if offsets is not None
          else [bytes(r) for r in sample_host])
    zb, zt0 = 0, time.perf_counter()
    while time.perf_counter() - zt0 < 2.0:
        for p in pk[:2048]:
            icrc_oracle.icrc(p, family)
            zb += len(p)
    zdt = time.perf_counter() - zt0
    oracle_gibs = sample_bytes * reps / dt / 2**30
    prod = product_cpu(sample_host, got_sample, size, min(5.0, budget_s), threads, offsets, lengths, family)
    if not isinstance(prod, float):
        raise SystemExit(f"bench: the product CPU path disagrees with the GPU on the CPU-baseline sample ({prod})")
    # value: the build's own CPU batch path (SURVEY.md 8(d)(3) names it the CPU
    # baseline); the C oracle's time on the same sample is a side key.
    return {
        "value": round(prod, 2),
        "unit": "GiB/s",
        "cores": threads,
        "kind": "port",
        "sample": f"{what} of the same synthetic batch; ricrc_batch_cpu (libroceicrc_cpu.so: the slice-by-16 fold of "
                  f"ricrc_one, the build's CPU path restating calc_icrc) on {threads} threads (this GPU's CPU share of "
                  f"{os.cpu_count()} visible host CPUs), ICRCs checked equal to the GPU's first",
        "cpu_model": cpu_model(),
        "oracle_port_GiBs": round(oracle_gibs, 2),
        "oracle_port": f"oracle/icrc_oracle.c slice-by-8 on the same sample and {threads} threads, {reps} passes in "
                       f"{dt:.1f} s (test infrastructure; the checker)",
        "zlib_1core_GiBs": round(zb / zdt / 2**30, 3),
    }


def c0_latency():
    """BASELINE configs[0]: ICRC of one 1 KiB RoCE packet on the CPU through the
    product's per-packet entry point (libroceicrc_cpu.so via ctypes, the way
    python/simulator.py's crossings would call it)."""
    import roce_icrc

    pkt = bytearray(os.urandom(1024))
    pkt[0], pkt[9], pkt[2], pkt[3], pkt[22], pkt[23] = 0x45, 17, 4, 0, 0x12, 0xB7
    n, t0 = 0, time.perf_counter()
    while time.perf_counter() - t0 < 0.5:
        for _ in range(1000):
            roce_icrc.icrc(pkt)
        n += 1000
    dt = time.perf_counter() - t0
    # the C call alone (no Python argument marshalling): ctypes with a raw pointer
    import ctypes

    buf = (ctypes.c_uint8 * 1024).from_buffer(pkt)
    f = roce_icrc.cpu.ricrc_one
    addr = ctypes.addressof(buf)
    m, t1 = 0, time.perf_counter()
    while time.perf_counter() - t1 < 0.5:
        for _ in range(1000):
            f(addr, 1024)
        m += 1000
    dt1 = time.perf_counter() - t1
    return {"config": "1 x 1024 B RoCEv2 packet, CPU, libroceicrc_cpu.so (BASELINE configs[0])",
            "us_per_packet_python_api": round(dt / n * 1e6, 3),
            "us_per_packet_ctypes_call": round(dt1 / m * 1e6, 3)}


def shard_plan(args, world):
    """The global batch and its per-rank cuts (no GPU): (T, cuts, lens_global).
    Fixed size: shard_range of T packets; --mix: one global length vector
    (PCG64 on the seed) cut at equal bytes."""
    import numpy as np

    from roce_icrc.dist import byte_balanced_cuts, shard_range

    T = args.global_count if args.global_count is not None else args.count * world
    if args.mix:
        lens_g = np.random.default_rng(args.seed).choice(np.array(MIX_SIZES, np.uint32), size=T)
        return T, byte_balanced_cuts(lens_g, world), lens_g
    cuts = [shard_range(T, world, r)[0] for r in range(world)] + [T]
    if args.slot_lengths:  # ring slots: equal slot counts per rank, a length per slot
        lo, hi = args.slot_lengths
        return T, cuts, np.random.default_rng(args.seed).integers(lo, hi + 1, size=T).astype(np.uint32)
    return T, cuts, None


def build_batch(torch, np, ctx, dev, stream, args, world, rank):
    """This rank's shard of the global batch, generated on `dev`.  Returns a
    dict: buf, d_offs, d_lens, h_offs, h_lens (ragged), cuts, sizes,
    lens_global (ragged), rank_bytes."""
    from roce_icrc.dist import cuts_to_sizes

    T, cuts, lens_g = shard_plan(args, world)
    lo, hi = cuts[rank], cuts[rank + 1]
    b = {}
    if args.mix:
        lens = np.ascontiguousarray(lens_g[lo:hi])
        offs = np.zeros(len(lens), np.uint64)
        if len(lens) > 1:
            offs[1:] = np.cumsum(lens[:-1], dtype=np.uint64)
        nbytes = int(lens.sum(dtype=np.uint64))
        buf = torch.empty(max(nbytes, 1), dtype=torch.uint8, device=dev)
        d_offs = torch.from_numpy(offs.view(np.int64)).to(dev)
        d_lens = torch.from_numpy(lens.view(np.int32)).to(dev)
        ctx.synth_ragged_device(buf, args.seed, lo, len(lens), d_offs, d_lens, stream=stream)
        b.update(buf=buf, d_offs=d_offs, d_lens=d_lens, h_offs=offs, h_lens=lens, lens_global=lens_g,
                 rank_bytes=nbytes)
    elif args.l3_offset or args.slot_lengths:  # a framed ring: the L3 packet at l3_offset in each stride-byte slot
        n = hi - lo
        buf = torch.zeros(max(n * args.stride, 1), dtype=torch.uint8, device=dev)
        h_lens = np.ascontiguousarray(lens_g[lo:hi]) if args.slot_lengths else np.full(n, args.pkt, np.uint32)
        d_lens = torch.from_numpy(h_lens.view(np.int32)).to(dev) if n else None
        if n:
            offs = torch.arange(n, dtype=torch.int64, device=dev) * args.stride + args.l3_offset
            ctx.synth_ragged_device(buf, args.seed, lo, n, offs, d_lens, stream=stream)
            stream.synchronize()
            del offs
        if not args.slot_lengths:  # every packet runs to its slot's end: no lengths array
            d_lens = None
        b.update(buf=buf, d_offs=None, d_lens=d_lens, h_lens=h_lens, lens_global=lens_g,
                 rank_bytes=int(h_lens.sum(dtype=np.uint64)))
    else:
        buf = torch.empty(max((hi - lo) * args.size, 1), dtype=torch.uint8, device=dev)
        ctx.synth_device(buf, args.seed, lo, hi - lo, args.size, stream=stream)
        b.update(buf=buf, d_offs=None, d_lens=None, lens_global=None, rank_bytes=(hi - lo) * args.size)
    b.update(cuts=cuts, sizes=cuts_to_sizes(cuts), T=T)
    return b


def plan_only(args, world, rank):
    """--plan-only: every rank computes the shard plan it would run, the ranks
    check over gloo (CPU, no GPU touched) that they agree, and rank 0 prints it
    as one JSON line -- the launcher / rendezvous / sharding exercised without
    a GPU."""
    import numpy as np
    import torch
    import torch.distributed as dist

    from roce_icrc.dist import cuts_to_sizes

    T, cuts, lens_g = shard_plan(args, world)
    sizes = cuts_to_sizes(cuts)
    lo, hi = cuts[rank], cuts[rank + 1]
    mine = int(lens_g[lo:hi].sum(dtype=np.uint64)) if lens_g is not None else (hi - lo) * args.pkt
    if world > 1:
        dist.init_process_group("gloo")
        got = [torch.zeros(2, dtype=torch.int64) for _ in range(world)]
        dist.all_gather(got, torch.tensor([hi - lo, mine], dtype=torch.int64))
        counts = [int(g[0]) for g in got]
        nbytes = [int(g[1]) for g in got]
        dist.destroy_process_group()
        if counts != sizes:
            raise SystemExit(f"bench: rank {rank}: ranks disagree on the shard plan {counts} != {sizes}")
    else:
        nbytes = [mine]
    if rank == 0:
        print(json.dumps({"plan_only": True, "n_gpus": world, "packets_total": T, "shard_packets": sizes,
                          "shard_bytes": nbytes, "scaling": "strong" if args.global_count is not None else "weak",
                          "workload": "mix" if args.mix else f"{args.size} B"}), flush=True)
    return 0


def relaunch(args, argv):
    cmd = launcher_argv(argv, args.gpus, _free_port())
    env = dict(os.environ, MASTER_ADDR="127.0.0.1")
    return subprocess.call(cmd, env=env)


def _count_label(n):
    return f"{n >> 20}M" if n and n % (1 << 20) == 0 else str(n)


def metric_for(args, T, count):
    """The metric string of the workload actually run: BASELINE.json's
    headline string only for its own config (1 M x 4096 B per GPU)."""
    if args.mix:
        scope = f"{_count_label(T)} in all" if args.global_count is not None else f"{_count_label(args.count)} per GPU"
        return (f"device-resident ICRC GiB/s on mixed-MTU (64/256/1024/4096 B) RoCE packets ({scope}); "
                "bit-exact vs reference")
    if args.slot_lengths:
        scope = f"{_count_label(T)} in all" if args.global_count is not None else f"{_count_label(args.count)} per GPU"
        lo, hi = args.slot_lengths
        return (f"device-resident ICRC GiB/s on {lo}-{hi}B RoCE packets in {args.stride}B ring slots with a length "
                f"per slot (L3 at offset {args.l3_offset}; {scope}); bit-exact vs reference")
    if args.l3_offset:
        scope = f"{_count_label(T)} in all" if args.global_count is not None else f"{_count_label(args.count)} per GPU"
        return (f"device-resident ICRC GiB/s on {args.pkt}B RoCE packets in {args.stride}B Ethernet-framed ring slots "
                f"(L3 at offset {args.l3_offset}; {scope}); bit-exact vs reference")
    if args.global_count is None and args.size == 4096 and args.count == 1 << 20:
        return METRIC
    if args.global_count is not None:
        return (f"device-resident ICRC GiB/s on {_count_label(T)}\u00d7{args.size}B RoCE packets (fixed total); "
                "bit-exact vs reference")
    return f"device-resident ICRC GiB/s on {_count_label(args.count)}\u00d7{args.size}B RoCE packets; bit-exact vs reference"


class HipBackend:
    """The product path of one rank: libroceicrc's gfx950 kernels on the
    rank's GPU (roce_icrc.Context), RCCL ("nccl") between ranks, HIP events on
    the compute stream.  run() drives it; tests/test_bench_dist.py drives
    run() with a CPU stand-in over gloo (the N > 1 loop without a GPU)."""

    dist_backend = "nccl"

    def __init__(self, local, pass_times=False):
        import torch

        import roce_icrc

        self.torch = torch
        torch.cuda.set_device(local)
        self.dev = torch.device("cuda", local)
        if pass_times:  # read once, by ricrc_create
            os.environ["RICRC_PASS_TIMES"] = "1"
        self.ctx = roce_icrc.Context(devices=[local])
        self.stream = torch.cuda.current_stream()

    def init_dist(self):
        import torch.distributed as dist

        dist.init_process_group("nccl", device_id=self.dev)

    def build(self, args, world, rank):
        import numpy as np

        return build_batch(self.torch, np, self.ctx, self.dev, self.stream, args, world, rank)

    def compute(self, b, count, out, args):
        if args.mix:
            self.ctx.batch_device(b["buf"], count, out, offsets=b["d_offs"], lengths=b["d_lens"], stream=self.stream,
                                  family=args.family)
        else:
            self.ctx.batch_device(b["buf"], count, out, stride=args.stride, l3_offset=args.l3_offset,
                                  lengths=b["d_lens"], stream=self.stream, family=args.family)

    def sync(self):
        self.torch.cuda.synchronize()

    def event(self):
        return self.torch.cuda.Event(enable_timing=True)

    def record(self, ev):
        ev.record(self.stream)

    def prime(self, ms):
        if ms > 0:
            self.ctx.prime(int(ms * 1000))

    def pass_times(self):
        return self.ctx.pass_times()

    def launch_info(self, b, count, args):
        """The dispatch's launch of this batch (ricrc_launch_info): grid, the
        per-XCD work-split weights and the recorded start XCD."""
        if args.mix:
            return self.ctx.launch_info(b["buf"], count, offsets=b["d_offs"], lengths=b["d_lens"])
        return self.ctx.launch_info(b["buf"], count, stride=args.stride, l3_offset=args.l3_offset,
                                    lengths=b["d_lens"])

    def release(self):
        self.torch.cuda.synchronize()
        self.torch.cuda.empty_cache()

    def host_bytes(self, b, nbytes):
        return b["buf"][:nbytes].cpu().numpy()

    # -- the host route (e2e): host in, host out --------------------------
    def host_pinned(self, b, nbytes):
        """A pinned host copy (ricrc_host_alloc) of the batch's first nbytes."""
        arr = self.ctx.host_alloc(nbytes)
        self.torch.from_numpy(arr).copy_(b["buf"][:nbytes])
        return arr

    def host_free(self, arr):
        self.ctx.host_free(arr)

    def host_batch(self, arr, args, count):
        return self.ctx.batch_host(arr, stride=args.size, count=count, family=args.family)

    def h2d_ms(self, arr, b, reps):
        """The host-to-device copy alone of the whole pinned batch (ms per copy)."""
        src = self.torch.from_numpy(arr)
        dst = b["buf"][:arr.size]
        e0, e1 = self.event(), self.event()
        dst.copy_(src, non_blocking=True)
        self.sync()
        self.record(e0)
        for _ in range(reps):
            dst.copy_(src, non_blocking=True)
        self.record(e1)
        self.sync()
        return e0.elapsed_time(e1) / reps

    def close(self):
        self.ctx.close()


def run(args, world, rank, be, distributed):
    """The timed loop of one rank on backend `be`; returns (result, ICRCs on
    the host, batch).  Steps: the hot path over the resident shard + (N > 1)
    the all-gather of the u32 results (IcrcGather, one collective per step,
    double-buffered; async on the collective's stream by default).  The K
    timed steps sit between barrier + synchronize on both sides; elapsed and
    kernel time are the max over ranks, bytes the sum."""
    import numpy as np
    import torch
    import torch.distributed as dist

    from roce_icrc.dist import IcrcGather

    if distributed and not dist.is_initialized():
        be.init_dist()
    b = be.build(args, world, rank)
    count, sizes = b["sizes"][rank], b["sizes"]
    if os.environ.get("RICRC_DEBUG") and hasattr(b["buf"], "data_ptr"):  # placement studies
        print("bench: buf %#x offs %#x lens %#x" % (b["buf"].data_ptr(), getattr(b.get("d_offs"), "data_ptr", int)(),
                                                    getattr(b.get("d_lens"), "data_ptr", int)()), file=sys.stderr)
    rank_bytes = b["rank_bytes"]
    do_gather = distributed and not args.no_gather
    g = IcrcGather(sizes)
    # Double-buffered results (padded to the longest shard).  Default: step
    # i's all-gather runs async on the collective's stream, overlapping step
    # i+1's kernel, and a buffer is reused only after the gather that read it
    # has been waited for.  --in-stream-gather: the gather is ordered after
    # the kernel on the compute stream.
    outs = [g.local_buffer(be.dev) for _ in range(2)]
    gathered = [g.gathered_buffer(be.dev) for _ in range(2)] if do_gather else None
    pending = [None, None]

    def step(i, ev=None):
        j = i & 1
        if pending[j] is not None:
            pending[j].wait()  # the current stream waits for the gather that read outs[j]
            pending[j] = None
        if ev is not None:
            be.record(ev[0])
        if count:
            be.compute(b, count, outs[j], args)
        if ev is not None:
            be.record(ev[1])
        if do_gather:
            pending[j] = g.start(outs[j], gathered[j], async_op=args.overlap_gather)

    def drain():
        for j in range(2):
            if pending[j] is not None:
                pending[j].wait()
                pending[j] = None

    be.sync()
    be.prime(args.prime_ms)
    if args.warm_ms > 0 and count:
        t_w = time.perf_counter()
        i = 0
        while True:
            be.compute(b, count, outs[i & 1], args)
            i += 1
            if i % 8 == 0:
                be.sync()
                if (time.perf_counter() - t_w) * 1e3 >= args.warm_ms:
                    break
    for i in range(args.warmup):
        step(i)
    drain()
    diag = {}
    if args.pass_times and hasattr(be, "pass_times"):
        be.sync()
        be.pass_times()  # forget the warmup's calls
        if not args.no_gpu_state:
            diag["gpu_state_before"] = gpu_state(be.dev.index)
            if args.gpu_state_delay > 0:
                time.sleep(args.gpu_state_delay)
    n_ev = args.steps if args.step_events else 1
    evs = [(be.event(), be.event()) for _ in range(n_ev)]
    be.sync()
    if distributed:
        dist.barrier()
    be.sync()
    t0 = time.perf_counter()
    if args.step_events:
        for i in range(args.steps):
            step(i, evs[i])
    else:
        be.record(evs[0][0])
        for i in range(args.steps):
            step(i)
        be.record(evs[0][1])
    drain()
    be.sync()
    if distributed:
        dist.barrier()
    be.sync()
    elapsed = time.perf_counter() - t0
    kern_ms = sum(a.elapsed_time(c) for a, c in evs) / max(args.steps, 1)
    if args.pass_times and hasattr(be, "pass_times"):
        if not args.no_gpu_state:
            diag["gpu_state_after"] = gpu_state(be.dev.index)
        calls, ms = be.pass_times()
        diag["pass_ms"] = {k: round(v / max(calls, 1), 4) for k, v in
                           zip(("bucket", "fold", "one_line", "gather"), ms)} if calls else None
        diag["pass_calls"] = calls

    # ---- N > 1, after the timed region: the step's two parts timed apart
    # (compute-only and with-gather scaling reported
    # separately), each as K more iterations between barrier + synchronize,
    # max over ranks -- so a shortfall of the driver's scaling run can be
    # pinned on the kernels or on the collective.
    split = None
    if distributed:
        def timed(fn):
            be.sync()
            dist.barrier()
            be.sync()
            t = time.perf_counter()
            for i in range(args.steps):
                fn(i)
            be.sync()
            dist.barrier()
            be.sync()
            return (time.perf_counter() - t) * 1e3 / max(args.steps, 1)

        def compute_only(i):
            if count:
                be.compute(b, count, outs[i & 1], args)

        split = {"compute_only_ms_per_step": timed(compute_only)}
        if do_gather:
            split["gather_ms"] = timed(lambda i: g.start(outs[0], gathered[0], async_op=False))

    # ---- after the timed region: correctness on every rank
    last = (args.steps - 1) & 1
    out = outs[last][:count]
    if do_gather:
        gv = gathered[last]
        if not torch.equal(g.shard_of(gv, rank), out):
            raise SystemExit("bench: all-gathered ICRCs do not contain this rank's shard")
        full = g.compact(gv)
    else:
        full = out
    full_h = full.cpu().numpy().view(np.uint32)
    if do_gather or world == 1:
        bad = oracle_check(full_h, sizes if do_gather else [count], b["cuts"] if do_gather else [0],
                           args, lens_global=b["lens_global"])
    else:  # --no-gather at N > 1: only this rank's own shard is here
        bad = oracle_check(np.concatenate([np.zeros(b["cuts"][rank], np.uint32), full_h]),
                           [0] * rank + [count], b["cuts"], args, lens_global=b["lens_global"])
    if bad:
        raise SystemExit(f"bench: rank {rank}: {bad} sampled ICRCs differ from the oracle")

    all_bytes = rank_bytes
    ranks = None
    if distributed:
        # every rank's own kernel time, wall time and shard:
        # a shortfall of the driver's multi-GPU run can then be pinned on one
        # slow rank, an unequal byte cut or the collective
        mine = torch.tensor([kern_ms, elapsed * 1e3 / max(args.steps, 1), float(rank_bytes), float(count)],
                            dtype=torch.float64, device=be.dev)
        every = [torch.zeros_like(mine) for _ in range(world)]
        dist.all_gather(every, mine)
        every = [[float(x) for x in t.cpu()] for t in every]
        km = [e[0] for e in every]
        sb = [int(e[2]) for e in every]
        ranks = {"kernel_ms": [round(v, 4) for v in km], "ms_per_step": [round(e[1], 4) for e in every],
                 "shard_bytes": sb, "shard_packets": [int(e[3]) for e in every],
                 "kernel_ms_min": round(min(km), 4), "kernel_ms_max": round(max(km), 4),
                 "slowest_rank": int(max(range(world), key=lambda r: km[r])),
                 "shard_bytes_min": min(sb), "shard_bytes_max": max(sb)}
        keys = sorted(split)
        t = torch.tensor([elapsed, kern_ms] + [split[k] for k in keys], dtype=torch.float64, device=be.dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed, kern_ms = float(t[0]), float(t[1])
        split = {k: round(float(v), 4) for k, v in zip(keys, t[2:])}
        nb = torch.tensor([rank_bytes], dtype=torch.int64, device=be.dev)
        dist.all_reduce(nb, op=dist.ReduceOp.SUM)
        all_bytes = int(nb[0])

    value = all_bytes * args.steps / elapsed / 2**30
    # per launch: packets read + ICRCs written (+ 12 B of offset/length descriptors per packet, ragged)
    # (+ 4 B of length per slot, rings with a length per slot)
    alg_bytes = rank_bytes + 4 * count + (12 * count if args.mix else 4 * count if args.slot_lengths else 0)
    achieved = alg_bytes / (kern_ms * 1e-3) / 1e9 if kern_ms > 0 else 0.0
    traffic = load_traffic(args, count)

    strong = args.global_count is not None
    base = b["buf"].data_ptr() if hasattr(b["buf"], "data_ptr") else 0x100000
    label = kernel_label(args, base, max(count, 1))  # from the library's own dispatch (ricrc_kernel_path)
    if args.mix:
        workload = (f"{b['T']} RoCEv2 packets in all ({'fixed total' if strong else f'{args.count} per GPU'}), "
                    "lengths uniform over 64/256/1024/4096 B, packed, uint64 offsets + uint32 lengths, "
                    f"shards cut at equal bytes; rank 0: {sizes[0]} packets, {rank_bytes if rank == 0 else '?'} B; "
                    f"device-resident, ragged path: {label}")
    elif args.slot_lengths:
        workload = (f"{b['T']} RoCEv2 packets of {args.slot_lengths[0]}-{args.slot_lengths[1]} B in all ({count} on "
                    f"rank 0, {rank_bytes if rank == 0 else '?'} B), each at offset {args.l3_offset} of a "
                    f"{args.stride} B ring slot, uint32 length per slot, device-resident, ragged path: {label}")
    elif args.l3_offset:
        workload = (f"{b['T']} x {args.pkt} B RoCEv2 packets in all ({count} on rank 0), each at offset "
                    f"{args.l3_offset} of a {args.stride} B Ethernet-framed ring slot, device-resident, " + label)
    else:
        workload = (f"{b['T']} x {args.size} B RoCEv2 packets in all ({count} on rank 0), device-resident, "
                    + label)
    if do_gather:
        workload += " + RCCL all-gather of the u32 ICRCs" + (" (overlapped)" if args.overlap_gather else "")
    result = {
        "metric": metric_for(args, b["T"], count),
        "value": round(value, 2),
        "unit": "GiB/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(elapsed * 1e3 / args.steps, 4),
        "higher_is_better": True,
        "scaling": "strong" if strong else "weak",
        "vs_baseline": None,
        "dtype": "u8",
        "data": "synthetic (device-generated RoCEv2 SEND_ONLY packets, seeded; reference P4 header template)",
        "config": {"workload": workload, "packets_total": b["T"], "packets_rank0": sizes[0], "family": args.family,
                   "packet_bytes": ("mix 64/256/1024/4096" if args.mix else
                                    f"{args.slot_lengths[0]}-{args.slot_lengths[1]}" if args.slot_lengths else args.pkt),
                   "parallelism": f"dp{world}" + (" (all-gather u32 results)" if do_gather else "")},
        "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic,
                     "kernel_ms": round(kern_ms, 4), "alg_bytes_per_launch": alg_bytes},
        "oracle_sampled_all_ranks": True,
        # how the number was taken: untimed, before the warmup
        # steps, ricrc_prime's streaming reads and the workload's own steps
        # (the board's power ramps over tens of ms of sustained load)
        "method": {"prime_ms": args.prime_ms, "warm_ms": args.warm_ms, "warmup_steps": args.warmup,
                   "timing": "one HIP event pair around the K steps on the kernels' stream; value from wall "
                             "time between barrier + synchronize"},
    }
    if args.l3_offset or args.slot_lengths:
        result["config"].update(l3_offset=args.l3_offset, slot_bytes=args.stride)
    if hasattr(be, "launch_info") and count:
        try:
            result["launch"] = be.launch_info(b, count, args)
        except Exception as e:  # diagnostics only
            result["launch"] = f"unavailable: {e}"
    result.update(diag)
    if distributed:
        result["world_size"] = dist.get_world_size()
        result["collective_backend"] = dist.get_backend()
        result["rccl_version"] = rccl_version()
        result.update(split)
        result["ranks"] = ranks
    return result, full_h, b


def e2e_route(be, b, args, count, want, reps=5):
    """The headline batch through ricrc_batch_host from pinned host memory
    (ricrc_host_alloc): host in, host out, PCIe included -- the north_star's
    end-to-end rate (the path starts and ends in host memory,
    python/simulator.py:49-55).  The library cuts the batch into <= 256 MiB
    chunks, double-buffered on two streams (H2D of chunk k+1 overlaps the
    kernel of chunk k), and copies the 4-byte results back.  Reported beside
    the host-to-device copy alone of the same bytes and the device-resident
    kernel time; the ICRCs are checked equal to the device-resident run's."""
    import numpy as np

    nbytes = count * args.size
    arr = be.host_pinned(b, nbytes)
    try:
        got = be.host_batch(arr, args, count)  # (warm: first-touch of the staging and the chunk plan)
        if not np.array_equal(got, want[:count]):
            raise SystemExit("bench: e2e host-route ICRCs differ from the device-resident run")
        t0 = time.perf_counter()
        for _ in range(reps):
            be.host_batch(arr, args, count)
        dt = (time.perf_counter() - t0) / reps
        h2d = be.h2d_ms(arr, b, reps)
    finally:
        be.host_free(arr)
    return {"value": round(nbytes / dt / 2**30, 2), "unit": "GiB/s", "ms_per_batch": round(dt * 1e3, 3),
            "reps": reps, "h2d_ms": round(h2d, 3), "h2d_GiBs": round(nbytes / (h2d * 1e-3) / 2**30, 2),
            "d2h_bytes": 4 * count, "route": "ricrc_batch_host, pinned host buffer (ricrc_host_alloc): "
            "hipMemcpyAsync H2D in <= 256 MiB chunks on two streams, each chunk's kernel behind its copy, "
            "4-byte results D2H; host wall time per call",
            "config": f"{count} x {args.size} B (the headline batch), host in, host out, ICRCs checked"}


def n1_extras(args, be, result, full_h, b):
    """N = 1 only: cpu_baseline, the C0 latency and (headline shape) e2e."""
    import numpy as np

    count = b["sizes"][0]
    ns = min(count, 32768)
    got = full_h[:ns]
    if args.mix:
        h_offs, h_lens = b["h_offs"], b["h_lens"]
        span = int(h_offs[ns - 1]) + int(h_lens[ns - 1])
        sample = be.host_bytes(b, span)
        result["cpu_baseline"] = cpu_baseline(sample, got, args.size, args.cpu_seconds,
                                              offsets=h_offs[:ns].copy(), lengths=h_lens[:ns].copy(),
                                              family=args.family)
    elif args.slot_lengths:  # ring slots with a length each
        sample = be.host_bytes(b, ns * args.stride)
        offs = np.arange(ns, dtype=np.uint64) * args.stride + args.l3_offset
        result["cpu_baseline"] = cpu_baseline(sample, got, args.pkt, args.cpu_seconds, offsets=offs,
                                              lengths=b["h_lens"][:ns].copy(), family=args.family)
    else:  # (a framed ring: its slots' L3 packets, contiguous on the host)
        sample = be.host_bytes(b, ns * args.stride).reshape(ns, args.stride)[:, args.l3_offset:]
        result["cpu_baseline"] = cpu_baseline(np.ascontiguousarray(sample), got, args.pkt, args.cpu_seconds,
                                              family=args.family)
    result["c0"] = c0_latency()
    if not (args.mix or args.l3_offset or args.slot_lengths) and hasattr(be, "host_batch"):
        try:
            result["e2e"] = e2e_route(be, b, args, count, full_h)
        except (Exception, SystemExit) as e:
            result["e2e"] = {"error": f"{type(e).__name__}: {e}"}


# BASELINE.json's other configs: measured after the main
# workload in the same process, each with its own warm phase and K steps.
# N = 1 also carries the anchors of the 8-GPU run: C3's
# 4 M x 4 KiB on one GPU (the denominator of its strong-scaling curve), C4's
# 524,288-packet shard stand-in, the 4 KiB framed NIC ring, and a NIC ring of
# 1 KiB slots with a length per slot (64-1010 B, the ragged pipeline).
SIDE_N1 = (("c1", ["--size", "64"]), ("c2", ["--size", "1024"]), ("c4", ["--mix"]),
           ("c3", ["--global-count", str(4 << 20)]), ("c4s", ["--mix", "--count", str(512 << 10)]),
           ("ring", ["--l3-offset", "14", "--stride", "4096"]),
           ("ring_len", ["--l3-offset", "14", "--stride", "1024", "--slot-lengths", "64:1010"]))
SIDE_NX = (("c3_strong", ["--global-count", str(4 << 20)]), ("c4_strong", ["--mix", "--global-count", str(4 << 20)]))
SIDE_KEYS = ("metric", "value", "unit", "ms_per_step", "scaling", "compute_only_ms_per_step", "gather_ms",
             "oracle_sampled_all_ranks", "launch", "ranks")


def side_args(args, extra):
    """The parsed arguments of a side config: the main run's K, W, seed,
    family, gather mode and warm phase (no second primer: the device is busy
    already), the config's own shape (--side-count overrides its count)."""
    argv = extra + ["--gpus", str(args.gpus), "--steps", str(args.steps), "--warmup", str(args.warmup),
                    "--seed", str(args.seed), "--family", args.family, "--prime-ms", "0",
                    "--warm-ms", str(args.warm_ms), "--no-side", "--no-cpu"]
    argv += ["--no-gather"] if args.no_gather else []
    argv += [] if args.overlap_gather else ["--in-stream-gather"]
    sa = parse(argv)
    if args.side_count is not None:
        if sa.global_count is not None:
            sa.global_count = args.side_count
        else:
            sa.count = args.side_count
    return sa


def run_side(args, world, rank, be, distributed):
    """{name: compact result} for the side configs of this world size."""
    out = {}
    for name, extra in (SIDE_N1 if world == 1 else SIDE_NX):
        sa = side_args(args, extra)
        try:
            r, _, sb = run(sa, world, rank, be, distributed)
            del sb
        except (Exception, SystemExit) as e:  # N = 1: one side config's failure must not lose the main line
            if distributed:  # the other ranks may wait in a collective: fail the job as before
                raise
            out[name] = {"error": f"{type(e).__name__}: {e}"}
            if hasattr(be, "release"):
                be.release()
            continue
        d = {k: r[k] for k in SIDE_KEYS if k in r}
        d["config"] = {k: r["config"][k] for k in ("workload", "packets_total", "packets_rank0")}
        d["roofline"] = {k: r["roofline"][k] for k in ("achieved", "frac", "traffic", "kernel_ms", "alg_bytes_per_launch")}
        out[name] = d
        if hasattr(be, "release"):
            be.release()
    return out


def main(argv=None):
    argv = sys.argv[1:] if argv is None else argv
    args = parse(argv)
    chk = check_world(args)
    if chk is not None:
        code, msg = chk
        if msg == "relaunch":  # --gpus N > 1 outside torchrun: N ranks, before any GPU call
            return relaunch(args, argv)
        print(msg, file=sys.stderr)
        return code
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if args.plan_only:
        return plan_only(args, world, rank)

    import numpy as np
    import torch.distributed as dist

    be = HipBackend(local, pass_times=args.pass_times)
    distributed = world > 1 or "MASTER_ADDR" in os.environ
    result, full_h, b = run(args, world, rank, be, distributed)
    count = b["sizes"][rank]

    if world == 1 and not args.no_cpu:
        n1_extras(args, be, result, full_h, b)

    if not args.no_side:  # the other BASELINE configs, by the same command
        del full_h, b
        if hasattr(be, "release"):
            be.release()
        result.update(run_side(args, world, rank, be, distributed))

    if rank == 0:
        print(json.dumps(result), flush=True)
    be.close()
    if distributed:
        dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())
