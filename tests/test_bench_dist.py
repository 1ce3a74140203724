"""CPU: bench.py's N > 1 timed loop, end to end, at world size 2 over gloo.

bench.run() is the loop the driver's multi-GPU bench executes on every rank
(double-buffered result vectors, the padded IcrcGather all-gather after every
step -- async and overlapped by default, in stream with --in-stream-gather,
absent with --no-gather -- the barrier + synchronize bracket, max-over-ranks
time, summed bytes, and the sampled oracle check of EVERY rank's gathered
ICRCs).  Here it runs with a CPU stand-in for the HIP backend: each rank
generates its shard with the generator's restatement and computes its ICRCs
with the CPU oracle (test code only; the product backend is HipBackend), so
everything but the kernels and RCCL is exercised before the driver's 8-GPU
run.  Anchor: SURVEY.md §8(e)."""
import json
import os
import socket
import sys
import time

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


class _Ev:
    def record(self, stream=None):
        self.t = time.perf_counter()

    def elapsed_time(self, other):
        return (other.t - self.t) * 1e3


class CpuOracleBackend:
    """HipBackend's interface on the CPU: gloo, host tensors, the oracle."""

    dist_backend = "gloo"

    def __init__(self):
        self.dev = torch.device("cpu")

    def init_dist(self):
        dist.init_process_group("gloo")

    def build(self, args, world, rank):
        import bench
        import oracle_c
        from roce_icrc.dist import cuts_to_sizes

        T, cuts, lens_g = bench.shard_plan(args, world)
        lo, hi = cuts[rank], cuts[rank + 1]
        if args.mix:
            lens = np.ascontiguousarray(lens_g[lo:hi])
            buf, offs = oracle_c.synth_ragged(args.seed, lo, lens)
            b = dict(buf=buf, h_offs=offs, h_lens=lens, lens_global=lens_g, rank_bytes=int(lens.sum(dtype=np.uint64)))
        elif args.l3_offset or args.slot_lengths:  # ring slots (a length per slot with --slot-lengths)
            n = hi - lo
            lens = np.ascontiguousarray(lens_g[lo:hi]) if args.slot_lengths else np.full(n, args.pkt, np.uint32)
            offs = np.arange(n, dtype=np.uint64) * args.stride + args.l3_offset
            buf, _ = oracle_c.synth_ragged(args.seed, lo, lens, offsets=offs, size=n * args.stride)
            b = dict(buf=buf, h_offs=offs, h_lens=lens, lens_global=lens_g, rank_bytes=int(lens.sum(dtype=np.uint64)))
        else:
            buf = oracle_c.synth_batch(args.seed, lo, hi - lo, args.size)
            b = dict(buf=buf, lens_global=None, rank_bytes=(hi - lo) * args.size)
        b.update(cuts=cuts, sizes=cuts_to_sizes(cuts), T=T)
        return b

    def compute(self, b, count, out, args):
        import oracle_c

        if b.get("h_offs") is not None:
            v = oracle_c.icrc_batch(b["buf"], offsets=b["h_offs"], lengths=b["h_lens"], family=args.family)
        else:
            v = oracle_c.icrc_batch(b["buf"], stride=args.size, family=args.family)
        out[:count] = torch.from_numpy(v.view(np.int32))

    def sync(self):
        pass

    def event(self):
        return _Ev()

    def record(self, ev):
        ev.record()

    def prime(self, ms):
        pass

    def host_bytes(self, b, nbytes):
        return b["buf"][:nbytes]

    # the host route (bench.e2e_route), on the CPU
    def host_pinned(self, b, nbytes):
        return np.array(b["buf"][:nbytes])

    def host_free(self, arr):
        pass

    def host_batch(self, arr, args, count):
        import oracle_c

        return oracle_c.icrc_batch(arr, stride=args.size, count=count, family=args.family)

    def h2d_ms(self, arr, b, reps):
        t = time.perf_counter()
        for _ in range(reps):
            np.copyto(b["buf"][:arr.size], arr)
        return (time.perf_counter() - t) * 1e3 / reps

    def close(self):
        pass


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _rank(rank, world, port, argv, q):
    sys.path.insert(0, ROOT)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    import bench

    try:
        args = bench.parse(argv)
        res, full_h, b = bench.run(args, world, rank, CpuOracleBackend(), True)
        q.put((rank, json.dumps(res), full_h.copy(), b["sizes"]))
    except BaseException as e:  # SystemExit from the bench's own checks included
        q.put((rank, f"ERROR {type(e).__name__}: {e}", None, None))
    finally:
        if dist.is_initialized():
            dist.destroy_process_group()


def _rank_side(rank, world, port, argv, q):
    """_rank, then bench.run_side: the N > 1 side configs (c3_strong, c4_strong)."""
    sys.path.insert(0, ROOT)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    import bench

    try:
        args = bench.parse(argv)
        be = CpuOracleBackend()
        res, full_h, b = bench.run(args, world, rank, be, True)
        res.update(bench.run_side(args, world, rank, be, True))
        q.put((rank, json.dumps(res), full_h.copy(), b["sizes"]))
    except BaseException as e:
        q.put((rank, f"ERROR {type(e).__name__}: {e}", None, None))
    finally:
        if dist.is_initialized():
            dist.destroy_process_group()


def run2(argv, world=2, target=None):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=target or _rank, args=(r, world, port, argv, q)) for r in range(world)]
    for p in procs:
        p.start()
    got = {}
    for _ in range(world):
        r, res, full, sizes = q.get(timeout=240)
        assert not res.startswith("ERROR"), f"rank {r}: {res}"
        got[r] = (json.loads(res), full, sizes)
    for p in procs:
        p.join(60)
        assert p.exitcode == 0
    return got


BASE = ["--gpus", "2", "--steps", "3", "--warmup", "1", "--prime-ms", "0", "--no-cpu"]


def _want(argv):
    """The single-process result vector of the whole global batch (oracle)."""
    import bench
    import oracle_c

    args = bench.parse(BASE + argv)
    T, cuts, lens_g = bench.shard_plan(args, 2)  # the global batch (independent of the cut)
    if args.mix:
        buf, offs = oracle_c.synth_ragged(args.seed, 0, lens_g)
        return oracle_c.icrc_batch(buf, offsets=offs, lengths=lens_g)
    return oracle_c.icrc_batch(oracle_c.synth_batch(args.seed, 0, T, args.size), stride=args.size)


@pytest.mark.parametrize("argv,scaling,total", [
    (["--size", "1024", "--count", "3000"], "weak", 6000),                      # headline shape, scaled down
    (["--size", "4096", "--global-count", "4097"], "strong", 4097),             # C3 shape (4 M in all), odd split
    (["--mix", "--count", "2500"], "weak", 5000),                               # C4: byte-balanced unequal shards
    (["--size", "64", "--count", "2000", "--in-stream-gather"], "weak", 4000),  # gather ordered after the kernel
])
def test_bench_run_world2_gloo(argv, scaling, total):
    got = run2(BASE + argv)
    res = got[0][0]
    assert res["n_gpus"] == 2 and res["scaling"] == scaling and res["steps"] == 3
    assert res["config"]["packets_total"] == total and res["config"]["parallelism"] == "dp2 (all-gather u32 results)"
    assert res["value"] > 0 and res["ms_per_step"] > 0 and res["oracle_sampled_all_ranks"]
    assert "cpu_baseline" not in res
    # the step's parts timed apart (compute-only, the collective alone), the
    # group's own world size, the collective library's version (None on gloo)
    assert res["world_size"] == 2 and res["collective_backend"] == "gloo" and "rccl_version" in res
    assert res["compute_only_ms_per_step"] > 0 and res["gather_ms"] > 0
    # every rank's own kernel time and shard, with their spread
    rk = res["ranks"]
    assert len(rk["kernel_ms"]) == 2 and len(rk["shard_bytes"]) == 2 and rk["slowest_rank"] in (0, 1)
    assert rk["kernel_ms_min"] == min(rk["kernel_ms"]) and rk["kernel_ms_max"] == max(rk["kernel_ms"])
    assert rk["shard_bytes_min"] == min(rk["shard_bytes"]) and rk["shard_bytes_max"] == max(rk["shard_bytes"])
    assert rk["shard_packets"] == got[0][2] and rk["kernel_ms_max"] == res["roofline"]["kernel_ms"]
    sizes = got[0][2]
    assert sum(sizes) == total
    if "--mix" in argv:
        assert sizes[0] != sizes[1] and "mixed-MTU" in res["metric"]
    want = _want(argv)
    for r in (0, 1):  # every rank ends with the whole vector, in packet order
        np.testing.assert_array_equal(got[r][1], want)
        assert got[r][0]["value"] == res["value"]  # max-over-ranks time, summed bytes: one number


def test_bench_run_world2_no_gather():
    """--no-gather: each rank keeps only its own shard; the oracle check runs on it."""
    argv = ["--size", "1024", "--count", "1500", "--no-gather"]
    got = run2(BASE + argv)
    want = _want(argv)
    assert got[0][0]["config"]["parallelism"] == "dp2"
    assert got[0][0]["compute_only_ms_per_step"] > 0 and "gather_ms" not in got[0][0]
    np.testing.assert_array_equal(got[0][1], want[:1500])
    np.testing.assert_array_equal(got[1][1], want[1500:])


def test_bench_side_configs_world2_gloo():
    """The driver's N > 1 command also runs BASELINE configs 3 and 4 as
    strong scaling: c3_strong (4 M x 4 KiB in all) and
    c4_strong (the 4 M mix in all, byte-balanced), each with its own
    compute-only and gather times -- here scaled down by --side-count."""
    got = run2(BASE + ["--size", "1024", "--count", "1000", "--side-count", "3001"], target=_rank_side)
    res = got[0][0]
    for k in ("c3_strong", "c4_strong"):
        d = res[k]
        assert d["scaling"] == "strong" and d["config"]["packets_total"] == 3001, k
        assert d["compute_only_ms_per_step"] > 0 and d["gather_ms"] > 0 and d["oracle_sampled_all_ranks"], k
        # (frac is rounded to 4 places: a CPU stand-in on a loaded host can round to 0)
        assert d["roofline"]["frac"] >= 0 and d["roofline"]["kernel_ms"] > 0 and d["value"] > 0, k
        assert got[1][0][k]["value"] == d["value"], k  # one number on every rank
        assert len(d["ranks"]["kernel_ms"]) == 2 and sum(d["ranks"]["shard_packets"]) == 3001, k
    assert "mixed-MTU" in res["c4_strong"]["metric"] and "fixed total" in res["c3_strong"]["metric"]
