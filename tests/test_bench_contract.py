"""bench.py's driver contract, checked on the CPU (no GPU needed).

The driver runs `python bench.py --gpus N --steps K --warmup W` (N > 1 under
torch.distributed.run) and parses ONE JSON line; these tests pin the argument
surface and the helpers that label the line (the GPU run itself is the
driver's and tests/test_gpu_parity.py's business)."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import pytest

import bench  # noqa: E402


def test_defaults_are_one_gpu_and_short(monkeypatch):
    monkeypatch.setattr(sys, "argv", ["bench.py"])
    a = bench.parse()
    assert a.gpus == 1 and a.steps > 0 and a.warmup >= 0
    assert a.count == 1 << 20 and a.size == 4096  # the BASELINE headline config
    assert a.overlap_gather is True  # N > 1: all-gather overlapped with the next kernel


def test_driver_flags_parse(monkeypatch):
    monkeypatch.setattr(sys, "argv", ["bench.py", "--gpus", "8", "--steps", "7", "--warmup", "3", "--in-stream-gather"])
    a = bench.parse()
    assert (a.gpus, a.steps, a.warmup, a.overlap_gather) == (8, 7, 3, False)


def test_mix_and_aliases_parse(monkeypatch):
    monkeypatch.setattr(sys, "argv", ["bench.py", "--mix"])
    a = bench.parse()
    assert a.mix and a.count == 4 << 20  # BASELINE configs[4]: 4 M mixed-MTU packets
    monkeypatch.setattr(sys, "argv", ["bench.py", "--mtu", "1024", "--count", "5", "--seed", "7"])
    a = bench.parse()
    assert (a.size, a.count, a.seed, a.mix) == (1024, 5, 7, False)
    assert bench.MIX_METRIC != bench.METRIC and bench.MIX_SIZES == (64, 256, 1024, 4096)


def test_gpus_n_relaunches_under_torchrun(monkeypatch):
    """--gpus N > 1 outside torchrun re-runs the script on N ranks (before any
    GPU call); inside torchrun WORLD_SIZE must equal --gpus."""
    a = bench.parse(["--gpus", "2", "--steps", "3"])
    assert bench.check_world(a, env={}) == (0, "relaunch")
    argv = bench.launcher_argv(["--gpus", "2", "--steps", "3"], 2, 29511)
    assert argv[1:3] == ["-m", "torch.distributed.run"]
    assert "--nproc-per-node=2" in argv and "--nnodes=1" in argv and "--master-addr=127.0.0.1" in argv
    assert "--master-port=29511" in argv
    assert argv[-4:] == ["--gpus", "2", "--steps", "3"] and argv[-5].endswith("bench.py")
    assert bench.check_world(a, env={"WORLD_SIZE": "2"}) is None
    assert bench.check_world(bench.parse([]), env={}) is None


def test_world_size_mismatch_exits_nonzero():
    env = dict(os.environ, WORLD_SIZE="2", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "1"], env=env,
                       capture_output=True, text=True, timeout=120)
    assert r.returncode != 0 and "WORLD_SIZE=2" in r.stderr and r.stdout == ""
    env["WORLD_SIZE"] = "8"
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "4"], env=env,
                       capture_output=True, text=True, timeout=120)
    assert r.returncode != 0 and r.stdout == ""


def test_global_count_is_strong_scaling(monkeypatch):
    a = bench.parse(["--global-count", "4194304"])
    assert a.global_count == 4 << 20 and a.count == 1 << 20
    a = bench.parse(["--mix", "--global-count", "1000"])
    assert a.mix and a.global_count == 1000


def test_cpu_share_respects_the_box_share(monkeypatch):
    monkeypatch.setenv("OMP_NUM_THREADS", "3")
    assert bench.cpu_share() == min(3, len(os.sched_getaffinity(0)))
    monkeypatch.delenv("OMP_NUM_THREADS")
    assert bench.cpu_share() == len(os.sched_getaffinity(0))
    assert isinstance(bench.cpu_model(), str)


def test_oracle_check_catches_a_wrong_shard():
    """The post-run checker regenerates every rank's sampled packets from the
    generator restatement: a correct gathered vector passes, a corrupted one
    (here: rank 1's shard of a 3-rank fixed batch, and one ragged packet) fails."""
    import numpy as np
    import oracle_c
    from roce_icrc.dist import byte_balanced_cuts, cuts_to_sizes, shard_range

    a = bench.parse(["--size", "256"])
    T, world = 3001, 3
    cuts = [shard_range(T, world, r)[0] for r in range(world)] + [T]
    full = oracle_c.icrc_batch(oracle_c.synth_batch(a.seed, 0, T, 256), stride=256)
    assert bench.oracle_check(full, cuts_to_sizes(cuts), cuts, a, per_rank=64) == 0
    bad = full.copy()
    bad[cuts[1] + 5] ^= 1
    assert bench.oracle_check(bad, cuts_to_sizes(cuts), cuts, a, per_rank=64) > 0
    a = bench.parse(["--mix"])
    lens = np.random.default_rng(a.seed).choice(np.array(bench.MIX_SIZES, np.uint32), size=2000)
    cuts = byte_balanced_cuts(lens, world)
    buf, offs = oracle_c.synth_ragged(a.seed, 0, lens)
    full = oracle_c.icrc_batch(buf, offsets=offs, lengths=lens)
    assert bench.oracle_check(full, cuts_to_sizes(cuts), cuts, a, lens_global=lens, per_rank=64) == 0
    full[cuts[2]] ^= 0x80
    assert bench.oracle_check(full, cuts_to_sizes(cuts), cuts, a, lens_global=lens, per_rank=64) > 0


def test_metric_matches_baseline_json():
    with open(os.path.join(ROOT, "BASELINE.json")) as f:
        assert json.load(f)["metric"] == bench.METRIC


def test_metric_names_the_workload_run():
    """Only BASELINE's own config carries BASELINE's metric string; C1/C2,
    the strong-scaling C3 batch and the C4 mix name what they ran."""
    m = lambda *a: bench.metric_for(bench.parse(list(a)), *((lambda x: (  # noqa: E731
        x.global_count if x.global_count is not None else x.count, x.count))(bench.parse(list(a)))))
    assert m() == bench.METRIC
    assert "1M\u00d764B" in m("--size", "64") and "4096B" not in m("--size", "64")
    assert "1M\u00d71024B" in m("--size", "1024")
    c3 = m("--global-count", "4194304")
    assert "4M\u00d74096B" in c3 and "fixed total" in c3 and c3 != bench.METRIC
    assert "1M\u00d74096B" not in m("--count", "4194304") and "4M\u00d74096B" in m("--count", "4194304")
    mix = m("--mix")
    assert "mixed-MTU" in mix and "4M per GPU" in mix
    assert "16M in all" in m("--mix", "--global-count", str(16 << 20))


def test_kernel_labels_follow_the_dispatch():
    """Labels come from the library's own dispatch (ricrc_kernel_path, no GPU
    needed): the kernels rocprofv3 shows for each BASELINE config."""
    lab = lambda *a: bench.kernel_label(bench.parse(list(a)))  # noqa: E731
    assert "(icrc_sck_kernel)" in lab() and "(icrc_sck_kernel)" in lab("--size", "1024")
    assert lab("--size", "64") == "quad ICRC kernel (64-byte packets, lane-quad transposes) (icrc_quad_kernel)"
    assert "(icrc_tsk_kernel)" in lab("--size", "256")
    mixa = bench.parse(["--mix"])
    mix = bench.kernel_label(mixa, count=mixa.count)  # C4's 4 M packets: eight chunks a workgroup, one launch
    wg = "workgroup-local ragged kernel (classify, fold, write in one launch) (icrc_rswg_kernel)"
    assert mix == wg
    # past ~4.6 M packets on 256 CUs: the three-pass pipeline, in launch order
    big = bench.kernel_label(bench.parse(["--mix", "--count", str(8 << 20)]), count=8 << 20)
    fold = "strided-chain fold (8 packets of >= 2 lines a group; one-line packets one a lane) (icrc_rsck_kernel)"
    assert big.split(" -> ") == ["bucket pass (rsck_bucket)", fold, "gather (rsck_gather)"]
    # C4's 8-GPU shard (about 524 K packets): one chunk a workgroup
    shard = bench.kernel_label(bench.parse(["--mix", "--count", "524288"]), count=524288)
    assert shard == wg
    # a framed 4 KiB NIC ring (L3 at 14): the SCK's framed variant over the slots
    assert "(icrc_sck_kernel)" in lab("--l3-offset", "14", "--stride", "4096")
    assert "(icrc_rswg_kernel)" in lab("--l3-offset", "14", "--stride", "1536")
    assert "family_fix_kernel" in lab("--size", "64", "--family", "v6")
    assert "family_fix_kernel" not in lab("--family", "v6")  # the SCK applies IPv6 masks natively
    assert "count/plan" not in mix and "scatter" not in mix


def test_cpu_baseline_value_is_the_product_cpu_path():
    """cpu_baseline.value is the build's own slice-by-16 CPU batch path
    (SURVEY.md 8(d)(3)); the oracle port's figure is a side key."""
    import oracle_c

    host = oracle_c.synth_batch(bench.SEED, 0, 64, 1024)
    want = oracle_c.icrc_batch(host, stride=1024)
    cb = bench.cpu_baseline(host, want, 1024, 0.05)
    assert cb["kind"] == "port" and cb["unit"] == "GiB/s" and cb["cores"] >= 1
    assert "ricrc_batch_cpu" in cb["sample"] and cb["value"] > 0
    assert cb["oracle_port_GiBs"] > 0 and "icrc_oracle.c" in cb["oracle_port"]
    with pytest.raises(SystemExit):  # a GPU result the CPU paths disagree with
        bad = want.copy()
        bad[3] ^= 1
        bench.cpu_baseline(host, bad, 1024, 0.05)


def test_traffic_is_tied_to_the_kernel_source(tmp_path):
    # only the headline kernel's own sources count (an edit of another kernel
    # must not null roofline.traffic)
    assert bench.SCK_SOURCES[0] == "icrc_sck.hip"
    h = bench.kernel_source_hash()
    assert len(h) == 16 and h == bench.kernel_source_hash()
    # profiles/pmc_traffic.json is only reported for the source it was measured on
    p = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    with open(p) as f:
        d = json.load(f)
    got = bench.load_traffic(bench.parse(["--size", str(d["size"]), "--count", str(d["count"])]), d["count"])
    assert (got is not None) == (d.get("kernel_src") == h)
    # the mix's record is tied to the ragged pipeline's sources, not the SCK's
    assert "icrc_rsck.hip" in bench.RAGGED_SOURCES and "icrc_rsck.hip" not in bench.SCK_SOURCES


def test_committed_traffic_matches_headline_kernel():
    """The committed PMC pass is of the headline config (1 M x 4 KiB) and of
    the SCK source at HEAD, so the default bench line carries a non-null
    roofline.traffic. An SCK edit fails this until tools/pmc_traffic.py is
    re-run on the GPU and profiles/pmc_traffic.json refreshed."""
    a = bench.parse([])
    with open(os.path.join(ROOT, "profiles", "pmc_traffic.json")) as f:
        d = json.load(f)
    assert (d["size"], d["count"]) == (a.size, 1 << 20)
    assert d["kernel_src"] == bench.kernel_source_hash()
    assert 0.99 < d["traffic_over_algorithmic"] < 1.05
    assert bench.load_traffic(a, 1 << 20) == d["hbm_bytes_per_launch"]


def test_bench_compiles_standalone():
    subprocess.check_call([sys.executable, "-m", "py_compile", os.path.join(ROOT, "bench.py")])


def test_gpus_2_relaunch_end_to_end_plan_only():
    """The real re-launch: `bench.py --gpus 2` outside torchrun starts 2 ranks
    through torch.distributed.run (rendezvous on 127.0.0.1), the ranks agree
    over gloo on the shard plan -- byte-balanced unequal shards for --mix,
    shard_range for --global-count -- and rank 0 prints one JSON line."""
    def run(*args):
        r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--plan-only", *args],
                           capture_output=True, text=True, timeout=300,
                           env={k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")})
        assert r.returncode == 0, r.stderr[-2000:]
        lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
        assert len(lines) == 1, r.stdout
        return json.loads(lines[0])

    d = run("--mix", "--count", "5000")
    assert d["n_gpus"] == 2 and d["packets_total"] == 10000 and sum(d["shard_packets"]) == 10000
    assert d["scaling"] == "weak" and abs(d["shard_bytes"][0] - d["shard_bytes"][1]) <= 2 * 4096
    d = run("--global-count", "4194304")
    assert d["scaling"] == "strong" and d["shard_packets"] == [2097152, 2097152]


def test_side_configs_are_the_baseline_configs():
    """The driver's one command also measures BASELINE's other configs
    (VERDICT r4 item 2): N = 1 adds c1 / c2 / c4, N > 1 c3_strong / c4_strong,
    each with the main run's K, W and seed."""
    a = bench.parse(["--steps", "7", "--warmup", "2", "--seed", "11"])
    got = {n: bench.side_args(a, x) for n, x in bench.SIDE_N1}
    assert set(got) == {"c1", "c2", "c4", "c3", "c4s", "ring", "ring_len"}
    # the 8-GPU run's anchors at N = 1
    assert (got["c3"].global_count, got["c3"].size, got["c3"].mix) == (4 << 20, 4096, False)
    assert got["c4s"].mix and got["c4s"].count == 524288
    assert (got["ring"].l3_offset, got["ring"].stride, got["ring"].count) == (14, 4096, 1 << 20)
    assert (got["ring_len"].l3_offset, got["ring_len"].stride, got["ring_len"].slot_lengths) == (14, 1024, (64, 1010))
    assert (got["c1"].size, got["c1"].count, got["c1"].mix) == (64, 1 << 20, False)
    assert (got["c2"].size, got["c2"].count, got["c2"].mix) == (1024, 1 << 20, False)
    assert got["c4"].mix and got["c4"].count == 4 << 20 and got["c4"].global_count is None
    for sa in got.values():
        assert (sa.steps, sa.warmup, sa.seed, sa.prime_ms, sa.no_side) == (7, 2, 11, 0.0, True)
    got = {n: bench.side_args(bench.parse(["--gpus", "8"]), x) for n, x in bench.SIDE_NX}
    assert set(got) == {"c3_strong", "c4_strong"}
    assert (got["c3_strong"].global_count, got["c3_strong"].size, got["c3_strong"].mix) == (4 << 20, 4096, False)
    assert got["c4_strong"].mix and got["c4_strong"].global_count == 4 << 20
    assert bench.side_args(bench.parse(["--side-count", "99"]), ["--mix"]).count == 99


def test_side_configs_run_at_n1_on_cpu_stand_in():
    """bench.run_side at N = 1 with the CPU stand-in backend (the oracle as
    the compute, test only): every side key carries its value, step time,
    kernel time, roofline fraction and the sampled oracle check."""
    from test_bench_dist import CpuOracleBackend

    a = bench.parse(["--steps", "2", "--warmup", "1", "--prime-ms", "0", "--warm-ms", "0", "--side-count", "1500"])
    res = bench.run_side(a, 1, 0, CpuOracleBackend(), False)
    assert set(res) == {"c1", "c2", "c4", "c3", "c4s", "ring", "ring_len"}
    assert not any("error" in d for d in res.values()), res
    for name, d in res.items():
        assert d["value"] > 0 and d["ms_per_step"] > 0 and d["oracle_sampled_all_ranks"], name
        # (frac is rounded to 4 places: a CPU stand-in on a loaded host can round to 0)
        assert d["roofline"]["frac"] >= 0 and d["roofline"]["kernel_ms"] > 0 and "traffic" in d["roofline"], name
        assert d["config"]["packets_total"] == 1500, name
    assert "mixed-MTU" in res["c4"]["metric"] and "64B" in res["c1"]["metric"] and "1024B" in res["c2"]["metric"]
    assert "fixed total" in res["c3"]["metric"] and "mixed-MTU" in res["c4s"]["metric"]
    assert "framed" in res["ring"]["metric"] and "length per slot" in res["ring_len"]["metric"]
    # the ring with a length per slot counts its packets' bytes and its lengths array
    rl = res["ring_len"]["roofline"]
    assert rl["alg_bytes_per_launch"] > 8 * 1500 and rl["alg_bytes_per_launch"] < 1500 * (1010 + 8)


def test_side_config_failure_keeps_the_main_line(monkeypatch):
    """A side config that raises is recorded as an error key (N = 1); the
    others still run (the headline must never be lost)."""
    from test_bench_dist import CpuOracleBackend

    a = bench.parse(["--steps", "1", "--warmup", "0", "--prime-ms", "0", "--warm-ms", "0", "--side-count", "600"])
    real = bench.run

    def flaky(sa, *rest):
        if sa.mix and flaky.n == 0:  # c4, the first mixed side config
            flaky.n += 1
            raise RuntimeError("out of memory (test)")
        return real(sa, *rest)
    flaky.n = 0
    monkeypatch.setattr(bench, "run", flaky)
    res = bench.run_side(a, 1, 0, CpuOracleBackend(), False)
    assert "error" in res["c4"] and "out of memory" in res["c4"]["error"]
    assert res["c1"]["value"] > 0 and res["c4s"]["value"] > 0


def test_n1_extras_carry_cpu_baseline_c0_and_e2e():
    """N = 1: cpu_baseline, C0, and the headline batch through the host route
    (e2e: host in, host out) -- on the CPU stand-in."""
    from test_bench_dist import CpuOracleBackend

    be = CpuOracleBackend()
    a = bench.parse(["--steps", "1", "--warmup", "0", "--prime-ms", "0", "--warm-ms", "0", "--count", "700",
                     "--size", "1024", "--cpu-seconds", "0.05"])
    res, full_h, b = bench.run(a, 1, 0, be, False)
    bench.n1_extras(a, be, res, full_h, b)
    assert res["cpu_baseline"]["value"] > 0 and res["c0"]["us_per_packet_ctypes_call"] > 0
    e = res["e2e"]
    assert "error" not in e, e
    assert e["value"] > 0 and e["h2d_ms"] > 0 and e["d2h_bytes"] == 4 * 700 and "ricrc_batch_host" in e["route"]
    # a ring with a length per slot: its CPU baseline takes offsets + lengths; no e2e (not the headline shape)
    a = bench.parse(["--steps", "1", "--warmup", "0", "--prime-ms", "0", "--warm-ms", "0", "--count", "500",
                     "--l3-offset", "14", "--stride", "1024", "--slot-lengths", "64:1010", "--cpu-seconds", "0.05"])
    res, full_h, b = bench.run(a, 1, 0, be, False)
    bench.n1_extras(a, be, res, full_h, b)
    assert res["cpu_baseline"]["value"] > 0 and "e2e" not in res


def test_slot_lengths_flag():
    """--slot-lengths LO:HI: a NIC ring with a completion length per slot
    (VERDICT r5 item 2), lengths uniform over [LO, HI] from the seed."""
    a = bench.parse(["--l3-offset", "14", "--stride", "1024", "--slot-lengths", "64:1010"])
    assert a.slot_lengths == (64, 1010) and a.pkt == 1010
    T, cuts, lens = bench.shard_plan(a, 1)
    assert T == 1 << 20 and cuts == [0, T] and lens.min() >= 64 and lens.max() <= 1010
    assert "(icrc_rswg_kernel)" in bench.kernel_label(a, count=a.count)  # 1 M slots: two chunks a workgroup
    assert bench.traffic_record(False, a.size, a.count, 14, 1024, (64, 1010))[0] == \
        "pmc_traffic_ring14_1024_len64-1010.json"
    for bad in (["--stride", "1024", "--slot-lengths", "64:1011", "--l3-offset", "14"],
                ["--stride", "1024", "--slot-lengths", "30:100"], ["--mix", "--slot-lengths", "64:100"],
                ["--stride", "1024", "--slot-lengths", "64"]):
        with pytest.raises(SystemExit):
            bench.parse(bad)


def test_framed_ring_flags():
    """--l3-offset / --stride: an Ethernet-framed fixed-slot ring (SURVEY
    8(f)-4); the packet is the slot minus the L3 offset."""
    a = bench.parse(["--l3-offset", "14", "--stride", "4096"])
    assert (a.l3_offset, a.stride, a.pkt) == (14, 4096, 4082)
    assert "framed" in bench.metric_for(a, a.count, a.count)
    assert bench.traffic_record(False, a.size, a.count, 14, 4096)[0] == "pmc_traffic_ring14_4096.json"
    with pytest.raises(SystemExit):
        bench.parse(["--mix", "--l3-offset", "14"])
