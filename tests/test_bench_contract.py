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


def test_metric_matches_baseline_json():
    with open(os.path.join(ROOT, "BASELINE.json")) as f:
        assert json.load(f)["metric"] == bench.METRIC


def test_kernel_labels_follow_the_dispatch():
    assert "icrc_sck_kernel" in bench.kernel_label(4096)
    assert "icrc_sck_kernel" in bench.kernel_label(1024)
    assert "icrc_tsk_kernel" in bench.kernel_label(256)
    assert "icrc_tsk_kernel" not in bench.kernel_label(64)


def test_traffic_is_tied_to_the_kernel_source(tmp_path):
    h = bench.kernel_source_hash()
    assert len(h) == 16 and h == bench.kernel_source_hash()
    # profiles/pmc_traffic.json is only reported for the source it was measured on
    p = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    with open(p) as f:
        d = json.load(f)
    got = bench.load_traffic(d["size"], d["count"])
    assert (got is not None) == (d.get("kernel_src") == h)


def test_bench_compiles_standalone():
    subprocess.check_call([sys.executable, "-m", "py_compile", os.path.join(ROOT, "bench.py")])
