"""The C ABI from compiled C / C++ callers (examples/): the
per-packet wire crossing against the HIP-free libroceicrc_cpu.so, and a NIC
ring of Ethernet frames through ricrc_batch_host against libroceicrc.so.
Built by examples/Makefile (also run by __graft_entry__.build())."""
import os
import re
import subprocess

import pytest

import icrc_oracle

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
EX = os.path.join(ROOT, "examples")


def _build():
    subprocess.run(["make", "-s", "-C", EX], check=True, capture_output=True, text=True)


def _crossing_packet():
    """The packet examples/cpu_crossing.c builds (before stamping)."""
    n = 1024
    p = bytearray(n)
    p[0], p[2], p[3], p[4], p[5], p[6], p[8], p[9] = 0x45, n >> 8, n & 0xFF, 0x12, 0x34, 0x40, 64, 17
    p[12:16] = bytes([192, 168, 1, 100])
    p[16:20] = bytes([192, 168, 1, 200])
    p[20], p[22], p[23], p[24], p[25] = 0xC0, 4791 >> 8, 4791 & 0xFF, (n - 20) >> 8, (n - 20) & 0xFF
    p[28], p[30], p[31], p[35], p[39] = 0x04, 0xFF, 0xFF, 0x11, 7
    for i in range(40, n - 4):
        p[i] = (i * 131 + 7) & 0xFF
    return bytes(p)


def test_c_caller_per_packet_crossing():
    _build()
    r = subprocess.run([os.path.join(EX, "cpu_crossing")], capture_output=True, text=True, timeout=60)
    assert r.returncode == 0, r.stderr
    assert r.stdout.strip().endswith("ok")
    got = int(re.search(r"icrc 0x([0-9a-f]{8})", r.stdout).group(1), 16)
    assert got == icrc_oracle.icrc(_crossing_packet())
    # the C program links only the HIP-free library
    deps = subprocess.run(["ldd", os.path.join(EX, "cpu_crossing")], capture_output=True, text=True).stdout
    assert "libroceicrc_cpu.so" in deps and "amdhip" not in deps


def test_cpp_caller_without_gpu_gets_enodev():
    """No CPU fallback for batch calls: without a GPU the ring program gets
    -ENODEV from ricrc_create and says so (exit 2)."""
    import torch

    if torch.cuda.device_count() > 0:  # counting devices does not initialise the GPU
        pytest.skip("a GPU is visible: tests/test_examples.py::test_cpp_caller_nic_ring covers it")
    _build()
    r = subprocess.run([os.path.join(EX, "nic_ring"), "100"], capture_output=True, text=True, timeout=120)
    assert r.returncode == 2 and "no GPU" in r.stdout, (r.returncode, r.stdout, r.stderr)


@pytest.mark.gpu
def test_cpp_caller_nic_ring():
    """Mixed-size Ethernet frames in a pinned ring, one ricrc_batch_host call,
    every ICRC equal to the per-packet CPU call; a bad frame length -EINVAL."""
    exe = os.path.join(EX, "nic_ring")
    assert os.path.exists(exe), "examples/nic_ring is built by __graft_entry__.build() / make -C examples"
    r = subprocess.run([exe, "200000"], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, (r.stdout, r.stderr)
    assert r.stdout.strip().endswith("ok")
