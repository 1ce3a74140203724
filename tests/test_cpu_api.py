"""CPU: the C-ABI library loads, exports what include/roce_icrc.h declares, and
its per-packet (CPU) entry points match the oracle.  No GPU compute here: the
batch calls are covered by tests/test_gpu_parity.py on the MI355X."""
import ctypes
import errno
import json
import os
import random
import re
import struct
import subprocess
import sys
import zlib

import numpy as np
import pytest

import icrc_oracle as O
import roce_icrc

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "roce_icrc.h")


def declared_symbols():
    text = open(HEADER).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(ricrc_[a-z_0-9]+)\s*\(", text)))


def test_header_declarations_exported():
    syms = declared_symbols()
    assert len(syms) >= 15
    lib = ctypes.CDLL(roce_icrc.LIB_PATH)
    for s in syms:
        assert hasattr(lib, s), s
    out = subprocess.run(["nm", "-D", "--defined-only", roce_icrc.LIB_PATH], capture_output=True, text=True).stdout
    for s in syms:
        assert re.search(rf"\bT {s}\b", out), f"{s} not exported as a text symbol"
    assert sorted(roce_icrc.EXPORTED) == syms


def test_library_is_gfx950_code_object():
    """The .so embeds gfx950 code objects (the HIP kernels), nothing else: every
    offload-bundle entry targets gfx950.  (Other gfx names may appear as host
    strings -- rocPRIM's architecture tables -- but not as bundle targets.)"""
    blob = open(roce_icrc.LIB_PATH, "rb").read()
    targets = set(re.findall(rb"amdgcn-amd-amdhsa--(gfx[0-9a-f]+)", blob))
    assert targets == {b"gfx950"}, targets


def test_one_matches_golden_and_random():
    meta = json.load(open(os.path.join(ROOT, "tests", "golden", "icrc_golden.json")))
    blob = open(os.path.join(ROOT, "tests", "golden", "icrc_golden.bin"), "rb").read()
    for c in meta["cases"]:
        pkt = blob[c["offset"]: c["offset"] + c["len"]]
        assert roce_icrc.icrc(pkt) == c["icrc"], c["desc"]
    rng = random.Random(9)
    for _ in range(300):
        pkt = bytes(rng.getrandbits(8) for _ in range(rng.randrange(4, 5000)))
        assert roce_icrc.icrc(pkt) == O.icrc(pkt)


def test_input_types_no_copy_paths():
    pkt = bytes.fromhex("450200301234400040110000c0a80164c0a80101457b12b7001c00001140ffff"
                        "0000001100000005000000016c1f7922")
    for v in (pkt, bytearray(pkt), memoryview(pkt), np.frombuffer(pkt, np.uint8).copy(), memoryview(bytearray(pkt))):
        assert roce_icrc.icrc(v) == 0x22791F6C


def test_verify_stamp_roundtrip():
    rng = random.Random(1)
    for n in (44, 64, 300, 1024, 4096):
        pkt = bytearray(rng.getrandbits(8) for _ in range(n))
        roce_icrc.stamp(pkt)
        assert roce_icrc.verify(pkt)
        assert O.residue_ok(bytes(pkt))
        assert struct.unpack("<I", bytes(pkt[-4:]))[0] == O.icrc(bytes(pkt))
        pkt[n - 5] ^= 0x40  # last covered byte (never a masked offset for n >= 44)
        assert not roce_icrc.verify(pkt)


def test_is_rocev2_classifier():
    pkt = bytes.fromhex("450200301234400040110000c0a80164c0a80101457b12b7001c00001140ffff"
                        "0000001100000005000000016c1f7922")
    assert roce_icrc.is_rocev2(pkt)
    bad = bytearray(pkt)
    bad[23] = 0xB8  # dport 4792
    assert not roce_icrc.is_rocev2(bad)
    bad = bytearray(pkt)
    bad[9] = 6  # TCP
    assert not roce_icrc.is_rocev2(bad)
    assert not roce_icrc.is_rocev2(pkt[:40])


def test_shift_and_combine_against_oracle_and_zlib():
    rng = random.Random(4)
    for _ in range(50):
        reg, n = rng.getrandbits(32), rng.randrange(0, 5000)
        assert roce_icrc.shift(reg, n) == O.crc_shift(reg, n) if n < 600 else True
        a = bytes(rng.getrandbits(8) for _ in range(rng.randrange(0, 300)))
        b = bytes(rng.getrandbits(8) for _ in range(rng.randrange(0, 300)))
        assert roce_icrc.combine(zlib.crc32(a), zlib.crc32(b), len(b)) == zlib.crc32(a + b)


def test_incremental_repair_after_header_rewrite():
    """The linearity the next-step 'repair' feature relies on: rewriting PSN
    (shuffle_egress.p4:665) changes the ICRC by shift(crc0(delta), tail)."""
    rng = random.Random(8)
    pkt = bytearray(rng.getrandbits(8) for _ in range(1024))
    old = roce_icrc.icrc(pkt)
    new_pkt = bytearray(pkt)
    new_pkt[37:40] = (0x123456).to_bytes(3, "big")
    delta = bytes(a ^ b for a, b in zip(pkt[:1020], new_pkt[:1020]))
    # crc0 of the delta stream (register from 0, no conditioning) = pure linear part
    reg = 0
    for byte in delta:
        reg ^= byte
        for _ in range(8):
            reg = (reg >> 1) ^ (0xEDB88320 if reg & 1 else 0)
    assert roce_icrc.icrc(new_pkt) == old ^ reg


def test_errors_never_abort():
    with pytest.raises(ValueError):
        roce_icrc.icrc(b"abc")
    assert roce_icrc.lib.ricrc_one(None, 100) == 0
    assert roce_icrc.lib.ricrc_verify_one(None, 100) == -errno.EINVAL
    assert roce_icrc.lib.ricrc_stamp_one(None, 100) == -errno.EINVAL
    assert roce_icrc.lib.ricrc_batch_host(None, None, None, None, 0, 1, 0, None) == -errno.EINVAL
    assert roce_icrc.lib.ricrc_batch_device(None, 0, None, None, None, 0, 1, 0, None, None) == -errno.EINVAL
    h = ctypes.c_void_p()
    assert roce_icrc.lib.ricrc_create(ctypes.byref(h), 0) == -errno.EINVAL
    for rc in (0, -errno.EINVAL, -errno.ENODEV, -errno.ENOMEM, -errno.EIO, -12345):
        assert roce_icrc.lib.ricrc_strerror(rc)


def test_status_entry_points_reject_bad_arguments():
    """The per-packet-status batch calls (ricrc_batch_device_st /
    ricrc_batch_host_st / ricrc_classify_device): NULL context, bad flags ->
    -EINVAL, never an abort; count 0 is a no-op only with a valid context."""
    L = roce_icrc.lib
    assert L.ricrc_batch_device_st(None, 0, None, None, None, 64, 1, 0, None, None, None, 0) == -errno.EINVAL
    assert L.ricrc_batch_host_st(None, None, None, None, 64, 1, 0, None, None, 0) == -errno.EINVAL
    assert L.ricrc_batch_host_st(None, None, None, None, 64, 1, 0, None, None, 0x400) == -errno.EINVAL
    assert L.ricrc_classify_device(None, 0, None, None, None, 64, 1, 0, None, None) == -errno.EINVAL
    assert roce_icrc.ST_OK == 0 and roce_icrc.ST_BADLEN == 1 and roce_icrc.ST_NOTROCE == 2
    text = open(HEADER).read()
    for name, v in (("RICRC_ST_OK", 0), ("RICRC_ST_BADLEN", 1), ("RICRC_ST_NOTROCE", 2),
                    ("RICRC_F_STRICT", 0x100), ("RICRC_F_VERIFY", 0x200)):
        assert re.search(rf"#define {name} {v:#x}u?\b" if v >= 0x100 else rf"#define {name} {v}\b", text), name


def test_hip_library_needs_no_newer_hip_than_torchs():
    """libroceicrc.so shares the process's HIP runtime with PyTorch-ROCm,
    whichever is loaded first -- on the GPU box that is torch's bundled
    libamdhip64 (ROCm 7.0), older than /opt/rocm's.  Every versioned HIP
    symbol the library imports must exist there (round 3 found hipStreamGetId,
    hip_7.1, missing from torch's copy: the library then fails to load)."""
    torch = pytest.importorskip("torch")
    thip = os.path.join(os.path.dirname(torch.__file__), "lib", "libamdhip64.so")
    if not os.path.exists(thip):
        pytest.skip("torch ships no libamdhip64")
    need = subprocess.run(["objdump", "-T", roce_icrc.LIB_PATH], capture_output=True, text=True).stdout
    have = subprocess.run(["nm", "-D", "--defined-only", thip], capture_output=True, text=True).stdout
    defined = set(re.findall(r"\b(hip\w+)@@?(hip_[\d.]+)", have))
    missing = [(s, v) for v, s in re.findall(r"\*UND\*\s+\S+\s+\((hip_[\d.]+)\)\s+(hip\w+)", need)
               if (s, v) not in defined]
    assert not missing, missing


def test_no_cpu_fallback_without_gpu():
    torch = pytest.importorskip("torch")
    if torch.cuda.is_available():
        pytest.skip("GPU present: the ENODEV path is not reachable")
    with pytest.raises(roce_icrc.ICRCError) as e:
        roce_icrc.Context()
    assert e.value.rc == -errno.ENODEV
    with pytest.raises(roce_icrc.ICRCError):
        roce_icrc.icrc_batch(np.zeros(4096, np.uint8), stride=4096)


def test_cpu_library_is_hip_free_and_exports_the_per_packet_section():
    """libroceicrc_cpu.so (the simulator drop-in) links nothing from ROCm, and
    importing roce_icrc for per-packet calls pulls in neither torch nor HIP."""
    out = subprocess.run(["ldd", roce_icrc.CPU_LIB_PATH], capture_output=True, text=True).stdout
    assert "amdhip" not in out and "rccl" not in out and "torch" not in out, out
    syms = subprocess.run(["nm", "-D", "--defined-only", roce_icrc.CPU_LIB_PATH], capture_output=True,
                          text=True).stdout
    for s in roce_icrc.CPU_EXPORTED:
        assert re.search(rf"\bT {s}\b", syms), s
    assert set(roce_icrc.CPU_EXPORTED) <= set(declared_symbols())
    code = ("import sys; sys.modules['torch'] = None; sys.path.insert(0, %r); import roce_icrc; "
            "p = bytes.fromhex('450200301234400040110000c0a80164c0a80101457b12b7001c00001140ffff"
            "0000001100000005000000016c1f7922'); assert roce_icrc.icrc(p) == 0x22791F6C; "
            "assert roce_icrc.verify(p); print('hip' in ' '.join(open('/proc/self/maps').read().split()))"
            % os.path.join(ROOT, "roce-test_amd"))
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    assert r.stdout.strip() == "False"  # libamdhip64 never mapped


def test_icrc_checked_length_and_classifier_contract():
    """ricrc_icrc: SURVEY §8(b)'s -EINVAL for n < 44 / n > 65535 / NULL, and
    with RICRC_F_STRICT -EPROTO for packets the ingress parser would not
    accept as RoCEv2 (shuffle_ingress_parser.p4:12-36)."""
    pkt = bytes.fromhex("450200301234400040110000c0a80164c0a80101457b12b7001c00001140ffff"
                        "0000001100000005000000016c1f7922")
    assert roce_icrc.icrc_checked(pkt) == 0x22791F6C == roce_icrc.icrc_checked(pkt, strict=True)
    assert roce_icrc.icrc_checked(pkt, family="auto", strict=True) == 0x22791F6C
    with pytest.raises(ValueError, match="-22"):
        roce_icrc.icrc_checked(pkt[:43])
    with pytest.raises(ValueError, match="-22"):
        roce_icrc.icrc_checked(bytes(65536))
    bad = bytearray(pkt)
    bad[23] ^= 1  # UDP dport != 4791
    assert roce_icrc.icrc_checked(bytes(bad)) == O.icrc(bytes(bad))  # not strict: any bytes
    with pytest.raises(ValueError, match="-71"):
        roce_icrc.icrc_checked(bytes(bad), strict=True)
    with pytest.raises(ValueError, match="-71"):
        roce_icrc.icrc_checked(pkt, family="v6", strict=True)  # an IPv4 packet
    out = ctypes.c_uint32(7)
    assert roce_icrc.cpu.ricrc_icrc(None, 100, 0, ctypes.byref(out)) == -errno.EINVAL
    assert roce_icrc.cpu.ricrc_icrc(pkt, len(pkt), 9, ctypes.byref(out)) == -errno.EINVAL
    assert out.value == 7


def test_framelen_padded_and_fcs_frames_cpu():
    """RICRC_F_FRAMELEN on the CPU entry points (ricrc_icrc, ricrc_batch_cpu)
    against the oracle's frame_l3_len restatement: the ACK known answer
    padded, with an FCS, both; RoCEv2/IPv6 with an FCS; frames whose IP
    header gives no usable length keep the descriptor's (ARP, total_len past
    the frame, total_len < 44), and a strict call still rejects those."""
    ack = bytes.fromhex("450200301234400040110000c0a80164c0a80101457b12b7001c00001140ffff"
                        "0000001100000005000000016c1f7922")
    fcs = bytes.fromhex("deadbeef")
    for tail in (bytes(2), fcs, bytes(2) + fcs, bytes(12)):
        frame = ack + tail
        assert O.frame_l3_len(frame) == len(ack)
        assert roce_icrc.icrc_checked(frame, strict=True, framelen=True) == 0x22791F6C
        with pytest.raises(ValueError, match="-71"):  # without the flag: total_len != descriptor length
            roce_icrc.icrc_checked(frame, strict=True)
    rng = np.random.default_rng(11)
    v6 = bytearray(rng.integers(0, 256, 100, dtype=np.uint8).tobytes())
    v6[0] = 0x60
    v6[4:6] = (60).to_bytes(2, "big")
    v6[6] = 17
    v6[42:44] = (4791).to_bytes(2, "big")
    assert O.frame_l3_len(bytes(v6) + fcs) == 100
    assert roce_icrc.icrc_checked(bytes(v6) + fcs, family="v6", strict=True, framelen=True) == O.icrc(bytes(v6), "v6")
    arp = bytes.fromhex("0001080006040001") + bytes(52)
    assert O.frame_l3_len(arp) == 60 and roce_icrc.icrc_checked(arp, framelen=True) == O.icrc(arp)
    long_t = bytearray(ack + fcs)
    long_t[2:4] = (200).to_bytes(2, "big")  # total_len past the frame
    short_t = bytearray(ack + fcs)
    short_t[2:4] = (40).to_bytes(2, "big")  # shorter than a RoCEv2 header
    for f in (bytes(long_t), bytes(short_t)):
        assert O.frame_l3_len(f) == len(f) and roce_icrc.icrc_checked(f, framelen=True) == O.icrc(f)
        with pytest.raises(ValueError, match="-71"):
            roce_icrc.icrc_checked(f, strict=True, framelen=True)
    # a batch of frames: lengths from the IP headers, slots of 128 bytes
    frames = [ack + bytes(2), ack + fcs, bytes(v6) + fcs, arp, bytes(long_t)]
    buf = np.zeros(128 * len(frames), np.uint8)
    for i, f in enumerate(frames):
        buf[128 * i:128 * i + len(f)] = np.frombuffer(f, np.uint8)
    lens = np.array([len(f) for f in frames], np.uint32)
    offs = np.arange(len(frames), dtype=np.uint64) * 128
    got = roce_icrc.icrc_batch_cpu(buf, offs, lens, framelen=True, family="auto")
    want = [O.icrc(f[:O.frame_l3_len(f)], "auto") for f in frames]
    np.testing.assert_array_equal(got, np.array(want, np.uint32))
