"""CPU: the batch dispatch (icrc_api.cpp choose_path), through
ricrc_kernel_path -- the same decision the launch makes, queried without a
GPU (the dispatch table).  Addresses are plain integers: only
their alignment and whether a descriptor array is given matter here."""
import pytest

roce_icrc = pytest.importorskip("roce_icrc")

BASE = 1 << 20  # 16-byte aligned
OFF, LEN = 0x10000, 0x20000  # "some device array"


def path(count=1000, **kw):
    base = kw.pop("base", BASE)
    return roce_icrc.kernel_path(base, count, **kw)


def test_fixed_size_batches():
    assert path(stride=4096) == "icrc_sck_kernel"
    assert path(stride=2048) == "icrc_sck_kernel"
    assert path(stride=1024) == "icrc_sck_kernel"
    assert path(stride=64) == "icrc_quad_kernel"
    assert path(stride=256) == "icrc_tsk_kernel"
    assert path(stride=1500 + 4) == "icrc_stream_kernel"  # 16-byte aligned stride, other length
    assert path(stride=4096, family="v6") == "icrc_sck_kernel"  # native masks
    assert path(stride=64, family="v6") == "icrc_quad_kernel+family_fix_kernel"


def test_framed_rings_full_slots():
    for slot in (1024, 2048, 4096):
        for l3 in (1, 14, 18, 22, 92):
            assert path(stride=slot, l3_offset=l3) == "icrc_sck_kernel", (slot, l3)
    assert path(stride=4096, l3_offset=93).startswith("rsck_bucket")  # a mask byte past line 0
    assert path(stride=1536, l3_offset=14).startswith("rsck_bucket")
    assert path(base=BASE + 2, stride=4096, l3_offset=14).startswith("rsck_bucket")
    assert path(stride=4096, l3_offset=14, family="auto") == "icrc_sck_kernel+family_fix_kernel"


def test_rings_with_slot_lengths():
    """Per-slot lengths: the ragged pipeline buckets them by line count (a
    strided-chain variant that stops each lane at its packet's end measured
    no faster overall; profiles/r05/NOTES.md)."""
    for slot in (1024, 2048, 4096):
        assert path(stride=slot, l3_offset=14, lengths=LEN).startswith("rsck_bucket")
    assert path(stride=4096, lengths=LEN, offsets=OFF).startswith("rsck_bucket")


def test_ragged_batches():
    """The fold kernel takes the one-line packets at every size (a separate
    one-line kernel only under RICRC_ONE_LINE_IN_GATHER=1 beyond 524,288 packets,
    tests/test_gpu_parity.py)."""
    assert path(count=4 << 20, offsets=OFF, lengths=LEN) == "rsck_bucket+icrc_rsck_kernel+rsck_gather"
    assert path(count=524288, offsets=OFF, lengths=LEN) == "rsck_bucket+icrc_rsck_kernel+rsck_gather"
