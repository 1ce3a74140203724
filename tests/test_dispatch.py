"""CPU: the batch dispatch (icrc_api.cpp choose_path), through
ricrc_kernel_path -- the same decision the launch makes, queried without a
GPU (the dispatch table).  Addresses are plain integers: only
their alignment and whether a descriptor array is given matter here."""
import pytest

roce_icrc = pytest.importorskip("roce_icrc")

BASE = 1 << 20  # 16-byte aligned
OFF, LEN = 0x10000, 0x20000  # "some device array"
RAGGED = ("rsck_bucket", "icrc_rswg_kernel")  # the three-pass pipeline, or its one-launch workgroup-local form


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
    assert path(stride=4096, l3_offset=93).startswith(RAGGED)  # a mask byte past line 0
    assert path(stride=1536, l3_offset=14).startswith(RAGGED)
    assert path(base=BASE + 2, stride=4096, l3_offset=14).startswith(RAGGED)
    assert path(stride=4096, l3_offset=14, family="auto") == "icrc_sck_kernel+family_fix_kernel"


def test_rings_with_slot_lengths():
    """Per-slot lengths: the ragged pipeline buckets them by line count (a
    strided-chain variant that stops each lane at its packet's end measured
    no faster overall; profiles/r05/NOTES.md)."""
    for slot in (1024, 2048, 4096):
        assert path(stride=slot, l3_offset=14, lengths=LEN).startswith(RAGGED)
    assert path(stride=4096, lengths=LEN, offsets=OFF).startswith(RAGGED)


def test_ragged_batches():
    """The fold kernel takes the one-line packets at every size (a separate
    one-line kernel only under RICRC_ONE_LINE_IN_GATHER=1 beyond 524,288 packets,
    tests/test_gpu_parity.py)."""
    assert path(count=4 << 20, offsets=OFF, lengths=LEN) == "icrc_rswg_kernel"  # C4: eight chunks a workgroup
    assert path(count=8 << 20, offsets=OFF, lengths=LEN) == "rsck_bucket+icrc_rsck_kernel+rsck_gather"
    # up to one chunk of 2304 packets per workgroup (C4's 8-GPU shard): one launch, workgroup-local
    assert path(count=524288, offsets=OFF, lengths=LEN) == "icrc_rswg_kernel"
    assert path(count=540_000, offsets=OFF, lengths=LEN) == "icrc_rswg_kernel"  # C4 strong, its largest rank
    assert path(count=1 << 20, stride=1024, l3_offset=14, lengths=LEN) == "icrc_rswg_kernel"  # 1 M ring slots: 2 chunks
    assert path(count=8 << 20, stride=1024, l3_offset=14, lengths=LEN).startswith("rsck_bucket")  # 8 M: the pipeline
    assert path(count=3, offsets=OFF, lengths=LEN) == "icrc_rswg_kernel"


def test_launch_info_reports_every_path():
    """ricrc_launch_info names the grid and the lanes per packet of every
    kernel path, so a C1 regression is attributable from
    the bench line; ctx = NULL: the dispatch on a 256-CU MI355X."""
    li = lambda count, **kw: roce_icrc.launch_info(BASE, count, **kw)  # noqa: E731
    c1 = li(1 << 20, stride=64)  # C1: 1 M x 64 B, the quad kernel
    assert c1["grid"] == 256 and c1["lanes_per_packet"] == 4
    assert li(1000, stride=64)["grid"] == 1  # 1000 packets: one 4 KiB wave step per 64 packets, 16 waves
    tsk = li(1 << 20, stride=256)
    assert tsk["grid"] == 256 and tsk["lanes_per_packet"] == 8
    st = li(1 << 20, stride=1504)  # the direct streaming kernel: 1500-byte chunks over 64-byte lanes
    assert st["grid"] == 256 and st["lanes_per_packet"] == 32
    head = li(1 << 20, stride=4096)  # the headline: 240 of 256 CUs, XCD-weighted
    assert head["grid"] == 240 and head["lanes_per_packet"] == 8 and head["xcd_weights"][0] > head["xcd_weights"][1]
    rag = li(8 << 20, offsets=OFF, lengths=LEN)  # past eight chunks a workgroup: the three-pass pipeline
    assert rag["grid"] == 256 and rag["pass_grid"] == 256 and rag["one_line_in"] == "fold"
    assert rag["lanes_per_packet"] == 8
    wg = li(4 << 20, offsets=OFF, lengths=LEN)  # C4: the workgroup-local kernel, no bucket / gather passes
    assert wg["grid"] == 256 and "pass_grid" not in wg and wg["passes"] == 1 and wg["one_line_in"] == "fold"
    with pytest.raises(roce_icrc.ICRCError):
        li(0, stride=64)
