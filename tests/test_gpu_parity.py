"""GPU parity: the gfx950 kernels (through the C ABI) against the CPU oracle.

Bit-exact comparison on the same bytes: integer arithmetic, no tolerance.
Inputs are built on the host (numpy, seeded) or by the device generator,
copied where needed, and every kernel result is compared with
oracle/icrc_oracle.c (itself pinned to zlib / the golden vectors by
tests/test_oracle.py).  Covers the streaming kernel (fixed length, 16-B
aligned), the ragged kernel (offsets, ragged lengths, any alignment,
multi-window jumbo packets, Ethernet l3_offset), verify mode, the host-buffer
path, and the full BASELINE headline size (1 M x 4096 B).
"""
import numpy as np
import pytest

torch = pytest.importorskip("torch")

import oracle_c  # noqa: E402
import icrc_oracle  # noqa: E402

pytestmark = pytest.mark.gpu

SEED = 0x1CEC0DE


def _dev(a: np.ndarray):
    return torch.from_numpy(np.ascontiguousarray(a)).to("cuda")


def _out(count):
    return torch.empty(count, dtype=torch.int32, device="cuda")


def _host_u32(t):
    torch.cuda.synchronize()
    return t.cpu().numpy().view(np.uint32)


def _stream():
    return torch.cuda.current_stream()


@pytest.mark.parametrize("n", [48, 64, 128, 256, 512, 1024, 1520, 2048, 4096, 4112, 8192, 9008, 16384])
def test_stream_kernel_fixed(ctx, n):
    count = 3000 if n <= 4096 else 600
    host = oracle_c.synth_batch(SEED, 0, count, n)
    want = oracle_c.icrc_batch(host, stride=n, threads=8)
    d = _dev(host)
    out = _out(count)
    ctx.batch_device(d, count, out, stride=n, stream=_stream())
    got = _host_u32(out)
    np.testing.assert_array_equal(got, want)


@pytest.mark.parametrize("count", [1, 2, 63, 64, 65, 4097])
def test_stream_kernel_tails(ctx, count):
    """Partial last wave-steps and tiny batches (lanes past the batch)."""
    for n in (64, 1024, 4096):
        host = oracle_c.synth_batch(SEED + count, 7, count, n)
        want = oracle_c.icrc_batch(host, stride=n)
        out = _out(count)
        ctx.batch_device(_dev(host), count, out, stride=n, stream=_stream())
        np.testing.assert_array_equal(_host_u32(out), want)


def test_device_synth_matches_host_restatement(ctx):
    for n, stride in ((64, 64), (1024, 1024), (4096, 4096), (1000, 1008)):
        count = 257
        d = torch.empty(count * stride, dtype=torch.uint8, device="cuda")
        ctx.synth_device(d, SEED, 1000, count, n, stride, stream=_stream())
        torch.cuda.synchronize()
        np.testing.assert_array_equal(d.cpu().numpy().reshape(count, stride),
                                      oracle_c.synth_batch(SEED, 1000, count, n, stride))


def _ragged(rng, count, lo, hi, align, l3_offset=0):
    lens = rng.integers(lo, hi + 1, size=count).astype(np.uint32)
    offs = np.zeros(count, dtype=np.uint64)
    pos = int(rng.integers(0, 16))
    for i in range(count):
        pos += int(rng.integers(0, 40))
        if align:
            pos = (pos + align - 1) // align * align
        offs[i] = pos
        pos += int(lens[i]) + l3_offset
    buf = rng.integers(0, 256, size=pos + 64, dtype=np.uint8)
    return buf, offs, lens


@pytest.mark.parametrize("lo,hi,align", [(4, 64, 1), (44, 300, 1), (44, 4096, 4), (44, 4096, 16),
                                         (3000, 9100, 1), (9000, 20000, 1), (44, 65535, 1)])
def test_ragged_kernel_lengths(ctx, lo, hi, align):
    rng = np.random.default_rng(lo * 7 + hi)
    count = 400 if hi <= 9100 else 40
    buf, offs, lens = _ragged(rng, count, lo, hi, align)
    want = oracle_c.icrc_batch(buf, offsets=offs, lengths=lens)
    out = _out(count)
    ctx.batch_device(_dev(buf), count, out, offsets=_dev(offs), lengths=_dev(lens), stream=_stream())
    np.testing.assert_array_equal(_host_u32(out), want)


def test_ragged_kernel_ethernet_offset(ctx):
    """l3_offset = 14: L3 starts 2 bytes past a 16-byte boundary."""
    rng = np.random.default_rng(14)
    count, n = 500, 1024
    frames = rng.integers(0, 256, size=(count, n + 14 + 2), dtype=np.uint8)  # 1040-B slots
    stride = frames.shape[1]
    want = oracle_c.icrc_batch(frames, stride=stride, l3_offset=14)
    out = _out(count)
    ctx.batch_device(_dev(frames), count, out, stride=stride, l3_offset=14, stream=_stream())
    np.testing.assert_array_equal(_host_u32(out), want)


def test_ragged_kernel_invalid_lengths_status(ctx):
    """Bad descriptor lengths: the plain call writes 0 (indistinguishable from
    an ICRC of 0); the status call tells them apart (RICRC_ST_BADLEN)."""
    import roce_icrc

    buf = np.arange(256, dtype=np.uint8)
    offs = np.array([0, 16, 32, 40, 48], dtype=np.uint64)
    lens = np.array([3, 0, 100, 43, 70000], dtype=np.uint32)
    out = _out(5)
    ctx.batch_device(_dev(buf), 5, out, offsets=_dev(offs), lengths=_dev(lens), stream=_stream())
    got = _host_u32(out)
    assert got[0] == 0 and got[1] == 0 and got[4] == 0
    assert got[2] == icrc_oracle.icrc(buf[32:132].tobytes())
    assert got[3] == icrc_oracle.icrc(buf[40:83].tobytes())  # 4 <= n < 44: computed by the plain call
    st = torch.empty(5, dtype=torch.uint8, device="cuda")
    ctx.batch_device_st(_dev(buf), 5, out, st, offsets=_dev(offs), lengths=_dev(lens), stream=_stream())
    torch.cuda.synchronize()
    B, OK = roce_icrc.ST_BADLEN, roce_icrc.ST_OK
    np.testing.assert_array_equal(st.cpu().numpy(), [B, B, OK, B, B])
    np.testing.assert_array_equal(_host_u32(out), [0, 0, got[2], 0, 0])


def test_ragged_kernel_c4_mix_many_waves(ctx):
    """BASELINE C4 shape (sizes uniform over 64/256/1024/4096, packed back to
    back): enough packets that every wave owns a range and the per-wave
    64-ary searches take several rounds; plus long runs of 64-byte packets
    (64 packets in one wave step)."""
    rng = np.random.default_rng(4)
    count = 200_000
    lens = rng.choice(np.array([64, 256, 1024, 4096], np.uint32), size=count)
    lens[1000:9000] = 64
    offs = np.zeros(count, np.uint64)
    offs[1:] = np.cumsum(lens[:-1], dtype=np.uint64)
    total = int(offs[-1] + lens[-1])
    buf = np.empty(total + 64, np.uint8)
    buf[:] = rng.integers(0, 256, size=buf.size, dtype=np.uint8)
    want = oracle_c.icrc_batch(buf, offsets=offs, lengths=lens, threads=16)
    out = _out(count)
    ctx.batch_device(_dev(buf), count, out, offsets=_dev(offs), lengths=_dev(lens), stream=_stream())
    np.testing.assert_array_equal(_host_u32(out), want)


@pytest.mark.parametrize("gcost", [1, 4, 40])
def test_ragged_work_split_does_not_change_results(ctx, ctx_env, gcost):
    """The ragged fold splits weighted work (lines + a per-group cost,
    RICRC_RS_GCOST, read by ricrc_create) over its waves: other splits move
    groups between waves and descriptor blocks but give the same ICRCs, on a
    C4-shaped mix with odd starts and Ethernet framing -- on the session
    context before and after (its workspace counters must be left clean)."""
    rng = np.random.default_rng(31)
    count = 20_000
    lens = rng.choice(np.array([64, 100, 256, 1024, 1500, 4096], np.uint32), size=count)
    offs = np.zeros(count, np.uint64)
    offs[1:] = np.cumsum(lens[:-1].astype(np.uint64) + 14, dtype=np.uint64)
    buf = rng.integers(0, 256, size=int(offs[-1] + lens[-1]) + 64 + 14, dtype=np.uint8)
    want = oracle_c.icrc_batch(buf[14:], offsets=offs, lengths=lens, threads=16)
    d_buf, d_offs, d_lens = _dev(buf), _dev(offs), _dev(lens)
    for c in (ctx, ctx_env(RICRC_RS_GCOST=gcost, RICRC_RSCK_GRID=37), ctx):
        out = _out(count)
        c.batch_device(d_buf, count, out, offsets=d_offs, lengths=d_lens, l3_offset=14, stream=_stream())
        np.testing.assert_array_equal(_host_u32(out), want)


@pytest.mark.parametrize("pass_grid", [1, 3, 7])
def test_ragged_bucket_pass_blocks_of_several_rounds(ctx, ctx_env, pass_grid):
    """The bucket pass lays each pass block's packets out by class; a block
    whose packets take several rounds (more than 16 per thread) counts them
    first and re-reads them to place them (stores from the registers; blocks
    of one round build their layout in LDS).  Few pass blocks
    (RICRC_RS_PASS_GRID) force that path: every size class (one-line, 2-3
    line, long), short packets computed in the pass itself (n < 44), invalid
    lengths, odd starts, in verify mode too -- and the session context after
    (the counters must be left clean)."""
    rng = np.random.default_rng(100 + pass_grid)
    count = 30_000
    lens = rng.choice(np.array([4, 20, 43, 44, 64, 100, 256, 1024, 1500, 4096, 9000], np.uint32), size=count)
    gaps = rng.integers(0, 9, size=count).astype(np.uint64)
    offs = np.zeros(count, np.uint64)
    offs[1:] = np.cumsum(lens[:-1].astype(np.uint64) + gaps[:-1], dtype=np.uint64)
    buf = rng.integers(0, 256, size=int(offs[-1] + lens[-1]) + 64, dtype=np.uint8)
    bad = rng.choice(count, size=50, replace=False)
    lens_dev = lens.copy()
    lens_dev[bad] = 70000  # invalid: 0, as the status-less call documents
    want = oracle_c.icrc_batch(buf, offsets=offs, lengths=lens, threads=16)
    want[bad] = 0
    d_buf, d_offs, d_lens = _dev(buf), _dev(offs), _dev(lens_dev)
    for c in (ctx_env(RICRC_RS_PASS_GRID=pass_grid), ctx):
        out = _out(count)
        c.batch_device(d_buf, count, out, offsets=d_offs, lengths=d_lens, stream=_stream())
        np.testing.assert_array_equal(_host_u32(out), want)
    stamped, want_v, badset = buf.copy(), np.zeros(count, np.uint32), set(bad.tolist())
    for i in range(0, count, 97):
        if i not in badset:
            stamped[int(offs[i]) + int(lens[i]) - 4:int(offs[i]) + int(lens[i])] = np.frombuffer(
                int(want[i]).to_bytes(4, "little"), np.uint8)
            want_v[i] = 1
    out = _out(count)
    ctx_env(RICRC_RS_PASS_GRID=pass_grid).batch_device(_dev(stamped), count, out, offsets=d_offs, lengths=d_lens,
                                                       stream=_stream(), verify=True)
    np.testing.assert_array_equal(_host_u32(out), want_v)


@pytest.mark.parametrize("hi", [6000, 30000])
def test_ragged_bucket_layout_lds_or_overflow(ctx, ctx_env, hi):
    """A pass block of one round builds its layout in LDS when the layout
    fits (its packets + the padding of each class's last group <= 16384 +
    512 entries): lengths up to 6000 B span <= 48 line classes (padding <=
    336, LDS); up to 30000 B, ~235 classes whose padding overflows the LDS
    room, so the block stores from its registers and the gather reads pool
    positions.  One pass block of 16384 packets (RICRC_RS_PASS_GRID=1)."""
    rng = np.random.default_rng(hi)
    count = 16384
    lens = rng.integers(44, hi + 1, size=count).astype(np.uint32)
    offs = np.zeros(count, np.uint64)
    offs[1:] = np.cumsum(lens[:-1].astype(np.uint64) + 3, dtype=np.uint64)
    buf = rng.integers(0, 256, size=int(offs[-1] + lens[-1]) + 64, dtype=np.uint8)
    want = oracle_c.icrc_batch(buf, offsets=offs, lengths=lens, threads=16)
    d_buf, d_offs, d_lens = _dev(buf), _dev(offs), _dev(lens)
    for c in (ctx_env(RICRC_RS_PASS_GRID=1), ctx):
        out = _out(count)
        c.batch_device(d_buf, count, out, offsets=d_offs, lengths=d_lens, stream=_stream())
        np.testing.assert_array_equal(_host_u32(out), want)


def test_ragged_bucket_17_per_thread_one_round_unstaged(ctx, ctx_env):
    """a pass block of 17 packets per thread (more than 16 x 1024
    packets on one block: RICRC_RS_PASS_GRID=1, 17400 packets) whose packets
    fit one round (<= 17 x 1024) but whose layout overflows the LDS stage
    (17920 entries; ~235 line classes of lengths up to 30000 B pad their last
    groups by ~800) places its packets from the registers, and the gather
    takes its unstaged path."""
    rng = np.random.default_rng(17000)
    count = 17400
    lens = rng.integers(44, 30001, size=count).astype(np.uint32)
    offs = np.zeros(count, np.uint64)
    offs[1:] = np.cumsum(lens[:-1].astype(np.uint64) + 5, dtype=np.uint64)
    buf = rng.integers(0, 256, size=int(offs[-1] + lens[-1]) + 64, dtype=np.uint8)
    want = oracle_c.icrc_batch(buf, offsets=offs, lengths=lens, threads=16)
    d_buf, d_offs, d_lens = _dev(buf), _dev(offs), _dev(lens)
    for c in (ctx_env(RICRC_RS_PASS_GRID=1), ctx):
        out = _out(count)
        c.batch_device(d_buf, count, out, offsets=d_offs, lengths=d_lens, stream=_stream())
        np.testing.assert_array_equal(_host_u32(out), want)


@pytest.mark.parametrize("count", [3000, 30_000, 200_000, 524_288])
def test_one_line_packets_three_ways(ctx, ctx_env, count):
    """The one-line packets of a ragged batch are folded by the fold kernel
    (default: rounds of 64, one lane per packet, dealt to wave slots 0..11
    before their groups; RICRC_SMALL_SLOTS=0: to every wave by its share of
    the work), or, with
    RICRC_ONE_LINE_IN_GATHER, by the gather: for batches whose bucket pass runs
    on at most half the CUs (<= 524,288 packets: 4 per thread on <= 128
    blocks) on twice the blocks, block nblk + b folding pass block b's
    one-line packets and writing their out[i] itself ("small sides"), or with
    RICRC_NO_GATHER_SPLIT too by the pass grid's own blocks.  Every class
    (one-line, 2-3 lines, long), short packets finished in the gather
    (n < 44), invalid lengths, verify mode -- the same words all three ways
    and from the oracle."""
    import roce_icrc

    rng = np.random.default_rng(count)
    lens = rng.choice(np.array([20, 44, 60, 64, 100, 124, 256, 1024, 1500, 4096], np.uint32), size=count)
    offs = np.zeros(count, np.uint64)
    offs[1:] = np.cumsum(lens[:-1].astype(np.uint64) + rng.integers(0, 5, size=count - 1).astype(np.uint64))
    buf = rng.integers(0, 256, size=int(offs[-1] + lens[-1]) + 64, dtype=np.uint8)
    bad = rng.choice(count, size=min(40, count // 50), replace=False)
    lens_dev = lens.copy()
    lens_dev[bad] = 70000
    want = oracle_c.icrc_batch(buf, offsets=offs, lengths=lens, threads=16)
    want[bad] = 0
    d_buf, d_offs, d_lens = _dev(buf), _dev(offs), _dev(lens_dev)
    pipe = ctx_env(RICRC_NO_WG=1)  # the three-pass pipeline (default here: the workgroup-local kernel)
    sides = ctx_env(RICRC_ONE_LINE_IN_GATHER=1)
    whole = ctx_env(RICRC_ONE_LINE_IN_GATHER=1, RICRC_NO_GATHER_SPLIT=1)
    prop = ctx_env(RICRC_SMALL_SLOTS=0, RICRC_NO_WG=1)  # the fold's rounds dealt by each wave's work
    lf, li, lw = (c.launch_info(d_buf, count, offsets=d_offs, lengths=d_lens) for c in (pipe, sides, whole))
    assert lf["one_line_in"] == "fold" and lf["gather_grid"] == lf["pass_grid"]
    assert li["one_line_in"] == "gather" and li["gather_grid"] == 2 * li["pass_grid"] <= 256
    assert lw["one_line_in"] == "gather" and lw["gather_grid"] == lw["pass_grid"] == li["pass_grid"]
    for c in (pipe, sides, whole):
        assert roce_icrc.kernel_path(d_buf, count, offsets=d_offs, lengths=d_lens, ctx=c) == \
            "rsck_bucket+icrc_rsck_kernel+rsck_gather"
    assert roce_icrc.kernel_path(d_buf, count, offsets=d_offs, lengths=d_lens, ctx=ctx) == "icrc_rswg_kernel"
    for c in (ctx, pipe, sides, whole, prop):
        out = _out(count)
        c.batch_device(d_buf, count, out, offsets=d_offs, lengths=d_lens, stream=_stream())
        np.testing.assert_array_equal(_host_u32(out), want)
    stamped = buf.copy()
    want_v = np.zeros(count, np.uint32)
    for i in range(0, count, 7):
        if lens_dev[i] != 70000 and lens[i] >= 4:
            o = int(offs[i]) + int(lens[i]) - 4
            stamped[o:o + 4] = np.frombuffer(int(want[i]).to_bytes(4, "little"), np.uint8)
            want_v[i] = 1
    for c in (ctx, pipe, sides, whole):
        out = _out(count)
        c.batch_device(_dev(stamped), count, out, offsets=d_offs, lengths=d_lens, stream=_stream(), verify=True)
        got = _host_u32(out)
        np.testing.assert_array_equal(got[::7], want_v[::7])


@pytest.mark.parametrize("n", [60, 64, 65, 66, 67])
def test_one_line_half_line_waves(ctx, n):
    """One-line packets that each sit in one aligned 64-byte half line, a
    whole wave of them: the coalesced half-line path folds 4 blocks, so only
    packets of <= 60 covered bytes (n <= 64) may take it; n = 65..67 still
    sit in one half line but need a fifth block for the 0xFF prefix."""
    rng = np.random.default_rng(n)
    count = 5000
    offs = (np.arange(count, dtype=np.uint64) * 128) + (rng.integers(0, 2, size=count).astype(np.uint64) * 64)
    lens = np.full(count, n, np.uint32)
    buf = rng.integers(0, 256, size=count * 128 + 64, dtype=np.uint8)
    want = oracle_c.icrc_batch(buf, offsets=offs, lengths=lens, threads=16)
    out = _out(count)
    ctx.batch_device(_dev(buf), count, out, offsets=_dev(offs), lengths=_dev(lens), stream=_stream())
    np.testing.assert_array_equal(_host_u32(out), want)


def test_ragged_kernel_offsets_only_and_lengths_only(ctx):
    """Descriptor modes: offsets with a fixed length (stride - l3_offset), and
    per-packet lengths at a fixed stride."""
    rng = np.random.default_rng(23)
    count, stride = 3000, 1536
    frames = rng.integers(0, 256, size=count * stride + 64, dtype=np.uint8)
    perm = rng.permutation(count).astype(np.uint64)
    offs = perm * stride + 3  # scattered, odd alignment
    want = oracle_c.icrc_batch(frames, offsets=offs, lengths=np.full(count, 1000, np.uint32))
    out = _out(count)
    ctx.batch_device(_dev(frames), count, out, stride=1000, offsets=_dev(offs), stream=_stream())
    np.testing.assert_array_equal(_host_u32(out), want)
    lens = rng.integers(44, stride - 14 + 1, size=count).astype(np.uint32)
    want = oracle_c.icrc_batch(frames, lengths=lens, stride=stride, count=count, l3_offset=14)
    ctx.batch_device(_dev(frames), count, out, stride=stride, lengths=_dev(lens), l3_offset=14,
                     stream=_stream())
    np.testing.assert_array_equal(_host_u32(out), want)


def test_ragged_kernel_uniform_misaligned_stride(ctx):
    """Fixed stride with the L3 start off 16-byte alignment (no descriptors:
    arithmetic piece map), several pieces per packet, many packets."""
    rng = np.random.default_rng(9)
    for n, l3, stride in ((1500, 14, 1520), (64, 2, 80), (4096, 6, 4112)):
        count = 20000 if n < 2000 else 5000
        frames = rng.integers(0, 256, size=count * stride + 64, dtype=np.uint8)
        want = oracle_c.icrc_batch(frames, stride=stride, count=count, l3_offset=l3, threads=16)
        out = _out(count)
        ctx.batch_device(_dev(frames), count, out, stride=stride, l3_offset=l3, stream=_stream())
        np.testing.assert_array_equal(_host_u32(out), want, err_msg=f"n={n} l3={l3}")


@pytest.mark.parametrize("n", [64, 1024, 4096, 1000])
def test_verify_mode(ctx, n):
    """Stamp with the oracle, corrupt some packets, verify on the GPU."""
    count = 1000
    stride = (n + 15) // 16 * 16 if n % 16 else n
    host = oracle_c.synth_batch(SEED, 0, count, n, stride)
    icrcs = oracle_c.icrc_batch(host, stride=stride) if n == stride else \
        oracle_c.icrc_batch(host, offsets=np.arange(count, dtype=np.uint64) * stride,
                            lengths=np.full(count, n, np.uint32))
    host[:, n - 4:n] = icrcs.view(np.uint8).reshape(count, 4)
    bad = np.arange(0, count, 7)
    flip_pos = 40 + (bad * 13) % (n - 44)   # an unmasked covered byte
    host[bad, flip_pos] ^= 0x10
    out = _out(count)
    if n == stride:
        ctx.batch_device(_dev(host), count, out, stride=n, stream=_stream(), verify=True)
    else:
        ctx.batch_device(_dev(host), count, out, offsets=_dev(np.arange(count, dtype=np.uint64) * stride),
                         lengths=_dev(np.full(count, n, np.uint32)), stream=_stream(), verify=True)
    got = _host_u32(out)
    want = np.ones(count, np.uint32)
    want[bad] = 0
    np.testing.assert_array_equal(got, want)


def test_mask_invariance_on_gpu(ctx):
    """Changing tos/ttl/checksums/FECN byte must not change the device ICRC."""
    count, n = 512, 1024
    host = oracle_c.synth_batch(SEED, 0, count, n)
    out1, out2 = _out(count), _out(count)
    ctx.batch_device(_dev(host), count, out1, stride=n, stream=_stream())
    for o in icrc_oracle.MASK_OFFSETS:
        host[:, o] ^= 0x5A
    ctx.batch_device(_dev(host), count, out2, stride=n, stream=_stream())
    np.testing.assert_array_equal(_host_u32(out1), _host_u32(out2))


def test_batch_host_paths(ctx):
    rng = np.random.default_rng(5)
    count, n = 2000, 4096
    host = oracle_c.synth_batch(SEED, 0, count, n)
    np.testing.assert_array_equal(ctx.batch_host(host, stride=n), oracle_c.icrc_batch(host, stride=n))
    buf, offs, lens = _ragged(rng, 1500, 44, 4096, 1)
    np.testing.assert_array_equal(ctx.batch_host(buf, offs, lens),
                                  oracle_c.icrc_batch(buf, offsets=offs, lengths=lens))


def test_batch_host_multi_chunk_pinned_and_registered(ctx):
    """> one 256 MiB staging chunk (slot alternation), through each route:
    pageable span (parallel CPU copy), pinned span (ricrc_host_alloc, direct
    DMA) and registered span (ricrc_host_register, direct DMA)."""
    count, n = 70000, 4096  # 287 MB -> 2 chunks
    host = oracle_c.synth_batch(SEED, 7, count, n)
    want = oracle_c.icrc_batch(host, stride=n, threads=8)
    np.testing.assert_array_equal(ctx.batch_host(host, stride=n), want)
    pinned = ctx.host_alloc(host.size)
    try:
        pinned[:] = host.reshape(-1)
        np.testing.assert_array_equal(ctx.batch_host(pinned, stride=n), want)
    finally:
        ctx.host_free(pinned)
    ring = host.reshape(-1).copy()
    ctx.host_register(ring)
    try:
        np.testing.assert_array_equal(ctx.batch_host(ring, stride=n), want)
    finally:
        ctx.host_unregister(ring)


@pytest.mark.parametrize("registered", [False, True])
def test_batch_host_ring_and_gather(ctx, registered):
    """Ragged ring (ascending offsets, small gaps, Ethernet l3_offset) takes
    the span route; the same packets with shuffled offsets take the gather
    route; fixed stride with per-packet lengths takes the span route with
    device offsets.  All bit-exact."""
    rng = np.random.default_rng(11)
    buf, offs, lens = _ragged(rng, 3000, 44, 4096, 1, l3_offset=14)
    want = oracle_c.icrc_batch(buf, offsets=offs, lengths=lens, l3_offset=14)
    if registered:
        ctx.host_register(buf)
    try:
        np.testing.assert_array_equal(ctx.batch_host(buf, offs, lens, l3_offset=14), want)
        perm = rng.permutation(len(offs))
        np.testing.assert_array_equal(ctx.batch_host(buf, offs[perm], lens[perm], l3_offset=14), want[perm])
    finally:
        if registered:
            ctx.host_unregister(buf)
    stride = 2048
    count = 1000
    fr = rng.integers(0, 256, size=count * stride + 64, dtype=np.uint8)
    ln = rng.integers(44, stride - 14 + 1, size=count).astype(np.uint32)
    want = oracle_c.icrc_batch(fr, lengths=ln, stride=stride, count=count, l3_offset=14)
    np.testing.assert_array_equal(ctx.batch_host(fr, lengths=ln, stride=stride, l3_offset=14, count=count), want)
    want = oracle_c.icrc_batch(fr, stride=stride, count=count, l3_offset=14)
    np.testing.assert_array_equal(ctx.batch_host(fr, stride=stride, l3_offset=14, count=count), want)


def test_host_register_errors(ctx):
    import roce_icrc

    a = np.zeros(1 << 16, np.uint8)
    ctx.host_register(a)
    try:
        with pytest.raises(roce_icrc.ICRCError):
            ctx.host_register(a)
    finally:
        ctx.host_unregister(a)
    with pytest.raises(roce_icrc.ICRCError):
        ctx.host_unregister(a)


def test_batch_host_rejects_bad_lengths(ctx):
    import roce_icrc

    buf = np.zeros(4096, np.uint8)
    with pytest.raises(roce_icrc.ICRCError):
        ctx.batch_host(buf, offsets=np.array([0], np.uint64), lengths=np.array([43], np.uint32))


@pytest.mark.slow
def test_headline_full_size_bit_exact(ctx):
    """BASELINE headline: 1,048,576 x 4096 B generated on the device, every
    ICRC compared with the C oracle on the very same bytes (copied back)."""
    count, n = 1 << 20, 4096
    d = torch.empty(count * n, dtype=torch.uint8, device="cuda")
    ctx.synth_device(d, SEED, 0, count, n, stream=_stream())
    out = _out(count)
    ctx.batch_device(d, count, out, stride=n, stream=_stream())
    got = _host_u32(out)
    host = d.cpu().numpy()
    want = oracle_c.icrc_batch(host, stride=n, threads=16)
    np.testing.assert_array_equal(got, want)
    # size-independent check: stamping every ICRC makes every residue verify
    host_pk = host.reshape(count, n)
    host_pk[:, n - 4:] = got.view(np.uint8).reshape(count, 4)
    d.copy_(torch.from_numpy(host))
    ctx.batch_device(d, count, out, stride=n, stream=_stream(), verify=True)
    assert int(_host_u32(out).sum()) == count


@pytest.mark.slow
def test_c2_full_size_bit_exact(ctx):
    """BASELINE C2: 1,048,576 x 1024 B (the SCK's 4 KiB super-groups of four
    packets) generated on the device, every ICRC compared with the C oracle
    on the very same bytes, then every trailer stamped and verified."""
    import roce_icrc

    count, n = 1 << 20, 1024
    d = torch.empty(count * n, dtype=torch.uint8, device="cuda")
    assert roce_icrc.kernel_path(d, count, stride=n, ctx=ctx) == "icrc_sck_kernel"
    ctx.synth_device(d, SEED ^ 2, 0, count, n, stream=_stream())
    out = _out(count)
    ctx.batch_device(d, count, out, stride=n, stream=_stream())
    got = _host_u32(out)
    host = d.cpu().numpy()
    np.testing.assert_array_equal(got, oracle_c.icrc_batch(host, stride=n, threads=16))
    host.reshape(count, n)[:, n - 4:] = got.view(np.uint8).reshape(count, 4)
    d.copy_(torch.from_numpy(host))
    ctx.batch_device(d, count, out, stride=n, stream=_stream(), verify=True)
    assert int(_host_u32(out).sum()) == count


@pytest.mark.slow
def test_c3_grid_path_bit_exact(ctx):
    """The strided-chain kernel on every CU (batches past 48 groups per wave
    of 240 CUs, C3's path: 256 CUs, XCD weights 1050 / 950): 1,600,000 x
    4096 B (6.6 GB, 200,000 groups) generated on the device, every ICRC
    compared with the C oracle on the very same bytes (copied back)."""
    import roce_icrc

    count, n = 1_600_000, 4096
    d = torch.empty(count * n, dtype=torch.uint8, device="cuda")
    assert roce_icrc.kernel_path(d, count, stride=n, ctx=ctx) == "icrc_sck_kernel"
    ctx.synth_device(d, SEED ^ 3, 0, count, n, stream=_stream())
    out = _out(count)
    ctx.batch_device(d, count, out, stride=n, stream=_stream())
    got = _host_u32(out)
    want = oracle_c.icrc_batch(d.cpu().numpy(), stride=n, threads=16)
    np.testing.assert_array_equal(got, want)


@pytest.mark.slow
def test_c4_full_size_bit_exact(ctx):
    """BASELINE C4 at full size: 4,194,304 packets of 64/256/1024/4096 B
    (PCG64 on the bench seed, packed back to back, 5.7 GB) generated on the
    device -- every pass block a full round of 16 packets per thread, its
    layout staged in LDS -- every ICRC compared with the C oracle on the very
    same bytes (copied back), then every trailer stamped and verified."""
    count = 4 << 20
    lens = np.random.default_rng(SEED).choice(np.array([64, 256, 1024, 4096], np.uint32), size=count)
    offs = np.zeros(count, np.uint64)
    offs[1:] = np.cumsum(lens[:-1], dtype=np.uint64)
    total = int(offs[-1] + lens[-1])
    d = torch.empty(total, dtype=torch.uint8, device="cuda")
    d_offs, d_lens = _dev(offs), _dev(lens)
    ctx.synth_ragged_device(d, SEED, 0, count, d_offs, d_lens, stream=_stream())
    out = _out(count)
    ctx.batch_device(d, count, out, offsets=d_offs, lengths=d_lens, stream=_stream())
    got = _host_u32(out)
    host = d.cpu().numpy()
    want = oracle_c.icrc_batch(host, offsets=offs, lengths=lens, threads=16)
    np.testing.assert_array_equal(got, want)
    # size-independent check: stamping every ICRC makes every trailer verify
    tail = (offs + lens.astype(np.uint64) - 4).astype(np.int64)
    idx = (tail[:, None] + np.arange(4, dtype=np.int64)[None, :]).reshape(-1)
    host[idx] = got.view(np.uint8)
    d.copy_(torch.from_numpy(host))
    ctx.batch_device(d, count, out, offsets=d_offs, lengths=d_lens, stream=_stream(), verify=True)
    assert int(_host_u32(out).astype(np.uint64).sum()) == count


@pytest.mark.slow
@pytest.mark.parametrize("route", ["wg", "pipeline"])
@pytest.mark.parametrize("shard", ["c4s", "c4_strong_rank7"])
def test_c4_shard_full_size_bit_exact(ctx, ctx_env, shard, route):
    """C4's 8-GPU shard at full size, as bench.py builds it: the stand-in
    (--mix --count 524288: the first 524,288 packets of the bench seed's mix)
    and rank 7 of C4 strong-scaled over 8 GPUs (4 M packets cut at equal
    bytes).  Both take the workgroup-local kernel (one launch: classify, lay
    out in LDS, fold with groups claimed from an LDS counter, write out[]);
    with RICRC_NO_WG=1 the three-pass pipeline -- the bucket pass at 4
    packets per thread on <= 128 blocks, the fold kernel folding the one-line
    packets before its groups, a plain gather.  Every ICRC is compared with
    the C oracle on the very same bytes, then every trailer stamped and
    verified."""
    import bench
    import roce_icrc
    from roce_icrc.dist import byte_balanced_cuts

    T = 524288 if shard == "c4s" else 4 << 20
    lens_g = np.random.default_rng(bench.SEED).choice(np.array(bench.MIX_SIZES, np.uint32), size=T)
    lo, hi = (0, T) if shard == "c4s" else byte_balanced_cuts(lens_g, 8)[7:9]
    lens = np.ascontiguousarray(lens_g[lo:hi])
    count = len(lens)
    assert 500_000 < count < 540_000
    offs = np.zeros(count, np.uint64)
    offs[1:] = np.cumsum(lens[:-1], dtype=np.uint64)
    d = torch.empty(int(offs[-1] + lens[-1]), dtype=torch.uint8, device="cuda")
    d_offs, d_lens = _dev(offs), _dev(lens)
    if route == "pipeline":
        ctx = ctx_env(RICRC_NO_WG=1)
        assert roce_icrc.kernel_path(d, count, offsets=d_offs, lengths=d_lens, ctx=ctx) == \
            "rsck_bucket+icrc_rsck_kernel+rsck_gather"
        li = ctx.launch_info(d, count, offsets=d_offs, lengths=d_lens)
        assert li["one_line_in"] == "fold" and li["pass_unroll"] == 4 and li["pass_grid"] <= 128
    else:
        assert roce_icrc.kernel_path(d, count, offsets=d_offs, lengths=d_lens, ctx=ctx) == "icrc_rswg_kernel"
    ctx.synth_ragged_device(d, bench.SEED, lo, count, d_offs, d_lens, stream=_stream())
    out = _out(count)
    ctx.batch_device(d, count, out, offsets=d_offs, lengths=d_lens, stream=_stream())
    got = _host_u32(out)
    host = d.cpu().numpy()
    np.testing.assert_array_equal(got, oracle_c.icrc_batch(host, offsets=offs, lengths=lens, threads=16))
    tail = (offs + lens.astype(np.uint64) - 4).astype(np.int64)
    host[(tail[:, None] + np.arange(4, dtype=np.int64)[None, :]).reshape(-1)] = got.view(np.uint8)
    d.copy_(torch.from_numpy(host))
    ctx.batch_device(d, count, out, offsets=d_offs, lengths=d_lens, stream=_stream(), verify=True)
    assert int(_host_u32(out).astype(np.uint64).sum()) == count


@pytest.mark.slow
def test_ragged_more_than_4m_packets(ctx):
    """More than 256 x 1024 x 16 packets (C4's byte-balanced shards at N > 1
    hold up to 4.2 M): the bucket and gather passes read 17 packets per
    thread so every block stays one staged round -- mixed classes, every ICRC
    against the oracle."""
    rng = np.random.default_rng(4242)
    count = 4_200_000
    lens = rng.choice(np.array([64, 100, 256, 1024], np.uint32), size=count, p=[0.4, 0.3, 0.25, 0.05])
    offs = np.zeros(count, np.uint64)
    offs[1:] = np.cumsum(lens[:-1], dtype=np.uint64)
    buf = rng.integers(0, 256, size=int(offs[-1] + lens[-1]) + 64, dtype=np.uint8)
    want = oracle_c.icrc_batch(buf, offsets=offs, lengths=lens, threads=16)
    out = _out(count)
    ctx.batch_device(_dev(buf), count, out, offsets=_dev(offs), lengths=_dev(lens), stream=_stream())
    np.testing.assert_array_equal(_host_u32(out), want)


@pytest.mark.parametrize("n", [1024, 2048, 4096])
@pytest.mark.parametrize("count,grid", [(1, None), (7, None), (9, None), (8 * 16 * 64 + 3, 1),
                                         (8 * 16 * 130 + 5, 1), (8 * 16 * 200, 2), (70001, None)])
def test_strided_chain_kernel(ctx, ctx_env, n, count, grid):
    """icrc_sck_kernel (back-to-back 1/2/4 KiB packets): partial 8-packet
    groups, waves with no groups, and -- with the grid capped -- waves that
    flush their 512 LDS result slots several times; compared with the oracle
    and with the transposed kernel on the same bytes."""
    if grid is not None:
        ctx = ctx_env(RICRC_SCK_GRID=grid)
    host = oracle_c.synth_batch(SEED ^ count, 3, count, n)
    want = oracle_c.icrc_batch(host, stride=n, threads=8)
    d = _dev(host)
    out = _out(count)
    ctx.batch_device(d, count, out, stride=n, stream=_stream())
    np.testing.assert_array_equal(_host_u32(out), want)
    out2 = _out(count)
    ctx_env(RICRC_NO_SCK=1).batch_device(d, count, out2, stride=n, stream=_stream())
    np.testing.assert_array_equal(_host_u32(out2), want)


@pytest.mark.parametrize("skew", [0, 25, 50, 500, "1,10000,3,7,5000,2,9,1"])
@pytest.mark.parametrize("count,grid", [(70001, None), (8 * 16 * 200 + 3, 3), (1 << 20 | 5, None)])
def test_xcd_weighted_split(ctx_env, skew, count, grid):
    """The work split weighted by XCD (xcd_share; RICRC_XCD_SKEW parity
    weights -- the product's defaults are 25 / 50 for the SCK, 40 for the
    ragged fold -- or RICRC_XCD_WEIGHTS, eight per-XCD weights, here lopsided
    ones), from the start XCD the kernels record: any weights give
    contiguous per-wave ranges covering every group exactly once -- odd
    grids (the last workgroup even), waves with no groups, more groups than
    the grid's waves -- on 4 KiB packets and on a ragged mix."""
    env = {"RICRC_XCD_WEIGHTS": skew} if isinstance(skew, str) else {"RICRC_XCD_SKEW": skew}
    if grid is not None:
        env["RICRC_SCK_GRID"] = grid
        env["RICRC_RSCK_GRID"] = grid
    c = ctx_env(**env)
    n = 4096
    m = min(count, 200000)
    seed = SEED ^ (skew if isinstance(skew, int) else 77)
    host = oracle_c.synth_batch(seed, 11, m, n)
    want = oracle_c.icrc_batch(host, stride=n, threads=16)
    out = _out(m)
    c.batch_device(_dev(host), m, out, stride=n, stream=_stream())
    np.testing.assert_array_equal(_host_u32(out), want)
    rng = np.random.default_rng(count + (skew if isinstance(skew, int) else 77))
    lens = rng.choice(np.array([64, 256, 1024, 4096], np.uint32), size=count)
    offs = np.zeros(count, np.uint64)
    offs[1:] = np.cumsum(lens[:-1], dtype=np.uint64)
    buf = rng.integers(0, 256, size=int(offs[-1] + lens[-1]) + 64, dtype=np.uint8)
    want = oracle_c.icrc_batch(buf, offsets=offs, lengths=lens, threads=16)
    out = _out(count)
    c.batch_device(_dev(buf), count, out, offsets=_dev(offs), lengths=_dev(lens), stream=_stream())
    np.testing.assert_array_equal(_host_u32(out), want)


@pytest.mark.parametrize("grid", [None, 1])
def test_ragged_strided_chain_mixed(ctx, ctx_env, grid):
    """Ragged strided-chain path: lengths from 44 B to 9 KiB, start offsets of
    any alignment (bytes before the first packet and between packets), so every
    line-count class, the one-line classes (lane-per-packet kernel) and byte-granular
    head/tail masks occur; with the fold grid capped to one workgroup each wave
    crosses many descriptor blocks and result rounds.  Verify mode on the same
    batch with a few corrupted packets."""
    if grid is not None:
        ctx = ctx_env(RICRC_RSCK_GRID=grid)
    rng = np.random.default_rng(7)
    count = 6000
    lens = rng.integers(44, 9001, size=count).astype(np.uint32)
    pick = rng.random(count) < 0.3  # a share of the BASELINE mix sizes
    lens[pick] = rng.choice(np.array([64, 256, 1024, 4096], np.uint32), size=int(pick.sum()))
    gaps = rng.integers(0, 200, size=count).astype(np.uint64)
    offs = np.zeros(count, np.uint64)
    offs[1:] = np.cumsum(lens[:-1].astype(np.uint64) + gaps[:-1])
    offs += 37
    total = int(offs[-1] + lens[-1]) + 64
    buf = rng.integers(0, 256, size=total, dtype=np.uint8)
    want = oracle_c.icrc_batch(buf, offsets=offs, lengths=lens, threads=8)
    d, d_off, d_len = _dev(buf), _dev(offs.view(np.int64)), _dev(lens.view(np.int32))
    out = _out(count)
    ctx.batch_device(d, count, out, offsets=d_off, lengths=d_len, stream=_stream())
    np.testing.assert_array_equal(_host_u32(out), want)
    # verify: stamp every packet, corrupt every 11th in an unmasked covered byte
    stamped = buf.copy()
    for i in range(count):
        o, n = int(offs[i]), int(lens[i])
        stamped[o + n - 4:o + n] = np.frombuffer(int(want[i]).to_bytes(4, "little"), np.uint8)
    bad = np.arange(0, count, 11)
    for i in bad:
        stamped[int(offs[i]) + 41] ^= 0x01
    ctx.batch_device(_dev(stamped), count, out, offsets=d_off, lengths=d_len, stream=_stream(), verify=True)
    exp = np.ones(count, np.uint32)
    exp[bad] = 0
    np.testing.assert_array_equal(_host_u32(out), exp)


@pytest.mark.gpu
def test_ragged_strided_chain_word_aligned(ctx):
    """Word-aligned ragged batches take the fold loop with whole-word edges
    (the count pass raises a device flag for any misaligned strided-chain
    packet): starts at every multiple of 4 inside a 128-byte line (headers
    running into line 1 included), lengths multiple of 4.  Then the same batch
    with ONE packet moved off the word grid (the flag must switch the launch to
    byte-granular edges), then the aligned batch again (the flag must not
    leak from the previous launch)."""
    rng = np.random.default_rng(11)
    count = 5000
    lens = (rng.integers(11, 2300, size=count) * 4).astype(np.uint32)
    gaps = (rng.integers(0, 50, size=count) * 4).astype(np.uint64)
    offs = np.zeros(count, np.uint64)
    offs[1:] = np.cumsum(lens[:-1].astype(np.uint64) + gaps[:-1])
    offs += 4
    total = int(offs[-1] + lens[-1]) + 128
    buf = rng.integers(0, 256, size=total, dtype=np.uint8)
    d = _dev(buf)
    odd_offs = offs.copy()
    odd_offs[count // 2] += 1  # one byte later and 4 shorter: stays inside its slot
    odd_lens = lens.copy()
    odd_lens[count // 2] -= 4
    for o, l in ((offs, lens), (odd_offs, odd_lens), (offs, lens)):
        want = oracle_c.icrc_batch(buf, offsets=o, lengths=l, threads=8)
        out = _out(count)
        ctx.batch_device(d, count, out, offsets=_dev(o.view(np.int64)), lengths=_dev(l.view(np.int32)),
                         stream=_stream())
        np.testing.assert_array_equal(_host_u32(out), want)


@pytest.mark.parametrize("grid", [None, 5])
def test_ragged_fold_line_count_runs(ctx, ctx_env, grid):
    """Word-aligned runs of C4's line counts L in {2, 3, 8, 9, 32, 33} next to
    other classes, through the ragged fold (icrc_rsck_kernel: the one fold;
    round 4's timing-only fold specialized on L is gone, round 5).  Starts at
    every multiple of 4 (headers running into line 1: a second head line);
    the default grid splits each workgroup's work exactly, so groups of every
    class are cut between waves (head and tail parts, every line offset), and
    a capped grid makes each wave take many groups of mixed classes.  Verify
    mode on the same batch."""
    if grid is not None:
        ctx = ctx_env(RICRC_RSCK_GRID=grid)
    rng = np.random.default_rng(404)
    count = 40_000
    lens = rng.choice(np.array([256, 1024, 4096, 2048, 1500, 64, 300, 8192], np.uint32), size=count,
                      p=[.25, .25, .25, .05, .05, .05, .05, .05])
    lens &= ~np.uint32(3)
    gaps = (rng.integers(0, 33, size=count) * 4).astype(np.uint64)
    gaps[rng.random(count) < 0.5] = 0  # runs packed back to back too
    offs = np.zeros(count, np.uint64)
    offs[1:] = np.cumsum(lens[:-1].astype(np.uint64) + gaps[:-1])
    offs += 12
    buf = rng.integers(0, 256, size=int(offs[-1] + lens[-1]) + 128, dtype=np.uint8)
    starts = (offs & 127).astype(np.int64)
    line_counts = (starts + lens.astype(np.int64) - 4 + 127) // 128
    for L in (2, 3, 8, 9, 32, 33):
        assert (line_counts == L).sum() > 500, L
    assert ((starts > 88) & np.isin(line_counts, [2, 3, 8, 9, 32, 33])).sum() > 1000  # second head lines
    want = oracle_c.icrc_batch(buf, offsets=offs, lengths=lens, threads=16)
    d, d_off, d_len = _dev(buf), _dev(offs.view(np.int64)), _dev(lens.view(np.int32))
    out = _out(count)
    ctx.batch_device(d, count, out, offsets=d_off, lengths=d_len, stream=_stream())
    np.testing.assert_array_equal(_host_u32(out), want)
    stamped = buf.copy()
    for i in range(0, count, 3):
        o, n = int(offs[i]), int(lens[i])
        stamped[o + n - 4:o + n] = np.frombuffer(int(want[i]).to_bytes(4, "little"), np.uint8)
    exp = np.zeros(count, np.uint32)
    exp[::3] = 1
    ctx.batch_device(_dev(stamped), count, out, offsets=d_off, lengths=d_len, stream=_stream(), verify=True)
    np.testing.assert_array_equal(_host_u32(out), exp)


def test_ragged_workspace_reuse_across_sizes_and_streams(ctx):
    """The ragged path's context-owned workspaces (one per stream, grown on
    demand, class counters re-zeroed by the last pass of every call): calls of
    growing and shrinking sizes on one stream, then interleaved on two more
    streams, all bit-exact."""
    rng = np.random.default_rng(77)
    cases = []
    for count in (500, 20000, 3, 70000, 1000):
        lens = rng.choice([64, 256, 1024, 4096, 61, 333], count).astype(np.uint32)
        offs = np.zeros(count, np.uint64)
        offs[1:] = np.cumsum(lens[:-1].astype(np.uint64) + 3)
        buf = rng.integers(0, 256, int(offs[-1]) + int(lens[-1]) + 16, dtype=np.uint8)
        cases.append((buf, offs, lens, oracle_c.icrc_batch(buf, offsets=offs, lengths=lens, threads=8)))
    streams = [torch.cuda.current_stream(), torch.cuda.Stream(), torch.cuda.Stream()]
    for rep in range(2):
        for k, (buf, offs, lens, want) in enumerate(cases):
            st = streams[0] if rep == 0 else streams[k % 3]
            out = _out(len(lens))
            with torch.cuda.stream(st):
                ctx.batch_device(_dev(buf), len(lens), out, offsets=_dev(offs), lengths=_dev(lens), stream=st)
            st.synchronize()
            np.testing.assert_array_equal(out.cpu().numpy().view(np.uint32), want)


@pytest.mark.parametrize("count", [1, 15, 16, 17, 63, 64, 65, 255, 256, 257, 4096 * 4 + 3, 1 << 20])
def test_quad_kernel_64B(ctx, ctx_env, count):
    """icrc_quad_kernel (back-to-back 64-byte packets, 4 lanes per packet,
    coalesced 1 KiB loads): partial loads, partial 4 KiB steps, partial
    rounds of result slots, waves with several rounds (C1's 1 M), verify
    mode with corruptions; and the direct kernel (RICRC_NO_QUAD) agrees."""
    n = 64
    host = oracle_c.synth_batch(SEED + count, 5, count, n)
    want = oracle_c.icrc_batch(host, stride=n, threads=16)
    d = _dev(host)
    out = _out(count)
    ctx.batch_device(d, count, out, stride=n, stream=_stream())
    np.testing.assert_array_equal(_host_u32(out), want)
    if count in (257, 4096 * 4 + 3):
        out2 = _out(count)
        ctx_env(RICRC_NO_QUAD=1).batch_device(d, count, out2, stride=n, stream=_stream())
        np.testing.assert_array_equal(_host_u32(out2), want)
    host[:, n - 4:] = want.view(np.uint8).reshape(count, 4)
    bad = np.arange(0, count, 5)
    host[bad, 40 + bad % 20] ^= 0x04
    ctx.batch_device(_dev(host), count, out, stride=n, stream=_stream(), verify=True)
    w = np.ones(count, np.uint32)
    w[bad] = 0
    np.testing.assert_array_equal(_host_u32(out), w)


@pytest.mark.parametrize("case", ["c4_64B_aligned", "mixed_starts", "one_spoiler_per_wave", "end_at_half_line_end"])
def test_one_line_packets_half_line_path(ctx, case):
    """The one-line kernel's coalesced half-line path (C4's 64-byte packets,
    64-byte aligned: every covered byte in one aligned 64-byte half line whose
    last unit holds the covered end) against the oracle, and waves where that
    condition fails for some lanes (start 4 bytes in, covered end exactly at
    the half line's end, one packet per 64 spoiling its wave) taking the
    per-lane path -- mixed with bigger packets so the classes interleave."""
    rng = np.random.default_rng(hash(case) & 0xFFFF)
    count = 40_000
    lens = rng.choice(np.array([64, 64, 64, 1024, 256], np.uint32), size=count)
    starts = np.zeros(count, np.uint64)
    if case == "mixed_starts":
        lens = np.where(lens == 64, rng.choice(np.array([53, 56, 60, 64], np.uint32), size=count), lens)
        starts = rng.choice(np.array([0, 0, 4], np.uint64), size=count)
    elif case == "one_spoiler_per_wave":
        starts[::64] = 2
    elif case == "end_at_half_line_end":
        lens = np.where(lens == 64, np.uint32(68), lens)  # covered end 64: the half line's last byte
    offs = np.zeros(count, np.uint64)
    pos = 0
    for i in range(count):  # each packet at a 64-byte boundary (+ its start offset)
        pos = (pos + 63) // 64 * 64
        offs[i] = pos + int(starts[i])
        pos = int(offs[i]) + int(lens[i])
    buf = rng.integers(0, 256, size=pos + 128, dtype=np.uint8)
    want = oracle_c.icrc_batch(buf, offsets=offs, lengths=lens, threads=16)
    out = _out(count)
    ctx.batch_device(_dev(buf), count, out, offsets=_dev(offs), lengths=_dev(lens), stream=_stream())
    np.testing.assert_array_equal(_host_u32(out), want)
