"""GPU: the workgroup-local ragged kernel (icrc_rsck.hip, icrc_rswg_kernel).

Batches of up to one chunk of 2304 packets per workgroup (C4's 8-GPU shard:
524,288 packets on 256 CUs) take the whole ragged path in one launch: each
workgroup classifies its contiguous range, lays the descriptors out in LDS
(one-line classes, then the big classes by descending line count), folds them
-- one-line packets one lane each, groups of 8 equal-L packets claimed from an
LDS counter -- and writes out[] from the layout.  Every test compares the
kernel with the C oracle and with the three-pass pipeline (RICRC_NO_WG=1) on
the same bytes; chunking (a workgroup taking its range in several chunks) is
forced with RICRC_WG_CHUNKS and a capped grid (RICRC_RSCK_GRID)."""
import numpy as np
import pytest

torch = pytest.importorskip("torch")

import oracle_c  # noqa: E402
import roce_icrc  # noqa: E402

pytestmark = pytest.mark.gpu


def _dev(a):
    a = np.ascontiguousarray(a)
    if a.dtype == np.uint64:
        a = a.view(np.int64)
    elif a.dtype == np.uint32:
        a = a.view(np.int32)
    return torch.from_numpy(a).cuda()


def _out(n):
    return torch.full((max(n, 1),), -1, dtype=torch.int32, device="cuda")


def _host(t, n):
    torch.cuda.synchronize()
    return t[:n].cpu().numpy().view(np.uint32)


def _batch(seed, count, sizes=None, lo=20, hi=9000, gap=64, align=1, base_pad=0):
    rng = np.random.default_rng(seed)
    if sizes is not None:
        lens = rng.choice(np.array(sizes, np.uint32), size=count)
    else:
        lens = rng.integers(lo, hi + 1, size=count).astype(np.uint32)
    gaps = (rng.integers(0, gap + 1, size=count) // align * align).astype(np.uint64)
    offs = np.zeros(count, np.uint64)
    if count > 1:
        offs[1:] = np.cumsum(lens[:-1].astype(np.uint64) + gaps[:-1])
    offs += base_pad
    buf = rng.integers(0, 256, size=int(offs[-1] + lens[-1]) + 128, dtype=np.uint8)
    return buf, offs, lens


def _check(ctx, pipe, buf, offs, lens, want=None, **kw):
    count = len(lens)
    if want is None:
        want = oracle_c.icrc_batch(buf, offsets=offs, lengths=np.where(lens > 65535, 0, lens).astype(np.uint32),
                                   threads=16)
    d, d_off, d_len = _dev(buf), _dev(offs), _dev(lens)
    got = []
    for c in (ctx, pipe):
        out = _out(count)
        c.batch_device(d, count, out, offsets=d_off, lengths=d_len, **kw)
        got.append(_host(out, count))
    np.testing.assert_array_equal(got[0], want)
    np.testing.assert_array_equal(got[1], want)
    return want


@pytest.fixture
def pipe(ctx_env):
    return ctx_env(RICRC_NO_WG=1)


@pytest.mark.parametrize("count", [1, 7, 8, 9, 63, 65, 2304, 3001, 70_001, 300_000])
def test_wg_mixed_lengths_any_alignment(ctx, pipe, count):
    """Lengths 20..9000 at any byte offset (the byte-granular edges), invalid
    and short packets included (n < 44: computed when out[] is written)."""
    buf, offs, lens = _batch(count, count, lo=20, hi=9000, gap=37, base_pad=5)
    if count > 50:
        bad = np.random.default_rng(count).choice(count, size=count // 50, replace=False)
        lens[bad[: len(bad) // 2]] = 70000
        lens[bad[len(bad) // 2:]] = 2
    assert roce_icrc.kernel_path(_dev(buf), count, offsets=_dev(offs), lengths=_dev(lens), ctx=ctx) == \
        "icrc_rswg_kernel"
    _check(ctx, pipe, buf, offs, lens)


@pytest.mark.parametrize("count", [4000, 131_072, 524_288])
def test_wg_c4_mix_word_aligned(ctx, pipe, count):
    """C4's sizes packed back to back (every start and end on a word: the
    whole-word edges), the shard's size included."""
    buf, offs, lens = _batch(1000 + count, count, sizes=[64, 256, 1024, 4096], gap=0)
    _check(ctx, pipe, buf, offs, lens)


def test_wg_every_line_count(ctx, pipe):
    """Lengths 44..65535: hundreds of line-count classes in one workgroup's
    chunk (runs of one group or less), the run lookup crossing many runs."""
    buf, offs, lens = _batch(5, 20_000, lo=44, hi=65535, gap=3)
    _check(ctx, pipe, buf, offs, lens)


@pytest.mark.parametrize("grid,count", [(1, 5000), (3, 20_000), (7, 100_000)])
def test_wg_chunks(ctx_env, pipe, grid, count):
    """A workgroup taking its range in several chunks of 2304 packets (a grid
    capped to a few workgroups, RICRC_WG_CHUNKS raised so the kernel is taken)."""
    wg = ctx_env(RICRC_RSCK_GRID=grid, RICRC_WG_CHUNKS=64)
    buf, offs, lens = _batch(grid * 7 + count, count, sizes=[64, 100, 256, 333, 1024, 1500, 4096], gap=9)
    assert roce_icrc.kernel_path(_dev(buf), count, offsets=_dev(offs), lengths=_dev(lens), ctx=wg) == \
        "icrc_rswg_kernel"
    _check(wg, pipe, buf, offs, lens)


def test_wg_large_batch_multi_chunk(ctx_env, pipe):
    """1 M packets on every CU with RICRC_WG_CHUNKS=8: two chunks per workgroup."""
    wg = ctx_env(RICRC_WG_CHUNKS=8)
    buf, offs, lens = _batch(77, 1 << 20, sizes=[64, 256, 1024, 1500], gap=0)
    _check(wg, pipe, buf, offs, lens)


@pytest.mark.parametrize("slot,lo,hi", [(1024, 64, 1010), (2048, 64, 2034), (1024, 200, 200)])
def test_wg_ring_slots_with_lengths(ctx, pipe, slot, lo, hi):
    """A NIC ring of fixed slots with a length per slot (no offsets array),
    the L3 packet at 14: byte-granular heads and tails."""
    count, l3 = 200_000, 14
    rng = np.random.default_rng(slot + lo)
    frames = rng.integers(0, 256, size=count * slot + 256, dtype=np.uint8)
    lens = rng.integers(lo, hi + 1, size=count).astype(np.uint32)
    want = oracle_c.icrc_batch(frames, lengths=lens, stride=slot, count=count, l3_offset=l3, threads=16)
    d, d_len = _dev(frames), _dev(lens)
    assert roce_icrc.kernel_path(d, count, stride=slot, lengths=d_len, l3_offset=l3, ctx=ctx) == "icrc_rswg_kernel"
    for c in (ctx, pipe):
        out = _out(count)
        c.batch_device(d, count, out, stride=slot, lengths=d_len, l3_offset=l3)
        np.testing.assert_array_equal(_host(out, count), want)


def test_wg_offsets_only_and_fixed(ctx, pipe):
    """Offsets with one length for all (no lengths array), and a misaligned
    fixed stride (neither array): both ragged, both through the kernel."""
    count = 30_000
    rng = np.random.default_rng(9)
    n = 700
    offs = np.arange(count, dtype=np.uint64) * 701  # byte-misaligned starts
    buf = rng.integers(0, 256, size=int(offs[-1]) + n + 64, dtype=np.uint8)
    want = oracle_c.icrc_batch(buf, offsets=offs, lengths=np.full(count, n, np.uint32), threads=16)
    d = _dev(buf)
    for c in (ctx, pipe):
        out = _out(count)
        c.batch_device(d, count, out, offsets=_dev(offs), stride=n)
        np.testing.assert_array_equal(_host(out, count), want)
    stride, l3 = 712, 6  # 16-byte multiple, misaligned L3: the ragged route
    frames = rng.integers(0, 256, size=count * stride + 64, dtype=np.uint8)
    want = oracle_c.icrc_batch(frames, stride=stride, count=count, l3_offset=l3, threads=16)
    d = _dev(frames)
    assert roce_icrc.kernel_path(d, count, stride=stride, l3_offset=l3, ctx=ctx) == "icrc_rswg_kernel"
    for c in (ctx, pipe):
        out = _out(count)
        c.batch_device(d, count, out, stride=stride, l3_offset=l3)
        np.testing.assert_array_equal(_host(out, count), want)


def test_wg_verify_mode(ctx, pipe):
    """Verify mode: stamped trailers give 1, corrupted packets 0 (short
    packets included: verified when out[] is written)."""
    buf, offs, lens = _batch(31, 50_000, sizes=[30, 64, 256, 1024, 1500, 4096], gap=5)
    want = oracle_c.icrc_batch(buf, offsets=offs, lengths=lens, threads=16)
    for i in range(len(lens)):
        o, n = int(offs[i]), int(lens[i])
        buf[o + n - 4:o + n] = np.frombuffer(int(want[i]).to_bytes(4, "little"), np.uint8)
    bad = np.arange(0, len(lens), 13)
    for i in bad:
        buf[int(offs[i]) + 42 if lens[i] > 46 else int(offs[i]) + 5] ^= 0x10
    exp = np.ones(len(lens), np.uint32)
    exp[bad] = 0
    _check(ctx, pipe, buf, offs, lens, want=exp, verify=True)


def test_wg_status_and_strict_calls(ctx, pipe):
    """The status call (the device pre-pass and status kernel around the
    ragged path) gives the same words and statuses through both routes."""
    buf, offs, lens = _batch(41, 40_000, sizes=[20, 64, 256, 1024, 70000], gap=3)
    count = len(lens)
    d, d_off, d_len = _dev(buf), _dev(offs), _dev(lens)
    res = []
    for c in (ctx, pipe):
        out = _out(count)
        st = torch.full((count,), 255, dtype=torch.uint8, device="cuda")
        c.batch_device_st(d, count, out, st, offsets=d_off, lengths=d_len)
        torch.cuda.synchronize()
        res.append((out.cpu().numpy().view(np.uint32), st.cpu().numpy()))
    np.testing.assert_array_equal(res[0][0], res[1][0])
    np.testing.assert_array_equal(res[0][1], res[1][1])
    ok = res[0][1] == roce_icrc.ST_OK
    want = oracle_c.icrc_batch(buf, offsets=offs, lengths=np.where(lens > 65535, 0, lens).astype(np.uint32),
                               threads=16)
    np.testing.assert_array_equal(res[0][0][ok], want[ok])


def test_wg_streams_back_to_back(ctx):
    """No workspace: calls of different sizes back to back on two streams."""
    streams = [torch.cuda.current_stream(), torch.cuda.Stream()]
    cases = [_batch(100 + k, n, sizes=[64, 256, 1500, 4096], gap=7) for k, n in enumerate((3, 40_000, 1000, 9000))]
    outs = []
    for k, (buf, offs, lens) in enumerate(cases):
        st = streams[k % 2]
        out = _out(len(lens))
        with torch.cuda.stream(st):
            ctx.batch_device(_dev(buf), len(lens), out, offsets=_dev(offs), lengths=_dev(lens), stream=st)
        outs.append(out)
    torch.cuda.synchronize()
    for (buf, offs, lens), out in zip(cases, outs):
        np.testing.assert_array_equal(_host(out, len(lens)), oracle_c.icrc_batch(buf, offsets=offs, lengths=lens,
                                                                                 threads=16))
