"""GPU: the buffer-extent contract of the batch calls.

The caller owns every buffer (the reference's huge_malloc MRs,
common/huge_malloc.h:12-22) and the plain device calls read packets in place
with no extent: include/roce_icrc.h states that a descriptor past the
caller's allocation is the caller's fault.  The extent-checked calls take the
buffer's size: ricrc_batch_host_bounded returns -EINVAL (status NULL) or
RICRC_ST_BADLEN per packet, ricrc_batch_device_bounded reports
RICRC_ST_BADLEN with out = 0 and never reads the packet; ricrc_batch_host
itself checks descriptors against a ricrc_host_alloc'd buffer's size.

What each test can see: on the device call the status pass sets out[i] = 0
for every RICRC_ST_BADLEN packet whatever was read, so the device tests check
statuses and the other packets' ICRCs (the device buffer is allocated larger
than the extent declared: a stray read there is neither a fault nor visible).
That no byte past the extent is READ is asserted on the host route, whose
buffer ends at a PROT_NONE guard page: a read past it is a SIGSEGV."""
import ctypes
import errno
import mmap

import numpy as np
import pytest

torch = pytest.importorskip("torch")

import icrc_oracle as O  # noqa: E402
import oracle_c  # noqa: E402
import roce_icrc  # noqa: E402

pytestmark = pytest.mark.gpu


def _ragged(count, seed, slack=0):
    rng = np.random.default_rng(seed)
    lens = rng.choice(np.array([64, 256, 1024, 1500, 4096], np.uint32), size=count)
    gaps = rng.integers(0, 8, size=count).astype(np.uint64) * 4
    offs = np.zeros(count, np.uint64)
    offs[1:] = np.cumsum(lens[:-1].astype(np.uint64) + gaps[:-1])
    buf = rng.integers(0, 256, size=int(offs[-1] + lens[-1]) + slack, dtype=np.uint8)
    return buf, offs, lens


def test_batch_host_bounded_rejects_descriptor_past_end(ctx):
    buf, offs, lens = _ragged(5000, 1)
    extent = int(offs[-1] + lens[-1])
    want = oracle_c.icrc_batch(buf, offsets=offs, lengths=lens, threads=16)
    np.testing.assert_array_equal(ctx.batch_host_bounded(buf, extent, offsets=offs, lengths=lens), want)
    # one byte short: the last packet ends past the buffer
    with pytest.raises(roce_icrc.ICRCError) as e:
        ctx.batch_host_bounded(buf, extent - 1, offsets=offs, lengths=lens)
    assert e.value.rc == -errno.EINVAL
    # with a status array: that packet is RICRC_ST_BADLEN, the others exact
    out, st = ctx.batch_host_bounded(buf, extent - 1, offsets=offs, lengths=lens, status=True)
    assert st[-1] == roce_icrc.ST_BADLEN and out[-1] == 0
    assert (st[:-1] == roce_icrc.ST_OK).all()
    np.testing.assert_array_equal(out[:-1], want[:-1])
    # an offset far past the end (an overflowing sum included)
    bad = offs.copy()
    bad[17] = np.uint64(2**64 - 8)
    bad[18] = np.uint64(extent + 4096)
    out, st = ctx.batch_host_bounded(buf, extent, offsets=bad, lengths=lens, status=True)
    assert st[17] == st[18] == roce_icrc.ST_BADLEN and out[17] == out[18] == 0
    ok = np.ones(len(lens), bool)
    ok[[17, 18]] = False
    np.testing.assert_array_equal(out[ok], want[ok])


def test_batch_host_checks_descriptors_in_a_host_alloc_buffer(ctx):
    """ricrc_batch_host knows the size of a buffer the context allocated
    (ricrc_host_alloc): a descriptor past its end is -EINVAL there."""
    buf, offs, lens = _ragged(3000, 2)
    n = int(offs[-1] + lens[-1])
    pinned = ctx.host_alloc(n)
    try:
        pinned[:] = buf[:n]
        want = oracle_c.icrc_batch(buf, offsets=offs, lengths=lens, threads=16)
        np.testing.assert_array_equal(ctx.batch_host(pinned, offsets=offs, lengths=lens), want)
        past = lens.copy()
        past[-1] += 4  # the last packet now ends 4 bytes past the allocation
        with pytest.raises(roce_icrc.ICRCError) as e:
            ctx.batch_host(pinned, offsets=offs, lengths=past)
        assert e.value.rc == -errno.EINVAL
    finally:
        ctx.host_free(pinned)


@pytest.mark.parametrize("framelen", [False, True])
def test_batch_device_bounded_flags_out_of_range_packets(ctx, framelen):
    count = 20000
    buf, offs, lens = _ragged(count, 3, slack=1 << 16)  # the device buffer extends past the declared extent
    rng = np.random.default_rng(4)
    extent = int(offs[count // 2])  # the second half lies past it ...
    inside = offs + lens <= extent
    bad = rng.choice(count // 2, size=50, replace=False)  # ... and so do 50 descriptors of the first half
    offs = offs.copy()
    offs[bad] = np.uint64(extent) - (lens[bad].astype(np.uint64) // 2)  # straddling the end
    inside[bad] = False
    if framelen:  # RICRC_F_FRAMELEN: random bytes sometimes read as an IPv4 / IPv6 header with a shorter length
        eff = np.array([O.frame_l3_len(buf[int(o):int(o) + int(n)].tobytes()) if ok else n
                        for o, n, ok in zip(offs, lens, inside)], np.uint32)
        want = oracle_c.icrc_batch(buf, offsets=offs, lengths=np.where(inside, eff, lens), threads=16)
    else:
        want = oracle_c.icrc_batch(buf, offsets=offs, lengths=lens, threads=16)
    d = torch.from_numpy(buf).cuda()
    d_off = torch.from_numpy(offs.view(np.int64)).cuda()
    d_len = torch.from_numpy(lens.view(np.int32)).cuda()
    out = torch.full((count,), -1, dtype=torch.int32, device="cuda")
    st = torch.full((count,), 255, dtype=torch.uint8, device="cuda")
    s = torch.cuda.current_stream()
    ctx.batch_device_bounded(d, extent, count, out, st, offsets=d_off, lengths=d_len, stream=s, framelen=framelen)
    torch.cuda.synchronize()
    got, status = out.cpu().numpy().view(np.uint32), st.cpu().numpy()
    assert (status[~inside] == roce_icrc.ST_BADLEN).all() and (got[~inside] == 0).all()
    assert (status[inside] == roce_icrc.ST_OK).all()
    np.testing.assert_array_equal(got[inside], want[inside])
    # a fixed-stride batch that does not fit is a call error
    with pytest.raises(roce_icrc.ICRCError) as e:
        ctx.batch_device_bounded(d, 4096 * 3 - 1, 3, out, st, stride=4096, stream=s)
    assert e.value.rc == -errno.EINVAL


def _guarded(nbytes):
    """A writable host array of nbytes that ends exactly at a PROT_NONE page."""
    page = mmap.PAGESIZE
    total = ((nbytes + page - 1) // page + 1) * page
    mm = mmap.mmap(-1, total, prot=mmap.PROT_READ | mmap.PROT_WRITE)
    addr = ctypes.addressof(ctypes.c_char.from_buffer(mm))
    libc = ctypes.CDLL(None, use_errno=True)
    assert libc.mprotect(ctypes.c_void_p(addr + total - page), ctypes.c_size_t(page), 0) == 0
    arr = np.frombuffer(mm, np.uint8, count=total - page)[total - page - nbytes:]
    return mm, arr


@pytest.mark.parametrize("l3_offset", [0, 14])
def test_batch_host_never_reads_past_the_extent(ctx, l3_offset):
    """a trailing descriptor a little past the buffer (or a frame
    starting within l3_offset bytes of its end) is RICRC_ST_BADLEN and none of
    its bytes is read -- the buffer ends at a guard page, so the span copy of
    the host route would fault if it stretched over such a packet."""
    rng = np.random.default_rng(7 + l3_offset)
    count = 3000
    lens = rng.choice(np.array([64, 256, 1024, 1500], np.uint32), size=count)
    frames = lens.astype(np.uint64) + l3_offset
    offs = np.zeros(count, np.uint64)
    offs[1:] = np.cumsum(frames[:-1])
    extent = int(offs[-1] + frames[-1])
    mm, buf = _guarded(extent)
    buf[:] = rng.integers(0, 256, size=extent, dtype=np.uint8)
    want = oracle_c.icrc_batch(buf, offsets=offs, lengths=lens, l3_offset=l3_offset, threads=16)
    got = ctx.batch_host_bounded(buf, extent, offsets=offs, lengths=lens, l3_offset=l3_offset)
    np.testing.assert_array_equal(got, want)
    cases = [  # (last offset, last length): just past the end; the frame inside, its L3 packet past it
        (extent - 10, 64), (extent - max(l3_offset, 1) + 0, 64), (extent + 64, 64),
        (extent - int(frames[-1]), int(lens[-1]) + 1)]
    for last_off, last_len in cases:
        o, n = offs.copy(), lens.copy()
        o[-1], n[-1] = last_off, last_len
        out, st = ctx.batch_host_bounded(buf, extent, offsets=o, lengths=n, l3_offset=l3_offset, status=True)
        assert st[-1] == roce_icrc.ST_BADLEN and out[-1] == 0, (last_off, last_len)
        assert (st[:-1] == roce_icrc.ST_OK).all()
        np.testing.assert_array_equal(out[:-1], want[:-1])
    # a bad descriptor in the middle of an ascending ring does not break it for the rest
    o = offs.copy()
    o[1500] = np.uint64(2**64 - 8)
    out, st = ctx.batch_host_bounded(buf, extent, offsets=o, lengths=lens, l3_offset=l3_offset, status=True)
    assert st[1500] == roce_icrc.ST_BADLEN and out[1500] == 0
    ok = np.ones(count, bool)
    ok[1500] = False
    np.testing.assert_array_equal(out[ok], want[ok])
    del buf
