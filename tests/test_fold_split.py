"""CPU: the ragged fold's work split (icrc_rsck.hip, icrc_rsck_kernel), restated.

The bucket pass lays out each pass block's packets as runs of 8-packet
groups of one line count L (one run per class) and reserves the block's
groups and weighted work with one atomic, so blocks sit in the big pool in
an arbitrary order, group order and work order agreeing.  The fold's waves
take contiguous shares [x0, x1) of the weighted work (equal, or weighted by
XCD: xcd_share, icrc_device.h), and each wave folds the groups whose work
starts in its share.  This test restates that rule on random layouts and
checks that it partitions the pool: every group folded by exactly one wave,
whatever the grid, the weights and the start XCD.  (Round 5 tried splitting
each workgroup's work exactly between its waves, cutting groups between two
waves and combining the halves by CRC linearity: correct, but the fold ran
slower, the waves' end times no tighter -- profiles/r05/NOTES.md.)"""
import random

KW = 16  # waves per workgroup (kWaves)
GC = 12  # group cost, quarter line-steps (kRsGroupCost)


def xcd_share(total, w, k, b, nb, wid):
    """icrc_device.h xcd_share: wave wid of workgroup b's [lo, hi)."""
    cyc = sum(w)

    def cum(n):
        return (n >> 3) * cyc + sum(w[(k + j) & 7] for j in range(n & 7))
    wb = w[(b + k) & 7]
    before = KW * cum(b) + wid * wb
    wtot = KW * cum(nb)
    f = float(total) / float(wtot)  # double precision, as the kernel (a monotonic map, exact at 0 and wtot)

    def at(x):
        r = int(float(x) * f)
        return total if x >= wtot or r > total else r
    return at(before), at(before + wb)


def layout(rng, nblk):
    """Pass blocks' runs in the big pool: (blocks, runs, NG, S)."""
    order = list(range(nblk))
    rng.shuffle(order)  # the reservation atomic's order
    runs_of = {b: [(L, rng.randint(1, 40)) for L in sorted(rng.sample([2, 3, 8, 9, 32, 33, 5, 12, 100],
                                                                   rng.randint(0, 6)))] for b in range(nblk)}
    g = s = 0
    blk, runs = [None] * nblk, [[] for _ in range(nblk)]
    for b in order:
        g0, s0 = g, s
        for L, G in runs_of[b]:
            runs[b].append(dict(g0=g, gs=G, L=L, s0=s, w=4 * L + GC))
            g += G
            s += G * (4 * L + GC)
        blk[b] = dict(g0=g0, s0=s0, work=s - s0, runs=len(runs_of[b]))
    return blk, runs, g, s


def first_at(blk, runs, NG, S, x):
    """The kernel's first_group_at: the first group whose work starts at or after x."""
    if x >= S:
        return NG
    b = next(b for b, B in enumerate(blk) if B["runs"] and B["s0"] <= x < B["s0"] + B["work"])
    R = next(R for R in runs[b] if R["s0"] <= x < R["s0"] + R["gs"] * R["w"])
    return min(R["g0"] + (x - R["s0"] + R["w"] - 1) // R["w"], R["g0"] + R["gs"], NG)


def test_wave_shares_partition_the_pool():
    rng = random.Random(7)
    for _ in range(80):
        blk, runs, NG, S = layout(rng, rng.choice([1, 2, 5, 40, 128, 256]))
        if NG == 0:
            continue
        grid = rng.choice([1, 3, 16, 64, 256])
        xw, xk = rng.choice([None, [1040, 960] * 4, [1025, 975] * 4, [3, 7, 1, 8000, 2, 2, 5, 9]]), rng.randrange(8)
        nw = grid * KW
        share = (S + nw - 1) // nw
        seen = [0] * NG
        for b in range(grid):
            for wid in range(KW):
                wave = b * KW + wid
                x0 = min(wave * share, S)
                x1 = x0 + share
                if xw:
                    x0, x1 = xcd_share(S, xw, xk, b, grid, wid)
                for q in range(first_at(blk, runs, NG, S, x0), first_at(blk, runs, NG, S, x1)):
                    seen[q] += 1
        assert seen == [1] * NG


def test_xcd_shares_tile_large_totals():
    """xcd_share's double-precision boundaries at the ragged pool's full range
    (total < 2^39.01) and the weight cap (8000): contiguous, ordered shares
    from 0 to total, wave after wave."""
    rng = random.Random(3)
    for _ in range(60):
        total = rng.choice([1, 7, 4096, rng.randrange(1, 1 << 39), (1 << 39) - 1])
        grid = rng.choice([1, 3, 240, 256])
        w = rng.choice([[1040, 960] * 4, [1025, 975] * 4, [8000] * 8, [rng.randrange(1, 8001) for _ in range(8)]])
        k = rng.randrange(8)
        prev = 0
        for b in range(grid):
            for wid in range(KW):
                lo, hi = xcd_share(total, w, k, b, grid, wid)
                assert lo == prev and lo <= hi <= total
                prev = hi
        assert prev == total


def small_rounds(NC, NG, S, grid, b, wid, x0, x1, slots):
    """icrc_rsck_kernel's small rounds [c_begin, c_end) of wave wid of
    workgroup b: dealt evenly to wave slots 0..slots-1, or (slots = 0, or
    no big pool) the wave's fraction [x0, x1) / T of them."""
    T = S if NG else NC
    c0, c1 = min(x0, T) * NC // T, min(x1, T) * NC // T
    if slots and NG:
        E, e = grid * slots, b * slots + wid
        c0, c1 = (e * NC // E, (e + 1) * NC // E) if wid < slots else (0, 0)
    return c0, c1


def test_small_rounds_partition_the_small_pool():
    """The fold's rounds of 64 one-line packets: every round folded by exactly
    one wave, for slot dealing (kRsSmallSlots = 12, RICRC_SMALL_SLOTS) and the
    share-proportional rule, with and without a big pool and XCD weights."""
    rng = random.Random(11)
    for _ in range(300):
        NC = rng.choice([1, 2, 63, 64, 2048, 16384, rng.randrange(1, 5000)])
        NG = rng.choice([0, 1, 7, 1000])
        S = NG * rng.choice([16, 20, 144])
        T = S if NG else NC
        grid = rng.choice([1, 3, 16, 256])
        slots = rng.choice([0, 1, 4, 12, 16])
        xw, xk = rng.choice([None, [1040, 960] * 4, [3, 7, 1, 8000, 2, 2, 5, 9]]), rng.randrange(8)
        nw = grid * KW
        share = (T + nw - 1) // nw
        seen = [0] * NC
        for b in range(grid):
            for wid in range(KW):
                x0 = min((b * KW + wid) * share, T)
                x1 = x0 + share
                if xw:
                    x0, x1 = xcd_share(T, xw, xk, b, grid, wid)
                c0, c1 = small_rounds(NC, NG, S, grid, b, wid, x0, x1, slots)
                for c in range(c0, c1):
                    seen[c] += 1
        assert seen == [1] * NC, (NC, NG, grid, slots)
