"""CPU check of the decomposition the gfx950 kernels use (no GPU needed).

The kernels split a packet into lane chunks folded from a zero register,
re-align each chunk register with a GF(2) multiply by x^(8 d) and XOR the
results; the ragged kernel additionally zero-extends packets to 64-byte
pieces from a 16-byte aligned base, aligns lanes to the end of a 64-piece wave
step, carries open packets across steps by x^(8*4096) and removes the
alignment and zero tail with x^-(8 z + 512 (63 - lane)).
These tests restate that algebra in pure Python -- using the oracle's
independent gf_mul / crc_shift -- and check it against zlib on random
packets, so a mistake in the *math* is caught on the CPU, before any GPU run.
"""
import random
import zlib

import icrc_oracle as o

POLY = o.POLY_REFLECTED
ONE = 0x80000000
SEED_REG = o.REGISTER_AFTER_PREFIX


def fold(reg, data: bytes):
    for b in data:
        reg ^= b
        for _ in range(8):
            reg = (reg >> 1) ^ (POLY if reg & 1 else 0)
    return reg


def x8n(n):
    return o.crc_shift(ONE, n)


def xinv():
    return ((POLY << 1) & 0xFFFFFFFF) | 1


def xinv8n(n):
    r, s = ONE, xinv()
    for _ in range(8 * n):
        r = o.gf_mul(r, s)
    return r


def masked(pkt):
    return bytearray(o.masked_body(pkt))


def test_inverse_of_x():
    assert o.gf_mul(xinv(), ONE >> 1) == ONE
    for n in (1, 3, 17):
        assert o.gf_mul(xinv8n(n), x8n(n)) == ONE


def test_stream_kernel_decomposition():
    """Lane c folds bytes [chunk*c, chunk*(c+1)) from 0 (lane 0 with the seed
    injected into its first word); K_c = x^(8 * bytes after chunk c)."""
    rng = random.Random(1)
    for n in (44, 64, 100, 1024, 1500, 4096):
        pkt = bytes(rng.randrange(256) for _ in range(n))
        m = masked(pkt)
        M = len(m)
        for chunk in (64, 128, 256):
            P = -(-M // chunk)
            acc = 0
            for c in range(P):
                part = bytearray(m[chunk * c: min(chunk * (c + 1), M)])
                if c == 0:
                    for k in range(4):
                        part[k] ^= (SEED_REG >> (8 * k)) & 0xFF
                r = fold(0, part)
                acc ^= o.gf_mul(r, x8n(M - min(chunk * (c + 1), M)))
            assert acc ^ 0xFFFFFFFF == zlib.crc32(o.PREFIX + bytes(m))


def _xinv8n_fast(n):
    r, sq, e = ONE, xinv8n(1), n
    while e:
        if e & 1:
            r = o.gf_mul(r, sq)
        sq = o.gf_mul(sq, sq)
        e >>= 1
    return r


def test_ragged_kernel_decomposition():
    """The ragged kernel's algebra (icrc_kernels.hip icrc_ragged_kernel):
    packets cut into 64-byte pieces from their 16-byte aligned base, 64
    consecutive pieces per wave step regardless of packet boundaries, lane l
    aligned to the step end by x^(512 (63-l)), packets reduced as
    P[last] ^ P[first-1] of a prefix XOR, packets open at lane 63 carried into
    the next step by x^(8*4096), and the last lane's x^-(8 z + 512 (63-l))."""
    rng = random.Random(3)
    sizes = [4, 5, 44, 48, 61, 64, 100, 256, 1024, 4096, 4100, 9001, 64, 64, 44, 300] * 2
    rng.shuffle(sizes)
    pkts, pieces = [], []  # pieces: (packet index, bytes)
    for i, n in enumerate(sizes):
        pkt = bytes(rng.randrange(256) for _ in range(n))
        m = masked(pkt)
        M, s = len(m), rng.randrange(16)
        P = max(1, (s + M + 63) // 64)
        D = bytearray(64 * P)
        D[s: s + M] = m
        for k in range(4):
            D[s + k] ^= (SEED_REG >> (8 * k)) & 0xFF
        pkts.append((m, s, P))
        pieces += [(i, D[64 * k: 64 * k + 64]) for k in range(P)]
    got, carry = {}, 0
    for g in range(0, len(pieces), 64):
        step = pieces[g: g + 64]
        vals = []
        for lane, (_, d) in enumerate(step):
            r = fold(0, d)
            vals.append(o.gf_mul(r, x8n(64 * (63 - lane))))
        vals[0] ^= carry
        pre, acc = [], 0
        for v in vals:
            acc ^= v
            pre.append(acc)
        carry = 0
        for lane, (i, _) in enumerate(step):
            first = next(l for l in range(64) if step[l][0] == i)
            seg = pre[lane] ^ (pre[first - 1] if first > 0 else 0)
            last_here = lane + 1 == len(step) or step[lane + 1][0] != i
            if not last_here:
                continue
            ends = g + lane + 1 == len(pieces) or pieces[g + lane + 1][0] != i
            if ends:
                m, s, P = pkts[i]
                z = 64 * P - s - len(m)
                got[i] = o.gf_mul(seg, _xinv8n_fast(z + 64 * (63 - lane))) ^ 0xFFFFFFFF
            else:  # open at lane 63
                assert lane == 63
                carry = o.gf_mul(seg, x8n(4096))
    for i, (m, _, _) in enumerate(pkts):
        assert got[i] == zlib.crc32(o.PREFIX + bytes(m)), (i, len(m))


def test_strided_chain_decomposition():
    """The strided-chain kernel's algebra (icrc_kernels.hip icrc_sck_kernel):
    8 lanes per packet, lane s loads the 16-byte slot s of every 128-byte line,
    and each of its 4 words is its own chain j = 4 s + i over words
    j, j + 32, j + 64, ... (one fold step = XOR the word, advance 128 bytes:
    tables T_124..T_127).  With the trailer word zeroed,
    register = XOR_j r_j * x^(-32 (j + 1)); the lane combines its four chains
    by Horner in x^-32 and multiplies once by x^(-32 (4 s + 1))."""
    rng = random.Random(7)
    X = _xinv8n_fast(4)
    for n in (128, 256, 1024, 4096):
        pkt = bytes(rng.randrange(256) for _ in range(n))
        body = bytearray(masked(pkt)) + bytes(4)  # trailer word zeroed
        words = [int.from_bytes(body[4 * t: 4 * t + 4], "little") for t in range(n // 4)]
        words[0] ^= SEED_REG
        chains = [0] * 32
        for t, w in enumerate(words):
            chains[t % 32] = o.crc_shift(chains[t % 32] ^ w, 128)
        flat = 0
        for j in range(32):
            flat ^= o.gf_mul(chains[j], _xinv8n_fast(4 * (j + 1)))
        horner = 0
        for s in range(8):
            u = chains[4 * s + 3]
            for i in (2, 1, 0):
                u = o.gf_mul(u, X) ^ chains[4 * s + i]
            horner ^= o.gf_mul(u, _xinv8n_fast(16 * s + 4))
        want = o.icrc(pkt) ^ 0xFFFFFFFF
        assert flat == want
        assert horner == want


def test_ragged_line_grid_decomposition():
    """The ragged strided-chain kernel's algebra (icrc_rsck.hip): a packet at
    any byte address is folded on the absolute 128-byte line grid -- lines
    [A, A + 128 L), A = addr & ~127 -- with bytes outside the covered range
    zeroed, the seed XORed into covered bytes 0..3 and the masks applied by
    packet-relative offset.  Chains j = t mod 32 as in the fixed-size kernel;
    lane s combines its 4 chains by Horner in x^-32 and multiplies by
    x^(-128 s); the packet register is the XOR over lanes times x^(-8 tz),
    tz = 128 L - a - M the zero tail of the last line."""
    rng = random.Random(11)
    X = _xinv8n_fast(4)
    for _ in range(40):
        n = rng.choice([44, 45, 60, 64, 100, 127, 128, 129, 256, 1000, 1500, 4096])
        a = rng.randrange(128)
        pkt = bytes(rng.randrange(256) for _ in range(n))
        M = n - 4
        L = (a + M + 127) // 128
        body = masked(pkt)
        stream = bytearray(128 * L)
        stream[a:a + M] = body
        for k in range(4):
            stream[a + k] ^= (SEED_REG >> (8 * k)) & 0xFF
        words = [int.from_bytes(stream[4 * t: 4 * t + 4], "little") for t in range(32 * L)]
        chains = [0] * 32
        for t, w in enumerate(words):
            chains[t % 32] = o.crc_shift(chains[t % 32] ^ w, 128)
        reg = 0
        for s in range(8):
            u = chains[4 * s + 3]
            for i in (2, 1, 0):
                u = o.gf_mul(u, X) ^ chains[4 * s + i]
            reg ^= o.gf_mul(u, _xinv8n_fast(16 * s))
        tz = 128 * L - a - M
        assert 0 <= tz < 128
        reg = o.gf_mul(reg, _xinv8n_fast(tz))
        assert reg ^ 0xFFFFFFFF == o.icrc(pkt), (n, a)



def _le_words(b: bytes):
    return [int.from_bytes(b[i:i + 4], "little") for i in range(0, len(b), 4)]


def _byte_span(lo, hi):
    lo, hi = max(0, min(4, lo)), max(0, min(4, hi))
    return sum(0xFF << (8 * k) for k in range(lo, hi))


def _small_word(w, r):  # icrc_rsck.hip small_word()
    keep = _byte_span(-r, 4)
    pre = _byte_span(-4 - r, -r)
    orm = 0
    for k in range(4):
        if (r + k) in o.MASK_OFFSETS:
            orm |= 0xFF << (8 * k)
    return (w & keep) | pre | orm


def test_small_lane_end_aligned_stream():
    """icrc_rsmall_kernel (one lane per packet): fold 16-byte blocks that END at
    the covered end e from a ZERO register -- 4 x 0xFF prefix (= init ~0 and the 8 x 0xFF of calc_icrc), masked body,
    leading zero blocks up to a wave-wide multiple-of-4 block count, units
    clamped to the packet's own, words by the 2-level funnel + alignbyte --
    and take ~register.  Restated on a byte image with arbitrary neighbours."""
    rng = random.Random(5)
    mem = bytearray(rng.getrandbits(8) for _ in range(1 << 14))
    for _ in range(400):
        n = rng.choice([44, 45, 47, 64, 100, 256, 255, 300, 380, rng.randrange(44, 400)])
        addr = rng.randrange(64, len(mem) - n - 64)
        M = n - 4
        e = addr + M
        K = (M + 4 + 15) >> 4
        Kmax = ((K + rng.randrange(0, 6)) + 3) & ~3  # the wave's maximum, rounded up
        t = e & 15
        ufirst, ulast = addr & ~15, (e - 1) & ~15
        unit = lambda u: _le_words(bytes(mem[min(max(u, ufirst), ulast):][:16]))  # noqa: E731
        reg = 0
        N = e - t - 16 * Kmax
        rel = M - 16 * Kmax
        for j in range(Kmax):
            W = unit(N) + unit(N + 16)
            X = [W[(t >> 2) + k] for k in range(5)]
            sb = t & 3
            for i in range(4):
                w = ((X[i + 1] << 32 | X[i]) >> (8 * sb)) & 0xFFFFFFFF
                if rel < 40:
                    w = _small_word(w, rel + 4 * i)
                reg = fold(reg, w.to_bytes(4, "little"))
            rel += 16
            N += 16
        assert (~reg) & 0xFFFFFFFF == o.icrc(bytes(mem[addr:addr + n])), (addr, n, Kmax)


def test_small_word_aligned_matches_bytewise():
    """icrc_rsck.hip small_word_aligned (whole-word masks, word-aligned waves)
    == small_word for every word-aligned packet-relative offset."""
    W0, W2, W6, W8 = 0x0000FF00, 0xFFFF00FF, 0xFFFF0000, 0x000000FF  # icrc_math.h kMaskW*
    rng = random.Random(8)
    for r in range(-64, 80, 4):
        for _ in range(20):
            w = rng.getrandbits(32)
            keep = 0xFFFFFFFF if r >= 0 else 0
            orm = (0xFFFFFFFF if r == -4 else 0) | (W0 if r == 0 else 0) | (W2 if r == 8 else 0) \
                | (W6 if r == 24 else 0) | (W8 if r == 32 else 0)
            assert (w & keep) | orm == _small_word(w, r), r


def test_small_lane_static_head_window():
    """icrc_rsmall_kernel masks only blocks 0..3 when every lane of the wave has
    M >= 16 Kmax - 24: then no byte at packet offset < 40 (prefix, invariant
    fields) or before the packet lies in a block >= 4."""
    for M in range(40, 400):
        K = (M + 4 + 15) >> 4
        for Kmax in range((K + 3) & ~3, ((K + 3) & ~3) + 12, 4):
            if M + 24 < 16 * Kmax:
                continue
            rel4 = M - 16 * Kmax + 64
            assert rel4 >= 40, (M, Kmax)
            assert M - 16 * Kmax >= -24


def _nib_mul(table, v):
    """icrc_rsck.hip nib_mul: v * (the table's constant) by 8 nibble lookups."""
    r = 0
    for w in range(8):
        r ^= table[16 * w + ((v >> (4 * w)) & 15)]
    return r


def test_ragged_finish_nibble_tables():
    """The ragged fold's finish tables (icrc_rsck_kernel): the x^-32 table
    entry (w, v) = (nibble v at bits 4w..4w+3) * x^-32, and lane slot s's
    table built the way the kernel builds it -- p = QS[s] x^(28 - 4w), then
    one x per bit from bit 4w + 3 down -- turn 8 lookups into the GF(2)
    multiply, so Horner and the x^(-128 s) alignment are unchanged."""
    rng = random.Random(17)
    X = _xinv8n_fast(4)
    xt = [o.gf_mul(X, v << (4 * w)) for w in range(8) for v in range(16)]
    mulx = lambda p: o.gf_mul(p, ONE >> 1)  # noqa: E731
    for s in range(8):
        qs = _xinv8n_fast(16 * s)  # host: QS[s] = x^(-128 s)
        qt = []
        for w in range(8):
            for v in range(16):
                p = qs
                for _ in range(28 - 4 * w):
                    p = mulx(p)
                e = 0
                for b in (3, 2, 1, 0):
                    e ^= p if (v >> b) & 1 else 0
                    p = mulx(p)
                qt.append(e)
        for _ in range(20):
            u = rng.getrandbits(32)
            assert _nib_mul(qt, u) == o.gf_mul(u, qs)
    for _ in range(200):
        u = rng.getrandbits(32)
        assert _nib_mul(xt, u) == o.gf_mul(u, X)


def test_fold_one_line_nibble_step():
    """icrc_rsck.hip StepNib (the fold kernel's one-line packets, whose LDS
    tables advance 128 bytes a step): the x^32 nibble table (icrc_math.h
    build_fin_tables, kFinStep4) gives the slice-by-4 step's register,
    r, w -> (r ^ w) x^32."""
    rng = random.Random(32)
    X32 = ONE
    for _ in range(32):
        X32 = o.gf_mul(X32, ONE >> 1)
    xt = [o.gf_mul(X32, v << (4 * w)) for w in range(8) for v in range(16)]
    for _ in range(300):
        r, w = rng.getrandbits(32), rng.getrandbits(32)
        assert _nib_mul(xt, r ^ w) == fold(r, w.to_bytes(4, "little"))


def test_ragged_tz_bases_compact():
    """Basis word 4q of x^(-8 tz) is x^(-8 tz) x^(31 - 4q) = x^(31 - 4 (2 tz + q)),
    so the kernel's table needs one entry per m = 2 tz + q (264 words, host
    icrc_api.cpp) instead of 128 x 8: every split of m gives the same word."""
    table = {}
    for tz in range(128):
        c = _xinv8n_fast(tz)
        for q in range(8):
            table.setdefault(2 * tz + q, set()).add(o.gf_mul(c, 1 << (4 * q)))
    assert len(table) == 262 and all(len(v) == 1 for v in table.values())
    for m, (v,) in table.items():  # the host's split: tz = min(m >> 1, 127), q = m - 2 tz
        tz = min(m >> 1, 127)
        assert o.gf_mul(_xinv8n_fast(tz), 1 << (4 * (m - 2 * tz))) == v


def test_ragged_whole_word_edges():
    """Whole-word edge masking of the ragged fold (word-aligned packets): keep
    = sign of ((rel - M) & ~rel) for 0 <= rel < M, then the head table's
    (or, xor) pair at k = min(rel >> 2, 15) -- equal to the bytewise rule:
    bytes outside [0, M) zeroed, the invariant fields forced to 0xFF, the seed
    XORed into bytes 0..3."""
    rng = random.Random(19)
    mask_off = {1, 8, 10, 11, 26, 27, 32}
    orm = [0] * 16
    for k in range(10):
        for b in range(4):
            if 4 * k + b in mask_off:
                orm[k] |= 0xFF << (8 * b)
    seed = [SEED_REG] + [0] * 15
    for _ in range(3000):
        M = 4 * rng.randrange(10, 1200)
        rel = 4 * rng.randrange(-40, 1300)
        w = rng.getrandbits(32)
        x = (rel - M) & ~rel & 0xFFFFFFFF
        keep = 0xFFFFFFFF if x >> 31 else 0
        k = min((rel & 0xFFFFFFFF) >> 2, 15)
        got = ((w & keep) | orm[k]) ^ seed[k]
        want = bytearray(w.to_bytes(4, "little"))
        for b in range(4):
            off = rel + b
            if not 0 <= off < M:
                want[b] = 0
            elif off in mask_off:
                want[b] = 0xFF
        wv = int.from_bytes(want, "little")
        if rel == 0:
            wv ^= SEED_REG
        assert got == wv, (rel, M)
