// GF(2) arithmetic and CRC-32 tables shared by the host library and the
// gfx950 kernels of libroceicrc.
//
// Representation: the reflected CRC-32 register (poly 0xEDB88320, the
// HashAlgorithm_t.CRC32 of p4/shuffle/shuffle_egress.p4:461).  Bit 31 of a
// 32-bit value is the coefficient of x^0, bit 0 the coefficient of x^31, so
// "advance the register over one zero bit" is multiplication by x.
//
// The register is linear over GF(2):   reg(A || B) = reg(A) * x^(8|B|) ^ reg0(B)
// (reg0 = register started from 0).  Every kernel in this library is built on
// that identity: lanes fold independent chunks from a zero register and the
// partial registers are re-aligned by a multiplication by x^(8 d).
#pragma once
#include <stdint.h>

#if defined(__HIPCC__)
#define RICRC_HD __host__ __device__
#else
#define RICRC_HD
#endif

namespace ricrc {

constexpr uint32_t kPoly = 0xEDB88320u;
constexpr uint32_t kOne = 0x80000000u;          // x^0
constexpr uint32_t kSeed = 0xDEBB20E3u;         // register after 8 x 0xFF from ~0 (shuffle_egress.p4:465)
constexpr uint32_t kMinLen = 20 + 8 + 12 + 4;   // IPv4 + UDP + BTH + ICRC
constexpr uint32_t kMaxLen = 65535;             // IPv4 total_len is 16 bits (header.p4:45)

// Invariant-field masks as bits of a 64-bit "byte is forced to 0xFF" map over
// L3 bytes [0,40): tos 1, ttl 8, IPv4 csum 10-11, UDP csum 26-27, BTH byte 4
// at 32 (shuffle_egress.p4:467,471,473,480,485).
constexpr uint64_t kMaskBits = (1ull << 1) | (1ull << 8) | (1ull << 10) | (1ull << 11) |
                               (1ull << 26) | (1ull << 27) | (1ull << 32);
// The same masks as little-endian OR-words for 4-aligned words 0, 2, 6, 8.
constexpr uint32_t kMaskW0 = 0x0000FF00u;
constexpr uint32_t kMaskW2 = 0xFFFF00FFu;
constexpr uint32_t kMaskW6 = 0xFFFF0000u;
constexpr uint32_t kMaskW8 = 0x000000FFu;

// IPv6 (RoCEv2 over IPv6; not in the IPv4-only reference, header.p4:42-53):
// the invariant fields of IBTA Annex A17 as the Linux rxe driver masks them
// (rxe_icrc.c) -- traffic class + flow label (byte 0 low nibble, bytes 1-3),
// hop limit 7, UDP checksum 46-47, BTH byte 4 at 52.  OR-words for 4-aligned
// words 0, 1, 11, 13.
constexpr uint32_t kMaskV6W0 = 0xFFFFFF0Fu;
constexpr uint32_t kMaskV6W1 = 0xFF000000u;
constexpr uint32_t kMaskV6W11 = 0xFFFF0000u;
constexpr uint32_t kMaskV6W13 = 0x000000FFu;

// Address families (the flags of the *_ex entry points, include/roce_icrc.h).
enum Family : uint32_t { kFamV4 = 0, kFamV6 = 1, kFamAuto = 2 };
constexpr uint32_t kMaskSpan = 56;  // every masked byte of either family lies in L3 [0, 56)

// OR-word w (bytes 4w..4w+3) of a family's masks.
RICRC_HD constexpr uint32_t mask_word(uint32_t fam, uint32_t w) {
  return fam == kFamV6 ? (w == 0 ? kMaskV6W0 : w == 1 ? kMaskV6W1 : w == 11 ? kMaskV6W11 : w == 13 ? kMaskV6W13 : 0u)
                       : (w == 0 ? kMaskW0 : w == 2 ? kMaskW2 : w == 6 ? kMaskW6 : w == 8 ? kMaskW8 : 0u);
}
RICRC_HD constexpr uint32_t mask_byte(uint32_t fam, uint32_t i) {
  return i < kMaskSpan ? (mask_word(fam, i >> 2) >> (8 * (i & 3))) & 0xFFu : 0u;
}

// RICRC_F_FRAMELEN (include/roce_icrc.h): the L3 length of a packet whose
// frame extends n bytes past its L3 start (an Ethernet NIC ring's frame may
// carry minimum-frame padding and the FCS after the datagram).  b0 = L3 byte
// 0, h2 / h4 = the big-endian 16-bit fields at L3 bytes 2 and 4 (read only
// when kMinLen <= n <= kMaxLen; a longer or shorter descriptor is a bad
// length whatever the header says): IPv4 total_len (header.p4:45), IPv6
// payload length + 40.  That length when it lies in [kMinLen, n], else n (a
// strict classification rejects such a packet).  Same rule:
// oracle/icrc_oracle.py frame_l3_len.
RICRC_HD constexpr bool frame_len_applies(uint32_t n) { return n >= kMinLen && n <= kMaxLen; }
RICRC_HD constexpr uint32_t frame_l3_len(uint32_t n, uint32_t b0, uint32_t h2, uint32_t h4) {
  const uint32_t v = b0 >> 4;
  const uint32_t t = v == 4u ? h2 : (v == 6u ? h4 + 40u : 0u);
  return (frame_len_applies(n) && t >= kMinLen && t <= n) ? t : n;
}

RICRC_HD constexpr uint32_t gf_mulx(uint32_t a) { return (a >> 1) ^ ((a & 1u) ? kPoly : 0u); }

// a * b mod P, both reflected.
RICRC_HD constexpr uint32_t gf_mul(uint32_t a, uint32_t b) {
  uint32_t p = 0;
  for (int i = 31; i >= 0; --i) {
    if ((a >> i) & 1u) p ^= b;
    b = gf_mulx(b);
  }
  return p;
}

// x^(8 n) mod P by square-and-multiply.
RICRC_HD constexpr uint32_t gf_x8n(uint64_t n) {
  uint32_t r = kOne, sq = kOne >> 8;  // x^8
  while (n) {
    if (n & 1u) r = gf_mul(r, sq);
    sq = gf_mul(sq, sq);
    n >>= 1;
  }
  return r;
}

// x^-1 mod P = (P(x) + 1) / x: in normal order x^31 + (0x04C11DB7 >> 1);
// reflected, that is bit 0 plus the reflected poly shifted left by one.
constexpr uint32_t kXInv = (kPoly << 1) | 1u;

// x^(-8 n) mod P.
RICRC_HD constexpr uint32_t gf_xinv8n(uint64_t n) {
  uint32_t r = kOne, sq = gf_mul(gf_mul(gf_mul(kXInv, kXInv), gf_mul(kXInv, kXInv)),
                                 gf_mul(gf_mul(kXInv, kXInv), gf_mul(kXInv, kXInv)));
  while (n) {
    if (n & 1u) r = gf_mul(r, sq);
    sq = gf_mul(sq, sq);
    n >>= 1;
  }
  return r;
}

// Multiplication basis of a constant K: q[j] = K * x^(31-j), so that
// r * K = XOR over set bits j of r of q[j] (bit j is the x^(31-j) term).
struct Basis {
  uint32_t q[32];
};
RICRC_HD constexpr Basis make_const_basis(uint32_t K) {
  Basis b{};
  b.q[31] = K;
  for (int j = 30; j >= 0; --j) b.q[j] = gf_mulx(b.q[j + 1]);
  return b;
}

// Slice-by-N tables: T[k][b] = register after byte b followed by k zero
// bytes, from a zero register (T[0] is the classic Sarwate table).
template <int N>
struct SliceTables {
  uint32_t t[N][256];
};

template <int N>
constexpr SliceTables<N> make_tables() {
  SliceTables<N> s{};
  for (uint32_t b = 0; b < 256; ++b) {
    uint32_t c = b;
    for (int k = 0; k < 8; ++k) c = (c >> 1) ^ ((c & 1u) ? kPoly : 0u);
    s.t[0][b] = c;
  }
  for (int k = 1; k < N; ++k)
    for (uint32_t b = 0; b < 256; ++b) s.t[k][b] = (s.t[k - 1][b] >> 8) ^ s.t[0][s.t[k - 1][b] & 0xFFu];
  return s;
}

// The strided-chain kernels' finish tables, the first words of their LDS
// (built on the host once per device, loaded by every workgroup): nibble
// tables of GF(2) constants -- entry 16 w + v = (nibble v at bits
// 4w..4w+3) * K, bit j of a value standing for x^(31 - j).
//   [0, 128)               K = x^-32
//   [128 + 132 s, + 128)   K = QS[s] = x^(-8 (16 s + trail)), lane slot s (rows padded to 132 words)
//   kFinSck = 1216 words (the SCK: trail = 4, its trailer word); the ragged
//   fold (trail = 0) adds [1184, 1216) its head masks (or, xor of word k)
//   and [1216, 1344), [1344, 1472) K = x^-64, x^-96, and [1472, 1600)
//   K = x^32 (one 4-byte CRC step for its one-line packets, whose 128 KiB
//   LDS tables are the 128-byte-stride ones): kFinFold = 1600.
constexpr uint32_t kFinQtStride = 132;
constexpr uint32_t kFinSck = 128 + 8 * kFinQtStride + 32;
constexpr uint32_t kFinFold = 128 + 8 * kFinQtStride + 32 + 384;
constexpr uint32_t kFinStep4 = 1472;  // the fold's x^32 nibble table
inline uint32_t nibble_entry(uint32_t K, uint32_t w, uint32_t v) {
  uint32_t e = 0;
  for (int b = 0; b < 4; ++b)
    if ((v >> b) & 1u) e ^= gf_mul(K, 1u << (4 * w + b));
  return e;
}
inline void build_fin_tables(uint32_t *t, bool fold) {
  const uint32_t n = fold ? kFinFold : kFinSck;
  for (uint32_t i = 0; i < n; ++i) t[i] = 0;
  uint32_t qs[8];
  for (uint32_t s = 0; s < 8; ++s) qs[s] = gf_xinv8n(16ull * s + (fold ? 0 : 4));
  const uint32_t x32 = gf_xinv8n(4), x64 = gf_xinv8n(8), x96 = gf_xinv8n(12);
  for (uint32_t w = 0; w < 8; ++w)
    for (uint32_t v = 0; v < 16; ++v) {
      t[16 * w + v] = nibble_entry(x32, w, v);
      for (uint32_t s = 0; s < 8; ++s) t[128 + kFinQtStride * s + 16 * w + v] = nibble_entry(qs[s], w, v);
      if (fold) {
        t[1216 + 16 * w + v] = nibble_entry(x64, w, v);
        t[1344 + 16 * w + v] = nibble_entry(x96, w, v);
        t[kFinStep4 + 16 * w + v] = nibble_entry(gf_x8n(4), w, v);
      }
    }
  if (fold)
    for (uint32_t k = 0; k < 16; ++k) {  // word k of the header (rel = 4k): IPv4 invariant fields -> 0xFF, the seed at 0
      t[1184 + 2 * k] = k == 0 ? kMaskW0 : k == 2 ? kMaskW2 : k == 6 ? kMaskW6 : k == 8 ? kMaskW8 : 0u;
      t[1184 + 2 * k + 1] = k == 0 ? kSeed : 0u;
    }
}

static_assert(gf_mul(kXInv, kOne >> 1) == kOne, "x * x^-1 must be 1");
static_assert(make_tables<1>().t[0][1] == 0x77073096u, "Sarwate table");

}  // namespace ricrc
