// Device-side building blocks shared by the gfx950 kernels of libroceicrc
// (icrc_kernels.hip, icrc_rsck.hip): LDS slice-by-4 tables, GF(2) multiplies,
// 3-input bit ops, cross-lane XOR reductions, buffer resources, byte masks.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "icrc_math.h"

namespace ricrc {

__device__ constexpr SliceTables<4> g_tab = make_tables<4>();

static constexpr int kWaves = 16;       // waves per workgroup
static constexpr int kBlock = 64 * kWaves;
static constexpr int kLdsWords = 32768;  // 128 KiB

// ---------------------------------------------------------------- helpers
// The share [lo, hi) of `total` units that wave `wid` of workgroup blockIdx.x
// takes when a wave on XCD x weighs w[x] (the odd-numbered XCDs' waves, and
// XCD 0's a little, stream HBM 5-10 % slower: tools/microbench/sck_skew.hip,
// xcd_slow.hip).  Workgroups are dealt round-robin over the 8 XCDs starting
// at XCD k, which changes between processes (tools/microbench/xcc_probe.hip):
// workgroup b is on XCD (b + k) % 8.  w and k come from the host or from an
// earlier kernel of the same stream, so every wave uses the same values: the
// shares are contiguous, in wave order, and cover [0, total) for any k; a
// wrong k costs speed, never a packet.
__device__ __forceinline__ void xcd_share(uint64_t total, const uint32_t (&w)[8], uint32_t k, uint32_t wid,
                                          uint64_t &lo, uint64_t &hi) {
  const uint64_t b = blockIdx.x, nb = gridDim.x;
  uint64_t cyc = 0;
#pragma unroll
  for (int x = 0; x < 8; ++x) cyc += w[x];
  auto cum = [&](uint64_t n) -> uint64_t {  // the weight of workgroups [0, n)
    uint64_t s = (n >> 3) * cyc;
    for (uint32_t j = 0; j < (uint32_t)(n & 7u); ++j) s += w[(k + j) & 7u];
    return s;
  };
  const uint64_t wb = w[(b + k) & 7u];
  const uint64_t before = (uint64_t)kWaves * cum(b) + wid * wb;
  const uint64_t wtot = (uint64_t)kWaves * cum(nb);
  // The boundary at weight x, total * x / wtot, in double precision: a
  // 64-bit integer division is a long software expansion ahead of the
  // wave's first loads.  Monotonic in x and the same for both waves that
  // share a boundary, exact at 0 and at wtot: still a partition.
  const double f = (double)total / (double)wtot;
  auto at = [&](uint64_t x) -> uint64_t {
    const uint64_t r = (uint64_t)((double)x * f);
    return x >= wtot || r > total ? total : r;
  };
  lo = at(before);
  hi = at(before + wb);
}

// Workgroup 0 records the XCD it runs on (HW_REG_XCC_ID) for the host's next
// launch (xcd_share's k): a system-scope store to pinned host memory.
__device__ __forceinline__ void xcd_record(uint32_t *rec) {
  if (rec != nullptr && blockIdx.x == 0 && threadIdx.x == 0)
    __hip_atomic_store(rec, (uint32_t)__builtin_amdgcn_s_getreg((3 << 11) | 20), __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_SYSTEM);
}

__device__ __forceinline__ uint32_t xor3(uint32_t a, uint32_t b, uint32_t c) {
  return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96);
}
__device__ __forceinline__ uint32_t and_xor(uint32_t a, uint32_t b, uint32_t c) {  // (a & b) ^ c
  return __builtin_amdgcn_bitop3_b32(a, b, c, 0x6A);
}
__device__ __forceinline__ uint32_t or_xor(uint32_t a, uint32_t b, uint32_t c) {  // (a | b) ^ c
  return __builtin_amdgcn_bitop3_b32(a, b, c, 0x56);
}

// Build the LDS tables: region 0 = {T3 | T2}, region 1 = {T1 | T0}, 256-byte
// rows of 32 copies x 4 B per half.
// One table entry per thread (4 x 256 = 1024 = kBlock): a single global load,
// then the entry's 32 copies (128 contiguous bytes) in 8 ds_write_b128.
__device__ __forceinline__ uint32_t table_entry(const SliceTables<4> &tab) {
  return tab.t[threadIdx.x >> 8][threadIdx.x & 255];
}
__device__ __forceinline__ void table_store_at(uint32_t *lds, uint32_t idx, uint32_t v) {  // entry idx & 255 of T_{idx >> 8}
  const uint32_t t = idx >> 8, e = idx & 255;
  const uint32_t region = t <= 1 ? 1u : 0u, half = (t == 0 || t == 2) ? 1u : 0u;  // T3 T2 | T1 T0
  typedef uint32_t v4 __attribute__((ext_vector_type(4)));
  v4 *dst = reinterpret_cast<v4 *>(lds + ((region << 14) | (e << 6) | (half << 5)));
#pragma unroll
  for (int k = 0; k < 8; ++k) dst[k] = v4{v, v, v, v};
}
__device__ __forceinline__ void table_store(uint32_t *lds, uint32_t v) { table_store_at(lds, threadIdx.x, v); }

// The whole 128 KiB set in address order: store k of thread t writes the 16
// bytes at 16 (1024 k + t), so a wave's store is one contiguous KiB and no
// two lanes share a bank; the thread loads the 8 entries it stores (from a
// 4 KiB table the L2 holds).  table_store -- one entry per thread, its 32
// copies as 128 contiguous bytes -- put every lane of a wave on the same four
// banks: the build took ~5 us at the start of the ragged fold
// (tools/microbench/shard.hip, profiles/r05/NOTES.md).  load early, write
// late: the loads' latency hides behind a kernel's first global loads.
struct TableRegs {
  uint32_t v[8];
};
__device__ __forceinline__ TableRegs table_load(const SliceTables<4> &tab) {
  static_assert(kBlock == 1024 && kLdsWords == 8 * 4 * kBlock, "8 stores of 16 bytes per thread");
  TableRegs r;
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    const uint32_t w = 4u * (1024u * k + threadIdx.x);  // the word the store starts at
    const uint32_t region = w >> 14, e = (w >> 6) & 255u, half = (w >> 5) & 1u;
    const uint32_t t = region ? (half ? 0u : 1u) : (half ? 2u : 3u);  // T3 T2 | T1 T0 (table_store_at)
    r.v[k] = tab.t[t][e];
  }
  return r;
}
__device__ __forceinline__ void table_write(uint32_t *lds, const TableRegs &r) {
  typedef uint32_t v4 __attribute__((ext_vector_type(4)));
  v4 *dst = reinterpret_cast<v4 *>(lds);
#pragma unroll
  for (int k = 0; k < 8; ++k) dst[1024u * k + threadIdx.x] = v4{r.v[k], r.v[k], r.v[k], r.v[k]};
}
__device__ __forceinline__ void fill_tables(uint32_t *lds, const SliceTables<4> &tab = g_tab) {
  table_write(lds, table_load(tab));
}

struct LaneTab {
  uint32_t lo0, lo1;  // copy offsets for region 0 / region 1
};

__device__ __forceinline__ uint32_t lds_at(const uint32_t *lds, uint32_t byte_addr) {
  return *reinterpret_cast<const uint32_t *>(reinterpret_cast<const char *>(lds) + byte_addr);
}

// One slice-by-4 step: register after folding word w into register r.
__device__ __forceinline__ uint32_t step4(const uint32_t *lds, LaneTab lt, uint32_t r, uint32_t w) {
  const uint32_t x = r ^ w;
  const uint32_t t3 = lds_at(lds, __builtin_amdgcn_perm(x, lt.lo0, 0x0C0C0400u));
  const uint32_t t2 = lds_at(lds, __builtin_amdgcn_perm(x, lt.lo0, 0x0C0C0500u) + 128);
  const uint32_t t1 = lds_at(lds, __builtin_amdgcn_perm(x, lt.lo1, 0x0C020600u));
  const uint32_t t0 = lds_at(lds, __builtin_amdgcn_perm(x, lt.lo1, 0x0C020700u) + 128);
  return xor3(t3, t2, t1 ^ t0);
}

// Same step, but returns (register ^ next word) directly: the word XOR rides
// in the second v_bitop3, so a step is 4 v_perm + 2 v_bitop3 + 4 ds_read_b32.
__device__ __forceinline__ uint32_t step4x(const uint32_t *lds, LaneTab lt, uint32_t x, uint32_t wnext) {
  const uint32_t t3 = lds_at(lds, __builtin_amdgcn_perm(x, lt.lo0, 0x0C0C0400u));
  const uint32_t t2 = lds_at(lds, __builtin_amdgcn_perm(x, lt.lo0, 0x0C0C0500u) + 128);
  const uint32_t t1 = lds_at(lds, __builtin_amdgcn_perm(x, lt.lo1, 0x0C020600u));
  const uint32_t t0 = lds_at(lds, __builtin_amdgcn_perm(x, lt.lo1, 0x0C020700u) + 128);
  return xor3(t3, t2, xor3(t1, t0, wnext));
}

// r * K where Q[j] = K * x^(31-j) (bit j of r is the x^(31-j) coefficient).
// Four independent accumulators keep the 32-term XOR off one dependency chain.
__device__ __forceinline__ uint32_t mul_basis(uint32_t r, const uint32_t (&Q)[32]) {
  uint32_t acc[4] = {0u, 0u, 0u, 0u};
#pragma unroll
  for (int j = 0; j < 32; ++j) {
    const uint32_t m = (uint32_t)(((int32_t)(r << (31 - j))) >> 31);
    acc[j & 3] = and_xor(m, Q[j], acc[j & 3]);
  }
  return xor3(acc[0], acc[1], acc[2] ^ acc[3]);
}

__device__ __forceinline__ void make_basis(uint32_t K, uint32_t (&Q)[32]) {
  Q[31] = K;
#pragma unroll
  for (int j = 30; j >= 0; --j) Q[j] = gf_mulx(Q[j + 1]);
}

__device__ __forceinline__ uint32_t gf_mul_dev(uint32_t a, uint32_t b) {
  uint32_t p = 0;
#pragma unroll 8
  for (int i = 31; i >= 0; --i) {
    const uint32_t m = (uint32_t)(((int32_t)(a << (31 - i))) >> 31);
    p = and_xor(m, b, p);
    b = gf_mulx(b);
  }
  return p;
}

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ uint32_t word_of(const u32x4 &v, int i) { return v[i]; }


__device__ __forceinline__ __amdgpu_buffer_rsrc_t make_rsrc(const void *base, uint32_t bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void *>(base), (short)0, (int)bytes, 0x00020000);
}

// Swizzled 16-byte slot of piece p in a 2 KiB round: the 8-lane groups of
// ds_write_b128 stay in one 128-byte row, and the 32-byte chunk reads of each
// 16-lane ds_read_b128 group hit 16 distinct bank quads.
__device__ __forceinline__ uint32_t stage_slot(uint32_t p) { return p ^ ((p >> 4) & 1u); }

// XOR of v over aligned groups of 2^levels lanes, result in every lane.
__device__ __forceinline__ uint32_t group_xor(uint32_t v, uint32_t levels) {
  if (levels > 0) v ^= __builtin_amdgcn_update_dpp(0u, v, 0xB1, 0xF, 0xF, true);   // quad_perm [1,0,3,2]
  if (levels > 1) v ^= __builtin_amdgcn_update_dpp(0u, v, 0x4E, 0xF, 0xF, true);   // quad_perm [2,3,0,1]
  if (levels > 2) v ^= __builtin_amdgcn_update_dpp(0u, v, 0x141, 0xF, 0xF, true);  // row_half_mirror
  if (levels > 3) v ^= __builtin_amdgcn_update_dpp(0u, v, 0x140, 0xF, 0xF, true);  // row_mirror
  if (levels > 4) {
    const auto p = __builtin_amdgcn_permlane16_swap(v, v, false, false);
    v = p[0] ^ p[1];
  }
  if (levels > 5) {
    const auto p = __builtin_amdgcn_permlane32_swap(v, v, false, false);
    v = p[0] ^ p[1];
  }
  return v;
}

// Branch-free variant for a run-time group size: level k is applied through
// a wave-uniform all-ones / zero mask, so the code stays one basic block and
// the scheduler can interleave it with the next step's table lookups.
__device__ __forceinline__ uint32_t group_xor_masked(uint32_t v, const uint32_t (&lm)[6]) {
  v = and_xor(__builtin_amdgcn_update_dpp(0u, v, 0xB1, 0xF, 0xF, true), lm[0], v);
  v = and_xor(__builtin_amdgcn_update_dpp(0u, v, 0x4E, 0xF, 0xF, true), lm[1], v);
  v = and_xor(__builtin_amdgcn_update_dpp(0u, v, 0x141, 0xF, 0xF, true), lm[2], v);
  v = and_xor(__builtin_amdgcn_update_dpp(0u, v, 0x140, 0xF, 0xF, true), lm[3], v);
  const auto p = __builtin_amdgcn_permlane16_swap(v, v, false, false);
  v = and_xor(p[0] ^ p[1] ^ v, lm[4], v);
  const auto q = __builtin_amdgcn_permlane32_swap(v, v, false, false);
  v = and_xor(q[0] ^ q[1] ^ v, lm[5], v);
  return v;
}

constexpr SliceTables<4> make_stride_tables(uint64_t gap) {
  SliceTables<4> s = make_tables<4>();
  const uint32_t g = gf_x8n(gap);
  for (int k = 0; k < 4; ++k)
    for (int b = 0; b < 256; ++b) s.t[k][b] = gf_mul(s.t[k][b], g);
  return s;
}
__device__ constexpr SliceTables<4> g_tab128 = make_stride_tables(124);  // word + 124 bytes = one line

// =======================================================================
// Byte-level helpers for packets that do not start or end on a word.
// =======================================================================
__device__ __forceinline__ uint32_t byte_span_mask(int lo, int hi) {  // bytes [lo,hi) of a word
  // Branch-free: 64-bit shifts of 0xFFFFFFFF handle the 0- and 32-bit ends.
  const uint32_t l = (uint32_t)(lo < 0 ? 0 : lo > 4 ? 4 : lo);
  const uint32_t h = (uint32_t)(hi < 0 ? 0 : hi > 4 ? 4 : hi);
  const uint32_t keep_hi = (uint32_t)(0xFFFFFFFFull >> (32u - 8u * h));
  const uint32_t keep_lo = (uint32_t)(0xFFFFFFFFull << (8u * l));
  return keep_hi & keep_lo;
}

__device__ __forceinline__ uint32_t expand_nibble(uint32_t b) {
  return ((b & 1u) ? 0x000000FFu : 0u) | ((b & 2u) ? 0x0000FF00u : 0u) | ((b & 4u) ? 0x00FF0000u : 0u) |
         ((b & 8u) ? 0xFF000000u : 0u);
}

// Loads through explicit global (address space 1) pointers: an address
// built from an integer is otherwise a flat access, and flat loads may retire
// out of order with global ones, which forces vmcnt(0) after each of them.
typedef const u32x4 __attribute__((address_space(1))) *gptr_u32x4;
typedef uint32_t __attribute__((aligned(1))) u32_unaligned;
typedef const u32_unaligned __attribute__((address_space(1))) *gptr_u32_unaligned;
__device__ __forceinline__ u32x4 gload16(uintptr_t addr) { return *reinterpret_cast<gptr_u32x4>(addr); }
__device__ __forceinline__ uint32_t gload4_unaligned(uintptr_t addr) {
  return *reinterpret_cast<gptr_u32_unaligned>(addr);
}

// ---------------------------------------------------------- lane quads (DPP)
// Lane quad transpose of 16-byte chunks: on entry lane 4 p + c holds chunk c
// of the packets in A[0..3] (A[k]: load k); on exit it holds chunks 0..3 of
// the packet that was in A[c].  swap(v, 1): the value of lane l ^ 1.
__device__ __forceinline__ uint32_t dpp_swap1(uint32_t v) {
  return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0xB1, 0xF, 0xF, false);  // quad_perm [1,0,3,2]
}
__device__ __forceinline__ uint32_t dpp_swap2(uint32_t v) {
  return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x4E, 0xF, 0xF, false);  // quad_perm [2,3,0,1]
}
__device__ __forceinline__ void quad_transpose(u32x4 (&A)[4], uint32_t c) {
  const bool o1 = (c & 1u) != 0, o2 = (c & 2u) != 0;
#pragma unroll
  for (int i = 0; i < 4; ++i) {  // round 1: registers k, k ^ 1 across lanes c, c ^ 1
    const uint32_t t0 = dpp_swap1(A[0][i]), t1 = dpp_swap1(A[1][i]);
    const uint32_t t2 = dpp_swap1(A[2][i]), t3 = dpp_swap1(A[3][i]);
    A[0][i] = o1 ? t1 : A[0][i];
    A[1][i] = o1 ? A[1][i] : t0;
    A[2][i] = o1 ? t3 : A[2][i];
    A[3][i] = o1 ? A[3][i] : t2;
  }
#pragma unroll
  for (int i = 0; i < 4; ++i) {  // round 2: registers k, k ^ 2 across lanes c, c ^ 2
    const uint32_t t0 = dpp_swap2(A[0][i]), t1 = dpp_swap2(A[1][i]);
    const uint32_t t2 = dpp_swap2(A[2][i]), t3 = dpp_swap2(A[3][i]);
    A[0][i] = o2 ? t2 : A[0][i];
    A[2][i] = o2 ? A[2][i] : t0;
    A[1][i] = o2 ? t3 : A[1][i];
    A[3][i] = o2 ? A[3][i] : t1;
  }
}

// The value v of lane 4 (l / 4) + c (c a constant 0..3): a quad broadcast.
template <int C>
__device__ __forceinline__ uint32_t dpp_quad_bcast(uint32_t v) {
  return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, C * 0x55, 0xF, 0xF, false);  // quad_perm [C,C,C,C]
}

}  // namespace ricrc
