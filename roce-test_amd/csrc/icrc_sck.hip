// gfx950 strided-chain ICRC kernel (SCK), the headline path: back-to-back
// RoCEv2 packets of 1, 2 or 4 KiB.  Its own translation unit
// so that the PMC traffic measured on it (profiles/pmc_traffic.json) is tied
// to exactly these sources (bench.py kernel_source_hash), not to edits of the
// other kernels.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "icrc_device.h"
#include "icrc_math.h"
#include "icrc_sck.h"

namespace ricrc {

// =======================================================================
// Strided-chain kernel (SCK): the headline path, packets of n = 128 L bytes
// back to back (L = 8, 16, 32: 1, 2, 4 KiB).
//
// A wave takes 8 packets at a time (a "group", 8 n bytes); lane 8 g + s
// belongs to packet g of the group and owns the 16-byte slot s of every
// 128-byte line of it.  Load k of a group is one buffer_load_dwordx4 that
// reads line k of all 8 packets -- whole 128-byte lines, which streams as
// fast as 1 KiB-contiguous loads on MI355X (tools/microbench/mb_lines.hip)
// -- and lands, with no LDS transpose, as one fold step for each of the
// lane's 4 chains: chain j = 4 s + i folds words j, j + 32, j + 64, ... of
// its packet, one word per line, so a fold step is "XOR the word, advance
// the register 128 bytes" with the slice-by-4 tables T_124..T_127 in LDS
// (same conflict-free layout as above).  Four independent chains per lane
// and no cross-lane traffic while folding.
//
// Algebra (tests/test_kernel_algebra.py::test_strided_chain_decomposition):
// with the trailer word zeroed, register = XOR_j r_j x^-32(j+1).  A lane
// combines its chains by Horner in x^-32 (uniform basis, SGPRs), multiplies
// once by x^-32(4 s + 1) (lane basis) and the 8 lanes of a packet XOR-reduce
// with three DPP steps.  That finish (4 GF(2) multiplies per lane per group,
// 4 per 8 packets instead of the transposed kernel's 2 per packet) runs in 8
// VALU slices inside the first fold steps of the next group.  Loads run D
// lines ahead through a rotating register ring; past the wave's span the
// buffer range check returns zeros, so no load is ever exec-masked.
// Results: lane l keeps packet 8 (l & 7) + (l >> 3) of each block of 8
// groups and the block leaves in one coalesced 64-dword store.
//
// ABL (timing-only ablations for tools/microbench; the product uses 0):
// 1 no table fold, 2 no finish, 8 no global loads, 16 no stores, 64 per-wave
// start/end s_memrealtime stamps into a.stamps, 128 no LDS table build.
// D: lines in flight per wave.  Every finish multiply goes through nibble
// tables, ONE copy each (the 16 entries of a nibble position sit in 16 banks:
// any lane pattern is conflict-free) -- x^-32 (128 words) and, per lane slot
// s, x^(-32 (4 s + 1)) (8 x 132 words) -- so the lane-basis multiply is 8
// lookups instead of 32 bit-select pairs and needs no basis VGPRs; the finish
// tables sit at the bottom of LDS so each lookup's constant part is a ds_read
// offset.  (Measured and retired in round 2, code in git history: the
// per-XCD dynamic group schedule, lane bases in LDS, and 32-copy x^-32
// tables with the lane basis in VGPRs -- DESIGN.md §4.)
// =======================================================================
// FAM: the address family's invariant masks, applied natively on line 0
// (kFamV4 = the reference's IPv4 masks; kFamV6; kFamAuto per packet from the
// IP version nibble, broadcast from lane 8 g to the packet's 8 lanes).
// PL < L (super-groups, 1 and 2 KiB packets): the wave streams lines exactly
// as for L-line packets -- a "super-packet" is S = L / PL consecutive packets,
// a group 8 S packets (32 KiB for L = 32) -- but each lane's chains are
// finished and restarted every PL lines, at the packet boundaries.  Load k of
// a group then reads line k of 8 super-packets 4 KiB apart, the access
// pattern of the 4 KiB packets, whose memory path alone streams ~8 % faster
// than 8 packets of 1 KiB side by side (profiles/r02/sck_abl_xt1_vs_xt2.txt:
// 0.628 ms per 4 GiB against 0.678 ms).  Sub-group m of a group (packets
// 8 S Q + S g + m) is finished S times per group; its results land in the
// slots in packet order, so the flush is unchanged.
// FR: a framed NIC ring -- 128 L-byte slots, the L3 packet at a.l3_offset in
// each, running to the slot's end.  The kernel folds the whole slot: with a
// zero register, the o = l3_offset leading bytes (zeroed) leave it at zero,
// so the register at the L3 start is seeded by XORing kSeed into L3 bytes
// 0..3 exactly as for o = 0.  Line 0's transform is per byte of the slot
// (zero before o, the IPv4 masks and the seed from o on) and is precomputed
// per lane (fr_and / fr_or / fr_xor); the trailer is still the slot's last
// word.  IPv4 masks only (other families: the linear fix-up after it).
template <int L, int ABL, int FAM = kFamV4, int PL = L, int D = 8, int FR = 0>
__global__ __launch_bounds__(kBlock) void icrc_sck_kernel(SckArgs a) {
  static_assert(L % PL == 0 && PL >= 8, "super-groups: whole packets");
  static_assert(!FR || FAM == kFamV4, "framed rings: IPv4 masks");
  constexpr uint32_t S = L / PL;  // packets per super-packet
  // finish tables | 128 KiB of slice-by-4 tables | result slots per wave
  constexpr uint32_t kSlots = 256;
  constexpr uint32_t kRoundMask = kSlots / 8 - 1;  // groups per round of slots - 1
  constexpr uint32_t kQtStride = kFinQtStride;  // words per lane slot's nibble table (padded across banks)
  constexpr uint32_t kFin = kFinSck;             // finish tables (build_fin_tables): a multiple of 32 words
  __shared__ uint32_t lds[kFin + kLdsWords + kWaves * kSlots];
  uint32_t *tab = lds + kFin;  // slice-by-4 tables
  const uint32_t *xtl = lds, *qtl = lds + 128;

  // D: lines in flight per wave
  static_assert(L % D == 0 || D == L, "ring indices must repeat every group");
  constexpr uint32_t N = 128u * L, GB = 8u * N;
  const uint32_t lane = threadIdx.x & 63;
  const uint32_t wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const uint32_t s = lane & 7;

  const uint64_t wave = (uint64_t)blockIdx.x * kWaves + wid;
  const uint64_t nwaves = (uint64_t)gridDim.x * kWaves;
  const uint32_t G = (uint32_t)((a.count + 8 * S - 1) / (8 * S));  // groups (of 8 S packets)
  const uint64_t total = a.count * (128u * PL);
  const uint32_t vo = (lane >> 3) * N + 16u * s;

  // The wave's groups: the contiguous block [g0, g1).  (A per-XCD dynamic
  // tail schedule balanced the waves' end times but measured slower,
  // tools/microbench/sck_tail.hip, profiles/r02/sck_tail.txt.)
  uint32_t g0, g1;
  if (a.xw[0] == 0u) {
    const uint64_t per = (G + nwaves - 1) / nwaves;
    g0 = (uint32_t)(wave * per < G ? wave * per : G);
    g1 = (uint32_t)(g0 + per < G ? g0 + per : G);
  } else {  // weighted by XCD
    uint64_t lo, hi;
    xcd_share(G, a.xw, a.xcd_k, wid, lo, hi);
    g0 = (uint32_t)lo;
    g1 = (uint32_t)hi;
  }
  auto after = [&](uint32_t q) -> uint32_t { return q + 1 < g1 ? q + 1 : G; };
  uint32_t qcur = g0 < g1 ? g0 : G;
  uint32_t qnext = qcur < G ? after(qcur) : G;

  // Line `line` of absolute group q (q >= G: no group, the range check reads zeros).
  auto load = [&](uint32_t q, uint32_t line) -> u32x4 {
    if (ABL & 8) return u32x4{q * 977u + line, lane, q, 5u};
    const uint64_t b = (uint64_t)q * GB;
    const uint32_t rem = q < G ? (uint32_t)(total - b < GB ? total - b : GB) : 0u;
    const __amdgpu_buffer_rsrc_t rs = make_rsrc(a.base + (q < G ? b : 0), rem);
    return __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(rs, vo + 128u * line, 0, 2));
  };
  // The first D lines are in flight while the workgroup builds its tables
  // (the table load is issued first, so waiting for it leaves them in flight).
  const uint64_t t_start = (ABL & 64) ? __builtin_amdgcn_s_memrealtime() : 0u;
  xcd_record(a.xcd_rec);
  const TableRegs tab_v = table_load(g_tab128);
  // the finish tables, built by the host (icrc_math.h build_fin_tables): two words per thread
  const uint32_t fin0 = a.fin[threadIdx.x], fin1 = a.fin[threadIdx.x + 1024u < kFin ? threadIdx.x + 1024u : 0u];
  u32x4 ring[D];
#pragma unroll
  for (int k = 0; k < D; ++k) {  // in order: the loop's vmcnt waits assume it
    __builtin_amdgcn_sched_barrier(0);
    ring[k] = load(k < L ? qcur : qnext, (uint32_t)(k % L));
  }
  __builtin_amdgcn_sched_barrier(0);
  if (!(ABL & 128)) table_write(tab, tab_v);
  if (!(ABL & 128)) {
    lds[threadIdx.x] = fin0;
    if (threadIdx.x + 1024u < kFin) lds[threadIdx.x + 1024u] = fin1;
  }
  __syncthreads();

  uint32_t *slots = lds + kFin + kLdsWords + wid * kSlots;
  const LaneTab lt{(lane & 31) << 2, ((lane & 31) << 2) | 0x10000u};
  const uint32_t mw0 = s == 0 ? kMaskW0 : (s == 2 ? kMaskW8 : 0u);  // bytes 1 / 32
  const uint32_t xw0 = s == 0 ? kSeed : 0u;
  const uint32_t mw2 = s == 0 ? kMaskW2 : (s == 1 ? kMaskW6 : 0u);  // bytes 8, 10-11 / 26-27
  // IPv6 (words 4s..4s+3 of line 0): bytes 0-3 / 7 (s = 0), 46-47 (s = 2), 52 (s = 3)
  const uint32_t m6w0 = s == 0 ? kMaskV6W0 : 0u;
  const uint32_t m6w1 = s == 0 ? kMaskV6W1 : (s == 3 ? kMaskV6W13 : 0u);
  const uint32_t m6w3 = s == 2 ? kMaskV6W11 : 0u;
  const uint32_t keep3 = s == 7 ? 0u : 0xFFFFFFFFu;                  // the trailer word
  const uint32_t *qrow = qtl + s * kQtStride;
  // FR: line 0's per-byte transform, bytes 16 s + 4 i .. + 3 of the slot
  uint32_t fr_and[4] = {}, fr_or[4] = {}, fr_xor[4] = {};
  if constexpr (FR) {
    const int o = (int)a.l3_offset;
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const int rel = (int)(16u * s) + 4 * i + k - o;  // the byte's L3 offset
        if (rel < 0) continue;
        fr_and[i] |= 0xFFu << (8 * k);
        fr_or[i] |= mask_byte(kFamV4, (uint32_t)rel) << (8 * k);
        if (rel < 4) fr_xor[i] |= ((kSeed >> (8 * rel)) & 0xFFu) << (8 * k);
      }
  }

  struct Fin {
    uint32_t r[4];    // chain registers
    uint32_t tr;      // trailer word (lane s = 7), for verify
    uint32_t acc[4];  // multiply accumulators
    uint32_t u;       // Horner value
  };
  auto take = [](Fin &f) -> uint32_t {
    const uint32_t v = xor3(f.acc[0], f.acc[1], f.acc[2] ^ f.acc[3]);
#pragma unroll
    for (int k = 0; k < 4; ++k) f.acc[k] = 0u;
    return v;
  };
  // Slice sl (0..7): u = ((r3 X ^ r2) X ^ r1) X ^ r0, then u * Q.
  auto fin_slice = [&](Fin &f, int sl) {
    if (ABL & 2) return;
    if (sl == 0) {
      f.u = f.r[3];
#pragma unroll
      for (int k = 0; k < 4; ++k) f.acc[k] = 0u;
    }
    {  // 4 nibble lookups of one table copy (x^-32, then the lane slot's)
      const uint32_t *t = sl < 6 ? xtl : qrow;
#pragma unroll
      for (int w = 4 * (sl & 1); w < 4 * (sl & 1) + 4; ++w) f.acc[w & 3] ^= t[16 * w + __builtin_amdgcn_ubfe(f.u, 4 * w, 4)];
    }
    if (sl == 1) f.u = take(f) ^ f.r[2];
    if (sl == 3) f.u = take(f) ^ f.r[1];
    if (sl == 5) f.u = take(f) ^ f.r[0];
    if (sl == 7) f.u = take(f);
  };
  const uint32_t vmask = __builtin_amdgcn_readfirstlane(a.verify ? 0xFFFFFFFFu : 0u);
  uint32_t sink = 0;
  // Results go to the wave's LDS slots (all 8 lanes of a packet write the
  // same value to the same slot: no exec mask) and leave for HBM once per
  // round of slots, so the streaming loop holds no global store: a store
  // shares vmcnt with the ring and every load queued behind it would wait
  // for its write acknowledgement.  j counts the wave's finished groups.
  auto flush = [&](uint32_t j_end) {  // the round of groups ending at local index j_end
    if (ABL & 16) return;
    const uint32_t j_lo = (j_end - 1) & ~kRoundMask;
    __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0): the slot writes have landed
    {  // consecutive groups: coalesced
      const uint64_t pb = ((uint64_t)g0 * S + j_lo) * 8u;
      const uint32_t valid = (j_end - j_lo) * 8u;  // slots written this round
      const uint32_t nout = (uint32_t)(a.count - pb < valid ? a.count - pb : valid);
      const __amdgpu_buffer_rsrc_t ro = make_rsrc(a.out + pb, 4u * nout);
#pragma unroll
      for (int h = 0; h < (int)kSlots / 256; ++h) {
        const u32x4 v = *reinterpret_cast<const u32x4 *>(slots + 256 * h + 4 * lane);
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(__attribute__((ext_vector_type(4))) uint32_t, v),
                                               ro, 1024u * h + 16u * lane, 0, 0);
      }
    }
  };
  auto fin_store = [&](Fin &f, uint32_t jf) {
    const uint32_t crc = (ABL & 2) ? (f.r[0] ^ f.r[1] ^ f.r[2] ^ f.r[3]) : f.u;
    const uint32_t v = group_xor(crc, 3);
    const uint32_t chk = group_xor(f.tr, 3) == ~v ? 1u : 0u;
    const uint32_t val = __builtin_amdgcn_bitop3_b32(vmask, chk, ~v, 0xCA);  // vmask ? chk : ~v, bitwise
    if (ABL & 16) {
      sink ^= val;
      return;
    }
    // sub-group jf's packet of lane group g: S (jf / S) * 8 + S g + jf % S in the round
    slots[(((jf & kRoundMask) & ~(S - 1)) << 3) | ((lane >> 3) * S) | (jf & (S - 1))] = val;
  };

  // Finish slices of the previous packet ride in its successor's steps 0..7
  // (0..6 for PL = 8, two in step 0), its result is written in the step after.
  constexpr int kStoreStep = PL >= 16 ? 8 : PL - 1;
  auto slice_step = [](int sl) constexpr { return PL >= 16 ? sl : sl * (PL - 1) / 8; };
  static_assert(PL >= 8, "finish needs 8 fold steps");
  // A packet's first line: the family's invariant masks and the seed.
  auto first_line = [&](u32x4 w, uint32_t (&x)[4]) {
    if constexpr (FR) {
#pragma unroll
      for (int i = 0; i < 4; ++i) w[i] = ((w[i] & fr_and[i]) | fr_or[i]) ^ fr_xor[i];
    } else if constexpr (FAM == kFamV4) {
      w[0] = or_xor(w[0], mw0, xw0);
      w[2] |= mw2;
    } else if constexpr (FAM == kFamV6) {
      w[0] = or_xor(w[0], m6w0, xw0);
      w[1] |= m6w1;
      w[3] |= m6w3;
    } else {  // per packet: IP version nibble of lane 8 g's first byte (ds_swizzle: lane & 0x18)
      const uint32_t b0 = (uint32_t)__builtin_amdgcn_ds_swizzle((int)w[0], 0x18);
      const uint32_t v6 = ((b0 >> 4) & 15u) == 6u ? 0xFFFFFFFFu : 0u;
      w[0] = or_xor(w[0], __builtin_amdgcn_bitop3_b32(v6, m6w0, mw0, 0xCA), xw0);
      w[1] |= v6 & m6w1;
      w[2] |= ~v6 & mw2;
      w[3] |= v6 & m6w3;
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) x[i] = w[i];  // chain register (0) ^ line-0 word
  };
  Fin pf{};
  uint32_t j = 0;  // the wave's packets of lane group 0 started so far (sub-groups)
  while (qcur < G) {  // qcur: wave-uniform
    const u32x4 w = ring[0];
    ring[0] = load(D < L ? qcur : qnext, (uint32_t)(D % L));
    uint32_t x[4];
    first_line(w, x);
    uint32_t tr = 0;
#pragma unroll
    for (int k = 0; k < L; ++k) {
      const int kp = k % PL;              // line within the packet
      const bool last = kp == PL - 1;     // the packet's last line
      // Fence each step: the scheduler would otherwise hoist the whole
      // group's ring refills to the top and drain vmcnt to zero there.
      __builtin_amdgcn_sched_barrier(0);
      u32x4 wn = {0u, 0u, 0u, 0u}, wf = {0u, 0u, 0u, 0u};
      if (k + 1 < L) {
        const u32x4 nx = ring[(k + 1) % D];
        ring[(k + 1) % D] = load(k + 1 + D < L ? qcur : qnext, (uint32_t)((k + 1 + D) % L));
        if (last) {
          wf = nx;  // the next packet's first line (PL < L)
        } else {
          wn = nx;
          if (kp + 1 == PL - 1) {
            tr = keep3 ? 0u : wn[3];
            wn[3] &= keep3;
          }
        }
      }
      uint32_t t[4][4];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        if (ABL & 1) {
          t[i][0] = __builtin_amdgcn_perm(x[i], lt.lo0, 0x0C0C0400u);
          t[i][1] = x[i] >> 7;
          t[i][2] = x[i] * 3u;
          t[i][3] = 0u;
        } else {
          t[i][0] = lds_at(tab, __builtin_amdgcn_perm(x[i], lt.lo0, 0x0C0C0400u));
          t[i][1] = lds_at(tab, __builtin_amdgcn_perm(x[i], lt.lo0, 0x0C0C0500u) + 128);
          t[i][2] = lds_at(tab, __builtin_amdgcn_perm(x[i], lt.lo1, 0x0C020600u));
          t[i][3] = lds_at(tab, __builtin_amdgcn_perm(x[i], lt.lo1, 0x0C020700u) + 128);
        }
      }
      // The previous packet's finish, in the shadow of the reads (for j = 0
      // it runs on zeros; its slot write is overwritten before any flush).
#pragma unroll
      for (int sl = 0; sl < 8; ++sl)
        if (slice_step(sl) == kp) fin_slice(pf, sl);
      if (kp == kStoreStep) {
        fin_store(pf, j - 1);
        if (j > 0 && ((j - 1) & kRoundMask) == kRoundMask) flush(j);  // wave-uniform: a full round of slots
      }
#pragma unroll
      for (int i = 0; i < 4; ++i) x[i] = xor3(t[i][0], t[i][1], xor3(t[i][2], t[i][3], wn[i]));
      if (last) {  // the packet is folded: hand its chains to the finish
#pragma unroll
        for (int i = 0; i < 4; ++i) pf.r[i] = x[i];
        pf.tr = tr;
        ++j;
        if (k + 1 < L) {
          first_line(wf, x);
          tr = 0;
        }
      }
    }
    qcur = qnext;  // advance the group sequence (wave-uniform)
    qnext = qcur < G ? after(qcur) : G;
  }
  if (j > 0) {
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int sl = 0; sl < 8; ++sl) fin_slice(pf, sl);
    fin_store(pf, j - 1);
    flush(j);
  }
  if (ABL & 16) a.out[wave * 64 + lane] = sink;
  if ((ABL & 64) && lane == 0) {  // diagnostic builds (tools/microbench/sck_tail.hip): start / end times
    a.stamps[2 * wave] = t_start;
    a.stamps[2 * wave + 1] = __builtin_amdgcn_s_memrealtime();
  }
}

// ----------------------------------------------------------- host launcher
template <int FAM>
hipError_t launch_sck_fam(const SckArgs &a, int grid, hipStream_t st) {
  const dim3 g(grid), b(kBlock);
  if (a.n == 4096) hipLaunchKernelGGL((icrc_sck_kernel<32, 0, FAM>), g, b, 0, st, a);
  // 1 KiB packets stream in 4 KiB super-packets (S = 4 packets each): 0.180 ->
  // 0.176 ms on 1 M; 2 KiB packets measured 2 % slower that way (0.346 ->
  // 0.353 ms, same box, profiles/r02/ab_super_1k_2k/) and keep L = 16
  else if (a.n == 2048) hipLaunchKernelGGL((icrc_sck_kernel<16, 0, FAM>), g, b, 0, st, a);
  else if (a.n == 1024) hipLaunchKernelGGL((icrc_sck_kernel<32, 0, FAM, 8>), g, b, 0, st, a);
  else return hipErrorInvalidValue;
  return hipGetLastError();
}

// Framed rings (a.l3_offset > 0): 1, 2 and 4 KiB slots, IPv4 masks.
hipError_t launch_sck_framed(const SckArgs &a, int grid, hipStream_t st) {
  const dim3 g(grid), b(kBlock);
  if (a.n == 4096) hipLaunchKernelGGL((icrc_sck_kernel<32, 0, kFamV4, 32, 8, 1>), g, b, 0, st, a);
  else if (a.n == 2048) hipLaunchKernelGGL((icrc_sck_kernel<16, 0, kFamV4, 16, 8, 1>), g, b, 0, st, a);
  else if (a.n == 1024) hipLaunchKernelGGL((icrc_sck_kernel<32, 0, kFamV4, 8, 8, 1>), g, b, 0, st, a);
  else return hipErrorInvalidValue;
  return hipGetLastError();
}

hipError_t launch_sck(const SckArgs &a, int grid, hipStream_t st) {
  (void)hipGetLastError();  // a stale error of an earlier, unrelated HIP call must not fail this launch
  if (a.l3_offset != 0) {
    if (a.family != kFamV4 || a.l3_offset > kSckMaxL3) return hipErrorInvalidValue;
    return launch_sck_framed(a, grid, st);
  }
  if (a.family == kFamV6) return launch_sck_fam<kFamV6>(a, grid, st);
  if (a.family == kFamAuto) return launch_sck_fam<kFamAuto>(a, grid, st);
  if (a.family != kFamV4) return hipErrorInvalidValue;
  return launch_sck_fam<kFamV4>(a, grid, st);
}

}  // namespace ricrc
