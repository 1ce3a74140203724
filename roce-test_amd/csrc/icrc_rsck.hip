// Ragged strided-chain path of libroceicrc (gfx950): batches with per-packet
// offsets and/or lengths, any alignment, any mix of sizes -- the C4 mixed-MTU
// configuration and NIC rings with Ethernet framing.
//
// The fixed-size strided-chain kernel (icrc_kernels.hip, icrc_sck_kernel)
// streams at the HBM read ceiling because a wave reads whole 128-byte lines
// of 8 packets per load and folds them without any transpose.  This path
// gives ragged batches the same inner loop:
//
//  1. rsck_bucket   classify every packet by its number of 128-byte lines on
//                   the ABSOLUTE line grid, L = ceil(((addr & 127) + n - 4) /
//                   128), and lay each pass block's packets out by class:
//                   small ones in a range of the small pool, big ones as runs
//                   of whole 8-packet groups of one L in a range of the big
//                   pool (block-local: no grid-wide count or plan, see the
//                   kernel);
//  2. icrc_rsck_kernel  folds groups of 8 equal-L packets (L > kRsSmallL)
//                   exactly like the SCK -- lane 8g+s owns slot s of every
//                   line of packet g, four chains per lane, T_124..T_127
//                   tables in LDS -- with a load cursor running ahead of the
//                   fold cursor across group boundaries, descriptors read 64
//                   at a time, waves splitting the big pool by weighted work;
//                   and, in rounds of 64 on wave slots 0..11, the one-line
//                   packets (C4's 64 B; 8 lanes per packet is too coarse for
//                   them) one lane per packet (RICRC_ONE_LINE_IN_GATHER: a
//                   separate icrc_rsmall_kernel, or the gather, folds them);
//  3. rsck_gather   out[i] = res[pos(i)] (verify mode: the trailer compared
//                   with it); packets too short for a RoCEv2 header
//                   (4 <= n < 44) are computed here by a scalar loop, invalid
//                   lengths yield 0.
//
// Lines are 128-byte aligned in memory (misaligned line grids measured 20 %
// slower, tools/microbench/mb_lines.hip), so a packet's first and last line
// generally hold bytes of its neighbours: bytes outside the covered range
// [addr, addr + n - 4) are zeroed (leading zeros do not change a register
// folded from 0), the seed and the invariant masks are applied by
// packet-relative byte offset on the packet's head lines, and the zero tail
// tz = 128 L - a - M of the last line is removed at the end by x^(-8 tz)
// (tests/test_kernel_algebra.py::test_ragged_line_grid_decomposition).
// Every load is a 16-byte slot of a line that holds packet bytes, i.e. in a
// page the packet occupies.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <type_traits>
#include <utility>

#include "icrc_device.h"
#include "icrc_kernels.h"
#include "icrc_math.h"

namespace ricrc {
namespace {

typedef const u32x4 __attribute__((address_space(1))) *gptr_u32x4_t;
__device__ __forceinline__ u32x4 gload16_nt(uint64_t addr) {
  return __builtin_nontemporal_load(reinterpret_cast<gptr_u32x4_t>((uintptr_t)addr));
}

// Packet i's L3 address and length.  OFF / LEN: the batch has per-packet
// offsets / lengths (template parameters of the pass kernels, so the loads of
// several packets issue back to back instead of behind per-packet branches).
template <bool OFF, bool LEN>
__device__ __forceinline__ void rs_packet(const RsckArgs &a, uint64_t i, uint64_t &addr, uint32_t &n) {
  addr = (uint64_t)(uintptr_t)a.base + (OFF ? a.off[i] : i * a.stride) + a.l3_offset;
  n = LEN ? a.len[i] : a.fixed_len;
}
__device__ __forceinline__ void rs_packet(const RsckArgs &a, uint64_t i, uint64_t &addr, uint32_t &n) {
  addr = (uint64_t)(uintptr_t)a.base + (a.off ? a.off[i] : i * a.stride) + a.l3_offset;
  n = a.len ? a.len[i] : a.fixed_len;
}

// Class of a packet (icrc_kernels.h): by 128-byte lines of the absolute grid
// its covered bytes span, or, for packets of <= kRsSmallL lines, by 64-byte
// pieces; 0 = not bucketed.
__device__ __forceinline__ uint32_t rs_class(uint64_t addr, uint32_t n) {
  if (n < kMinLen || n > kMaxLen) return 0u;
  const uint32_t M = n - 4u;
  const uint32_t L = (uint32_t)(((addr & 127u) + M + 127u) >> 7);
  if (L <= (uint32_t)kRsSmallL) return 1u + (uint32_t)(((addr & 15u) + M + 63u) >> 6);
  return (uint32_t)kRsBigBase + L;
}

// ICRC of a packet shorter than a RoCEv2 header (4 <= n < 44): Sarwate loop.
__device__ uint32_t icrc_small(uint64_t addr, uint32_t n) {
  const uint8_t *p = reinterpret_cast<const uint8_t *>((uintptr_t)addr);
  uint32_t r = kSeed;
  for (uint32_t i = 0; i < n - 4u; ++i) {
    const uint32_t b = p[i] | mask_byte(kFamV4, i);
    r = g_tab.t[0][(r ^ b) & 0xFFu] ^ (r >> 8);
  }
  return ~r;
}

// Pass blocks own contiguous packet ranges.
constexpr int kPassBlock = 1024;
constexpr int kPassBlocks = 256;  // pass grid cap: one 1024-thread block per CU, all resident at once
constexpr int kPassUnroll = 16;   // packets per thread whose descriptors are read at once (C4: one round)
// Batches of more than kPassBlocks x kPassBlock x 16 packets (4 M; C4's
// byte-balanced shards at N > 1 hold up to 4.2 M) read 17 per thread, so
// their blocks stay on the one-round, LDS-staged path up to 4.46 M.
constexpr int kPassUnrollBig = 17;
__device__ __forceinline__ void pass_range(uint64_t count, uint64_t &lo, uint64_t &hi) {
  const uint64_t per = ((count + gridDim.x - 1) / gridDim.x + kPassBlock - 1) / kPassBlock * kPassBlock;
  lo = (uint64_t)blockIdx.x * per;
  lo = lo < count ? lo : count;
  hi = lo + per < count ? lo + per : count;
}

// Inclusive sum over the wave's lanes (6 bpermute steps).
template <typename T>
__device__ __forceinline__ T wave_scan(T v) {
  const int lane = (int)(threadIdx.x & 63u);
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const T u = __shfl_up(v, (unsigned)d);
    if (lane >= d) v += u;
  }
  return v;
}

// The bucket pass: ONE kernel, no grid-wide dependency.  Round 2 counted
// the classes over the whole batch first (a count pass, then a plan in its
// last workgroup: class-contiguous buckets), so every packet's descriptors
// were read twice and the pipeline paid a launch and a serial plan tail.
// The fold does not need classes to be contiguous over the batch, only
// groups of 8 equal-L packets and a work prefix in group order: so each
// block buckets its own packets --
//   1. read the descriptors (kept in registers when the block's packets fit
//      one round of kPassUnroll per thread: C4's 4 M packets on 256 blocks),
//      classify, rank each packet in its class by an LDS atomic (packets
//      that are not bucketed -- n < 44, invalid lengths -- are left to the
//      gather pass);
//   2. scan the block's class counts (one class per thread): small classes
//      are laid out back to back, big classes as runs of whole groups;
//   3. reserve the block's small range and its big range -- groups and
//      weighted work packed in ONE 64-bit atomic, so the big pool's group
//      order and work order agree -- and publish the block's runs (RsBlock,
//      RsRun) for the fold's work split;
//   4. write each descriptor to its position (and pos_of[i]); the packet
//      ranked last in its class pads the run's last group with copies of
//      itself.  When the block's packets fit one round, the block's layout
//      is built in LDS first and leaves in coalesced 8-byte stores: its
//      small range and its big range are each contiguous in the pools, so
//      LDS entry j maps to a pool position by one offset.  (Stored straight
//      from the registers, every wave scattered 4-byte stores over its
//      classes' ranges: 25 of the pass's 46 us on C4, against 5 us
//      coalesced; tools/microbench/bucket_abl.hip.)
// Blocks whose packets take several rounds re-read them for step 4 (ranks
// from a second LDS cursor: any order of ranks is a valid layout) and store
// from the registers.
// ABL (timing-only ablations, tools/microbench/bucket_abl.hip): 1 stop after
// the ranking round, 2 no LDS atomics (rank 0), 4 stop after the reservation,
// 8 no pos_of stores, 16 no descriptor stores, 32 no LDS staging.
// LDS layout entries of a block: a round's packets + room for group padding
// (U <= 4: room for the worst case, 7 padding entries for each of kRsRuns
// classes, so every block of such a batch is staged: PassShape::fused.)
__host__ __device__ constexpr uint32_t stage_entries(int U) {
  return (uint32_t)U * kPassBlock + (U <= 4 ? 7u * (uint32_t)kRsRuns : 512u);
}
template <bool OFF, bool LEN, int ABL = 0, int U = kPassUnroll>
__global__ __launch_bounds__(kPassBlock) void rsck_bucket(RsckArgs a) {
  constexpr uint32_t kStage = stage_entries(U);
  __shared__ uint32_t h[kRsClasses], at[kRsClasses], cur[kRsClasses];
  __shared__ uint32_t wg[16], wsm[16], wf[16];
  __shared__ uint64_t ww[16];
  __shared__ uint32_t blk_g0, blk_small, blk_stot, blk_total;
  __shared__ uint64_t blk_s0;
  __shared__ uint64_t stage[kStage];  // the block's layout: small range | big range (132 / 140 KiB)
  // The XCD this launch's workgroup 0 runs on: the fold that follows on the
  // same stream starts dealing its workgroups there too
  // (tools/microbench/xcd_slow.hip), and splits its work by it (xcd_share).
  if (blockIdx.x == 0 && threadIdx.x == 0) a.ctr->xcd = __builtin_amdgcn_s_getreg((3 << 11) | 20);
  for (int t = threadIdx.x; t < kRsClasses; t += blockDim.x) {
    h[t] = 0;
    cur[t] = 0;
  }
  __syncthreads();
  // 32-bit packet indexes (count <= kRsMaxCount): fewer registers per packet in flight
  uint32_t lo, hi;
  {
    uint64_t l, h_;
    pass_range(a.count, l, h_);
    lo = (uint32_t)l;
    hi = (uint32_t)h_;
  }
  const bool one = hi - lo <= (uint32_t)U * blockDim.x;  // block-uniform
  int odd = 0;  // a big packet not starting or ending on a 4-byte word
  // Per packet, packed (3 VGPRs): the descriptor words and class | rank << 10.
  uint32_t dlo[U], dhi[U], cr[U];
  // One round: descriptors of U packets per thread read at once
  // (raw loads first, unconditional with the index clamped, arithmetic after:
  // an add on a loaded value inside a per-packet branch made the compiler
  // wait for each load before issuing the next), then classified and ranked
  // in their class by an LDS atomic on `ctr` (h in the first sweep, cur in
  // the second); packets that are not bucketed are marked for the gather.
  auto round = [&](uint32_t r0, uint32_t *ctr, bool first) {
    uint64_t addr[U];
    uint32_t n[U];
#pragma unroll
    for (int k = 0; k < U; ++k) {
      uint32_t i = r0 + (uint32_t)k * blockDim.x + threadIdx.x;
      i = i < hi ? i : hi - 1;
      addr[k] = OFF ? a.off[i] : (uint64_t)i * a.stride;
      n[k] = LEN ? a.len[i] : a.fixed_len;
    }
#pragma unroll
    for (int k = 0; k < U; ++k) {
      const uint32_t i = r0 + (uint32_t)k * blockDim.x + threadIdx.x;
      const uint64_t ad = addr[k] + (uint64_t)(uintptr_t)a.base + a.l3_offset;
      const uint32_t c = i < hi ? rs_class(ad, n[k]) : 0u;
      const uint32_t rk = (c && !(ABL & 2)) ? atomicAdd(&ctr[c], 1u) : 0u;
      odd |= (c > (uint32_t)kRsBigBase && ((ad | n[k]) & 3u)) ? 1 : 0;
      if (first && i < hi && !c) a.pos_of[i] = 0xFFFFFFFFu;  // the gather pass computes it
      dlo[k] = (uint32_t)ad;
      dhi[k] = (uint32_t)(ad >> 32) | (n[k] << 16);
      cr[k] = c | (rk << 10);
    }
  };
  for (uint32_t r0 = lo; r0 < hi; r0 += U * blockDim.x) round(r0, h, true);  // block-uniform
  if (__syncthreads_or(odd) && threadIdx.x == 0) atomicOr(&a.ctr->odd, 1u);
  if (ABL & 1) {  // keep the round's results live
    uint32_t x = 0;
#pragma unroll
    for (int k = 0; k < U; ++k) x ^= cr[k] ^ dlo[k] ^ dhi[k];
    if (x == 0x9E3779B9u) a.pos_of[threadIdx.x] = x;
    return;
  }

  // Block scan over the classes, one per thread (one barrier: each wave
  // scans its 64 classes, then adds the totals of the waves before it).
  const uint32_t t = threadIdx.x, wid = t >> 6;
  const uint32_t cnt = t < (uint32_t)kRsClasses ? h[t] : 0u;
  const bool big = t > (uint32_t)kRsBigBase && t < (uint32_t)kRsClasses;
  const uint32_t L = big ? t - (uint32_t)kRsBigBase : 0u;
  const uint32_t G = big ? (cnt + 7u) >> 3 : 0u;
  const uint32_t Sm = big ? 0u : cnt;  // class 0 is never counted
  const uint32_t f = (big && cnt) ? 1u : 0u;
  const uint64_t W = (uint64_t)G * (4u * L + a.group_cost);
  uint32_t ig = wave_scan(G), is = wave_scan(Sm), jf = wave_scan(f);
  uint64_t iw = wave_scan(W);
  if ((t & 63u) == 63u) {
    wg[wid] = ig;
    wsm[wid] = is;
    wf[wid] = jf;
    ww[wid] = iw;
  }
  __syncthreads();
  for (uint32_t w = 0; w < wid; ++w) {  // wave-uniform
    ig += wg[w];
    is += wsm[w];
    jf += wf[w];
    iw += ww[w];
  }
  if (t == blockDim.x - 1) {  // block totals: reserve the ranges
    const unsigned long long old =
        ig ? atomicAdd(&a.ctr->pool, ((unsigned long long)iw << kRsGroupBits) | ig) : 0ull;
    blk_g0 = (uint32_t)(old & ((1ull << kRsGroupBits) - 1u));
    blk_s0 = old >> kRsGroupBits;
    blk_small = is ? atomicAdd(&a.ctr->small, is) : 0u;
    blk_stot = is;
    blk_total = is + 8u * ig;
    const bool st = !(ABL & 32) && one && is + 8u * ig <= kStage;
    a.blk[blockIdx.x] = RsBlock{blk_g0, ig, ig ? jf : 0u, blk_small, is, st ? 1u : 0u, blk_s0, iw};
  }
  __syncthreads();
  const uint32_t Stot = blk_stot, total = blk_total;
  const bool staged = !(ABL & 32) && one && total <= kStage;  // block-uniform
  // at[c]: the class's first position -- in the LDS layout when staged, else in its pool
  if (t < (uint32_t)kRsClasses)
    at[t] = staged ? (big ? Stot + 8u * (ig - G) : is - Sm) : big ? 8u * (blk_g0 + ig - G) : blk_small + is - Sm;
  if (f) a.runs[(uint64_t)blockIdx.x * kRsRuns + (jf - 1u)] = RsRun{blk_g0 + ig - G, G, L, 0u, blk_s0 + iw - W};
  __syncthreads();
  if (ABL & 4) {
    uint32_t x = 0;
#pragma unroll
    for (int k = 0; k < U; ++k) x ^= cr[k] ^ dlo[k] ^ dhi[k];
    if (x == 0x9E3779B9u) a.pos_of[threadIdx.x] = x;
    return;
  }

  auto place = [&](uint32_t r0) {
#pragma unroll
    for (int k = 0; k < U; ++k) {
      const uint32_t i = r0 + (uint32_t)k * blockDim.x + threadIdx.x;
      const uint32_t c = cr[k] & 1023u, rk = cr[k] >> 10;
      if (i >= hi || !c) continue;
      const RsDesc d{dlo[k], dhi[k]};
      const bool bc = c > (uint32_t)kRsBigBase;
      const uint32_t p = at[c] + rk;
      RsDesc *D = bc ? a.bdesc : a.desc;
      // streaming stores: the folds that follow read these once, and dirty
      // lines left in the caches would be written back into their read stream
      if (!(ABL & 16)) {
        __builtin_nontemporal_store(d.lo, &D[p].lo);
        __builtin_nontemporal_store(d.hi, &D[p].hi);
      }
      if (!(ABL & 8)) __builtin_nontemporal_store(bc ? a.small_cap + p : p, &a.pos_of[i]);
      if (bc && rk + 1u == h[c])  // the class's last packet pads its run's last group with copies of itself
        for (uint32_t q = p + 1u; q & 7u; ++q) a.bdesc[q] = d;
    }
  };
  if (staged) {  // block-uniform: the round's descriptors are still in registers
    const uint32_t big0 = 8u * blk_g0, small0 = blk_small;
#pragma unroll
    for (int k = 0; k < U; ++k) {
      const uint32_t i = lo + (uint32_t)k * blockDim.x + threadIdx.x;
      const uint32_t c = cr[k] & 1023u, rk = cr[k] >> 10;
      if (i >= hi || !c) continue;
      const uint64_t d = ((uint64_t)dhi[k] << 32) | dlo[k];
      const bool bc = c > (uint32_t)kRsBigBase;
      const uint32_t lp = at[c] + rk;
      stage[lp] = d;
      if (!(ABL & 8)) __builtin_nontemporal_store(lp, &a.pos_of[i]);  // the gather maps the block's layout back
      if (bc && rk + 1u == h[c])  // the class's last packet pads its run's last group with copies of itself
        for (uint32_t q = lp + 1u; (q - Stot) & 7u; ++q) stage[q] = d;
    }
    __syncthreads();
    if (ABL & 16) return;
    uint64_t *sm = reinterpret_cast<uint64_t *>(a.desc) + small0;
    uint64_t *bg = reinterpret_cast<uint64_t *>(a.bdesc) + big0 - Stot;
    // streaming stores: the folds that follow read these once, and dirty
    // lines left in the caches would be written back into their read stream
#pragma unroll 4
    for (uint32_t j = threadIdx.x; j < total; j += blockDim.x)
      __builtin_nontemporal_store(stage[j], (j < Stot ? sm : bg) + j);
    return;
  }
  if (one) {  // block-uniform: the round's descriptors are still in registers
    place(lo);
    return;
  }
  for (uint32_t r0 = lo; r0 < hi; r0 += U * blockDim.x) {
    round(r0, cur, false);
    place(r0);
  }
}

// out[i] for packet i, which the bucket pass left to the gather (n < 44:
// Sarwate loop here; an invalid length: 0), or from its result v.
__device__ __forceinline__ uint32_t gather_one(const RsckArgs &a, uint64_t i, uint32_t p, uint32_t v) {
  if (p == 0xFFFFFFFFu) {
    uint64_t addr;
    uint32_t n;
    rs_packet(a, i, addr, n);
    v = 0u;
    if (n >= 4u && n <= kMaxLen) {
      v = icrc_small(addr, n);
      if (a.verify) v = gload4_unaligned((uintptr_t)(addr + n - 4u)) == v ? 1u : 0u;
    }
    return v;
  }
  if (a.verify) {  // out = trailer holds the ICRC
    uint64_t addr;
    uint32_t n;
    rs_packet(a, i, addr, n);
    v = gload4_unaligned((uintptr_t)(addr + n - 4u)) == v ? 1u : 0u;
  }
  return v;
}

// Bytes [0, M) of the packet kept, invariant masks, seed: word i of a slot whose
// first byte is packet-relative offset rel (any sign, any alignment).  Branch
// free (one-direction 64-bit shifts + selects): a divergent branch here made
// the compiler drain vmcnt(0) at its join, stalling the whole load ring.
__device__ __forceinline__ uint32_t edge_word(uint32_t w, int rel, int M) {
  const uint32_t keep = byte_span_mask(-rel, M - rel);
  const uint32_t sh = (uint32_t)(rel + 3 < 0 ? 0 : rel + 3 > 63 ? 63 : rel + 3);  // byte b <-> bit/byte rel + b
  const uint32_t bits = (uint32_t)(((kMaskBits << 3) >> sh) & 0xFu);
  const uint32_t orm = (rel > -4 && rel < 40) ? (expand_nibble(bits) & keep) : 0u;
  const uint64_t s64 = (uint64_t)kSeed << 24;  // seed byte k at byte k + 3
  const uint32_t sx = (rel > -4 && rel < 4) ? (uint32_t)(s64 >> (8u * (sh & 7u))) : 0u;
  return ((w & keep) | orm) ^ sx;
}

// edge_word with no end (M past the word) as two masks for a word at offset
// rel: edge_word(w, rel, inf) = (w & ~drop) ^ set, so a fold that XORed w in
// whole fixes it with xr ^= (w & drop) ^ set.
__device__ __forceinline__ uint32_t __attribute__((ext_vector_type(2))) head_masks(int rel) {
  const uint32_t keep = byte_span_mask(-rel, 4);
  const uint32_t sh = (uint32_t)(rel + 3 < 0 ? 0 : rel + 3 > 63 ? 63 : rel + 3);
  const uint32_t bits = (uint32_t)(((kMaskBits << 3) >> sh) & 0xFu);
  const uint32_t orm = (rel > -4 && rel < 40) ? (expand_nibble(bits) & keep) : 0u;
  const uint64_t s64 = (uint64_t)kSeed << 24;
  const uint32_t sx = (rel > -4 && rel < 4) ? (uint32_t)(s64 >> (8u * (sh & 7u))) : 0u;
  return {~(keep & ~orm), orm ^ sx};
}


}  // namespace

// f(integral_constant<0>), ..., f(integral_constant<N - 1>), unrolled.
template <class F, uint32_t... I>
__device__ __forceinline__ void static_for_impl(F &&f, std::integer_sequence<uint32_t, I...>) {
  (f(std::integral_constant<uint32_t, I>{}), ...);
}
template <uint32_t N, class F>
__device__ __forceinline__ void static_for(F &&f) {
  static_for_impl(f, std::make_integer_sequence<uint32_t, N>{});
}

// ABL (timing-only ablations, tools/microbench/shard.hip, bucket_abl.hip):
// 1 no table fold, 2 no finish, 8 no edge masks, 16 no result
// slots / stores, 16384 no line loads,
// 524288 per-wave s_memrealtime stamps into a.out, 8 words per wave: entry,
// tables built (the barrier), work split found, end, first line arrived,
// counters arrived, table build's own instructions done, the work of the
// wave's groups.
// =======================================================================
// Small packets of the ragged path (<= kRsSmallL lines: the 64 / 256-byte
// share of C4): ONE LANE PER PACKET, descriptors [0, ctr->small) of the
// buckets.  8 lanes per packet (the fold above) is too coarse for them, and
// the round-1 piece kernel (one 64-byte piece per lane; git history) paid a
// GF(2) re-alignment, prefix XOR and end multiply per packet.  Here a lane folds its
// packet's whole byte stream from a ZERO register with no multiply at all:
//
//   stream = 4 x 0xFF || masked L3[0, M)        (M = n - 4)
//
// (the CRC-32 init ~0 folded over the 8-byte 0xFF prefix of calc_icrc,
// shuffle_egress.p4:465, is the zero register over 00 x 4 || FF x 4, and
// leading zeros are free; tests/test_kernel_algebra.py::
// test_small_lane_end_aligned_stream), ICRC = ~register.  The
// stream is cut into 16-byte blocks that END at the packet's covered end
// e = addr + M, so no trailing byte is ever folded; leading bytes before the
// prefix are zeros, which a zero register ignores.  That lets every lane of
// a wave fold the same number of blocks Kmax (a multiple of 4: lanes with
// shorter packets start with all-zero blocks), so the loop has no divergence
// and no exec-masked memory op.  Block j needs the 16-byte native units N and
// N + 16 (N = e - (e & 15) - 16 (Kmax - j)), requested up to 17 at a time
// before the fold (memory-level parallelism); loads are clamped to the units
// that hold packet bytes (never another page) and whatever a clamped unit
// holds is masked away by packet-relative offset.  A block's words come out
// of the two units by a 2-level word funnel and v_alignbyte (phase e & 15).
// =======================================================================
__device__ __forceinline__ uint32_t small_word(uint32_t w, int r) {  // r = packet-relative offset of byte 0
  const uint32_t keep = byte_span_mask(-r, 4);            // bytes at r >= 0: packet data
  const uint32_t pre = byte_span_mask(-4 - r, -r);        // bytes at -4 <= r < 0: the 0xFF prefix
  // invariant fields -> 0xFF; outside [0, 40) the shifted map is empty, so no
  // range test (a select on r became a divergent branch)
  const uint32_t sh = (uint32_t)(r + 3 < 0 ? 0 : r + 3 > 63 ? 63 : r + 3);
  const uint32_t bits = (uint32_t)(((kMaskBits << 3) >> sh) & 0xFu);
  return (w & keep) | pre | (expand_nibble(bits) & keep);
}

// small_word for a word-aligned r (a multiple of 4): whole-word keep, the
// 0xFF prefix word at -4, the IPv4 mask words of offsets 0, 8, 24, 32.
__device__ __forceinline__ uint32_t small_word_aligned(uint32_t w, int r) {
  const uint32_t keep = (uint32_t)(r >= 0) * 0xFFFFFFFFu;
  const uint32_t orm = ((uint32_t)(r == -4) * 0xFFFFFFFFu) | ((uint32_t)(r == 0) * kMaskW0) |
                       ((uint32_t)(r == 8) * kMaskW2) | ((uint32_t)(r == 24) * kMaskW6) |
                       ((uint32_t)(r == 32) * kMaskW8);
  return (w & keep) | orm;
}

// One packet's stream in icrc_rsmall_kernel.
struct SmallPk {
  uint64_t ufirst, ulast, N0;  // the packet's first / last 16-byte unit, native unit of block 0
  uint32_t sb, m2, m1;         // end phase: byte shift, word-shift selects (all ones / zero)
  int rel;                     // packet-relative offset of the next block
  uint32_t reg;

  __device__ __forceinline__ void init(const RsDesc &d, uint32_t Kmax) {
    const uint64_t addr = ((uint64_t)(d.hi & 0xFFFFu) << 32) | d.lo;
    const uint32_t M = (d.hi >> 16) - 4u;
    const uint64_t e = addr + M;
    const uint32_t t = (uint32_t)(e & 15u);
    sb = t & 3u;
    m2 = 0u - ((t >> 3) & 1u);
    m1 = 0u - ((t >> 2) & 1u);
    ufirst = addr & ~15ull;
    ulast = (e - 1u) & ~15ull;
    N0 = e - t - 16ull * Kmax;
    rel = (int)M - 16 * (int)Kmax;
    reg = 0u;
  }
  __device__ __forceinline__ u32x4 unit(uint32_t k) const {  // native unit k, clamped to the packet's
    uint64_t u = N0 + 16ull * k;
    u = u < ufirst ? ufirst : (u > ulast ? ulast : u);
    return gload16(u);  // plain: non-temporal scattered unit reads took 69 instead of 40 us on C4
  }
  // Blocks j0 .. j0 + KB - 1: all KB + 1 units they need are requested at
  // once, then folded.  (A ring of 4-8 units in flight measured ~2x slower
  // on C4's scattered small packets, tools/microbench/mb_scatter.hip: the
  // memory-level parallelism of one lane is what these reads need.)
  // WA: every packet of the wave starts and ends on a 4-byte word (the wave-
  // uniform common case: C4, NIC rings): no byte shift, whole-word masks.
  // MASK: which blocks get the head masks (prefix / invariant fields / bytes
  // before the packet), branch-free: 1 = blocks 0..3 (the first chunk of a
  // wave whose packets all start their heads there: M >= 16 Kmax - 24), 2 = all
  // (lanes with shorter packets start later), 0 = none.  (A wave-uniform
  // branch on "is some lane in its head" made the compiler wait for every
  // outstanding load (vmcnt(0)) before each block: 2x slower.)
  template <int KB, bool WA, int MASK, class Step>
  __device__ __forceinline__ void chunk(const Step &step, uint32_t j0) {
    u32x4 U[KB + 1];
#pragma unroll
    for (int k = 0; k <= KB; ++k) U[k] = unit(j0 + k);
    blocks<KB, WA, MASK>(step, U);
  }
  // Fold blocks 0 .. KB-1 of units U (block j from units j, j + 1).
  template <int KB, bool WA, int MASK, class Step>
  __device__ __forceinline__ void blocks(const Step &step, const u32x4 (&U)[KB + 1]) {
#pragma unroll
    for (int j = 0; j < KB; ++j) {
      // Block j's 4 words from units j, j + 1: X[k] = W[(t >> 2) + k] by
      // bitwise selects (written as ternaries, the compiler turned the
      // funnel into a dynamically indexed array in scratch), then
      // v_alignbyte by the byte phase.
      const u32x4 c = U[j], n = U[j + 1];
      const uint32_t W[8] = {c[0], c[1], c[2], c[3], n[0], n[1], n[2], n[3]};
      uint32_t V[6], X[5], w[4];
#pragma unroll
      for (int k = 0; k < 6; ++k) V[k] = __builtin_amdgcn_bitop3_b32(m2, W[k + 2], W[k], 0xCA);
#pragma unroll
      for (int k = 0; k < 5; ++k) X[k] = __builtin_amdgcn_bitop3_b32(m1, V[k + 1], V[k], 0xCA);
#pragma unroll
      for (int i = 0; i < 4; ++i) w[i] = WA ? X[i] : __builtin_amdgcn_alignbyte(X[i + 1], X[i], sb);
      if (MASK == 2 || (MASK == 1 && j < 4)) {
#pragma unroll
        for (int i = 0; i < 4; ++i) w[i] = WA ? small_word_aligned(w[i], rel + 4 * i) : small_word(w[i], rel + 4 * i);
      }
#pragma unroll
      for (int i = 0; i < 4; ++i) reg = step(reg, w[i]);
      rel += 16;
    }
  }
};

// small_icrc's CRC step over the slice-by-4 tables in LDS (fill_tables).
struct Step4 {
  const uint32_t *lds;
  LaneTab lt;
  __device__ __forceinline__ uint32_t operator()(uint32_t r, uint32_t w) const { return step4(lds, lt, r, w); }
};
// ... through the nibble table of x^32 (16 entries per nibble position, in 16
// banks: conflict-free for any lane pattern): 8 lookups instead of 4, for
// the fold kernel, whose 128 KiB of LDS tables advance 128 bytes a step.
struct StepNib {
  const uint32_t *t;  // [128]: entry 16 w + v = (nibble v at bits 4w..4w+3) * x^32
  __device__ __forceinline__ uint32_t operator()(uint32_t r, uint32_t w) const {
    const uint32_t v = r ^ w;
    uint32_t e[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) e[k] = t[16 * k + __builtin_amdgcn_ubfe(v, 4 * k, 4)];
    return xor3(xor3(e[0], e[1], e[2]), xor3(e[3], e[4], e[5]), e[6] ^ e[7]);
  }
};

// The ICRC of every lane's one-line packet d: wave-collective (every lane of
// the wave calls it together; a lane without a packet passes a copy of a
// valid descriptor and ignores the result), since the wave's shape -- its
// largest block count, whether every packet is word-aligned, half-line --
// is decided by ballots.  step(r, w): the register after folding word w
// into r (step4 over the slice-by-4 tables, fill_tables; or nibble lookups).
template <class Step>
__device__ __forceinline__ uint32_t small_icrc(const Step &step, const RsDesc &d, uint32_t lane) {
  uint32_t K = (((d.hi >> 16) - 4u) + 4u + 15u) >> 4;  // this lane's blocks
  // the wave's largest, rounded up to a multiple of 4: by ballots for
  // one-line packets (K <= 8), a shuffle reduction beyond
  uint32_t Kmax;
  if (__builtin_amdgcn_ballot_w64(K > 4u) == 0) {
    Kmax = 4u;
  } else if (__builtin_amdgcn_ballot_w64(K > 8u) == 0) {
    Kmax = 8u;
  } else {
#pragma unroll
    for (int w = 32; w >= 1; w >>= 1) K = max(K, (uint32_t)__shfl_xor((int)K, w));
    Kmax = __builtin_amdgcn_readfirstlane((K + 3u) & ~3u);
  }
  // wave-uniform variants: word-aligned packets; every packet's head in blocks 0..3
  const bool wa = __builtin_amdgcn_ballot_w64(((d.lo | (d.hi >> 16)) & 3u) != 0) == 0;
  // heads in blocks 0..3: rel_4 = M - 16 Kmax + 64 >= 40 for every lane
  const bool uk = __builtin_amdgcn_ballot_w64((d.hi >> 16) - 4u + 24u < 16u * Kmax) == 0;
  // Half-line packets: every covered byte in one aligned 64-byte half
  // line hb .. hb + 63 whose last 16-byte unit holds the covered end, not
  // at the half line's end (C4's 64-byte packets: 64-byte aligned, 60
  // covered bytes).  For a wave of them the 5 units of the 4 blocks are
  // the half line's units 0, 0, 1, 2, 3, and they are read coalesced: in
  // load c the 4 lanes of quad p read units 0..3 of lane 4 p + c's half
  // line (64 contiguous bytes), and a 4 x 4 quad transpose hands every lane
  // its own -- instead of every lane reading its packet's units alone, 64
  // lines apart (the access pattern that costs C1's direct kernel, see the
  // quad kernel in icrc_kernels.hip).  (Kmax = 4: a half-line packet of
  // 61..63 covered bytes needs a fifth block for its prefix.)
  const uint64_t pa = ((uint64_t)(d.hi & 0xFFFFu) << 32) | d.lo;
  const uint64_t pe = pa + ((d.hi >> 16) - 4u);
  const uint64_t hb = (pe - 1u) & ~63ull;
  const bool half = pa >= hb && ((uint32_t)pe & 63u) > 48u;
  SmallPk P;
  if (Kmax == 4u && __builtin_amdgcn_ballot_w64(!half) == 0) {  // wave-uniform: a wave of half-line packets
    const uint32_t hlo = (uint32_t)hb, hhi = (uint32_t)(hb >> 32), q = lane & 3u;
    auto at = [&](uint32_t lo, uint32_t hi) { return ((uint64_t)hi << 32 | lo) + 16u * q; };
    u32x4 H[4];
    H[0] = gload16(at(dpp_quad_bcast<0>(hlo), dpp_quad_bcast<0>(hhi)));
    H[1] = gload16(at(dpp_quad_bcast<1>(hlo), dpp_quad_bcast<1>(hhi)));
    H[2] = gload16(at(dpp_quad_bcast<2>(hlo), dpp_quad_bcast<2>(hhi)));
    H[3] = gload16(at(dpp_quad_bcast<3>(hlo), dpp_quad_bcast<3>(hhi)));
    quad_transpose(H, lane & 3u);
    const u32x4 U[5] = {H[0], H[0], H[1], H[2], H[3]};
    P.init(d, 4u);
    if (wa && uk)
      P.blocks<4, true, 1>(step, U);
    else if (uk)
      P.blocks<4, false, 1>(step, U);
    else
      P.blocks<4, false, 2>(step, U);
    return ~P.reg;
  }
  P.init(d, Kmax);
  auto run = [&](auto words, auto uniform) __attribute__((always_inline)) {
    constexpr bool WA = decltype(words)::value;
    constexpr int M1 = decltype(uniform)::value ? 1 : 2, M2 = decltype(uniform)::value ? 0 : 2;
    // Kmax = 8 q + r (r = 0 or 4): a first chunk of r or 8 blocks, then
    // chunks of 8 (one-line packets: M <= 124, Kmax <= 8 -- one chunk, at
    // most 9 units = 36 VGPRs in flight)
    uint32_t j = 0;
    if ((Kmax & 7u) == 4u) {  // wave-uniform
      P.chunk<4, WA, M1>(step, 0);
      j = 4;
    } else {
      P.chunk<8, WA, M1>(step, 0);
      j = 8;
    }
    for (; j < Kmax; j += 8) P.chunk<8, WA, M2>(step, j);
  };
  if (wa && uk)
    run(std::true_type{}, std::true_type{});
  else if (uk)
    run(std::false_type{}, std::true_type{});
  else
    run(std::false_type{}, std::false_type{});
  return ~P.reg;
}

template <int ABL>
__global__ __launch_bounds__(kBlock) void icrc_rsck_kernel(RsckArgs a) {
  // Result slots per wave (a round of 8 groups leaves in one store; a store
  // holds back every load queued behind it in vmcnt until its write is
  // acknowledged: the stores cost ~4 % of the fold on a 4 GiB mix, the same
  // for rounds of 8 or 16 groups and 4- or 8-byte stores, profiles/r02/rsck_abl_*.txt).
  constexpr uint32_t kSlots = 64, kRound = kSlots / 8;
  constexpr uint32_t kBlk = 128;                          // words per descriptor block (8 groups x 8 x 8 B)
  constexpr uint32_t kWaveWords = kSlots + 2 * kBlk + 64;  // slots | 2-block ring | 8-group info FIFO
  // lines in flight per wave: 6 (with the quiet blocks below, 8 lines in
  // flight left no registers for them: 128 VGPRs and spills; fold of a
  // C4-shaped 5.3 GiB batch 953 -> 930 us, profiles/r03/fold_var.txt)
  constexpr int D = 6;
  // Finish tables first, so every lookup's constant part fits a ds_read's
  // 16-bit offset: x^-32 nibble table (128 words) | x^(-128 s) nibble tables
  // (8 x 132 words: rows padded by 4 words so the 8 lane slots spread over
  // the banks) | head masks (32 words) | x^-64, x^-96, x^32 nibble tables
  // (3 x 128 words) | 128 KiB slice-by-4 tables | 1 KiB tz bases | 1.5 KiB
  // per wave = 159.3 KiB.
  constexpr uint32_t kQtStride = kFinQtStride, kSmallWords = kFinFold;  // 1600 (build_fin_tables): a multiple of 32 words
  __shared__ uint32_t lds[kSmallWords + kLdsWords + kTzWords + kWaves * kWaveWords];
  uint32_t *xtl = lds;
  uint32_t *qtl = lds + 128;
  uint32_t *etl = lds + 128 + 8 * kQtStride;  // whole-word head masks: (or, xor) of word k = rel / 4
  uint32_t *x2tl = etl + 32, *x3tl = etl + 160;  // nibble tables of x^-64, x^-96
  uint32_t *tab = lds + kSmallWords;
  uint32_t *tzl = tab + kLdsWords;

  const uint32_t lane = threadIdx.x & 63;
  const uint32_t wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const uint32_t s = lane & 7, g = lane >> 3;
  const uint32_t t_entry = (ABL & 524288) ? (uint32_t)__builtin_amdgcn_s_memrealtime() : 0u;

  // Everything a wave needs from memory before it can stream is requested at
  // once, ahead of the table build: its table entries, the counters and
  // every pass block's work range.  The work split then costs one more round
  // trip (the runs of the two pass blocks holding the wave's share ends),
  // issued before the table build too, and the wave's first descriptors and
  // lines are in flight before the workgroup barrier.  (The round-4 fold
  // chased blocks and runs through up to a dozen dependent loads after the
  // barrier: at C4's 8-GPU shard its waves found their share 11 us after
  // entry at the median, 27 us at worst, tools/microbench/shard.hip,
  // profiles/r05/s1_mb_shard_baseline.txt.)
  const TableRegs tab_v = table_load(g_tab128);
  const uint32_t fin0 = a.fin[threadIdx.x], fin1 = a.fin[threadIdx.x + 1024u < kSmallWords ? threadIdx.x + 1024u : 0u];
  const uint32_t tz_v = a.tzb[threadIdx.x < kTzWords ? threadIdx.x : 0];
  const RsCounters C = *a.ctr;
  constexpr int kBq = kPassBlocks / 64;  // pass blocks per lane
  uint64_t bs0[kBq], bwk[kBq];
  uint32_t brn[kBq];
#pragma unroll
  for (int k = 0; k < kBq; ++k) {  // unconditional loads, index clamped: issued back to back
    const uint32_t bb = 64u * (uint32_t)k + lane;
    const RsBlock *B = a.blk + (bb < a.nblk ? bb : 0u);
    bs0[k] = B->s0;
    bwk[k] = B->work;
    brn[k] = B->runs;
  }
  // The big pool: NG groups, S weighted work (the bucket pass's packed
  // counter); block b's groups [g0, g0 + groups) hold work [s0, s0 + work),
  // its runs split that range by class.
  const uint32_t NG = (uint32_t)(C.pool & ((1ull << kRsGroupBits) - 1u));
  const uint64_t S = C.pool >> kRsGroupBits;
  // The small pool's one-line packets (a.small_in_fold): rounds of 64, one
  // lane per packet, split over the waves in the proportion of their big
  // work (below) -- spread thin, as one round costs a wave two round trips
  // that a wave with many of them could not hide.
  const uint32_t NS = a.small_in_fold ? C.small : 0u;
  const uint32_t NC = (NS + 63u) >> 6;
  if (NG == 0 && NC == 0) return;  // nothing to fold: every wave leaves here (no barrier above)
  const uint32_t t_ctr = (ABL & 524288) ? (uint32_t)__builtin_amdgcn_s_memrealtime() : 0u;
#pragma unroll
  for (int k = 0; k < kBq; ++k) brn[k] = 64u * (uint32_t)k + lane < a.nblk ? brn[k] : 0u;
  // This wave's groups: those whose first line lies in its share of the work.
  const uint64_t wave = (uint64_t)blockIdx.x * kWaves + wid;
  const uint64_t nwaves = (uint64_t)gridDim.x * kWaves;
  const uint64_t T = NG ? S : NC;  // the work split's total (the small rounds when no packet has >= 2 lines)
  uint64_t x0, x1;
  if (a.xw[0] != 0u) {
    xcd_share(T, a.xw, C.xcd, wid, x0, x1);  // weighted by XCD
  } else {
    const uint64_t share = (T + nwaves - 1) / nwaves;
    x0 = wave * share < T ? wave * share : T;
    x1 = x0 + share;
  }
  // the pass block whose work range holds x (ballots over the loaded ranges)
  auto block_of = [&](uint64_t x) -> uint32_t {
    uint32_t b = 0;
#pragma unroll
    for (int k = 0; k < kBq; ++k) {
      const uint64_t m = __ballot(brn[k] != 0u && bs0[k] <= x && x - bs0[k] < bwk[k]);
      if (m) b = 64u * (uint32_t)k + (uint32_t)__builtin_ctzll(m);
    }
    return __builtin_amdgcn_readfirstlane(b);
  };
  auto runs_of = [&](uint32_t b) -> uint32_t {  // (scalar selects: a VGPR select became a scratch array)
    uint32_t v = 0;
#pragma unroll
    for (int k = 0; k < kBq; ++k) {
      const uint32_t c = __builtin_amdgcn_readlane(brn[k], b & 63u);
      v = (b >> 6) == (uint32_t)k ? c : v;
    }
    return v;
  };
  const uint32_t b0 = block_of(x0), b1 = block_of(x1);
  const uint32_t n0 = runs_of(b0), n1 = runs_of(b1);
  const RsRun *R0 = a.runs + (uint64_t)b0 * kRsRuns, *R1 = a.runs + (uint64_t)b1 * kRsRuns;
  RsRun Q0 = R0[lane < n0 ? lane : 0u], Q1 = R1[lane < n1 ? lane : 0u];  // in flight during the table stores

  // The tables' words arrived with the counters: LDS stores only.  (Built
  // in the kernel from kernel-argument bases, the finish tables indexed the
  // arguments by lane -- vector loads from the argument segment, each
  // waiting for every load before it, the runs included: ~4 us of the
  // fold's start at C4's 8-GPU shard, profiles/r05/NOTES.md.)
  table_write(tab, tab_v);
  if (threadIdx.x < kTzWords) tzl[threadIdx.x] = tz_v;
  lds[threadIdx.x] = fin0;  // the finish tables, built by the host (icrc_math.h build_fin_tables)
  if (threadIdx.x + 1024u < kSmallWords) lds[threadIdx.x + 1024u] = fin1;

  // First group whose work starts at or after x: the run of the pass block
  // (b, its nr runs at R; Q = this lane's run of the first 64) holding x.
  auto group_at = [&](uint64_t x, uint32_t nr, const RsRun *R, RsRun Q) -> uint32_t {
    if (x >= S) return NG;  // wave-uniform
    for (uint32_t r0 = 0; r0 < nr; r0 += 64) {  // (more than 64 classes in one pass block: rare)
      if (r0 != 0) Q = R[r0 + lane < nr ? r0 + lane : r0];
      const uint64_t m = __ballot(r0 + lane < nr && Q.s0 <= x &&
                                  x - Q.s0 < (uint64_t)Q.groups * (4u * Q.L + a.group_cost));
      if (m) {  // wave-uniform
        const uint32_t r = (uint32_t)__builtin_ctzll(m);
        const uint32_t g0 = __builtin_amdgcn_readlane(Q.g0, r), gs = __builtin_amdgcn_readlane(Q.groups, r);
        const uint32_t L = __builtin_amdgcn_readlane(Q.L, r);
        const uint64_t s0 = ((uint64_t)__builtin_amdgcn_readlane((uint32_t)(Q.s0 >> 32), r) << 32) |
                            __builtin_amdgcn_readlane((uint32_t)Q.s0, r);
        // x - s0 < gs w, the run's work: below 2^31 for every product shape
        // (a one-round pass block holds <= 17 K packets, gs w < 2^23), so a
        // 32-bit division (a 64-bit one is a long expansion on the start-up's
        // critical path); blocks of several rounds (RICRC_RS_PASS_GRID) can
        // hold runs past it: 64 bits there (wave-uniform)
        const uint32_t w = 4u * L + a.group_cost;  // quarter line-steps
        const uint64_t dx = x - s0;
        const uint64_t q = g0 + (dx < (1ull << 31) ? ((uint32_t)dx + w - 1u) / w : (dx + w - 1u) / w);
        const uint32_t gend = g0 + gs < NG ? g0 + gs : NG;  // (never past the pool)
        return q < gend ? (uint32_t)q : gend;
      }
    }
    return NG;  // (not reached: x < S lies in a run)
  };
  const uint32_t t_tb = (ABL & 524288) ? (uint32_t)__builtin_amdgcn_s_memrealtime() : 0u;
  const uint32_t q_begin = group_at(x0, n0, R0, Q0), q_end = group_at(x1, n1, R1, Q1);
  const uint32_t t_split = (ABL & 524288) ? (uint32_t)__builtin_amdgcn_s_memrealtime() : 0u;
  const bool work = q_begin < q_end;  // wave-uniform
  // Small rounds [c_begin, c_end): dealt evenly to the waves of slots
  // 0 .. small_slots - 1 (12: the four youngest slots of a workgroup, the
  // last to finish their equal shares, take none; at C4's 8-GPU shard 0.1542
  // -> 0.1512 ms per step against folding them in the gather, at C4 0.9825 ->
  // 0.9730, where slots 0..15 measured 0.981 and a share by each wave's work
  // 0.984, profiles/r05/NOTES.md), or -- small_slots = 0, or no packet of
  // >= 2 lines -- the wave's fraction [x0, x1) / T of them (consecutive
  // waves' fractions meet, so the rounds are dealt exactly once).
  uint32_t c_begin = (uint32_t)((x0 < T ? x0 : T) * NC / T), c_end = (uint32_t)((x1 < T ? x1 : T) * NC / T);
  if (a.small_slots != 0u && NG != 0u) {  // wave-uniform
    const uint32_t sl = a.small_slots;
    const uint64_t E = (uint64_t)gridDim.x * sl, e = (uint64_t)blockIdx.x * sl + wid;
    c_begin = wid < sl ? (uint32_t)(e * NC / E) : 0u;
    c_end = wid < sl ? (uint32_t)((e + 1u) * NC / E) : 0u;
  }
  auto small_desc = [&](uint32_t c) {
    const uint32_t j = 64u * c + lane;
    return a.desc[j < NS ? j : NS - 1u];
  };
  // the first round's descriptors, requested with the first descriptor blocks
  RsDesc sd{0u, 0u};
  if (c_begin < c_end) sd = small_desc(c_begin);

  const LaneTab lt{(lane & 31) << 2, ((lane & 31) << 2) | 0x10000u};
  const uint32_t *qrow = qtl + s * kQtStride;
  uint32_t *slots = tzl + kTzWords + wid * kWaveWords;
  uint32_t *dring = slots + kSlots;
  uint32_t *fifo = dring + 2 * kBlk;
  const uint64_t npos = 8ull * NG;

  // Descriptor blocks (8 groups = 64 descriptors of 8 B, lane l holding
  // descriptor l) go through a 2-slot LDS ring, block b in slot b & 1; only
  // the load cursor reads them.  Entering block b it stores block b + 1
  // (loaded into NB when it entered block b - 1, >= 8 lines ago) into the
  // slot block b - 1 used, and requests block b + 2 into NB.  (LDS-DMA would
  // skip the register, but the compiler then waits for it before every LDS
  // read -- the table lookups included.)  The fold cursor gets (a, M) of each
  // group through an 8-entry LDS FIFO the load cursor fills (the fold lags
  // at most 8 lines = 8 groups; each step folds before it loads, so an entry
  // is read before it is reused).
  typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
  auto load_block = [&](uint32_t b) -> u32x2 {
    uint64_t e = (uint64_t)b * 64u + lane;
    e = e < npos ? e : npos - 1;
    return *reinterpret_cast<const u32x2 __attribute__((address_space(1))) *>(
        (uintptr_t)reinterpret_cast<const uint32_t *>(a.bdesc + e));
  };
  auto put_block = [&](uint32_t b, const u32x2 &v) {
    *reinterpret_cast<u32x2 *>(dring + (b & 1u) * kBlk + 2u * lane) = v;
  };
  const uint32_t qb = q_begin, qe = q_end;
  struct LInfo {
    uint64_t line0;  // lane's slot in the packet's first line
  };
  // Load cursor enters group q: line base, L, and (a, M) into the FIFO.
  auto ld_enter = [&](uint32_t q, LInfo &li) -> uint32_t {
    const u32x2 d = *reinterpret_cast<const u32x2 *>(dring + ((q >> 3) & 1u) * kBlk + 2u * (8u * (q & 7u) + g));
    const uint64_t addr = ((uint64_t)(d[1] & 0xFFFFu) << 32) | d[0];
    const uint32_t gM = (d[1] >> 16) - 4u;
    const uint32_t ga = (uint32_t)addr & 127u;
    li.line0 = (addr & ~127ull) + 16u * s;
    fifo[((q & 7u) << 3) | g] = (gM << 7) | ga;
    return __builtin_amdgcn_readfirstlane((ga + gM + 127u) >> 7);  // equal within a group
  };
  // (ABL 16384, timing only: no line loads, a value derived from the address)
  auto line_load = [&](uint64_t addr) -> u32x4 {
    if (ABL & 16384) return u32x4{(uint32_t)addr, (uint32_t)(addr >> 7), lane, (uint32_t)addr * 3u};
    return gload16_nt(addr);
  };
  LInfo ld;
  u32x2 NB = {0u, 0u};
  uint32_t ld_q = qb, ld_k = 0, ld_L = 1;
  auto ld_issue = [&]() -> u32x4 { return line_load(ld.line0 + 128ull * ld_k); };
  auto ld_advance = [&]() {
    if (++ld_k == ld_L) {  // wave-uniform
      ld_k = 0;
      if (ld_q + 1 < qe) {
        ++ld_q;
        if ((ld_q & 7u) == 0) {
          put_block((ld_q >> 3) + 1, NB);
          NB = load_block((ld_q >> 3) + 2);
        }
        ld_L = ld_enter(ld_q, ld);
      } else {
        ld_L = 1;  // done: re-read line 0 of the last group (ld_k wraps to 0 every step)
      }
    }
  };
  // The wave's first descriptor blocks and D lines, requested before the
  // barrier: they arrive while the other waves finish the tables.
  u32x4 ring[D];
  if (work) {  // wave-uniform
    const uint32_t b = qb >> 3;
    put_block(b, load_block(b));
    put_block(b + 1, load_block(b + 1));
    NB = load_block(b + 2);
    __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0)
    ld_L = ld_enter(ld_q, ld);
#pragma unroll
    for (int u = 0; u < D; ++u) {
      __builtin_amdgcn_sched_barrier(0);
      ring[u] = ld_issue();
      ld_advance();
    }
    __builtin_amdgcn_sched_barrier(0);
  }
  __syncthreads();  // the tables are built
  const uint32_t t_tab = (ABL & 524288) ? (uint32_t)__builtin_amdgcn_s_memrealtime() : 0u;
  const uint64_t wave8 = 8ull * wave;
  if ((ABL & 524288) && lane == 0) {
    a.out[wave8] = t_entry;
    a.out[wave8 + 1] = t_tab;
    a.out[wave8 + 2] = t_split;
    a.out[wave8 + 3] = t_split;
    a.out[wave8 + 4] = work ? q_end - q_begin : 0u;
    a.out[wave8 + 5] = t_ctr;
  }
  // The wave's small rounds first, while its first lines are in flight.
  // small_icrc is wave-collective: every lane folds one packet (lanes past
  // the pool a copy of the last, result dropped).
  if (c_begin < c_end) {  // wave-uniform
    const __amdgpu_buffer_rsrc_t ro = make_rsrc(a.res, 4u * NS);
    const StepNib step{lds + kFinStep4};
    auto put = [&](uint32_t c, uint32_t v) {
      const uint32_t pos = 64u * c + lane;
      __builtin_amdgcn_raw_buffer_store_b32(v, ro, pos < NS ? 4u * pos : 0x7FFFFFF0u, 0, 0);
    };
    RsDesc d = sd;
#pragma unroll 1
    for (uint32_t c = c_begin; c < c_end; ++c) {
      const RsDesc dn = small_desc(c + 1u < c_end ? c + 1u : c);  // the next round's, in flight meanwhile
      put(c, small_icrc(step, d, lane));
      d = dn;
    }
  }
  uint32_t done_work = 0;  // (ABL 524288: the work of the wave's groups)
  if (work) {  // wave-uniform
    uint32_t round_q0 = q_begin;  // first group of the current round of result slots
    uint32_t sink = 0;             // timing ablations: values kept live
    auto flush = [&](uint32_t q_stop) {  // groups [round_q0, q_stop) of the round
      const uint32_t valid = 8u * (q_stop - round_q0);
      const __amdgpu_buffer_rsrc_t ro = make_rsrc(a.bres + 8ull * round_q0, 4u * valid);
      __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0): the slot writes have landed
      // slots past `valid` fall outside the range check
      __builtin_amdgcn_raw_buffer_store_b32(slots[lane], ro, 4u * lane, 0, 16);
    };
    // A group's finish: its chain registers rr (after its last line), L lines,
    // first-byte offsets ga and covered lengths gM of its 8 packets (per lane
    // group), its position q in the big pool -> the ICRC into the wave's slot.
    auto finish_group = [&](uint32_t (&rr)[4], uint32_t Lg, uint32_t ga, uint32_t gM, uint32_t q) {
      uint32_t R;
      if (ABL & 2) {
        R = group_xor(rr[0] ^ rr[1] ^ rr[2] ^ rr[3], 3);
      } else {
        // Horner by x^-32 through the nibble table: 8 lookups per multiply
        // (one copy: the 16 entries of a nibble position sit in 16 banks, so
        // any lane pattern is conflict-free) instead of 32 bit-selects.
        // v * (table's constant) ^ x: 8 nibble lookups, an XOR tree of 3-input XORs
        auto nib_mul = [](const uint32_t *t, uint32_t v, uint32_t x) -> uint32_t {
          uint32_t e[8];
#pragma unroll
          for (int w = 0; w < 8; ++w) e[w] = t[16 * w + __builtin_amdgcn_ubfe(v, 4 * w, 4)];
          return xor3(xor3(e[0], e[1], e[2]), xor3(e[3], e[4], e[5]), xor3(e[6], e[7], x));
        };
        // r3 x^-96 + r2 x^-64 + r1 x^-32 + r0: three independent multiplies
        // (Horner chained them: four dependent LDS round trips per finish,
        // which the 2-3-line groups of 256-byte packets could not hide)
        const uint32_t u = nib_mul(x3tl, rr[3], nib_mul(x2tl, rr[2], nib_mul(xtl, rr[1], rr[0])));
        R = group_xor(nib_mul(qrow, u, 0u), 3);  // u * x^(-128 s): lane slot s's nibble table
        // x^(-8 tz), distributed: lane s takes bits 4s..4s+3 of R; basis word
        // 4s from LDS, 4s+1..4s+3 by successive x^-1.
        const uint32_t tz = 128u * Lg - ga - gM;
        uint32_t bw = tzl[2u * tz + s], p = 0;
#pragma unroll
        for (int t = 0; t < 4; ++t) {
          const uint32_t m = (uint32_t)__builtin_amdgcn_sbfe((int)R, (int)(4u * s + t), 1);
          p = and_xor(m, bw, p);
          bw = and_xor((uint32_t)((int32_t)bw >> 31), kXInv, bw << 1);
        }
        R = group_xor(p, 3);
      }
      if (ABL & 524288) done_work += 4u * Lg + a.group_cost;
      if (ABL & 16) {
        sink ^= R;  // keep the value live
        return;
      }
      slots[((q - round_q0) << 3) | g] = ~R;
      if (q + 1 - round_q0 == kRound) {  // wave-uniform
        flush(q + 1);
        round_q0 = q + 1;
      }
    };

    // The fold over groups [qb, qe): any mix of line counts, byte- or
    // word-granular edges (two cursors, quiet blocks).
    uint32_t fd_q = qb, fd_k = 0, fd_L, fd_a, fd_M;
    auto fd_enter = [&](uint32_t q) {
      const uint32_t v = fifo[((q & 7u) << 3) | g];
      fd_a = v & 127u;
      fd_M = v >> 7;
      fd_L = __builtin_amdgcn_readfirstlane((fd_a + fd_M + 127u) >> 7);
    };
    fd_enter(fd_q);
    // head lines of the group: 2 when some packet's header runs into line 1 (a
    // plain uint32 so the edge test below is SALU arithmetic and one branch:
    // short-circuit || on a ballot-derived bool compiled to five branches per
    // step, and C4's fold ran 1.5 % slower)
    uint32_t fd_hl = __ballot(fd_a > 88u) != 0 ? 2u : 1u;
    // edge line <=> fd_k < fd_hl or fd_k == fd_L - 1 <=> (fd_k - fd_hl) >= fd_span, unsigned
    uint32_t fd_span = fd_L - 1u > fd_hl ? fd_L - 1u - fd_hl : 0u;  // 0: every line is an edge line

    uint32_t r[4] = {0u, 0u, 0u, 0u};
    // Two copies of the fold loop: one with whole-word edges when the bucket
    // pass found every strided-chain packet word-aligned in start and length
    // (a per-group choice inside the loop made the compiler rotate the load
    // ring through copies and drain vmcnt(0) at the loop head).
    // The fold keeps xr = r ^ (the current line's word), the lookup input: the
    // XOR with the next line's word rides in the step's last 3-input XOR (as in
    // the SCK), 4 VALU per line fewer.  An edge line corrects xr by
    // w ^ masked(w) on its own step; a group's last line leaves the next
    // group's first word alone in xr (its chains start from zero).
    uint32_t xr[4] = {ring[0][0], ring[0][1], ring[0][2], ring[0][3]};
    if ((ABL & 524288) && lane == 0) a.out[wave8 + 4] = (uint32_t)__builtin_amdgcn_s_memrealtime() + (xr[0] == 0x9E3779B9u);
    // Quiet steps.  Per-step cursor control cost the fold 16 SALU and 4.5
    // branches per wave step against 1.7 and 0.1 in the SCK (rocprofv3 --pmc,
    // profiles/r03/pmc_insts.txt).  A run of steps in which neither cursor
    // changes group and the fold cursor's line is no edge line (not a head
    // line, not the group's last) needs none of it: a step is then the 16
    // lookups, the XORs and a load.  Every full step computes the length of
    // the run that follows it (quiet); a block of D steps that starts with a
    // run of >= D ahead is D quiet steps with no per-step test at all, and
    // shorter runs go through full steps (a per-step quiet / full branch
    // measured 17 % slower: 1115 against 953 us, profiles/r03/fold_var.txt).
    uint32_t quiet = 0;
    auto quiet_step = [&](int u, uint32_t ahead) {  // ahead: lines the load cursor is past ld_k within the block
      const u32x4 wn = ring[(u + 1) % D];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const uint32_t t0 = lds_at(tab, __builtin_amdgcn_perm(xr[i], lt.lo0, 0x0C0C0400u));
        const uint32_t t1 = lds_at(tab, __builtin_amdgcn_perm(xr[i], lt.lo0, 0x0C0C0500u) + 128);
        const uint32_t t2 = lds_at(tab, __builtin_amdgcn_perm(xr[i], lt.lo1, 0x0C020600u));
        const uint32_t t3 = lds_at(tab, __builtin_amdgcn_perm(xr[i], lt.lo1, 0x0C020700u) + 128);
        xr[i] = xor3(t0, t1, xor3(t2, t3, wn[i]));
      }
      ring[u] = line_load(ld.line0 + 128ull * (ld_k + ahead));
    };
    auto fold_loop = [&](auto words) {
      // One full step: edge masks, group finish and both cursors' group changes.
      auto full_step = [&](int u, bool &done) {
        const u32x4 wn = ring[(u + 1) % D];  // the next line, raw
        if (!(ABL & 8) && fd_k - fd_hl >= fd_span) {  // wave-uniform: an edge line
          const u32x4 wc = ring[u];
          const int rel0 = (int)(128u * fd_k + 16u * s) - (int)fd_a;
          if constexpr (decltype(words)::value) {
            if (fd_k < fd_hl) {  // wave-uniform: a head line
#pragma unroll
              for (int i = 0; i < 4; ++i) {
                // whole words: keep 0 <= rel < M by sign arithmetic (compare +
                // select pairs needed hazard NOPs), head masks from a 16-entry
                // table (rel >= 40 and rel < 0 index the zero entry 15)
                const int rel = rel0 + 4 * i;
                const uint32_t keep = (uint32_t)(((rel - (int)fd_M) & ~rel) >> 31);
                const uint32_t k = __builtin_elementwise_min((uint32_t)rel >> 2, 15u);
                typedef uint32_t u32x2e __attribute__((ext_vector_type(2)));
                const u32x2e e = *reinterpret_cast<const u32x2e *>(etl + 2 * k);
                xr[i] = xor3(xr[i], wc[i], ((wc[i] & keep) | e[0]) ^ e[1]);
              }
            } else {
              // the group's last line past its head lines: rel >= 40 (no head
              // masks), only the bytes at rel >= M dropped -- 3 VALU a word
              // instead of 10 and a table read
              const int lim = (int)fd_M - 1 - rel0;
#pragma unroll
              for (int i = 0; i < 4; ++i) xr[i] ^= wc[i] & (uint32_t)((lim - 4 * i) >> 31);
            }
          } else if (fd_k < fd_hl) {  // wave-uniform: a head line (byte-granular)
#pragma unroll
            for (int i = 0; i < 4; ++i) xr[i] = xor3(xr[i], wc[i], edge_word(wc[i], rel0 + 4 * i, (int)fd_M));
          } else {
            // the group's last line past its head lines, byte-granular: rel
            // >= 40 (no head masks), only the bytes at rel >= M dropped -- the
            // word keeps its low clamp(M - rel, 0, 4) bytes (5 VALU a word
            // instead of edge_word's ~20)
#pragma unroll
            for (int i = 0; i < 4; ++i) {
              const int r = (int)fd_M - (rel0 + 4 * i);
              const uint32_t c = 8u * (uint32_t)__builtin_elementwise_min(__builtin_elementwise_max(r, 0), 4);
              const uint32_t keep = (uint32_t)((1ull << c) - 1u);
              xr[i] ^= wc[i] & ~keep;
            }
          }
        }
        uint32_t t[4][4];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          if (ABL & 1) {
            t[i][0] = __builtin_amdgcn_perm(xr[i], lt.lo0, 0x0C0C0400u);
            t[i][1] = xr[i] >> 7;
            t[i][2] = 0u;
            t[i][3] = 0u;
          } else {
            t[i][0] = lds_at(tab, __builtin_amdgcn_perm(xr[i], lt.lo0, 0x0C0C0400u));
            t[i][1] = lds_at(tab, __builtin_amdgcn_perm(xr[i], lt.lo0, 0x0C0C0500u) + 128);
            t[i][2] = lds_at(tab, __builtin_amdgcn_perm(xr[i], lt.lo1, 0x0C020600u));
            t[i][3] = lds_at(tab, __builtin_amdgcn_perm(xr[i], lt.lo1, 0x0C020700u) + 128);
          }
        }
        if (++fd_k == fd_L) {  // wave-uniform: group fd_q folded
#pragma unroll
          for (int i = 0; i < 4; ++i) r[i] = xor3(t[i][0], t[i][1], t[i][2] ^ t[i][3]);
          finish_group(r, fd_L, fd_a, fd_M, fd_q);
#pragma unroll
          for (int i = 0; i < 4; ++i) xr[i] = wn[i];
          fd_k = 0;
          if (fd_q + 1 < qe) {
            ++fd_q;
            fd_enter(fd_q);
            fd_hl = __ballot(fd_a > 88u) != 0 ? 2u : 1u;
            fd_span = fd_L - 1u > fd_hl ? fd_L - 1u - fd_hl : 0u;
          } else {
            done = true;
            fd_L = 0xFFFFFFFFu;
          }
        } else {
#pragma unroll
          for (int i = 0; i < 4; ++i) xr[i] = xor3(t[i][0], t[i][1], xor3(t[i][2], t[i][3], wn[i]));
        }
        // Refill after folding: the FIFO entry the fold just read may be
        // rewritten by this step's load-cursor advance.
        ring[u] = ld_issue();
        ld_advance();
        // The quiet run that follows: fold lines fd_k .. fd_L - 2 past the head
        // lines, loads up to the line before the load cursor's group change
        // (ld_L = 1 once every group is loaded: no run).
        const uint32_t nf = (fd_k >= fd_hl && fd_k + 1 < fd_L) ? fd_L - 1u - fd_k : 0u;
        const uint32_t nl = ld_L - 1u - ld_k;
        quiet = nf < nl ? nf : nl;
      };
      bool done = false;
      while (!done) {
        if (!(ABL & 8) && quiet >= (uint32_t)D) {  // wave-uniform: D quiet steps, no per-step control
#pragma unroll
          for (int u = 0; u < D; ++u) {
            __builtin_amdgcn_sched_barrier(0);
            quiet_step(u, (uint32_t)u);
          }
          quiet -= D;
          fd_k += D;
          ld_k += D;
          continue;
        }
#pragma unroll
        for (int u = 0; u < D; ++u) {  // full steps (correct in any state; each one measures the next run)
          __builtin_amdgcn_sched_barrier(0);
          full_step(u, done);
        }
      }
    };
    if (C.odd == 0)
      fold_loop(std::true_type{});
    else
      fold_loop(std::false_type{});
    if (!(ABL & 16) && q_end != round_q0) flush(q_end);
    if ((ABL & 16) && sink == 0x12345678u) a.bres[0] = sink;
  }
  if ((ABL & 524288) && lane == 0) {  // timing only: end stamp after every store has left
    __builtin_amdgcn_s_waitcnt(0);
    a.out[wave8 + 3] = (uint32_t)__builtin_amdgcn_s_memrealtime();
    a.out[wave8 + 6] = t_tb;
    a.out[wave8 + 7] = done_work;
  }
}

// The small pool [0, ctr->small), one round of 64 packets per wave at a time
// (two rounds batched per wave, their coalesced loads all issued before the
// first fold, measured slower: 29.4 against 26.7 us on C4's mix,
// profiles/r04/s6_mb_class_rates.txt).  Batches whose gather pass folds its
// blocks' one-line packets itself (PassShape::fused) do not launch it.
__global__ __launch_bounds__(kBlock) void icrc_rsmall_kernel(RsckArgs a) {
  __shared__ uint32_t lds[kLdsWords];
  const uint32_t count = a.ctr->small;
  if (count == 0) return;  // no one-line packets (wave-uniform): no table build either
  fill_tables(lds);
  __syncthreads();
  const uint32_t lane = threadIdx.x & 63;
  const uint32_t wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const LaneTab lt{(lane & 31) << 2, ((lane & 31) << 2) | 0x10000u};
  const uint32_t step = gridDim.x * kWaves * 64u;
  const __amdgpu_buffer_rsrc_t ro = make_rsrc(a.res, 4u * count);
  auto desc_at = [&](uint32_t pos) -> RsDesc { return a.desc[pos < count ? pos : count - 1u]; };
  uint32_t base = (blockIdx.x * kWaves + wid) * 64u;
  RsDesc dn = desc_at(base + lane);
  for (; base < count; base += step) {
    const RsDesc d = dn;
    dn = desc_at(base + step + lane);  // the next round's descriptors, in flight meanwhile
    const uint32_t v = small_icrc(Step4{lds, lt}, d, lane);
    const uint32_t pos = base + lane;
    __builtin_amdgcn_raw_buffer_store_b32(v, ro, pos < count ? 4u * pos : 0x7FFFFFF0u, 0, 0);
  }
}

// =======================================================================
// The ragged path in ONE launch, workgroup-local (icrc_rswg_kernel): for
// batches of up to about kWgCap packets per workgroup (C4's 8-GPU shard:
// 524,288 packets on 256 CUs).  The three-pass pipeline above pays, at that
// size, the bucket pass (~11 us), the gather (~4.5 us), two launch
// boundaries and the fold's start-up of four dependent round trips (counters
// and block ranges, runs, descriptor blocks, lines: ~10 us), for ~130 us of
// streaming (profiles/r05/NOTES.md).  Here each workgroup takes a contiguous
// range of the batch (XCD-weighted packet counts) and, per chunk of <=
// kWgCap packets:
//   1. reads its descriptors (3 per thread), classifies them as rsck_bucket
//      does (rs_class) and ranks each in its class by an LDS atomic;
//   2. scans the class counts -- one-line classes first, then the big
//      classes by DESCENDING line count, so the groups claimed last are the
//      short ones -- and lays the descriptors out in LDS (no padding: a
//      class's last group repeats its last packet in the lanes past its
//      end); each packet's layout position goes to out[i] (scratch);
//   3. folds: the one-line packets in rounds of 64 on wave slots 0..11
//      (small_icrc, as the fold kernel), then the groups of 8 equal-L
//      packets, CLAIMED one at a time from an LDS counter -- the waves of a
//      workgroup end within a group of each other, instead of spreading by
//      wave slot as static shares do (the memory system serves a SIMD's
//      older waves first: mean end by slot 104 -> 124 us at the shard, r6s1);
//      the result of each packet overwrites its layout entry;
//   4. writes out[i] from the layout (out[i] held its position), computing
//      the packets not bucketed (n < 44: Sarwate loop; invalid: 0) there.
// The fold loop is the fold kernel's (two cursors, quiet blocks, edge masks,
// the finish through nibble tables); a group's descriptors come from the
// layout in LDS instead of global descriptor blocks, and the fold cursor
// reads (a, M) of each group from the layout too (a per-wave FIFO carries the
// group's layout range from the load cursor).
// =======================================================================
constexpr uint32_t kWgCap = kRsWgCap;                             // packets per workgroup chunk
constexpr uint32_t kWgPer = (kWgCap + kBlock - 1) / kBlock;       // ... per thread
constexpr uint32_t kWgFifo = 8;                                   // group ranges between the cursors, per wave
template <int ABL>
__global__ __launch_bounds__(kBlock) void icrc_rswg_kernel(RsckArgs a) {
  constexpr int D = 6;  // lines in flight per wave (as the fold kernel)
  constexpr uint32_t kLayW = 2 * kWgCap;          // (lo, hi) per layout entry; lo <- the ICRC once folded
  constexpr uint32_t kScrW = 2 * kRsClasses;      // class counts | class starts; then the runs
  constexpr uint32_t kFifoW = kWaves * kWgFifo * 2;
  constexpr uint32_t kMiscW = 16;
  constexpr int kHeadLo = -16, kHeadHi = 44;  // head words' offsets: rel0 clamped to [lo, hi], + 4 i
  constexpr uint32_t kHeadN = kHeadHi + 12 - kHeadLo + 1, kHeadW = 2 * kHeadN;
  __shared__ uint32_t lds[kFinFold + kLdsWords + kTzWords + kLayW + kScrW + kFifoW + kMiscW + kHeadW];
  uint32_t *xtl = lds;
  uint32_t *qtl = lds + 128;
  uint32_t *etl = lds + 128 + 8 * kFinQtStride;  // whole-word head masks: (or, xor) of word k = rel / 4
  uint32_t *x2tl = etl + 32, *x3tl = etl + 160;  // nibble tables of x^-64, x^-96
  uint32_t *tab = lds + kFinFold;
  uint32_t *tzl = tab + kLdsWords;
  uint32_t *lay = tzl + kTzWords;
  uint32_t *hcnt = lay + kLayW, *cstart = hcnt + kRsClasses;
  uint32_t *runs = hcnt;  // after the placement: run r = (g0 | L << 16, e0 | cnt << 16)
  uint32_t *fifo_all = hcnt + kScrW;
  uint32_t *misc = fifo_all + kFifoW;  // 0 groups, 1 one-line packets, 2 claim counter, 3.. scan totals
  uint32_t *htl = misc + kMiscW;       // byte-granular head words: (drop, set) by offset (head_masks)
  static_assert(sizeof(lds) <= 160 * 1024, "LDS");
  static_assert(kWgCap < 65536 && kRsClasses <= kBlock, "16-bit layout fields, one class per thread");

  const uint32_t lane = threadIdx.x & 63;
  const uint32_t wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const uint32_t s = lane & 7, g = lane >> 3;
  // ABL 524288 (timing only, tools/microbench/wg.hip): per-wave s_memrealtime
  // stamps into a.pos_of, 8 words per wave: entry, layout done, one-line
  // rounds done, fold done, end, descriptors in, ranks counted (the first
  // chunk's), the XCD
  uint32_t st_w[8] = {};
  auto stamp = [&](int k) {
    if (ABL & 524288) st_w[k] = (uint32_t)__builtin_amdgcn_s_memrealtime();
  };
  stamp(0);
  if (ABL & 524288) st_w[7] = (uint32_t)__builtin_amdgcn_s_getreg((3 << 11) | 20);  // HW_REG_XCC_ID
  xcd_record(a.xcd_rec);
  // This workgroup's packets: the union of its waves' XCD-weighted shares.
  uint64_t w_lo, w_hi;
  {
    uint64_t l0, h0, l1, h1;
    if (a.xw[0] != 0u) {
      xcd_share(a.count, a.xw, a.xcd_k, 0, l0, h0);
      xcd_share(a.count, a.xw, a.xcd_k, kWaves - 1, l1, h1);
    } else {
      const uint64_t per = (a.count + gridDim.x - 1) / gridDim.x;
      l0 = (uint64_t)blockIdx.x * per < a.count ? (uint64_t)blockIdx.x * per : a.count;
      h1 = l0 + per < a.count ? l0 + per : a.count;
    }
    w_lo = l0;
    w_hi = h1;
  }
  // The first chunk's descriptor lines, one load a 128-byte line, requested
  // before the tables: their HBM round trip runs beside the tables' and the
  // chunk's own descriptor loads find them in L2.
  uint32_t pf = 0;
  if (w_lo < w_hi) {
    const uint64_t P0 = w_hi - w_lo < kWgCap ? w_hi - w_lo : kWgCap;
    const uint32_t t = threadIdx.x;
    const uint32_t no = a.off ? (uint32_t)((8u * P0 + 127u) >> 7) + 1u : 0u;
    const uint32_t nl = a.len ? (uint32_t)((4u * P0 + 127u) >> 7) + 1u : 0u;
    if (t < no)
      pf = (uint32_t)a.off[w_lo + (16ull * t < P0 ? 16ull * t : P0 - 1u)];
    else if (t < no + nl)
      pf = a.len[w_lo + (32ull * (t - no) < P0 ? 32ull * (t - no) : P0 - 1u)];
  }
  const TableRegs tab_v = table_load(g_tab128);
  const uint32_t fin0 = a.fin[threadIdx.x], fin1 = a.fin[threadIdx.x + 1024u < kFinFold ? threadIdx.x + 1024u : 0u];
  const uint32_t tz_v = a.tzb[threadIdx.x < kTzWords ? threadIdx.x : 0];
  table_write(tab, tab_v);
  if (threadIdx.x < kTzWords) tzl[threadIdx.x] = tz_v;
  lds[threadIdx.x] = fin0;  // the finish tables, built by the host (icrc_math.h build_fin_tables)
  if (threadIdx.x + 1024u < kFinFold) lds[threadIdx.x + 1024u] = fin1;
  if (threadIdx.x < kHeadN) {
    const auto hm = head_masks((int)threadIdx.x + kHeadLo);
    htl[2u * threadIdx.x] = hm[0];
    htl[2u * threadIdx.x + 1u] = hm[1];
  }
  asm volatile("" ::"v"(pf));  // (the prefetch lands here, not in the chunk loop)

  const LaneTab lt{(lane & 31) << 2, ((lane & 31) << 2) | 0x10000u};
  const uint32_t *qrow = qtl + s * kFinQtStride;
  uint32_t *fifo = fifo_all + wid * (kWgFifo * 2);
  typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
  auto lay_at = [&](uint32_t e) -> u32x2 { return *reinterpret_cast<const u32x2 *>(lay + 2u * e); };

  for (uint64_t c0 = w_lo; c0 < w_hi; c0 += kWgCap) {  // workgroup-uniform: chunks of <= kWgCap packets
    const uint32_t P = (uint32_t)(w_hi - c0 < kWgCap ? w_hi - c0 : kWgCap);
    for (uint32_t t = threadIdx.x; t < kRsClasses; t += kBlock) hcnt[t] = 0;
    if (threadIdx.x < kMiscW) misc[threadIdx.x] = 0;
    __syncthreads();  // (the first chunk: the tables are written too)

    // 1. descriptors, classes, ranks (loads first, index clamped: issued back to back)
    uint64_t addr[kWgPer];
    uint32_t n[kWgPer], cr[kWgPer];
#pragma unroll
    for (int k = 0; k < (int)kWgPer; ++k) {
      const uint32_t j = (uint32_t)k * kBlock + threadIdx.x;
      const uint64_t i = c0 + (j < P ? j : P - 1u);
      addr[k] = a.off ? a.off[i] : i * a.stride;
      n[k] = a.len ? a.len[i] : a.fixed_len;
    }
    int odd = 0;
    if (ABL & 524288) {  // (timing: the descriptors' arrival)
      __builtin_amdgcn_s_waitcnt(0);
      if (c0 == w_lo) stamp(5);
    }
#pragma unroll
    for (int k = 0; k < (int)kWgPer; ++k) {
      const uint32_t j = (uint32_t)k * kBlock + threadIdx.x;
      addr[k] += (uint64_t)(uintptr_t)a.base + a.l3_offset;
      const uint32_t c = j < P ? rs_class(addr[k], n[k]) : 0u;
      const uint32_t rk = c ? atomicAdd(&hcnt[c], 1u) : 0u;
      odd |= (c > (uint32_t)kRsBigBase && ((addr[k] | n[k]) & 3u)) ? 1 : 0;
      cr[k] = c | (rk << 10);
    }
    const bool words = __syncthreads_or(odd) == 0;  // (a barrier: the counts are complete)
    if (c0 == w_lo) stamp(6);

    // 2. scan by key: one-line classes 1..kRsBigBase (keys 0..7), then the big
    //    classes by descending L (key 8 + j: class kRsClasses - 1 - j)
    const uint32_t t = threadIdx.x, wv = t >> 6;
    const bool key = t < (uint32_t)kRsClasses - 1u;
    const uint32_t c = !key ? 0u : t < (uint32_t)kRsBigBase ? t + 1u : (uint32_t)kRsClasses - 1u - (t - kRsBigBase);
    const bool big = c > (uint32_t)kRsBigBase;
    const uint32_t cnt = key ? hcnt[c] : 0u;
    const uint32_t G = big ? (cnt + 7u) >> 3 : 0u;
    const uint32_t f = (big && cnt) ? 1u : 0u;
    const uint32_t Sm = big ? 0u : cnt;
    uint32_t ie = wave_scan(cnt), ig = wave_scan(G), ir = wave_scan(f), is = wave_scan(Sm);
    uint32_t *wt = fifo_all;  // per-wave totals (the FIFOs are not in use yet)
    if (lane == 63) {
      wt[4 * wv] = ie;
      wt[4 * wv + 1] = ig;
      wt[4 * wv + 2] = ir;
      wt[4 * wv + 3] = is;
    }
    __syncthreads();
    for (uint32_t w = 0; w < wv; ++w) {  // wave-uniform
      ie += wt[4 * w];
      ig += wt[4 * w + 1];
      ir += wt[4 * w + 2];
      is += wt[4 * w + 3];
    }
    const uint32_t e0 = ie - cnt, g0 = ig - G, r0 = ir - f;  // exclusive prefixes
    if (key) cstart[c] = e0;
    if (t == kBlock - 1) {
      misc[0] = ig;  // groups
      misc[1] = is;  // one-line packets: layout entries [0, is)
    }
    __syncthreads();
    // placement; out[i] <- the packet's layout position (or ~0: not bucketed)
#pragma unroll
    for (int k = 0; k < (int)kWgPer; ++k) {
      const uint32_t j = (uint32_t)k * kBlock + threadIdx.x;
      if (j >= P) continue;
      const uint32_t ck = cr[k] & 1023u;
      uint32_t pos = 0xFFFFFFFFu;
      if (ck) {
        pos = cstart[ck] + (cr[k] >> 10);
        *reinterpret_cast<u32x2 *>(lay + 2u * pos) =
            u32x2{(uint32_t)addr[k], (uint32_t)(addr[k] >> 32) | (n[k] << 16)};
      }
      __builtin_nontemporal_store(pos, a.out + c0 + j);
    }
    __syncthreads();
    if (f) {  // the runs, in key order (g0 ascending)
      runs[2u * r0] = g0 | ((c - (uint32_t)kRsBigBase) << 16);
      runs[2u * r0 + 1u] = e0 | (cnt << 16);
    }
    __syncthreads();
    const uint32_t NG = misc[0], NS = misc[1];
    if (c0 == w_lo) stamp(1);

    // 3a. the one-line packets: rounds of 64 dealt evenly to wave slots 0..11
    {
      const uint32_t NC = (NS + 63u) >> 6;
      const uint32_t sl = kRsSmallSlots;
      const uint32_t cb = wid < sl ? wid * NC / sl : 0u, ce = wid < sl ? (wid + 1u) * NC / sl : 0u;
      const StepNib step{lds + kFinStep4};
#pragma unroll 1
      for (uint32_t cc = cb; cc < ce; ++cc) {  // wave-uniform
        const uint32_t jj = 64u * cc + lane;
        const u32x2 dv = lay_at(jj < NS ? jj : NS - 1u);
        const uint32_t v = small_icrc(step, RsDesc{dv[0], dv[1]}, lane);
        if (jj < NS) lay[2u * jj] = v;
      }
    }

    if (c0 == w_lo) stamp(2);
    // 3b. the groups, claimed one at a time
    auto claim = [&]() -> uint32_t {
      uint32_t v = 0;
      if (lane == 0) v = atomicAdd(&misc[2], 1u);
      return v;  // (readfirstlane when used: the atomic's return lands meanwhile)
    };
    uint32_t run_i = 0;  // the run of the load cursor's group (runs in g0 order, groups claimed ascending)
    uint32_t run_g0 = 0, run_L = 0, run_e0 = 0, run_cnt = 0, run_g1 = 0;
    auto run_load = [&](uint32_t r) {
      const u32x2 rv = *reinterpret_cast<const u32x2 *>(runs + 2u * r);
      run_g0 = __builtin_amdgcn_readfirstlane(rv[0] & 0xFFFFu);
      run_L = __builtin_amdgcn_readfirstlane(rv[0] >> 16);
      run_e0 = __builtin_amdgcn_readfirstlane(rv[1] & 0xFFFFu);
      run_cnt = __builtin_amdgcn_readfirstlane(rv[1] >> 16);
      run_g1 = run_g0 + ((run_cnt + 7u) >> 3);
    };
    if (NG != 0u) run_load(0);
    uint32_t q_pend = claim();  // (lane 0's claim in flight)
    const uint32_t q_first = __builtin_amdgcn_readfirstlane(q_pend);
    if (q_first < NG) {  // wave-uniform
      uint32_t q_next = q_first;
      q_pend = claim();
      uint32_t ld_seq = 0;  // groups the load cursor entered - 1
      struct LInfo {
        uint64_t line0;
      } ld;
      // Load cursor enters claimed group q: its layout range, line base and L;
      // the range goes into the FIFO slot of its sequence number.
      auto ld_enter = [&](uint32_t q, uint32_t seq) -> uint32_t {
        while (q >= run_g1) run_load(++run_i);  // wave-uniform (claims ascend)
        const uint32_t eb = run_e0 + 8u * (q - run_g0), el = run_e0 + run_cnt - 1u;
        const uint32_t e = eb + g < el ? eb + g : el;
        const u32x2 dv = lay_at(e);
        const uint64_t ad = ((uint64_t)(dv[1] & 0xFFFFu) << 32) | dv[0];
        ld.line0 = (ad & ~127ull) + 16u * s;
        if (lane == 0) *reinterpret_cast<u32x2 *>(fifo + 2u * (seq & (kWgFifo - 1u))) = u32x2{eb, el};
        return run_L;
      };
      auto line_load = [&](uint64_t ad) -> u32x4 {
        if (ABL & 16384) return u32x4{(uint32_t)ad, (uint32_t)(ad >> 7), lane, (uint32_t)ad * 3u};
        return gload16_nt(ad);
      };
      uint32_t ld_k = 0, ld_L = ld_enter(q_next, 0);
      bool ld_more = true;  // a claimed group follows the load cursor's current one
      auto ld_issue = [&]() -> u32x4 { return line_load(ld.line0 + 128ull * ld_k); };
      auto ld_advance = [&]() {
        if (++ld_k == ld_L) {  // wave-uniform
          ld_k = 0;
          if (ld_more) {
            const uint32_t qn = __builtin_amdgcn_readfirstlane(q_pend);
            if (qn < NG) {
              q_pend = claim();
              ++ld_seq;
              ld_L = ld_enter(qn, ld_seq);
              return;
            }
            ld_more = false;
          }
          ld_L = 1;  // done: re-read line 0 of the last group (ld_k wraps to 0 every step)
        }
      };
      u32x4 ring[D];
#pragma unroll
      for (int u = 0; u < D; ++u) {
        __builtin_amdgcn_sched_barrier(0);
        ring[u] = ld_issue();
        ld_advance();
      }
      __builtin_amdgcn_sched_barrier(0);

      // A group's finish (the fold kernel's): chains rr after its last line,
      // L lines, first-byte offsets ga and covered lengths gM per lane group,
      // its layout entry e -> ~ICRC into lay[2 e].
      auto finish_group = [&](uint32_t (&rr)[4], uint32_t Lg, uint32_t ga, uint32_t gM, uint32_t e) {
        uint32_t R;
        if (ABL & 2) {
          R = group_xor(rr[0] ^ rr[1] ^ rr[2] ^ rr[3], 3);
        } else {
          // v * (table's constant) ^ x: nibble w's entry at byte 64 w + 4 n_w of
          // the tables; the 4 n_w sit in the bytes of two masked shifts of v, one
          // byte extract (or SDWA add to a lane's base) per lookup
          auto nib_mul = [](const uint32_t *tb, uint32_t v, uint32_t x) -> uint32_t {
            uint32_t lo4 = (v << 2) & 0x3C3C3C3Cu, hi4 = (v >> 2) & 0x3C3C3C3Cu;
            asm volatile("" : "+v"(lo4), "+v"(hi4));  // (else folded back into a shift and mask per nibble)
            const char *tc = reinterpret_cast<const char *>(tb);
            uint32_t ev[8];
#pragma unroll
            for (int k = 0; k < 4; ++k) {
              ev[2 * k] = *reinterpret_cast<const uint32_t *>(tc + 128 * k + ((lo4 >> (8 * k)) & 0xFFu));
              ev[2 * k + 1] = *reinterpret_cast<const uint32_t *>(tc + 128 * k + 64 + ((hi4 >> (8 * k)) & 0xFFu));
            }
            return xor3(xor3(ev[0], ev[1], ev[2]), xor3(ev[3], ev[4], ev[5]), xor3(ev[6], ev[7], x));
          };
          const uint32_t u = nib_mul(x3tl, rr[3], nib_mul(x2tl, rr[2], nib_mul(xtl, rr[1], rr[0])));
          R = group_xor(nib_mul(qrow, u, 0u), 3);
          const uint32_t tz = 128u * Lg - ga - gM;
          uint32_t bw = tzl[2u * tz + s], p = 0;
#pragma unroll
          for (int tt = 0; tt < 4; ++tt) {
            const uint32_t m = (uint32_t)__builtin_amdgcn_sbfe((int)R, (int)(4u * s + tt), 1);
            p = and_xor(m, bw, p);
            bw = and_xor((uint32_t)((int32_t)bw >> 31), kXInv, bw << 1);
          }
          R = group_xor(p, 3);
        }
        if (ABL & 16) return;
        if (s == 0) lay[2u * e] = ~R;  // (the group's entries are dead: both cursors are past it)
      };

      uint32_t fd_seq = 0, fd_k = 0, fd_L, fd_a, fd_M, fd_e;
      auto fd_enter = [&](uint32_t seq) {
        const u32x2 rg = *reinterpret_cast<const u32x2 *>(fifo + 2u * (seq & (kWgFifo - 1u)));
        const uint32_t eb = __builtin_amdgcn_readfirstlane(rg[0]), el = __builtin_amdgcn_readfirstlane(rg[1]);
        fd_e = eb + g < el ? eb + g : el;
        const u32x2 dv = lay_at(fd_e);
        fd_a = dv[0] & 127u;
        fd_M = (dv[1] >> 16) - 4u;
        fd_L = __builtin_amdgcn_readfirstlane((fd_a + fd_M + 127u) >> 7);
      };
      fd_enter(0);
      uint32_t fd_hl = __ballot(fd_a > 88u) != 0 ? 2u : 1u;
      uint32_t fd_span = fd_L - 1u > fd_hl ? fd_L - 1u - fd_hl : 0u;
      uint32_t r[4] = {0u, 0u, 0u, 0u};
      uint32_t xr[4] = {ring[0][0], ring[0][1], ring[0][2], ring[0][3]};
      uint32_t quiet = 0;
      auto quiet_step = [&](int u, uint32_t ahead) {
        const u32x4 wn = ring[(u + 1) % D];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const uint32_t t0 = lds_at(tab, __builtin_amdgcn_perm(xr[i], lt.lo0, 0x0C0C0400u));
          const uint32_t t1 = lds_at(tab, __builtin_amdgcn_perm(xr[i], lt.lo0, 0x0C0C0500u) + 128);
          const uint32_t t2 = lds_at(tab, __builtin_amdgcn_perm(xr[i], lt.lo1, 0x0C020600u));
          const uint32_t t3 = lds_at(tab, __builtin_amdgcn_perm(xr[i], lt.lo1, 0x0C020700u) + 128);
          xr[i] = xor3(t0, t1, xor3(t2, t3, wn[i]));
        }
        ring[u] = line_load(ld.line0 + 128ull * (ld_k + ahead));
      };
      auto fold_loop = [&](auto wordsv) {
        auto full_step = [&](int u, bool &done) {
          const u32x4 wn = ring[(u + 1) % D];
          if (!(ABL & 8) && fd_k - fd_hl >= fd_span) {  // wave-uniform: an edge line
            const u32x4 wc = ring[u];
            const int rel0 = (int)(128u * fd_k + 16u * s) - (int)fd_a;
            if constexpr (decltype(wordsv)::value) {
              if (fd_k < fd_hl) {  // wave-uniform: a head line
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                  const int rel = rel0 + 4 * i;
                  const uint32_t keep = (uint32_t)(((rel - (int)fd_M) & ~rel) >> 31);
                  const uint32_t k = __builtin_elementwise_min((uint32_t)rel >> 2, 15u);
                  const u32x2 ev = *reinterpret_cast<const u32x2 *>(etl + 2 * k);
                  xr[i] = xor3(xr[i], wc[i], ((wc[i] & keep) | ev[0]) ^ ev[1]);
                }
              } else {
                const int lim = (int)fd_M - 1 - rel0;
#pragma unroll
                for (int i = 0; i < 4; ++i) xr[i] ^= wc[i] & (uint32_t)((lim - 4 * i) >> 31);
              }
            } else {
              if (fd_k < fd_hl) {  // wave-uniform: a head line (byte-granular): the word -> (word & ~drop) ^ set
                const int rc = __builtin_elementwise_min(__builtin_elementwise_max(rel0, kHeadLo), kHeadHi);
                const uint32_t *h = htl + 2 * (rc - kHeadLo);
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                  const u32x2 dm = *reinterpret_cast<const u32x2 *>(h + 8 * i);
                  xr[i] ^= (wc[i] & dm[0]) ^ dm[1];
                }
              }
              if (fd_k >= fd_hl || fd_k + 1u == fd_L) {  // wave-uniform: the last line: bytes past M dropped
                // (past M >= 40 the head masks are identity, so the two apply in turn);
                // word i keeps its low clamp(M - rel0 - 4 i, 0, 4) bytes
                const int rb8 = 8 * ((int)fd_M - rel0);
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                  int t8 = rb8 - 32 * i;
                  asm volatile("" : "+v"(t8));  // (one med3, not max/sub/min)
                  const uint32_t cb = (uint32_t)__builtin_elementwise_min(__builtin_elementwise_max(t8, 0), 32);
                  xr[i] ^= wc[i] & (uint32_t)(~0ull << cb);
                }
              }
            }
          }
          uint32_t tl[4][4];
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            tl[i][0] = lds_at(tab, __builtin_amdgcn_perm(xr[i], lt.lo0, 0x0C0C0400u));
            tl[i][1] = lds_at(tab, __builtin_amdgcn_perm(xr[i], lt.lo0, 0x0C0C0500u) + 128);
            tl[i][2] = lds_at(tab, __builtin_amdgcn_perm(xr[i], lt.lo1, 0x0C020600u));
            tl[i][3] = lds_at(tab, __builtin_amdgcn_perm(xr[i], lt.lo1, 0x0C020700u) + 128);
          }
          if (++fd_k == fd_L) {  // wave-uniform: the group is folded
#pragma unroll
            for (int i = 0; i < 4; ++i) r[i] = xor3(tl[i][0], tl[i][1], tl[i][2] ^ tl[i][3]);
            finish_group(r, fd_L, fd_a, fd_M, fd_e);
#pragma unroll
            for (int i = 0; i < 4; ++i) xr[i] = wn[i];
            fd_k = 0;
            if (fd_seq < ld_seq) {  // wave-uniform: the load cursor entered a next group
              ++fd_seq;
              fd_enter(fd_seq);
              fd_hl = __ballot(fd_a > 88u) != 0 ? 2u : 1u;
              fd_span = fd_L - 1u > fd_hl ? fd_L - 1u - fd_hl : 0u;
            } else {
              done = true;
              fd_L = 0xFFFFFFFFu;
            }
          } else {
#pragma unroll
            for (int i = 0; i < 4; ++i) xr[i] = xor3(tl[i][0], tl[i][1], xor3(tl[i][2], tl[i][3], wn[i]));
          }
          ring[u] = ld_issue();
          ld_advance();
          const uint32_t nf = (fd_k >= fd_hl && fd_k + 1 < fd_L) ? fd_L - 1u - fd_k : 0u;
          const uint32_t nl = ld_L - 1u - ld_k;
          quiet = nf < nl ? nf : nl;
        };
        bool done = false;
        while (!done) {
          if (!(ABL & 8)) {
            while (quiet >= (uint32_t)D) {  // wave-uniform: D quiet steps, no per-step control
#pragma unroll
              for (int u = 0; u < D; ++u) {
                __builtin_amdgcn_sched_barrier(0);
                quiet_step(u, (uint32_t)u);
              }
              quiet -= D;
              fd_k += D;
              ld_k += D;
            }
          }
#pragma unroll
          for (int u = 0; u < D; ++u) {
            __builtin_amdgcn_sched_barrier(0);
            full_step(u, done);
          }
        }
      };
      if (words)
        fold_loop(std::true_type{});
      else
        fold_loop(std::false_type{});
    }
    stamp(3);
    // 4. out[i] from the layout (out[i] held the packet's position)
    uint32_t pv[kWgPer];
#pragma unroll
    for (int k = 0; k < (int)kWgPer; ++k) {
      const uint32_t j = (uint32_t)k * kBlock + threadIdx.x;
      pv[k] = j < P ? __builtin_nontemporal_load(a.out + c0 + j) : 0xFFFFFFFFu;
    }
    __syncthreads();  // every group folded
#pragma unroll
    for (int k = 0; k < (int)kWgPer; ++k) {
      const uint32_t j = (uint32_t)k * kBlock + threadIdx.x;
      if (j >= P) continue;
      const uint32_t v = pv[k] != 0xFFFFFFFFu ? lay[2u * pv[k]] : 0u;
      __builtin_nontemporal_store(gather_one(a, c0 + j, pv[k], v), a.out + c0 + j);
    }
    __syncthreads();  // the layout is read: the next chunk may overwrite it
  }
  if ((ABL & 524288) && lane == 0) {
    __builtin_amdgcn_s_waitcnt(0);
    stamp(4);
    const uint64_t w8 = 8ull * ((uint64_t)blockIdx.x * kWaves + wid);
#pragma unroll
    for (int k = 0; k < 8; ++k) a.pos_of[w8 + k] = st_w[k];
  }
}

// Gather: block b serves pass block b's packets.  A staged block's results
// sit in two contiguous ranges (its small range, its big range): they are
// read coalesced into LDS in the block's layout order and pos_of indexes
// that copy, instead of one 4-byte read per packet scattered over the class
// runs of the pools.  SMALL (PassShape::fused): the block's one-line packets
// (its small range, descriptors at desc[small0, small0 + small)) are folded
// here, one lane per packet, instead of by icrc_rsmall_kernel: at C4's
// 8-GPU shard that kernel took 11.4 us (its launch, its table build, one
// round of loads) for 131 K packets, profiles/r05/s1_prof_c4s.txt.  With a
// grid of 2 x nblk (PassShape::split: the pass ran on at most half the CUs)
// the one-line packets of pass block b are folded by block nblk + b, the
// "small side", on the CUs the pass left idle: it inverts the block's
// positions in LDS and writes those packets' out[i] itself, while block b
// gathers the others -- no result crosses between the two, so neither waits.
__device__ __forceinline__ void pass_range_of(uint64_t count, uint32_t nblk, uint32_t b, uint32_t &lo,
                                              uint32_t &hi) {
  const uint64_t per = ((count + nblk - 1) / nblk + kPassBlock - 1) / kPassBlock * kPassBlock;
  const uint64_t l = (uint64_t)b * per < count ? (uint64_t)b * per : count;
  lo = (uint32_t)l;
  hi = (uint32_t)(l + per < count ? l + per : count);
}

template <int PU, bool SMALL, bool SPLIT = false>  // the bucket pass's packets per thread
__global__ __launch_bounds__(kPassBlock) void rsck_gather(RsckArgs a) {
  static_assert(SMALL || !SPLIT, "small sides fold one-line packets");
  constexpr uint32_t kStage = stage_entries(PU);
  __shared__ uint32_t lres[kStage];
  __shared__ uint32_t tab[SMALL ? kLdsWords : 1];
  constexpr bool split = SPLIT;  // a grid of 2 x nblk
  const bool small_side = split && blockIdx.x >= a.nblk;
  const uint32_t pb = small_side ? blockIdx.x - a.nblk : blockIdx.x;
  TableRegs tab_v{};
  if (SMALL) tab_v = table_load(g_tab);
  // The counters are dead now (the bucket pass and both folds have read
  // them): zero them for the next call on this workspace.
  if (blockIdx.x == 0 && threadIdx.x == 0) *a.ctr = RsCounters{};
  uint32_t lo, hi;
  pass_range_of(a.count, a.nblk, pb, lo, hi);
  const RsBlock B = a.blk[pb];
  const uint32_t lane = threadIdx.x & 63;
  const LaneTab lt{(lane & 31) << 2, ((lane & 31) << 2) | 0x10000u};
  // SMALL: the first of this thread's one-line descriptors (every lane of a
  // wave with a valid one: the fold is wave-collective), requested with the
  // other loads; C4's shard blocks hold ~1 K one-line packets, one per thread
  auto small_desc = [&](uint32_t j) { return a.desc[B.small0 + (j < B.small ? j : B.small - 1u)]; };
  auto small_fold = [&](const RsDesc &sd0, auto store) {  // fold the block's small range, store(j, icrc)
    table_write(tab, tab_v);
    __syncthreads();
#pragma unroll 1
    for (uint32_t j0 = 0; j0 < B.small; j0 += blockDim.x) {
      const uint32_t j = j0 + threadIdx.x;
      if (j0 + (threadIdx.x & ~63u) < B.small) {  // wave-uniform
        const uint32_t v = small_icrc(Step4{tab, lt}, j0 ? small_desc(j) : sd0, lane);
        if (j < B.small) store(j, v);
      }
    }
  };
  constexpr int U = 4;  // packets per thread in flight at once
  if (small_side) {  // block-uniform
    if (!B.staged || B.small == 0) return;  // (an unstaged block's gather side folds them)
    uint32_t p[PU];
#pragma unroll
    for (int k = 0; k < PU; ++k) {
      const uint32_t i = lo + (uint32_t)k * blockDim.x + threadIdx.x;
      p[k] = i < hi ? __builtin_nontemporal_load(a.pos_of + i) : 0xFFFFFFFFu;
    }
    const RsDesc sd0 = small_desc(threadIdx.x);
    uint32_t *idx = lres;  // small position j -> packet index i
#pragma unroll
    for (int k = 0; k < PU; ++k)
      if (p[k] < B.small) idx[p[k]] = lo + (uint32_t)k * blockDim.x + threadIdx.x;
    small_fold(sd0, [&](uint32_t j, uint32_t x) {
      const uint32_t i = idx[j];
      __builtin_nontemporal_store(gather_one(a, i, j, x), a.out + i);
    });
    return;
  }
  RsDesc sd0{0u, 0u};
  if (SMALL && !split && B.small) sd0 = small_desc(threadIdx.x);
  if (B.staged) {  // block-uniform (a staged block's packets fit one round: hi - lo <= PU x blockDim)
    // every load of the block issued before the barrier: the positions, then
    // the results into LDS
    uint32_t p[PU];
#pragma unroll
    for (int k = 0; k < PU; ++k) {
      const uint32_t i = lo + (uint32_t)k * blockDim.x + threadIdx.x;
      p[k] = i < hi ? __builtin_nontemporal_load(a.pos_of + i) : 0xFFFFFFFFu;
    }
    const uint32_t total = B.small + 8u * B.groups;
    const uint32_t *rs = a.res + B.small0, *rb = a.bres + 8ull * B.g0 - B.small;
    const uint32_t from = SMALL ? B.small : 0u;  // SMALL: the small range is folded here or by the small side
    constexpr int R = (kStage + kPassBlock - 1) / kPassBlock;
    uint32_t v[R];
#pragma unroll
    for (int k = 0; k < R; ++k) {
      const uint32_t j = (uint32_t)k * blockDim.x + threadIdx.x;
      v[k] = j >= from && j < total ? __builtin_nontemporal_load((j < B.small ? rs : rb) + j) : 0u;
    }
#pragma unroll
    for (int k = 0; k < R; ++k) {
      const uint32_t j = (uint32_t)k * blockDim.x + threadIdx.x;
      if (j >= from && j < total) lres[j] = v[k];
    }
    if (SMALL && !split && B.small) small_fold(sd0, [&](uint32_t j, uint32_t x) { lres[j] = x; });
    __syncthreads();
#pragma unroll
    for (int k = 0; k < PU; ++k) {
      const uint32_t i = lo + (uint32_t)k * blockDim.x + threadIdx.x;
      if (i < hi && !(split && p[k] < B.small))  // split: the small side wrote those
        __builtin_nontemporal_store(gather_one(a, i, p[k], p[k] != 0xFFFFFFFFu ? lres[p[k]] : 0u), a.out + i);
    }
    return;
  }
  // not staged: the small results go to the pool first (a workgroup-scope
  // barrier orders those stores before the reads below)
  if (SMALL && B.small) {
    small_fold(small_desc(threadIdx.x), [&](uint32_t j, uint32_t x) { a.res[B.small0 + j] = x; });
    __syncthreads();
  }
  for (uint32_t i0 = lo + threadIdx.x; i0 < hi; i0 += U * blockDim.x) {
    uint32_t p[U], v[U];
#pragma unroll
    for (int k = 0; k < U; ++k) p[k] = i0 + k * blockDim.x < hi ? a.pos_of[i0 + k * blockDim.x] : 0xFFFFFFFFu;
#pragma unroll
    for (int k = 0; k < U; ++k) v[k] = p[k] != 0xFFFFFFFFu ? a.res[p[k]] : 0u;
#pragma unroll
    for (int k = 0; k < U; ++k) {
      const uint32_t i = i0 + k * blockDim.x;
      if (i >= hi) break;
      a.out[i] = gather_one(a, i, p[k], v[k]);
    }
  }
}

// Positions: the small pool [0, small_cap), the big pool after it; the big
// pool holds every big packet plus at most 7 padding copies per run (a run
// needs a packet: at most min(count, kRsRuns x pass blocks) runs).
static uint64_t rs_small_cap(uint64_t count) { return (count + 7) & ~7ull; }
static uint64_t rs_npos(uint64_t count) {
  const uint64_t runs = count < (uint64_t)kRsRuns * kPassBlocks ? count : (uint64_t)kRsRuns * kPassBlocks;
  return rs_small_cap(count) + ((count + 7 * runs + 7) & ~7ull);
}

uint64_t rs_workspace_bytes(uint64_t count) {
  const uint64_t npos = rs_npos(count);
  auto al = [](uint64_t b) { return (b + 255) & ~255ull; };
  return al(sizeof(RsCounters)) + al(sizeof(RsBlock) * kPassBlocks) + al(sizeof(RsRun) * kRsRuns * kPassBlocks) +
         al(sizeof(RsDesc) * npos) + al(4 * count) + al(4 * npos);
}

hipError_t rs_zero_counters(void *ws, hipStream_t st) {  // the counters are the workspace's first region
  return hipMemsetAsync(ws, 0, sizeof(RsCounters), st);
}

void rs_bind_workspace(RsckArgs &a, void *ws) {
  const uint64_t npos = rs_npos(a.count);
  auto al = [](uint64_t b) { return (b + 255) & ~255ull; };
  char *p = static_cast<char *>(ws);
  a.ctr = reinterpret_cast<RsCounters *>(p), p += al(sizeof(RsCounters));
  a.blk = reinterpret_cast<RsBlock *>(p), p += al(sizeof(RsBlock) * kPassBlocks);
  a.runs = reinterpret_cast<RsRun *>(p), p += al(sizeof(RsRun) * kRsRuns * kPassBlocks);
  a.desc = reinterpret_cast<RsDesc *>(p), p += al(sizeof(RsDesc) * npos);
  a.pos_of = reinterpret_cast<uint32_t *>(p), p += al(4 * a.count);
  a.res = reinterpret_cast<uint32_t *>(p);
  a.small_cap = (uint32_t)rs_small_cap(a.count);
  a.bdesc = a.desc + a.small_cap;
  a.bres = a.res + a.small_cap;
}

template <int U>
static void launch_bucket_u(const RsckArgs &a, int pgrid, hipStream_t st) {
  static_assert(kPassBlock == 1024 && kRsClasses <= kPassBlock, "one class per thread in the bucket pass's scan");
  if (a.off && a.len) hipLaunchKernelGGL((rsck_bucket<true, true, 0, U>), dim3(pgrid), dim3(kPassBlock), 0, st, a);
  else if (a.off) hipLaunchKernelGGL((rsck_bucket<true, false, 0, U>), dim3(pgrid), dim3(kPassBlock), 0, st, a);
  else if (a.len) hipLaunchKernelGGL((rsck_bucket<false, true, 0, U>), dim3(pgrid), dim3(kPassBlock), 0, st, a);
  else hipLaunchKernelGGL((rsck_bucket<false, false, 0, U>), dim3(pgrid), dim3(kPassBlock), 0, st, a);
}
// The bucket and gather passes' shape for a batch: packets per thread U (the
// smallest of 4, 8, 16, 17 whose round covers the batch on 256 blocks) and
// pass blocks (as many as one round of U per thread needs).  A latency-bound
// pass: at C4's 8-GPU shard (524 K packets) the round-4 shape, U = 16 on 256
// blocks (2 live packets per thread, 14 clamped loads), took 16.3 us; U = 4
// on 128 blocks 10.2, U = 2 on 256 blocks 12.4, U = 8 on 64 blocks 11.4
// (tools/microbench/shard.hip, profiles/r05/s1_mb_shard_baseline.txt).
struct PassShape {
  int grid, U;
  bool fused;  // the gather folds the one-line packets (U = 4, one staged round per block): no icrc_rsmall_kernel
  bool split;  // fused on at most half the pass blocks: the gather runs on 2 x grid, small sides beside it
};
static PassShape pass_shape(uint64_t count, int pass_cap, bool no_split = false) {
  int U = kPassUnrollBig;
  for (int u : {4, 8, kPassUnroll})
    if (count <= (uint64_t)kPassBlocks * kPassBlock * u) {
      U = u;
      break;
    }
  const uint64_t want = (count + (uint64_t)U * kPassBlock - 1) / ((uint64_t)U * kPassBlock);
  int grid = (int)(want < (uint64_t)kPassBlocks ? (want ? want : 1) : kPassBlocks);
  if (pass_cap > 0 && pass_cap < grid) grid = pass_cap;  // RICRC_RS_PASS_GRID (blocks then take several rounds)
  const bool fused = U == 4 && (uint64_t)grid * 4u * kPassBlock >= count;
  return PassShape{grid, U, fused, fused && !no_split && 2 * grid <= kPassBlocks};
}
bool rs_fused(uint64_t count, int pass_cap) { return count > 0 && pass_shape(count, pass_cap).fused; }
void rs_pass_info(uint64_t count, int pass_cap, bool no_split, int *grid, int *unroll, bool *fused, int *ggrid) {
  const PassShape ps = pass_shape(count, pass_cap, no_split);
  *grid = ps.grid;
  *unroll = ps.U;
  *fused = ps.fused;
  *ggrid = ps.split ? 2 * ps.grid : ps.grid;
}
static void launch_bucket(const RsckArgs &a, const PassShape &ps, hipStream_t st) {
  switch (ps.U) {
    case 4: launch_bucket_u<4>(a, ps.grid, st); break;
    case 8: launch_bucket_u<8>(a, ps.grid, st); break;
    case kPassUnroll: launch_bucket_u<kPassUnroll>(a, ps.grid, st); break;
    default: launch_bucket_u<kPassUnrollBig>(a, ps.grid, st); break;
  }
}
static void launch_gather(const RsckArgs &a, const PassShape &ps, hipStream_t st) {
  switch (ps.U) {  // the gather's blocks are the bucket pass's (block b serves pass block b's packets)
    case 4:
      if (ps.split) hipLaunchKernelGGL((rsck_gather<4, true, true>), dim3(2 * ps.grid), dim3(kPassBlock), 0, st, a);
      else if (ps.fused) hipLaunchKernelGGL((rsck_gather<4, true>), dim3(ps.grid), dim3(kPassBlock), 0, st, a);
      else hipLaunchKernelGGL((rsck_gather<4, false>), dim3(ps.grid), dim3(kPassBlock), 0, st, a);
      break;
    case 8: hipLaunchKernelGGL((rsck_gather<8, false>), dim3(ps.grid), dim3(kPassBlock), 0, st, a); break;
    case kPassUnroll: hipLaunchKernelGGL((rsck_gather<kPassUnroll, false>), dim3(ps.grid), dim3(kPassBlock), 0, st, a); break;
    default: hipLaunchKernelGGL((rsck_gather<kPassUnrollBig, false>), dim3(ps.grid), dim3(kPassBlock), 0, st, a); break;
  }
}

hipError_t launch_rswg(const RsckArgs &a, int grid, hipStream_t st, hipEvent_t *pass_ev) {
  (void)hipGetLastError();  // a stale error of an earlier, unrelated HIP call must not fail this launch
  if (a.count == 0) return hipSuccess;
  if (a.count > kRsMaxCount) return hipErrorInvalidValue;
  // RICRC_PASS_TIMES: the one kernel counts as the fold (bucket, one-line and gather 0)
  if (pass_ev) {
    (void)hipEventRecord(pass_ev[0], st);
    (void)hipEventRecord(pass_ev[1], st);
  }
  hipLaunchKernelGGL((icrc_rswg_kernel<0>), dim3(grid), dim3(kBlock), 0, st, a);
  if (pass_ev)
    for (int k = 2; k < 5; ++k) (void)hipEventRecord(pass_ev[k], st);
  return hipGetLastError();
}

uint64_t rs_wg_chunks(uint64_t count, int grid, const uint32_t (&w)[8]) {
  // the heaviest workgroup's share: count x w_max / w_mean (xcd_share), rounded up
  uint64_t wsum = 0, wmax = 0;
  for (int x = 0; x < 8; ++x) {
    wsum += w[x];
    wmax = w[x] > wmax ? w[x] : wmax;
  }
  const uint64_t g = grid > 0 ? (uint64_t)grid : 1u;
  const uint64_t share = wsum ? (count * wmax * 8u + wsum * g - 1u) / (wsum * g) + 1u : (count + g - 1u) / g;
  return (share + kWgCap - 1u) / kWgCap;
}

hipError_t launch_rsck(RsckArgs &a, int grid, int pass_cap, hipStream_t st, hipEvent_t *pass_ev) {
  (void)hipGetLastError();  // a stale error of an earlier, unrelated HIP call must not fail this launch
  if (a.count == 0) return hipSuccess;
  if (a.count > kRsMaxCount) return hipErrorInvalidValue;
  // a.ctr is zero here: zeroed when the workspace was allocated, and again
  // by rsck_gather at the end of every call.
  PassShape ps = pass_shape(a.count, pass_cap, a.no_split != 0);
  if (a.small_in_fold) ps.fused = ps.split = false;  // the fold takes the one-line packets: a plain gather
  a.nblk = (uint32_t)ps.grid;
  // RICRC_PASS_TIMES: timing events between the passes on st (diagnostics)
  auto mark = [&](int k) { if (pass_ev) (void)hipEventRecord(pass_ev[k], st); };
  mark(0);
  launch_bucket(a, ps, st);
  mark(1);
  hipLaunchKernelGGL((icrc_rsck_kernel<0>), dim3(grid), dim3(kBlock), 0, st, a);
  mark(2);
  // RICRC_ONE_LINE_IN_GATHER: the small pool [0, ctr->small) one lane per
  // packet here, unless the gather folds each block's one-line packets
  // itself (ps.fused); by default the fold took them.  (Round 4 ran it
  // on 1/16 of the CUs on a second stream beside the fold instead: the step
  // took 1.050 against 0.999 ms -- its scattered half-line reads slowed the
  // fold by 60 us, profiles/r04/s2_*.)
  if (!ps.fused && !a.small_in_fold) hipLaunchKernelGGL(icrc_rsmall_kernel, dim3(grid), dim3(kBlock), 0, st, a);
  mark(3);
  launch_gather(a, ps, st);
  mark(4);
  return hipGetLastError();
}

}  // namespace ricrc
