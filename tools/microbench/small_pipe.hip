// The one-line kernel, software-pipelined (round 4).  The product's
// icrc_rsmall_kernel<1> takes one round of 64 packets per wave at a time:
// its half-line loads are issued, then waited for, then folded, and the
// result store goes out before the next round's loads -- so every round pays
// a full memory latency, and in the in-order vmcnt the next round's wait also
// covers the previous round's store.  Batching two rounds (R = 2) measured
// slower (profiles/r04/s6_*).  Here round r + 1's half-line loads are issued
// before round r is folded (one round in flight behind the fold; its
// descriptors two rounds ahead), so a wave waits on memory once at its start.
// Compared with the product kernel on the same bucketed batches (results
// bit-exact, times alternating): C4's mix (4 M packets, 1 M of them 64 B)
// and 1 M back-to-back 64-byte packets.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 small_pipe.hip -o small_pipe
#include "../../roce-test_amd/csrc/icrc_kernels.hip"
#include "../../roce-test_amd/csrc/icrc_rsck.hip"
#include <stdio.h>
#include <stdlib.h>

#include <vector>
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s line %d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)

namespace ricrc {
namespace {
__global__ __launch_bounds__(kBlock) void rsmall_pipe(RsckArgs a) {
  __shared__ uint32_t lds[kLdsWords];
  const uint32_t count = a.ctr->small;
  if (count == 0) return;
  const uint32_t tab_v = table_entry(g_tab);
  table_store(lds, tab_v);
  __syncthreads();
  const uint32_t lane = threadIdx.x & 63;
  const uint32_t wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const LaneTab lt{(lane & 31) << 2, ((lane & 31) << 2) | 0x10000u};
  const uint32_t step = gridDim.x * kWaves * 64u;
  const __amdgpu_buffer_rsrc_t ro = make_rsrc(a.res, 4u * count);
  auto desc_at = [&](uint32_t pos) -> RsDesc { return a.desc[pos < count ? pos : count - 1u]; };
  struct Round {
    RsDesc d;
    uint32_t Kmax;
    bool wa, uk, halfw;
    uint64_t hb;
  };
  auto shape = [&](const RsDesc &d) __attribute__((always_inline)) -> Round {
    Round o;
    o.d = d;
    uint32_t K = (((d.hi >> 16) - 4u) + 4u + 15u) >> 4;
    if (__builtin_amdgcn_ballot_w64(K > 4u) == 0) {
      o.Kmax = 4u;
    } else if (__builtin_amdgcn_ballot_w64(K > 8u) == 0) {
      o.Kmax = 8u;
    } else {
#pragma unroll
      for (int w = 32; w >= 1; w >>= 1) K = max(K, (uint32_t)__shfl_xor((int)K, w));
      o.Kmax = __builtin_amdgcn_readfirstlane((K + 3u) & ~3u);
    }
    o.wa = __builtin_amdgcn_ballot_w64(((d.lo | (d.hi >> 16)) & 3u) != 0) == 0;
    o.uk = __builtin_amdgcn_ballot_w64((d.hi >> 16) - 4u + 24u < 16u * o.Kmax) == 0;
    const uint64_t pa = ((uint64_t)(d.hi & 0xFFFFu) << 32) | d.lo;
    const uint64_t pe = pa + ((d.hi >> 16) - 4u);
    o.hb = (pe - 1u) & ~63ull;
    const bool half = pa >= o.hb && ((uint32_t)pe & 63u) > 48u;
    o.halfw = o.Kmax == 4u && __builtin_amdgcn_ballot_w64(!half) == 0;
    return o;
  };
  // the lane's quad reads 64 contiguous bytes of lane 4 p + c's half line;
  // hb lies in the last 64-byte block of a packet byte, so the load is in a
  // page the packet occupies whatever the round's shape
  auto half_line_load = [&](const Round &o, u32x4 (&H)[4]) __attribute__((always_inline)) {
    const uint32_t hlo = (uint32_t)o.hb, hhi = (uint32_t)(o.hb >> 32), q = lane & 3u;
    auto at = [&](uint32_t lo, uint32_t hi) { return ((uint64_t)hi << 32 | lo) + 16u * q; };
    H[0] = gload16(at(dpp_quad_bcast<0>(hlo), dpp_quad_bcast<0>(hhi)));
    H[1] = gload16(at(dpp_quad_bcast<1>(hlo), dpp_quad_bcast<1>(hhi)));
    H[2] = gload16(at(dpp_quad_bcast<2>(hlo), dpp_quad_bcast<2>(hhi)));
    H[3] = gload16(at(dpp_quad_bcast<3>(hlo), dpp_quad_bcast<3>(hhi)));
  };
  auto half_line_fold = [&](const Round &o, u32x4 (&H)[4], uint32_t pos, auto words,
                            auto uniform) __attribute__((always_inline)) {
    constexpr bool WA = decltype(words)::value;
    constexpr int M1 = decltype(uniform)::value ? 1 : 2;
    quad_transpose(H, lane & 3u);
    const u32x4 U[5] = {H[0], H[0], H[1], H[2], H[3]};
    SmallPk P;
    P.init(o.d, 4u);
    P.blocks<4, WA, M1>(lds, lt, U);
    __builtin_amdgcn_raw_buffer_store_b32(~P.reg, ro, pos < count ? 4u * pos : 0x7FFFFFF0u, 0, 0);
  };
  // any other round: the product's one_round (its own loads, then its fold)
  auto other_round = [&](const Round &o, uint32_t pos) __attribute__((always_inline)) {
    if (o.halfw) {
      u32x4 H[4];
      half_line_load(o, H);
      if (o.uk)
        half_line_fold(o, H, pos, std::false_type{}, std::true_type{});
      else
        half_line_fold(o, H, pos, std::false_type{}, std::false_type{});
      return;
    }
    SmallPk P;
    P.init(o.d, o.Kmax);
    auto run = [&](auto words, auto uniform) __attribute__((always_inline)) {
      constexpr bool WA = decltype(words)::value;
      constexpr int M1 = decltype(uniform)::value ? 1 : 2, M2 = decltype(uniform)::value ? 0 : 2;
      uint32_t j = 0;
      if ((o.Kmax & 7u) == 4u) {
        P.chunk<4, WA, M1>(lds, lt, 0);
        j = 4;
      } else {
        P.chunk<8, WA, M1>(lds, lt, 0);
        j = 8;
      }
      for (; j < o.Kmax; j += 8) P.chunk<8, WA, M2>(lds, lt, j);
    };
    if (o.wa && o.uk)
      run(std::true_type{}, std::true_type{});
    else if (o.uk)
      run(std::false_type{}, std::true_type{});
    else
      run(std::false_type{}, std::false_type{});
    __builtin_amdgcn_raw_buffer_store_b32(~P.reg, ro, pos < count ? 4u * pos : 0x7FFFFFF0u, 0, 0);
  };
  auto hot_of = [](const Round &o) { return o.halfw && o.wa && o.uk; };
  uint32_t base = (blockIdx.x * kWaves + wid) * 64u;
  if (base >= count) return;  // wave-uniform; no barrier below
  RsDesc dn = desc_at(base + step + lane);
  Round o = shape(desc_at(base + lane));
  bool hot = hot_of(o);  // wave-uniform: a round of word-aligned half-line packets (C4's 64 B)
  u32x4 H[4];
  if (hot) half_line_load(o, H);
  for (; base < count; base += step) {
    const RsDesc dnn = desc_at(base + 2u * step + lane);
    const Round on = shape(dn);
    const bool nhot = hot_of(on);
    u32x4 HN[4];
    if (hot) {  // wave-uniform
      if (nhot) half_line_load(on, HN);  // the next round's loads in flight before this round's fold
      __builtin_amdgcn_sched_barrier(0);
      half_line_fold(o, H, base + lane, std::true_type{}, std::true_type{});
    } else {
      other_round(o, base + lane);
      if (nhot) half_line_load(on, HN);
    }
    o = on;
    hot = nhot;
    dn = dnn;
#pragma unroll
    for (int k = 0; k < 4; ++k) H[k] = HN[k];
  }
}
}  // namespace
}  // namespace ricrc
using namespace ricrc;

template <typename F> float timeit(F launch, int reps) {
  hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  for (int w = 0; w < 3; ++w) launch();
  CK(hipDeviceSynchronize()); CK(hipEventRecord(e0));
  for (int i = 0; i < reps; ++i) launch();
  CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1)); float ms; CK(hipEventElapsedTime(&ms, e0, e1));
  CK(hipEventDestroy(e0)); CK(hipEventDestroy(e1));
  return 1e3f * ms / reps;
}

int main() {
  hipDeviceProp_t p; CK(hipGetDeviceProperties(&p, 0));
  const int grid = p.multiProcessorCount;
  struct Cfg { const char *name; std::vector<uint32_t> sizes; uint64_t count; };
  const Cfg cfgs[] = {{"C4 mix 64/256/1024/4096", {64, 256, 1024, 4096}, 4ull << 20},
                      {"64 B only", {64}, 1ull << 20},
                      {"mix 44..1500 B, any alignment", {}, 1ull << 20}};
  const uint64_t cap = 4ull << 20, cap_bytes = (4ull << 20) * 1360ull + (1ull << 20) * 4096ull;
  uint8_t *buf; CK(hipMalloc(&buf, cap_bytes + 4096));
  {
    std::vector<uint64_t> h(cap_bytes / 8);
    uint64_t x = 0x5EEDull;
    for (auto &v : h) { x ^= x << 13; x ^= x >> 7; x ^= x << 17; v = x; }
    CK(hipMemcpy(buf, h.data(), cap_bytes, hipMemcpyHostToDevice));
  }
  uint64_t *d_off; uint32_t *d_len, *out, *tzb;
  CK(hipMalloc(&d_off, 8 * cap)); CK(hipMalloc(&d_len, 4 * cap)); CK(hipMalloc(&out, 4 * cap));
  CK(hipMalloc(&tzb, 4 * 1024)); CK(hipMemset(tzb, 0x35, 4 * 1024));
  void *ws; CK(hipMalloc(&ws, rs_workspace_bytes(cap)));
  int fails = 0;
  for (const Cfg &c : cfgs) {
    CK(rs_zero_counters(ws, 0));
    std::vector<uint64_t> off(c.count);
    std::vector<uint32_t> len(c.count);
    uint64_t x = 0x1CEC0DEull, pos = 0;
    for (uint64_t i = 0; i < c.count; ++i) {
      x ^= x << 13; x ^= x >> 7; x ^= x << 17;
      if (c.sizes.empty()) {  // ragged, unaligned: one-line and multi-line small packets, big ones
        len[i] = 44 + (uint32_t)((x >> 20) % 1457);
        pos += (x >> 40) & 7;
      } else {
        len[i] = c.sizes[(x >> 33) % c.sizes.size()];
      }
      off[i] = pos;
      pos += len[i];
    }
    if (pos > cap_bytes) { printf("%s: %llu bytes exceed the buffer\n", c.name, (unsigned long long)pos); return 1; }
    CK(hipMemcpy(d_off, off.data(), 8 * c.count, hipMemcpyHostToDevice));
    CK(hipMemcpy(d_len, len.data(), 4 * c.count, hipMemcpyHostToDevice));
    RsckArgs a{};
    a.base = buf; a.off = d_off; a.len = d_len; a.count = c.count;
    a.out = out; a.tzb = tzb; a.group_cost = kRsGroupCost;
    rs_bind_workspace(a, ws);
    const uint64_t want = (c.count + kPassBlock - 1) / kPassBlock;
    a.nblk = (uint32_t)(want < kPassBlocks ? want : kPassBlocks);
    launch_bucket(a, (int)a.nblk, 0);
    CK(hipDeviceSynchronize());
    RsCounters ctr; CK(hipMemcpy(&ctr, a.ctr, sizeof ctr, hipMemcpyDeviceToHost));
    const uint32_t ns = ctr.small;
    std::vector<uint32_t> r1(ns), r2(ns);
    CK(hipMemset(a.res, 0, 4ull * ns));
    hipLaunchKernelGGL((icrc_rsmall_kernel<1>), dim3(grid), dim3(kBlock), 0, 0, a);
    CK(hipDeviceSynchronize());
    CK(hipMemcpy(r1.data(), a.res, 4ull * ns, hipMemcpyDeviceToHost));
    CK(hipMemset(a.res, 0, 4ull * ns));
    hipLaunchKernelGGL(rsmall_pipe, dim3(grid), dim3(kBlock), 0, 0, a);
    CK(hipDeviceSynchronize());
    CK(hipMemcpy(r2.data(), a.res, 4ull * ns, hipMemcpyDeviceToHost));
    uint64_t bad = 0;
    for (uint32_t i = 0; i < ns; ++i) bad += r1[i] != r2[i];
    fails += bad != 0;
    printf("%-30s %8llu packets, %u in the small pool: pipelined vs product %s (%llu differ)\n", c.name,
           (unsigned long long)c.count, ns, bad ? "DIFFER" : "bit-exact", (unsigned long long)bad);
    for (int r = 0; r < 5; ++r) {
      const float s1 = timeit([&] { hipLaunchKernelGGL((icrc_rsmall_kernel<1>), dim3(grid), dim3(kBlock), 0, 0, a); }, 20);
      const float sp = timeit([&] { hipLaunchKernelGGL(rsmall_pipe, dim3(grid), dim3(kBlock), 0, 0, a); }, 20);
      const float s2 = timeit([&] { hipLaunchKernelGGL((icrc_rsmall_kernel<2>), dim3(grid), dim3(kBlock), 0, 0, a); }, 20);
      printf("    round %d: product (R = 1) %6.1f | pipelined %6.1f | R = 2 %6.1f us\n", r, s1, sp, s2);
    }
  }
  return fails;
}
