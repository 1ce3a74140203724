// C4's 8-GPU shard (about 524 K mixed packets per GPU):
// where the ragged pipeline's time goes at this size.  Timing only.
//   1. the product pipeline (launch_rsck) with events between its passes, and
//      back to back without events (the per-call time with the launch gaps);
//   2. the fold's per-wave timeline (ABL 524288 stamps: entry, tables built,
//      work split found, end);
//   3. the bucket pass by packets per thread (template U);
//   4. the floor: a plain streaming read of the same bytes on the same grid.
// Batch: lengths uniform over {64, 256, 1024, 4096} (xorshift), packed back to
// back, random bytes.  Args: [count] (default 524288).
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 shard.hip -o shard
#include "../../roce-test_amd/csrc/icrc_kernels.hip"
#include "../../roce-test_amd/csrc/icrc_rsck.hip"
#include "mb_fin.h"
#include <stdio.h>
#include <stdlib.h>

#include <algorithm>
#include <vector>
using namespace ricrc;
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s line %d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)

template <typename F> float timeit(F launch, int reps) {
  hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  for (int w = 0; w < 3; ++w) launch();
  CK(hipDeviceSynchronize()); CK(hipEventRecord(e0));
  for (int i = 0; i < reps; ++i) launch();
  CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1)); float ms; CK(hipEventElapsedTime(&ms, e0, e1));
  CK(hipEventDestroy(e0)); CK(hipEventDestroy(e1));
  return 1e3f * ms / reps;
}

// Streaming floor: wave w reads 16-byte slots nt over [lo, hi) of the bytes in
// 1 KiB wave steps, 8 in flight, and XORs them into one word.
template <bool STAMP = false>
__global__ __launch_bounds__(1024) void stream_floor(const uint8_t *p, uint64_t bytes, uint32_t *sink) {
  const uint32_t t_entry = STAMP ? (uint32_t)__builtin_amdgcn_s_memrealtime() : 0u;
  const uint64_t nw = (uint64_t)gridDim.x * 16, w = (uint64_t)blockIdx.x * 16 + (threadIdx.x >> 6);
  const uint64_t steps = bytes / 1024, per = (steps + nw - 1) / nw;
  const uint64_t s0 = w * per, s1 = s0 + per < steps ? s0 + per : steps;
  u32x4 acc = {0, 0, 0, 0};
  const uint32_t lane = threadIdx.x & 63;
  uint64_t s = s0;
  for (; s + 8 <= s1; s += 8) {
    u32x4 v[8];
#pragma unroll
    for (int k = 0; k < 8; ++k)
      v[k] = __builtin_nontemporal_load(reinterpret_cast<const u32x4 *>(p + (s + k) * 1024 + 16 * lane));
#pragma unroll
    for (int k = 0; k < 8; ++k) acc ^= v[k];
  }
  for (; s < s1; ++s) acc ^= __builtin_nontemporal_load(reinterpret_cast<const u32x4 *>(p + s * 1024 + 16 * lane));
  const uint32_t x = acc[0] ^ acc[1] ^ acc[2] ^ acc[3];
  if (x == 0x12345678u) sink[0] = x;
  if (STAMP && lane == 0) {
    sink[2 * w] = t_entry;
    sink[2 * w + 1] = (uint32_t)__builtin_amdgcn_s_memrealtime() + (x == 0x12345678u ? 1u : 0u);
  }
}

int main(int argc, char **argv) {
  hipDeviceProp_t p; CK(hipGetDeviceProperties(&p, 0));
  const int grid = p.multiProcessorCount;
  const uint64_t count = argc > 1 ? strtoull(argv[1], nullptr, 0) : 524288ull;
  std::vector<uint64_t> off(count);
  std::vector<uint32_t> len(count);
  const uint32_t sizes[4] = {64, 256, 1024, 4096};
  uint64_t x = 0x1CEC0DEull, pos = 0, fold_bytes = 0;
  for (uint64_t i = 0; i < count; ++i) {
    x ^= x << 13; x ^= x >> 7; x ^= x << 17;
    len[i] = sizes[(x >> 33) & 3];
    off[i] = pos;
    pos += len[i];
    fold_bytes += len[i] > 64 ? len[i] : 0;
  }
  uint8_t *buf; CK(hipMalloc(&buf, pos + 4096));
  {
    std::vector<uint64_t> h((pos + 4096) / 8);
    uint64_t y = 0x5EEDull;
    for (auto &v : h) { y ^= y << 13; y ^= y >> 7; y ^= y << 17; v = y; }
    CK(hipMemcpy(buf, h.data(), 8 * h.size(), hipMemcpyHostToDevice));
  }
  uint64_t *d_off; uint32_t *d_len, *out, *tzb, *sink;
  CK(hipMalloc(&d_off, 8 * count)); CK(hipMalloc(&d_len, 4 * count));
  CK(hipMalloc(&out, 4 * (count > 65536 ? count : 65536)));
  CK(hipMalloc(&tzb, 4 * 1024)); CK(hipMemset(tzb, 0x35, 4 * 1024));
  CK(hipMalloc(&sink, 8 * 8192 * 4));
  CK(hipMemcpy(d_off, off.data(), 8 * count, hipMemcpyHostToDevice));
  CK(hipMemcpy(d_len, len.data(), 4 * count, hipMemcpyHostToDevice));
  void *ws; CK(hipMalloc(&ws, rs_workspace_bytes(count)));
  CK(rs_zero_counters(ws, 0));
  RsckArgs a{};
  a.base = buf; a.off = d_off; a.len = d_len; a.count = count;
  a.out = out; a.tzb = tzb; a.group_cost = kRsGroupCost;
  a.small_in_fold = 1u; a.small_slots = kRsSmallSlots;  // the product's defaults (icrc_api.cpp)
  a.fin = mb_fin();
  for (int k = 0; k < 8; ++k) a.xw[k] = 1000u + ((k & 1) ? -40 : 40);
  rs_bind_workspace(a, ws);
  const double alg = (double)pos + 16.0 * (double)count;
  printf("shard batch: %llu packets, %.1f MB (%.1f MB in packets of >= 2 lines), alg %.1f MB; fold grid %d\n",
         (unsigned long long)count, pos / 1e6, fold_bytes / 1e6, alg / 1e6, grid);

  hipEvent_t ev[5];
  for (auto &evk : ev) CK(hipEventCreate(&evk));
  // out of the idle power state: 200 ms of the pipeline
  {
    hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
    float ms = 0;
    while (ms < 200.f) {
      CK(hipEventRecord(e0));
      for (int i = 0; i < 100; ++i) CK(launch_rsck(a, grid, 0, 0, nullptr));
      CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
      float d; CK(hipEventElapsedTime(&d, e0, e1)); ms += d;
    }
  }
  const char *pass[4] = {"bucket", "fold", "one-line", "gather"};
  for (int r = 0; r < 3; ++r) {
    double sum[4] = {0, 0, 0, 0};
    const int reps = 20;
    for (int it = 0; it < 3 + reps; ++it) {
      CK(launch_rsck(a, grid, 0, 0, ev));
      CK(hipEventSynchronize(ev[4]));
      if (it < 3) continue;
      for (int k = 0; k < 4; ++k) { float ms; CK(hipEventElapsedTime(&ms, ev[k], ev[k + 1])); sum[k] += 1e3 * ms / reps; }
    }
    const float back = timeit([&] { CK(launch_rsck(a, grid, 0, 0, nullptr)); }, 50);
    printf("pipeline round %d: back to back %.1f us/call (%.3f of 8 TB/s) | with events:", r, back, alg / back / 8e6);
    for (int k = 0; k < 4; ++k) printf(" %s %.1f", pass[k], sum[k]);
    printf(" = %.1f\n", sum[0] + sum[1] + sum[2] + sum[3]);
  }
  // the fold alone, after one bucket pass (the gather would zero the counters)
  const PassShape ps = pass_shape(count, 0);
  a.nblk = (uint32_t)ps.grid;
  printf("pass shape: %d blocks x %d packets per thread\n", ps.grid, ps.U);
  CK(rs_zero_counters(ws, 0));
  launch_bucket(a, ps, 0);
  CK(hipDeviceSynchronize());
  {
    const int nw = grid * kWaves;
    std::vector<uint32_t> st(8 * nw);
    for (int r = 0; r < 3; ++r) {
      const float f0 = timeit([&] { hipLaunchKernelGGL((icrc_rsck_kernel<0>), dim3(grid), dim3(kBlock), 0, 0, a); }, 20);
      const float fm = timeit([&] { hipLaunchKernelGGL((icrc_rsck_kernel<3>), dim3(grid), dim3(kBlock), 0, 0, a); }, 20);
      const float fs = timeit([&] { hipLaunchKernelGGL(stream_floor<false>, dim3(grid), dim3(1024), 0, 0, buf, pos, sink); }, 20);
      printf("fold alone %.1f us (%.2f TB/s of its packets) | memory path %.1f | plain stream of all %.1f MB %.1f us (%.2f TB/s)\n",
             f0, fold_bytes / f0 / 1e6, fm, pos / 1e6, fs, pos / fs / 1e6);
      hipLaunchKernelGGL((icrc_rsck_kernel<524288>), dim3(grid), dim3(kBlock), 0, 0, a);
      CK(hipDeviceSynchronize());
      CK(hipMemcpy(st.data(), out, 4 * st.size(), hipMemcpyDeviceToHost));
      uint32_t t0 = st[0];
      for (int w = 0; w < nw; ++w) t0 = (int32_t)(st[8 * w] - t0) < 0 ? st[8 * w] : t0;
      std::vector<double> en(nw), tb(nw), sp(nw), ent(nw), c1(nw), l1(nw), work;
      for (int w = 0; w < nw; ++w) {
        ent[w] = (int32_t)(st[8 * w] - t0) / 100.0;
        tb[w] = (int32_t)(st[8 * w + 1] - t0) / 100.0;
        sp[w] = (int32_t)(st[8 * w + 2] - t0) / 100.0;
        en[w] = (int32_t)(st[8 * w + 3] - t0) / 100.0;
        l1[w] = (int32_t)(st[8 * w + 4] - t0) / 100.0;
        c1[w] = (int32_t)(st[8 * w + 5] - t0) / 100.0;
      }
      auto pct = [](std::vector<double> v, double q) { std::sort(v.begin(), v.end()); return v[(size_t)(q * (v.size() - 1))]; };
      printf("  timeline (us from the first entry): entry p50 %.1f max %.1f | tables p50 %.1f max %.1f | split p50 %.1f max %.1f | "
             "end p1 %.1f p10 %.1f p50 %.1f p90 %.1f p99 %.1f max %.1f\n",
             pct(ent, 0.5), pct(ent, 1), pct(tb, 0.5), pct(tb, 1), pct(sp, 0.5), pct(sp, 1), pct(en, 0.01), pct(en, 0.1),
             pct(en, 0.5), pct(en, 0.9), pct(en, 0.99), pct(en, 1));
      printf("  counters arrived p50 %.1f max %.1f | first line arrived p10 %.1f p50 %.1f max %.1f\n", pct(c1, 0.5),
             pct(c1, 1), pct(l1, 0.1), pct(l1, 0.5), pct(l1, 1));
      std::vector<double> tb2(nw);
      for (int w = 0; w < nw; ++w) tb2[w] = (int32_t)(st[8 * w + 6] - t0) / 100.0;
      printf("  table build's instructions done p50 %.1f max %.1f", pct(tb2, 0.5), pct(tb2, 1));
      printf("\n  mean end by wave slot:");
      for (int sl = 0; sl < kWaves; ++sl) { double m = 0; for (int b = 0; b < grid; ++b) m += en[b * kWaves + sl]; printf(" %.0f", m / grid); }
      printf("\n");
      // the plain stream's own timeline
      hipLaunchKernelGGL(stream_floor<true>, dim3(grid), dim3(1024), 0, 0, buf, pos, sink);
      CK(hipDeviceSynchronize());
      std::vector<uint32_t> ss(2 * nw);
      CK(hipMemcpy(ss.data(), sink, 4 * ss.size(), hipMemcpyDeviceToHost));
      uint32_t s0 = ss[0];
      for (int w = 0; w < nw; ++w) s0 = (int32_t)(ss[2 * w] - s0) < 0 ? ss[2 * w] : s0;
      std::vector<double> se(nw);
      for (int w = 0; w < nw; ++w) se[w] = (int32_t)(ss[2 * w + 1] - s0) / 100.0;
      printf("  plain stream timeline: end p1 %.1f p10 %.1f p50 %.1f p90 %.1f p99 %.1f max %.1f\n", pct(se, 0.01),
             pct(se, 0.1), pct(se, 0.5), pct(se, 0.9), pct(se, 0.99), pct(se, 1));
    }
  }
  // the gather alone (after the bucket pass and the fold above): split into
  // gather + small sides (product), fused on the pass grid, and the plain
  // gather with the one-line kernel before it
  {
    CK(rs_zero_counters(ws, 0));
    launch_bucket(a, ps, 0);
    hipLaunchKernelGGL((icrc_rsck_kernel<0>), dim3(grid), dim3(kBlock), 0, 0, a);
    CK(hipDeviceSynchronize());
    const int g = ps.grid;
    for (int r = 0; r < 3; ++r) {
      const float gs = timeit([&] { hipLaunchKernelGGL((rsck_gather<4, true, true>), dim3(2 * g), dim3(kPassBlock), 0, 0, a); }, 20);
      const float gf = timeit([&] { hipLaunchKernelGGL((rsck_gather<4, true>), dim3(g), dim3(kPassBlock), 0, 0, a); }, 20);
      const float gp = timeit([&] { hipLaunchKernelGGL((rsck_gather<4, false>), dim3(g), dim3(kPassBlock), 0, 0, a); }, 20);
      printf("gather alone: small sides beside it (%d blocks) %.1f us | one-line folded in the gather (%d) %.1f | plain gather %.1f\n",
             2 * g, gs, g, gf, gp);
    }
  }
  // the bucket pass by packets per thread (one round when U x 1024 x blocks >= count)
  auto bucket_u = [&](auto uc, int pg) {
    constexpr int U = decltype(uc)::value;
    a.nblk = (uint32_t)pg;
    return timeit([&] {
      CK(rs_zero_counters(ws, 0));
      hipLaunchKernelGGL((rsck_bucket<true, true, 0, U>), dim3(pg), dim3(kPassBlock), 0, 0, a);
    }, 20);
  };
  const float zero = timeit([&] { CK(rs_zero_counters(ws, 0)); }, 20);
  for (int r = 0; r < 3; ++r) {
    printf("bucket (incl. a %.1f us counter memset): U=16 x 256 %.1f | U=4 x 256 %.1f | U=2 x 256 %.1f | U=4 x 128 %.1f | U=8 x 64 %.1f\n",
           zero, bucket_u(std::integral_constant<int, 16>{}, 256), bucket_u(std::integral_constant<int, 4>{}, 256),
           bucket_u(std::integral_constant<int, 2>{}, 256), bucket_u(std::integral_constant<int, 4>{}, 128),
           bucket_u(std::integral_constant<int, 8>{}, 64));
  }
  return 0;
}
