// NIC rings with a length per slot: where the ragged
// pipeline's time goes by line count.  Timing only.
//   1. the product pipeline (launch_rsck) with events between its passes;
//   2. the fold alone, product build and timing ablations: memory path (no
//      table fold, no finish: ABL 3), no finish (2), no edge masks (8), no
//      result stores (16), compute with no line loads (16384);
//   3. the fold's per-wave timeline (ABL 524288 stamps);
//   4. a plain stream of the same lines in the fold's access order floor: a
//      wave reads 8 slots' line k per load, as the fold does.
// Ring: count slots of `slot` bytes, the L3 packet at 14 in each, lengths
// uniform over [lo, hi] (xorshift), random bytes.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 ring_len.hip -o ring_len
//   ./ring_len slot lo hi [count]      e.g. ./ring_len 1024 64 1010
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

// The lines of the ring's packets (each slot's lines 0 .. L-1 from its start),
// read 8 slots per wave load as the fold reads a group: wave w takes groups of
// 8 consecutive slots, lane 8 g + s reads slot s of line k of slot g.
__global__ __launch_bounds__(1024) void slot_stream(const uint8_t *p, const uint32_t *len, uint64_t count,
                                                    uint32_t slot, uint32_t *sink) {
  const uint64_t nw = (uint64_t)gridDim.x * 16, w = (uint64_t)blockIdx.x * 16 + (threadIdx.x >> 6);
  const uint32_t lane = threadIdx.x & 63, g = lane >> 3, s = lane & 7;
  const uint64_t groups = count / 8, per = (groups + nw - 1) / nw;
  const uint64_t q0 = w * per, q1 = q0 + per < groups ? q0 + per : groups;
  u32x4 acc = {0, 0, 0, 0};
  for (uint64_t q = q0; q < q1; ++q) {
    const uint64_t i = 8 * q + g;
    const uint32_t L = (14u + len[i] - 4u + 127u) >> 7;
    const uint32_t Lw = __builtin_amdgcn_readfirstlane(L);
    for (uint32_t k = 0; k < Lw; ++k)
      acc ^= __builtin_nontemporal_load(reinterpret_cast<const u32x4 *>(p + i * slot + 128u * k + 16u * s));
  }
  const uint32_t x = acc[0] ^ acc[1] ^ acc[2] ^ acc[3];
  if (x == 0x12345678u) sink[0] = x;
}

int main(int argc, char **argv) {
  hipDeviceProp_t p; CK(hipGetDeviceProperties(&p, 0));
  const int grid = p.multiProcessorCount;
  if (argc < 4) { printf("usage: ring_len slot lo hi [count]\n"); return 2; }
  const uint32_t slot = (uint32_t)atoi(argv[1]), lo = (uint32_t)atoi(argv[2]), hi = (uint32_t)atoi(argv[3]);
  const uint64_t count = argc > 4 ? strtoull(argv[4], nullptr, 0) : (1ull << 20);
  const uint32_t l3 = 14;
  std::vector<uint32_t> len(count);
  uint64_t x = 0x1CEC0DEull, bytes = 0, lines = 0;
  for (uint64_t i = 0; i < count; ++i) {
    x ^= x << 13; x ^= x >> 7; x ^= x << 17;
    len[i] = lo + (uint32_t)((x >> 20) % (hi - lo + 1));
    bytes += len[i];
    lines += (l3 + len[i] - 4 + 127) / 128;
  }
  uint8_t *buf; CK(hipMalloc(&buf, count * slot + 4096));
  {
    std::vector<uint64_t> h((count * slot + 4096) / 8);
    uint64_t y = 0x5EEDull;
    for (auto &v : h) { y ^= y << 13; y ^= y >> 7; y ^= y << 17; v = y; }
    CK(hipMemcpy(buf, h.data(), 8 * h.size(), hipMemcpyHostToDevice));
  }
  uint32_t *d_len, *out, *tzb, *sink;
  CK(hipMalloc(&d_len, 4 * count));
  CK(hipMalloc(&out, 4 * (count > 65536 ? count : 65536)));
  CK(hipMalloc(&tzb, 4 * 1024)); CK(hipMemset(tzb, 0x35, 4 * 1024));
  CK(hipMalloc(&sink, 8 * 8192 * 4));
  CK(hipMemcpy(d_len, len.data(), 4 * count, hipMemcpyHostToDevice));
  void *ws; CK(hipMalloc(&ws, rs_workspace_bytes(count)));
  CK(rs_zero_counters(ws, 0));
  RsckArgs a{};
  a.base = buf; a.off = nullptr; a.len = d_len; a.stride = slot; a.l3_offset = l3; a.count = count;
  a.out = out; a.tzb = tzb; a.group_cost = kRsGroupCost;
  a.small_in_fold = 1u; a.small_slots = kRsSmallSlots;
  a.fin = mb_fin();
  for (int k = 0; k < 8; ++k) a.xw[k] = 1000u + ((k & 1) ? -40 : 40);
  rs_bind_workspace(a, ws);
  const double alg = (double)bytes + 8.0 * (double)count;
  printf("ring: %llu slots of %u B, lengths %u-%u, %.1f MB of packets, %.2f lines per packet, alg %.1f MB "
         "(%.1f us at 8 TB/s); fold grid %d\n", (unsigned long long)count, slot, lo, hi, bytes / 1e6,
         (double)lines / count, alg / 1e6, alg / 8e6, grid);
  {  // out of the idle power state: 200 ms of the pipeline
    hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
    float ms = 0;
    while (ms < 200.f) {
      CK(hipEventRecord(e0));
      for (int i = 0; i < 100; ++i) CK(launch_rsck(a, grid, 0, 0, nullptr));
      CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
      float d; CK(hipEventElapsedTime(&d, e0, e1)); ms += d;
    }
  }
  hipEvent_t ev[5];
  for (auto &evk : ev) CK(hipEventCreate(&evk));
  const char *pass[4] = {"bucket", "fold", "one-line", "gather"};
  for (int r = 0; r < 2; ++r) {
    double sum[4] = {0, 0, 0, 0};
    const int reps = 20;
    for (int it = 0; it < 3 + reps; ++it) {
      CK(launch_rsck(a, grid, 0, 0, ev));
      CK(hipEventSynchronize(ev[4]));
      if (it < 3) continue;
      for (int k = 0; k < 4; ++k) { float ms; CK(hipEventElapsedTime(&ms, ev[k], ev[k + 1])); sum[k] += 1e3 * ms / reps; }
    }
    const float back = timeit([&] { CK(launch_rsck(a, grid, 0, 0, nullptr)); }, 50);
    printf("pipeline: back to back %.1f us/call (%.3f of 8 TB/s) | with events:", back, alg / back / 8e6);
    for (int k = 0; k < 4; ++k) printf(" %s %.1f", pass[k], sum[k]);
    printf("\n");
  }
  const PassShape ps = pass_shape(count, 0);
  a.nblk = (uint32_t)ps.grid;
  CK(rs_zero_counters(ws, 0));
  launch_bucket(a, ps, 0);
  CK(hipDeviceSynchronize());
  const int nw = grid * kWaves;
  std::vector<uint32_t> st(8 * nw);
  for (int r = 0; r < 2; ++r) {
    const float f0 = timeit([&] { hipLaunchKernelGGL((icrc_rsck_kernel<0>), dim3(grid), dim3(kBlock), 0, 0, a); }, 20);
    const float fm = timeit([&] { hipLaunchKernelGGL((icrc_rsck_kernel<3>), dim3(grid), dim3(kBlock), 0, 0, a); }, 20);
    const float f2 = timeit([&] { hipLaunchKernelGGL((icrc_rsck_kernel<2>), dim3(grid), dim3(kBlock), 0, 0, a); }, 20);
    const float f8 = timeit([&] { hipLaunchKernelGGL((icrc_rsck_kernel<8>), dim3(grid), dim3(kBlock), 0, 0, a); }, 20);
    const float f16 = timeit([&] { hipLaunchKernelGGL((icrc_rsck_kernel<16>), dim3(grid), dim3(kBlock), 0, 0, a); }, 20);
    const float fn = timeit([&] { hipLaunchKernelGGL((icrc_rsck_kernel<16384>), dim3(grid), dim3(kBlock), 0, 0, a); }, 20);
    const float fnn = timeit([&] { hipLaunchKernelGGL((icrc_rsck_kernel<16384 | 3>), dim3(grid), dim3(kBlock), 0, 0, a); }, 20);
    const float fs = timeit([&] { hipLaunchKernelGGL(slot_stream, dim3(grid), dim3(1024), 0, 0, buf, d_len, count, slot, sink); }, 20);
    printf("fold alone %.1f us | memory path (ABL 3) %.1f | no finish %.1f | no edge masks %.1f | no stores %.1f | "
           "no loads %.1f | control only (no loads, no fold, no finish) %.1f | slot stream of the same lines %.1f\n",
           f0, fm, f2, f8, f16, fn, fnn, fs);
    hipLaunchKernelGGL((icrc_rsck_kernel<524288>), dim3(grid), dim3(kBlock), 0, 0, a);
    CK(hipDeviceSynchronize());
    CK(hipMemcpy(st.data(), out, 4 * st.size(), hipMemcpyDeviceToHost));
    uint32_t t0 = st[0];
    for (int w = 0; w < nw; ++w) t0 = (int32_t)(st[8 * w] - t0) < 0 ? st[8 * w] : t0;
    std::vector<double> en(nw), tb(nw), sp(nw), l1(nw);
    for (int w = 0; w < nw; ++w) {
      tb[w] = (int32_t)(st[8 * w + 1] - t0) / 100.0;
      sp[w] = (int32_t)(st[8 * w + 2] - t0) / 100.0;
      en[w] = (int32_t)(st[8 * w + 3] - t0) / 100.0;
      l1[w] = (int32_t)(st[8 * w + 4] - t0) / 100.0;
    }
    auto pct = [](std::vector<double> v, double q) { std::sort(v.begin(), v.end()); return v[(size_t)(q * (v.size() - 1))]; };
    printf("  timeline (us): tables p50 %.1f | split p50 %.1f | first line p50 %.1f | end p1 %.1f p50 %.1f p99 %.1f max %.1f\n",
           pct(tb, 0.5), pct(sp, 0.5), pct(l1, 0.5), pct(en, 0.01), pct(en, 0.5), pct(en, 0.99), pct(en, 1));
  }
  return 0;
}
