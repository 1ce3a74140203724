// The workgroup-local ragged kernel (icrc_rswg_kernel) at C4's 8-GPU shard
// or a NIC ring with per-slot lengths: where its time goes.  Timing only.
//   1. the product kernel, and timing ablations: memory path (no table fold,
//      no finish: ABL 3), compute with no line loads (16384), control only
//      (16384 | 3);
//   2. its per-wave timeline (ABL 524288 stamps: entry, layout done, one-line
//      rounds done, fold done, end), the mean fold end by wave slot and the
//      spread of the workgroups' ends;
//   3. the floor: a plain streaming read of the batch's bytes on the same grid.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 wg.hip -o wg
//   ./wg mix [count]                 C4's mix, packed (default 524288)
//   ./wg ring slot lo hi [count]     slots of `slot` bytes, L3 at 14, lengths lo..hi
#include "../../roce-test_amd/csrc/icrc_kernels.hip"
#include "../../roce-test_amd/csrc/icrc_rsck.hip"
#include "mb_fin.h"
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

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

__global__ __launch_bounds__(1024) void stream_floor(const uint8_t *p, uint64_t bytes, uint32_t *sink) {
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
}

int main(int argc, char **argv) {
  hipDeviceProp_t p; CK(hipGetDeviceProperties(&p, 0));
  const int grid = p.multiProcessorCount;
  const bool ring = argc > 1 && !strcmp(argv[1], "ring");
  uint32_t slot = 0, lo = 0, hi = 0;
  uint64_t count;
  if (ring) {
    if (argc < 5) { printf("usage: wg ring slot lo hi [count]\n"); return 2; }
    slot = (uint32_t)atoi(argv[2]); lo = (uint32_t)atoi(argv[3]); hi = (uint32_t)atoi(argv[4]);
    count = argc > 5 ? strtoull(argv[5], nullptr, 0) : (1ull << 20);
  } else {
    count = argc > 2 ? strtoull(argv[2], nullptr, 0) : 524288ull;
  }
  std::vector<uint64_t> off(count);
  std::vector<uint32_t> len(count);
  const uint32_t sizes[4] = {64, 256, 1024, 4096};
  uint64_t x = 0x1CEC0DEull, pos = 0, bytes = 0;
  for (uint64_t i = 0; i < count; ++i) {
    x ^= x << 13; x ^= x >> 7; x ^= x << 17;
    if (ring) {
      len[i] = lo + (uint32_t)((x >> 20) % (hi - lo + 1));
      off[i] = i * slot;
    } else {
      len[i] = sizes[(x >> 33) & 3];
      off[i] = pos;
      pos += len[i];
    }
    bytes += len[i];
  }
  const uint64_t buf_bytes = ring ? count * slot + 4096 : pos + 4096;
  uint8_t *buf; CK(hipMalloc(&buf, buf_bytes));
  {
    std::vector<uint64_t> h(buf_bytes / 8);
    uint64_t y = 0x5EEDull;
    for (auto &v : h) { y ^= y << 13; y ^= y >> 7; y ^= y << 17; v = y; }
    CK(hipMemcpy(buf, h.data(), 8 * h.size(), hipMemcpyHostToDevice));
  }
  uint64_t *d_off; uint32_t *d_len, *out, *tzb, *sink, *stamps;
  CK(hipMalloc(&d_off, 8 * count)); CK(hipMalloc(&d_len, 4 * count));
  CK(hipMalloc(&out, 4 * count));
  CK(hipMalloc(&tzb, 4 * 1024)); CK(hipMemset(tzb, 0x35, 4 * 1024));
  CK(hipMalloc(&sink, 64));
  const int nw = grid * kWaves;
  CK(hipMalloc(&stamps, 4 * 8 * nw));
  CK(hipMemcpy(d_off, off.data(), 8 * count, hipMemcpyHostToDevice));
  CK(hipMemcpy(d_len, len.data(), 4 * count, hipMemcpyHostToDevice));
  RsckArgs a{};
  a.base = buf; a.len = d_len; a.count = count;
  if (ring) { a.off = nullptr; a.stride = slot; a.l3_offset = 14; } else { a.off = d_off; }
  a.out = out; a.tzb = tzb; a.group_cost = kRsGroupCost; a.fin = mb_fin();
  const int skew = getenv("WG_SKEW") ? atoi(getenv("WG_SKEW")) : 40;  // per-mille moved to even XCD slots
  for (int k = 0; k < 8; ++k) a.xw[k] = skew ? 1000u + ((k & 1) ? -skew : skew) : 0u;
  if (getenv("WG_XW")) {  // eight weights, per XCD slot relative to block 0's XCD
    const char *c = getenv("WG_XW");
    for (int k = 0; k < 8 && *c; ++k) { a.xw[k] = (uint32_t)atoi(c); while (*c && *c != ',') ++c; if (*c) ++c; }
  }
  printf("xcd weights:"); for (int k = 0; k < 8; ++k) printf(" %u", a.xw[k]); printf("\n");
  a.pos_of = stamps;
  const double alg = (double)bytes + (ring ? 8.0 : 16.0) * (double)count;
  printf("%s: %llu packets, %.1f MB, alg %.1f MB (%.1f us at 8 TB/s); grid %d, chunks on the heaviest workgroup %llu\n",
         ring ? "ring" : "C4 mix", (unsigned long long)count, bytes / 1e6, alg / 1e6, alg / 8e6, grid,
         (unsigned long long)rs_wg_chunks(count, grid, a.xw));
  auto run = [&](auto abl) { hipLaunchKernelGGL((icrc_rswg_kernel<decltype(abl)::value>), dim3(grid), dim3(kBlock), 0, 0, a); };
  {  // out of the idle power state
    float ms = 0;
    hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
    while (ms < 200.f) {
      CK(hipEventRecord(e0));
      for (int i = 0; i < 100; ++i) run(std::integral_constant<int, 0>{});
      CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
      float d; CK(hipEventElapsedTime(&d, e0, e1)); ms += d;
    }
  }
  std::vector<uint32_t> st(8 * nw);
  {  // the XCD block 0 runs on (the product passes the last launch's record as xcd_k)
    run(std::integral_constant<int, 524288>{});
    CK(hipDeviceSynchronize());
    CK(hipMemcpy(st.data(), stamps, 4 * st.size(), hipMemcpyDeviceToHost));
    a.xcd_k = st[7] & 7u;
    printf("xcd_k %u\n", a.xcd_k);
  }
  for (int r = 0; r < 3; ++r) {
    const float f0 = timeit([&] { run(std::integral_constant<int, 0>{}); }, 20);
    const float fm = timeit([&] { run(std::integral_constant<int, 3>{}); }, 20);
    const float fn = timeit([&] { run(std::integral_constant<int, 16384>{}); }, 20);
    const float fc = timeit([&] { run(std::integral_constant<int, 16384 | 3>{}); }, 20);
    const float fs = timeit([&] { hipLaunchKernelGGL(stream_floor, dim3(grid), dim3(1024), 0, 0, buf, buf_bytes - 4096, sink); }, 20);
    printf("kernel %.1f us (%.3f of 8 TB/s) | memory path %.1f | no loads %.1f | control only %.1f | plain stream of %.1f MB %.1f us\n",
           f0, alg / f0 / 8e6, fm, fn, fc, (buf_bytes - 4096) / 1e6, fs);
    run(std::integral_constant<int, 524288>{});
    CK(hipDeviceSynchronize());
    CK(hipMemcpy(st.data(), stamps, 4 * st.size(), hipMemcpyDeviceToHost));
    uint32_t t0 = st[0];
    for (int w = 0; w < nw; ++w) t0 = (int32_t)(st[8 * w] - t0) < 0 ? st[8 * w] : t0;
    std::vector<double> ent(nw), lay(nw), sm(nw), fd(nw), en(nw), grp(nw), ranks(nw), wgend(grid, 0.0), wgfold(grid, 0.0);
    for (int w = 0; w < nw; ++w) {
      ent[w] = (int32_t)(st[8 * w] - t0) / 100.0;
      lay[w] = (int32_t)(st[8 * w + 1] - t0) / 100.0;
      sm[w] = (int32_t)(st[8 * w + 2] - t0) / 100.0;
      fd[w] = (int32_t)(st[8 * w + 3] - t0) / 100.0;
      en[w] = (int32_t)(st[8 * w + 4] - t0) / 100.0;
      grp[w] = (int32_t)(st[8 * w + 5] - t0) / 100.0;  // descriptors in
      ranks[w] = (int32_t)(st[8 * w + 6] - t0) / 100.0;
      wgend[w / kWaves] = std::max(wgend[w / kWaves], en[w]);
      wgfold[w / kWaves] = std::max(wgfold[w / kWaves], fd[w]);
    }
    auto pct = [](std::vector<double> v, double q) { std::sort(v.begin(), v.end()); return v[(size_t)(q * (v.size() - 1))]; };
    printf("  timeline (us): entry p50 %.1f max %.1f | layout p50 %.1f max %.1f | one-line done p50 %.1f max %.1f | "
           "fold done p1 %.1f p50 %.1f p99 %.1f max %.1f | end p50 %.1f max %.1f\n",
           pct(ent, .5), pct(ent, 1), pct(lay, .5), pct(lay, 1), pct(sm, .5), pct(sm, 1), pct(fd, .01), pct(fd, .5),
           pct(fd, .99), pct(fd, 1), pct(en, .5), pct(en, 1));
    printf("  layout phase: descriptors in p50 %.1f max %.1f | ranks counted p50 %.1f max %.1f | layout done p50 %.1f\n",
           pct(grp, .5), pct(grp, 1), pct(ranks, .5), pct(ranks, 1), pct(lay, .5));
    printf("  workgroups' fold end: p1 %.1f p10 %.1f p50 %.1f p90 %.1f max %.1f\n",
           pct(wgfold, .01), pct(wgfold, .1), pct(wgfold, .5), pct(wgfold, .9), pct(wgfold, 1));
    printf("  fold end by wave slot:");
    for (int sl = 0; sl < kWaves; ++sl) { double m = 0; for (int b = 0; b < grid; ++b) m += fd[b * kWaves + sl]; printf(" %.0f", m / grid); }
    printf("\n  fold end by XCD slot (block %% 8):");
    for (int xs = 0; xs < 8; ++xs) { double m = 0; int c = 0; for (int b = xs; b < grid; b += 8) { m += wgfold[b]; ++c; } printf(" %.1f", m / c); }
    printf("\n  fold end by physical XCD (HW_REG_XCC_ID) [workgroups]:");
    for (int xc = 0; xc < 8; ++xc) {
      double m = 0; int c = 0;
      for (int b = 0; b < grid; ++b) if ((st[8 * (b * kWaves) + 7] & 7u) == (uint32_t)xc) { m += wgfold[b]; ++c; }
      printf(" %.1f[%d]", c ? m / c : 0.0, c);
    }
    printf("  (block 0 on XCD %u)\n", st[7] & 7u);
  }
  return 0;
}
