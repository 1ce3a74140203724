// Ablation timing of the ragged strided-chain fold (icrc_rsck_kernel) next to
// the fixed-size SCK on the same bytes (timing only: outputs are meaningless
// for ABL != 0).  Build:
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 rsck_abl.hip -o rsck_abl
#include "../../roce-test_amd/csrc/icrc_kernels.hip"
#include "../../roce-test_amd/csrc/icrc_rsck.hip"
#include "../../roce-test_amd/csrc/icrc_sck.hip"
#include <stdio.h>
#include <stdlib.h>
#include <vector>
using namespace ricrc;
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s\n", hipGetErrorString(e)); exit(1); } } while (0)

template <typename F> float timeit(F launch, int reps) {
  hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  for (int w = 0; w < 3; ++w) launch();
  CK(hipDeviceSynchronize()); CK(hipEventRecord(e0));
  for (int i = 0; i < reps; ++i) launch();
  CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1)); float ms; CK(hipEventElapsedTime(&ms, e0, e1));
  return ms / reps;
}

int main(int argc, char **argv) {
  hipDeviceProp_t p; CK(hipGetDeviceProperties(&p, 0));
  const int grid = p.multiProcessorCount;
  const uint64_t bytes = 4ull << 30;
  uint8_t *buf; CK(hipMalloc(&buf, bytes + 4096));
  {
    std::vector<uint64_t> h(bytes / 8);
    uint64_t x = 0x9E3779B97F4A7C15ull;
    for (auto &v : h) { x ^= x << 13; x ^= x >> 7; x ^= x << 17; v = x; }
    CK(hipMemcpy(buf, h.data(), bytes, hipMemcpyHostToDevice));
  }
  uint32_t *out; CK(hipMalloc(&out, 4ull * (17u << 20)));
  uint32_t *tzb; CK(hipMalloc(&tzb, 4 * 1024)); CK(hipMemset(tzb, 0x35, 4 * 1024));
  auto rep = [&](const char *nm, float ms, double b) { printf("%-44s %8.1f us  %7.1f GB/s\n", nm, ms * 1e3, b / (ms * 1e-3) / 1e9); };

  auto ragged = [&](const char *tag, uint64_t count, const uint64_t *d_off, const uint32_t *d_len, uint32_t n, double b) {
    RsckArgs a{};
    a.base = buf; a.off = d_off; a.len = d_len; a.stride = n; a.count = count; a.fixed_len = n;
    a.out = out; a.tzb = tzb; a.group_cost = kRsGroupCost;
    for (int j = 0; j < 32; ++j) { a.XB[j] = 0x85EBCA6Bu * (j + 3); a.XB2[j] = 0x27D4EB2Fu * (j + 5); a.XB3[j] = 0x165667B1u * (j + 7); }
    for (int s = 0; s < 8; ++s) a.QS[s] = 0x9E3779B9u * (s + 1);
    void *ws; CK(hipMalloc(&ws, rs_workspace_bytes(count)));
    CK(rs_zero_counters(ws, 0));
    rs_bind_workspace(a, ws);
    const uint64_t want = (count + kPassBlock - 1) / kPassBlock;
    const int pgrid = (int)(want < kPassBlocks ? want : kPassBlocks);
    { a.nblk = (uint32_t)(pgrid); launch_bucket(a, (int)(pgrid), 0); }
    CK(hipDeviceSynchronize());
    char nm[128];
    for (int r = 0; r < 2; ++r) {
      snprintf(nm, sizeof nm, "%s rsck full", tag);
      rep(nm, timeit([&] { hipLaunchKernelGGL((icrc_rsck_kernel<0>), dim3(grid), dim3(kBlock), 0, 0, a); }, 10), b);
      snprintf(nm, sizeof nm, "%s rsck no finish", tag);
      rep(nm, timeit([&] { hipLaunchKernelGGL((icrc_rsck_kernel<2>), dim3(grid), dim3(kBlock), 0, 0, a); }, 10), b);
      snprintf(nm, sizeof nm, "%s rsck memory path", tag);
      rep(nm, timeit([&] { hipLaunchKernelGGL((icrc_rsck_kernel<3>), dim3(grid), dim3(kBlock), 0, 0, a); }, 10), b);
      snprintf(nm, sizeof nm, "%s rsck no edges", tag);
      rep(nm, timeit([&] { hipLaunchKernelGGL((icrc_rsck_kernel<8>), dim3(grid), dim3(kBlock), 0, 0, a); }, 10), b);
      snprintf(nm, sizeof nm, "%s rsck no stores", tag);
      rep(nm, timeit([&] { hipLaunchKernelGGL((icrc_rsck_kernel<16>), dim3(grid), dim3(kBlock), 0, 0, a); }, 10), b);
      snprintf(nm, sizeof nm, "%s rsck no finish, 192 slots", tag);
      rep(nm, timeit([&] { hipLaunchKernelGGL((icrc_rsck_kernel<2 | 512>), dim3(grid), dim3(kBlock), 0, 0, a); }, 10), b);
      snprintf(nm, sizeof nm, "%s rsck no finish, no global stores", tag);
      rep(nm, timeit([&] { hipLaunchKernelGGL((icrc_rsck_kernel<2 | 32>), dim3(grid), dim3(kBlock), 0, 0, a); }, 10), b);
      snprintf(nm, sizeof nm, "%s rsck no finish, nt stores", tag);
      rep(nm, timeit([&] { hipLaunchKernelGGL((icrc_rsck_kernel<2 | 1024>), dim3(grid), dim3(kBlock), 0, 0, a); }, 10), b);
      snprintf(nm, sizeof nm, "%s rsck no finish, default-policy stores", tag);
      rep(nm, timeit([&] { hipLaunchKernelGGL((icrc_rsck_kernel<2 | 2048>), dim3(grid), dim3(kBlock), 0, 0, a); }, 10), b);
      snprintf(nm, sizeof nm, "%s rsck no finish, sc0 sc1 stores", tag);
      rep(nm, timeit([&] { hipLaunchKernelGGL((icrc_rsck_kernel<2 | 4096>), dim3(grid), dim3(kBlock), 0, 0, a); }, 10), b);
      snprintf(nm, sizeof nm, "%s rsck no global stores", tag);
      rep(nm, timeit([&] { hipLaunchKernelGGL((icrc_rsck_kernel<32>), dim3(grid), dim3(kBlock), 0, 0, a); }, 10), b);
      snprintf(nm, sizeof nm, "%s rsck memory path, no edges, no stores", tag);
      rep(nm, timeit([&] { hipLaunchKernelGGL((icrc_rsck_kernel<3 | 8 | 16>), dim3(grid), dim3(kBlock), 0, 0, a); }, 10), b);
      if (!d_off) {
        snprintf(nm, sizeof nm, "%s rsck arith desc", tag);
        rep(nm, timeit([&] { hipLaunchKernelGGL((icrc_rsck_kernel<4>), dim3(grid), dim3(kBlock), 0, 0, a); }, 10), b);
        snprintf(nm, sizeof nm, "%s rsck arith desc, memory path", tag);
        rep(nm, timeit([&] { hipLaunchKernelGGL((icrc_rsck_kernel<7>), dim3(grid), dim3(kBlock), 0, 0, a); }, 10), b);
      }
      snprintf(nm, sizeof nm, "%s small kernel", tag);
      rep(nm, timeit([&] { hipLaunchKernelGGL((icrc_rsmall_kernel<kSmallRounds>), dim3(grid), dim3(kBlock), 0, 0, a); }, 10), b);
    }
    if (d_off) {  // the bench's order: passes, fold, small, gather per step; fold timed inside
      hipEvent_t f0, f1; CK(hipEventCreate(&f0)); CK(hipEventCreate(&f1));
      for (int r = 0; r < 2; ++r) {
        float tot = 0;
        for (int it = 0; it < 13; ++it) {
          // the counters (and the count pass's ticket) must start at zero: the
          // product's gather zeroes them, the variants above never ran it
          CK(rs_zero_counters(ws, 0));
          { a.nblk = (uint32_t)(pgrid); launch_bucket(a, (int)(pgrid), 0); }
          CK(hipEventRecord(f0, 0));
          hipLaunchKernelGGL((icrc_rsck_kernel<0>), dim3(grid), dim3(kBlock), 0, 0, a);
          CK(hipEventRecord(f1, 0));
          hipLaunchKernelGGL((icrc_rsmall_kernel<kSmallRounds>), dim3(grid), dim3(kBlock), 0, 0, a);
          hipLaunchKernelGGL(rsck_gather<kPassUnroll>, dim3(pgrid), dim3(kPassBlock), 0, 0, a);
          CK(hipEventSynchronize(f1));
          float ms; CK(hipEventElapsedTime(&ms, f0, f1));
          if (it >= 3) tot += ms;
        }
        snprintf(nm, sizeof nm, "%s rsck full, inside the bench's step sequence", tag);
        rep(nm, tot / 10, b);
      }
    }
    CK(hipFree(ws));
  };

  {  // out of the idle power state before timing anything
    SckArgs s{}; s.base = buf; s.count = bytes / 4096; s.out = out; s.n = 4096;
    for (int i = 0; i < 300; ++i) hipLaunchKernelGGL((icrc_sck_kernel<32, 0>), dim3(grid), dim3(kBlock), 0, 0, s);
    CK(hipDeviceSynchronize());
  }
  const bool mix_only = argc > 1 && argv[1][0] == 'm';  // "mix": the mixed batch only
  const bool u256_only = argc > 1 && argv[1][0] == 'u';  // "u256": uniform 256 B only
  const bool s1k = argc > 1 && argv[1][0] == 's';        // "s1k": uniform 1 KiB, full vs no global stores only (PMC)
  // uniform 4 KiB and 1 KiB, natural order (SCK reference on the same bytes)
  for (uint32_t n : {4096u, 1024u, 256u}) {
    if (mix_only) break;
    if (u256_only && n != 256) continue;
    if (s1k) {
      if (n != 1024) continue;
      RsckArgs a{};
      a.base = buf; a.stride = n; a.count = bytes / n; a.fixed_len = n; a.out = out; a.tzb = tzb; a.group_cost = kRsGroupCost;
      for (int j = 0; j < 32; ++j) { a.XB[j] = 0x85EBCA6Bu * (j + 3); a.XB2[j] = 0x27D4EB2Fu * (j + 5); a.XB3[j] = 0x165667B1u * (j + 7); }
      for (int k = 0; k < 8; ++k) a.QS[k] = 0x9E3779B9u * (k + 1);
      void *ws; CK(hipMalloc(&ws, rs_workspace_bytes(a.count)));
      CK(rs_zero_counters(ws, 0));
      rs_bind_workspace(a, ws);
      const uint64_t want = (a.count + kPassBlock - 1) / kPassBlock;
      { a.nblk = (uint32_t)((int)(want < kPassBlocks ? want : kPassBlocks)); launch_bucket(a, (int)((int)(want < kPassBlocks ? want : kPassBlocks)), 0); }
      CK(hipDeviceSynchronize());
      for (int r = 0; r < 3; ++r) {
        rep("1 KiB full", timeit([&] { hipLaunchKernelGGL((icrc_rsck_kernel<0>), dim3(grid), dim3(kBlock), 0, 0, a); }, 5), (double)bytes);
        rep("1 KiB no global stores", timeit([&] { hipLaunchKernelGGL((icrc_rsck_kernel<32>), dim3(grid), dim3(kBlock), 0, 0, a); }, 5), (double)bytes);
      }
      CK(hipFree(ws));
      return 0;
    }
    const uint64_t count = bytes / n;
    SckArgs s{}; s.base = buf; s.count = count; s.out = out; s.n = n;
    for (int j = 0; j < 32; ++j) s.XB[j] = 0x85EBCA6Bu * (j + 3);
    for (int k = 0; k < 8; ++k) s.QS[k] = 0x9E3779B9u * (k + 1);
    char tag[32]; snprintf(tag, sizeof tag, "%u B x %llu", n, (unsigned long long)count);
    char nm[128]; snprintf(nm, sizeof nm, "%s sck", tag);
    if (n == 256) {}
    else if (n == 4096) rep(nm, timeit([&] { hipLaunchKernelGGL((icrc_sck_kernel<32, 0>), dim3(grid), dim3(kBlock), 0, 0, s); }, 10), (double)bytes);
    else rep(nm, timeit([&] { hipLaunchKernelGGL((icrc_sck_kernel<8, 0>), dim3(grid), dim3(kBlock), 0, 0, s); }, 10), (double)bytes);
    ragged(tag, count, nullptr, nullptr, n, (double)bytes);
  }
  // C4 mix: 64/256/1024/4096 uniformly, packed, within the 4 GiB buffer
  if (!u256_only) {
    std::vector<uint64_t> off; std::vector<uint32_t> len;
    uint64_t x = 0x1234567ull, pos = 0, big = 0;
    const uint32_t sizes[4] = {64, 256, 1024, 4096};
    for (;;) {
      x ^= x << 13; x ^= x >> 7; x ^= x << 17;
      const uint32_t n = sizes[x & 3];
      if (pos + n > bytes) break;
      off.push_back(pos); len.push_back(n); pos += n; if (n >= 1024) big += n;
    }
    uint64_t *d_off; uint32_t *d_len;
    CK(hipMalloc(&d_off, 8 * off.size())); CK(hipMalloc(&d_len, 4 * len.size()));
    CK(hipMemcpy(d_off, off.data(), 8 * off.size(), hipMemcpyHostToDevice));
    CK(hipMemcpy(d_len, len.data(), 4 * len.size(), hipMemcpyHostToDevice));
    if (getenv("SYNTH")) {  // the bench's bytes: RoCEv2 headers from the P4 template, mix64 payload
      SynthArgs sa{}; sa.buf = buf; sa.seed = 0x5EED; sa.first = 0; sa.count = off.size(); sa.off = d_off; sa.len = d_len;
      CK(launch_synth_ragged(sa, 0)); CK(hipDeviceSynchronize());
      printf("(synthetic RoCEv2 packets)\n");
    }
    printf("mix: %zu packets, %llu B (%llu B in 1/4 KiB packets)\n", off.size(), (unsigned long long)pos, (unsigned long long)big);
    ragged("mix", off.size(), d_off, d_len, 0, (double)big);
  }
  return 0;
}
