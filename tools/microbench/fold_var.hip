// The ragged fold (icrc_rsck_kernel) alone on a C4-shaped batch: 4 M packets, lengths uniform over 64/256/1024/4096 B,
// packed back to back (random bytes).  The passes run once; each variant's
// fold is timed (HIP events, 10 launches, 3 rounds).   hipcc --offload-arch=gfx950 -O3 -std=c++17 fold_var.hip -o fold_var
#include "../../roce-test_amd/csrc/icrc_kernels.hip"
#include "../../roce-test_amd/csrc/icrc_rsck.hip"
#include <stdio.h>
#include <stdlib.h>

#include <vector>
using namespace ricrc;
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s line %d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)

template <typename F> float timeit(F launch, int reps) {
  hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  for (int w = 0; w < 3; ++w) launch();
  CK(hipDeviceSynchronize()); CK(hipEventRecord(e0));
  for (int i = 0; i < reps; ++i) launch();
  CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1)); float ms; CK(hipEventElapsedTime(&ms, e0, e1));
  return ms / reps;
}

int main() {
  hipDeviceProp_t p; CK(hipGetDeviceProperties(&p, 0));
  const int grid = p.multiProcessorCount;
  const uint64_t count = 4ull << 20;
  std::vector<uint64_t> off(count);
  std::vector<uint32_t> len(count);
  uint64_t x = 0x1CEC0DEull, pos = 0;
  const uint32_t sizes[4] = {64, 256, 1024, 4096};
  for (uint64_t i = 0; i < count; ++i) {
    x ^= x << 13; x ^= x >> 7; x ^= x << 17;
    len[i] = sizes[(x >> 33) & 3];
    off[i] = pos;
    pos += len[i];
  }
  const uint64_t bytes = pos;
  uint8_t *buf; CK(hipMalloc(&buf, bytes + 4096));
  {
    std::vector<uint64_t> h((bytes + 7) / 8);
    for (auto &v : h) { x ^= x << 13; x ^= x >> 7; x ^= x << 17; v = x; }
    CK(hipMemcpy(buf, h.data(), bytes, hipMemcpyHostToDevice));
  }
  uint64_t *d_off; uint32_t *d_len, *out, *tzb;
  CK(hipMalloc(&d_off, 8 * count)); CK(hipMalloc(&d_len, 4 * count)); CK(hipMalloc(&out, 4 * count));
  CK(hipMemcpy(d_off, off.data(), 8 * count, hipMemcpyHostToDevice));
  CK(hipMemcpy(d_len, len.data(), 4 * count, hipMemcpyHostToDevice));
  CK(hipMalloc(&tzb, 4 * 1024)); CK(hipMemset(tzb, 0x35, 4 * 1024));
  RsckArgs a{};
  a.base = buf; a.off = d_off; a.len = d_len; a.count = count;
  a.out = out; a.tzb = tzb; a.group_cost = kRsGroupCost;
  for (int j = 0; j < 32; ++j) { a.XB[j] = 0x85EBCA6Bu * (j + 3); a.XB2[j] = 0x27D4EB2Fu * (j + 5); a.XB3[j] = 0x165667B1u * (j + 7); }
  for (int s = 0; s < 8; ++s) a.QS[s] = 0x9E3779B9u * (s + 1);
  void *ws; CK(hipMalloc(&ws, rs_workspace_bytes(count)));
  CK(rs_zero_counters(ws, 0));
  rs_bind_workspace(a, ws);
  const uint64_t want = (count + kPassBlock - 1) / kPassBlock;
  { a.nblk = (uint32_t)((int)(want < kPassBlocks ? want : kPassBlocks)); launch_bucket(a, (int)((int)(want < kPassBlocks ? want : kPassBlocks)), 0); }
  CK(hipDeviceSynchronize());
  const uint64_t npos = rs_npos(count);
  std::vector<uint32_t> ref(npos), got(npos);
  auto check = [&](const char *nm) {
    CK(hipDeviceSynchronize());
    CK(hipMemcpy(got.data(), a.res, 4 * npos, hipMemcpyDeviceToHost));
    uint64_t bad = 0;
    for (uint64_t i = 0; i < npos; ++i) bad += got[i] != ref[i];
    printf("  %-28s results %s (%llu differ)\n", nm, bad ? "DIFFER" : "match", (unsigned long long)bad);
  };
  // reference: the generic fold (the product)
  hipLaunchKernelGGL((icrc_rsck_kernel<0>), dim3(grid), dim3(kBlock), 0, 0, a);
  CK(hipDeviceSynchronize());
  CK(hipMemcpy(ref.data(), a.res, 4 * npos, hipMemcpyDeviceToHost));
  printf("%.2f GiB in %llu packets\n", bytes / 1073741824.0, (unsigned long long)count);
  CK(hipMemset(a.res, 0, 4 * npos));
  hipLaunchKernelGGL((icrc_rsck_kernel<131072>), dim3(grid), dim3(kBlock), 0, 0, a);
  check("specialized fold vs generic");
  // (Round-3 variants, measured on this harness and since removed from the
  // kernel: the round-2 fold 952-955 us; one-compare edge test 949-952;
  // + blocks of D quiet steps, D = 8 (spills) 945-949; D = 6 929-933 (kept);
  // a per-step quiet / full branch 1114-1120; D = 6 alone 954.)
  // Round 4: the fold specialized on the line count (ABL 131072) against the
  // generic fold (product), alternating, same process.  Session r4s2 (then
  // the specialized fold was the product): 921.5 / 918.5 us, 921.7 / 919.8.
  for (int r = 0; r < 1; ++r) {
    printf("fold generic (product)     %8.1f us\n", 1e3f * timeit([&] { hipLaunchKernelGGL((icrc_rsck_kernel<0>), dim3(grid), dim3(kBlock), 0, 0, a); }, 10));
    printf("fold specialized           %8.1f us\n", 1e3f * timeit([&] { hipLaunchKernelGGL((icrc_rsck_kernel<131072>), dim3(grid), dim3(kBlock), 0, 0, a); }, 10));
  }
  // What the result stores cost the fold (ABL 32: result slots kept, no
  // global stores; with the product's XCD weights), alternating.
  if (getenv("FOLD_STORES")) {
    for (int r = 0; r < 3; ++r) {  // round size: 64 vs 192 result slots per wave (both without the finish)
      RsckArgs k = a;
      for (int x = 0; x < 8; ++x) k.xw[x] = (x & 1) ? 960u : 1040u;
      const float v0 = 1e3f * timeit([&] { hipLaunchKernelGGL((icrc_rsck_kernel<2>), dim3(grid), dim3(kBlock), 0, 0, k); }, 10);
      const float v1 = 1e3f * timeit([&] { hipLaunchKernelGGL((icrc_rsck_kernel<2 | 512>), dim3(grid), dim3(kBlock), 0, 0, k); }, 10);
      const float v2 = 1e3f * timeit([&] { hipLaunchKernelGGL((icrc_rsck_kernel<2 | 32>), dim3(grid), dim3(kBlock), 0, 0, k); }, 10);
      printf("no finish, round %d: 64 slots (8 groups per store) %6.1f | 192 slots (24 groups) %6.1f | no global stores %6.1f us\n",
             r, v0, v1, v2);
    }
    for (int r = 0; r < 2; ++r) {
      RsckArgs k = a;
      for (int x = 0; x < 8; ++x) k.xw[x] = (x & 1) ? 960u : 1040u;
      const float t0 = 1e3f * timeit([&] { hipLaunchKernelGGL((icrc_rsck_kernel<0>), dim3(grid), dim3(kBlock), 0, 0, k); }, 10);
      const float t1 = 1e3f * timeit([&] { hipLaunchKernelGGL((icrc_rsck_kernel<32>), dim3(grid), dim3(kBlock), 0, 0, k); }, 10);
      const float t2 = 1e3f * timeit([&] { hipLaunchKernelGGL((icrc_rsck_kernel<3>), dim3(grid), dim3(kBlock), 0, 0, k); }, 10);
      const float t3 = 1e3f * timeit([&] { hipLaunchKernelGGL((icrc_rsck_kernel<35>), dim3(grid), dim3(kBlock), 0, 0, k); }, 10);
      printf("stores, round %d: product %6.1f | no global stores %6.1f | memory path %6.1f | memory path, no global stores %6.1f us\n",
             r, t0, t1, t2, t3);

    }
  }
  // Round 4: the product fold with its work split weighted by XCD parity
  // (a.xw by XCD parity, xcd_share), alternating.
  {
    const uint32_t W[][2] = {{0, 0}, {1000, 1000}, {1020, 980}, {1040, 960}, {1060, 940}, {1080, 920}};
    for (int r = 0; r < 3; ++r) {
      printf("xcd weights, round %d:", r);
      for (const auto &w : W) {
        RsckArgs k = a;
        for (int x = 0; x < 8; ++x) k.xw[x] = w[x & 1];
        printf(" | %u/%u %6.1f", w[0], w[1], 1e3f * timeit([&] { hipLaunchKernelGGL((icrc_rsck_kernel<0>), dim3(grid), dim3(kBlock), 0, 0, k); }, 10));
      }
      printf("\n");
    }
    // grids x weights (FOLD_GRIDS="224,240,256" in the environment)
    if (const char *gs = getenv("FOLD_GRIDS")) {
      std::vector<int> grids;
      for (const char *c = gs; *c;) {
        grids.push_back(atoi(c));
        while (*c && *c != ',') ++c;
        if (*c == ',') ++c;
      }
      const uint32_t S[] = {0, 20, 40, 60};
      for (int r = 0; r < 2; ++r)
        for (int gr : grids) {
          printf("grid %d, round %d:", gr, r);
          for (uint32_t d : S) {
            RsckArgs k = a;
            for (int x = 0; x < 8; ++x) k.xw[x] = d ? ((x & 1) ? 1000 - d : 1000 + d) : 0u;
            printf(" | skew %u %6.1f", d, 1e3f * timeit([&] { hipLaunchKernelGGL((icrc_rsck_kernel<0>), dim3(gr), dim3(kBlock), 0, 0, k); }, 10));
          }
          printf("\n");
        }
    }
    RsckArgs k = a;
    for (int x = 0; x < 8; ++x) k.xw[x] = (x & 1) ? 960u : 1040u;
    CK(hipMemset(a.res, 0, 4 * npos));
    hipLaunchKernelGGL((icrc_rsck_kernel<0>), dim3(grid), dim3(kBlock), 0, 0, k);
    check("fold 1040/960 vs 0/0");
  }
  return 0;
}
