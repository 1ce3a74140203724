// The fold's line-load cache policy (round 4).  The fold (icrc_rsck_kernel)
// streams every line with non-temporal 16-byte loads.  A line that holds the
// end of one packet and the start of the next is fetched once per class
// (PMC: the fold's 4 % over-read); here the fold on C4's batch (one bucket
// pass, counters restored before each launch) with its line loads at the
// default policy (ABL 524288), and with only the packets' first and last
// lines at the default policy (ABL 1048576), against the product,
// alternating; results compared over the whole big pool.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 fold_policy.hip -o fold_policy
#include "../../roce-test_amd/csrc/icrc_kernels.hip"
#include "../../roce-test_amd/csrc/icrc_rsck.hip"
#include <stdio.h>
#include <stdlib.h>

#include <vector>
using namespace ricrc;
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s line %d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)

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
  uint64_t *d_off; uint32_t *d_len, *out, *out2, *tzb, *idx;
  CK(hipMalloc(&d_off, 8 * count)); CK(hipMalloc(&d_len, 4 * count));
  CK(hipMalloc(&out, 4 * count)); CK(hipMalloc(&out2, 4 * count));
  CK(hipMemcpy(d_off, off.data(), 8 * count, hipMemcpyHostToDevice));
  CK(hipMemcpy(d_len, len.data(), 4 * count, hipMemcpyHostToDevice));
  CK(hipMalloc(&tzb, 4 * 1024)); CK(hipMemset(tzb, 0x35, 4 * 1024));
  RsckArgs a{};
  a.base = buf; a.off = d_off; a.len = d_len; a.count = count;
  a.out = out; a.tzb = tzb; a.group_cost = kRsGroupCost;
  for (int k = 0; k < 8; ++k) a.xw[k] = (k & 1) ? 960u : 1040u;
  for (int j = 0; j < 32; ++j) { a.XB[j] = 0x85EBCA6Bu * (j + 3); a.XB2[j] = 0x27D4EB2Fu * (j + 5); a.XB3[j] = 0x165667B1u * (j + 7); }
  for (int s = 0; s < 8; ++s) a.QS[s] = 0x9E3779B9u * (s + 1);
  void *ws; CK(hipMalloc(&ws, rs_workspace_bytes(count)));
  CK(rs_zero_counters(ws, 0));
  rs_bind_workspace(a, ws);
  const uint64_t want = (count + kPassBlock - 1) / kPassBlock;
  const int pgrid = (int)(want < kPassBlocks ? want : kPassBlocks);
  a.nblk = (uint32_t)pgrid;

  // one bucket pass; its counters restored before every fold
  launch_bucket(a, pgrid, 0);
  CK(hipDeviceSynchronize());
  RsCounters ctr; CK(hipMemcpy(&ctr, a.ctr, sizeof ctr, hipMemcpyDeviceToHost));
  RsCounters *ctr_saved; CK(hipMalloc(&ctr_saved, sizeof ctr));
  CK(hipMemcpy(ctr_saved, a.ctr, sizeof ctr, hipMemcpyDeviceToDevice));
  const uint64_t npos = 8ull * (uint32_t)(ctr.pool & ((1ull << kRsGroupBits) - 1u));
  auto restore = [&] { CK(hipMemcpyAsync(a.ctr, ctr_saved, sizeof ctr, hipMemcpyDeviceToDevice, 0)); };
  auto fold = [&](auto abl) {
    constexpr int ABL = decltype(abl)::value;
    return [&, abl] {
      (void)abl;
      restore();
      hipLaunchKernelGGL((icrc_rsck_kernel<ABL>), dim3(grid), dim3(kBlock), 0, 0, a);
    };
  };
  auto f0 = fold(std::integral_constant<int, 0>{});
  auto f1 = fold(std::integral_constant<int, 524288>{});
  auto f2 = fold(std::integral_constant<int, 1048576>{});
  auto results = [&](auto f) {
    CK(hipMemset(a.bres, 0, 4 * npos));
    f();
    CK(hipDeviceSynchronize());
    std::vector<uint32_t> r(npos);
    CK(hipMemcpy(r.data(), a.bres, 4 * npos, hipMemcpyDeviceToHost));
    return r;
  };
  const std::vector<uint32_t> r0 = results(f0), r1 = results(f1), r2 = results(f2);
  printf("%llu packets, %.2f GiB, %llu big-pool positions: default-policy loads %s, edge lines only %s\n",
         (unsigned long long)count, bytes / 1073741824.0, (unsigned long long)npos, r1 == r0 ? "bit-exact" : "DIFFER",
         r2 == r0 ? "bit-exact" : "DIFFER");
  if (r1 != r0 || r2 != r0) return 1;
  hipEvent_t t0, t1; CK(hipEventCreate(&t0)); CK(hipEventCreate(&t1));
  auto timeit = [&](auto step) {
    for (int r = 0; r < 3; ++r) step();
    CK(hipDeviceSynchronize());
    CK(hipEventRecord(t0, 0));
    for (int r = 0; r < 10; ++r) step();
    CK(hipEventRecord(t1, 0));
    CK(hipEventSynchronize(t1));
    float ms; CK(hipEventElapsedTime(&ms, t0, t1));
    return 1e3f * ms / 10;
  };
  for (int r = 0; r < 5; ++r)
    printf("round %d: fold, nt line loads (product) %7.1f | default policy %7.1f | default on edge lines %7.1f us\n", r,
           timeit(f0), timeit(f1), timeit(f2));
  return 0;
}
