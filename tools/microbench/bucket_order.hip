// The bucket pass's reservation order (round 4).  After its block scan, a
// pass block reserves its small and big ranges with two device-scope atomics
// (all 256 blocks on the same two counters).  Round 3 waited for them before
// building the block's LDS layout; the product now builds the layout while
// they are in flight and waits only before the final stores (rsck_bucket,
// ABL 64 = the round-3 order).  Each launch is timed alone (HIP events
// around it, the counter reset before the first event), alternating, on
// C4's batch (4 M packets of 64/256/1024/4096 B) and on its N = 8 shard
// (512 K packets).
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 bucket_order.hip -o bucket_order
#include "../../roce-test_amd/csrc/icrc_kernels.hip"
#include "../../roce-test_amd/csrc/icrc_rsck.hip"
#include <stdio.h>
#include <stdlib.h>

#include <vector>
using namespace ricrc;
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s line %d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)

int main() {
  const uint64_t cap = 4ull << 20;
  std::vector<uint64_t> off(cap);
  std::vector<uint32_t> len(cap);
  uint64_t x = 0x1CEC0DEull, pos = 0;
  const uint32_t sizes[4] = {64, 256, 1024, 4096};
  for (uint64_t i = 0; i < cap; ++i) {
    x ^= x << 13; x ^= x >> 7; x ^= x << 17;
    len[i] = sizes[(x >> 33) & 3];
    off[i] = pos;
    pos += len[i];
  }
  // the pass reads only descriptors: any base address will do (no packet bytes are read)
  uint8_t *buf; CK(hipMalloc(&buf, 4096));
  uint64_t *d_off; uint32_t *d_len;
  CK(hipMalloc(&d_off, 8 * cap)); CK(hipMalloc(&d_len, 4 * cap));
  CK(hipMemcpy(d_off, off.data(), 8 * cap, hipMemcpyHostToDevice));
  CK(hipMemcpy(d_len, len.data(), 4 * cap, hipMemcpyHostToDevice));
  void *ws; CK(hipMalloc(&ws, rs_workspace_bytes(cap)));
  hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  for (uint64_t count : {cap, cap / 8}) {
    RsckArgs a{};
    a.base = buf; a.off = d_off; a.len = d_len; a.count = count;
    a.group_cost = kRsGroupCost;
    rs_bind_workspace(a, ws);
    const uint64_t want = (count + kPassBlock - 1) / kPassBlock;
    const int pgrid = (int)(want < kPassBlocks ? want : kPassBlocks);
    a.nblk = (uint32_t)pgrid;
    if (pass_big(a, pgrid)) { printf("unexpected: 17 packets per thread\n"); return 1; }
    auto one = [&](auto abl) {
      constexpr int ABL = decltype(abl)::value;
      CK(rs_zero_counters(ws, 0));
      CK(hipEventRecord(e0, 0));
      hipLaunchKernelGGL((rsck_bucket<true, true, ABL, kPassUnroll>), dim3(pgrid), dim3(kPassBlock), 0, 0, a);
      CK(hipEventRecord(e1, 0));
      CK(hipEventSynchronize(e1));
      float ms; CK(hipEventElapsedTime(&ms, e0, e1));
      return 1e3f * ms;
    };
    auto avg = [&](auto abl) {
      for (int r = 0; r < 3; ++r) one(abl);
      float s = 0;
      for (int r = 0; r < 20; ++r) s += one(abl);
      return s / 20;
    };
    // both orders leave the same pools: compare the block records' sizes and the counters
    RsCounters c0, c1;
    one(std::integral_constant<int, 0>{});
    CK(hipMemcpy(&c0, a.ctr, sizeof c0, hipMemcpyDeviceToHost));
    one(std::integral_constant<int, 64>{});
    CK(hipMemcpy(&c1, a.ctr, sizeof c1, hipMemcpyDeviceToHost));
    printf("%llu packets on %d pass blocks: small %u / %u, pool %llx / %llx (%s)\n", (unsigned long long)count, pgrid,
           c0.small, c1.small, c0.pool, c1.pool, c0.small == c1.small && c0.pool == c1.pool ? "same" : "DIFFER");
    for (int r = 0; r < 5; ++r)
      printf("  round %d: product (layout while the reservation is in flight) %6.2f | round-3 order %6.2f us\n", r,
             avg(std::integral_constant<int, 0>{}), avg(std::integral_constant<int, 64>{}));
  }
  return 0;
}
