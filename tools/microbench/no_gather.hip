// The "no gather" layout against the current fold (round 4, VERDICT r3 item
// 1(b)).  The product's fold leaves its results in class order (rounds of 64
// in 256-byte stores into the big pool's result slots) and the gather pass
// maps them back to packet order: out[i] = res[pos(i)].  The alternative
// writes every result straight to out[i] from the fold's finish, with the
// packet index carried next to the descriptor, and has no gather pass.  This
// prototype measures the fold's side of it on C4's batch (4 M packets of
// 64/256/1024/4096 B, back to back): the packet indexes of the big pool are
// built on the host from one bucket pass (pos_of and the pass blocks'
// ranges, inverted) and handed to the fold's ABL 262144 variant, which loads
// the next round's 64 indexes at each flush and stores each result at
// out[i] -- 4-byte stores scattered over the pass block's packets instead of
// 256-byte bursts.  Timed, alternating, with the counters restored before
// each step:
//   product    fold + gather (the gather's work on the small pool included)
//   no gather  fold with the scattered stores
// The small pool's results are left out of the second variant (its kernel
// would scatter them the same way), so the comparison favours it.  The
// scattered results are checked against the product's out[] for every big
// packet.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 no_gather.hip -o no_gather
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

  // the product's results (the whole pipeline; the gather zeroes the counters)
  CK(launch_rsck(a, grid, 0, 0, nullptr));
  CK(hipDeviceSynchronize());
  std::vector<uint32_t> ref(count);
  CK(hipMemcpy(ref.data(), out, 4 * count, hipMemcpyDeviceToHost));

  // one bucket pass; its counters kept for every step below
  launch_bucket(a, pgrid, 0);
  CK(hipDeviceSynchronize());
  RsCounters ctr; CK(hipMemcpy(&ctr, a.ctr, sizeof ctr, hipMemcpyDeviceToHost));
  RsCounters *ctr_saved; CK(hipMalloc(&ctr_saved, sizeof ctr));
  CK(hipMemcpy(ctr_saved, a.ctr, sizeof ctr, hipMemcpyDeviceToDevice));
  const uint32_t NG = (uint32_t)(ctr.pool & ((1ull << kRsGroupBits) - 1u));
  const uint64_t npos = 8ull * NG;
  std::vector<uint32_t> pos_of(count);
  std::vector<RsBlock> blk(pgrid);
  CK(hipMemcpy(pos_of.data(), a.pos_of, 4 * count, hipMemcpyDeviceToHost));
  CK(hipMemcpy(blk.data(), a.blk, sizeof(RsBlock) * pgrid, hipMemcpyDeviceToHost));
  // invert: big-pool position -> packet index (pass_range's blocks)
  const uint64_t per = ((count + pgrid - 1) / pgrid + kPassBlock - 1) / kPassBlock * kPassBlock;
  std::vector<uint32_t> ix(npos, 0xFFFFFFFFu);
  uint64_t nbig = 0, staged = 0;
  for (uint64_t i = 0; i < count; ++i) {
    const uint32_t q = pos_of[i];
    if (q == 0xFFFFFFFFu) continue;
    const RsBlock &B = blk[i / per];
    uint64_t bp;
    if (B.staged) {
      if (q < B.small) continue;
      bp = 8ull * B.g0 + (q - B.small);
    } else {
      if (q < a.small_cap) continue;
      bp = q - a.small_cap;
    }
    if (bp >= npos) { printf("position %llu outside the big pool\n", (unsigned long long)bp); return 1; }
    ix[bp] = (uint32_t)i;
    ++nbig;
  }
  for (const RsBlock &B : blk) staged += B.staged;
  // padding copies follow their class's last packet
  for (uint64_t j = 1; j < npos; ++j)
    if (ix[j] == 0xFFFFFFFFu) ix[j] = ix[j - 1];
  if (ix[0] == 0xFFFFFFFFu) { printf("big pool starts with a pad\n"); return 1; }
  CK(hipMalloc(&idx, 4 * npos));
  CK(hipMemcpy(idx, ix.data(), 4 * npos, hipMemcpyHostToDevice));
  printf("%llu packets, %.2f GiB; %u big groups, %llu big packets, small pool %u; %llu of %d pass blocks staged\n",
         (unsigned long long)count, bytes / 1073741824.0, NG, (unsigned long long)nbig, ctr.small,
         (unsigned long long)staged, pgrid);

  RsckArgs b = a;
  b.pos_of = idx;
  b.out = out2;
  auto restore = [&] { CK(hipMemcpyAsync(a.ctr, ctr_saved, sizeof ctr, hipMemcpyDeviceToDevice, 0)); };
  auto gather = [&] {
    if (pass_big(a, pgrid)) hipLaunchKernelGGL(rsck_gather<kPassUnrollBig>, dim3(pgrid), dim3(kPassBlock), 0, 0, a);
    else hipLaunchKernelGGL(rsck_gather<kPassUnroll>, dim3(pgrid), dim3(kPassBlock), 0, 0, a);
  };
  auto prod = [&] {
    restore();
    hipLaunchKernelGGL((icrc_rsck_kernel<0>), dim3(grid), dim3(kBlock), 0, 0, a);
    gather();
  };
  auto nog = [&] {
    restore();
    hipLaunchKernelGGL((icrc_rsck_kernel<262144>), dim3(grid), dim3(kBlock), 0, 0, b);
  };
  // check: every big packet's result from the scattered stores
  CK(hipMemset(out2, 0, 4 * count));
  nog();
  CK(hipDeviceSynchronize());
  {
    std::vector<uint32_t> got(count);
    CK(hipMemcpy(got.data(), out2, 4 * count, hipMemcpyDeviceToHost));
    uint64_t bad = 0;
    for (uint64_t j = 0; j < npos; ++j) bad += got[ix[j]] != ref[ix[j]];
    printf("no-gather fold vs product: %s (%llu of %llu big-pool positions differ)\n", bad ? "DIFFER" : "bit-exact",
           (unsigned long long)bad, (unsigned long long)npos);
    if (bad) return 1;
  }
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
  auto fold_only = [&] {
    restore();
    hipLaunchKernelGGL((icrc_rsck_kernel<0>), dim3(grid), dim3(kBlock), 0, 0, a);
  };
  for (int r = 0; r < 5; ++r)
    printf("round %d: product fold + gather %7.1f | no-gather fold %7.1f | product fold alone %7.1f us per step\n", r,
           timeit(prod), timeit(nog), timeit(fold_only));
  return 0;
}
