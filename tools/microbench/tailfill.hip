// The one-line kernel in the fold's tail (round 4).  The fold's waves end
// between ~600 and ~930 us (profiles/r03/s17_bucket_abl.txt): in its last
// ~100 us CUs fall idle one by one.  Both kernels hold 128+ KiB of LDS, so
// one workgroup of either fits a CU: if the fold's 256 workgroups are
// dispatched first, the one-line kernel's workgroups can only take CUs the
// fold has released -- its work fills the tail instead of competing with the
// fold (round 4's side stream ran it beside the fold from the start on 1/16
// of the CUs: 1.050 vs 0.999 ms).  Variants on the C4-shaped batch, each
// timed from before the bucket pass to after the gather (HIP events on the
// main stream), alternating:
//   seq       the product: bucket, fold, one-line, gather on one stream
//   tail      fold on the main stream; the one-line kernel on a second
//             stream after the bucket pass's event; the gather waits for it
//   tail_pri  the same with the main stream at the highest priority and the
//             second at the lowest (the fold's workgroups dispatched first)
// Results are compared with seq's (bit-exact).
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 tailfill.hip -o tailfill
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
  uint64_t *d_off; uint32_t *d_len, *out, *tzb;
  CK(hipMalloc(&d_off, 8 * count)); CK(hipMalloc(&d_len, 4 * count)); CK(hipMalloc(&out, 4 * count));
  CK(hipMemcpy(d_off, off.data(), 8 * count, hipMemcpyHostToDevice));
  CK(hipMemcpy(d_len, len.data(), 4 * count, hipMemcpyHostToDevice));
  CK(hipMalloc(&tzb, 4 * 1024)); CK(hipMemset(tzb, 0x35, 4 * 1024));
  RsckArgs a{};
  a.base = buf; a.off = d_off; a.len = d_len; a.count = count;
  a.out = out; a.tzb = tzb; a.group_cost = kRsGroupCost; for (int x = 0; x < 8; ++x) a.xw[x] = (x & 1) ? 960u : 1040u;
  for (int j = 0; j < 32; ++j) { a.XB[j] = 0x85EBCA6Bu * (j + 3); a.XB2[j] = 0x27D4EB2Fu * (j + 5); a.XB3[j] = 0x165667B1u * (j + 7); }
  for (int s = 0; s < 8; ++s) a.QS[s] = 0x9E3779B9u * (s + 1);
  void *ws; CK(hipMalloc(&ws, rs_workspace_bytes(count)));
  CK(rs_zero_counters(ws, 0));
  rs_bind_workspace(a, ws);
  const uint64_t want = (count + kPassBlock - 1) / kPassBlock;
  const int pgrid = (int)(want < kPassBlocks ? want : kPassBlocks);
  a.nblk = (uint32_t)pgrid;

  int lo_pri = 0, hi_pri = 0;
  CK(hipDeviceGetStreamPriorityRange(&lo_pri, &hi_pri));
  hipStream_t mainst, side, main_hp, side_lp;
  CK(hipStreamCreateWithFlags(&mainst, hipStreamNonBlocking));
  CK(hipStreamCreateWithFlags(&side, hipStreamNonBlocking));
  CK(hipStreamCreateWithPriority(&main_hp, hipStreamNonBlocking, hi_pri));
  CK(hipStreamCreateWithPriority(&side_lp, hipStreamNonBlocking, lo_pri));
  hipEvent_t ev_b, ev_s, t0, t1;
  CK(hipEventCreateWithFlags(&ev_b, hipEventDisableTiming));
  CK(hipEventCreateWithFlags(&ev_s, hipEventDisableTiming));
  CK(hipEventCreate(&t0)); CK(hipEventCreate(&t1));

  auto gather = [&](hipStream_t st) {
    if (pass_big(a, pgrid)) hipLaunchKernelGGL(rsck_gather<kPassUnrollBig>, dim3(pgrid), dim3(kPassBlock), 0, st, a);
    else hipLaunchKernelGGL(rsck_gather<kPassUnroll>, dim3(pgrid), dim3(kPassBlock), 0, st, a);
  };
  auto step = [&](int v) {  // 0 seq, 1 tail, 2 tail_pri
    hipStream_t m = v == 2 ? main_hp : mainst, s = v == 2 ? side_lp : side;
    if (v == 0) {
      CK(launch_rsck(a, grid, 0, m, nullptr));
      return m;
    }
    launch_bucket(a, pgrid, m);
    CK(hipEventRecord(ev_b, m));
    hipLaunchKernelGGL((icrc_rsck_kernel<0>), dim3(grid), dim3(kBlock), 0, m, a);
    CK(hipStreamWaitEvent(s, ev_b, 0));
    hipLaunchKernelGGL((icrc_rsmall_kernel<kSmallRounds>), dim3(grid), dim3(kBlock), 0, s, a);
    CK(hipEventRecord(ev_s, s));
    CK(hipStreamWaitEvent(m, ev_s, 0));
    gather(m);
    return m;
  };
  auto timeit = [&](int v) {
    hipStream_t m = v == 2 ? main_hp : mainst;
    for (int r = 0; r < 3; ++r) step(v);
    CK(hipDeviceSynchronize());
    CK(hipEventRecord(t0, m));
    for (int r = 0; r < 10; ++r) step(v);
    CK(hipEventRecord(t1, m));
    CK(hipEventSynchronize(t1));
    CK(hipDeviceSynchronize());
    float ms; CK(hipEventElapsedTime(&ms, t0, t1));
    return 1e3f * ms / 10;
  };
  std::vector<uint32_t> ref(count), got(count);
  step(0);
  CK(hipDeviceSynchronize());
  CK(hipMemcpy(ref.data(), out, 4 * count, hipMemcpyDeviceToHost));
  for (int v = 1; v < 3; ++v) {
    CK(hipMemset(out, 0, 4 * count));
    step(v);
    CK(hipDeviceSynchronize());
    CK(hipMemcpy(got.data(), out, 4 * count, hipMemcpyDeviceToHost));
    uint64_t bad = 0;
    for (uint64_t i = 0; i < count; ++i) bad += got[i] != ref[i];
    printf("variant %d vs seq: %s (%llu differ)\n", v, bad ? "DIFFER" : "match", (unsigned long long)bad);
  }
  printf("%.2f GiB in %llu packets; stream priorities %d (least) .. %d (greatest)\n", bytes / 1073741824.0,
         (unsigned long long)count, lo_pri, hi_pri);
  for (int r = 0; r < 4; ++r)
    printf("round %d: seq %7.1f | tail %7.1f | tail_pri %7.1f us per step\n", r, timeit(0), timeit(1), timeit(2));
  return 0;
}
