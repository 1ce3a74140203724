// C4's per-process spread, inside one process: the ragged
// pipeline on FOUR copies of the same C4-shaped batch (4 M packets, 64/256/
// 1024/4096 B, back to back) in four separate 5.7 GB allocations, each with
// its own workspace, alternating copy by copy for several rounds -- and every
// batch with the first copy's workspace.  If a copy's time stays apart from
// the others' round after round, the physical placement of the batch (or of
// the workspace) is what differs between bench processes; if all copies read
// the same, placement is ruled out within a process.  Then (round 4, the
// microbench's fold read 911 us where bench.py's process read 925 by rocprof
// and 965-993 by its pass events): copy 1 regenerated with the product's
// synthetic RoCE packets (synth_ragged_kernel, bench.py's data) against the
// random bytes of copy 0, each timed with a host sync after every step (as
// above) and as 10 steps back to back (as bench.py runs them).
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 placement.hip -o placement
#include "../../roce-test_amd/csrc/icrc_kernels.hip"
#include "../../roce-test_amd/csrc/icrc_rsck.hip"
#include "mb_fin.h"
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
  constexpr int kCopies = 4;
  uint8_t *buf[kCopies];
  void *ws[kCopies];
  uint64_t *d_off; uint32_t *d_len, *out, *tzb;
  {
    std::vector<uint64_t> h((bytes + 7) / 8);
    for (auto &v : h) { x ^= x << 13; x ^= x >> 7; x ^= x << 17; v = x; }
    for (int c = 0; c < kCopies; ++c) {
      CK(hipMalloc(&buf[c], bytes + 4096));
      CK(hipMemcpy(buf[c], h.data(), bytes, hipMemcpyHostToDevice));
      CK(hipMalloc(&ws[c], rs_workspace_bytes(count)));
      CK(rs_zero_counters(ws[c], 0));
    }
  }
  CK(hipMalloc(&d_off, 8 * count)); CK(hipMalloc(&d_len, 4 * count)); CK(hipMalloc(&out, 4 * count));
  CK(hipMemcpy(d_off, off.data(), 8 * count, hipMemcpyHostToDevice));
  CK(hipMemcpy(d_len, len.data(), 4 * count, hipMemcpyHostToDevice));
  CK(hipMalloc(&tzb, 4 * 1024)); CK(hipMemset(tzb, 0x35, 4 * 1024));
  hipEvent_t ev[5];
  for (auto &evk : ev) CK(hipEventCreate(&evk));
  auto run = [&](int c, int w, int reps, double (&sum)[4]) {
    RsckArgs a{};
    a.base = buf[c]; a.off = d_off; a.len = d_len; a.count = count;
    a.out = out; a.tzb = tzb; a.group_cost = kRsGroupCost;
    a.fin = mb_fin();
    rs_bind_workspace(a, ws[w]);
    for (int k = 0; k < 4; ++k) sum[k] = 0;
    for (int r = 0; r < 3 + reps; ++r) {
      CK(launch_rsck(a, grid, 0, 0, ev));
      CK(hipEventSynchronize(ev[4]));
      if (r < 3) continue;
      for (int k = 0; k < 4; ++k) {
        float ms; CK(hipEventElapsedTime(&ms, ev[k], ev[k + 1]));
        sum[k] += 1e3 * ms / reps;
      }
    }
  };
  printf("%.2f GiB in %llu packets, %d copies (batch at %p %p %p %p)\n", bytes / 1073741824.0,
         (unsigned long long)count, kCopies, (void *)buf[0], (void *)buf[1], (void *)buf[2], (void *)buf[3]);
  for (int round = 0; round < 4; ++round) {
    for (int c = 0; c < kCopies; ++c) {
      double own[4], first[4];
      run(c, c, 10, own);
      run(c, 0, 10, first);
      printf("round %d copy %d: own workspace: bucket %5.1f fold %6.1f one-line %5.1f gather %5.1f | "
             "copy 0's workspace: bucket %5.1f fold %6.1f one-line %5.1f gather %5.1f us\n",
             round, c, own[0], own[1], own[2], own[3], first[0], first[1], first[2], first[3]);
    }
  }
  // Data and cadence.
  {
    SynthArgs sa{};
    sa.buf = buf[1]; sa.seed = 0x1CEC0DEull; sa.first = 0; sa.count = count; sa.off = d_off; sa.len = d_len;
    CK(launch_synth_ragged(sa, 0));
    CK(hipDeviceSynchronize());
  }
  constexpr int kB2B = 10;
  std::vector<hipEvent_t> bev(5 * kB2B);
  for (auto &evk : bev) CK(hipEventCreate(&evk));
  auto b2b = [&](int c, double (&sum)[4]) {
    RsckArgs a{};
    a.base = buf[c]; a.off = d_off; a.len = d_len; a.count = count;
    a.out = out; a.tzb = tzb; a.group_cost = kRsGroupCost;
    a.fin = mb_fin();
    rs_bind_workspace(a, ws[c]);
    for (int r = 0; r < 3; ++r) CK(launch_rsck(a, grid, 0, 0, nullptr));  // warm, back to back
    for (int i = 0; i < kB2B; ++i) CK(launch_rsck(a, grid, 0, 0, &bev[5 * i]));
    CK(hipDeviceSynchronize());
    for (int k = 0; k < 4; ++k) sum[k] = 0;
    for (int i = 0; i < kB2B; ++i)
      for (int k = 0; k < 4; ++k) {
        float ms; CK(hipEventElapsedTime(&ms, bev[5 * i + k], bev[5 * i + k + 1]));
        sum[k] += 1e3 * ms / kB2B;
      }
  };
  for (int round = 0; round < 3; ++round) {
    for (int c = 0; c < 2; ++c) {
      double sy[4], bb[4];
      run(c, c, 10, sy);
      b2b(c, bb);
      printf("round %d %-22s synced: bucket %5.1f fold %6.1f one-line %5.1f gather %5.1f | back to back: bucket %5.1f "
             "fold %6.1f one-line %5.1f gather %5.1f us\n", round, c ? "synthetic RoCE packets" : "random bytes",
             sy[0], sy[1], sy[2], sy[3], bb[0], bb[1], bb[2], bb[3]);
    }
  }
  return 0;
}
