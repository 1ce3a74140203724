// The ragged pipeline's rate per packet-size class (round 4):
// the same pipeline (bucket -> fold -> one-line -> gather, launch_rsck with
// timing events between the passes) over ragged batches of ONE size each --
// 64, 256, 1024 and 4096 B, back to back -- and over C4's mix of the four, so
// the mix's fold time can be set against the sum of its classes' fold times
// at their own rates.  Algorithmic bytes: the packets' bytes + 16 per packet
// (offset, length, result), as bench.py counts them.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 class_rates.hip -o class_rates
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
  CK(hipEventDestroy(e0)); CK(hipEventDestroy(e1));
  return 1e3f * ms / reps;
}

struct Cfg {
  const char *name;
  std::vector<uint32_t> sizes;  // drawn uniformly per packet
  uint64_t count;
};

int main() {
  hipDeviceProp_t p; CK(hipGetDeviceProperties(&p, 0));
  const int grid = p.multiProcessorCount;
  const Cfg cfgs[] = {
      {"C4 mix 64/256/1024/4096", {64, 256, 1024, 4096}, 4ull << 20},
      {"64 B only", {64}, 1ull << 20},
      {"256 B only", {256}, 1ull << 20},
      {"1024 B only", {1024}, 1ull << 20},
      {"4096 B only", {4096}, 1ull << 20},
  };
  const uint64_t cap = 4ull << 20;
  const uint64_t cap_bytes = (4ull << 20) * 1360ull + (1ull << 20) * 4096ull;
  uint8_t *buf; CK(hipMalloc(&buf, cap_bytes + 4096));
  {
    std::vector<uint64_t> h(cap_bytes / 8);
    uint64_t x = 0x5EEDull;
    for (auto &v : h) { x ^= x << 13; x ^= x >> 7; x ^= x << 17; v = x; }
    CK(hipMemcpy(buf, h.data(), cap_bytes, hipMemcpyHostToDevice));
  }
  uint64_t *d_off; uint32_t *d_len, *out, *tzb;
  CK(hipMalloc(&d_off, 8 * cap)); CK(hipMalloc(&d_len, 4 * cap)); CK(hipMalloc(&out, 4 * cap));
  CK(hipMalloc(&tzb, 4 * 1024)); CK(hipMemset(tzb, 0x35, 4 * 1024));
  void *ws; CK(hipMalloc(&ws, rs_workspace_bytes(cap)));
  CK(rs_zero_counters(ws, 0));
  hipEvent_t ev[5];
  for (auto &evk : ev) CK(hipEventCreate(&evk));
  const char *pass[4] = {"bucket", "fold", "one-line", "gather"};
  for (const Cfg &c : cfgs) {
    std::vector<uint64_t> off(c.count);
    std::vector<uint32_t> len(c.count);
    uint64_t x = 0x1CEC0DEull, pos = 0, fold_bytes = 0;
    for (uint64_t i = 0; i < c.count; ++i) {
      x ^= x << 13; x ^= x >> 7; x ^= x << 17;
      len[i] = c.sizes[(x >> 33) % c.sizes.size()];
      off[i] = pos;
      pos += len[i];
      fold_bytes += len[i] > 64 ? len[i] : 0;  // 64-B packets at 64-B offsets span one line: the one-line kernel's
    }
    if (pos > cap_bytes) { printf("%s: %llu bytes exceed the buffer\n", c.name, (unsigned long long)pos); return 1; }
    CK(hipMemcpy(d_off, off.data(), 8 * c.count, hipMemcpyHostToDevice));
    CK(hipMemcpy(d_len, len.data(), 4 * c.count, hipMemcpyHostToDevice));
    RsckArgs a{};
    a.base = buf; a.off = d_off; a.len = d_len; a.count = c.count;
    a.out = out; a.tzb = tzb; a.group_cost = kRsGroupCost;
    for (int j = 0; j < 32; ++j) { a.XB[j] = 0x85EBCA6Bu * (j + 3); a.XB2[j] = 0x27D4EB2Fu * (j + 5); a.XB3[j] = 0x165667B1u * (j + 7); }
    for (int s = 0; s < 8; ++s) a.QS[s] = 0x9E3779B9u * (s + 1);
    rs_bind_workspace(a, ws);
    const double alg = (double)pos + 16.0 * (double)c.count;
    double sum[4] = {0, 0, 0, 0};
    const int warm = 5, reps = 20;
    for (int r = 0; r < warm + reps; ++r) {
      CK(launch_rsck(a, grid, 0, 0, ev));
      CK(hipEventSynchronize(ev[4]));
      if (r < warm) continue;
      for (int k = 0; k < 4; ++k) {
        float ms; CK(hipEventElapsedTime(&ms, ev[k], ev[k + 1]));
        sum[k] += 1e3 * ms / reps;
      }
    }
    const double tot = sum[0] + sum[1] + sum[2] + sum[3];
    printf("%-26s %8llu packets %6.3f GB | total %7.1f us %5.2f TB/s (%.3f of 8) |", c.name,
           (unsigned long long)c.count, pos / 1e9, tot, alg / tot / 1e6, alg / tot / 8e6);
    for (int k = 0; k < 4; ++k) printf(" %s %6.1f", pass[k], sum[k]);
    printf(" | fold %.2f TB/s of its packets' bytes\n", fold_bytes ? fold_bytes / sum[1] / 1e6 : 0.0);
    // The fold alone after one bucket pass (it leaves the counters as they
    // are; the gather would zero them), by variant: the product, the fold
    // specialized on the line count, the memory path (no table fold, no
    // finish), no finish, and the compute alone (no line loads).
    const uint64_t want = (c.count + kPassBlock - 1) / kPassBlock;
    a.nblk = (uint32_t)(want < kPassBlocks ? want : kPassBlocks);
    launch_bucket(a, (int)a.nblk, 0);
    CK(hipDeviceSynchronize());
    if (fold_bytes) {
      for (int r = 0; r < 2; ++r) {
        const float f0 = timeit([&] { hipLaunchKernelGGL((icrc_rsck_kernel<0>), dim3(grid), dim3(kBlock), 0, 0, a); }, 10);
        const float f1 = timeit([&] { hipLaunchKernelGGL((icrc_rsck_kernel<131072>), dim3(grid), dim3(kBlock), 0, 0, a); }, 10);
        const float f2 = timeit([&] { hipLaunchKernelGGL((icrc_rsck_kernel<3>), dim3(grid), dim3(kBlock), 0, 0, a); }, 10);
        const float f3 = timeit([&] { hipLaunchKernelGGL((icrc_rsck_kernel<2>), dim3(grid), dim3(kBlock), 0, 0, a); }, 10);
        const float f4 = timeit([&] { hipLaunchKernelGGL((icrc_rsck_kernel<16384>), dim3(grid), dim3(kBlock), 0, 0, a); }, 10);
        printf("    fold alone: product %6.1f | specialized %6.1f | memory path %6.1f | no finish %6.1f | "
               "compute, no loads %6.1f us\n", f0, f1, f2, f3, f4);
      }
    }
    // the one-line kernel alone by rounds batched per wave (R = 1: one
    // round at a time; the product runs kSmallRounds)
    if (fold_bytes != pos) {
      for (int r = 0; r < 3; ++r) {
        const float s1 = timeit([&] { hipLaunchKernelGGL((icrc_rsmall_kernel<1>), dim3(grid), dim3(kBlock), 0, 0, a); }, 10);
        const float s2 = timeit([&] { hipLaunchKernelGGL((icrc_rsmall_kernel<2>), dim3(grid), dim3(kBlock), 0, 0, a); }, 10);
        const float s4 = timeit([&] { hipLaunchKernelGGL((icrc_rsmall_kernel<4>), dim3(grid), dim3(kBlock), 0, 0, a); }, 10);
        printf("    one-line alone: R = 1 %6.1f | R = 2 %6.1f | R = 4 %6.1f us\n", s1, s2, s4);
      }
    }
    // the next configuration's bucket pass starts from zeroed counters
    CK(rs_zero_counters(ws, 0));
    CK(hipDeviceSynchronize());
  }
  return 0;
}
