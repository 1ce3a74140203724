// Ablation timing of the TSK kernel (timing only: outputs are meaningless
// for ABL != 0).  Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 abl.hip -o abl
#include "../../roce-test_amd/csrc/icrc_kernels.hip"
#include <stdio.h>
#include <stdlib.h>
using namespace ricrc;
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s\n", hipGetErrorString(e)); exit(1); } } while (0)
template <int ABL> float run(TskArgs a, int grid, int reps) {
  hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  hipLaunchKernelGGL((icrc_tsk_kernel<true, ABL>), dim3(grid), dim3(kBlock), 0, 0, a);
  CK(hipDeviceSynchronize()); CK(hipEventRecord(e0));
  for (int i = 0; i < reps; ++i) hipLaunchKernelGGL((icrc_tsk_kernel<true, ABL>), dim3(grid), dim3(kBlock), 0, 0, a);
  CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1)); float ms; CK(hipEventElapsedTime(&ms, e0, e1)); return ms / reps;
}
int main() {
  const uint64_t n = 4096, count = 1 << 20;
  uint8_t *buf; uint32_t *out; CK(hipMalloc(&buf, n * count)); CK(hipMalloc(&out, 4 * count + (1 << 20)));
  {  // random bytes (DVFS: constant data runs at a higher clock than real traffic)
    uint8_t *h = (uint8_t *)malloc(n * count);
    uint64_t x = 0x9E3779B97F4A7C15ull;
    for (uint64_t i = 0; i < n * count / 8; ++i) { x ^= x << 13; x ^= x >> 7; x ^= x << 17; ((uint64_t *)h)[i] = x; }
    CK(hipMemcpy(buf, h, n * count, hipMemcpyHostToDevice));
    free(h);
  }
  hipDeviceProp_t p; CK(hipGetDeviceProperties(&p, 0));
  TskArgs a{}; a.base = buf; a.stride = n; a.count = count; a.out = out; a.n_iters = count * n / 4096; a.log2C = 7;
  for (int i = 0; i < 128; ++i) a.K[i] = 0x9E3779B9u * (i + 1);
  for (int j = 0; j < 32; ++j) a.YB[j] = 0x85EBCA6Bu * (j + 3);
  const int grid = p.multiProcessorCount;
  auto rep = [&](const char *nm, float ms) { printf("%-36s %7.3f ms  %7.1f GB/s\n", nm, ms, n * count / (ms * 1e-3) / 1e9); };
  for (int r = 0; r < 3; ++r) { char nm[64]; snprintf(nm, 64, "full #%d (x20)", r); rep(nm, run<0>(a, grid, 20)); }
  rep("exp: one store per wave", run<512>(a, grid, 20));
  rep("full", run<0>(a, grid, 20));
  rep("exp: one store per wave", run<512>(a, grid, 20));
  rep("full", run<0>(a, grid, 10));
  rep("no fold", run<1>(a, grid, 10));
  rep("no transpose", run<2>(a, grid, 10));
  rep("no combine", run<4>(a, grid, 10));
  rep("no loads", run<8>(a, grid, 10));
  rep("no loads, no transpose", run<8 | 2>(a, grid, 10));
  rep("no fold, no combine (mem+transpose)", run<1 | 4>(a, grid, 10));
  rep("no fold, no combine, no transpose", run<1 | 4 | 2>(a, grid, 10));
  rep("fold only (no loads/transpose/comb)", run<8 | 2 | 4>(a, grid, 10));
  rep("loads+fold (no transpose/comb)", run<2 | 4>(a, grid, 10));
  rep("no stores", run<16>(a, grid, 10));
  rep("exp: no drain at step", run<64>(a, grid, 10));
  rep("exp: s_sleep 1 at step", run<256>(a, grid, 10));
  rep("full again", run<0>(a, grid, 10));
  {
    const int nw = grid * kWaves;
    uint64_t *st; CK(hipMalloc(&st, 3 * 8 * nw)); a.stamps = st;
    rep("stamps (diag)", run<32>(a, grid, 3));
    rep("stamps no loads (diag)", run<32 | 8>(a, grid, 3));
    uint64_t *h = (uint64_t *)malloc(3 * 8 * nw);
    for (int v = 0; v < 2; ++v) {
      if (v == 0) run<32>(a, grid, 1); else run<32 | 8>(a, grid, 1);
      CK(hipMemcpy(h, st, 3 * 8 * nw, hipMemcpyDeviceToHost));
      double s0 = 0, s1 = 0, s2 = 0;
      for (int w = 0; w < nw; ++w) { s0 += h[3 * w]; s1 += h[3 * w + 1]; s2 += h[3 * w + 2]; }
      const double iters = (double)a.n_iters / nw;
      printf("%s per wave-iteration (ticks): staging+wait %.0f, fold+finish %.0f, total %.0f\n",
             v == 0 ? "full    " : "no loads", s0 / nw / iters, s1 / nw / iters, s2 / nw / iters);
    }
  }
  return 0;
}
