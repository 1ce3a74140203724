// Ablation / variant timing of the strided-chain kernel (timing only: outputs
// are meaningless for ABL != 0).  Build:
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 sck_abl.hip -o sck_abl
#include "../../roce-test_amd/csrc/icrc_kernels.hip"
#include "../../roce-test_amd/csrc/icrc_sck.hip"
#include "mb_fin.h"
#include <stdio.h>
#include <stdlib.h>
using namespace ricrc;
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s\n", hipGetErrorString(e)); exit(1); } } while (0)
template <int L, int ABL, int PL = L> float run(SckArgs a, int grid, int reps) {
  hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  for (int w = 0; w < 3; ++w) hipLaunchKernelGGL((icrc_sck_kernel<L, ABL, kFamV4, PL>), dim3(grid), dim3(kBlock), 0, 0, a);
  CK(hipDeviceSynchronize()); CK(hipEventRecord(e0));
  for (int i = 0; i < reps; ++i) hipLaunchKernelGGL((icrc_sck_kernel<L, ABL, kFamV4, PL>), dim3(grid), dim3(kBlock), 0, 0, a);
  CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1)); float ms; CK(hipEventElapsedTime(&ms, e0, e1)); return ms / reps;
}
int main(int argc, char **argv) {
  const uint64_t n = 4096, count = 1 << 20;
  uint8_t *buf; uint32_t *out; CK(hipMalloc(&buf, n * count)); CK(hipMalloc(&out, 4 * (4ull << 20) + (1 << 22)));  // room for the L = 8 run (4 M packets) + ABL sink
  {  // random bytes (DVFS: constant data runs at a higher clock than real traffic)
    uint8_t *h = (uint8_t *)malloc(n * count);
    uint64_t x = 0x9E3779B97F4A7C15ull;
    for (uint64_t i = 0; i < n * count / 8; ++i) { x ^= x << 13; x ^= x >> 7; x ^= x << 17; ((uint64_t *)h)[i] = x; }
    CK(hipMemcpy(buf, h, n * count, hipMemcpyHostToDevice));
    free(h);
  }
  hipDeviceProp_t p; CK(hipGetDeviceProperties(&p, 0));
  SckArgs a{}; a.base = buf; a.count = count; a.out = out; a.n = n;
  a.fin = mb_fin();
  const int grid = p.multiProcessorCount;
  auto rep = [&](const char *nm, float ms) { printf("%-36s %7.3f ms  %7.1f GB/s\n", nm, ms, 4294967296.0 / (ms * 1e-3) / 1e9); };
  const bool quick = argc > 1 && argv[1][0] == 'x';  // "xt": finish-table variants only
  for (int r = 0; r < 2; ++r) {
    rep("full (one-copy finish tables)", run<32, 0>(a, grid, 20));
    rep("no loads", run<32, 8>(a, grid, 20));
    rep("memory path", run<32, 1 | 2>(a, grid, 20));
    if (quick) continue;
    rep("full D8", run<32, 0>(a, grid, 20));
    rep("no stores", run<32, 16>(a, grid, 20));
    rep("no fold (VALU stand-in)", run<32, 1>(a, grid, 20));
    rep("no finish", run<32, 2>(a, grid, 20));
    rep("no loads", run<32, 8>(a, grid, 20));
    rep("no fold, no finish (memory path)", run<32, 1 | 2>(a, grid, 20));
    rep("no loads, no finish (fold only)", run<32, 8 | 2>(a, grid, 20));
    rep("no loads, no fold (finish only)", run<32, 8 | 1>(a, grid, 20));
  }
  // 1 KiB packets (C2): L = 8, the ring spans exactly one group; 4 M and 1 M packets
  for (uint64_t cnt : {4ull << 20, 1ull << 20}) {
    SckArgs b = a; b.n = 1024; b.count = cnt;
    const double by = 1024.0 * cnt;
    auto rep8 = [&](const char *nm, float ms) { printf("%-36s %7.3f ms  %7.1f GB/s  (%llu x 1 KiB)\n", nm, ms, by / (ms * 1e-3) / 1e9, (unsigned long long)cnt); };
    for (int r = 0; r < 2; ++r) {
      rep8("L8 full", run<8, 0>(b, grid, 20));
      rep8("L8 no loads", run<8, 8>(b, grid, 20));
      rep8("L8 memory path", run<8, 1 | 2>(b, grid, 20));
      rep8("L32/PL8 super-groups full", run<32, 0, 8>(b, grid, 20));
      rep8("L32/PL8 super-groups no loads", run<32, 8, 8>(b, grid, 20));
      rep8("L32/PL8 super-groups memory path", run<32, 1 | 2, 8>(b, grid, 20));
      if (quick) continue;
      rep8("L8 full", run<8, 0>(b, grid, 20));
      rep8("L8 no finish", run<8, 2>(b, grid, 20));
      rep8("L8 no fold", run<8, 1>(b, grid, 20));
      rep8("L8 no loads", run<8, 8>(b, grid, 20));
    }
  }
  return 0;
}
