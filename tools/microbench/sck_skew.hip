// XCD-weighted work split of the strided-chain kernel (round 4).  Every
// per-wave timeline of rounds 2-3 shows the waves of odd-indexed workgroups
// (XCDs 1, 3, 5, 7: workgroup b runs on XCD b % 8) ending 5-9 % after those
// of even ones with equal work (profiles/r02/sck_tail.txt: even XCDs by
// 574-578 us, odd by 627-637 us; the ragged fold's "mean end by blockIdx % 8"
// lines of profiles/r03/s17_bucket_abl.txt).  Here the headline batch (1 M x
// 4 KiB, random bytes, the product's 240-CU grid) runs with the waves of
// even workgroups taking W[0] parts of the groups and odd ones W[1] (xw),
// alternating over several rounds, and with per-wave stamps per XCD.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 sck_skew.hip -o sck_skew
#include "../../roce-test_amd/csrc/icrc_kernels.hip"
#include "../../roce-test_amd/csrc/icrc_sck.hip"
#include "mb_fin.h"
#include <stdio.h>
#include <stdlib.h>

#include <algorithm>
#include <array>
#include <string.h>
#include <vector>
using namespace ricrc;
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s line %d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)

int main(int argc, char **argv) {
  const int L = argc > 1 ? atoi(argv[1]) : 32;  // 32: 4 KiB packets; 8: 1 KiB (super-groups)
  const uint64_t count = argc > 3 ? strtoull(argv[3], nullptr, 0) : 1ull << 20;  // C3: 4194304
  const uint64_t n = L == 32 ? 4096 : 1024;
  const uint64_t bytes = count * n;
  uint8_t *buf; uint32_t *out; uint64_t *stamps;
  CK(hipMalloc(&buf, bytes)); CK(hipMalloc(&out, 4 * count));
  {
    std::vector<uint64_t> h(bytes / 8);
    uint64_t x = 0x9E3779B97F4A7C15ull;
    for (auto &v : h) { x ^= x << 13; x ^= x >> 7; x ^= x << 17; v = x; }
    CK(hipMemcpy(buf, h.data(), bytes, hipMemcpyHostToDevice));
  }
  hipDeviceProp_t p; CK(hipGetDeviceProperties(&p, 0));
  // the product's grid for 1 M packets, or argv[2]
  const int grid = argc > 2 ? atoi(argv[2]) : p.multiProcessorCount - p.multiProcessorCount / 16;
  const int waves = grid * kWaves;
  CK(hipMalloc(&stamps, 16ull * waves));
  SckArgs a{};
  a.base = buf; a.count = count; a.out = out; a.n = (uint32_t)n;
  a.fin = mb_fin();
  hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  auto launch = [&](const SckArgs &k, bool stamp) {
    if (L == 32) {
      if (stamp) hipLaunchKernelGGL((icrc_sck_kernel<32, 64>), dim3(grid), dim3(kBlock), 0, 0, k);
      else hipLaunchKernelGGL((icrc_sck_kernel<32, 0>), dim3(grid), dim3(kBlock), 0, 0, k);
    } else {
      if (stamp) hipLaunchKernelGGL((icrc_sck_kernel<32, 64, kFamV4, 8>), dim3(grid), dim3(kBlock), 0, 0, k);
      else hipLaunchKernelGGL((icrc_sck_kernel<32, 0, kFamV4, 8>), dim3(grid), dim3(kBlock), 0, 0, k);
    }
  };
  auto timeit = [&](const SckArgs &k) {
    for (int r = 0; r < 5; ++r) launch(k, false);
    CK(hipEventRecord(e0));
    for (int r = 0; r < 20; ++r) launch(k, false);
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms; CK(hipEventElapsedTime(&ms, e0, e1));
    return 1e3f * ms / 20;
  };
  // (session r4s13: 0/0 632.5-633.1, 1000/1000 629.0-629.6, 1030/970
  // 618.6-621.1, 1050/950 625.6-626.3, 1070/930 635, 1100/900 642, 970/1030
  // 640-641 us on 4 KiB packets)
  // (session r4s14, 240 CUs: 0/0 630-631, 1000/1000 628.5-629, 1010/990
  // 624-625, 1020/980 620-621, 1030/970 619-621, 1040/960 625-627, 1050/950
  // 628-629; 256 CUs: 0/0 645-647, 1030/970 636-640, 1050/950 622-625 us)
  const uint32_t W240[][2] = {{0, 0}, {1000, 1000}, {1015, 985}, {1020, 980}, {1025, 975}, {1030, 970}, {1035, 965}};
  const uint32_t W256[][2] = {{0, 0}, {1000, 1000}, {1040, 960}, {1050, 950}, {1060, 940}, {1070, 930}, {1080, 920}};
  std::vector<std::array<uint32_t, 2>> W;
  if (argc > 4) {  // per-mille skews, comma-separated ("0" = the equal ceil split)
    for (char *t = strtok(argv[4], ","); t; t = strtok(nullptr, ",")) {
      const uint32_t d = (uint32_t)atoi(t);
      W.push_back(d ? std::array<uint32_t, 2>{1000 + d, 1000 - d} : std::array<uint32_t, 2>{0, 0});
    }
  } else {
    for (const auto &w : (grid >= p.multiProcessorCount ? W256 : W240)) W.push_back({w[0], w[1]});
  }
  const int nv = (int)W.size();
  printf("%llu x %llu B, grid %d; us per launch (HIP events, 20 launches), variants alternating\n",
         (unsigned long long)count, (unsigned long long)n, grid);
  for (int r = 0; r < 3; ++r) {
    printf("round %d:", r);
    for (int v = 0; v < nv; ++v) {
      SckArgs k = a;
      for (int x = 0; x < 8; ++x) k.xw[x] = W[v][0] ? W[v][x & 1] : 0u;
      printf(" | %u/%u %6.1f", W[v][0], W[v][1], timeit(k));
    }
    printf("\n");
  }
  // per-XCD wave ends for three of them
  for (int v : {0, std::min(4, nv - 1)}) {  // the first and the fifth variant
    SckArgs k = a;
    for (int x = 0; x < 8; ++x) k.xw[x] = W[v][0] ? W[v][x & 1] : 0u; k.stamps = stamps;
    for (int r = 0; r < 5; ++r) launch(k, true);
    CK(hipDeviceSynchronize());
    std::vector<uint64_t> st(2 * waves);
    CK(hipMemcpy(st.data(), stamps, 16ull * waves, hipMemcpyDeviceToHost));
    uint64_t t0 = ~0ull, t1 = 0;
    for (int w = 0; w < waves; ++w) { t0 = std::min(t0, st[2 * w]); t1 = std::max(t1, st[2 * w + 1]); }
    printf("%u/%u: span %.1f us; per XCD mean / max wave end:", W[v][0], W[v][1], (t1 - t0) / 100.0);
    for (int xcd = 0; xcd < 8; ++xcd) {
      double sum = 0, mx = 0; int c = 0;
      for (int w = 0; w < waves; ++w)
        if ((w / kWaves) % 8 == xcd) { const double e = (st[2 * w + 1] - t0) / 100.0; sum += e; mx = std::max(mx, e); ++c; }
      printf(" %d: %.0f/%.0f", xcd, sum / c, mx);
    }
    printf("\n");
  }
  return 0;
}
