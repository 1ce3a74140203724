// Per-XCD weights of the strided-chain kernel's split beyond parity (round
// 4): with the start XCD recorded by the previous launch (as the product
// does), the headline batch (1 M x 4 KiB, 240 CUs) under equal shares, the
// product's parity weights (+-25 per mille) and parity weights that also
// spare XCD 0 (whose waves end after the other even XCDs', profiles/r04/
// s27_mb_xcd_slow.txt), alternating; then per-XCD mean wave ends (stamps).
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 sck_xw.hip -o sck_xw
#include "../../roce-test_amd/csrc/icrc_kernels.hip"
#include "../../roce-test_amd/csrc/icrc_sck.hip"
#include "mb_fin.h"
#include <stdio.h>
#include <stdlib.h>

#include <vector>
using namespace ricrc;
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s line %d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)

int main() {
  const uint64_t count = 1ull << 20, n = 4096, bytes = count * n;
  uint8_t *buf; uint32_t *out; uint64_t *stamps;
  CK(hipMalloc(&buf, bytes)); CK(hipMalloc(&out, 4 * count));
  {
    std::vector<uint64_t> h(bytes / 8);
    uint64_t x = 0x9E3779B97F4A7C15ull;
    for (auto &v : h) { x ^= x << 13; x ^= x >> 7; x ^= x << 17; v = x; }
    CK(hipMemcpy(buf, h.data(), bytes, hipMemcpyHostToDevice));
  }
  uint32_t *h_rec, *d_rec;
  CK(hipHostMalloc((void **)&h_rec, 64, hipHostMallocCoherent));
  *h_rec = 0;
  CK(hipHostGetDevicePointer((void **)&d_rec, h_rec, 0));
  const int grid = 240, waves = grid * kWaves;
  CK(hipMalloc(&stamps, 16ull * waves));
  SckArgs a{};
  a.base = buf; a.count = count; a.out = out; a.n = 4096; a.xcd_rec = d_rec;
  a.fin = mb_fin();
  const uint32_t W[][8] = {
      {0, 0, 0, 0, 0, 0, 0, 0},
      {1025, 975, 1025, 975, 1025, 975, 1025, 975},
      {1015, 970, 1030, 980, 1030, 980, 1030, 980},
      {1005, 965, 1035, 985, 1035, 985, 1035, 985},
      {1015, 960, 1030, 985, 1030, 985, 1030, 985},
  };
  const int nv = sizeof(W) / sizeof(W[0]);
  hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  auto launch = [&](int v, bool stamp) {
    SckArgs k = a;
    for (int x = 0; x < 8; ++x) k.xw[x] = W[v][x];
    k.xcd_k = __atomic_load_n(h_rec, __ATOMIC_RELAXED) & 7u;
    if (stamp) {
      k.stamps = stamps;
      hipLaunchKernelGGL((icrc_sck_kernel<32, 64>), dim3(grid), dim3(kBlock), 0, 0, k);
    } else {
      hipLaunchKernelGGL((icrc_sck_kernel<32, 0>), dim3(grid), dim3(kBlock), 0, 0, k);
    }
  };
  auto timeit = [&](int v) {
    for (int r = 0; r < 5; ++r) launch(v, false);
    CK(hipEventRecord(e0));
    for (int r = 0; r < 20; ++r) launch(v, false);
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms; CK(hipEventElapsedTime(&ms, e0, e1));
    return 1e3f * ms / 20;
  };
  for (int r = 0; r < 4; ++r) {
    printf("round %d (start XCD %u):", r, *h_rec & 7u);
    for (int v = 0; v < nv; ++v) printf(" | v%d %6.1f", v, timeit(v));
    printf(" us\n");
  }
  std::vector<uint64_t> st(2 * waves);
  for (int v = 0; v < nv; ++v) {
    for (int r = 0; r < 3; ++r) launch(v, true);
    CK(hipDeviceSynchronize());
    CK(hipMemcpy(st.data(), stamps, 16ull * waves, hipMemcpyDeviceToHost));
    const uint32_t k = *h_rec & 7u;
    uint64_t t0 = ~0ull, t1 = 0;
    for (int w = 0; w < waves; ++w) { t0 = std::min(t0, st[2 * w]); t1 = std::max(t1, st[2 * w + 1]); }
    double sum[8] = {0}; int c[8] = {0};
    for (int w = 0; w < waves; ++w) { const int x = (int)((w / kWaves + k) % 8); sum[x] += (st[2 * w + 1] - t0) / 100.0; ++c[x]; }
    printf("v%d (%u %u %u %u %u %u %u %u): span %.1f us, mean wave end by XCD:", v, W[v][0], W[v][1], W[v][2], W[v][3],
           W[v][4], W[v][5], W[v][6], W[v][7], (t1 - t0) / 100.0);
    for (int x = 0; x < 8; ++x) printf(" %.0f", sum[x] / c[x]);
    printf("\n");
  }
  return 0;
}
