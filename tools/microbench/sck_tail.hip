// Per-wave start / end times of the strided-chain kernel (ABL = 64 stamps,
// s_memrealtime at 100 MHz) over a 1 M x 4 KiB and a 1 M x 1 KiB batch:
// how much of a launch is the tail (waves done early waiting for the last).
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 sck_tail.hip -o sck_tail
#include "../../roce-test_amd/csrc/icrc_kernels.hip"
#include "../../roce-test_amd/csrc/icrc_sck.hip"
#include "mb_fin.h"
#include <stdio.h>
#include <stdlib.h>

#include <algorithm>
#include <vector>
using namespace ricrc;
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s\n", hipGetErrorString(e)); exit(1); } } while (0)

template <int L>
void run(uint8_t *buf, uint32_t *out, uint64_t count, int grid) {
  SckArgs a{};
  a.base = buf; a.count = count; a.out = out; a.n = 128 * L;
  a.fin = mb_fin();
  const int waves = grid * kWaves;
  CK(hipMalloc(&a.stamps, 16ull * waves));
  hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  for (int r = 0; r < 10; ++r) hipLaunchKernelGGL((icrc_sck_kernel<L, 64>), dim3(grid), dim3(kBlock), 0, 0, a);
  CK(hipEventRecord(e0));
  for (int r = 0; r < 20; ++r) hipLaunchKernelGGL((icrc_sck_kernel<L, 64>), dim3(grid), dim3(kBlock), 0, 0, a);
  CK(hipEventRecord(e1));
  CK(hipDeviceSynchronize());
  float ms; CK(hipEventElapsedTime(&ms, e0, e1));
  printf("%s L=%d count=%llu: %.1f us per launch (HIP events, 20 launches)\n", "STATIC ", L,
         (unsigned long long)count, ms * 1000.f / 20);
  std::vector<uint64_t> st(2 * waves);
  CK(hipMemcpy(st.data(), a.stamps, 16ull * waves, hipMemcpyDeviceToHost));
  uint64_t t0 = ~0ull, t1 = 0;
  std::vector<double> ends, starts;
  for (int w = 0; w < waves; ++w) { t0 = std::min(t0, st[2 * w]); t1 = std::max(t1, st[2 * w + 1]); }
  for (int w = 0; w < waves; ++w) { starts.push_back((st[2 * w] - t0) / 100.0); ends.push_back((st[2 * w + 1] - t0) / 100.0); }
  std::sort(ends.begin(), ends.end());
  std::sort(starts.begin(), starts.end());
  auto q = [&](std::vector<double> &v, double f) { return v[std::min(v.size() - 1, (size_t)(f * v.size()))]; };
  printf("  L=%d count=%llu: span %.1f us; wave start p50 %.1f p99 %.1f max %.1f us; wave end min %.1f p10 %.1f p50 %.1f p90 %.1f max %.1f us\n",
         L, (unsigned long long)count, (t1 - t0) / 100.0, q(starts, 0.5), q(starts, 0.99), starts.back(),
         ends.front(), q(ends, 0.1), q(ends, 0.5), q(ends, 0.9), ends.back());
  // per XCD (workgroup w -> XCD w % 8)
  for (int x = 0; x < 8; ++x) {
    double mx = 0, mn = 1e30;
    for (int w = 0; w < waves; ++w) if ((w / kWaves) % 8 == x) { double e = (st[2 * w + 1] - t0) / 100.0; mx = std::max(mx, e); mn = std::min(mn, e); }
    printf("    xcd %d: end min %.1f max %.1f us\n", x, mn, mx);
  }
  CK(hipFree(a.stamps));
}

int main() {
  const uint64_t bytes = 4ull << 30;
  uint8_t *buf; uint32_t *out;
  CK(hipMalloc(&buf, bytes)); CK(hipMalloc(&out, 4ull << 22));
  {  // random bytes (DVFS: constant data runs at a higher clock than real traffic)
    uint8_t *h = (uint8_t *)malloc(bytes);
    uint64_t x = 0x9E3779B97F4A7C15ull;
    for (uint64_t i = 0; i < bytes / 8; ++i) { x ^= x << 13; x ^= x >> 7; x ^= x << 17; ((uint64_t *)h)[i] = x; }
    CK(hipMemcpy(buf, h, bytes, hipMemcpyHostToDevice));
    free(h);
  }
  hipDeviceProp_t p; CK(hipGetDeviceProperties(&p, 0));
  for (int r = 0; r < 2; ++r) {
    run<32>(buf, out, 1ull << 20, p.multiProcessorCount);
    run<8>(buf, out, 1ull << 20, p.multiProcessorCount);
  }
  return 0;
}
