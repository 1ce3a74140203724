// Does a load that touches only half of each 128-byte line fetch half the
// bytes?  The ragged fold reads a packet's first and last line whole, even
// the 16-byte slots outside the packet (a line shared by two packets of
// different classes is then fetched by both).  Three kernels stream the same
// 2 GiB in the strided-chain pattern (lane 8g + s reads slot s of line k of
// packet g, 8 packets of 4 KiB per wave step, nt loads): all slots; only
// slots 4..7 (exec-masked loads); slots 0..3 redirected onto slot 4..7 of the
// same line.  Time per launch here; FETCH_SIZE per kernel under
// rocprofv3 --pmc FETCH_SIZE.  Build:
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 half_line.hip -o half_line
#include "../../roce-test_amd/csrc/icrc_kernels.hip"
#include "../../roce-test_amd/csrc/icrc_sck.hip"
#include <stdint.h>
#include "mb_fin.h"
#include <stdio.h>
#include <stdlib.h>
using namespace ricrc;

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s\n", hipGetErrorString(e)); exit(1); } } while (0)
typedef const u32x4 __attribute__((address_space(1))) *gp_t;

// MODE 0 all slots, 1 upper half only (masked), 2 lower half redirected to
// the upper half; group order (all slots): 0 group q = wave + i nw
// (interleaved), 3 a contiguous block of groups per wave (the SCK's order),
// 4 / 5 chunks of 8 / 2 consecutive groups interleaved over the waves.
template <int MODE>
__global__ __launch_bounds__(1024) void stream_kernel(const uint8_t *buf, uint64_t groups, uint32_t *sink) {
  const uint32_t lane = threadIdx.x & 63, s = lane & 7, g = lane >> 3;
  const uint64_t wave = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const uint64_t nw = ((uint64_t)gridDim.x * blockDim.x) >> 6;
  u32x4 acc = {0u, 0u, 0u, 0u};
  const uint64_t per = (groups + nw - 1) / nw;
  constexpr uint64_t CH = MODE == 4 ? 8 : MODE == 5 ? 2 : 1;
  for (uint64_t i = 0; i < per; ++i) {
    uint64_t q = MODE == 3 ? wave * per + i : ((i / CH) * nw + wave) * CH + i % CH;
    if (q >= groups) break;
    const uint8_t *pk = buf + (8 * q + g) * 4096;
#pragma unroll 8
    for (int k = 0; k < 32; ++k) {
      uint32_t slot = s;
      if (MODE == 2) slot = s | 4u;
      const uintptr_t addr = (uintptr_t)(pk + 128 * k + 16 * slot);
      if (MODE == 1) {
        if (s >= 4) acc ^= __builtin_nontemporal_load(reinterpret_cast<gp_t>(addr));
      } else {
        acc ^= __builtin_nontemporal_load(reinterpret_cast<gp_t>(addr));
      }
    }
  }
  const uint32_t v = acc[0] ^ acc[1] ^ acc[2] ^ acc[3];
  if (v == 0x9E3779B9u) sink[threadIdx.x] = v;
}

template <typename F> float timeit(F launch, int reps) {
  hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  for (int w = 0; w < 3; ++w) launch();
  CK(hipDeviceSynchronize()); CK(hipEventRecord(e0));
  for (int i = 0; i < reps; ++i) launch();
  CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1)); float ms; CK(hipEventElapsedTime(&ms, e0, e1));
  return ms / reps;
}

int main() {
  const uint64_t bytes = 4ull << 30, groups = bytes / (8 * 4096);
  uint8_t *buf; CK(hipMalloc(&buf, bytes));
  {  // random bytes (constant data runs at a higher clock than real traffic)
    uint64_t *h = (uint64_t *)malloc(bytes);
    uint64_t x = 0x9E3779B97F4A7C15ull;
    for (uint64_t i = 0; i < bytes / 8; ++i) { x ^= x << 13; x ^= x >> 7; x ^= x << 17; h[i] = x; }
    CK(hipMemcpy(buf, h, bytes, hipMemcpyHostToDevice));
    free(h);
  }
  uint32_t *out; CK(hipMalloc(&out, 4ull << 22));
  SckArgs sa{}; sa.base = buf; sa.count = bytes / 4096; sa.out = out; sa.n = 4096;
  sa.fin = mb_fin();
  uint32_t *sink; CK(hipMalloc(&sink, 4096));
  const int grid = 256;
  if (getenv("SIZE_SWEEP")) {  // SCK at 256 vs 240 workgroups by batch size (4 KiB packets), alternating
    uint8_t *big; CK(hipMalloc(&big, 16ull << 30));
    CK(hipMemset(big, 0x6B, 16ull << 30));
    for (uint64_t cnt : {1ull << 20, 3ull << 19, 2ull << 20, 3ull << 20, 4ull << 20}) {
      SckArgs b = sa; b.base = big; b.count = cnt;
      uint32_t *o2; CK(hipMalloc(&o2, 4 * cnt)); b.out = o2;
      printf("%llu x 4 KiB:", (unsigned long long)cnt);
      for (int r = 0; r < 3; ++r)
        for (int g : {256, 240}) {
          const float t = timeit([&] { hipLaunchKernelGGL((icrc_sck_kernel<32, 0>), dim3(g), dim3(kBlock), 0, 0, b); }, 10);
          printf(" %d:%.1f", g, t * 1e3);
        }
      printf(" us\n");
      CK(hipFree(o2));
    }
    return 0;
  }
  if (getenv("GRID_SWEEP")) {  // SCK grid sweep, alternating (one 1024-thread workgroup per CU used)
    SckArgs s2 = sa; s2.n = 1024; s2.count = 1 << 20;  // C2: 1 M x 1 KiB (super-groups)
    for (int r = 0; r < 3; ++r) {
      printf("SCK 4 KiB grid sweep round %d:", r);
      for (int g : {256, 252, 248, 244, 240, 236, 232, 228, 224, 216}) {
        const float t = timeit([&] { hipLaunchKernelGGL((icrc_sck_kernel<32, 0>), dim3(g), dim3(kBlock), 0, 0, sa); }, 20);
        printf(" %d:%.1f", g, t * 1e3);
      }
      printf(" us\n");
      printf("SCK 1 KiB (C2) grid sweep round %d:", r);
      for (int g : {256, 248, 240, 232, 224, 216, 208, 192}) {
        const float t = timeit([&] { hipLaunchKernelGGL((icrc_sck_kernel<32, 0, kFamV4, 8>), dim3(g), dim3(kBlock), 0, 0, s2); }, 20);
        printf(" %d:%.1f", g, t * 1e3);
      }
      printf(" us\n");
    }
    return 0;
  }
  for (int r = 0; r < 3; ++r) {
    const float a = timeit([&] { hipLaunchKernelGGL((stream_kernel<0>), dim3(grid), dim3(1024), 0, 0, buf, groups, sink); }, 10);
    const float b = timeit([&] { hipLaunchKernelGGL((stream_kernel<1>), dim3(grid), dim3(1024), 0, 0, buf, groups, sink); }, 10);
    const float c = timeit([&] { hipLaunchKernelGGL((stream_kernel<2>), dim3(grid), dim3(1024), 0, 0, buf, groups, sink); }, 10);
    printf("4 GiB of lines: all slots %.1f us (%.0f GB/s of lines) | upper half, masked %.1f us | lower half redirected %.1f us\n",
           a * 1e3, bytes / (a * 1e-3) / 1e9, b * 1e3, c * 1e3);
    const float d = timeit([&] { hipLaunchKernelGGL((stream_kernel<3>), dim3(grid), dim3(1024), 0, 0, buf, groups, sink); }, 10);
    const float e = timeit([&] { hipLaunchKernelGGL((stream_kernel<4>), dim3(grid), dim3(1024), 0, 0, buf, groups, sink); }, 10);
    const float f = timeit([&] { hipLaunchKernelGGL((stream_kernel<5>), dim3(grid), dim3(1024), 0, 0, buf, groups, sink); }, 10);
    printf("group order: interleaved %.1f us | contiguous block per wave (SCK) %.1f us (%.0f GB/s) | chunks of 8 %.1f us | chunks of 2 %.1f us\n",
           a * 1e3, d * 1e3, bytes / (d * 1e-3) / 1e9, e * 1e3, f * 1e3);
    const float sf = timeit([&] { hipLaunchKernelGGL((icrc_sck_kernel<32, 0>), dim3(grid), dim3(kBlock), 0, 0, sa); }, 10);
    const float sm = timeit([&] { hipLaunchKernelGGL((icrc_sck_kernel<32, 1 | 2>), dim3(grid), dim3(kBlock), 0, 0, sa); }, 10);
    const float sn = timeit([&] { hipLaunchKernelGGL((icrc_sck_kernel<32, 1 | 2 | 16>), dim3(grid), dim3(kBlock), 0, 0, sa); }, 10);
    printf("same bytes: SCK full %.1f us (%.0f GB/s) | SCK memory path (no fold, no finish) %.1f us | memory path, no stores %.1f us\n",
           sf * 1e3, bytes / (sf * 1e-3) / 1e9, sm * 1e3, sn * 1e3);
    const float st = timeit([&] { hipLaunchKernelGGL((icrc_sck_kernel<32, 1 | 2 | 16 | 128>), dim3(grid), dim3(kBlock), 0, 0, sa); }, 10);
    const float s8 = timeit([&] { hipLaunchKernelGGL((icrc_sck_kernel<32, 8>), dim3(grid), dim3(kBlock), 0, 0, sa); }, 10);
    const float s1 = timeit([&] { hipLaunchKernelGGL((icrc_sck_kernel<32, 1>), dim3(grid), dim3(kBlock), 0, 0, sa); }, 10);
    const float s2 = timeit([&] { hipLaunchKernelGGL((icrc_sck_kernel<32, 2>), dim3(grid), dim3(kBlock), 0, 0, sa); }, 10);
    printf("  SCK memory path, no stores, no table build %.1f us | no loads (compute only) %.1f us | no fold %.1f us | no finish %.1f us\n",
           st * 1e3, s8 * 1e3, s1 * 1e3, s2 * 1e3);
  }
  return 0;
}
