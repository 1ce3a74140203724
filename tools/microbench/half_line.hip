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
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s\n", hipGetErrorString(e)); exit(1); } } while (0)
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef const u32x4 __attribute__((address_space(1))) *gp_t;

template <int MODE>  // 0 all slots, 1 upper half only (masked), 2 lower half redirected to the upper half
__global__ __launch_bounds__(1024) void stream_kernel(const uint8_t *buf, uint64_t groups, uint32_t *sink) {
  const uint32_t lane = threadIdx.x & 63, s = lane & 7, g = lane >> 3;
  const uint64_t wave = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const uint64_t nw = ((uint64_t)gridDim.x * blockDim.x) >> 6;
  u32x4 acc = {0u, 0u, 0u, 0u};
  for (uint64_t q = wave; q < groups; q += nw) {
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
  const uint64_t bytes = 2ull << 30, groups = bytes / (8 * 4096);
  uint8_t *buf; CK(hipMalloc(&buf, bytes)); CK(hipMemset(buf, 0x3C, bytes));
  uint32_t *sink; CK(hipMalloc(&sink, 4096));
  const int grid = 256;
  for (int r = 0; r < 3; ++r) {
    const float a = timeit([&] { hipLaunchKernelGGL((stream_kernel<0>), dim3(grid), dim3(1024), 0, 0, buf, groups, sink); }, 10);
    const float b = timeit([&] { hipLaunchKernelGGL((stream_kernel<1>), dim3(grid), dim3(1024), 0, 0, buf, groups, sink); }, 10);
    const float c = timeit([&] { hipLaunchKernelGGL((stream_kernel<2>), dim3(grid), dim3(1024), 0, 0, buf, groups, sink); }, 10);
    printf("2 GiB of lines: all slots %.1f us (%.0f GB/s of lines) | upper half, masked %.1f us | lower half redirected %.1f us\n",
           a * 1e3, bytes / (a * 1e-3) / 1e9, b * 1e3, c * 1e3);
  }
  return 0;
}
