// A stand-in for bench.py's N > 1 step: the strided-chain kernel of step j + 1
// on one stream while the results of step j are moved by another kernel on a
// second stream (RCCL's all-gather kernel at N = 8 moves 28 MB into each GPU,
// DESIGN.md §6).  The SCK keeps one 1024-thread workgroup per CU for its
// whole run (152 KiB of LDS), so a kernel on another stream finds no CU free
// until SCK workgroups finish -- and every SCK workgroup that starts late
// ends late by its full static share.  Measured: K steps back to back with
//   (a) no second kernel, (b) a copy kernel of B blocks after each step,
// with the SCK grid at 256 CUs or leaving R CUs to the copy.  Build:
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 overlap.hip -o overlap
#include "../../roce-test_amd/csrc/icrc_kernels.hip"
#include "../../roce-test_amd/csrc/icrc_sck.hip"
#include "mb_fin.h"
#include <stdio.h>
#include <stdlib.h>
using namespace ricrc;
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s\n", hipGetErrorString(e)); exit(1); } } while (0)

// The gather stand-in: copy n16 16-byte units (grid-stride), 256 threads per block.
__global__ __launch_bounds__(256) void copy_kernel(const u32x4 *src, u32x4 *dst, uint64_t n16) {
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n16; i += (uint64_t)gridDim.x * blockDim.x)
    dst[i] = src[i];
}

// The same copy holding 24 units per thread in flight (~100 VGPRs, like a
// collective kernel's): it cannot share a SIMD with the SCK's waves (the
// SCK leaves 64 VGPRs per SIMD lane free), so it waits for whole CUs.
__global__ __launch_bounds__(256) void copy_kernel_fat(const u32x4 *src, u32x4 *dst, uint64_t n16) {
  const uint64_t T = (uint64_t)gridDim.x * blockDim.x;
  for (uint64_t i0 = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i0 < n16; i0 += 24 * T) {
    u32x4 v[24];
#pragma unroll
    for (int k = 0; k < 24; ++k) v[k] = i0 + k * T < n16 ? __builtin_nontemporal_load(src + i0 + k * T) : u32x4{0u, 0u, 0u, 0u};
#pragma unroll
    for (int k = 0; k < 24; ++k)
      if (i0 + k * T < n16) dst[i0 + k * T] = v[k];
  }
}

int main() {
  const uint64_t count = 1 << 20, n = 4096, bytes = count * n;
  uint8_t *buf; CK(hipMalloc(&buf, bytes));
  {
    uint64_t *h = (uint64_t *)malloc(bytes);
    uint64_t x = 0x9E3779B97F4A7C15ull;
    for (uint64_t i = 0; i < bytes / 8; ++i) { x ^= x << 13; x ^= x >> 7; x ^= x << 17; h[i] = x; }
    CK(hipMemcpy(buf, h, bytes, hipMemcpyHostToDevice));
    free(h);
  }
  uint32_t *out; CK(hipMalloc(&out, 4 * count));
  const uint64_t gbytes = 28ull << 20;  // what one GPU receives of an 8-GPU all-gather of 4 MB shards
  u32x4 *gsrc, *gdst; CK(hipMalloc(&gsrc, gbytes)); CK(hipMalloc(&gdst, gbytes)); CK(hipMemset(gsrc, 1, gbytes));
  SckArgs sa{}; sa.base = buf; sa.count = count; sa.out = out; sa.n = 4096;
  sa.fin = mb_fin();
  hipStream_t sk, sg; CK(hipStreamCreateWithFlags(&sk, hipStreamNonBlocking)); CK(hipStreamCreateWithFlags(&sg, hipStreamNonBlocking));
  const int K = 20;
  hipEvent_t done[K], e0, e1;
  for (int i = 0; i < K; ++i) CK(hipEventCreateWithFlags(&done[i], hipEventDisableTiming));
  CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  auto run = [&](int grid, int cblocks, bool fat = false) -> float {
    for (int w = 0; w < 5; ++w) hipLaunchKernelGGL((icrc_sck_kernel<32, 0>), dim3(grid), dim3(kBlock), 0, sk, sa);
    CK(hipDeviceSynchronize());
    CK(hipEventRecord(e0, sk));
    for (int i = 0; i < K; ++i) {
      hipLaunchKernelGGL((icrc_sck_kernel<32, 0>), dim3(grid), dim3(kBlock), 0, sk, sa);
      if (cblocks) {
        CK(hipEventRecord(done[i], sk));
        CK(hipStreamWaitEvent(sg, done[i], 0));
        if (fat) hipLaunchKernelGGL(copy_kernel_fat, dim3(cblocks), dim3(256), 0, sg, gsrc, gdst, gbytes / 16);
        else hipLaunchKernelGGL(copy_kernel, dim3(cblocks), dim3(256), 0, sg, gsrc, gdst, gbytes / 16);
      }
    }
    CK(hipStreamWaitEvent(sk, done[K - 1], 0));
    if (cblocks) {  // the last copy too
      hipEvent_t g; CK(hipEventCreateWithFlags(&g, hipEventDisableTiming)); CK(hipEventRecord(g, sg)); CK(hipStreamWaitEvent(sk, g, 0));
    }
    CK(hipEventRecord(e1, sk)); CK(hipEventSynchronize(e1));
    float ms; CK(hipEventElapsedTime(&ms, e0, e1));
    return ms / K;
  };
  {  // the copy alone, by block count
    for (int cb : {8, 16, 32, 64}) {
      for (int w = 0; w < 3; ++w) hipLaunchKernelGGL(copy_kernel, dim3(cb), dim3(256), 0, sg, gsrc, gdst, gbytes / 16);
      CK(hipEventRecord(e0, sg));
      for (int i = 0; i < 10; ++i) hipLaunchKernelGGL(copy_kernel, dim3(cb), dim3(256), 0, sg, gsrc, gdst, gbytes / 16);
      CK(hipEventRecord(e1, sg)); CK(hipEventSynchronize(e1));
      float ms; CK(hipEventElapsedTime(&ms, e0, e1));
      printf("copy of 28 MiB alone, %2d blocks: %.1f us\n", cb, ms * 100.0f);
    }
  }
  for (int r = 0; r < 3; ++r) {
    printf("-- round %d: ms per step (SCK 1 M x 4 KiB; + a 28 MiB copy on a second stream after each step)\n", r);
    printf("grid 256, no copy %.4f | grid 256 + copy 32 blocks %.4f | grid 256 + copy 8 blocks %.4f\n",
           run(256, 0), run(256, 32), run(256, 8));
    printf("grid 248, no copy %.4f | grid 248 + copy 8 blocks %.4f | grid 240 + copy 16 blocks %.4f | grid 240, no copy %.4f\n",
           run(248, 0), run(248, 8), run(240, 16), run(240, 0));
    printf("fat copy (no SIMD sharing): grid 256 + 32 blocks %.4f | grid 256 + 8 blocks %.4f | grid 248 + 8 blocks %.4f | grid 240 + 16 blocks %.4f\n",
           run(256, 32, true), run(256, 8, true), run(248, 8, true), run(240, 16, true));
  }
  return 0;
}
