// Static vs dynamic (device-counter) group schedule of the strided-chain
// kernel, alone and with a concurrent "interference" kernel holding K CUs for
// ~T us (what RCCL's all-gather does when it overlaps the next step's kernel).
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 sck_dyn.hip -o sck_dyn
#include "../../roce-test_amd/csrc/icrc_kernels.hip"
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
using namespace ricrc;
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e)); exit(1); } } while (0)

__global__ void spin(uint64_t ticks) {  // one block per CU, holds it for `ticks` of the 100 MHz clock
  __shared__ uint32_t pad[16384];
  const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
  while (__builtin_amdgcn_s_memrealtime() - t0 < ticks) __builtin_amdgcn_s_sleep(8);
  if (threadIdx.x == 1024) pad[0] = 1;  // keep the LDS allocation
}

int main() {
  const uint64_t n = 4096, count = 1 << 20;
  uint8_t *buf; uint32_t *out0, *out1, *work;
  CK(hipMalloc(&buf, n * count)); CK(hipMalloc(&out0, 4 * count)); CK(hipMalloc(&out1, 4 * count));
  CK(hipMalloc(&work, 64)); CK(hipMemset(work, 0, 64));
  {
    uint8_t *h = (uint8_t *)malloc(n * count);
    uint64_t x = 0x9E3779B97F4A7C15ull;
    for (uint64_t i = 0; i < n * count / 8; ++i) { x ^= x << 13; x ^= x >> 7; x ^= x << 17; ((uint64_t *)h)[i] = x; }
    CK(hipMemcpy(buf, h, n * count, hipMemcpyHostToDevice));
    free(h);
  }
  hipDeviceProp_t p; CK(hipGetDeviceProperties(&p, 0));
  const int grid = p.multiProcessorCount;
  SckArgs a{}; a.base = buf; a.count = count; a.n = n; a.work = work;
  for (int j = 0; j < 32; ++j) a.XB[j] = 0x85EBCA6Bu * (j + 3);
  for (int s = 0; s < 8; ++s) a.QS[s] = 0x9E3779B9u * (s + 1);
  hipStream_t s1, s2; CK(hipStreamCreateWithFlags(&s1, hipStreamNonBlocking)); CK(hipStreamCreateWithFlags(&s2, hipStreamNonBlocking));
  hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  auto run = [&](bool dyn, int kcu, double spin_us, int reps, uint32_t *out) -> float {
    a.dynamic = dyn; a.out = out;
    float tot = 0;
    for (int r = 0; r < reps + 3; ++r) {
      if (kcu) hipLaunchKernelGGL(spin, dim3(kcu), dim3(256), 0, s2, (uint64_t)(spin_us * 100.0));
      CK(hipEventRecord(e0, s1));
      CK(launch_sck(a, grid, s1));
      CK(hipEventRecord(e1, s1));
      CK(hipDeviceSynchronize());
      float ms; CK(hipEventElapsedTime(&ms, e0, e1));
      if (r >= 3) tot += ms;
    }
    return tot / reps;
  };
  for (int rep = 0; rep < 2; ++rep) {
    printf("static  alone            %.4f ms\n", run(false, 0, 0, 20, out0));
    printf("dynamic alone            %.4f ms\n", run(true, 0, 0, 20, out1));
    printf("static  + 16 CUs 100 us  %.4f ms\n", run(false, 16, 100, 20, out0));
    printf("dynamic + 16 CUs 100 us  %.4f ms\n", run(true, 16, 100, 20, out1));
    printf("static  + 32 CUs 150 us  %.4f ms\n", run(false, 32, 150, 20, out0));
    printf("dynamic + 32 CUs 150 us  %.4f ms\n", run(true, 32, 150, 20, out1));
  }
  uint32_t *h0 = (uint32_t *)malloc(4 * count), *h1 = (uint32_t *)malloc(4 * count);
  CK(hipMemcpy(h0, out0, 4 * count, hipMemcpyDeviceToHost)); CK(hipMemcpy(h1, out1, 4 * count, hipMemcpyDeviceToHost));
  uint32_t w[2]; CK(hipMemcpy(w, work, 8, hipMemcpyDeviceToHost));
  printf("static == dynamic results: %s; counter after: %u %u\n", memcmp(h0, h1, 4 * count) == 0 ? "yes" : "NO", w[0], w[1]);
  return 0;
}
