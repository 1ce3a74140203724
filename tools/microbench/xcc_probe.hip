// Which XCD does workgroup b of a launch run on?  (round 4: the XCD-parity
// weighted split assumes "block b on XCD (b + k) % 8" with k even.)  Every
// workgroup records s_getreg(HW_REG_XCC_ID); per launch we print k = the XCD
// of block 0 and how many blocks break "XCD = (b + k) % 8".  The probe
// kernels hold 128 KiB of LDS and 1024 threads (one per CU, like the ICRC
// kernels).  Scenarios, in one process:
//   A  ten launches of 240 workgroups back to back (the headline SCK's grid)
//   B  241-, then 256-workgroup launches, five times (bucket pass -> fold)
//   C  256-workgroup launches while a second stream launches 7-workgroup
//      kernels (a stand-in for RCCL's kernels at N > 1)
//   D  a 240-workgroup launch after a host sync and a 1 ms sleep, ten times
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 xcc_probe.hip -o xcc_probe
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <unistd.h>

#include <vector>
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s line %d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)

__global__ __launch_bounds__(1024) void probe(uint32_t *out, uint32_t spin) {
  __shared__ uint32_t lds[32768];  // 128 KiB: one workgroup per CU
  lds[threadIdx.x] = threadIdx.x;
  __syncthreads();
  if (threadIdx.x == 0) {
    const uint32_t xcc = __builtin_amdgcn_s_getreg((3 << 11) | 20);  // HW_REG_XCC_ID bits 3:0
    out[blockIdx.x] = xcc | (lds[5] << 8);
  }
  // keep the workgroup resident a little (so launches overlap like real kernels)
  const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
  while (__builtin_amdgcn_s_memrealtime() - t0 < spin) {
  }
}

__global__ void small(uint32_t *sink) {
  if (threadIdx.x == 0) sink[blockIdx.x] = blockIdx.x;
}

int main() {
  constexpr int kMaxLaunch = 64, kMaxBlocks = 256;
  uint32_t *out, *sink;
  CK(hipMalloc(&out, 4 * kMaxLaunch * kMaxBlocks));
  CK(hipMalloc(&sink, 4096));
  hipStream_t s1, s2;
  CK(hipStreamCreateWithFlags(&s1, hipStreamNonBlocking));
  CK(hipStreamCreateWithFlags(&s2, hipStreamNonBlocking));
  std::vector<uint32_t> h(kMaxLaunch * kMaxBlocks);
  auto report = [&](const char *what, const std::vector<int> &grids) {
    CK(hipDeviceSynchronize());
    CK(hipMemcpy(h.data(), out, 4 * kMaxLaunch * kMaxBlocks, hipMemcpyDeviceToHost));
    printf("%s\n", what);
    for (size_t l = 0; l < grids.size(); ++l) {
      const uint32_t *o = &h[l * kMaxBlocks];
      const int k = (int)((o[0] & 15u) + 8u) % 8;
      int bad = 0;
      for (int b = 0; b < grids[l]; ++b) bad += (int)(o[b] & 15u) != (b + k) % 8;
      printf("  launch %2zu: %3d workgroups, block 0 on XCD %d (k %s), %d break XCD = (b + k) %% 8; first 10:", l,
             grids[l], k, k % 2 ? "odd" : "even", bad);
      for (int b = 0; b < 10; ++b) printf(" %u", o[b] & 15u);
      printf("\n");
    }
  };
  const uint32_t spin = 2000;  // 20 us at 100 MHz
  {  // A
    std::vector<int> g;
    for (int l = 0; l < 10; ++l) { hipLaunchKernelGGL(probe, dim3(240), dim3(1024), 0, s1, out + l * kMaxBlocks, spin); g.push_back(240); }
    report("A: 240-workgroup launches back to back", g);
  }
  {  // B
    std::vector<int> g;
    for (int l = 0; l < 10; ++l) {
      const int n = l % 2 ? 256 : 241;
      hipLaunchKernelGGL(probe, dim3(n), dim3(1024), 0, s1, out + l * kMaxBlocks, spin);
      g.push_back(n);
    }
    report("B: 241- then 256-workgroup launches (bucket pass -> fold)", g);
  }
  {  // C
    std::vector<int> g;
    for (int l = 0; l < 10; ++l) {
      hipLaunchKernelGGL(small, dim3(7), dim3(64), 0, s2, sink);
      hipLaunchKernelGGL(probe, dim3(256), dim3(1024), 0, s1, out + l * kMaxBlocks, spin);
      hipLaunchKernelGGL(small, dim3(7), dim3(64), 0, s2, sink);
      g.push_back(256);
    }
    report("C: 256-workgroup launches with 7-workgroup kernels on a second stream", g);
  }
  {  // D
    std::vector<int> g;
    for (int l = 0; l < 10; ++l) {
      CK(hipDeviceSynchronize());
      usleep(1000);
      hipLaunchKernelGGL(probe, dim3(240), dim3(1024), 0, s1, out + l * kMaxBlocks, spin);
      g.push_back(240);
    }
    report("D: 240-workgroup launches after a host sync and 1 ms", g);
  }
  return 0;
}
