// The XCD-parity weights with the start XCD taken from the previous launch's
// record (the product, round 4) against the same weights assuming workgroup
// b on XCD b % 8 (the first version) and against equal shares, on the
// headline batch (1 M x 4 KiB, 240 CUs, skew 25), alternating.  "cold"
// (argv[1]) skips the host copy of the data first: in such processes the
// launches start dealing at XCD 7 (tools/microbench/xcd_slow.hip), which
// flips which workgroups are on the slow XCDs.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 xcd_fix.hip -o xcd_fix
#include "../../roce-test_amd/csrc/icrc_kernels.hip"
#include "../../roce-test_amd/csrc/icrc_sck.hip"
#include "mb_fin.h"
#include <stdio.h>
#include <stdlib.h>

#include <vector>
using namespace ricrc;
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s line %d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)

__global__ __launch_bounds__(1024) void lds_one(uint32_t *out) {  // one 1024-thread, 128 KiB-LDS workgroup
  __shared__ uint32_t lds[32768];
  lds[threadIdx.x] = threadIdx.x;
  __syncthreads();
  if (threadIdx.x == 0) out[0] = lds[7];
}

int main(int argc, char **argv) {
  const bool cold = argc > 1;
  const uint64_t count = 1ull << 20, n = 4096, bytes = count * n;
  uint8_t *buf; uint32_t *out;
  CK(hipMalloc(&buf, bytes)); CK(hipMalloc(&out, 4 * count));
  if (!cold) {
    std::vector<uint64_t> h(bytes / 8);
    uint64_t x = 0x9E3779B97F4A7C15ull;
    for (auto &v : h) { x ^= x << 13; x ^= x >> 7; x ^= x << 17; v = x; }
    CK(hipMemcpy(buf, h.data(), bytes, hipMemcpyHostToDevice));
  }
  uint32_t *h_rec, *d_rec;
  CK(hipHostMalloc((void **)&h_rec, 64, hipHostMallocCoherent));
  *h_rec = 0;
  CK(hipHostGetDevicePointer((void **)&d_rec, h_rec, 0));
  const int grid = 240;
  SckArgs a{};
  a.base = buf; a.count = count; a.out = out; a.n = 4096; a.xcd_rec = d_rec;
  a.fin = mb_fin();
  hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  hipStream_t st = 0;
  auto run = [&](int v) {  // 0 equal shares, 1 skew assuming k = 0, 2 skew with the recorded k
    SckArgs k = a;
    if (v) for (int x = 0; x < 8; ++x) k.xw[x] = (x & 1) ? 975u : 1025u;
    k.xcd_k = v == 2 ? __atomic_load_n(h_rec, __ATOMIC_RELAXED) & 7u : 0u;
    hipLaunchKernelGGL((icrc_sck_kernel<32, 0>), dim3(grid), dim3(kBlock), 0, st, k);
  };
  auto timeit = [&](int v) {
    for (int r = 0; r < 5; ++r) run(v);
    CK(hipEventRecord(e0, st));
    for (int r = 0; r < 20; ++r) run(v);
    CK(hipEventRecord(e1, st));
    CK(hipEventSynchronize(e1));
    float ms; CK(hipEventElapsedTime(&ms, e0, e1));
    return 1e3f * ms / 20;
  };
  printf("%s; 1 M x 4 KiB, 240 CUs\n", cold ? "cold (no host copy first)" : "data copied from the host first");
  // a fresh stream per round (the start XCD has changed after stream creation, xcd_slow.hip)
  for (int r = 0; r < 8; ++r) {
    CK(hipStreamCreateWithFlags(&st, r % 2 ? hipStreamNonBlocking : hipStreamDefault));
    // (xcd_slow.hip: after such a one-workgroup kernel the launches of a
    // cold process started dealing at XCD 7)
    hipLaunchKernelGGL(lds_one, dim3(1), dim3(1024), 0, st, out);
    const float t0 = timeit(0), t1 = timeit(1), t2 = timeit(2);
    printf("round %d (recorded start XCD %u): equal %6.1f | skew 25, k = 0 assumed %6.1f | skew 25, k recorded %6.1f us\n",
           r, *h_rec & 7u, t0, t1, t2);
    CK(hipStreamDestroy(st));
  }
  return 0;
}
