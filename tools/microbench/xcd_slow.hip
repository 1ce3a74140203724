// Are the slow workgroups of the strided-chain kernel the odd-NUMBERED ones
// (relative to where a launch starts dealing workgroups) or the ones on
// odd-NUMBERED XCDs?  (round 4: tools/microbench/xcc_probe.hip showed that
// which XCD gets workgroup 0 changes between launches of one process, k = 6
// or 7.)  Per trial: a fresh stream; a probe kernel reads HW_REG_XCC_ID of
// every workgroup (k = XCD of workgroup 0; the stamped kernel that follows
// on the same stream is assumed to start there too, and a second probe after
// it checks that); then the SCK with per-wave start / end stamps, equal
// shares (ABL 64).  Mean wave end by blockIdx % 8 and by physical XCD.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 xcd_slow.hip -o xcd_slow
#include "../../roce-test_amd/csrc/icrc_kernels.hip"
#include "../../roce-test_amd/csrc/icrc_sck.hip"
#include "mb_fin.h"
#include <stdio.h>
#include <stdlib.h>

#include <vector>
using namespace ricrc;
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s line %d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)

__global__ void xcc_one(uint32_t *out) {  // one 64-thread workgroup: the XCD it lands on
  if (threadIdx.x == 0) out[0] = __builtin_amdgcn_s_getreg((3 << 11) | 20);
}

__global__ __launch_bounds__(1024) void xcc_probe(uint32_t *out) {
  __shared__ uint32_t lds[32768];  // 128 KiB: one workgroup per CU, like the SCK
  lds[threadIdx.x] = threadIdx.x;
  __syncthreads();
  if (threadIdx.x == 0) out[blockIdx.x] = __builtin_amdgcn_s_getreg((3 << 11) | 20) | (lds[1] << 8);
}

int main(int argc, char **argv) {
  const bool cold = argc > 1;  // "cold": no host copy first (the kernels are the process's first GPU work)
  const uint64_t count = 1ull << 20, n = 4096, bytes = count * n;
  uint8_t *buf; uint32_t *out, *xo; uint64_t *stamps;
  CK(hipMalloc(&buf, bytes)); CK(hipMalloc(&out, 4 * count)); CK(hipMalloc(&xo, 4 * 512));
  if (!cold) {
    std::vector<uint64_t> h(bytes / 8);
    uint64_t x = 0x9E3779B97F4A7C15ull;
    for (auto &v : h) { x ^= x << 13; x ^= x >> 7; x ^= x << 17; v = x; }
    CK(hipMemcpy(buf, h.data(), bytes, hipMemcpyHostToDevice));
  }
  const int grid = 240, waves = grid * kWaves;
  CK(hipMalloc(&stamps, 16ull * waves));
  SckArgs a{};
  a.base = buf; a.count = count; a.out = out; a.n = 4096; a.stamps = stamps;
  a.fin = mb_fin();
  std::vector<uint32_t> hx(512);
  std::vector<uint64_t> st(2 * waves);
  uint32_t *sink; CK(hipMalloc(&sink, 4096));
  auto trial = [&](const char *what, hipStream_t s, int pre) {
    for (int w = 0; w < 3; ++w) hipLaunchKernelGGL((icrc_sck_kernel<32, 0>), dim3(grid), dim3(kBlock), 0, s, a);
    if (pre > 0) hipLaunchKernelGGL(xcc_probe, dim3(pre), dim3(1024), 0, s, sink);
    hipLaunchKernelGGL(xcc_one, dim3(1), dim3(64), 0, s, xo + 511);
    hipLaunchKernelGGL(xcc_probe, dim3(grid), dim3(1024), 0, s, xo);
    hipLaunchKernelGGL((icrc_sck_kernel<32, 64>), dim3(grid), dim3(kBlock), 0, s, a);
    hipLaunchKernelGGL(xcc_probe, dim3(grid), dim3(1024), 0, s, xo + 256);
    CK(hipStreamSynchronize(s));
    CK(hipMemcpy(hx.data(), xo, 4 * 512, hipMemcpyDeviceToHost));
    CK(hipMemcpy(st.data(), stamps, 16ull * waves, hipMemcpyDeviceToHost));
    const int k0 = (int)(hx[0] & 15u), k1 = (int)(hx[256] & 15u);
    uint64_t t0 = ~0ull, t1 = 0;
    for (int w = 0; w < waves; ++w) { t0 = std::min(t0, st[2 * w]); t1 = std::max(t1, st[2 * w + 1]); }
    double byb[8] = {0}, byx[8] = {0};
    int cb[8] = {0}, cx[8] = {0};
    for (int w = 0; w < waves; ++w) {
      const int b = w / kWaves;
      const double e = (st[2 * w + 1] - t0) / 100.0;
      byb[b % 8] += e; ++cb[b % 8];
      byx[(b + k0) % 8] += e; ++cx[(b + k0) % 8];
    }
    printf("%-34s 1-workgroup detector %u;", what, hx[511] & 15u);
    printf(" k before %d after %d; span %.1f us | mean end by blockIdx%%8:", k0, k1, (t1 - t0) / 100.0);
    for (int i = 0; i < 8; ++i) printf(" %.0f", byb[i] / cb[i]);
    printf(" | by XCD:");
    for (int i = 0; i < 8; ++i) printf(" %.0f", byx[i] / cx[i]);
    double ev = 0, od = 0, evx = 0, odx = 0;
    for (int i = 0; i < 8; i += 2) { ev += byb[i] / cb[i]; od += byb[i + 1] / cb[i + 1]; evx += byx[i] / cx[i]; odx += byx[i + 1] / cx[i + 1]; }
    printf(" | odd-even blocks %+.0f, odd-even XCDs %+.0f us\n", (od - ev) / 4, (odx - evx) / 4);
  };
  char nm[64];
  for (int t = 0; t < 12; ++t) {
    hipStream_t s;
    CK(hipStreamCreateWithFlags(&s, t % 2 ? hipStreamNonBlocking : hipStreamDefault));
    const int pre = t % 4 == 1 ? 1 : t % 4 == 2 ? 7 : t % 4 == 3 ? 3 : 0;
    snprintf(nm, sizeof nm, "trial %2d (%d-workgroup kernel first)", t, pre);
    trial(nm, s, pre);
    CK(hipStreamDestroy(s));
  }
  return 0;
}
