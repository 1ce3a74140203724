// Floor of the C1 configuration (1 M x 64 B = 64 MiB): how fast can any kernel
// read 64 MiB and write one u32 per 64-byte packet on MI355X?  No CRC at all:
// each lane XORs its packet's four 16-byte units.  Variants: one packet per
// lane over a full grid, or a persistent grid with P packets per lane in
// flight; default vs non-temporal loads.  Median of 50 HIP-event timings.
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 mb_small.hip -o mb_small
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#include <algorithm>
#include <vector>

#define CK(x)                                                                 \
  do {                                                                        \
    hipError_t e = (x);                                                       \
    if (e != hipSuccess) {                                                    \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e)); \
      exit(1);                                                                \
    }                                                                         \
  } while (0)

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

// Lane-per-packet: lane loads 4 x 16 B of its packet (4 instructions, each
// covering 64 x 16 B at a 64-byte stride = 4 KiB contiguous per wave).
template <int P, bool NT>
__global__ __launch_bounds__(256) void lane_pkt(const uint8_t *buf, uint64_t count, uint32_t *out) {
  const uint64_t t0 = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const uint64_t nt = (uint64_t)gridDim.x * blockDim.x;
  for (uint64_t base = t0; base < count; base += nt * P) {
    u32x4 v[P][4];
#pragma unroll
    for (int p = 0; p < P; ++p) {
      const uint64_t i = base + (uint64_t)p * nt;
      const u32x4 *q = (const u32x4 *)(buf + (i < count ? i : 0) * 64);
#pragma unroll
      for (int k = 0; k < 4; ++k) v[p][k] = NT ? __builtin_nontemporal_load(q + k) : q[k];
    }
#pragma unroll
    for (int p = 0; p < P; ++p) {
      const uint64_t i = base + (uint64_t)p * nt;
      const u32x4 a = v[p][0] ^ v[p][1] ^ v[p][2] ^ v[p][3];
      if (i < count) out[i] = a.x ^ a.y ^ a.z ^ a.w;
    }
  }
}

// Coalesced: lane l of a wave reads unit l of each KiB (16 packets per KiB);
// the four lanes of a packet XOR-reduce with shuffles.
template <bool NT>
__global__ __launch_bounds__(256) void coal(const uint8_t *buf, uint64_t count, uint32_t *out) {
  const uint64_t units = count * 4;
  const uint64_t t0 = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const uint64_t nt = (uint64_t)gridDim.x * blockDim.x;
  for (uint64_t u = t0; u < units; u += nt) {
    const u32x4 *q = (const u32x4 *)(buf + u * 16);
    const u32x4 a = NT ? __builtin_nontemporal_load(q) : *q;
    uint32_t x = a.x ^ a.y ^ a.z ^ a.w;
    x ^= __shfl_xor(x, 1);
    x ^= __shfl_xor(x, 2);
    if ((u & 3) == 0) out[u >> 2] = x;
  }
}

template <typename F>
float time_it(F f) {
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  std::vector<float> ts;
  for (int r = 0; r < 70; ++r) {
    CK(hipEventRecord(a, 0));
    f();
    CK(hipEventRecord(b, 0));
    CK(hipEventSynchronize(b));
    float ms;
    CK(hipEventElapsedTime(&ms, a, b));
    if (r >= 20) ts.push_back(ms);
  }
  std::sort(ts.begin(), ts.end());
  return ts[ts.size() / 2] * 1e3f;
}

int main() {
  const uint64_t count = 1ull << 20, bytes = count * 64;
  uint8_t *buf;
  uint32_t *out;
  CK(hipMalloc(&buf, bytes));
  CK(hipMalloc(&out, count * 4));
  CK(hipMemset(buf, 0x5A, bytes));
  const double alg = bytes + 4.0 * count;
  auto rep = [&](const char *name, float us) {
    printf("%-36s %7.2f us  %6.0f GiB/s  %.3f of 8 TB/s\n", name, us, bytes / (us * 1e-6) / (1 << 30),
           alg / (us * 1e-6) / 8e12);
  };
  const unsigned full = (unsigned)(count / 256);
  rep("lane_pkt P1 full grid", time_it([&] { hipLaunchKernelGGL((lane_pkt<1, false>), dim3(full), dim3(256), 0, 0, buf, count, out); }));
  rep("lane_pkt P1 full grid nt", time_it([&] { hipLaunchKernelGGL((lane_pkt<1, true>), dim3(full), dim3(256), 0, 0, buf, count, out); }));
  for (unsigned g : {1024u, 2048u}) {
    char nm[64];
    snprintf(nm, sizeof nm, "lane_pkt P2 grid %u", g);
    rep(nm, time_it([&] { hipLaunchKernelGGL((lane_pkt<2, false>), dim3(g), dim3(256), 0, 0, buf, count, out); }));
    snprintf(nm, sizeof nm, "lane_pkt P4 grid %u", g);
    rep(nm, time_it([&] { hipLaunchKernelGGL((lane_pkt<4, false>), dim3(g), dim3(256), 0, 0, buf, count, out); }));
  }
  rep("coal full grid", time_it([&] { hipLaunchKernelGGL((coal<false>), dim3((unsigned)(count * 4 / 256)), dim3(256), 0, 0, buf, count, out); }));
  rep("coal full grid nt", time_it([&] { hipLaunchKernelGGL((coal<true>), dim3((unsigned)(count * 4 / 256)), dim3(256), 0, 0, buf, count, out); }));
  rep("empty launch", time_it([&] { hipLaunchKernelGGL((lane_pkt<1, false>), dim3(1), dim3(64), 0, 0, buf, 0, out); }));
  CK(hipFree(buf));
  CK(hipFree(out));
  return 0;
}
