// C1 (1 M x 64 B) attribution: what bounds the 16 us launch?  Timing only.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 c1_probe.hip -o c1_probe && ./c1_probe
// Variants over the same 64 MiB (random bytes), 20 launches each, HIP events:
//   empty      the launch alone (grid x 1024 threads, 128 KiB LDS declared)
//   fill       + the 128 KiB 32-copy table fill
//   lane64     memory path, each lane loads its packet's 64 B (4 x 16 B at
//              64 l + 16 k: the product's direct kernel pattern)
//   coal       memory path, coalesced: load k of a wave reads 1 KiB at 1024 k + 16 l
//   direct     icrc_stream_kernel<1, true> (the round-2 C1 kernel)
//   quad       icrc_quad_kernel<4> as the library launches it (round 3)
// Memory variants request all of a wave's bytes before using any (the whole
// batch is ~4 steps per wave), XOR them and write one word per wave.
// Per-wave s_memrealtime start / end stamps for `coal` and `lane64`.
#include "../../roce-test_amd/csrc/icrc_kernels.hip"

#include <stdio.h>
#include <stdlib.h>

#include <algorithm>
#include <vector>
using namespace ricrc;
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s line %d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)

template <int MODE, bool FILL, int STEPS, bool LDS = true>
__global__ __launch_bounds__(1024) void probe(const uint8_t *buf, uint64_t bytes, uint32_t *sink, uint64_t *stamps) {
  __shared__ uint32_t lds[LDS ? kLdsWords : 64];
  const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
  const uint32_t lane = threadIdx.x & 63;
  const uint64_t wave = (uint64_t)blockIdx.x * 16 + (threadIdx.x >> 6);
  const uint64_t nwaves = (uint64_t)gridDim.x * 16;
  u32x4 acc = {0u, 0u, 0u, 0u};
  if (MODE != 0) {
    // the wave's block of STEPS x 4 KiB
    const uint64_t base = wave * (uint64_t)STEPS * 4096u;
    u32x4 v[4 * STEPS];
#pragma unroll
    for (int k = 0; k < 4 * STEPS; ++k) {
      const uint32_t o = MODE == 1 ? (uint32_t)(4096 * (k >> 2) + 64 * lane + 16 * (k & 3))  // lane64
                                   : (uint32_t)(1024 * k + 16 * lane);                          // coalesced
      v[k] = base + o < bytes ? __builtin_nontemporal_load(reinterpret_cast<const u32x4 *>(buf + base + o))
                              : u32x4{0u, 0u, 0u, 0u};
    }
    if (FILL) {
      const uint32_t tv = table_entry(g_tab);
      table_store(lds, tv);
      __syncthreads();
      acc[0] ^= lds[(lane * 97) & (kLdsWords - 1)];
    }
#pragma unroll
    for (int k = 0; k < 4 * STEPS; ++k) acc ^= v[k];
  } else if (FILL) {
    const uint32_t tv = table_entry(g_tab);
    table_store(lds, tv);
    __syncthreads();
    acc[0] ^= lds[(lane * 97) & (kLdsWords - 1)];
  }
  const uint32_t x = acc[0] ^ acc[1] ^ acc[2] ^ acc[3];
  if (x == 0x12345678u) sink[wave] = x;
  if (stamps && lane == 0) {
    stamps[2 * wave] = t0;
    stamps[2 * wave + 1] = __builtin_amdgcn_s_memrealtime();
  }
}

template <class F>
float timeit(F f, int reps = 20) {
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  for (int i = 0; i < 5; ++i) f();
  CK(hipDeviceSynchronize());
  CK(hipEventRecord(e0));
  for (int i = 0; i < reps; ++i) f();
  CK(hipEventRecord(e1));
  CK(hipEventSynchronize(e1));
  float ms;
  CK(hipEventElapsedTime(&ms, e0, e1));
  return ms * 1000.f / reps;
}

void timeline(const char *nm, std::vector<uint64_t> &st, int waves) {
  uint64_t t0 = ~0ull, t1 = 0;
  for (int w = 0; w < waves; ++w) t0 = std::min(t0, st[2 * w]), t1 = std::max(t1, st[2 * w + 1]);
  std::vector<double> s, e;
  for (int w = 0; w < waves; ++w) s.push_back((st[2 * w] - t0) / 100.0), e.push_back((st[2 * w + 1] - t0) / 100.0);
  std::sort(s.begin(), s.end());
  std::sort(e.begin(), e.end());
  auto q = [&](std::vector<double> &v, double f) { return v[std::min(v.size() - 1, (size_t)(f * v.size()))]; };
  printf("  %-8s span %.2f us | wave start p10 %.2f p50 %.2f p90 %.2f max %.2f | end min %.2f p10 %.2f p50 %.2f p90 %.2f max %.2f\n",
         nm, (t1 - t0) / 100.0, q(s, .1), q(s, .5), q(s, .9), s.back(), e.front(), q(e, .1), q(e, .5), q(e, .9), e.back());
}

int main() {
  const uint64_t count = 1 << 20, n = 64, bytes = count * n;
  uint8_t *buf;
  uint32_t *out, *sink;
  uint64_t *stamps;
  CK(hipMalloc(&buf, bytes));
  CK(hipMalloc(&out, 4 * count));
  CK(hipMalloc(&sink, 4 << 20));
  CK(hipMalloc(&stamps, 16ull << 16));
  {
    std::vector<uint64_t> h(bytes / 8);
    uint64_t x = 0x9E3779B97F4A7C15ull;
    for (auto &v : h) x ^= x << 13, x ^= x >> 7, x ^= x << 17, v = x;
    CK(hipMemcpy(buf, h.data(), bytes, hipMemcpyHostToDevice));
  }
  hipDeviceProp_t p;
  CK(hipGetDeviceProperties(&p, 0));
  const int cu = p.multiProcessorCount;
  printf("1 M x 64 B = %.1f MiB, %d CUs; roofline (64 MiB + 4 MiB) / 8 TB/s = %.2f us\n", bytes / 1048576.0, cu,
         (bytes + 4.0 * count) / 8e12 * 1e6);
  // the product kernel exactly as icrc_api.cpp launches it for 64-byte packets
  StreamArgs a{};
  a.base = buf; a.stride = n; a.count = count; a.out = out; a.len = n;
  a.P = 1; a.log2P2 = 0; a.nw_last = 15; a.n_iters = count / 64; a.verify = 0;
  a.K[0] = gf_x8n(0);
  const int pgrid = (int)std::min<uint64_t>(cu, (a.n_iters + 15) / 16);
  QuadArgs q{};
  q.base = buf; q.count = count; q.out = out;
  for (int r = 0; r < 3; ++r) {
    printf("round %d\n", r);
    printf("  empty         %7.2f us\n", timeit([&] { hipLaunchKernelGGL((probe<0, false, 4>), dim3(cu), dim3(1024), 0, 0, buf, bytes, sink, nullptr); }));
    printf("  fill          %7.2f us\n", timeit([&] { hipLaunchKernelGGL((probe<0, true, 4>), dim3(cu), dim3(1024), 0, 0, buf, bytes, sink, nullptr); }));
    printf("  lane64        %7.2f us\n", timeit([&] { hipLaunchKernelGGL((probe<1, false, 4>), dim3(cu), dim3(1024), 0, 0, buf, bytes, sink, nullptr); }));
    printf("  lane64+fill   %7.2f us\n", timeit([&] { hipLaunchKernelGGL((probe<1, true, 4>), dim3(cu), dim3(1024), 0, 0, buf, bytes, sink, nullptr); }));
    printf("  coal          %7.2f us\n", timeit([&] { hipLaunchKernelGGL((probe<2, false, 4>), dim3(cu), dim3(1024), 0, 0, buf, bytes, sink, nullptr); }));
    printf("  coal+fill     %7.2f us\n", timeit([&] { hipLaunchKernelGGL((probe<2, true, 4>), dim3(cu), dim3(1024), 0, 0, buf, bytes, sink, nullptr); }));
    printf("  coal 2xgrid   %7.2f us  (2 steps per wave)\n", timeit([&] { hipLaunchKernelGGL((probe<2, false, 2>), dim3(2 * cu), dim3(1024), 0, 0, buf, bytes, sink, nullptr); }));
    printf("  coal 4xgrid   %7.2f us  (1 step per wave)\n", timeit([&] { hipLaunchKernelGGL((probe<2, false, 1>), dim3(4 * cu), dim3(1024), 0, 0, buf, bytes, sink, nullptr); }));
    printf("  direct        %7.2f us  (icrc_stream_kernel<1,true>, grid %d)\n", timeit([&] { CK(launch_stream(a, 1, pgrid, 0)); }), pgrid);
    printf("  quad          %7.2f us  (icrc_quad_kernel<4>, grid %d)\n", timeit([&] { CK(launch_quad(q, cu, 0)); }), cu);
    printf("  empty noLDS   %7.2f us\n", timeit([&] { hipLaunchKernelGGL((probe<0, false, 4, false>), dim3(cu), dim3(1024), 0, 0, buf, bytes, sink, nullptr); }));
    printf("  empty 256thr  %7.2f us\n", timeit([&] { hipLaunchKernelGGL((probe<0, false, 4>), dim3(cu), dim3(256), 0, 0, buf, bytes, sink, nullptr); }));
    printf("  empty 64 WGs  %7.2f us\n", timeit([&] { hipLaunchKernelGGL((probe<0, false, 4>), dim3(64), dim3(1024), 0, 0, buf, bytes, sink, nullptr); }));
    printf("  quad W8       %7.2f us  (512-thread workgroups)\n", timeit([&] { hipLaunchKernelGGL((icrc_quad_kernel<0, 2, 2, 8>), dim3(cu), dim3(512), 0, 0, q); }));
    printf("  quad W8 R4F2  %7.2f us  (512-thread workgroups)\n", timeit([&] { hipLaunchKernelGGL((icrc_quad_kernel<0, 4, 2, 8>), dim3(cu), dim3(512), 0, 0, q); }));
    printf("  quad R4F2 IP  %7.2f us  (in-place ring)\n", timeit([&] { hipLaunchKernelGGL((icrc_quad_kernel<0, 4, 2, 16, true>), dim3(cu), dim3(kBlock), 0, 0, q); }));
    printf("  quad R2F2 IP  %7.2f us  (in-place ring)\n", timeit([&] { hipLaunchKernelGGL((icrc_quad_kernel<0, 2, 2, 16, true>), dim3(cu), dim3(kBlock), 0, 0, q); }));
    printf("  quad R4F1 IP  %7.2f us  (in-place ring)\n", timeit([&] { hipLaunchKernelGGL((icrc_quad_kernel<0, 4, 1, 16, true>), dim3(cu), dim3(kBlock), 0, 0, q); }));
    printf("  quad R2F1 IP  %7.2f us  (in-place ring)\n", timeit([&] { hipLaunchKernelGGL((icrc_quad_kernel<0, 2, 1, 16, true>), dim3(cu), dim3(kBlock), 0, 0, q); }));
    printf("  quad R1F1 IP  %7.2f us  (in-place ring)\n", timeit([&] { hipLaunchKernelGGL((icrc_quad_kernel<0, 1, 1, 16, true>), dim3(cu), dim3(kBlock), 0, 0, q); }));
    printf("  quad R2F2 IP W8 %5.2f us  (in-place ring, 512 threads)\n", timeit([&] { hipLaunchKernelGGL((icrc_quad_kernel<0, 2, 2, 8, true>), dim3(cu), dim3(512), 0, 0, q); }));
    printf("  quad R4 F1    %7.2f us\n", timeit([&] { hipLaunchKernelGGL((icrc_quad_kernel<0, 4, 1>), dim3(cu), dim3(kBlock), 0, 0, q); }));
    printf("  quad R2 F1    %7.2f us\n", timeit([&] { hipLaunchKernelGGL((icrc_quad_kernel<0, 2, 1>), dim3(cu), dim3(kBlock), 0, 0, q); }));
    printf("  quad R1 F1    %7.2f us\n", timeit([&] { hipLaunchKernelGGL((icrc_quad_kernel<0, 1, 1>), dim3(cu), dim3(kBlock), 0, 0, q); }));
    printf("  quad R4 F2    %7.2f us\n", timeit([&] { hipLaunchKernelGGL((icrc_quad_kernel<0, 4, 2>), dim3(cu), dim3(kBlock), 0, 0, q); }));
  }
  // Round 4, the one launch-trim A/B: the product launch
  // against fewer, fatter workgroups (half the grid: 8 steps per wave, half
  // the table fills and dispatches) and against two 512-thread workgroups
  // per CU (a CU starts folding after half the table fill), alternating.
  printf("launch-trim A/B\n");
  for (int r = 0; r < 5; ++r) {
    const float t0 = timeit([&] { CK(launch_quad(q, cu, 0)); });
    const float t1 = timeit([&] { hipLaunchKernelGGL((icrc_quad_kernel<0, 2, 2, 16, true>), dim3(cu / 2), dim3(kBlock), 0, 0, q); });
    const float t2 = timeit([&] { hipLaunchKernelGGL((icrc_quad_kernel<0, 2, 2, 8, true>), dim3(2 * cu), dim3(512), 0, 0, q); });
    printf("  product %d x 1024 %6.2f us | %d x 1024 %6.2f us | %d x 512 %6.2f us\n", cu, t0, cu / 2, t1, 2 * cu, t2);
  }
  for (int m : {1, 2, 3}) {
    std::vector<uint64_t> st(2 * 16 * cu);
    QuadArgs qs = q;
    qs.stamps = stamps;
    for (int i = 0; i < 5; ++i) {
      if (m == 1) hipLaunchKernelGGL((probe<1, true, 4>), dim3(cu), dim3(1024), 0, 0, buf, bytes, sink, stamps);
      else if (m == 2) hipLaunchKernelGGL((probe<2, true, 4>), dim3(cu), dim3(1024), 0, 0, buf, bytes, sink, stamps);
      else hipLaunchKernelGGL((icrc_quad_kernel<64, 2, 2, 16, true>), dim3(cu), dim3(kBlock), 0, 0, qs);
    }
    CK(hipDeviceSynchronize());
    CK(hipMemcpy(st.data(), stamps, st.size() * 8, hipMemcpyDeviceToHost));
    timeline(m == 1 ? "lane64" : m == 2 ? "coal" : "quad", st, 16 * cu);
  }
  return 0;
}
