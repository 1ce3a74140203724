// Memory-pattern microbenchmark for a strided-chain ICRC layout: a wave
// reads a group of 64/LPP packets of 4096 B; load k gives lane 16*... the
// 16-byte slot s = lane % LPP of "line" k (16*LPP bytes) of packet lane / LPP.
// LPP = 64 is the fully coalesced 1 KiB-per-instruction pattern.  Loads are
// issued D steps ahead (rotating registers).  Random data (DVFS).
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 mb_lines.hip -o mb_lines
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#define CK(x)                                                                 \
  do {                                                                        \
    hipError_t e = (x);                                                       \
    if (e != hipSuccess) {                                                    \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e)); \
      exit(1);                                                                \
    }                                                                         \
  } while (0)

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ __amdgpu_buffer_rsrc_t make_rsrc(const void *base, uint32_t bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void *>(base), (short)0, (int)bytes, 0x00020000);
}

// Gathered variant: packet slot g of group q is packet perm[8 q + g] (random
// order, as after bucketing a ragged batch by size), lines offset by SHIFT bytes
// from 128-byte alignment; global loads with 64-bit addresses.
template <int SHIFT, int D, bool NT>
__global__ __launch_bounds__(1024) void gather_lines(const uint8_t *buf, const uint32_t *perm, uint64_t npkt,
                                                     uint32_t *sink) {
  constexpr uint32_t PKT = 4096, STEPS = PKT / 128;
  const uint32_t lane = threadIdx.x & 63;
  const uint64_t wave = (uint64_t)blockIdx.x * 16 + (threadIdx.x >> 6);
  const uint64_t nw = (uint64_t)gridDim.x * 16;
  const uint64_t ngroups = npkt / 8 - 1;  // the shifted last packet would run past the buffer
  const uint64_t per = (ngroups + nw - 1) / nw;
  const uint64_t g0 = wave * per < ngroups ? wave * per : ngroups;
  const uint64_t g1 = g0 + per < ngroups ? g0 + per : ngroups;
  const uint64_t nsteps = (g1 - g0) * STEPS;
  auto addr = [&](uint64_t t) -> const u32x4 * {
    uint64_t g = g0 + t / STEPS;
    if (g >= g1) g = g0;
    const uint32_t k = (uint32_t)(t % STEPS);
    const uint64_t pk = perm[8 * g + (lane >> 3)];
    return (const u32x4 *)(buf + pk * PKT + SHIFT + 128 * k + 16 * (lane & 7));
  };
  u32x4 acc = {0, 0, 0, 0};
  u32x4 v[D];
#pragma unroll
  for (int d = 0; d < D; ++d) v[d] = NT ? __builtin_nontemporal_load(addr(d)) : *addr(d);
  for (uint64_t t = 0; t < nsteps; t += D) {
#pragma unroll
    for (int d = 0; d < D; ++d) {
      acc ^= v[d];
      v[d] = NT ? __builtin_nontemporal_load(addr(t + D + d)) : *addr(t + D + d);
    }
  }
  sink[blockIdx.x * blockDim.x + threadIdx.x] = acc.x ^ acc.y ^ acc.z ^ acc.w;
}

template <int LPP, int D, int AUX, int WAVES>
__global__ __launch_bounds__(64 * WAVES) void read_lines(const uint8_t *buf, uint64_t npkt, uint32_t *sink) {
  constexpr uint32_t PKT = 4096, PPG = 64 / LPP, LINE = 16 * LPP, STEPS = PKT / LINE, GB = PPG * PKT;
  const uint32_t lane = threadIdx.x & 63;
  const uint64_t wave = (uint64_t)blockIdx.x * WAVES + (threadIdx.x >> 6);
  const uint64_t nw = (uint64_t)gridDim.x * WAVES;
  const uint64_t ngroups = npkt / PPG;
  const uint64_t per = (ngroups + nw - 1) / nw;
  const uint64_t g0 = wave * per < ngroups ? wave * per : ngroups;
  const uint64_t g1 = g0 + per < ngroups ? g0 + per : ngroups;
  const uint64_t nsteps = (g1 - g0) * STEPS;
  const __amdgpu_buffer_rsrc_t rs = make_rsrc(buf + g0 * GB, (uint32_t)((g1 - g0) * GB));
  const uint32_t vo = (lane / LPP) * PKT + (lane % LPP) * 16;
  auto addr = [&](uint64_t t) -> uint32_t {
    const uint32_t g = (uint32_t)(t / STEPS), k = (uint32_t)(t % STEPS);
    return g * GB + k * LINE;
  };
  u32x4 acc = {0, 0, 0, 0};
  u32x4 v[D];
#pragma unroll
  for (int d = 0; d < D; ++d)
    v[d] = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(rs, vo, addr(d), AUX));
  for (uint64_t t = 0; t < nsteps; t += D) {
#pragma unroll
    for (int d = 0; d < D; ++d) {
      acc ^= v[d];
      v[d] = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(rs, vo, addr(t + D + d), AUX));
    }
  }
  sink[blockIdx.x * blockDim.x + threadIdx.x] = acc.x ^ acc.y ^ acc.z ^ acc.w;
}

template <typename F>
static float timeit(F f, int reps) {
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  f();
  f();
  CK(hipDeviceSynchronize());
  CK(hipEventRecord(a));
  for (int i = 0; i < reps; ++i) f();
  CK(hipEventRecord(b));
  CK(hipEventSynchronize(b));
  float ms;
  CK(hipEventElapsedTime(&ms, a, b));
  return ms / reps;
}

int main() {
  const uint64_t bytes = 4ull << 30, npkt = bytes / 4096;
  hipDeviceProp_t prop;
  CK(hipGetDeviceProperties(&prop, 0));
  const int ncu = prop.multiProcessorCount;
  uint8_t *buf;
  uint32_t *sink;
  CK(hipMalloc(&buf, bytes));
  CK(hipMalloc(&sink, 64ull << 20));
  {
    uint64_t *h = (uint64_t *)malloc(bytes);
    uint64_t x = 0x9E3779B97F4A7C15ull;
    for (uint64_t i = 0; i < bytes / 8; ++i) { x ^= x << 13; x ^= x >> 7; x ^= x << 17; h[i] = x; }
    CK(hipMemcpy(buf, h, bytes, hipMemcpyHostToDevice));
    free(h);
  }
  printf("CUs %d, buffer %.2f GiB\n", ncu, bytes / 1073741824.0);
  auto rep = [&](const char *name, float ms) {
    printf("%-30s %8.3f ms  %7.1f GB/s  (%5.1f%% of 8 TB/s)\n", name, ms, bytes / (ms * 1e-3) / 1e9,
           100.0 * bytes / (ms * 1e-3) / 8e12);
  };
#define RUN(LPP, D, AUX, W)                                                                          \
  rep("LPP " #LPP " D " #D " aux " #AUX " w" #W,                                                      \
      timeit([&] { hipLaunchKernelGGL((read_lines<LPP, D, AUX, W>), dim3(ncu * 16 / W), dim3(64 * W), 0, 0, buf, npkt, sink); }, 20))
  uint32_t *perm_id, *perm_rnd;
  {
    uint32_t *h = (uint32_t *)malloc(4 * npkt);
    for (uint64_t i = 0; i < npkt; ++i) h[i] = (uint32_t)i;
    CK(hipMalloc(&perm_id, 4 * npkt));
    CK(hipMemcpy(perm_id, h, 4 * npkt, hipMemcpyHostToDevice));
    uint64_t x = 12345;
    for (uint64_t i = npkt - 1; i > 0; --i) {
      x ^= x << 13; x ^= x >> 7; x ^= x << 17;
      const uint64_t j = x % (i + 1);
      const uint32_t t = h[i]; h[i] = h[j]; h[j] = t;
    }
    CK(hipMalloc(&perm_rnd, 4 * npkt));
    CK(hipMemcpy(perm_rnd, h, 4 * npkt, hipMemcpyHostToDevice));
    free(h);
  }
#define GRUN(NAME, SHIFT, D, NT, PERM)                                                                  \
  rep(NAME, timeit([&] { hipLaunchKernelGGL((gather_lines<SHIFT, D, NT>), dim3(ncu), dim3(1024), 0, 0, buf, PERM, npkt, sink); }, 20))
  for (int rep2 = 0; rep2 < 2; ++rep2) {
    GRUN("gather id  shift0  D8 nt", 0, 8, true, perm_id);
    GRUN("gather id  shift64 D8 nt", 64, 8, true, perm_id);
    GRUN("gather id  shift16 D8 nt", 16, 8, true, perm_id);
    GRUN("gather rnd shift0  D8 nt", 0, 8, true, perm_rnd);
    GRUN("gather rnd shift64 D8 nt", 64, 8, true, perm_rnd);
    GRUN("gather rnd shift0  D8", 0, 8, false, perm_rnd);
    GRUN("gather rnd shift64 D8", 64, 8, false, perm_rnd);
    RUN(64, 2, 2, 16);
    RUN(64, 4, 2, 16);
    RUN(64, 4, 0, 16);
    RUN(16, 4, 2, 16);
    RUN(16, 4, 0, 16);
    RUN(8, 2, 2, 16);
    RUN(8, 4, 2, 16);
    RUN(8, 8, 2, 16);
    RUN(8, 4, 0, 16);
    RUN(8, 8, 0, 16);
    RUN(4, 4, 2, 16);
    RUN(4, 8, 2, 16);
    RUN(4, 4, 0, 16);
    RUN(4, 8, 0, 16);
    RUN(8, 4, 2, 8);
    RUN(8, 8, 2, 8);
  }
  return 0;
}
