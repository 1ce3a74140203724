// Microbenchmarks that bound the ICRC streaming kernel on MI355X:
//   read_coal  : pure streaming read, lane i reads 16 B at i*16 (+1 KiB per piece)
//   read_chunk : pure streaming read, lane i reads its own 64 B chunk (kernel's pattern)
//   fold_only  : the slice-by-4 LDS fold + lane combine with NO global loads
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 mb.hip -o mb
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#include "../../roce-test_amd/csrc/icrc_math.h"

#define CK(x)                                                                 \
  do {                                                                        \
    hipError_t e = (x);                                                       \
    if (e != hipSuccess) {                                                    \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e)); \
      exit(1);                                                                \
    }                                                                         \
  } while (0)

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

template <int WAVES, int DEPTH, bool NT>
__global__ __launch_bounds__(64 * WAVES) void read_coal(const uint8_t *buf, uint64_t nblk, uint32_t *sink) {
  const int lane = threadIdx.x & 63;
  const uint64_t wave = (uint64_t)blockIdx.x * WAVES + (threadIdx.x >> 6);
  const uint64_t nw = (uint64_t)gridDim.x * WAVES;
  u32x4 acc = {0, 0, 0, 0};
  for (uint64_t b = wave * DEPTH; b < nblk; b += nw * DEPTH) {
    u32x4 v[4 * DEPTH];
#pragma unroll
    for (int d = 0; d < DEPTH; ++d)
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const u32x4 *p = (const u32x4 *)(buf + (b + d) * 4096 + k * 1024 + lane * 16);
        v[d * 4 + k] = NT ? __builtin_nontemporal_load(p) : *p;
      }
#pragma unroll
    for (int k = 0; k < 4 * DEPTH; ++k) acc ^= v[k];
  }
  sink[blockIdx.x * blockDim.x + threadIdx.x] = acc.x ^ acc.y ^ acc.z ^ acc.w;
}

template <int WAVES, int DEPTH, bool NT>
__global__ __launch_bounds__(64 * WAVES) void read_chunk(const uint8_t *buf, uint64_t nblk, uint32_t *sink) {
  const int lane = threadIdx.x & 63;
  const uint64_t wave = (uint64_t)blockIdx.x * WAVES + (threadIdx.x >> 6);
  const uint64_t nw = (uint64_t)gridDim.x * WAVES;
  u32x4 acc = {0, 0, 0, 0};
  for (uint64_t b = wave * DEPTH; b < nblk; b += nw * DEPTH) {
    u32x4 v[4 * DEPTH];
#pragma unroll
    for (int d = 0; d < DEPTH; ++d)
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const u32x4 *p = (const u32x4 *)(buf + (b + d) * 4096 + lane * 64 + k * 16);
        v[d * 4 + k] = NT ? __builtin_nontemporal_load(p) : *p;
      }
#pragma unroll
    for (int k = 0; k < 4 * DEPTH; ++k) acc ^= v[k];
  }
  sink[blockIdx.x * blockDim.x + threadIdx.x] = acc.x ^ acc.y ^ acc.z ^ acc.w;
}

__device__ constexpr ricrc::SliceTables<4> g_tab = ricrc::make_tables<4>();

__device__ __forceinline__ uint32_t lds_at(const uint32_t *lds, uint32_t a) {
  return *(const uint32_t *)((const char *)lds + a);
}

// Fold-only: 16 dependent slice-by-4 steps per lane per "block" + 32-bit
// basis multiply + 6-level butterfly, on data synthesised in registers.
template <int CHAINS>
__global__ __launch_bounds__(1024) void fold_only(uint64_t nblk, uint32_t *sink) {
  __shared__ uint32_t lds[32768];
  for (int i = threadIdx.x; i < 32768; i += 1024) {
    const int region = i >> 14, e = (i >> 6) & 255, half = (i >> 5) & 1;
    lds[i] = g_tab.t[region ? (half ? 0 : 1) : (half ? 2 : 3)][e];
  }
  __syncthreads();
  const int lane = threadIdx.x & 63;
  const uint32_t lo0 = (lane & 31) << 2, lo1 = lo0 | 0x10000u;
  uint32_t Q[32];
  Q[31] = 0x12345678u ^ lane;
#pragma unroll
  for (int j = 30; j >= 0; --j) Q[j] = ricrc::gf_mulx(Q[j + 1]);
  const uint64_t wave = (uint64_t)blockIdx.x * 16 + (threadIdx.x >> 6);
  const uint64_t nw = (uint64_t)gridDim.x * 16;
  uint32_t total = 0;
  for (uint64_t b = wave * CHAINS; b < nblk; b += nw * CHAINS) {
    uint32_t r[CHAINS];
#pragma unroll
    for (int c = 0; c < CHAINS; ++c) r[c] = 0;
#pragma unroll
    for (int j = 0; j < 16; ++j) {
#pragma unroll
      for (int c = 0; c < CHAINS; ++c) {
        const uint32_t x = r[c] ^ (uint32_t)(b * 977 + j * 131 + lane + c);
        const uint32_t t3 = lds_at(lds, __builtin_amdgcn_perm(x, lo0, 0x0C0C0400u));
        const uint32_t t2 = lds_at(lds, __builtin_amdgcn_perm(x, lo0, 0x0C0C0500u) + 128);
        const uint32_t t1 = lds_at(lds, __builtin_amdgcn_perm(x, lo1, 0x0C020600u));
        const uint32_t t0 = lds_at(lds, __builtin_amdgcn_perm(x, lo1, 0x0C020700u) + 128);
        r[c] = __builtin_amdgcn_bitop3_b32(t3, t2, t1 ^ t0, 0x96);
      }
    }
#pragma unroll
    for (int c = 0; c < CHAINS; ++c) {
      uint32_t acc = 0;
#pragma unroll
      for (int j = 0; j < 32; ++j) {
        const uint32_t m = (uint32_t)(((int32_t)(r[c] << (31 - j))) >> 31);
        acc = __builtin_amdgcn_bitop3_b32(m, Q[j], acc, 0x6A);
      }
#pragma unroll
      for (int s = 1; s < 64; s <<= 1) acc ^= __shfl_xor(acc, s);
      total ^= acc;
    }
  }
  sink[blockIdx.x * blockDim.x + threadIdx.x] = total;
}


__device__ __forceinline__ __amdgpu_buffer_rsrc_t make_rsrc(const void *base, uint32_t bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void *>(base), (short)0, (int)bytes, 0x00020000);
}

template <int AUX>
__global__ __launch_bounds__(1024) void read_chunk_buf(const uint8_t *buf, uint64_t nblk, uint32_t *sink) {
  const int lane = threadIdx.x & 63;
  const uint64_t wave = (uint64_t)blockIdx.x * 16 + (threadIdx.x >> 6);
  const uint64_t nw = (uint64_t)gridDim.x * 16;
  u32x4 acc = {0, 0, 0, 0};
  for (uint64_t b = wave * 2; b < nblk; b += nw * 2) {
    const __amdgpu_buffer_rsrc_t rs = make_rsrc(buf + b * 4096, 8192);
    u32x4 v[8];
#pragma unroll
    for (int d = 0; d < 2; ++d)
#pragma unroll
      for (int k = 0; k < 4; ++k)
        v[d * 4 + k] = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(rs, d * 4096 + lane * 64 + k * 16, 0, AUX));
#pragma unroll
    for (int k = 0; k < 8; ++k) acc ^= v[k];
  }
  sink[blockIdx.x * blockDim.x + threadIdx.x] = acc.x ^ acc.y ^ acc.z ^ acc.w;
}
template <int AUX>
__global__ __launch_bounds__(1024) void read_coal_buf(const uint8_t *buf, uint64_t nblk, uint32_t *sink) {
  const int lane = threadIdx.x & 63;
  const uint64_t wave = (uint64_t)blockIdx.x * 16 + (threadIdx.x >> 6);
  const uint64_t nw = (uint64_t)gridDim.x * 16;
  u32x4 acc = {0, 0, 0, 0};
  for (uint64_t b = wave * 2; b < nblk; b += nw * 2) {
    const __amdgpu_buffer_rsrc_t rs = make_rsrc(buf + b * 4096, 8192);
    u32x4 v[8];
#pragma unroll
    for (int d = 0; d < 2; ++d)
#pragma unroll
      for (int k = 0; k < 4; ++k)
        v[d * 4 + k] = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(rs, d * 4096 + k * 1024 + lane * 16, 0, AUX));
#pragma unroll
    for (int k = 0; k < 8; ++k) acc ^= v[k];
  }
  sink[blockIdx.x * blockDim.x + threadIdx.x] = acc.x ^ acc.y ^ acc.z ^ acc.w;
}

template <typename F>
static float timeit(F f, int reps) {
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
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
  const uint64_t bytes = 4ull << 30, nblk = bytes / 4096;
  hipDeviceProp_t prop;
  CK(hipGetDeviceProperties(&prop, 0));
  const int ncu = prop.multiProcessorCount;
  uint8_t *buf;
  uint32_t *sink;
  CK(hipMalloc(&buf, bytes));
  CK(hipMalloc(&sink, 64ull << 20));
  CK(hipMemset(buf, 0x5a, bytes));
  printf("CUs %d, buffer %.2f GiB\n", ncu, bytes / 1073741824.0);
  auto rep = [&](const char *name, float ms) {
    printf("%-34s %8.3f ms  %7.1f GB/s  (%5.1f%% of 8 TB/s)\n", name, ms, bytes / (ms * 1e-3) / 1e9,
           100.0 * bytes / (ms * 1e-3) / 8e12);
  };
#define RUN(NAME, KERN, GRID, BLK) rep(NAME, timeit([&] { hipLaunchKernelGGL(KERN, dim3(GRID), dim3(BLK), 0, 0, buf, nblk, sink); }, 10))
  RUN("read_coal  w16 d1", (read_coal<16, 1, false>), ncu, 1024);
  RUN("read_coal  w16 d2", (read_coal<16, 2, false>), ncu, 1024);
  RUN("read_coal  w16 d1 nt", (read_coal<16, 1, true>), ncu, 1024);
  RUN("read_coal  w16 d2 nt", (read_coal<16, 2, true>), ncu, 1024);
  RUN("read_coal  w8x2 d2", (read_coal<8, 2, false>), ncu * 2, 512);
  RUN("read_coal  w16 d1 grid x4", (read_coal<16, 1, false>), ncu * 4, 1024);
  RUN("read_chunk w16 d1", (read_chunk<16, 1, false>), ncu, 1024);
  RUN("read_chunk w16 d2", (read_chunk<16, 2, false>), ncu, 1024);
  RUN("read_chunk w16 d1 nt", (read_chunk<16, 1, true>), ncu, 1024);
  RUN("read_chunk w16 d2 nt", (read_chunk<16, 2, true>), ncu, 1024);
  RUN("read_chunk w16 d4 nt", (read_chunk<16, 4, true>), ncu, 1024);
  RUN("chunk_buf aux0", (read_chunk_buf<0>), ncu, 1024);
  RUN("chunk_buf aux1 sc0", (read_chunk_buf<1>), ncu, 1024);
  RUN("chunk_buf aux2 nt", (read_chunk_buf<2>), ncu, 1024);
  RUN("chunk_buf aux3 sc0nt", (read_chunk_buf<3>), ncu, 1024);
  RUN("chunk_buf aux16 sc1", (read_chunk_buf<16>), ncu, 1024);
  RUN("chunk_buf aux17", (read_chunk_buf<17>), ncu, 1024);
  RUN("chunk_buf aux18", (read_chunk_buf<18>), ncu, 1024);
  RUN("chunk_buf aux19", (read_chunk_buf<19>), ncu, 1024);
  RUN("coal_buf aux0", (read_coal_buf<0>), ncu, 1024);
  RUN("coal_buf aux2 nt", (read_coal_buf<2>), ncu, 1024);
  RUN("coal_buf aux3", (read_coal_buf<3>), ncu, 1024);
  RUN("coal_buf aux16 sc1", (read_coal_buf<16>), ncu, 1024);
  RUN("coal_buf aux18", (read_coal_buf<18>), ncu, 1024);
  rep("fold_only chains1", timeit([&] { hipLaunchKernelGGL((fold_only<1>), dim3(ncu), dim3(1024), 0, 0, nblk, sink); }, 5));
  rep("fold_only chains2", timeit([&] { hipLaunchKernelGGL((fold_only<2>), dim3(ncu), dim3(1024), 0, 0, nblk, sink); }, 5));
  rep("fold_only chains4", timeit([&] { hipLaunchKernelGGL((fold_only<4>), dim3(ncu), dim3(1024), 0, 0, nblk, sink); }, 5));
  return 0;
}
