// Floor of reading C4's small packets where they lie: the 64-byte and
// 256-byte packets of a mixed-MTU batch (lengths uniform over 64/256/1024/4096,
// packed back to back, 5.3 GiB) read one lane per packet in 16-byte units,
// XOR-folded (no CRC), one word out per packet -- versus the same packets
// packed contiguously.  Tells whether the ragged path's small-packet kernels
// (~185 us for 2 M packets) are bound by the scattered DRAM accesses or by
// their own work.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 mb_scatter.hip -o mb_scatter && ./mb_scatter
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#include <algorithm>
#include <random>
#include <vector>

#include "../../roce-test_amd/csrc/icrc_device.h"
using namespace ricrc;

#define CK(x)                                                                  \
  do {                                                                         \
    hipError_t e_ = (x);                                                       \
    if (e_ != hipSuccess) {                                                    \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      exit(1);                                                                 \
    }                                                                          \
  } while (0)


// Lane per packet: UNITS 16-byte loads from base + off[i].
template <int UNITS>
__global__ __launch_bounds__(256) void read_lane(const uint8_t *base, const uint64_t *off, uint32_t n, uint32_t *out) {
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
    const u32x4 *p = reinterpret_cast<const u32x4 *>(base + off[i]);
    u32x4 acc = {0u, 0u, 0u, 0u};
#pragma unroll
    for (int k = 0; k < UNITS; ++k) acc ^= p[k];
    out[i] = acc[0] ^ acc[1] ^ acc[2] ^ acc[3];
  }
}

// 4 lanes per 64-byte piece, coalesced within the piece.
__global__ __launch_bounds__(256) void read_quad(const uint8_t *base, const uint64_t *off, uint32_t n, uint32_t pieces,
                                                 uint32_t *out) {
  const uint64_t total = (uint64_t)n * pieces * 4;
  for (uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; t < total; t += (uint64_t)gridDim.x * blockDim.x) {
    const uint64_t i = t / (pieces * 4), r = t % (pieces * 4);
    const u32x4 v = *reinterpret_cast<const u32x4 *>(base + off[i] + 16 * r);
    uint32_t x = v[0] ^ v[1] ^ v[2] ^ v[3];
    x ^= __shfl_xor(x, 1);
    x ^= __shfl_xor(x, 2);
    if ((t & 3) == 0) out[t >> 2] = x;
  }
}

// The ragged path's small-packet fold (icrc_rsck.hip icrc_rsmall_kernel,
// one lane per packet, end-aligned 16-byte blocks, ring of D units, LDS
// slice-by-4) on packets of ONE length n (K = ceil((n - 4 + 4) / 16) blocks,
// rounded to D), with ablations: ABL & 1 no table fold (XOR), ABL & 2 no
// loads (register data), ABL & 4 no realign funnel.
template <int ABL, int D>
__global__ __launch_bounds__(1024) void fold_lane(const uint8_t *base, const uint64_t *off, uint32_t count, uint32_t n,
                                                  uint32_t *out) {
  __shared__ uint32_t lds[kLdsWords];
  fill_tables(lds);
  __syncthreads();
  const uint32_t lane = threadIdx.x & 63;
  const LaneTab lt{(lane & 31) << 2, ((lane & 31) << 2) | 0x10000u};
  const uint32_t M = n - 4;
  const uint32_t Kmax = ((M + 4 + 15) / 16 + D - 1) / D * D;
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < count; i += gridDim.x * blockDim.x) {
    const uint64_t addr = (uint64_t)(uintptr_t)base + off[i];
    const uint64_t e = addr + M;
    const uint32_t t = (uint32_t)(e & 15u), sb = t & 3u;
    const uint32_t m2 = 0u - ((t >> 3) & 1u), m1 = 0u - ((t >> 2) & 1u);
    const uint64_t ufirst = addr & ~15ull, ulast = (e - 1u) & ~15ull;
    const uint64_t N0 = e - t - 16ull * Kmax;
    auto unit = [&](uint32_t k) -> u32x4 {
      if (ABL & 2) return u32x4{k, (uint32_t)addr, t, k * 7u};
      uint64_t u = N0 + 16ull * k;
      u = u < ufirst ? ufirst : (u > ulast ? ulast : u);
      return gload16(u);
    };
    u32x4 ring[D];
#pragma unroll
    for (int k = 0; k < D; ++k) {
      __builtin_amdgcn_sched_barrier(0);
      ring[k] = unit(k);
    }
    uint32_t reg = 0u;
    for (uint32_t j = 0; j < Kmax; j += D) {
#pragma unroll
      for (int u = 0; u < D; ++u) {
        __builtin_amdgcn_sched_barrier(0);
        const u32x4 c = ring[u], nn = ring[(u + 1) % D];
        uint32_t w[4];
        if (ABL & 4) {
          for (int q = 0; q < 4; ++q) w[q] = c[q] ^ nn[q];
        } else {
          const uint32_t W[8] = {c[0], c[1], c[2], c[3], nn[0], nn[1], nn[2], nn[3]};
          uint32_t V[6], X[5];
#pragma unroll
          for (int k = 0; k < 6; ++k) V[k] = __builtin_amdgcn_bitop3_b32(m2, W[k + 2], W[k], 0xCA);
#pragma unroll
          for (int k = 0; k < 5; ++k) X[k] = __builtin_amdgcn_bitop3_b32(m1, V[k + 1], V[k], 0xCA);
#pragma unroll
          for (int q = 0; q < 4; ++q) w[q] = __builtin_amdgcn_alignbyte(X[q + 1], X[q], sb);
        }
        __builtin_amdgcn_sched_barrier(0);
        ring[u] = unit(j + u + D);
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int q = 0; q < 4; ++q) reg = (ABL & 1) ? ((reg ^ w[q]) * 3u) : step4(lds, lt, reg, w[q]);
      }
    }
    out[i] = ~reg;
  }
}

// Load-all variant: the packet's KM + 1 units are all requested up front
// (statically unrolled), then folded -- the memory-level parallelism of
// read_lane.
template <int KM, bool MASK = false>
__global__ __launch_bounds__(1024) void fold_all(const uint8_t *base, const uint64_t *off, uint32_t count, uint32_t n,
                                                 uint32_t *out) {
  __shared__ uint32_t lds[kLdsWords];
  fill_tables(lds);
  __syncthreads();
  const uint32_t lane = threadIdx.x & 63;
  const LaneTab lt{(lane & 31) << 2, ((lane & 31) << 2) | 0x10000u};
  const uint32_t M = n - 4;
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < count; i += gridDim.x * blockDim.x) {
    const uint64_t addr = (uint64_t)(uintptr_t)base + off[i];
    const uint64_t e = addr + M;
    const uint32_t t = (uint32_t)(e & 15u), sb = t & 3u;
    const uint32_t m2 = 0u - ((t >> 3) & 1u), m1 = 0u - ((t >> 2) & 1u);
    const uint64_t ufirst = addr & ~15ull, ulast = (e - 1u) & ~15ull;
    const uint64_t N0 = e - t - 16ull * KM;
    u32x4 U[KM + 1];
#pragma unroll
    for (int k = 0; k <= KM; ++k) {
      uint64_t u = N0 + 16ull * k;
      u = u < ufirst ? ufirst : (u > ulast ? ulast : u);
      U[k] = gload16(u);
    }
    uint32_t reg = 0u;
#pragma unroll
    for (int j = 0; j < KM; ++j) {
      const u32x4 c = U[j], nn = U[j + 1];
      const uint32_t W[8] = {c[0], c[1], c[2], c[3], nn[0], nn[1], nn[2], nn[3]};
      uint32_t V[6], X[5], w[4];
#pragma unroll
      for (int k = 0; k < 6; ++k) V[k] = __builtin_amdgcn_bitop3_b32(m2, W[k + 2], W[k], 0xCA);
#pragma unroll
      for (int k = 0; k < 5; ++k) X[k] = __builtin_amdgcn_bitop3_b32(m1, V[k + 1], V[k], 0xCA);
#pragma unroll
      for (int q = 0; q < 4; ++q) w[q] = __builtin_amdgcn_alignbyte(X[q + 1], X[q], sb);
      if (MASK) {
        const int rel = (int)M - 16 * KM + 16 * j;
        if (__builtin_amdgcn_ballot_w64(rel < 40) != 0) {
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            const int r = rel + 4 * q;
            const uint32_t keep = (uint32_t)(r >= 0) * 0xFFFFFFFFu;
            const uint32_t orm = ((uint32_t)(r == -4) * 0xFFFFFFFFu) | ((uint32_t)(r == 0) * 0xFF00u) |
                                 ((uint32_t)(r == 8) * 0xFFFF00FFu) | ((uint32_t)(r == 24) * 0xFFFF0000u) |
                                 ((uint32_t)(r == 32) * 0xFFu);
            w[q] = (w[q] & keep) | orm;
          }
        }
      }
#pragma unroll
      for (int q = 0; q < 4; ++q) reg = step4(lds, lt, reg, w[q]);
    }
    out[i] = ~reg;
  }
}

__global__ void flush_kernel(const u32x4 *p, uint64_t n16, uint32_t *sink) {
  u32x4 acc = {0u, 0u, 0u, 0u};
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n16; i += (uint64_t)gridDim.x * blockDim.x)
    acc ^= p[i];
  if ((acc[0] ^ acc[1] ^ acc[2] ^ acc[3]) == 0x12345678u) sink[0] = 1;
}
static const u32x4 *g_flush;
static uint32_t *g_sink;
static const uint64_t kFlushBytes = 1ull << 30;  // 4x the 256 MB Infinity Cache
static void flush() { flush_kernel<<<2048, 256>>>(g_flush, kFlushBytes / 16, g_sink); }

template <class F>
float timeit_cold(F f, int reps = 20);

template <class F>
float timeit(F f, int reps = 20) {
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  for (int i = 0; i < 5; ++i) f();
  CK(hipEventRecord(a));
  for (int i = 0; i < reps; ++i) f();
  CK(hipEventRecord(b));
  CK(hipEventSynchronize(b));
  float ms;
  CK(hipEventElapsedTime(&ms, a, b));
  return ms * 1000.f / reps;
}

// Each launch after a 1 GiB streaming read (caches cold, as after the
// ragged path's big-packet fold); the flush alone is timed and subtracted.
template <class F>
float timeit_cold(F f, int reps) {
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  auto run = [&](bool with) {
    for (int i = 0; i < 3; ++i) { flush(); if (with) f(); }
    CK(hipEventRecord(a));
    for (int i = 0; i < reps; ++i) { flush(); if (with) f(); }
    CK(hipEventRecord(b));
    CK(hipEventSynchronize(b));
    float ms;
    CK(hipEventElapsedTime(&ms, a, b));
    return ms * 1000.f / reps;
  };
  const float both = run(true), alone = run(false);
  return both - alone;
}

int main() {
  const uint32_t count = 4u << 20;
  std::mt19937_64 rng(0x1CEC0DE);
  const uint32_t sizes[4] = {64, 256, 1024, 4096};
  std::vector<uint32_t> len(count);
  std::vector<uint64_t> off(count);
  uint64_t at = 0;
  for (uint32_t i = 0; i < count; ++i) {
    len[i] = sizes[rng() & 3];
    off[i] = at;
    at += len[i];
  }
  std::vector<uint64_t> o64, o256, c64, c256;
  for (uint32_t i = 0; i < count; ++i) {
    if (len[i] == 64) o64.push_back(off[i]);
    if (len[i] == 256) o256.push_back(off[i]);
  }
  // class-bucket order of the ragged path's scatter pass: ascending by pass
  // block, shuffled within windows of ~256 packets of a class (LDS atomics)
  std::vector<uint64_t> s64 = o64, s256 = o256;
  for (size_t w = 0; w < s64.size(); w += 256) std::shuffle(s64.begin() + w, s64.begin() + std::min(s64.size(), w + 256), rng);
  for (size_t w = 0; w < s256.size(); w += 256) std::shuffle(s256.begin() + w, s256.begin() + std::min(s256.size(), w + 256), rng);
  for (size_t i = 0; i < o64.size(); ++i) c64.push_back(64ull * i);
  for (size_t i = 0; i < o256.size(); ++i) c256.push_back(256ull * i);
  uint8_t *buf;
  CK(hipMalloc(&buf, at));
  CK(hipMemset(buf, 0x5A, at));
  uint64_t *d64, *d256, *dc64, *dc256, *ds64, *ds256;
  uint32_t *out;
  CK(hipMalloc(&d64, o64.size() * 8));
  CK(hipMalloc(&d256, o256.size() * 8));
  CK(hipMalloc(&dc64, c64.size() * 8));
  CK(hipMalloc(&ds64, s64.size() * 8));
  CK(hipMalloc(&ds256, s256.size() * 8));
  CK(hipMemcpy(ds64, s64.data(), s64.size() * 8, hipMemcpyHostToDevice));
  CK(hipMemcpy(ds256, s256.data(), s256.size() * 8, hipMemcpyHostToDevice));
  CK(hipMalloc(&dc256, c256.size() * 8));
  CK(hipMalloc(&out, (size_t)count * 16 * 4));
  CK(hipMemcpy(d64, o64.data(), o64.size() * 8, hipMemcpyHostToDevice));
  CK(hipMemcpy(d256, o256.data(), o256.size() * 8, hipMemcpyHostToDevice));
  CK(hipMemcpy(dc64, c64.data(), c64.size() * 8, hipMemcpyHostToDevice));
  CK(hipMemcpy(dc256, c256.data(), c256.size() * 8, hipMemcpyHostToDevice));
  const uint32_t n64 = (uint32_t)o64.size(), n256 = (uint32_t)o256.size();
  const dim3 g(4096), b(256);
  CK(hipMalloc((void **)&g_flush, kFlushBytes));
  CK(hipMemset((void *)g_flush, 1, kFlushBytes));
  CK(hipMalloc(&g_sink, 4));
  printf("batch %.2f GiB, %u x 64 B, %u x 256 B\n", at / 1073741824.0, n64, n256);
  printf("64 B  lane  scattered(C4) %.1f us   contiguous %.1f us\n",
         timeit([&] { read_lane<4><<<g, b>>>(buf, d64, n64, out); }),
         timeit([&] { read_lane<4><<<g, b>>>(buf, dc64, n64, out); }));
  printf("256 B lane  scattered(C4) %.1f us   contiguous %.1f us\n",
         timeit([&] { read_lane<16><<<g, b>>>(buf, d256, n256, out); }),
         timeit([&] { read_lane<16><<<g, b>>>(buf, dc256, n256, out); }));
  printf("64 B  quad  scattered(C4) %.1f us   contiguous %.1f us\n",
         timeit([&] { read_quad<<<g, b>>>(buf, d64, n64, 1, out); }),
         timeit([&] { read_quad<<<g, b>>>(buf, dc64, n64, 1, out); }));
  printf("256 B quad  scattered(C4) %.1f us   contiguous %.1f us\n",
         timeit([&] { read_quad<<<g, b>>>(buf, d256, n256, 4, out); }),
         timeit([&] { read_quad<<<g, b>>>(buf, dc256, n256, 4, out); }));
  const dim3 fg(256), fb(1024);
#define FOLD(ABL, D)                                                                                   \
  printf("fold ABL=%d D=%d: 64 B %.1f us, 256 B %.1f us (scattered)\n", ABL, D,                       \
         timeit([&] { fold_lane<ABL, D><<<fg, fb>>>(buf, d64, n64, 64, out); }),                       \
         timeit([&] { fold_lane<ABL, D><<<fg, fb>>>(buf, d256, n256, 256, out); }));
  printf("fold_all: 64 B %.1f us, 256 B %.1f us (scattered); 256 B contiguous %.1f us\n",
         timeit([&] { fold_all<4><<<fg, fb>>>(buf, d64, n64, 64, out); }),
         timeit([&] { fold_all<16><<<fg, fb>>>(buf, d256, n256, 256, out); }),
         timeit([&] { fold_all<16><<<fg, fb>>>(buf, dc256, n256, 256, out); }));
  printf("COLD read_lane scattered: 64 B %.1f us, 256 B %.1f us; contiguous 64 B %.1f us, 256 B %.1f us\n",
         timeit_cold([&] { read_lane<4><<<g, b>>>(buf, d64, n64, out); }, 20),
         timeit_cold([&] { read_lane<16><<<g, b>>>(buf, d256, n256, out); }, 20),
         timeit_cold([&] { read_lane<4><<<g, b>>>(buf, dc64, n64, out); }, 20),
         timeit_cold([&] { read_lane<16><<<g, b>>>(buf, dc256, n256, out); }, 20));
  printf("COLD fold_all scattered: 64 B %.1f us, 256 B %.1f us\n",
         timeit_cold([&] { fold_all<4><<<fg, fb>>>(buf, d64, n64, 64, out); }, 20),
         timeit_cold([&] { fold_all<16><<<fg, fb>>>(buf, d256, n256, 256, out); }, 20));
  printf("COLD fold_all + head masks: 64 B %.1f us, 256 B %.1f us\n",
         timeit_cold([&] { fold_all<4, true><<<fg, fb>>>(buf, d64, n64, 64, out); }, 20),
         timeit_cold([&] { fold_all<16, true><<<fg, fb>>>(buf, d256, n256, 256, out); }, 20));
  printf("COLD fold ring D=4 scattered: 64 B %.1f us, 256 B %.1f us\n",
         timeit_cold([&] { fold_lane<0, 4><<<fg, fb>>>(buf, d64, n64, 64, out); }, 20),
         timeit_cold([&] { fold_lane<0, 4><<<fg, fb>>>(buf, d256, n256, 256, out); }, 20));
  printf("fold_all, window-shuffled order: 64 B %.1f us, 256 B %.1f us\n",
         timeit([&] { fold_all<4><<<fg, fb>>>(buf, ds64, n64, 64, out); }),
         timeit([&] { fold_all<16><<<fg, fb>>>(buf, ds256, n256, 256, out); }));
  printf("read_lane, window-shuffled order: 64 B %.1f us, 256 B %.1f us\n",
         timeit([&] { read_lane<4><<<g, b>>>(buf, ds64, n64, out); }),
         timeit([&] { read_lane<16><<<g, b>>>(buf, ds256, n256, out); }));
  FOLD(0, 4) FOLD(1, 4) FOLD(2, 4) FOLD(4, 4) FOLD(5, 4) FOLD(3, 4) FOLD(0, 2) FOLD(0, 8)
  printf("both, lane, scattered: %.1f us\n", timeit([&] {
           read_lane<4><<<g, b>>>(buf, d64, n64, out);
           read_lane<16><<<g, b>>>(buf, d256, n256, out + n64);
         }));
  return 0;
}
