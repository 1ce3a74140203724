// The memory floor of a NIC ring with a length per slot: read exactly the
// 128-byte lines each packet covers (L3 at 14, the ICRC's bytes), in the
// fused kernel's pattern (a wave load = line k of 8 slots, lane 8 g + s
// reading 16 bytes), with every line of a group issued before any is used
// (up to 32 loads in flight a wave), on one 1024-thread workgroup per CU.
// Timing only: no CRC, the bytes XOR-reduced into a sink.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 ring_floor.hip -o ring_floor
//   ./ring_floor slot lo hi [count]
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#include <algorithm>
#include <vector>
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s line %d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

// MAXL: the slot's lines (8 for 1 KiB); groups of 8 consecutive slots per
// wave in a grid-contiguous share.
template <int MAXL>
__global__ __launch_bounds__(1024) void ring_lines(const uint8_t *p, const uint32_t *len, uint64_t count,
                                                   uint32_t slot, uint32_t *sink) {
  const uint64_t nw = (uint64_t)gridDim.x * 16, w = (uint64_t)blockIdx.x * 16 + (threadIdx.x >> 6);
  const uint32_t lane = threadIdx.x & 63, g = lane >> 3, s = lane & 7;
  const uint64_t groups = count / 8, per = (groups + nw - 1) / nw;
  const uint64_t q0 = w * per, q1 = q0 + per < groups ? q0 + per : groups;
  u32x4 acc = {0, 0, 0, 0};
  for (uint64_t q = q0; q < q1; ++q) {
    const uint64_t i = 8 * q + g;
    const uint64_t a0 = i * slot + 14u;
    const uint32_t L = (uint32_t)(((a0 & 127u) + len[i] - 4u + 127u) >> 7);
    const uint8_t *b = p + (a0 & ~127ull) + 16u * s;
    u32x4 v[MAXL];
#pragma unroll
    for (int k = 0; k < MAXL; ++k) {
      v[k] = u32x4{0, 0, 0, 0};
      if ((uint32_t)k < L) v[k] = __builtin_nontemporal_load(reinterpret_cast<const u32x4 *>(b + 128u * k));
    }
#pragma unroll
    for (int k = 0; k < MAXL; ++k) acc ^= v[k];
  }
  const uint32_t x = acc[0] ^ acc[1] ^ acc[2] ^ acc[3];
  if (x == 0x12345678u) sink[0] = x;
}

// The same lines in the fused kernel's layout order: within each chunk of
// 2304 slots, the packets sorted by line count (class), groups of 8 of one
// class; idx[] holds the slot of each layout position (host-built: by class,
// then either in slot order or shuffled within the class as the LDS
// atomics leave them).
template <int MAXL>
__global__ __launch_bounds__(1024) void ring_lines_idx(const uint8_t *p, const uint32_t *len, const uint32_t *idx,
                                                       uint64_t count, uint32_t slot, uint32_t *sink) {
  const uint64_t nw = (uint64_t)gridDim.x * 16, w = (uint64_t)blockIdx.x * 16 + (threadIdx.x >> 6);
  const uint32_t lane = threadIdx.x & 63, g = lane >> 3, s = lane & 7;
  const uint64_t groups = count / 8, per = (groups + nw - 1) / nw;
  const uint64_t q0 = w * per, q1 = q0 + per < groups ? q0 + per : groups;
  u32x4 acc = {0, 0, 0, 0};
  for (uint64_t q = q0; q < q1; ++q) {
    const uint64_t i = idx[8 * q + g];
    const uint64_t a0 = i * slot + 14u;
    const uint32_t L = (uint32_t)(((a0 & 127u) + len[i] - 4u + 127u) >> 7);
    const uint8_t *b = p + (a0 & ~127ull) + 16u * s;
    u32x4 v[MAXL];
#pragma unroll
    for (int k = 0; k < MAXL; ++k) {
      v[k] = u32x4{0, 0, 0, 0};
      if ((uint32_t)k < L) v[k] = __builtin_nontemporal_load(reinterpret_cast<const u32x4 *>(b + 128u * k));
    }
#pragma unroll
    for (int k = 0; k < MAXL; ++k) acc ^= v[k];
  }
  const uint32_t x = acc[0] ^ acc[1] ^ acc[2] ^ acc[3];
  if (x == 0x12345678u) sink[0] = x;
}

int main(int argc, char **argv) {
  if (argc < 4) { printf("usage: ring_floor slot lo hi [count]\n"); return 2; }
  const uint32_t slot = (uint32_t)atoi(argv[1]), lo = (uint32_t)atoi(argv[2]), hi = (uint32_t)atoi(argv[3]);
  const uint64_t count = argc > 4 ? strtoull(argv[4], nullptr, 0) : (1ull << 20);
  hipDeviceProp_t prop; CK(hipGetDeviceProperties(&prop, 0));
  const int grid = prop.multiProcessorCount;
  std::vector<uint32_t> len(count);
  uint64_t x = 0x1CEC0DEull, bytes = 0, lines = 0;
  for (uint64_t i = 0; i < count; ++i) {
    x = x * 6364136223846793005ull + 1442695040888963407ull;
    len[i] = lo + (uint32_t)((x >> 33) % (hi - lo + 1));
    bytes += len[i];
    lines += ((14u + len[i] - 4u + 127u) >> 7);
  }
  uint8_t *d; uint32_t *dl, *sink;
  CK(hipMalloc(&d, count * slot + 256)); CK(hipMalloc(&dl, 4 * count)); CK(hipMalloc(&sink, 4));
  CK(hipMemset(d, 0x5A, count * slot + 256));
  CK(hipMemcpy(dl, len.data(), 4 * count, hipMemcpyHostToDevice));
  const double alg = (double)bytes + 8.0 * count;
  printf("ring: %llu slots of %u B, lengths %u-%u, %.1f MB of packets, %.2f lines a packet, %.1f MB of lines; alg %.1f MB\n",
         (unsigned long long)count, slot, lo, hi, bytes / 1e6, (double)lines / count, lines * 128.0 / 1e6, alg / 1e6);
  auto launch = [&]() {
    if (slot <= 1024) hipLaunchKernelGGL((ring_lines<8>), dim3(grid), dim3(1024), 0, 0, d, dl, count, slot, sink);
    else if (slot <= 2048) hipLaunchKernelGGL((ring_lines<16>), dim3(grid), dim3(1024), 0, 0, d, dl, count, slot, sink);
    else hipLaunchKernelGGL((ring_lines<32>), dim3(grid), dim3(1024), 0, 0, d, dl, count, slot, sink);
  };
  hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  for (int r = 0; r < 3; ++r) {
    for (int w = 0; w < 5; ++w) launch();
    CK(hipDeviceSynchronize()); CK(hipEventRecord(e0));
    const int reps = 20;
    for (int i = 0; i < reps; ++i) launch();
    CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
    float ms; CK(hipEventElapsedTime(&ms, e0, e1)); ms /= reps;
    printf("  lines read, every line of a group in flight: %.1f us (alg %.3f of 8 TB/s; lines at %.2f TB/s)\n",
           ms * 1e3, alg / (ms * 1e-3) / 8e12, lines * 128.0 / (ms * 1e-3) / 1e12);
  }
  // layout orders: by class within chunks of 2304 slots (one workgroup's
  // chunk), in slot order or shuffled within the class
  for (int shuffled = 0; shuffled < 2; ++shuffled) {
    std::vector<uint32_t> idx(count);
    uint64_t rs = 0x9E3779B97F4A7C15ull;
    for (uint64_t c0 = 0; c0 < count; c0 += 2304) {
      const uint64_t c1 = c0 + 2304 < count ? c0 + 2304 : count;
      std::vector<std::vector<uint32_t>> by(64);
      for (uint64_t i = c0; i < c1; ++i) by[(14u + len[i] - 4u + 127u) >> 7].push_back((uint32_t)i);
      uint64_t o = c0;
      for (int L = 63; L >= 0; --L) {
        auto &v = by[L];
        if (shuffled)
          for (size_t j = v.size(); j > 1; --j) {
            rs = rs * 6364136223846793005ull + 1442695040888963407ull;
            std::swap(v[j - 1], v[(rs >> 33) % j]);
          }
        for (uint32_t x : v) idx[o++] = x;
      }
    }
    uint32_t *di; CK(hipMalloc(&di, 4 * count));
    CK(hipMemcpy(di, idx.data(), 4 * count, hipMemcpyHostToDevice));
    auto li = [&]() {
      if (slot <= 1024) hipLaunchKernelGGL((ring_lines_idx<8>), dim3(grid), dim3(1024), 0, 0, d, dl, di, count, slot, sink);
      else hipLaunchKernelGGL((ring_lines_idx<16>), dim3(grid), dim3(1024), 0, 0, d, dl, di, count, slot, sink);
    };
    for (int r = 0; r < 2; ++r) {
      for (int w = 0; w < 5; ++w) li();
      CK(hipDeviceSynchronize()); CK(hipEventRecord(e0));
      const int reps = 20;
      for (int i = 0; i < reps; ++i) li();
      CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
      float ms; CK(hipEventElapsedTime(&ms, e0, e1)); ms /= reps;
      printf("  class order (%s within a class): %.1f us (alg %.3f of 8 TB/s)\n", shuffled ? "shuffled" : "slot order",
             ms * 1e3, alg / (ms * 1e-3) / 8e12);
    }
    CK(hipFree(di));
  }
  return 0;
}
