// Attribution of the ragged path's bucket pass (rsck_bucket) on a C4-shaped
// batch: 4 M packets, lengths uniform over {64, 256, 1024, 4096}, packed back
// to back (the bench's --mix layout).  Timing only.  Cumulative stops:
//   loads + classify | + LDS ranking atomics | + scan and pool reservation |
//   full | full without pos_of stores | full without descriptor stores,
// next to a plain copy of the same descriptor bytes (12 B in, 12 B out per
// packet) and the other passes of the pipeline over a group-cost sweep.  Build:
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 bucket_abl.hip -o bucket_abl
#include "../../roce-test_amd/csrc/icrc_kernels.hip"
#include "../../roce-test_amd/csrc/icrc_rsck.hip"
#include "mb_fin.h"
#include <stdio.h>
#include <stdlib.h>
#include <string>
#include <vector>
#include <algorithm>
using namespace ricrc;
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s\n", hipGetErrorString(e)); exit(1); } } while (0)

template <typename F> float timeit(F launch, int reps) {
  hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  for (int w = 0; w < 3; ++w) launch();
  CK(hipDeviceSynchronize()); CK(hipEventRecord(e0));
  for (int i = 0; i < reps; ++i) launch();
  CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1)); float ms; CK(hipEventElapsedTime(&ms, e0, e1));
  return ms / reps;
}

// The floor: read each packet's offset and length, write 8 + 4 bytes at the
// packet's own index (coalesced), 16 packets per thread, same grid.
__global__ __launch_bounds__(1024) void copy_floor(const uint64_t *off, const uint32_t *len, uint64_t count,
                                                    RsDesc *d, uint32_t *pos) {
  const uint64_t T = (uint64_t)gridDim.x * blockDim.x;
  uint64_t o[16]; uint32_t n[16];
#pragma unroll
  for (int k = 0; k < 16; ++k) {
    uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x + k * T;
    i = i < count ? i : count - 1;
    o[k] = off[i]; n[k] = len[i];
  }
#pragma unroll
  for (int k = 0; k < 16; ++k) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x + k * T;
    if (i >= count) break;
    __builtin_nontemporal_store((uint32_t)o[k], &d[i].lo);
    __builtin_nontemporal_store((uint32_t)(o[k] >> 32) | (n[k] << 16), &d[i].hi);
    __builtin_nontemporal_store((uint32_t)i, &pos[i]);
  }
}

__global__ void fill_random(uint64_t *p, uint64_t n) {
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
    uint64_t x = (i + 1) * 0x9E3779B97F4A7C15ull;
    x ^= x >> 31; x *= 0xBF58476D1CE4E5B9ull; x ^= x >> 27;
    p[i] = x;
  }
}

int main(int argc, char **argv) {
  hipDeviceProp_t p; CK(hipGetDeviceProperties(&p, 0));
  const int grid = p.multiProcessorCount;
  // "shard": C4's 8-GPU shard, 524,288 packets, on the product's pass shape (U = 4, 128 blocks)
  const bool shard = argc > 1 && std::string(argv[1]) == "shard";
  const uint64_t count = shard ? 524288ull : 4ull << 20;
  std::vector<uint64_t> off(count); std::vector<uint32_t> len(count);
  uint64_t x = 0x1234567ull, pos = 0;
  const uint32_t sizes[4] = {64, 256, 1024, 4096};
  for (uint64_t i = 0; i < count; ++i) {
    x ^= x << 13; x ^= x >> 7; x ^= x << 17;
    off[i] = pos; len[i] = sizes[x & 3]; pos += len[i];
  }
  uint8_t *buf; CK(hipMalloc(&buf, pos + 4096));
  // random bytes (constant data can run at another clock than real traffic)
  hipLaunchKernelGGL(fill_random, dim3(4096), dim3(256), 0, 0, reinterpret_cast<uint64_t *>(buf), (pos + 4096) / 8);
  CK(hipDeviceSynchronize());
  uint64_t *d_off; uint32_t *d_len;
  CK(hipMalloc(&d_off, 8 * count)); CK(hipMalloc(&d_len, 4 * count));
  CK(hipMemcpy(d_off, off.data(), 8 * count, hipMemcpyHostToDevice));
  CK(hipMemcpy(d_len, len.data(), 4 * count, hipMemcpyHostToDevice));
  uint32_t *out; CK(hipMalloc(&out, 4 * count));
  uint32_t *tzb; CK(hipMalloc(&tzb, 4 * 1024)); CK(hipMemset(tzb, 0x35, 4 * 1024));
  RsckArgs a{};
  a.base = buf; a.off = d_off; a.len = d_len; a.count = count; a.out = out; a.tzb = tzb; a.group_cost = kRsGroupCost;
  a.fin = mb_fin();
  void *ws; CK(hipMalloc(&ws, rs_workspace_bytes(count)));
  CK(rs_zero_counters(ws, 0));
  rs_bind_workspace(a, ws);
  const int pgrid = shard ? 128 : kPassBlocks;
  a.nblk = pgrid;
  printf("C4-shaped batch: %llu packets, %llu B; pass grid %d x %d, fold grid %d\n", (unsigned long long)count,
         (unsigned long long)pos, pgrid, kPassBlock, grid);
  {  // out of the idle power state
    for (int i = 0; i < 200; ++i) hipLaunchKernelGGL(copy_floor, dim3(256), dim3(1024), 0, 0, d_off, d_len, count, a.desc, a.pos_of);
    CK(hipDeviceSynchronize());
  }
  auto rep = [&](const char *nm, float ms) { printf("%-52s %8.2f us\n", nm, ms * 1e3); };
  // every variant starts from zeroed counters (the product's gather zeroes them)
  auto bucket = [&](auto abl) {
    constexpr int ABL = decltype(abl)::value;
    return timeit([&] {
      CK(rs_zero_counters(ws, 0));
      if (shard) hipLaunchKernelGGL((rsck_bucket<true, true, ABL, 4>), dim3(pgrid), dim3(kPassBlock), 0, 0, a);
      else hipLaunchKernelGGL((rsck_bucket<true, true, ABL>), dim3(pgrid), dim3(kPassBlock), 0, 0, a);
    }, 20);
  };
  const float zero = timeit([&] { CK(rs_zero_counters(ws, 0)); }, 20);
  for (int r = 0; r < 3; ++r) {
    printf("-- round %d (bucket rows include a %.2f us counter memset)\n", r, zero * 1e3);
    rep("copy floor (12 B in, 12 B out per packet)", timeit([&] {
      hipLaunchKernelGGL(copy_floor, dim3(256), dim3(1024), 0, 0, d_off, d_len, count, a.desc, a.pos_of); }, 20));
    rep("bucket: loads + classify", bucket(std::integral_constant<int, 1 | 2>{}));
    rep("bucket: + LDS ranking atomics", bucket(std::integral_constant<int, 1>{}));
    rep("bucket: + scan + pool reservation", bucket(std::integral_constant<int, 4>{}));
    rep("bucket: full (LDS-staged layout)", bucket(std::integral_constant<int, 0>{}));
    rep("bucket: full, no LDS staging (stores from registers)", bucket(std::integral_constant<int, 32>{}));
    rep("bucket: full, no pos_of stores", bucket(std::integral_constant<int, 8>{}));
    rep("bucket: full, no descriptor stores", bucket(std::integral_constant<int, 16>{}));
    rep("bucket: full, no stores", bucket(std::integral_constant<int, 8 | 16>{}));
    rep("bucket: no staging, no pos_of stores", bucket(std::integral_constant<int, 32 | 8>{}));
    rep("bucket: no staging, no descriptor stores", bucket(std::integral_constant<int, 32 | 16>{}));
    if (shard) continue;  // (the rest times the 4 M layout's other passes)
    // the rest of the pipeline on the product's layout
    CK(rs_zero_counters(ws, 0));
    hipLaunchKernelGGL((rsck_bucket<true, true, 0>), dim3(pgrid), dim3(kPassBlock), 0, 0, a);
    CK(hipDeviceSynchronize());
    auto fold_report = [&](uint32_t gc) {
      a.group_cost = gc;
      CK(rs_zero_counters(ws, 0));
      hipLaunchKernelGGL((rsck_bucket<true, true, 0>), dim3(pgrid), dim3(kPassBlock), 0, 0, a);
      CK(hipDeviceSynchronize());
      char nm[96]; snprintf(nm, sizeof nm, "fold (icrc_rsck_kernel), group cost %u", gc);
      rep(nm, timeit([&] { hipLaunchKernelGGL((icrc_rsck_kernel<0>), dim3(grid), dim3(kBlock), 0, 0, a); }, 10));
    };
    if (r == 0) for (uint32_t gc : {4u, 8u, 16u}) fold_report(gc);
    fold_report(kRsGroupCost);
    // (the fold's per-wave timeline: tools/microbench/shard.hip, ABL 524288)
    rep("fold, no line loads (compute only)", timeit([&] { hipLaunchKernelGGL((icrc_rsck_kernel<16384>), dim3(grid), dim3(kBlock), 0, 0, a); }, 10));
    rep("fold, memory path (no table fold, no finish)", timeit([&] { hipLaunchKernelGGL((icrc_rsck_kernel<3>), dim3(grid), dim3(kBlock), 0, 0, a); }, 10));
    rep("fold, no edge masks", timeit([&] { hipLaunchKernelGGL((icrc_rsck_kernel<8>), dim3(grid), dim3(kBlock), 0, 0, a); }, 10));
    rep("fold, no finish", timeit([&] { hipLaunchKernelGGL((icrc_rsck_kernel<2>), dim3(grid), dim3(kBlock), 0, 0, a); }, 10));
    rep("fold, memory path, no edges, no stores", timeit([&] { hipLaunchKernelGGL((icrc_rsck_kernel<3 | 8 | 16>), dim3(grid), dim3(kBlock), 0, 0, a); }, 10));
    rep("one-line (icrc_rsmall_kernel)", timeit([&] { hipLaunchKernelGGL((icrc_rsmall_kernel), dim3(grid), dim3(kBlock), 0, 0, a); }, 20));
    {  // the gather zeroes the counters: restore them before each timed launch
      RsCounters *saved; CK(hipMalloc(&saved, sizeof(RsCounters)));
      CK(hipMemcpy(saved, a.ctr, sizeof(RsCounters), hipMemcpyDeviceToDevice));
      hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
      float tot = 0;
      for (int it = 0; it < 23; ++it) {
        CK(hipMemcpyAsync(a.ctr, saved, sizeof(RsCounters), hipMemcpyDeviceToDevice, 0));
        CK(hipEventRecord(e0, 0));
        hipLaunchKernelGGL((rsck_gather<kPassUnroll, false>), dim3(pgrid), dim3(kPassBlock), 0, 0, a);
        CK(hipEventRecord(e1, 0)); CK(hipEventSynchronize(e1));
        float ms; CK(hipEventElapsedTime(&ms, e0, e1));
        if (it >= 3) tot += ms;
      }
      rep("gather (one launch between events)", tot / 20);
      CK(hipFree(saved));
    }
  }
  {  // placement: the same batch at a second address (a second 5.7 GB allocation), fold on each, alternating
    uint8_t *buf2; CK(hipMalloc(&buf2, pos + 4096));
    CK(hipMemcpy(buf2, buf, pos + 4096, hipMemcpyDeviceToDevice));
    printf("placement: batch A at %p, batch B at %p\n", (void *)buf, (void *)buf2);
    for (int r = 0; r < 4; ++r) {
      for (int which = 0; which < 2; ++which) {
        a.base = which ? buf2 : buf;
        a.group_cost = kRsGroupCost;
        CK(rs_zero_counters(ws, 0));
        hipLaunchKernelGGL((rsck_bucket<true, true, 0>), dim3(pgrid), dim3(kPassBlock), 0, 0, a);
        CK(hipDeviceSynchronize());
        rep(which ? "placement: fold on batch B" : "placement: fold on batch A",
            timeit([&] { hipLaunchKernelGGL((icrc_rsck_kernel<0>), dim3(grid), dim3(kBlock), 0, 0, a); }, 10));
      }
    }
    a.base = buf;
    CK(hipFree(buf2));
  }
  return 0;
}