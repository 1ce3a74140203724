// Ablation timing of the ragged kernel on the C4 mix (timing only: outputs
// are meaningless for ABL != 0).
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 ragged_abl.hip -o ragged_abl
#include "../../roce-test_amd/csrc/icrc_kernels.hip"
#include <stdio.h>
#include <stdlib.h>
#include <vector>
using namespace ricrc;
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s\n", hipGetErrorString(e)); exit(1); } } while (0)
template <int MODE, int ABL> float run(RaggedArgs a, int grid, int reps) {
  hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  hipLaunchKernelGGL((icrc_ragged_kernel<MODE, 1024, ABL>), dim3(grid), dim3(1024), 0, 0, a);
  CK(hipDeviceSynchronize()); CK(hipEventRecord(e0));
  for (int i = 0; i < reps; ++i) hipLaunchKernelGGL((icrc_ragged_kernel<MODE, 1024, ABL>), dim3(grid), dim3(1024), 0, 0, a);
  CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1)); float ms; CK(hipEventElapsedTime(&ms, e0, e1)); return ms / reps;
}
int main(int argc, char **argv) {
  const bool only_full = argc > 1;  // counters: one variant only
  const uint64_t count = 4 << 20;
  std::vector<uint32_t> len(count);
  std::vector<uint64_t> off(count), ps(count + 1);
  uint64_t x = 0x9E3779B97F4A7C15ull, pos = 0;
  const uint32_t sizes[4] = {64, 256, 1024, 4096};
  for (uint64_t i = 0; i < count; ++i) {
    x ^= x << 13; x ^= x >> 7; x ^= x << 17;
    len[i] = sizes[x & 3]; off[i] = pos; pos += len[i];
    ps[i + 1] = ps[i] + ragged_pieces(0, len[i]);
  }
  uint8_t *buf; uint32_t *out, *inv; uint64_t *d_off, *d_ps; uint32_t *d_len;
  CK(hipMalloc(&buf, pos + 64)); CK(hipMalloc(&out, 4 * count)); CK(hipMalloc(&inv, 4 * 4097));
  CK(hipMalloc(&d_off, 8 * count)); CK(hipMalloc(&d_ps, 8 * (count + 1))); CK(hipMalloc(&d_len, 4 * count));
  {
    std::vector<uint64_t> h((pos + 64) / 8);
    for (auto &v : h) { x ^= x << 13; x ^= x >> 7; x ^= x << 17; v = x; }
    CK(hipMemcpy(buf, h.data(), h.size() * 8, hipMemcpyHostToDevice));
  }
  CK(hipMemset(inv, 0x5A, 4 * 4097));
  CK(hipMemcpy(d_off, off.data(), 8 * count, hipMemcpyHostToDevice));
  CK(hipMemcpy(d_len, len.data(), 4 * count, hipMemcpyHostToDevice));
  CK(hipMemcpy(d_ps, ps.data(), 8 * (count + 1), hipMemcpyHostToDevice));
  hipDeviceProp_t p; CK(hipGetDeviceProperties(&p, 0));
  RaggedArgs a{}; a.base = buf; a.off = d_off; a.len = d_len; a.ps = d_ps; a.count = count; a.out = out;
  a.inv_tab = inv;
  u32x4_t *inv4; CK(hipMalloc(&inv4, 16 * 4097)); CK(hipMemset(inv4, 0x3C, 16 * 4097)); a.inv4 = inv4;
  for (int l = 0; l < 64; ++l) a.K[l] = gf_x8n(64ull * (63 - l));
  const int grid = p.multiProcessorCount;
  auto rep = [&](const char *nm, float ms) { printf("%-40s %7.3f ms  %7.1f GB/s\n", nm, ms, pos / (ms * 1e-3) / 1e9); };
  rep("full", run<1, 0>(a, grid, 10));
  if (only_full) return 0;
  rep("full", run<1, 0>(a, grid, 10));
  rep("no fold", run<1, 1>(a, grid, 10));
  rep("no finish", run<1, 2>(a, grid, 10));
  rep("no loads", run<1, 4>(a, grid, 10));
  rep("no mask", run<1, 8>(a, grid, 10));
  rep("no fold, no finish", run<1, 3>(a, grid, 10));
  rep("no fold, no finish, no mask", run<1, 11>(a, grid, 10));
  rep("only map (no fold/finish/mask/loads)", run<1, 15>(a, grid, 10));
  rep("no loads, no mask (compute)", run<1, 12>(a, grid, 10));
  rep("no stores (one per wave)", run<1, 32>(a, grid, 10));
  rep("no end multiply", run<1, 64>(a, grid, 10));
  rep("no carry multiply", run<1, 128>(a, grid, 10));
  rep("no lane alignment", run<1, 256>(a, grid, 10));
  rep("no end/carry/lane multiplies", run<1, 64 | 128 | 256>(a, grid, 10));
  rep("full again", run<1, 0>(a, grid, 10));
  return 0;
}
