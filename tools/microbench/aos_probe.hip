// Address-order single-pass ragged fold: an optimistic SKELETON, timed next
// to the product's bucketed pipeline on the same C4-shaped batch, same process
// ("measure the alternative ... before committing").
//
// C4 shape: 4 M packets, lengths uniform over 64/256/1024/4096 B, packed back
// to back, random bytes.  Every 128-byte line is read once in address order:
// lane 8 g + s owns slot s of every line of its group's stream, 4 chains per
// lane folded through the 128-byte-stride slice-by-4 tables (the SCK's
// inner loop).  Variants:
//   floor     the batch's lines split evenly over the 8 groups of every wave,
//             folded with no packet boundaries at all: the stream + fold floor
//             of any address-order design;
//   skeleton  each group streams the lines of a byte-balanced packet range
//             and at every packet boundary it meets does the bookkeeping an
//             address-order fold cannot avoid -- the group's next boundary
//             from its descriptors (a register window of 8, refilled ahead),
//             the ended packet's chains pushed to a per-wave LDS queue and
//             reset, and per 8 queued packets one batched finish (four
//             nibble-table GF(2) multiplies and the 8-lane reduction) and a
//             result store -- but WITHOUT the per-word edge masks (keep,
//             invariant fields, seed) and tail removal the real fold needs.
//             Any real address-order fold costs at least this.
//   product   the bucketed pipeline (bucket, fold, one-line, gather) and its
//             fold alone.
// Timing only (results are not ICRCs).  Build (GPU box):
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 aos_probe.hip -o aos_probe
#include "../../roce-test_amd/csrc/icrc_kernels.hip"
#include "../../roce-test_amd/csrc/icrc_rsck.hip"
#include "mb_fin.h"
#include <stdio.h>
#include <stdlib.h>

#include <vector>
using namespace ricrc;
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s line %d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)

template <typename F> float timeit(F launch, int reps) {
  hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  for (int w = 0; w < 3; ++w) launch();
  CK(hipDeviceSynchronize()); CK(hipEventRecord(e0));
  for (int i = 0; i < reps; ++i) launch();
  CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1)); float ms; CK(hipEventElapsedTime(&ms, e0, e1));
  return ms / reps;
}

struct AosArgs {
  const uint8_t *base;
  const uint64_t *off;
  const uint32_t *len;
  const uint32_t *gfirst;  // [groups + 1]: group k's packets [gfirst[k], gfirst[k + 1]) (skeleton)
  uint64_t lines;          // floor: lines of the batch
  uint32_t *out;
  uint32_t XB[32];
};

constexpr int kD = 8;

template <int SKEL>
__global__ __launch_bounds__(kBlock) void aos_kernel(AosArgs a) {
  __shared__ uint32_t lds[kLdsWords + 256 + kWaves * 8 * 32];  // tables | x^-32 nibble table | per-wave queue (8 entries x 32 words)
  uint32_t *tab = lds, *xtl = lds + kLdsWords;
  table_store(tab, table_entry(g_tab128));
  if (threadIdx.x < 128) {
    const uint32_t w = threadIdx.x >> 4, v = threadIdx.x & 15u;
    uint32_t t = 0;
    for (int b = 0; b < 4; ++b) t ^= ((v >> b) & 1u) ? a.XB[4 * w + b] : 0u;
    xtl[threadIdx.x] = t;
  }
  __syncthreads();
  const uint32_t lane = threadIdx.x & 63, s = lane & 7, g = lane >> 3;
  const uint32_t wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  uint32_t *queue = lds + kLdsWords + 256 + wid * 8 * 32;
  const LaneTab lt{(lane & 31) << 2, ((lane & 31) << 2) | 0x10000u};
  const uint64_t gk = ((uint64_t)blockIdx.x * kWaves + wid) * 8 + g;  // this lane's group
  const uint64_t G = (uint64_t)gridDim.x * kWaves * 8;
  // the group's line range
  uint64_t l_lo, l_hi;
  uint32_t pk = 0, p_end = 0;
  if (SKEL) {
    pk = a.gfirst[gk];
    p_end = a.gfirst[gk + 1];
    l_lo = pk < p_end ? a.off[pk] >> 7 : 0;
    l_hi = pk < p_end ? ((a.off[p_end - 1] + a.len[p_end - 1] - 5) >> 7) + 1 : 0;
  } else {
    l_lo = a.lines * gk / G;
    l_hi = a.lines * (gk + 1) / G;
  }
  const uint64_t nlines = l_hi - l_lo;
  uint32_t maxl = (uint32_t)nlines;  // the wave runs its longest group's line count
#pragma unroll
  for (int o = 8; o < 64; o <<= 1) maxl = max(maxl, (uint32_t)__shfl_xor((int)maxl, o));
  const uint32_t steps = __builtin_amdgcn_readfirstlane(maxl);
  const uint8_t *gbase = a.base + (l_lo << 7) + 16u * s;
  auto load = [&](uint32_t k) -> u32x4 {
    const uint32_t kk = k < nlines ? k : (nlines ? (uint32_t)nlines - 1 : 0);
    return gload16((uintptr_t)(gbase + ((uint64_t)kk << 7)));
  };
  // skeleton: the group's packet cursor -- the current packet's last line
  // (absolute), descriptor windows of 8 packets (lane s of the group holds
  // packet w0 + s's last covered line) read through ds_bpermute
  uint32_t w0 = pk, wl = 0, nl = 0;  // window base, this lane's window packet's last line, the next window's
  auto win_load = [&](uint32_t base) -> uint32_t {
    const uint32_t i = base + s < p_end ? base + s : (p_end ? p_end - 1 : 0);
    return (uint32_t)((a.off[i] + a.len[i] - 5u) >> 7);
  };
  if (SKEL) {
    wl = win_load(w0);
    nl = win_load(w0 + 8);
  }
  auto last_line_of = [&](uint32_t k) -> uint32_t {
    return (uint32_t)__builtin_amdgcn_ds_bpermute((int)((8 * g + (k - w0)) << 2), (int)wl);
  };
  uint32_t nb = SKEL && pk < p_end ? last_line_of(pk) : 0xFFFFFFFFu;
  uint32_t qn = 0;  // queued packets (wave)
  uint32_t sink = 0;
  u32x4 ring[kD];
#pragma unroll
  for (int k = 0; k < kD; ++k) ring[k] = load(k);
  uint32_t r[4] = {0u, 0u, 0u, 0u};
  const uint32_t line0 = (uint32_t)l_lo;
  for (uint32_t k0 = 0; k0 < steps; k0 += kD) {
#pragma unroll
    for (int u = 0; u < kD; ++u) {
      __builtin_amdgcn_sched_barrier(0);
      const uint32_t k = k0 + u;
      const u32x4 w = ring[u];
      ring[u] = load(k + kD);
      uint32_t x[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) x[i] = r[i] ^ w[i];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const uint32_t t0 = lds_at(tab, __builtin_amdgcn_perm(x[i], lt.lo0, 0x0C0C0400u));
        const uint32_t t1 = lds_at(tab, __builtin_amdgcn_perm(x[i], lt.lo0, 0x0C0C0500u) + 128);
        const uint32_t t2 = lds_at(tab, __builtin_amdgcn_perm(x[i], lt.lo1, 0x0C020600u));
        const uint32_t t3 = lds_at(tab, __builtin_amdgcn_perm(x[i], lt.lo1, 0x0C020700u) + 128);
        r[i] = xor3(t0, t1, t2 ^ t3);
      }
      if (SKEL) {
        // every packet ending in this line: push its chains, take the next
        // packet (tiny packets: several per line)
        bool e = line0 + k == nb && k < nlines;
        while (__ballot(e)) {  // wave-uniform
          const uint64_t m = __ballot(e && s == 0);
          const uint32_t rank = __builtin_popcountll(m & ((1ull << lane) - 1ull));
          if (e) {
            const uint32_t slot = (qn + rank) & 7u;
            *reinterpret_cast<u32x4 *>(queue + slot * 32 + 4 * s) = u32x4{r[0], r[1], r[2], r[3]};
#pragma unroll
            for (int i = 0; i < 4; ++i) r[i] = 0u;
            ++pk;
            if (pk - w0 == 8u) {  // next window (loaded 8 packets ago), and request the one after
              w0 += 8;
              wl = nl;
              nl = win_load(w0 + 8);
            }
            nb = pk < p_end ? last_line_of(pk) : 0xFFFFFFFFu;
          }
          qn += __builtin_popcountll(m);
          if (qn >= 8u) {  // a batched finish of 8 queued packets: lane 8 q + s takes entry q's slot s
            const u32x4 v = *reinterpret_cast<const u32x4 *>(queue + ((qn - 8u + g) & 7u) * 32 + 4 * s);
            auto nib = [&](uint32_t val, uint32_t acc) {
              uint32_t e8[8];
#pragma unroll
              for (int ww = 0; ww < 8; ++ww) e8[ww] = xtl[16 * ww + __builtin_amdgcn_ubfe(val, 4 * ww, 4)];
              return xor3(xor3(e8[0], e8[1], e8[2]), xor3(e8[3], e8[4], e8[5]), xor3(e8[6], e8[7], acc));
            };
            const uint32_t f = group_xor(nib(nib(nib(v[3], v[2]), v[1]), nib(v[0], 0u)), 3);
            sink ^= f;
            qn -= 8u;
          }
          e = line0 + k == nb && k < nlines;
        }
      }
    }
  }
  a.out[gk * 8 + s] = r[0] ^ r[1] ^ r[2] ^ r[3] ^ sink;
}

int main() {
  hipDeviceProp_t p; CK(hipGetDeviceProperties(&p, 0));
  const int grid = p.multiProcessorCount;
  const uint64_t count = 4ull << 20;
  std::vector<uint64_t> off(count);
  std::vector<uint32_t> len(count);
  uint64_t x = 0x1CEC0DEull, pos = 0;
  const uint32_t sizes[4] = {64, 256, 1024, 4096};
  for (uint64_t i = 0; i < count; ++i) {
    x ^= x << 13; x ^= x >> 7; x ^= x << 17;
    len[i] = sizes[(x >> 33) & 3];
    off[i] = pos;
    pos += len[i];
  }
  const uint64_t bytes = pos;
  uint8_t *buf; CK(hipMalloc(&buf, bytes + 8192));
  {
    std::vector<uint64_t> h((bytes + 7) / 8);
    for (auto &v : h) { x ^= x << 13; x ^= x >> 7; x ^= x << 17; v = x; }
    CK(hipMemcpy(buf, h.data(), bytes, hipMemcpyHostToDevice));
  }
  uint64_t *d_off; uint32_t *d_len, *out, *tzb;
  CK(hipMalloc(&d_off, 8 * count)); CK(hipMalloc(&d_len, 4 * count)); CK(hipMalloc(&out, 4 * count));
  CK(hipMemcpy(d_off, off.data(), 8 * count, hipMemcpyHostToDevice));
  CK(hipMemcpy(d_len, len.data(), 4 * count, hipMemcpyHostToDevice));
  CK(hipMalloc(&tzb, 4 * 1024)); CK(hipMemset(tzb, 0x35, 4 * 1024));
  // byte-balanced packet ranges of the skeleton's groups
  const uint64_t G = (uint64_t)grid * kWaves * 8;
  std::vector<uint32_t> gfirst(G + 1);
  {
    uint64_t i = 0;
    for (uint64_t k = 0; k <= G; ++k) {
      const uint64_t t = bytes * k / G;
      while (i < count && off[i] < t) ++i;
      gfirst[k] = (uint32_t)i;
    }
    gfirst[G] = (uint32_t)count;
  }
  uint32_t *d_gfirst, *aout; CK(hipMalloc(&d_gfirst, 4 * (G + 1))); CK(hipMalloc(&aout, 4 * G * 8));
  CK(hipMemcpy(d_gfirst, gfirst.data(), 4 * (G + 1), hipMemcpyHostToDevice));
  AosArgs aa{};
  aa.base = buf; aa.off = d_off; aa.len = d_len; aa.gfirst = d_gfirst; aa.lines = (bytes + 127) / 128; aa.out = aout;
  for (int j = 0; j < 32; ++j) aa.XB[j] = 0x85EBCA6Bu * (j + 3);
  // the product pipeline on the same batch
  RsckArgs a{};
  a.base = buf; a.off = d_off; a.len = d_len; a.count = count;
  a.out = out; a.tzb = tzb; a.group_cost = kRsGroupCost;
  a.fin = mb_fin();
  void *ws; CK(hipMalloc(&ws, rs_workspace_bytes(count)));
  CK(rs_zero_counters(ws, 0));
  rs_bind_workspace(a, ws);
  const double alg = (double)bytes + 16.0 * count;
  printf("%.2f GiB in %llu packets (%llu lines); algorithmic bytes %.0f (8 TB/s: %.1f us)\n", bytes / 1073741824.0,
         (unsigned long long)count, (unsigned long long)aa.lines, alg, alg / 8e12 * 1e6);
  // the product fold alone needs a bucketed workspace: one pipeline run first
  CK(launch_rsck(a, grid, 0, 0)); CK(hipDeviceSynchronize());
  for (int r = 0; r < 3; ++r) {
    const float t0 = 1e3f * timeit([&] { hipLaunchKernelGGL(aos_kernel<0>, dim3(grid), dim3(kBlock), 0, 0, aa); }, 10);
    const float t1 = 1e3f * timeit([&] { hipLaunchKernelGGL(aos_kernel<1>, dim3(grid), dim3(kBlock), 0, 0, aa); }, 10);
    const float t2 = 1e3f * timeit([&] { (void)launch_rsck(a, grid, 0, 0); }, 10);
    const float t3 = 1e3f * timeit([&] { hipLaunchKernelGGL((icrc_rsck_kernel<0>), dim3(grid), dim3(kBlock), 0, 0, a); }, 10);
    printf("round %d: address-order floor %7.1f us | address-order skeleton (no masks) %7.1f us | "
           "product pipeline %7.1f us, its fold alone %7.1f us\n", r, t0, t1, t2, t3);
  }
  return 0;
}
