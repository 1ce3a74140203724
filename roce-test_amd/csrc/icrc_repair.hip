// Batch incremental ICRC repair on gfx950 (ricrc_repair_device).
//
// The switch's egress rewrites a few header bytes of packets that already
// carry a valid ICRC -- PSN / MSN / opcode patches, p4/shuffle/shuffle_egress.p4:
// 635-671 -- which is why the reference turns ICRC checking off on its NICs
// (scripts/icrc/disable-icrc.sh:13,30).  The CRC is linear over GF(2): for two
// equal-length packets that differ only in bytes [off, off+len),
//   icrc(new) = icrc(old) ^ crc0(masked delta) * x^(8 (n - 4 - off - len))
// (init and xorout cancel), so a repair touches 2 len + 8 bytes of a packet
// instead of n.  Same identity and masks as ricrc_repair_one (icrc_cpu.cpp).
//
// One lane per packet: the work per packet is a handful of dependent byte
// loads and one GF(2) multiply, so the kernel is bound by the latency of
// scattered loads (one or two cache lines per packet), not by bytes; a
// grid-stride loop with many waves per CU keeps enough of them in flight.
#include <hip/hip_runtime.h>

#include "icrc_device.h"
#include "icrc_kernels.h"

namespace ricrc {
namespace {

__device__ __forceinline__ uint32_t load_le32(const uint8_t *p) {
  if (((uintptr_t)p & 3u) == 0) return *reinterpret_cast<const uint32_t *>(p);
  return (uint32_t)p[0] | ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16) | ((uint32_t)p[3] << 24);
}

__device__ __forceinline__ void store_le32(uint8_t *p, uint32_t v) {
  if (((uintptr_t)p & 3u) == 0) {
    *reinterpret_cast<uint32_t *>(p) = v;
    return;
  }
  p[0] = (uint8_t)v;
  p[1] = (uint8_t)(v >> 8);
  p[2] = (uint8_t)(v >> 16);
  p[3] = (uint8_t)(v >> 24);
}

// Small ranges (rlen <= kSmallRange, the PSN / MSN / opcode patches): the
// range, the trailer and the shift constant are loaded up front with
// independent loads (unrolled, guarded), so one packet costs one round of
// memory latency instead of one per byte, and the range comes as whole
// dwords: the kernel is bound by L2 requests per packet (range, trailer,
// trailer store) more than by bytes.  Then the byte chain in LDS.
constexpr uint32_t kSmallRange = 16;

template <bool kSmall>
__global__ __launch_bounds__(256) void repair_kernel(RepairArgs a) {
  __shared__ uint32_t tab[256];  // Sarwate table (slice 0)
  tab[threadIdx.x] = g_tab.t[0][threadIdx.x];
  __syncthreads();
  const uint64_t nthreads = (uint64_t)gridDim.x * blockDim.x;
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < a.count; i += nthreads) {
    const uint32_t n = a.len ? a.len[i] : a.fixed_len;
    uint8_t *p = a.base + (a.off ? a.off[i] : i * a.stride) + a.l3_offset;
    const uint8_t *old = a.old_bytes + i * a.old_stride;
    uint32_t res = 0;
    // Packets too short for the rewritten range, or too long: out = 0, no stamp.
    const bool ok = n >= 4 && n <= kMaxLen && a.roff <= n - 4 && a.rlen <= n - 4 - a.roff;
    if (ok) {
      const bool v6 = a.family == kFamV6 || (a.family == kFamAuto && (p[0] >> 4) == 6);
      const bool same_family =
          a.family != kFamAuto || a.roff != 0 || a.rlen == 0 || (old[0] >> 4) == (p[0] >> 4);
      uint8_t *trailer = p + (n - 4);
      const uint32_t t_old = load_le32(trailer);
      const uint32_t shift = a.x8n[n - 4 - a.roff - a.rlen];
      uint32_t c = 0;
      if constexpr (kSmall) {
        const uint32_t *mw = v6 ? a.mask6 : a.mask4;  // byte k: invariant-field bits of range byte k
        // New bytes: the aligned dwords that hold the range (one L2 request
        // each, instead of one per byte; never outside the packet), realigned
        // with v_alignbyte so that word j holds range bytes 4j..4j+3.
        const uintptr_t q = (uintptr_t)(p + a.roff);
        const uint32_t *qw = reinterpret_cast<const uint32_t *>(q & ~(uintptr_t)3);
        const uint32_t sh = (uint32_t)(q & 3u);
        uint32_t nw[kSmallRange / 4 + 1];
#pragma unroll
        for (uint32_t j = 0; j <= kSmallRange / 4; ++j) nw[j] = 4 * j < sh + a.rlen ? qw[j] : 0u;
        uint8_t ob[kSmallRange];  // old bytes: a compact array, coalesced across lanes
#pragma unroll
        for (uint32_t k = 0; k < kSmallRange; ++k)
          if (k < a.rlen) ob[k] = old[k];
#pragma unroll
        for (uint32_t j = 0; j < kSmallRange / 4; ++j) {
          const uint32_t w = __builtin_amdgcn_alignbyte(nw[j + 1], nw[j], sh);
#pragma unroll
          for (uint32_t b = 0; b < 4; ++b) {
            const uint32_t k = 4 * j + b;
            if (k < a.rlen) {
              const uint32_t d = ((w >> (8 * b)) ^ ob[k]) & ~(mw[j] >> (8 * b)) & 0xFFu;
              c = tab[(c ^ d) & 0xFFu] ^ (c >> 8);
            }
          }
        }
      } else {
        const uint32_t fam = v6 ? kFamV6 : kFamV4;
        for (uint32_t k = 0; k < a.rlen; ++k) {
          const uint32_t d = (uint32_t)(p[a.roff + k] ^ old[k]) & ~mask_byte(fam, a.roff + k) & 0xFFu;
          c = tab[(c ^ d) & 0xFFu] ^ (c >> 8);
        }
      }
      if (same_family) {
        res = t_old ^ gf_mul_dev(c, shift);
        if (a.stamp) store_le32(trailer, res);
      }
    }
    if (a.out) a.out[i] = res;
  }
}

// Address-family fix-up (ricrc_batch_device_ex & co.).  The batch kernels
// apply the reference's IPv4 masks.  A packet's register is linear in its
// bytes and the two families' masks differ only in L3 [0, 56), so
//   icrc_v6(P) = icrc_v4(P) ^ crc0(D) * x^(8 (n - 4 - h)),
//   D = (P|m4) ^ (P|m6) over the h = min(56, n-4) header bytes,
// byte k of D being (m4[k] ^ m6[k]) & ~P[k].  One lane per packet reads the
// header (aligned dwords, never outside the packet), folds D with the Sarwate
// chain in LDS and applies the shift; verify mode compares with the trailer
// here (the batch kernel ran in compute mode).
__global__ __launch_bounds__(256) void family_fix_kernel(FamilyFixArgs a) {
  __shared__ uint32_t tab[256];
  tab[threadIdx.x] = g_tab.t[0][threadIdx.x];
  __syncthreads();
  constexpr uint32_t kH = kMaskSpan;  // 56
  const uint64_t nthreads = (uint64_t)gridDim.x * blockDim.x;
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < a.count; i += nthreads) {
    const uint32_t n = a.len ? a.len[i] : a.fixed_len;
    if (n < 4 || n > kMaxLen) {
      a.out[i] = 0;  // the batch kernel's value for an invalid length, in both modes
      continue;
    }
    const uint8_t *p = a.base + (a.off ? a.off[i] : i * a.stride) + a.l3_offset;
    uint32_t r = a.out[i];
    const bool v6 = a.family == kFamV6 || (a.family == kFamAuto && (p[0] >> 4) == 6);
    if (v6) {
      const uint32_t h = n - 4 < kH ? n - 4 : kH;
      const uintptr_t q = (uintptr_t)p;
      const uint32_t *qw = reinterpret_cast<const uint32_t *>(q & ~(uintptr_t)3);
      const uint32_t sh = (uint32_t)(q & 3u);
      uint32_t hw[kH / 4 + 1];
#pragma unroll
      for (uint32_t j = 0; j <= kH / 4; ++j) hw[j] = 4 * j < sh + h ? qw[j] : 0u;
      uint32_t c = 0;
#pragma unroll
      for (uint32_t j = 0; j < kH / 4; ++j) {
        const uint32_t w = __builtin_amdgcn_alignbyte(hw[j + 1], hw[j], sh);
        const uint32_t dm = mask_word(kFamV4, j) ^ mask_word(kFamV6, j);  // compile-time per j
#pragma unroll
        for (uint32_t b = 0; b < 4; ++b) {
          const uint32_t k = 4 * j + b;
          if (k < h) {
            const uint32_t d = (dm >> (8 * b)) & ~(w >> (8 * b)) & 0xFFu;
            c = tab[(c ^ d) & 0xFFu] ^ (c >> 8);
          }
        }
      }
      r ^= gf_mul_dev(c, a.x8n[n - 4 - h]);
    }
    if (a.verify) r = load_le32(p + (n - 4)) == r ? 1u : 0u;
    a.out[i] = r;
  }
}

}  // namespace

hipError_t launch_family_fix(const FamilyFixArgs &a, int grid, hipStream_t st) {
  (void)hipGetLastError();  // a stale error of an earlier, unrelated HIP call must not fail this launch
  if (a.count == 0) return hipSuccess;
  const uint64_t need = (a.count + 255) / 256;
  const unsigned blocks = (unsigned)std::min<uint64_t>(need, (uint64_t)grid);
  hipLaunchKernelGGL(family_fix_kernel, dim3(blocks), dim3(256), 0, st, a);
  return hipGetLastError();
}

hipError_t launch_repair(const RepairArgs &a, int grid, hipStream_t st) {
  (void)hipGetLastError();  // a stale error of an earlier, unrelated HIP call must not fail this launch
  if (a.count == 0) return hipSuccess;
  const uint64_t need = (a.count + 255) / 256;
  const unsigned blocks = (unsigned)std::min<uint64_t>(need, (uint64_t)grid);
  RepairArgs b = a;
  for (uint32_t w = 0; w < 4; ++w) b.mask4[w] = b.mask6[w] = 0;
  for (uint32_t k = 0; k < kSmallRange && k < a.rlen; ++k) {
    b.mask4[k >> 2] |= mask_byte(kFamV4, a.roff + k) << (8 * (k & 3));
    b.mask6[k >> 2] |= mask_byte(kFamV6, a.roff + k) << (8 * (k & 3));
  }
  if (a.rlen <= kSmallRange)
    hipLaunchKernelGGL(repair_kernel<true>, dim3(blocks), dim3(256), 0, st, b);
  else
    hipLaunchKernelGGL(repair_kernel<false>, dim3(blocks), dim3(256), 0, st, b);
  return hipGetLastError();
}

}  // namespace ricrc
