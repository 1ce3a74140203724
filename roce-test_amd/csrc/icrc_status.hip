// Per-packet status and RoCEv2 classification of device batches (gfx950).
//
// The reference accepts a frame as RoCEv2 only along one parser path
// (p4/shuffle/shuffle_ingress_parser.p4:12-36): Ethernet ether_type 0x0800
// (ETHERTYPE_IPV4, p4/common/header.p4:8) -> IPv4 protocol 17 -> UDP dst_port
// 4791 (UDP_PORT_ROCE, header.p4:14) -> BTH; anything else falls through to
// `accept` without a BTH and is not RoCE.  ricrc_classify (icrc_cpu.cpp) is
// the same accept path on one L3 packet (plus IHL 5 / total_len == n, and
// the IPv6 path of IBTA Annex A17); this kernel applies it to every packet of
// a batch, after the ICRC kernels ran:
//
//   status[i] = RICRC_ST_BADLEN   n outside [RICRC_MIN_LEN, RICRC_MAX_LEN]
//             = RICRC_ST_NOTROCE  strict and the packet is not RoCEv2 of an
//                                 accepted family (or its frame's EtherType,
//                                 the two bytes before L3, is not that
//                                 family's when the batch is Ethernet framed)
//             = RICRC_ST_OK       otherwise
//   out[i]    = 0 wherever status[i] != RICRC_ST_OK
//
// or, classify-only, cls[i] = 4 / 6 / 0.  One thread per packet, four packets
// per thread with their descriptor and header loads issued before any is
// used; header fields are read as bytes (L3 starts at any alignment).  This
// pass reads <= 44 header bytes (+2 EtherType bytes) and 12 descriptor bytes
// per packet and writes 1 (+4) bytes.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "icrc_kernels.h"
#include "icrc_math.h"

namespace ricrc {
namespace {

constexpr int kStBlock = 256;
constexpr int kStUnroll = 4;

typedef const uint8_t __attribute__((address_space(1))) *gbyte;

__device__ __forceinline__ uint32_t be16(gbyte p) { return ((uint32_t)p[0] << 8) | p[1]; }

// 4: RoCEv2 over IPv4, 6: over IPv6, 0: neither (ricrc_classify's rules).
__device__ __forceinline__ uint32_t classify_l3(gbyte l3, uint32_t n) {
  if (n < kMinLen || n > kMaxLen) return 0u;
  const uint32_t b0 = l3[0];
  if (b0 == 0x45u) {  // ipv4_h: version 4, IHL 5 (header.p4:42-53, no options)
    const bool ok = l3[9] == 17u && be16(l3 + 2) == n && be16(l3 + 22) == 4791u;
    return ok ? 4u : 0u;
  }
  if ((b0 >> 4) == 6u && n >= 40u + 8u + 12u + 4u) {  // IPv6 || UDP || BTH || ICRC
    const bool ok = l3[6] == 17u && be16(l3 + 4) == n - 40u && be16(l3 + 42) == 4791u;
    return ok ? 6u : 0u;
  }
  return 0u;
}

__global__ __launch_bounds__(kStBlock) void icrc_status_kernel(StatusArgs a) {
  const uint64_t T = (uint64_t)gridDim.x * blockDim.x;
  for (uint64_t i0 = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i0 < a.count; i0 += kStUnroll * T) {
    uint64_t addr[kStUnroll];
    uint32_t n[kStUnroll];
#pragma unroll
    for (int k = 0; k < kStUnroll; ++k) {
      uint64_t i = i0 + k * T;
      i = i < a.count ? i : a.count - 1;
      addr[k] = (uint64_t)(uintptr_t)a.base + (a.off ? a.off[i] : i * a.stride) + a.l3_offset;
      n[k] = a.len ? a.len[i] : a.fixed_len;
    }
#pragma unroll
    for (int k = 0; k < kStUnroll; ++k) {
      const uint64_t i = i0 + k * T;
      if (i >= a.count) break;
      const bool len_ok = n[k] >= kMinLen && n[k] <= kMaxLen;
      uint32_t c = 0u;
      if (len_ok && (a.accept || a.cls)) {
        const gbyte l3 = reinterpret_cast<gbyte>((uintptr_t)addr[k]);
        c = classify_l3(l3, n[k]);
        if (c && a.ether) c = be16(l3 - 2) == (c == 4u ? 0x0800u : 0x86DDu) ? c : 0u;
      }
      if (a.cls) {
        a.cls[i] = (uint8_t)c;
        continue;
      }
      const bool accepted = !a.accept || (c == 4u && (a.accept & 1u)) || (c == 6u && (a.accept & 2u));
      const uint8_t st = !len_ok ? (uint8_t)kStBadLen : accepted ? (uint8_t)kStOk : (uint8_t)kStNotRoce;
      a.status[i] = st;
      if (st != kStOk && a.out) a.out[i] = 0u;
    }
  }
}

// RICRC_F_FRAMELEN and / or an extent: one thread per packet, four packets
// per thread with the descriptor loads, then the 6 header bytes, issued
// before any is used.
__global__ __launch_bounds__(kStBlock) void icrc_framelen_kernel(FrameLenArgs a) {
  const uint64_t T = (uint64_t)gridDim.x * blockDim.x;
  for (uint64_t i0 = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i0 < a.count; i0 += kStUnroll * T) {
    uint64_t addr[kStUnroll];
    uint32_t n[kStUnroll], b0[kStUnroll], h2[kStUnroll], h4[kStUnroll];
#pragma unroll
    for (int k = 0; k < kStUnroll; ++k) {
      uint64_t i = i0 + k * T;
      i = i < a.count ? i : a.count - 1;
      const uint64_t fo = a.off ? a.off[i] : i * a.stride;
      addr[k] = (uint64_t)(uintptr_t)a.base + fo + a.l3_offset;
      n[k] = a.len ? a.len[i] : a.fixed_len;
      // outside the caller's allocation: length 0 (nothing reads it)
      if (a.extent && (fo > a.extent || (uint64_t)a.l3_offset + n[k] > a.extent - fo)) n[k] = 0u;
    }
#pragma unroll
    for (int k = 0; k < kStUnroll; ++k) {
      b0[k] = h2[k] = h4[k] = 0u;
      if (a.framelen && frame_len_applies(n[k])) {  // the frame holds at least the IPv4 / BTH headers: bytes 0..5 are in it
        const gbyte l3 = reinterpret_cast<gbyte>((uintptr_t)addr[k]);
        b0[k] = l3[0];
        h2[k] = be16(l3 + 2);
        h4[k] = be16(l3 + 4);
      }
    }
#pragma unroll
    for (int k = 0; k < kStUnroll; ++k) {
      const uint64_t i = i0 + k * T;
      if (i < a.count) a.eff[i] = a.framelen ? frame_l3_len(n[k], b0[k], h2[k], h4[k]) : n[k];
    }
  }
}

}  // namespace

hipError_t launch_framelen(const FrameLenArgs &a, int n_cu, hipStream_t st) {
  (void)hipGetLastError();
  if (a.count == 0) return hipSuccess;
  const uint64_t want = (a.count + kStBlock * kStUnroll - 1) / (kStBlock * kStUnroll);
  const uint64_t cap = 8ull * (uint64_t)n_cu;
  const int grid = (int)(want < cap ? (want ? want : 1) : cap);
  hipLaunchKernelGGL(icrc_framelen_kernel, dim3(grid), dim3(kStBlock), 0, st, a);
  return hipGetLastError();
}

hipError_t launch_status(const StatusArgs &a, int n_cu, hipStream_t st) {
  (void)hipGetLastError();  // a stale error of an earlier, unrelated HIP call must not fail this launch
  if (a.count == 0) return hipSuccess;
  const uint64_t want = (a.count + kStBlock * kStUnroll - 1) / (kStBlock * kStUnroll);
  const uint64_t cap = 8ull * (uint64_t)n_cu;
  const int grid = (int)(want < cap ? (want ? want : 1) : cap);
  hipLaunchKernelGGL(icrc_status_kernel, dim3(grid), dim3(kStBlock), 0, st, a);
  return hipGetLastError();
}

}  // namespace ricrc
