// Kernel arguments + launcher of the strided-chain kernel (icrc_sck.hip), the
// headline path.  Kept apart from icrc_kernels.h so the headline kernel's
// sources are exactly icrc_sck.{h,hip} + icrc_device.h + icrc_math.h.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace ricrc {

// Back-to-back packets of n = 128 * L bytes (L = 8, 16, 32), 16-byte aligned:
// the strided-chain kernel.  8 lanes per packet, 8 packets per wave group.
struct SckArgs {
  const uint8_t *base;
  uint64_t count;
  uint32_t *out;
  uint32_t n;        // == stride (the slot, for a framed ring)
  uint32_t l3_offset;  // 0, or a framed ring's L3 offset in each slot (<= kSckMaxL3)
  uint32_t verify;
  const uint32_t *fin;  // finish tables (kFinSck words: x^-32 and x^(-32 (4 s + 1)) nibble tables), the context's
  uint32_t family;   // kFamV4 / kFamV6 / kFamAuto: masks applied by the kernel itself
  uint64_t *stamps;  // diagnostic builds only (tools/microbench); null in the product
  // Per-wave share of the groups by XCD (xcd_share): a wave on XCD x takes
  // xw[x] parts; workgroup b runs on XCD (b + xcd_k) % 8.  xw[0] == 0: equal
  // contiguous blocks of ceil(G / waves).  xcd_rec: where workgroup 0
  // records its XCD (or null).
  uint32_t xw[8];
  uint32_t xcd_k;
  uint32_t *xcd_rec;
};

// A framed ring's L3 offset: line 0 of the slot must hold the L3 bytes the
// IPv4 masks and the seed touch (L3 bytes 0..32), so o + 33 <= 128.
constexpr uint32_t kSckMaxL3 = 92;

// Returns hipErrorInvalidValue for an n it has no instantiation for.
hipError_t launch_sck(const SckArgs &a, int grid, hipStream_t st);

}  // namespace ricrc
