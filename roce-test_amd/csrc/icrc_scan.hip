// Piece prefix for the ragged kernel (icrc_kernels.hip): ps[i] = number of
// 64-byte pieces of packets [0, i), ps[count] = total.  A stream-ordered
// hipCUB exclusive scan over a transform of the descriptors (offsets,
// lengths): 12 B read + 8 B written per packet, next to the packet bytes.
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>

#include "icrc_kernels.h"

namespace ricrc {
namespace {

struct PieceCount {
  const uint8_t *base;
  const uint64_t *off;
  const uint32_t *len;
  uint64_t stride, count;
  uint32_t fixed_len, l3_offset;
  __host__ __device__ uint64_t operator()(uint64_t i) const {
    if (i >= count) return 0;
    const uintptr_t start = (uintptr_t)base + (off ? off[i] : i * stride) + l3_offset;
    return ragged_pieces(start, len ? len[i] : fixed_len);
  }
};

}  // namespace

hipError_t ragged_piece_scan(const RaggedArgs &a, uint64_t *ps, hipStream_t st) {
  const PieceCount f{a.base, a.off, a.len, a.stride, a.count, a.fixed_len, a.l3_offset};
  hipcub::CountingInputIterator<uint64_t> idx(0);
  hipcub::TransformInputIterator<uint64_t, PieceCount, hipcub::CountingInputIterator<uint64_t>> in(idx, f);
  const uint64_t n = a.count + 1;
  size_t bytes = 0;
  hipError_t e = hipcub::DeviceScan::ExclusiveSum(nullptr, bytes, in, ps, n, st);
  if (e != hipSuccess) return e;
  void *tmp = nullptr;
  e = hipMallocAsync(&tmp, bytes ? bytes : 1, st);
  if (e != hipSuccess) return e;
  e = hipcub::DeviceScan::ExclusiveSum(tmp, bytes, in, ps, n, st);
  const hipError_t e2 = hipFreeAsync(tmp, st);
  return e != hipSuccess ? e : e2;
}

}  // namespace ricrc
