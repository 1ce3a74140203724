// Kernel argument blocks and launchers shared by icrc_kernels.hip and the
// host API (icrc_api.cpp).  Plain structs passed by value as kernargs.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "icrc_sck.h"  // SckArgs / launch_sck (the headline kernel)

namespace ricrc {

struct u32x4_t {
  uint32_t v[4];
};

// Fixed-length batch, packet i at base + i*stride, 16-byte aligned.
struct StreamArgs {
  const uint8_t *base;  // first packet's L3 start
  uint64_t stride;
  uint64_t count;
  uint32_t *out;
  uint64_t n_iters;   // wave steps = ceil(count / (64 >> log2P2))
  uint32_t len;       // n (L3 bytes incl. trailer)
  uint32_t P;         // lanes per packet that hold data
  uint32_t log2P2;    // lanes per packet rounded up to a power of two
  uint32_t nw_last;   // words folded by the last lane of a packet
  uint32_t verify;    // 0: out = ICRC, 1: out = (trailer == ICRC)
  uint32_t K[64];     // per chunk c: x^(8 * bytes after chunk c)
};

// Back-to-back packets of n = 32 * 2^log2C bytes (2 <= 2^log2C <= 128),
// 16-byte aligned: the coalesced + LDS-transposed kernel.
struct TskArgs {
  const uint8_t *base;
  uint64_t stride;  // == n
  uint64_t count;
  uint32_t *out;
  uint64_t n_iters;  // 4 KiB regions = ceil(count * n / 4096)
  uint32_t log2C;
  uint32_t verify;
  uint32_t K[128];   // per chunk position: x^(8 (n - 4 - 32 (pos + 1)))
  uint32_t YB[32];   // x^(8*2048) * x^(31-j): uniform basis for 4 KiB packets
  uint64_t *stamps;  // diagnostic builds only (tools/microbench); null in the product
};

// 8-byte descriptor in class order: lo = address bits 0..31, hi = address
// bits 32..47 | n << 16 (device addresses are 48-bit, n <= 65535).  Padding
// entries of a class's last group repeat the class's last packet.
struct RsDesc {
  uint32_t lo, hi;
};

// Ragged batches (any alignment, per-packet offsets and/or lengths): the
// batch is cut into 64-byte pieces, packet by packet -- packet i covers
// pieces [ps[i], ps[i+1]) laid from its start rounded down to 16 B -- and a
// wave step maps 64 consecutive pieces onto its 64 lanes, however many
// packets they belong to.
struct RaggedArgs {
  const uint8_t *base;
  const uint64_t *off;     // may be null (then p * stride)
  const uint32_t *len;     // may be null (then fixed_len)
  const uint64_t *ps;      // exclusive prefix of pieces, count + 1 entries; null: uniform
  uint64_t stride;
  uint64_t count;
  uint32_t *out;
  const uint32_t *inv_tab;  // x^(-8 z), z in [0, 4096]
  const u32x4_t *inv4;      // entry t: x^(8 (k - t)) for k = 0..3, t in [0, 4096]
  uint32_t fixed_len;
  uint32_t l3_offset;
  uint32_t verify;
  uint32_t P;              // pieces per packet when ps == null
  uint32_t K[64];          // x^(8*64*(63-lane)): lane piece end -> step end
  // Descriptor mode (the small packets of the ragged strided-chain path):
  // packet i is desc[i], the count is *dev_count (device memory).
  const RsDesc *desc;
  const uint32_t *dev_count;
};

// Pieces of a packet of n bytes whose L3 header starts at address `start`:
// the CRC'd bytes [0, n-4) plus the start's offset inside its 16-byte unit,
// in 64-byte pieces (at least one; invalid lengths get one and yield 0).
__host__ __device__ inline uint32_t ragged_pieces(uintptr_t start, uint32_t n) {
  if (n < 4 || n > 65535) return 1u;
  const uint32_t p = ((uint32_t)(start & 15u) + (n - 4u) + 63u) >> 6;
  return p ? p : 1u;
}

// Ragged strided-chain path (icrc_rsck.hip): any packet addresses and
// lengths, packets bucketed by their number of 128-byte lines on the device,
// 8 packets of equal line count per group, folded as in the SCK.
// Classes: 0 = not bucketed (n < 44 or n > 65535: done in the count pass);
// 1 + P for packets spanning <= kRsSmallL lines, by their 64-byte piece count P
// (they go to the piece kernel: 8 lanes per packet is too coarse for them);
// kRsBigBase + L for the rest, by line count L (the strided-chain fold).
#ifndef RICRC_RS_SMALL_L  // tools/microbench only
#define RICRC_RS_SMALL_L 1
#endif
constexpr int kRsSmallL = RICRC_RS_SMALL_L;
constexpr int kRsBigBase = 8;                  // small classes 2..8 (P <= 7 for L <= 3)
constexpr int kRsClasses = kRsBigBase + 514;   // L <= 513 (n <= 65535, any start offset)
constexpr int kTzWords = 264;                  // tz bases: m = 2 tz + q <= 2 * 127 + 7
struct RsPlan {
  uint32_t nc;        // non-empty big classes
  uint32_t ngroups;   // 8-packet groups over all classes
  uint64_t nsteps;    // weighted work over all groups: lines + a per-group finish cost
  uint32_t L[kRsClasses];   // compact, ascending
  uint32_t g0[kRsClasses];  // first group of the class
  uint64_t s0[kRsClasses];  // weighted work before the class's first group
  uint64_t ps0[kRsClasses]; // small classes: first piece of the class (by class index)
};
struct RsckArgs {
  const uint8_t *base;
  const uint64_t *off;  // may be null (then p * stride)
  const uint32_t *len;  // may be null (then fixed_len)
  uint64_t stride;
  uint64_t count;
  uint32_t fixed_len;
  uint32_t l3_offset;
  uint32_t verify;
  uint32_t piece;       // the small region goes to the piece kernel (RICRC_RS_PIECE): write its piece prefix
  uint32_t group_cost;  // a group's finish in line-steps of the fold's work split (launch_rsck sets it)
  uint32_t *out;
  // device workspace (icrc_api.cpp sizes it: rs_workspace_bytes)
  uint32_t *counts;   // [kRsClasses + 2], zeroed before the count pass: class counts, "misaligned" flag, count-pass ticket
  uint32_t *cursor;   // [kRsClasses], zeroed by the plan pass
  uint32_t *bucket;   // [kRsClasses] first position of each class
  RsPlan *plan;
  RsDesc *desc;       // [count + 8 kRsClasses] in class order
  uint32_t *pos_of;   // [count] position of packet i, or ~0 (written by the scatter pass)
  uint32_t *res;      // [count + 8 kRsClasses] results in class order
  uint32_t *hist;     // [pass blocks][kRsClasses] per-block class counts
  uint64_t *ps;       // [count + 8 kRsClasses + 1] piece prefix of the small region
  uint32_t *small_pos;  // positions of the small region (device count for the piece kernel)
  const uint32_t *tzb;  // [kTzWords]: entry m = x^(31 - 4 m), i.e. basis word 4 q of x^(-8 tz) at m = 2 tz + q
  uint32_t XB[32];      // basis of x^-32
  uint32_t XB2[32];     // basis of x^-64
  uint32_t XB3[32];     // basis of x^-96
  uint32_t QS[8];       // x^(-8*16 s): lane slot s -> line start
};
uint64_t rs_workspace_bytes(uint64_t count);
// Carves the workspace (rs_workspace_bytes(count) bytes at ws) into a.
void rs_bind_workspace(RsckArgs &a, void *ws);
// Zeroes a workspace's class counters (on allocation; afterwards every call
// leaves them zero).
hipError_t rs_zero_counters(void *ws, hipStream_t st);
// The whole ragged pipeline on `st`: count/classify, plan, scatter, fold, gather.
// `small` carries the piece kernel's tables (inv_tab, inv4, K) for the small packets.
hipError_t launch_rsck(RsckArgs &a, const RaggedArgs &small, int grid, hipStream_t st);

struct SynthArgs {
  uint8_t *buf;
  uint64_t seed, first, count;
  uint32_t n, stride;    // stride % 8 == 0, n <= stride (fixed-size batches)
  const uint64_t *off;   // ragged batches (launch_synth_ragged): packet k at buf + off[k],
  const uint32_t *len;   //   len[k] bytes
};

// Incremental repair (icrc_repair.hip): packet i's bytes [roff, roff+rlen)
// were old_bytes + i*old_stride when its trailer was stamped.
struct RepairArgs {
  uint8_t *base;
  const uint64_t *off;  // may be null (then i * stride)
  const uint32_t *len;  // may be null (then fixed_len)
  const uint8_t *old_bytes;
  const uint32_t *x8n;  // x^(8 k), k in [0, 65536)
  uint32_t *out;        // may be null (stamp only)
  uint64_t stride, old_stride, count;
  uint32_t fixed_len, l3_offset;
  uint32_t roff, rlen;
  uint32_t family;      // kFamV4 / kFamV6 / kFamAuto
  uint32_t stamp;
  uint32_t mask4[4], mask6[4];  // set by launch_repair: byte k = mask bits of range byte k (k < 16)
};
hipError_t launch_repair(const RepairArgs &a, int grid, hipStream_t st);

// Address-family fix-up after a batch kernel ran with the IPv4 masks
// (icrc_repair.hip): out[i] (the IPv4-mask ICRC) becomes the family's ICRC,
// or, with verify, 1/0 = trailer matches it.
struct FamilyFixArgs {
  const uint8_t *base;
  const uint64_t *off;  // may be null (then i * stride)
  const uint32_t *len;  // may be null (then fixed_len)
  const uint32_t *x8n;  // x^(8 k), k in [0, 65536)
  uint32_t *out;
  uint64_t stride, count;
  uint32_t fixed_len, l3_offset;
  uint32_t family;      // kFamV6 / kFamAuto
  uint32_t verify;
};
hipError_t launch_family_fix(const FamilyFixArgs &a, int grid, hipStream_t st);

hipError_t launch_stream(const StreamArgs &a, int cpl, int grid, hipStream_t st);
hipError_t launch_tsk(const TskArgs &a, int grid, hipStream_t st);
hipError_t launch_ragged(const RaggedArgs &a, int grid, hipStream_t st);
// ps[0..count] = exclusive prefix of ragged_pieces over the batch (stream
// ordered; temporary storage from the stream-ordered allocator).
hipError_t ragged_piece_scan(const RaggedArgs &a, uint64_t *ps, hipStream_t st);
hipError_t launch_synth(const SynthArgs &a, hipStream_t st);
hipError_t launch_synth_ragged(const SynthArgs &a, hipStream_t st);
// ricrc_prime's streaming read of `bytes` (a multiple of 16) of scratch.
hipError_t launch_prime(const void *scratch, uint64_t bytes, uint32_t *sink, int n_cu, hipStream_t st);

}  // namespace ricrc
