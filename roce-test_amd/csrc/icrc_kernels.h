// Kernel argument blocks and launchers shared by icrc_kernels.hip and the
// host API (icrc_api.cpp).  Plain structs passed by value as kernargs.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "icrc_sck.h"  // SckArgs / launch_sck (the headline kernel)

namespace ricrc {

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

// Ragged strided-chain path (icrc_rsck.hip): any packet addresses and
// lengths, packets bucketed by their number of 128-byte lines on the device,
// 8 packets of equal line count per group, folded as in the SCK.
// Classes: 0 = not bucketed (n < 44 or n > 65535: done in the bucket pass);
// 1 + P for packets spanning <= kRsSmallL lines, by their 64-byte piece count P
// (one lane per packet, in the fold's small rounds: 8 lanes per packet is too coarse
// for them); kRsBigBase + L for the rest, by line count L (the strided-chain
// fold).
#ifndef RICRC_RS_SMALL_L  // tools/microbench only
#define RICRC_RS_SMALL_L 1
#endif
constexpr int kRsSmallL = RICRC_RS_SMALL_L;
constexpr int kRsBigBase = 8;                  // small classes 2..8 (P <= 7 for L <= 3)
constexpr int kRsClasses = kRsBigBase + 514;   // L <= 513 (n <= 65535, any start offset)
constexpr int kRsRuns = kRsClasses - kRsBigBase;  // big classes a pass block can hold
constexpr int kTzWords = 264;                  // tz bases: m = 2 tz + q <= 2 * 127 + 7
// Bucket layout (block-local, one pass): pass block b lays its packets out
// by class -- the small ones in a range of the small pool, the big ones as
// "runs" of whole 8-packet groups in a range of the big pool (each run is one
// class, its last group padded with copies of its last packet) -- and
// reserves both ranges with one atomic each.  The big pool's counter packs
// groups (bits 0..25) and weighted work (bits 26..63) so a block's groups and
// its work prefix come from ONE atomic: group order and work order agree.
constexpr int kRsGroupBits = 26;
struct RsCounters {
  uint32_t odd;                // a big packet not starting or ending on a 4-byte word
  uint32_t small;              // small-pool packets
  unsigned long long pool;     // big pool: groups | work << kRsGroupBits
  uint32_t xcd;                // the XCD the bucket pass's workgroup 0 ran on (the fold's xcd_share k)
  uint32_t pad;
};
struct RsBlock {               // pass block b's ranges (runs == 0: no big packets)
  uint32_t g0, groups, runs;   // big pool: groups [g0, g0 + groups), its runs
  uint32_t small0, small;      // small pool: positions [small0, small0 + small)
  uint32_t staged;             // 1: pos_of holds positions in the block's layout (small range | big range)
  uint64_t s0, work;           // big pool: weighted work [s0, s0 + work)
};
struct RsRun {                 // one class of one pass block: groups [g0, g0 + groups) of L lines
  uint32_t g0, groups, L, pad;
  uint64_t s0;                 // weighted work before the run's first group
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
  uint32_t group_cost;  // a group's finish in line-steps of the fold's work split (launch_rsck sets it)
  uint32_t xw[8];            // the fold's work split by XCD (xcd_share; xw[0] == 0: equal shares)
  uint32_t no_split;         // host: keep the fused gather on the pass grid (RICRC_NO_GATHER_SPLIT)
  uint32_t small_in_fold;    // the fold takes the one-line packets (host: unless RICRC_ONE_LINE_IN_GATHER)
  uint32_t small_slots;      // ... dealt to wave slots 0..s-1 (0: to every wave by its work)
  uint32_t *out;
  // device workspace (icrc_api.cpp sizes it: rs_workspace_bytes)
  RsCounters *ctr;      // zeroed on allocation and by the gather pass of every call
  RsBlock *blk;         // [pass blocks]
  RsRun *runs;          // [pass blocks][kRsRuns]
  RsDesc *desc;         // small pool [0, count) | big pool [small_cap, ...) (positions)
  RsDesc *bdesc;        // desc + small_cap: the big pool, group q at 8 q
  uint32_t *pos_of;     // [count] position of packet i (in its pool, or in its block's layout when the
                        // block is staged), or ~0 (written by the bucket pass)
  uint32_t *res;        // results by position, like desc
  uint32_t *bres;       // res + small_cap
  uint32_t small_cap;   // count rounded up to 8
  uint32_t nblk;        // pass blocks of this call (launch_rsck sets it)
  const uint32_t *tzb;  // [kTzWords]: entry m = x^(31 - 4 m), i.e. basis word 4 q of x^(-8 tz) at m = 2 tz + q
  const uint32_t *fin;  // the fold's finish tables (kFinFold words, icrc_math.h build_fin_tables), the context's
  uint32_t xcd_k;       // icrc_rswg_kernel: the start XCD of its work split (the SCK's record, xcd_share)
  uint32_t *xcd_rec;    // ... where its workgroup 0 records its XCD for the next launch
};
// Work of a group in line-steps: its L lines plus the per-group finish
// (GF(2) multiplies through nibble tables, reductions, descriptor and slot
// traffic).  Waves split the total weighted work, not the lines: split by
// lines, a wave that drew 64-byte packets (one line per group) ran ~8x longer
// than one that drew 4 KiB packets.  Swept on C4 (same box, tools/ab_env.sh
// with RICRC_RS_GCOST, profiles/r02/ab_c4_group_cost.txt): 0 -> 1.52 ms per
// step, 1 -> 1.16, 2 -> 1.060-1.081, 3 -> 1.061-1.062, 4 -> 1.065-1.086,
// 6 (round 1's estimate) -> 1.073-1.076, 10 -> 1.09, 16 -> 1.13.  In quarter
// line-steps 10..14 are within the run-to-run noise (profiles/r02/
// ab_c4_group_cost_quarters.txt).
// (RICRC_RS_GCOST, read by ricrc_create, overrides it for schedule studies.)
constexpr uint32_t kRsGroupCost = 12;  // quarter line-steps (3 lines)
// The fold's one-line packets go to wave slots 0 .. kRsSmallSlots - 1 of
// every workgroup (icrc_rsck_kernel; RICRC_SMALL_SLOTS overrides, 0: every
// wave in proportion to its work).
constexpr uint32_t kRsSmallSlots = 12;
uint64_t rs_workspace_bytes(uint64_t count);
// Carves the workspace (rs_workspace_bytes(count) bytes at ws) into a.
void rs_bind_workspace(RsckArgs &a, void *ws);
// Zeroes a workspace's counters (on allocation; afterwards every call
// leaves them zero).
hipError_t rs_zero_counters(void *ws, hipStream_t st);
// The whole ragged pipeline on `st`: bucket, fold (one-line packets included), gather.
// count <= kRsMaxCount (the host cuts larger batches: the big pool's group
// count must fit kRsGroupBits).
constexpr uint64_t kRsMaxCount = 1ull << 28;
// pass_ev (diagnostics, RICRC_PASS_TIMES): 5 timing events recorded on st
// before the bucket pass and after the bucket, fold, one-line and gather
// passes.
hipError_t launch_rsck(RsckArgs &a, int grid, int pass_cap, hipStream_t st, hipEvent_t *pass_ev = nullptr);
// Whether a batch of `count` packets takes the fused pipeline (bucket, fold,
// gather folding the one-line packets: no icrc_rsmall_kernel launch).
bool rs_fused(uint64_t count, int pass_cap);
// The bucket / gather passes' blocks and packets per thread for such a batch (ricrc_launch_info).
void rs_pass_info(uint64_t count, int pass_cap, bool no_split, int *grid, int *unroll, bool *fused, int *ggrid);
// The workgroup-local ragged kernel (icrc_rswg_kernel: classify, lay out,
// fold and write out[] in one launch, no workspace) on `grid` workgroups.
// Any count <= kRsMaxCount is exact (a workgroup takes its packets in chunks
// of kRsWgCap); the dispatch sends it batches of about one chunk per
// workgroup (rs_wg_chunks).
constexpr uint32_t kRsWgCap = 2304;
hipError_t launch_rswg(const RsckArgs &a, int grid, hipStream_t st, hipEvent_t *pass_ev = nullptr);
// Chunks the most loaded workgroup takes for a batch of `count` packets on
// `grid` workgroups with the XCD weights w (0: equal shares).
uint64_t rs_wg_chunks(uint64_t count, int grid, const uint32_t (&w)[8]);

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

// Back-to-back 64-byte packets (C1), 16-byte aligned: the quad kernel
// (coalesced 1 KiB loads, lane-quad transposes).
struct QuadArgs {
  const uint8_t *base;
  uint64_t count;
  uint32_t *out;
  uint32_t verify;
  uint64_t *stamps;   // diagnostic builds only (tools/microbench); null in the product
};
hipError_t launch_quad(const QuadArgs &a, int grid, hipStream_t st);

hipError_t launch_stream(const StreamArgs &a, int cpl, int grid, hipStream_t st);
hipError_t launch_tsk(const TskArgs &a, int grid, hipStream_t st);
hipError_t launch_synth(const SynthArgs &a, hipStream_t st);

// Per-packet status / RoCEv2 classification after a batch ran (icrc_status.hip):
// the reference's ingress accept path, shuffle_ingress_parser.p4:12-36.
constexpr uint32_t kStOk = 0, kStBadLen = 1, kStNotRoce = 2;  // RICRC_ST_* (include/roce_icrc.h)
struct StatusArgs {
  const uint8_t *base;
  const uint64_t *off;  // may be null (then i * stride)
  const uint32_t *len;  // may be null (then fixed_len)
  uint64_t stride, count;
  uint32_t fixed_len, l3_offset;
  uint32_t accept;  // bit 0: RoCEv2/IPv4, bit 1: RoCEv2/IPv6 accepted; 0: lengths only (no header read)
  uint32_t ether;   // frames are Ethernet: the EtherType (2 bytes before L3) must match the family
  uint32_t *out;    // zeroed where status != OK (may be null)
  uint8_t *status;  // status mode: per-packet RICRC_ST_*
  uint8_t *cls;     // classify mode (non-null): per-packet 4 / 6 / 0 instead of a status
};
hipError_t launch_status(const StatusArgs &a, int n_cu, hipStream_t st);
// RICRC_F_FRAMELEN (icrc_status.hip): eff[i] = the L3 length of packet i
// from its IP header when its descriptor length is the frame's extent past
// L3 (frame_l3_len, icrc_math.h); the batch then runs on eff as lengths.
// With an extent (ricrc_batch_device_bounded), a packet whose bytes do not
// all lie in [base, base + extent) gets eff[i] = 0 -- a bad length, so no
// later pass reads it -- and its header is not read here either.
struct FrameLenArgs {
  const uint8_t *base;
  const uint64_t *off;  // may be null (then i * stride)
  const uint32_t *len;  // may be null (then fixed_len)
  uint64_t stride, count;
  uint32_t fixed_len, l3_offset;
  uint32_t *eff;
  uint64_t extent;      // 0: no bound
  uint32_t framelen;    // 1: the IP-header rule (RICRC_F_FRAMELEN); 0: the descriptor length
};
hipError_t launch_framelen(const FrameLenArgs &a, int n_cu, hipStream_t st);
hipError_t launch_synth_ragged(const SynthArgs &a, hipStream_t st);
// ricrc_prime's streaming read of `bytes` (a multiple of 16) of scratch.
hipError_t launch_prime(const void *scratch, uint64_t bytes, uint32_t *sink, int n_cu, hipStream_t st);

}  // namespace ricrc
