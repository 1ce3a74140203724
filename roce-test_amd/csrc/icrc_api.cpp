// Host side of libroceicrc: contexts, kernel selection, host-buffer staging
// and multi-GPU sharding.  Everything here is plumbing around the gfx950
// kernels in icrc_kernels.hip; there is no CPU compute path for batches.
//
// Conventions follow the reference's C++: 0 / negative
// errno returns (endpoint/shuffle_endpoint.hpp:364-389), no aborts
// (common/logger.hpp:190 logassert only logs), caller-owned buffers
// (common/huge_malloc.h:12-22).
#include <dlfcn.h>
#include <errno.h>
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <new>
#include <type_traits>
#include <thread>
#include <vector>

#include "../../include/roce_icrc.h"
#include "icrc_kernels.h"
#include "icrc_math.h"
#include "icrc_plan.h"

using namespace ricrc;

namespace {

constexpr uint64_t kStageBytes = 256ull << 20;  // per staging slot (bytes of packets)
constexpr uint64_t kStagePkts = 1ull << 20;     // per staging slot (packets)
// Ragged-path workspaces per device, one per recently used stream: batch_host's
// two slot streams + the context stream + callers' streams.
constexpr size_t kMaxWorkspaces = 8;
// ... and at most this many bytes of them per device (one workspace for a
// 2^28-packet chunk is ~7.5 GB): least recently used ones are freed first
// when a workspace grows; the one in use is never evicted.
constexpr uint64_t kMaxWorkspaceBytes = 12ull << 30;
constexpr uint64_t kRsChunk = kRsMaxCount;  // the ragged pipeline's group counter is 26-bit: longer batches are cut

// Environment knobs, read ONCE by ricrc_create (diagnostics, tests and
// schedule studies; the launch path never calls getenv).
struct Knobs {
  bool no_sck = false;     // RICRC_NO_SCK: fixed 1/2/4 KiB batches take the transposed kernel
  bool no_framed = false;  // RICRC_NO_FRAMED: framed 1/2/4 KiB rings take the ragged pipeline
  bool no_gather_split = false;  // RICRC_NO_GATHER_SPLIT: the fused gather folds its one-line packets itself
  bool no_tsk = false;     // RICRC_NO_TSK: ... and 128-512 B batches the direct streaming kernel
  bool no_quad = false;    // RICRC_NO_QUAD: 64 B batches take the direct streaming kernel
  int sck_grid = 0;        // RICRC_SCK_GRID: cap the strided-chain grid (tests: many groups per wave)
  int rsck_grid = 0;       // RICRC_RSCK_GRID: cap the ragged fold grid (tests)
  uint32_t gcost = 0;      // RICRC_RS_GCOST: the ragged fold's per-group cost, quarter lines (0: kRsGroupCost)
  bool one_line_in_gather = false;  // RICRC_ONE_LINE_IN_GATHER: the gather / a one-line kernel folds the one-line packets
  int small_slots = -1;    // RICRC_SMALL_SLOTS: wave slots taking the fold's one-line packets (-1: kRsSmallSlots)
  int wg_chunks = 8;       // RICRC_WG_CHUNKS: ragged batches of up to this many kRsWgCap chunks per workgroup take
                           // the workgroup-local kernel (0: never; RICRC_NO_WG = 0)
  int pass_grid = 0;       // RICRC_RS_PASS_GRID: cap the ragged bucket / gather pass grid (schedule studies)
  bool pass_times = false; // RICRC_PASS_TIMES: timing events between the ragged passes (ricrc_pass_times)
  long fail_chunk = -1;    // RICRC_FAIL_CHUNK: the next ricrc_batch_host fails after queueing chunk k (tests; once)
  int host_threads = 16;   // RICRC_HOST_THREADS: CPU copy threads of ricrc_batch_host
  int xcd_skew = -1;       // RICRC_XCD_SKEW: per-mille work moved to even XCDs (-1: per kernel, 0: equal shares)
  uint32_t xcd_w[8] = {};  // RICRC_XCD_WEIGHTS=w0,...,w7: parts per wave on XCD x (overrides the skew)
};

// Work split by XCD parity (xcd_share in icrc_device.h): a wave of an
// even-indexed workgroup takes (1000 + skew) parts, of an odd one (1000 -
// skew).  On every MI355X box of rounds 2-4 the odd XCDs' waves ended 5-10 %
// after the even ones' with equal work (profiles/r02/sck_tail.txt,
// profiles/r03/s17_bucket_abl.txt); weighting them evens the ends
// (tools/microbench/sck_skew.hip, fold_var.hip, profiles/r04/s15_*): 1 M x
// 4 KiB on 240 CUs 630.7-631.1 -> 618.1-619.7 us at 25; 4 M x 4 KiB on 256
// CUs 2558-2568 -> 2485-2488 us at 50; the C4 fold 919.5-924.1 -> 912.6-912.9
// us at 40.  The 1 KiB super-group schedule gains nothing (0).
struct XcdWeights {
  uint32_t w[8];  // parts per wave on XCD x; w[0] == 0: equal shares
};
// The start XCD of the next launch on this device: the latest one a kernel
// recorded (it is stable over many launches; a stale value costs speed only).
uint32_t xcd_start(const uint32_t *h_xcd) { return h_xcd ? __atomic_load_n(h_xcd, __ATOMIC_RELAXED) & 7u : 0u; }

XcdWeights xcd_weights(const Knobs &kn, int auto_skew) {
  XcdWeights r{};
  if (kn.xcd_w[0] != 0u) {  // RICRC_XCD_WEIGHTS
    for (int x = 0; x < 8; ++x) r.w[x] = kn.xcd_w[x];
    return r;
  }
  const int skew = kn.xcd_skew >= 0 ? kn.xcd_skew : auto_skew;
  if (skew <= 0) return r;  // the kernels' equal-share split
  for (int x = 0; x < 8; ++x) r.w[x] = (x & 1) ? 1000u - (uint32_t)skew : 1000u + (uint32_t)skew;
  return r;
}
bool g_debug = false;  // RICRC_DEBUG: print the HIP/RCCL error behind an -EIO

struct Slot {
  uint8_t *d_buf = nullptr;
  uint64_t *d_off = nullptr;
  uint32_t *d_len = nullptr;
  uint32_t *d_out = nullptr;
  uint8_t *h_buf = nullptr;  // pinned
  uint64_t *h_off = nullptr;
  uint32_t *h_len = nullptr;
  uint32_t *h_out = nullptr;
  hipStream_t st = nullptr;  // per slot: chunk k+1's H2D overlaps chunk k's kernel/D2H
  hipEvent_t done = nullptr;
};

struct Dev {
  int id = 0;
  int n_cu = 0;
  Knobs knobs;
  hipStream_t stream = nullptr;
  uint32_t *d_tzb = nullptr;   // [kTzWords]: basis words 4q of x^(-8 tz) at 2 tz + q (ragged strided-chain path)
  uint32_t *d_fin = nullptr;   // [kFinSck + kFinFold]: the strided-chain kernels' finish tables (build_fin_tables)
  uint32_t *d_x8n = nullptr;   // x^(8 k), k < 65536 (incremental repair)
  // Pinned word where workgroup 0 of the SCK records its XCD; the next SCK
  // launch passes it as xcd_k (xcd_share in icrc_device.h).  (The ragged
  // fold reads the XCD its own call's bucket pass recorded, RsCounters::xcd.)
  uint32_t *h_xcd = nullptr;
  uint32_t *d_xcd_rec = nullptr;  // the same word as the device addresses it
  Slot slot[2];
  uint8_t *d_status[2] = {nullptr, nullptr};  // batch_host_st: per-slot status staging (device / pinned)
  uint8_t *h_status[2] = {nullptr, nullptr};
  bool staged = false;
  // Ragged-path workspaces, one per stream that used this device (work on
  // one stream is ordered, so its workspace is never shared by two calls in
  // flight), grown on demand with the stream-ordered allocator; the class
  // counters inside are zeroed on allocation and re-zeroed by the last pass
  // of every call (rsck_gather), so a call costs no allocation and no memset.
  // Kept in LRU order (front = least recently used).  `done` is recorded
  // after every use: evicting a workspace (or reusing it on a stream handle
  // that may name a new stream) orders the free / the reuse after that event
  // on the GPU -- no host or device-wide wait.
  struct Ws {
    hipStream_t st;
    void *p;
    uint64_t bytes;
    bool dirty;  // a call failed part-way: zero the counters before the next one
    hipEvent_t done;
  };
  // RICRC_PASS_TIMES: kPtSets sets of 5 timing events, one set per ragged
  // call in turn; ricrc_pass_times sums the sets recorded since its last call.
  static constexpr int kPtSets = 64;
  std::vector<hipEvent_t> pt_ev;
  int pt_next = 0, pt_used = 0;
  std::vector<Ws> ws;
  std::vector<hipEvent_t> spare;  // events of workspaces evicted for bytes, reused by the next new one
};

int hip_err(hipError_t e) {
  if (e != hipSuccess && g_debug) fprintf(stderr, "libroceicrc: HIP error %d: %s\n", (int)e, hipGetErrorString(e));
  return e == hipSuccess ? 0 : (e == hipErrorOutOfMemory ? -ENOMEM : -EIO);
}

#define HIP_TRY(x)                          \
  do {                                      \
    hipError_t e_ = (x);                    \
    if (e_ != hipSuccess) return hip_err(e_); \
  } while (0)

class DeviceGuard {
 public:
  explicit DeviceGuard(int dev) {
    if (hipGetDevice(&prev_) != hipSuccess) prev_ = -1;
    ok_ = hipSetDevice(dev) == hipSuccess;
  }
  ~DeviceGuard() {
    if (prev_ >= 0) (void)hipSetDevice(prev_);
  }
  bool ok() const { return ok_; }

 private:
  int prev_ = -1;
  bool ok_ = false;
};

uint32_t x8n_host(uint64_t n) { return gf_x8n(n); }

}  // namespace

struct HostRange {
  uintptr_t lo, hi;
  bool owned;  // ricrc_host_alloc (else ricrc_host_register)
};

struct ricrc_ctx {
  std::vector<Dev> devs;
  std::vector<HostRange> pinned;  // host ranges the DMA engines may read directly
  Knobs knobs;
  // RICRC_FAIL_CHUNK's one-shot state (tests): consumed by a compare-exchange,
  // so two host threads sharing a context cannot both fire it.
  std::atomic<long> fail_once{-1};
  std::vector<ncclComm_t> comms;  // ricrc_comm_init: one RCCL communicator per device
};

namespace {

int init_dev(Dev &d) {
  DeviceGuard g(d.id);
  if (!g.ok()) return -ENODEV;
  hipDeviceProp_t prop;
  HIP_TRY(hipGetDeviceProperties(&prop, d.id));
  d.n_cu = prop.multiProcessorCount > 0 ? prop.multiProcessorCount : 256;
  HIP_TRY(hipStreamCreateWithFlags(&d.stream, hipStreamNonBlocking));
  // Basis word 4q of x^(-8 tz) is x^(-8 tz) x^(31 - 4q) = x^(31 - 4 (2 tz + q)):
  // one entry per m = 2 tz + q; the kernel derives words 4q+1..4q+3 by x^-1.
  std::vector<uint32_t> tzb(kTzWords);
  for (int m = 0; m < kTzWords; ++m) {
    const int tz = std::min(m >> 1, 127), q = m - 2 * tz;
    tzb[m] = q < 8 ? gf_mul(gf_xinv8n((uint64_t)tz), 1u << (4 * q)) : 0u;
  }
  // (a speed hint only: without it the SCK assumes workgroup b on XCD b % 8)
  if (hipHostMalloc((void **)&d.h_xcd, 64, hipHostMallocCoherent) == hipSuccess) {
    *d.h_xcd = 0;  // until a kernel has recorded it: workgroup b on XCD b % 8
    if (hipHostGetDevicePointer((void **)&d.d_xcd_rec, d.h_xcd, 0) != hipSuccess) d.d_xcd_rec = nullptr;
  } else {
    d.h_xcd = nullptr;
  }
  (void)hipGetLastError();
  HIP_TRY(hipMalloc(&d.d_tzb, tzb.size() * sizeof(uint32_t)));
  HIP_TRY(hipMemcpy(d.d_tzb, tzb.data(), tzb.size() * sizeof(uint32_t), hipMemcpyHostToDevice));
  std::vector<uint32_t> fin(kFinSck + kFinFold);
  build_fin_tables(fin.data(), false);
  build_fin_tables(fin.data() + kFinSck, true);
  HIP_TRY(hipMalloc(&d.d_fin, fin.size() * sizeof(uint32_t)));
  HIP_TRY(hipMemcpy(d.d_fin, fin.data(), fin.size() * sizeof(uint32_t), hipMemcpyHostToDevice));
  std::vector<uint32_t> x8n(65536);  // x^(8 k): a repair's shift over the bytes after the rewrite
  uint32_t w = kOne;
  for (size_t k = 0; k < x8n.size(); ++k) {
    x8n[k] = w;
    for (int b = 0; b < 8; ++b) w = gf_mulx(w);
  }
  HIP_TRY(hipMalloc(&d.d_x8n, x8n.size() * sizeof(uint32_t)));
  HIP_TRY(hipMemcpy(d.d_x8n, x8n.data(), x8n.size() * sizeof(uint32_t), hipMemcpyHostToDevice));
  return 0;
}

int ensure_staging(Dev &d) {
  if (d.staged) return 0;
  DeviceGuard g(d.id);
  for (Slot &s : d.slot) {
    HIP_TRY(hipMalloc(&s.d_buf, kStageBytes + 64));
    HIP_TRY(hipMalloc(&s.d_off, kStagePkts * sizeof(uint64_t)));
    HIP_TRY(hipMalloc(&s.d_len, kStagePkts * sizeof(uint32_t)));
    HIP_TRY(hipMalloc(&s.d_out, kStagePkts * sizeof(uint32_t)));
    HIP_TRY(hipHostMalloc(&s.h_buf, kStageBytes + 64, hipHostMallocDefault));
    HIP_TRY(hipHostMalloc(&s.h_off, kStagePkts * sizeof(uint64_t), hipHostMallocDefault));
    HIP_TRY(hipHostMalloc(&s.h_len, kStagePkts * sizeof(uint32_t), hipHostMallocDefault));
    HIP_TRY(hipHostMalloc(&s.h_out, kStagePkts * sizeof(uint32_t), hipHostMallocDefault));
    HIP_TRY(hipStreamCreateWithFlags(&s.st, hipStreamNonBlocking));
    HIP_TRY(hipEventCreateWithFlags(&s.done, hipEventDisableTiming));
  }
  for (int k = 0; k < 2; ++k) {
    HIP_TRY(hipMalloc(&d.d_status[k], kStagePkts));
    HIP_TRY(hipHostMalloc(&d.h_status[k], kStagePkts, hipHostMallocDefault));
  }
  d.staged = true;
  return 0;
}

void free_dev(Dev &d) {
  DeviceGuard g(d.id);
  for (Slot &s : d.slot) {
    if (s.done) (void)hipEventSynchronize(s.done), (void)hipEventDestroy(s.done);
    (void)hipFree(s.d_buf), (void)hipFree(s.d_off), (void)hipFree(s.d_len), (void)hipFree(s.d_out);
    (void)hipHostFree(s.h_buf), (void)hipHostFree(s.h_off), (void)hipHostFree(s.h_len), (void)hipHostFree(s.h_out);
    if (s.st) (void)hipStreamDestroy(s.st);
  }
  for (int k = 0; k < 2; ++k) (void)hipFree(d.d_status[k]), (void)hipHostFree(d.h_status[k]);
  for (Dev::Ws &w : d.ws) {  // wait for each workspace's last use (its stream may be gone already)
    if (w.done) (void)hipEventSynchronize(w.done), (void)hipEventDestroy(w.done);
    (void)hipFree(w.p);
  }
  d.ws.clear();
  for (hipEvent_t e : d.spare) (void)hipEventSynchronize(e), (void)hipEventDestroy(e);
  d.spare.clear();
  for (hipEvent_t e : d.pt_ev) (void)hipEventDestroy(e);
  d.pt_ev.clear();
  (void)hipFree(d.d_tzb);
  (void)hipFree(d.d_fin);
  (void)hipFree(d.d_x8n);
  if (d.h_xcd) (void)hipDeviceSynchronize(), (void)hipHostFree(d.h_xcd);  // no kernel may still record into it
  if (d.stream) (void)hipStreamDestroy(d.stream);
}

int ilog2_ceil(uint32_t v) {
  int l = 0;
  while ((1u << l) < v) ++l;
  return l;
}

// The ragged-path workspace of stream st on device d, at least `bytes`.
// launch_rsck_range records the workspace's `done` event after the call's kernels.
int ragged_ws(Dev &d, hipStream_t st, uint64_t bytes, Dev::Ws **out) {
  size_t at = d.ws.size();
  for (size_t k = 0; k < d.ws.size(); ++k)
    if (d.ws[k].st == st) at = k;
  if (at < d.ws.size()) {
    Dev::Ws w = d.ws[at];
    d.ws.erase(d.ws.begin() + at);
    // Same handle: the same stream (ordered already) or a new stream that
    // reuses a destroyed one's handle (not ordered after its last call).
    // The HIP runtime torch ships has no hipStreamGetId to tell them apart,
    // so a last use that is still in flight is waited for on the GPU.
    const hipError_t q = hipEventQuery(w.done);
    if (q == hipErrorNotReady) HIP_TRY(hipStreamWaitEvent(st, w.done, 0));
    else if (q != hipSuccess) return hip_err(q);
    d.ws.push_back(w);  // most recently used
  } else {
    Dev::Ws w{st, nullptr, 0, true, nullptr};
    if (d.ws.size() >= kMaxWorkspaces) {  // evict the least recently used, in stream order on st
      Dev::Ws old = d.ws.front();
      d.ws.erase(d.ws.begin());
      HIP_TRY(hipStreamWaitEvent(st, old.done, 0));
      if (old.p) HIP_TRY(hipFreeAsync(old.p, st));
      w.done = old.done;  // re-recorded after this call
    } else if (!d.spare.empty()) {
      w.done = d.spare.back();
      d.spare.pop_back();
    } else {
      HIP_TRY(hipEventCreateWithFlags(&w.done, hipEventDisableTiming));
    }
    d.ws.push_back(w);
  }
  Dev::Ws *w = &d.ws.back();
  if (w->bytes < bytes) {
    if (w->p) HIP_TRY(hipFreeAsync(w->p, st));
    w->p = nullptr;
    w->bytes = 0;
    const uint64_t grow = std::max<uint64_t>(bytes, bytes + bytes / 4);
    // Byte cap: free least recently used workspaces (in stream order on st,
    // after their last use) until this one fits beside the rest.
    uint64_t others = 0;
    for (size_t k = 0; k + 1 < d.ws.size(); ++k) others += d.ws[k].bytes;
    while (d.ws.size() > 1 && others + grow > kMaxWorkspaceBytes) {
      Dev::Ws old = d.ws.front();
      d.ws.erase(d.ws.begin());
      HIP_TRY(hipStreamWaitEvent(st, old.done, 0));
      if (old.p) HIP_TRY(hipFreeAsync(old.p, st));
      others -= old.bytes;
      d.spare.push_back(old.done);
    }
    w = &d.ws.back();
    HIP_TRY(hipMallocAsync(&w->p, grow, st));
    w->bytes = grow;
    w->dirty = true;
    if (g_debug) fprintf(stderr, "libroceicrc: ragged workspace %p (%llu B) for stream %p\n", w->p,
                         (unsigned long long)grow, (void *)st);
  }
  if (w->dirty) {
    HIP_TRY(rs_zero_counters(w->p, st));
    w->dirty = false;
  }
  *out = w;
  return 0;
}

// Kernel selection + launch for one device-resident batch.
// The strided-chain kernel's grid for a batch, or 0 if the batch does not
// take it (it needs back-to-back 1, 2 or 4 KiB packets, 16-byte aligned); it
// applies any address family natively.
// A framed NIC ring the strided-chain kernel folds slot by slot (FR,
// icrc_sck.hip): 1, 2 or 4 KiB slots, 16-byte aligned, the L3 packet at
// 0 < l3_offset <= kSckMaxL3 running to the slot's end.
bool sck_framed(const Knobs &kn, const uint8_t *base, const uint64_t *off, const uint32_t *len, uint64_t stride,
                uint32_t l3_offset) {
  return !off && !len && l3_offset > 0 && l3_offset <= kSckMaxL3 && (uintptr_t)base % 16 == 0 && !kn.no_sck &&
         !kn.no_framed && (stride == 1024 || stride == 2048 || stride == 4096);
}

int sck_grid(const Dev &d, const uint8_t *base, const uint64_t *off, const uint32_t *len, uint64_t stride,
             uint64_t count, uint32_t l3_offset) {
  if (l3_offset != 0 && !sck_framed(d.knobs, base, off, len, stride, l3_offset)) return 0;
  if (off || len || ((uintptr_t)base % 16) != 0 || d.knobs.no_sck || count == 0) return 0;
  if (stride != 1024 && stride != 2048 && stride != 4096) return 0;
  const uint64_t groups = (count + 7) / 8;
  // One workgroup per CU.  Batches of up to 48 groups per wave (6 GiB of
  // 4 KiB packets on 256 CUs) run on 15/16 of the CUs (240 of 256): the grid
  // on every CU took 1-3 % longer there (1 M x 4 KiB: 641 against 626 us,
  // 1.5 M: 972-992 against 957-980; 1 M x 1 KiB: 163-165 against 162; grids
  // of 248 / 244 read 670) and left no CU to a collective kernel on another
  // stream (bench.py's overlapped RCCL all-gather at N > 1); from 2 M x 4 KiB
  // on, every CU is as fast or faster (profiles/r03/s31_sck_grid_sweep.txt,
  // s32_sck_grid_sweep_4k_1k.txt, s33_ab_sck_grid_15_16.txt,
  // s34_sck_grid_by_batch_size.txt, s30_sck_overlap_standin.txt).
  const uint64_t full = (uint64_t)d.n_cu;
  const uint64_t cus = groups <= 48ull * 16ull * full ? (uint64_t)std::max(1, d.n_cu - d.n_cu / 16) : full;
  int g = (int)std::max<uint64_t>(1, std::min<uint64_t>(cus, (groups + 15) / 16));
  if (d.knobs.sck_grid > 0) g = std::min(g, d.knobs.sck_grid);
  return g;
}

// Whether a ragged range of `count` packets takes the workgroup-local kernel
// (icrc_rswg_kernel, one launch) rather than the bucket / fold / gather
// pipeline: up to RICRC_WG_CHUNKS (default 8) chunks of kRsWgCap packets on
// the most loaded workgroup -- every batch up to ~4.6 M packets on 256 CUs
// (C4, its 8-GPU shard, NIC rings of up to 4 M slots).  Same-box A/B
// (profiles/r06/): the shard 0.148 -> 0.131 ms of kernel per step, C4's 4 M
// (eight chunks) 0.971-0.974 -> 0.963-0.967 (session 20), 4 M x 4 KiB ring
// slots of 64-4082 B 1.46 -> 1.40; larger batches keep the pipeline.
// One decision for the launch, ricrc_kernel_path and ricrc_launch_info.
bool rs_use_wg(const Dev &d, uint64_t count) {
  if (d.knobs.wg_chunks <= 0 || count == 0) return false;
  if (d.knobs.one_line_in_gather || d.knobs.pass_grid > 0) return false;  // (knobs of the three-pass pipeline)
  int rgrid = d.n_cu;
  if (d.knobs.rsck_grid > 0) rgrid = std::min(rgrid, d.knobs.rsck_grid);
  const XcdWeights xw = xcd_weights(d.knobs, 40);
  return rs_wg_chunks(count, rgrid, xw.w) <= (uint64_t)d.knobs.wg_chunks;
}

// The ragged strided-chain pipeline (icrc_rsck.hip) on packets [0, count) of
// the batch, count < 2^31.
int launch_rsck_range(Dev &d, const uint8_t *base, const uint64_t *off, const uint32_t *len, uint64_t stride,
                      uint64_t count, uint32_t fixed_len, uint32_t l3_offset, uint32_t *out, hipStream_t st,
                      bool verify) {
  RsckArgs k{};
  k.base = base;
  k.off = off;
  k.len = len;
  k.stride = stride;
  k.count = count;
  k.fixed_len = fixed_len;
  k.l3_offset = l3_offset;
  k.verify = verify ? 1u : 0u;
  k.group_cost = d.knobs.gcost ? d.knobs.gcost : kRsGroupCost;
  k.small_in_fold = d.knobs.one_line_in_gather ? 0u : 1u;
  k.small_slots = d.knobs.small_slots < 0 ? kRsSmallSlots : (uint32_t)d.knobs.small_slots;
  const XcdWeights xw = xcd_weights(d.knobs, 40);
  for (int x = 0; x < 8; ++x) k.xw[x] = xw.w[x];
  k.no_split = d.knobs.no_gather_split ? 1u : 0u;
  k.out = out;
  k.tzb = d.d_tzb;
  k.fin = d.d_fin + kFinSck;  // the fold's finish tables
  int rgrid = d.n_cu;
  if (d.knobs.rsck_grid > 0) rgrid = std::min(rgrid, d.knobs.rsck_grid);
  const bool wg = rs_use_wg(d, count);
  Dev::Ws *ws = nullptr;
  if (!wg) {
    const int wrc = ragged_ws(d, st, rs_workspace_bytes(count), &ws);
    if (wrc) return wrc;
    rs_bind_workspace(k, ws->p);
  } else {
    k.xcd_k = xcd_start(d.h_xcd);
    k.xcd_rec = d.d_xcd_rec;
  }
  hipEvent_t *pev = nullptr;
  if (d.knobs.pass_times && count > 0 && count <= kRsMaxCount) {  // (launch_rsck records all five events then)
    if (d.pt_ev.empty()) {
      d.pt_ev.resize(5 * Dev::kPtSets);
      for (hipEvent_t &ev : d.pt_ev) HIP_TRY(hipEventCreate(&ev));
    }
    pev = &d.pt_ev[5 * d.pt_next];  // a ring: the last kPtSets calls are kept
    d.pt_next = (d.pt_next + 1) % Dev::kPtSets;
    d.pt_used = std::min(d.pt_used + 1, Dev::kPtSets);
  }
  if (wg) return hip_err(launch_rswg(k, rgrid, st, pev));  // no workspace
  const hipError_t e = launch_rsck(k, rgrid, d.knobs.pass_grid, st, pev);
  if (e != hipSuccess) ws->dirty = true;
  const hipError_t e2 = hipEventRecord(ws->done, st);
  return hip_err(e != hipSuccess ? e : e2);
}

// The kernel path of a batch: ONE decision, used by launch_batch_v4 and by
// ricrc_kernel_path (which bench.py and the tests query, so the labels of a
// run cannot drift from what ran).
enum class Path { kSck, kSckFramed, kQuad, kTsk, kStream, kRagged };

// Chunks of a fixed-length batch per lane of the direct streaming kernel
// (1, 2 or 4), or 0 if its packets are too long for it.
int stream_cpl(uint32_t fixed_len) {
  const uint32_t M = fixed_len - 4;
  for (int c : {1, 2, 4})
    if ((M + 64u * c - 1) / (64u * c) <= 64) return c;
  return 0;
}

Path choose_path(const Knobs &kn, const uint8_t *base, const uint64_t *off, const uint32_t *len, uint64_t stride,
                 uint32_t l3_offset) {
  const uint8_t *first = base + l3_offset;
  const uint32_t fixed_len = stride > l3_offset ? (uint32_t)std::min<uint64_t>(stride - l3_offset, 0xFFFFFFFFu) : 0u;
  const bool aligned = ((uintptr_t)first % 16 == 0) && (stride % 16 == 0);
  // An Ethernet-framed ring of 1, 2 or 4 KiB slots: the strided-chain kernel over the slots.
  if (sck_framed(kn, base, off, len, stride, l3_offset) && fixed_len >= kMinLen) return Path::kSckFramed;
  if (off || len || !aligned || fixed_len < kMinLen || fixed_len > kMaxLen || fixed_len % 4 != 0) return Path::kRagged;
  // Back-to-back 1, 2 or 4 KiB packets: the strided-chain kernel (no LDS transpose).
  if (l3_offset == 0 && (uintptr_t)base % 16 == 0 && !kn.no_sck && (stride == 1024 || stride == 2048 || stride == 4096))
    return Path::kSck;
  // Back-to-back 64-byte packets (C1): the quad kernel, coalesced 1 KiB loads.
  if (fixed_len == 64 && stride == 64 && l3_offset == 0 && (uintptr_t)base % 16 == 0 && !kn.no_quad) return Path::kQuad;
  const int cpl = stream_cpl(fixed_len);
  // Back-to-back packets of 32 * 2^j bytes: coalesced + LDS-transposed kernel.
  // (64-byte packets: the direct streaming kernel is faster, 20.1 vs 23.8 us on 1 M x 64 B.)
  if (cpl && l3_offset == 0 && stride == fixed_len && fixed_len >= 128 && fixed_len <= 4096 &&
      (fixed_len & (fixed_len - 1)) == 0 && ((uintptr_t)base % 16 == 0) && !kn.no_tsk)
    return Path::kTsk;
  // any other fixed length up to 16 KiB: lanes fold 64 CPL-byte chunks
  return cpl ? Path::kStream : Path::kRagged;
}

const char *path_kernels(Path p, bool one_line_pass, bool wg = false) {
  switch (p) {
    case Path::kSck:
    case Path::kSckFramed: return "icrc_sck_kernel";
    case Path::kQuad: return "icrc_quad_kernel";
    case Path::kTsk: return "icrc_tsk_kernel";
    case Path::kStream: return "icrc_stream_kernel";
    default:
      if (wg) return "icrc_rswg_kernel";
      return one_line_pass ? "rsck_bucket+icrc_rsck_kernel+icrc_rsmall_kernel+rsck_gather" : "rsck_bucket+icrc_rsck_kernel+rsck_gather";
  }
}

// Grids of the fixed-length kernels (one decision for the launch and
// ricrc_launch_info): one 1024-thread workgroup per CU at most, 16 waves of
// work per workgroup.
int quad_grid(const Dev &d, uint64_t count) {  // a wave step reads 4 KiB (64 packets)
  const uint64_t steps = (count * 64 + 4095) / 4096;
  return (int)std::max<uint64_t>(1, std::min<uint64_t>((uint64_t)d.n_cu, (steps + 15) / 16));
}
int tsk_grid(const Dev &d, uint64_t count, uint64_t stride) {  // a wave step re-lays a 4 KiB region
  const uint64_t n_iters = (count * stride + 4095) / 4096;
  return (int)std::max<uint64_t>(1, std::min<uint64_t>((uint64_t)d.n_cu, (n_iters + 15) / 16));
}
// The direct streaming kernel's packets: P lanes of 64 cpl bytes each,
// 64 >> log2(P) packets per wave step.
uint32_t stream_lanes(uint32_t fixed_len, int cpl) { return (fixed_len - 4 + 64u * cpl - 1) / (64u * cpl); }
int stream_grid(const Dev &d, uint64_t count, uint32_t P) {
  const uint64_t ppw = 64u >> ilog2_ceil(P);
  const uint64_t n_iters = (count + ppw - 1) / ppw;
  return (int)std::max<uint64_t>(1, std::min<uint64_t>((uint64_t)d.n_cu, (n_iters + 15) / 16));
}

int launch_batch_v4(Dev &d, const uint8_t *base, const uint64_t *off, const uint32_t *len, uint64_t stride,
                    uint64_t count, uint32_t l3_offset, uint32_t *out, hipStream_t st, bool verify,
                    uint32_t family = kFamV4) {
  if (count == 0) return 0;
  const uint8_t *first = base + l3_offset;
  const uint32_t fixed_len = stride > l3_offset ? (uint32_t)std::min<uint64_t>(stride - l3_offset, 0xFFFFFFFFu) : 0u;
  const Path path = choose_path(d.knobs, base, off, len, stride, l3_offset);
  if (path != Path::kRagged) {
    // Back-to-back 1, 2 or 4 KiB packets: the strided-chain kernel (no LDS transpose).
    if (path == Path::kSck || path == Path::kSckFramed) {
      const int sgrid = sck_grid(d, base, off, len, stride, count, l3_offset);
      SckArgs k{};
      k.family = family;
      k.base = base;
      k.count = count;
      k.out = out;
      k.n = (uint32_t)stride;
      k.l3_offset = l3_offset;
      k.verify = verify ? 1u : 0u;
      k.fin = d.d_fin;  // the SCK's finish tables
      const XcdWeights xw = xcd_weights(d.knobs, stride != 4096 ? 0 : sgrid < d.n_cu ? 25 : 50);
      for (int x = 0; x < 8; ++x) k.xw[x] = xw.w[x];
      k.xcd_k = xcd_start(d.h_xcd);
      k.xcd_rec = d.d_xcd_rec;
      return hip_err(launch_sck(k, sgrid, st));
    }
    const uint32_t M = fixed_len - 4;
    if (path == Path::kQuad) {
      QuadArgs q{};
      q.base = base;
      q.count = count;
      q.out = out;
      q.verify = verify ? 1u : 0u;
      return hip_err(launch_quad(q, quad_grid(d, count), st));
    }
    const int cpl = stream_cpl(fixed_len);
    if (path == Path::kTsk) {
      TskArgs t{};
      t.base = base;
      t.stride = stride;
      t.count = count;
      t.out = out;
      t.n_iters = (count * stride + 4095) / 4096;
      t.log2C = (uint32_t)ilog2_ceil(fixed_len / 32);
      t.verify = verify ? 1u : 0u;
      for (uint32_t p = 0; p < 128; ++p) {
        const int64_t dd = (int64_t)M - 32 * (int64_t)(p + 1);
        t.K[p] = p < fixed_len / 32 ? (dd >= 0 ? gf_x8n((uint64_t)dd) : gf_xinv8n((uint64_t)-dd)) : 0u;
      }
      const uint32_t y = gf_x8n(2048);
      for (int j = 0; j < 32; ++j) t.YB[j] = gf_mul(y, 1u << j);
      return hip_err(launch_tsk(t, tsk_grid(d, count, stride), st));
    }
    {  // Path::kStream: any other fixed length up to 16 KiB, lanes fold 64 CPL-byte chunks
      StreamArgs a{};
      const uint32_t chunk = 64u * cpl;
      a.base = first;
      a.stride = stride;
      a.count = count;
      a.out = out;
      a.len = fixed_len;
      a.P = stream_lanes(fixed_len, cpl);
      a.log2P2 = (uint32_t)ilog2_ceil(a.P);
      a.nw_last = (M - chunk * (a.P - 1)) / 4;
      const uint64_t ppw = 64u >> a.log2P2;
      a.n_iters = (count + ppw - 1) / ppw;
      a.verify = verify ? 1u : 0u;
      for (uint32_t c = 0; c < 64; ++c) {
        if (c >= a.P) a.K[c] = 0;
        else a.K[c] = x8n_host((uint64_t)M - std::min<uint64_t>((uint64_t)chunk * (c + 1), M));
      }
      return hip_err(launch_stream(a, cpl, stream_grid(d, count, a.P), st));
    }
  }
  // Everything else (offsets, lengths, any alignment, Ethernet framing): the
  // ragged strided-chain pipeline, packets bucketed on the device by line
  // count; cut into ranges of kRsChunk packets (its positions are 32-bit).
  for (uint64_t lo = 0; lo < count; lo += kRsChunk) {
    const uint64_t m = std::min<uint64_t>(kRsChunk, count - lo);
    const uint8_t *b = off ? base : base + lo * stride;  // no offsets: the range's first frame at lo * stride
    const int rc = launch_rsck_range(d, b, off ? off + lo : nullptr, len ? len + lo : nullptr, stride, m,
                                     fixed_len, l3_offset, out + lo, st, verify);
    if (rc) return rc;
  }
  return 0;
}

// Any address family: the IPv4-mask kernels, then (IPv6 / AUTO) the linear
// header fix-up, which also does the verify compare in that case.
int launch_batch(Dev &d, const uint8_t *base, const uint64_t *off, const uint32_t *len, uint64_t stride,
                 uint64_t count, uint32_t l3_offset, uint32_t *out, hipStream_t st, bool verify,
                 uint32_t family = kFamV4) {
  if (family == kFamV4 || count == 0)
    return launch_batch_v4(d, base, off, len, stride, count, l3_offset, out, st, verify);
  if (choose_path(d.knobs, base, off, len, stride, l3_offset) == Path::kSck)  // masks native in the kernel
    return launch_batch_v4(d, base, off, len, stride, count, l3_offset, out, st, verify, family);
  const int rc = launch_batch_v4(d, base, off, len, stride, count, l3_offset, out, st, false);
  if (rc) return rc;
  FamilyFixArgs f{};
  f.base = base;
  f.off = off;
  f.len = len;
  f.x8n = d.d_x8n;
  f.out = out;
  f.stride = stride;
  f.count = count;
  f.fixed_len = stride > l3_offset ? (uint32_t)std::min<uint64_t>(stride - l3_offset, 0xFFFFFFFFu) : 0u;
  f.l3_offset = l3_offset;
  f.family = family;
  f.verify = verify ? 1u : 0u;
  return hip_err(launch_family_fix(f, 16 * d.n_cu, st));
}

// ------------------------------------------------------------------- RCCL
// Resolved at run time (dlopen), so libroceicrc carries no link-time RCCL
// dependency and shares the process's RCCL when one is already loaded (e.g.
// torch's, same SONAME librccl.so.1).  Single process, N devices:
// ncclCommInitAll; the one collective is the all-gather of
// the 4-byte results.
struct Rccl {
  bool tried = false, ok = false;
  ncclResult_t (*init_all)(ncclComm_t *, int, const int *) = nullptr;
  ncclResult_t (*destroy)(ncclComm_t) = nullptr;
  ncclResult_t (*all_gather)(const void *, void *, size_t, ncclDataType_t, ncclComm_t, hipStream_t) = nullptr;
  ncclResult_t (*send)(const void *, size_t, ncclDataType_t, int, ncclComm_t, hipStream_t) = nullptr;
  ncclResult_t (*recv)(void *, size_t, ncclDataType_t, int, ncclComm_t, hipStream_t) = nullptr;
  ncclResult_t (*group_start)() = nullptr;
  ncclResult_t (*group_end)() = nullptr;
  const char *(*err_str)(ncclResult_t) = nullptr;
};

Rccl &rccl() {
  static Rccl r;
  if (r.tried) return r;
  r.tried = true;
  void *h = dlopen("librccl.so.1", RTLD_NOW | RTLD_NOLOAD);
  if (!h) h = dlopen("librccl.so.1", RTLD_NOW);
  if (!h) h = dlopen("/opt/rocm/lib/librccl.so.1", RTLD_NOW);
  if (!h) return r;
  auto sym = [&](auto &fp, const char *name) {
    fp = reinterpret_cast<std::remove_reference_t<decltype(fp)>>(dlsym(h, name));
    return fp != nullptr;
  };
  r.ok = sym(r.init_all, "ncclCommInitAll") && sym(r.destroy, "ncclCommDestroy") &&
         sym(r.all_gather, "ncclAllGather") && sym(r.send, "ncclSend") && sym(r.recv, "ncclRecv") &&
         sym(r.group_start, "ncclGroupStart") && sym(r.group_end, "ncclGroupEnd") &&
         sym(r.err_str, "ncclGetErrorString");
  return r;
}

int nccl_err(ncclResult_t e) {
  if (e == ncclSuccess) return 0;
  if (g_debug) fprintf(stderr, "libroceicrc: RCCL error %d: %s\n", (int)e, rccl().err_str(e));
  return -EIO;
}

void comm_destroy(ricrc_ctx *ctx) {
  if (ctx->comms.empty()) return;
  for (size_t k = 0; k < ctx->comms.size(); ++k) {
    DeviceGuard g(ctx->devs[k].id);
    (void)hipStreamSynchronize(ctx->devs[k].stream);
    if (ctx->comms[k]) (void)rccl().destroy(ctx->comms[k]);
  }
  ctx->comms.clear();
}

// All-gather of per-device result vectors in place: device k's d_out[k]
// holds its shard's counts[k] results at offset sum(counts[<k]) and ends with
// all of them.  The calls come from allgather_plan (icrc_plan.h, checked on
// the CPU): equal shards, one in-place ncclAllGather per device; unequal
// shards, ncclSend / ncclRecv pairs; every device's calls in one group.
int comm_allgather(ricrc_ctx *ctx, const uint64_t *counts, uint32_t *const *d_out) {
  Rccl &r = rccl();
  const std::vector<ricrc_xfer> plan = allgather_plan((int)ctx->devs.size(), counts);
  if (plan.empty()) return 0;  // one device (or nothing to move): already in place
  int rc = nccl_err(r.group_start());
  if (rc) return rc;
  for (const ricrc_xfer &x : plan) {
    const ncclComm_t comm = ctx->comms[x.dev];
    const hipStream_t st = ctx->devs[x.dev].stream;
    uint32_t *buf = d_out[x.dev];
    if (x.kind == RICRC_XFER_ALLGATHER)
      rc = nccl_err(r.all_gather(buf + x.offset, buf, (size_t)x.count, ncclUint32, comm, st));
    else if (x.kind == RICRC_XFER_SEND)
      rc = nccl_err(r.send(buf + x.offset, (size_t)x.count, ncclUint32, x.peer, comm, st));
    else
      rc = nccl_err(r.recv(buf + x.offset, (size_t)x.count, ncclUint32, x.peer, comm, st));
    if (rc) break;
  }
  const int rc2 = nccl_err(r.group_end());
  return rc ? rc : rc2;
}

// Per-packet status (or classification) of a batch after its ICRC kernels,
// in stream order (icrc_status.hip).  accept: bit 0 RoCEv2/IPv4, bit 1
// RoCEv2/IPv6 (0: lengths only); ether: check the EtherType before L3.
// A fixed-length batch checked for lengths only is all RICRC_ST_OK (its one
// length was validated by the caller): a memset, no kernel.
int launch_status_pass(Dev &d, const uint8_t *base, const uint64_t *off, const uint32_t *len, uint64_t stride,
                       uint64_t count, uint32_t l3_offset, uint32_t accept, bool ether, uint32_t *out,
                       uint8_t *status, uint8_t *cls, hipStream_t st) {
  if (count == 0) return 0;
  if (!cls && !len && !accept) return hip_err(hipMemsetAsync(status, (int)kStOk, count, st));
  StatusArgs a{};
  a.base = base;
  a.off = off;
  a.len = len;
  a.stride = stride;
  a.count = count;
  a.fixed_len = stride > l3_offset ? (uint32_t)std::min<uint64_t>(stride - l3_offset, 0xFFFFFFFFu) : 0u;
  a.l3_offset = l3_offset;
  a.accept = accept;
  a.ether = ether ? 1u : 0u;
  a.out = out;
  a.status = status;
  a.cls = cls;
  return hip_err(launch_status(a, d.n_cu, st));
}

// flags of the *_st calls: a family | RICRC_F_STRICT | RICRC_F_VERIFY | RICRC_F_FRAMELEN.
struct StFlags {
  uint32_t fam;
  bool strict, verify, framelen;
  uint32_t accept;  // StatusArgs::accept
};
bool decode_st_flags(uint32_t flags, StFlags &f) {
  if (flags & ~(3u | RICRC_F_STRICT | RICRC_F_VERIFY | RICRC_F_FRAMELEN)) return false;
  f.fam = flags & 3u;
  if (f.fam > RICRC_F_AUTO) return false;
  f.strict = (flags & RICRC_F_STRICT) != 0;
  f.verify = (flags & RICRC_F_VERIFY) != 0;
  f.framelen = (flags & RICRC_F_FRAMELEN) != 0;
  f.accept = !f.strict ? 0u : f.fam == RICRC_F_IPV4 ? 1u : f.fam == RICRC_F_IPV6 ? 2u : 3u;
  return true;
}

Knobs read_knobs() {
  Knobs k;
  auto num = [](const char *name, long dflt) -> long {
    const char *e = getenv(name);
    return e ? atol(e) : dflt;
  };
  k.no_sck = getenv("RICRC_NO_SCK") != nullptr;
  k.no_framed = getenv("RICRC_NO_FRAMED") != nullptr;
  k.no_gather_split = getenv("RICRC_NO_GATHER_SPLIT") != nullptr;
  k.no_tsk = getenv("RICRC_NO_TSK") != nullptr;
  k.no_quad = getenv("RICRC_NO_QUAD") != nullptr;
  k.sck_grid = (int)std::max(0L, num("RICRC_SCK_GRID", 0));
  k.rsck_grid = (int)std::max(0L, num("RICRC_RSCK_GRID", 0));
  k.gcost = (uint32_t)std::min(1024L, std::max(0L, num("RICRC_RS_GCOST", 0)));  // the packed work counter's range
  k.one_line_in_gather = getenv("RICRC_ONE_LINE_IN_GATHER") != nullptr;
  k.small_slots = (int)std::min(16L, std::max(-1L, num("RICRC_SMALL_SLOTS", -1)));  // (16 waves a workgroup)
  k.wg_chunks = getenv("RICRC_NO_WG") ? 0 : (int)std::min(64L, std::max(0L, num("RICRC_WG_CHUNKS", 8)));
  k.pass_grid = (int)std::max(0L, num("RICRC_RS_PASS_GRID", 0));
  k.pass_times = getenv("RICRC_PASS_TIMES") != nullptr;
  k.fail_chunk = num("RICRC_FAIL_CHUNK", -1);
  k.xcd_skew = (int)std::min(500L, std::max(-1L, num("RICRC_XCD_SKEW", -1)));
  // Eight weights in 1..8000, else ignored.  The bound keeps xcd_share's
  // 64-bit products exact: total work S < 2^28 packets x 2064 quarter-steps
  // = 2^39.01, times the weight sum of 256 workgroups x 16 waves (at most
  // 512 x 64000 < 2^24.97) stays below 2^64.
  if (const char *e = getenv("RICRC_XCD_WEIGHTS")) {
    uint32_t w[8];
    int n = 0;
    for (const char *c = e; *c && n < 8;) {
      const long v = atol(c);
      if (v < 1 || v > 8000) break;
      w[n++] = (uint32_t)v;
      while (*c && *c != ',') ++c;
      if (*c == ',') ++c;
    }
    if (n == 8)
      for (int x = 0; x < 8; ++x) k.xcd_w[x] = w[x];
  }
  const unsigned hw = std::thread::hardware_concurrency();
  k.host_threads = (int)std::max(1L, std::min(64L, num("RICRC_HOST_THREADS", (long)std::min(16u, std::max(1u, hw)))));
  return k;
}

}  // namespace

extern "C" {

int ricrc_create_devices(ricrc_ctx **ctx, const int *devices, int n) {
  if (!ctx || !devices || n <= 0) return -EINVAL;
  *ctx = nullptr;
  int avail = 0;
  if (hipGetDeviceCount(&avail) != hipSuccess || avail <= 0) {
    (void)hipGetLastError();
    return -ENODEV;
  }
  for (int i = 0; i < n; ++i)
    if (devices[i] < 0 || devices[i] >= avail) return -ENODEV;
  ricrc_ctx *c = new (std::nothrow) ricrc_ctx;
  if (!c) return -ENOMEM;
  c->knobs = read_knobs();
  c->fail_once.store(c->knobs.fail_chunk);
  g_debug = getenv("RICRC_DEBUG") != nullptr;
  c->devs.resize(n);
  for (int i = 0; i < n; ++i) {
    c->devs[i].id = devices[i];
    c->devs[i].knobs = c->knobs;
    const int rc = init_dev(c->devs[i]);
    if (rc) {
      ricrc_destroy(c);
      return rc;
    }
  }
  *ctx = c;
  return 0;
}

int ricrc_create(ricrc_ctx **ctx, int n_gpus) {
  if (!ctx || n_gpus == 0) return -EINVAL;
  *ctx = nullptr;
  int avail = 0;
  if (hipGetDeviceCount(&avail) != hipSuccess || avail <= 0) {
    (void)hipGetLastError();
    return -ENODEV;
  }
  const int n = n_gpus < 0 ? avail : n_gpus;
  if (n > avail) return -ENODEV;
  std::vector<int> ids(n);
  for (int i = 0; i < n; ++i) ids[i] = i;
  return ricrc_create_devices(ctx, ids.data(), n);
}

void ricrc_destroy(ricrc_ctx *ctx) {
  if (!ctx) return;
  comm_destroy(ctx);
  for (Dev &d : ctx->devs) free_dev(d);
  for (const HostRange &r : ctx->pinned) {
    if (r.owned) (void)hipHostFree((void *)r.lo);
    else (void)hipHostUnregister((void *)r.lo);
  }
  delete ctx;
}

int ricrc_device_count(const ricrc_ctx *ctx) { return ctx ? (int)ctx->devs.size() : 0; }

void *ricrc_stream(ricrc_ctx *ctx, int dev) {
  if (!ctx || dev < 0 || dev >= (int)ctx->devs.size()) return nullptr;
  return ctx->devs[dev].stream;
}

int ricrc_pass_times(ricrc_ctx *ctx, int dev, float *ms, int n) {
  if (!ctx || dev < 0 || dev >= (int)ctx->devs.size() || (n > 0 && !ms)) return -EINVAL;
  Dev &d = ctx->devs[dev];
  DeviceGuard g(d.id);
  if (!g.ok()) return -ENODEV;
  for (int k = 0; k < n; ++k) ms[k] = 0.f;
  const int used = d.pt_used;
  d.pt_used = 0;  // forgotten whatever happens below: a failed query does not fail every later one
  for (int c = 0; c < used; ++c) {  // the oldest recorded set first
    hipEvent_t *e = &d.pt_ev[5 * ((d.pt_next - used + c + Dev::kPtSets) % Dev::kPtSets)];
    HIP_TRY(hipEventSynchronize(e[4]));
    for (int k = 0; k < 4 && k < n; ++k) {
      float t = 0.f;
      HIP_TRY(hipEventElapsedTime(&t, e[k], e[k + 1]));
      ms[k] += t;
    }
  }
  return used;
}

const char *ricrc_kernel_path(const ricrc_ctx *ctx, const void *d_base, const uint64_t *d_off, const uint32_t *d_len,
                              uint32_t stride, uint64_t count, uint32_t l3_offset, uint32_t flags) {
  if (!d_base || flags > RICRC_F_AUTO || count == 0) return nullptr;
  if ((!d_off && stride == 0) || (!d_len && stride <= l3_offset)) return nullptr;
  const Knobs kn = ctx ? ctx->knobs : Knobs{};
  const Path p = choose_path(kn, (const uint8_t *)d_base, d_off, d_len, stride, l3_offset);
  // the ragged pipeline's first range (launch_batch_v4 cuts at kRsChunk) decides the one-line pass:
  // none when the fold (the default) or the gather (a fused pass shape) folds those packets
  const bool one_line_pass = kn.one_line_in_gather && !rs_fused(std::min<uint64_t>(count, kRsChunk), kn.pass_grid);
  // ... and whether it takes the workgroup-local kernel (ctx NULL: a 256-CU MI355X)
  Dev nodev{};
  nodev.n_cu = 256;
  nodev.knobs = kn;
  const bool wg = rs_use_wg(ctx && !ctx->devs.empty() ? ctx->devs[0] : nodev, std::min<uint64_t>(count, kRsChunk));
  if (flags == RICRC_F_IPV4 || p == Path::kSck) return path_kernels(p, one_line_pass, wg);  // the SCK applies every family natively
  if (p == Path::kRagged && wg) return "icrc_rswg_kernel+family_fix_kernel";
  switch (p) {  // IPv6 / AUTO: the IPv4-mask kernels, then the linear header fix-up
    case Path::kSckFramed: return "icrc_sck_kernel+family_fix_kernel";
    case Path::kQuad: return "icrc_quad_kernel+family_fix_kernel";
    case Path::kTsk: return "icrc_tsk_kernel+family_fix_kernel";
    case Path::kStream: return "icrc_stream_kernel+family_fix_kernel";
    default:
      return one_line_pass ? "rsck_bucket+icrc_rsck_kernel+icrc_rsmall_kernel+rsck_gather+family_fix_kernel"
                           : "rsck_bucket+icrc_rsck_kernel+rsck_gather+family_fix_kernel";
  }
}

int ricrc_launch_info(const ricrc_ctx *ctx, int dev, const void *d_base, const uint64_t *d_off,
                      const uint32_t *d_len, uint32_t stride, uint64_t count, uint32_t l3_offset,
                      ricrc_launch_info_t *info) {
  if (!info || dev < 0 || (ctx && dev >= (int)ctx->devs.size()) || (!ctx && dev != 0) || !d_base || count == 0)
    return -EINVAL;
  if ((!d_off && stride == 0) || (!d_len && stride <= l3_offset)) return -EINVAL;
  // ctx NULL: the dispatch on a 256-CU MI355X with the default knobs (no GPU needed)
  Dev nodev{};
  nodev.n_cu = 256;
  const Dev &d = ctx ? ctx->devs[dev] : nodev;
  *info = ricrc_launch_info_t{};
  info->start_xcd = xcd_start(d.h_xcd);
  const uint8_t *base = (const uint8_t *)d_base;
  const Path p = choose_path(d.knobs, base, d_off, d_len, stride, l3_offset);
  XcdWeights xw{};
  const uint32_t fixed_len = stride > l3_offset ? (uint32_t)std::min<uint64_t>(stride - l3_offset, 0xFFFFFFFFu) : 0u;
  if (p == Path::kSck || p == Path::kSckFramed) {
    info->grid = (uint32_t)sck_grid(d, base, d_off, d_len, stride, count, l3_offset);
    xw = xcd_weights(d.knobs, stride != 4096 ? 0 : (int)info->grid < d.n_cu ? 25 : 50);
    info->lanes_per_packet = 8;  // lane 8 g + s: slot s of every line of packet g
  } else if (p == Path::kQuad) {
    info->grid = (uint32_t)quad_grid(d, count);
    info->lanes_per_packet = 4;  // a lane quad per 64-byte packet
  } else if (p == Path::kTsk) {
    info->grid = (uint32_t)tsk_grid(d, count, stride);
    info->lanes_per_packet = fixed_len / 32;  // contiguous 32-byte chunks per lane
  } else if (p == Path::kStream) {
    const uint32_t P = stream_lanes(fixed_len, stream_cpl(fixed_len));
    info->grid = (uint32_t)stream_grid(d, count, P);
    info->lanes_per_packet = 1u << ilog2_ceil(P);  // P chunk lanes, padded to a power of two
  } else if (p == Path::kRagged && rs_use_wg(d, std::min<uint64_t>(count, kRsChunk))) {
    info->lanes_per_packet = 8;  // the fold's groups (one-line packets: one lane each)
    info->grid = (uint32_t)(d.knobs.rsck_grid > 0 ? std::min(d.n_cu, d.knobs.rsck_grid) : d.n_cu);
    xw = xcd_weights(d.knobs, 40);
    info->one_line = 2;  // folded by the kernel; no bucket / gather passes (pass_grid 0)
  } else if (p == Path::kRagged) {
    info->lanes_per_packet = 8;  // the fold's groups (one-line packets: one lane each)
    info->grid = (uint32_t)(d.knobs.rsck_grid > 0 ? std::min(d.n_cu, d.knobs.rsck_grid) : d.n_cu);
    xw = xcd_weights(d.knobs, 40);
    int pg = 0, pu = 0, gg = 0;
    bool fused = false;
    rs_pass_info(std::min<uint64_t>(count, kRsChunk), d.knobs.pass_grid, d.knobs.no_gather_split, &pg, &pu, &fused,
                 &gg);
    info->pass_grid = (uint32_t)pg;
    info->pass_unroll = (uint32_t)pu;
    const bool in_fold = !d.knobs.one_line_in_gather;
    info->one_line = in_fold ? 2u : fused ? 1u : 0u;
    info->gather_grid = in_fold ? (uint32_t)pg : (uint32_t)gg;
  }
  for (int x = 0; x < 8; ++x) info->xcd_weights[x] = xw.w[x];
  return 0;
}

static int batch_device_impl(ricrc_ctx *ctx, int dev, const void *d_base, const uint64_t *d_off,
                             const uint32_t *d_len, uint32_t stride, uint64_t count, uint32_t l3_offset,
                             uint32_t *d_out, void *stream, bool verify, uint32_t flags = RICRC_F_IPV4) {
  if (!ctx || dev < 0 || dev >= (int)ctx->devs.size()) return -EINVAL;
  if (flags > RICRC_F_AUTO) return -EINVAL;
  if (count == 0) return 0;
  if (!d_base || !d_out) return -EINVAL;
  if (!d_off && stride == 0) return -EINVAL;
  if (!d_len && (stride <= l3_offset)) return -EINVAL;
  Dev &d = ctx->devs[dev];
  DeviceGuard g(d.id);
  if (!g.ok()) return -ENODEV;
  hipStream_t st = (hipStream_t)stream;  // NULL = the HIP null stream, like any HIP API
  return launch_batch(d, (const uint8_t *)d_base, d_off, d_len, stride, count, l3_offset, d_out, st, verify, flags);
}

int ricrc_batch_device(ricrc_ctx *ctx, int dev, const void *d_base, const uint64_t *d_off,
                       const uint32_t *d_len, uint32_t stride, uint64_t count, uint32_t l3_offset,
                       uint32_t *d_out, void *stream) {
  return batch_device_impl(ctx, dev, d_base, d_off, d_len, stride, count, l3_offset, d_out, stream, false);
}

int ricrc_verify_device(ricrc_ctx *ctx, int dev, const void *d_base, const uint64_t *d_off,
                        const uint32_t *d_len, uint32_t stride, uint64_t count, uint32_t l3_offset,
                        uint32_t *d_out, void *stream) {
  return batch_device_impl(ctx, dev, d_base, d_off, d_len, stride, count, l3_offset, d_out, stream, true);
}

int ricrc_batch_device_ex(ricrc_ctx *ctx, int dev, const void *d_base, const uint64_t *d_off,
                          const uint32_t *d_len, uint32_t stride, uint64_t count, uint32_t l3_offset,
                          uint32_t *d_out, void *stream, uint32_t flags) {
  return batch_device_impl(ctx, dev, d_base, d_off, d_len, stride, count, l3_offset, d_out, stream, false, flags);
}

int ricrc_verify_device_ex(ricrc_ctx *ctx, int dev, const void *d_base, const uint64_t *d_off,
                           const uint32_t *d_len, uint32_t stride, uint64_t count, uint32_t l3_offset,
                           uint32_t *d_out, void *stream, uint32_t flags) {
  return batch_device_impl(ctx, dev, d_base, d_off, d_len, stride, count, l3_offset, d_out, stream, true, flags);
}

// The *_st device calls; extent > 0 (ricrc_batch_device_bounded): packets
// must lie in [d_base, d_base + extent).
static int batch_device_st_impl(ricrc_ctx *ctx, int dev, const void *d_base, uint64_t extent, const uint64_t *d_off,
                                const uint32_t *d_len, uint32_t stride, uint64_t count, uint32_t l3_offset,
                                uint32_t *d_out, uint8_t *d_status, void *stream, uint32_t flags) {
  StFlags f;
  if (!ctx || dev < 0 || dev >= (int)ctx->devs.size() || !decode_st_flags(flags, f)) return -EINVAL;
  if (count == 0) return 0;
  if (!d_base || !d_out || !d_status) return -EINVAL;
  if (!d_off && stride == 0) return -EINVAL;
  if (!d_len && (stride <= l3_offset || stride - l3_offset < kMinLen || stride - l3_offset > kMaxLen))
    return -EINVAL;  // one length for the whole batch: a call error, not a per-packet status
  // a fixed-stride batch either lies in the extent or is a call error
  if (extent && !d_off && !d_len && ((count - 1) > (extent / stride) || (count - 1) * stride + stride > extent))
    return -EINVAL;
  Dev &d = ctx->devs[dev];
  DeviceGuard g(d.id);
  if (!g.ok()) return -ENODEV;
  hipStream_t st = (hipStream_t)stream;
  const uint8_t *base = (const uint8_t *)d_base;
  // RICRC_F_FRAMELEN (the packets' L3 lengths from their IP headers) and / or
  // an extent over per-packet descriptors: one pre-pass writes the lengths
  // every later pass runs on (0 for a packet outside the extent), into the
  // tail of the stream's ragged workspace -- the batch takes the ragged
  // pipeline on them, whose workspace that is (no allocation per call).
  const bool pre = f.framelen || (extent && (d_off || d_len));
  Dev::Ws *ws = nullptr;
  if (pre) {
    const uint64_t at = (rs_workspace_bytes(std::min<uint64_t>(count, kRsChunk)) + 255) & ~255ull;
    const int wrc = ragged_ws(d, st, at + count * sizeof(uint32_t), &ws);
    if (wrc) return wrc;
    uint32_t *eff = reinterpret_cast<uint32_t *>(static_cast<char *>(ws->p) + at);
    FrameLenArgs fa{};
    fa.base = base;
    fa.off = d_off;
    fa.len = d_len;
    fa.stride = stride;
    fa.count = count;
    fa.fixed_len = d_len ? 0u : stride - l3_offset;
    fa.l3_offset = l3_offset;
    fa.eff = eff;
    fa.extent = extent;
    fa.framelen = f.framelen ? 1u : 0u;
    const int rc = hip_err(launch_framelen(fa, d.n_cu, st));
    if (rc) return rc;
    d_len = eff;  // every later pass runs on these lengths
  }
  int rc = launch_batch(d, base, d_off, d_len, stride, count, l3_offset, d_out, st, f.verify, f.fam);
  if (!rc)
    rc = launch_status_pass(d, base, d_off, d_len, stride, count, l3_offset, f.accept, f.strict && l3_offset >= 14,
                            d_out, d_status, nullptr, st);
  // the workspace's last use is the status pass (it reads the lengths): a
  // later reuse from another stream waits for it
  if (ws) {
    const int rc2 = hip_err(hipEventRecord(ws->done, st));
    if (!rc) rc = rc2;
  }
  return rc;
}

int ricrc_batch_device_st(ricrc_ctx *ctx, int dev, const void *d_base, const uint64_t *d_off,
                          const uint32_t *d_len, uint32_t stride, uint64_t count, uint32_t l3_offset,
                          uint32_t *d_out, uint8_t *d_status, void *stream, uint32_t flags) {
  return batch_device_st_impl(ctx, dev, d_base, 0, d_off, d_len, stride, count, l3_offset, d_out, d_status, stream,
                              flags);
}

int ricrc_batch_device_bounded(ricrc_ctx *ctx, int dev, const void *d_base, uint64_t base_bytes,
                               const uint64_t *d_off, const uint32_t *d_len, uint32_t stride, uint64_t count,
                               uint32_t l3_offset, uint32_t *d_out, uint8_t *d_status, void *stream, uint32_t flags) {
  if (base_bytes == 0) return -EINVAL;
  return batch_device_st_impl(ctx, dev, d_base, base_bytes, d_off, d_len, stride, count, l3_offset, d_out, d_status,
                              stream, flags);
}

int ricrc_classify_device(ricrc_ctx *ctx, int dev, const void *d_base, const uint64_t *d_off,
                          const uint32_t *d_len, uint32_t stride, uint64_t count, uint32_t l3_offset,
                          uint8_t *d_class, void *stream) {
  if (!ctx || dev < 0 || dev >= (int)ctx->devs.size()) return -EINVAL;
  if (count == 0) return 0;
  if (!d_base || !d_class) return -EINVAL;
  if (!d_off && stride == 0) return -EINVAL;
  if (!d_len && stride <= l3_offset) return -EINVAL;
  Dev &d = ctx->devs[dev];
  DeviceGuard g(d.id);
  if (!g.ok()) return -ENODEV;
  return launch_status_pass(d, (const uint8_t *)d_base, d_off, d_len, stride, count, l3_offset, 3u,
                            l3_offset >= 14, nullptr, nullptr, d_class, (hipStream_t)stream);
}

int ricrc_repair_device(ricrc_ctx *ctx, int dev, void *d_base, const uint64_t *d_off, const uint32_t *d_len,
                        uint32_t stride, uint64_t count, uint32_t l3_offset, uint32_t off, uint32_t len,
                        const uint8_t *d_old_bytes, uint32_t old_stride, uint32_t flags, uint32_t stamp,
                        uint32_t *d_out, void *stream) {
  if (!ctx || dev < 0 || dev >= (int)ctx->devs.size()) return -EINVAL;
  if (flags > RICRC_F_AUTO) return -EINVAL;
  if (len > RICRC_REPAIR_MAX || (uint64_t)off + len > kMaxLen - 4) return -EINVAL;
  if (count == 0) return 0;
  if (!d_base || (len && !d_old_bytes) || (!d_out && !stamp)) return -EINVAL;
  if (count > 1 && old_stride < len) return -EINVAL;
  if (!d_off && stride == 0) return -EINVAL;
  if (!d_len && stride <= l3_offset) return -EINVAL;
  Dev &d = ctx->devs[dev];
  DeviceGuard g(d.id);
  if (!g.ok()) return -ENODEV;
  RepairArgs a{};
  a.base = (uint8_t *)d_base;
  a.off = d_off;
  a.len = d_len;
  a.old_bytes = d_old_bytes;
  a.x8n = d.d_x8n;
  a.out = d_out;
  a.stride = stride;
  a.old_stride = old_stride;
  a.count = count;
  a.fixed_len = stride > l3_offset ? (uint32_t)std::min<uint64_t>(stride - l3_offset, 0xFFFFFFFFu) : 0u;
  a.l3_offset = l3_offset;
  a.roff = off;
  a.rlen = len;
  a.family = flags;
  a.stamp = stamp ? 1u : 0u;
  return hip_err(launch_repair(a, 16 * d.n_cu, (hipStream_t)stream));
}

int ricrc_synth_device(ricrc_ctx *ctx, int dev, uint64_t seed, uint64_t first, uint64_t count, uint32_t n,
                       uint32_t stride, void *d_buf, void *stream) {
  if (!ctx || dev < 0 || dev >= (int)ctx->devs.size() || !d_buf) return -EINVAL;
  if (stride % 8 != 0 || n > stride || n < 4) return -EINVAL;
  Dev &d = ctx->devs[dev];
  DeviceGuard g(d.id);
  if (!g.ok()) return -ENODEV;
  SynthArgs a{(uint8_t *)d_buf, seed, first, count, n, stride, nullptr, nullptr};
  return hip_err(launch_synth(a, (hipStream_t)stream));
}

int ricrc_synth_ragged_device(ricrc_ctx *ctx, int dev, uint64_t seed, uint64_t first, uint64_t count,
                              const uint64_t *d_off, const uint32_t *d_len, void *d_buf, void *stream) {
  if (!ctx || dev < 0 || dev >= (int)ctx->devs.size()) return -EINVAL;
  if (count == 0) return 0;
  if (!d_buf || !d_off || !d_len) return -EINVAL;
  Dev &d = ctx->devs[dev];
  DeviceGuard g(d.id);
  if (!g.ok()) return -ENODEV;
  SynthArgs a{(uint8_t *)d_buf, seed, first, count, 0u, 0u, d_off, d_len};
  return hip_err(launch_synth_ragged(a, (hipStream_t)stream));
}

// Bring a device out of its idle power state before a latency-sensitive
// burst: a streaming read of a 256 MiB scratch buffer (icrc_prime_kernel, at
// HBM speed like the ICRC kernels), back to back, for `usec` microseconds.  Measured (tools/ramp_probe.py, profiles/r02/
// ramp_probe.jsonl): after >= 20 ms of GPU idle the 5th-12th launches of the
// 1 M x 4 KiB batch run 700-750 us instead of 645-650 us; 20 ms of busy work
// first removes that transient.
int ricrc_prime(ricrc_ctx *ctx, int dev, uint32_t usec) {
  if (!ctx || dev < 0 || dev >= (int)ctx->devs.size()) return -EINVAL;
  if (usec == 0) return 0;
  Dev &d = ctx->devs[dev];
  DeviceGuard g(d.id);
  if (!g.ok()) return -ENODEV;
  constexpr uint64_t kPkts = 65536, kN = 4096;
  uint8_t *buf = nullptr;
  uint32_t *out = nullptr;
  HIP_TRY(hipMalloc(&buf, kPkts * kN));
  int rc = hip_err(hipMalloc(&out, 256 * sizeof(uint32_t)));
  if (!rc) rc = hip_err(hipMemsetAsync(buf, 0, kPkts * kN, d.stream));
  const auto t0 = std::chrono::steady_clock::now();
  while (!rc) {
    for (int k = 0; k < 16 && !rc; ++k) rc = hip_err(launch_prime(buf, kPkts * kN, out, d.n_cu, d.stream));
    if (!rc) rc = hip_err(hipStreamSynchronize(d.stream));
    const auto us = std::chrono::duration_cast<std::chrono::microseconds>(std::chrono::steady_clock::now() - t0);
    if (us.count() >= (long long)usec) break;
  }
  (void)hipStreamSynchronize(d.stream);
  (void)hipFree(out);
  (void)hipFree(buf);
  return rc;
}

void *ricrc_host_alloc(ricrc_ctx *ctx, uint64_t bytes) {
  if (!ctx || bytes == 0) return nullptr;
  void *p = nullptr;
  if (hipHostMalloc(&p, bytes, hipHostMallocPortable) != hipSuccess) {
    (void)hipGetLastError();
    return nullptr;
  }
  ctx->pinned.push_back({(uintptr_t)p, (uintptr_t)p + bytes, true});
  return p;
}

void ricrc_host_free(ricrc_ctx *ctx, void *p) {
  if (!ctx || !p) return;
  for (size_t i = 0; i < ctx->pinned.size(); ++i)
    if (ctx->pinned[i].owned && ctx->pinned[i].lo == (uintptr_t)p) {
      ctx->pinned.erase(ctx->pinned.begin() + i);
      (void)hipHostFree(p);
      return;
    }
}

int ricrc_host_register(ricrc_ctx *ctx, void *p, uint64_t bytes) {
  if (!ctx || !p || bytes == 0) return -EINVAL;
  const uintptr_t lo = (uintptr_t)p, hi = lo + bytes;
  for (const HostRange &r : ctx->pinned)
    if (lo < r.hi && r.lo < hi) return -EINVAL;  // overlaps a context range (HIP itself may accept it)
  const hipError_t e = hipHostRegister(p, bytes, hipHostRegisterPortable);
  if (e != hipSuccess) {
    (void)hipGetLastError();
    return e == hipErrorHostMemoryAlreadyRegistered ? -EINVAL : (e == hipErrorOutOfMemory ? -ENOMEM : -EIO);
  }
  ctx->pinned.push_back({(uintptr_t)p, (uintptr_t)p + bytes, false});
  return 0;
}

int ricrc_host_unregister(ricrc_ctx *ctx, void *p) {
  if (!ctx || !p) return -EINVAL;
  for (size_t i = 0; i < ctx->pinned.size(); ++i)
    if (!ctx->pinned[i].owned && ctx->pinned[i].lo == (uintptr_t)p) {
      ctx->pinned.erase(ctx->pinned.begin() + i);
      return hipHostUnregister(p) == hipSuccess ? 0 : ((void)hipGetLastError(), -EIO);
    }
  return -EINVAL;
}

int ricrc_comm_init(ricrc_ctx *ctx) {
  if (!ctx || ctx->devs.empty()) return -EINVAL;
  if (!ctx->comms.empty()) return 0;
  Rccl &r = rccl();
  if (!r.ok) return -ENODEV;
  std::vector<int> ids;
  for (const Dev &d : ctx->devs) ids.push_back(d.id);
  std::vector<ncclComm_t> comms(ids.size(), nullptr);
  const int rc = nccl_err(r.init_all(comms.data(), (int)ids.size(), ids.data()));
  if (rc) return rc;
  ctx->comms = comms;
  return 0;
}

int ricrc_allgather(ricrc_ctx *ctx, const uint64_t *counts, uint32_t *const *d_out) {
  if (!ctx || !counts || !d_out) return -EINVAL;
  if (ctx->comms.empty()) return -EINVAL;  // ricrc_comm_init first
  for (size_t k = 0; k < ctx->devs.size(); ++k)
    if (!d_out[k]) return -EINVAL;
  return comm_allgather(ctx, counts, d_out);
}

int ricrc_batch_device_all(ricrc_ctx *ctx, const void *const *d_base, const uint64_t *const *d_off,
                           const uint32_t *const *d_len, uint32_t stride, const uint64_t *counts,
                           uint32_t l3_offset, uint32_t *const *d_out, uint32_t flags) {
  if (!ctx || !d_base || !counts || !d_out || flags > RICRC_F_AUTO) return -EINVAL;
  if (ctx->comms.empty()) return -EINVAL;  // ricrc_comm_init first
  const int n = (int)ctx->devs.size();
  uint64_t at = 0;
  for (int k = 0; k < n; ++k) {
    if (!d_out[k] || (counts[k] && !d_base[k])) return -EINVAL;
    const uint64_t *off = d_off ? d_off[k] : nullptr;
    const uint32_t *len = d_len ? d_len[k] : nullptr;
    if (counts[k] && ((!off && stride == 0) || (!len && stride <= l3_offset))) return -EINVAL;
  }
  for (int k = 0; k < n; ++k) {
    Dev &d = ctx->devs[k];
    DeviceGuard g(d.id);
    if (!g.ok()) return -ENODEV;
    if (counts[k]) {
      const int rc = launch_batch(d, (const uint8_t *)d_base[k], d_off ? d_off[k] : nullptr, d_len ? d_len[k] : nullptr,
                                  stride, counts[k], l3_offset, d_out[k] + at, d.stream, false, flags);
      if (rc) return rc;
    }
    at += counts[k];
  }
  return comm_allgather(ctx, counts, d_out);
}

int ricrc_sync(ricrc_ctx *ctx) {
  if (!ctx) return -EINVAL;
  for (Dev &d : ctx->devs) {
    DeviceGuard g(d.id);
    if (!g.ok()) return -ENODEV;
    HIP_TRY(hipStreamSynchronize(d.stream));
  }
  return 0;
}

}  // extern "C"

namespace {

// True if [p, p+n) lies in host memory the DMA engines can read without a
// CPU bounce: a context range (ricrc_host_alloc / ricrc_host_register) or
// memory some other owner pinned (hipHostMalloc / hipHostRegister, e.g. a
// torch pinned tensor), as reported by the HIP pointer attributes.
bool dma_readable(const ricrc_ctx *ctx, const void *p, uint64_t n) {
  const uintptr_t lo = (uintptr_t)p, hi = lo + n;
  for (const HostRange &r : ctx->pinned)
    if (lo >= r.lo && hi <= r.hi) return true;
  hipPointerAttribute_t at;
  if (hipPointerGetAttributes(&at, p) != hipSuccess) {
    (void)hipGetLastError();
    return false;
  }
  if (at.type != hipMemoryTypeHost) return false;
  uintptr_t rs = 0;
  size_t rn = 0;
  if (hipPointerGetAttribute(&rs, HIP_POINTER_ATTRIBUTE_RANGE_START_ADDR, (hipDeviceptr_t)p) != hipSuccess ||
      hipPointerGetAttribute(&rn, HIP_POINTER_ATTRIBUTE_RANGE_SIZE, (hipDeviceptr_t)p) != hipSuccess) {
    (void)hipGetLastError();
    return false;
  }
  return lo >= rs && hi <= rs + rn;
}

// Run fn(lo, hi) over [0, n) on up to `threads` threads (the caller is one).
template <class F>
void par_for(uint64_t n, int threads, uint64_t grain, F fn) {
  const uint64_t t = std::max<uint64_t>(1, std::min<uint64_t>((uint64_t)threads, n / std::max<uint64_t>(1, grain)));
  if (t <= 1) {
    fn(0, n);
    return;
  }
  std::vector<std::thread> th;
  th.reserve(t - 1);
  for (uint64_t k = 1; k < t; ++k) th.emplace_back(fn, n * k / t, n * (k + 1) / t);
  fn(0, n / t);
  for (auto &x : th) x.join();
}

}  // namespace

// Host batches (host in, host out; the NIC-ring path of SURVEY §8f-4).  The
// batch is cut into byte-balanced shards, one per device; each device walks
// its shard in chunks alternating between two staging slots with their own
// streams, so chunk k+1's CPU copy + H2D overlap chunk k's kernel + D2H.
// A chunk reaches the device in one of three ways:
//   span/DMA   the packets form a contiguous, ascending span (fixed stride,
//              or a ring of ascending offsets with little slack) in
//              DMA-readable memory: one hipMemcpyAsync straight from the
//              caller's buffer, no CPU copy;
//   span/copy  same span in pageable memory: parallel memcpy into the pinned
//              slot, then one DMA;
//   gather     anything else: packets copied one by one (in parallel) into
//              the pinned slot, 16-byte aligned, with new offsets (and, when
//              the EtherType is checked, the 2 bytes before each L3 header).
// With a status array (ricrc_batch_host_st) a descriptor length outside
// [RICRC_MIN_LEN, RICRC_MAX_LEN] is not an error: the packet is staged as 0
// bytes, the device reports RICRC_ST_BADLEN for it and out[i] = 0.
// extent: the bytes from base the caller's buffer holds (0: unknown).  The
// plain calls know it when base lies in a context range (ricrc_host_alloc /
// ricrc_host_register); ricrc_batch_host_bounded takes it from the caller.
// A packet outside it is -EINVAL (with a status array: RICRC_ST_BADLEN), and
// none of its bytes is read.
static int batch_host_impl(ricrc_ctx *ctx, const uint8_t *base, const uint64_t *off, const uint32_t *len,
                           uint32_t stride, uint64_t count, uint32_t l3_offset, uint32_t *out, uint8_t *status,
                           const StFlags &f, uint64_t extent = 0) {
  if (!ctx || ctx->devs.empty()) return -EINVAL;
  if (count == 0) return 0;
  if (!base || !out) return -EINVAL;
  if (!off && stride == 0) return -EINVAL;
  if (!len && stride <= l3_offset) return -EINVAL;
  // The plain calls know the buffer's size only for a buffer the context
  // allocated (ricrc_host_alloc): a registered range may be a part of a
  // larger caller buffer (or one of several adjacent ones), so it bounds
  // nothing.
  if (extent == 0)
    for (const HostRange &r : ctx->pinned)
      if (r.owned && (uintptr_t)base >= r.lo && (uintptr_t)base < r.hi) extent = r.hi - (uintptr_t)base;
  auto len_ok = [](uint64_t n) { return n >= kMinLen && n <= kMaxLen; };
  auto frame = [&](uint64_t i) -> uint64_t { return off ? off[i] : i * (uint64_t)stride; };
  // packet i's descriptor bytes [frame + l3_offset, + n) inside the extent
  auto in_ext = [&](uint64_t i, uint64_t n) {
    const uint64_t fo = frame(i);
    return extent == 0 || (fo <= extent && (uint64_t)l3_offset + n <= extent - fo);
  };
  const int T = ctx->knobs.host_threads;
  // RICRC_F_FRAMELEN: every packet's L3 length from its IP header
  // (frame_l3_len), read once, in parallel (the headers of a NIC ring sit in
  // separate slots: one cache miss each, which the passes below would
  // otherwise pay five times over).
  std::vector<uint32_t> flen;
  if (f.framelen) {
    flen.resize(count);
    par_for(count, T, 4096, [&](uint64_t a, uint64_t b) {
      for (uint64_t i = a; i < b; ++i) {
        uint32_t n = len ? len[i] : stride - l3_offset;
        if (frame_len_applies(n) && in_ext(i, n)) {  // (its header only when the frame is in the buffer)
          const uint8_t *l3 = base + frame(i) + l3_offset;
          n = frame_l3_len(n, l3[0], (uint32_t)l3[2] << 8 | l3[3], (uint32_t)l3[4] << 8 | l3[5]);
        }
        flen[i] = n;
      }
    });
  }
  // Bytes staged for packet i (0 for a bad length under a status array).
  auto desc_len = [&](uint64_t i) -> uint64_t { return len ? len[i] : (uint64_t)stride - l3_offset; };
  auto pkt_len = [&](uint64_t i) -> uint64_t {
    const uint64_t n = f.framelen ? flen[i] : desc_len(i);
    return (status && (!len_ok(n) || !in_ext(i, desc_len(i)))) ? 0 : n;
  };
  if (!len && !len_ok((uint64_t)stride - l3_offset)) return -EINVAL;  // the batch's one length
  uint64_t total = 0;
  for (uint64_t i = 0; i < count; ++i) {
    const uint64_t n = pkt_len(i);
    if (!status && (!len_ok(n) || !in_ext(i, desc_len(i)))) return -EINVAL;
    total += n;
  }
  const int ndev = (int)ctx->devs.size();
  for (Dev &d : ctx->devs) {
    const int rc = ensure_staging(d);
    if (rc) return rc;
  }
  // Byte-balanced shard boundaries.
  std::vector<uint64_t> cut(ndev + 1, count);
  cut[0] = 0;
  {
    uint64_t acc = 0;
    int k = 1;
    for (uint64_t i = 0; i < count && k < ndev; ++i) {
      acc += pkt_len(i);
      while (k < ndev && acc * ndev >= total * k) cut[k++] = i + 1;
    }
  }
  struct Cur {
    uint64_t next, end;
    int slot;
    uint64_t pend_lo[2], pend_hi[2];
    bool pend[2];
  };
  std::vector<Cur> cur(ndev);
  for (int k = 0; k < ndev; ++k) cur[k] = Cur{cut[k], cut[k + 1], 0, {0, 0}, {0, 0}, {false, false}};
  const bool ether = f.strict && l3_offset >= 14;  // the EtherType is checked: gather keeps its 2 bytes

  auto drain = [&](Dev &d, Cur &c, int s) -> int {
    if (!c.pend[s]) return 0;
    HIP_TRY(hipEventSynchronize(d.slot[s].done));
    memcpy(out + c.pend_lo[s], d.slot[s].h_out, (c.pend_hi[s] - c.pend_lo[s]) * sizeof(uint32_t));
    if (status) memcpy(status + c.pend_lo[s], d.h_status[s], c.pend_hi[s] - c.pend_lo[s]);
    c.pend[s] = false;
    return 0;
  };

  // Debug knob (tests): RICRC_FAIL_CHUNK=k fails the context's next host
  // call with -EIO right after chunk k (0-based, counted over devices) has
  // been queued; later calls run normally.
  const long fail_chunk = ctx->fail_once.load();
  long chunk_no = 0;

  auto run = [&]() -> int {
    bool busy = true;
    while (busy) {
      busy = false;
      for (int k = 0; k < ndev; ++k) {
        Dev &d = ctx->devs[k];
        Cur &c = cur[k];
        if (c.next >= c.end) continue;
        busy = true;
        DeviceGuard g(d.id);
        if (!g.ok()) return -ENODEV;
        const int s = c.slot;
        int rc = drain(d, c, s);
        if (rc) return rc;
        Slot &sl = d.slot[s];
        const uint64_t lo = c.next;
        // Span plan: the largest [lo, hi) whose frames ascend without overlap
        // and whose byte span [first frame, end of the last packet) fits the
        // slot with at most 25 % slack.  The span lands at d_buf + pad so that
        // its first packet's L3 header is 16-byte aligned on the device (so
        // are the others when the frames are 16 apart, e.g. a fixed stride).
        // A packet staged as 0 bytes (with a status array: a bad length, or a
        // frame outside the extent) is read by nobody: it neither starts,
        // stretches nor ends a span, so no byte outside the extent is copied
        // (its device descriptor is length 0 at the span's start).
        const uint64_t pad = (16u - (l3_offset & 15u)) & 15u;
        uint64_t hi = lo, s_lo = 0, s_hi = 0, used = 0;
        bool any = false, empty = false;
        while (hi < c.end && hi - lo < kStagePkts) {
          const uint64_t n = pkt_len(hi);
          if (n == 0) {
            empty = true;
            ++hi;
            continue;
          }
          const uint64_t fs = frame(hi), fe = fs + l3_offset + n;
          if (!any) {
            s_lo = s_hi = fs;
            any = true;
          } else if (fs < s_hi) {
            break;  // not ascending / overlapping
          }
          if (fe - s_lo > kStageBytes) break;
          s_hi = fe;
          used += n;
          ++hi;
        }
        const bool span = hi > lo && (s_hi - s_lo) <= used + used / 4 + 64;
        uint64_t m, bytes;
        uint32_t kl3 = l3_offset;
        if (span) {
          m = hi - lo;
          bytes = s_hi - s_lo;
          const uint8_t *src = base + s_lo;
          if (dma_readable(ctx, src, bytes)) {
            HIP_TRY(hipMemcpyAsync(sl.d_buf + pad, src, bytes, hipMemcpyHostToDevice, sl.st));
          } else {
            par_for(bytes, T, 4u << 20, [&](uint64_t a, uint64_t b) { memcpy(sl.h_buf + a, src + a, b - a); });
            HIP_TRY(hipMemcpyAsync(sl.d_buf + pad, sl.h_buf, bytes, hipMemcpyHostToDevice, sl.st));
          }
          if (off || len || f.framelen || empty)
            for (uint64_t i = lo; i < hi; ++i) sl.h_off[i - lo] = pkt_len(i) ? frame(i) - s_lo + pad : pad;
        } else {
          // Gather: packed L3 packets, 16-byte aligned each (after `pre`
          // EtherType bytes when those are checked).
          const uint32_t pre = ether ? 2u : 0u;
          hi = lo;
          bytes = 0;
          while (hi < c.end && hi - lo < kStagePkts) {
            const uint64_t padded = (pre ? 16u : 0u) + ((pkt_len(hi) + 15) & ~15ull);
            if (bytes + padded > kStageBytes) break;
            sl.h_off[hi - lo] = bytes + (pre ? 16u - pre : 0u);
            bytes += padded;
            ++hi;
          }
          m = hi - lo;
          par_for(m, T, 4096, [&](uint64_t a, uint64_t b) {
            for (uint64_t i = a; i < b; ++i) {
              const uint64_t n = pkt_len(lo + i);
              if (n) memcpy(sl.h_buf + sl.h_off[i], base + frame(lo + i) + l3_offset - pre, n + pre);
            }
          });
          HIP_TRY(hipMemcpyAsync(sl.d_buf, sl.h_buf, bytes, hipMemcpyHostToDevice, sl.st));
          kl3 = pre;
        }
        // frames at i*stride from d_buf + pad (no packet staged as 0 bytes: those need their length 0)
        const bool fixed = span && !off && !len && !f.framelen && !empty;
        const uint8_t *dbase = fixed ? sl.d_buf + pad : sl.d_buf;
        const uint64_t *doff = nullptr;
        const uint32_t *dlen = nullptr;
        const uint32_t dstride = fixed ? stride : 0;
        if (!fixed) {
          HIP_TRY(hipMemcpyAsync(sl.d_off, sl.h_off, m * sizeof(uint64_t), hipMemcpyHostToDevice, sl.st));
          for (uint64_t i = 0; i < m; ++i) sl.h_len[i] = (uint32_t)pkt_len(lo + i);
          HIP_TRY(hipMemcpyAsync(sl.d_len, sl.h_len, m * sizeof(uint32_t), hipMemcpyHostToDevice, sl.st));
          doff = sl.d_off;
          dlen = sl.d_len;
        }
        rc = launch_batch(d, dbase, doff, dlen, dstride, m, kl3, sl.d_out, sl.st, f.verify, f.fam);
        if (!rc && status)
          rc = launch_status_pass(d, dbase, doff, dlen, dstride, m, kl3, f.accept, ether, sl.d_out, d.d_status[s],
                                  nullptr, sl.st);
        if (rc) return rc;
        HIP_TRY(hipMemcpyAsync(sl.h_out, sl.d_out, m * sizeof(uint32_t), hipMemcpyDeviceToHost, sl.st));
        if (status) HIP_TRY(hipMemcpyAsync(d.h_status[s], d.d_status[s], m, hipMemcpyDeviceToHost, sl.st));
        HIP_TRY(hipEventRecord(sl.done, sl.st));
        c.pend[s] = true;
        c.pend_lo[s] = lo;
        c.pend_hi[s] = hi;
        c.next = hi;
        c.slot ^= 1;
        if (chunk_no++ == fail_chunk) {
          long armed = fail_chunk;
          if (ctx->fail_once.compare_exchange_strong(armed, -1)) return -EIO;
        }
      }
    }
    for (int k = 0; k < ndev; ++k)
      for (int s = 0; s < 2; ++s) {
        const int rc = drain(ctx->devs[k], cur[k], s);
        if (rc) return rc;
      }
    return 0;
  };
  const int rc = run();
  if (rc) {
    // Leave nothing in flight: earlier chunks may still be reading the
    // caller's buffer or the pinned slots and writing h_out; the next call
    // reuses the slots.  Every staged slot stream of every device is drained
    // (best effort: the first error is what the caller gets).
    for (Dev &d : ctx->devs) {
      DeviceGuard g(d.id);
      for (Slot &sl : d.slot)
        if (sl.st) (void)hipStreamSynchronize(sl.st);
    }
    (void)hipGetLastError();
    return rc;
  }
  return 0;
}

extern "C" {

int ricrc_batch_host(ricrc_ctx *ctx, const uint8_t *base, const uint64_t *off, const uint32_t *len,
                     uint32_t stride, uint64_t count, uint32_t l3_offset, uint32_t *out) {
  return ricrc_batch_host_ex(ctx, base, off, len, stride, count, l3_offset, out, RICRC_F_IPV4);
}

int ricrc_batch_host_ex(ricrc_ctx *ctx, const uint8_t *base, const uint64_t *off, const uint32_t *len,
                        uint32_t stride, uint64_t count, uint32_t l3_offset, uint32_t *out, uint32_t flags) {
  StFlags f;
  if (flags > RICRC_F_AUTO || !decode_st_flags(flags, f)) return -EINVAL;
  return batch_host_impl(ctx, base, off, len, stride, count, l3_offset, out, nullptr, f);
}

int ricrc_batch_host_st(ricrc_ctx *ctx, const uint8_t *base, const uint64_t *off, const uint32_t *len,
                        uint32_t stride, uint64_t count, uint32_t l3_offset, uint32_t *out, uint8_t *status,
                        uint32_t flags) {
  StFlags f;
  if (!decode_st_flags(flags, f) || (count && !status)) return -EINVAL;
  return batch_host_impl(ctx, base, off, len, stride, count, l3_offset, out, status, f);
}

int ricrc_batch_host_bounded(ricrc_ctx *ctx, const uint8_t *base, uint64_t base_bytes, const uint64_t *off,
                             const uint32_t *len, uint32_t stride, uint64_t count, uint32_t l3_offset, uint32_t *out,
                             uint8_t *status, uint32_t flags) {
  StFlags f;
  if (!decode_st_flags(flags, f) || base_bytes == 0) return -EINVAL;
  if (!status && (flags & (RICRC_F_STRICT | RICRC_F_VERIFY))) return -EINVAL;  // those report per packet
  return batch_host_impl(ctx, base, off, len, stride, count, l3_offset, out, status, f, base_bytes);
}

}  // extern "C"
