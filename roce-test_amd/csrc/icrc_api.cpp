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
#include <chrono>
#include <new>
#include <type_traits>
#include <thread>
#include <vector>

#include "../../include/roce_icrc.h"
#include "icrc_kernels.h"
#include "icrc_math.h"

using namespace ricrc;

namespace {

constexpr uint64_t kStageBytes = 256ull << 20;  // per staging slot (bytes of packets)
constexpr uint64_t kStagePkts = 1ull << 20;     // per staging slot (packets)
constexpr uint32_t kWorkSlots = 64;
constexpr size_t kMaxWorkspaces = 4;  // ragged-path workspaces per device (one per recent stream)

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
  hipStream_t stream = nullptr;
  uint32_t *d_inv = nullptr;   // x^(-8 z), z <= 4096
  uint32_t *d_inv4 = nullptr;  // t: x^(8 (k - t)), k = 0..3, t <= 4096
  uint32_t *d_tzb = nullptr;   // [kTzWords]: basis words 4q of x^(-8 tz) at 2 tz + q (ragged strided-chain path)
  uint32_t *d_x8n = nullptr;   // x^(8 k), k < 65536 (incremental repair)
  uint32_t *d_work = nullptr;  // kWorkSlots x kSckWorkWords counters (dynamic SCK schedule)
  uint32_t work_next = 0;      // round-robin slot: launches in flight on different streams never share one
  Slot slot[2];
  bool staged = false;
  // Ragged-path workspaces, one per stream that used this device (work on
  // one stream is ordered, so its workspace is never shared by two calls in
  // flight), grown on demand with the stream-ordered allocator; the class
  // counters inside are zeroed on allocation and re-zeroed by the last pass
  // of every call (rsck_gather), so a call costs no allocation and no memset.
  struct Ws {
    hipStream_t st;
    void *p;
    uint64_t bytes;
    bool dirty;  // a call failed part-way: zero the counters before the next one
  };
  std::vector<Ws> ws;
};

int hip_err(hipError_t e) {
  if (e != hipSuccess && getenv("RICRC_DEBUG")) fprintf(stderr, "libroceicrc: HIP error %d: %s\n", (int)e, hipGetErrorString(e));
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
  int host_threads = 1;           // CPU copy threads for pageable host batches
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
  std::vector<uint32_t> inv(4097);  // z in [0, 4096]
  const uint32_t step = gf_xinv8n(1);
  uint32_t v = kOne;
  for (int z = 0; z <= 4096; ++z) {
    inv[z] = v;
    v = gf_mul(v, step);
  }
  HIP_TRY(hipMalloc(&d.d_inv, 4097 * sizeof(uint32_t)));
  HIP_TRY(hipMemcpy(d.d_inv, inv.data(), 4097 * sizeof(uint32_t), hipMemcpyHostToDevice));
  std::vector<uint32_t> inv4(4097 * 4);  // t, k: x^(8 (k - t))
  for (int t = 0; t <= 4096; ++t)
    for (int k = 0; k < 4; ++k) inv4[4 * t + k] = k >= t ? gf_x8n((uint64_t)(k - t)) : gf_xinv8n((uint64_t)(t - k));
  HIP_TRY(hipMalloc(&d.d_inv4, inv4.size() * sizeof(uint32_t)));
  HIP_TRY(hipMemcpy(d.d_inv4, inv4.data(), inv4.size() * sizeof(uint32_t), hipMemcpyHostToDevice));
  // Basis word 4q of x^(-8 tz) is x^(-8 tz) x^(31 - 4q) = x^(31 - 4 (2 tz + q)):
  // one entry per m = 2 tz + q; the kernel derives words 4q+1..4q+3 by x^-1.
  std::vector<uint32_t> tzb(kTzWords);
  for (int m = 0; m < kTzWords; ++m) {
    const int tz = std::min(m >> 1, 127), q = m - 2 * tz;
    tzb[m] = q < 8 ? gf_mul(gf_xinv8n((uint64_t)tz), 1u << (4 * q)) : 0u;
  }
  HIP_TRY(hipMalloc(&d.d_tzb, tzb.size() * sizeof(uint32_t)));
  HIP_TRY(hipMemcpy(d.d_tzb, tzb.data(), tzb.size() * sizeof(uint32_t), hipMemcpyHostToDevice));
  std::vector<uint32_t> x8n(65536);  // x^(8 k): a repair's shift over the bytes after the rewrite
  uint32_t w = kOne;
  for (size_t k = 0; k < x8n.size(); ++k) {
    x8n[k] = w;
    for (int b = 0; b < 8; ++b) w = gf_mulx(w);
  }
  HIP_TRY(hipMalloc(&d.d_x8n, x8n.size() * sizeof(uint32_t)));
  HIP_TRY(hipMemcpy(d.d_x8n, x8n.data(), x8n.size() * sizeof(uint32_t), hipMemcpyHostToDevice));
  HIP_TRY(hipMalloc(&d.d_work, kWorkSlots * kSckWorkWords * sizeof(uint32_t)));
  HIP_TRY(hipMemset(d.d_work, 0, kWorkSlots * kSckWorkWords * sizeof(uint32_t)));
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
  if (!d.ws.empty()) (void)hipDeviceSynchronize();  // the workspaces' streams may be gone already
  for (Dev::Ws &w : d.ws) (void)hipFree(w.p);
  d.ws.clear();
  (void)hipFree(d.d_inv);
  (void)hipFree(d.d_inv4);
  (void)hipFree(d.d_tzb);
  (void)hipFree(d.d_x8n);
  (void)hipFree(d.d_work);
  if (d.stream) (void)hipStreamDestroy(d.stream);
}

int ilog2_ceil(uint32_t v) {
  int l = 0;
  while ((1u << l) < v) ++l;
  return l;
}

// The ragged-path workspace of stream st on device d, at least `bytes`.
int ragged_ws(Dev &d, hipStream_t st, uint64_t bytes, Dev::Ws **out) {
  Dev::Ws *w = nullptr;
  for (Dev::Ws &x : d.ws)
    if (x.st == st) w = &x;
  if (!w) {
    if (d.ws.size() >= kMaxWorkspaces) {  // bound the pool: drop the oldest (its stream may be gone)
      HIP_TRY(hipDeviceSynchronize());
      (void)hipFree(d.ws.front().p);
      d.ws.erase(d.ws.begin());
    }
    d.ws.push_back(Dev::Ws{st, nullptr, 0, true});
    w = &d.ws.back();
  }
  if (w->bytes < bytes) {
    if (w->p) HIP_TRY(hipFreeAsync(w->p, st));
    w->p = nullptr;
    w->bytes = 0;
    const uint64_t grow = std::max<uint64_t>(bytes, bytes + bytes / 4);
    HIP_TRY(hipMallocAsync(&w->p, grow, st));
    w->bytes = grow;
    w->dirty = true;
  }
  if (w->dirty) {
    HIP_TRY(rs_zero_counters(w->p, st));
    w->dirty = false;
  }
  *out = w;
  return 0;
}

// Kernel selection + launch for one device-resident batch.
// True if the batch takes the strided-chain kernel (back-to-back 1, 2 or 4
// KiB packets, 16-byte aligned), which applies any address family natively.
bool sck_batch(const uint8_t *base, const uint64_t *off, const uint32_t *len, uint64_t stride, uint64_t count,
               uint32_t l3_offset, int n_cu) {
  if (off || len || l3_offset != 0 || ((uintptr_t)base % 16) != 0 || getenv("RICRC_NO_SCK") != nullptr) return false;
  if (stride != 1024 && stride != 2048 && stride != 4096) return false;
  const uint64_t groups = (count + 7) / 8;
  int sgrid = (int)std::max<uint64_t>(1, std::min<uint64_t>((uint64_t)n_cu, (groups + 15) / 16));
  if (const char *e = getenv("RICRC_SCK_GRID")) sgrid = std::max(1, std::min(sgrid, atoi(e)));  // tests
  const uint64_t waves = 16ull * (uint64_t)sgrid;
  return (groups + waves - 1) / waves * 8ull * stride < (1ull << 31);  // each wave's span: a 31-bit buffer offset
}

int launch_batch_v4(Dev &d, const uint8_t *base, const uint64_t *off, const uint32_t *len, uint64_t stride,
                    uint64_t count, uint32_t l3_offset, uint32_t *out, hipStream_t st, bool verify,
                    uint32_t family = kFamV4) {
  if (count == 0) return 0;
  const uint8_t *first = base + l3_offset;
  const uint32_t fixed_len = stride > l3_offset ? (uint32_t)std::min<uint64_t>(stride - l3_offset, 0xFFFFFFFFu) : 0u;
  const bool aligned = ((uintptr_t)first % 16 == 0) && (stride % 16 == 0);
  if (!off && !len && aligned && fixed_len >= kMinLen && fixed_len <= kMaxLen && fixed_len % 4 == 0) {
    const uint32_t M = fixed_len - 4;
    int cpl = 0;
    for (int c : {1, 2, 4})
      if ((M + 64u * c - 1) / (64u * c) <= 64) {
        cpl = c;
        break;
      }
    if (cpl) {
      StreamArgs a{};
      const uint32_t chunk = 64u * cpl;
      a.base = first;
      a.stride = stride;
      a.count = count;
      a.out = out;
      a.len = fixed_len;
      a.P = (M + chunk - 1) / chunk;
      a.log2P2 = (uint32_t)ilog2_ceil(a.P);
      a.nw_last = (M - chunk * (a.P - 1)) / 4;
      const uint64_t ppw = 64u >> a.log2P2;
      a.n_iters = (count + ppw - 1) / ppw;
      a.verify = verify ? 1u : 0u;
      for (uint32_t c = 0; c < 64; ++c) {
        if (c >= a.P) a.K[c] = 0;
        else a.K[c] = x8n_host((uint64_t)M - std::min<uint64_t>((uint64_t)chunk * (c + 1), M));
      }
      const uint64_t want = (a.n_iters + 15) / 16;
      const int grid = (int)std::max<uint64_t>(1, std::min<uint64_t>((uint64_t)d.n_cu, want));
      // Back-to-back 1, 2 or 4 KiB packets: the strided-chain kernel (no LDS
      // transpose), as long as each wave's span fits a 31-bit buffer offset.
      if (sck_batch(base, off, len, stride, count, l3_offset, d.n_cu)) {
        const uint64_t groups = (count + 7) / 8;
        int sgrid = (int)std::max<uint64_t>(1, std::min<uint64_t>((uint64_t)d.n_cu, (groups + 15) / 16));
        if (const char *e = getenv("RICRC_SCK_GRID")) sgrid = std::max(1, std::min(sgrid, atoi(e)));  // tests
        {
          SckArgs k{};
          k.family = family;
          k.base = base;
          k.count = count;
          k.out = out;
          k.n = fixed_len;
          k.verify = verify ? 1u : 0u;
          const uint32_t xi = gf_xinv8n(4);
          for (int j = 0; j < 32; ++j) k.XB[j] = gf_mul(xi, 1u << j);
          for (int s = 0; s < 8; ++s) k.QS[s] = gf_xinv8n(16ull * s + 4);
          // Dynamic schedule (groups from a device counter): robust when other
          // kernels (RCCL) hold CUs while this one starts.  RICRC_SCK_STATIC=1:
          // contiguous per-wave blocks.
          k.dynamic = getenv("RICRC_SCK_DYNAMIC") != nullptr ? 1u : 0u;
          k.work = d.d_work + kSckWorkWords * (d.work_next++ % kWorkSlots);
          return hip_err(launch_sck(k, sgrid, st));
        }
      }
      // Back-to-back packets of 32 * 2^j bytes: coalesced + LDS-transposed kernel.
      // (64-byte packets: the direct streaming kernel is faster, 20.1 vs 23.8 us on 1 M x 64 B.)
      if (l3_offset == 0 && stride == fixed_len && fixed_len >= 128 && fixed_len <= 4096 &&
          (fixed_len & (fixed_len - 1)) == 0 && ((uintptr_t)base % 16 == 0) && getenv("RICRC_NO_TSK") == nullptr) {
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
        const uint64_t tw = (t.n_iters + 15) / 16;
        const int tgrid = (int)std::max<uint64_t>(1, std::min<uint64_t>((uint64_t)d.n_cu, tw));
        return hip_err(launch_tsk(t, tgrid, st));
      }
      return hip_err(launch_stream(a, cpl, grid, st));
    }
  }
  // Everything else (offsets, lengths, any alignment, Ethernet framing): the
  // ragged strided-chain pipeline (icrc_rsck.hip), packets bucketed on the
  // device by line count.  RICRC_NO_RSCK=1 selects the older piece-based
  // ragged kernel below (kept for comparison and as a second implementation).
  if (getenv("RICRC_NO_RSCK") == nullptr && count < (1ull << 31)) {
    RsckArgs k{};
    k.base = base;
    k.off = off;
    k.len = len;
    k.stride = stride;
    k.count = count;
    k.fixed_len = fixed_len;
    k.l3_offset = l3_offset;
    k.verify = verify ? 1u : 0u;
    k.out = out;
    k.tzb = d.d_tzb;
    const uint32_t xi = gf_xinv8n(4);
    const uint32_t xi2 = gf_xinv8n(8), xi3 = gf_xinv8n(12);
    for (int j = 0; j < 32; ++j) {
      k.XB[j] = gf_mul(xi, 1u << j);
      k.XB2[j] = gf_mul(xi2, 1u << j);
      k.XB3[j] = gf_mul(xi3, 1u << j);
    }
    for (int s = 0; s < 8; ++s) k.QS[s] = gf_xinv8n(16ull * s);
    RaggedArgs small{};
    small.inv_tab = d.d_inv;
    small.inv4 = reinterpret_cast<const u32x4_t *>(d.d_inv4);
    for (uint32_t l = 0; l < 64; ++l) small.K[l] = x8n_host(64ull * (63 - l));
    Dev::Ws *ws = nullptr;
    const int wrc = ragged_ws(d, st, rs_workspace_bytes(count), &ws);
    if (wrc) return wrc;
    rs_bind_workspace(k, ws->p);
    int rgrid = d.n_cu;
    if (const char *e = getenv("RICRC_RSCK_GRID")) rgrid = std::max(1, std::min(rgrid, atoi(e)));  // tests
    const hipError_t e = launch_rsck(k, small, rgrid, st);
    if (e != hipSuccess) ws->dirty = true;
    return hip_err(e);
  }
  // The piece-based ragged kernel.  Pieces from a device-side scan of the
  // descriptors, or arithmetic when every packet has the same length and
  // 16-byte phase.
  RaggedArgs r{};
  r.base = base;
  r.off = off;
  r.len = len;
  r.stride = stride;
  r.count = count;
  r.out = out;
  r.inv_tab = d.d_inv;
  r.inv4 = reinterpret_cast<const u32x4_t *>(d.d_inv4);
  r.fixed_len = fixed_len;
  r.l3_offset = l3_offset;
  r.verify = verify ? 1u : 0u;
  for (uint32_t l = 0; l < 64; ++l) r.K[l] = x8n_host(64ull * (63 - l));
  const int grid = (int)std::max<uint64_t>(1, std::min<uint64_t>((uint64_t)d.n_cu, (count + 63) / 64));
  if (!off && !len && stride % 16 == 0) {
    r.P = ragged_pieces((uintptr_t)base + l3_offset, fixed_len);
    return hip_err(launch_ragged(r, grid, st));
  }
  uint64_t *ps = nullptr;
  HIP_TRY(hipMallocAsync((void **)&ps, (count + 1) * sizeof(uint64_t), st));
  r.ps = ps;
  hipError_t e = ragged_piece_scan(r, ps, st);
  if (e == hipSuccess) e = launch_ragged(r, grid, st);
  const hipError_t e2 = hipFreeAsync(ps, st);
  return hip_err(e != hipSuccess ? e : e2);
}

// Any address family: the IPv4-mask kernels, then (IPv6 / AUTO) the linear
// header fix-up, which also does the verify compare in that case.
int launch_batch(Dev &d, const uint8_t *base, const uint64_t *off, const uint32_t *len, uint64_t stride,
                 uint64_t count, uint32_t l3_offset, uint32_t *out, hipStream_t st, bool verify,
                 uint32_t family = kFamV4) {
  if (family == kFamV4 || count == 0)
    return launch_batch_v4(d, base, off, len, stride, count, l3_offset, out, st, verify);
  if (sck_batch(base, off, len, stride, count, l3_offset, d.n_cu))  // masks native in the kernel
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
  if (getenv("RICRC_DEBUG")) fprintf(stderr, "libroceicrc: RCCL error %d: %s\n", (int)e, rccl().err_str(e));
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
// all of them.  Equal shards: one in-place ncclAllGather per device; unequal
// shards: ncclSend / ncclRecv pairs, every device's calls in one group.
int comm_allgather(ricrc_ctx *ctx, const uint64_t *counts, uint32_t *const *d_out) {
  Rccl &r = rccl();
  const int n = (int)ctx->devs.size();
  std::vector<uint64_t> at(n + 1, 0);
  bool equal = true;
  for (int k = 0; k < n; ++k) {
    at[k + 1] = at[k] + counts[k];
    equal = equal && counts[k] == counts[0];
  }
  if (n == 1) return 0;  // already in place
  int rc = nccl_err(r.group_start());
  if (rc) return rc;
  for (int k = 0; k < n && !rc; ++k) {
    Dev &d = ctx->devs[k];
    if (equal) {
      rc = nccl_err(r.all_gather(d_out[k] + at[k], d_out[k], (size_t)counts[k], ncclUint32, ctx->comms[k], d.stream));
      continue;
    }
    for (int p = 0; p < n && !rc; ++p) {
      if (p == k) continue;
      if (counts[k]) rc = nccl_err(r.send(d_out[k] + at[k], (size_t)counts[k], ncclUint32, p, ctx->comms[k], d.stream));
      if (!rc && counts[p]) rc = nccl_err(r.recv(d_out[k] + at[p], (size_t)counts[p], ncclUint32, p, ctx->comms[k], d.stream));
    }
  }
  const int rc2 = nccl_err(r.group_end());
  return rc ? rc : rc2;
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
  {
    const unsigned hw = std::thread::hardware_concurrency();
    int t = (int)std::min(16u, std::max(1u, hw));
    if (const char *e = getenv("RICRC_HOST_THREADS")) t = std::max(1, std::min(64, atoi(e)));
    c->host_threads = t;
  }
  c->devs.resize(n);
  for (int i = 0; i < n; ++i) {
    c->devs[i].id = devices[i];
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

extern "C" {

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
//              the pinned slot, 16-byte aligned, with new offsets.
int ricrc_batch_host(ricrc_ctx *ctx, const uint8_t *base, const uint64_t *off, const uint32_t *len,
                     uint32_t stride, uint64_t count, uint32_t l3_offset, uint32_t *out) {
  return ricrc_batch_host_ex(ctx, base, off, len, stride, count, l3_offset, out, RICRC_F_IPV4);
}

int ricrc_batch_host_ex(ricrc_ctx *ctx, const uint8_t *base, const uint64_t *off, const uint32_t *len,
                        uint32_t stride, uint64_t count, uint32_t l3_offset, uint32_t *out, uint32_t flags) {
  if (!ctx || ctx->devs.empty() || flags > RICRC_F_AUTO) return -EINVAL;
  if (count == 0) return 0;
  if (!base || !out) return -EINVAL;
  if (!off && stride == 0) return -EINVAL;
  auto pkt_len = [&](uint64_t i) -> uint64_t { return len ? len[i] : (uint64_t)stride - l3_offset; };
  auto frame = [&](uint64_t i) -> uint64_t { return off ? off[i] : i * (uint64_t)stride; };
  if (!len && stride <= l3_offset) return -EINVAL;
  uint64_t total = 0;
  for (uint64_t i = 0; i < count; ++i) {
    const uint64_t n = pkt_len(i);
    if (n < kMinLen || n > kMaxLen) return -EINVAL;
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
  const int T = ctx->host_threads;

  auto drain = [&](Dev &d, Cur &c, int s) -> int {
    if (!c.pend[s]) return 0;
    HIP_TRY(hipEventSynchronize(d.slot[s].done));
    memcpy(out + c.pend_lo[s], d.slot[s].h_out, (c.pend_hi[s] - c.pend_lo[s]) * sizeof(uint32_t));
    c.pend[s] = false;
    return 0;
  };

  // Debug knob (tests): RICRC_FAIL_CHUNK=k fails the call with -EIO right
  // after chunk k (0-based, counted over devices) has been queued.
  long fail_chunk = -1;
  if (const char *e = getenv("RICRC_FAIL_CHUNK")) fail_chunk = atol(e);
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
        // and whose byte span [frame(lo), end of hi-1) fits the slot with at
        // most 25 % slack.  The span lands at d_buf + pad so that packet lo's
        // L3 header is 16-byte aligned on the device (so are the others when
        // the frames are 16 apart, e.g. a fixed stride).
        const uint64_t s_lo = frame(lo);
        const uint64_t pad = (16u - (l3_offset & 15u)) & 15u;
        uint64_t hi = lo, s_hi = s_lo, used = 0;
        while (hi < c.end && hi - lo < kStagePkts) {
          const uint64_t fs = frame(hi), fe = fs + l3_offset + pkt_len(hi);
          if (fs < s_hi && hi > lo) break;  // not ascending / overlapping
          if (fe - s_lo > kStageBytes) break;
          s_hi = fe;
          used += pkt_len(hi);
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
          if (off || len)
            for (uint64_t i = lo; i < hi; ++i) sl.h_off[i - lo] = frame(i) - s_lo + pad;
        } else {
          // Gather: packed L3 packets, 16-byte aligned each.
          hi = lo;
          bytes = 0;
          while (hi < c.end && hi - lo < kStagePkts) {
            const uint64_t padded = (pkt_len(hi) + 15) & ~15ull;
            if (bytes + padded > kStageBytes) break;
            sl.h_off[hi - lo] = bytes;
            bytes += padded;
            ++hi;
          }
          m = hi - lo;
          par_for(m, T, 4096, [&](uint64_t a, uint64_t b) {
            for (uint64_t i = a; i < b; ++i)
              memcpy(sl.h_buf + sl.h_off[i], base + frame(lo + i) + l3_offset, pkt_len(lo + i));
          });
          HIP_TRY(hipMemcpyAsync(sl.d_buf, sl.h_buf, bytes, hipMemcpyHostToDevice, sl.st));
          kl3 = 0;
        }
        const bool fixed = span && !off && !len;  // frames at i*stride from d_buf + pad
        if (fixed) {
          rc = launch_batch(d, sl.d_buf + pad, nullptr, nullptr, stride, m, kl3, sl.d_out, sl.st, false, flags);
        } else {
          HIP_TRY(hipMemcpyAsync(sl.d_off, sl.h_off, m * sizeof(uint64_t), hipMemcpyHostToDevice, sl.st));
          for (uint64_t i = 0; i < m; ++i) sl.h_len[i] = (uint32_t)pkt_len(lo + i);
          HIP_TRY(hipMemcpyAsync(sl.d_len, sl.h_len, m * sizeof(uint32_t), hipMemcpyHostToDevice, sl.st));
          rc = launch_batch(d, sl.d_buf, sl.d_off, sl.d_len, 0, m, kl3, sl.d_out, sl.st, false, flags);
        }
        if (rc) return rc;
        HIP_TRY(hipMemcpyAsync(sl.h_out, sl.d_out, m * sizeof(uint32_t), hipMemcpyDeviceToHost, sl.st));
        HIP_TRY(hipEventRecord(sl.done, sl.st));
        c.pend[s] = true;
        c.pend_lo[s] = lo;
        c.pend_hi[s] = hi;
        c.next = hi;
        c.slot ^= 1;
        if (chunk_no++ == fail_chunk) return -EIO;
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

}  // extern "C"
