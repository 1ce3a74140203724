// Host side of libroceicrc: contexts, kernel selection, host-buffer staging
// and multi-GPU sharding.  Everything here is plumbing around the gfx950
// kernels in icrc_kernels.hip; there is no CPU compute path for batches.
//
// Conventions follow the reference's C++: 0 / negative
// errno returns (endpoint/shuffle_endpoint.hpp:364-389), no aborts
// (common/logger.hpp:190 logassert only logs), caller-owned buffers
// (common/huge_malloc.h:12-22).
#include <errno.h>
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <new>
#include <vector>

#include "../../include/roce_icrc.h"
#include "icrc_kernels.h"
#include "icrc_math.h"

using namespace ricrc;

namespace {

constexpr uint64_t kStageBytes = 256ull << 20;  // per staging slot (bytes of packets)
constexpr uint64_t kStagePkts = 1ull << 20;     // per staging slot (packets)

struct Slot {
  uint8_t *d_buf = nullptr;
  uint64_t *d_off = nullptr;
  uint32_t *d_len = nullptr;
  uint32_t *d_out = nullptr;
  uint8_t *h_buf = nullptr;  // pinned
  uint64_t *h_off = nullptr;
  uint32_t *h_len = nullptr;
  uint32_t *h_out = nullptr;
  hipEvent_t done = nullptr;
};

struct Dev {
  int id = 0;
  int n_cu = 0;
  hipStream_t stream = nullptr;
  uint32_t *d_inv = nullptr;  // x^(-8 z), z <= 4096
  Slot slot[2];
  bool staged = false;
};

int hip_err(hipError_t e) { return e == hipSuccess ? 0 : (e == hipErrorOutOfMemory ? -ENOMEM : -EIO); }

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

struct ricrc_ctx {
  std::vector<Dev> devs;
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
  }
  (void)hipFree(d.d_inv);
  if (d.stream) (void)hipStreamDestroy(d.stream);
}

int ilog2_ceil(uint32_t v) {
  int l = 0;
  while ((1u << l) < v) ++l;
  return l;
}

// Kernel selection + launch for one device-resident batch.
int launch_batch(Dev &d, const uint8_t *base, const uint64_t *off, const uint32_t *len, uint64_t stride,
                 uint64_t count, uint32_t l3_offset, uint32_t *out, hipStream_t st, bool verify) {
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
      // Back-to-back packets of 32 * 2^j bytes: coalesced + LDS-transposed kernel.
      if (l3_offset == 0 && stride == fixed_len && fixed_len >= 64 && fixed_len <= 4096 &&
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
  GeneralArgs g{};
  g.base = base;
  g.off = off;
  g.len = len;
  g.stride = stride;
  g.count = count;
  g.out = out;
  g.inv_tab = d.d_inv;
  g.fixed_len = fixed_len;
  g.l3_offset = l3_offset;
  g.x4096 = x8n_host(4096);
  g.verify = verify ? 1u : 0u;
  for (uint32_t l = 0; l < 64; ++l) g.K[l] = x8n_host(64ull * (63 - l));
  const uint64_t want = (count + 15) / 16;
  const int grid = (int)std::max<uint64_t>(1, std::min<uint64_t>((uint64_t)d.n_cu, want));
  return hip_err(launch_general(g, grid, st));
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
  for (Dev &d : ctx->devs) free_dev(d);
  delete ctx;
}

int ricrc_device_count(const ricrc_ctx *ctx) { return ctx ? (int)ctx->devs.size() : 0; }

void *ricrc_stream(ricrc_ctx *ctx, int dev) {
  if (!ctx || dev < 0 || dev >= (int)ctx->devs.size()) return nullptr;
  return ctx->devs[dev].stream;
}

static int batch_device_impl(ricrc_ctx *ctx, int dev, const void *d_base, const uint64_t *d_off,
                             const uint32_t *d_len, uint32_t stride, uint64_t count, uint32_t l3_offset,
                             uint32_t *d_out, void *stream, bool verify) {
  if (!ctx || dev < 0 || dev >= (int)ctx->devs.size()) return -EINVAL;
  if (count == 0) return 0;
  if (!d_base || !d_out) return -EINVAL;
  if (!d_off && stride == 0) return -EINVAL;
  if (!d_len && (stride <= l3_offset)) return -EINVAL;
  Dev &d = ctx->devs[dev];
  DeviceGuard g(d.id);
  if (!g.ok()) return -ENODEV;
  hipStream_t st = (hipStream_t)stream;  // NULL = the HIP null stream, like any HIP API
  return launch_batch(d, (const uint8_t *)d_base, d_off, d_len, stride, count, l3_offset, d_out, st, verify);
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

int ricrc_synth_device(ricrc_ctx *ctx, int dev, uint64_t seed, uint64_t first, uint64_t count, uint32_t n,
                       uint32_t stride, void *d_buf, void *stream) {
  if (!ctx || dev < 0 || dev >= (int)ctx->devs.size() || !d_buf) return -EINVAL;
  if (stride % 8 != 0 || n > stride || n < 4) return -EINVAL;
  Dev &d = ctx->devs[dev];
  DeviceGuard g(d.id);
  if (!g.ok()) return -ENODEV;
  SynthArgs a{(uint8_t *)d_buf, seed, first, count, n, stride};
  return hip_err(launch_synth(a, (hipStream_t)stream));
}

void *ricrc_host_alloc(ricrc_ctx *ctx, uint64_t bytes) {
  if (!ctx || bytes == 0) return nullptr;
  void *p = nullptr;
  if (hipHostMalloc(&p, bytes, hipHostMallocPortable) != hipSuccess) return nullptr;
  return p;
}

void ricrc_host_free(ricrc_ctx *ctx, void *p) {
  (void)ctx;
  if (p) (void)hipHostFree(p);
}

// Host batches: the batch is cut into byte-balanced shards, one per device;
// each device walks its shard in chunks that alternate between two staging
// slots so the CPU gather of chunk k+1 overlaps H2D + kernel + D2H of chunk k.
int ricrc_batch_host(ricrc_ctx *ctx, const uint8_t *base, const uint64_t *off, const uint32_t *len,
                     uint32_t stride, uint64_t count, uint32_t l3_offset, uint32_t *out) {
  if (!ctx || ctx->devs.empty()) return -EINVAL;
  if (count == 0) return 0;
  if (!base || !out) return -EINVAL;
  if (!off && stride == 0) return -EINVAL;
  auto pkt_len = [&](uint64_t i) -> uint64_t { return len ? len[i] : (uint64_t)stride - l3_offset; };
  auto pkt_start = [&](uint64_t i) -> uint64_t { return (off ? off[i] : i * (uint64_t)stride) + l3_offset; };
  if (!len && stride <= l3_offset) return -EINVAL;
  for (uint64_t i = 0; i < count; ++i) {
    const uint64_t n = pkt_len(i);
    if (n < kMinLen || n > kMaxLen) return -EINVAL;
  }
  const int ndev = (int)ctx->devs.size();
  for (Dev &d : ctx->devs) {
    const int rc = ensure_staging(d);
    if (rc) return rc;
  }
  // Byte-balanced shard boundaries.
  uint64_t total = 0;
  for (uint64_t i = 0; i < count; ++i) total += pkt_len(i);
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
  // Per device cursor; round-robin chunk issue across devices.
  struct Cur {
    uint64_t next, end;
    int slot;
    uint64_t pend_lo[2], pend_hi[2];
    bool pend[2];
  };
  std::vector<Cur> cur(ndev);
  for (int k = 0; k < ndev; ++k) cur[k] = Cur{cut[k], cut[k + 1], 0, {0, 0}, {0, 0}, {false, false}};

  auto drain = [&](Dev &d, Cur &c, int s) -> int {
    if (!c.pend[s]) return 0;
    HIP_TRY(hipEventSynchronize(d.slot[s].done));
    memcpy(out + c.pend_lo[s], d.slot[s].h_out, (c.pend_hi[s] - c.pend_lo[s]) * sizeof(uint32_t));
    c.pend[s] = false;
    return 0;
  };

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
      // Gather packets [lo, hi) into the pinned slot, 16-byte aligned each.
      const uint64_t lo = c.next;
      uint64_t hi = lo, bytes = 0;
      while (hi < c.end && hi - lo < kStagePkts) {
        const uint64_t n = pkt_len(hi), padded = (n + 15) & ~15ull;
        if (bytes + padded > kStageBytes) break;
        sl.h_off[hi - lo] = bytes;
        sl.h_len[hi - lo] = (uint32_t)n;
        memcpy(sl.h_buf + bytes, base + pkt_start(hi), n);
        bytes += padded;
        ++hi;
      }
      const uint64_t m = hi - lo;
      HIP_TRY(hipMemcpyAsync(sl.d_buf, sl.h_buf, bytes, hipMemcpyHostToDevice, d.stream));
      const bool uniform = !len && !off;  // contiguous fixed-size -> streaming kernel
      if (uniform && (pkt_len(lo) % 16 == 0)) {
        rc = launch_batch(d, sl.d_buf, nullptr, nullptr, pkt_len(lo), m, 0, sl.d_out, d.stream, false);
      } else {
        HIP_TRY(hipMemcpyAsync(sl.d_off, sl.h_off, m * sizeof(uint64_t), hipMemcpyHostToDevice, d.stream));
        HIP_TRY(hipMemcpyAsync(sl.d_len, sl.h_len, m * sizeof(uint32_t), hipMemcpyHostToDevice, d.stream));
        rc = launch_batch(d, sl.d_buf, sl.d_off, sl.d_len, 0, m, 0, sl.d_out, d.stream, false);
      }
      if (rc) return rc;
      HIP_TRY(hipMemcpyAsync(sl.h_out, sl.d_out, m * sizeof(uint32_t), hipMemcpyDeviceToHost, d.stream));
      HIP_TRY(hipEventRecord(sl.done, d.stream));
      c.pend[s] = true;
      c.pend_lo[s] = lo;
      c.pend_hi[s] = hi;
      c.next = hi;
      c.slot ^= 1;
    }
  }
  for (int k = 0; k < ndev; ++k)
    for (int s = 0; s < 2; ++s) {
      const int rc = drain(ctx->devs[k], cur[k], s);
      if (rc) return rc;
    }
  return 0;
}

}  // extern "C"
