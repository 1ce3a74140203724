// A NIC receive ring handled the way an endpoint of the reference would
// (endpoint/shuffle_endpoint.hpp style: 0 / negative errno returns, a
// logassert-like check): Ethernet frames of mixed sizes back to back in one
// pinned host ring (ricrc_host_alloc, the role of huge_malloc,
// common/huge_malloc.h:12-22), per-frame lengths, the L3 packet 14 bytes into
// each frame; ICRCs of the whole ring in one ricrc_batch_host call (sharded
// over the context's GPUs), checked against the per-packet CPU call.
//
//   g++ -std=c++17 -O2 -I include examples/nic_ring.cpp
//       -L roce-test_amd/roce_icrc -lroceicrc -o examples/nic_ring   (examples/Makefile)
//
// Exits 0 and prints "ok" when every ICRC matches; 2 when there is no GPU.
#include <errno.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <chrono>
#include <vector>

#include "roce_icrc.h"

#define CHECK(cond, ...)                      \
  do {                                        \
    if (!(cond)) {                            \
      fprintf(stderr, "nic_ring: " __VA_ARGS__); \
      fprintf(stderr, "\n");                  \
      return 1;                               \
    }                                         \
  } while (0)

int main(int argc, char **argv) {
  const uint64_t count = argc > 1 ? strtoull(argv[1], nullptr, 10) : 200000;
  ricrc_ctx *ctx = nullptr;
  int rc = ricrc_create(&ctx, -1);
  if (rc == -ENODEV) {
    printf("no GPU: %s\n", ricrc_strerror(rc));
    return 2;
  }
  CHECK(rc == 0, "ricrc_create: %s", ricrc_strerror(rc));

  const uint32_t sizes[4] = {64, 256, 1024, 4096};
  std::vector<uint64_t> off(count);
  std::vector<uint32_t> len(count);
  uint64_t pos = 0, x = 0x9E3779B97F4A7C15ull;
  for (uint64_t i = 0; i < count; ++i) {
    x ^= x << 13, x ^= x >> 7, x ^= x << 17;
    len[i] = sizes[x & 3];
    off[i] = pos;
    pos += 14 + len[i];  // Ethernet header + L3 packet
  }
  uint8_t *ring = static_cast<uint8_t *>(ricrc_host_alloc(ctx, pos));
  CHECK(ring != nullptr, "ricrc_host_alloc(%llu)", (unsigned long long)pos);
  for (uint64_t i = 0; i < count; ++i) {
    uint8_t *p = ring + off[i] + 14;
    const uint32_t n = len[i];
    for (uint32_t b = 0; b < n; ++b) {
      x ^= x << 13, x ^= x >> 7, x ^= x << 17;
      p[b] = (uint8_t)x;
    }
    p[0] = 0x45;  // IPv4, IHL 5; the rest of the header is whatever the wire held
    p[2] = (uint8_t)(n >> 8);
    p[3] = (uint8_t)n;
  }

  std::vector<uint32_t> icrc(count);
  // the first call sizes the context's staging and ragged workspaces; time the second
  rc = ricrc_batch_host(ctx, ring, off.data(), len.data(), 0, count, 14, icrc.data());
  CHECK(rc == 0, "ricrc_batch_host: %s", ricrc_strerror(rc));
  const auto t0 = std::chrono::steady_clock::now();
  rc = ricrc_batch_host(ctx, ring, off.data(), len.data(), 0, count, 14, icrc.data());
  const double s = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
  CHECK(rc == 0, "ricrc_batch_host: %s", ricrc_strerror(rc));
  for (uint64_t i = 0; i < count; ++i)
    CHECK(icrc[i] == ricrc_one(ring + off[i] + 14, len[i]), "packet %llu: gpu 0x%08x cpu 0x%08x",
          (unsigned long long)i, icrc[i], ricrc_one(ring + off[i] + 14, len[i]));

  // a frame with a bad length is refused before any GPU work
  len[count / 2] = 20;
  rc = ricrc_batch_host(ctx, ring, off.data(), len.data(), 0, count, 14, icrc.data());
  CHECK(rc == -EINVAL, "bad length must be -EINVAL, got %d", rc);

  printf("%llu frames, %llu bytes, %d GPU(s), %.2f GiB/s host-to-host\nok\n", (unsigned long long)count,
         (unsigned long long)pos, ricrc_device_count(ctx), pos / s / (1u << 30));
  ricrc_host_free(ctx, ring);
  ricrc_destroy(ctx);
  return 0;
}
