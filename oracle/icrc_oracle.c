/*
 * CPU oracle for the RoCEv2 ICRC -- TEST INFRASTRUCTURE ONLY.
 *
 * Linked/loaded only by tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline leg, as the checker.  Never part of the product library.
 *
 * Restates calc_icrc() of the reference (p4/shuffle/shuffle_egress.p4:461-494):
 *   CRC-32 (reflected poly 0xEDB88320, init/xorout 0xFFFFFFFF; Tofino's
 *   HashAlgorithm_t.CRC32, :461) over
 *     0xFF x 8                                   (:465)
 *     || L3 bytes [0, n-4) with bytes 1 (tos, :467), 8 (ttl, :471),
 *        10-11 (IPv4 csum, :473), 26-27 (UDP csum, :480) and
 *        32 (BTH FECN/BECN/resv, :485) forced to 0xFF,
 *   all other bytes unmasked (BTH rest :482-487, AETH :489-490).  The P4
 *   field list ends at the AETH (calc_icrc is written for 48-byte write ACKs);
 *   bytes after BTH other than an AETH (extension headers, payload, pad) are
 *   covered unmasked as IBTA Annex A17 / Linux rxe do -- a deliberate
 *   generalisation that equals calc_icrc on the reference's ACK shape.
 *   Offsets from p4/common/header.p4:42-53 (ipv4_h), :67-72 (udp_h),
 *   :75-85 (bth_h).  The trailer carries the value little-endian (:493).
 *
 * Three independent formulations (bitwise, Sarwate byte table, slice-by-8)
 * are exported so the tests can cross-check them against each other and
 * against Python's zlib.  Parity is "unpinned" by reference fixtures (the
 * reference has none); see DESIGN.md.
 *
 * Also: the CPU restatement of the synthetic packet generator used by
 * bench.py / the device generator (so device-generated batches can be
 * regenerated and checked on the host).
 */
#include <pthread.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#define POLY 0xEDB88320u

/* {L3 offset, OR value}.  IPv4: shuffle_egress.p4:467,471,473,480,485.
 * IPv6 (not in the IPv4-only reference): IBTA Annex A17 as Linux rxe applies
 * it (rxe_icrc.c): priority nibble (byte 0 low), flow label bytes 1-3, hop
 * limit 7, UDP checksum 46-47, BTH byte 4 at 52. */
static const int kMaskV4[][2] = {{1, 0xFF}, {8, 0xFF}, {10, 0xFF}, {11, 0xFF}, {26, 0xFF}, {27, 0xFF}, {32, 0xFF}};
static const int kMaskV6[][2] = {{0, 0x0F}, {1, 0xFF}, {2, 0xFF}, {3, 0xFF}, {7, 0xFF}, {46, 0xFF}, {47, 0xFF}, {52, 0xFF}};
#define HEAD 56 /* every masked byte of either family lies in [0, 56) */

static uint32_t bit_update(uint32_t crc, const uint8_t *p, size_t n) {
  for (size_t i = 0; i < n; ++i) {
    crc ^= p[i];
    for (int k = 0; k < 8; ++k) crc = (crc >> 1) ^ ((crc & 1u) ? POLY : 0u);
  }
  return crc;
}

static uint32_t T[8][256];
static pthread_once_t g_once = PTHREAD_ONCE_INIT;

static void init_tables(void) {
  for (uint32_t b = 0; b < 256; ++b) {
    uint32_t c = b;
    for (int k = 0; k < 8; ++k) c = (c >> 1) ^ ((c & 1u) ? POLY : 0u);
    T[0][b] = c;
  }
  for (int t = 1; t < 8; ++t)
    for (uint32_t b = 0; b < 256; ++b)
      T[t][b] = (T[t - 1][b] >> 8) ^ T[0][T[t - 1][b] & 0xFF];
}

/* family: 0 IPv4, 1 IPv6, 2 per packet from the version nibble. */
static int fam_of(const uint8_t *l3, uint32_t n, int family) {
  if (family == 2) return (n > 0 && (l3[0] >> 4) == 6) ? 1 : 0;
  return family == 1 ? 1 : 0;
}

/* First min(n-4, HEAD) bytes with the invariant masks applied. */
static size_t masked_head(const uint8_t *l3, uint32_t n, int family, uint8_t head[HEAD]) {
  size_t m = n - 4, h = m < HEAD ? m : HEAD;
  memcpy(head, l3, h);
  if (fam_of(l3, n, family)) {
    for (size_t i = 0; i < sizeof(kMaskV6) / sizeof(kMaskV6[0]); ++i)
      if ((size_t)kMaskV6[i][0] < h) head[kMaskV6[i][0]] |= (uint8_t)kMaskV6[i][1];
  } else {
    for (size_t i = 0; i < sizeof(kMaskV4) / sizeof(kMaskV4[0]); ++i)
      if ((size_t)kMaskV4[i][0] < h) head[kMaskV4[i][0]] |= (uint8_t)kMaskV4[i][1];
  }
  return h;
}

uint32_t oracle_icrc_bitwise_ex(const uint8_t *l3, uint32_t n, int family) {
  if (n < 4) return 0;
  static const uint8_t ff[8] = {0xFF, 0xFF, 0xFF, 0xFF, 0xFF, 0xFF, 0xFF, 0xFF};
  uint8_t head[HEAD];
  size_t h = masked_head(l3, n, family, head);
  uint32_t c = bit_update(0xFFFFFFFFu, ff, 8);
  c = bit_update(c, head, h);
  c = bit_update(c, l3 + h, (n - 4) - h);
  return ~c;
}
uint32_t oracle_icrc_bitwise(const uint8_t *l3, uint32_t n) { return oracle_icrc_bitwise_ex(l3, n, 0); }

static uint32_t byte_update(uint32_t c, const uint8_t *p, size_t n) {
  for (size_t i = 0; i < n; ++i) c = T[0][(c ^ p[i]) & 0xFF] ^ (c >> 8);
  return c;
}

uint32_t oracle_icrc_bytewise_ex(const uint8_t *l3, uint32_t n, int family) {
  pthread_once(&g_once, init_tables);
  if (n < 4) return 0;
  static const uint8_t ff[8] = {0xFF, 0xFF, 0xFF, 0xFF, 0xFF, 0xFF, 0xFF, 0xFF};
  uint8_t head[HEAD];
  size_t h = masked_head(l3, n, family, head);
  uint32_t c = byte_update(0xFFFFFFFFu, ff, 8);
  c = byte_update(c, head, h);
  c = byte_update(c, l3 + h, (n - 4) - h);
  return ~c;
}
uint32_t oracle_icrc_bytewise(const uint8_t *l3, uint32_t n) { return oracle_icrc_bytewise_ex(l3, n, 0); }

static uint32_t s8_update(uint32_t c, const uint8_t *p, size_t n) {
  while (n >= 8) {
    uint32_t lo, hi;
    memcpy(&lo, p, 4);
    memcpy(&hi, p + 4, 4);
    lo ^= c;
    c = T[7][lo & 0xFF] ^ T[6][(lo >> 8) & 0xFF] ^ T[5][(lo >> 16) & 0xFF] ^ T[4][lo >> 24] ^
        T[3][hi & 0xFF] ^ T[2][(hi >> 8) & 0xFF] ^ T[1][(hi >> 16) & 0xFF] ^ T[0][hi >> 24];
    p += 8;
    n -= 8;
  }
  return byte_update(c, p, n);
}

uint32_t oracle_icrc_fast_ex(const uint8_t *l3, uint32_t n, int family) {
  pthread_once(&g_once, init_tables);
  if (n < 4) return 0;
  uint8_t head[HEAD];
  size_t h = masked_head(l3, n, family, head);
  uint32_t c = 0xDEBB20E3u; /* register after the 8 x 0xFF prefix */
  c = s8_update(c, head, h);
  c = s8_update(c, l3 + h, (n - 4) - h);
  return ~c;
}
uint32_t oracle_icrc_fast(const uint8_t *l3, uint32_t n) { return oracle_icrc_fast_ex(l3, n, 0); }

/* ---------------------------------------------------------------- batch */
typedef uint32_t (*icrc_fn)(const uint8_t *, uint32_t, int);

struct job {
  const uint8_t *base;
  const uint64_t *off;
  const uint32_t *len;
  uint64_t stride, lo, hi;
  uint32_t l3_offset;
  uint32_t *out;
  icrc_fn fn;
  int family;
};

static void *run_job(void *arg) {
  struct job *j = (struct job *)arg;
  for (uint64_t i = j->lo; i < j->hi; ++i) {
    uint64_t o = j->off ? j->off[i] : i * j->stride;
    uint32_t n = j->len ? j->len[i] : (uint32_t)(j->stride - j->l3_offset);
    j->out[i] = j->fn(j->base + o + j->l3_offset, n, j->family);
  }
  return NULL;
}

/* kind: 0 = bitwise, 1 = bytewise, 2 = slice-by-8; family: 0 IPv4, 1 IPv6,
 * 2 per packet.  Returns 0. */
int oracle_icrc_batch_ex(const uint8_t *base, const uint64_t *off, const uint32_t *len,
                         uint64_t stride, uint64_t count, uint32_t l3_offset, uint32_t *out,
                         int threads, int kind, int family) {
  pthread_once(&g_once, init_tables);
  icrc_fn fn = kind == 0 ? oracle_icrc_bitwise_ex : kind == 1 ? oracle_icrc_bytewise_ex : oracle_icrc_fast_ex;
  if (threads < 1) threads = 1;
  if ((uint64_t)threads > count) threads = count ? (int)count : 1;
  pthread_t tid[256];
  struct job jobs[256];
  if (threads > 256) threads = 256;
  for (int t = 0; t < threads; ++t) {
    jobs[t] = (struct job){base, off, len, stride, count * t / threads, count * (t + 1) / threads,
                           l3_offset, out, fn, family};
    if (threads == 1) run_job(&jobs[0]);
    else pthread_create(&tid[t], NULL, run_job, &jobs[t]);
  }
  if (threads > 1)
    for (int t = 0; t < threads; ++t) pthread_join(tid[t], NULL);
  return 0;
}

int oracle_icrc_batch(const uint8_t *base, const uint64_t *off, const uint32_t *len,
                      uint64_t stride, uint64_t count, uint32_t l3_offset, uint32_t *out,
                      int threads, int kind) {
  return oracle_icrc_batch_ex(base, off, len, stride, count, l3_offset, out, threads, kind, 0);
}

/* ------------------------------------------------- synthetic generator
 * Restatement of the device generator (roce-test_amd/csrc/icrc_synth.hip):
 * packet i (global index), 8-byte block j:  LE64(mix(mix(seed + i) + j)),
 * then the RoCEv2 SEND_ONLY header template of the reference overwrites
 * bytes [0,40): IPv4 per shuffle_ingress.p4:717-724 (ver_ihl 0x45, id
 * 0x1234, flags 0x4000, proto 17), src 192.168.1.100 / dst 192.168.1.(1+i%4)
 * (switchd/vswitchd.hpp:52-56, shuffle_drv.hpp:15), UDP sport 0x457b
 * (shuffle_drv.hpp:16), dport 4791 (header.p4:14), BTH opcode 0x04,
 * se/m/pad/tver 0x40, pkey 0xffff (shuffle_ingress.p4:734-735), ackreq 0,
 * psn = i mod 2^24.  tos, ttl, both checksums, the FECN/BECN byte, dqpn and
 * the payload stay random, so every masked field is exercised.
 */
static inline uint64_t mix64(uint64_t z) {
  z += 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

void oracle_synth_packet(uint64_t seed, uint64_t i, uint32_t n, uint32_t stride, uint8_t *dst) {
  uint64_t h = mix64(seed + i);
  for (uint32_t j = 0; j * 8 < stride; ++j) {
    uint64_t r = mix64(h + j);
    uint32_t lim = stride - j * 8 < 8 ? stride - j * 8 : 8;
    for (uint32_t k = 0; k < lim; ++k) dst[j * 8 + k] = (j * 8 + k < n) ? (uint8_t)(r >> (8 * k)) : 0;
  }
  if (n < 40) return;
  dst[0] = 0x45;
  dst[2] = (uint8_t)(n >> 8);
  dst[3] = (uint8_t)n;
  dst[4] = 0x12; dst[5] = 0x34; dst[6] = 0x40; dst[7] = 0x00;
  dst[9] = 17;
  dst[12] = 192; dst[13] = 168; dst[14] = 1; dst[15] = 100;
  dst[16] = 192; dst[17] = 168; dst[18] = 1; dst[19] = (uint8_t)(1 + (i & 3));
  dst[20] = 0x45; dst[21] = 0x7b; dst[22] = 0x12; dst[23] = 0xb7;
  dst[24] = (uint8_t)((n - 20) >> 8);
  dst[25] = (uint8_t)(n - 20);
  dst[28] = 0x04; dst[29] = 0x40; dst[30] = 0xff; dst[31] = 0xff;
  dst[36] = 0;
  dst[37] = (uint8_t)(i >> 16); dst[38] = (uint8_t)(i >> 8); dst[39] = (uint8_t)i;
}

void oracle_synth_batch(uint64_t seed, uint64_t first, uint64_t count, uint32_t n, uint32_t stride,
                        uint8_t *buf) {
  for (uint64_t k = 0; k < count; ++k) oracle_synth_packet(seed, first + k, n, stride, buf + k * stride);
}

/* Ragged restatement (ricrc_synth_ragged_device): packet k is global packet
 * first + k, len[k] bytes at buf + off[k]; bytes between packets untouched. */
void oracle_synth_ragged(uint64_t seed, uint64_t first, uint64_t count, const uint64_t *off,
                         const uint32_t *len, uint8_t *buf) {
  for (uint64_t k = 0; k < count; ++k) oracle_synth_packet(seed, first + k, len[k], len[k], buf + off[k]);
}
