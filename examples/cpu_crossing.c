/* One wire crossing of the reference simulator (python/simulator.py:49-55) as
 * a C caller would do it with the per-packet section of the C ABI, linked
 * against the HIP-free libroceicrc_cpu.so: build a RoCEv2 SEND_ONLY packet
 * (the field values of the reference's P4 template, shuffle_ingress.p4:717-735),
 * stamp its ICRC on transmit, verify it on arrival, and show the error
 * contract of the checked call.
 *
 *   cc -std=c99 -I include examples/cpu_crossing.c
 *      -L roce-test_amd/roce_icrc -lroceicrc_cpu -o examples/cpu_crossing   (examples/Makefile)
 *
 * Prints "icrc 0x........" for the packet and "ok"; exits non-zero on any
 * mismatch. */
#include <errno.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>

#include "roce_icrc.h"

static int fail(const char *what) {
  fprintf(stderr, "cpu_crossing: %s\n", what);
  return 1;
}

int main(void) {
  enum { N = 1024 };
  uint8_t pkt[N];
  memset(pkt, 0, sizeof pkt);
  /* IPv4: version 4 / IHL 5, total_len N, id 0x1234, DF, TTL 64, UDP */
  pkt[0] = 0x45;
  pkt[2] = N >> 8;
  pkt[3] = N & 0xFF;
  pkt[4] = 0x12;
  pkt[5] = 0x34;
  pkt[6] = 0x40;
  pkt[8] = 64;
  pkt[9] = 17;
  const uint8_t src[4] = {192, 168, 1, 100}, dst[4] = {192, 168, 1, 200};
  memcpy(pkt + 12, src, 4);
  memcpy(pkt + 16, dst, 4);
  /* UDP: sport 49152, dport 4791 (RoCEv2), length N - 20 */
  pkt[20] = 0xC0;
  pkt[22] = 4791 >> 8;
  pkt[23] = 4791 & 0xFF;
  pkt[24] = (N - 20) >> 8;
  pkt[25] = (N - 20) & 0xFF;
  /* BTH: opcode SEND_ONLY (RC 0x04), pkey 0xFFFF, dest QP 0x000011, PSN 7 */
  pkt[28] = 0x04;
  pkt[30] = 0xFF;
  pkt[31] = 0xFF;
  pkt[35] = 0x11;
  pkt[39] = 7;
  for (int i = 40; i < N - 4; ++i) pkt[i] = (uint8_t)(i * 131u + 7u);

  if (!ricrc_is_rocev2(pkt, N)) return fail("packet does not classify as RoCEv2");
  uint32_t icrc = 0;
  if (ricrc_icrc(pkt, N, RICRC_F_IPV4 | RICRC_F_STRICT, &icrc) != 0) return fail("ricrc_icrc");
  if (icrc != ricrc_one(pkt, N)) return fail("ricrc_icrc != ricrc_one");

  /* transmit: stamp; arrival: verify (what the NIC check does) */
  if (ricrc_stamp_one(pkt, N) != 0) return fail("stamp");
  const uint32_t trailer = (uint32_t)pkt[N - 4] | (uint32_t)pkt[N - 3] << 8 | (uint32_t)pkt[N - 2] << 16 |
                           (uint32_t)pkt[N - 1] << 24;
  if (trailer != icrc) return fail("trailer is not the little-endian ICRC");
  if (ricrc_verify_one(pkt, N) != 1) return fail("verify of a stamped packet");

  /* the switch rewrites TTL / checksum (invariant fields): still verifies */
  pkt[8] = 63;
  pkt[10] ^= 0x5A;
  if (ricrc_verify_one(pkt, N) != 1) return fail("verify after invariant-field rewrite");
  /* a flipped payload bit on the wire: caught, the receiver drops the packet */
  pkt[500] ^= 0x10;
  if (ricrc_verify_one(pkt, N) != 0) return fail("corruption not caught");
  pkt[500] ^= 0x10;

  /* error contract of the checked call */
  uint32_t v = 0xABCDu;
  if (ricrc_icrc(pkt, 43, RICRC_F_IPV4, &v) != -EINVAL || v != 0xABCDu) return fail("n < 44 must be -EINVAL");
  if (ricrc_icrc(NULL, N, RICRC_F_IPV4, &v) != -EINVAL) return fail("NULL must be -EINVAL");
  pkt[23] = 0; /* UDP dport 4791 -> 4608: not RoCEv2 */
  if (ricrc_icrc(pkt, N, RICRC_F_IPV4 | RICRC_F_STRICT, &v) != -EPROTO) return fail("strict must be -EPROTO");
  if (ricrc_icrc(pkt, N, RICRC_F_IPV4, &v) != 0) return fail("non-strict call must still compute");
  printf("icrc 0x%08x\nstrerror(-EPROTO): %s\nok\n", icrc, ricrc_strerror(-EPROTO));
  return 0;
}
