// Per-packet CPU entry points of libroceicrc (no GPU involved).
//
// ricrc_one is the per-packet call the reference's simulator crossings need
// (python/simulator.py:49-55, 59-82): one L3 packet in, one 32-bit ICRC out.
// It restates calc_icrc() (p4/shuffle/shuffle_egress.p4:463-494) with a
// slice-by-16 table fold; the 8 x 0xFF prefix (:465) is folded into the
// starting register kSeed, the masked fields (:467-485) are applied to a
// 40-byte copy of the header, and everything after it (:489-490) is folded
// straight from the caller's buffer.
#include <errno.h>
#include <string.h>

#include "../../include/roce_icrc.h"
#include "icrc_math.h"

namespace {

constexpr ricrc::SliceTables<16> kT = ricrc::make_tables<16>();

inline uint32_t load_le32(const uint8_t *p) {
  uint32_t v;
  memcpy(&v, p, 4);
  return v;
}

uint32_t fold_bytes(uint32_t c, const uint8_t *p, size_t n) {
  while (n >= 16) {
    uint32_t w0 = load_le32(p) ^ c, w1 = load_le32(p + 4), w2 = load_le32(p + 8), w3 = load_le32(p + 12);
    c = kT.t[15][w0 & 0xFF] ^ kT.t[14][(w0 >> 8) & 0xFF] ^ kT.t[13][(w0 >> 16) & 0xFF] ^ kT.t[12][w0 >> 24] ^
        kT.t[11][w1 & 0xFF] ^ kT.t[10][(w1 >> 8) & 0xFF] ^ kT.t[9][(w1 >> 16) & 0xFF] ^ kT.t[8][w1 >> 24] ^
        kT.t[7][w2 & 0xFF] ^ kT.t[6][(w2 >> 8) & 0xFF] ^ kT.t[5][(w2 >> 16) & 0xFF] ^ kT.t[4][w2 >> 24] ^
        kT.t[3][w3 & 0xFF] ^ kT.t[2][(w3 >> 8) & 0xFF] ^ kT.t[1][(w3 >> 16) & 0xFF] ^ kT.t[0][w3 >> 24];
    p += 16;
    n -= 16;
  }
  while (n--) c = kT.t[0][(c ^ *p++) & 0xFF] ^ (c >> 8);
  return c;
}

// Register over 0xFF x 8 || masked L3[0, n-4); n >= 4.
uint32_t icrc_register(const uint8_t *l3, uint32_t n) {
  const size_t m = n - 4, h = m < 40 ? m : 40;
  uint8_t head[40];
  memcpy(head, l3, h);
  for (int i = 0; i < 40; ++i)
    if (((ricrc::kMaskBits >> i) & 1u) && (size_t)i < h) head[i] = 0xFF;
  uint32_t c = fold_bytes(ricrc::kSeed, head, h);
  return fold_bytes(c, l3 + h, m - h);
}

}  // namespace

extern "C" {

uint32_t ricrc_one(const uint8_t *l3, uint32_t n) {
  if (!l3 || n < 4) return 0;
  return ~icrc_register(l3, n);
}

int ricrc_verify_one(const uint8_t *l3, uint32_t n) {
  if (!l3 || n < 4) return -EINVAL;
  return ricrc_one(l3, n) == load_le32(l3 + n - 4) ? 1 : 0;
}

int ricrc_stamp_one(uint8_t *l3, uint32_t n) {
  if (!l3 || n < 4) return -EINVAL;
  const uint32_t v = ricrc_one(l3, n);
  memcpy(l3 + n - 4, &v, 4);  // little-endian host == LE32 on the wire
  return 0;
}

int ricrc_is_rocev2(const uint8_t *l3, uint32_t n) {
  if (!l3 || n < RICRC_MIN_LEN) return 0;
  if (l3[0] != 0x45 || l3[9] != 17) return 0;                // ipv4_h ver_ihl / protocol
  if (((uint32_t)l3[2] << 8 | l3[3]) != n) return 0;         // total_len
  if (((uint32_t)l3[22] << 8 | l3[23]) != 4791) return 0;    // udp_h dst_port == UDP_PORT_ROCE
  return 1;
}

uint32_t ricrc_shift(uint32_t reg, uint64_t nbytes) { return ricrc::gf_mul(reg, ricrc::gf_x8n(nbytes)); }

uint32_t ricrc_combine(uint32_t crc1, uint32_t crc2, uint64_t len2) {
  return ricrc::gf_mul(crc1, ricrc::gf_x8n(len2)) ^ crc2;
}

const char *ricrc_strerror(int err) {
  switch (err) {
    case 0: return "success";
    case -EINVAL: return "invalid argument (length out of range, NULL pointer or misaligned buffer)";
    case -ENODEV: return "no usable GPU device";
    case -ENOMEM: return "out of memory";
    case -EIO: return "HIP/RCCL runtime error";
    default: return "unknown error";
  }
}

}  // extern "C"
