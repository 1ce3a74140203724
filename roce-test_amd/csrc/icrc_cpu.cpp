// Per-packet CPU entry points of libroceicrc (no GPU involved).
//
// ricrc_one is the per-packet call the reference's simulator crossings need
// (python/simulator.py:49-55, 59-82): one L3 packet in, one 32-bit ICRC out.
// It restates calc_icrc() (p4/shuffle/shuffle_egress.p4:463-494) with a
// slice-by-16 table fold; the 8 x 0xFF prefix (:465) is folded into the
// starting register kSeed, the masked fields (:467-485) are applied to a
// copy of the header, and everything after it (the AETH of :489-490, and, as
// IBTA Annex A17 generalises calc_icrc beyond the ACK it was written for,
// extension headers and payload) is folded straight
// from the caller's buffer.  The *_ex variants add RoCEv2 over IPv6 (masks of
// IBTA Annex A17 / Linux rxe) and per-packet family detection.
#include <errno.h>
#include <string.h>

#include <algorithm>
#include <thread>
#include <vector>

#include "../../include/roce_icrc.h"
#include "icrc_math.h"
#include "icrc_plan.h"

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

uint32_t family_of(const uint8_t *l3, uint32_t n, uint32_t flags) {
  if (flags == ricrc::kFamAuto) return (n > 0 && (l3[0] >> 4) == 6) ? ricrc::kFamV6 : ricrc::kFamV4;
  return flags == ricrc::kFamV6 ? ricrc::kFamV6 : ricrc::kFamV4;
}

// Register over 0xFF x 8 || masked L3[0, n-4); n >= 4.  The masked bytes
// (either family) all lie in the first kMaskSpan bytes: they are applied to a
// copy of that head, the rest is folded from the caller's buffer.
uint32_t icrc_register(const uint8_t *l3, uint32_t n, uint32_t fam) {
  const size_t m = n - 4, h = m < ricrc::kMaskSpan ? m : ricrc::kMaskSpan;
  uint8_t head[ricrc::kMaskSpan];
  memcpy(head, l3, h);
  for (size_t i = 0; i < h; ++i) head[i] |= (uint8_t)ricrc::mask_byte(fam, (uint32_t)i);
  uint32_t c = fold_bytes(ricrc::kSeed, head, h);
  return fold_bytes(c, l3 + h, m - h);
}

bool flags_ok(uint32_t flags) { return flags <= ricrc::kFamAuto; }

// RICRC_F_FRAMELEN: the L3 length of the packet whose frame extends n bytes past l3.
uint32_t frame_len(const uint8_t *l3, uint32_t n) {
  if (!ricrc::frame_len_applies(n)) return n;
  return ricrc::frame_l3_len(n, l3[0], (uint32_t)l3[2] << 8 | l3[3], (uint32_t)l3[4] << 8 | l3[5]);
}

}  // namespace

extern "C" {

uint32_t ricrc_one_ex(const uint8_t *l3, uint32_t n, uint32_t flags) {
  if (!l3 || n < 4 || !flags_ok(flags)) return 0;
  return ~icrc_register(l3, n, family_of(l3, n, flags));
}

uint32_t ricrc_one(const uint8_t *l3, uint32_t n) { return ricrc_one_ex(l3, n, RICRC_F_IPV4); }

int ricrc_icrc(const uint8_t *l3, uint32_t n, uint32_t flags, uint32_t *out) {
  const uint32_t fam = flags & ~(RICRC_F_STRICT | RICRC_F_FRAMELEN);
  if (!l3 || !out || !flags_ok(fam)) return -EINVAL;
  if (flags & RICRC_F_FRAMELEN) n = frame_len(l3, n);
  if (n < RICRC_MIN_LEN || n > RICRC_MAX_LEN) return -EINVAL;
  if (flags & RICRC_F_STRICT) {
    const int c = ricrc_classify(l3, n);
    const uint32_t want = fam == RICRC_F_AUTO ? 0u : (fam == RICRC_F_IPV6 ? 6u : 4u);
    if (c == 0 || (want && (uint32_t)c != want)) return -EPROTO;
  }
  *out = ~icrc_register(l3, n, family_of(l3, n, fam));
  return 0;
}

int ricrc_verify_one_ex(const uint8_t *l3, uint32_t n, uint32_t flags) {
  if (!l3 || n < 4 || !flags_ok(flags)) return -EINVAL;
  return ricrc_one_ex(l3, n, flags) == load_le32(l3 + n - 4) ? 1 : 0;
}

int ricrc_verify_one(const uint8_t *l3, uint32_t n) { return ricrc_verify_one_ex(l3, n, RICRC_F_IPV4); }

int ricrc_stamp_one_ex(uint8_t *l3, uint32_t n, uint32_t flags) {
  if (!l3 || n < 4 || !flags_ok(flags)) return -EINVAL;
  const uint32_t v = ricrc_one_ex(l3, n, flags);
  memcpy(l3 + n - 4, &v, 4);  // little-endian host == LE32 on the wire
  return 0;
}

int ricrc_stamp_one(uint8_t *l3, uint32_t n) { return ricrc_stamp_one_ex(l3, n, RICRC_F_IPV4); }

int ricrc_repair_one(const uint8_t *l3, uint32_t n, uint32_t off, const uint8_t *old_bytes, uint32_t len,
                     uint32_t old_icrc, uint32_t flags, uint32_t *new_icrc) {
  if (!l3 || !old_bytes || !new_icrc || n < 4 || !flags_ok(flags)) return -EINVAL;
  const uint32_t m = n - 4;
  if (off > m || len > m - off) return -EINVAL;  // only covered bytes [0, n-4) can change
  const uint32_t fam = family_of(l3, n, flags);
  if (flags == ricrc::kFamAuto && off == 0 && len > 0 && (old_bytes[0] >> 4) != (l3[0] >> 4))
    return -EINVAL;  // the rewrite changed the address family: recompute instead
  // Linearity: the register moves by crc0(delta) advanced over the covered
  // bytes after the range; masked bytes contribute nothing to either side.
  uint32_t c = 0;
  for (uint32_t i = 0; i < len; ++i) {
    const uint32_t mb = ricrc::mask_byte(fam, off + i);
    const uint8_t d = (uint8_t)((l3[off + i] ^ old_bytes[i]) & ~mb);
    c = kT.t[0][(c ^ d) & 0xFF] ^ (c >> 8);
  }
  *new_icrc = old_icrc ^ ricrc_shift(c, (uint64_t)(m - off - len));
  return 0;
}

int ricrc_classify(const uint8_t *l3, uint32_t n) {
  if (!l3 || n < RICRC_MIN_LEN || n > RICRC_MAX_LEN) return 0;
  if (ricrc_is_rocev2(l3, n)) return 4;
  // IPv6: version 6, next header UDP, payload length = n - 40, dport 4791.
  if (n < 40 + 8 + 12 + 4 || (l3[0] >> 4) != 6 || l3[6] != 17) return 0;
  if (((uint32_t)l3[4] << 8 | l3[5]) != n - 40) return 0;
  if (((uint32_t)l3[42] << 8 | l3[43]) != 4791) return 0;
  return 6;
}

int ricrc_is_rocev2(const uint8_t *l3, uint32_t n) {
  if (!l3 || n < RICRC_MIN_LEN) return 0;
  if (l3[0] != 0x45 || l3[9] != 17) return 0;                // ipv4_h ver_ihl / protocol
  if (((uint32_t)l3[2] << 8 | l3[3]) != n) return 0;         // total_len
  if (((uint32_t)l3[22] << 8 | l3[23]) != 4791) return 0;    // udp_h dst_port == UDP_PORT_ROCE
  return 1;
}

int ricrc_batch_cpu(const uint8_t *base, const uint64_t *off, const uint32_t *len, uint32_t stride, uint64_t count,
                    uint32_t l3_offset, uint32_t *out, uint32_t flags, int threads) {
  if (count == 0) return 0;
  const bool framelen = (flags & RICRC_F_FRAMELEN) != 0;
  flags &= ~RICRC_F_FRAMELEN;
  if (!base || !out || !flags_ok(flags)) return -EINVAL;
  if (!off && stride == 0) return -EINVAL;
  if (!len && stride <= l3_offset) return -EINVAL;
  auto pkt = [&](uint64_t i, uint32_t &n) -> const uint8_t * {
    n = len ? len[i] : stride - l3_offset;
    const uint8_t *p = base + (off ? off[i] : i * (uint64_t)stride) + l3_offset;
    if (framelen) n = frame_len(p, n);
    return p;
  };
  for (uint64_t i = 0; i < count; ++i) {
    uint32_t n;
    (void)pkt(i, n);
    if (n < RICRC_MIN_LEN || n > RICRC_MAX_LEN) return -EINVAL;
  }
  auto work = [&](uint64_t lo, uint64_t hi) {
    for (uint64_t i = lo; i < hi; ++i) {
      uint32_t n;
      const uint8_t *p = pkt(i, n);
      out[i] = ~icrc_register(p, n, family_of(p, n, flags));
    }
  };
  const uint64_t t = (uint64_t)std::max(1, std::min(threads, 256));
  const uint64_t nt = std::min<uint64_t>(t, count);
  // A thread that cannot be created must not throw across the C ABI: its
  // range (and every later one) runs on the caller's thread instead.
  std::vector<std::thread> th;
  uint64_t k = 1;
  try {
    th.reserve(nt - 1);
    for (; k < nt; ++k) th.emplace_back(work, count * k / nt, count * (k + 1) / nt);
  } catch (...) {
  }
  work(0, count / nt);
  if (k < nt) work(count * k / nt, count);
  for (auto &x : th) x.join();
  return 0;
}

int ricrc_allgather_plan(int n, const uint64_t *counts, ricrc_xfer *ops, int max_ops) {
  if (n < 1 || !counts || (max_ops > 0 && !ops)) return -EINVAL;
  const std::vector<ricrc_xfer> plan = ricrc::allgather_plan(n, counts);
  for (int i = 0; i < (int)plan.size() && i < max_ops; ++i) ops[i] = plan[i];
  return (int)plan.size();
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
    case -EPROTO: return "not a RoCEv2 packet of the requested address family (RICRC_F_STRICT)";
    default: return "unknown error";
  }
}

}  // extern "C"
