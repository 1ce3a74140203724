/*
 * libroceicrc -- MI355X-native RoCEv2 Invariant-CRC engine, C ABI.
 *
 * What this replaces (reference = cqzhangyu/roce-test):
 *   - calc_icrc()            p4/shuffle/shuffle_egress.p4:463-494 (the only ICRC
 *                            arithmetic in the reference; its call is commented
 *                            out at :669, so rewritten packets carry stale ICRCs)
 *   - scripts/icrc/{disable,enable,query}-icrc.sh:12-41 (turn NIC ICRC checking
 *                            off because of the above; with correct ICRCs that
 *                            is no longer needed)
 *   - the per-packet "ICRC of a Packet" hook python/simulator.py would call at
 *     its wire crossings (simulator.py:49-55, 59-82) via ctypes.
 * The reference has no FFI for this path; the signatures below follow its C++
 * conventions instead: 0 / negative-errno returns (shuffle_endpoint.hpp:364-389,
 * 447-471), errors reported, never aborting (logassert, common/logger.hpp:190),
 * caller-owned buffers (huge_malloc MRs, common/huge_malloc.h:12-22).
 *
 * Packet convention: an "n-byte packet" is the L3 RoCEv2 packet with IPv4
 * total_len = n: IPv4(20) || UDP(8) || BTH(12) || ext || payload+pad || ICRC(4)
 * (p4/common/header.p4:42-112).  The ICRC covers 0xFF x 8 || L3[0, n-4) with the
 * invariant fields masked; the returned value v is put on the wire as LE32(v)
 * (shuffle_egress.p4:493), i.e. trailer bytes = v & 0xff, v >> 8, ...
 * calc_icrc's own field list stops at the AETH: it is written for the
 * switch's 48-byte write ACKs (IPv4 || UDP || BTH || AETH), for which the two
 * definitions hash the same bytes; covering every byte after the BTH for
 * every other packet is IBTA Annex A17's ICRC (as Linux rxe and NICs compute
 * it), a deliberate generalisation.
 *
 * Errors: 0 = success, negative errno: -EINVAL (bad length / NULL / alignment),
 * -ENODEV (no GPU), -ENOMEM, -EIO (HIP / RCCL failure), -EPROTO (not RoCEv2,
 * strict mode).  Nothing aborts.
 *
 * Two shared libraries implement this header:
 *   libroceicrc.so      everything (gfx950 kernels + host runtime + RCCL);
 *   libroceicrc_cpu.so  the CPU section only (ricrc_one .. ricrc_combine,
 *                       ricrc_icrc, ricrc_batch_cpu, ricrc_strerror), built by g++ with no HIP,
 *                       RCCL or torch dependency: the simulator drop-in
 *                       (python/simulator.py:49-55) loads it on any host.
 */
#ifndef ROCE_ICRC_H
#define ROCE_ICRC_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define RICRC_MIN_LEN 44u    /* IPv4 20 + UDP 8 + BTH 12 + ICRC 4 */
#define RICRC_MAX_LEN 65535u /* IPv4 total_len is 16 bits */

typedef struct ricrc_ctx ricrc_ctx;

/* ------------------------------------------------------------ per packet (CPU)
 * ricrc_one: ICRC of one L3 packet of n bytes (n >= 4; masks that fall beyond
 * n-4 are skipped).  Pure, re-entrant, thread-safe.  Returns 0 for n < 4.
 * Replaces calc_icrc() (shuffle_egress.p4:463-494) for the simulator's
 * one-packet-at-a-time crossings, where a GPU launch would be pure overhead. */
uint32_t ricrc_one(const uint8_t *l3, uint32_t n);

/* Checked per-packet call with the SURVEY §8(b) length contract: *out = the
 * ICRC, return 0; -EINVAL for NULL, n outside [RICRC_MIN_LEN, RICRC_MAX_LEN]
 * or bad flags.  flags = a family (RICRC_F_IPV4/IPV6/AUTO, below), optionally
 * | RICRC_F_STRICT: the packet must also classify as RoCEv2 of that family
 * (ricrc_classify: the ingress parser's accept path,
 * shuffle_ingress_parser.p4:12-36), else -EPROTO and *out is untouched. */
int ricrc_icrc(const uint8_t *l3, uint32_t n, uint32_t flags, uint32_t *out);

/* 1 if the trailer holds the right ICRC, 0 if not, -EINVAL if n < 4 / NULL.
 * The check NICs perform and scripts/icrc/disable-icrc.sh:27-33 turns off. */
int ricrc_verify_one(const uint8_t *l3, uint32_t n);

/* Writes the ICRC into the trailer (bytes n-4..n-1, LE32).  0 / -EINVAL. */
int ricrc_stamp_one(uint8_t *l3, uint32_t n);

/* 1 if l3 is a RoCEv2 packet this engine accepts: IPv4, IHL 5, protocol 17,
 * UDP dport 4791, total_len == n, RICRC_MIN_LEN <= n (the ingress parser's
 * accept path, p4/shuffle/shuffle_ingress_parser.p4:12-36, header.p4:14). */
int ricrc_is_rocev2(const uint8_t *l3, uint32_t n);

/* CPU batch: out[i] = ICRC of packet i, addressed as in the GPU batch calls
 * below, folded by the slice-by-16 code of ricrc_one on `threads` host
 * threads (the caller's thread included).  For hosts without a GPU and the
 * CPU figure bench.py reports next to the GPU's; the GPU batch calls never
 * fall back to it.  0, or -EINVAL (NULL, bad flags, a length outside
 * [RICRC_MIN_LEN, RICRC_MAX_LEN]; nothing is written then). */
int ricrc_batch_cpu(const uint8_t *base, const uint64_t *off, const uint32_t *len, uint32_t stride, uint64_t count,
                    uint32_t l3_offset, uint32_t *out, uint32_t flags, int threads);

/* ------------------------------------------------------- address families
 * The reference is IPv4-only (header.p4:42-53, shuffle_ingress_parser.p4:16-19)
 * and every entry point without a flags argument keeps exactly its masks.
 * The *_ex entry points take one of:
 *   RICRC_F_IPV4  IPv4 masks (as the plain entry points);
 *   RICRC_F_IPV6  RoCEv2 over IPv6: traffic class + flow label (L3 byte 0 low
 *                 nibble, bytes 1-3), hop limit (7), UDP checksum (46-47),
 *                 BTH byte 4 (52) forced to ones -- IBTA Annex A17 as the
 *                 Linux rxe driver applies it (rxe_icrc.c);
 *   RICRC_F_AUTO  per packet from the IP version nibble (6: IPv6, else IPv4).
 * Any other value: -EINVAL (per-packet calls returning a value: 0). */
#define RICRC_F_IPV4 0u
#define RICRC_F_IPV6 1u
#define RICRC_F_AUTO 2u
#define RICRC_F_STRICT 0x100u /* ricrc_icrc / *_st calls: reject packets that do not classify */
/* ricrc_icrc / ricrc_batch_cpu / *_st calls: the length a descriptor gives
 * (n, len[i], or stride - l3_offset) is the FRAME's extent past the L3
 * start, which on an Ethernet NIC ring may include minimum-frame padding (a
 * 44-byte SEND_ONLY in a 60-byte frame: 2 bytes) and a kept FCS (4 bytes).
 * The packet's L3 length is then its IP header's -- IPv4 total_len, IPv6
 * payload length + 40 -- whenever that lies in [RICRC_MIN_LEN, the
 * descriptor length]; otherwise the descriptor length stands (and
 * RICRC_F_STRICT rejects the packet, its total_len not matching).  The
 * reference's parser takes each header's fields from the packet and never
 * uses a descriptor length (shuffle_ingress_parser.p4:12-36; total_len at
 * header.p4:45).  Without this flag the descriptor length is the L3 length. */
#define RICRC_F_FRAMELEN 0x400u

uint32_t ricrc_one_ex(const uint8_t *l3, uint32_t n, uint32_t flags);
int ricrc_verify_one_ex(const uint8_t *l3, uint32_t n, uint32_t flags);
int ricrc_stamp_one_ex(uint8_t *l3, uint32_t n, uint32_t flags);

/* 4: RoCEv2 over IPv4 (as ricrc_is_rocev2), 6: RoCEv2 over IPv6 (version 6,
 * next header 17, payload length n-40, UDP dport 4791, n >= 64), 0: neither
 * (also for n outside [RICRC_MIN_LEN, RICRC_MAX_LEN]). */
int ricrc_classify(const uint8_t *l3, uint32_t n);

/* Incremental repair after a header rewrite (the switch's PSN/MSN/opcode
 * patches, shuffle_egress.p4:635-671): l3 is the packet AFTER the rewrite,
 * bytes [off, off+len) held old_bytes before it and old_icrc was its ICRC.
 * *new_icrc = the rewritten packet's ICRC in O(len), not O(n):
 * old ^ shift(crc0(masked delta), n-4-off-len).  0, or -EINVAL (NULL,
 * n < 4, range past n-4, bad flags, or an AUTO rewrite that changes the IP
 * version). */
int ricrc_repair_one(const uint8_t *l3, uint32_t n, uint32_t off, const uint8_t *old_bytes, uint32_t len,
                     uint32_t old_icrc, uint32_t flags, uint32_t *new_icrc);

/* GF(2) helpers on the (un-inverted) CRC register -- the linear algebra behind
 * incremental repair after header rewrites (shuffle_egress.p4:635-671):
 *   ricrc_shift(reg, k)          = register advanced over k zero bytes
 *   ricrc_combine(c1, c2, len2)  = ICRC-style crc32 of A||B from crc32(A),
 *                                  crc32(B) and |B| (zlib crc32_combine). */
uint32_t ricrc_shift(uint32_t reg, uint64_t nbytes);
uint32_t ricrc_combine(uint32_t crc1, uint32_t crc2, uint64_t len2);

/* ------------------------------------------------------------------ context
 * n_gpus > 0: use devices 0..n_gpus-1; n_gpus < 0: every visible device;
 * n_gpus == 0 -> -EINVAL.  No GPU -> -ENODEV (there is no CPU fallback).
 * The context owns per-device streams, staging buffers and kernel state
 * (including one pinned 64-byte word per device where the big kernels record
 * which XCD their first workgroup ran on, a scheduling hint for the next
 * launch); it is not thread-safe (lock externally), exactly like the
 * reference's endpoint objects. */
int ricrc_create(ricrc_ctx **ctx, int n_gpus);
/* Same, on an explicit device list (one process per GPU: pass {LOCAL_RANK}). */
int ricrc_create_devices(ricrc_ctx **ctx, const int *devices, int n);
void ricrc_destroy(ricrc_ctx *ctx);
int ricrc_device_count(const ricrc_ctx *ctx);

/* ------------------------------------------------------------- batch calls
 * Packet i starts at base + (off ? off[i] : i * stride) + l3_offset and is
 * len ? len[i] : (stride - l3_offset) bytes long; out[i] = its ICRC.
 *
 * ricrc_batch_host: host buffers in and out.  Packets are sharded over the
 * context's GPUs by bytes, staged through pinned memory by parallel CPU
 * copies (or DMA'd directly if base was allocated by ricrc_host_alloc /
 * registered with ricrc_host_register / is otherwise pinned), computed on
 * the GPUs and copied back; chunks are double-buffered per GPU.  Synchronous.  Validates every length
 * (RICRC_MIN_LEN..RICRC_MAX_LEN) before touching a GPU.
 *
 * ricrc_batch_device: device-resident batch on context device `dev`
 * (pointers are device pointers on that device; off/len may be NULL).
 * Asynchronous on `stream` (a hipStream_t; NULL = the HIP null stream;
 * ricrc_stream() returns the context's own non-blocking stream).  Lengths
 * are not read on the host: a device length outside [4, RICRC_MAX_LEN]
 * yields out[i] = 0 -- which is also a possible ICRC: callers that must tell
 * bad descriptors apart use ricrc_batch_device_st (a status per packet).
 * 16-byte aligned packet starts with a fixed length take the streaming
 * kernels; anything else (offsets, lengths, any alignment or mix of sizes)
 * the ragged pipeline, several packets per wave.
 *
 * Buffer extent.  The caller owns the buffers (the reference's huge_malloc
 * MRs, common/huge_malloc.h:12-22) and every descriptor must lie inside the
 * caller's allocation: packet i's bytes [off[i] + l3_offset, + len[i]).  The
 * device calls take no extent and read the packets in place: a descriptor
 * past the end of the allocation makes the kernels read out of bounds (a GPU
 * memory fault, as a DMA engine given a bad descriptor would), it is NOT
 * reported as -EINVAL.  Callers whose descriptors are not trusted use
 * ricrc_batch_device_bounded / ricrc_batch_host_bounded below.
 * ricrc_batch_host checks the descriptors against the buffer when it knows
 * the buffer's size -- base inside a ricrc_host_alloc'd buffer -- and returns
 * -EINVAL (reading nothing) for one past its end.  A ricrc_host_register'ed
 * range bounds nothing (it may be one part of a larger caller buffer). */
int ricrc_batch_host(ricrc_ctx *ctx, const uint8_t *base, const uint64_t *off, const uint32_t *len,
                     uint32_t stride, uint64_t count, uint32_t l3_offset, uint32_t *out);
int ricrc_batch_device(ricrc_ctx *ctx, int dev, const void *d_base, const uint64_t *d_off,
                       const uint32_t *d_len, uint32_t stride, uint64_t count, uint32_t l3_offset,
                       uint32_t *d_out, void *stream);

/* Verify mode on the device: out[i] = 1 if packet i's trailer holds its ICRC,
 * else 0.  Same addressing/asynchrony as ricrc_batch_device. */
int ricrc_verify_device(ricrc_ctx *ctx, int dev, const void *d_base, const uint64_t *d_off,
                        const uint32_t *d_len, uint32_t stride, uint64_t count, uint32_t l3_offset,
                        uint32_t *d_out, void *stream);

/* Address-family variants of the batch calls (flags as the *_ex per-packet
 * calls: RICRC_F_IPV4 / RICRC_F_IPV6 / RICRC_F_AUTO by each packet's version
 * nibble).  The batch kernels apply the IPv4 masks; for IPV6 / AUTO one more
 * pass per packet corrects the result from the first min(56, n-4) header
 * bytes (the families' masks differ only there; the register is linear), and
 * does the verify compare.  Bad flags: -EINVAL.  Otherwise as the plain calls,
 * which are these with RICRC_F_IPV4. */
int ricrc_batch_host_ex(ricrc_ctx *ctx, const uint8_t *base, const uint64_t *off, const uint32_t *len,
                        uint32_t stride, uint64_t count, uint32_t l3_offset, uint32_t *out, uint32_t flags);
int ricrc_batch_device_ex(ricrc_ctx *ctx, int dev, const void *d_base, const uint64_t *d_off,
                          const uint32_t *d_len, uint32_t stride, uint64_t count, uint32_t l3_offset,
                          uint32_t *d_out, void *stream, uint32_t flags);
int ricrc_verify_device_ex(ricrc_ctx *ctx, int dev, const void *d_base, const uint64_t *d_off,
                           const uint32_t *d_len, uint32_t stride, uint64_t count, uint32_t l3_offset,
                           uint32_t *d_out, void *stream, uint32_t flags);

/* ------------------------------------------- batches with a per-packet status
 * For NIC rings that carry more than RoCEv2 and descriptors that may be bad.
 * The reference only ever computes an ICRC for frames its ingress parser
 * accepted as RoCEv2 (EtherType 0x0800 -> IPv4 protocol 17 -> UDP dport 4791,
 * p4/shuffle/shuffle_ingress_parser.p4:12-36, header.p4:8,14); these calls
 * apply that accept path per packet on the device and report, per packet:
 *   RICRC_ST_OK       out[i] is the ICRC (RICRC_F_VERIFY: 1/0, trailer check);
 *   RICRC_ST_BADLEN   its length is outside [RICRC_MIN_LEN, RICRC_MAX_LEN];
 *   RICRC_ST_NOTROCE  RICRC_F_STRICT and the packet is not RoCEv2 of an
 *                     accepted family: ricrc_classify's rules (IPv4: version
 *                     4 + IHL 5, protocol 17, total_len == n, dport 4791;
 *                     IPv6: version 6, next header 17, payload length n-40,
 *                     dport 4791), and, for Ethernet frames (l3_offset >=
 *                     14), the EtherType in the two bytes before L3 must be
 *                     the family's (0x0800 / 0x86DD);
 * and out[i] = 0 whenever status[i] != RICRC_ST_OK.
 * flags = a family (RICRC_F_IPV4 / IPV6 / AUTO; with RICRC_F_STRICT, IPV4 or
 * IPV6 accepts only that family, AUTO either) | RICRC_F_STRICT |
 * RICRC_F_VERIFY.  A batch without per-packet lengths whose one length
 * (stride - l3_offset) is out of range is a call error (-EINVAL).
 *
 * ricrc_batch_device_st: as ricrc_batch_device_ex, plus d_status (count
 *   bytes, device).  Asynchronous on `stream`.
 * ricrc_batch_host_st: as ricrc_batch_host_ex, plus status (count bytes,
 *   host); a bad descriptor length is a per-packet RICRC_ST_BADLEN here, not
 *   -EINVAL, and its bytes are never read.
 * ricrc_classify_device: d_class[i] = ricrc_classify of packet i (4 / 6 / 0),
 *   with the EtherType check above when l3_offset >= 14.  No ICRC.
 * 0, -EINVAL (NULL, bad flags), -ENODEV, -ENOMEM, -EIO. */
#define RICRC_F_VERIFY 0x200u /* *_st calls: out[i] = 1 if the trailer holds the ICRC, else 0 */
#define RICRC_ST_OK 0
#define RICRC_ST_BADLEN 1
#define RICRC_ST_NOTROCE 2
int ricrc_batch_device_st(ricrc_ctx *ctx, int dev, const void *d_base, const uint64_t *d_off,
                          const uint32_t *d_len, uint32_t stride, uint64_t count, uint32_t l3_offset,
                          uint32_t *d_out, uint8_t *d_status, void *stream, uint32_t flags);
int ricrc_batch_host_st(ricrc_ctx *ctx, const uint8_t *base, const uint64_t *off, const uint32_t *len,
                        uint32_t stride, uint64_t count, uint32_t l3_offset, uint32_t *out, uint8_t *status,
                        uint32_t flags);
int ricrc_classify_device(ricrc_ctx *ctx, int dev, const void *d_base, const uint64_t *d_off,
                          const uint32_t *d_len, uint32_t stride, uint64_t count, uint32_t l3_offset,
                          uint8_t *d_class, void *stream);

/* Extent-checked batches, for descriptors that are not trusted: base_bytes
 * is the size of the caller's buffer at base (> 0, else -EINVAL).
 * ricrc_batch_device_bounded: as ricrc_batch_device_st; a packet whose bytes
 *   do not all lie in [d_base, d_base + base_bytes) is never read and gets
 *   RICRC_ST_BADLEN and out[i] = 0.  A fixed-stride batch (no d_off, no
 *   d_len) that does not fit is -EINVAL.  Per-packet descriptors cost one
 *   pre-pass over them (12 bytes per packet, the RICRC_F_FRAMELEN pass).
 * ricrc_batch_host_bounded: as ricrc_batch_host_st with status != NULL (a
 *   packet outside the buffer: RICRC_ST_BADLEN, never read); with status ==
 *   NULL (flags: a family, optionally | RICRC_F_FRAMELEN) any packet outside
 *   the buffer, or of a bad length, is -EINVAL and nothing is computed. */
int ricrc_batch_device_bounded(ricrc_ctx *ctx, int dev, const void *d_base, uint64_t base_bytes,
                               const uint64_t *d_off, const uint32_t *d_len, uint32_t stride, uint64_t count,
                               uint32_t l3_offset, uint32_t *d_out, uint8_t *d_status, void *stream, uint32_t flags);
int ricrc_batch_host_bounded(ricrc_ctx *ctx, const uint8_t *base, uint64_t base_bytes, const uint64_t *off,
                             const uint32_t *len, uint32_t stride, uint64_t count, uint32_t l3_offset, uint32_t *out,
                             uint8_t *status, uint32_t flags);

/* Batch incremental repair on the device, after a header rewrite of packets
 * that were already stamped -- the switch egress's PSN/MSN/opcode patches
 * (shuffle_egress.p4:635-671), the reason the reference disables NIC ICRC
 * checking (scripts/icrc/disable-icrc.sh:13,30).  Packet i is addressed as in
 * ricrc_batch_device (d_base is writable); its bytes [off, off+len) held
 * d_old_bytes + i*old_stride before the rewrite and its trailer still holds
 * the old packet's ICRC.  d_out[i] (d_out may be NULL when stamp != 0) = the
 * rewritten packet's ICRC, computed from 2*len + 4 bytes of the packet
 * instead of n (ricrc_repair_one's identity); stamp != 0 also writes it
 * LE32 into the trailer.  flags as the *_ex calls.  Per packet, a length
 * outside [4, RICRC_MAX_LEN], a range past n-4, or an AUTO rewrite that
 * changes the IP version nibble gives d_out[i] = 0 and leaves the trailer
 * alone.  A wrong old trailer stays wrong (repair is incremental, not a
 * check: verify first where that matters).  0, -EINVAL (NULL pointers,
 * len > RICRC_REPAIR_MAX, off + len > RICRC_MAX_LEN - 4, old_stride < len,
 * bad flags), -ENODEV, -EIO.  Asynchronous on `stream`. */
#define RICRC_REPAIR_MAX 256u
int ricrc_repair_device(ricrc_ctx *ctx, int dev, void *d_base, const uint64_t *d_off, const uint32_t *d_len,
                        uint32_t stride, uint64_t count, uint32_t l3_offset, uint32_t off, uint32_t len,
                        const uint8_t *d_old_bytes, uint32_t old_stride, uint32_t flags, uint32_t stamp,
                        uint32_t *d_out, void *stream);

/* ----------------------------------------------- multi-GPU, one process
 * The reference's only scale-out is N endpoints behind one switch
 * (switchd/vswitchd.hpp:150-154); here a batch is sharded over the
 * context's GPUs and the 4-byte results are all-gathered over xGMI with RCCL
 * (the multi-process form is torch.distributed in bench.py).
 *
 * ricrc_comm_init: one RCCL communicator per context device, ncclCommInitAll
 * over the context's device list.  RCCL is resolved at run time (dlopen of
 * librccl.so.1, sharing one already loaded in the process).  Idempotent;
 * freed by ricrc_destroy.  0, -EINVAL, -ENODEV (no RCCL), -EIO.
 *
 * ricrc_batch_device_all: shard k lives on context device k: counts[k]
 * packets at d_base[k], addressed as in ricrc_batch_device (d_off / d_len
 * may be NULL, or arrays of per-device pointers, entries NULL too).  d_out[k]
 * is a buffer on device k of sum(counts) uint32; shard j's ICRCs go to
 * offset counts[0] + ... + counts[j-1] of every d_out[k].  Equal counts: one
 * in-place ncclAllGather; unequal counts (byte-balanced ragged cuts):
 * ncclSend/ncclRecv pairs in one group.  Asynchronous on each device's
 * context stream (ricrc_stream); ricrc_sync waits for all of them.  flags as
 * the *_ex calls.  0, -EINVAL (also: ricrc_comm_init not called), -EIO.
 *
 * ricrc_allgather: only the exchange, for shards computed by the caller into
 * d_out[k] + counts[0] + ... + counts[k-1] (on ricrc_stream(ctx, k)).
 *
 * Status: with more than one device this exchange is unverified on hardware
 * (the development boxes have one GPU); its plan (ricrc_allgather_plan,
 * below) is checked on the CPU by simulating RCCL's semantics. */
int ricrc_comm_init(ricrc_ctx *ctx);
int ricrc_batch_device_all(ricrc_ctx *ctx, const void *const *d_base, const uint64_t *const *d_off,
                           const uint32_t *const *d_len, uint32_t stride, const uint64_t *counts,
                           uint32_t l3_offset, uint32_t *const *d_out, uint32_t flags);
int ricrc_allgather(ricrc_ctx *ctx, const uint64_t *counts, uint32_t *const *d_out);

/* The exchange ricrc_allgather / ricrc_batch_device_all issue for n devices
 * and these counts, one entry per RCCL call (CPU only, no GPU, no RCCL; in
 * both libraries): equal counts -> one in-place ALLGATHER per device (offset
 * = k * count, RCCL's in-place condition); unequal -> SEND of device k's
 * shard to every peer and RECV of every peer's shard at its offset, all in
 * one RCCL group.  Offsets and counts are in uint32 elements of d_out[dev].
 * Returns the number of calls (entries beyond max_ops are not written),
 * -EINVAL for n < 1 or NULL counts. */
#define RICRC_XFER_ALLGATHER 0
#define RICRC_XFER_SEND 1
#define RICRC_XFER_RECV 2
typedef struct ricrc_xfer {
  int32_t dev;     /* context device (RCCL rank) that issues the call */
  int32_t kind;    /* RICRC_XFER_* */
  int32_t peer;    /* SEND / RECV: the other device; ALLGATHER: -1 */
  int32_t reserved;
  uint64_t offset; /* ALLGATHER / SEND: the shard sent from d_out[dev] + offset; RECV: lands at d_out[dev] + offset */
  uint64_t count;
} ricrc_xfer;
int ricrc_allgather_plan(int n, const uint64_t *counts, ricrc_xfer *ops, int max_ops);
int ricrc_sync(ricrc_ctx *ctx);

/* Pinned host memory for NIC-ring style buffers (the role of huge_malloc in
 * common/huge_malloc.h:12-22).  NULL on failure.  ricrc_batch_host DMAs
 * straight out of such memory (no CPU copy) whenever a chunk's packets form
 * an ascending span -- a fixed stride, or ring offsets with little slack. */
void *ricrc_host_alloc(ricrc_ctx *ctx, uint64_t bytes);
void ricrc_host_free(ricrc_ctx *ctx, void *p);

/* Pin an existing host buffer (e.g. a hugepage NIC ring from huge_malloc,
 * common/huge_malloc.h:12-22, or a numpy array) for the lifetime of the
 * registration, so ricrc_batch_host reads it by DMA.  0, -EINVAL (NULL, zero
 * size, already registered / not registered), -ENOMEM, -EIO.  Registrations
 * still live at ricrc_destroy are released there. */
int ricrc_host_register(ricrc_ctx *ctx, void *p, uint64_t bytes);
int ricrc_host_unregister(ricrc_ctx *ctx, void *p);

/* Synthetic RoCEv2 SEND_ONLY batch generator on device `dev` (bench / tests):
 * packet k of the buffer is global packet first+k, n bytes, at d_buf + k*stride.
 * Header template of the reference (shuffle_ingress.p4:717-724,734-735),
 * masked fields and payload seeded-random.  Asynchronous on `stream`. */
int ricrc_synth_device(ricrc_ctx *ctx, int dev, uint64_t seed, uint64_t first, uint64_t count,
                       uint32_t n, uint32_t stride, void *d_buf, void *stream);

/* Ragged variant: packet k is global packet first+k (same bytes as
 * ricrc_synth_device makes for that index and length), len[k] bytes at
 * d_buf + off[k] (device arrays).  Bytes between packets are left alone. */
int ricrc_synth_ragged_device(ricrc_ctx *ctx, int dev, uint64_t seed, uint64_t first, uint64_t count,
                              const uint64_t *d_off, const uint32_t *d_len, void *d_buf, void *stream);

/* Bring context device dev out of its idle power state: streams a 256 MiB
 * scratch buffer at HBM speed, back to back, for usec microseconds
 * (synchronous; ~20000 is enough on MI355X).  After >= 20 ms of idle, the
 * first ~12 launches of a burst otherwise run up to 15 % slower (DESIGN.md §4
 * "Power ramp").  A NIC-ring service calls it when traffic resumes; bench.py
 * calls it once before its warmup.  0, -EINVAL, -ENODEV, -ENOMEM, -EIO. */
int ricrc_prime(ricrc_ctx *ctx, int dev, uint32_t usec);

/* The context's own stream (a hipStream_t) for context device dev. */
void *ricrc_stream(ricrc_ctx *ctx, int dev);

/* The gfx950 kernel(s) ricrc_batch_device(_ex) launches for a batch of this
 * shape, from the same dispatch code: a static string of '+'-joined kernel
 * names as rocprofv3 reports them, e.g. "icrc_sck_kernel" (back-to-back 1, 2,
 * 4 KiB packets), "icrc_quad_kernel" (back-to-back 64 B) or
 * "rsck_bucket+icrc_rsck_kernel+icrc_rsmall_kernel+rsck_gather" (the ragged
 * pipeline), "+family_fix_kernel" for IPv6 / AUTO where the kernel applies
 * IPv4 masks.  No GPU is touched: d_base is inspected only for its alignment;
 * ctx may be NULL (the dispatch without the context's RICRC_NO_* test knobs).
 * NULL for a call ricrc_batch_device would reject (flags as the *_ex calls).
 * Bench and test labels come from here, so they name what actually ran. */
const char *ricrc_kernel_path(const ricrc_ctx *ctx, const void *d_base, const uint64_t *d_off, const uint32_t *d_len,
                              uint32_t stride, uint64_t count, uint32_t l3_offset, uint32_t flags);

/* How a batch of that shape would be launched on context device dev, as the
 * dispatch decides it (no GPU work): the main kernel's workgroups, the
 * per-XCD weights of its work split (all 0: equal shares; the SCK's 4 KiB
 * path and the ragged fold weight the odd-numbered XCDs, which stream HBM a
 * few per cent slower), the XCD the device's last strided-chain launch
 * started on (the next launch's k in the split), and for the ragged
 * pipeline its bucket / gather pass blocks, packets per thread and whether
 * the gather folds the one-line packets; for every path the lanes that fold
 * one packet.  ctx may be NULL (dev 0): the dispatch on a 256-CU MI355X
 * with the default knobs, no GPU needed.  bench.py reports it next to its
 * numbers.  0, or -EINVAL as ricrc_kernel_path's NULL. */
typedef struct {
  uint32_t grid;           /* workgroups of the main kernel (0: not reported for this path) */
  uint32_t xcd_weights[8]; /* the main kernel's work split by XCD; all 0 = equal shares */
  uint32_t start_xcd;      /* recorded by the last strided-chain kernel on this device */
  uint32_t pass_grid;      /* ragged: bucket / gather blocks (0 otherwise) */
  uint32_t pass_unroll;    /* ragged: packets per thread of those passes */
  uint32_t one_line;       /* ragged: who folds the one-line packets: 2 the fold (default), 1 the gather,
                              0 a separate one-line kernel (RICRC_ONE_LINE_IN_GATHER selects 1 or 0) */
  uint32_t gather_grid;    /* ragged: gather blocks (2 x pass_grid when one-line sides run beside them) */
  uint32_t lanes_per_packet; /* lanes of a wave that fold one packet (SCK and the ragged fold 8, the quad
                                kernel 4, TSK n / 32, the streaming kernel its chunk lanes; the ragged
                                pipeline's one-line packets take one lane each) */
} ricrc_launch_info_t;
int ricrc_launch_info(const ricrc_ctx *ctx, int dev, const void *d_base, const uint64_t *d_off,
                      const uint32_t *d_len, uint32_t stride, uint64_t count, uint32_t l3_offset,
                      ricrc_launch_info_t *info);

/* Diagnostics: with RICRC_PASS_TIMES set when the context was created, every
 * ragged-pipeline call on device dev records timing events between its
 * passes (costing a few microseconds per call); this waits for the recorded
 * calls, writes into ms[0..min(n,4)) the summed milliseconds of the bucket
 * pass, the fold, the one-line kernel (with the wait for its side launch)
 * and the gather, and returns how many calls were summed (then forgets
 * them; the last 64 calls are kept).
 * 0 without RICRC_PASS_TIMES; -EINVAL, -ENODEV, -EIO. */
int ricrc_pass_times(ricrc_ctx *ctx, int dev, float *ms, int n);

const char *ricrc_strerror(int err);

#ifdef __cplusplus
}
#endif

#endif /* ROCE_ICRC_H */
