// The all-gather plan of ricrc_batch_device_all / ricrc_allgather (pure host
// code, no HIP): which RCCL call each context device issues so that every
// device's d_out[k] ends with all shards in shard order.  Kept apart from the
// RCCL calls so the plan is checked on the CPU (ricrc_allgather_plan,
// tests/test_cpu_api.py) before any multi-GPU run.
//
// Invariants (RCCL's rules for the two forms):
//  * equal counts c: one in-place ncclAllGather per device k with
//    sendbuff = d_out[k] + k c == recvbuff + rank * c (RCCL's in-place
//    condition), count c -- every device in one group;
//  * unequal counts (byte-balanced ragged cuts): for every ordered pair
//    k != p with counts[k] > 0, device k sends its shard [at[k], at[k] +
//    counts[k]) to p and p receives it at the same offset at[k] of its own
//    buffer; every (k -> p) send has exactly one matching (p <- k) receive of
//    the same count; nothing is sent to oneself; zero-length shards issue
//    nothing; all calls of all devices in ONE ncclGroupStart/End (a device
//    that sent before posting its receives would otherwise deadlock).
#pragma once
#include <stdint.h>

#include <vector>

#include "../../include/roce_icrc.h"

namespace ricrc {

inline std::vector<ricrc_xfer> allgather_plan(int n, const uint64_t *counts) {
  std::vector<ricrc_xfer> ops;
  if (n <= 1) return ops;  // one device: the shard is already in place
  std::vector<uint64_t> at(n + 1, 0);
  bool equal = true;
  for (int k = 0; k < n; ++k) {
    at[k + 1] = at[k] + counts[k];
    equal = equal && counts[k] == counts[0];
  }
  for (int k = 0; k < n; ++k) {
    if (equal) {
      if (counts[k]) ops.push_back(ricrc_xfer{k, RICRC_XFER_ALLGATHER, -1, 0, at[k], counts[k]});
      continue;
    }
    for (int p = 0; p < n; ++p) {
      if (p == k) continue;
      if (counts[k]) ops.push_back(ricrc_xfer{k, RICRC_XFER_SEND, p, 0, at[k], counts[k]});
      if (counts[p]) ops.push_back(ricrc_xfer{k, RICRC_XFER_RECV, p, 0, at[p], counts[p]});
    }
  }
  return ops;
}

}  // namespace ricrc
