// Timing-only microbenches: a device buffer standing in for the context's
// finish tables (SckArgs::fin, RsckArgs::fin; the product builds them with
// build_fin_tables).  Arbitrary words: the microbenches time, never check.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
static const uint32_t *mb_fin() {
  static uint32_t *p = nullptr;
  if (!p && hipMalloc(&p, 4 * 2048) == hipSuccess) (void)hipMemset(p, 0x5A, 4 * 2048);
  return p;
}
