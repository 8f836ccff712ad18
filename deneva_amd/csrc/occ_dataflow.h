// Key table of the OCC dataflow solver (occ_dataflow.hip): the survivors'
// write keys, open addressing with linear probes, KEY_EMPTY = free.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "dcc_device.h"
#include "occ_kernels.h"

namespace dcc {

__device__ inline uint32_t df_hash(uint64_t key, uint32_t bits) {
  return (uint32_t)(fmix64(key) >> (64 - bits));
}

// Insert-or-find (linear probes).  A plain agent-scope read first: a hot key's
// writers must not all CAS one word; a stale EMPTY only costs a CAS that then
// returns the truth.  Keys are never removed during an epoch.
__device__ inline uint32_t df_insert(uint64_t* tab, uint32_t bits, uint64_t key) {
  const uint32_t mask = (1u << bits) - 1u;
  uint32_t h = df_hash(key, bits);
  for (uint32_t n = 0; n <= mask; n++) {
    const uint64_t cur = __hip_atomic_load(&tab[h], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (cur == key) return h;
    if (cur == KEY_EMPTY) {
      const unsigned long long prev = atomicCAS((unsigned long long*)&tab[h], (unsigned long long)KEY_EMPTY,
                                                (unsigned long long)key);
      if (prev == KEY_EMPTY || prev == key) return h;
    }
    h = (h + 1) & mask;
  }
  return DF_NONE;
}
__device__ inline uint32_t df_find(const uint64_t* tab, uint32_t bits, uint64_t key) {
  const uint32_t mask = (1u << bits) - 1u;
  uint32_t h = df_hash(key, bits);
  for (uint32_t n = 0; n <= mask; n++) {
    const uint64_t cur = tab[h];
    if (cur == key) return h;
    if (cur == KEY_EMPTY) return DF_NONE;
    h = (h + 1) & mask;
  }
  return DF_NONE;
}

}  // namespace dcc
