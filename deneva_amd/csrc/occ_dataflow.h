// Buckets of the OCC dataflow solver (occ_dataflow.hip): a write key's bucket.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "dcc_device.h"
#include "occ_kernels.h"

namespace dcc {

__device__ inline uint32_t df_bucket(uint64_t key, uint32_t bits) {
  return (uint32_t)(fmix64(key) >> (64 - bits));
}

}  // namespace dcc
