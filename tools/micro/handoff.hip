// Microbenchmark: latency of a chain of cross-workgroup hand-offs through
// u32 flags, per polling form.  Block k (k >= 1) waits until flag[k-1] is
// set, then sets flag[k]; blocks are spread over XCDs by dispatch order.
// All blocks are co-resident (grid <= CUs); every spin is bounded.
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>

__device__ inline uint32_t ld_atomic(const uint32_t* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ inline uint32_t ld_rmw(uint32_t* p) { return atomicAdd(p, 0u); }
__device__ inline uint32_t ld_acq(const uint32_t* p) {
  return __hip_atomic_load(p, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT);
}

template <int MODE>
__global__ void chain(uint32_t* flags, uint32_t* timeout, int stride) {
  if (threadIdx.x != 0) return;
  const int k = blockIdx.x;
  uint32_t* prev = flags + (k - 1) * stride;
  if (k > 0) {
    unsigned spins = 0;
    for (;;) {
      uint32_t v;
      if (MODE == 0) v = ld_atomic(prev);
      else if (MODE == 1) v = ld_rmw(prev);
      else v = ld_acq(prev);
      if (v) break;
      if (++spins > (1u << 24)) { atomicOr(timeout, 1u); break; }
      __builtin_amdgcn_s_sleep(1);
    }
  }
  __hip_atomic_store(flags + k * stride, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

int main() {
  const int nb = 256, stride = 32;
  uint32_t *flags, *to;
  hipMalloc(&flags, nb * stride * 4);
  hipMalloc(&to, 4);
  const char* names[3] = {"relaxed agent atomic load", "atomicAdd(0) rmw", "acquire agent load"};
  for (int mode = 0; mode < 3; mode++) {
    for (int rep = 0; rep < 4; rep++) {
      hipMemset(flags, 0, nb * stride * 4);
      hipMemset(to, 0, 4);
      hipDeviceSynchronize();
      hipEvent_t a, b;
      hipEventCreate(&a);
      hipEventCreate(&b);
      hipEventRecord(a);
      if (mode == 0) chain<0><<<nb, 64>>>(flags, to, stride);
      if (mode == 1) chain<1><<<nb, 64>>>(flags, to, stride);
      if (mode == 2) chain<2><<<nb, 64>>>(flags, to, stride);
      hipEventRecord(b);
      hipEventSynchronize(b);
      float ms;
      hipEventElapsedTime(&ms, a, b);
      uint32_t t;
      hipMemcpy(&t, to, 4, hipMemcpyDeviceToHost);
      if (rep == 3) printf("%-28s chain of %d hops: %8.1f us  (%.2f us/hop)%s\n", names[mode], nb - 1,
                           ms * 1e3, ms * 1e3 / (nb - 1), t ? "  TIMEOUT" : "");
    }
  }
  return 0;
}
