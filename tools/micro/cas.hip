// Micro-benchmark: cost of 64-bit global atomicCAS vs plain load/store, from
// 8 workgroups x 1024 threads into a 4 MiB table (the pre-pass's pattern).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <vector>
__device__ inline uint32_t hsh(uint64_t k) { return (uint32_t)k * 0x9E3779B1u; }
template <int MODE>
__global__ __launch_bounds__(1024) void k(uint64_t* t, uint32_t mask, uint64_t* out, uint64_t seed) {
  const uint64_t key = seed + (uint64_t)blockIdx.x * 1024 + threadIdx.x;
  const uint32_t h = (hsh(key) >> 8) & mask;
  __syncthreads();
  const uint64_t t0 = clock64();
  uint64_t r = 0;
  if (MODE == 0) r = atomicCAS((unsigned long long*)&t[h], ~0ull, (unsigned long long)key);
  if (MODE == 1) { r = t[h]; }
  if (MODE == 2) { t[h] = key; }
  if (MODE == 3) r = __hip_atomic_fetch_add(&t[h], 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  if (MODE == 4) r = __hip_atomic_compare_exchange_strong(&t[h], &r, key, __ATOMIC_RELAXED, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) ? 1 : 0;
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  const uint64_t t1 = clock64();
  if (threadIdx.x == 0) out[blockIdx.x] = t1 - t0;
  if (r == 12345) out[1000] = r;
}
int main() {
  uint64_t *t, *o;
  hipMalloc(&t, 4 << 20);
  hipMalloc(&o, 8192);
  const char* nm[] = {"atomicCAS", "plain load", "plain store", "fetch_add agent", "cas wg-scope"};
  for (int rep = 0; rep < 2; rep++)
    for (int mode = 0; mode < 5; mode++) {
      hipMemset(t, 0xFF, 4 << 20);
      for (int grid : {1, 8, 256}) {
        if (mode == 0) k<0><<<grid, 1024>>>(t, (1u << 19) - 1, o, 77 + rep * 1000000);
        if (mode == 1) k<1><<<grid, 1024>>>(t, (1u << 19) - 1, o, 77);
        if (mode == 2) k<2><<<grid, 1024>>>(t, (1u << 19) - 1, o, 77);
        if (mode == 3) k<3><<<grid, 1024>>>(t, (1u << 19) - 1, o, 77);
        if (mode == 4) k<4><<<grid, 1024>>>(t, (1u << 19) - 1, o, 77 + rep * 1000000);
        hipDeviceSynchronize();
        std::vector<uint64_t> h(grid);
        hipMemcpy(h.data(), o, grid * 8, hipMemcpyDeviceToHost);
        double s = 0;
        for (auto x : h) s += x;
        printf("rep %d %-16s grid %3d: %.0f cycles (1024 threads, 1 op each)\n", rep, nm[mode], grid, s / grid);
      }
    }
  return 0;
}
