// LDS operation throughput on one workgroup of 1024 threads (gfx950): cycles
// per wave-instruction for reads, atomics and byte stores at random and
// contended addresses -- the costs the fixed-point pass (occ_sweep.hip) is
// built from.  hipcc --offload-arch=gfx950 -O3 lds_ops.hip -o lds_ops
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdint>

constexpr int NW = 16384;  // LDS words
constexpr int ITER = 64;   // operations per thread

__device__ inline uint32_t rnd(uint32_t x) {
  x ^= x >> 16;
  x *= 0x7feb352du;
  x ^= x >> 15;
  x *= 0x846ca68bu;
  x ^= x >> 16;
  return x;
}

// mode: 0 read random, 1 atomicMin random, 2 atomicMin 8 addresses per wave,
// 3 atomicMin one address per wave, 4 atomicOr one word per 32 lanes,
// 5 byte store random, 6 byte store 64 consecutive bytes, 7 read same address
// 8 atomicMin random, half the lanes masked
__global__ __launch_bounds__(1024) void k_lds(int mode, uint64_t* out, uint32_t* sink) {
  __shared__ uint32_t w[NW];
  const uint32_t j = threadIdx.x, lane = j & 63, wv = j >> 6;
  for (int q = j; q < NW; q += 1024) w[q] = q;
  __syncthreads();
  uint32_t addr[ITER];
#pragma unroll
  for (int i = 0; i < ITER; i++) {
    const uint32_t r = rnd(j * 7919u + i * 104729u + 17u);
    switch (mode) {
      case 2: addr[i] = rnd(wv * 131u + i * 7u + (lane & 7)) % NW; break;
      case 3: addr[i] = rnd(wv * 131u + i * 7u) % NW; break;
      case 4: addr[i] = (rnd(wv * 131u + i * 7u) % (NW / 2)) * 2 + (lane >> 5); break;
      case 6: addr[i] = (rnd(wv * 131u + i * 7u) % (NW * 4 - 64)) & ~63u; break;
      case 7: addr[i] = 5; break;
      default: addr[i] = r % NW;
    }
  }
  __syncthreads();
  const uint64_t t0 = __builtin_amdgcn_s_memtime();
  uint32_t acc = 0;
#pragma unroll
  for (int i = 0; i < ITER; i++) {
    switch (mode) {
      case 0:
      case 7: acc += w[addr[i]]; break;
      case 1:
      case 2:
      case 3: atomicMin(&w[addr[i]], j + i); break;
      case 4: atomicOr(&w[addr[i]], 1u << (lane & 31)); break;
      case 5: ((uint8_t*)w)[(addr[i] * 4 + (lane & 3)) % (NW * 4)] = (uint8_t)i; break;
      case 6: ((uint8_t*)w)[addr[i] + lane] = (uint8_t)i; break;
      case 8: if (lane & 1) atomicMin(&w[addr[i]], j + i); break;
    }
  }
  __builtin_amdgcn_s_waitcnt(0);
  __syncthreads();
  const uint64_t t1 = __builtin_amdgcn_s_memtime();
  if (j == 0) out[mode] = t1 - t0;
  if (acc == 0xdeadbeef) sink[0] = acc;
}

int main() {
  uint64_t* out;
  uint32_t* sink;
  hipMalloc(&out, 16 * 8);
  hipMalloc(&sink, 64);
  const char* name[] = {"read random", "atomicMin random", "atomicMin 8 addr/wave", "atomicMin 1 addr/wave",
                        "atomicOr 1 word/32 lanes", "byte store random", "byte store 64 consecutive",
                        "read same address", "atomicMin random, half lanes"};
  for (int rep = 0; rep < 2; rep++)
    for (int m = 0; m < 9; m++) {
      k_lds<<<1, 1024>>>(m, out, sink);
      hipDeviceSynchronize();
      uint64_t c;
      hipMemcpy(&c, out + m, 8, hipMemcpyDeviceToHost);
      if (rep) printf("%-30s %8.1f cycles per wave-instruction (16 waves x %d)\n", name[m], (double)c / (16.0 * ITER), ITER);
    }
  return 0;
}
