// Where do a CU-masked stream's workgroups run?  (measurement aid)
//
// Launches a grid on streams created with hipExtStreamCreateWithCUMask and
// records, per workgroup, the XCD (HW_REG_XCC_ID) and the CU within it
// (HW_REG_HW_ID: SE, SH, CU fields); prints per mask the XCDs used and the
// distinct CUs.  Used to map mask bits to XCDs before giving each pipeline
// lane its own XCD (occ_pipe.cpp).
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>

#include <cstdio>
#include <set>
#include <vector>

__global__ void k_where(uint32_t* out, uint32_t spin) {
  uint32_t hw, xcc;
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
  const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
  while (__builtin_amdgcn_s_memrealtime() - t0 < spin) __builtin_amdgcn_s_sleep(4);
  if (threadIdx.x == 0) {
    out[2 * blockIdx.x] = xcc & 0xF;
    out[2 * blockIdx.x + 1] = hw;
  }
}

int main() {
  const int G = 4096;
  uint32_t* d;
  if (hipMalloc(&d, G * 8) != hipSuccess) return 1;
  std::vector<uint32_t> h(2 * G);
  struct M {
    const char* name;
    std::vector<uint32_t> m;
  };
  std::vector<M> masks;
  auto bits = [](auto pred) {
    std::vector<uint32_t> m(8, 0);
    for (int i = 0; i < 256; i++)
      if (pred(i)) m[i / 32] |= 1u << (i % 32);
    return m;
  };
  masks.push_back({"all", bits([](int) { return true; })});
  masks.push_back({"bits 0-31", bits([](int i) { return i < 32; })});
  masks.push_back({"bits i%8==0", bits([](int i) { return i % 8 == 0; })});
  masks.push_back({"bits i%8==3", bits([](int i) { return i % 8 == 3; })});
  masks.push_back({"bits 0-63", bits([](int i) { return i < 64; })});
  masks.push_back({"bits 224-255", bits([](int i) { return i >= 224; })});
  masks.push_back({"bit 5", bits([](int i) { return i == 5; })});
  for (auto& mk : masks) {
    hipStream_t s;
    if (hipExtStreamCreateWithCUMask(&s, 8, mk.m.data()) != hipSuccess) {
      printf("%s: hipExtStreamCreateWithCUMask failed\n", mk.name);
      continue;
    }
    hipMemsetAsync(d, 0xFF, G * 8, s);
    k_where<<<G, 64, 0, s>>>(d, 200);  // 2 us each
    hipStreamSynchronize(s);
    hipMemcpy(h.data(), d, G * 8, hipMemcpyDeviceToHost);
    int per_xcc[16] = {0};
    std::set<uint32_t> cus;
    for (int b = 0; b < G; b++) {
      const uint32_t x = h[2 * b], hw = h[2 * b + 1];
      per_xcc[x & 15]++;
      // SE 15:13, SH 12, CU 11:8
      cus.insert((x << 16) | (((hw >> 13) & 7) << 8) | (((hw >> 12) & 1) << 4) | ((hw >> 8) & 15));
    }
    printf("%-14s xcc:", mk.name);
    for (int x = 0; x < 8; x++) printf(" %4d", per_xcc[x]);
    printf("  distinct CUs %zu  first:", cus.size());
    int k = 0;
    for (uint32_t c : cus) {
      if (k++ == 6) break;
      printf(" x%u/se%u/sh%u/cu%u", c >> 16, (c >> 8) & 7, (c >> 4) & 1, c & 15);
    }
    printf("\n");
    hipStreamDestroy(s);
  }
  return 0;
}
