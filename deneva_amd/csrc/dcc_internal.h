// Host-side internals shared by libdcc translation units (not part of the ABI).
#pragma once
#include <algorithm>
#include <atomic>
#include <cstdint>
#include <thread>
#include <vector>

namespace dcc {

// myrand, system/helper.cpp:140-147:
//   seed = (seed * 1103515247 + 12345) % 2^63;  return (seed / 65537) % RAND_MAX
// (u64 wrap-around before the modulus; RAND_MAX = 2^31-1 on glibc).
struct MyRand {
  uint64_t seed = 0;
  void init(uint64_t s) { seed = s; }
  uint64_t next() {
    seed = (seed * 1103515247ull + 12345ull) % (1ull << 63);
    return (seed / 65537) % 2147483647ull;
  }
};

inline uint64_t splitmix64(uint64_t x) {
  x += 0x9E3779B97F4A7C15ull;
  x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
  x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
  return x ^ (x >> 31);
}

// Per-chunk generator stream seed.
inline uint64_t chunk_seed(uint64_t seed, uint64_t chunk) {
  return splitmix64(seed ^ splitmix64(chunk + 1));
}

double zeta_cached(uint64_t n, double theta);

inline unsigned host_threads(unsigned requested) {
  if (requested) return requested;
  unsigned hc = std::thread::hardware_concurrency();
  if (hc == 0) hc = 1;
  return std::min(hc, 16u);  // the GPU box grants 16 cores per GPU
}

template <class F>
void parallel_for(uint64_t n, unsigned threads, F&& f) {
  threads = host_threads(threads);
  if (n == 0) return;
  if (threads <= 1 || n == 1) {
    for (uint64_t i = 0; i < n; i++) f(i);
    return;
  }
  std::atomic<uint64_t> next{0};
  std::vector<std::thread> pool;
  const unsigned nt = (unsigned)std::min<uint64_t>(threads, n);
  for (unsigned t = 0; t < nt; t++)
    pool.emplace_back([&] {
      for (uint64_t i; (i = next.fetch_add(1)) < n;) f(i);
    });
  for (auto& th : pool) th.join();
}

}  // namespace dcc
