// gfx950 stable LSD radix sort of (key, u32 value) pairs — see radix_sort.h.
#include <hip/hip_runtime.h>

#include <cstdlib>

#include "dcc_device.h"
#include "dcc_env.h"
#include "radix_sort.h"

namespace dcc {

// Lanes of the wave whose 8-bit digit equals this lane's (8 ballots).
__device__ inline uint64_t digit_peers(uint32_t d, bool act) {
  uint64_t m = ballot64(act);
#pragma unroll
  for (int b = 0; b < 8; b++) {
    const uint64_t bb = ballot64((d >> b) & 1u);
    m &= ((d >> b) & 1u) ? bb : ~bb;
  }
  return act ? m : 0ull;
}

__device__ inline uint64_t lanemask_lt() {
  const uint32_t l = lane_id();
  return l == 0 ? 0ull : (~0ull >> (64 - l));
}

constexpr uint32_t RS_W = RS_THREADS / 64;  // waves per workgroup
static_assert(RS_THREADS >= 256, "one thread per digit");

// Exclusive scan of one u32 per thread over the workgroup.
__device__ inline uint32_t block_excl_scan(uint32_t v, uint32_t* sh /*[RS_W]*/, uint32_t& total) {
  const uint32_t lane = lane_id(), wv = threadIdx.x >> 6;
  uint32_t x = v;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const uint32_t y = __shfl_up(x, d);
    if (lane >= (uint32_t)d) x += y;
  }
  __syncthreads();
  if (lane == 63) sh[wv] = x;
  __syncthreads();
  uint32_t off = 0;
  total = 0;
#pragma unroll
  for (uint32_t w = 0; w < RS_W; w++) {
    if (w < wv) off += sh[w];
    total += sh[w];
  }
  return off + x - v;
}

// Per-tile digit counts: one LDS histogram per wave, summed at the end.
// Thread t counts the tile's items [16t, 16t + 16) (16-B loads): a run of
// equal digits -- a hot row's requests are adjacent once the lower digits
// are sorted -- costs one LDS atomic, not one per item (the skewed top-digit
// pass of a YCSB key sort took 34 us with an atomic per item, the others
// ~16-19; adding once per digit per wave instruction, via digit_peers, 41).
template <typename K, uint32_t IT>
__global__ __launch_bounds__(RS_THREADS) void k_rs_hist(const K* __restrict__ keys, uint64_t m,
                                                        uint32_t shift, uint32_t* __restrict__ cnt,
                                                        uint32_t tiles) {
  constexpr uint32_t W = RS_W;
  constexpr uint32_t V = 16 / sizeof(K);  // keys per 16-B load
  __shared__ uint32_t s_h[W][256];
  const uint32_t wv = threadIdx.x >> 6;
  for (uint32_t q = threadIdx.x; q < W * 256; q += RS_THREADS) (&s_h[0][0])[q] = 0;
  __syncthreads();
  const uint64_t p0 = (uint64_t)blockIdx.x * (RS_THREADS * IT) + (uint64_t)threadIdx.x * IT;
  K k[IT];
  if (p0 + IT <= m && ((uintptr_t)(keys + p0) & 15) == 0) {
#pragma unroll
    for (uint32_t q = 0; q < IT / V; q++) {
      const uint4 x = ((const uint4*)(keys + p0))[q];
      const K* xk = (const K*)&x;
#pragma unroll
      for (uint32_t i = 0; i < V; i++) k[q * V + i] = xk[i];
    }
  } else {
#pragma unroll
    for (uint32_t i = 0; i < IT; i++) k[i] = p0 + i < m ? keys[p0 + i] : (K)0;
  }
  const uint32_t n = p0 >= m ? 0u : (uint32_t)min<uint64_t>(IT, m - p0);
  uint32_t run_d = (uint32_t)(k[0] >> shift) & 255u, run_n = 0;
#pragma unroll
  for (uint32_t i = 0; i < IT; i++) {
    const uint32_t d = (uint32_t)(k[i] >> shift) & 255u;
    if (i < n) {
      if (d != run_d) {
        if (run_n) atomicAdd(&s_h[wv][run_d], run_n);
        run_d = d;
        run_n = 0;
      }
      run_n++;
    }
  }
  if (run_n) atomicAdd(&s_h[wv][run_d], run_n);
  __syncthreads();
  if (threadIdx.x < 256) {
    uint32_t c = 0;
#pragma unroll
    for (uint32_t w = 0; w < W; w++) c += s_h[w][threadIdx.x];
    cnt[(uint64_t)threadIdx.x * tiles + blockIdx.x] = c;
  }
}

// One workgroup per digit: exclusive scan of cnt[d][0..tiles) in place,
// digit total to tot[d].
__global__ __launch_bounds__(RS_THREADS) void k_rs_scan(uint32_t* __restrict__ cnt, uint32_t tiles,
                                                        uint32_t* __restrict__ tot) {
  __shared__ uint32_t sh[RS_W];
  uint32_t* row = cnt + (uint64_t)blockIdx.x * tiles;
  uint32_t run = 0;
  for (uint32_t c0 = 0; c0 < tiles; c0 += RS_THREADS * 4) {
    uint32_t v[4], s = 0;
#pragma unroll
    for (int q = 0; q < 4; q++) {
      const uint32_t i = c0 + threadIdx.x * 4 + q;
      v[q] = i < tiles ? row[i] : 0u;
      s += v[q];
    }
    uint32_t total;
    uint32_t pre = run + block_excl_scan(s, sh, total);
#pragma unroll
    for (int q = 0; q < 4; q++) {
      const uint32_t i = c0 + threadIdx.x * 4 + q;
      if (i < tiles) row[i] = pre;
      pre += v[q];
    }
    run += total;
  }
  if (threadIdx.x == 0) tot[blockIdx.x] = run;
}

// Stable scatter of one tile.  Wave w owns the tile's items
// [w * 1024, w * 1024 + 1024) (item it of lane l at w * 1024 + 64 it + l), so
// position order is (wave, round, lane): each wave ranks its own items with a
// running per-digit count in its own LDS row -- no workgroup barrier per
// round (a wave's LDS operations execute in order) -- and the waves' counts
// are combined once.  Then the tile is staged in LDS in digit order and
// written out with coalesced runs per digit.
template <typename K, uint32_t IT>
__global__ __launch_bounds__(RS_THREADS) void k_rs_scatter(const K* __restrict__ kin,
                                                           const uint32_t* __restrict__ vin,
                                                           K* __restrict__ kout,
                                                           uint32_t* __restrict__ vout, uint64_t m,
                                                           uint32_t shift,
                                                           const uint32_t* __restrict__ cnt,
                                                           const uint32_t* __restrict__ tot,
                                                           uint32_t tiles) {
  constexpr uint32_t TILE = RS_THREADS * IT;
  constexpr uint32_t W = RS_W, WI = TILE / W;  // waves, items per wave
  __shared__ K s_key[TILE];
  __shared__ uint32_t s_val[TILE];
  __shared__ uint32_t s_wc[W][256];  // per wave: running digit count, then its base in the tile
  __shared__ uint32_t s_gb[256];     // global destination base per digit
  __shared__ uint32_t s_tb[256];     // tile-local base per digit
  __shared__ uint32_t sh[RS_W];
  const uint32_t tid = threadIdx.x, lane = lane_id(), wv = tid >> 6;
  const bool dig = tid < 256;  // this thread owns digit tid
  const uint64_t base = (uint64_t)blockIdx.x * TILE;
  const uint64_t wbase = base + (uint64_t)wv * WI;

  K k[IT];
  uint32_t v[IT];
#pragma unroll
  for (uint32_t it = 0; it < IT; it++) {
    const uint64_t p = wbase + it * 64 + lane;
    k[it] = p < m ? kin[p] : (K)0;
    v[it] = p < m ? vin[p] : 0u;
  }
  {
    uint32_t total;
    const uint32_t g = block_excl_scan(dig ? tot[tid] : 0u, sh, total);
    if (dig) s_gb[tid] = g + cnt[(uint64_t)tid * tiles + blockIdx.x];
  }
  for (uint32_t q = tid; q < W * 256; q += RS_THREADS) (&s_wc[0][0])[q] = 0;
  __syncthreads();

  const uint64_t lt = lanemask_lt();
  uint32_t loc[IT];
  uint32_t* wc = s_wc[wv];
#pragma unroll
  for (uint32_t it = 0; it < IT; it++) {
    const uint64_t p = wbase + it * 64 + lane;
    const bool act = p < m;
    const uint32_t d = (uint32_t)(k[it] >> shift) & 255u;
    const uint64_t peers = digit_peers(d, act);
    const uint32_t lr = (uint32_t)__builtin_popcountll(peers & lt);
    const uint32_t before = wc[d];
    loc[it] = before + lr;
    // the digit's first lane advances the count; the read above and this
    // write are the same wave's, in order
    if (act && lr == 0) wc[d] = before + (uint32_t)__builtin_popcountll(peers);
  }
  __syncthreads();
  {
    uint32_t c[W], t = 0;
#pragma unroll
    for (uint32_t w = 0; w < W; w++) {
      c[w] = dig ? s_wc[w][tid] : 0u;
      t += c[w];
    }
    uint32_t total;
    uint32_t b = block_excl_scan(t, sh, total);
    __syncthreads();  // every wave's counts read before they become bases
    if (dig) {
      s_tb[tid] = b;
#pragma unroll
      for (uint32_t w = 0; w < W; w++) {
        s_wc[w][tid] = b;
        b += c[w];
      }
    }
  }
  __syncthreads();
#pragma unroll
  for (uint32_t it = 0; it < IT; it++) {
    const uint64_t p = wbase + it * 64 + lane;
    if (p < m) {
      const uint32_t d = (uint32_t)(k[it] >> shift) & 255u;
      const uint32_t pos = wc[d] + loc[it];
      s_key[pos] = k[it];
      s_val[pos] = v[it];
    }
  }
  __syncthreads();
  const uint32_t n_here = (uint32_t)min<uint64_t>(TILE, m - base);
  for (uint32_t j = tid; j < n_here; j += RS_THREADS) {
    const K kk = s_key[j];
    const uint32_t d = (uint32_t)(kk >> shift) & 255u;
    const uint64_t dst = (uint64_t)s_gb[d] + (j - s_tb[d]);
    kout[dst] = kk;
    vout[dst] = s_val[j];
  }
}

template <typename K, uint32_t IT>
static int radix_sort_run(K* k[2], uint32_t* v[2], uint64_t m, uint32_t bits, uint32_t* scratch,
                          hipStream_t st) {
  int cur = 0;
  const uint32_t tiles = (uint32_t)((m + RS_THREADS * IT - 1) / (RS_THREADS * IT));
  uint32_t* cnt = scratch;
  uint32_t* tot = scratch + 256ull * tiles;
  for (uint32_t shift = 0; shift < bits; shift += 8) {
    k_rs_hist<K, IT><<<tiles, RS_THREADS, 0, st>>>(k[cur], m, shift, cnt, tiles);
    k_rs_scan<<<256, RS_THREADS, 0, st>>>(cnt, tiles, tot);
    k_rs_scatter<K, IT><<<tiles, RS_THREADS, 0, st>>>(k[cur], v[cur], k[cur ^ 1], v[cur ^ 1], m, shift,
                                                      cnt, tot, tiles);
    cur ^= 1;
  }
  return cur;
}
// small sorts (the Calvin rank of 1M orders, index builds) take 2,048-pair
// tiles: four times the workgroups of the 8,192-pair tiles, each with a
// quarter of the latency-bound chain
template <typename K>
static int radix_sort_impl(K* k[2], uint32_t* v[2], uint64_t m, uint32_t bits, uint32_t* scratch,
                           hipStream_t st) {
  if (m <= 1 || bits == 0) return 0;
  static const bool small_on = [] {  // DCC_RS_SMALL=0: 8,192-pair tiles at every size (A/B)
    const char* e = DCC_ENV("DCC_RS_SMALL");
    return !(e && e[0] == '0');
  }();
  if (small_on && m <= RS_SMALL) return radix_sort_run<K, RS_ITEMS_SMALL>(k, v, m, bits, scratch, st);
  return radix_sort_run<K, RS_ITEMS>(k, v, m, bits, scratch, st);
}

int radix_sort_u32(uint32_t* k[2], uint32_t* v[2], uint64_t m, uint32_t bits, uint32_t* scratch,
                   hipStream_t st) {
  return radix_sort_impl<uint32_t>(k, v, m, bits > 32 ? 32 : bits, scratch, st);
}
int radix_sort_u64(uint64_t* k[2], uint32_t* v[2], uint64_t m, uint32_t bits, uint32_t* scratch,
                   hipStream_t st) {
  return radix_sort_impl<uint64_t>(k, v, m, bits > 64 ? 64 : bits, scratch, st);
}

void rs_scan_one(uint32_t* row, uint32_t len, uint32_t* total, hipStream_t st) {
  k_rs_scan<<<1, RS_THREADS, 0, st>>>(row, len, total);
}
void rs_scan_rows(uint32_t* cnt, uint32_t rows, uint32_t len, uint32_t* tot, hipStream_t st) {
  k_rs_scan<<<rows, RS_THREADS, 0, st>>>(cnt, len, tot);
}

KeyPack make_keypack(uint64_t varying) {
  KeyPack p{};
  uint32_t dst = 0;
  for (uint32_t b = 0; b < 64;) {
    if (!((varying >> b) & 1ull)) {
      b++;
      continue;
    }
    uint32_t w = 0;
    while (b + w < 64 && ((varying >> (b + w)) & 1ull)) w++;
    p.src[p.nruns] = (uint8_t)b;
    p.width[p.nruns] = (uint8_t)w;
    p.dst[p.nruns] = (uint8_t)dst;
    p.nruns++;
    dst += w;
    b += w;
  }
  p.bits = dst;
  return p;
}

}  // namespace dcc
