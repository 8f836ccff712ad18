// Device-resident OCC history: append, level build, trim (occ_history.h).
//
// Reference: central_finish pushes every committed write set onto `history`
// with tn = ++tnc (concurrency_control/occ.cpp:277-286); central_validate
// scans the entries with start_tn < tn <= finish_tn against the read set
// (occ.cpp:160-180).  Here an epoch's committed writes are appended on the
// device in index (= tn) order and the per-key tn runs are rebuilt by a
// stable radix sort, so the host never copies the batch back.
#include <hip/hip_runtime.h>

#include <algorithm>

#include "dcc_device.h"
#include "occ_history.h"
#include "occ_kernels.h"
#include "radix_sort.h"

namespace dcc {

constexpr uint32_t HB = 1024;  // txns per block of the append kernels
constexpr uint32_t FIN_INSERT_WG = 512;  // k_fin_insert: the grid walks the appended pairs

// committed writes of txn t (0 when it did not commit or is read-only)
__device__ inline uint32_t hist_writes_of(uint64_t t, const uint32_t* off, const uint8_t* acctype,
                                          uint64_t nnz, const uint64_t* tn, uint32_t& a0) {
  a0 = 0;
  if (!tn[t]) return 0;
  const uint64_t o0 = min((uint64_t)off[t], nnz), o1 = min((uint64_t)off[t + 1], nnz);
  if (o1 <= o0) return 0;
  a0 = (uint32_t)o0;
  uint32_t c = 0;
  for (uint64_t x = o0; x < o1 && x < o0 + MAX_TXN_LEN; x++) c += acctype[x] == DCC_WR;
  return c;
}

// exclusive scan over the block (1024 threads = 16 waves); returns the block total
__device__ inline uint32_t block_excl_scan1024(uint32_t v, uint32_t& excl) {
  __shared__ uint32_t s_w[HB / 64];
  const uint32_t lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  uint32_t x = v;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const uint32_t y = __shfl_up(x, d);
    if (lane >= (uint32_t)d) x += y;
  }
  if (lane == 63) s_w[w] = x;
  __syncthreads();
  uint32_t before = 0, total = 0;
#pragma unroll
  for (uint32_t q = 0; q < HB / 64; q++) {
    const uint32_t s = s_w[q];
    if (q < w) before += s;
    total += s;
  }
  excl = before + x - v;
  return total;
}

__global__ __launch_bounds__(HB) void k_hist_count(uint64_t n, const uint32_t* off,
                                                   const uint8_t* acctype, uint64_t nnz,
                                                   const uint64_t* tn, uint32_t* bsum) {
  const uint64_t t = (uint64_t)blockIdx.x * HB + threadIdx.x;
  uint32_t a0;
  const uint32_t c = t < n ? hist_writes_of(t, off, acctype, nnz, tn, a0) : 0u;
  uint32_t ex;
  const uint32_t tot = block_excl_scan1024(c, ex);
  if (threadIdx.x == 0) bsum[blockIdx.x] = tot;
}

__global__ __launch_bounds__(HB) void k_hist_emit(uint64_t n, const uint32_t* off,
                                                  const uint64_t* keys, const uint8_t* acctype,
                                                  uint64_t nnz, const uint64_t* tn,
                                                  const uint32_t* bsum, uint64_t* out_k,
                                                  uint64_t* out_t, unsigned long long* kmax) {
  __shared__ unsigned long long s_mx;
  const uint64_t t = (uint64_t)blockIdx.x * HB + threadIdx.x;
  uint32_t a0 = 0;
  const uint32_t c = t < n ? hist_writes_of(t, off, acctype, nnz, tn, a0) : 0u;
  uint32_t ex;
  (void)block_excl_scan1024(c, ex);
  if (threadIdx.x == 0) s_mx = 0;
  __syncthreads();
  uint64_t mx = 0;
  if (c) {
    uint64_t p = (uint64_t)bsum[blockIdx.x] + ex;
    const uint64_t my_tn = tn[t];
    for (uint64_t x = a0; p < (uint64_t)bsum[blockIdx.x] + ex + c; x++) {
      if (acctype[x] != DCC_WR) continue;
      const uint64_t k = keys[x];
      out_k[p] = k;
      out_t[p] = my_tn;
      mx = max(mx, k);
      p++;
    }
  }
  for (int d = 32; d > 0; d >>= 1) mx = max(mx, (uint64_t)__shfl_xor(mx, d));
  if ((threadIdx.x & 63) == 0 && mx) atomicMax(&s_mx, (unsigned long long)mx);
  __syncthreads();
  if (threadIdx.x == 0 && s_mx) atomicMax(kmax, s_mx);  // one per workgroup
}

// ---------------------------------------------------------------------------
// central_finish in three launches (OccFinArgs, occ_kernels.h).  Per 1024-txn
// block: the committed writers (cflag) and, when appending, their writes and
// largest key; one workgroup scans the block counts from dyn->tnc and
// dyn->hist_m; then each committed writer takes its tn and emits its write set
// at its position.  Only committed writers (a few per thousand under
// contention) read their access lists.
__device__ inline uint32_t fin_writes(uint64_t t, const OccFinArgs& a, uint64_t& o0, uint64_t& o1,
                                      uint64_t& kmx) {
  o0 = min((uint64_t)a.off[t], a.nnz);
  o1 = min((uint64_t)a.off[t + 1], a.nnz);
  if (o1 < o0) o1 = o0;
  o1 = min(o1, o0 + MAX_TXN_LEN);
  uint32_t c = 0;
  for (uint64_t x = o0; x < o1; x++)
    if (a.acctype[x] == DCC_WR) {
      c++;
      kmx = max(kmx, a.keys[x]);
    }
  return c;
}

// block-wide exclusive scans of two counters (1024 threads); returns both totals
__device__ inline void block_excl_scan2(uint32_t v0, uint32_t v1, uint32_t& e0, uint32_t& e1,
                                        uint32_t& t0, uint32_t& t1) {
  __shared__ uint32_t s_w[2][HB / 64];
  const uint32_t lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  uint32_t x0 = v0, x1 = v1;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const uint32_t y0 = __shfl_up(x0, d), y1 = __shfl_up(x1, d);
    if (lane >= (uint32_t)d) {
      x0 += y0;
      x1 += y1;
    }
  }
  if (lane == 63) {
    s_w[0][w] = x0;
    s_w[1][w] = x1;
  }
  __syncthreads();
  uint32_t b0 = 0, b1 = 0;
  t0 = t1 = 0;
#pragma unroll
  for (uint32_t q = 0; q < HB / 64; q++) {
    if (q < w) {
      b0 += s_w[0][q];
      b1 += s_w[1][q];
    }
    t0 += s_w[0][q];
    t1 += s_w[1][q];
  }
  e0 = b0 + x0 - v0;
  e1 = b1 + x1 - v1;
}

__global__ __launch_bounds__(HB) void k_fin_count(OccFinArgs a) {
  __shared__ unsigned long long s_mx;
  const uint64_t t = (uint64_t)blockIdx.x * HB + threadIdx.x;
  const bool app = a.dyn->app_k != nullptr;
  const uint32_t c = (t < a.n && a.cflag[t]) ? 1u : 0u;
  uint64_t o0, o1, kmx = 0;
  const uint32_t w = (c && app) ? fin_writes(t, a, o0, o1, kmx) : 0u;
  if (threadIdx.x == 0) s_mx = 0;
  uint32_t e0, e1, t0, t1;
  block_excl_scan2(c, w, e0, e1, t0, t1);  // its barrier orders s_mx's reset
  for (int d = 32; d > 0; d >>= 1) kmx = max(kmx, (uint64_t)__shfl_xor(kmx, d));
  if ((threadIdx.x & 63) == 0 && kmx) atomicMax(&s_mx, (unsigned long long)kmx);
  __syncthreads();
  if (threadIdx.x == 0) {
    a.part[3 * blockIdx.x] = t0;
    a.part[3 * blockIdx.x + 1] = t1;
    a.part[3 * blockIdx.x + 2] = s_mx;
  }
}

// exclusive scans of the block counts from dyn->tnc / dyn->hist_m (one
// workgroup, 1024 blocks per step), totals to pinned memory
__global__ __launch_bounds__(1024) void k_fin_sums(OccFinArgs a, uint64_t nb) {
  __shared__ uint64_t s_w[2][16];
  __shared__ uint64_t s_carry[2];
  __shared__ unsigned long long s_mx;
  const uint32_t lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  if (threadIdx.x == 0) {
    s_carry[0] = a.dyn->tnc;
    s_carry[1] = a.dyn->hist_m;
    s_mx = 0;
  }
  __syncthreads();
  const uint64_t c0_base = s_carry[0], c1_base = s_carry[1];
  uint64_t mx = 0;
  for (uint64_t c0 = 0; c0 < nb; c0 += 1024) {
    const uint64_t q = c0 + threadIdx.x;
    const uint64_t v0 = q < nb ? a.part[3 * q] : 0ull, v1 = q < nb ? a.part[3 * q + 1] : 0ull;
    if (q < nb) mx = max(mx, a.part[3 * q + 2]);
    uint64_t x0 = v0, x1 = v1;
    for (int d = 1; d < 64; d <<= 1) {
      const uint64_t y0 = __shfl_up(x0, d), y1 = __shfl_up(x1, d);
      if (lane >= (uint32_t)d) {
        x0 += y0;
        x1 += y1;
      }
    }
    if (lane == 63) {
      s_w[0][wv] = x0;
      s_w[1][wv] = x1;
    }
    __syncthreads();
    uint64_t b0 = s_carry[0], b1 = s_carry[1];
    for (uint32_t w = 0; w < wv; w++) {
      b0 += s_w[0][w];
      b1 += s_w[1][w];
    }
    if (q < nb) {
      a.part[3 * q] = b0 + x0 - v0;
      a.part[3 * q + 1] = b1 + x1 - v1;
    }
    __syncthreads();
    if (threadIdx.x == 1023) {
      s_carry[0] = b0 + x0;
      s_carry[1] = b1 + x1;
    }
    __syncthreads();
  }
  for (int d = 32; d > 0; d >>= 1) mx = max(mx, (uint64_t)__shfl_xor(mx, d));
  if (lane == 0 && mx) atomicMax(&s_mx, (unsigned long long)mx);
  __syncthreads();
  if (threadIdx.x == 0) {
    a.totals[0] = s_carry[0] - c0_base;
    a.totals[1] = s_carry[1] - c1_base;
    a.totals[2] = s_mx;
    a.part[3 * nb + 1] = s_carry[1] - c1_base;  // the appended count, for k_fin_insert
  }
}

__global__ __launch_bounds__(HB) void k_fin_apply(OccFinArgs a) {
  const uint64_t t = (uint64_t)blockIdx.x * HB + threadIdx.x;
  uint64_t* app_k = a.dyn->app_k;
  const uint32_t c = (t < a.n && a.cflag[t]) ? 1u : 0u;
  uint64_t o0 = 0, o1 = 0, kmx = 0;
  const uint32_t w = (c && app_k) ? fin_writes(t, a, o0, o1, kmx) : 0u;
  uint32_t e0, e1, t0, t1;
  block_excl_scan2(c, w, e0, e1, t0, t1);
  if (t >= a.n) return;
  const uint64_t my_tn = c ? a.part[3 * blockIdx.x] + e0 + 1 : 0;
  a.tn[t] = my_tn;
  if (w) {
    uint64_t* app_t = a.dyn->app_t;
    uint64_t p = a.part[3 * blockIdx.x + 1] + e1;
    for (uint64_t x = o0; x < o1; x++)
      if (a.acctype[x] == DCC_WR) {
        app_k[p] = a.keys[x];
        app_t[p] = my_tn;
        p++;
      }
  }
}

// the appended pairs into the delta's table (a thread per pair), then its
// overflow flag to pinned memory by the last workgroup to finish
__global__ __launch_bounds__(256) void k_fin_insert(OccFinArgs a, uint64_t nb) {
  const HistInsert ins = a.dyn->ins;
  if (!ins.hash) {
    if (blockIdx.x == 0 && threadIdx.x == 0) a.totals[3] = 0;
    return;
  }
  const uint64_t p0 = a.dyn->hist_m, cnt = a.part[3 * nb + 1];
  for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < cnt; i += (uint64_t)gridDim.x * 256)
    hist_insert(ins, p0 + i, ins.fk[p0 + i], ins.ft[p0 + i]);
  __shared__ bool s_last;
  __syncthreads();
  if (threadIdx.x == 0) {
    __threadfence();
    s_last = atomicAdd(&ins.over[1], 1u) == gridDim.x - 1;
  }
  __syncthreads();
  if (s_last && threadIdx.x == 0) {
    __threadfence();
    a.totals[3] = atomicAdd(&ins.over[0], 0u);
    ins.over[1] = 0;  // ready for the next epoch
  }
}

void launch_fin(const OccFinArgs& a, hipStream_t st) {
  const uint64_t nb = (a.n + HB - 1) / HB;
  const unsigned g = (unsigned)(nb ? nb : 1);
  k_fin_count<<<g, HB, 0, st>>>(a);
  k_fin_sums<<<1, 1024, 0, st>>>(a, nb);
  k_fin_apply<<<g, HB, 0, st>>>(a);
  k_fin_insert<<<FIN_INSERT_WG, 256, 0, st>>>(a, nb);
}

__global__ __launch_bounds__(256) void k_hist_insert(HistInsert h, uint64_t from, uint64_t to) {
  for (uint64_t p = from + (uint64_t)blockIdx.x * 256 + threadIdx.x; p < to; p += (uint64_t)gridDim.x * 256)
    hist_insert(h, p, h.fk[p], h.ft[p]);
}
void launch_hist_insert(const HistInsert& h, uint64_t from, uint64_t to, hipStream_t st) {
  if (to <= from) return;
  const uint64_t g = std::min<uint64_t>((to - from + 255) / 256, 4096);
  k_hist_insert<<<(unsigned)g, 256, 0, st>>>(h, from, to);
}

void launch_hist_count(uint64_t n, const uint32_t* off, const uint8_t* acctype, uint64_t nnz,
                       const uint64_t* tn, uint32_t* bsum, hipStream_t st) {
  const unsigned g = (unsigned)((n + HB - 1) / HB);
  k_hist_count<<<g ? g : 1, HB, 0, st>>>(n, off, acctype, nnz, tn, bsum);
}
void launch_hist_emit(uint64_t n, const uint32_t* off, const uint64_t* keys, const uint8_t* acctype,
                      uint64_t nnz, const uint64_t* tn, const uint32_t* bsum, uint64_t* out_k,
                      uint64_t* out_t, unsigned long long* kmax, hipStream_t st) {
  const unsigned g = (unsigned)((n + HB - 1) / HB);
  k_hist_emit<<<g ? g : 1, HB, 0, st>>>(n, off, keys, acctype, nnz, tn, bsum, out_k, out_t, kmax);
}

// ---------------------------------------------------------------- level build
__global__ __launch_bounds__(256) void k_hist_init(const uint64_t* src, uint64_t m, uint64_t* k,
                                                   uint32_t* v) {
  for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < m; i += (uint64_t)gridDim.x * 256) {
    k[i] = src[i];
    v[i] = (uint32_t)i;
  }
}
// second key of a two-pass sort: k[i] = fk[perm[i]], v[i] = perm[i]
__global__ __launch_bounds__(256) void k_hist_regather(const uint64_t* fk, const uint32_t* perm,
                                                       uint64_t m, uint64_t* k, uint32_t* v) {
  for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < m; i += (uint64_t)gridDim.x * 256) {
    const uint32_t p = perm[i];
    k[i] = fk[p];
    v[i] = p;
  }
}
__global__ __launch_bounds__(256) void k_hist_gather(const uint64_t* sk, const uint32_t* perm,
                                                     const uint64_t* ft, uint64_t m, uint64_t* skey,
                                                     uint64_t* stn) {
  for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < m; i += (uint64_t)gridDim.x * 256) {
    skey[i] = sk[i];
    stn[i] = ft[perm[i]];
  }
}
// the first pair of each key's run enters the table: (key, first)
__global__ __launch_bounds__(256) void k_hist_heads(const uint64_t* skey, uint64_t m,
                                                    uint64_t* hash, uint32_t hbits) {
  const uint64_t mask = (1ull << hbits) - 1;
  uint64_t* side = hash + (2ull << hbits);
  for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < m; i += (uint64_t)gridDim.x * 256) {
    const uint64_t key = skey[i];
    if (i > 0 && skey[i - 1] == key) continue;
    uint64_t s = hist_hash_slot(key, hbits);
    for (;;) {
      const unsigned long long prev = atomicCAS((unsigned long long*)&hash[2 * s],
                                                (unsigned long long)DCC_KEY_RESERVED,
                                                (unsigned long long)key);
      if (prev == DCC_KEY_RESERVED) break;
      s = (s + 1) & mask;  // keys are unique here: a taken slot is another key's
    }
    side[2 * s] = i;
  }
}
// the last pair of each run completes its slot: count = last + 1 - first,
// and the run's tn range
__global__ __launch_bounds__(256) void k_hist_tails(const uint64_t* skey, const uint64_t* stn, uint64_t m,
                                                    uint64_t* hash, uint32_t hbits) {
  const uint64_t mask = (1ull << hbits) - 1;
  uint64_t* side = hash + (2ull << hbits);
  for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < m; i += (uint64_t)gridDim.x * 256) {
    const uint64_t key = skey[i];
    if (i + 1 < m && skey[i + 1] == key) continue;
    uint64_t s = hist_hash_slot(key, hbits);
    while (hash[2 * s] != key) s = (s + 1) & mask;
    const uint64_t first = side[2 * s];
    side[2 * s] = first | ((i + 1 - first) << 32);
    side[2 * s + 1] = stn[first];
    hash[2 * s + 1] = ~stn[i];
  }
}

static unsigned hgrid(uint64_t m) {
  uint64_t g = (m + 255) / 256;
  return (unsigned)(g == 0 ? 1 : g > 4096 ? 4096 : g);
}

int hist_build_level(const HistBuild& b, hipStream_t st) {
  if (b.m == 0) return 0;
  uint64_t* K[2] = {b.K[0], b.K[1]};
  uint32_t* V[2] = {b.V[0], b.V[1]};
  int r;
  if (b.mono) {
    // append order is tn order within every key: one stable sort by key
    k_hist_init<<<hgrid(b.m), 256, 0, st>>>(b.fk, b.m, K[0], V[0]);
    r = radix_sort_u64(K, V, b.m, b.kbits, b.scratch, st);
  } else {
    // LSD over (key, tn): by tn, then stably by key
    k_hist_init<<<hgrid(b.m), 256, 0, st>>>(b.ft, b.m, K[0], V[0]);
    const int r1 = radix_sort_u64(K, V, b.m, b.tbits, b.scratch, st);
    k_hist_regather<<<hgrid(b.m), 256, 0, st>>>(b.fk, V[r1], b.m, K[r1 ^ 1], V[r1 ^ 1]);
    uint64_t* K2[2] = {K[r1 ^ 1], K[r1]};
    uint32_t* V2[2] = {V[r1 ^ 1], V[r1]};
    const int r2 = radix_sort_u64(K2, V2, b.m, b.kbits, b.scratch, st);
    K[0] = K2[r2];
    V[0] = V2[r2];
    r = 0;
  }
  k_hist_gather<<<hgrid(b.m), 256, 0, st>>>(K[r], V[r], b.ft, b.m, b.skey, b.stn);
  if (hipMemsetAsync(b.hash, 0xFF, (32ull << b.hbits), st) != hipSuccess) return -1;
  k_hist_heads<<<hgrid(b.m), 256, 0, st>>>(b.skey, b.m, b.hash, b.hbits);
  k_hist_tails<<<hgrid(b.m), 256, 0, st>>>(b.skey, b.stn, b.m, b.hash, b.hbits);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

// ---------------------------------------------------------------- key bitmap
__global__ __launch_bounds__(256) void k_hist_bm(const uint64_t* keys, uint64_t m, uint32_t* bm) {
  for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < m; i += (uint64_t)gridDim.x * 256) {
    const uint32_t b = hist_bm_bit(keys[i]);
    atomicOr(&bm[b >> 5], 1u << (b & 31u));
  }
}
__global__ __launch_bounds__(256) void k_hist_bm_or(const uint32_t* a, const uint32_t* b, uint32_t* out) {
  for (uint32_t i = blockIdx.x * 256 + threadIdx.x; i < (1u << HIST_BM_LOG) / 32; i += gridDim.x * 256)
    out[i] = (a ? a[i] : 0u) | (b ? b[i] : 0u);
}
void launch_hist_bm(const uint64_t* keys, uint64_t m, uint32_t* bm, hipStream_t st) {
  (void)hipMemsetAsync(bm, 0, (1u << HIST_BM_LOG) / 8, st);
  if (m) k_hist_bm<<<hgrid(m), 256, 0, st>>>(keys, m, bm);
}
void launch_hist_bm_or(const uint32_t* a, const uint32_t* b, uint32_t* out, hipStream_t st) {
  k_hist_bm_or<<<16, 256, 0, st>>>(a, b, out);
}

// ---------------------------------------------------------------- trim
__global__ __launch_bounds__(256) void k_hist_trim(const uint64_t* ak, const uint64_t* at,
                                                   uint64_t na, const uint64_t* bk,
                                                   const uint64_t* bt, uint64_t nb, uint64_t floor,
                                                   uint64_t* ok, uint64_t* ot,
                                                   unsigned long long* cnt) {
  for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < na + nb;
       i += (uint64_t)gridDim.x * 256) {
    const uint64_t k = i < na ? ak[i] : bk[i - na];
    const uint64_t t = i < na ? at[i] : bt[i - na];
    if (t <= floor) continue;
    const unsigned long long p = atomicAdd(cnt, 1ull);
    ok[p] = k;
    ot[p] = t;
  }
}
void launch_hist_trim(const uint64_t* ak, const uint64_t* at, uint64_t na, const uint64_t* bk,
                      const uint64_t* bt, uint64_t nb, uint64_t floor, uint64_t* ok, uint64_t* ot,
                      unsigned long long* cnt, hipStream_t st) {
  k_hist_trim<<<hgrid(na + nb), 256, 0, st>>>(ak, at, na, bk, bt, nb, floor, ok, ot, cnt);
}

}  // namespace dcc
