// Device-resident OCC history: append, level build, trim (occ_history.h).
//
// Reference: central_finish pushes every committed write set onto `history`
// with tn = ++tnc (concurrency_control/occ.cpp:277-286); central_validate
// scans the entries with start_tn < tn <= finish_tn against the read set
// (occ.cpp:160-180).  Here an epoch's committed writes are appended on the
// device in index (= tn) order and the per-key tn runs are rebuilt by a
// stable radix sort, so the host never copies the batch back.
#include <hip/hip_runtime.h>

#include "dcc_device.h"
#include "occ_history.h"
#include "occ_kernels.h"
#include "radix_sort.h"

namespace dcc {

constexpr uint32_t HB = 1024;  // txns per block of the append kernels

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
    hash[2 * s + 1] = i;
  }
}
// the last pair of each run completes its slot: count = last + 1 - first
__global__ __launch_bounds__(256) void k_hist_tails(const uint64_t* skey, uint64_t m,
                                                    uint64_t* hash, uint32_t hbits) {
  const uint64_t mask = (1ull << hbits) - 1;
  for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < m; i += (uint64_t)gridDim.x * 256) {
    const uint64_t key = skey[i];
    if (i + 1 < m && skey[i + 1] == key) continue;
    uint64_t s = hist_hash_slot(key, hbits);
    while (hash[2 * s] != key) s = (s + 1) & mask;
    const uint64_t first = hash[2 * s + 1];
    hash[2 * s + 1] = first | ((i + 1 - first) << 32);
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
  if (hipMemsetAsync(b.hash, 0xFF, (16ull << b.hbits), st) != hipSuccess) return -1;
  k_hist_heads<<<hgrid(b.m), 256, 0, st>>>(b.skey, b.m, b.hash, b.hbits);
  k_hist_tails<<<hgrid(b.m), 256, 0, st>>>(b.skey, b.m, b.hash, b.hbits);
  return hipGetLastError() == hipSuccess ? 0 : -1;
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
