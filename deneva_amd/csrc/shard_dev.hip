// Device-side key-shard partition ("a device-side partition
// kernel"): the sub-context of rank r of a multi-GPU context keeps only the
// accesses whose key it owns (dcc_key_shard(key, R) == r, shard.cpp), as a CSR
// over every txn of the epoch, plus each kept access's index in the batch
// (Calvin grant groups go back to batch order through it).  The batch is read
// once from HBM -- its own staging copy, or the caller's device batch (on
// this GPU, or a peer's over xGMI) -- instead of being split on one host
// thread every epoch.
//
//   k_sh_count    one txn per thread: its own-shard accesses; per-block sums
//   rs_scan_one   exclusive scan of the block sums
//   k_sh_scatter  offsets, and the kept keys / types / batch indices
#include <hip/hip_runtime.h>

#include <algorithm>

#include "dcc.h"
#include "dcc_ctx.h"
#include "dcc_device.h"
#include "radix_sort.h"

#define CK(expr)                                           \
  do {                                                     \
    hipError_t e_ = (expr);                                \
    if (e_ != hipSuccess) return ctx->hip_fail(e_, #expr); \
  } while (0)
#define CR(expr)                 \
  do {                           \
    int r_ = (expr);             \
    if (r_ != DCC_OK) return r_; \
  } while (0)

namespace {

// dcc_key_shard (shard.cpp) on the device: splitmix64 finaliser, multiply-high
__device__ inline uint32_t key_shard(uint64_t key, uint32_t nranks) {
  uint64_t x = (key ^ 0x5DEECE66Dull) + 0x9E3779B97F4A7C15ull;
  x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
  x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
  x ^= x >> 31;
  return (uint32_t)__umul64hi(x, (uint64_t)nranks);
}

constexpr uint32_t SH_B = 256;

__device__ inline uint32_t sh_count(const uint32_t* off, const uint64_t* keys, uint64_t nnz,
                                    uint64_t t, uint32_t rank, uint32_t R) {
  const uint64_t s = min((uint64_t)off[t], nnz), e = min((uint64_t)off[t + 1], nnz);
  uint32_t c = 0;
  for (uint64_t x = s; x < e; x++) c += key_shard(keys[x], R) == rank;
  return c;
}

__global__ __launch_bounds__(SH_B) void k_sh_count(const uint32_t* off, const uint64_t* keys,
                                                   uint64_t n, uint64_t nnz, uint32_t rank,
                                                   uint32_t R, uint32_t* cnt, uint32_t* bsum) {
  __shared__ uint32_t s_w[SH_B / 64];
  const uint64_t t = (uint64_t)blockIdx.x * SH_B + threadIdx.x;
  const uint32_t c = t < n ? sh_count(off, keys, nnz, t, rank, R) : 0u;
  if (t < n) cnt[t] = c;
  uint32_t v = c;
  for (int d = 32; d > 0; d >>= 1) v += __shfl_xor(v, d);
  if ((threadIdx.x & 63) == 0) s_w[threadIdx.x >> 6] = v;
  __syncthreads();
  if (threadIdx.x == 0) {
    uint32_t b = 0;
    for (uint32_t w = 0; w < SH_B / 64; w++) b += s_w[w];
    bsum[blockIdx.x] = b;
  }
}

__global__ __launch_bounds__(SH_B) void k_sh_scatter(const uint32_t* off, const uint64_t* keys,
                                                     const uint8_t* at, uint64_t n, uint64_t nnz,
                                                     uint32_t rank, uint32_t R, const uint32_t* cnt,
                                                     const uint32_t* bsum, const uint32_t* total,
                                                     uint32_t* off_out, uint64_t* keys_out,
                                                     uint8_t* at_out, uint32_t* src_out) {
  __shared__ uint32_t s_w[SH_B / 64];
  const uint32_t lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const uint64_t t = (uint64_t)blockIdx.x * SH_B + threadIdx.x;
  const uint32_t c = t < n ? cnt[t] : 0u;
  uint32_t x = c;
  for (int d = 1; d < 64; d <<= 1) {
    const uint32_t y = __shfl_up(x, d);
    if (lane >= (uint32_t)d) x += y;
  }
  if (lane == 63) s_w[wv] = x;
  __syncthreads();
  uint32_t o = bsum[blockIdx.x] + x - c;
  for (uint32_t w = 0; w < wv; w++) o += s_w[w];
  if (t < n) {
    off_out[t] = o;
    const uint64_t s = min((uint64_t)off[t], nnz), e = min((uint64_t)off[t + 1], nnz);
    for (uint64_t q = s; q < e; q++) {
      const uint64_t k = keys[q];
      if (key_shard(k, R) != rank) continue;
      keys_out[o] = k;
      at_out[o] = at[q];
      src_out[o] = (uint32_t)q;
      o++;
    }
  }
  if (t == 0) off_out[n] = *total;
}

// Calvin grant groups of a shard back to batch order (device outputs: the
// caller's array may sit on a peer GPU, written over xGMI)
__global__ __launch_bounds__(SH_B) void k_sh_groups(const uint32_t* grp, const uint32_t* src,
                                                    uint64_t m, uint32_t* out) {
  for (uint64_t j = (uint64_t)blockIdx.x * SH_B + threadIdx.x; j < m; j += (uint64_t)gridDim.x * SH_B)
    out[src[j]] = grp[j];
}

inline unsigned blocks(uint64_t n) { return (unsigned)std::max<uint64_t>(1, (n + SH_B - 1) / SH_B); }

}  // namespace

// Rank `rank` of R: this context's shard of batch b as a device batch `sb`
// (DCC_DEVICE_PTRS; the per-txn windows / order stay those of the staged or
// caller's batch).  One host synchronisation: the shard's access count.
int dcc_ctx::shard_stage(const dcc_batch* b, uint32_t rank, uint32_t R, dcc_batch& sb,
                         DevBatch* full_out) {
  dcc_ctx* ctx = this;
  DevBatch full;
  CR(stage_batch(b, full));
  if (full_out) *full_out = full;
  const uint64_t n = full.n, nnz = full.nnz;
  const unsigned nb = blocks(n);
  CR(sh_off.ensure(this, (n + 1) * 4 + 64, "shard offsets"));
  CR(sh_keys.ensure(this, std::max<uint64_t>(8, nnz * 8), "shard keys"));
  CR(sh_at.ensure(this, std::max<uint64_t>(16, nnz), "shard types"));
  CR(sh_src.ensure(this, std::max<uint64_t>(16, nnz * 4), "shard batch indices"));
  CR(sh_cnt.ensure(this, n * 4 + 64, "shard counts"));
  CR(sh_bsum.ensure(this, (nb + 2) * 4, "shard block sums"));
  uint32_t* bs = (uint32_t*)sh_bsum.p;
  k_sh_count<<<nb, SH_B, 0, stream>>>(full.off, full.keys, n, nnz, rank, R, (uint32_t*)sh_cnt.p, bs);
  dcc::rs_scan_one(bs, nb, bs + nb, stream);
  k_sh_scatter<<<nb, SH_B, 0, stream>>>(full.off, full.keys, full.acctype, n, nnz, rank, R,
                                        (const uint32_t*)sh_cnt.p, bs, bs + nb, (uint32_t*)sh_off.p,
                                        (uint64_t*)sh_keys.p, (uint8_t*)sh_at.p, (uint32_t*)sh_src.p);
  CK(hipGetLastError());
  CK(hipMemcpyAsync(hmisc, bs + nb, 4, hipMemcpyDeviceToHost, stream));
  CK(hipStreamSynchronize(stream));
  sb = *b;
  sb.flags = (b->flags | DCC_DEVICE_PTRS) & ~DCC_COMPACT_FLAGS;  // stage_batch widened them
  sb.n_txn = n;
  sb.nnz = *(const uint32_t*)hmisc;
  sb.offsets = (const uint32_t*)sh_off.p;
  sb.keys = (const uint64_t*)sh_keys.p;
  sb.acctype = (const uint8_t*)sh_at.p;
  sb.start_tn = full.start_tn;
  sb.finish_tn = full.finish_tn;
  sb.order = full.order;
  return DCC_OK;
}

int dcc_ctx::shard_groups(const uint32_t* grp, uint64_t m, uint32_t* out_dev) {
  dcc_ctx* ctx = this;
  if (!m) return DCC_OK;
  k_sh_groups<<<(unsigned)std::min<uint64_t>(4096, blocks(m)), SH_B, 0, stream>>>(
      grp, (const uint32_t*)sh_src.p, m, out_dev);
  CK(hipGetLastError());
  return DCC_OK;
}
