// GPU index probe and the Calvin wave dispatch lists.
//
// Index: the key -> row lookup IndexHash gives execution (index_insert /
// index_read, storage/index_hash.cpp:58-137, BucketHeader::insert_item /
// read_item :160-231) as one HBM open-addressing table probed for a whole
// epoch at once.  The reference's bucket chains return the most recently
// inserted item of a key (insert_item prepends, read_item takes the head);
// here every insert carries an ordinal and the slot keeps the largest, so
// the newest insert wins for duplicate keys inside one build and across
// builds.  A missing key is the reference's assertion failure
// (M_ASSERT_V, index_hash.cpp:221); here it is DCC_ROW_NONE and counted.
//
// Dispatch: the Calvin wave levels (dcc_calvin_order_epoch's out_wave: the
// schedule level at which TxnTable::restart_txn, txn_table.cpp:151-176,
// releases a txn after the lock_release promotions of row_lock.cpp:317-357)
// turned into what a dispatcher consumes: per wave, its txns in sequence
// order (a stable counting sort by wave on the GPU).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstring>

#include "dcc.h"
#include "dcc_ctx.h"
#include "dcc_device.h"
#include "radix_sort.h"

using namespace dcc;

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

__device__ inline uint64_t ix_hash(uint64_t key, uint32_t bits) {
  return (key * 0x9E3779B97F4A7C15ull) >> (64 - bits);
}

// slot words: key (DCC_KEY_RESERVED = empty) and the largest insert ordinal
__global__ __launch_bounds__(256) void k_ix_insert(const uint64_t* keys, uint64_t n, uint64_t base,
                                                   uint64_t* tk, unsigned long long* tord,
                                                   uint32_t bits, uint32_t* cnt) {
  const uint64_t mask = (1ull << bits) - 1;
  uint32_t fresh = 0, bad = 0;
  for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (uint64_t)gridDim.x * 256) {
    const uint64_t key = keys[i];
    if (key == DCC_KEY_RESERVED) {
      bad++;
      continue;
    }
    uint64_t s = ix_hash(key, bits);
    for (uint64_t q = 0; q <= mask; q++, s = (s + 1) & mask) {
      uint64_t v = tk[s];
      if (v == DCC_KEY_RESERVED) {
        const unsigned long long prev = atomicCAS((unsigned long long*)&tk[s],
                                                  (unsigned long long)DCC_KEY_RESERVED,
                                                  (unsigned long long)key);
        if (prev == DCC_KEY_RESERVED) fresh++;
        v = prev == DCC_KEY_RESERVED ? key : prev;
      }
      if (v == key) {
        atomicMax(&tord[s], (unsigned long long)(base + i));
        break;
      }
    }
  }
  for (int d = 32; d > 0; d >>= 1) {
    fresh += __shfl_xor(fresh, d);
    bad += __shfl_xor(bad, d);
  }
  if ((threadIdx.x & 63) == 0) {
    if (fresh) atomicAdd(&cnt[0], fresh);
    if (bad) atomicAdd(&cnt[1], bad);
  }
}

// one probe per key: the row of its newest insert, or DCC_ROW_NONE
__global__ __launch_bounds__(256) void k_ix_probe(const uint64_t* keys, uint64_t n,
                                                  const uint64_t* tk,
                                                  const unsigned long long* tord,
                                                  const uint64_t* rows, uint32_t bits,
                                                  uint64_t* out, uint32_t* cnt) {
  const uint64_t mask = (1ull << bits) - 1;
  uint32_t miss = 0;
  for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (uint64_t)gridDim.x * 256) {
    const uint64_t key = keys[i];
    uint64_t r = DCC_ROW_NONE;
    uint64_t s = ix_hash(key, bits);
    for (uint64_t q = 0; q <= mask; q++, s = (s + 1) & mask) {
      const uint64_t v = tk[s];
      if (v == key) {
        r = rows[tord[s]];
        break;
      }
      if (v == DCC_KEY_RESERVED) break;
    }
    miss += r == DCC_ROW_NONE;
    out[i] = r;
  }
  for (int d = 32; d > 0; d >>= 1) miss += __shfl_xor(miss, d);
  if ((threadIdx.x & 63) == 0 && miss) atomicAdd(&cnt[2], miss);
}

__global__ __launch_bounds__(256) void k_ix_rehash(const uint64_t* ok, const unsigned long long* oo,
                                                   uint64_t ocap, uint64_t* tk,
                                                   unsigned long long* tord, uint32_t bits) {
  const uint64_t mask = (1ull << bits) - 1;
  for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < ocap; i += (uint64_t)gridDim.x * 256) {
    const uint64_t key = ok[i];
    if (key == DCC_KEY_RESERVED) continue;
    uint64_t s = ix_hash(key, bits);
    while (atomicCAS((unsigned long long*)&tk[s], (unsigned long long)DCC_KEY_RESERVED,
                     (unsigned long long)key) != DCC_KEY_RESERVED)
      s = (s + 1) & mask;  // keys are unique in the old table
    tord[s] = oo[i];
  }
}

inline unsigned g256(uint64_t n) {
  const uint64_t g = (n + 255) / 256;
  return (unsigned)std::max<uint64_t>(1, std::min<uint64_t>(g, 16384));
}

// ---------------------------------------------------------------- dispatch
__global__ __launch_bounds__(256) void k_wv_max(const uint32_t* wave, uint64_t n, uint32_t* mx) {
  uint32_t m = 0;
  for (uint64_t t = (uint64_t)blockIdx.x * 256 + threadIdx.x; t < n; t += (uint64_t)gridDim.x * 256)
    m = max(m, wave[t]);
  for (int d = 32; d > 0; d >>= 1) m = max(m, (uint32_t)__shfl_xor(m, d));
  if ((threadIdx.x & 63) == 0) atomicMax(mx, m);
}
// sort keys: the wave of the txn at sequence position q; value: the txn
__global__ __launch_bounds__(256) void k_wv_keys(const uint32_t* wave, const uint32_t* seq,
                                                 uint64_t n, uint32_t* k, uint32_t* v) {
  for (uint64_t q = (uint64_t)blockIdx.x * 256 + threadIdx.x; q < n; q += (uint64_t)gridDim.x * 256) {
    const uint32_t t = seq ? seq[q] : (uint32_t)q;
    k[q] = wave[t];
    v[q] = t;
  }
}
// wave offsets from the sorted waves: off[w] = first position of wave w
__global__ __launch_bounds__(256) void k_wv_off(const uint32_t* sk, uint64_t n, uint32_t nw,
                                                uint32_t* off) {
  for (uint64_t p = (uint64_t)blockIdx.x * 256 + threadIdx.x; p < n; p += (uint64_t)gridDim.x * 256) {
    const uint32_t w = sk[p], pw = p ? sk[p - 1] : 0u;
    if (p == 0)
      for (uint32_t x = 0; x <= w; x++) off[x] = 0;
    else
      for (uint32_t x = pw + 1; x <= w; x++) off[x] = (uint32_t)p;
    if (p + 1 == n)
      for (uint32_t x = w + 1; x <= nw; x++) off[x] = (uint32_t)n;
  }
}
__global__ __launch_bounds__(256) void k_wv_order_keys(const uint64_t* order, uint64_t n,
                                                       uint64_t* k, uint32_t* v) {
  for (uint64_t t = (uint64_t)blockIdx.x * 256 + threadIdx.x; t < n; t += (uint64_t)gridDim.x * 256) {
    k[t] = order[t];
    v[t] = (uint32_t)t;
  }
}

}  // namespace

// ---------------------------------------------------------------- index API
int dcc_ctx::index_reserve(uint64_t want) {
  dcc_ctx* ctx = this;
  if (ix_bits && 2 * want <= (1ull << ix_bits)) return DCC_OK;
  uint32_t bits = std::max<uint32_t>(ix_bits, 12);
  while ((1ull << bits) < 2 * want) bits++;
  if (bits > 34) return fail(DCC_ERANGE, "index: more than 2^33 keys");
  const uint64_t cap = 1ull << bits;
  // the new table: released on every error return, moved in on success
  DevBuf nk, no;
  struct Guard {
    DevBuf *a, *b;
    ~Guard() {
      if (a) a->release();
      if (b) b->release();
    }
  } guard{&nk, &no};
  CR(nk.ensure(this, cap * 8, "index keys"));
  CR(no.ensure(this, cap * 8, "index ordinals"));
  CK(hipMemsetAsync(nk.p, 0xFF, cap * 8, stream));
  CK(hipMemsetAsync(no.p, 0, cap * 8, stream));
  if (ix_bits)
    k_ix_rehash<<<g256(1ull << ix_bits), 256, 0, stream>>>(
        (const uint64_t*)ix_keys.p, (const unsigned long long*)ix_ord.p, 1ull << ix_bits,
        (uint64_t*)nk.p, (unsigned long long*)no.p, bits);
  CK(hipGetLastError());
  CK(hipStreamSynchronize(stream));
  ix_keys.release();
  ix_ord.release();
  ix_keys = nk;
  ix_ord = no;
  guard.a = guard.b = nullptr;
  ix_bits = bits;
  return DCC_OK;
}

extern "C" int dcc_index_insert(dcc_ctx* ctx, const uint64_t* keys, const uint64_t* rows,
                                uint64_t n) {
  if (!ctx || (n && (!keys || !rows))) return DCC_EINVAL;
  if (ctx->multi) return ctx->fail(DCC_ENOTSUP, "index: single-GPU");
  if (n == 0) return DCC_OK;
  if (hipSetDevice(ctx->device) != hipSuccess) return DCC_ENODEV;
  CR(ctx->index_reserve(ctx->ix_nkeys + n));
  // the rows of every insert so far, by ordinal (grow-with-copy)
  const uint64_t base = ctx->ix_nrows;
  if ((base + n) * 8 > ctx->ix_rows.cap) {
    DevBuf nr;
    CR(nr.ensure(ctx, std::max<uint64_t>((base + n) * 8 * 3 / 2, 4096), "index rows"));
    if (base) CK(hipMemcpy(nr.p, ctx->ix_rows.p, base * 8, hipMemcpyDeviceToDevice));
    ctx->ix_rows.release();
    ctx->ix_rows = nr;
  }
  // host keys staged in the context's grow-only scratch (no per-call allocation)
  DevBuf& tk = ctx->ix_scr;
  CR(tk.ensure(ctx, n * 8, "index insert keys"));
  CR(ctx->ix_cnt.ensure(ctx, 64, "index counters"));
  CK(hipMemcpyAsync(tk.p, keys, n * 8, hipMemcpyHostToDevice, ctx->stream));
  CK(hipMemcpyAsync((uint64_t*)ctx->ix_rows.p + base, rows, n * 8, hipMemcpyHostToDevice, ctx->stream));
  CK(hipMemsetAsync(ctx->ix_cnt.p, 0, 16, ctx->stream));
  k_ix_insert<<<g256(n), 256, 0, ctx->stream>>>((const uint64_t*)tk.p, n, base,
                                                (uint64_t*)ctx->ix_keys.p,
                                                (unsigned long long*)ctx->ix_ord.p, ctx->ix_bits,
                                                (uint32_t*)ctx->ix_cnt.p);
  CK(hipGetLastError());
  uint32_t c[2];
  CK(hipMemcpyAsync(c, ctx->ix_cnt.p, 8, hipMemcpyDeviceToHost, ctx->stream));
  CK(hipStreamSynchronize(ctx->stream));
  ctx->ix_nkeys += c[0];
  ctx->ix_nrows += n;
  if (c[1]) return ctx->fail(DCC_EINVAL, "index: key equal to DCC_KEY_RESERVED");
  return DCC_OK;
}

extern "C" int dcc_index_probe(dcc_ctx* ctx, const uint64_t* keys, uint64_t n, uint64_t* out_rows,
                               uint32_t flags, uint64_t* out_missing) {
  if (!ctx || (n && (!keys || !out_rows))) return DCC_EINVAL;
  if (ctx->multi) return ctx->fail(DCC_ENOTSUP, "index: single-GPU");
  if (hipSetDevice(ctx->device) != hipSuccess) return DCC_ENODEV;
  if (out_missing) *out_missing = 0;
  if (n == 0) return DCC_OK;
  const bool dev = (flags & DCC_DEVICE_PTRS) != 0;
  CR(ctx->ix_cnt.ensure(ctx, 64, "index counters"));
  if (!ctx->ix_bits) CR(ctx->index_reserve(1));
  if (!ctx->ix_rows.p) CR(ctx->ix_rows.ensure(ctx, 4096, "index rows"));
  const uint64_t* dk = keys;
  uint64_t* dout = out_rows;
  if (!dev) {  // host pointers: keys and rows staged in the grow-only scratch
    CR(ctx->ix_scr.ensure(ctx, n * 16, "probe keys + rows"));
    uint64_t* tk = (uint64_t*)ctx->ix_scr.p;
    CK(hipMemcpyAsync(tk, keys, n * 8, hipMemcpyHostToDevice, ctx->stream));
    dk = tk;
    dout = tk + n;
  }
  CK(hipMemsetAsync(ctx->ix_cnt.p, 0, 16, ctx->stream));
  CK(hipEventRecord(ctx->ev0, ctx->stream));
  k_ix_probe<<<g256(n), 256, 0, ctx->stream>>>(dk, n, (const uint64_t*)ctx->ix_keys.p,
                                               (const unsigned long long*)ctx->ix_ord.p,
                                               (const uint64_t*)ctx->ix_rows.p, ctx->ix_bits, dout,
                                               (uint32_t*)ctx->ix_cnt.p);
  CK(hipGetLastError());
  CK(hipEventRecord(ctx->ev1, ctx->stream));
  if (!dev) CK(hipMemcpyAsync(out_rows, dout, n * 8, hipMemcpyDeviceToHost, ctx->stream));
  uint32_t c[3];
  CK(hipMemcpyAsync(c, ctx->ix_cnt.p, 12, hipMemcpyDeviceToHost, ctx->stream));
  CK(hipStreamSynchronize(ctx->stream));
  float ms = 0;
  CK(hipEventElapsedTime(&ms, ctx->ev0, ctx->ev1));
  ctx->ix_last_ms = ms;
  if (out_missing) *out_missing = c[2];
  return DCC_OK;
}

extern "C" uint64_t dcc_index_size(const dcc_ctx* ctx) { return ctx ? ctx->ix_nkeys : 0; }
extern "C" double dcc_index_last_ms(const dcc_ctx* ctx) { return ctx ? ctx->ix_last_ms : 0.0; }

extern "C" int dcc_index_clear(dcc_ctx* ctx) {
  if (!ctx) return DCC_EINVAL;
  ctx->ix_keys.release();
  ctx->ix_ord.release();
  ctx->ix_rows.release();
  ctx->ix_bits = 0;
  ctx->ix_nkeys = ctx->ix_nrows = 0;
  return DCC_OK;
}

// ---------------------------------------------------------------- dispatch API
extern "C" int dcc_calvin_dispatch(dcc_ctx* ctx, const uint32_t* wave, const uint64_t* order,
                                   uint64_t n, uint32_t flags, uint32_t* out_wave_off,
                                   uint64_t off_cap, uint32_t* out_txn, uint32_t* out_n_waves) {
  if (!ctx || !out_n_waves || (n && (!wave || !out_txn))) return DCC_EINVAL;
  if (ctx->multi) return ctx->fail(DCC_ENOTSUP, "dispatch: single-GPU");
  if (hipSetDevice(ctx->device) != hipSuccess) return DCC_ENODEV;
  *out_n_waves = 0;
  if (n == 0) {
    if (out_wave_off && off_cap) out_wave_off[0] = 0;
    return DCC_OK;
  }
  if (n >= 0xFFFFFFFFull) return ctx->fail(DCC_ERANGE, "dispatch: n exceeds 2^32-1");
  const bool dev = (flags & DCC_DEVICE_PTRS) != 0;
  hipStream_t st = ctx->stream;
  CR(ctx->wv_buf.ensure(ctx, n * 4 * 6 + n * 8 * 2 + 64, "dispatch workspace"));
  uint64_t* ok[2] = {(uint64_t*)ctx->wv_buf.p, (uint64_t*)ctx->wv_buf.p + n};  // 8-B aligned first
  uint32_t* w = (uint32_t*)(ok[1] + n);
  uint32_t* kb[2] = {w, w + n};
  uint32_t* vb[2] = {w + 2 * n, w + 3 * n};
  uint32_t* seqb = w + 4 * n;
  uint32_t* mx = w + 5 * n;
  const uint32_t* dwave = wave;
  const uint64_t* dorder = order;
  // host pointers: order and waves staged in the grow-only scratch
  if (!dev) {
    CR(ctx->wv_hbuf.ensure(ctx, n * 8 + n * 4 + 64, "dispatch staging"));
    uint64_t* to = (uint64_t*)ctx->wv_hbuf.p;
    uint32_t* tw = (uint32_t*)(to + n);
    CK(hipMemcpyAsync(tw, wave, n * 4, hipMemcpyHostToDevice, st));
    dwave = tw;
    if (order) {
      CK(hipMemcpyAsync(to, order, n * 8, hipMemcpyHostToDevice, st));
      dorder = to;
    }
  }
  CR(ctx->cv_scratch.ensure(ctx, rs_scratch_words(n) * 4 + 64, "radix scratch"));
  // sequence positions (stable: ties keep index order), as dcc_calvin_order_epoch
  const uint32_t* seq = nullptr;
  if (dorder) {
    k_wv_order_keys<<<g256(n), 256, 0, st>>>(dorder, n, ok[0], vb[0]);
    const int c = radix_sort_u64(ok, vb, n, 64, (uint32_t*)ctx->cv_scratch.p, st);
    CK(hipMemcpyAsync(seqb, vb[c], n * 4, hipMemcpyDeviceToDevice, st));
    seq = seqb;
  }
  CK(hipMemsetAsync(mx, 0, 4, st));
  k_wv_max<<<g256(n), 256, 0, st>>>(dwave, n, mx);
  k_wv_keys<<<g256(n), 256, 0, st>>>(dwave, seq, n, kb[0], vb[0]);
  uint32_t hmx = 0;
  CK(hipMemcpyAsync(&hmx, mx, 4, hipMemcpyDeviceToHost, st));
  CK(hipStreamSynchronize(st));
  const uint32_t nw = hmx + 1;
  *out_n_waves = nw;
  if (out_wave_off && off_cap < (uint64_t)nw + 1)
    return ctx->fail(DCC_ERANGE, "dispatch: %u waves need %u offsets", nw, nw + 1);
  uint32_t bits = 0;
  while (bits < 32 && (1ull << bits) <= hmx) bits++;
  const int c = radix_sort_u32(kb, vb, n, bits, (uint32_t*)ctx->cv_scratch.p, st);
  uint32_t* doff = dev ? out_wave_off : nullptr;
  if (out_wave_off && !dev) {
    CR(ctx->wv_obuf.ensure(ctx, ((uint64_t)nw + 1) * 4, "dispatch offsets"));
    doff = (uint32_t*)ctx->wv_obuf.p;
  }
  if (doff) k_wv_off<<<g256(n), 256, 0, st>>>(kb[c], n, nw, doff);
  CK(hipGetLastError());
  if (dev) {
    CK(hipMemcpyAsync(out_txn, vb[c], n * 4, hipMemcpyDeviceToDevice, st));
  } else {
    CK(hipMemcpyAsync(out_txn, vb[c], n * 4, hipMemcpyDeviceToHost, st));
    if (doff) CK(hipMemcpyAsync(out_wave_off, doff, ((uint64_t)nw + 1) * 4, hipMemcpyDeviceToHost, st));
  }
  CK(hipStreamSynchronize(st));
  return DCC_OK;
}
