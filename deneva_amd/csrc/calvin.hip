// Calvin epoch lock ordering on gfx950.
//
// Reference semantics (parity target): the sequencer fixes a global order of
// the epoch (Sequencer::process_txn / send_next_batch, sequencer.cpp:184-326;
// QWorkQueue::sched_dequeue, work_queue.cpp:105-151); one lock thread walks
// the epoch in that order calling acquire_locks (calvin_thread.cpp:40-100,
// ycsb_txn.cpp:49-88), which requests every row once (txn.cpp:778-782) in SH
// for RD/SCAN, else EX (row.cpp:191) from Row_lock in CALVIN mode: FIFO, no
// barging past waiters (row_lock.cpp:78-81, 152-170); lock_release promotes
// the compatible head of the waiter queue (row_lock.cpp:317-357).
//
// Against an empty lock table that is a pure per-row function of the
// requests in sequence order:
//   grant group of a request = number of group boundaries before it on its
//     row, where consecutive requests start a new group iff either is EX
//     (an SH run shares one group, every EX is alone);
//   acquire_locks returns RCOK iff every request of the txn is in group 0;
//   wave(txn) = 1 + max over its requests of the max wave of the row's
//     previous group (0 when all requests are in group 0): the txn's place in
//     a schedule where every ready txn runs and then releases all its locks.
//
// Device pipeline (one stream, one host sync after the prep reduction):
//   k_cv_prep      OR/AND of keys and of order -> which bits vary
//   rank           stable radix sort of packed order -> seq (sched order)
//   k_cv_layout    requests in sequence order: packed key, (txn, j, EX) value
//   key sort       stable radix sort by packed key -> per-row FIFO runs
//   k_cv_up/top/down  one segmented scan (monoid below) -> group, dedup,
//                  readiness, and the group links the wave kernel needs
//   waves          (optional) wave levels: the one-CU sequence-order walk
//                  (calvin_wave.h) for txns of at most 32 requests, else
//                  k_cv_wave, dependency-driven, one txn per wave64
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>

#include "calvin_bucket.h"
#include "calvin_gl.h"
#include "calvin_wave.h"
#include "dcc.h"
#include "dcc_ctx.h"
#include "dcc_device.h"
#include "dcc_env.h"
#include "occ_kernels.h"
#include "prep_body.h"
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
// helper workgroups of the wave walk (calvin_wave.hip), each on a CU of its
// own (experiments builds: DCC_CW_HELPERS, 0 = the walker's workgroup alone;
// C4: 0 34.7 ms, 16 18.1, 32 18.1 -- profiles/r06/cwhelp/)
constexpr uint32_t CW_NH = 16;
uint32_t cw_helpers(int n_cu) {
  uint32_t nh = CW_NH;
  if (const char* e = DCC_ENV("DCC_CW_HELPERS")) nh = (uint32_t)atoi(e);
  return std::min<uint32_t>(nh, n_cu > 1 ? (uint32_t)n_cu - 1u : 0u);
}

constexpr uint32_t NOPOS = 0xFFFFFFFFu;
constexpr uint32_t CV_MAX_TXN = 1u << 25;  // value = txn:25 | j:6 | EX:1
constexpr unsigned CV_PREP_BLOCKS = 1024;
constexpr uint32_t CV_ITEMS = 16;                  // scan elements per thread
constexpr uint32_t CV_TILE = 256 * CV_ITEMS;       // scan elements per workgroup
constexpr uint64_t CV_PUT_MIN = 1ull << 21;        // requests from which groups go out windowed
constexpr uint32_t ERR_WAVE_TIMEOUT = 1u << 8;

struct CvPart {
  uint64_t kor, kand, oor, oand;
  uint32_t nex, unsorted, pad[2];  // EX requests; positions t with order[t] > order[t + 1]
};
constexpr size_t CV_COUNT_OFF = 65536;  // CvCount partials inside part / hpart (after the prep's)

// ---------------------------------------------------------------- prep
// Workgroups [0, CV_PREP_BLOCKS): the key / order bit reductions; the rest
// run the batch validation (prep_body.h: offsets, lengths) beside them in the
// same launch.
__global__ __launch_bounds__(256) void k_cv_prep(const uint64_t* __restrict__ keys, uint64_t nnz,
                                                 const uint8_t* __restrict__ at,
                                                 const uint64_t* __restrict__ order, uint64_t n,
                                                 const uint64_t* __restrict__ hkeys, uint64_t nh,
                                                 CvPart* __restrict__ part, const uint32_t* off,
                                                 PrepPart* pp) {
  if (blockIdx.x >= CV_PREP_BLOCKS) {
    prep_body(off, n, at, nnz, 0, pp, blockIdx.x - CV_PREP_BLOCKS, gridDim.x - CV_PREP_BLOCKS);
    return;
  }
  __shared__ uint64_t s[4][4];
  __shared__ uint32_t s_ex[4];
  uint64_t kor = 0, kand = ~0ull, oor = 0, oand = ~0ull;
  uint32_t nex = 0, uns = 0;
  const uint64_t tid = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const uint64_t stride = (uint64_t)CV_PREP_BLOCKS * blockDim.x;
  // 16-B loads: two keys, sixteen access types per load (when aligned)
  const uint64_t n2 = ((uintptr_t)keys & 15) ? 0 : nnz / 2;
  const uint64_t n16 = ((uintptr_t)at & 15) ? 0 : nnz / 16;
  for (uint64_t x = tid; x < n2; x += stride) {
    const ulonglong2 k = ((const ulonglong2*)keys)[x];
    kor |= k.x | k.y;
    kand &= k.x & k.y;
  }
  for (uint64_t x = 2 * n2 + tid; x < nnz; x += stride) {
    kor |= keys[x];
    kand &= keys[x];
  }
  for (uint64_t x = tid; x < n16; x += stride) {
    const uint4 q = ((const uint4*)at)[x];
    const uint32_t w[4] = {q.x, q.y, q.z, q.w};
#pragma unroll
    for (int b = 0; b < 4; b++)
#pragma unroll
      for (int c = 0; c < 4; c++) {
        const uint32_t a = (w[b] >> (8 * c)) & 255u;
        nex += (a != DCC_RD && a != DCC_SCAN) ? 1u : 0u;
      }
  }
  for (uint64_t x = 16 * n16 + tid; x < nnz; x += stride) {
    const uint8_t a = at[x];
    nex += (a != DCC_RD && a != DCC_SCAN) ? 1u : 0u;
  }
  for (uint64_t x = tid; x < nh; x += stride) {  // rows of the held prefix
    const uint64_t k = hkeys[x];
    kor |= k;
    kand &= k;
  }
  if (order)
    for (uint64_t t = tid; t < n; t += stride) {
      const uint64_t o = order[t];
      oor |= o;
      oand &= o;
      // already in sequence order (a sequencer hands its batch over origin by
      // origin, FIFO): the stable rank is the identity and needs no sort
      uns += (t + 1 < n && o > order[t + 1]) ? 1u : 0u;
    }
  for (int d = 32; d > 0; d >>= 1) {
    kor |= __shfl_xor(kor, d);
    kand &= __shfl_xor(kand, d);
    oor |= __shfl_xor(oor, d);
    oand &= __shfl_xor(oand, d);
    nex += __shfl_xor(nex, d);
    uns += __shfl_xor(uns, d);
  }
  __shared__ uint32_t s_un[4];
  const uint32_t wv = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) {
    s[wv][0] = kor;
    s[wv][1] = kand;
    s[wv][2] = oor;
    s[wv][3] = oand;
    s_ex[wv] = nex;
    s_un[wv] = uns;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    CvPart p{0, ~0ull, 0, ~0ull, 0, 0, {0, 0}};
    for (int w = 0; w < 4; w++) {
      p.kor |= s[w][0];
      p.kand &= s[w][1];
      p.oor |= s[w][2];
      p.oand &= s[w][3];
      p.nex += s_ex[w];
      p.unsorted += s_un[w];
    }
    part[blockIdx.x] = p;
  }
}

// ---------------------------------------------------------------- rank
template <typename K>
__global__ __launch_bounds__(256) void k_cv_order_init(const uint64_t* __restrict__ order,
                                                       uint64_t n, KeyPack kp, K* __restrict__ ok,
                                                       uint32_t* __restrict__ ov) {
  const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= n) return;
  ok[t] = (K)keypack_apply(kp, order[t]);
  ov[t] = (uint32_t)t;
}

// lengths in sequence order, then per-tile sums (u32 exclusive scan, pass 1)
__global__ __launch_bounds__(256) void k_cv_len_tiles(const uint32_t* __restrict__ off,
                                                      const uint32_t* __restrict__ seq, uint64_t n,
                                                      uint32_t* __restrict__ len,
                                                      uint32_t* __restrict__ tsum) {
  __shared__ uint32_t sh[4];
  const uint64_t base = (uint64_t)blockIdx.x * CV_TILE;
  uint32_t s = 0;
  for (uint32_t it = 0; it < CV_ITEMS; it++) {
    const uint64_t q = base + it * 256 + threadIdx.x;
    if (q < n) {
      const uint32_t t = seq[q];
      const uint32_t l = off[t + 1] - off[t];
      len[q] = l;
      s += l;
    }
  }
  for (int d = 32; d > 0; d >>= 1) s += __shfl_xor(s, d);
  if ((threadIdx.x & 63) == 0) sh[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) tsum[blockIdx.x] = sh[0] + sh[1] + sh[2] + sh[3];
}

// exclusive scan of len (tile prefix from the scanned tsum) -> off2 [n+1]
__global__ __launch_bounds__(256) void k_cv_len_apply(const uint32_t* __restrict__ len, uint64_t n,
                                                      const uint32_t* __restrict__ tpre,
                                                      uint32_t nnz, uint32_t* __restrict__ off2) {
  __shared__ uint32_t sh[4];
  const uint64_t base = (uint64_t)blockIdx.x * CV_TILE + (uint64_t)threadIdx.x * CV_ITEMS;
  uint32_t v[CV_ITEMS], s = 0;
  for (uint32_t i = 0; i < CV_ITEMS; i++) {
    v[i] = base + i < n ? len[base + i] : 0u;
    s += v[i];
  }
  const uint32_t lane = lane_id(), wv = threadIdx.x >> 6;
  uint32_t x = s;
  for (int d = 1; d < 64; d <<= 1) {
    const uint32_t y = __shfl_up(x, d);
    if (lane >= (uint32_t)d) x += y;
  }
  if (lane == 63) sh[wv] = x;
  __syncthreads();
  uint32_t run = tpre[blockIdx.x] + x - s;
  for (uint32_t w = 0; w < wv; w++) run += sh[w];
  for (uint32_t i = 0; i < CV_ITEMS; i++) {
    if (base + i < n) off2[base + i] = run;
    run += v[i];
  }
  if (blockIdx.x == 0 && threadIdx.x == 0) off2[n] = nnz;
}

// ---------------------------------------------------------------- layout
// Requests in sequence order: position q's txn t = seq[q] writes its requests
// to [off2[q], off2[q+1]) as (packed key, t:25 | j:6 | EX:1).  One wave per
// 64 positions: the lanes walk the wave's whole request range together (the
// txn of each output found by a search of the wave's length prefix in LDS),
// so both the key / type reads and the writes are coalesced instead of one
// lane streaming one txn.
template <typename K>
__global__ __launch_bounds__(256) void k_cv_layout(const uint32_t* __restrict__ off,
                                                   const uint32_t* __restrict__ seq,
                                                   const uint32_t* __restrict__ off2, uint64_t n,
                                                   const uint64_t* __restrict__ keys,
                                                   const uint8_t* __restrict__ at, KeyPack kp,
                                                   uint32_t base, uint32_t ulen, K* __restrict__ ak,
                                                   uint32_t* __restrict__ av) {
  __shared__ uint32_t s_src[4][64], s_pre[4][65], s_t[4][64];
  const uint32_t lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const uint64_t q0 = ((uint64_t)blockIdx.x * 4 + w) * 64;
  if (q0 >= n) return;  // whole wave: no barrier below is workgroup-wide
  const uint64_t q = q0 + lane;
  uint32_t t = 0, src = 0, len = 0;
  if (q < n) {
    t = seq ? seq[q] : (uint32_t)q;
    src = off[t];
    len = off[t + 1] - src;
  }
  uint32_t x = len;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const uint32_t y = __shfl_up(x, d);
    if (lane >= (uint32_t)d) x += y;
  }
  const uint32_t total = __shfl(x, 63);
  s_src[w][lane] = src;
  s_pre[w][lane] = x - len;
  s_t[w][lane] = t;
  if (lane == 0) s_pre[w][64] = total;
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  // the wave's first request in sequence order: q0 * len for uniform txns,
  // else the sequence-order offsets (identity order: the batch's own)
  const uint64_t d0 = (uint64_t)base + (ulen ? q0 * ulen : (off2 ? off2[q0] : off[q0]));
  for (uint32_t jj = lane; jj < total; jj += 64) {
    // largest k with pre[k] <= jj (empty txns share a prefix value: take the last)
    uint32_t lo = 0, hi = 64;
    while (hi - lo > 1) {
      const uint32_t mid = (lo + hi) >> 1;
      if (s_pre[w][mid] <= jj) lo = mid;
      else hi = mid;
    }
    const uint32_t j = jj - s_pre[w][lo];
    const uint32_t xs = s_src[w][lo] + j;
    const uint8_t a = at[xs];
    ak[d0 + jj] = (K)keypack_apply(kp, keys[xs]);
    av[d0 + jj] = (s_t[w][lo] << 7) | (j << 1) | ((a != DCC_RD && a != DCC_SCAN) ? 1u : 0u);
  }
}

// The held prefix (rows still locked when the epoch starts, row_lock.cpp:
// 219-372: owners first, then waiters, per row in FIFO order) ahead of the
// epoch's requests: request i is pseudo-txn n + i, so it is never a duplicate
// and has no output slot.
template <typename K>
__global__ __launch_bounds__(256) void k_cv_layout_held(const uint64_t* __restrict__ hkeys,
                                                        const uint8_t* __restrict__ hat, uint64_t nh,
                                                        uint32_t n, KeyPack kp, K* __restrict__ ak,
                                                        uint32_t* __restrict__ av) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= nh) return;
  const uint8_t a = hat[i];
  ak[i] = (K)keypack_apply(kp, hkeys[i]);
  av[i] = ((n + (uint32_t)i) << 7) | ((a != DCC_RD && a != DCC_SCAN) ? 1u : 0u);
}

// ---------------------------------------------------------------- group scan
// Segmented scan over the key-sorted requests.  State of an interval "since
// the last row start" (flag = the interval holds a row start):
//   ft/fpos  first non-dup lock type and its position, lt last one
//   cnt      group boundaries between consecutive non-dup requests
//   ns       group starts inside the interval; gs / pgs the last two
//   gnd      non-dup requests since the last group start (all if ns == 0)
//   nd       non-dup requests
// A de-duplicated request (same row, same txn as its predecessor — a txn's
// requests on one row are adjacent after the stable sort) is neutral.
struct Gs {
  uint32_t flag, ft, lt, fpos, cnt, ns, gs, pgs, gnd, nd;
};

__device__ inline Gs gs_identity() { return Gs{0, CV_NONE, CV_NONE, 0, 0, 0, NOPOS, NOPOS, 0, 0}; }

__device__ inline Gs gs_combine(const Gs& A, const Gs& B) {
  if (B.flag) return B;
  Gs R;
  R.flag = A.flag;
  const bool bnd = A.lt != CV_NONE && B.ft != CV_NONE && (A.lt == CV_EX || B.ft == CV_EX);
  const bool af = A.ft != CV_NONE;
  R.ft = af ? A.ft : B.ft;
  R.fpos = af ? A.fpos : B.fpos;
  R.lt = B.lt != CV_NONE ? B.lt : A.lt;
  R.cnt = A.cnt + B.cnt + (bnd ? 1u : 0u);
  R.ns = A.ns + B.ns + (bnd ? 1u : 0u);
  if (B.ns >= 1) {
    R.gs = B.gs;
    R.gnd = B.gnd;
    R.pgs = B.ns >= 2 ? B.pgs : (bnd ? B.fpos : A.gs);
  } else if (bnd) {
    R.gs = B.fpos;
    R.gnd = B.nd;
    R.pgs = A.gs;
  } else {
    R.gs = A.gs;
    R.gnd = A.gnd + B.nd;
    R.pgs = A.pgs;
  }
  R.nd = A.nd + B.nd;
  return R;
}

template <typename K>
__device__ inline Gs gs_element(uint64_t p, K key, uint32_t val, K pkey, uint32_t pval) {
  const bool start = p == 0 || key != pkey;
  const uint32_t typ = (val & 1u) ? CV_EX : CV_SH;
  if (start) return Gs{1, typ, typ, (uint32_t)p, 0, 1, (uint32_t)p, NOPOS, 1, 1};
  if ((val >> 7) == (pval >> 7)) return gs_identity();  // duplicate row of the same txn
  return Gs{0, typ, typ, (uint32_t)p, 0, 0, NOPOS, NOPOS, 1, 1};
}

struct ScanOut {
  const uint32_t* off;
  uint32_t ulen;    // every txn has this many requests (off[t] = t * ulen), or 0: ragged
  uint32_t n;       // epoch txns: values with txn >= n are the held prefix (no outputs)
  uint32_t* group;  // [nnz] or null
  uint8_t* rc;      // [n]
  uint32_t* pgx;    // [nnz] previous group start per request (waves) or null
  uint32_t* gsx;    // [nnz] own group start per request (waves) or null
  uint32_t* gsize;  // [nnz] group size by start position (waves) or null
  // the one-CU walk (calvin_wave.h) instead of pgx / gsize: gsx holds the own
  // group start | has-previous-group << 31, glast [m] the sorted position of
  // each group's last element (by group start; only groups with a successor)
  uint32_t* glast;
};

// Ordered tree reduction of 256 per-thread states (LDS).
__device__ inline Gs block_reduce_gs(Gs v, Gs* s) {
  s[threadIdx.x] = v;
  __syncthreads();
  for (uint32_t w = 1; w < 256; w <<= 1) {
    if ((threadIdx.x & (2 * w - 1)) == 0) s[threadIdx.x] = gs_combine(s[threadIdx.x], s[threadIdx.x + w]);
    __syncthreads();
  }
  return s[0];
}

// Exclusive scan of 256 per-thread states (Hillis-Steele in LDS).
__device__ inline Gs block_excl_gs(Gs v, Gs* s) {
  s[threadIdx.x] = v;
  __syncthreads();
  for (uint32_t d = 1; d < 256; d <<= 1) {
    Gs r = s[threadIdx.x];
    if (threadIdx.x >= d) r = gs_combine(s[threadIdx.x - d], r);
    __syncthreads();
    s[threadIdx.x] = r;
    __syncthreads();
  }
  const Gs ex = threadIdx.x ? s[threadIdx.x - 1] : gs_identity();
  __syncthreads();
  return ex;
}

// The tile's keys / values staged through LDS with coalesced global loads
// (one padding word per 16, so a thread's 16 consecutive items are read
// bank-conflict free), then each thread takes its run of CV_ITEMS and the
// element before it.
template <typename K>
__device__ inline void load_run(const K* sk, const uint32_t* sv, uint64_t m, K* lk, uint32_t* lv,
                                K* k, uint32_t* v, K& pk, uint32_t& pv) {
  const uint64_t base = (uint64_t)blockIdx.x * CV_TILE;
  for (uint32_t i = threadIdx.x; i < CV_TILE; i += 256) {
    const uint64_t p = base + i;
    const uint32_t li = i + (i >> 4);
    lk[li] = p < m ? sk[p] : (K)0;
    lv[li] = p < m ? sv[p] : 0u;
  }
  __syncthreads();
  const uint32_t b = threadIdx.x * (CV_ITEMS + 1);
#pragma unroll
  for (uint32_t i = 0; i < CV_ITEMS; i++) {
    k[i] = lk[b + i];
    v[i] = lv[b + i];
  }
  if (threadIdx.x) {
    pk = lk[b - 2];  // item 16 * tid - 1 sits at 17 * tid - 2
    pv = lv[b - 2];
  } else {
    pk = base ? sk[base - 1] : (K)0;
    pv = base ? sv[base - 1] : 0u;
  }
}
constexpr uint32_t CV_LDS = CV_TILE + CV_TILE / 16;

template <typename K>
__global__ __launch_bounds__(256) void k_cv_up(const K* __restrict__ sk,
                                               const uint32_t* __restrict__ sv, uint64_t m,
                                               Gs* __restrict__ agg) {
  __shared__ Gs s[256];
  __shared__ K lk[CV_LDS];
  __shared__ uint32_t lv[CV_LDS];
  const uint64_t p0 = (uint64_t)blockIdx.x * CV_TILE + (uint64_t)threadIdx.x * CV_ITEMS;
  K k[CV_ITEMS];
  uint32_t v[CV_ITEMS];
  K pk;
  uint32_t pv;
  load_run(sk, sv, m, lk, lv, k, v, pk, pv);
  Gs acc = gs_identity();
  if (p0 < m) {
#pragma unroll
    for (uint32_t i = 0; i < CV_ITEMS; i++) {
      if (p0 + i < m) acc = gs_combine(acc, gs_element(p0 + i, k[i], v[i], pk, pv));
      pk = k[i];
      pv = v[i];
    }
  }
  const Gs r = block_reduce_gs(acc, s);
  if (threadIdx.x == 0) agg[blockIdx.x] = r;
}

// one workgroup: exclusive scan of the tile aggregates in place; each thread
// folds 16 consecutive aggregates, so one block scan covers 4096 tiles
__global__ __launch_bounds__(256) void k_cv_top(Gs* __restrict__ agg, uint32_t tiles) {
  __shared__ Gs s[256];
  __shared__ Gs s_last;
  Gs carry = gs_identity();
  for (uint32_t c0 = 0; c0 < tiles; c0 += 256 * 16) {
    const uint32_t i0 = c0 + threadIdx.x * 16;
    Gs v = gs_identity();
    for (uint32_t q = 0; q < 16 && i0 + q < tiles; q++) v = gs_combine(v, agg[i0 + q]);
    const Gs ex = block_excl_gs(v, s);
    Gs run = gs_combine(carry, ex);
    for (uint32_t q = 0; q < 16 && i0 + q < tiles; q++) {
      const Gs a = agg[i0 + q];
      agg[i0 + q] = run;
      run = gs_combine(run, a);
    }
    if (threadIdx.x == 255) s_last = gs_combine(ex, v);
    __syncthreads();
    carry = gs_combine(carry, s_last);
    __syncthreads();
  }
}

template <typename K>
__global__ __launch_bounds__(256) void k_cv_down(const K* __restrict__ sk,
                                                 const uint32_t* __restrict__ sv, uint64_t m,
                                                 const Gs* __restrict__ pre, ScanOut o) {
  __shared__ Gs s[256];
  __shared__ K lk[CV_LDS];
  __shared__ uint32_t lv[CV_LDS];
  const uint64_t p0 = (uint64_t)blockIdx.x * CV_TILE + (uint64_t)threadIdx.x * CV_ITEMS;
  K k[CV_ITEMS];
  uint32_t v[CV_ITEMS];
  K pk0 = 0;
  uint32_t pv0 = 0;
  load_run(sk, sv, m, lk, lv, k, v, pk0, pv0);
  Gs acc = gs_identity();
  if (p0 < m) {
    K pk = pk0;
    uint32_t pv = pv0;
#pragma unroll
    for (uint32_t i = 0; i < CV_ITEMS; i++) {
      if (p0 + i < m) acc = gs_combine(acc, gs_element(p0 + i, k[i], v[i], pk, pv));
      pk = k[i];
      pv = v[i];
    }
  }
  Gs run = gs_combine(pre[blockIdx.x], block_excl_gs(acc, s));
  if (p0 >= m) return;
  // group of each request, straight to its place in request order (a random
  // 4-B scatter: measured no slower than partitioning by destination first
  // and placing window by window, profiles/r02/calvin_*)
  // every request's txn offset first, all in flight together (a dependent
  // random load per item inside the loop serialised 16 round trips)
  uint32_t xo[CV_ITEMS];
#pragma unroll
  for (uint32_t i = 0; i < CV_ITEMS; i++) {
    const uint32_t t = v[i] >> 7;
    xo[i] = (p0 + i < m && t < o.n) ? (o.ulen ? t * o.ulen : o.off[t]) : 0u;
  }
  K pk = pk0;
  uint32_t pv = pv0;
  uint32_t last_gs = NOPOS, last_gnd = 0;
#pragma unroll
  for (uint32_t i = 0; i < CV_ITEMS; i++) {
    if (p0 + i >= m) break;
    const uint64_t p = p0 + i;
    const Gs e = gs_element(p, k[i], v[i], pk, pv);
    const bool dup = !e.flag && e.ft == CV_NONE;
    run = gs_combine(run, e);
    pk = k[i];
    pv = v[i];
    const uint32_t t = v[i] >> 7, j = (v[i] >> 1) & 63u;
    if (t >= o.n) continue;  // held-prefix request: part of the scan only (no waves)
    const uint32_t x = xo[i] + j;
    if (dup) {
      o.group[x] = DCC_GROUP_NONE;
      if (o.gsx) o.gsx[x] = NOPOS;
      if (o.pgx) o.pgx[x] = NOPOS;
      continue;
    }
    o.group[x] = run.cnt;
    if (o.glast) {
      o.gsx[x] = run.gs | (run.cnt ? 0x80000000u : 0u);
      if (run.cnt && run.gs == (uint32_t)p) o.glast[run.pgs] = (uint32_t)p - 1u;
    } else if (o.pgx) {
      o.pgx[x] = run.cnt ? run.pgs : NOPOS;
      o.gsx[x] = run.gs;
      if (last_gs != NOPOS && last_gs != run.gs) atomicMax(&o.gsize[last_gs], last_gnd);
      last_gs = run.gs;
      last_gnd = run.gnd;
    }
  }
  if (o.gsize && last_gs != NOPOS) atomicMax(&o.gsize[last_gs], last_gnd);
}

// ---- the same scan when no wave levels are asked for: only the grant group
// count is needed, so the state packs into one word (calvin_gl.h) and the
// block scans are wave shuffles instead of 10-word LDS trees.  Same monoid as
// Gs restricted to (flag, ft, lt, cnt).
template <typename K>
__device__ inline uint32_t gl_element(uint64_t p, K key, uint32_t val, K pkey, uint32_t pval) {
  const bool start = p == 0 || key != pkey;
  const uint32_t typ = (val & 1u) ? CV_EX : CV_SH;
  if (start) return gl_pack(1, typ, typ, 0);
  if ((val >> 7) == (pval >> 7)) return GL_ID;  // duplicate row of the same txn
  return gl_pack(0, typ, typ, 0);
}
template <typename K>
__global__ __launch_bounds__(256) void k_cv_up_l(const K* __restrict__ sk,
                                                 const uint32_t* __restrict__ sv, uint64_t m,
                                                 uint32_t* __restrict__ agg, uint32_t dshift,
                                                 uint32_t* __restrict__ hcnt) {
  __shared__ uint32_t s_w[4];
  __shared__ uint32_t s_h[256];
  __shared__ K lk[CV_LDS];
  __shared__ uint32_t lv[CV_LDS];
  const uint64_t p0 = (uint64_t)blockIdx.x * CV_TILE + (uint64_t)threadIdx.x * CV_ITEMS;
  K k[CV_ITEMS];
  uint32_t v[CV_ITEMS];
  K pk;
  uint32_t pv;
  load_run(sk, sv, m, lk, lv, k, v, pk, pv);
  uint32_t acc = GL_ID;
  if (p0 < m) {
#pragma unroll
    for (uint32_t i = 0; i < CV_ITEMS; i++) {
      if (p0 + i < m) acc = gl_combine(acc, gl_element(p0 + i, k[i], v[i], pk, pv));
      pk = k[i];
      pv = v[i];
    }
  }
  uint32_t total;
  (void)gl_block_excl(acc, s_w, total);
  if (threadIdx.x == 0) agg[blockIdx.x] = total;
  if (hcnt) {  // the tile's counts of the write-out partition digit (txn's top bits)
    s_h[threadIdx.x] = 0;
    __syncthreads();
#pragma unroll
    for (uint32_t i = 0; i < CV_ITEMS; i++)
      if (p0 + i < m) atomicAdd(&s_h[(v[i] >> dshift) & 255u], 1u);
    __syncthreads();
    hcnt[(uint64_t)threadIdx.x * gridDim.x + blockIdx.x] = s_h[threadIdx.x];
  }
}

// one workgroup: exclusive scan of the tile aggregates in place (16 per thread)
__global__ __launch_bounds__(256) void k_cv_top_l(uint32_t* __restrict__ agg, uint32_t tiles) {
  __shared__ uint32_t s_w[4];
  uint32_t carry = GL_ID;
  for (uint32_t c0 = 0; c0 < tiles; c0 += 256 * 16) {
    const uint32_t i0 = c0 + threadIdx.x * 16;
    uint32_t a[16], v = GL_ID;
#pragma unroll
    for (uint32_t q = 0; q < 16; q++) {
      a[q] = i0 + q < tiles ? agg[i0 + q] : GL_ID;
      v = gl_combine(v, a[q]);
    }
    uint32_t total;
    uint32_t run = gl_combine(carry, gl_block_excl(v, s_w, total));
#pragma unroll
    for (uint32_t q = 0; q < 16; q++) {
      if (i0 + q < tiles) agg[i0 + q] = run;
      run = gl_combine(run, a[q]);
    }
    carry = gl_combine(carry, total);
  }
}

// The windowed put's partition, written by the scan itself: (value, group)
// pairs into 256 buckets of the txn's top bits (the order inside a bucket is
// free: every pair carries its destination); hcnt holds the per-digit
// exclusive prefix over tiles (k_cv_up_l's counts, scanned), tot the digit
// totals.
struct PartOut {
  uint32_t dshift;
  const uint32_t* hcnt;
  const uint32_t* tot;
  uint32_t* ko;
  uint32_t* go;
};

template <typename K>
__global__ __launch_bounds__(256) void k_cv_down_l(const K* __restrict__ sk,
                                                   const uint32_t* __restrict__ sv, uint64_t m,
                                                   const uint32_t* __restrict__ pre, ScanOut o,
                                                   PartOut po) {
  __shared__ uint32_t s_w[4];
  __shared__ uint32_t s_tb[256], s_gb[256], s_run[256];
  __shared__ K lk[CV_LDS];
  __shared__ uint32_t lv[CV_LDS];
  const uint64_t p0 = (uint64_t)blockIdx.x * CV_TILE + (uint64_t)threadIdx.x * CV_ITEMS;
  K k[CV_ITEMS];
  uint32_t v[CV_ITEMS];
  K pk0 = 0;
  uint32_t pv0 = 0;
  load_run(sk, sv, m, lk, lv, k, v, pk0, pv0);
  uint32_t acc = GL_ID;
  if (p0 < m) {
    K pk = pk0;
    uint32_t pv = pv0;
#pragma unroll
    for (uint32_t i = 0; i < CV_ITEMS; i++) {
      if (p0 + i < m) acc = gl_combine(acc, gl_element(p0 + i, k[i], v[i], pk, pv));
      pk = k[i];
      pv = v[i];
    }
  }
  uint32_t total;
  uint32_t run = gl_combine(pre[blockIdx.x], gl_block_excl(acc, s_w, total));
  if (po.ko) {
    // (1) per digit: the tile's count (LDS), its tile-local base (scan over
    // digits) and its global base (digit totals before it + this tile's
    // prefix among the tiles)
    const uint32_t tid = threadIdx.x;
    s_run[tid] = 0;
    __syncthreads();
    uint32_t g[CV_ITEMS], dg[CV_ITEMS];
    {
      K pk = pk0;
      uint32_t pv = pv0;
#pragma unroll
      for (uint32_t i = 0; i < CV_ITEMS; i++) {
        g[i] = 0;
        dg[i] = (v[i] >> po.dshift) & 255u;
        if (p0 + i < m) {
          const uint32_t e = gl_element(p0 + i, k[i], v[i], pk, pv);
          run = gl_combine(run, e);
          g[i] = e == GL_ID ? DCC_GROUP_NONE : run >> 5;
          atomicAdd(&s_run[dg[i]], 1u);
        }
        pk = k[i];
        pv = v[i];
      }
    }
    __syncthreads();
    {
      const uint32_t c = s_run[tid], t = po.tot[tid];
      uint32_t x = c, y = t;  // inclusive wave scans of the tile counts and the totals
#pragma unroll
      for (uint32_t d = 1; d < 64; d <<= 1) {
        const uint32_t xu = __shfl_up(x, d), yu = __shfl_up(y, d);
        if ((tid & 63u) >= d) {
          x += xu;
          y += yu;
        }
      }
      __shared__ uint32_t s_wx[4], s_wy[4];
      if ((tid & 63u) == 63u) {
        s_wx[tid >> 6] = x;
        s_wy[tid >> 6] = y;
      }
      __syncthreads();
      uint32_t bx = 0, by = 0;
      for (uint32_t w = 0; w < (tid >> 6); w++) {
        bx += s_wx[w];
        by += s_wy[w];
      }
      s_tb[tid] = bx + x - c;
      s_gb[tid] = by + y - t + po.hcnt[(uint64_t)tid * gridDim.x + blockIdx.x];
      s_run[tid] = bx + x - c;
    }
    __syncthreads();
    // (2) the tile's pairs in digit order through LDS (any order within a digit)
    uint32_t* lvv = lv;
    uint32_t* lgg = (uint32_t*)lk;
#pragma unroll
    for (uint32_t i = 0; i < CV_ITEMS; i++)
      if (p0 + i < m) {
        const uint32_t q = atomicAdd(&s_run[dg[i]], 1u);
        lvv[q] = v[i];
        lgg[q] = g[i];
      }
    __syncthreads();
    // (3) coalesced runs per digit
    const uint64_t base = (uint64_t)blockIdx.x * CV_TILE;
    const uint32_t n_here = (uint32_t)min<uint64_t>(CV_TILE, m - base);
    for (uint32_t j = tid; j < n_here; j += 256) {
      const uint32_t vv = lvv[j], d = (vv >> po.dshift) & 255u;
      const uint32_t dst = s_gb[d] + (j - s_tb[d]);
      po.ko[dst] = vv;
      po.go[dst] = lgg[j];
    }
    return;
  }
  if (p0 >= m) return;
  uint32_t xo[CV_ITEMS];
#pragma unroll
  for (uint32_t i = 0; i < CV_ITEMS; i++) {
    const uint32_t t = v[i] >> 7;
    xo[i] = (p0 + i < m && t < o.n) ? (o.ulen ? t * o.ulen : o.off[t]) : 0u;
  }
  K pk = pk0;
  uint32_t pv = pv0;
#pragma unroll
  for (uint32_t i = 0; i < CV_ITEMS; i++) {
    if (p0 + i >= m) break;
    const uint32_t e = gl_element(p0 + i, k[i], v[i], pk, pv);
    run = gl_combine(run, e);
    pk = k[i];
    pv = v[i];
    const uint32_t t = v[i] >> 7, j = (v[i] >> 1) & 63u;
    if (t >= o.n) continue;  // held-prefix request: part of the scan only
    o.group[xo[i] + j] = e == GL_ID ? DCC_GROUP_NONE : run >> 5;
  }
}

// The windowed group write-out (uniform request counts, large epochs).  The
// direct store from k_cv_down_l puts each request's group at a random place:
// one 32-B sector write per 4-B store (PMC: 521 MB written for 67 MB).
// Instead k_cv_down_l writes the (value, group) pairs already partitioned by
// the txn's top 8 bits (bucket offsets from k_cv_up_l's per-tile digit counts
// scanned by rs_scan_rows), and each workgroup here owns
// a window of the group array (a bucket's requests are contiguous there):
// it places its bucket's groups into the window in LDS and stores the window
// with coalesced stores.
constexpr uint32_t CV_WIN = 40448;  // u32 window per workgroup (158 KiB of LDS)
__global__ __launch_bounds__(1024) void k_cv_put(const uint32_t* __restrict__ sv,
                                                 const uint32_t* __restrict__ sg,
                                                 const uint32_t* __restrict__ tot, uint32_t n,
                                                 uint32_t ulen, uint32_t tsh, uint32_t H,
                                                 uint32_t wh, uint32_t* __restrict__ group) {
  __shared__ uint32_t win[CV_WIN];
  __shared__ uint32_t s_rng[2];
  const uint32_t bkt = blockIdx.x / H, h = blockIdx.x % H;
  const uint64_t t_lo = (uint64_t)bkt << tsh;
  if (t_lo >= n) return;  // whole workgroup
  const uint64_t d_lo = t_lo * ulen + (uint64_t)h * wh;
  const uint64_t d_end = min<uint64_t>(t_lo + (1ull << tsh), n) * ulen;
  if (d_lo >= d_end) return;  // whole workgroup
  const uint32_t w = (uint32_t)min<uint64_t>(wh, d_end - d_lo);
  // the bucket's pairs: the digit totals before it (bucket order)
  if (threadIdx.x < 2) s_rng[threadIdx.x] = 0;
  __syncthreads();
  if (threadIdx.x < bkt) atomicAdd(&s_rng[0], tot[threadIdx.x]);
  if (threadIdx.x == bkt) s_rng[1] = tot[bkt];
  __syncthreads();
  const uint32_t p_lo = s_rng[0], p_hi = s_rng[0] + s_rng[1];
  constexpr uint32_t U = 8;  // pairs in flight per thread
  for (uint32_t p0 = p_lo + threadIdx.x; p0 < p_hi; p0 += 1024 * U) {
    uint32_t vv[U], gg[U];
#pragma unroll
    for (uint32_t u = 0; u < U; u++) {
      const uint32_t p = p0 + u * 1024;
      vv[u] = p < p_hi ? sv[p] : 0xFFFFFFFFu;  // txn 2^25 - 1 >= n: skipped
      gg[u] = p < p_hi ? sg[p] : 0u;
    }
#pragma unroll
    for (uint32_t u = 0; u < U; u++) {
      const uint32_t t = vv[u] >> 7;
      if (t >= n) continue;  // held-prefix request (or past the bucket)
      const uint64_t x = (uint64_t)t * ulen + ((vv[u] >> 1) & 63u);
      if (x >= d_lo && x < d_lo + w) win[x - d_lo] = gg[u];
    }
  }
  __syncthreads();
  for (uint32_t i = threadIdx.x; i < w; i += 1024) group[d_lo + i] = win[i];
}

// acquire_locks' return (ycsb_txn.cpp:76-79): RCOK iff every request of the
// txn is in group 0.  One wave per 64 txns walks their contiguous requests.
__global__ __launch_bounds__(256) void k_cv_ready(const uint32_t* __restrict__ off, uint64_t n,
                                                  const uint32_t* __restrict__ group,
                                                  uint8_t* __restrict__ rc) {
  __shared__ uint32_t s_o[4][65];
  __shared__ uint32_t s_w[4][64];
  const uint32_t lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const uint64_t t0 = ((uint64_t)blockIdx.x * 4 + w) * 64;
  if (t0 >= n) return;
  const uint64_t t = t0 + lane;
  const uint64_t tl = min<uint64_t>(n, t0 + 64);
  s_o[w][lane] = off[min(t, tl)];
  if (lane == 0) s_o[w][64] = off[tl];
  s_w[w][lane] = 0;
  __builtin_amdgcn_wave_barrier();
  const uint32_t a0 = s_o[w][0], a1 = s_o[w][64];
  for (uint32_t x = a0 + lane; x < a1; x += 64) {
    const uint32_t g = group[x];
    if (g == 0 || g == DCC_GROUP_NONE) continue;
    uint32_t lo = 0, hi = 64;  // largest k with s_o[k] <= x
    while (hi - lo > 1) {
      const uint32_t mid = (lo + hi) >> 1;
      if (s_o[w][mid] <= x) lo = mid;
      else hi = mid;
    }
    s_w[w][lo] = 1;
  }
  __builtin_amdgcn_wave_barrier();
  if (t < n) rc[t] = s_w[w][lane] ? DCC_RC_WAIT : DCC_RC_RCOK;
}

// ---------------------------------------------------------------- waves
// Dependency-driven wave levels.  Wave w of the persistent grid takes the
// sequence positions w, w+W, ... in order; lanes are the txn's requests.  A
// request in group g > 0 waits until every member of the row's previous
// group has published (done == size), then the txn's level is 1 + the max
// published level over those groups; it publishes max(level) into its own
// groups and counts itself done.  Every dependency is an earlier sequence
// position, every wave owns at most one unfinished position and the grid is
// co-resident, so the earliest unfinished position always progresses.  Spins
// are bounded by a wall-clock budget; on expiry the error word is raised.
struct WaveArgs {
  uint64_t n;
  const uint32_t* seq;  // or null (index order)
  const uint32_t* off;
  const uint32_t* pgx;
  const uint32_t* gsx;
  const uint32_t* gsize;
  uint32_t* done;
  uint32_t* maxl;
  uint32_t* wave;
  uint32_t* err;
  uint64_t budget;  // s_memrealtime ticks (100 MHz)
};

__global__ __launch_bounds__(256) void k_cv_wave(WaveArgs a) {
  const uint32_t lane = lane_id();
  const uint64_t W = (uint64_t)gridDim.x * (blockDim.x >> 6);
  const uint64_t w = (uint64_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
  const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
  bool expired = false;
  for (uint64_t q = w; q < a.n; q += W) {
    const uint32_t t = a.seq ? a.seq[q] : (uint32_t)q;
    const uint32_t s = a.off[t], len = a.off[t + 1] - s;
    const bool act = lane < len;
    const uint32_t pg = act ? a.pgx[s + lane] : NOPOS;
    const uint32_t g = act ? a.gsx[s + lane] : NOPOS;
    const uint32_t need = pg != NOPOS ? a.gsize[pg] : 0u;
    uint32_t lvl = 0;
    if (ballot64(pg != NOPOS)) {
      bool ok = pg == NOPOS;
      while (!expired) {
        if (!ok) ok = __hip_atomic_load(&a.done[pg], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) >= need;
        if (ballot64(!ok) == 0) break;
        __builtin_amdgcn_s_sleep(1);
        if (__builtin_amdgcn_s_memrealtime() - t0 > a.budget) expired = true;
      }
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      if (pg != NOPOS)
        lvl = __hip_atomic_load(&a.maxl[pg], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) + 1u;
      for (int d = 32; d > 0; d >>= 1) lvl = max(lvl, (uint32_t)__shfl_xor(lvl, d));
    }
    if (g != NOPOS) __hip_atomic_fetch_max(&a.maxl[g], lvl, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    if (g != NOPOS) __hip_atomic_fetch_add(&a.done[g], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (lane == 0) a.wave[t] = lvl;
  }
  if (expired && lane == 0) atomicOr(a.err, ERR_WAVE_TIMEOUT);
}

// ---------------------------------------------------------------- counts
struct CvCount {
  uint32_t ready, maxwave, pad0, pad1;
};
__global__ __launch_bounds__(256) void k_cv_count(const uint8_t* __restrict__ rc,
                                                  const uint32_t* __restrict__ wave, uint64_t n,
                                                  CvCount* __restrict__ part) {
  __shared__ uint32_t s[2][4];
  uint32_t r = 0, mw = 0;
  const uint64_t tid = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  for (uint64_t t = tid; t < n; t += (uint64_t)gridDim.x * blockDim.x) {
    r += rc[t] == DCC_RC_RCOK;
    if (wave) mw = max(mw, wave[t]);
  }
  for (int d = 32; d > 0; d >>= 1) {
    r += __shfl_xor(r, d);
    mw = max(mw, (uint32_t)__shfl_xor(mw, d));
  }
  if ((threadIdx.x & 63) == 0) {
    s[0][threadIdx.x >> 6] = r;
    s[1][threadIdx.x >> 6] = mw;
  }
  __syncthreads();
  if (threadIdx.x == 0)
    part[blockIdx.x] = CvCount{s[0][0] + s[0][1] + s[0][2] + s[0][3],
                               max(max(s[1][0], s[1][1]), max(s[1][2], s[1][3])), 0, 0};
}

inline unsigned grid1(uint64_t n, unsigned b) {
  const uint64_t g = (n + b - 1) / b;
  return (unsigned)(g ? g : 1);
}

}  // namespace

// ---------------------------------------------------------------- driver
template <typename K>
static int calvin_sort_and_scan(dcc_ctx* ctx, const DevBatch& d, const uint32_t* seq,
                                const uint32_t* off2, const KeyPack& kp, const ScanOut& so,
                                const uint64_t* hkeys, const uint8_t* hat, uint64_t nh,
                                bool prof, const uint32_t** sv_out) {
  const uint64_t m = nh + d.nnz;
  hipStream_t st = ctx->stream;
  CR(ctx->calvin_a.ensure(ctx, std::max<uint64_t>(16, m * sizeof(K)), "calvin keys a"));
  CR(ctx->calvin_b.ensure(ctx, std::max<uint64_t>(16, m * sizeof(K)), "calvin keys b"));
  CR(ctx->calvin_c.ensure(ctx, std::max<uint64_t>(16, m * 4), "calvin vals a"));
  CR(ctx->calvin_d.ensure(ctx, std::max<uint64_t>(16, m * 4), "calvin vals b"));
  const uint64_t tiles = (m + CV_TILE - 1) / CV_TILE;
  // the radix passes' counts, or the scan's write-out partition counts
  // ([256][tiles] + 256 totals)
  CR(ctx->cv_scratch.ensure(ctx, std::max<uint64_t>(rs_scratch_words(m), 256 * (tiles + 1)) * 4 + 64,
                            "radix scratch"));
  CR(ctx->cv_agg.ensure(ctx, std::max<uint64_t>(1, tiles) * sizeof(Gs), "calvin scan"));
  K* kb[2] = {(K*)ctx->calvin_a.p, (K*)ctx->calvin_b.p};
  uint32_t* vb[2] = {(uint32_t*)ctx->calvin_c.p, (uint32_t*)ctx->calvin_d.p};
  if (nh)
    k_cv_layout_held<K><<<grid1(nh, 256), 256, 0, st>>>(hkeys, hat, nh, (uint32_t)d.n, kp, kb[0],
                                                         vb[0]);
  k_cv_layout<K><<<grid1(d.n, 256), 256, 0, st>>>(d.off, seq, off2, d.n, d.keys, d.acctype, kp,
                                                  (uint32_t)nh, so.ulen, kb[0], vb[0]);  // 4 waves x 64
  if (prof) CK(hipEventRecord(ctx->pev[1], st));
  int cur;
  if (sizeof(K) == 4)
    cur = radix_sort_u32((uint32_t**)kb, vb, m, kp.bits, (uint32_t*)ctx->cv_scratch.p, st);
  else
    cur = radix_sort_u64((uint64_t**)kb, vb, m, kp.bits, (uint32_t*)ctx->cv_scratch.p, st);
  if (prof) CK(hipEventRecord(ctx->pev[2], st));
  *sv_out = vb[cur];
  if (so.gsx) {  // wave levels: the full scan state
    Gs* agg = (Gs*)ctx->cv_agg.p;
    k_cv_up<K><<<(unsigned)tiles, 256, 0, st>>>(kb[cur], vb[cur], m, agg);
    k_cv_top<<<1, 256, 0, st>>>(agg, (uint32_t)tiles);
    k_cv_down<K><<<(unsigned)tiles, 256, 0, st>>>(kb[cur], vb[cur], m, agg, so);
  } else {  // grant groups only: the one-word state
    uint32_t* agg = (uint32_t*)ctx->cv_agg.p;
    const bool put = so.ulen && d.nnz >= CV_PUT_MIN;
    const uint64_t tmax = d.n + nh - 1;
    const uint32_t tb = tmax ? 64u - (uint32_t)__builtin_clzll(tmax) : 1u;
    const uint32_t tsh = tb > 8 ? tb - 8 : 0;
    uint32_t* hcnt = (uint32_t*)ctx->cv_scratch.p;
    uint32_t* htot = hcnt + 256 * tiles;
    k_cv_up_l<K><<<(unsigned)tiles, 256, 0, st>>>(kb[cur], vb[cur], m, agg, 7 + tsh,
                                                  put ? hcnt : nullptr);
    k_cv_top_l<<<1, 256, 0, st>>>(agg, (uint32_t)tiles);
    if (put) {
      // the scan writes (value, group) pairs straight into 256 buckets of the
      // txn's top 8 bits (counted by the up pass); the windowed put places
      // each bucket's groups in request order
      rs_scan_rows(hcnt, 256, (uint32_t)tiles, htot, st);
      uint32_t* ko = (uint32_t*)kb[1 - cur];
      uint32_t* go = vb[1 - cur];
      k_cv_down_l<K><<<(unsigned)tiles, 256, 0, st>>>(kb[cur], vb[cur], m, agg, so,
                                                      PartOut{7 + tsh, hcnt, htot, ko, go});
      const uint64_t span = (1ull << tsh) * so.ulen;
      const uint32_t H = (uint32_t)((span + CV_WIN - 1) / CV_WIN);
      const uint32_t wh = (uint32_t)((span + H - 1) / H);
      k_cv_put<<<256 * H, 1024, 0, st>>>(ko, go, htot, (uint32_t)d.n, so.ulen, tsh, H, wh, so.group);
    } else {
      k_cv_down_l<K><<<(unsigned)tiles, 256, 0, st>>>(kb[cur], vb[cur], m, agg, so,
                                                      PartOut{0, nullptr, nullptr, nullptr, nullptr});
    }
  }
  CK(hipGetLastError());
  return DCC_OK;
}

int dcc_ctx::calvin_epoch(const dcc_batch* b, const dcc_calvin_held* held, uint32_t* out_group,
                          uint8_t* out_rc, uint32_t* out_wave, dcc_stats* st) {
  dcc_ctx* ctx = this;
  const auto t_wall0 = std::chrono::steady_clock::now();
  CR(check_batch(b));
  const bool dev_out = (b->flags & DCC_DEVICE_PTRS) != 0;
  dcc_stats S;
  memset(&S, 0, sizeof S);
  S.n_shards = (uint32_t)comm_ranks();
  if (b->n_txn == 0) {
    if (st) *st = S;
    return DCC_OK;
  }
  if (out_wave && comm_ranks() > 1)
    return fail(DCC_ENOTSUP, "calvin: wave levels need the whole epoch on one GPU");
  const uint64_t nh = held ? held->n : 0;
  if (nh && (!held->keys || !held->acctype)) return fail(DCC_EINVAL, "calvin: null held arrays");
  if (nh && out_wave)
    return fail(DCC_ENOTSUP, "calvin: wave levels need an empty lock table (no held prefix)");
  if (b->n_txn + nh >= CV_MAX_TXN)
    return fail(DCC_ERANGE, "calvin: n_txn + held %llu exceeds %u per epoch",
                (unsigned long long)(b->n_txn + nh), CV_MAX_TXN - 1);
  if (b->nnz + nh >= 0xFFFFFFFFull) return fail(DCC_ERANGE, "calvin: requests exceed 2^32-1");
  DevBatch d;
  CR(stage_batch(b, d));
  // the held prefix: device arrays alongside a device batch, else uploaded
  const uint64_t* hkeys = nullptr;
  const uint8_t* hat = nullptr;
  if (nh) {
    if (dev_out) {
      hkeys = held->keys;
      hat = held->acctype;
    } else {
      CR(cv_hkeys.ensure(this, nh * 8, "calvin held keys"));
      CR(cv_hat.ensure(this, nh, "calvin held types"));
      CK(hipMemcpyAsync(cv_hkeys.p, held->keys, nh * 8, hipMemcpyHostToDevice, stream));
      CK(hipMemcpyAsync(cv_hat.p, held->acctype, nh, hipMemcpyHostToDevice, stream));
      hkeys = (const uint64_t*)cv_hkeys.p;
      hat = (const uint8_t*)cv_hat.p;
    }
  }
  // ---- outputs / workspaces (they depend on the shape only)
  CR(rc.ensure(this, d.n + 16, "rc"));
  uint8_t* rc_dev = (dev_out && out_rc) ? out_rc : (uint8_t*)rc.p;
  // groups are always produced (readiness is derived from them)
  uint32_t* grp_dev = nullptr;
  if (out_group && dev_out) {
    grp_dev = out_group;
  } else {
    CR(cv_group.ensure(this, std::max<uint64_t>(16, d.nnz * 4), "calvin group"));
    grp_dev = (uint32_t*)cv_group.p;
  }
  const bool waves = out_wave != nullptr;
  uint32_t* err = (uint32_t*)misc.p;
  const bool cv_graph_ok = !profiling && !waves && nh == 0 && !sharded() &&
                           !DCC_ENV("DCC_NO_GRAPH");
  CvGraphKey gk;
  memset(&gk, 0, sizeof gk);
  gk.off = d.off;
  gk.keys = d.keys;
  gk.acc = d.acctype;
  gk.order = d.order;
  gk.grp = grp_dev;
  gk.rc = rc_dev;
  gk.n = d.n;
  gk.nnz = d.nnz;
  gk.gen = buf_gen;

  CK(hipEventRecord(ev0, stream));
  if (profiling) CK(hipEventRecord(pev[0], stream));

  // ---- prep: offsets/length validation + which key / order bits vary
  CvPart* cvp = (CvPart*)((char*)part.p + 16384);
  k_cv_prep<<<CV_PREP_BLOCKS + PREP_BLOCKS, 256, 0, stream>>>(d.keys, d.nnz, d.acctype, d.order, d.n,
                                                              hkeys, nh, cvp, d.off, (PrepPart*)part.p);
  CK(hipGetLastError());
  CK(hipMemcpyAsync(hpart, part.p, 16384 + CV_PREP_BLOCKS * sizeof(CvPart), hipMemcpyDeviceToHost,
                    stream));
  // The rest of the epoch reads the prep's results (key / order packings, the
  // plan) as launch constants, so it would wait for a host round trip.  When
  // this batch shape already has a captured graph, the graph is launched
  // right behind the prep on the results it was captured with -- a
  // speculation the host checks once the epoch is done: the epoch is redone
  // (from the prep results already read) if they changed.  A stable key
  // universe and sequencer keep them equal from epoch to epoch.
  auto same_shape = [&](const CvGraphKey& k) {
    return k.off == gk.off && k.keys == gk.keys && k.acc == gk.acc && k.order == gk.order &&
           k.grp == gk.grp && k.rc == gk.rc && k.n == gk.n && k.nnz == gk.nnz && k.gen == gk.gen;
  };
  // (only a bucket-path graph: it never reads the offsets, which the prep
  // is still validating, so a malformed batch cannot steer its accesses)
  // (uniform txns only: the ragged form reads the offsets)
  const bool spec = cv_graph_ok && cv_graph_exec && cv_graph_key.bucket && cv_graph_key.ulen &&
                    same_shape(cv_graph_key);
  // the tail of every epoch: device clock, outputs to the host, counts
  auto enqueue_tail = [&](const uint32_t* wave_dev) -> int {
    CK(hipEventRecord(ev1, stream));
    if (!dev_out) {
      if (out_rc) CK(hipMemcpyAsync(out_rc, rc_dev, d.n, hipMemcpyDeviceToHost, stream));
      if (out_group && d.nnz)
        CK(hipMemcpyAsync(out_group, grp_dev, d.nnz * 4, hipMemcpyDeviceToHost, stream));
      if (waves) CK(hipMemcpyAsync(out_wave, wave_dev, d.n * 4, hipMemcpyDeviceToHost, stream));
    }
    CK(hipMemcpyAsync(hmisc, misc.p, 64, hipMemcpyDeviceToHost, stream));
    CK(hipMemcpyAsync((char*)hpart + CV_COUNT_OFF, (char*)part.p + CV_COUNT_OFF,
                      CV_PREP_BLOCKS * sizeof(CvCount), hipMemcpyDeviceToHost, stream));
    CK(hipStreamSynchronize(stream));
    return DCC_OK;
  };
  if (spec) {
    CK(hipGraphLaunch(cv_graph_exec, stream));
    CR(enqueue_tail(nullptr));
  } else {
    CK(hipStreamSynchronize(stream));
  }
  uint32_t maxlen = 0, perr = 0, unsorted = 0;
  uint64_t kor = 0, kand = ~0ull, oor = 0, oand = ~0ull, nex = 0;
  {
    const PrepPart* pp = (const PrepPart*)hpart;
    for (unsigned q = 0; q < PREP_BLOCKS; q++) {
      perr |= pp[q].err;
      maxlen = std::max(maxlen, pp[q].maxlen);
    }
    const CvPart* cp = (const CvPart*)((const char*)hpart + 16384);
    for (unsigned q = 0; q < CV_PREP_BLOCKS; q++) {
      kor |= cp[q].kor;
      kand &= cp[q].kand;
      oor |= cp[q].oor;
      oand &= cp[q].oand;
      nex += cp[q].nex;
      unsorted += cp[q].unsorted;
    }
  }
  if (perr & ERR_OFFSETS) return fail(DCC_EINVAL, "batch: malformed offsets");
  if (maxlen > MAX_TXN_LEN)
    return fail(DCC_ERANGE, "batch: a txn has %u accesses (> MAX_ROW_PER_TXN=%u)", maxlen,
                MAX_TXN_LEN);
  const KeyPack kp = make_keypack(d.nnz + nh ? (kor ^ kand) : 0);
  // uniform txn length (YCSB's fixed request count): a request's place in
  // request order is t * len + j, no offset lookup per request
  const uint32_t ulen = (maxlen && d.nnz == (uint64_t)d.n * maxlen) ? maxlen : 0u;
  // a varying order that is already non-decreasing ranks as the identity
  const bool have_seq = d.order && (oor ^ oand) && unsorted != 0;
  const KeyPack op = have_seq ? make_keypack(oor ^ oand) : KeyPack{};
  static_assert(sizeof(KeyPack) <= sizeof(CvGraphKey::kp), "key image");
  // the bucket path (calvin_bucket.h) for large epochs, uniform or ragged
  // txns (TPC-C, a key-sharded rank's share of YCSB);
  // DCC_OPT_CALVIN_PATH: 1 keeps the global sort + scan, 2 takes the bucket
  // path at every size it applies to (0: the bucket path on large epochs)
  const int cb_mode = cv_path == 1 ? 0 : cv_path == 2 ? 1 : -1;
  CbPlan cbp{};
  // The hashed carry table (packed keys of 25-28 bits) only when asked for
  // (DCC_OPT_CALVIN_PATH 2) and unless an epoch of this context overflowed
  // one: on TPC-C (28 bits at 128 warehouses, 262,144 txns) it measured
  // 0.82 ms against the sort path's 0.28 (tools/calvin_tpcc_probe.py)
  const bool use_cb = d.nnz && cb_mode != 0 && !waves && nh == 0 &&
                      (cb_mode == 1 || d.nnz >= CV_PUT_MIN) && cb_plan(d.n, d.nnz, ulen, maxlen, kp.bits, &cbp) &&
                      !(cbp.hashed && (cb_hash_off || cb_mode != 1));
  gk.ulen = ulen;
  gk.have_seq = have_seq ? 1u : 0u;
  gk.bucket = use_cb ? 1u : 0u;
  memcpy(gk.kp, &kp, sizeof kp);
  memcpy(gk.op, &op, sizeof op);
  cv_last_sorted = d.order && !have_seq;
  cv_last_bucket = use_cb;
  uint32_t* wave_dev = nullptr;
  if (!(spec && !memcmp(&gk, &cv_graph_key, sizeof gk))) {
  cv_spec_miss += spec ? 1 : 0;
  ScanOut so{d.off, ulen, (uint32_t)d.n, grp_dev, rc_dev, nullptr, nullptr, nullptr, nullptr};
  const uint32_t* sv = nullptr;  // the sorted request values (waves)
  // wave levels: the one-CU walk for txns of at most CW_LMAX requests, the
  // dataflow grid (k_cv_wave) for longer ones
  CwPlan cwp{};
  const bool cw = waves && !DCC_ENV("DCC_CV_WAVE_GRID") && cw_plan(d.n, maxlen, &cwp);
  const uint32_t cw_nh = cw && cwp.nch > 2 ? cw_helpers(n_cu) : 0u;
  if (waves) {
    if (dev_out) {
      wave_dev = out_wave;
    } else {
      CR(cv_wave.ensure(this, d.n * 4 + 16, "calvin wave"));
      wave_dev = (uint32_t*)cv_wave.p;
    }
    const uint64_t m = std::max<uint64_t>(16, d.nnz * 4);
    CR(cv_gsx.ensure(this, m, "calvin gsx"));
    so.gsx = (uint32_t*)cv_gsx.p;
    if (cw) {
      CR(cv_pgx.ensure(this, m, "calvin group last"));
      CK(hipMemsetAsync(cv_pgx.p, 0xFF, m, stream));
      so.glast = (uint32_t*)cv_pgx.p;
      const uint64_t sb = std::max<uint64_t>(16, cwp.slots * 4);
      CR(cv_gsize.ensure(this, sb, "calvin wave records"));
      CR(cv_done.ensure(this, sb, "calvin wave previous"));
      CR(cv_maxl.ensure(this, sb, "calvin wave own"));
      CR(cv_cwmax.ensure(this, sb, "calvin wave maxima"));
      CR(cv_cwpos.ensure(this, d.n * 4 + 16, "calvin seqpos"));
      CR(cv_cwmark.ensure(this, cwp.slots + 16, "calvin wave marks"));
      CR(cv_cwhot.ensure(this, (uint64_t)cwp.nch * cwp.C * 32 + 16, "calvin wave compact records"));
      CR(cv_cwpa.ensure(this, sb, "calvin wave read addresses"));
      CR(cv_cwoa.ensure(this, sb, "calvin wave publish addresses"));
      if (cw_nh) {
        CR(cv_cwhelp.ensure(this, cw_help_words(cwp) * 4, "calvin wave helper hand-offs"));
        CR(cv_cwrec2.ensure(this, sb, "calvin wave two-chunk records"));
      }
    } else {
      CR(cv_pgx.ensure(this, m, "calvin pgx"));
      CR(cv_gsize.ensure(this, m, "calvin gsize"));
      CR(cv_done.ensure(this, m, "calvin done"));
      CR(cv_maxl.ensure(this, m, "calvin maxl"));
      CK(hipMemsetAsync(cv_gsize.p, 0, m, stream));
      CK(hipMemsetAsync(cv_done.p, 0, m, stream));
      CK(hipMemsetAsync(cv_maxl.p, 0, m, stream));
      so.pgx = (uint32_t*)cv_pgx.p;
      so.gsize = (uint32_t*)cv_gsize.p;
    }
  }

  // ---- the rest of the epoch as one captured HIP graph: the launches below
  // depend only on the batch's buffers and shape, the key / order packings
  // and the outputs, so the second epoch of a shape is captured and later
  // ones replay it (speculatively, above, or here after the prep read-back)
  const bool cv_replay = cv_graph_ok && cv_graph_exec && !memcmp(&gk, &cv_graph_key, sizeof gk);
  const bool cv_cap = cv_graph_ok && !cv_replay && cv_seen && !memcmp(&gk, &cv_seen_key, sizeof gk);
  struct CvCapture {  // a failure while capturing still ends the capture
    hipStream_t s;
    bool on;
    ~CvCapture() {
      if (on) {
        hipGraph_t g = nullptr;
        (void)hipStreamEndCapture(s, &g);
        if (g) (void)hipGraphDestroy(g);
        (void)hipGetLastError();
      }
    }
  } cap{stream, false};
  if (cv_replay) {
    CK(hipGraphLaunch(cv_graph_exec, stream));
  } else {
  if (cv_cap) {
    if (cv_graph_exec) {
      (void)hipGraphExecDestroy(cv_graph_exec);
      cv_graph_exec = nullptr;
    }
    CK(hipStreamBeginCapture(stream, hipStreamCaptureModeThreadLocal));
    cap.on = true;
  }
  CK(hipMemsetAsync(err, 0, 4, stream));

  // ---- rank: seq[q] = txn at sequence position q (stable in index order)
  const uint32_t* seq = nullptr;
  const uint32_t* off2 = nullptr;
  if (have_seq) {
    CR(perm.ensure(this, d.n * 4 + 16, "calvin seq a"));
    CR(cv_seq_b.ensure(this, d.n * 4 + 16, "calvin seq b"));
    CR(cv_ok.ensure(this, d.n * 8 * 2 + 32, "calvin order keys"));
    CR(cv_scratch.ensure(this, rs_scratch_words(std::max<uint64_t>(d.n, d.nnz + nh)) * 4 + 64,
                         "radix scratch"));
    uint32_t* vb[2] = {(uint32_t*)perm.p, (uint32_t*)cv_seq_b.p};
    int cur;
    if (op.bits <= 32) {
      uint32_t* kb[2] = {(uint32_t*)cv_ok.p, (uint32_t*)cv_ok.p + d.n + 4};
      k_cv_order_init<uint32_t><<<grid1(d.n, 256), 256, 0, stream>>>(d.order, d.n, op, kb[0], vb[0]);
      cur = radix_sort_u32(kb, vb, d.n, op.bits, (uint32_t*)cv_scratch.p, stream);
    } else {
      uint64_t* kb[2] = {(uint64_t*)cv_ok.p, (uint64_t*)cv_ok.p + d.n + 2};
      k_cv_order_init<uint64_t><<<grid1(d.n, 256), 256, 0, stream>>>(d.order, d.n, op, kb[0], vb[0]);
      cur = radix_sort_u64(kb, vb, d.n, op.bits, (uint32_t*)cv_scratch.p, stream);
    }
    seq = vb[cur];
  }
  // request offsets in sequence order (uniform txns: q * len, no pass)
  if (have_seq && !ulen && !use_cb) {  // (the bucket path builds its own per wave)
    const uint64_t lt = (d.n + CV_TILE - 1) / CV_TILE;
    CR(cv_len.ensure(this, d.n * 4 + 16, "calvin len"));
    CR(cv_off2.ensure(this, (d.n + 1) * 4 + 16, "calvin off2"));
    CR(cv_tsum.ensure(this, (lt + 1) * 4 + 16, "calvin tile sums"));
    uint32_t* tsum = (uint32_t*)cv_tsum.p;
    k_cv_len_tiles<<<(unsigned)lt, 256, 0, stream>>>(d.off, seq, d.n, (uint32_t*)cv_len.p, tsum);
    rs_scan_one(tsum, (uint32_t)lt, tsum + lt, stream);
    k_cv_len_apply<<<(unsigned)lt, 256, 0, stream>>>((const uint32_t*)cv_len.p, d.n, tsum,
                                                     (uint32_t)d.nnz, (uint32_t*)cv_off2.p);
    off2 = (const uint32_t*)cv_off2.p;
  }
  CK(hipGetLastError());

  // ---- requests in sequence order -> sorted by row -> group scan
  if (use_cb) {
    CR(cb_e.ensure(this, cbp.elem_bytes, "calvin bucket requests"));
    CR(cb_out.ensure(this, cbp.out_bytes, "calvin bucket pairs"));
    CR(cb_cnt.ensure(this, cbp.cnt_bytes, "calvin bucket counts"));
    CR(cb_small.ensure(this, cbp.small_bytes, "calvin bucket totals"));
    const CbArgs ca{d.keys,         d.acctype,           seq,     d.off,  d.n, d.nnz, ulen, kp, (uint64_t*)cb_e.p,
                    (uint64_t*)cb_out.p, (uint32_t*)cb_cnt.p, (uint32_t*)cb_small.p, grp_dev, rc_dev, err};
    CK(cb_run(cbp, ca, stream, profiling ? pev[1] : nullptr, profiling ? pev[2] : nullptr));
  } else if (d.nnz) {
    if (kp.bits <= 32)
      CR(calvin_sort_and_scan<uint32_t>(this, d, seq, off2, kp, so, hkeys, hat, nh, profiling, &sv));
    else
      CR(calvin_sort_and_scan<uint64_t>(this, d, seq, off2, kp, so, hkeys, hat, nh, profiling, &sv));
  } else if (profiling) {
    CK(hipEventRecord(pev[1], stream));
    CK(hipEventRecord(pev[2], stream));
  }
  if (use_cb) {
    // readiness came with the bucket path's window stores
  } else if (d.nnz) {
    k_cv_ready<<<grid1(d.n, 256), 256, 0, stream>>>(d.off, d.n, grp_dev, rc_dev);
  } else {
    CK(hipMemsetAsync(rc_dev, DCC_RC_RCOK, d.n, stream));
  }
  CK(hipGetLastError());
  if (profiling) CK(hipEventRecord(pev[3], stream));

  // ---- sharded: grant groups are per row, hence shard-local; a txn is
  // ready only if it is ready on every shard (WAIT = 3 > RCOK = 0)
  if (sharded()) CR(comm_allreduce_max_u8(rc_dev, d.n));

  // ---- wave levels
  if (cw) {
    const CwArgs ca{d.n, seq, d.off, ulen, so.gsx, so.glast, sv, (uint32_t*)cv_cwpos.p,
                    (uint32_t*)cv_gsize.p, (uint32_t*)cv_done.p, (uint32_t*)cv_maxl.p,
                    (uint32_t*)cv_cwmax.p, (uint8_t*)cv_cwmark.p, (uint32_t*)cv_cwpa.p,
                    (uint32_t*)cv_cwoa.p, (uint32_t*)cv_cwhot.p,
                    wave_dev, err, nullptr, (uint32_t*)cv_cwhelp.p, cw_nh ? (uint32_t*)cv_cwrec2.p : nullptr, cw_nh};
    if (DCC_ENV("DCC_CW_DBG")) {  // experiments builds: the walker's timing counters
      static uint64_t* dbg = nullptr;
      if (!dbg) CK(hipMalloc(&dbg, 256));
      CK(hipMemsetAsync(dbg, 0, 256, stream));
      CwArgs cd = ca;
      cd.dbg = dbg;
      CK(cw_run(cwp, cd, stream));
      uint64_t h[18];
      CK(hipMemcpyAsync(h, dbg, 144, hipMemcpyDeviceToHost, stream));
      CK(hipStreamSynchronize(stream));
      fprintf(stderr, "cw: chunks %u C %u H %u walk %.3f ms rounds-loop %.3f ms barriers %.3f ms rounds %llu"
              " | staging: maxima+fence %.3f sync %.3f bounds %.3f rest %.3f ms | clock %.0f MHz"
              " | sub-chunks with intra %llu overflow %llu plain rounds %llu"
              " | helpers: staging poll %.3f, helper 0 wait %.3f busy %.3f ms"
              " | boundary: walk wait %.3f refill %.3f adds %.3f ms\n",
              cwp.nch, cwp.C, cwp.H, h[0] * 1e-5, h[1] * 1e-5, h[2] * 1e-5, (unsigned long long)h[3],
              h[4] * 1e-5, h[5] * 1e-5, h[6] * 1e-5, h[7] * 1e-5,
              h[9] ? (double)h[8] / (h[9] * 1e-2) : 0.0, (unsigned long long)h[10],
              (unsigned long long)h[11], (unsigned long long)h[12], h[13] * 1e-5, h[14] * 1e-5,
              h[15] * 1e-5, h[16] * 1e-5, h[17] * 1e-5, h[7] * 1e-5);
    } else {
      CK(cw_run(cwp, ca, stream));
    }
  } else if (waves) {
    WaveArgs wa{d.n, seq, d.off, so.pgx, so.gsx, so.gsize, (uint32_t*)cv_done.p,
                (uint32_t*)cv_maxl.p, wave_dev, err, 100000000ull * 20};
    // co-resident persistent grid: 4 workgroups of 4 waves per CU
    const unsigned g = (unsigned)std::min<uint64_t>((uint64_t)n_cu * 4, (d.n + 3) / 4);
    k_cv_wave<<<g ? g : 1, 256, 0, stream>>>(wa);
    CK(hipGetLastError());
  }
  if (profiling) CK(hipEventRecord(pev[4], stream));
  CvCount* cc = (CvCount*)((char*)part.p + CV_COUNT_OFF);
  k_cv_count<<<CV_PREP_BLOCKS, 256, 0, stream>>>(rc_dev, wave_dev, d.n, cc);
  CK(hipGetLastError());
  if (cv_cap) {
    cap.on = false;
    hipGraph_t g = nullptr;
    CK(hipStreamEndCapture(stream, &g));
    const hipError_t ie = hipGraphInstantiate(&cv_graph_exec, g, nullptr, nullptr, 0);
    (void)hipGraphDestroy(g);
    if (ie != hipSuccess) {
      cv_graph_exec = nullptr;
      return fail(DCC_EIO, "hipGraphInstantiate: %s", hipGetErrorString(ie));
    }
    cv_graph_key = gk;
    CK(hipGraphLaunch(cv_graph_exec, stream));
  }
  if (cv_graph_ok) {  // the shape this call enqueued, with the workspaces it left
    cv_seen_key = gk;
    cv_seen_key.gen = buf_gen;
    cv_seen = true;
  }
  }  // not replayed
  CR(enqueue_tail(wave_dev));
  }  // not a confirmed speculation
  if (*(const uint32_t*)hmisc & (ERR_WAVE_TIMEOUT | CW_ERR_SPIN))
    return fail(DCC_EIO, "calvin: wave kernel exceeded its time budget");
  if (*(const uint32_t*)hmisc & CB_ERR_TAB) {
    // a bucket held more rows than the hashed carry table: this context's
    // epochs take the sort path from now on, this one again
    cb_hash_off = true;
    return calvin_epoch(b, held, out_group, out_rc, out_wave, st);
  }
  uint64_t ready = 0;
  uint32_t maxwave = 0;
  for (unsigned q = 0; q < CV_PREP_BLOCKS; q++) {
    const CvCount& c = ((const CvCount*)((const char*)hpart + CV_COUNT_OFF))[q];
    ready += c.ready;
    maxwave = std::max(maxwave, c.maxwave);
  }
  float ms = 0;
  CK(hipEventElapsedTime(&ms, ev0, ev1));
  S.rounds = waves ? maxwave + 1 : 0;
  S.n_commit = ready;
  S.n_abort = d.n - ready;
  S.nnz_w = nex;
  S.alg_bytes = dcc_calvin_alg_bytes(d.n, d.nnz, d.order != nullptr, waves);
  S.device_ms = ms;
  S.fallback = use_cb ? 1u : 0u;  // Calvin: the grant groups came from the bucket path
  if (profiling) {
    float t[4] = {0, 0, 0, 0};
    CK(hipEventElapsedTime(&t[0], pev[0], pev[1]));  // prep + rank + layout
    CK(hipEventElapsedTime(&t[1], pev[1], pev[2]));  // key sort
    CK(hipEventElapsedTime(&t[2], pev[2], pev[3]));  // group scan
    CK(hipEventElapsedTime(&t[3], pev[3], pev[4]));  // waves
    for (int q = 0; q < 4; q++) S.phase_ms[q] = t[q];
  }
  const auto t_wall1 = std::chrono::steady_clock::now();
  S.total_ms = std::chrono::duration<double, std::milli>(t_wall1 - t_wall0).count();
  if (st) *st = S;
  return DCC_OK;
}

extern "C" uint64_t dcc_calvin_alg_bytes(uint64_t n_txn, uint64_t nnz, int with_order,
                                         int with_wave) {
  // offsets, key + acctype per request, group per request, RC byte per txn,
  // order per txn (if given), wave per txn (if requested)
  return 4 * (n_txn + 1) + 9 * nnz + 4 * nnz + n_txn + (with_order ? 8 * n_txn : 0) +
         (with_wave ? 4 * n_txn : 0);
}

extern "C" int dcc_calvin_order_epoch(dcc_ctx* ctx, const dcc_batch* batch, uint32_t* out_group,
                                      uint8_t* out_rc, uint32_t* out_wave, dcc_stats* st) {
  if (!ctx) return DCC_EINVAL;
  if (ctx->multi) return dcc_multi_calvin_epoch(ctx, batch, nullptr, out_group, out_rc, out_wave, st);
  if (hipSetDevice(ctx->device) != hipSuccess) return DCC_ENODEV;
  return ctx->calvin_epoch(batch, nullptr, out_group, out_rc, out_wave, st);
}

extern "C" int dcc_calvin_order_epoch_held(dcc_ctx* ctx, const dcc_batch* batch,
                                           const dcc_calvin_held* held, uint32_t* out_group,
                                           uint8_t* out_rc, uint32_t* out_wave, dcc_stats* st) {
  if (!ctx) return DCC_EINVAL;
  if (ctx->multi) return dcc_multi_calvin_epoch(ctx, batch, held, out_group, out_rc, out_wave, st);
  if (hipSetDevice(ctx->device) != hipSuccess) return DCC_ENODEV;
  return ctx->calvin_epoch(batch, held, out_group, out_rc, out_wave, st);
}
