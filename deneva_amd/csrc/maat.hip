// MaaT epoch validation on gfx950.
//
// Reference: Maat::validate / find_bound (concurrency_control/maat.cpp:29-191)
// over the per-row soft locks of Row_maat (row_maat.cpp:38-314).  The epoch
// model (include/dcc.h, dcc_maat_validate_epoch): every txn accesses its rows
// (index order), then in index order each txn validates and commits or aborts.
// A txn's copied uncommitted sets then hold only earlier txns, decided and
// released by the time it validates, so the set loops of Maat::validate never
// tighten anything; what reaches txn i is the forward validation of earlier
// commits (Row_maat::commit) and the row timestamps copied at access time:
//
//   L_i = max(gwts_i + 1, grts_i + 1, max{cts_j + 1 : j < i committed, j read a row i wrote})
//   U_i = min(UINT64_MAX, min{cts_j - 1 : j < i committed, j wrote a row i accessed})
//   commit iff L_i < U_i, with commit timestamp cts_i = L_i (find_bound)
//
// (oracle/maat_ref.c restates both the literal replay and this formula).
// L only grows and U only shrinks as earlier txns commit, so the GPU decides
// by rounds: accesses sorted by row (stable, so index order within a row),
// one segmented scan per round gives each (row, txn) group the max commit
// timestamp of earlier committed readers, the min of earlier committed
// writers and whether an earlier reader / writer is still undecided; a txn
// whose known L >= known U aborts (final), one with no undecided relevant
// predecessor commits at L, the rest wait for the next round.  The smallest
// undecided txn always decides, so the rounds terminate.
//
// Row timestamps (timestamp_last_read / _write, row_maat.h:38-39) persist
// in an HBM open-addressing table across epochs; committed txns raise them
// with atomicMax at the end of the epoch (row_maat.cpp:249-251, 276-278).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>

#include "dcc.h"
#include "dcc_ctx.h"
#include "dcc_device.h"
#include "dcc_env.h"
#include "occ_kernels.h"
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

constexpr uint64_t U64MAX = ~0ull;
constexpr uint32_t MT_ITEMS = 16;
constexpr uint32_t MT_TILE = 256 * MT_ITEMS;
constexpr uint32_t MT_RING = 64;          // per-round undecided counters
constexpr uint32_t MT_BATCH = 12;         // rounds enqueued per host check (A/B: tools/ab_maat_batch.sh)
constexpr uint64_t MT_LONG = 1u << 22;    // scans longer than this: a check after every round
constexpr uint64_t MT_PREFIX = 1024;      // txns of the prefix level (DCC_MT_PREFIX; 0: none)
constexpr uint8_t ST_UND = 0, ST_COM = 1, ST_ABO = 2;
// sorted-position flags
constexpr uint8_t F_R = 1, F_W = 2, F_LAST = 4, F_START = 8;
constexpr uint32_t MT_ERR_OFF = 1, MT_ERR_KEY = 2, MT_ERR_FULL = 4;

__device__ inline uint64_t mt_hash(uint64_t key, uint32_t bits) {
  return (key * 0x9E3779B97F4A7C15ull) >> (64 - bits);
}

// ---------------------------------------------------------------- row table
// One 32-B slot per row: the key and its two timestamps side by side, so the
// access that finds a row has its timestamps in the same 64-B line (three
// separate arrays cost three random HBM lines per access).
struct __attribute__((aligned(32))) MtSlot {
  uint64_t key, lr, lw, pad;
};
static_assert(sizeof(MtSlot) == 32, "row slot");
// insert-or-find the row of `key` (ins: this call created it); its lr / lw
// stay 0 until an epoch commits
// (a walk past MT_WALK slots reports MT_ERR_FULL: the host grows the table
// and runs the epoch again)
constexpr uint64_t MT_WALK = 256;
__device__ inline uint32_t mt_row(MtSlot* rt, uint32_t bits, uint64_t key, bool& ins,
                                  uint32_t* err) {
  const uint64_t mask = (1ull << bits) - 1;
  uint64_t s = mt_hash(key, bits);
  ins = false;
  for (uint64_t q = 0; q <= mask && q < MT_WALK; q++) {
    const uint64_t v = rt[s].key;
    if (v == key) return (uint32_t)s;
    if (v == DCC_KEY_RESERVED) {
      const unsigned long long prev = atomicCAS((unsigned long long*)&rt[s].key,
                                                (unsigned long long)DCC_KEY_RESERVED,
                                                (unsigned long long)key);
      if (prev == DCC_KEY_RESERVED) {
        ins = true;
        return (uint32_t)s;
      }
      if (prev == key) return (uint32_t)s;
    }
    s = (s + 1) & mask;
  }
  atomicOr(err, MT_ERR_FULL);
  return 0;
}

// one atomic per workgroup for a per-thread count (256 threads)
__device__ inline void block_add(uint32_t c, uint32_t* ctr) {
  __shared__ uint32_t s_c[4];
  for (int d = 32; d > 0; d >>= 1) c += __shfl_xor(c, d);
  if ((threadIdx.x & 63) == 0) s_c[threadIdx.x >> 6] = c;
  __syncthreads();
  if (threadIdx.x == 0) {
    const uint32_t v = s_c[0] + s_c[1] + s_c[2] + s_c[3];
    if (v) atomicAdd(ctr, v);
  }
}

// rehash: every row of the old table into the new one (values carried)
__global__ __launch_bounds__(256) void k_mt_rehash(const MtSlot* ot, uint64_t ocap, MtSlot* nt,
                                                   uint32_t nbits, uint32_t* nrows, uint32_t* err) {
  uint32_t c = 0;
  for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < ocap; i += (uint64_t)gridDim.x * 256) {
    const MtSlot o = ot[i];
    if (o.key == DCC_KEY_RESERVED) continue;
    bool ins;
    const uint32_t s = mt_row(nt, nbits, o.key, ins, err);
    c += ins;
    nt[s].lr = o.lr;
    nt[s].lw = o.lw;
  }
  block_add(c, nrows);
}
// an empty table: every key KEY_RESERVED, timestamps 0
__global__ __launch_bounds__(256) void k_mt_clear(MtSlot* rt, uint64_t cap) {
  for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < cap; i += (uint64_t)gridDim.x * 256)
    rt[i] = MtSlot{DCC_KEY_RESERVED, 0, 0, 0};
}

// host-seeded rows (dcc_maat_rows_set): insert and overwrite the timestamps
__global__ __launch_bounds__(256) void k_mt_seed(const uint64_t* keys, const uint64_t* lr,
                                                 const uint64_t* lw, uint64_t n, MtSlot* rt,
                                                 uint32_t bits, uint32_t* nrows, uint32_t* err) {
  uint32_t c = 0;
  for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (uint64_t)gridDim.x * 256) {
    if (keys[i] == DCC_KEY_RESERVED) {
      atomicOr(err, MT_ERR_KEY);
      continue;
    }
    bool ins;
    const uint32_t s = mt_row(rt, bits, keys[i], ins, err);
    c += ins;
    rt[s].lr = lr[i];
    rt[s].lw = lw[i];
  }
  block_add(c, nrows);
}
__global__ __launch_bounds__(256) void k_mt_get(const uint64_t* keys, uint64_t n, const MtSlot* rt,
                                                uint32_t bits, uint64_t* lr, uint64_t* lw) {
  const uint64_t mask = (1ull << bits) - 1;
  for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (uint64_t)gridDim.x * 256) {
    const uint64_t key = keys[i];
    uint64_t s = mt_hash(key, bits), a = 0, b = 0;
    for (uint64_t q = 0; q <= mask; q++) {
      const uint64_t v = rt[s].key;
      if (v == key) {
        a = rt[s].lr;
        b = rt[s].lw;
        break;
      }
      if (v == DCC_KEY_RESERVED) break;
      s = (s + 1) & mask;
    }
    lr[i] = a;
    lw[i] = b;
  }
}

// ---------------------------------------------------------------- check
// The batch's validity before the persistent row table changes: offsets
// (monotone, 0 .. nnz, <= MAX_ROW_PER_TXN per txn) and no reserved key.  A
// rejected epoch leaves the row table (rows and timestamps) untouched.
__global__ __launch_bounds__(256) void k_mt_check(const uint32_t* off, uint64_t n,
                                                  const uint64_t* keys, uint64_t nnz,
                                                  uint32_t* err) {
  uint32_t e = 0;
  const uint64_t t0 = (uint64_t)blockIdx.x * 256 + threadIdx.x, stride = (uint64_t)gridDim.x * 256;
  for (uint64_t t = t0; t < n; t += stride) {
    const uint32_t o0 = off[t], o1 = off[t + 1];
    if (o1 < o0 || o1 - o0 > MAX_TXN_LEN) e |= MT_ERR_OFF;
    if ((t == 0 && o0 != 0) || (t + 1 == n && o1 != nnz)) e |= MT_ERR_OFF;
  }
  for (uint64_t x = t0; x < nnz; x += stride)
    if (keys[x] == DCC_KEY_RESERVED) e |= MT_ERR_KEY;
  if (e) atomicOr(err, e);
}

// ---------------------------------------------------------------- base
// The txn's lower bound from the row timestamps copied at access time: gwts
// over rows read or written, grts over rows written (Row_maat::read /
// prewrite, row_maat.cpp:115-117, 150-156; Maat::validate raises lower past
// them, maat.cpp:46-49, 69-72).  Every access first finds or enters its row
// in the table (its slot id, written twice: the sort's key buffer and the
// finish's copy) and reads the row's timestamps from the same slot.  A wave
// per 64 txns walks their contiguous accesses 64 at a time (coalesced key /
// type loads, four rounds in flight),
// finds each access's txn in the wave's LDS offset prefix and folds the row
// timestamps per txn with LDS atomicMax.  Each access's sort value packs its
// txn and R / W bits, so the sorted groups need no gathers.
struct BaseArgs {
  uint64_t n, nnz;
  const uint32_t* off;
  const uint8_t* at;
  uint32_t rw_all;
  const uint64_t* keys;
  MtSlot* rt;
  uint32_t bits;
  uint32_t* slot;   // [nnz] row slot per access
  uint32_t* slot2;  // [nnz] the same (the sort's first key buffer)
  uint32_t* nrows;
  uint32_t* sval;   // [nnz] txn << 2 | R << 1 | W
  uint64_t* base;   // [n]
  uint8_t* state;   // [n] zeroed here
  uint64_t* lacc;   // [n] 0
  uint64_t* uacc;   // [n] U64MAX
  uint32_t* pend;   // [n] 0
  uint32_t* err;
};
constexpr uint32_t SV_R = 2, SV_W = 1;
__global__ __launch_bounds__(256) void k_mt_base(BaseArgs a) {
  __shared__ uint32_t s_o[4][65];
  __shared__ unsigned long long s_gw[4][64], s_gr[4][64];
  const uint32_t lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const uint64_t t0 = ((uint64_t)blockIdx.x * 4 + w) * 64;
  if (t0 >= a.n) return;
  const uint32_t nt = (uint32_t)min<uint64_t>(64, a.n - t0);
  const uint64_t t = t0 + lane;
  if (lane < nt) {
    const uint32_t o0 = a.off[t], o1 = a.off[t + 1];
    if (o1 < o0 || o1 - o0 > MAX_TXN_LEN) atomicOr(a.err, MT_ERR_OFF);
    if ((t == 0 && o0 != 0) || (t + 1 == a.n && o1 != a.nnz)) atomicOr(a.err, MT_ERR_OFF);
  }
  // clamped, made monotone: a malformed batch is reported, never overrun
  uint32_t ov = lane <= nt ? (uint32_t)min<uint64_t>(a.off[t0 + lane], a.nnz) : 0u;
  for (int d = 1; d < 64; d <<= 1) {
    const uint32_t y = __shfl_up(ov, d);
    if (lane >= (uint32_t)d && lane <= nt) ov = max(ov, y);
  }
  s_o[w][lane] = ov;
  if (lane == 0) s_o[w][64] = 0;
  s_gw[w][lane] = 0;
  s_gr[w][lane] = 0;
  __builtin_amdgcn_wave_barrier();
  if (nt == 64 && lane == 0)
    s_o[w][64] = max(s_o[w][63], (uint32_t)min<uint64_t>(a.off[t0 + 64], a.nnz));
  __builtin_amdgcn_wave_barrier();
  const uint32_t a0 = s_o[w][0], a1 = s_o[w][nt];
  uint32_t nins = 0;
  for (uint32_t x0 = a0; x0 < a1; x0 += 4 * 64) {
    uint64_t key[4];
    uint8_t ty[4];
#pragma unroll
    for (uint32_t u = 0; u < 4; u++) {
      const uint32_t x = min(x0 + 64 * u + lane, a1 - 1);
      key[u] = a.keys[x];
      ty[u] = a.at[x];
    }
    uint32_t sl[4];
#pragma unroll
    for (uint32_t u = 0; u < 4; u++) {
      sl[u] = 0;
      if (x0 + 64 * u + lane < a1 && key[u] != DCC_KEY_RESERVED) {  // the check rejected reserved keys
        bool ins;
        sl[u] = mt_row(a.rt, a.bits, key[u], ins, a.err);
        nins += ins;
      }
    }
    uint64_t lw[4], lr[4];
#pragma unroll
    for (uint32_t u = 0; u < 4; u++) {
      lw[u] = a.rt[sl[u]].lw;
      lr[u] = a.rt[sl[u]].lr;
    }
#pragma unroll
    for (uint32_t u = 0; u < 4; u++) {
      const uint32_t x = x0 + 64 * u + lane;
      if (x >= a1) continue;
      a.slot[x] = sl[u];
      a.slot2[x] = sl[u];
      uint32_t lo = 0, hi = nt;  // largest k < nt with s_o[k] <= x
      while (hi - lo > 1) {
        const uint32_t mid = (lo + hi) >> 1;
        if (s_o[w][mid] <= x) lo = mid;
        else hi = mid;
      }
      const bool rd = a.rw_all || ty[u] == DCC_RD, wr = a.rw_all || ty[u] == DCC_WR;
      if (rd || wr) atomicMax(&s_gw[w][lo], (unsigned long long)lw[u]);
      if (wr) atomicMax(&s_gr[w][lo], (unsigned long long)lr[u]);
      a.sval[x] = ((uint32_t)(t0 + lo) << 2) | (rd ? SV_R : 0u) | (wr ? SV_W : 0u);
    }
  }
  for (int d = 32; d > 0; d >>= 1) nins += __shfl_xor(nins, d);
  if (lane == 0 && nins) atomicAdd(a.nrows, nins);
  __builtin_amdgcn_wave_barrier();
  if (lane < nt) {
    a.base[t] = max(s_gw[w][lane], s_gr[w][lane]) + 1;
    a.state[t] = ST_UND;
    a.lacc[t] = 0;
    a.uacc[t] = U64MAX;
    a.pend[t] = 0;
  }
}

// Group flags per sorted position: a (row, txn) group is a run of equal
// (slot, txn); its last position carries the OR of its R / W bits.
__global__ __launch_bounds__(256) void k_mt_groups(const uint32_t* ss, const uint32_t* sv,
                                                   uint64_t m, uint8_t* sfl, uint32_t* stx) {
  for (uint64_t p = (uint64_t)blockIdx.x * 256 + threadIdx.x; p < m; p += (uint64_t)gridDim.x * 256) {
    const uint32_t s = ss[p], v = sv[p], t = v >> 2;
    uint8_t f = 0;
    if (p == 0 || ss[p - 1] != s) f |= F_START;
    const bool last = p + 1 == m || ss[p + 1] != s || (sv[p + 1] >> 2) != t;
    if (last) {
      f |= F_LAST;
      for (uint64_t q = p;; q--) {  // the group's accesses (<= MAX_ROW_PER_TXN)
        const uint32_t vq = sv[q];
        if (vq & SV_R) f |= F_R;
        if (vq & SV_W) f |= F_W;
        if (q == 0 || ss[q - 1] != s || (sv[q - 1] >> 2) != t) break;
      }
    }
    sfl[p] = f;
    stx[p] = t;
  }
}

// ---------------------------------------------------------------- round scan
// State of an interval since the last row start: flag = holds a row start;
// rmax / wmin over committed readers / writers; und bit 0 / 1 = an undecided
// reader / writer.  Contributions sit at each group's last position, so the
// exclusive prefix at a group excludes the group's own txn.
struct Ms {
  uint32_t flag, und;
  uint64_t rmax, wmin;
};
__device__ inline Ms ms_id() { return Ms{0, 0, 0, U64MAX}; }
__device__ inline Ms ms_comb(const Ms& A, const Ms& B) {
  if (B.flag) return B;
  return Ms{A.flag, A.und | B.und, max(A.rmax, B.rmax), min(A.wmin, B.wmin)};
}
__device__ inline Ms ms_elem(uint8_t f, uint8_t st, uint64_t cts) {
  Ms e = ms_id();
  if (f & F_START) e.flag = 1;
  if (f & F_LAST) {
    if (st == ST_COM) {
      if (f & F_R) e.rmax = cts;
      if (f & F_W) e.wmin = cts;
    } else if (st == ST_UND) {
      e.und = ((f & F_R) ? 1u : 0u) | ((f & F_W) ? 2u : 0u);
    }
  }
  return e;
}

struct MtRoundArgs {
  uint64_t m, n;
  const uint8_t* sfl;
  const uint32_t* stx;
  const uint8_t* state;
  const uint64_t* cts;
  uint64_t* lacc;
  uint64_t* uacc;
  uint32_t* pend;
  Ms* agg;
};

// wave shuffles of the four fields, then the four waves' totals through LDS
__device__ inline Ms ms_shfl_up(const Ms& v, uint32_t d) {
  Ms r;
  r.flag = __shfl_up(v.flag, d);
  r.und = __shfl_up(v.und, d);
  r.rmax = __shfl_up(v.rmax, d);
  r.wmin = __shfl_up(v.wmin, d);
  return r;
}
__device__ inline Ms wave_incl_ms(Ms x) {
  const uint32_t lane = threadIdx.x & 63;
#pragma unroll
  for (uint32_t d = 1; d < 64; d <<= 1) {
    const Ms y = ms_shfl_up(x, d);
    if (lane >= d) x = ms_comb(y, x);
  }
  return x;
}
__device__ inline Ms block_reduce_ms(Ms v, Ms* s) {
  const Ms x = wave_incl_ms(v);
  if ((threadIdx.x & 63) == 63) s[threadIdx.x >> 6] = x;
  __syncthreads();
  Ms r = s[0];
  for (uint32_t w = 1; w < 4; w++) r = ms_comb(r, s[w]);
  __syncthreads();
  return r;
}
__device__ inline Ms block_excl_ms(Ms v, Ms* s) {
  const uint32_t lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const Ms x = wave_incl_ms(v);
  if (lane == 63) s[wv] = x;
  __syncthreads();
  Ms pre = ms_id();
  for (uint32_t w = 0; w < wv; w++) pre = ms_comb(pre, s[w]);
  Ms ex = ms_shfl_up(x, 1);
  if (lane == 0) ex = ms_id();
  __syncthreads();
  return ms_comb(pre, ex);
}

// A tile's flags and txns in the blocked arrangement the scans need (thread
// t: positions 16t .. 16t + 15 of the tile), loaded with coalesced 16-B loads
// (flags: 4 per thread, txns: 16 words per thread as 4 loads) through LDS --
// a thread reading its own 16 consecutive positions straight from memory
// spreads every wave instruction over 64 lines.  Past the end: flags 0, an
// identity element of every scan.
struct MtTileLds {
  uint4 f[MT_TILE / 16];
  uint4 x[MT_TILE / 4];
};
__device__ inline void mt_load_tile(const uint8_t* sfl, const uint32_t* stx, uint64_t m, uint64_t base,
                                    MtTileLds& L, uint8_t (&f)[MT_ITEMS], uint32_t (&tx)[MT_ITEMS]) {
  const uint32_t tid = threadIdx.x;
  const uint64_t n_here = m > base ? min<uint64_t>(MT_TILE, m - base) : 0;
  const bool full = n_here == MT_TILE && ((uintptr_t)(sfl + base) & 15) == 0 &&
                    ((uintptr_t)(stx + base) & 15) == 0;
  if (full) {
    L.f[tid] = ((const uint4*)(sfl + base))[tid];
#pragma unroll
    for (uint32_t i = 0; i < 4; i++) L.x[i * 256 + tid] = ((const uint4*)(stx + base))[i * 256 + tid];
  } else {
    uint8_t* lf = (uint8_t*)L.f;
    uint32_t* lx = (uint32_t*)L.x;
    for (uint32_t q = tid; q < MT_TILE; q += 256) {
      lf[q] = q < n_here ? sfl[base + q] : (uint8_t)0;
      lx[q] = q < n_here ? stx[base + q] : 0u;
    }
  }
  __syncthreads();
  const uint4 fw = L.f[tid];
  const uint32_t w4[4] = {fw.x, fw.y, fw.z, fw.w};
#pragma unroll
  for (uint32_t i = 0; i < MT_ITEMS; i++) f[i] = (uint8_t)(w4[i >> 2] >> (8 * (i & 3)));
#pragma unroll
  for (uint32_t i = 0; i < 4; i++) {
    const uint4 v = L.x[tid * 4 + i];
    tx[4 * i] = v.x;
    tx[4 * i + 1] = v.y;
    tx[4 * i + 2] = v.z;
    tx[4 * i + 3] = v.w;
  }
  __syncthreads();  // the caller may reuse L
}

// ---------------------------------------------------------------- fused round
// The round scan in one launch (one read of each tile, no
// aggregate pass): a single-pass scan with decoupled look-back.  Tile j
// publishes its aggregate as soon as it has it, then wave 0 looks back 64
// tiles at a time (lane 0 the nearest) until it meets a published inclusive
// prefix, combines what it read in order, and publishes its own inclusive
// prefix.  Status words carry the round's tag (tag << 2 | 1 aggregate, | 2
// inclusive), so nothing is reset between rounds.  Workgroups are dispatched
// in index order, so every tile a look-back waits on is running or done; the
// spins are bounded anyway (release/acquire recipe and timeout flag of
// grid_barrier, occ_kernels.hip): a timeout raises MT_ERR_SPIN and the host
// fails the epoch.
struct __attribute__((aligned(64))) MtLb {
  uint64_t agg_rmax, agg_wmin, inc_rmax, inc_wmin;
  uint32_t agg_fu, inc_fu;  // flag | und << 1
  uint32_t status, pad[5];
};
static_assert(sizeof(MtLb) == 64, "one line per tile");
constexpr uint32_t MT_ERR_SPIN = 8;

// Every field is written and read with device-scope atomics (coherent across
// the XCDs' L2s without a cache write-back per tile).  The status word is the
// flag of a message-passing pair, ordered by the hardware rather than by the
// HIP memory model's release/acquire: the payload's agent-scope stores are
// write-through (`sc1`) and `s_waitcnt vmcnt(0)` holds the status store until
// each of them is acknowledged at the coherence point, and a reader issues its
// payload loads (also `sc1`, read at that point) only after the status load
// has returned the tag (the spin's branch depends on it).  The model's own
// recipe -- a release store (`buffer_wbl2 sc1`, a write-back of the whole XCD
// L2) per publish and an acquire load (`buffer_inv sc1`) per poll -- is what
// the first version of this scan used, at 517-548 us per 16.7 M-position
// round against 252 us.
template <typename T>
__device__ inline void st_dev(T* p, T v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
template <typename T>
__device__ inline T ld_dev(T* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ inline void mt_publish(MtLb* e, const Ms& v, bool incl, uint32_t tag) {
  if (incl) {
    st_dev(&e->inc_rmax, v.rmax);
    st_dev(&e->inc_wmin, v.wmin);
    st_dev(&e->inc_fu, v.flag | (v.und << 1));
  } else {
    st_dev(&e->agg_rmax, v.rmax);
    st_dev(&e->agg_wmin, v.wmin);
    st_dev(&e->agg_fu, v.flag | (v.und << 1));
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  st_dev(&e->status, (tag << 2) | (incl ? 2u : 1u));
}
__device__ inline Ms mt_read(MtLb* e, bool incl) {
  const uint32_t fu = ld_dev(incl ? &e->inc_fu : &e->agg_fu);
  return Ms{fu & 1u, fu >> 1, ld_dev(incl ? &e->inc_rmax : &e->agg_rmax),
            ld_dev(incl ? &e->inc_wmin : &e->agg_wmin)};
}
// ordered wave reduction, lane 0 rightmost: lane 0 gets v63 (x) ... (x) v0
__device__ inline Ms wave_rcomb_ms(Ms x) {
  const uint32_t lane = threadIdx.x & 63;
#pragma unroll
  for (uint32_t d = 1; d < 64; d <<= 1) {
    Ms y;
    y.flag = __shfl_down(x.flag, d);
    y.und = __shfl_down(x.und, d);
    y.rmax = __shfl_down(x.rmax, d);
    y.wmin = __shfl_down(x.wmin, d);
    if (lane + d < 64) x = ms_comb(y, x);
  }
  return x;
}

__global__ __launch_bounds__(256) void k_mt_round(MtRoundArgs a, MtLb* lb, uint32_t tag, uint32_t* err,
                                                  const uint32_t* prev_und) {
  __shared__ Ms s[4];
  __shared__ Ms s_pre;
  __shared__ MtTileLds L;
  // a round enqueued after the list was already decided (a batch runs a
  // fixed number of rounds between host checks): nothing to do
  if (prev_und && *prev_und == 0) return;
  const uint32_t tile = blockIdx.x, lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const uint64_t base = (uint64_t)tile * MT_TILE;
  const uint64_t p0 = base + (uint64_t)threadIdx.x * MT_ITEMS;
  uint8_t f[MT_ITEMS], st[MT_ITEMS];
  uint32_t tx[MT_ITEMS];
  uint64_t c[MT_ITEMS];
  mt_load_tile(a.sfl, a.stx, a.m, base, L, f, tx);
#pragma unroll
  for (uint32_t i = 0; i < MT_ITEMS; i++) {
    st[i] = (f[i] & F_LAST) ? a.state[tx[i]] : ST_ABO;
    c[i] = 0;
  }
#pragma unroll
  for (uint32_t i = 0; i < MT_ITEMS; i++)
    if (st[i] == ST_COM) c[i] = a.cts[tx[i]];
  Ms acc = ms_id();
#pragma unroll
  for (uint32_t i = 0; i < MT_ITEMS; i++) acc = ms_comb(acc, ms_elem(f[i], st[i], c[i]));
  // block exclusive prefix per thread and the tile's total
  const Ms x = wave_incl_ms(acc);
  if (lane == 63) s[wv] = x;
  __syncthreads();
  Ms pre = ms_id(), tot = ms_id();
#pragma unroll
  for (uint32_t w = 0; w < 4; w++) {
    if (w < wv) pre = ms_comb(pre, s[w]);
    tot = ms_comb(tot, s[w]);
  }
  Ms ex = ms_shfl_up(x, 1);
  if (lane == 0) ex = ms_id();
  ex = ms_comb(pre, ex);
  if (wv == 0) {
    Ms P = ms_id();
    if (tile == 0) {
      if (lane == 0) mt_publish(&lb[0], tot, true, tag);
    } else {
      if (lane == 0) mt_publish(&lb[tile], tot, false, tag);
      bool timed_out = false;
      for (int64_t hi = (int64_t)tile - 1; hi >= 0; hi -= 64) {
        const int64_t j = hi - (int64_t)lane;
        uint32_t stw = 0;
        if (j >= 0) {
          const uint64_t t0 = spin_clock();
          while (((stw = ld_dev(&lb[j].status)) >> 2) != tag) {
            __builtin_amdgcn_s_sleep(1);
            if (spin_clock() - t0 > SPIN_TICKS) {
              timed_out = true;
              break;
            }
          }
        }
        if (ballot64(timed_out)) {
          if (lane == 0) atomicOr(err, MT_ERR_SPIN);
          break;
        }
        const bool inc = j >= 0 && (stw & 3u) == 2u;
        const uint64_t im = ballot64(inc);
        const uint32_t stop = im ? (uint32_t)__builtin_ctzll(im) : 63u;
        Ms v = ms_id();
        if (j >= 0 && lane <= stop) v = mt_read(&lb[j], inc);
        P = ms_comb(wave_rcomb_ms(v), P);  // lane 0's value is the batch's
        if (im) break;
      }
      if (lane == 0) mt_publish(&lb[tile], ms_comb(P, tot), true, tag);
    }
    if (lane == 0) s_pre = P;
  }
  __syncthreads();
  Ms run = ms_comb(s_pre, ex);
#pragma unroll
  for (uint32_t i = 0; i < MT_ITEMS; i++) {
    const uint64_t p = p0 + i;
    if (p >= a.m) break;
    if (f[i] & F_START) run = Ms{1, 0, 0, U64MAX};  // own group excluded: contributions at its end
    if ((f[i] & F_LAST) && (f[i] & (F_R | F_W)) && st[i] == ST_UND) {
      const uint32_t t = tx[i];
      if ((f[i] & F_W) && run.rmax) atomicMax((unsigned long long*)&a.lacc[t], run.rmax + 1);
      if (run.wmin != U64MAX) atomicMin((unsigned long long*)&a.uacc[t], run.wmin - 1);
      if ((run.und & 2u) || ((f[i] & F_W) && (run.und & 1u))) a.pend[t] = 1u;
    }
    run = ms_comb(run, ms_elem(f[i] & ~F_START, st[i], c[i]));
  }
}

// decide: abort when the known bounds are already empty, commit when no
// relevant predecessor is undecided; reset the accumulators
// (over the undecided-txn list ul[0, *ulen) when given, else txns [0, n))
__global__ __launch_bounds__(256) void k_mt_decide(uint64_t n, const uint32_t* ul, const uint32_t* ulen,
                                                   const uint64_t* base, uint8_t* state,
                                                   uint64_t* cts, uint64_t* lacc, uint64_t* uacc,
                                                   uint32_t* pend, uint32_t* und_out,
                                                   uint32_t* und_zero, const uint32_t* prev_und) {
  __shared__ uint32_t sh[4];
  if (prev_und && *prev_und == 0) {  // already decided: this round's count stays 0
    if (blockIdx.x == 0 && threadIdx.x == 0) *und_zero = 0;
    return;
  }
  uint32_t und = 0;
  const uint64_t cnt = ul ? *ulen : n;
  for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < cnt; i += (uint64_t)gridDim.x * 256) {
    const uint64_t t = ul ? ul[i] : i;
    if (state[t] != ST_UND) continue;
    const uint64_t L = max(base[t], lacc[t]);
    const uint64_t U = uacc[t];
    if (L >= U) {
      state[t] = ST_ABO;
    } else if (!pend[t]) {
      state[t] = ST_COM;
      cts[t] = L;
    } else {
      und++;
    }
    lacc[t] = 0;
    uacc[t] = U64MAX;
    pend[t] = 0;
  }
  for (int d = 32; d > 0; d >>= 1) und += __shfl_xor(und, d);
  if ((threadIdx.x & 63) == 0) sh[threadIdx.x >> 6] = und;
  __syncthreads();
  if (threadIdx.x == 0) {
    const uint32_t s = sh[0] + sh[1] + sh[2] + sh[3];
    if (s) atomicAdd(und_out, s);
    if (blockIdx.x == 0) *und_zero = 0;
  }
}

// the undecided txns of a list (any order: each is decided on its own)
__global__ __launch_bounds__(256) void k_mt_ucompact(const uint32_t* ul, const uint32_t* ulen, uint64_t n,
                                                     const uint8_t* state, uint32_t* out,
                                                     uint32_t* out_len) {
  // one counter atomic per workgroup and step (same-address atomics
  // serialise: one per wave cost 190 us over a 1M-txn list)
  __shared__ uint32_t s_n[4], s_b;
  const uint64_t cnt = ul ? *ulen : n;
  const uint32_t lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  for (uint64_t i0 = (uint64_t)blockIdx.x * 256; i0 < cnt; i0 += (uint64_t)gridDim.x * 256) {
    const uint64_t i = i0 + threadIdx.x;
    uint32_t t = 0;
    bool keep = false;
    if (i < cnt) {
      t = ul ? ul[i] : (uint32_t)i;
      keep = state[t] == ST_UND;
    }
    const uint64_t bm = ballot64(keep);
    if (lane == 0) s_n[wv] = (uint32_t)__popcll(bm);
    __syncthreads();
    if (threadIdx.x == 0) {
      const uint32_t tot = s_n[0] + s_n[1] + s_n[2] + s_n[3];
      s_b = tot ? atomicAdd(out_len, tot) : 0u;
    }
    __syncthreads();
    uint32_t b = s_b;
    for (uint32_t w = 0; w < wv; w++) b += s_n[w];
    if (keep) out[b + (uint32_t)__popcll(bm & ((1ull << lane) - 1ull))] = t;
    __syncthreads();
  }
}

// ---------------------------------------------------------------- compaction
// Between rounds the scan input shrinks to what can still matter: the last
// position of every group of an undecided or committed txn (aborted txns
// never constrain anyone; a group's other positions carry nothing).  Rows
// keep their order, so per-row index order is kept; row starts are
// recomputed from the slots.
__device__ inline bool mt_keep(uint8_t f, uint8_t st) {
  return (f & F_LAST) && (f & (F_R | F_W)) && st != ST_ABO;
}
__global__ __launch_bounds__(256) void k_mt_keep_count(uint64_t m, const uint8_t* sfl,
                                                       const uint32_t* stx, const uint8_t* state,
                                                       uint32_t* tcnt) {
  __shared__ uint32_t s_c[4];
  // the count only: positions in the striped order (coalesced loads)
  const uint64_t base = (uint64_t)blockIdx.x * MT_TILE;
  uint32_t c = 0;
#pragma unroll
  for (uint32_t i = 0; i < MT_ITEMS; i++) {
    const uint64_t p = base + i * 256 + threadIdx.x;
    if (p < m) {
      const uint8_t f = sfl[p];
      if ((f & F_LAST) && mt_keep(f, state[stx[p]])) c++;
    }
  }
  for (int d = 32; d > 0; d >>= 1) c += __shfl_xor(c, d);
  if ((threadIdx.x & 63) == 0) s_c[threadIdx.x >> 6] = c;
  __syncthreads();
  if (threadIdx.x == 0) tcnt[blockIdx.x] = s_c[0] + s_c[1] + s_c[2] + s_c[3];
}
// the kept positions of a tile, in order: blocked arrangement for the
// prefix (loads through LDS), the kept ones staged in LDS at their tile
// offsets, then stored with coalesced stores
__global__ __launch_bounds__(256) void k_mt_keep_scatter(uint64_t m, const uint8_t* sfl,
                                                         const uint32_t* stx, const uint32_t* ss,
                                                         const uint8_t* state, const uint32_t* tpre,
                                                         uint8_t* sfl2, uint32_t* stx2, uint32_t* ss2) {
  __shared__ uint32_t s_w[4];
  __shared__ MtTileLds L;
  __shared__ uint32_t s_ss[MT_TILE];
  const uint64_t base = (uint64_t)blockIdx.x * MT_TILE;
  const uint64_t n_here = m > base ? min<uint64_t>(MT_TILE, m - base) : 0;
  for (uint32_t q = threadIdx.x; q < MT_TILE; q += 256) s_ss[q] = q < n_here ? ss[base + q] : 0u;
  uint8_t f[MT_ITEMS];
  uint32_t tx[MT_ITEMS];
  mt_load_tile(sfl, stx, m, base, L, f, tx);  // (its barriers also cover s_ss)
  uint32_t keep = 0, c = 0;
#pragma unroll
  for (uint32_t i = 0; i < MT_ITEMS; i++)
    if ((f[i] & F_LAST) && mt_keep(f[i], state[tx[i]])) {
      keep |= 1u << i;
      c++;
    }
  // exclusive scan of c over the workgroup (thread order = position order)
  const uint32_t lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  uint32_t x = c;
  for (int d = 1; d < 64; d <<= 1) {
    const uint32_t y = __shfl_up(x, d);
    if (lane >= (uint32_t)d) x += y;
  }
  if (lane == 63) s_w[w] = x;
  __syncthreads();
  uint32_t q = x - c, tot = 0;
  for (uint32_t v = 0; v < 4; v++) {
    if (v < w) q += s_w[v];
    tot += s_w[v];
  }
  // stage the kept positions at their tile offsets (flags in L.f, txns in
  // L.x, slots back in s_ss once every thread holds its own)
  uint32_t sv[MT_ITEMS];
#pragma unroll
  for (uint32_t i = 0; i < MT_ITEMS; i++) sv[i] = s_ss[threadIdx.x * MT_ITEMS + i];
  __syncthreads();
  uint8_t* of = (uint8_t*)L.f;
  uint32_t* ox = (uint32_t*)L.x;
#pragma unroll
  for (uint32_t i = 0; i < MT_ITEMS; i++) {
    if (!((keep >> i) & 1u)) continue;
    of[q] = f[i] & (F_R | F_W | F_LAST);
    ox[q] = tx[i];
    s_ss[q] = sv[i];
    q++;
  }
  __syncthreads();
  const uint32_t ob = tpre[blockIdx.x];
  for (uint32_t j = threadIdx.x; j < tot; j += 256) {
    sfl2[ob + j] = of[j];
    stx2[ob + j] = ox[j];
    ss2[ob + j] = s_ss[j];
  }
}
__global__ __launch_bounds__(256) void k_mt_starts(uint64_t m, const uint32_t* ss, uint8_t* sfl) {
  for (uint64_t q = (uint64_t)blockIdx.x * 256 + threadIdx.x; q < m; q += (uint64_t)gridDim.x * 256)
    if (q == 0 || ss[q - 1] != ss[q]) sfl[q] |= F_START;
}

// ---------------------------------------------------------------- finish
// RC bytes, commit timestamps, counts; committed txns raise their rows'
// timestamps (Row_maat::commit, row_maat.cpp:249-251, 276-278)
struct FinArgs {
  uint64_t n, nnz;
  const uint32_t* off;
  const uint8_t* at;
  uint32_t rw_all;
  const uint8_t* state;
  const uint64_t* cts;
  const uint32_t* slot;
  MtSlot* rt;
  uint8_t* rc;
  uint64_t* cts_out;
  uint32_t* cnt;  // [0] commits, [1] undecided, [2] write accesses
  const uint32_t* err;
};
__global__ __launch_bounds__(256) void k_mt_finish(FinArgs a) {
  __shared__ uint32_t sh[3][4];
  uint32_t com = 0, und = 0, nw = 0;
  // a full row table left some accesses without their row: the epoch runs
  // again on a bigger table, and this one's timestamps must not land anywhere
  const bool keep = (*(volatile const uint32_t*)a.err & MT_ERR_FULL) == 0;
  for (uint64_t t = (uint64_t)blockIdx.x * 256 + threadIdx.x; t < a.n; t += (uint64_t)gridDim.x * 256) {
    const uint8_t s = a.state[t];
    const bool ok = s == ST_COM;
    a.rc[t] = ok ? DCC_RC_RCOK : DCC_RC_ABORT;
    if (a.cts_out) a.cts_out[t] = ok ? a.cts[t] : 0;
    com += ok;
    und += s == ST_UND;
    const uint64_t o0 = min((uint64_t)a.off[t], a.nnz), o1 = min((uint64_t)a.off[t + 1], a.nnz);
    const uint64_t c = ok ? a.cts[t] : 0;
    for (uint64_t x = o0; x < o1; x++) {
      const uint8_t ty = a.at[x];
      nw += ty == DCC_WR;
      if (!ok || !keep) continue;
      const uint32_t sl = a.slot[x];
      if (a.rw_all || ty == DCC_RD) atomicMax((unsigned long long*)&a.rt[sl].lr, c);
      if (a.rw_all || ty == DCC_WR) atomicMax((unsigned long long*)&a.rt[sl].lw, c);
    }
  }
  for (int d = 32; d > 0; d >>= 1) {
    com += __shfl_xor(com, d);
    und += __shfl_xor(und, d);
    nw += __shfl_xor(nw, d);
  }
  if ((threadIdx.x & 63) == 0) {
    sh[0][threadIdx.x >> 6] = com;
    sh[1][threadIdx.x >> 6] = und;
    sh[2][threadIdx.x >> 6] = nw;
  }
  __syncthreads();
  if (threadIdx.x < 3) {
    const uint32_t v = sh[threadIdx.x][0] + sh[threadIdx.x][1] + sh[threadIdx.x][2] + sh[threadIdx.x][3];
    if (v) atomicAdd(&a.cnt[threadIdx.x], v);
  }
}

inline unsigned g1(uint64_t n, uint64_t cap = 8192) {
  uint64_t g = (n + 255) / 256;
  return (unsigned)std::max<uint64_t>(1, std::min<uint64_t>(g, cap));
}

}  // namespace

// ---------------------------------------------------------------- prefix level
// The sweep idea: the epoch's first P txns are decided alone
// by rounds on their own accesses (a txn's constraints come only from earlier
// txns), then every later txn is checked against their commits -- per row the
// max commit timestamp of the committed prefix readers and the min of its
// writers (MtPTab, an open-addressing table on row slots) -- and aborted when
// its bounds are already empty: L only grows and U only shrinks as more
// earlier txns commit, so such a txn aborts in the full replay too.  The
// rounds then run on the survivors' accesses plus the prefix's (its commits
// constrain the survivors), so the first rounds scan ~2 M positions instead
// of the epoch's 16.7 M.
struct MtPTab {
  uint32_t* key;               // row slot, ~0u empty
  unsigned long long* rmax;    // max cts of committed prefix readers (0: none)
  unsigned long long* wmin;    // min cts of committed prefix writers (U64MAX: none)
  uint32_t mask;
  uint32_t* bits;              // one-hash presence bitmap of the slots (MT_PBITS bits)
};
constexpr uint32_t MT_PBITS_LOG = 18;  // 32 KiB: the filter's LDS copy
__device__ inline uint32_t mt_pbit(uint32_t s) { return (s * 0x9E3779B1u) >> (32 - MT_PBITS_LOG); }
__device__ inline uint32_t mt_phash(uint32_t s) { return (s * 2654435761u) ^ (s >> 15); }

// committed prefix txns' accesses into the table (16 lanes per prefix txn)
__global__ __launch_bounds__(256) void k_mt_ptab(const uint32_t* off, uint32_t P, const uint8_t* at, uint32_t rw_all,
                                                 const uint32_t* slot, const uint8_t* state, const uint64_t* cts,
                                                 MtPTab tb) {
  const uint32_t g = blockIdx.x * 256 + threadIdx.x, t = g >> 4;
  if (t >= P || state[t] != ST_COM) return;
  const uint64_t c = cts[t];
  for (uint32_t x = off[t] + (g & 15u); x < off[t + 1]; x += 16) {
    const uint8_t ty = at[x];
    const bool rd = rw_all || ty == DCC_RD, wr = rw_all || ty == DCC_WR;
    if (!rd && !wr) continue;
    const uint32_t sl = slot[x];
    uint32_t h = mt_phash(sl) & tb.mask;
    for (uint32_t q = 0; q <= tb.mask; q++, h = (h + 1) & tb.mask) {
      const uint32_t k = atomicCAS(&tb.key[h], ~0u, sl);
      if (k == ~0u || k == sl) break;
    }
    const uint32_t b = mt_pbit(sl);
    atomicOr(&tb.bits[b >> 5], 1u << (b & 31u));
    if (rd) atomicMax(&tb.rmax[h], (unsigned long long)c);
    if (wr) atomicMin(&tb.wmin[h], (unsigned long long)c);
  }
}

// every later access against the table: the round scan's folds (k_mt_round)
// with the committed prefix as the only earlier committed txns.  Persistent
// workgroups with the presence bitmap in LDS: an access whose bit is clear
// (almost every access of a row the prefix did not commit) never leaves the CU.
__global__ __launch_bounds__(256) void k_mt_filter(const uint32_t* slot, const uint32_t* sval, uint64_t x0,
                                                   uint64_t nnz, MtPTab tb, uint64_t* lacc, uint64_t* uacc) {
  __shared__ uint32_t s_bits[(1u << MT_PBITS_LOG) / 32];
  for (uint32_t q = threadIdx.x; q < (1u << MT_PBITS_LOG) / 32; q += 256) s_bits[q] = tb.bits[q];
  __syncthreads();
  constexpr uint32_t U = 4;
  for (uint64_t xb = x0 + (uint64_t)blockIdx.x * 256 * U; xb < nnz; xb += (uint64_t)gridDim.x * 256 * U) {
    uint32_t v[U], sl[U];
#pragma unroll
    for (uint32_t u = 0; u < U; u++) {
      const uint64_t x = min(xb + u * 256 + threadIdx.x, nnz - 1);
      v[u] = sval[x];
      sl[u] = slot[x];
    }
#pragma unroll
    for (uint32_t u = 0; u < U; u++) {
      if (xb + u * 256 + threadIdx.x >= nnz || !(v[u] & (SV_R | SV_W))) continue;
      const uint32_t b = mt_pbit(sl[u]);
      if (!((s_bits[b >> 5] >> (b & 31u)) & 1u)) continue;
      const uint32_t t = v[u] >> 2;
      uint32_t h = mt_phash(sl[u]) & tb.mask;
      for (uint32_t q = 0; q <= tb.mask; q++, h = (h + 1) & tb.mask) {
        const uint32_t k = tb.key[h];
        if (k == ~0u) break;
        if (k != sl[u]) continue;
        const uint64_t r = tb.rmax[h], w = tb.wmin[h];
        if ((v[u] & SV_W) && r) atomicMax((unsigned long long*)&lacc[t], (unsigned long long)(r + 1));
        if (w != U64MAX) atomicMin((unsigned long long*)&uacc[t], (unsigned long long)(w - 1));
        break;
      }
    }
  }
}

// the filter's decision for txns [P, n): abort when the bounds are empty
// (nothing commits here: later txns wait for the rounds); accumulators reset
__global__ __launch_bounds__(256) void k_mt_fdecide(uint64_t n, uint64_t P, const uint64_t* base, uint8_t* state,
                                                    uint64_t* lacc, uint64_t* uacc) {
  for (uint64_t t = P + (uint64_t)blockIdx.x * 256 + threadIdx.x; t < n; t += (uint64_t)gridDim.x * 256) {
    if (state[t] != ST_UND) continue;
    if (max(base[t], lacc[t]) >= uacc[t]) state[t] = ST_ABO;
    lacc[t] = 0;
    uacc[t] = U64MAX;
  }
}

// The prefix's rounds in one workgroup: its sorted positions (<= 16,384) and
// its txns' state (<= 1,024 txns, ids < 1,024) live in LDS, a round is a
// block scan plus the decisions, with barriers instead of launches and host
// checks -- the same per-round rule as k_mt_round + k_mt_decide (ms_elem /
// ms_comb over the state at the round's start, then every undecided txn
// decided from what the scan folded into it).
constexpr uint32_t MS_T = 1024, MS_ITEMS = 16, MS_MAXPOS = MS_T * MS_ITEMS, MS_MAXTXN = MS_T;
__global__ __launch_bounds__(MS_T) void k_mt_small(const uint8_t* sfl, const uint32_t* stx, uint32_t mp, uint32_t P,
                                                   const uint64_t* base, uint8_t* state, uint64_t* cts,
                                                   uint32_t* rounds_out) {
  __shared__ uint8_t s_f[MS_MAXPOS];
  __shared__ uint16_t s_t[MS_MAXPOS];
  __shared__ uint8_t s_st[MS_MAXTXN];
  __shared__ unsigned long long s_cts[MS_MAXTXN], s_l[MS_MAXTXN], s_u[MS_MAXTXN], s_b[MS_MAXTXN];
  __shared__ uint32_t s_pend[MS_MAXTXN];
  __shared__ Ms s_w[MS_T / 64];
  __shared__ uint32_t s_und[MS_T / 64];
  const uint32_t tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  for (uint32_t q = tid; q < MS_MAXPOS; q += MS_T) {
    s_f[q] = q < mp ? sfl[q] : (uint8_t)0;
    s_t[q] = q < mp ? (uint16_t)stx[q] : (uint16_t)0;
  }
  if (tid < P) {
    s_st[tid] = state[tid];
    s_b[tid] = base[tid];
    s_cts[tid] = 0;
    s_l[tid] = 0;
    s_u[tid] = U64MAX;
    s_pend[tid] = 0;
  }
  __syncthreads();
  uint32_t r = 0;
  for (;; r++) {
    // the thread's positions are read from LDS twice (fold, then down pass)
    // rather than held in registers across the block scan
    Ms acc = ms_id();
    for (uint32_t i = 0; i < MS_ITEMS; i++) {
      const uint8_t f = s_f[tid * MS_ITEMS + i];
      const uint32_t tx = s_t[tid * MS_ITEMS + i];
      const uint8_t st = (f & F_LAST) ? s_st[tx] : ST_ABO;
      acc = ms_comb(acc, ms_elem(f, st, st == ST_COM ? (uint64_t)s_cts[tx] : 0));
    }
    const Ms x = wave_incl_ms(acc);
    if (lane == 63) s_w[wv] = x;
    __syncthreads();
    Ms pre = ms_id();
    for (uint32_t w = 0; w < wv; w++) pre = ms_comb(pre, s_w[w]);
    Ms ex = ms_shfl_up(x, 1);
    if (lane == 0) ex = ms_id();
    Ms run = ms_comb(pre, ex);
    for (uint32_t i = 0; i < MS_ITEMS; i++) {
      if (tid * MS_ITEMS + i >= mp) break;
      const uint8_t f = s_f[tid * MS_ITEMS + i];
      const uint32_t t = s_t[tid * MS_ITEMS + i];
      const uint8_t st = (f & F_LAST) ? s_st[t] : ST_ABO;
      if (f & F_START) run = Ms{1, 0, 0, U64MAX};
      if ((f & F_LAST) && (f & (F_R | F_W)) && st == ST_UND) {
        if ((f & F_W) && run.rmax) atomicMax(&s_l[t], (unsigned long long)(run.rmax + 1));
        if (run.wmin != U64MAX) atomicMin(&s_u[t], (unsigned long long)(run.wmin - 1));
        if ((run.und & 2u) || ((f & F_W) && (run.und & 1u))) s_pend[t] = 1u;
      }
      run = ms_comb(run, ms_elem(f & ~F_START, st, st == ST_COM ? (uint64_t)s_cts[t] : 0));
    }
    __syncthreads();
    uint32_t und = 0;
    if (tid < P && s_st[tid] == ST_UND) {
      const uint64_t L = max((uint64_t)s_b[tid], (uint64_t)s_l[tid]);
      const uint64_t U = s_u[tid];
      if (L >= U) {
        s_st[tid] = ST_ABO;
      } else if (!s_pend[tid]) {
        s_st[tid] = ST_COM;
        s_cts[tid] = L;
      } else {
        und = 1;
      }
      s_l[tid] = 0;
      s_u[tid] = U64MAX;
      s_pend[tid] = 0;
    }
    for (int d = 32; d > 0; d >>= 1) und += __shfl_xor(und, d);
    if (lane == 0) s_und[wv] = und;
    __syncthreads();
    uint32_t tot = 0;
    for (uint32_t w = 0; w < MS_T / 64; w++) tot += s_und[w];
    if (tot == 0 || r > P + 8) break;  // uniform; the smallest undecided txn decides every round
    __syncthreads();  // s_w / s_und of the next round
  }
  if (tid < P) {
    state[tid] = s_st[tid];
    if (s_st[tid] == ST_COM) cts[tid] = s_cts[tid];
  }
  if (tid == 0) *rounds_out = r + 1;
}

// txns [0, P) as an undecided list
__global__ __launch_bounds__(256) void k_mt_iota(uint32_t* ul, uint32_t* ulen, uint32_t P) {
  for (uint32_t i = blockIdx.x * 256 + threadIdx.x; i < P; i += gridDim.x * 256) ul[i] = i;
  if (blockIdx.x == 0 && threadIdx.x == 0) *ulen = P;
}

// The rounds' input after the filter: the accesses of every txn that is not
// aborted (the prefix's commits and the survivors), in index order, as the
// sort's (slot, txn << 2 | R / W) pairs.  Per 256-txn block: its count, then
// (after the scan of the counts) its pairs at the block's base.
__device__ inline uint32_t mt_keep_len(const uint32_t* off, uint64_t n, const uint8_t* state, uint64_t t) {
  return (t < n && state[t] != ST_ABO) ? off[t + 1] - off[t] : 0u;
}
__global__ __launch_bounds__(256) void k_mt_gcount(const uint32_t* off, uint64_t n, const uint8_t* state,
                                                   uint32_t* bsum) {
  __shared__ uint32_t sh[4];
  const uint64_t t = (uint64_t)blockIdx.x * 256 + threadIdx.x;
  uint32_t c = mt_keep_len(off, n, state, t);
  for (int d = 32; d > 0; d >>= 1) c += __shfl_xor(c, d);
  if ((threadIdx.x & 63) == 0) sh[threadIdx.x >> 6] = c;
  __syncthreads();
  if (threadIdx.x == 0) bsum[blockIdx.x] = sh[0] + sh[1] + sh[2] + sh[3];
}
__global__ __launch_bounds__(256) void k_mt_gscatter(const uint32_t* off, uint64_t n, const uint8_t* state,
                                                     const uint8_t* at, uint32_t rw_all, const uint32_t* slot,
                                                     const uint32_t* bsum, uint32_t* okey, uint32_t* oval) {
  __shared__ uint32_t sh[4];
  const uint32_t lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const uint64_t t = (uint64_t)blockIdx.x * 256 + threadIdx.x;
  const uint32_t len = mt_keep_len(off, n, state, t);
  const uint32_t o0 = t < n ? off[t] : 0u;
  uint32_t x = len;  // inclusive prefix of the wave's kept lengths
  for (uint32_t d = 1; d < 64; d <<= 1) {
    const uint32_t y = __shfl_up(x, d);
    if (lane >= d) x += y;
  }
  if (lane == 63) sh[wv] = x;
  __syncthreads();
  uint32_t b = bsum[blockIdx.x];
  for (uint32_t w = 0; w < wv; w++) b += sh[w];
  const uint32_t tot = __shfl(x, 63), ex = x - len;
  // lanes over the wave's kept accesses (coalesced stores): output q belongs
  // to the first lane whose inclusive prefix exceeds q
  for (uint32_t q0 = 0; q0 < tot; q0 += 64) {
    const uint32_t q = q0 + lane;
    uint32_t lo = 0;
#pragma unroll
    for (uint32_t st = 32; st > 0; st >>= 1)
      if (__shfl(x, lo + st - 1) <= q) lo += st;
    const uint32_t src = __shfl(o0, lo) + (q - __shfl(ex, lo));
    const uint32_t tt = (uint32_t)(blockIdx.x * 256 + wv * 64 + lo);
    if (q < tot) {
      const uint8_t ty = at[src];
      const bool rd = rw_all || ty == DCC_RD, wr = rw_all || ty == DCC_WR;
      okey[b + q] = slot[src];
      oval[b + q] = (tt << 2) | (rd ? SV_R : 0u) | (wr ? SV_W : 0u);
    }
  }
}

// ---------------------------------------------------------------- host
// Row table capacity for `want` rows at <= 50 % load (rehash on growth).
int dcc_ctx::maat_rows_reserve(uint64_t want) {
  dcc_ctx* ctx = this;
  uint32_t* cnt = (uint32_t*)mt_misc.p;  // [0] rows, [1] errors
  if (mt_bits && (2 * want) <= (1ull << mt_bits)) return DCC_OK;
  uint32_t bits = std::max<uint32_t>(mt_bits, 12);
  while ((1ull << bits) < 2 * want) bits++;
  if (bits > 31) return fail(DCC_ERANGE, "maat: row table exceeds 2^31 slots");
  const uint64_t cap = 1ull << bits;
  DevBuf nt;
  CR(nt.ensure(this, cap * sizeof(MtSlot), "maat row table"));
  k_mt_clear<<<g1(cap, 16384), 256, 0, stream>>>((MtSlot*)nt.p, cap);
  CK(hipMemsetAsync(cnt, 0, 8, stream));
  if (mt_bits) {
    const uint64_t ocap = 1ull << mt_bits;
    k_mt_rehash<<<g1(ocap), 256, 0, stream>>>((const MtSlot*)mt_rk.p, ocap, (MtSlot*)nt.p, bits, cnt,
                                              cnt + 1);
  }
  CK(hipGetLastError());
  CK(hipMemcpyAsync(hmisc, cnt + 1, 4, hipMemcpyDeviceToHost, stream));
  CK(hipStreamSynchronize(stream));
  mt_rk.release();
  mt_rk = nt;
  mt_bits = bits;
  if (*(const uint32_t*)hmisc & MT_ERR_FULL) {  // a rehash walk ran past MT_WALK: bigger still
    CK(hipMemsetAsync(cnt + 1, 0, 4, stream));
    return maat_rows_reserve(2 * want);
  }
  return DCC_OK;
}

// The row table is sized for the rows the epoch is expected to add (the last
// epoch's count with a quarter of headroom, a quarter of the accesses the
// first time) instead of one row per access: at the headline 3.3 M distinct
// rows of 16.7 M accesses that is a 256-MB table instead of 1 GB.  An epoch
// that finds it full runs again on a table sized for every access.
int dcc_ctx::maat_epoch(const dcc_batch* b, uint8_t* out_rc, uint64_t* out_cts, dcc_stats* st) {
  bool full = false;
  const int e = maat_epoch_try(b, out_rc, out_cts, st, false, &full);
  if (e != DCC_OK || !full) return e;
  mt_full_redo++;
  const int e2 = maat_epoch_try(b, out_rc, out_cts, st, true, &full);
  if (e2 == DCC_OK && full) return fail(DCC_EIO, "maat: row table full");
  return e2;
}

int dcc_ctx::maat_epoch_try(const dcc_batch* b, uint8_t* out_rc, uint64_t* out_cts, dcc_stats* st,
                            bool all_rows, bool* full) {
  dcc_ctx* ctx = this;
  *full = false;
  const auto t_wall0 = std::chrono::steady_clock::now();
  CR(check_batch(b));
  if (comm_ranks() > 1) return fail(DCC_ENOTSUP, "maat: single-GPU engine");
  const bool dev = (b->flags & DCC_DEVICE_PTRS) != 0;
  const uint32_t rw_all = (b->flags & DCC_MAAT_READ_AND_PREWRITE) ? 1u : 0u;
  dcc_stats S;
  memset(&S, 0, sizeof S);
  S.n_shards = 1;
  if (b->n_txn == 0) {
    if (st) *st = S;
    return DCC_OK;
  }
  DevBatch d;
  CR(stage_batch(b, d));
  const uint64_t n = d.n, m = d.nnz;
  CR(mt_misc.ensure(this, 64 + MT_RING * 4, "maat counters"));
  uint32_t* cnt = (uint32_t*)mt_misc.p;  // [0] rows, [1] err, [2..4] finish counts, ring at 8
  uint32_t* ring = cnt + 8;
  // the row counter survives between epochs in mt_rows (host copy)
  {
    const uint64_t est = mt_new_last ? mt_new_last + mt_new_last / 4 + 4096 : m / 4 + 4096;
    CR(maat_rows_reserve(mt_rows + (all_rows ? m : std::min<uint64_t>(m, est))));
  }
  const uint64_t rows_before = mt_rows;
  mt_rows32 = (uint32_t)mt_rows;
  CK(hipMemcpyAsync(cnt, &mt_rows32, 4, hipMemcpyHostToDevice, stream));
  CK(hipMemsetAsync(cnt + 1, 0, 4 * 7 + MT_RING * 4, stream));
  const uint64_t mm = std::max<uint64_t>(m, 1);
  CR(mt_slot.ensure(this, mm * 4, "maat slots"));
  CR(mt_sval.ensure(this, mm * 4, "maat sort values"));
  CR(mt_slot2.ensure(this, mm * 4, "maat slots b"));
  CR(mt_sval2.ensure(this, mm * 4, "maat sort values b"));
  CR(mt_sfl.ensure(this, mm, "maat flags"));
  CR(mt_sflB.ensure(this, mm, "maat flags b"));
  CR(mt_stxB.ensure(this, mm * 4, "maat sorted txns b"));
  CR(mt_k1.ensure(this, mm * 4, "maat sort keys b"));
  CR(mt_tcnt.ensure(this, (std::max<uint64_t>((mm + MT_TILE - 1) / MT_TILE, (n + 255) / 256) + 2) * 4,
                     "maat tile / block counts"));
  CR(mt_stx.ensure(this, mm * 4, "maat sorted txns"));
  CR(mt_txn.ensure(this, n * (8 * 4 + 4 + 1) + 64, "maat txn state"));
  CR(cv_scratch.ensure(this, rs_scratch_words(mm) * 4 + 64, "radix scratch"));
  const uint64_t tiles = (m + MT_TILE - 1) / MT_TILE;
  CR(mt_agg.ensure(this, std::max<uint64_t>(1, tiles) * sizeof(Ms), "maat scan"));
  {
    // any reallocation is cleared, even at the old address (its grown tail
    // holds the previous owner's words; see occ_begin's fin_part)
    const size_t old_cap = mt_lb.cap;
    CR(mt_lb.ensure(this, std::max<uint64_t>(1, tiles) * sizeof(MtLb), "maat look-back status"));
    if (mt_lb.cap != old_cap || mt_tag + 64 >= (1u << 30)) {  // reallocated, or the tags wrap
      CK(hipMemsetAsync(mt_lb.p, 0, mt_lb.cap, stream));
      mt_tag = 0;
    }
  }
  uint64_t* base = (uint64_t*)mt_txn.p;
  uint64_t* cts = base + n;
  uint64_t* lacc = cts + n;
  uint64_t* uacc = lacc + n;
  uint32_t* pend = (uint32_t*)(uacc + n);
  uint8_t* state = (uint8_t*)(pend + n);
  CR(rc.ensure(this, n + 16, "rc"));
  uint8_t* rc_dev = (dev && out_rc) ? out_rc : (uint8_t*)rc.p;
  uint64_t* cts_dev = nullptr;
  if (out_cts) {
    if (dev) {
      cts_dev = out_cts;
    } else {
      CR(tn.ensure(this, n * 8, "maat cts"));
      cts_dev = (uint64_t*)tn.p;
    }
  }

  // reject a malformed batch before the row table changes (one small sync)
  k_mt_check<<<g1(std::max<uint64_t>(n, m), 2048), 256, 0, stream>>>(d.off, n, d.keys, m, cnt + 1);
  CK(hipGetLastError());
  CK(hipMemcpyAsync(hmisc, cnt + 1, 4, hipMemcpyDeviceToHost, stream));
  CK(hipStreamSynchronize(stream));
  {
    const uint32_t e = *(const uint32_t*)hmisc;
    if (e & MT_ERR_OFF) return fail(DCC_EINVAL, "batch: malformed offsets");
    if (e & MT_ERR_KEY) return fail(DCC_EINVAL, "batch: key equal to DCC_KEY_RESERVED");
  }
  CK(hipEventRecord(ev0, stream));
  // the check passed: the offsets cover every access once, so the base pass
  // writes every slot and sort value (no clears)
  BaseArgs ba{n,     m,     d.off, d.acctype, rw_all, d.keys, (MtSlot*)mt_rk.p, mt_bits,
              (uint32_t*)mt_slot.p, (uint32_t*)mt_slot2.p, cnt, (uint32_t*)mt_sval.p,
              base,  state, lacc,  uacc,      pend,   cnt + 1};
  k_mt_base<<<(unsigned)((n + 255) / 256), 256, 0, stream>>>(ba);  // a wave per 64 txns
  // rows sorted by slot (stable: index order within a row); the sorted slots
  // and the other key buffer become the two slot arrays of the compaction
  uint8_t* sflb[2] = {(uint8_t*)mt_sfl.p, (uint8_t*)mt_sflB.p};
  uint32_t* stxb[2] = {(uint32_t*)mt_stx.p, (uint32_t*)mt_stxB.p};
  uint32_t* ssb[2] = {(uint32_t*)mt_slot2.p, (uint32_t*)mt_k1.p};
  // sort the first mm pairs of (mt_slot2, mt_sval) and flag their groups
  // into sflb[0] / stxb[0]; ssb / svb point at the sorted pairs afterwards
  auto sort_groups = [&](uint64_t mm) {
    uint32_t* kk[2] = {(uint32_t*)mt_slot2.p, (uint32_t*)mt_k1.p};
    uint32_t* vb[2] = {(uint32_t*)mt_sval.p, (uint32_t*)mt_sval2.p};
    const int cur = mm ? radix_sort_u32(kk, vb, mm, mt_bits, (uint32_t*)cv_scratch.p, stream) : 0;
    ssb[0] = kk[cur];
    ssb[1] = kk[cur ^ 1];
    if (mm) k_mt_groups<<<g1(mm), 256, 0, stream>>>(ssb[0], vb[cur], mm, sflb[0], stxb[0]);
  };

  // ---- rounds: one, then MT_BATCH between host checks; after each check
  // the scan input is compacted to the groups that can still matter
  uint32_t rounds = 0;
  const bool mt_debug = DCC_ENV("DCC_MT_DEBUG") != nullptr;
  CR(mt_ul.ensure(this, 2 * n * 4 + 64, "maat undecided lists"));
  uint32_t* ul_buf[2] = {(uint32_t*)mt_ul.p, (uint32_t*)mt_ul.p + n};
  uint32_t* ulen_w = cnt + 5;  // two count words: cnt[5], cnt[6]
  uint32_t* tcnt = (uint32_t*)mt_tcnt.p;
  // Rounds until the txns of the undecided list (null: every txn) are all
  // decided, over the mc sorted positions in sflb[0] / stxb[0] / ssb[0]; the
  // list is compacted whenever the undecided count falls well below it
  // (into ul_buf[ub], alternating).
  auto solve = [&](uint64_t mc, const uint32_t* ul_cur, const uint32_t* ulen_cur, uint64_t ulen_host,
                   int ub) -> int {
    bool done = false;
    int cb = 0;  // current buffer set
    const uint32_t r0 = rounds;  // this solve's first round (no earlier count of its own)
    while (!done) {
      const uint32_t k0 = rounds;
      const uint64_t tiles_c = (mc + MT_TILE - 1) / MT_TILE;
      MtRoundArgs ra{mc, n, sflb[cb], stxb[cb], state, cts, lacc, uacc, pend, (Ms*)mt_agg.p};
      // one round per host check while the scan is long (each check may
      // compact it), MT_BATCH once it is short
      static const uint32_t batch = [] {  // DCC_MT_BATCH / DCC_MT_LONG: tuning experiments
        const char* e = DCC_ENV("DCC_MT_BATCH");
        return e && atoi(e) > 0 ? (uint32_t)atoi(e) : MT_BATCH;
      }();
      static const uint64_t long_scan = [] {
        const char* e = DCC_ENV("DCC_MT_LONG");
        return e && atoll(e) > 0 ? (uint64_t)atoll(e) : MT_LONG;
      }();
      const uint32_t nb = (rounds == 0 || mc > long_scan) ? 1u : batch;
      for (uint32_t q = 0; q < nb; q++, rounds++) {
        const uint32_t* prev = rounds > r0 ? &ring[(rounds - 1) % MT_RING] : nullptr;
        if (mc) {
          if (mt_tag + 1 >= (1u << 30)) {
            CK(hipMemsetAsync(mt_lb.p, 0, mt_lb.cap, stream));
            mt_tag = 0;
          }
          k_mt_round<<<(unsigned)tiles_c, 256, 0, stream>>>(ra, (MtLb*)mt_lb.p, ++mt_tag, cnt + 1, prev);
        }
        k_mt_decide<<<g1(ulen_host, 2048), 256, 0, stream>>>(n, ul_cur, ulen_cur, base, state, cts, lacc,
                                                              uacc, pend, &ring[rounds % MT_RING],
                                                              &ring[(rounds + 1) % MT_RING], prev);
      }
      if (mc) {
        k_mt_keep_count<<<(unsigned)tiles_c, 256, 0, stream>>>(mc, sflb[cb], stxb[cb], state, tcnt);
        rs_scan_one(tcnt, (uint32_t)tiles_c, tcnt + tiles_c, stream);
      }
      // the ring, the kept-position total and the error word into pinned
      // memory with one gather launch (three copies cost ~13 us of device time)
      GatherArgs ga{};
      ga.job[ga.n++] = CopyJob{ring, (uint32_t*)hmisc_dev, MT_RING};
      if (mc) ga.job[ga.n++] = CopyJob{tcnt + tiles_c, (uint32_t*)hmisc_dev + MT_RING, 1};
      ga.job[ga.n++] = CopyJob{cnt + 1, (uint32_t*)hmisc_dev + MT_RING + 1, 1};
      launch_gather(ga, stream);
      CK(hipGetLastError());
      CK(hipStreamSynchronize(stream));
      const uint32_t* hr = (const uint32_t*)hmisc;
      if (hr[MT_RING + 1] & MT_ERR_SPIN) return fail(DCC_EIO, "maat: round scan look-back timed out");
      if (hr[MT_RING + 1] & MT_ERR_FULL) return DCC_OK;  // the epoch runs again (maat_epoch)
      if (mt_debug)  // DCC_MT_DEBUG: undecided txns after each round, scan length
        for (uint32_t q = k0; q < rounds; q++)
          fprintf(stderr, "maat round %u: undecided %u, scan positions %llu\n", q + 1, hr[q % MT_RING],
                  (unsigned long long)mc);
      for (uint32_t q = k0; q < rounds; q++)
        if (hr[q % MT_RING] == 0) {
          rounds = q + 1;
          done = true;
          break;
        }
      if (!done && rounds > n + 8) return fail(DCC_EIO, "maat: rounds did not converge");
      if (!done) {
        const uint32_t und = hr[(rounds - 1) % MT_RING];
        if ((uint64_t)und * 10 < ulen_host * 3) {  // shrinks to < 30 %: worth a pass
          CK(hipMemsetAsync(ulen_w + ub, 0, 4, stream));
          k_mt_ucompact<<<g1(ulen_host, 2048), 256, 0, stream>>>(ul_cur, ulen_cur, n, state, ul_buf[ub],
                                                                ulen_w + ub);
          ul_cur = ul_buf[ub];
          ulen_cur = ulen_w + ub;
          ulen_host = und;
          ub ^= 1;
        }
      }
      if (!done && mc && (uint64_t)hr[MT_RING] * 10 <= mc * 9) {  // compact when it drops >= 10 %
        const uint64_t m2 = hr[MT_RING];
        k_mt_keep_scatter<<<(unsigned)tiles_c, 256, 0, stream>>>(mc, sflb[cb], stxb[cb], ssb[cb], state,
                                                               tcnt, sflb[cb ^ 1], stxb[cb ^ 1],
                                                               ssb[cb ^ 1]);
        if (m2) k_mt_starts<<<g1(m2), 256, 0, stream>>>(m2, ssb[cb ^ 1], sflb[cb ^ 1]);
        CK(hipGetLastError());
        cb ^= 1;
        mc = m2;
      }
    }
    return DCC_OK;
  };

  // the prefix level (DCC_MT_PREFIX txns, 0: off; epochs of > 4 prefixes)
  static const uint64_t prefix = [] {
    const char* e = DCC_ENV("DCC_MT_PREFIX");
    return e ? (uint64_t)atoll(e) : (uint64_t)MT_PREFIX;
  }();
  if (m != 0 && prefix != 0 && n > 4 * prefix) {
    const uint32_t P = (uint32_t)prefix;
    uint32_t mp = 0;
    {
      GatherArgs ga{};
      ga.job[ga.n++] = CopyJob{d.off + P, (uint32_t*)hmisc_dev, 1};
      launch_gather(ga, stream);
      CK(hipGetLastError());
      CK(hipStreamSynchronize(stream));
    }
    mp = *(const uint32_t*)hmisc;
    // 1. the prefix alone: its accesses are the first mp pairs of the base
    //    pass's (slot, value) buffers
    sort_groups(mp);
    uint32_t* small_rounds = cnt + 7;  // k_mt_small's round count (0: not used)
    if (P <= MS_MAXTXN && mp <= MS_MAXPOS) {
      k_mt_small<<<1, MS_T, 0, stream>>>(sflb[0], stxb[0], mp, P, base, state, cts, small_rounds);
      CK(hipGetLastError());
    } else {
      k_mt_iota<<<g1(P), 256, 0, stream>>>(ul_buf[0], ulen_w, P);
      CK(hipGetLastError());
      CR(solve(mp, ul_buf[0], ulen_w, P, 1));
    }
    // 2. its commits per row, then every later access against them
    uint64_t cap = 1024;
    while (cap < 4ull * std::max<uint32_t>(mp, 1)) cap <<= 1;
    const size_t pbytes = (1u << MT_PBITS_LOG) / 8;
    CR(mt_ptab.ensure(this, cap * 20 + pbytes, "maat prefix table"));
    MtPTab tb{(uint32_t*)mt_ptab.p, (unsigned long long*)((uint32_t*)mt_ptab.p + cap),
              (unsigned long long*)((uint32_t*)mt_ptab.p + cap) + cap, (uint32_t)(cap - 1),
              (uint32_t*)((char*)mt_ptab.p + cap * 20)};
    CK(hipMemsetAsync(tb.key, 0xFF, cap * 4, stream));
    CK(hipMemsetAsync(tb.rmax, 0, cap * 8, stream));
    CK(hipMemsetAsync(tb.wmin, 0xFF, cap * 8, stream));
    CK(hipMemsetAsync(tb.bits, 0, pbytes, stream));
    k_mt_ptab<<<(16 * P + 255) / 256, 256, 0, stream>>>(d.off, P, d.acctype, rw_all, (const uint32_t*)mt_slot.p,
                                                       state, cts, tb);
    const unsigned fgrid = (unsigned)std::max<uint64_t>(1, std::min<uint64_t>((m - mp + 1023) / 1024, 4ull * n_cu));
    k_mt_filter<<<fgrid, 256, 0, stream>>>((const uint32_t*)mt_slot.p, (const uint32_t*)mt_sval.p, mp, m, tb, lacc,
                                           uacc);
    k_mt_fdecide<<<g1(n - P), 256, 0, stream>>>(n, P, base, state, lacc, uacc);
    // 3. the survivors (undecided list) and the rounds' input: every access of
    //    a txn not aborted, in index order
    CK(hipMemsetAsync(ulen_w, 0, 4, stream));
    k_mt_ucompact<<<g1(n, 2048), 256, 0, stream>>>(nullptr, nullptr, n, state, ul_buf[0], ulen_w);
    const uint32_t nblk = (uint32_t)((n + 255) / 256);
    uint32_t* gb = tcnt;  // tile counts are free here (nblk <= tiles + 2)
    k_mt_gcount<<<nblk, 256, 0, stream>>>(d.off, n, state, gb);
    rs_scan_one(gb, nblk, gb + nblk, stream);
    k_mt_gscatter<<<nblk, 256, 0, stream>>>(d.off, n, state, d.acctype, rw_all, (const uint32_t*)mt_slot.p, gb,
                                            (uint32_t*)mt_slot2.p, (uint32_t*)mt_sval.p);
    CK(hipGetLastError());
    {
      GatherArgs ga{};
      ga.job[ga.n++] = CopyJob{gb + nblk, (uint32_t*)hmisc_dev, 1};
      ga.job[ga.n++] = CopyJob{ulen_w, (uint32_t*)hmisc_dev + 1, 1};
      ga.job[ga.n++] = CopyJob{small_rounds, (uint32_t*)hmisc_dev + 2, 1};
      launch_gather(ga, stream);
      CK(hipGetLastError());
      CK(hipStreamSynchronize(stream));
    }
    const uint32_t m2 = ((const uint32_t*)hmisc)[0], nsurv = ((const uint32_t*)hmisc)[1];
    rounds += ((const uint32_t*)hmisc)[2];  // the prefix's rounds when k_mt_small ran them
    if (mt_debug)
      fprintf(stderr, "maat prefix %u txns (%u accesses, %u rounds): %u survivors, %u positions\n", P, mp,
              rounds, nsurv, m2);
    if (nsurv) {
      sort_groups(m2);
      CK(hipGetLastError());
      CR(solve(m2, ul_buf[0], ulen_w, nsurv, 1));
    }
  } else {
    sort_groups(m);
    CK(hipGetLastError());
    CR(solve(m, nullptr, nullptr, n, 0));
  }
  FinArgs fa{n, m, d.off, d.acctype, rw_all, state, cts, (const uint32_t*)mt_slot.p,
             (MtSlot*)mt_rk.p, rc_dev, cts_dev, cnt + 2, cnt + 1};
  k_mt_finish<<<g1(n, 2048), 256, 0, stream>>>(fa);
  CK(hipGetLastError());
  CK(hipEventRecord(ev1, stream));
  if (!dev) {
    if (out_rc) CK(hipMemcpyAsync(out_rc, rc_dev, n, hipMemcpyDeviceToHost, stream));
    if (out_cts) CK(hipMemcpyAsync(out_cts, cts_dev, n * 8, hipMemcpyDeviceToHost, stream));
  }
  CK(hipMemcpyAsync(hmisc, cnt, 32, hipMemcpyDeviceToHost, stream));
  CK(hipStreamSynchronize(stream));
  const uint32_t* hc = (const uint32_t*)hmisc;
  mt_rows = hc[0];  // rows inserted this epoch stay in the table whatever follows
  if (hc[1] & MT_ERR_OFF) return fail(DCC_EINVAL, "batch: malformed offsets");
  if (hc[1] & MT_ERR_KEY) return fail(DCC_EINVAL, "batch: key equal to DCC_KEY_RESERVED");
  if (hc[1] & MT_ERR_FULL) {
    *full = true;
    return DCC_OK;
  }
  if (hc[1] & MT_ERR_SPIN) return fail(DCC_EIO, "maat: round scan look-back timed out");
  if (hc[3]) return fail(DCC_EIO, "maat: %u undecided transactions", hc[3]);
  mt_new_last = mt_rows - rows_before;
  float ms = 0;
  CK(hipEventElapsedTime(&ms, ev0, ev1));
  S.rounds = rounds;
  S.n_commit = hc[2];
  S.n_abort = n - hc[2];
  S.nnz_w = hc[4];
  S.alg_bytes = dcc_maat_alg_bytes(n, m);
  S.device_ms = ms;
  S.total_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t_wall0)
                   .count();
  if (st) *st = S;
  return DCC_OK;
}

extern "C" uint64_t dcc_maat_alg_bytes(uint64_t n_txn, uint64_t nnz) {
  // offsets, key + acctype per access, one 24-B row-table slot read (key,
  // lr, lw) and one timestamp update per access, RC byte + commit timestamp
  return 4 * (n_txn + 1) + 9 * nnz + 24 * nnz + 8 * nnz + n_txn + 8 * n_txn;
}

extern "C" int dcc_maat_validate_epoch(dcc_ctx* ctx, const dcc_batch* batch, uint8_t* out_rc,
                                       uint64_t* out_commit_ts, dcc_stats* out_stats) {
  if (!ctx) return DCC_EINVAL;
  if (ctx->multi) {  // the whole epoch on rank 0 (dcc_multi.cpp)
    dcc_ctx* s = dcc_multi_rank0(ctx);
    dcc_comm_state* const cm = s->comm;  // one GPU's engine: no collective
    s->comm = nullptr;
    const int e = s->maat_epoch(batch, out_rc, out_commit_ts, out_stats);
    s->comm = cm;
    if (e != DCC_OK) ctx->last_error = s->last_error;
    return e;
  }
  if (hipSetDevice(ctx->device) != hipSuccess) return DCC_ENODEV;
  return ctx->maat_epoch(batch, out_rc, out_commit_ts, out_stats);
}

extern "C" int dcc_maat_rows_clear(dcc_ctx* ctx) {
  if (!ctx) return DCC_EINVAL;
  if (ctx->multi) return dcc_maat_rows_clear(dcc_multi_rank0(ctx));
  if (hipSetDevice(ctx->device) != hipSuccess) return DCC_ENODEV;
  if (ctx->mt_bits) {
    const uint64_t cap = 1ull << ctx->mt_bits;
    k_mt_clear<<<g1(cap, 16384), 256, 0, ctx->stream>>>((MtSlot*)ctx->mt_rk.p, cap);
    if (hipGetLastError() != hipSuccess || hipStreamSynchronize(ctx->stream) != hipSuccess)
      return ctx->hip_fail(hipGetLastError(), "maat rows clear");
  }
  ctx->mt_rows = 0;
  return DCC_OK;
}

extern "C" int dcc_maat_rows_set(dcc_ctx* ctx, const uint64_t* keys, const uint64_t* last_read,
                                 const uint64_t* last_write, uint64_t n) {
  if (!ctx || (n && (!keys || !last_read || !last_write))) return DCC_EINVAL;
  if (ctx->multi) return dcc_maat_rows_set(dcc_multi_rank0(ctx), keys, last_read, last_write, n);
  if (n == 0) return DCC_OK;
  if (hipSetDevice(ctx->device) != hipSuccess) return DCC_ENODEV;
  CR(ctx->mt_misc.ensure(ctx, 64 + MT_RING * 4, "maat counters"));
  CR(ctx->maat_rows_reserve(ctx->mt_rows + n));
  DevBuf tmp;
  CR(tmp.ensure(ctx, n * 24, "maat seed"));
  uint64_t* t = (uint64_t*)tmp.p;
  uint32_t* cnt = (uint32_t*)ctx->mt_misc.p;
  ctx->mt_rows32 = (uint32_t)ctx->mt_rows;
  CK(hipMemcpyAsync(cnt, &ctx->mt_rows32, 4, hipMemcpyHostToDevice, ctx->stream));
  CK(hipMemsetAsync(cnt + 1, 0, 4, ctx->stream));
  CK(hipMemcpyAsync(t, keys, n * 8, hipMemcpyHostToDevice, ctx->stream));
  CK(hipMemcpyAsync(t + n, last_read, n * 8, hipMemcpyHostToDevice, ctx->stream));
  CK(hipMemcpyAsync(t + 2 * n, last_write, n * 8, hipMemcpyHostToDevice, ctx->stream));
  k_mt_seed<<<g1(n), 256, 0, ctx->stream>>>(t, t + n, t + 2 * n, n, (MtSlot*)ctx->mt_rk.p,
                                            ctx->mt_bits, cnt, cnt + 1);
  CK(hipGetLastError());
  uint32_t hc[2];
  CK(hipMemcpyAsync(hc, cnt, 8, hipMemcpyDeviceToHost, ctx->stream));
  CK(hipStreamSynchronize(ctx->stream));
  tmp.release();
  if (hc[1] & MT_ERR_KEY) return ctx->fail(DCC_EINVAL, "maat rows: key equal to DCC_KEY_RESERVED");
  if (hc[1] & MT_ERR_FULL) return ctx->fail(DCC_EIO, "maat: row table full");
  ctx->mt_rows = hc[0];
  return DCC_OK;
}

extern "C" int dcc_maat_rows_get(dcc_ctx* ctx, const uint64_t* keys, uint64_t* last_read,
                                 uint64_t* last_write, uint64_t n) {
  if (!ctx || (n && (!keys || !last_read || !last_write))) return DCC_EINVAL;
  if (ctx->multi) return dcc_maat_rows_get(dcc_multi_rank0(ctx), keys, last_read, last_write, n);
  if (n == 0) return DCC_OK;
  if (hipSetDevice(ctx->device) != hipSuccess) return DCC_ENODEV;
  if (!ctx->mt_bits) {
    memset(last_read, 0, n * 8);
    memset(last_write, 0, n * 8);
    return DCC_OK;
  }
  DevBuf tmp;
  CR(tmp.ensure(ctx, n * 24, "maat get"));
  uint64_t* t = (uint64_t*)tmp.p;
  CK(hipMemcpyAsync(t, keys, n * 8, hipMemcpyHostToDevice, ctx->stream));
  k_mt_get<<<g1(n), 256, 0, ctx->stream>>>(t, n, (const MtSlot*)ctx->mt_rk.p, ctx->mt_bits,
                                           t + n, t + 2 * n);
  CK(hipGetLastError());
  CK(hipMemcpyAsync(last_read, t + n, n * 8, hipMemcpyDeviceToHost, ctx->stream));
  CK(hipMemcpyAsync(last_write, t + 2 * n, n * 8, hipMemcpyDeviceToHost, ctx->stream));
  CK(hipStreamSynchronize(ctx->stream));
  tmp.release();
  return DCC_OK;
}

extern "C" uint64_t dcc_maat_rows_size(const dcc_ctx* ctx) {
  if (ctx && ctx->multi) return dcc_multi_sub((dcc_ctx*)ctx, 0)->mt_rows;
  return ctx ? ctx->mt_rows : 0;
}
