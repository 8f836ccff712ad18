// gfx950 kernels of the asynchronous OCC solver.
//
// The serial decision of txn i (central_validate in index order,
// occ.cpp:116-239) is the unique fixed point of
//
//   abort(i)  <=> some key K of i has a writer j < i with commit(j)
//   commit(i) <=> every writer j < i of every key K of i aborted
//
// For one key, every accessor sees the same thing: the FIRST non-aborted
// writer f(K) of K in txn order.  f(K) < i committed -> i is killed;
// f(K) < i undecided -> i waits; no such writer (or f(K) >= i) -> K is clear
// for i, for good.  So with each key's writers sorted by txn index and a
// per-key cursor that only ever moves past writers seen ABORTED (final), every
// fact a wave reads is either final or conservatively "wait" — stale reads
// cost a retry, never a wrong decision.  The solver therefore needs no
// rounds, no grid barriers and no host synchronisation: persistent waves
// claim chunks of txns in index order (a ticket), so every txn a chunk waits
// on sits in the same or an earlier chunk, held by a running wave, and the
// lowest undecided txn can always decide (no deadlock at any grid size).
//
//   k_acount    insert write keys, count writers per key (LDS-combined)
//   k_aalloc    allocate each key's writer segment (bump pointer)
//   k_ascatter  write the writer txn ids into their segments (LDS-combined)
//   k_asort     sort each segment by txn (thread per short segment,
//               workgroup bitonic in LDS for long ones)
//   k_async     the chunked asynchronous evaluation
#include <hip/hip_runtime.h>

#include "dcc_device.h"
#include "occ_kernels.h"

namespace dcc {

constexpr uint32_t AST_UND = 0, AST_COMMIT = 1, AST_ABORT = 2;
constexpr int COMB = 1024;  // LDS combiner slots per workgroup (sid -> count)

__device__ inline uint32_t ald(const uint32_t* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ inline void ast(uint32_t* p, uint32_t v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Per-workgroup LDS combiner sid -> (count, base): equal keys of a workgroup
// (zipf-hot rows) reach the global counter once instead of once per writer.
struct LdsCount {
  uint32_t sid[COMB];
  uint32_t cnt[COMB];
  uint32_t base[COMB];
  __device__ void init() {
    for (uint32_t q = threadIdx.x; q < COMB; q += blockDim.x) {
      sid[q] = SID_NONE;
      cnt[q] = 0;
    }
  }
  // slot of `s` in the combiner, or -1 when its probe window is full
  __device__ int find(uint32_t s, bool insert) {
    uint32_t h = (s * 2654435761u) >> (32 - 10);
#pragma unroll 1
    for (int q = 0; q < 8; q++) {
      const uint32_t cur = sid[h];
      if (cur == s) return (int)h;
      if (cur == SID_NONE) {
        if (!insert) return -1;
        const uint32_t prev = atomicCAS(&sid[h], SID_NONE, s);
        if (prev == SID_NONE || prev == s) return (int)h;
      }
      h = (h + 1) & (COMB - 1);
    }
    return -1;
  }
};

// Tile prologue shared by the preprocessing kernels: lane l < nt owns txn
// j0 + l; map[] gives the lane of every staged access (0xFF: none).
struct ATile {
  uint32_t nt, A0, A1;
  bool live;
};
__device__ inline ATile atile(const AsyncArgs& a, uint32_t tw, uint64_t j0, uint8_t* map,
                              bool& und, uint32_t& s, uint32_t& e) {
  const uint32_t lane = lane_id();
  ATile T;
  T.nt = j0 < a.m ? (uint32_t)min((uint64_t)tw, a.m - j0) : 0u;
  s = e = 0;
  und = false;
  if (lane < T.nt) {
    s = a.off[j0 + lane];
    e = a.off[j0 + lane + 1];
    und = a.state[j0 + lane] == ST_UNDECIDED;
  }
  T.A0 = T.A1 = 0;
  if (T.nt) {
    T.A0 = __shfl(s, 0);
    T.A1 = __shfl(e, T.nt - 1);
  }
  T.live = T.nt != 0 && T.A1 - T.A0 <= (uint32_t)ASYNC_CAP;
  if (T.nt && !T.live && lane == 0) atomicOr(a.err, ERR_TILE);
  if (T.live && lane < T.nt)
    for (uint32_t x = s; x < e; x++) map[x - T.A0] = und ? (uint8_t)lane : (uint8_t)0xFF;
  return T;
}

// ---------------------------------------------------------------------------
// k_acount: insert the write keys of undecided txns, count writers per key;
// also initialise the working state words.
template <int WAVES>
__global__ __launch_bounds__(WAVES * 64) void k_acount(AsyncArgs a) {
  __shared__ uint8_t s_map[WAVES][ASYNC_CAP];
  __shared__ uint8_t s_hw[WAVES][64], s_und[WAVES][64];
  __shared__ LdsCount comb;
  const uint32_t wv = threadIdx.x >> 6, lane = lane_id();
  uint8_t* map = s_map[wv];
  comb.init();
  __syncthreads();
  const uint64_t per = (uint64_t)WAVES * a.tw_pre;
  for (uint64_t c0 = (uint64_t)blockIdx.x * per; c0 < a.m; c0 += (uint64_t)gridDim.x * per) {
    const uint64_t j0 = c0 + (uint64_t)wv * a.tw_pre;
    bool und;
    uint32_t s, e;
    const ATile T = atile(a, a.tw_pre, j0, map, und, s, e);
    if (lane < T.nt)
      ast(&a.st32[j0 + lane],
          und ? AST_UND : a.state[j0 + lane] == ST_COMMIT ? AST_COMMIT : AST_ABORT);
    // has-write bytes cover every txn, decided ones too: the map of this
    // kernel names every txn's lane and s_und says which ones take part
    if (T.live && lane < T.nt)
      for (uint32_t x = s; x < e; x++) map[x - T.A0] = (uint8_t)lane;
    s_hw[wv][lane] = 0;
    s_und[wv][lane] = und ? 1 : 0;
    __syncthreads();
    if (T.live) {
      for (uint32_t x = T.A0 + lane; x < T.A1; x += 64) {
        const uint8_t at = a.acctype[x];
        const uint32_t l = map[x - T.A0];
        if (at == 1) s_hw[wv][l] = 1;
        if (!s_und[wv][l] || at != 1 /* WR */) continue;
        const uint64_t key = a.keys[x];
        if (key == KEY_EMPTY) {
          atomicOr(a.err, ERR_KEY);
          continue;
        }
        const uint32_t sid = table_insert(a.tab, a.mask, key);
        if (sid == SID_NONE) {
          atomicOr(a.err, ERR_FULL);
          continue;
        }
        const int c = comb.find(sid, true);
        if (c >= 0) atomicAdd(&comb.cnt[c], 1u);
        else atomicAdd(&a.wcnt[sid], 1u);
      }
    }
    __syncthreads();
    if (a.hasw && T.live && lane < T.nt) a.hasw[j0 + lane] = s_hw[wv][lane];
  }
  for (uint32_t q = threadIdx.x; q < COMB; q += blockDim.x)
    if (comb.sid[q] != SID_NONE) atomicAdd(&a.wcnt[comb.sid[q]], comb.cnt[q]);
}

// ---------------------------------------------------------------------------
// k_aclear: one launch clears the key table, the per-key counters and
// cursors, and the solver's device counters.
__global__ __launch_bounds__(256) void k_aclear(AsyncArgs a, uint64_t cap) {
  const uint64_t t0 = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const uint64_t st = (uint64_t)gridDim.x * blockDim.x;
  const uint4 ff = make_uint4(~0u, ~0u, ~0u, ~0u);
  for (uint64_t q = t0; q < cap; q += st) {
    *reinterpret_cast<uint4*>(&a.tab[q]) = ff;
    a.wcnt[q] = 0;
    a.cursor[q] = 0;
  }
  if (t0 == 0) {
    *a.bump = 0;
    *a.nbig = 0;
    *a.ticket = 0ull;
  }
}

// ---------------------------------------------------------------------------
// k_aalloc: segment start per key: ALLOC_PER consecutive keys per thread, a
// workgroup scan, one bump-pointer add per workgroup; keys with more than
// ASORT_SMALL writers are listed for the workgroup sort.
constexpr int ALLOC_PER = 8;
__global__ __launch_bounds__(256) void k_aalloc(AsyncArgs a) {
  __shared__ uint32_t s_w[4];
  __shared__ uint32_t s_base;
  const uint32_t lane = lane_id(), wv = threadIdx.x >> 6;
  const uint64_t s0 = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) * ALLOC_PER;
  uint32_t c[ALLOC_PER];
  uint32_t sum = 0;
#pragma unroll
  for (int q = 0; q < ALLOC_PER; q++) {
    c[q] = s0 + q <= a.mask ? a.wcnt[s0 + q] : 0u;
    sum += c[q];
  }
  uint32_t x = sum;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const uint32_t y = __shfl_up(x, d);
    if (lane >= (uint32_t)d) x += y;
  }
  if (lane == 63) s_w[wv] = x;
  __syncthreads();
  if (threadIdx.x == 0) {
    const uint32_t tot = s_w[0] + s_w[1] + s_w[2] + s_w[3];
    s_base = tot ? atomicAdd(a.bump, tot) : 0u;
  }
  __syncthreads();
  uint32_t run = s_base + x - sum;
  for (uint32_t k = 0; k < wv; k++) run += s_w[k];
#pragma unroll
  for (int q = 0; q < ALLOC_PER; q++) {
    if (s0 + q > a.mask) break;
    a.wstart[s0 + q] = run;
    a.wfill[s0 + q] = 0;
    if (c[q] > ASORT_SMALL) a.big[atomicAdd(a.nbig, 1u)] = (uint32_t)(s0 + q);
    run += c[q];
  }
}

// ---------------------------------------------------------------------------
// k_ascatter: writer txn ids into their key segments (unordered).
template <int WAVES>
__global__ __launch_bounds__(WAVES * 64) void k_ascatter(AsyncArgs a) {
  __shared__ uint8_t s_map[WAVES][ASYNC_CAP];
  __shared__ LdsCount comb;
  const uint32_t wv = threadIdx.x >> 6, lane = lane_id();
  uint8_t* map = s_map[wv];
  const uint64_t per = (uint64_t)WAVES * a.tw_pre;
  for (uint64_t c0 = (uint64_t)blockIdx.x * per; c0 < a.m; c0 += (uint64_t)gridDim.x * per) {
    comb.init();
    __syncthreads();
    const uint64_t j0 = c0 + (uint64_t)wv * a.tw_pre;
    bool und;
    uint32_t s, e;
    const ATile T = atile(a, a.tw_pre, j0, map, und, s, e);
    __syncthreads();
    // pass 1: count this step's writers per key in LDS
    uint32_t sidv[ASYNC_CAP / 64];
#pragma unroll
    for (int u = 0; u < ASYNC_CAP / 64; u++) {
      const uint32_t x = T.A0 + 64 * u + lane;
      sidv[u] = SID_NONE;
      if (T.live && x < T.A1 && map[x - T.A0] != 0xFFu && a.acctype[x] == 1) {
        const uint64_t key = a.keys[x];
        if (key != KEY_EMPTY) sidv[u] = table_find(a.tab, a.mask, key);
        if (sidv[u] != SID_NONE) {
          const int c = comb.find(sidv[u], true);
          if (c >= 0) atomicAdd(&comb.cnt[c], 1u);
        }
      }
    }
    __syncthreads();
    // reserve: one global add per (workgroup, key)
    for (uint32_t q = threadIdx.x; q < COMB; q += blockDim.x)
      if (comb.sid[q] != SID_NONE) {
        comb.base[q] = a.wstart[comb.sid[q]] + atomicAdd(&a.wfill[comb.sid[q]], comb.cnt[q]);
        comb.cnt[q] = 0;
      }
    __syncthreads();
    // pass 2: place
#pragma unroll
    for (int u = 0; u < ASYNC_CAP / 64; u++) {
      if (sidv[u] == SID_NONE) continue;
      const uint32_t x = T.A0 + 64 * u + lane;
      const uint32_t txn = (uint32_t)(j0 + map[x - T.A0]);
      const int c = comb.find(sidv[u], false);
      uint32_t pos;
      if (c >= 0) pos = comb.base[c] + atomicAdd(&comb.cnt[c], 1u);
      else pos = a.wstart[sidv[u]] + atomicAdd(&a.wfill[sidv[u]], 1u);
      a.writers[pos] = txn;
    }
    __syncthreads();
  }
}

// ---------------------------------------------------------------------------
// k_asort_small: thread per key, insertion sort of a short segment.
__global__ __launch_bounds__(256) void k_asort_small(AsyncArgs a) {
  const uint64_t sid = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (sid > a.mask) return;
  const uint32_t c = a.wcnt[sid];
  if (c < 2 || c > ASORT_SMALL) return;
  uint32_t v[ASORT_SMALL];
  uint32_t* p = a.writers + a.wstart[sid];
#pragma unroll
  for (int q = 0; q < ASORT_SMALL; q++) v[q] = q < (int)c ? p[q] : 0xFFFFFFFFu;
  // odd-even transposition network over the fixed width (registers only)
#pragma unroll
  for (int r = 0; r < ASORT_SMALL; r++) {
#pragma unroll
    for (int q = r & 1; q + 1 < ASORT_SMALL; q += 2) {
      const uint32_t lo = min(v[q], v[q + 1]), hi = max(v[q], v[q + 1]);
      v[q] = lo;
      v[q + 1] = hi;
    }
  }
#pragma unroll
  for (int q = 0; q < ASORT_SMALL; q++)
    if (q < (int)c) p[q] = v[q];
}

// k_asort_big: workgroup per long segment, bitonic sort in LDS (<= ASORT_BIG).
__global__ __launch_bounds__(1024) void k_asort_big(AsyncArgs a) {
  __shared__ uint32_t v[ASORT_BIG];
  const uint32_t nb = *a.nbig;
  for (uint32_t b = blockIdx.x; b < nb; b += gridDim.x) {
    const uint32_t sid = a.big[b];
    const uint32_t c = a.wcnt[sid];
    if (c > ASORT_BIG) {
      if (threadIdx.x == 0) atomicOr(a.err, ERR_SEG);
      continue;
    }
    uint32_t n2 = 1;
    while (n2 < c) n2 <<= 1;
    uint32_t* p = a.writers + a.wstart[sid];
    for (uint32_t q = threadIdx.x; q < n2; q += blockDim.x) v[q] = q < c ? p[q] : 0xFFFFFFFFu;
    __syncthreads();
    for (uint32_t k = 2; k <= n2; k <<= 1) {
      for (uint32_t j = k >> 1; j > 0; j >>= 1) {
        for (uint32_t q = threadIdx.x; q < n2; q += blockDim.x) {
          const uint32_t r = q ^ j;
          if (r > q) {
            const bool up = (q & k) == 0;
            const uint32_t x = v[q], y = v[r];
            if ((x > y) == up) {
              v[q] = y;
              v[r] = x;
            }
          }
        }
        __syncthreads();
      }
    }
    for (uint32_t q = threadIdx.x; q < c; q += blockDim.x) p[q] = v[q];
    __syncthreads();
  }
}

// ---------------------------------------------------------------------------
// k_async: persistent waves; a chunk (one wave tile of tw txns) is claimed by
// ticket in index order.  Per pending access the LDS holds its key's slot,
// the position of the candidate first non-aborted writer in the key's sorted
// segment and that writer's txn: a pass costs ONE state load per pending
// access, and only an aborted candidate makes it walk on (taking the shared
// cursor's progress).  Passes repeat until the chunk decides.
template <int WAVES>
__global__ __launch_bounds__(WAVES * 64) void k_async(AsyncArgs a) {
  __shared__ uint8_t s_map[WAVES][ASYNC_KCAP];
  __shared__ uint32_t s_sid[WAVES][ASYNC_KCAP];
  __shared__ uint32_t s_pos[WAVES][ASYNC_KCAP];
  __shared__ uint32_t s_cw[WAVES][ASYNC_KCAP];
  __shared__ uint32_t s_flag[WAVES][64];
  const uint32_t wv = threadIdx.x >> 6, lane = lane_id();
  uint8_t* map = s_map[wv];
  uint32_t* sidl = s_sid[wv];
  uint32_t* posl = s_pos[wv];
  uint32_t* cwl = s_cw[wv];
  if (*a.err & ERR_SEG) return;  // an unsorted segment: the host re-runs with rounds
  const uint64_t nchunk = (a.m + a.tw - 1) / a.tw;
  uint32_t max_pass = 0;
  for (;;) {
    uint64_t ch = 0;
    if (lane == 0) ch = atomicAdd(a.ticket, 1ull);
    ch = __shfl(ch, 0);
    if (ch >= nchunk) break;
    const uint64_t j0 = ch * a.tw;
    const uint32_t nt = (uint32_t)min((uint64_t)a.tw, a.m - j0);
    uint32_t s = 0, e = 0;
    bool und = false;
    if (lane < nt) {
      s = a.off[j0 + lane];
      e = a.off[j0 + lane + 1];
      und = a.state[j0 + lane] == ST_UNDECIDED;
    }
    const uint32_t A0 = __shfl(s, 0), A1 = __shfl(e, nt - 1);
    if (A1 - A0 > (uint32_t)ASYNC_KCAP) {
      if (lane == 0) atomicOr(a.err, ERR_TILE);
      continue;
    }
    if (lane < nt)
      for (uint32_t x = s; x < e; x++) map[x - A0] = und ? (uint8_t)lane : (uint8_t)0xFF;
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    const uint32_t i_own = (uint32_t)(j0 + lane);
    // stage: candidate first writer per access (clear at once when the key
    // has no writer before the txn)
    for (uint32_t x = A0 + lane; x < A1; x += 64) {
      uint32_t sid = SID_NONE;
      const uint32_t l = map[x - A0];
      if (l != 0xFFu) {
        const uint64_t key = a.keys[x];
        if (key != KEY_EMPTY) sid = table_find(a.tab, a.mask, key);
        if (sid != SID_NONE) {
          const uint32_t c = ald(&a.cursor[sid]);
          const uint32_t w = c < a.wcnt[sid] ? a.writers[a.wstart[sid] + c] : 0xFFFFFFFFu;
          if (w >= (uint32_t)(j0 + l)) sid = SID_NONE;
          posl[x - A0] = c;
          cwl[x - A0] = w;
        }
      }
      sidl[x - A0] = sid;
    }
    bool pend = lane < nt && und;  // this lane's txn is undecided
    uint32_t pass = 0;
    while (__ballot(pend)) {
      if (++pass > ASYNC_MAX_PASS) {
        if (lane == 0) atomicOr(a.err, ERR_ASYNC);
        break;
      }
      s_flag[wv][lane] = 0;  // bit0 blocked, bit1 killed
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
      for (uint32_t xb = A0; xb < A1; xb += 64) {  // uniform trip count
        const uint32_t x = xb + lane;
        uint32_t sid = SID_NONE, l = 0xFFu;
        if (x < A1) {
          sid = sidl[x - A0];
          l = map[x - A0];
        }
        const bool act = sid != SID_NONE && l != 0xFFu;
        const uint32_t i = (uint32_t)(j0 + (l & 63u));
        uint32_t res = 0;
        bool walk = false;
        if (act) {
          const uint32_t sw = ald(&a.st32[cwl[x - A0]]);
          if (sw == AST_ABORT) walk = true;
          else res = sw == AST_COMMIT ? 2u : 1u;
        }
        // walk on past aborted writers: one walk per distinct key among the
        // walking lanes (every accessor of a key sees the same first
        // non-aborted writer), 64 writers per step with their states loaded
        // in parallel
        uint64_t wm = __ballot(walk);
        while (wm) {
          const uint32_t L = (uint32_t)__builtin_ctzll(wm);
          const uint32_t sidL = __shfl(sid, L);
          const bool mine = walk && sid == sidL;
          wm &= ~__ballot(mine);
          uint32_t cL = __shfl(walk ? posl[x - A0] + 1 : 0u, L);
          const uint32_t baseL = a.wstart[sidL], lenL = a.wcnt[sidL];
          const uint32_t cg = ald(&a.cursor[sidL]);
          if (cg > cL) cL = cg;
          uint32_t wL = 0xFFFFFFFFu, sL = AST_UND;
          for (;;) {
            const uint32_t pos = cL + lane;
            uint32_t w2 = 0xFFFFFFFFu, st2 = AST_UND;
            bool stop = true;  // end of the segment
            if (pos < lenL) {
              w2 = a.writers[baseL + pos];
              st2 = ald(&a.st32[w2]);
              stop = st2 != AST_ABORT;
            }
            const uint64_t sm = __ballot(stop);
            if (sm) {
              const uint32_t f = (uint32_t)__builtin_ctzll(sm);
              wL = __shfl(w2, f);
              sL = __shfl(st2, f);
              cL += f;
              break;
            }
            cL += 64;
          }
          if (lane == 0 && cL > cg) atomicMax(&a.cursor[sidL], cL);
          if (mine) {
            // the key's first non-aborted writer is wL (none past the end)
            posl[x - A0] = cL;
            cwl[x - A0] = wL;
            if (cL >= lenL || wL >= i) {
              res = 0;
              sidl[x - A0] = SID_NONE;  // clear for good
            } else {
              res = sL == AST_COMMIT ? 2u : 1u;
            }
          }
        }
        if (act && res) atomicOr(&s_flag[wv][l], res);
      }
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
      if (pend) {
        const uint32_t f = s_flag[wv][lane];
        if (f & 2u) {
          ast(&a.st32[i_own], AST_ABORT);
          a.state[i_own] = ST_ABORT;
          pend = false;
          for (uint32_t x = s; x < e; x++) map[x - A0] = 0xFF;  // stop evaluating it
        } else if (f == 0u) {
          ast(&a.st32[i_own], AST_COMMIT);
          a.state[i_own] = ST_COMMIT;
          pend = false;
        }
      }
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
      if (__ballot(pend)) __builtin_amdgcn_s_sleep(1);
    }
    max_pass = max(max_pass, pass);
  }
  if (lane == 0 && max_pass) atomicMax(a.passes, max_pass);
}

// ---------------------------------------------------------------------------
static inline unsigned agrid(uint64_t m, uint32_t tw, unsigned waves, unsigned cap) {
  const uint64_t per = (uint64_t)waves * tw;
  uint64_t g = (m + per - 1) / per;
  if (g > cap) g = cap;
  return g ? (unsigned)g : 1u;
}
void launch_async(const AsyncArgs& a, uint64_t cap, unsigned n_cu, hipStream_t st) {
  uint64_t gc = (cap + 255) / 256;
  if (gc > (uint64_t)n_cu * 8) gc = (uint64_t)n_cu * 8;
  k_aclear<<<(unsigned)gc, 256, 0, st>>>(a, cap);
  k_acount<4><<<agrid(a.m, a.tw_pre, 4, n_cu * 8), 256, 0, st>>>(a);
  const uint64_t slots = (uint64_t)a.mask + 1;
  k_aalloc<<<(unsigned)((slots + 256 * ALLOC_PER - 1) / (256 * ALLOC_PER)), 256, 0, st>>>(a);
  k_ascatter<4><<<agrid(a.m, a.tw_pre, 4, n_cu * 8), 256, 0, st>>>(a);
  k_asort_small<<<(unsigned)((slots + 255) / 256), 256, 0, st>>>(a);
  k_asort_big<<<n_cu, 1024, 0, st>>>(a);
  k_async<ASYNC_WAVES><<<agrid(a.m, a.tw, ASYNC_WAVES, n_cu * 4), ASYNC_WAVES * 64, 0, st>>>(a);
}

}  // namespace dcc
