// gfx950 kernels of the OCC sweep solver.
//
// The serial decision (central_validate in index order, occ.cpp:116-239,
// then central_finish) is
//
//   abort(i)  <=>  some EARLIER committed txn j wrote a key i reads or writes
//
// so a txn that touches a key in the committed write set C of the txns before
// it is dead, whatever else happens.  Under contention C covers the hot rows
// after a few hundred txns, and almost every later txn dies on them.  The
// solver therefore alternates two very different passes over a LIST of txns
// (level 0 = the epoch in index order, level l+1 = the survivors of level l,
// still in index order):
//
//   k_sw_pre     (grid)   per 64-txn tile of the list's first p_max txns:
//                         stage the tile's keys, the local txn of every
//                         access and the intra-tile dependency masks
//                         dep[t] = {u < t : W_u and keys(t) intersect}
//   k_sw_seq     (1 CU)   the exact serial decision, tile by tile, with C in
//                         LDS: a txn dies if a key is in C or an earlier
//                         committed txn of its tile writes one of its keys
//                         (a bit-parallel fixed point over the 64 dep masks);
//                         committed write keys join C.  Stops at p_max txns
//                         or when C would outgrow its LDS table.
//   k_sw_filter  (grid)   one streaming pass over the rest of the list: a txn
//                         touching a key of C dies (its committed writer is
//                         earlier); the survivors are compacted in index
//                         order (decoupled look-back) into the next level.
//
// Exactness: a dead txn never commits, so it neither kills nor blocks anyone;
// a survivor's fate depends only on earlier survivors (every committed key
// before it that it touches would have killed it).  So deciding the survivors
// in their own order reproduces the serial replay (the argument of the prefix
// peel, occ_peel.hip).
#include <hip/hip_runtime.h>

#include "dcc_device.h"
#include "occ_kernels.h"

namespace dcc {

constexpr uint32_t SW_U = SW_TA / 1024;  // accesses per thread of a tile (1024 threads)
constexpr uint32_t SW_MAP = 8192;        // LDS key -> writer-mask map of k_sw_pre
constexpr uint64_t ST_INCL = 2ull << 62, ST_AGG = 1ull << 62;
constexpr uint64_t LB_VAL = (1ull << 62) - 1;
constexpr uint32_t LB_ACC_BITS = 34;
constexpr uint32_t SPIN_LIMIT = 1u << 22;

__device__ inline uint32_t sw_hash(uint64_t key, uint32_t log2s) {
  const uint32_t h = (uint32_t)key * 0x9E3779B1u ^ (uint32_t)(key >> 32) * 0x85EBCA77u;
  return h >> (32 - log2s);
}

// Level key table in global memory: 4-slot buckets (32 B) filled in slot
// order, so one read answers most lookups; a key's id is its slot.  Slots
// never change once set: a plain read that sees the key is exact and a stale
// EMPTY only costs a CAS.
__device__ inline uint32_t gtab_insert(uint64_t* gt, uint32_t gbits, uint64_t key) {
  const uint32_t nbm = (1u << (gbits - 2)) - 1u;
  uint32_t b = sw_hash(key, gbits - 2);
  for (uint32_t q = 0; q <= nbm; q++) {
#pragma unroll
    for (uint32_t i = 0; i < 4; i++) {
      uint64_t* slot = gt + 4 * b + i;
      const uint64_t v = *slot;
      if (v == key) return 4 * b + i;
      if (v == KEY_EMPTY) {
        const unsigned long long prev = atomicCAS((unsigned long long*)slot,
                                                  (unsigned long long)KEY_EMPTY,
                                                  (unsigned long long)key);
        if (prev == KEY_EMPTY || prev == key) return 4 * b + i;
      }
    }
    b = (b + 1) & nbm;
  }
  return 0;  // unreachable: the access budget keeps the table <= 50% full
}
// slot of `key`, or ~0u when absent
__device__ inline uint32_t gtab_find(const uint64_t* gt, uint32_t gbits, uint64_t key) {
  const uint32_t nbm = (1u << (gbits - 2)) - 1u;
  uint32_t b = sw_hash(key, gbits - 2);
  for (uint32_t q = 0; q <= nbm; q++) {
    const uint4* p = (const uint4*)(gt + 4 * b);
    const uint4 x = p[0], y = p[1];
    const uint64_t v0 = ((uint64_t)x.y << 32) | x.x, v1 = ((uint64_t)x.w << 32) | x.z;
    const uint64_t v2 = ((uint64_t)y.y << 32) | y.x, v3 = ((uint64_t)y.w << 32) | y.z;
    if (v0 == key) return 4 * b;
    if (v1 == key) return 4 * b + 1;
    if (v2 == key) return 4 * b + 2;
    if (v3 == key) return 4 * b + 3;
    if (v3 == KEY_EMPTY) return ~0u;
    b = (b + 1) & nbm;
  }
  return ~0u;
}

// Two Bloom-filter bits of a key (2^SW_BLOOM_LOG bits).
__device__ inline void bloom_bits(uint64_t key, uint32_t& b1, uint32_t& b2) {
  const uint32_t h = (uint32_t)key * 0x9E3779B1u ^ (uint32_t)(key >> 32) * 0x85EBCA77u;
  b1 = h >> (32 - SW_BLOOM_LOG);
  b2 = (h * 0xC2B2AE35u + 0x27D4EB2Fu) >> (32 - SW_BLOOM_LOG);
}

// LDS set of u64 keys in 4-slot buckets (32 B, two ds_read_b128 per bucket).
// A bucket fills in slot order and a key moves to the next bucket only when
// its bucket is full, so a bucket with a free last slot ends every chain:
// the common lookup is one bucket read, no loop, no divergence.
template <uint32_t S>
__device__ inline bool lset_find(const uint64_t* cs, uint64_t key) {
  constexpr uint32_t NB = S / 4, LB = __builtin_ctz(NB);
  uint32_t b = sw_hash(key, LB);
#pragma unroll 1
  for (uint32_t q = 0; q < NB; q++) {
    const uint4* p = (const uint4*)(cs + 4 * b);
    const uint4 x = p[0], y = p[1];
    const uint64_t v0 = ((uint64_t)x.y << 32) | x.x, v1 = ((uint64_t)x.w << 32) | x.z;
    const uint64_t v2 = ((uint64_t)y.y << 32) | y.x, v3 = ((uint64_t)y.w << 32) | y.z;
    if (v0 == key || v1 == key || v2 == key || v3 == key) return true;
    if (v3 == KEY_EMPTY) return false;
    b = (b + 1) & (NB - 1);
  }
  return false;
}
// true when the key was not yet present
template <uint32_t S>
__device__ inline bool lset_insert(uint64_t* cs, uint64_t key) {
  constexpr uint32_t NB = S / 4, LB = __builtin_ctz(NB);
  uint32_t b = sw_hash(key, LB);
#pragma unroll 1
  for (uint32_t q = 0; q < NB; q++) {
#pragma unroll
    for (uint32_t i = 0; i < 4; i++) {
      uint64_t* slot = cs + 4 * b + i;
      const uint64_t v = *slot;
      if (v == key) return false;
      if (v == KEY_EMPTY) {
        const unsigned long long prev = atomicCAS((unsigned long long*)slot,
                                                  (unsigned long long)KEY_EMPTY,
                                                  (unsigned long long)key);
        if (prev == KEY_EMPTY) return true;
        if (prev == key) return false;
      }
    }
    b = (b + 1) & (NB - 1);
  }
  return false;
}

// any bit of [lo, lo+len) in an LDS bitmap (len <= 64 for valid input)
__device__ inline bool range_any(const uint64_t* bm, uint32_t lo, uint32_t len) {
  if (len == 0) return false;
  const uint32_t hi = lo + len - 1;
  const uint32_t w0 = lo >> 6, w1 = hi >> 6;
  uint64_t acc = 0;
  for (uint32_t w = w0; w <= w1; w++) {
    uint64_t m = ~0ull;
    if (w == w0) m &= ~0ull << (lo & 63);
    if (w == w1) m &= ~0ull >> (63 - (hi & 63));
    acc |= bm[w] & m;
  }
  return acc != 0;
}
// first set bit at position >= lo and < hi, or hi
__device__ inline uint32_t range_next(const uint64_t* bm, uint32_t lo, uint32_t hi) {
  for (uint32_t w = lo >> 6; (w << 6) < hi; w++) {
    uint64_t v = bm[w];
    if (w == (lo >> 6)) v &= ~0ull << (lo & 63);
    if (v) {
      const uint32_t x = (w << 6) + (uint32_t)__builtin_ctzll(v);
      return x < hi ? x : hi;
    }
  }
  return hi;
}
__device__ inline void range_set(uint64_t* bm, uint32_t lo, uint32_t len) {
  if (len == 0) return;
  const uint32_t hi = lo + len - 1;
  const uint32_t w0 = lo >> 6, w1 = hi >> 6;
  for (uint32_t w = w0; w <= w1; w++) {
    uint64_t m = ~0ull;
    if (w == w0) m &= ~0ull << (lo & 63);
    if (w == w1) m &= ~0ull >> (63 - (hi & 63));
    atomicOr((unsigned long long*)&bm[w], (unsigned long long)m);
  }
}

__device__ inline uint64_t wave_or64(uint64_t v) {
#pragma unroll
  for (int d = 32; d > 0; d >>= 1) v |= __shfl_xor(v, d);
  return v;
}
__device__ inline uint64_t wave_sum64(uint64_t v) {
#pragma unroll
  for (int d = 32; d > 0; d >>= 1) v += __shfl_xor(v, d);
  return v;
}
__device__ inline uint32_t wave_max32(uint32_t v) {
#pragma unroll
  for (int d = 32; d > 0; d >>= 1) v = max(v, (uint32_t)__shfl_xor(v, d));
  return v;
}
__device__ inline uint32_t wave_excl_u32(uint32_t v, uint32_t& total) {
  const uint32_t lane = lane_id();
  uint32_t x = v;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const uint32_t y = __shfl_up(x, d);
    if (lane >= (uint32_t)d) x += y;
  }
  total = __shfl(x, 63);
  return x - v;
}
__device__ inline uint64_t lanemask_lt() {
  const uint32_t l = lane_id();
  return l ? (~0ull >> (64 - l)) : 0ull;
}

__device__ inline uint32_t list_len(const uint32_t* m_dev, uint32_t m_host) {
  return m_dev ? *m_dev : m_host;
}

// ---------------------------------------------------------------------------
// k_sw_pre: tile records (SwRec) of list txns [0, min(m, p_max)), 64 txns
// per tile: keys, (local txn | W << 7) bytes, spans and intra-tile masks.
__global__ __launch_bounds__(1024) void k_sw_pre(SwPreArgs a) {
  __shared__ uint64_t mkey[SW_MAP];
  __shared__ uint64_t mmask[SW_MAP];
  __shared__ uint64_t s_dep[SW_T];
  __shared__ uint32_t s_off[SW_T + 1];
  __shared__ uint64_t s_hw;
  __shared__ uint32_t s_bad;
  if (*a.abandon) return;
  const uint32_t m = list_len(a.m_dev, a.m_host);
  const uint32_t lim = min(m, a.p_max);
  const uint32_t ntiles = (lim + SW_T - 1) / SW_T;
  const uint32_t j = threadIdx.x, lane = lane_id();
  const uint64_t nnz = a.in.nnz;
  for (uint32_t k = blockIdx.x; k < ntiles; k += gridDim.x) {
    const uint32_t i0 = k * SW_T;
    const uint32_t nt = min(SW_T, lim - i0);
    if (j <= nt) s_off[j] = (uint32_t)min((uint64_t)a.in.off[i0 + j], nnz);
    if (j < SW_T) s_dep[j] = 0;
    if (j == 0) {
      s_hw = 0;
      s_bad = 0;
    }
    for (uint32_t q = j; q < SW_MAP; q += 1024) {
      mkey[q] = KEY_EMPTY;
      mmask[q] = 0;
    }
    __syncthreads();
    if (j < nt && s_off[j + 1] < s_off[j]) atomicOr(&s_bad, ERR_OFFSETS);
    const uint32_t A0 = s_off[0];
    __syncthreads();
    const uint32_t A1 = s_off[nt];
    const uint32_t cnt = A1 >= A0 ? A1 - A0 : 0u;
    if (cnt > SW_TA) s_bad |= ERR_TILE;  // benign race: same value
    __syncthreads();
    const uint32_t bad = s_bad;
    // the level's key table holds `budget` accesses: the serial pass stops here
    if (!bad && (uint64_t)A1 - min((uint64_t)a.in.off[0], nnz) > a.budget) {
      if (j == 0) {
        a.tinfo[k] = SwTile{0, SW_STOP, 0, 0};
        a.rec[k].nt = 0;
        a.rec[k].cnt = SW_STOP;
      }
      __syncthreads();
      continue;
    }
    if (bad) {
      if (j == 0) {
        atomicOr(a.err, bad);
        a.tinfo[k] = SwTile{0, 0, 0, 0};
        a.rec[k].nt = 0;
        a.rec[k].cnt = 0;
        a.rec[k].prekill = 0;
        a.rec[k].hasw = 0;
      }
      __syncthreads();
      continue;
    }
    uint64_t key[SW_U];
    uint32_t lt[SW_U];
    bool w[SW_U], v[SW_U];
#pragma unroll
    for (uint32_t u = 0; u < SW_U; u++) {
      const uint32_t xr = j + 1024 * u;
      v[u] = xr < cnt;
      key[u] = KEY_EMPTY;
      lt[u] = 0;
      w[u] = false;
      if (v[u]) {
        const uint32_t x = A0 + xr;
        key[u] = a.in.keys[x];
        if (key[u] == KEY_EMPTY) atomicOr(a.err, ERR_KEY);  // reserved: reported by the host
        w[u] = a.in.acctype[x] == 1;  // WR (occ.cpp:379-383)
        // largest t < nt with s_off[t] <= x (empty txns never own an access)
        uint32_t lo = 0, hi = nt;  // invariant: s_off[lo] <= x < s_off[hi]
        while (hi - lo > 1) {
          const uint32_t mid = (lo + hi) >> 1;
          if (s_off[mid] <= x) lo = mid;
          else hi = mid;
        }
        lt[u] = lo;
        const uint8_t pkv = (uint8_t)(lo | (w[u] ? 0x80u : 0u));
        // key id = its slot in the level's global key table (insert-or-find;
        // a slot never changes once set, so a plain read that sees the key is
        // exact and a stale EMPTY only costs a CAS)
        const uint32_t h = gtab_insert(a.gtab, a.gbits, key[u]);
        if (xr < SW_REC_ACC) {
          a.rec[k].id[xr] = h;
          a.rec[k].pk[xr] = pkv;
        } else {
          const uint64_t o = (uint64_t)k * (SW_TA - SW_REC_ACC) + (xr - SW_REC_ACC);
          a.id_ovf[o] = h;
          a.rp_ovf[o] = pkv;
        }
        if (w[u]) {
          uint32_t h = sw_hash(key[u], 13);
          for (uint32_t q = 0; q < SW_MAP; q++) {
            const unsigned long long prev = atomicCAS((unsigned long long*)&mkey[h],
                                                      (unsigned long long)KEY_EMPTY,
                                                      (unsigned long long)key[u]);
            if (prev == KEY_EMPTY || prev == key[u]) break;
            h = (h + 1) & (SW_MAP - 1);
          }
          atomicOr((unsigned long long*)&mmask[h], 1ull << lo);
        }
      }
      const uint64_t hw = wave_or64(v[u] && w[u] ? (1ull << lt[u]) : 0ull);
      if (lane == 0 && hw) atomicOr((unsigned long long*)&s_hw, (unsigned long long)hw);
    }
    __syncthreads();
#pragma unroll
    for (uint32_t u = 0; u < SW_U; u++) {
      if (!v[u]) continue;
      uint32_t h = sw_hash(key[u], 13);
      uint64_t wm = 0;
      for (uint32_t q = 0; q < SW_MAP; q++) {
        const uint64_t kv = mkey[h];
        if (kv == key[u]) {
          wm = mmask[h];
          break;
        }
        if (kv == KEY_EMPTY) break;
        h = (h + 1) & (SW_MAP - 1);
      }
      wm &= (1ull << lt[u]) - 1ull;  // earlier writers of the tile only
      if (wm) atomicOr((unsigned long long*)&s_dep[lt[u]], (unsigned long long)wm);
    }
    __syncthreads();
    if (j < SW_T) {
      const uint64_t r = (uint64_t)k * SW_T + j;
      a.rec[k].dep[j] = s_dep[j];
      a.rec[k].span[j] = j < nt ? (s_off[j] - A0) | ((s_off[j + 1] - s_off[j]) << 16) : 0u;
      a.rtid[r] = j < nt ? (a.in.tid ? a.in.tid[i0 + j] : i0 + j) : 0u;
      // identity lists carry decisions made before the solver (history window)
      const bool pre = j < nt && a.state && a.state[i0 + j] != ST_UNDECIDED;
      const uint64_t pk = ballot64(pre);
      if (j == 0) {
        a.tinfo[k] = SwTile{nt, cnt, pk, s_hw};
        a.rec[k].nt = nt;
        a.rec[k].cnt = cnt;
        a.rec[k].prekill = pk;
        a.rec[k].hasw = s_hw;
      }
    }
    __syncthreads();  // LDS reuse by the next tile
  }
}

// ---------------------------------------------------------------------------
// k_sw_seq: one workgroup decides the tiles in order (see header).  Tile
// records reach LDS SW_SEQ_B at a time as one contiguous copy whose loads
// are issued a super-step ahead (registers), so the loop itself touches
// global memory only on the rare long-tile path; decisions and C go out
// after the last tile.
constexpr uint32_t SEQ_N16 = SW_SEQ_B * sizeof(SwRec) / 16;  // uint4 per super-step
constexpr uint32_t SEQ_R = (SEQ_N16 + 1023) / 1024;           // uint4 per thread
static_assert(sizeof(SwRec) == 6144, "SwRec layout");
static_assert(SEQ_R == 3, "super-step copy width");

__global__ __launch_bounds__(1024) void k_sw_seq(SwSeqArgs a) {
  __shared__ __attribute__((aligned(16))) SwRec ring[SW_SEQ_B];
  __shared__ uint32_t cbits[(1u << SW_GBITS_MAX) / 32];  // committed set over key ids
  __shared__ uint64_t s_hit[SW_TA / 64];
  __shared__ uint64_t s_M[SW_PMAX_TILES];  // commit mask per decided tile
  __shared__ uint64_t s_stamp[128 * 4];    // DCC_SW_DEBUG clock stamps
  __shared__ uint32_t sbloom[(1u << SW_BLOOM_LOG) / 32];
  __shared__ uint32_t s_cnt;
  const uint32_t j = threadIdx.x, lane = lane_id(), wv = j >> 6;
  if (*a.abandon) return;
  const uint32_t m = list_len(a.m_dev, a.m_host);
  const uint32_t lim = min(m, a.p_max);
  const uint32_t ntiles = min((lim + SW_T - 1) / SW_T, SW_PMAX_TILES);
  for (uint32_t q = j; q < (1u << SW_BLOOM_LOG) / 32; q += 1024) sbloom[q] = 0;
  const uint32_t nsup = (ntiles + SW_SEQ_B - 1) / SW_SEQ_B;
  // the filter of this level starts from a clean look-back and ticket; the
  // next level's list is empty unless the filter writes it
  for (uint32_t q = j; q < a.status_n; q += 1024) a.status[q] = 0;
  if (j == 0) {
    a.lv->ticket = 0;
    a.lv_next->m = 0;
    a.lv_next->acc = 0;
    a.next_off[0] = 0;
    s_cnt = 0;
  }
  const uint32_t nwords = (1u << a.gbits) / 32;
  for (uint32_t q = j; q < nwords; q += 1024) cbits[q] = 0;

  const uint4* src = (const uint4*)a.rec;
  uint4* dst = (uint4*)ring;
  // named registers per thread: an array captured by a lambda would live in
  // scratch
  uint4 R0, R1, R2;
  const uint32_t c0 = j, c1 = j + 1024, c2 = min(j + 2048, SEQ_N16 - 1);
#define SEQ_LOAD(sidx)                                     \
  do {                                                     \
    const uint4* p_ = src + (uint64_t)(sidx) * SEQ_N16;    \
    R0 = p_[c0];                                           \
    R1 = p_[c1];                                           \
    R2 = p_[c2];                                           \
  } while (0)
#define SEQ_STORE()  \
  do {               \
    dst[c0] = R0;    \
    dst[c1] = R1;    \
    dst[c2] = R2;    \
  } while (0)
  uint64_t* dbg = a.dbg;
  auto stamp = [&](uint32_t k, uint32_t i) {
    if (dbg && j == 0 && k < 128) s_stamp[k * 4 + i] = clock64();
  };

  // one tile; false = stopped before it (C at capacity, or the level's
  // access budget ends)
  auto step = [&](const SwRec& T, uint32_t k) -> bool {
    const uint32_t nt = T.nt, cnt = T.cnt;
    if ((uint64_t)s_cnt + cnt > a.cap) return false;  // uniform: read after a barrier
    stamp(k, 0);
    uint32_t xi[SW_U], xp[SW_U];
    xi[0] = T.id[j];
    xp[0] = T.pk[j];
#pragma unroll
    for (uint32_t u = 1; u < SW_U; u++) {  // long tiles: accesses beyond the record
      xi[u] = 0;
      xp[u] = 0;
      if (j + 1024 * u < cnt) {
        const uint64_t o = (uint64_t)k * (SW_TA - SW_REC_ACC) + j + 1024 * (u - 1);
        xi[u] = a.id_ovf[o];
        xp[u] = a.rp_ovf[o];
        // consume here: loads still pending at the merge would make the
        // common path wait for the super-step prefetch (vmcnt is in order)
        asm volatile("" ::"v"(xi[u]), "v"(xp[u]));
      }
    }
    // (1) probe C (one bitmap word per access); hit ballots into the tile bitmap
#pragma unroll
    for (uint32_t u = 0; u < SW_U; u++) {
      if (u && cnt <= 1024 * u) break;  // uniform
      const uint32_t xr = j + 1024 * u;
      const bool hit = xr < cnt && ((cbits[xi[u] >> 5] >> (xi[u] & 31u)) & 1u);
      const uint64_t b = ballot64(hit);
      if (lane == 0) s_hit[wv + 16 * u] = b;
    }
    __syncthreads();
    stamp(k, 1);
    // (2) wave 0: kills, then the tile's serial order as a fixed point over
    // the dependency masks
    if (wv == 0) {
      const bool valid = lane < nt;
      bool kill = ((T.prekill >> lane) & 1ull) != 0;
      const uint32_t span = T.span[lane];
      if (valid && !kill) kill = range_any(s_hit, span & 0xFFFFu, span >> 16);
      uint64_t U = ballot64(valid && !kill), M = 0;
      const uint64_t dep = T.dep[lane];
#pragma unroll 1
      while (U) {
        const bool mine = ((U >> lane) & 1ull) != 0;
        const bool c = mine && (dep & (M | U)) == 0;
        const bool ab = mine && (dep & M) != 0;
        const uint64_t cm = ballot64(c), am = ballot64(ab);
        M |= cm;
        U &= ~(cm | am);
      }
      if (lane == 0) s_M[k] = M;
    }
    __syncthreads();
    stamp(k, 2);
    // (3) committed write keys join C
    const uint64_t M = s_M[k];
#pragma unroll
    for (uint32_t u = 0; u < SW_U; u++) {
      if (u && cnt <= 1024 * u) break;
      const uint32_t xr = j + 1024 * u;
      const uint32_t pk = xp[u];
      bool nw = false;
      if (xr < cnt && (pk & 0x80u) && ((M >> (pk & 63u)) & 1ull)) {
        const uint32_t bit = 1u << (xi[u] & 31u);
        nw = (atomicOr(&cbits[xi[u] >> 5], bit) & bit) == 0;
      }
      const uint64_t nb = ballot64(nw);  // one counter atomic per wave
      if (lane == 0 && nb) atomicAdd(&s_cnt, (uint32_t)__popcll(nb));
    }
    __syncthreads();
    stamp(k, 3);
    return true;
  };

  __syncthreads();
  if (nsup) {
    SEQ_LOAD(0);
    SEQ_STORE();
  }
  __syncthreads();
  uint32_t k = 0;
  bool stop = false;
  for (uint32_t sidx = 0; sidx < nsup && !stop; sidx++) {
    SEQ_LOAD(min(sidx + 1, nsup - 1));  // unconditional: exact wait counts
#pragma unroll 1
    for (uint32_t b = 0; b < SW_SEQ_B; b++) {
      if (k >= ntiles || !step(ring[b], k)) {
        stop = true;
        break;
      }
      k++;
    }
    if (stop || sidx + 1 == nsup) break;
    SEQ_STORE();  // every wave passed the last step's barrier: the ring is free
    __syncthreads();
  }
#undef SEQ_LOAD
#undef SEQ_STORE
  // ---- write-out: decisions of tiles [0, k), the level's committed keys
  for (uint32_t q = j; q < k * SW_T; q += 1024) {
    const uint32_t kk = q / SW_T, t = q % SW_T;
    const SwTile ti = a.tinfo[kk];
    if (t >= ti.nt) continue;
    const uint32_t tid = a.rtid[q];
    if (!((ti.prekill >> t) & 1ull)) a.state[tid] = ((s_M[kk] >> t) & 1ull) ? ST_COMMIT : ST_ABORT;
    if (a.write_hasw) a.hasw[tid] = (uint8_t)((ti.hasw >> t) & 1ull);
  }
  // C for the filter: the committed-id bitmap and a Bloom filter of the keys
  for (uint32_t q = j; q < nwords; q += 1024) {
    uint32_t w = cbits[q];
    a.cbits_out[q] = w;
    while (w) {
      const uint32_t id = q * 32 + (uint32_t)__builtin_ctz(w);
      w &= w - 1;
      uint32_t b1, b2;
      bloom_bits(a.gtab[id], b1, b2);
      atomicOr(&sbloom[b1 >> 5], 1u << (b1 & 31));
      atomicOr(&sbloom[b2 >> 5], 1u << (b2 & 31));
    }
  }
  __syncthreads();
  for (uint32_t q = j; q < (1u << SW_BLOOM_LOG) / 32; q += 1024) a.bloom_out[q] = sbloom[q];
  const uint32_t ncid = s_cnt;
  if (dbg)
    for (uint32_t q = j; q < min(k, 128u) * 4; q += 1024) dbg[q] = s_stamp[q];
  if (j == 0) {
    a.lv->pos = min(k * SW_T, lim);
    a.lv->ccount = ncid;
  }
}

// ---------------------------------------------------------------------------
// k_sw_filter: list txns [pos, m) against C; survivors -> next level's list.
// Chunks of SW_CHUNK txns are taken by ticket (so every chunk a look-back
// waits on is held by a running workgroup); 16 waves x 64 txns per chunk.
__device__ inline uint64_t lb_pack(uint32_t t, uint64_t acc) {
  return ((uint64_t)t << LB_ACC_BITS) | acc;
}

// wave 0: decoupled look-back; returns the exclusive prefix of chunk c
__device__ uint64_t lookback(unsigned long long* status, uint32_t c, uint64_t agg, uint32_t* err) {
  const uint32_t lane = lane_id();
  if (c == 0) {
    if (lane == 0) __hip_atomic_store(&status[0], ST_INCL | agg, __ATOMIC_RELAXED,
                                      __HIP_MEMORY_SCOPE_AGENT);
    return 0;
  }
  if (lane == 0)
    __hip_atomic_store(&status[c], ST_AGG | agg, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  uint64_t excl = 0;
  int64_t j0 = (int64_t)c - 1;
  uint32_t spins = 0;
  for (;;) {
    const int64_t idx = j0 - (int64_t)lane;
    const unsigned long long v =
        idx >= 0 ? __hip_atomic_load(&status[idx], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
                 : ST_INCL;
    const uint32_t fl = (uint32_t)(v >> 62);
    const uint64_t notready = ballot64(fl == 0);
    const uint64_t incl = ballot64(fl == 2);
    const uint32_t fi = incl ? (uint32_t)__builtin_ctzll(incl) : 64u;
    const uint64_t need = fi >= 63 ? ~0ull : ((2ull << fi) - 1ull);
    if (notready & need) {
      if (++spins > SPIN_LIMIT) {
        if (lane == 0) atomicOr(err, ERR_SPIN);
        break;
      }
      __builtin_amdgcn_s_sleep(1);
      continue;
    }
    excl += wave_sum64(lane <= fi ? (uint64_t)(v & LB_VAL) : 0ull);
    if (fi < 64) break;
    j0 -= 64;
  }
  if (lane == 0)
    __hip_atomic_store(&status[c], ST_INCL | (excl + agg), __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_AGENT);
  return excl;
}

constexpr uint32_t FW = SW_CHUNK / 64;  // waves per filter workgroup
constexpr uint32_t FK = 16;             // access rounds kept in registers (1024 accesses)

// exact membership of a Bloom-positive key: its slot in the level's key
// table (a committed key always has one), then the committed-id bit
__device__ inline bool c_exact(const SwFilterArgs& a, uint64_t key) {
  const uint32_t id = gtab_find(a.gtab, a.gbits, key);
  return id != ~0u && ((a.cbits[id >> 5] >> (id & 31u)) & 1u);
}

__global__ __launch_bounds__(SW_CHUNK) void k_sw_filter(SwFilterArgs a) {
  __shared__ uint32_t bl[(1u << SW_BLOOM_LOG) / 32];
  __shared__ uint64_t s_hit[FW][SW_TA / 64];
  __shared__ uint64_t s_wr[FW][SW_TA / 64];
  __shared__ uint64_t s_sv[FW][SW_TA / 64];
  __shared__ uint32_t s_wt[FW], s_wa[FW];
  __shared__ uint64_t s_base;
  __shared__ uint32_t s_c;
  const uint32_t j = threadIdx.x, lane = lane_id(), wv = j >> 6;
  if (*a.abandon) return;
  uint64_t* fdbg = a.dbg ? a.dbg + (uint64_t)(blockIdx.x & 255) * 8 : nullptr;
  if (blockIdx.x > 255) fdbg = nullptr;
  if (fdbg && j == 0) fdbg[0] = clock64();
  const uint32_t m = list_len(a.m_dev, a.m_host);
  const uint32_t pos = a.lv->pos;
  // the next level's key table (its pre-pass runs after this kernel)
  for (uint64_t q = (uint64_t)blockIdx.x * SW_CHUNK + j; q < a.gclear_n;
       q += (uint64_t)gridDim.x * SW_CHUNK)
    a.gclear[q] = KEY_EMPTY;
  if (pos >= m) return;
  const uint32_t nchunks = (m - pos + SW_CHUNK - 1) / SW_CHUNK;
  const uint64_t nnz = a.in.nnz;
  {
    const uint4* src = (const uint4*)a.bloom;
    uint4* dst = (uint4*)bl;
    for (uint32_t q = j; q < (1u << SW_BLOOM_LOG) / 128; q += SW_CHUNK) dst[q] = src[q];
  }
  __syncthreads();
  if (fdbg && j == 0) fdbg[1] = clock64();
  uint32_t nchunk_done = 0;
  uint64_t* hit = s_hit[wv];
  uint64_t* wr = s_wr[wv];
  uint64_t* sv = s_sv[wv];
  for (;;) {
    if (j == 0) s_c = atomicAdd(&a.lv->ticket, 1u);
    __syncthreads();
    const uint32_t c = s_c;
    if (c >= nchunks) break;
    // ---- this wave's 64 list txns
    const uint32_t p = pos + c * SW_CHUNK + wv * 64 + lane;
    const bool valid = p < m;
    uint32_t s = 0, e = 0, tid = 0;
    bool cand = false;
    if (valid) {
      s = (uint32_t)min((uint64_t)a.in.off[p], nnz);
      e = (uint32_t)min((uint64_t)a.in.off[p + 1], nnz);
      if (e < s) e = s;
      tid = a.in.tid ? a.in.tid[p] : p;
      cand = a.cand_state ? a.state[p] == ST_UNDECIDED : true;
    }
    const uint64_t vm = ballot64(valid);
    const uint32_t A0 = vm ? __shfl(s, 0) : 0u;
    const uint32_t A1 = wave_max32(valid ? e : 0u);
    uint32_t span = A1 > A0 ? A1 - A0 : 0u;
    if (span > SW_TA) {  // malformed offsets (the host reports them): skip
      if (lane == 0) atomicOr(a.err, ERR_TILE);
      span = 0;
    }
    const uint32_t nw = (span + 63) / 64;
    for (uint32_t q = lane; q < nw; q += 64) sv[q] = 0;
    // probe every access: FK loads in flight per lane, kept for the copy
    uint64_t key[FK];
    uint8_t at[FK];
    for (uint32_t b0 = 0; b0 < span; b0 += 64 * FK) {
#pragma unroll
      for (uint32_t u = 0; u < FK; u++) {
        const uint32_t xr = b0 + 64 * u + lane;
        const uint32_t x = A0 + (xr < span ? xr : 0u);
        key[u] = a.in.keys[x];
        at[u] = a.in.acctype[x];
      }
#pragma unroll
      for (uint32_t u = 0; u < FK; u++) {
        const uint32_t xr = b0 + 64 * u + lane;
        if (b0 + 64 * u >= span) break;  // uniform
        const bool in = xr < span;
        if (ballot64(in && key[u] == KEY_EMPTY) && lane == 0) atomicOr(a.err, ERR_KEY);
        bool h = false;
        if (in) {
          uint32_t b1, b2;
          bloom_bits(key[u], b1, b2);
          h = ((bl[b1 >> 5] >> (b1 & 31u)) & (bl[b2 >> 5] >> (b2 & 31u)) & 1u) != 0;
        }
        const uint64_t hb = ballot64(h), wb = ballot64(in && at[u] == 1);
        if (lane == 0) {
          hit[(b0 >> 6) + u] = hb;
          wr[(b0 >> 6) + u] = wb;
        }
      }
    }
    // per txn: killed / has-write (the wave's own LDS rows: no barrier needed)
    const uint32_t rlo = s - A0, rlen = e - s;
    const bool ok = valid && (rlen == 0 || (uint64_t)rlo + rlen <= span);
    // Bloom-positive accesses of the txn, verified one by one (almost always
    // the first is a true hit): one key reload + key table + committed bit
    bool killed = false;
    if (ok && rlen) {
      for (uint32_t x = rlo; x < rlo + rlen; x++) {
        const uint32_t nx = range_next(hit, x, rlo + rlen);
        if (nx >= rlo + rlen) break;
        if (c_exact(a, a.in.keys[A0 + nx])) {
          killed = true;
          break;
        }
        x = nx;
      }
    }
    if (valid && a.write_hasw) a.hasw[tid] = ok && rlen && range_any(wr, rlo, rlen) ? 1 : 0;
    if (cand && killed) a.state[tid] = ST_ABORT;
    if (cand && ok && rlen == 0) a.state[tid] = ST_COMMIT;  // no keys: nothing can kill it
    const bool surv = cand && ok && rlen && !killed;
    if (surv) range_set(sv, rlo, rlen);
    const uint64_t sm = ballot64(surv);
    if (fdbg && j == 0 && nchunk_done == 0) fdbg[2] = clock64();
    uint32_t wa_tot;
    const uint32_t aex = wave_excl_u32(surv ? rlen : 0u, wa_tot);
    if (lane == 0) {
      s_wt[wv] = (uint32_t)__popcll(sm);
      s_wa[wv] = wa_tot;
    }
    __syncthreads();
    if (wv == 0) {
      const uint32_t t = lane < FW ? s_wt[lane] : 0u, ac = lane < FW ? s_wa[lane] : 0u;
      const uint64_t agg = wave_sum64(lb_pack(t, ac));
      const uint64_t ex = lookback(a.status, c, agg, a.err);
      if (lane == 0) s_base = ex;
      if (c == nchunks - 1 && lane == 0) {
        const uint64_t inc = ex + agg;
        const uint32_t tot = (uint32_t)(inc >> LB_ACC_BITS);
        const uint64_t acc = inc & ((1ull << LB_ACC_BITS) - 1);
        a.lv_next->m = tot;
        a.lv_next->acc = (uint32_t)acc;
        a.off_out[tot] = (uint32_t)acc;
        const uint32_t in_n = m - pos;
        if (tot > a.abandon_min && (uint64_t)tot * a.abandon_den > (uint64_t)in_n * a.abandon_num)
          atomicMax(a.abandon_out, a.level + 1);
      }
    }
    __syncthreads();
    if (fdbg && j == 0 && nchunk_done == 0) fdbg[3] = clock64();
    uint32_t tb = (uint32_t)(s_base >> LB_ACC_BITS);
    uint32_t ab = (uint32_t)(s_base & ((1ull << LB_ACC_BITS) - 1));
    for (uint32_t q = 0; q < wv; q++) {
      tb += s_wt[q];
      ab += s_wa[q];
    }
    if (surv) {
      const uint32_t r = tb + (uint32_t)__popcll(sm & lanemask_lt());
      a.tid_out[r] = tid;
      a.off_out[r] = ab + aex;
    }
    if (sm) {
      // copy the survivors' accesses (index order kept): word prefix counts
      const uint64_t wsv = lane < nw ? sv[lane] : 0ull;
      uint32_t ptot;
      const uint32_t wpre = wave_excl_u32((uint32_t)__popcll(wsv), ptot);
      if (span <= 64 * FK) {
        // every access is still in registers
#pragma unroll
        for (uint32_t u = 0; u < FK; u++) {
          if (64 * u >= span) break;  // uniform
          const uint64_t word = __shfl(wsv, u);
          const uint32_t wbase = __shfl(wpre, u);  // all lanes active
          if ((word >> lane) & 1ull) {
            const uint32_t dst = ab + wbase + (uint32_t)__popcll(word & lanemask_lt());
            a.keys_out[dst] = key[u];
            a.acc_out[dst] = at[u];
          }
        }
      } else {
        for (uint32_t b0 = 0; b0 < span; b0 += 64) {
          const uint32_t wi = b0 >> 6;
          const uint64_t word = __shfl(wsv, wi);
          if (!word) continue;  // uniform
          const uint32_t wbase = __shfl(wpre, wi);
          if ((word >> lane) & 1ull) {
            const uint32_t x = A0 + b0 + lane;
            const uint32_t dst = ab + wbase + (uint32_t)__popcll(word & lanemask_lt());
            a.keys_out[dst] = a.in.keys[x];
            a.acc_out[dst] = a.in.acctype[x];
          }
        }
      }
    }
    __syncthreads();  // s_c / s_base / s_wt reuse
    if (fdbg && j == 0 && nchunk_done == 0) fdbg[4] = clock64();
    nchunk_done++;
  }
  if (fdbg && j == 0) {
    fdbg[5] = clock64();
    fdbg[6] = nchunk_done;
  }
}

// ---------------------------------------------------------------------------
void launch_sw_pre(const SwPreArgs& a, unsigned grid, hipStream_t st) {
  k_sw_pre<<<grid ? grid : 1u, 1024, 0, st>>>(a);
}
void launch_sw_seq(const SwSeqArgs& a, hipStream_t st) { k_sw_seq<<<1, 1024, 0, st>>>(a); }
void launch_sw_filter(const SwFilterArgs& a, unsigned grid, hipStream_t st) {
  k_sw_filter<<<grid ? grid : 1u, SW_CHUNK, 0, st>>>(a);
}

}  // namespace dcc
