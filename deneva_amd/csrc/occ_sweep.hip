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
constexpr uint32_t LB_ACC_BITS = 34;

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
// k_sw_pre: tile records (SwRec) of list txns [0, min(m, p_max)), 128 txns
// per tile: key ids, (local txn | W << 7) bytes, spans and the intra-tile
// dependency masks, built in two passes over an LDS key -> writer-mask map
// (writers 0..63, then 64..127).
__device__ inline uint32_t map_slot(uint64_t* mkey, uint64_t key, bool insert) {
  uint32_t h = sw_hash(key, 13);
  for (uint32_t q = 0; q < SW_MAP; q++) {
    if (insert) {
      const unsigned long long prev = atomicCAS((unsigned long long*)&mkey[h],
                                                (unsigned long long)KEY_EMPTY,
                                                (unsigned long long)key);
      if (prev == KEY_EMPTY || prev == key) return h;
    } else {
      const uint64_t kv = mkey[h];
      if (kv == key) return h;
      if (kv == KEY_EMPTY) return ~0u;
    }
    h = (h + 1) & (SW_MAP - 1);
  }
  return ~0u;
}

// k_sw_ids: key ids of the level's serial range (list accesses [off[0],
// min(off[lim], off[0] + budget))), spread over the whole grid: one home
// bucket read + one CAS per access (the rare lost race or full bucket: the
// slow path).  Random table traffic costs a CU ~4 cycles per lane, so it must
// not sit on the one CU of a tile.
__global__ __launch_bounds__(256) void k_sw_ids(SwPreArgs a) {
  if (*a.abandon) return;
  const uint32_t m = list_len(a.m_dev, a.m_host);
  const uint32_t lim = min(m, a.p_max);
  const uint64_t nnz = a.in.nnz;
  const uint64_t off0 = min((uint64_t)a.in.off[0], nnz);
  const uint64_t end = min(min((uint64_t)a.in.off[lim], nnz), off0 + a.budget);
  for (uint64_t x = off0 + (uint64_t)blockIdx.x * 256 + threadIdx.x; x < end;
       x += (uint64_t)gridDim.x * 256) {
    const uint64_t key = a.in.keys[x];
    const uint32_t hb = sw_hash(key, a.gbits - 2);
    const uint4* p = (const uint4*)(a.gtab + 4 * (uint64_t)hb);
    const uint4 bx = p[0], by = p[1];
    const uint64_t sv[4] = {((uint64_t)bx.y << 32) | bx.x, ((uint64_t)bx.w << 32) | bx.z,
                            ((uint64_t)by.y << 32) | by.x, ((uint64_t)by.w << 32) | by.z};
    uint32_t id = ~0u, fre = 4;
#pragma unroll
    for (uint32_t i = 0; i < 4; i++) {
      if (sv[i] == key && id == ~0u) id = 4 * hb + i;
      if (sv[i] == KEY_EMPTY && fre == 4) fre = i;
    }
    if (id == ~0u && fre < 4) {
      const unsigned long long prev =
          atomicCAS((unsigned long long*)(a.gtab + 4 * (uint64_t)hb + fre),
                    (unsigned long long)KEY_EMPTY, (unsigned long long)key);
      if (prev == KEY_EMPTY || prev == key) id = 4 * hb + fre;
    }
    if (id == ~0u) id = gtab_insert(a.gtab, a.gbits, key);
    a.ids[x - off0] = id;
  }
}

__global__ __launch_bounds__(1024) void k_sw_pre(SwPreArgs a) {
  __shared__ uint64_t mkey[SW_MAP];
  __shared__ uint64_t mmask[SW_MAP];
  __shared__ uint64_t s_dep[2][SW_T];
  __shared__ uint32_t s_off[SW_T + 1];
  __shared__ uint64_t s_hw[2];
  __shared__ uint32_t s_bad;
  if (*a.abandon) return;
  const uint32_t m = list_len(a.m_dev, a.m_host);
  const uint32_t lim = min(m, a.p_max);
  const uint32_t ntiles = (lim + SW_T - 1) / SW_T;
  const uint32_t j = threadIdx.x, lane = lane_id();
  const uint64_t nnz = a.in.nnz;
  const uint64_t off0 = min((uint64_t)a.in.off[0], nnz);
  uint64_t* pd = (a.dbg && blockIdx.x < 64) ? a.dbg + blockIdx.x * 8 : nullptr;
  if (pd && j == 0) pd[0] = clock64();
  for (uint32_t k = blockIdx.x; k < ntiles; k += gridDim.x) {
    const uint32_t i0 = k * SW_T;
    const uint32_t nt = min(SW_T, lim - i0);
    if (j <= nt) s_off[j] = (uint32_t)min((uint64_t)a.in.off[i0 + j], nnz);
    if (j < 2 * SW_T) s_dep[j / SW_T][j % SW_T] = 0;
    if (j < 2) s_hw[j] = 0;
    if (j == 0) s_bad = 0;
    __syncthreads();
    if (j < nt && s_off[j + 1] < s_off[j]) atomicOr(&s_bad, ERR_OFFSETS);
    const uint32_t A0 = s_off[0], A1 = s_off[nt];
    const uint32_t cnt = A1 >= A0 ? A1 - A0 : 0u;
    __syncthreads();
    uint32_t bad = s_bad;
    if (cnt > SW_TA) bad |= ERR_TILE;
    if (bad) {
      if (j == 0) {
        atomicOr(a.err, bad);
        a.tinfo[k] = SwTile{0, 0, {0, 0}, {0, 0}};
        a.rec[k].nt = 0;
        a.rec[k].cnt = 0;
      }
      __syncthreads();
      continue;
    }
    // the level's key table holds `budget` accesses: the serial pass stops here
    if ((uint64_t)A1 - off0 > a.budget) {
      if (j == 0) {
        a.tinfo[k] = SwTile{0, SW_STOP, {0, 0}, {0, 0}};
        a.rec[k].nt = 0;
        a.rec[k].cnt = SW_STOP;
      }
      __syncthreads();
      continue;
    }
    if (pd && j == 0 && k == blockIdx.x) pd[1] = clock64();
    uint64_t key[SW_U];
    uint32_t lt[SW_U];
    bool w[SW_U], v[SW_U];
    uint64_t hw0 = 0, hw1 = 0;
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
        if (w[u]) {
          if (lo < 64) hw0 |= 1ull << lo;
          else hw1 |= 1ull << (lo - 64);
        }
      }
    }
    // key ids (assigned by k_sw_ids) into the record
#pragma unroll
    for (uint32_t u = 0; u < SW_U; u++) {
      if (u && cnt <= 1024 * u) break;  // uniform
      if (!v[u]) continue;
      const uint32_t xr = j + 1024 * u;
      const uint32_t id = a.ids[(A0 - off0) + xr];
      const uint8_t pkv = (uint8_t)(lt[u] | (w[u] ? 0x80u : 0u));
      if (xr < SW_REC_ACC) {
        a.rec[k].id[xr] = id;
        a.rec[k].pk[xr] = pkv;
      } else {
        const uint64_t o = (uint64_t)k * (SW_TA - SW_REC_ACC) + (xr - SW_REC_ACC);
        a.id_ovf[o] = id;
        a.rp_ovf[o] = pkv;
      }
    }
    hw0 = wave_or64(hw0);
    hw1 = wave_or64(hw1);
    if (lane == 0 && hw0) atomicOr((unsigned long long*)&s_hw[0], (unsigned long long)hw0);
    if (lane == 0 && hw1) atomicOr((unsigned long long*)&s_hw[1], (unsigned long long)hw1);
    __syncthreads();
    if (pd && j == 0 && k == blockIdx.x) pd[2] = clock64();
    // dependency masks: half h = writers 64h .. 64h+63
    for (uint32_t h = 0; h < 2; h++) {
      for (uint32_t q = j; q < SW_MAP; q += 1024) {
        mkey[q] = KEY_EMPTY;
        mmask[q] = 0;
      }
      __syncthreads();
#pragma unroll
      for (uint32_t u = 0; u < SW_U; u++) {
        if (!v[u] || !w[u] || (lt[u] >> 6) != h) continue;
        const uint32_t sl = map_slot(mkey, key[u], true);
        if (sl != ~0u) atomicOr((unsigned long long*)&mmask[sl], 1ull << (lt[u] & 63));
      }
      __syncthreads();
#pragma unroll
      for (uint32_t u = 0; u < SW_U; u++) {
        if (!v[u] || lt[u] <= 64 * h) continue;  // no writer of this half precedes it
        const uint32_t sl = map_slot(mkey, key[u], false);
        if (sl == ~0u) continue;
        const uint32_t rel = lt[u] - 64 * h;  // earlier writers of the half only
        const uint64_t wm = mmask[sl] & (rel >= 64 ? ~0ull : ((1ull << rel) - 1ull));
        if (wm) atomicOr((unsigned long long*)&s_dep[h][lt[u]], (unsigned long long)wm);
      }
      __syncthreads();
    }
    if (j < SW_T) {
      const uint64_t r = (uint64_t)k * SW_T + j;
      a.rec[k].dep[0][j] = s_dep[0][j];
      a.rec[k].dep[1][j] = s_dep[1][j];
      a.rec[k].span[j] = j < nt ? (s_off[j] - A0) | ((s_off[j + 1] - s_off[j]) << 16) : 0u;
      a.rtid[r] = j < nt ? (a.in.tid ? a.in.tid[i0 + j] : i0 + j) : 0u;
      // identity lists carry decisions made before the solver (history window)
      const bool pre = j < nt && a.state && a.state[i0 + j] != ST_UNDECIDED;
      const uint64_t pk = ballot64(pre);
      if (lane == 0) {
        a.tinfo[k].prekill[j >> 6] = pk;
        a.rec[k].prekill[j >> 6] = pk;
      }
      if (j == 0) {
        a.tinfo[k].nt = nt;
        a.tinfo[k].cnt = cnt;
        a.tinfo[k].hasw[0] = s_hw[0];
        a.tinfo[k].hasw[1] = s_hw[1];
        a.rec[k].nt = nt;
        a.rec[k].cnt = cnt;
        a.rec[k].hasw[0] = s_hw[0];
        a.rec[k].hasw[1] = s_hw[1];
      }
    }
    if (pd && j == 0 && k == blockIdx.x) pd[3] = clock64();
    __syncthreads();  // LDS reuse by the next tile
    if (pd && j == 0 && k == blockIdx.x) pd[4] = clock64();
  }
  if (pd && j == 0) pd[5] = clock64();
}

// ---------------------------------------------------------------------------
// k_sw_seq: one workgroup decides the tiles in order (see header).  Tile
// records reach LDS SW_SEQ_B at a time as one contiguous copy whose loads
// are issued a super-step ahead (registers), so the loop itself touches
// global memory only on the rare long-tile path; decisions and C go out
// after the last tile.
constexpr uint32_t SEQ_N16 = SW_SEQ_B * sizeof(SwRec) / 16;  // uint4 per super-step
constexpr uint32_t SEQ_R = (SEQ_N16 + 1023) / 1024;           // uint4 per thread
static_assert(sizeof(SwRec) == 12864, "SwRec layout");
static_assert(SEQ_R == 4, "super-step copy width");
constexpr uint32_t SEQ_UR = SW_REC_ACC / 1024;  // accesses per thread held in the record

__global__ __launch_bounds__(1024) void k_sw_seq(SwSeqArgs a) {
  __shared__ __attribute__((aligned(16))) SwRec ring[SW_SEQ_B];
  __shared__ uint32_t cbits[(1u << SW_GBITS_MAX) / 32];  // committed set over key ids
  __shared__ uint64_t s_hit[SW_TA / 64];
  __shared__ uint64_t s_M[SW_PMAX_TILES][2];  // commit masks per decided tile
  __shared__ uint64_t s_stamp[128 * 4];       // DCC_SW_DEBUG clock stamps
  __shared__ uint32_t sbloom[(1u << SW_BLOOM_LOG) / 32];
  __shared__ uint32_t s_cnt, s_kc;
  const uint32_t j = threadIdx.x, lane = lane_id(), wv = j >> 6;
  if (*a.abandon) return;
  const uint32_t m = list_len(a.m_dev, a.m_host);
  const uint32_t lim = min(m, a.p_max);
  const uint32_t ntiles = min((lim + SW_T - 1) / SW_T, SW_PMAX_TILES);
  for (uint32_t q = j; q < (1u << SW_BLOOM_LOG) / 32; q += 1024) sbloom[q] = 0;
  if (j == 0) s_kc = 0;
  const uint32_t nsup = (ntiles + SW_SEQ_B - 1) / SW_SEQ_B;
  // the filter of this level starts from a clean look-back and ticket; the
  // next level's list is empty unless the filter writes it
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
  uint4 R0, R1, R2, R3;
  const uint32_t c0 = j, c1 = j + 1024, c2 = j + 2048, c3 = min(j + 3072, SEQ_N16 - 1);
#define SEQ_LOAD(sidx)                                     \
  do {                                                     \
    const uint4* p_ = src + (uint64_t)(sidx) * SEQ_N16;    \
    R0 = p_[c0];                                           \
    R1 = p_[c1];                                           \
    R2 = p_[c2];                                           \
    R3 = p_[c3];                                           \
  } while (0)
#define SEQ_STORE()  \
  do {               \
    dst[c0] = R0;    \
    dst[c1] = R1;    \
    dst[c2] = R2;    \
    dst[c3] = R3;    \
  } while (0)
  uint64_t* dbg = a.dbg;
  auto stamp = [&](uint32_t k, uint32_t i) {
    if (dbg && j == 0 && k < 128) s_stamp[k * 4 + i] = clock64();
  };

  // one tile; false = stopped before it (the level's access budget ends)
  const uint32_t idmask = (1u << a.gbits) - 1u;
  auto step = [&](const SwRec& T, uint32_t k) -> bool {
    const uint32_t nt = T.nt, cnt = T.cnt;
    if (cnt == SW_STOP) return false;  // uniform
    stamp(k, 0);
    // the common path: a thread's two accesses of the record, branch-free
    // (ids past cnt are masked: records are not cleared between tiles)
    const uint32_t i0 = T.id[j] & idmask, i1 = T.id[j + 1024] & idmask;
    const uint32_t p0 = T.pk[j], p1 = T.pk[j + 1024];
    const bool v0 = j < cnt, v1 = j + 1024 < cnt;
    // (1) probe C: one bitmap word per access; hit ballots into the tile bitmap
    {
      const uint32_t w0 = cbits[i0 >> 5], w1 = cbits[i1 >> 5];  // unconditional reads
      const bool h0 = ((w0 >> (i0 & 31u)) & (uint32_t)v0) != 0;
      const bool h1 = ((w1 >> (i1 & 31u)) & (uint32_t)v1) != 0;
      const uint64_t b0 = ballot64(h0), b1 = ballot64(h1);
      if (lane == 0) {
        s_hit[wv] = b0;
        s_hit[wv + 16] = b1;
      }
    }
    if (cnt > SW_REC_ACC) {  // long tiles (scalar branch): accesses beyond the record
      for (uint32_t u = SEQ_UR; u < SW_U; u++) {
        const uint32_t xr = j + 1024 * u;
        bool h = false;
        if (xr < cnt) {
          const uint32_t id =
              a.id_ovf[(uint64_t)k * (SW_TA - SW_REC_ACC) + xr - SW_REC_ACC] & idmask;
          h = (cbits[id >> 5] >> (id & 31u)) & 1u;
        }
        const uint64_t b = ballot64(h);
        if (lane == 0) s_hit[wv + 16 * u] = b;
      }
    }
    __syncthreads();
    stamp(k, 1);
    // (2) wave 0: kills, then the tile's serial order as a fixed point over
    // the dependency masks (lane l holds txns l and l + 64)
    if (wv == 0) {
      const bool va = lane < nt, vb = lane + 64 < nt;
      bool ka = ((T.prekill[0] >> lane) & 1ull) != 0;
      bool kb = ((T.prekill[1] >> lane) & 1ull) != 0;
      const uint32_t spa = T.span[lane], spb = T.span[lane + 64];
      if (va && !ka) ka = range_any(s_hit, spa & 0xFFFFu, spa >> 16);
      if (vb && !kb) kb = range_any(s_hit, spb & 0xFFFFu, spb >> 16);
      const uint64_t d0 = T.dep[0][lane];                                   // txn l < 64
      const uint64_t d1l = T.dep[0][lane + 64], d1h = T.dep[1][lane + 64];  // txn l + 64
      uint64_t Ul = ballot64(va && !ka), Uh = ballot64(vb && !kb), Ml = 0, Mh = 0;
#pragma unroll 1
      while (Ul | Uh) {
        const bool m0 = ((Ul >> lane) & 1ull) != 0, m1 = ((Uh >> lane) & 1ull) != 0;
        const bool c0 = m0 && (d0 & (Ml | Ul)) == 0;
        const bool a0 = m0 && (d0 & Ml) != 0;
        const bool c1 = m1 && ((d1l & (Ml | Ul)) | (d1h & (Mh | Uh))) == 0;
        const bool a1 = m1 && ((d1l & Ml) | (d1h & Mh)) != 0;
        const uint64_t cl = ballot64(c0), al = ballot64(a0), ch = ballot64(c1), ah = ballot64(a1);
        Ml |= cl;
        Mh |= ch;
        Ul &= ~(cl | al);
        Uh &= ~(ch | ah);
      }
      if (lane == 0) {
        s_M[k][0] = Ml;
        s_M[k][1] = Mh;
      }
    }
    __syncthreads();
    stamp(k, 2);
    // (3) committed write keys join C (no-return atomics: nothing waits)
    const uint64_t Ml = s_M[k][0], Mh = s_M[k][1];
    {
      const bool c0 = v0 && (p0 & 0x80u) && ((((p0 & 64u) ? Mh : Ml) >> (p0 & 63u)) & 1ull);
      const bool c1 = v1 && (p1 & 0x80u) && ((((p1 & 64u) ? Mh : Ml) >> (p1 & 63u)) & 1ull);
      if (c0) atomicOr(&cbits[i0 >> 5], 1u << (i0 & 31u));
      if (c1) atomicOr(&cbits[i1 >> 5], 1u << (i1 & 31u));
    }
    if (cnt > SW_REC_ACC) {
      for (uint32_t u = SEQ_UR; u < SW_U; u++) {
        const uint32_t xr = j + 1024 * u;
        if (xr >= cnt) continue;
        const uint64_t o = (uint64_t)k * (SW_TA - SW_REC_ACC) + xr - SW_REC_ACC;
        const uint32_t pk = a.rp_ovf[o];
        if ((pk & 0x80u) && ((((pk & 64u) ? Mh : Ml) >> (pk & 63u)) & 1ull)) {
          const uint32_t id = a.id_ovf[o] & idmask;
          atomicOr(&cbits[id >> 5], 1u << (id & 31u));
        }
      }
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
    const SwTile& ti = a.tinfo[kk];
    if (t >= ti.nt) continue;
    const uint32_t tid = a.rtid[q];
    const uint32_t h = t >> 6, b = t & 63;
    if (!((ti.prekill[h] >> b) & 1ull))
      a.state[tid] = ((s_M[kk][h] >> b) & 1ull) ? ST_COMMIT : ST_ABORT;
    if (a.write_hasw) a.hasw[tid] = (uint8_t)((ti.hasw[h] >> b) & 1ull);
  }
  // C for the filter: the committed-id bitmap and a Bloom filter of the keys
  {
    // keys of the committed ids, 8 table reads in flight per thread
    uint32_t ids[8];
    uint32_t nid = 0;
    auto flush = [&]() {
      uint64_t kk[8];
#pragma unroll
      for (uint32_t i = 0; i < 8; i++) kk[i] = i < nid ? a.gtab[ids[i]] : 0ull;
#pragma unroll
      for (uint32_t i = 0; i < 8; i++) {
        if (i >= nid) break;
        uint32_t b1, b2;
        bloom_bits(kk[i], b1, b2);
        atomicOr(&sbloom[b1 >> 5], 1u << (b1 & 31));
        atomicOr(&sbloom[b2 >> 5], 1u << (b2 & 31));
        a.ckeys_out[atomicAdd(&s_kc, 1u)] = kk[i];
      }
      nid = 0;
    };
    for (uint32_t q = j; q < nwords; q += 1024) {
      uint32_t w = cbits[q];
      a.cbits_out[q] = w;
      while (w) {
        ids[nid & 7] = q * 32 + (uint32_t)__builtin_ctz(w);
        w &= w - 1;
        if (++nid == 8) flush();
      }
    }
    flush();
  }
  __syncthreads();
  for (uint32_t q = j; q < (1u << SW_BLOOM_LOG) / 32; q += 1024) a.bloom_out[q] = sbloom[q];
  {
    uint32_t c = 0;
    for (uint32_t q = j; q < nwords; q += 1024) c += (uint32_t)__popc(cbits[q]);
    for (int dd = 32; dd > 0; dd >>= 1) c += __shfl_xor(c, dd);
    if (lane == 0) atomicAdd(&s_cnt, c);
  }
  __syncthreads();
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

constexpr uint32_t FW = SW_CHUNK / 64;  // waves per filter workgroup
constexpr uint32_t FK = 16;             // access rounds kept in registers (1024 accesses)
constexpr uint32_t F_EXACT = 2048;      // LDS exact set of small C (<= 1024 keys)
constexpr uint32_t SW_CMP_MAXR = 4096;  // tiles of one filter workgroup

// exact membership of a Bloom-positive key: its slot in the level's key
// table (a committed key always has one), then the committed-id bit.  The
// home bucket and its committed nibble (bucket b's 4 slots are bits
// 4(b & 7) .. +3 of cbits word b >> 3) are read together: one round trip.
__device__ inline bool c_exact(const SwFilterArgs& a, uint64_t key) {
  const uint32_t nbm = (1u << (a.gbits - 2)) - 1u;
  uint32_t b = sw_hash(key, a.gbits - 2);
  for (uint32_t q = 0; q <= nbm; q++) {
    const uint4* p = (const uint4*)(a.gtab + 4 * (uint64_t)b);
    const uint4 x = p[0], y = p[1];
    const uint32_t nib = (a.cbits[b >> 3] >> ((b & 7u) * 4u)) & 15u;
    const uint64_t v0 = ((uint64_t)x.y << 32) | x.x, v1 = ((uint64_t)x.w << 32) | x.z;
    const uint64_t v2 = ((uint64_t)y.y << 32) | y.x, v3 = ((uint64_t)y.w << 32) | y.z;
    if (v0 == key) return nib & 1u;
    if (v1 == key) return (nib >> 1) & 1u;
    if (v2 == key) return (nib >> 2) & 1u;
    if (v3 == key) return (nib >> 3) & 1u;
    if (v3 == KEY_EMPTY) return false;
    b = (b + 1) & nbm;
  }
  return false;
}
constexpr uint32_t F_STASH = 256;  // Bloom-positive keys kept in LDS per wave

// ---------------------------------------------------------------------------
// k_sw_filter: list txns [pos, m) against C, 64 per wave, grid-stride (no
// cross-workgroup waits).  A txn touching a key of C is killed; the others
// get a survivor bit and per-tile counts for the compaction.
__global__ __launch_bounds__(SW_CHUNK) void k_sw_filter(SwFilterArgs a) {
  __shared__ uint32_t bl[(1u << SW_BLOOM_LOG) / 32];
  __shared__ __attribute__((aligned(16))) uint64_t cex[F_EXACT];
  __shared__ uint64_t s_hit[FW][SW_WA / 64];
  __shared__ uint64_t s_wr[FW][SW_WA / 64];
  __shared__ uint64_t s_stash[FW][F_STASH];
  __shared__ uint32_t s_wpre[FW][SW_WA / 64];
  const uint32_t j = threadIdx.x, lane = lane_id(), wv = j >> 6;
  if (*a.abandon) return;
  const uint32_t m = list_len(a.m_dev, a.m_host);
  const uint32_t pos = a.lv->pos;
  const uint32_t ccount = a.lv->ccount;
  // the next level's key table (its pre-pass runs after this kernel)
  for (uint64_t q = (uint64_t)blockIdx.x * SW_CHUNK + j; q < a.gclear_n;
       q += (uint64_t)gridDim.x * SW_CHUNK)
    a.gclear[q] = KEY_EMPTY;
  if (pos >= m) return;
  const uint32_t n64 = (m - pos + 63) / 64;
  const uint64_t nnz = a.in.nnz;
  const bool small = ccount <= F_EXACT / 2;  // exact checks in LDS
  {
    const uint4* src = (const uint4*)a.bloom;
    uint4* dst = (uint4*)bl;
    for (uint32_t q = j; q < (1u << SW_BLOOM_LOG) / 128; q += SW_CHUNK) dst[q] = src[q];
    if (small)
      for (uint32_t q = j; q < F_EXACT; q += SW_CHUNK) cex[q] = KEY_EMPTY;
  }
  __syncthreads();
  if (small) {
    for (uint32_t q = j; q < ccount; q += SW_CHUNK) lset_insert<F_EXACT>(cex, a.ckeys[q]);
    __syncthreads();
  }
  uint64_t* hit = s_hit[wv];
  uint64_t* wr = s_wr[wv];
  uint64_t* stash = s_stash[wv];
  // workgroup g: tiles [g R, (g + 1) R), its total into bsum[g] (two-level scan)
  const uint32_t R = (n64 + gridDim.x - 1) / gridDim.x;
  const uint32_t t_lo = min(blockIdx.x * R, n64), t_hi = min(t_lo + R, n64);
  uint64_t wsum = 0;
  for (uint32_t wt = t_lo + wv; wt < t_hi; wt += FW) {
    const uint32_t p = pos + wt * 64 + lane;
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
    if (span > SW_WA) {  // malformed offsets (the host reports them): skip
      if (lane == 0) atomicOr(a.err, ERR_TILE);
      span = 0;
    }
    const uint32_t nw = (span + 63) / 64;
    // probe every access: FK loads in flight per lane; Bloom-positive keys
    // are stashed in LDS for the per-txn exact check
    uint32_t npos = 0;  // Bloom-positive accesses so far (wave-uniform)
    bool bad_key = false;
    for (uint32_t b0 = 0; b0 < span; b0 += 64 * FK) {
      uint64_t key[FK];
      uint32_t at[FK];
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
        if (b0 + 64 * u >= span) continue;  // uniform; no break: the loop must unroll
        const bool in = xr < span;
        bad_key |= in && key[u] == KEY_EMPTY;
        uint32_t b1, b2;
        bloom_bits(key[u], b1, b2);
        const uint32_t wa = bl[b1 >> 5], wb = bl[b2 >> 5];
        const bool h = in && (((wa >> (b1 & 31u)) & (wb >> (b2 & 31u)) & 1u) != 0);
        const uint64_t hb = ballot64(h), wbm = ballot64(in && at[u] == 1);
        if (h) {
          const uint32_t ci = npos + (uint32_t)__popcll(hb & lanemask_lt());
          if (ci < F_STASH) stash[ci] = key[u];
        }
        npos += (uint32_t)__popcll(hb);
        if (lane == 0) {
          hit[(b0 >> 6) + u] = hb;
          wr[(b0 >> 6) + u] = wbm;
        }
      }
    }
    if (ballot64(bad_key) && lane == 0) atomicOr(a.err, ERR_KEY);
    // per txn (the wave's own LDS rows: no barrier needed)
    const uint32_t rlo = s - A0, rlen = e - s;
    const bool ok = valid && (rlen == 0 || (uint64_t)rlo + rlen <= span);
    {
      const uint32_t pw = lane < nw ? (uint32_t)__popcll(hit[lane]) : 0u;
      uint32_t ptot;
      const uint32_t pre = wave_excl_u32(pw, ptot);
      if (lane < nw) s_wpre[wv][lane] = pre;
    }
    // Bloom-positive accesses of the txn, verified one by one (almost always
    // the first is a true hit): the key from the LDS stash, then the exact set
    bool killed = false;
    if (cand && ok && rlen) {
      for (uint32_t x = rlo; x < rlo + rlen; x++) {
        const uint32_t nx = range_next(hit, x, rlo + rlen);
        if (nx >= rlo + rlen) break;
        const uint32_t ci = s_wpre[wv][nx >> 6] +
                            (uint32_t)__popcll(hit[nx >> 6] & ((1ull << (nx & 63)) - 1ull));
        const uint64_t kx = ci < F_STASH ? stash[ci] : a.in.keys[A0 + nx];
        if (small ? lset_find<F_EXACT>(cex, kx) : c_exact(a, kx)) {
          killed = true;
          break;
        }
        x = nx;
      }
    }
    if (valid && a.write_hasw) a.hasw[tid] = ok && rlen && range_any(wr, rlo, rlen) ? 1 : 0;
    if (killed) a.state[tid] = ST_ABORT;
    if (cand && ok && rlen == 0) a.state[tid] = ST_COMMIT;  // no keys: nothing can kill it
    const bool surv = cand && ok && rlen && !killed;
    const uint64_t sm = ballot64(surv);
    const uint64_t acc = wave_sum64(surv ? rlen : 0u);
    const uint64_t cnt = ((uint64_t)__popcll(sm) << LB_ACC_BITS) | acc;
    wsum += cnt;
    if (lane == 0) {
      a.sflag[wt] = sm;
      a.tcount[wt] = cnt;
    }
  }
  __shared__ unsigned long long s_bs[FW];
  if (lane == 0) s_bs[wv] = wsum;
  __syncthreads();
  if (j == 0) {
    uint64_t t = 0;
    for (uint32_t w = 0; w < FW; w++) t += s_bs[w];
    a.bsum[blockIdx.x] = t;
  }
}

// ---------------------------------------------------------------------------
// k_sw_scan (one workgroup): exclusive scan of the filter workgroups' totals
// (16 per thread, loaded together); the next list's length, closing offset
// and the hand-off decision.
__global__ __launch_bounds__(1024) void k_sw_scan(SwFilterArgs a) {
  constexpr uint32_t PT = 16;
  __shared__ unsigned long long s_w[16];
  __shared__ unsigned long long s_carry;
  const uint32_t j = threadIdx.x, lane = lane_id(), wv = j >> 6;
  if (*a.abandon) return;
  const uint32_t m = list_len(a.m_dev, a.m_host);
  const uint32_t pos = a.lv->pos;
  if (pos >= m) return;
  const uint32_t nb = a.nblocks;
  if (j == 0) s_carry = 0;
  __syncthreads();
  for (uint32_t c0 = 0; c0 < nb; c0 += 1024 * PT) {
    const uint32_t q0 = c0 + j * PT;
    uint64_t v[PT], t = 0;
#pragma unroll
    for (uint32_t i = 0; i < PT; i++) v[i] = q0 + i < nb ? a.bsum[q0 + i] : 0ull;
#pragma unroll
    for (uint32_t i = 0; i < PT; i++) t += v[i];
    uint64_t x = t;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
      const uint64_t y = __shfl_up(x, d);
      if (lane >= (uint32_t)d) x += y;
    }
    if (lane == 63) s_w[wv] = x;
    __syncthreads();
    uint64_t base = s_carry;
    for (uint32_t w = 0; w < wv; w++) base += s_w[w];
    uint64_t run = base + x - t;  // exclusive prefix of this thread's first block
#pragma unroll
    for (uint32_t i = 0; i < PT; i++) {
      if (q0 + i < nb) a.bsum[q0 + i] = run;
      run += v[i];
    }
    __syncthreads();
    if (j == 1023) s_carry = base + x;
    __syncthreads();
  }
  if (j == 0) {
    const uint64_t inc = s_carry;
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

// ---------------------------------------------------------------------------
// k_sw_compact: the survivors, in index order, into the next level's list.
__global__ __launch_bounds__(SW_CHUNK) void k_sw_compact(SwFilterArgs a) {
  const uint32_t lane = lane_id(), wv = threadIdx.x >> 6;
  // a hand-off decided by this level's scan still needs its list
  const uint32_t ab = *a.abandon;
  if (ab && ab != a.level + 1) return;
  const uint32_t m = list_len(a.m_dev, a.m_host);
  const uint32_t pos = a.lv->pos;
  if (pos >= m) return;
  const uint32_t n64 = (m - pos + 63) / 64;
  const uint64_t nnz = a.in.nnz;
  // the filter's block ranges: block base from the scan, tile bases in LDS
  const uint32_t R = (n64 + a.nblocks - 1) / a.nblocks;
  const uint32_t t_lo = min(blockIdx.x * R, n64), t_hi = min(t_lo + R, n64);
  __shared__ unsigned long long s_tb[SW_CMP_MAXR];
  if (R > SW_CMP_MAXR) {
    if (threadIdx.x == 0) atomicOr(a.err, ERR_TILE);
    return;
  }
  if (wv == 0) {
    uint64_t run = a.bsum[blockIdx.x];
    for (uint32_t c0 = t_lo; c0 < t_hi; c0 += 64) {
      const uint32_t q = c0 + lane;
      const uint64_t v = q < t_hi ? a.tcount[q] : 0ull;
      uint64_t x = v;
#pragma unroll
      for (int d = 1; d < 64; d <<= 1) {
        const uint64_t y = __shfl_up(x, d);
        if (lane >= (uint32_t)d) x += y;
      }
      if (q < t_hi) s_tb[q - t_lo] = run + x - v;
      run += __shfl(x, 63);
    }
  }
  __syncthreads();
  for (uint32_t wt = t_lo + wv; wt < t_hi; wt += FW) {
    const uint64_t word = a.sflag[wt];
    if (!word) continue;  // uniform
    const uint64_t base = s_tb[wt - t_lo];
    const uint32_t tb = (uint32_t)(base >> LB_ACC_BITS);
    const uint32_t abase = (uint32_t)(base & ((1ull << LB_ACC_BITS) - 1));
    const bool surv = (word >> lane) & 1ull;
    const uint32_t p = pos + wt * 64 + lane;
    uint32_t s = 0, len = 0, tid = 0;
    if (surv) {
      s = (uint32_t)min((uint64_t)a.in.off[p], nnz);
      len = (uint32_t)min((uint64_t)a.in.off[p + 1], nnz) - s;
      tid = a.in.tid ? a.in.tid[p] : p;
    }
    uint32_t atot;
    const uint32_t aex = wave_excl_u32(len, atot);
    if (surv) {
      const uint32_t r = tb + (uint32_t)__popcll(word & lanemask_lt());
      a.tid_out[r] = tid;
      a.off_out[r] = abase + aex;
    }
    // accesses: lanes over the wave's survivor accesses; output position q
    // belongs to the first lane whose inclusive access prefix exceeds q
    const uint32_t incl = aex + len;
    for (uint32_t q0 = 0; q0 < atot; q0 += 64 * 4) {
      uint32_t src[4];
      bool in[4];
#pragma unroll
      for (uint32_t r = 0; r < 4; r++) {
        const uint32_t q = q0 + 64 * r + lane;
        uint32_t lo = 0;  // first lane l with incl[l] > q (all lanes take part)
#pragma unroll
        for (uint32_t st = 32; st > 0; st >>= 1) {
          const uint32_t v = __shfl(incl, lo + st - 1);
          if (v <= q) lo += st;
        }
        in[r] = q < atot;
        src[r] = __shfl(s, lo) + (q - __shfl(aex, lo));
      }
      uint64_t kk[4];
      uint8_t aa[4];
#pragma unroll
      for (uint32_t r = 0; r < 4; r++) {
        kk[r] = in[r] ? a.in.keys[src[r]] : 0ull;
        aa[r] = in[r] ? a.in.acctype[src[r]] : (uint8_t)0;
      }
#pragma unroll
      for (uint32_t r = 0; r < 4; r++) {
        if (!in[r]) continue;
        const uint32_t q = q0 + 64 * r + lane;
        a.keys_out[abase + q] = kk[r];
        a.acc_out[abase + q] = aa[r];
      }
    }
  }
}

// ---------------------------------------------------------------------------
void launch_sw_ids(const SwPreArgs& a, unsigned grid, hipStream_t st) {
  k_sw_ids<<<grid ? grid : 1u, 256, 0, st>>>(a);
}
void launch_sw_pre(const SwPreArgs& a, unsigned grid, hipStream_t st) {
  k_sw_pre<<<grid ? grid : 1u, 1024, 0, st>>>(a);
}
void launch_sw_seq(const SwSeqArgs& a, hipStream_t st) { k_sw_seq<<<1, 1024, 0, st>>>(a); }
void launch_sw_filter(const SwFilterArgs& a, unsigned grid, hipStream_t st) {
  k_sw_filter<<<grid ? grid : 1u, SW_CHUNK, 0, st>>>(a);
}
void launch_sw_scan(const SwFilterArgs& a, hipStream_t st) { k_sw_scan<<<1, 1024, 0, st>>>(a); }
void launch_sw_compact(const SwFilterArgs& a, unsigned grid, hipStream_t st) {
  k_sw_compact<<<grid ? grid : 1u, SW_CHUNK, 0, st>>>(a);
}

}  // namespace dcc
