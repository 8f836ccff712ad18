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
//   k_sw_pre     (grid)   one 64-txn tile of the list's first p_max txns per
//                         workgroup: key ids (slots of the level's global key
//                         table, each distinct key entered once per tile via
//                         an LDS map), txn-major id rows and the intra-tile
//                         dependency masks dep[t] = {u < t : W_u and keys(t)
//                         intersect}
//   k_sw_seq     (1 wave) the exact serial decision, tile by tile, with C as
//                         an LDS bitmap over key ids: a txn dies if a key is
//                         in C or an earlier committed txn of its tile writes
//                         one of its keys (a bit-parallel fixed point over the
//                         64 dep masks); committed write keys join C.  No
//                         barrier inside the loop; records are prefetched
//                         into registers.  Stops at p_max txns or when the
//                         level's key table budget ends.
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

#include <algorithm>

#include "dcc_device.h"
#include "occ_kernels.h"
#include "prep_body.h"

namespace dcc {

constexpr uint32_t LB_ACC_BITS = 34;

__device__ inline uint32_t sw_hash(uint64_t key, uint32_t log2s) {
  const uint32_t h = (uint32_t)key * 0x9E3779B1u ^ (uint32_t)(key >> 32) * 0x85EBCA77u;
  return h >> (32 - log2s);
}

// Level key table in global memory: 4-slot buckets (32 B); a key's id is its
// slot.  A key's probe sequence is the slots of its home bucket in its own
// cyclic order, starting at its preferred slot (the two hash bits below the
// bucket bits), then the next bucket's the same way; an insert CASes the
// slots of its sequence in turn (no reads) and stops at the first that was
// empty or holds the key.  Slots never change once set, so every inserter of
// a key stops at the same slot (no duplicates), and a key lives beyond its
// home bucket only if that bucket is full (a lookup stops at a bucket with a
// free slot).  The table is kept sparse, so most inserts settle with one CAS.
__device__ inline uint32_t gtab_step(uint64_t key, uint32_t gbits, uint32_t step) {
  const uint32_t h = sw_hash(key, gbits);  // bucket bits, then the preferred slot
  const uint32_t nbm = (1u << (gbits - 2)) - 1u;
  const uint32_t b = ((h >> 2) + (step >> 2)) & nbm;
  return 4 * b + (((h & 3u) + step) & 3u);
}
__device__ inline unsigned long long gtab_cas(uint64_t* gt, uint32_t slot, uint64_t key) {
  return atomicCAS((unsigned long long*)(gt + slot), (unsigned long long)KEY_EMPTY,
                   (unsigned long long)key);
}
// the key's slot, walking its sequence from `step`
__device__ inline uint32_t gtab_insert(uint64_t* gt, uint32_t gbits, uint64_t key, uint32_t step) {
  for (uint32_t q = step; q < (4u << (gbits - 2)); q++) {
    const uint32_t sl = gtab_step(key, gbits, q);
    const unsigned long long prev = gtab_cas(gt, sl, key);
    if (prev == KEY_EMPTY || prev == key) return sl;
  }
  return 0;  // unreachable: the table is far from full
}

// Two Bloom-filter bits of a key (2^SW_BLOOM_LOG bits).
__device__ inline void bloom_bits(uint64_t key, uint32_t& b1, uint32_t& b2) {
  const uint32_t h = (uint32_t)key * 0x9E3779B1u ^ (uint32_t)(key >> 32) * 0x85EBCA77u;
  b1 = h >> (32 - SW_BLOOM_LOG);
  b2 = (h * 0xC2B2AE35u + 0x27D4EB2Fu) >> (32 - SW_BLOOM_LOG);
}

// The epoch's committed-writer table (WrTab, occ_kernels.h): linear probes
// from the key's hash, at most wt.probes slots.
__device__ inline void wt_insert(const WrTab& wt, uint64_t key, uint32_t tid) {
  const uint32_t mask = (1u << wt.bits) - 1u;
  uint32_t s = sw_hash(key, wt.bits);
  for (uint32_t q = 0; q < wt.probes; q++, s = (s + 1) & mask) {
    const unsigned long long prev = atomicCAS((unsigned long long*)&wt.slot[s].key,
                                              (unsigned long long)KEY_EMPTY, (unsigned long long)key);
    if (prev == KEY_EMPTY || prev == key) {
      wt.slot[s].tid = tid;  // one committed writer per key: a single value
      return;
    }
  }
  atomicOr(wt.full, 1u);
}
// the key's committed writer, or ~0u (one 16-B load per probe)
__device__ inline uint32_t wt_find(const WrTab& wt, uint64_t key) {
  const uint32_t mask = (1u << wt.bits) - 1u;
  uint32_t s = sw_hash(key, wt.bits);
  for (uint32_t q = 0; q < wt.probes; q++, s = (s + 1) & mask) {
    const uint4 v = *(const uint4*)&wt.slot[s];
    const uint64_t k = ((uint64_t)v.y << 32) | v.x;
    if (k == key) return v.z;
    if (k == KEY_EMPTY) break;
  }
  return ~0u;
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

// 64-txn tiles per filter workgroup (filter, apply and compaction agree): at
// least one per wave, so a short list keeps fewer workgroups busy, each with
// all its waves, and the idle ones leave at once instead of running a second
// generation of half-empty workgroups through the whole setup
__device__ inline uint32_t sw_tiles_per_wg(uint32_t n64, uint32_t nblocks) {
  return max((n64 + nblocks - 1) / nblocks, SW_CHUNK / 64);
}

// ---------------------------------------------------------------------------
// k_sw_pre: tile records (SwRec) of list txns [0, min(m, p_max)), one 64-txn
// tile per workgroup: key ids, dependency masks, per-txn meta.  Each distinct
// key of a tile is entered once in an LDS map (key -> writer mask, key id);
// only its first access touches the level's global key table, so a hot key
// costs one global CAS per tile rather than one per access.
constexpr uint32_t PRE_MAP = 4096;       // LDS map slots (<= 2048 distinct keys per pass)
constexpr uint32_t PRE_B = 1024;          // threads per workgroup

__device__ inline uint32_t pre_map_insert(uint64_t* mkey, uint64_t key, bool& first) {
  uint32_t h = sw_hash(key, 12);
  for (uint32_t q = 0; q < PRE_MAP; q++) {
    const uint64_t v = mkey[h];
    if (v == key) {
      first = false;
      return h;
    }
    if (v == KEY_EMPTY) {
      const unsigned long long prev = atomicCAS((unsigned long long*)&mkey[h],
                                                (unsigned long long)KEY_EMPTY,
                                                (unsigned long long)key);
      if (prev == KEY_EMPTY) {
        first = true;
        return h;
      }
      if (prev == key) {
        first = false;
        return h;
      }
    }
    h = (h + 1) & (PRE_MAP - 1);
  }
  first = false;
  return 0;  // unreachable: a pass holds <= PRE_MAP distinct keys
}

// the tile's accesses, U per thread (j + PRE_B u): key ids, writer /
// accessor masks, dependency masks, first-writer / last-accessor positions.
// Instantiated for U = 2, 4, 8 and chosen per tile, so the common short tile
// (<= 1024 accesses) runs without the register pressure of the longest.
struct PreLds {
  uint64_t mkey[PRE_MAP];
  uint64_t mmask[PRE_MAP];   // writers of the key in the tile
  uint64_t mamask[PRE_MAP];  // accessors of the key in the tile
  uint32_t mgid[PRE_MAP];
  uint64_t s_dep[SW_T];
  uint32_t s_off[SW_T + 1];
  uint32_t s_meta[SW_T];
  uint32_t s_bad;
};
template <uint32_t U>
__device__ inline void pre_tile(const SwPreArgs& a, PreLds& L, uint32_t k, uint32_t j, uint32_t nt,
                                uint32_t A0, uint32_t cnt, uint64_t off0) {
  uint64_t* const mkey = L.mkey;
  uint64_t* const mmask = L.mmask;
  uint64_t* const mamask = L.mamask;
  uint32_t* const mgid = L.mgid;
  uint64_t* const s_dep = L.s_dep;
  const uint32_t* const s_off = L.s_off;
  uint32_t* const s_meta = L.s_meta;
  // per-thread accesses j + PRE_B u; flags packed into bit masks over u.
  // Every load is issued first (clamped addresses), then the accesses are
  // classified, so the loads of a thread are in flight together.
  uint64_t key[U];
  uint32_t lt[U], slot[U];
  uint32_t vm = 0, wmk = 0;
  {
    uint8_t atv[U];
    const uint32_t xmax = cnt ? A0 + cnt - 1 : A0;
#pragma unroll
    for (uint32_t u = 0; u < U; u++) {
      const uint32_t x = min(A0 + j + PRE_B * u, xmax);
      key[u] = a.in.keys[x];
      atv[u] = a.in.acctype[x];
    }
    uint32_t bad_key = 0;
#pragma unroll
    for (uint32_t u = 0; u < U; u++) {
      lt[u] = 0;
      slot[u] = 0;
      const uint32_t xr = j + PRE_B * u;
      if (xr >= cnt) continue;
      const uint32_t x = A0 + xr;
      // largest t < nt with s_off[t] <= x (empty txns never own an access)
      uint32_t lo = 0, hi = nt;  // invariant: s_off[lo] <= x < s_off[hi]
      while (hi - lo > 1) {
        const uint32_t mid = (lo + hi) >> 1;
        if (s_off[mid] <= x) lo = mid;
        else hi = mid;
      }
      lt[u] = lo;
      if (atv[u] == 1) {  // WR (get_rw_set, occ.cpp:296-317)
        wmk |= 1u << u;
        atomicOr(&s_meta[lo], SWM_HASW);
      }
      if (key[u] == KEY_EMPTY) {
        // the reserved key is reported by the host; it gets no key id (its
        // access is recorded as an unused entry)
        bad_key = 1;
        a.aent[A0 - (uint32_t)off0 + xr] = SW_A_NONE;
        a.apos[A0 - (uint32_t)off0 + xr] = k * SW_T;
      } else {
        vm |= 1u << u;
      }
    }
    if (bad_key) atomicOr(a.err, ERR_KEY);
  }
  // passes over key-hash classes keep each map pass <= 2048 distinct keys
  const uint32_t P = cnt <= PRE_MAP / 2 ? 1u : 2u;
  for (uint32_t p = 0; p < P; p++) {
    for (uint32_t q = j; q < PRE_MAP; q += PRE_B) {
      mkey[q] = KEY_EMPTY;
      mmask[q] = 0;
      mamask[q] = 0;
    }
    __syncthreads();
  if (a.dbg && blockIdx.x == 0 && threadIdx.x == 0) a.dbg[3] = __builtin_amdgcn_s_memrealtime();
    uint32_t pm = vm;  // this pass's accesses
    if (P > 1)
#pragma unroll
      for (uint32_t u = 0; u < U; u++)
        if ((sw_hash(key[u], 13) & 1u) != p) pm &= ~(1u << u);
    uint32_t fm = 0;
#pragma unroll
    for (uint32_t u = 0; u < U; u++) {
      if (!((pm >> u) & 1u)) continue;
      bool first;
      slot[u] = pre_map_insert(mkey, key[u], first);
      if (first) fm |= 1u << u;
      if ((wmk >> u) & 1u) atomicOr((unsigned long long*)&mmask[slot[u]], 1ull << lt[u]);
      atomicOr((unsigned long long*)&mamask[slot[u]], 1ull << lt[u]);
    }
    if (a.dbg && blockIdx.x == 0) {  // debug only: phase boundaries of the block
      __syncthreads();
      if (j == 0 && p == 0) a.dbg[12] = __builtin_amdgcn_s_memrealtime();
    }
    // the first access of each key enters it in the global table: every
    // CAS of the first slot of the key's sequence in flight at once; a
    // lost slot (another key holds it) takes the next slot in a second
    // round, and only a second loss walks on alone
    {
      unsigned long long prev[U];
      uint32_t gid[U];
#pragma unroll
      for (uint32_t u = 0; u < U; u++) {
        gid[u] = gtab_step(key[u], a.gbits, 0);
        prev[u] = KEY_EMPTY;
        if ((fm >> u) & 1u) prev[u] = gtab_cas(a.gtab, gid[u], key[u]);
      }
      uint32_t lost = 0;
#pragma unroll
      for (uint32_t u = 0; u < U; u++)
        if (((fm >> u) & 1u) && prev[u] != KEY_EMPTY && prev[u] != key[u]) lost |= 1u << u;
      if (a.dbg && blockIdx.x == 0) {
        __syncthreads();
        if (j == 0 && p == 0) a.dbg[13] = __builtin_amdgcn_s_memrealtime();
      }
#pragma unroll
      for (uint32_t u = 0; u < U; u++)
        if ((lost >> u) & 1u) {
          gid[u] = gtab_step(key[u], a.gbits, 1);
          prev[u] = gtab_cas(a.gtab, gid[u], key[u]);
        }
      uint32_t slow = 0;
#pragma unroll
      for (uint32_t u = 0; u < U; u++)
        if (((lost >> u) & 1u) && prev[u] != KEY_EMPTY && prev[u] != key[u]) slow |= 1u << u;
      if (a.dbg && blockIdx.x == 0) {
        __syncthreads();
        if (j == 0 && p == 0) a.dbg[14] = __builtin_amdgcn_s_memrealtime();
        if (lost) atomicAdd((unsigned long long*)&a.dbg[15], (unsigned long long)__popc(lost));
        if (fm) atomicAdd((unsigned long long*)&a.dbg[16], (unsigned long long)__popc(fm));
      }
#pragma unroll
      for (uint32_t u = 0; u < U; u++) {
        if (!((fm >> u) & 1u)) continue;
        if ((slow >> u) & 1u) gid[u] = gtab_insert(a.gtab, a.gbits, key[u], 2);
        mgid[slot[u]] = gid[u];
      }
    }
    __syncthreads();
  if (a.dbg && blockIdx.x == 0 && threadIdx.x == 0) a.dbg[4] = __builtin_amdgcn_s_memrealtime();
#pragma unroll
    for (uint32_t u = 0; u < U; u++) {
      if (!((pm >> u) & 1u)) continue;
      const uint32_t t = lt[u];
      const uint64_t wmask = mmask[slot[u]];
      const uint64_t wm = wmask & ((1ull << t) - 1ull);  // earlier writers only
      if (wm) atomicOr((unsigned long long*)&s_dep[t], (unsigned long long)wm);
      const uint32_t gid = mgid[slot[u]];
      // the key's first writer and last accessor in the level's serial
      // range (list positions), once per distinct key of the tile
      if ((fm >> u) & 1u) {
        if (wmask) atomicMin(&a.first_w[gid], k * SW_T + (uint32_t)__builtin_ctzll(wmask));
        atomicMax(&a.last_a[gid], k * SW_T + 63u - (uint32_t)__builtin_clzll(mamask[slot[u]]));
      }
      const uint32_t xo = A0 - (uint32_t)off0 + j + PRE_B * u;
      a.aent[xo] = sw_apack(gid, (wmk >> u) & 1u);
      a.apos[xo] = k * SW_T + t;
    }
    __syncthreads();  // map reuse by the next pass
  if (a.dbg && blockIdx.x == 0 && threadIdx.x == 0) a.dbg[5] = __builtin_amdgcn_s_memrealtime();
  }
}

__global__ __launch_bounds__(PRE_B) void k_sw_pre(SwPreArgs a) {
  __shared__ PreLds L;
  uint64_t* const s_dep = L.s_dep;
  uint32_t* const s_off = L.s_off;
  uint32_t* const s_meta = L.s_meta;
  uint32_t& s_bad = L.s_bad;
  // every control word and the tile's offsets, txn ids and states are read
  // at once (indices clamped to the host's list bound m_host, which every
  // list buffer covers), before the first branch on any of them: one
  // dependent round trip instead of four
  const uint32_t j = threadIdx.x;
  const uint32_t k = blockIdx.x;  // one tile per workgroup (one workgroup per tile of p_max)
  const uint32_t i0 = k * SW_T;
  const uint32_t ab = *a.abandon;
  const uint32_t m = list_len(a.m_dev, a.m_host);
  const uint32_t xj = min(i0 + j, a.m_host);
  const uint32_t o_raw = a.in.off[xj], o0_raw = a.in.off[0];
  const uint32_t tid_raw = a.in.tid ? a.in.tid[xj] : i0 + j;
  const uint8_t st_raw = a.state ? a.state[xj] : (uint8_t)ST_UNDECIDED;
  if (ab) return;
    if (a.dbg && blockIdx.x == 0 && threadIdx.x == 0) a.dbg[0] = __builtin_amdgcn_s_memrealtime();
  const uint32_t lim = min(m, a.p_max);
  const uint32_t ntiles = (lim + SW_T - 1) / SW_T;
  const uint64_t nnz = a.in.nnz;
  const uint64_t off0 = min((uint64_t)o0_raw, nnz);
  if (k >= ntiles) return;
  {
    SwRec& R = a.rec[k];
    const uint32_t nt = min(SW_T, lim - i0);
    if (j <= nt) s_off[j] = (uint32_t)min((uint64_t)o_raw, nnz);
    // per-txn inputs of the record (used at the end); identity lists carry
    // decisions made before the solver (history window)
    const uint32_t my_tid = j < nt ? tid_raw : 0u;
    const bool my_pre = j < nt && st_raw != ST_UNDECIDED;
    if (j < SW_T) {
      s_dep[j] = 0;
      s_meta[j] = 0;
    }
    if (j == 0) s_bad = 0;
    __syncthreads();
    if (a.dbg && blockIdx.x == 0 && threadIdx.x == 0) a.dbg[1] = __builtin_amdgcn_s_memrealtime();
    if (j < nt && s_off[j + 1] < s_off[j]) atomicOr(&s_bad, ERR_OFFSETS);
    const uint32_t A0 = s_off[0], A1 = s_off[nt];
    const uint32_t cnt = A1 >= A0 ? A1 - A0 : 0u;
    __syncthreads();
    if (a.dbg && blockIdx.x == 0 && threadIdx.x == 0) a.dbg[2] = __builtin_amdgcn_s_memrealtime();
    uint32_t bad = s_bad;
    if (cnt > SW_TA) bad |= ERR_TILE;
    // the level's key table holds `budget` accesses: the serial pass stops here
    const bool stop = !bad && (uint64_t)A1 - off0 > a.budget;
    if (bad || stop) {
      if (bad && j == 0) atomicOr(a.err, bad);
      // a malformed tile is reported by the host; both end the serial pass
      if (j < SW_T) R.meta[j] = SWM_STOP;
      return;
    }
    if (cnt <= PRE_B) pre_tile<1>(a, L, k, j, nt, A0, cnt, off0);
    else if (cnt <= 2 * PRE_B) pre_tile<2>(a, L, k, j, nt, A0, cnt, off0);
    else pre_tile<4>(a, L, k, j, nt, A0, cnt, off0);
    // the per-txn words (k_sw_rows adds the row length)
    if (j < SW_T) {
      uint32_t mt = s_meta[j];
      if (j < nt) {
        mt |= SWM_VALID;
        if (my_pre) mt |= SWM_PRE;
      }
      R.meta[j] = mt;
      R.dep[j] = s_dep[j];
      R.rtid[j] = my_tid;
    }
    if (a.dbg && blockIdx.x == 0 && j == 0) {
      __builtin_amdgcn_s_waitcnt(0);
      a.dbg[6] = __builtin_amdgcn_s_memrealtime();
    }
  }
}

// ---------------------------------------------------------------------------
// k_sw_rows: the tile's two lists, one wave per tile (lane = txn): only the
// accesses the serial pass must look at.  An access is probed when an earlier
// txn of the serial range writes its key ("live": otherwise the key cannot be
// in C when the txn is decided); a write is inserted into the pass's C when a
// later txn of the range accesses the key ("needed").  Probes are grouped by
// txn (prefix sum over the lanes).  The full C of the level (every committed
// write) is listed afterwards by k_sw_cout.
__global__ __launch_bounds__(256) void k_sw_rows(SwPreArgs a) {
  __shared__ uint32_t s_off[SW_T + 1];
  __shared__ uint32_t s_ent[SW_TA];  // the tile's access entries (sw_apack)
  __shared__ uint8_t s_flag[SW_TA];  // live | needed << 1 per access
  const uint32_t k = blockIdx.x, j = threadIdx.x, lane = lane_id();
  // control words, the tile's stop mark and offsets in one round trip
  // (indices clamped to the host's list bound; records of tiles past the
  // list are never read by the serial pass)
  const uint32_t ab = *a.abandon;
  const uint32_t m = list_len(a.m_dev, a.m_host);
  SwRec& R = a.rec[k];
  const uint32_t meta0 = R.meta[0];
  const uint32_t o_raw = a.in.off[min(k * SW_T + j, a.m_host)], o0_raw = a.in.off[0];
  if (ab) return;
  const uint32_t lim = min(m, a.p_max);
  const uint32_t ntiles = (lim + SW_T - 1) / SW_T;
  if (k >= ntiles) return;
  if (meta0 & SWM_STOP) {  // uniform: written on every txn of a stopped tile
    if (j == 0) R.hdr = SWH_STOP;
    return;
  }
  uint64_t* dbg = (a.dbg && k == 0) ? a.dbg : nullptr;
  if (dbg && j == 0) dbg[8] = __builtin_amdgcn_s_memrealtime();
  const uint64_t nnz = a.in.nnz;
  const uint32_t off0 = (uint32_t)min((uint64_t)o0_raw, nnz);
  const uint32_t nt = min(SW_T, lim - k * SW_T);
  if (j <= nt) s_off[j] = (uint32_t)min((uint64_t)o_raw, nnz);
  __syncthreads();
  if (dbg && j == 0) dbg[9] = __builtin_amdgcn_s_memrealtime();
  const uint32_t A0 = s_off[0];
  const uint32_t cnt = min(s_off[nt] >= A0 ? s_off[nt] - A0 : 0u, SW_TA);  // pre checked it
  const uint32_t idlim = 1u << a.gbits;
  // (1) access-parallel: coalesced entry / position loads, then the random
  // first-writer / last-accessor lookups, four accesses per thread in flight
  for (uint32_t x0 = 0; x0 < cnt; x0 += 1024) {
    uint32_t e[4], pp[4], fw[4], la[4];
#pragma unroll
    for (uint32_t u = 0; u < 4; u++) {
      const uint32_t x = min(x0 + j + 256 * u, cnt - 1);
      e[u] = a.aent[A0 - off0 + x];
      pp[u] = a.apos[A0 - off0 + x];
    }
#pragma unroll
    for (uint32_t u = 0; u < 4; u++) {
      const uint32_t id = sw_aid(e[u]);
      const uint32_t ic = id < idlim ? id : 0u;
      fw[u] = a.first_w[ic];
      la[u] = a.last_a[ic];
    }
#pragma unroll
    for (uint32_t u = 0; u < 4; u++) {
      const uint32_t x = x0 + j + 256 * u;
      if (x >= cnt) continue;
      const bool in = sw_aid(e[u]) < idlim;
      // live | needed << 1 | the access's txn in the tile << 2
      const uint32_t f = (in && fw[u] < pp[u] ? 1u : 0u) |
                         (in && (e[u] & 32u) && la[u] > pp[u] ? 2u : 0u) | ((pp[u] & 63u) << 2);
      s_ent[x] = e[u];
      s_flag[x] = (uint8_t)f;
    }
  }
  __syncthreads();
  if (dbg && j == 0) dbg[10] = __builtin_amdgcn_s_memrealtime();
  // (2) the two lists in access order, which is txn order (so the probes
  // come grouped by txn): per 64-access chunk the live / needed ballots and
  // counts (the four waves take every fourth chunk), an exclusive scan of the
  // chunk counts (wave 0: at most 64 chunks), then every wave writes its
  // chunks' entries in place
  __shared__ uint64_t s_bl[SW_TA / 64 + 1];  // live ballot per chunk (+ a zero word)
  __shared__ uint32_t s_cp[SW_TA / 64 + 1], s_ci[SW_TA / 64 + 1];
  const uint32_t wv = j >> 6;
  const uint32_t nch = (cnt + 63) / 64;
  const uint64_t lt = lanemask_lt();
  for (uint32_t c = wv; c < nch; c += 4) {
    const uint32_t x = c * 64 + lane;
    const uint32_t f = x < cnt ? s_flag[x] : 0u;
    const uint64_t bl = ballot64(f & 1u), bn = ballot64((f >> 1) & 1u);
    if (lane == 0) {
      s_bl[c] = bl;
      s_cp[c] = (uint32_t)__popcll(bl);
      s_ci[c] = (uint32_t)__popcll(bn);
    }
  }
  __syncthreads();
  if (wv == 0) {
    const uint32_t vp = lane < nch ? s_cp[lane] : 0u, vi = lane < nch ? s_ci[lane] : 0u;
    uint32_t tp, ti;
    const uint32_t ep = wave_excl_u32(vp, tp), ei = wave_excl_u32(vi, ti);
    if (lane < nch) {
      s_cp[lane] = ep;
      s_ci[lane] = ei;
    }
    if (lane == 0) {
      s_cp[nch] = tp;
      s_ci[nch] = ti;
      s_bl[nch] = 0;
    }
  }
  __syncthreads();
  const uint32_t np = s_cp[nch], ni = s_ci[nch];
  uint32_t* ovf = a.lst_ovf + (uint64_t)k * SW_OVF;
  for (uint32_t c = wv; c < nch; c += 4) {
    const uint32_t x = c * 64 + lane;
    const uint32_t f = x < cnt ? s_flag[x] : 0u;
    const uint64_t bn = ballot64((f >> 1) & 1u);
    if (!(f & 3u)) continue;
    const uint32_t id = sw_aid(s_ent[x]);
    if (f & 1u) {
      const uint32_t q = s_cp[c] + (uint32_t)__popcll(s_bl[c] & lt);
      const uint32_t e = sw_ppack(id);
      if (q < SW_PL) R.probe[q] = e;
      else ovf[q - SW_PL] = e;
    }
    if (f & 2u) {
      const uint32_t q = s_ci[c] + (uint32_t)__popcll(bn & lt);
      const uint32_t e = sw_ipack(id, f >> 2);
      if (q < SW_IL) R.ins[q] = e;
      else ovf[SW_TA + q - SW_IL] = e;
    }
  }
  if (wv != 0) return;
  // lane = txn: its probe span (the live accesses before its first and past
  // its last access), the register-chunk masks, no-op padding, the header
  const uint32_t t = lane;
  uint32_t xlo = cnt, xhi = cnt;
  if (t < nt) {
    const uint32_t s0 = s_off[t] - A0;
    const uint32_t len = s_off[t + 1] > s_off[t] ? min(s_off[t + 1] - s_off[t], MAX_TXN_LEN) : 0u;
    xlo = min(s0, cnt);
    xhi = min(s0 + len, cnt);
  }
  auto live_before = [&](uint32_t x) {
    const uint32_t w = x >> 6, b = x & 63u;
    return s_cp[w] + (uint32_t)__popcll(s_bl[w] & (b ? ~0ull >> (64 - b) : 0ull));
  };
  const uint32_t ps = live_before(xlo), pe = live_before(xhi);
  R.pspan[t] = ps | (pe << 16);
  if (t == 0) {
    R.np = np;
    R.ni = ni;
    R.hdr = (np > SW_RC * 64 ? SWH_PLONG : 0u) | (ni > SW_RC_I * 64 ? SWH_ILONG : 0u);
  }
#pragma unroll
  for (uint32_t c = 0; c < SW_RC; c++) {
    const uint32_t lo = max(ps, c * 64), hi = min(pe, c * 64 + 64);
    const uint32_t nb = hi > lo ? hi - lo : 0u;
    R.seg[c][t] = nb ? (nb >= 64 ? ~0ull : ((1ull << nb) - 1ull)) << (lo - c * 64) : 0ull;
    if (c * 64 + t >= np) R.probe[c * 64 + t] = SW_P_NONE;
    if (c * 64 + t >= ni) R.ins[c * 64 + t] = sw_idummy(t);
  }
  if (dbg && t == 0) {
    __builtin_amdgcn_s_waitcnt(0);
    dbg[11] = __builtin_amdgcn_s_memrealtime();
  }
}

// ---------------------------------------------------------------------------
// k_sw_seq: the exact serial decision of the level's tiles, in order, by ONE
// wave (lane t = txn t of the tile): no barriers inside the loop.  The
// committed set C lives in LDS as a bitmap over key ids; a wave's LDS
// operations complete in order, so a tile's inserts are visible to the next
// tile's probes.  The other 15 waves stream the tile records from global
// memory into an LDS ring ahead of it (one tile per wave in flight; ready and
// consumed counters in LDS), then all 16 join for the write-out.
constexpr uint32_t SEQ_RING = 12;  // LDS record slots (73,728 B)
constexpr uint32_t SEQ_B = 1024;   // threads of the serial pass's workgroup
constexpr uint32_t SEQ_PROD = SEQ_B / 64 - 1;  // producer waves
constexpr uint32_t SEQ_V4 = sizeof(SwRec) / 16;  // uint4 per record
static_assert(SW_RC * 64 <= SW_PL && SW_RC_I * 64 <= SW_IL, "register chunks inside the record");
static_assert(sizeof(SwRec) % (16 * 64) == 0, "record copy: whole uint4 per lane");

// A load the compiler's wait-count tracking does not see: it completes inside
// the asm (vmcnt(0)); used on the rare overflow path of long txns.
__device__ inline uint32_t ld_sync(const uint32_t* p) {
  uint32_t v;
  asm volatile("global_load_dword %0, %1, off\n\ts_waitcnt vmcnt(0)" : "=v"(v) : "v"(p));
  return v;
}
// workgroup-scope acquire / release on the LDS hand-off counters
__device__ inline uint32_t lds_ld(uint32_t* p) {
  return __hip_atomic_load(p, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP);
}
__device__ inline uint32_t lds_ld_rlx(uint32_t* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}
__device__ inline void lds_st(uint32_t* p, uint32_t v) {
  __hip_atomic_store(p, v, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
}

// committed-set bitmap probe of a probe entry (sw_ppack): its bit
__device__ inline uint32_t cb_probe(const uint32_t* cb, uint32_t e) {
  return (*(const uint32_t*)((const char*)cb + (e >> 5)) >> (e & 31u)) & 1u;
}
// insert entry (sw_ipack): the key joins C if its txn committed (bit of M);
// ORs 0 otherwise
__device__ inline void cb_insert_m(uint32_t* cb, uint32_t e, uint64_t M) {
  const uint32_t b = (uint32_t)(M >> (e & 63u)) & 1u;
  atomicOr((uint32_t*)((char*)cb + (e >> 11)), b << ((e >> 6) & 31u));
}
// any bit of hm (entries q0 .. q0+63) inside the entry range [ps, pe)
__device__ inline bool seg_any(uint64_t hm, uint32_t ps, uint32_t pe, uint32_t q0) {
  const uint32_t lo = max(ps, q0), hi = min(pe, q0 + 64);
  if (hi <= lo) return false;
  const uint32_t n = hi - lo;
  const uint64_t msk = n >= 64 ? ~0ull : ((1ull << n) - 1ull);
  return ((hm >> (lo - q0)) & msk) != 0;
}

__global__ __launch_bounds__(SEQ_B) void k_sw_seq(SwSeqArgs a) {
  // one block, the committed bitmap first: its word addresses are the list
  // entries' shifted fields with no base to add
  struct Lds {
    uint32_t cbits[(1u << SW_GBITS_MAX) / 32 + 1 + 64];  // + the SW_ID_NONE word, spare words
    uint32_t s_ready[SEQ_RING];
    uint32_t s_done, s_stop, s_k;
    uint64_t s_M[SW_PMAX_TILES];  // commit mask per decided tile
    SwRec ring[SEQ_RING];
  };
  __shared__ __attribute__((aligned(16))) Lds L;
  uint32_t* const cbits = L.cbits;
  uint32_t* const s_ready = L.s_ready;
  uint32_t &s_done = L.s_done, &s_stop = L.s_stop, &s_k = L.s_k;
  uint64_t* const s_M = L.s_M;
  SwRec* const ring = L.ring;
  const uint32_t j = threadIdx.x, lane = lane_id(), wv = j >> 6;
  const uint32_t ab = *a.abandon;
  const uint32_t m = list_len(a.m_dev, a.m_host);
  if (ab) return;
  const uint32_t lim = min(m, a.p_max);
  const uint32_t ntiles = min((lim + SW_T - 1) / SW_T, SW_PMAX_TILES);
  // the filter of this level starts from a clean look-back and ticket; the
  // next level's list is empty unless the filter writes it
  if (j == 0) {
    a.lv->ticket = 0;
    a.lv_next->m = 0;
    a.lv_next->acc = 0;
    a.next_off[0] = 0;
    s_k = 0;
    s_done = 0;
    s_stop = 0;
  }
  if (j < SEQ_RING) s_ready[j] = 0;
  uint64_t* dbg = a.dbg;
  if (dbg && j == 0) dbg[0] = __builtin_amdgcn_s_memrealtime();
  const uint32_t nwords = (1u << a.gbits) / 32;
  for (uint32_t q = j; q < nwords; q += SEQ_B) cbits[q] = 0;
  if (j == 0) cbits[SW_ID_NONE / 32] = 0;  // the word padding probes read
  __syncthreads();

  if (dbg && j == 0) dbg[1] = __builtin_amdgcn_s_memrealtime();
  if (wv > 0) {
    uint32_t pw = 0;
    // producers: wave p copies tiles p-1, p-1+15, ... into slot k % SEQ_RING
    for (uint32_t k = wv - 1; k < ntiles; k += SEQ_PROD) {
      const uint32_t slot = k % SEQ_RING;
      bool stopped = false;
      while (true) {
        if (lds_ld(&s_stop)) {
          stopped = true;
          break;
        }
        if (lds_ld(&s_done) + SEQ_RING > k) break;
        pw++;
        __builtin_amdgcn_s_sleep(8);
      }
      if (stopped) break;
      const uint4* src = (const uint4*)(a.rec + k);
      uint4* dst = (uint4*)&ring[slot];
      uint4 v[SEQ_V4 / 64];
#pragma unroll
      for (uint32_t q = 0; q < SEQ_V4 / 64; q++) v[q] = src[q * 64 + lane];
#pragma unroll
      for (uint32_t q = 0; q < SEQ_V4 / 64; q++) dst[q * 64 + lane] = v[q];
      if (lane == 0) lds_st(&s_ready[slot], k + 1);  // release: the record is in LDS
    }
    if (dbg && lane == 0 && pw) atomicAdd((unsigned long long*)&dbg[7], (unsigned long long)pw);
  } else if (ntiles) {
    // software pipelined: while tile k resolves, tile k+1's record (per-txn
    // words and the first SW_RC chunks of its lists) is read into registers
    // behind tile k's probes, and tile k+2's ready flag with it
    uint32_t k = 0, cw = 0, st_it = 0;
    uint64_t st_u = 0;
    __builtin_amdgcn_s_setprio(3);  // the serial wave issues ahead of the producers
    const uint64_t cyc0 = __builtin_amdgcn_s_memtime();
    while (lds_ld(&s_ready[0]) != 1u) {
      cw++;
      __builtin_amdgcn_s_sleep(1);
    }
    uint64_t cdep, cseg[SW_RC];
    uint32_t cmeta, chdr, cpe[SW_RC], cie[SW_RC_I];
    auto read_rec = [&](const SwRec& T) {
      cdep = T.dep[lane];
      cmeta = T.meta[lane];
      chdr = T.hdr;
#pragma unroll
      for (uint32_t c = 0; c < SW_RC; c++) {
        cpe[c] = T.probe[c * 64 + lane];
        cseg[c] = T.seg[c][lane];
      }
#pragma unroll
      for (uint32_t c = 0; c < SW_RC_I; c++) cie[c] = T.ins[c * 64 + lane];
    };
    read_rec(ring[0]);
    if (ntiles > 1)
      while (lds_ld(&s_ready[1 % SEQ_RING]) != 2u) {
        cw++;
        __builtin_amdgcn_s_sleep(1);
      }
    uint32_t fl = 0, slot = 0;
    for (; k < ntiles; k++) {
      const uint32_t hdr = __builtin_amdgcn_readfirstlane(chdr);
      if (hdr & SWH_STOP) break;
      const uint64_t dep = cdep;
      const uint32_t meta = cmeta;
      uint64_t seg[SW_RC];
      uint32_t pe[SW_RC], ie[SW_RC_I];
#pragma unroll
      for (uint32_t c = 0; c < SW_RC; c++) {
        seg[c] = cseg[c];
        pe[c] = cpe[c];
      }
#pragma unroll
      for (uint32_t c = 0; c < SW_RC_I; c++) ie[c] = cie[c];
      const uint32_t kn = k + 1, sn = slot + 1 == SEQ_RING ? 0u : slot + 1;
      // (1) probe C with the register chunks: a txn touching a committed key
      // is dead (padding entries read the always-zero word)
      uint32_t h[SW_RC];
#pragma unroll
      for (uint32_t c = 0; c < SW_RC; c++) h[c] = cb_probe(cbits, pe[c]);
      // tile k+1's record (its ready flag was checked during tile k-1; a
      // wave's LDS operations complete in order, so these reads see the
      // producer's writes; a slot past the last tile is read but never used)
      // and tile k+2's flag share the probes' round trip
      read_rec(ring[sn]);
      fl = lds_ld_rlx(&s_ready[sn + 1 == SEQ_RING ? 0u : sn + 1]);
      uint64_t kv = 0;
#pragma unroll
      for (uint32_t c = 0; c < SW_RC; c++) kv |= ballot64(h[c] != 0) & seg[c];
      uint64_t K = ballot64(kv != 0);
      if (hdr & SWH_PLONG) {  // long probe lists (rare)
        const uint32_t np = __builtin_amdgcn_readfirstlane(ring[slot].np);
        const uint32_t sp = ring[slot].pspan[lane];
        const uint32_t ps = sp & 0xFFFFu, pe2 = sp >> 16;
        const uint32_t* ovf = a.lst_ovf + (uint64_t)k * SW_OVF;
        bool kill = false;
        for (uint32_t q0 = SW_RC * 64; q0 < np; q0 += 64) {
          const uint32_t q = q0 + lane;
          uint32_t e = SW_P_NONE;
          if (q < np) e = q < SW_PL ? ring[slot].probe[q] : ld_sync(ovf + (q - SW_PL));
          kill |= seg_any(ballot64(cb_probe(cbits, e) != 0), ps, pe2, q0);
        }
        K |= ballot64(kill);
      }
      // (2) the tile's serial order: fixed point over the dependency masks
      // (round 1: candidates with no earlier candidate conflict commit)
      uint64_t U = ballot64((meta & (SWM_VALID | SWM_PRE)) == SWM_VALID) & ~K, M = 0;
      st_u += __builtin_popcountll(U);
      if (U) {
        const uint64_t d = ballot64((dep & U) == 0);
        M = U & d;
        U &= ~d;
        while (U) {
          const uint64_t cm = U & ballot64((dep & (M | U)) == 0);
          const uint64_t am = U & ballot64((dep & M) != 0);
          M |= cm;
          U &= ~(cm | am);
          st_it++;
        }
      }
      // tile k+2's record must be in its slot before tile k+1 reads it
      if (kn + 1 < ntiles)
        while (fl != kn + 2) {
          cw++;
          __builtin_amdgcn_s_sleep(1);
          fl = lds_ld_rlx(&s_ready[sn + 1 == SEQ_RING ? 0u : sn + 1]);
        }
      __atomic_signal_fence(__ATOMIC_SEQ_CST);
      // (3) needed writes of committed txns join C: a fixed number of LDS
      // operations per tile, so the next tile's wait counts stay exact
#pragma unroll
      for (uint32_t c = 0; c < SW_RC_I; c++) cb_insert_m(cbits, ie[c], M);
      if (hdr & SWH_ILONG) {  // long insert lists (rare)
        const uint32_t ni = __builtin_amdgcn_readfirstlane(ring[slot].ni);
        const uint32_t* ovf = a.lst_ovf + (uint64_t)k * SW_OVF;
        for (uint32_t q0 = SW_RC_I * 64; q0 < ni; q0 += 64) {
          const uint32_t q = q0 + lane;
          uint32_t e = sw_idummy(lane);
          if (q < ni) e = q < SW_IL ? ring[slot].ins[q] : ld_sync(ovf + SW_TA + (q - SW_IL));
          cb_insert_m(cbits, e, M);
        }
      }
      s_M[k] = M;  // every lane stores the same word (no exec branch)
      // free tile k's slot: LDS executes this wave's operations in order, so
      // a producer that sees kn has the slot's reads behind it
      __hip_atomic_store(&s_done, kn, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
      slot = sn;
    }
    if (lane == 0) {
      s_k = k;
      lds_st(&s_stop, 1u);
      if (dbg) {
        dbg[2] = __builtin_amdgcn_s_memrealtime();
        dbg[5] = cw;
        dbg[6] = k;
        dbg[8] = __builtin_amdgcn_s_memtime() - cyc0;
        dbg[9] = st_u;
        dbg[10] = st_it;
      }
    }
  }
  __syncthreads();
  const uint32_t k = s_k;
  // ---- write-out: decisions of tiles [0, k), the level's committed keys.
  // WO_U positions per thread and step, their record words loaded together
  // (one round trip per step instead of one per position)
  constexpr uint32_t WO_U = 8;
  for (uint32_t q0 = 0; q0 < k * SW_T; q0 += SEQ_B * WO_U) {  // uniform trip count (ballots)
    uint32_t mt[WO_U], tid[WO_U];
#pragma unroll
    for (uint32_t u = 0; u < WO_U; u++) {
      const uint32_t q = q0 + u * SEQ_B + j;
      mt[u] = 0;
      tid[u] = 0;
      if (q < k * SW_T) {
        mt[u] = a.rec[q / SW_T].meta[q % SW_T];
        tid[u] = a.rec[q / SW_T].rtid[q % SW_T];
      }
    }
    bool cw[WO_U];
#pragma unroll
    for (uint32_t u = 0; u < WO_U; u++) {
      const uint32_t q = q0 + u * SEQ_B + j;
      cw[u] = false;
      if (mt[u] & SWM_VALID) {
        const bool com = (s_M[q / SW_T] >> (q % SW_T)) & 1ull;
        if (!(mt[u] & SWM_PRE)) a.state[tid[u]] = com ? ST_COMMIT : ST_ABORT;
        if (a.write_hasw) a.hasw[tid[u]] = (mt[u] & SWM_HASW) ? 1 : 0;
        cw[u] = com && !(mt[u] & SWM_PRE) && (mt[u] & SWM_HASW);
      }
    }
    if (a.cw_list) {  // the committed writers, for the writer table (k_sw_wall)
      uint64_t bm[WO_U];
      uint32_t tot = 0;
#pragma unroll
      for (uint32_t u = 0; u < WO_U; u++) {
        bm[u] = ballot64(cw[u]);
        tot += (uint32_t)__popcll(bm[u]);
      }
      uint32_t base = 0;
      if (lane == 0 && tot) base = atomicAdd(a.cw_count, tot);
      base = __shfl(base, 0);
#pragma unroll
      for (uint32_t u = 0; u < WO_U; u++) {
        if (cw[u]) a.cw_list[base + (uint32_t)__popcll(bm[u] & lanemask_lt())] = tid[u];
        base += (uint32_t)__popcll(bm[u]);
      }
    }
  }
  if (dbg) {
    __syncthreads();
    if (j == 0) dbg[3] = __builtin_amdgcn_s_memrealtime();
  }
  // C for the filter is listed by k_sw_cout from the committed masks: clear
  // its bitmap, Bloom filter and count here
  for (uint32_t q = j; q < k; q += SEQ_B) a.mg[q] = s_M[q];
  for (uint32_t q = j; q < nwords; q += SEQ_B) a.cbits_out[q] = 0;
  for (uint32_t q = j; q < (1u << SW_BLOOM_LOG) / 32; q += SEQ_B) a.bloom_out[q] = 0;
  if (j == 0) {
    a.lv->pos = min(k * SW_T, lim);
    a.lv->ccount = 0;  // k_sw_cout's fill counter
    if (dbg) dbg[4] = __builtin_amdgcn_s_memrealtime();
  }
}

// ---------------------------------------------------------------------------
// k_sw_cout: the level's committed set C for the filter, across the grid:
// every WR access of a committed txn of the serial range [0, pos) gives its
// key (Bloom filter, key list with wave-aggregated positions: the filter
// uses them as a set) and its key id (bitmap for the exact check).
__global__ __launch_bounds__(256) void k_sw_cout(SwCoutArgs a) {
  __shared__ uint32_t s_cnt[4];
  __shared__ uint32_t s_base;
  // workgroups past the listing's (level 0 only): the batch validation pass
  // -- the host reads its partials after the epoch -- and the clear of the
  // epoch's committed-writer table (used only after the last level)
  if (blockIdx.x >= a.cout_grid) {
    const uint32_t b = blockIdx.x - a.cout_grid, nb = gridDim.x - a.cout_grid;
    prep_body_hasw(a.prep_off, a.prep_n, a.prep_at, a.prep_nnz, a.hasw, a.prep_part, b, nb, a.prep_err);
    const uint4 e = make_uint4(~0u, ~0u, ~0u, ~0u);
    for (uint64_t q = (uint64_t)b * 256 + threadIdx.x; q < a.wclear_n16; q += (uint64_t)nb * 256)
      a.wclear[q] = e;
    return;
  }
  const uint32_t ab = *a.abandon;
  const uint32_t pos = a.lv->pos;
  const uint32_t m = list_len(a.m_dev, a.m_host);
  const uint32_t o0_raw = a.in.off[0];
  if (ab) return;
  if (a.skip_done && pos >= m) return;
  const uint32_t lane = lane_id(), wv = threadIdx.x >> 6;
  const uint64_t nnz = a.in.nnz;
  const uint32_t off0 = (uint32_t)min((uint64_t)o0_raw, nnz);
  const uint32_t range = (uint32_t)min((uint64_t)a.in.off[pos], nnz) - off0;
  // 1024 accesses per workgroup round (wave w: [256w, 256w + 256)), one
  // fill-counter atomic per round
  for (uint32_t x0 = blockIdx.x * 1024; x0 < range; x0 += gridDim.x * 1024) {
    // each access's entry, position and key loaded together (the position
    // and key of an access that is not a write are read and ignored), then
    // the commit-mask word: two round trips instead of four
    uint32_t ent[4], ap[4];
    uint64_t kx[4];
    bool c[4];
#pragma unroll
    for (uint32_t u = 0; u < 4; u++) {
      const uint32_t x = x0 + wv * 256 + u * 64 + lane;
      const bool in = x < range;
      ent[u] = in ? a.aent[x] : 0u;
      ap[u] = in ? a.apos[x] : 0u;
      kx[u] = in ? a.in.keys[off0 + x] : 0ull;
    }
    uint64_t mw[4];
#pragma unroll
    for (uint32_t u = 0; u < 4; u++) mw[u] = (ent[u] & 32u) ? a.mg[ap[u] >> 6] : 0ull;
#pragma unroll
    for (uint32_t u = 0; u < 4; u++) c[u] = (ent[u] & 32u) && ((mw[u] >> (ap[u] & 63u)) & 1ull);
    uint64_t cm[4];
    uint32_t wc = 0;
#pragma unroll
    for (uint32_t u = 0; u < 4; u++) {
      cm[u] = ballot64(c[u]);
      wc += (uint32_t)__popcll(cm[u]);
    }
    if (lane == 0) s_cnt[wv] = wc;
    __syncthreads();
    if (threadIdx.x == 0) {
      const uint32_t tot = s_cnt[0] + s_cnt[1] + s_cnt[2] + s_cnt[3];
      s_base = tot ? atomicAdd(&a.lv->ccount, tot) : 0u;
    }
    __syncthreads();
    uint32_t base = s_base;
    for (uint32_t w = 0; w < wv; w++) base += s_cnt[w];
#pragma unroll
    for (uint32_t u = 0; u < 4; u++) {
      if (c[u]) {
        const uint64_t key = kx[u];
        a.ckeys_out[base + (uint32_t)__popcll(cm[u] & lanemask_lt())] = key;
        const uint32_t id = sw_aid(ent[u]);
        if (id < SW_ID_NONE) atomicOr(&a.cbits_out[id >> 5], 1u << (id & 31u));
        uint32_t b1, b2;
        bloom_bits(key, b1, b2);
        atomicOr(&a.bloom_out[b1 >> 5], 1u << (b1 & 31));
        atomicOr(&a.bloom_out[b2 >> 5], 1u << (b2 & 31));
      }
      base += (uint32_t)__popcll(cm[u]);
    }
    __syncthreads();  // s_cnt / s_base of the next round
  }
}

// ---------------------------------------------------------------------------
// k_sw_filter: list txns [pos, m) against C; survivors -> next level's list.
// Chunks of SW_CHUNK txns are taken by ticket (so every chunk a look-back
// waits on is held by a running workgroup); 16 waves x 64 txns per chunk.

constexpr uint32_t FW = SW_CHUNK / 64;  // waves per filter workgroup
constexpr uint32_t FK = 16;             // access rounds kept in registers (1024 accesses)
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
    // a bucket with a free slot ends the chain (gtab_insert)
    if (v0 == KEY_EMPTY || v1 == KEY_EMPTY || v2 == KEY_EMPTY || v3 == KEY_EMPTY) return false;
    b = (b + 1) & nbm;
  }
  return false;
}
constexpr uint32_t F_STASH = 256;  // Bloom-positive keys kept in LDS per wave
#ifndef DCC_F_XS
#define DCC_F_XS 2048
#endif
#ifndef DCC_F_WPE
#define DCC_F_WPE 1
#endif
constexpr uint32_t F_XS = DCC_F_XS;    // small-C filter instance: LDS exact-set slots
constexpr uint32_t F_XCAP = F_XS / 2;  // ... for C of up to this many keys (<= 50% load)
constexpr uint32_t F_XBITS_LOG = 16;  // ... its one-hash bitmap of C (8 KiB)

// ---------------------------------------------------------------------------
// k_sw_filter: list txns [pos, m) against C, 64 per wave, grid-stride (no
// cross-workgroup waits).  A txn touching a key of C is killed; the others
// get a survivor bit and per-tile counts for the compaction.
// Two modes, chosen per launch from |C|: exact (X) when C has <= F_XCAP keys
// -- C as an LDS hash set behind a one-hash LDS bitmap, nothing global --
// and the level's Bloom filter with exact checks in the global key table
// otherwise.  Their LDS overlaps (36 KB in all: four workgroups fit a CU).
__global__ __launch_bounds__(SW_CHUNK, DCC_F_WPE) void k_sw_filter(SwFilterArgs a) {
  constexpr uint32_t B = SW_CHUNK, FW = B / 64;
  constexpr uint32_t CS = F_XS;  // exact-set slots (X)
  struct XSet {
    uint32_t bl[(1u << F_XBITS_LOG) / 32];
    uint64_t cex[F_XS];
  };
  union FSet {
    XSet x;
    uint32_t bl[(1u << SW_BLOOM_LOG) / 32];
  };
  __shared__ __attribute__((aligned(16))) FSet fs;
  uint32_t* const bl = fs.bl;     // both modes' bitmaps start the union
  uint64_t* const cex = fs.x.cex;
  __shared__ uint64_t s_hit[FW][SW_WA / 64];
  __shared__ uint64_t s_stash[FW][F_STASH];
  __shared__ uint32_t s_wpre[FW][SW_WA / 64];
  const uint32_t j = threadIdx.x, lane = lane_id(), wv = j >> 6;
  const uint32_t ab = *a.abandon;
  const uint32_t m = list_len(a.m_dev, a.m_host);
  const uint32_t pos = a.lv->pos;
  const uint32_t ccount = a.lv->ccount;
  if (ab) return;
  const bool X = ccount <= F_XCAP;  // uniform
  // DCC_SW_DEBUG: wave 0 of workgroups < 256 stamps start / setup / loads /
  // exact checks / writes / end and counts its tiles
  uint64_t* dbg = (a.dbg && blockIdx.x < 256 && j == 0) ? a.dbg + 8 * blockIdx.x : nullptr;
  if (dbg) dbg[0] = __builtin_amdgcn_s_memrealtime();
  // the serial pass decided the whole list: no next level (the epoch's first
  // level table is filled by the epoch's setup); sharded ranks still serve
  // the merged serial range of the next level
  if (pos >= m && !a.kill_out) return;
  // the next level's key table (its pre-pass runs after this kernel)
  for (uint64_t q = (uint64_t)blockIdx.x * B + j; q < a.gclear_n;
       q += (uint64_t)gridDim.x * B) {
    a.gclear[q] = KEY_EMPTY;
    a.fw_clear[q] = ~0u;
    a.la_clear[q] = 0u;
  }
  if (pos >= m) return;
  const uint32_t n64 = (m - pos + 63) / 64;
  const uint64_t nnz = a.in.nnz;
  // workgroup g: tiles [g R, (g + 1) R), its total into bsum[g] (two-level scan)
  const uint32_t R = sw_tiles_per_wg(n64, gridDim.x);
  const uint32_t t_lo = min(blockIdx.x * R, n64), t_hi = min(t_lo + R, n64);
  if (t_lo >= t_hi) {  // idle: no setup
    if (!a.kill_out && j == 0) {
      a.bsum[blockIdx.x] = 0;
      if (a.ro_split) a.rbsum[blockIdx.x] = 0;
    }
    return;
  }
  const bool small = X;  // exact checks in LDS
  {
    if (!X) {
      const uint4* src = (const uint4*)a.bloom;
      uint4* dst = (uint4*)bl;
      for (uint32_t q = j; q < (1u << SW_BLOOM_LOG) / 128; q += B) dst[q] = src[q];
    } else {
      for (uint32_t q = j; q < (1u << F_XBITS_LOG) / 32; q += B) bl[q] = 0;
      for (uint32_t q = j; q < CS; q += B) cex[q] = KEY_EMPTY;
    }
  }
  __syncthreads();
  if (small) {
    for (uint32_t q = j; q < ccount; q += B) {
      const uint64_t kq = a.ckeys[q];
      lset_insert<CS>(cex, kq);
      if (X) {
        uint32_t b1, b2;
        bloom_bits(kq, b1, b2);
        b1 >>= SW_BLOOM_LOG - F_XBITS_LOG;
        atomicOr(&bl[b1 >> 5], 1u << (b1 & 31u));
      }
    }
    __syncthreads();
  }
  if (dbg) dbg[1] = __builtin_amdgcn_s_memrealtime();
  uint64_t* hit = s_hit[wv];
  uint64_t* stash = s_stash[wv];
  uint64_t wsum = 0, rsum = 0;
  // the per-txn words of a wave's next tile are loaded while the current
  // tile's keys are in flight (branch-free, clamped: they issue together)
  uint32_t ns = 0, ne = 0, ntid = 0, nst = 0, nhw = 1;
  auto prefetch = [&](uint32_t wt) {
    const uint32_t pc = min(pos + wt * 64 + lane, m - 1);
    ns = a.in.off[pc];
    ne = a.in.off[pc + 1];
    ntid = a.in.tid ? a.in.tid[pc] : pc;
    nst = a.cand_state ? a.state[pc] : 0u;
    if (a.ro_split) nhw = a.hasw[pc];  // identity list: pc is the txn
  };
  if (t_lo + wv < t_hi) prefetch(t_lo + wv);
  for (uint32_t wt = t_lo + wv; wt < t_hi; wt += FW) {
    const uint32_t p = pos + wt * 64 + lane;
    const bool valid = p < m;
    uint32_t s = 0, e = 0, tid = 0;
    bool cand = false, ro = false;
    if (valid) {
      s = (uint32_t)min((uint64_t)ns, nnz);
      e = (uint32_t)min((uint64_t)ne, nnz);
      if (e < s) e = s;
      tid = ntid;
      cand = nst == ST_UNDECIDED;
      ro = nhw == 0;
    }
    bool pref = false;
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
#pragma unroll
      for (uint32_t u = 0; u < FK; u++) {
        const uint32_t xr = b0 + 64 * u + lane;
        const uint32_t x = A0 + (xr < span ? xr : 0u);
        key[u] = a.in.keys[x];
      }
      if (!pref) {
        pref = true;
        if (wt + FW < t_hi) prefetch(wt + FW);
      }
#pragma unroll
      for (uint32_t u = 0; u < FK; u++) {
        const uint32_t xr = b0 + 64 * u + lane;
        if (b0 + 64 * u >= span) continue;  // uniform; no break: the loop must unroll
        const bool in = xr < span;
        bad_key |= in && key[u] == KEY_EMPTY;
        bool h;
        uint32_t b1, b2;
        bloom_bits(key[u], b1, b2);
        if (X) {
          b1 >>= SW_BLOOM_LOG - F_XBITS_LOG;
          h = in && ((bl[b1 >> 5] >> (b1 & 31u)) & 1u) != 0;
        } else {
          const uint32_t wa = bl[b1 >> 5], wb = bl[b2 >> 5];
          h = in && (((wa >> (b1 & 31u)) & (wb >> (b2 & 31u)) & 1u) != 0);
        }
        const uint64_t hb = ballot64(h);
        if (h) {
          const uint32_t ci = npos + (uint32_t)__popcll(hb & lanemask_lt());
          if (ci < F_STASH) stash[ci] = key[u];
        }
        npos += (uint32_t)__popcll(hb);
        if (lane == 0) hit[(b0 >> 6) + u] = hb;
      }
    }
    if (!pref && wt + FW < t_hi) prefetch(wt + FW);  // a tile without accesses
    if (ballot64(bad_key) && lane == 0) atomicOr(a.err, ERR_KEY);
    if (dbg && wt == t_lo) dbg[2] = __builtin_amdgcn_s_memrealtime();
    // per txn (the wave's own LDS rows: no barrier needed)
    const uint32_t rlo = s - A0, rlen = e - s;
    const bool ok = valid && (rlen == 0 || (uint64_t)rlo + rlen <= span);
    bool killed = false;
    {
      {
        const uint32_t pw = lane < nw ? (uint32_t)__popcll(hit[lane]) : 0u;
        uint32_t ptot;
        const uint32_t pre = wave_excl_u32(pw, ptot);
        if (lane < nw) s_wpre[wv][lane] = pre;
      }
      // Bloom-positive accesses of the txn, verified one by one (almost always
      // the first is a true hit): the key from the LDS stash, then the exact set
      if (cand && ok && rlen) {
        for (uint32_t x = rlo; x < rlo + rlen; x++) {
          const uint32_t nx = range_next(hit, x, rlo + rlen);
          if (nx >= rlo + rlen) break;
          const uint32_t ci = s_wpre[wv][nx >> 6] +
                              (uint32_t)__popcll(hit[nx >> 6] & ((1ull << (nx & 63)) - 1ull));
          const uint64_t kx = ci < F_STASH ? stash[ci] : a.in.keys[A0 + nx];
          if (small ? lset_find<CS>(cex, kx) : c_exact(a, kx)) {
            killed = true;
            break;
          }
          x = nx;
        }
      }
    }
    if (dbg && wt == t_lo) dbg[3] = __builtin_amdgcn_s_memrealtime();
    if (dbg) dbg[6]++;
    if (a.kill_out) {  // key-sharded: this shard's kill bits only (k_sw_apply decides)
      const uint64_t km = ballot64(valid && killed);
      if (lane == 0) a.kill_out[wt] = km;
      continue;
    }
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
    if (a.ro_split) {  // read-only survivors, counted apart (k_sw_compact splits them off)
      const uint64_t rm = ballot64(surv && ro);
      const uint64_t racc = wave_sum64(surv && ro ? rlen : 0u);
      const uint64_t rc = ((uint64_t)__popcll(rm) << LB_ACC_BITS) | racc;
      rsum += rc;
      if (lane == 0) {
        a.rflag[wt] = rm;
        a.rtcount[wt] = rc;
      }
    }
    if (dbg && wt == t_lo) {
      __builtin_amdgcn_s_waitcnt(0);
      dbg[4] = __builtin_amdgcn_s_memrealtime();
    }
  }
  if (a.kill_out) return;
  __shared__ unsigned long long s_bs[FW][2];
  if (lane == 0) {
    s_bs[wv][0] = wsum;
    s_bs[wv][1] = rsum;
  }
  __syncthreads();
  if (j == 0) {
    uint64_t t = 0, r = 0;
    for (uint32_t w = 0; w < FW; w++) {
      t += s_bs[w][0];
      r += s_bs[w][1];
    }
    a.bsum[blockIdx.x] = t;
    if (a.ro_split) a.rbsum[blockIdx.x] = r;
  }
  if (dbg) {
    __builtin_amdgcn_s_waitcnt(0);
    dbg[5] = __builtin_amdgcn_s_memrealtime();
  }
}

// ---------------------------------------------------------------------------
// Key-sharded sweep: every rank holds all txns but only the
// accesses of its key shard.
//
// k_sw_apply: after the MAX all-reduce of the filters' kill bits, the level's
// decision on every rank alike: a candidate killed on any shard aborts, every
// other candidate survives (also one without accesses on this shard: another
// shard may hold them; a txn with none at all commits in a later serial pass).
// Same tile -> workgroup mapping as the filter (survivor words, counts, totals
// for k_sw_compact).
__global__ __launch_bounds__(SW_CHUNK) void k_sw_apply(SwFilterArgs a) {
  const uint32_t lane = lane_id(), wv = threadIdx.x >> 6;
  if (*a.abandon) return;
  const uint32_t m = list_len(a.m_dev, a.m_host);
  const uint32_t pos = a.lv->pos;
  if (pos >= m) return;
  const uint32_t n64 = (m - pos + 63) / 64;
  const uint64_t nnz = a.in.nnz;
  const uint32_t R = sw_tiles_per_wg(n64, gridDim.x);
  const uint32_t t_lo = min(blockIdx.x * R, n64), t_hi = min(t_lo + R, n64);
  uint64_t wsum = 0, rsum = 0;
  for (uint32_t wt = t_lo + wv; wt < t_hi; wt += SW_CHUNK / 64) {
    const uint32_t p = pos + wt * 64 + lane;
    // a kill on any shard wins: the OR of every rank's word of this tile
    uint64_t kw = 0;
    for (uint32_t r = 0; r < a.kill_ranks; r++) kw |= a.kill_in[r * a.kill_stride + wt];
    const bool kill = (kw >> lane) & 1ull;
    bool surv = false, ro = false;
    uint32_t len = 0;
    if (p < m) {
      const uint32_t tid = a.in.tid ? a.in.tid[p] : p;
      const bool cand = a.cand_state ? a.state[p] == ST_UNDECIDED : true;
      const uint32_t s = (uint32_t)min((uint64_t)a.in.off[p], nnz);
      const uint32_t e = (uint32_t)min((uint64_t)a.in.off[p + 1], nnz);
      len = e > s ? e - s : 0u;
      if (cand && kill) a.state[tid] = ST_ABORT;
      surv = cand && !kill;
      ro = a.ro_split && a.hasw[tid] == 0;  // the has-write bytes are the whole batch's
    }
    const uint64_t sm = ballot64(surv);
    const uint64_t acc = wave_sum64(surv ? len : 0u);
    const uint64_t cnt = ((uint64_t)__popcll(sm) << LB_ACC_BITS) | acc;
    wsum += cnt;
    if (lane == 0) {
      a.sflag[wt] = sm;
      a.tcount[wt] = cnt;
    }
    if (a.ro_split) {  // read-only survivors counted apart (as the filter does)
      const uint64_t rm = ballot64(surv && ro);
      const uint64_t racc = wave_sum64(surv && ro ? len : 0u);
      const uint64_t rc = ((uint64_t)__popcll(rm) << LB_ACC_BITS) | racc;
      rsum += rc;
      if (lane == 0) {
        a.rflag[wt] = rm;
        a.rtcount[wt] = rc;
      }
    }
  }
  __shared__ unsigned long long s_bs[SW_CHUNK / 64][2];
  if (lane == 0) {
    s_bs[wv][0] = wsum;
    s_bs[wv][1] = rsum;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    uint64_t t = 0, r = 0;
    for (uint32_t w = 0; w < SW_CHUNK / 64; w++) {
      t += s_bs[w][0];
      r += s_bs[w][1];
    }
    a.bsum[blockIdx.x] = t;
    if (a.ro_split) a.rbsum[blockIdx.x] = r;
  }
}

// k_sw_sg_scan (one workgroup): the offsets of the first P = min(p_max, *m)
// list txns' whole access lists (soff[0..P]); k_sw_sg_copy: their keys and
// types, 16 lanes per txn.  The serial range of a level of a key-sharded
// epoch whose ranks hold the whole batch (DCC_SHARD_SELF).
constexpr uint32_t SG_T = 1024;
__global__ __launch_bounds__(SG_T) void k_sw_sg_scan(const uint32_t* tid, const uint32_t* m_dev, uint32_t p_max,
                                                     const uint32_t* full_off, uint64_t full_nnz, uint32_t* soff,
                                                     uint32_t* err) {
  __shared__ uint32_t s_w[SG_T / 64];
  __shared__ uint32_t s_carry;
  const uint32_t P = min(p_max, *m_dev), lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  if (threadIdx.x == 0) s_carry = 0;
  __syncthreads();
  for (uint32_t q0 = 0; q0 < P; q0 += SG_T) {
    const uint32_t q = q0 + threadIdx.x;
    uint32_t len = 0;
    if (q < P) {
      const uint32_t t = tid[q];
      const uint64_t s = min((uint64_t)full_off[t], full_nnz), e = min((uint64_t)full_off[t + 1], full_nnz);
      len = e > s ? (uint32_t)(e - s) : 0u;
      if (len > MAX_TXN_LEN) {
        atomicOr(err, ERR_OFFSETS);
        len = 0;
      }
    }
    uint32_t x = len;
    for (int d = 1; d < 64; d <<= 1) {
      const uint32_t y = __shfl_up(x, d);
      if (lane >= (uint32_t)d) x += y;
    }
    if (lane == 63) s_w[wv] = x;
    __syncthreads();
    uint32_t b = s_carry;
    for (uint32_t w = 0; w < wv; w++) b += s_w[w];
    if (q < P) soff[q] = b + x - len;
    __syncthreads();
    if (threadIdx.x == SG_T - 1) s_carry = b + x;
    __syncthreads();
  }
  if (threadIdx.x == 0) soff[P] = s_carry;
}
__global__ __launch_bounds__(256) void k_sw_sg_copy(const uint32_t* tid, const uint32_t* m_dev, uint32_t p_max,
                                                    const uint32_t* full_off, const uint64_t* full_keys,
                                                    const uint8_t* full_at, uint64_t full_nnz, const uint32_t* soff,
                                                    uint64_t* skeys, uint8_t* sat) {
  const uint32_t P = min(p_max, *m_dev), sl = threadIdx.x & 15u;
  for (uint32_t q = (blockIdx.x * 256 + threadIdx.x) >> 4; q < P; q += gridDim.x * 16) {
    const uint32_t t = tid[q], o = soff[q], len = soff[q + 1] - o;
    const uint64_t s = min((uint64_t)full_off[t], full_nnz);
    for (uint32_t x = sl; x < len; x += 16) {
      skeys[o + x] = full_keys[s + x];
      sat[o + x] = full_at[s + x];
    }
  }
}

// k_sw_share (one thread): a key-sharded level's sizes in this rank's slots
// of the size exchange: list length (every rank alike), the abandon word, the
// serial range's txn count and this rank's accesses of it.
__global__ void k_sw_share(const uint32_t* m_dev, uint32_t m_host, const uint32_t* abandon,
                           const uint32_t* off, uint32_t p_max, uint32_t rank, uint32_t* cnt) {
  const uint32_t m = m_dev ? *m_dev : m_host;
  const uint32_t P = min(p_max, m);
  cnt[0] = m;
  cnt[1] = *abandon;
  cnt[2 + rank] = m ? off[P] - off[0] : 0u;
}

// k_sw_export: this rank's accesses of the level's serial range (list txns
// [0, P)) as 12-byte records {key, txn | type << 30} into its all-gather
// contribution (padded with 0xFF records up to the largest share).
__global__ __launch_bounds__(256) void k_sw_export(SwList in, uint32_t P, uint32_t* rec) {
  const uint64_t nnz = in.nnz;
  const uint32_t off0 = (uint32_t)min((uint64_t)in.off[0], nnz);
  for (uint32_t t = blockIdx.x * 4 + (threadIdx.x >> 6); t < P; t += gridDim.x * 4) {
    const uint32_t s = (uint32_t)min((uint64_t)in.off[t], nnz);
    const uint32_t e = (uint32_t)min((uint64_t)in.off[t + 1], nnz);
    for (uint32_t x = s + lane_id(); x < e; x += 64) {
      const uint64_t k = in.keys[x];
      uint32_t* r = rec + 3ull * (x - off0);
      r[0] = (uint32_t)k;
      r[1] = (uint32_t)(k >> 32);
      r[2] = t | ((uint32_t)(in.acctype[x] & 3u) << 30);
    }
  }
}

// k_sw_mcount / k_sw_mscan / k_sw_mscatter: every rank's records merged into
// one CSR of the serial range, grouped by txn (a counting sort; the order of a
// txn's accesses is irrelevant to OCC, which compares sets).
// (records whose txn field is >= P are all-gather padding: skipped)
__global__ __launch_bounds__(256) void k_sw_mcount(const uint32_t* rec, uint32_t n, uint32_t P,
                                                   uint32_t* cnt) {
  for (uint32_t i = blockIdx.x * 256 + threadIdx.x; i < n; i += gridDim.x * 256) {
    const uint32_t t = rec[3ull * i + 2] & 0x3FFFFFFFu;
    if (t < P) atomicAdd(&cnt[t], 1u);
  }
}
__global__ __launch_bounds__(1024) void k_sw_mscan(uint32_t* cnt, uint32_t P, uint32_t* off,
                                                   uint32_t* cur) {
  __shared__ uint32_t s_w[16];
  __shared__ uint32_t s_carry;
  const uint32_t j = threadIdx.x, lane = lane_id(), wv = j >> 6;
  if (j == 0) s_carry = 0;
  __syncthreads();
  for (uint32_t c0 = 0; c0 < P; c0 += 1024) {
    const uint32_t t = c0 + j;
    const uint32_t v = t < P ? cnt[t] : 0u;
    uint32_t tot;
    const uint32_t ex = wave_excl_u32(v, tot);
    if (lane == 0) s_w[wv] = tot;
    __syncthreads();
    uint32_t base = s_carry;
    for (uint32_t w = 0; w < wv; w++) base += s_w[w];
    if (t < P) {
      off[t] = base + ex;
      cur[t] = base + ex;
    }
    __syncthreads();
    if (j == 0) {
      uint32_t all = 0;
      for (uint32_t w = 0; w < 16; w++) all += s_w[w];
      s_carry += all;
    }
    __syncthreads();
  }
  if (j == 0) off[P] = s_carry;
}
__global__ __launch_bounds__(256) void k_sw_mscatter(const uint32_t* rec, uint32_t n, uint32_t P,
                                                     uint32_t* cur, uint64_t* keys,
                                                     uint8_t* at) {
  for (uint32_t i = blockIdx.x * 256 + threadIdx.x; i < n; i += gridDim.x * 256) {
    const uint32_t w2 = rec[3ull * i + 2];
    if ((w2 & 0x3FFFFFFFu) >= P) continue;  // padding
    const uint32_t q = atomicAdd(&cur[w2 & 0x3FFFFFFFu], 1u);
    keys[q] = ((uint64_t)rec[3ull * i + 1] << 32) | rec[3ull * i];
    at[q] = (uint8_t)(w2 >> 30);
  }
}

// ---------------------------------------------------------------------------
// k_sw_compact: the survivors, in index order, into the next level's list.
__global__ __launch_bounds__(SW_CHUNK) void k_sw_compact(SwFilterArgs a) {
  const uint32_t lane = lane_id(), wv = threadIdx.x >> 6;
  // an earlier level's hand-off: nothing to compact (this level's own
  // decision is made below and still needs its list)
  const uint32_t ab = *a.abandon;
  const uint32_t m = list_len(a.m_dev, a.m_host);
  const uint32_t pos = a.lv->pos;
  if (ab && ab != a.level + 1) return;
  if (pos >= m) return;
  const uint32_t n64 = (m - pos + 63) / 64;
  const uint64_t nnz = a.in.nnz;
  // the filter's block ranges: block base from the scan, tile bases in LDS
  const uint32_t R = sw_tiles_per_wg(n64, a.nblocks);
  const uint32_t t_lo = min(blockIdx.x * R, n64), t_hi = min(t_lo + R, n64);
  if (t_lo >= t_hi && blockIdx.x) return;  // idle (workgroup 0 closes the level)
  uint64_t* dbg = (a.cdbg && blockIdx.x == 0 && threadIdx.x == 0) ? a.cdbg : nullptr;
  if (dbg) dbg[0] = __builtin_amdgcn_s_memrealtime();
  __shared__ unsigned long long s_tb[SW_CMP_MAXR];
  __shared__ unsigned long long s_part[SW_CHUNK / 64][4];
  __shared__ uint32_t s_split, s_rnext;  // RO list: next position of this workgroup's block
  if (R > SW_CMP_MAXR) {
    if (threadIdx.x == 0) atomicOr(a.err, ERR_TILE);
    return;
  }
  // this workgroup's base: the filter workgroups' totals before it (no
  // separate scan pass); workgroup 0 also closes the level with the total.
  // Read-only survivors (ro_split) leave the list for the RO list unless the
  // level hands off (every workgroup takes the same decision from the same
  // totals): packed count|accesses words subtract field by field.
  {
    uint64_t pre = 0, all = 0, rpre = 0, rall = 0;
    // every total of this thread loaded before the first is added (the
    // filter grid is at most 4 x n_CU: four per thread at 256 CUs), not one
    // dependent round trip per step
    constexpr uint32_t TU = 4;
    for (uint32_t q0 = threadIdx.x; q0 < a.nblocks; q0 += SW_CHUNK * TU) {
      uint64_t v[TU], r[TU];
#pragma unroll
      for (uint32_t u = 0; u < TU; u++) {
        const uint32_t q = q0 + u * SW_CHUNK;
        v[u] = q < a.nblocks ? a.bsum[q] : 0ull;
        r[u] = (a.ro_split && q < a.nblocks) ? a.rbsum[q] : 0ull;
      }
#pragma unroll
      for (uint32_t u = 0; u < TU; u++) {
        const uint32_t q = q0 + u * SW_CHUNK;
        all += v[u];
        rall += r[u];
        if (q < blockIdx.x) {
          pre += v[u];
          rpre += r[u];
        }
      }
    }
    pre = wave_sum64(pre);
    all = wave_sum64(all);
    rpre = wave_sum64(rpre);
    rall = wave_sum64(rall);
    if (lane == 0) {
      s_part[wv][0] = pre;
      s_part[wv][1] = all;
      s_part[wv][2] = rpre;
      s_part[wv][3] = rall;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
      uint64_t p0 = 0, a0 = 0, rp = 0, ra = 0;
      for (uint32_t w = 0; w < SW_CHUNK / 64; w++) {
        p0 += s_part[w][0];
        a0 += s_part[w][1];
        rp += s_part[w][2];
        ra += s_part[w][3];
      }
      const uint32_t tot = (uint32_t)(a0 >> LB_ACC_BITS);
      const uint32_t in_n = m - pos;
      const bool handoff =
          tot > a.abandon_min && (uint64_t)tot * a.abandon_den > (uint64_t)in_n * a.abandon_num;
      const bool split = a.ro_split && !handoff;
      s_split = split ? 1u : 0u;
      s_part[0][0] = split ? p0 - rp : p0;
      s_rnext = (uint32_t)(rp >> LB_ACC_BITS);
      if (blockIdx.x == 0) {
        const uint64_t keep = split ? a0 - ra : a0;
        const uint32_t kt = (uint32_t)(keep >> LB_ACC_BITS);
        const uint64_t acc = keep & ((1ull << LB_ACC_BITS) - 1);
        a.lv_next->m = kt;
        a.lv_next->acc = (uint32_t)acc;
        a.off_out[kt] = (uint32_t)acc;
        if (a.ro_split) *a.ro_count = split ? (uint32_t)(ra >> LB_ACC_BITS) : 0u;
        if (handoff) atomicMax(a.abandon_out, a.level + 1);
      }
    }
    __syncthreads();
  }
  const bool split = s_split != 0;
  if (dbg) dbg[1] = __builtin_amdgcn_s_memrealtime();
  if (wv == 0) {
    uint64_t run = s_part[0][0];
    for (uint32_t c0 = t_lo; c0 < t_hi; c0 += 64) {
      const uint32_t q = c0 + lane;
      const uint64_t v = (q < t_hi ? a.tcount[q] : 0ull) - ((split && q < t_hi) ? a.rtcount[q] : 0ull);
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
  if (dbg) dbg[2] = __builtin_amdgcn_s_memrealtime();
  // a wave's tiles CB at a time: every survivor word, offset pair and txn id
  // of the CB tiles in flight together, then each tile's moves
  constexpr uint32_t CB = 4;
  for (uint32_t w0 = t_lo + wv; w0 < t_hi; w0 += FW * CB) {
    uint64_t wordv[CB], rwordv[CB];
    uint32_t sv[CB], ev[CB], tv[CB];
#pragma unroll
    for (uint32_t i = 0; i < CB; i++) {
      const uint32_t wt = w0 + FW * i;
      const uint32_t pc = min(pos + min(wt, n64 - 1) * 64 + lane, m - 1);
      wordv[i] = wt < t_hi ? a.sflag[wt] : 0ull;
      rwordv[i] = (split && wt < t_hi) ? a.rflag[wt] : 0ull;
      sv[i] = a.in.off[pc];
      ev[i] = a.in.off[pc + 1];
      tv[i] = a.in.tid ? a.in.tid[pc] : pc;
    }
#pragma unroll
    for (uint32_t i = 0; i < CB; i++) {
      const uint32_t wt = w0 + FW * i;
      const uint64_t rword = rwordv[i];
      const uint64_t word = wordv[i] & ~rword;
      if (rword) {  // uniform: the RO list's order is free (its txns are decided alone)
        uint32_t rb = 0;
        if (lane == 0) rb = atomicAdd(&s_rnext, (uint32_t)__popcll(rword));
        rb = __shfl(rb, 0);
        if ((rword >> lane) & 1ull) {
          const uint32_t rs = (uint32_t)min((uint64_t)sv[i], nnz);
          a.ro_out[rb + (uint32_t)__popcll(rword & lanemask_lt())] =
              RoEnt{tv[i], rs, max(rs, (uint32_t)min((uint64_t)ev[i], nnz)), 0u};
        }
      }
      if (!word) continue;  // uniform
      const uint64_t base = s_tb[wt - t_lo];
      const uint32_t tb = (uint32_t)(base >> LB_ACC_BITS);
      const uint32_t abase = (uint32_t)(base & ((1ull << LB_ACC_BITS) - 1));
      const bool surv = (word >> lane) & 1ull;
      uint32_t s = 0, len = 0;
      if (surv) {
        s = (uint32_t)min((uint64_t)sv[i], nnz);
        len = (uint32_t)min((uint64_t)ev[i], nnz) - s;
      }
      uint32_t atot;
      const uint32_t aex = wave_excl_u32(len, atot);
      if (surv) {
        const uint32_t r = tb + (uint32_t)__popcll(word & lanemask_lt());
        a.tid_out[r] = tv[i];
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
  if (dbg) {
    __builtin_amdgcn_s_waitcnt(0);
    dbg[4] = __builtin_amdgcn_s_memrealtime();
  }
}

// ---------------------------------------------------------------------------
// k_sw_ro: the read-only txns level 0 split off, 4 lanes per txn, each lane
// four accesses per step (accesses sl, sl + 4, sl + 8, sl + 12 of the step)
// with their key loads and first probes in flight together: a key whose
// committed writer precedes the txn kills it.  Read-only txns never kill or
// block anyone, so each is decided alone once every writer is.  (Round 5 ran
// 16 lanes per txn, one access each: twice the waves for the same probes,
// ~12 us of the whole chip per headline epoch.)
__global__ __launch_bounds__(256) void k_sw_ro(SwRoArgs a) {
  const uint32_t cnt = *a.ro_count;
  const uint32_t lane = lane_id(), g = lane >> 2, sl = lane & 3u;
  const uint32_t ng = gridDim.x * 64;
  const uint32_t mask = (1u << a.wt.bits) - 1u;
  for (uint32_t i = (blockIdx.x * 256 + threadIdx.x) >> 2; i < cnt; i += ng) {
    uint4 r = *(const uint4*)&a.ro[i];  // tid, first access, end
    if (a.full_off) {  // key-sharded: the txn's accesses in the whole batch
      r.y = a.full_off[r.x];
      r.z = a.full_off[r.x + 1];
    }
    bool kill = false;
    for (uint32_t x0 = r.y + sl; x0 < r.z && !kill; x0 += 16) {
      uint64_t k[4];
      bool in[4];
#pragma unroll
      for (uint32_t u = 0; u < 4; u++) {
        in[u] = x0 + 4 * u < r.z;
        k[u] = in[u] ? a.keys[x0 + 4 * u] : KEY_EMPTY;
      }
      uint32_t sv[4];
      uint4 v[4];
#pragma unroll
      for (uint32_t u = 0; u < 4; u++) {
        sv[u] = sw_hash(k[u], a.wt.bits);
        v[u] = in[u] ? *(const uint4*)&a.wt.slot[sv[u]] : make_uint4(~0u, ~0u, ~0u, ~0u);
      }
#pragma unroll
      for (uint32_t u = 0; u < 4; u++) {
        if (!in[u]) continue;
        // the first slot was loaded above; the rest of the probe sequence
        // (rare at the table's ~10 % load) as wt_find walks it
        uint32_t q = 0, s0 = sv[u];
        for (;;) {
          const uint64_t kk = ((uint64_t)v[u].y << 32) | v[u].x;
          if (kk == k[u]) {
            kill |= v[u].z < r.x;
            break;
          }
          if (kk == KEY_EMPTY || ++q >= a.wt.probes) break;
          s0 = (s0 + 1) & mask;
          v[u] = *(const uint4*)&a.wt.slot[s0];
        }
      }
    }
    const uint64_t b = ballot64(kill);
    if (sl == 0) a.state[r.x] = ((b >> (4 * g)) & 0xFull) ? ST_ABORT : ST_COMMIT;
  }
}

// k_sw_wall: the committed writers' writes into the writer table, 16 lanes
// per txn, four txns per wave step: the txns the serial passes listed, or
// (fallback) every committed txn with a write found in the epoch's state and
// has-write bytes (64 per wave).
__device__ inline void wall_txn(const SwWallArgs& a, uint64_t tt, uint32_t sl) {
  const uint64_t s = min((uint64_t)a.off[tt], a.nnz), e = min((uint64_t)a.off[tt + 1], a.nnz);
  for (uint64_t x = s + sl; x < e; x += 16)
    if (a.acctype[x] == 1) wt_insert(a.wt, a.keys[x], (uint32_t)tt);
}
__global__ __launch_bounds__(256) void k_sw_wall(SwWallArgs a) {
  const uint32_t lane = lane_id(), g = lane >> 4, sl = lane & 15u;
  if (a.cw_list) {
    const uint32_t cnt = *a.cw_count;
    for (uint32_t i = (blockIdx.x * 256 + threadIdx.x) >> 4; i < cnt; i += gridDim.x * 16)
      wall_txn(a, a.cw_list[i], sl);
    return;
  }
  for (uint64_t t0 = ((uint64_t)blockIdx.x * 256 + threadIdx.x) & ~63ull; t0 < a.n;
       t0 += (uint64_t)gridDim.x * 256) {
    const uint64_t t = t0 + lane;
    const bool cw = t < a.n && a.state[t] == ST_COMMIT && a.hasw[t];
    uint64_t w = ballot64(cw);
    while (w) {  // uniform: up to four committed writers per step
      uint32_t pick[4];
#pragma unroll
      for (int q = 0; q < 4; q++) {
        pick[q] = w ? (uint32_t)__builtin_ctzll(w) : 64u;
        if (w) w &= w - 1;
      }
      if (pick[g] < 64) wall_txn(a, t0 + pick[g], sl);
    }
  }
}

// ---------------------------------------------------------------------------
void launch_sw_ro(const SwRoArgs& a, unsigned grid, hipStream_t st) {
  k_sw_ro<<<grid ? grid : 1u, 256, 0, st>>>(a);
}
void launch_sw_wall(const SwWallArgs& a, unsigned grid, hipStream_t st) {
  k_sw_wall<<<grid ? grid : 1u, 256, 0, st>>>(a);
}
void launch_sw_pre(const SwPreArgs& a, unsigned grid, hipStream_t st) {
  k_sw_pre<<<grid ? grid : 1u, PRE_B, 0, st>>>(a);
}
void launch_sw_seq(const SwSeqArgs& a, hipStream_t st) {
  k_sw_seq<<<1, SEQ_B, 0, st>>>(a);
}
void launch_sw_rows(const SwPreArgs& a, unsigned grid, hipStream_t st) {
  k_sw_rows<<<grid ? grid : 1u, 256, 0, st>>>(a);  // one workgroup per tile
}
void launch_sw_cout(const SwCoutArgs& a0, unsigned grid, hipStream_t st) {
  SwCoutArgs a = a0;
  a.cout_grid = grid ? grid : 1u;
  k_sw_cout<<<a.cout_grid + (a.prep_part ? SW_PREP_BLOCKS : 0u), 256, 0, st>>>(a);
}
void launch_sw_filter(const SwFilterArgs& a, unsigned grid, hipStream_t st) {
  k_sw_filter<<<grid ? grid : 1u, SW_CHUNK, 0, st>>>(a);
}
void launch_sw_share(const uint32_t* m_dev, uint32_t m_host, const uint32_t* abandon,
                     const uint32_t* off, uint32_t p_max, uint32_t rank, uint32_t* cnt,
                     hipStream_t st) {
  k_sw_share<<<1, 1, 0, st>>>(m_dev, m_host, abandon, off, p_max, rank, cnt);
}
void launch_sw_sgather(const uint32_t* tid, const uint32_t* m_dev, uint32_t p_max,
                       const uint32_t* full_off, const uint64_t* full_keys, const uint8_t* full_at,
                       uint64_t full_nnz, uint32_t* soff, uint64_t* skeys, uint8_t* sat,
                       uint32_t* err, hipStream_t st) {
  k_sw_sg_scan<<<1, SG_T, 0, st>>>(tid, m_dev, p_max, full_off, full_nnz, soff, err);
  k_sw_sg_copy<<<std::max<uint32_t>(1, std::min<uint32_t>((p_max + 15) / 16, 1024)), 256, 0, st>>>(
      tid, m_dev, p_max, full_off, full_keys, full_at, full_nnz, soff, skeys, sat);
}
void launch_sw_apply(const SwFilterArgs& a, unsigned grid, hipStream_t st) {
  k_sw_apply<<<grid ? grid : 1u, SW_CHUNK, 0, st>>>(a);
}
void launch_sw_merge(const SwList& in, uint32_t P, uint32_t* xbuf, uint32_t xoff_words,
                     uint32_t n_all, uint32_t* cnt, uint32_t* cur, uint32_t* moff,
                     uint64_t* mkeys, uint8_t* mat, bool export_only, hipStream_t st) {
  if (export_only) {
    k_sw_export<<<256, 256, 0, st>>>(in, P, xbuf + xoff_words);
    return;
  }
  const unsigned g = (unsigned)std::min<uint32_t>((n_all + 255) / 256 + 1, 2048);
  k_sw_mcount<<<g, 256, 0, st>>>(xbuf, n_all, P, cnt);
  k_sw_mscan<<<1, 1024, 0, st>>>(cnt, P, moff, cur);
  k_sw_mscatter<<<g, 256, 0, st>>>(xbuf, n_all, P, cur, mkeys, mat);
}
void launch_sw_compact(const SwFilterArgs& a, unsigned grid, hipStream_t st) {
  k_sw_compact<<<grid ? grid : 1u, SW_CHUNK, 0, st>>>(a);
}

}  // namespace dcc
