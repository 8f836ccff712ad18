// gfx950 kernels of the OCC prefix peel.
//
// Serial validation order (occ.cpp:116-239 in index order, then
// central_finish) kills every txn that touches a key written by an EARLIER
// committed txn.  At YCSB/TPC-C contention the committed write sets of a
// short prefix already cover the hot keys, so the epoch is decided as
//
//   1. solve the prefix [0, p) exactly (the round engine, occ_kernels.hip)
//   2. k_cset:    gather the committed write keys C_p of the prefix
//   3. k_filter:  one streaming pass over [p, n): a txn touching any key of
//                 C_p aborts (its committed writer j < p <= i); probes hit a
//                 per-workgroup LDS hash set of C_p
//   4. k_compact: the survivors (no key in C_p) become a dense CSR sub-batch,
//                 still in index order
//   5. solve the sub-batch; k_scatter writes its decisions back.
//
// Exactness: a killed txn never commits, so it neither kills nor blocks
// anyone; a survivor's decision depends only on earlier survivors (no prefix
// commit touches its keys, every prefix abort is inert).  Hence deciding the
// survivors in their own index order reproduces the serial replay.
#include <hip/hip_runtime.h>

#include "dcc_device.h"
#include "occ_kernels.h"

namespace dcc {

constexpr uint32_t CS_LDS_SLOTS = 8192;  // LDS set: 64 KiB of u64 keys
constexpr uint32_t CS_LDS_MAX = CS_LDS_SLOTS / 2;

__device__ inline uint32_t cs_hash(uint64_t key) { return (uint32_t)fmix64(key); }

// ---------------------------------------------------------------------------
// k_cset: committed write keys of txns [0, p) -> ckeys[0..*ccount) and the
// exact global set gset (capacity gmask+1, used when C_p outgrows LDS).
// Wave tiles of tw txns, lanes over their accesses (coalesced).
template <int WAVES>
__global__ __launch_bounds__(WAVES * 64) void k_cset(CsetArgs a) {
  __shared__ uint8_t s_map[WAVES][FILTER_CAP];
  __shared__ uint8_t s_com[WAVES][64];
  const uint32_t wv = threadIdx.x >> 6, lane = lane_id();
  uint8_t* map = s_map[wv];
  const uint64_t step = (uint64_t)gridDim.x * WAVES * a.tw;
  for (uint64_t c0 = (uint64_t)blockIdx.x * WAVES * a.tw; c0 < a.p; c0 += step) {
    const uint64_t j0 = c0 + (uint64_t)wv * a.tw;
    const uint32_t nt = j0 < a.p ? (uint32_t)min((uint64_t)a.tw, a.p - j0) : 0u;
    const bool own = lane < nt;
    uint32_t s = 0, e = 0;
    bool com = false;
    if (own) {
      s = a.off[j0 + lane];
      e = a.off[j0 + lane + 1];
      com = a.state[j0 + lane] == ST_COMMIT;
    }
    uint32_t A0 = 0, A1 = 0;
    if (nt) {
      A0 = __shfl(s, 0);
      A1 = __shfl(e, nt - 1);
    }
    const bool live = nt != 0 && A1 - A0 <= (uint32_t)FILTER_CAP;
    if (live && own)
      for (uint32_t x = s; x < e; x++) map[x - A0] = (uint8_t)lane;
    s_com[wv][lane] = com ? 1 : 0;
    __syncthreads();
    if (live) {
      for (uint32_t x = A0 + lane; x < A1; x += 64) {
        if (!s_com[wv][map[x - A0]] || a.acctype[x] != 1 /* WR */) continue;
        const uint64_t key = a.keys[x];
        // exact global set (insert-or-find); a key has one committed writer
        uint32_t h = cs_hash(key) & a.gmask;
        for (uint32_t q = 0; q <= a.gmask; q++) {
          const unsigned long long prev =
              atomicCAS((unsigned long long*)&a.gset[h], (unsigned long long)KEY_EMPTY,
                        (unsigned long long)key);
          if (prev == KEY_EMPTY) {
            a.ckeys[atomicAdd(a.ccount, 1u)] = key;
            break;
          }
          if (prev == key) break;
          h = (h + 1) & a.gmask;
        }
      }
    }
    __syncthreads();
  }
}

// ---------------------------------------------------------------------------
// Block ranges: block b owns txns [t0 + b*per_blk, t0 + (b+1)*per_blk) so the
// per-block survivor counts, scanned, give survivors their index-ordered
// positions.  Inside a block, WAVES wave-tiles of tw txns per step.
template <int WAVES>
__device__ inline void blk_range(uint64_t t0, uint64_t n, uint64_t per_blk, uint64_t& b0,
                                 uint64_t& b1) {
  b0 = t0 + (uint64_t)blockIdx.x * per_blk;
  b1 = b0 + per_blk;
  if (b0 > n) b0 = n;
  if (b1 > n) b1 = n;
}

__device__ inline uint32_t wave_excl_scan(uint32_t v, uint32_t& total) {
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

// ---------------------------------------------------------------------------
// k_filter: txns [t0, n) with state UNDECIDED and any key in C_p -> killed.
// Also has-write bytes for every txn of [0, n) it covers (blocks start at 0:
// prefix txns get hasw, never a kill).  Per-block survivor partials.
template <int WAVES>
__global__ __launch_bounds__(WAVES * 64) void k_filter(FilterArgs a) {
  __shared__ uint64_t cs[CS_LDS_SLOTS];
  __shared__ uint8_t s_map[WAVES][FILTER_CAP];
  __shared__ uint32_t s_txn[WAVES][64];
  __shared__ uint8_t s_kill[WAVES][64];
  __shared__ uint32_t s_w[WAVES][64];  // write accesses per txn
  __shared__ uint32_t s_red[WAVES][3];
  const uint32_t wv = threadIdx.x >> 6, lane = lane_id();
  const uint32_t cnt = *a.ccount;
  const bool use_lds = cnt <= CS_LDS_MAX;
  if (use_lds) {
    for (uint32_t q = threadIdx.x; q < CS_LDS_SLOTS; q += blockDim.x) cs[q] = KEY_EMPTY;
    __syncthreads();
    for (uint32_t q = threadIdx.x; q < cnt; q += blockDim.x) {
      const uint64_t key = a.ckeys[q];
      uint32_t h = cs_hash(key) & (CS_LDS_SLOTS - 1);
      while (atomicCAS((unsigned long long*)&cs[h], (unsigned long long)KEY_EMPTY,
                       (unsigned long long)key) != KEY_EMPTY)
        h = (h + 1) & (CS_LDS_SLOTS - 1);  // keys are distinct: never equal
    }
  }
  __syncthreads();
  uint64_t b0, b1;
  blk_range<WAVES>(0, a.n, a.per_blk, b0, b1);
  uint32_t st_t = 0, st_a = 0, st_w = 0;  // survivors: txns, accesses, writes
  uint8_t* map = s_map[wv];
  // every wave runs the same number of steps (uniform workgroup barriers)
  for (uint64_t c0 = b0; c0 < b1; c0 += (uint64_t)WAVES * a.tw) {
    const uint64_t j0 = c0 + (uint64_t)wv * a.tw;
    const uint32_t nt = j0 < b1 ? (uint32_t)min((uint64_t)a.tw, b1 - j0) : 0u;
    const bool own = lane < nt;
    const uint64_t i = j0 + lane;
    uint32_t s = 0, e = 0;
    uint8_t st = ST_COMMIT;
    if (own) {
      s = a.off[i];
      e = a.off[i + 1];
      st = a.state[i];
    }
    uint32_t A0 = 0, A1 = 0;
    if (nt) {
      A0 = __shfl(s, 0);
      A1 = __shfl(e, nt - 1);
    }
    bool live = nt != 0;
    if (A1 - A0 > (uint32_t)FILTER_CAP) {
      if (lane == 0) atomicOr(a.err, ERR_TILE);
      live = false;
    }
    // probing txns: undecided and past the prefix
    const bool probe = live && own && i >= a.t0 && st == ST_UNDECIDED;
    if (live && own)
      for (uint32_t x = s; x < e; x++) map[x - A0] = (uint8_t)lane;
    s_kill[wv][lane] = 0;
    s_w[wv][lane] = 0;
    s_txn[wv][lane] = probe ? 1u : 0u;
    __syncthreads();
    if (live) {
      for (uint32_t base = A0; base < A1; base += 64 * FILTER_ILP) {
        uint64_t key[FILTER_ILP];
        uint32_t lt[FILTER_ILP];
        uint8_t at[FILTER_ILP];
        // unconditional, clamped loads: branch-free code keeps all of them
        // in flight (a conditional load gets its own vmcnt(0) wait)
#pragma unroll
        for (int u = 0; u < FILTER_ILP; u++) {
          const uint32_t x = base + 64 * u + lane;
          const uint32_t xs = x < A1 ? x : A0;
          lt[u] = x < A1 ? map[x - A0] : 0xFFu;
          key[u] = a.keys[xs];
          at[u] = a.acctype[xs];
        }
#pragma unroll
        for (int u = 0; u < FILTER_ILP; u++) {
          if (lt[u] == 0xFFu) continue;
          if (at[u] == 1) atomicAdd(&s_w[wv][lt[u]], 1u);
          if (!s_txn[wv][lt[u]]) continue;
          bool hit = false;
          if (use_lds) {
            uint32_t h = cs_hash(key[u]) & (CS_LDS_SLOTS - 1);
            for (;;) {
              const uint64_t v = cs[h];
              if (v == key[u]) { hit = true; break; }
              if (v == KEY_EMPTY) break;
              h = (h + 1) & (CS_LDS_SLOTS - 1);
            }
          } else {
            uint32_t h = cs_hash(key[u]) & a.gmask;
            for (uint32_t q = 0; q <= a.gmask; q++) {
              const uint64_t v = a.gset[h];
              if (v == key[u]) { hit = true; break; }
              if (v == KEY_EMPTY) break;
              h = (h + 1) & a.gmask;
            }
          }
          if (hit) s_kill[wv][lt[u]] = 1;  // racing stores of the same byte
        }
      }
    }
    __syncthreads();
    if (live && own) {
      a.hasw[i] = s_w[wv][lane] ? 1 : 0;
      if (probe) {
        if (s_kill[wv][lane]) {
          if (a.kill) a.kill[i] = 2;
          else a.state[i] = ST_ABORT;
        } else if (!a.kill) {
          // sharded: survivors are counted after the all-reduce (k_survivors)
          st_t++;
          st_a += e - s;
          st_w += s_w[wv][lane];
        }
      }
    }
    __syncthreads();  // LDS reuse by the next step
  }
  // block partials (waves reduce, then lane 0 of wave 0 combines)
  for (int d = 32; d > 0; d >>= 1) {
    st_t += __shfl_xor(st_t, d);
    st_a += __shfl_xor(st_a, d);
    st_w += __shfl_xor(st_w, d);
  }
  if (lane == 0) {
    s_red[wv][0] = st_t;
    s_red[wv][1] = st_a;
    s_red[wv][2] = st_w;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    uint32_t t = 0, ac = 0, w = 0;
    for (int q = 0; q < WAVES; q++) {
      t += s_red[q][0];
      ac += s_red[q][1];
      w += s_red[q][2];
    }
    a.part[blockIdx.x] = SurvPart{t, ac, w, 0};
  }
}

// ---------------------------------------------------------------------------
// k_survivors (sharded): after the kill bytes were all-reduced, apply them and
// count this shard's survivors per block (same block ranges as k_filter).
template <int WAVES>
__global__ __launch_bounds__(WAVES * 64) void k_survivors(FilterArgs a) {
  __shared__ uint32_t s_red[WAVES][3];
  const uint32_t wv = threadIdx.x >> 6, lane = lane_id();
  uint64_t b0, b1;
  blk_range<WAVES>(0, a.n, a.per_blk, b0, b1);
  uint32_t st_t = 0, st_a = 0, st_w = 0;
  for (uint64_t i = b0 + threadIdx.x; i < b1; i += blockDim.x) {
    if (i < a.t0 || a.state[i] != ST_UNDECIDED) continue;
    if (a.kill[i]) {
      a.state[i] = ST_ABORT;
      a.kill[i] = 0;
      continue;
    }
    const uint32_t s = a.off[i], e = a.off[i + 1];
    st_t++;
    st_a += e - s;
    for (uint32_t x = s; x < e; x++) st_w += a.acctype[x] == 1;
  }
  for (int d = 32; d > 0; d >>= 1) {
    st_t += __shfl_xor(st_t, d);
    st_a += __shfl_xor(st_a, d);
    st_w += __shfl_xor(st_w, d);
  }
  if (lane == 0) {
    s_red[wv][0] = st_t;
    s_red[wv][1] = st_a;
    s_red[wv][2] = st_w;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    uint32_t t = 0, ac = 0, w = 0;
    for (int q = 0; q < WAVES; q++) {
      t += s_red[q][0];
      ac += s_red[q][1];
      w += s_red[q][2];
    }
    a.part[blockIdx.x] = SurvPart{t, ac, w, 0};
  }
}

// ---------------------------------------------------------------------------
// k_surv_scan: exclusive scan of the per-block partials (one workgroup);
// totals go to tot[0..2] and the sub-batch's closing offset.
__global__ __launch_bounds__(1024) void k_surv_scan(SurvPart* part, uint32_t nb, uint32_t* tot,
                                                    uint32_t* sub_off) {
  __shared__ uint32_t sw[16][2];
  __shared__ unsigned long long s_w64[16];
  __shared__ uint32_t carry[3];
  const uint32_t lane = lane_id(), wv = threadIdx.x >> 6;
  if (threadIdx.x == 0) carry[0] = carry[1] = carry[2] = 0;
  __syncthreads();
  for (uint32_t c0 = 0; c0 < nb; c0 += 1024) {
    const uint32_t q = c0 + threadIdx.x;
    const SurvPart v = q < nb ? part[q] : SurvPart{0, 0, 0, 0};
    uint32_t tt, ta;
    const uint32_t et = wave_excl_scan(v.t, tt);
    const uint32_t ea = wave_excl_scan(v.a, ta);
    unsigned long long w = v.w;
    for (int d = 32; d > 0; d >>= 1) w += __shfl_xor(w, d);
    if (lane == 0) {
      sw[wv][0] = tt;
      sw[wv][1] = ta;
      s_w64[wv] = w;
    }
    __syncthreads();
    uint32_t bt = carry[0], ba = carry[1];
    for (uint32_t k = 0; k < wv; k++) {
      bt += sw[k][0];
      ba += sw[k][1];
    }
    if (q < nb) part[q] = SurvPart{bt + et, ba + ea, v.w, 0};
    __syncthreads();
    if (threadIdx.x == 0) {
      for (uint32_t k = 0; k < 16; k++) {
        carry[0] += sw[k][0];
        carry[1] += sw[k][1];
        carry[2] += (uint32_t)s_w64[k];
        sw[k][0] = sw[k][1] = 0;
        s_w64[k] = 0;
      }
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    tot[0] = carry[0];
    tot[1] = carry[1];
    tot[2] = carry[2];
    sub_off[carry[0]] = carry[1];
  }
}

// ---------------------------------------------------------------------------
// k_compact: survivors of each block, in index order, into the sub-batch
// (tid, offsets, keys, acctype).  Same block ranges as k_filter.
template <int WAVES>
__global__ __launch_bounds__(WAVES * 64) void k_compact(CompactArgs a) {
  __shared__ uint32_t s_cnt[WAVES][2];
  __shared__ uint32_t s_dst[WAVES][64], s_src[WAVES][64];
  const uint32_t wv = threadIdx.x >> 6, lane = lane_id();
  uint64_t b0, b1;
  blk_range<WAVES>(0, a.n, a.per_blk, b0, b1);
  const SurvPart base = a.part[blockIdx.x];
  uint32_t run_t = base.t, run_a = base.a;
  const uint64_t step = (uint64_t)WAVES * 64;
  for (uint64_t c0 = b0; c0 < b1; c0 += step) {
    const uint64_t i = c0 + (uint64_t)wv * 64 + lane;
    bool sv = false;
    uint32_t s = 0, len = 0;
    if (i < b1 && i >= a.t0 && a.state[i] == ST_UNDECIDED) {
      sv = true;
      s = a.off[i];
      len = a.off[i + 1] - s;
    }
    uint32_t tt, ta;
    const uint32_t et = wave_excl_scan(sv ? 1u : 0u, tt);
    const uint32_t ea = wave_excl_scan(len, ta);
    if (lane == 0) {
      s_cnt[wv][0] = tt;
      s_cnt[wv][1] = ta;
    }
    __syncthreads();
    uint32_t bt = run_t, ba = run_a;
    for (uint32_t k = 0; k < wv; k++) {
      bt += s_cnt[k][0];
      ba += s_cnt[k][1];
    }
    if (sv) {
      a.sub_tid[bt + et] = (uint32_t)i;
      a.sub_off[bt + et] = ba + ea;
    }
    // copy the wave's survivor accesses: one survivor at a time, lanes over
    // its accesses (<= 64 per txn, MAX_ROW_PER_TXN)
    const uint64_t sm = ballot64(sv);
    s_dst[wv][lane] = ba + ea;
    s_src[wv][lane] = s;
    __syncthreads();
    uint64_t rem = sm;
    while (rem) {
      const uint32_t l = (uint32_t)__builtin_ctzll(rem);
      rem &= rem - 1;
      const uint32_t ln = __shfl(len, l);
      const uint32_t src = s_src[wv][l], dst = s_dst[wv][l];
      if (lane < ln) {
        a.sub_keys[dst + lane] = a.keys[src + lane];
        a.sub_acctype[dst + lane] = a.acctype[src + lane];
      }
    }
    __syncthreads();
    for (uint32_t k = 0; k < WAVES; k++) {
      run_t += s_cnt[k][0];
      run_a += s_cnt[k][1];
    }
    __syncthreads();
  }
}

// ---------------------------------------------------------------------------
// k_scatter: sub-batch decisions back to the epoch's state bytes.
__global__ __launch_bounds__(256) void k_scatter(const uint8_t* __restrict__ sub_state,
                                                 const uint32_t* __restrict__ sub_tid,
                                                 const uint32_t* __restrict__ n_sub,
                                                 uint8_t* __restrict__ state) {
  const uint32_t m = *n_sub;
  for (uint32_t j = blockIdx.x * blockDim.x + threadIdx.x; j < m; j += gridDim.x * blockDim.x) {
    const uint8_t s = sub_state[j];
    state[sub_tid[j]] = s == ST_COMMIT ? ST_COMMIT : s == ST_UNDECIDED ? ST_UNDECIDED : ST_ABORT;
  }
}

// ---------------------------------------------------------------------------
void launch_cset(const CsetArgs& a, hipStream_t st) {
  const uint64_t per = (uint64_t)4 * a.tw;
  uint64_t g = (a.p + per - 1) / per;
  if (g > 1024) g = 1024;
  k_cset<4><<<g ? (unsigned)g : 1u, 256, 0, st>>>(a);
}
void launch_filter(const FilterArgs& a, unsigned grid, hipStream_t st) {
  k_filter<FILTER_WAVES><<<grid, FILTER_WAVES * 64, 0, st>>>(a);
}
void launch_survivors(const FilterArgs& a, unsigned grid, hipStream_t st) {
  k_survivors<FILTER_WAVES><<<grid, FILTER_WAVES * 64, 0, st>>>(a);
}
void launch_surv_scan(SurvPart* part, uint32_t nb, uint32_t* tot, uint32_t* sub_off,
                      hipStream_t st) {
  k_surv_scan<<<1, 1024, 0, st>>>(part, nb, tot, sub_off);
}
void launch_compact(const CompactArgs& a, unsigned grid, hipStream_t st) {
  k_compact<FILTER_WAVES><<<grid, FILTER_WAVES * 64, 0, st>>>(a);
}
void launch_scatter(const uint8_t* sub_state, const uint32_t* sub_tid, const uint32_t* n_sub,
                    uint64_t m_bound, uint8_t* state, hipStream_t st) {
  unsigned g = (unsigned)((m_bound + 255) / 256);
  if (g > 1024) g = 1024;
  k_scatter<<<g ? g : 1, 256, 0, st>>>(sub_state, sub_tid, n_sub, state);
}

}  // namespace dcc
