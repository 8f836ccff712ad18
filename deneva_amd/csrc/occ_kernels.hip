// gfx950 kernels of the batched OCC validator.
//
// Semantics (parity target): validating every txn of an epoch in index order
// with OptCC::central_validate (concurrency_control/occ.cpp:116-239) and then
// finishing all of them (central_finish, occ.cpp:248-294) decides
//
//   abort(i)  <=>  hist(i)  OR  exists j < i: commit(j) AND W_j ∩ (R_i ∪ W_i) != {}
//
// (active entries are checked against R then W, occ.cpp:185-199; read-only and
// aborted txns never sit in `active`, occ.cpp:151-154 / 219-235; hist(i) is the
// history window check of occ.cpp:160-180).  Every key has at most one
// committed writer, so a key is "resolved" as soon as its minimum non-aborted
// writer commits.  The kernels compute the unique fixed point in rounds:
//
//   k_build          insert every write key, own[1] = min writer     (round 1 owners)
//   k_round<KEYS>    round r over a CSR list of undecided txns:
//                      per access: own[r&1] -> KILLED (committed writer < i)
//                                              BLOCKED (undecided writer < i)
//                      per txn:    KILLED -> Abort, clear -> Commit (+ publish
//                                  tag-0 words), BLOCKED -> next list; its
//                                  writes publish round r+1 owners into own[(r+1)&1]
//   k_final          RC bytes, counts, commit tn (central_finish's tnc++).
//
// Tile = one wave owns up to `tw` consecutive list txns (one per lane) whose
// accesses (<= 1024) are staged through LDS; per-access lanes are coalesced
// and the per-txn reduction is a ballot segmented OR (no per-lane LDS atomics).
#include <hip/hip_runtime.h>

#include <algorithm>

#include "dcc_device.h"
#include "dcc_env.h"
#include "occ_kernels.h"
#include "prep_body.h"

namespace dcc {

// --------------------------------------------------------------------------
// k_prep: offset validation, max txn length and write count (prep_body.h).
__global__ __launch_bounds__(256) void k_prep(const uint32_t* __restrict__ off, uint64_t n,
                                              const uint8_t* __restrict__ at, uint64_t nnz,
                                              uint64_t p, PrepPart* __restrict__ part) {
  prep_body(off, n, at, nnz, p, part, blockIdx.x, gridDim.x);
}

// --------------------------------------------------------------------------
// k_hist: the history window check (occ.cpp:160-180): if finish_tn > start_tn,
// txn i aborts when a committed history entry with start_tn < tn <= finish_tn
// wrote a key i READ (history is checked against the read set only).  The
// history is the device's base + delta levels (occ_history.h).  A workgroup
// holds the history's key bitmap in LDS; a wave takes 64 txns and walks their
// contiguous accesses 64 at a time (coalesced key and type loads, one access
// per lane), finding each access's txn in the wave's LDS offset prefix; only a
// read whose key bit is set probes the levels, and a hit marks its txn
// aborted (every writer stores the same byte).  Offsets are clamped to nnz
// and made monotone; a malformed batch is reported.
constexpr uint32_t HIST_WAVES = 16;
constexpr uint32_t HIST_U = 2;  // accesses per lane in flight
constexpr uint32_t HIST_MAP = 2048;  // accesses per wave with an LDS access -> txn map
__global__ __launch_bounds__(HIST_WAVES * 64, 8) void k_hist(HistArgs a) {
  __shared__ uint32_t s_bm[(1u << HIST_BM_LOG) / 32];
  __shared__ uint32_t s_o[HIST_WAVES][65];
  __shared__ uint64_t s_lo[HIST_WAVES][64], s_hi[HIST_WAVES][64];
  __shared__ uint8_t s_live[HIST_WAVES][64];  // window open and not yet found aborted
  __shared__ uint8_t s_map[HIST_WAVES][HIST_MAP];  // access - a0 -> the wave's txn
  const HistView hv = a.dyn->view;  // by value: registers, not a reload per probe
  for (uint32_t i = threadIdx.x; i < (1u << HIST_BM_LOG) / 32; i += HIST_WAVES * 64)
    s_bm[i] = hv.bm ? hv.bm[i] : ~0u;
  __syncthreads();
  const uint32_t lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  // a resident grid: each wave takes 64-txn tiles in turn (the bitmap loaded
  // once per workgroup, not once per 1,024 txns)
  for (uint64_t t0 = ((uint64_t)blockIdx.x * HIST_WAVES + w) * 64; t0 < a.n;
       t0 += (uint64_t)gridDim.x * HIST_WAVES * 64) {
  const uint32_t nt = (uint32_t)min<uint64_t>(64, a.n - t0);
  const uint64_t t = t0 + lane;
  uint64_t lo = 0, hi = 0;
  if (lane < nt) {
    lo = a.start_tn[t];
    hi = a.finish_tn[t];
    const uint32_t o0 = a.off[t], o1 = a.off[t + 1];
    if (o1 < o0 || o1 - o0 > MAX_TXN_LEN) atomicOr(a.err, ERR_OFFSETS);
  }
  s_lo[w][lane] = lo;
  s_hi[w][lane] = hi;
  s_live[w][lane] = lane < nt && hi > lo;
  uint32_t ov = lane <= nt ? (uint32_t)min<uint64_t>(a.off[t0 + lane], a.nnz) : 0u;
  for (int d = 1; d < 64; d <<= 1) {
    const uint32_t y = __shfl_up(ov, d);
    if (lane >= (uint32_t)d && lane <= nt) ov = max(ov, y);
  }
  s_o[w][lane] = ov;
  __builtin_amdgcn_wave_barrier();
  if (lane == 0) s_o[w][64] = nt == 64 ? max(s_o[w][63], (uint32_t)min<uint64_t>(a.off[t0 + 64], a.nnz)) : 0u;
  __builtin_amdgcn_wave_barrier();
  // no txn of the wave has an open window: nothing to check
  if (!ballot64(lane < nt && hi > lo)) continue;
  const uint32_t a0 = s_o[w][0], a1 = s_o[w][nt];
  // each access's txn: from the LDS map when the wave's accesses fit, else a
  // binary search of the offsets
  const bool mapped = a1 - a0 <= HIST_MAP;
  if (mapped && lane < nt) {
    for (uint32_t x = s_o[w][lane]; x < s_o[w][lane + 1]; x++) s_map[w][x - a0] = (uint8_t)lane;
  }
  __builtin_amdgcn_wave_barrier();
  for (uint32_t x0 = a0; x0 < a1; x0 += 64 * HIST_U) {
    uint64_t key[HIST_U];
    uint8_t ty[HIST_U];
#pragma unroll
    for (uint32_t u = 0; u < HIST_U; u++) {  // every load of the step issued before any use
      const uint32_t x = min(x0 + 64 * u + lane, a1 - 1);
      // streamed once: non-temporal, so the batch does not evict the tables from L2
      key[u] = __builtin_nontemporal_load(a.keys + x);
      ty[u] = __builtin_nontemporal_load(a.acctype + x);
    }
    uint32_t txn[HIST_U];
    bool want[HIST_U];
#pragma unroll
    for (uint32_t u = 0; u < HIST_U; u++) {
      const uint32_t x = x0 + 64 * u + lane;
      const uint32_t b = hist_bm_bit(key[u]);
      want[u] = x < a1 && ty[u] != 1 /* WR */ && ((a.var & 2u) || ((s_bm[b >> 5] >> (b & 31u)) & 1u));
      txn[u] = 0;
      if (a.var & 1u) want[u] = false;
      if (want[u] && !(a.var & 4u)) {
        uint32_t l = 0;
        if (mapped) {
          l = s_map[w][x - a0];
        } else {
          uint32_t h = nt;  // largest k < nt with s_o[k] <= x
          while (h - l > 1) {
            const uint32_t mid = (l + h) >> 1;
            if (s_o[w][mid] <= x) l = mid;
            else h = mid;
          }
        }
        txn[u] = l;
        want[u] = s_live[w][l] != 0;
      }
    }
    // level by level, the U probes of a lane in lockstep: every home slot
    // loaded together, then each round of the collision walks (linear
    // probing) loaded together, until no lane of the wave has a walk left --
    // a step costs the longest walk's round trips, not the sum of them
#pragma unroll
    for (int q = 1; q >= 0; q--) {
      const HistLevel& L = hv.lv[q];
      if (!L.on) continue;
      const uint64_t mask = (1ull << L.hbits) - 1;
      uint64_t slot[HIST_U];
      HistSlot S[HIST_U];
#pragma unroll
      for (uint32_t u = 0; u < HIST_U; u++) {
        slot[u] = hist_hash_slot(key[u], L.hbits);
        S[u] = want[u] ? hist_slot_ld(L.hash, slot[u]) : HistSlot{DCC_KEY_RESERVED, 0};
      }
      // every key sits within HIST_WALK of its home (occ_history.h)
      for (uint32_t it = 1; it < HIST_WALK; it++) {
        uint32_t walk = 0;
#pragma unroll
        for (uint32_t u = 0; u < HIST_U; u++)
          walk |= (want[u] && S[u].key != key[u] && S[u].key != DCC_KEY_RESERVED) ? 1u << u : 0u;
        if (!ballot64(walk != 0) || (a.var & 8u)) break;
#pragma unroll
        for (uint32_t u = 0; u < HIST_U; u++) {
          if ((walk >> u) & 1u) {
            slot[u] = (slot[u] + 1) & mask;
            S[u] = hist_slot_ld(L.hash, slot[u]);
          }
        }
      }
#pragma unroll
      for (uint32_t u = 0; u < HIST_U; u++) {
        if (!want[u] || S[u].key != key[u]) continue;
        const uint32_t l = txn[u];
        if (hist_found_hit(L, slot[u], ~S[u].ntmax, s_lo[w][l], s_hi[w][l])) {
          a.state[t0 + l] = ST_ABORT;
          s_live[w][l] = 0;
          want[u] = false;  // decided: the other level need not be probed
        }
      }
    }
  }
  __builtin_amdgcn_wave_barrier();  // the tile's LDS rows are reused by the next
  }
}

// --------------------------------------------------------------------------
// Shared tile prologue: lane l < tw owns list txn j0 + l; map[] gives the
// local txn of every staged access (0xFF = not participating).
struct Tile {
  uint32_t nt;     // txns in this wave
  uint32_t A0, A1; // access range
};

template <int CAP>
__device__ inline bool tile_open(uint64_t j0, uint32_t tw, uint64_t m, const uint32_t* tid,
                                 const uint32_t* coff, uint32_t end_total, bool part_in,
                                 uint8_t* map, uint32_t* txnL, Tile& T, uint32_t& txn,
                                 uint32_t& s, uint32_t& e, uint32_t* err) {
  const uint32_t lane = lane_id();
  if (j0 >= m) return false;
  T.nt = (uint32_t)min((uint64_t)tw, m - j0);
  const bool own = lane < T.nt;
  const uint64_t j = j0 + lane;
  txn = 0;
  s = e = 0;
  if (own) {
    txn = tid ? tid[j] : (uint32_t)j;
    s = coff[j];
    // identity lists (tid == nullptr) index the batch CSR, which has m+1 offsets
    e = (j + 1 < m || tid == nullptr) ? coff[j + 1] : end_total;
  }
  T.A0 = __shfl(s, 0);
  T.A1 = __shfl(e, T.nt - 1);
  if (T.A1 - T.A0 > (uint32_t)CAP) {
    if (lane == 0) atomicOr(err, ERR_TILE);
    return false;
  }
  if (own) {
    const uint8_t tag = part_in ? (uint8_t)lane : (uint8_t)0xFF;
    for (uint32_t x = s; x < e; x++) map[x - T.A0] = tag;
    txnL[lane] = txn;
  }
  return true;
}

// 16-byte slot read: key and owner word in one load.
struct SlotV {
  uint64_t key;
  uint32_t own;
};
__device__ inline SlotV ld_slot(const Slot* p) {
  const uint4 v = *reinterpret_cast<const uint4*>(p);
  return SlotV{((uint64_t)v.y << 32) | v.x, v.z};
}

// List geometry of a round.  Round 1 reads the batch CSR (one segment,
// identity txn ids); later rounds read the NSEG segments written by the
// previous round, whose sizes sit in its device counters (so the host can
// enqueue rounds without synchronising).  A workgroup-tile never straddles
// two segments.
struct ListGeo {
  uint64_t pre[NSEG + 1];  // prefix of workgroup-tiles per segment
  uint64_t m[NSEG];
  uint32_t end[NSEG];
  uint32_t nseg;
};

__device__ inline void list_geo(const unsigned long long* m_in, uint64_t m_host, uint32_t end_host,
                                uint64_t per_wg, ListGeo& G) {
  G.pre[0] = 0;
  if (!m_in) {
    G.nseg = 1;
    G.m[0] = m_host;
    G.end[0] = end_host;
    G.pre[1] = (m_host + per_wg - 1) / per_wg;
    return;
  }
  G.nseg = NSEG;
#pragma unroll
  for (uint32_t q = 0; q < NSEG; q++) {
    const unsigned long long c = m_in[q];
    G.m[q] = c >> CTR_E_BITS;
    G.end[q] = (uint32_t)(c & CTR_E_MASK);
    G.pre[q + 1] = G.pre[q] + (G.m[q] + per_wg - 1) / per_wg;
  }
}

__device__ inline uint32_t geo_seg(const ListGeo& G, uint64_t g) {
  uint32_t q = 0;
  while (q + 1 < G.nseg && g >= G.pre[q + 1]) q++;
  return q;
}

constexpr int ILP = 4;  // 64-access steps in flight per wave

// --------------------------------------------------------------------------
// Software grid barrier for a fully resident grid (host sizes the grid well
// under the co-residency limit).  Release/acquire recipe of the CDNA guide
// (§6 Guideline 16): every storing wave drains, one lane releases and
// arrives on a device-scope counter, the last arriver flips the generation
// word; waiters poll it relaxed with s_sleep and acquire once.  Spins are
// bounded: on timeout the flag is raised and the host fails the call.
struct GridBar {
  unsigned count;
  unsigned gen;
  unsigned timeout;
  unsigned pad;
};

__device__ inline void grid_barrier(GridBar* b) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const unsigned a = __hip_atomic_fetch_add(&b->count, 1u, __ATOMIC_RELAXED,
                                              __HIP_MEMORY_SCOPE_AGENT);
    if (a == gridDim.x - 1) {
      __hip_atomic_store(&b->gen, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    } else {
      const uint64_t t0 = spin_clock();
      while (__hip_atomic_load(&b->gen, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == 0u) {
        __builtin_amdgcn_s_sleep(2);
        if (spin_clock() - t0 > SPIN_TICKS / 10) {  // 2 s: a resident grid meets in microseconds
          __hip_atomic_store(&b->timeout, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          break;
        }
      }
    }
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  __syncthreads();
}

// --------------------------------------------------------------------------
// k_build: insert write keys, round-1 owners (min writer), has-write flag.
template <int CAP, int WAVES>
__global__ __launch_bounds__(WAVES * 64) void k_build(BuildArgs a) {
  __shared__ uint8_t s_map[WAVES][CAP];
  __shared__ uint32_t s_txn[WAVES][64];
  __shared__ uint32_t s_stat[WAVES][64];
  const uint32_t wv = threadIdx.x >> 6, lane = lane_id();
  uint8_t* map = s_map[wv];
  const uint32_t tag1 = own_word(round_tag(1), 0);
  for (uint64_t tile = blockIdx.x; tile * WAVES * a.tw < a.n; tile += gridDim.x) {
    const uint64_t j0 = (tile * WAVES + wv) * a.tw;
    Tile T;
    uint32_t txn, s, e;
    bool part = true;
    if (lane < a.tw && j0 + lane < a.n) part = a.state[j0 + lane] == ST_UNDECIDED;
    const bool live = tile_open<CAP>(j0, a.tw, a.n, nullptr, a.off, 0, part, map, s_txn[wv], T,
                                     txn, s, e, a.err);
    s_stat[wv][lane] = 0;
    __syncthreads();
    if (live) {
      for (uint32_t base = T.A0; base < T.A1; base += 64 * ILP) {
        uint32_t lt[ILP];
        bool w[ILP];
        uint64_t key[ILP];
        // unconditional, clamped loads: branch-free code keeps every load of
        // the step in flight (a conditional load gets its own vmcnt(0) wait)
#pragma unroll
        for (int u = 0; u < ILP; u++) {
          const uint32_t x = base + 64 * u + lane;
          const uint32_t xs = x < T.A1 ? x : T.A0;
          lt[u] = x < T.A1 ? map[x - T.A0] : 0xFFu;
          const uint8_t at = a.acctype[xs];
          key[u] = a.keys[xs];
          w[u] = lt[u] != 0xFFu && at == 1 /* WR */;
        }
#pragma unroll
        for (int u = 0; u < ILP; u++) {
          if (w[u]) {
            if (key[u] == KEY_EMPTY) {
              atomicOr(a.err, ERR_KEY);
            } else {
              const uint32_t sid = table_insert(a.tab, a.mask, key[u]);
              if (sid == SID_NONE) atomicOr(a.err, ERR_FULL);
              else own_min(&a.tab[sid].own, tag1 | s_txn[wv][lt[u]]);
            }
          }
          bool head;
          const uint32_t v = segment_or2(lt[u], w[u] ? 1u : 0u, head);
          if (head && lt[u] != 0xFFu && v) atomicOr(&s_stat[wv][lt[u]], v);
        }
      }
    }
    __syncthreads();
    if (live && lane < T.nt) a.hasw[j0 + lane] = s_stat[wv][lane] ? 1 : 0;
  }
}

// --------------------------------------------------------------------------
// k_round: one fixed-point round over a CSR list of undecided txns.
//
// Per access (list entry):
//   round 1       find the key's slot; owner word -> blocked/killed/clear
//   entry with B  state[blocker]: COMMIT -> killed, UNDECIDED -> still blocked,
//                 ABORT -> re-read the owner word (published for this round)
//   write entry   clear (a clear access stays clear: writers are only ever
//                 decided, never added) — kept only to publish owners
// Per txn: killed -> Abort, clear -> Commit (+ tag-0 owner words), blocked ->
// next list (entries that were blocked or are writes).
//
// SHARD (key-sharded across GPUs): the shard sees only its
// keys, so it cannot decide.  It reports the txn's local status into gst
// (killed dominates blocked), keeps every txn it did not kill in the next
// list, and publishes nothing; the host all-reduces gst (MAX) and k_decide
// applies the verdict, identical on every shard.
template <bool FROM_KEYS, bool SHARD, int CAP, int WAVES>
__global__ __launch_bounds__(WAVES * 64) void k_round(RoundArgs a) {
  __shared__ uint8_t s_map[WAVES][CAP];
  __shared__ uint64_t s_ent[WAVES][CAP];
  __shared__ uint32_t s_txn[WAVES][64];
  __shared__ uint32_t s_stat[WAVES][64];
  __shared__ uint32_t s_opos[WAVES][64];
  __shared__ uint32_t s_wt[WAVES], s_we[WAVES], s_wk[WAVES];
  __shared__ unsigned long long s_base;
  __shared__ ListGeo G;  // in LDS: runtime-indexed register arrays go to scratch
  __shared__ TileOut s_rec[RECHECK_TILES];
  __shared__ uint32_t s_nrec;

  const uint32_t wv = threadIdx.x >> 6, lane = lane_id();
  uint8_t* map = s_map[wv];
  uint64_t* ent = s_ent[wv];
  if (threadIdx.x == 0) s_nrec = 0;
  const uint32_t tag_r = round_tag(a.r);
  const uint8_t cur_abort = st_abort(a.k);
  const uint64_t per_wg = (uint64_t)WAVES * a.tw;
  if (threadIdx.x == 0) list_geo(a.m_in, a.m, a.end_total, per_wg, G);
  if (blockIdx.x == 0 && threadIdx.x < NSEG) a.ctr_zero[threadIdx.x] = 0ull;
  if (blockIdx.x == 0 && threadIdx.x == 0) *a.kill_zero = 0u;
  if (blockIdx.x == 0 && threadIdx.x < 4 && a.bar_zero) a.bar_zero[threadIdx.x] = 0u;
  __syncthreads();

  for (uint64_t tile = blockIdx.x; tile < G.pre[G.nseg]; tile += gridDim.x) {
    const uint32_t sg = geo_seg(G, tile);
    const uint64_t m = G.m[sg];
    const uint32_t* tid_s = a.tid ? a.tid + sg * a.seg_ts : nullptr;
    const uint32_t* coff_s = a.m_in ? a.coff + sg * a.seg_ts : a.coff;
    const uint64_t* cent_s = a.cent ? a.cent + sg * a.seg_es : nullptr;
    const uint64_t j0 = (tile - G.pre[sg]) * per_wg + (uint64_t)wv * a.tw;
    // output segment of this workgroup-tile
    const uint32_t og = (uint32_t)(tile % NSEG);
    uint32_t* tid_o = a.tid_out + og * a.seg_ts;
    uint32_t* coff_o = a.coff_out + og * a.seg_ts;
    uint64_t* cent_o = a.cent_out + og * a.seg_es;
    Tile T;
    uint32_t txn, s, e;
    bool part = true;
    if (lane < a.tw && j0 + lane < m)  // txns killed by the previous round's recheck are skipped
      part = a.state[tid_s ? tid_s[j0 + lane] : (uint32_t)(j0 + lane)] == ST_UNDECIDED;
    const bool live = tile_open<CAP>(j0, a.tw, m, tid_s, coff_s, G.end[sg], part, map,
                                     s_txn[wv], T, txn, s, e, a.err);
    s_stat[wv][lane] = 0;
    __syncthreads();

    // ---- phase 1: resolve every access of the tile (coalesced, ILP steps)
    if (live) {
      for (uint32_t base = T.A0; base < T.A1; base += 64 * ILP) {
        uint32_t lt[ILP], lo[ILP], blk[ILP], ps[ILP];
#pragma unroll
        for (int u = 0; u < ILP; u++) {
          const uint32_t x = base + 64 * u + lane;
          lt[u] = x < T.A1 ? map[x - T.A0] : 0xFFu;
        }
        if (FROM_KEYS) {
          uint64_t key[ILP];
          bool w[ILP];
          uint32_t h[ILP], stp[ILP];
          SlotV sv[ILP];
#pragma unroll
          for (int u = 0; u < ILP; u++) {
            const uint32_t x = base + 64 * u + lane;
            const uint32_t xs = x < T.A1 ? x : T.A0;  // clamped: branch-free loads
            const uint64_t k = a.keys[xs];
            const uint8_t at = a.acctype[xs];
            key[u] = lt[u] != 0xFFu ? k : KEY_EMPTY;
            w[u] = lt[u] != 0xFFu && at == 1 /* WR */;
          }
#pragma unroll
          for (int u = 0; u < ILP; u++) {
            h[u] = slot_home(key[u], a.mask);
            sv[u] = ld_slot(&a.tab[h[u]]);  // unconditional: all probes in flight
          }
#pragma unroll
          for (int u = 0; u < ILP; u++) {
            lo[u] = SID_NONE;
            blk[u] = 0;
            ps[u] = 0;
            if (lt[u] != 0xFFu) {
              if (key[u] == KEY_EMPTY) atomicOr(a.err, ERR_KEY);
              stp[u] = slot_step(key[u], a.mask);
              // double hashing; the home probe was issued above
              for (uint32_t q = 0; q <= a.mask; q++) {
                if (sv[u].key == key[u]) {
                  lo[u] = h[u];
                  ps[u] = own_status(sv[u].own, tag_r, s_txn[wv][lt[u]]);
                  blk[u] = own_idx(sv[u].own);
                  break;
                }
                if (sv[u].key == KEY_EMPTY) break;
                h[u] = (h[u] + stp[u]) & a.mask;
                sv[u] = ld_slot(&a.tab[h[u]]);
              }
              lo[u] |= w[u] ? ENT_WRITE : 0u;
            }
          }
        } else {
          uint64_t en[ILP];
          uint8_t bs[ILP];
          // clamped, unconditional loads (branch-free: all in flight together)
#pragma unroll
          for (int u = 0; u < ILP; u++) {
            const uint32_t x = base + 64 * u + lane;
            const uint64_t e = cent_s[x < T.A1 ? x : T.A0];
            en[u] = lt[u] != 0xFFu ? e : (uint64_t)SID_NONE;
          }
#pragma unroll
          for (int u = 0; u < ILP; u++) {
            lo[u] = (uint32_t)en[u];
            blk[u] = (uint32_t)(en[u] >> 32);
            const uint8_t b = a.state[(lo[u] & ENT_BLOCK) ? blk[u] : 0u];
            bs[u] = (lo[u] & ENT_BLOCK) ? b : ST_COMMIT;
          }
          uint32_t ow[ILP];
          bool need[ILP];
#pragma unroll
          for (int u = 0; u < ILP; u++) {
            // only an access whose blocker aborted in an EARLIER round needs
            // the owner word (republished by k_pub since); an abort of this
            // round keeps blocking until the next one
            need[u] = (lo[u] & ENT_BLOCK) && bs[u] >= ST_ABORT && bs[u] != cur_abort;
            const uint32_t o = a.tab[need[u] ? (lo[u] & ENT_SID) : 0u].own;
            ow[u] = need[u] ? o : OWN_EMPTY;
          }
#pragma unroll
          for (int u = 0; u < ILP; u++) {
            ps[u] = 0;
            if (lo[u] & ENT_BLOCK) {
              if (bs[u] == ST_COMMIT) {
                ps[u] = PS_KILLED;
              } else if (need[u]) {
                ps[u] = own_status(ow[u], tag_r, s_txn[wv][lt[u]]);
                blk[u] = own_idx(ow[u]);
              } else {
                ps[u] = PS_BLOCKED;  // undecided, or aborted this very round
              }
            }
            lo[u] &= ~ENT_BLOCK;
          }
        }
#pragma unroll
        for (int u = 0; u < ILP; u++) {
          const uint32_t x = base + 64 * u + lane;
          if (ps[u] & PS_BLOCKED) lo[u] |= ENT_BLOCK;
          if (x < T.A1) ent[x - T.A0] = ((uint64_t)blk[u] << 32) | lo[u];
          bool head;
          uint32_t v;
          if (SHARD) {
            const bool wk = (lo[u] & ENT_WRITE) && (lo[u] & ENT_SID) != SID_NONE;
            v = segment_or<3>(lt[u], ps[u] | (wk ? PS_WRITE : 0u), head);
          } else {
            v = segment_or2(lt[u], ps[u], head);
          }
          if (head && lt[u] != 0xFFu && v) atomicOr(&s_stat[wv][lt[u]], v);
        }
      }
    }
    __syncthreads();

    // ---- phase 2: per-txn decision (lane = txn)
    uint32_t dec = 0;  // 0 none, 1 commit, 2 abort, 3 blocked
    if (live && lane < T.nt && part) {
      const uint32_t st = s_stat[wv][lane];
      if (SHARD) {
        // keep what can still matter here: a blocked txn (its blocked
        // entries) or a clear one with a local write (its owner words); a
        // clear read-only txn reports 0 on this shard from now on
        dec = (st & PS_KILLED) ? 2u : (st & (PS_BLOCKED | PS_WRITE)) ? 3u : 0u;
        const uint8_t v = (st & PS_KILLED) ? 2 : (st & PS_BLOCKED) ? 1 : 0;
        if (v) a.gst[txn] = v;
      } else {
        dec = (st & PS_KILLED) ? 2u : (st & PS_BLOCKED) ? 3u : 1u;
        if (dec != 3u) a.state[txn] = dec == 1u ? ST_COMMIT : cur_abort;
      }
    }
    if (live) s_stat[wv][lane] = dec;
    __syncthreads();

    // ---- phase 3: count kept entries in access order; record each blocked
    // txn's output start.  Kept: txn blocked, slot known, and the access is a
    // write (feeds owner words) or is blocked.
    uint32_t wave_e = 0;
    if (live) {
      for (uint32_t base = T.A0; base < T.A1; base += 64) {
        const uint32_t x = base + lane;
        const bool act = x < T.A1;
        const uint32_t lt = act ? map[x - T.A0] : 0xFFu;
        const uint32_t lo = act ? (uint32_t)ent[x - T.A0] : SID_NONE;
        const bool keep = lt != 0xFFu && s_stat[wv][lt] == 3u && (lo & ENT_SID) != SID_NONE &&
                          (lo & (ENT_WRITE | ENT_BLOCK));
        const uint64_t km = ballot64(keep);
        const uint32_t below = (uint32_t)__builtin_popcountll(km & ((1ull << lane) - 1ull));
        const bool first = act && lt != 0xFFu && (x == T.A0 || map[x - 1 - T.A0] != lt);
        if (first) s_opos[wv][lt] = wave_e + below;
        wave_e += (uint32_t)__builtin_popcountll(km);
      }
    }
    const uint64_t bm = ballot64(live && lane < T.nt && dec == 3u);
    const uint32_t wave_t = (uint32_t)__builtin_popcountll(bm);
    const uint32_t wave_k = (uint32_t)__builtin_popcountll(ballot64(live && lane < T.nt && dec == 2u));
    if (lane == 0) {
      s_wt[wv] = wave_t;
      s_we[wv] = wave_e;
      s_wk[wv] = wave_k;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
      unsigned long long tt = 0, te = 0, tk = 0;
      for (int w = 0; w < WAVES; w++) {
        tt += s_wt[w];
        te += s_we[w];
        tk += s_wk[w];
      }
      unsigned long long base = 0;
      if (tt) base = atomicAdd(&a.ctr[og], (tt << CTR_E_BITS) | te);
      if (tk) *a.kill_flag = 1u;  // benign racing plain stores of the same value
      s_base = base;
      if (tt && s_nrec < RECHECK_TILES)
        s_rec[s_nrec++] = TileOut{og, (uint32_t)(base >> CTR_E_BITS), (uint32_t)tt,
                                  (uint32_t)(base & CTR_E_MASK), (uint32_t)te};
    }
    __syncthreads();
    uint64_t bt = s_base >> CTR_E_BITS, be = s_base & CTR_E_MASK;
    for (uint32_t w = 0; w < wv; w++) {
      bt += s_wt[w];
      be += s_we[w];
    }

    // ---- phase 4: emit list entries, publish committed writers
    if (live) {
      if (lane < T.nt && dec == 3u) {
        const uint32_t p = (uint32_t)__builtin_popcountll(bm & ((1ull << lane) - 1ull));
        tid_o[bt + p] = txn;
        coff_o[bt + p] = (uint32_t)(be + s_opos[wv][lane]);
      }
      uint32_t run = 0;
      for (uint32_t base = T.A0; base < T.A1; base += 64) {
        const uint32_t x = base + lane;
        const bool act = x < T.A1;
        const uint32_t lt = act ? map[x - T.A0] : 0xFFu;
        const uint64_t en = act ? ent[x - T.A0] : (uint64_t)SID_NONE;
        const uint32_t lo = (uint32_t)en;
        const uint32_t d = lt != 0xFFu ? s_stat[wv][lt] : 0u;
        const uint32_t sid = lo & ENT_SID;
        const bool has = sid != SID_NONE;
        const bool keep = d == 3u && has && (lo & (ENT_WRITE | ENT_BLOCK));
        const uint64_t km = ballot64(keep);
        if (keep) {
          const uint32_t below = (uint32_t)__builtin_popcountll(km & ((1ull << lane) - 1ull));
          cent_o[be + run + below] = en;
        }
        run += (uint32_t)__builtin_popcountll(km);
        // committed writer: tag-0 word (never displaced)
        if (d == 1u && has && (lo & ENT_WRITE)) atomicMin(&a.tab[sid].own, own_word(0, s_txn[wv][lt]));
      }
    }
    __syncthreads();  // LDS reuse by the next tile
  }

  // ---- recheck: after every workgroup's decisions are visible, abort the
  // emitted txns whose recorded blocker committed in this round (the work of
  // the next round's kill wave, done without re-reading the table).
  // Entry-parallel and coalesced: the tile's output offsets go to LDS and a
  // hit finds its txn by binary search.
  if (a.bar) {
    grid_barrier(a.bar);
    uint32_t* s_off = reinterpret_cast<uint32_t*>(&s_map[0][0]);  // >= WAVES*64+1 words
    const uint32_t nrec = s_nrec;
    bool any = false;
    for (uint32_t q = 0; q < nrec; q++) {
      const TileOut r = s_rec[q];
      const uint32_t* tid_o = a.tid_out + r.og * a.seg_ts;
      const uint32_t* coff_o = a.coff_out + r.og * a.seg_ts;
      const uint64_t* cent_o = a.cent_out + r.og * a.seg_es;
      for (uint32_t p = threadIdx.x; p < r.nt; p += blockDim.x) s_off[p] = coff_o[r.bt + p];
      if (threadIdx.x == 0) s_off[r.nt] = r.be + r.ne;
      __syncthreads();
      for (uint32_t x = r.be + threadIdx.x; x < r.be + r.ne; x += blockDim.x) {
        const uint64_t en = cent_o[x];
        if (((uint32_t)en & ENT_BLOCK) && a.state[(uint32_t)(en >> 32)] == ST_COMMIT) {
          uint32_t lo = 0, hi = r.nt;  // last p with s_off[p] <= x
          while (hi - lo > 1) {
            const uint32_t mid = (lo + hi) >> 1;
            if (s_off[mid] <= x) lo = mid;
            else hi = mid;
          }
          a.state[tid_o[r.bt + lo]] = cur_abort;  // racing stores of the same byte
          any = true;
        }
      }
      __syncthreads();
    }
    if (any) *a.kill_flag = 1u;
  }
}

// --------------------------------------------------------------------------
// k_pub: after a round that aborted something, the writers of keys whose
// owner aborted publish the next round's owner words (tag r+1).  Those are
// exactly the write entries whose recorded blocker aborted: every undecided
// writer of a key carries the key's current owner as its blocker, so when the
// owner aborts all of them become candidates and atomicMin elects the new
// minimum.  A key whose owner is still undecided keeps its (older-tag) word,
// which is never consulted — only accesses whose blocker aborted re-read
// owner words.  A round without aborts publishes nothing.
template <int CAP, int WAVES>
__global__ __launch_bounds__(WAVES * 64) void k_pub(PubArgs a) {
  __shared__ uint8_t s_map[WAVES][CAP];
  __shared__ uint32_t s_txn[WAVES][64];
  __shared__ ListGeo G;
  __shared__ LdsMin<PUB_LDS> comb;
  __shared__ uint8_t s_com[WAVES][64];
  if (*a.kill_flag == 0u) return;  // uniform: no aborts last round
  const uint32_t wv = threadIdx.x >> 6, lane = lane_id();
  uint8_t* map = s_map[wv];
  const uint64_t per_wg = (uint64_t)WAVES * a.tw;
  const uint32_t tagw = own_word(round_tag(a.r), 0);
  if (threadIdx.x == 0) list_geo(a.m_in, 0, 0, per_wg, G);
  comb.init();
  __syncthreads();
  for (uint64_t tile = blockIdx.x; tile < G.pre[G.nseg]; tile += gridDim.x) {
    const uint32_t sg = geo_seg(G, tile);
    const uint64_t m = G.m[sg];
    const uint64_t j0 = (tile - G.pre[sg]) * per_wg + (uint64_t)wv * a.tw;
    const uint64_t* cent_s = a.cent + sg * a.seg_es;
    const uint32_t* tid_s = a.tid + sg * a.seg_ts;
    Tile T;
    uint32_t txn, s, e;
    // a txn aborted by the recheck publishes nothing; a txn committed by the
    // last sharded decision (only sharded lists hold one) publishes its tag-0
    // words, which an unsharded round does at commit time
    bool part = true, com = false;
    if (lane < a.tw && j0 + lane < m) {
      const uint8_t st = a.state[tid_s[j0 + lane]];
      part = st == ST_UNDECIDED || st == ST_COMMIT;
      com = st == ST_COMMIT;
    }
    s_com[wv][lane] = com ? 1 : 0;
    const bool live = tile_open<CAP>(j0, a.tw, m, tid_s, a.coff + sg * a.seg_ts, G.end[sg], part,
                                     map, s_txn[wv], T, txn, s, e, a.err);
    __syncthreads();
    if (live) {
      for (uint32_t base = T.A0; base < T.A1; base += 64 * ILP) {
        uint64_t en[ILP];
        uint32_t lt[ILP];
        uint8_t bs[ILP];
#pragma unroll
        for (int u = 0; u < ILP; u++) {
          const uint32_t x = base + 64 * u + lane;
          lt[u] = x < T.A1 ? map[x - T.A0] : 0xFFu;
          const uint64_t e = cent_s[x < T.A1 ? x : T.A0];  // clamped: branch-free
          en[u] = lt[u] != 0xFFu ? e : 0ull;
        }
#pragma unroll
        for (int u = 0; u < ILP; u++) {
          const uint32_t lo = (uint32_t)en[u];
          const bool wb = (lo & ENT_WRITE) && (lo & ENT_BLOCK) && !a.force;
          const uint8_t b = a.state[wb ? (uint32_t)(en[u] >> 32) : 0u];
          bs[u] = wb ? b : ST_UNDECIDED;
        }
#pragma unroll
        for (int u = 0; u < ILP; u++) {
          const uint32_t lo = (uint32_t)en[u];
          const bool com = lt[u] != 0xFFu && s_com[wv][lt[u]];
          const bool cand = (lo & ENT_WRITE) &&
                            (com || a.force || ((lo & ENT_BLOCK) && bs[u] >= ST_ABORT));
          if (cand) {
            const uint32_t sid = lo & ENT_SID;
            const uint32_t wd = (com ? 0u : tagw) | s_txn[wv][lt[u]];
            if (!comb.add(sid, wd)) own_min(&a.tab[sid].own, wd);
          }
        }
      }
    }
    __syncthreads();
  }
  comb.flush(a.tab);
}

// --------------------------------------------------------------------------
// k_retag: after MAX_ROUND_TAG rounds, drop every non-committed owner word.
__global__ __launch_bounds__(256) void k_retag(Slot* __restrict__ tab, uint64_t cap) {
  const uint64_t sidx = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (sidx >= cap) return;
  const uint32_t w = tab[sidx].own;
  if ((w >> IDX_BITS) != 0) tab[sidx].own = OWN_EMPTY;
}

// --------------------------------------------------------------------------
// k_decide (sharded): 16 txns per thread step; one atomic per workgroup.
constexpr unsigned DECIDE_BLOCKS = 128;
__global__ __launch_bounds__(256) void k_decide(uint8_t* __restrict__ state,
                                                uint8_t* __restrict__ gst, uint64_t n,
                                                uint8_t abort_byte, uint32_t* __restrict__ und,
                                                uint32_t* __restrict__ und_next) {
  __shared__ uint32_t sh[4];
  if (blockIdx.x == 0 && threadIdx.x == 0) *und_next = 0;
  uint32_t cnt = 0;
  const uint64_t tid = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  for (uint64_t t0 = tid * 16; t0 < n; t0 += stride * 16) {
    const uint64_t t1 = t0 + 16 < n ? t0 + 16 : n;
    for (uint64_t t = t0; t < t1; t++) {
      const uint8_t s = state[t];
      if (s != ST_UNDECIDED) continue;
      const uint8_t g = gst[t];
      if (g >= 2) state[t] = abort_byte;
      else if (g == 0) state[t] = ST_COMMIT;
      else cnt++;
      gst[t] = 0;
    }
  }
  const uint32_t tot = block_sum_u32(cnt, sh);
  if (threadIdx.x == 0 && tot) atomicAdd(und, tot);
}

// --------------------------------------------------------------------------
// k_final: RC bytes, commit flags for the tn scan, per-block count partials.
__global__ __launch_bounds__(256) void k_final(FinalArgs a, GatherArgs g) {
  __shared__ uint32_t sh[4];
  uint32_t c = 0, ab = 0, ro = 0, und = 0, cw = 0;
  // what the host reads back besides the partials (error words, the sweep's
  // control block), copied by the last workgroup into pinned host memory: no
  // separate gather launch
  if (blockIdx.x == gridDim.x - 1)
    for (uint32_t q = 0; q < g.n; q++) {
      const CopyJob& cj = g.job[q];
      for (uint32_t i = threadIdx.x; i < cj.words; i += blockDim.x) cj.dst[i] = cj.src[i];
    }
  auto one = [&](uint8_t st, bool w) -> uint32_t {  // counts; returns the commit flag
    c += st == ST_COMMIT;
    ab += st >= ST_ABORT;
    und += st == ST_UNDECIDED;
    ro += w ? 0u : 1u;
    const uint32_t f = (st == ST_COMMIT && w) ? 1u : 0u;
    cw += f;
    return f;
  };
  const uint64_t tid = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  // four txns per thread and step (word loads / stores) when the output is
  // word-aligned (state / has-write / flags are the engine's own buffers)
  const uint64_t n4 = ((uintptr_t)a.rc & 3u) == 0 ? a.n / 4 : 0;
  for (uint64_t q = tid; q < n4; q += stride) {
    const uint32_t s4 = ((const uint32_t*)a.state)[q], h4 = ((const uint32_t*)a.hasw)[q];
    uint32_t r4 = 0, fl[4];
#pragma unroll
    for (uint32_t b = 0; b < 4; b++) {
      const uint8_t st = (uint8_t)(s4 >> (8 * b));
      fl[b] = one(st, ((h4 >> (8 * b)) & 0xFFu) != 0);
      r4 |= (st == ST_COMMIT ? 0u /* RCOK */ : 2u /* Abort */) << (8 * b);
    }
    ((uint32_t*)a.rc)[q] = r4;
    if (a.cflag) ((uint4*)a.cflag)[q] = make_uint4(fl[0], fl[1], fl[2], fl[3]);
  }
  for (uint64_t t = 4 * n4 + tid; t < a.n; t += stride) {
    const uint8_t st = a.state[t];
    const uint32_t f = one(st, a.hasw[t] != 0);
    a.rc[t] = st == ST_COMMIT ? 0 /* RCOK */ : 2 /* Abort */;
    if (a.cflag) a.cflag[t] = f;
  }
  const uint32_t s0 = block_sum_u32(c, sh), s1 = block_sum_u32(ab, sh),
                 s2 = block_sum_u32(ro, sh), s3 = block_sum_u32(cw, sh),
                 s4 = block_sum_u32(und, sh);
  if (threadIdx.x == 0) a.part[blockIdx.x] = FinalPart{s0, s1, s2, s3, s4, 0, 0, 0};
}

// --------------------------------------------------------------------------
// Exclusive scan of u32 flags -> commit tn (tnc + rank + 1), 3 kernels.
__global__ __launch_bounds__(1024) void k_scan_blocks(const uint32_t* __restrict__ f, uint64_t n,
                                                      uint64_t* __restrict__ bsum) {
  __shared__ uint32_t s[16];
  const uint64_t t = (uint64_t)blockIdx.x * 1024 + threadIdx.x;
  uint32_t v = t < n ? f[t] : 0;
  for (int d = 32; d > 0; d >>= 1) v += __shfl_xor(v, d);
  if ((threadIdx.x & 63) == 0) s[threadIdx.x >> 6] = v;
  __syncthreads();
  if (threadIdx.x == 0) {
    uint64_t tot = 0;
    for (int w = 0; w < 16; w++) tot += s[w];
    bsum[blockIdx.x] = tot;
  }
}

// exclusive scan of the block sums in place: one workgroup, 1024 sums per
// step (a serial loop over 256+ sums took 30 us)
__global__ __launch_bounds__(1024) void k_scan_sums(uint64_t* __restrict__ bsum, uint64_t nb) {
  __shared__ uint64_t s_w[16];
  __shared__ uint64_t s_carry;
  const uint32_t lane = lane_id(), wv = threadIdx.x >> 6;
  if (threadIdx.x == 0) s_carry = 0;
  __syncthreads();
  for (uint64_t c0 = 0; c0 < nb; c0 += 1024) {
    const uint64_t q = c0 + threadIdx.x;
    const uint64_t v = q < nb ? bsum[q] : 0ull;
    uint64_t x = v;
    for (int d = 1; d < 64; d <<= 1) {
      const uint64_t y = __shfl_up(x, d);
      if (lane >= (uint32_t)d) x += y;
    }
    if (lane == 63) s_w[wv] = x;
    __syncthreads();
    uint64_t base = s_carry;
    for (uint32_t w = 0; w < wv; w++) base += s_w[w];
    if (q < nb) bsum[q] = base + x - v;
    __syncthreads();
    if (threadIdx.x == 1023) s_carry = base + x;
    __syncthreads();
  }
}

__global__ __launch_bounds__(1024) void k_scan_apply(const uint32_t* __restrict__ f, uint64_t n,
                                                     const uint64_t* __restrict__ bsum,
                                                     uint64_t tnc, uint64_t* __restrict__ tn) {
  __shared__ uint32_t s[16];
  const uint64_t t = (uint64_t)blockIdx.x * 1024 + threadIdx.x;
  const uint32_t v = t < n ? f[t] : 0;
  // inclusive wave scan
  uint32_t x = v;
  const uint32_t lane = lane_id();
  for (int d = 1; d < 64; d <<= 1) {
    const uint32_t y = __shfl_up(x, d);
    if (lane >= (uint32_t)d) x += y;
  }
  if (lane == 63) s[threadIdx.x >> 6] = x;
  __syncthreads();
  uint32_t woff = 0;
  for (uint32_t w = 0; w < (threadIdx.x >> 6); w++) woff += s[w];
  if (t < n) tn[t] = v ? tnc + bsum[blockIdx.x] + woff + x : 0;
}

// --------------------------------------------------------------------------
// host launchers (the templates stay private to this translation unit)
static inline unsigned grid_for(uint64_t n, unsigned b) { return (unsigned)((n + b - 1) / b); }

void launch_prep(const uint32_t* off, uint64_t n, const uint8_t* at, uint64_t nnz, uint64_t p,
                 PrepPart* part, hipStream_t st) {
  k_prep<<<PREP_BLOCKS, 256, 0, st>>>(off, n, at, nnz, p, part);
}
void launch_hist(const HistArgs& a0, hipStream_t st) {
  HistArgs a = a0;
#ifdef DCC_EXPERIMENTS
  if (const char* e = DCC_ENV("DCC_HIST_VAR")) a.var = (uint32_t)atoi(e);  // timing variants (wrong results)
#else
  a.var = 0;
#endif
  // two workgroups per CU (LDS), each wave looping over 64-txn tiles
  k_hist<<<(unsigned)std::min<uint64_t>(grid_for(a.n, HIST_WAVES * 64), 512), HIST_WAVES * 64, 0, st>>>(a);
}
static unsigned tile_grid(uint64_t m, uint32_t tw, unsigned max_grid) {
  const uint64_t waves = (m + tw - 1) / tw;
  unsigned g = grid_for(waves, TILE_WAVES);
  if (g > max_grid) g = max_grid;
  return g ? g : 1;
}
void launch_build(const BuildArgs& a, unsigned max_grid, hipStream_t st) {
  k_build<TILE_CAP, TILE_WAVES><<<tile_grid(a.n, a.tw, max_grid), TILE_WAVES * 64, 0, st>>>(a);
}
void launch_round(const RoundArgs& a, bool from_keys, uint64_t m_bound, unsigned max_grid,
                  hipStream_t st) {
  const unsigned g = tile_grid(m_bound, a.tw, max_grid);
  constexpr unsigned B = TILE_WAVES * 64;
  if (a.gst) {
    if (from_keys) k_round<true, true, ROUND_CAP, TILE_WAVES><<<g, B, 0, st>>>(a);
    else k_round<false, true, ROUND_CAP, TILE_WAVES><<<g, B, 0, st>>>(a);
  } else {
    if (from_keys) k_round<true, false, ROUND_CAP, TILE_WAVES><<<g, B, 0, st>>>(a);
    else k_round<false, false, ROUND_CAP, TILE_WAVES><<<g, B, 0, st>>>(a);
  }
}
void launch_decide(uint8_t* state, uint8_t* gst, uint64_t n, uint8_t abort_byte, uint32_t* und,
                   uint32_t* und_next, hipStream_t st) {
  k_decide<<<DECIDE_BLOCKS, 256, 0, st>>>(state, gst, n, abort_byte, und, und_next);
}
void launch_retag(Slot* tab, uint64_t cap, hipStream_t st) {
  k_retag<<<grid_for(cap, 256), 256, 0, st>>>(tab, cap);
}
void launch_pub(const PubArgs& a, uint64_t m_bound, unsigned max_grid, hipStream_t st) {
  // tiles here are PUB_WAVES waves; the list geometry is recomputed in-kernel
  const uint64_t waves = (m_bound + a.tw - 1) / a.tw + NSEG * TILE_WAVES;
  unsigned g = grid_for(waves, PUB_WAVES);
  if (g > max_grid) g = max_grid;
  k_pub<ROUND_CAP, PUB_WAVES><<<g ? g : 1, PUB_WAVES * 64, 0, st>>>(a);
}
__global__ __launch_bounds__(256) void k_fill(FillArgs a) {
  const uint64_t t = (uint64_t)blockIdx.x * 256 + threadIdx.x, stride = (uint64_t)gridDim.x * 256;
  for (uint32_t q = 0; q < a.n; q++) {
    const FillJob& f = a.job[q];
    if (f.src)
      for (uint64_t i = t; i < f.words; i += stride) f.p[i] = f.src[i];
    else
      for (uint64_t i = t; i < f.words; i += stride) f.p[i] = f.value;
  }
}
void launch_fill(const FillArgs& a, hipStream_t st) {
  uint64_t mx = 1;
  for (uint32_t q = 0; q < a.n; q++) mx = a.job[q].words > mx ? a.job[q].words : mx;
  const unsigned grid = (unsigned)std::min<uint64_t>((mx + 255) / 256, 2048);
  k_fill<<<grid, 256, 0, st>>>(a);
}
__global__ __launch_bounds__(256) void k_gather(GatherArgs a) {
  for (uint32_t q = 0; q < a.n; q++) {
    const CopyJob& c = a.job[q];
    for (uint32_t i = blockIdx.x * 256 + threadIdx.x; i < c.words; i += gridDim.x * 256)
      c.dst[i] = c.src[i];
  }
}
void launch_gather(const GatherArgs& a, hipStream_t st) { k_gather<<<16, 256, 0, st>>>(a); }

void launch_final(const FinalArgs& a, const GatherArgs& g, hipStream_t st) {
  k_final<<<FINAL_BLOCKS, 256, 0, st>>>(a, g);
}
void launch_commit_tn(const uint32_t* cflag, uint64_t n, uint64_t* bsum, uint64_t tnc,
                      uint64_t* tn, hipStream_t st) {
  const unsigned nb = grid_for(n, 1024);
  k_scan_blocks<<<nb, 1024, 0, st>>>(cflag, n, bsum);
  k_scan_sums<<<1, 1024, 0, st>>>(bsum, nb);
  k_scan_apply<<<nb, 1024, 0, st>>>(cflag, n, bsum, tnc, tn);
}

// ---------------------------------------------------------------------------
// k_finish_flags: the commit flags of a deferred central_finish (global RC).
__global__ __launch_bounds__(256) void k_finish_flags(const uint8_t* __restrict__ frc,
                                                      const uint8_t* __restrict__ state,
                                                      const uint8_t* __restrict__ hasw, uint64_t n,
                                                      uint32_t* __restrict__ cflag,
                                                      uint32_t* __restrict__ cnt) {
  __shared__ uint32_t sh[4];
  uint32_t c = 0, bad = 0;
  for (uint64_t t = (uint64_t)blockIdx.x * 256 + threadIdx.x; t < n; t += (uint64_t)gridDim.x * 256) {
    const bool g = frc[t] == 0 /* DCC_RC_RCOK */, local = state[t] == ST_COMMIT;
    const uint32_t f = (g && local && hasw[t]) ? 1u : 0u;
    cflag[t] = f;
    c += f;
    bad += (g && !local) ? 1u : 0u;
  }
  const uint32_t sc = block_sum_u32(c, sh), sb = block_sum_u32(bad, sh);
  if (threadIdx.x == 0) {
    if (sc) atomicAdd(&cnt[0], sc);
    if (sb) atomicAdd(&cnt[1], sb);
  }
}
void launch_finish_flags(const uint8_t* final_rc, const uint8_t* state, const uint8_t* hasw,
                         uint64_t n, uint32_t* cflag, uint32_t* cnt, hipStream_t st) {
  k_finish_flags<<<grid_for(n, 256) < 1024 ? grid_for(n, 256) : 1024, 256, 0, st>>>(
      final_rc, state, hasw, n, cflag, cnt);
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

void launch_scatter(const uint8_t* sub_state, const uint32_t* sub_tid, const uint32_t* n_sub,
                    uint64_t m_bound, uint8_t* state, hipStream_t st) {
  unsigned g = (unsigned)((m_bound + 255) / 256);
  if (g > 1024) g = 1024;
  k_scatter<<<g ? g : 1, 256, 0, st>>>(sub_state, sub_tid, n_sub, state);
}


// --------------------------------------------------------------------------
// k_widen: the compact transfer forms (dcc.h DCC_KEYS_U32 / DCC_ACCTYPE_2BIT /
// DCC_TN_U32) back to the engine's layout.  Four accesses per thread and step
// (one 16-B key load, two 16-B key stores, one packed type byte in, one 4-byte
// type word out) when the arrays are 16-B aligned, else one.
__global__ __launch_bounds__(256) void k_widen(WidenArgs a) {
  const uint64_t tid = (uint64_t)blockIdx.x * 256 + threadIdx.x;
  const uint64_t stride = (uint64_t)gridDim.x * 256;
  if (a.k32) {
    const bool vec = (((uintptr_t)a.k32 | (uintptr_t)a.k64) & 15u) == 0;
    const uint64_t n4 = vec ? a.nnz / 4 : 0;
    for (uint64_t q = tid; q < n4; q += stride) {
      const uint4 v = ((const uint4*)a.k32)[q];
      ((uint4*)a.k64)[2 * q] = make_uint4(v.x, 0u, v.y, 0u);
      ((uint4*)a.k64)[2 * q + 1] = make_uint4(v.z, 0u, v.w, 0u);
    }
    for (uint64_t x = 4 * n4 + tid; x < a.nnz; x += stride) a.k64[x] = a.k32[x];
  }
  if (a.a2) {
    const bool vec = ((uintptr_t)a.a8 & 3u) == 0;
    const uint64_t n4 = vec ? a.nnz / 4 : 0;
    for (uint64_t q = tid; q < n4; q += stride) {
      const uint32_t p = a.a2[q];
      ((uint32_t*)a.a8)[q] = (p & 3u) | ((p >> 2) & 3u) << 8 | ((p >> 4) & 3u) << 16 | ((p >> 6) & 3u) << 24;
    }
    for (uint64_t x = 4 * n4 + tid; x < a.nnz; x += stride) a.a8[x] = (a.a2[x >> 2] >> (2 * (x & 3))) & 3u;
  }
  if (a.s32)
    for (uint64_t t = tid; t < a.n; t += stride) {
      a.s64[t] = a.s32[t];
      a.f64[t] = a.f32[t];
    }
}

void launch_widen(const WidenArgs& a, unsigned n_cu, hipStream_t st) {
  const uint64_t work = std::max<uint64_t>(a.nnz / 4, a.n);
  const uint64_t g = std::min<uint64_t>((work + 255) / 256, 8ull * n_cu);
  k_widen<<<(unsigned)std::max<uint64_t>(g, 1), 256, 0, st>>>(a);
}


// --------------------------------------------------------------------------
// k_copy16: the bandwidth reference (dcc_copy_bandwidth): 16 B per lane per
// load.  Grid-stride form: four loads in flight per thread before their
// stores.  Chunked form: each workgroup copies one contiguous range (DRAM
// pages stay open), eight loads in flight per thread, non-temporal loads and
// stores (the copy is read and written once).
__global__ __launch_bounds__(256) void k_copy16(const uint4* __restrict__ src, uint4* __restrict__ dst,
                                                uint64_t n16) {
  const uint64_t stride = (uint64_t)gridDim.x * 256;
  uint64_t q = (uint64_t)blockIdx.x * 256 + threadIdx.x;
  for (; q + 3 * stride < n16; q += 4 * stride) {
    const uint4 a = src[q], b = src[q + stride], c = src[q + 2 * stride], d = src[q + 3 * stride];
    dst[q] = a;
    dst[q + stride] = b;
    dst[q + 2 * stride] = c;
    dst[q + 3 * stride] = d;
  }
  for (; q < n16; q += stride) dst[q] = src[q];
}
__global__ __launch_bounds__(256) void k_copy16_chunk(const uint4* __restrict__ src, uint4* __restrict__ dst,
                                                      uint64_t n16) {
  constexpr uint32_t U = 8;
  const uint64_t per = (n16 + gridDim.x - 1) / gridDim.x;
  const uint64_t lo = (uint64_t)blockIdx.x * per, hi = min(n16, lo + per);
  typedef unsigned int v4u __attribute__((ext_vector_type(4)));
  const v4u* s4 = (const v4u*)src;
  v4u* d4 = (v4u*)dst;
  uint64_t q = lo + threadIdx.x;
  for (; q + (U - 1) * 256 < hi; q += U * 256) {
    v4u v[U];
#pragma unroll
    for (uint32_t u = 0; u < U; u++) v[u] = __builtin_nontemporal_load(s4 + q + u * 256);
#pragma unroll
    for (uint32_t u = 0; u < U; u++) __builtin_nontemporal_store(v[u], d4 + q + u * 256);
  }
  for (; q < hi; q += 256) dst[q] = src[q];
}
void launch_copy16(const void* src, void* dst, uint64_t bytes, unsigned grid, hipStream_t st) {
  k_copy16<<<grid ? grid : 1u, 256, 0, st>>>((const uint4*)src, (uint4*)dst, bytes / 16);
}
void launch_copy16_chunk(const void* src, void* dst, uint64_t bytes, unsigned grid, hipStream_t st) {
  k_copy16_chunk<<<grid ? grid : 1u, 256, 0, st>>>((const uint4*)src, (uint4*)dst, bytes / 16);
}

}  // namespace dcc
