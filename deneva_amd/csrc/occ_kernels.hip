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

#include "dcc_device.h"
#include "occ_kernels.h"

namespace dcc {

// --------------------------------------------------------------------------
// k_prep: offset validation + max txn length (one pass over offsets).
__global__ __launch_bounds__(256) void k_prep(const uint32_t* __restrict__ off, uint64_t n,
                                              uint64_t nnz, uint32_t* __restrict__ info) {
  // info[0] = error bits, info[1] = max length
  const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  uint32_t len = 0, bad = 0;
  if (t < n) {
    const uint32_t a = off[t], b = off[t + 1];
    if (b < a) bad = ERR_OFFSETS;
    else len = b - a;
    if (t == 0 && a != 0) bad = ERR_OFFSETS;
    if (t == n - 1 && b != nnz) bad = ERR_OFFSETS;
  }
  // wave reduce
  for (int d = 32; d > 0; d >>= 1) {
    len = max(len, (uint32_t)__shfl_xor(len, d));
    bad |= (uint32_t)__shfl_xor(bad, d);
  }
  if ((threadIdx.x & 63) == 0) {
    if (len) atomicMax(&info[1], len);
    if (bad) atomicOr(&info[0], bad);
  }
}

// --------------------------------------------------------------------------
// k_hist: the history window check (occ.cpp:160-180): if finish_tn > start_tn,
// txn i aborts when a committed history entry with start_tn < tn <= finish_tn
// wrote a key i READ (history is checked against the read set only).
// History is a CSR sorted by key: hkeys[u] unique ascending, htn[hoff[u]..)
// ascending.  One thread per txn (this path is off under TS_CLOCK).
__device__ inline int64_t hist_find(const uint64_t* hk, uint64_t nk, uint64_t key) {
  uint64_t lo = 0, hi = nk;
  while (lo < hi) {
    const uint64_t mid = (lo + hi) >> 1;
    if (hk[mid] < key) lo = mid + 1;
    else hi = mid;
  }
  return (lo < nk && hk[lo] == key) ? (int64_t)lo : -1;
}

__global__ __launch_bounds__(256) void k_hist(HistArgs a) {
  const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= a.n) return;
  const uint64_t s_tn = a.start_tn[t], f_tn = a.finish_tn[t];
  if (!(f_tn > s_tn)) return;
  for (uint32_t x = a.off[t]; x < a.off[t + 1]; x++) {
    if (a.acctype[x] == 1 /* WR */) continue;
    const int64_t u = hist_find(a.hkeys, a.nkeys, a.keys[x]);
    if (u < 0) continue;
    // any tn in (s_tn, f_tn]: first tn > s_tn, then test <= f_tn
    uint64_t lo = a.hoff[u], hi = a.hoff[u + 1];
    while (lo < hi) {
      const uint64_t mid = (lo + hi) >> 1;
      if (a.htn[mid] <= s_tn) lo = mid + 1;
      else hi = mid;
    }
    if (lo < a.hoff[u + 1] && a.htn[lo] <= f_tn) {
      a.state[t] = ST_ABORT;
      return;
    }
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

// --------------------------------------------------------------------------
// k_build: insert write keys, round-1 owners, per-txn has-write flag.
template <int CAP, int WAVES>
__global__ __launch_bounds__(WAVES * 64) void k_build(BuildArgs a) {
  __shared__ uint8_t s_map[WAVES][CAP];
  __shared__ uint32_t s_txn[WAVES][64];
  __shared__ uint32_t s_stat[WAVES][64];
  __shared__ uint32_t s_nw[WAVES];
  const uint32_t wv = threadIdx.x >> 6, lane = lane_id();
  const uint64_t j0 = ((uint64_t)blockIdx.x * WAVES + wv) * a.tw;
  uint8_t* map = s_map[wv];
  Tile T;
  uint32_t txn, s, e;
  bool part = true;
  if (lane < a.tw && j0 + lane < a.n) part = a.state[j0 + lane] == ST_UNDECIDED;
  const bool live = tile_open<CAP>(j0, a.tw, a.n, nullptr, a.off, 0, part, map, s_txn[wv], T,
                                   txn, s, e, a.err);
  s_stat[wv][lane] = 0;
  __syncthreads();
  uint32_t nw = 0;
  if (live) {
    const uint32_t tag1 = own_word(round_tag(1), 0);
    for (uint32_t base = T.A0; base < T.A1; base += 64) {
      const uint32_t x = base + lane;
      const bool act = x < T.A1;
      const uint32_t lt = act ? map[x - T.A0] : 0xFFu;
      bool w = false;
      if (lt != 0xFFu) {
        w = a.acctype[x] == 1 /* WR */;
        if (w) {
          const uint64_t key = a.keys[x];
          if (key == KEY_EMPTY) {
            atomicOr(a.err, ERR_KEY);
          } else {
            const uint32_t sid = table_insert(a.tab, a.mask, key);
            if (sid == SID_NONE) atomicOr(a.err, ERR_FULL);
            else own_min(&a.tab[sid].own[1], tag1 | s_txn[wv][lt]);
          }
        }
      }
      nw += w ? 1u : 0u;
      bool head;
      const uint32_t v = segment_or2(lt, w ? 1u : 0u, head);
      if (head && lt != 0xFFu && v) atomicOr(&s_stat[wv][lt], v);
    }
  }
  for (int d = 32; d > 0; d >>= 1) nw += __shfl_xor(nw, d);
  if (lane == 0) s_nw[wv] = nw;
  __syncthreads();
  if (live && lane < T.nt) a.hasw[j0 + lane] = s_stat[wv][lane] ? 1 : 0;
  if (threadIdx.x == 0) {
    uint32_t tot = 0;
    for (int w = 0; w < WAVES; w++) tot += s_nw[w];
    if (tot) atomicAdd((unsigned long long*)a.nnz_w, (unsigned long long)tot);
  }
}

// --------------------------------------------------------------------------
// k_round: one fixed-point round over a CSR list of undecided txns.
template <bool FROM_KEYS, int CAP, int WAVES>
__global__ __launch_bounds__(WAVES * 64) void k_round(RoundArgs a) {
  __shared__ uint8_t s_map[WAVES][CAP];
  __shared__ uint32_t s_ent[WAVES][CAP];
  __shared__ uint32_t s_txn[WAVES][64];
  __shared__ uint32_t s_stat[WAVES][64];
  __shared__ uint32_t s_opos[WAVES][64];
  __shared__ uint32_t s_wt[WAVES], s_we[WAVES];
  __shared__ unsigned long long s_base;

  const uint32_t wv = threadIdx.x >> 6, lane = lane_id();
  const uint64_t j0 = ((uint64_t)blockIdx.x * WAVES + wv) * a.tw;
  uint8_t* map = s_map[wv];
  uint32_t* ent = s_ent[wv];
  const uint32_t rb = a.r & 1u, nb = (a.r + 1) & 1u;
  const uint32_t tag_r = round_tag(a.r);
  const uint32_t tag_n = own_word(round_tag(a.r + 1), 0);

  Tile T;
  uint32_t txn, s, e;
  bool part = true;
  if (FROM_KEYS && lane < a.tw && j0 + lane < a.m) part = a.state[j0 + lane] == ST_UNDECIDED;
  const bool live = tile_open<CAP>(j0, a.tw, a.m, a.tid, a.coff, a.end_total, part, map,
                                   s_txn[wv], T, txn, s, e, a.err);
  s_stat[wv][lane] = 0;
  __syncthreads();

  // ---- phase 1: probe every access of the tile (coalesced)
  if (live) {
    for (uint32_t base = T.A0; base < T.A1; base += 64) {
      const uint32_t x = base + lane;
      const bool act = x < T.A1;
      const uint32_t lt = act ? map[x - T.A0] : 0xFFu;
      uint32_t en = SID_NONE, ps = 0;
      if (lt != 0xFFu) {
        const uint32_t i = s_txn[wv][lt];
        if (FROM_KEYS) {
          const uint64_t key = a.keys[x];
          const bool w = a.acctype[x] == 1 /* WR */;
          if (key == KEY_EMPTY) atomicOr(a.err, ERR_KEY);
          en = table_find(a.tab, a.mask, key) | (w ? ENT_WRITE : 0u);
        } else {
          en = a.cent[x];
        }
        const uint32_t sid = en & ENT_SID;
        if (sid != SID_NONE) ps = own_status(a.tab[sid].own[rb], tag_r, i);
        if (ps & PS_BLOCKED) en |= ENT_BLOCK;
      }
      if (act) ent[x - T.A0] = en;
      bool head;
      const uint32_t v = segment_or2(lt, ps, head);
      if (head && lt != 0xFFu && v) atomicOr(&s_stat[wv][lt], v);
    }
  }
  __syncthreads();

  // ---- phase 2: per-txn decision (lane = txn)
  uint32_t dec = 0;  // 0 none, 1 commit, 2 abort, 3 blocked
  if (live && lane < T.nt && part) {
    const uint32_t st = s_stat[wv][lane];
    dec = (st & PS_KILLED) ? 2u : (st & PS_BLOCKED) ? 3u : 1u;
    if (dec != 3u) a.state[txn] = (uint8_t)dec;
  }
  if (live) s_stat[wv][lane] = dec;
  __syncthreads();

  // ---- phase 3: count kept entries in access order; record each blocked
  // txn's output start.  A kept entry: txn blocked, slot known, and the access
  // is a write (feeds next-round owners) or was blocking.  A read that was
  // clear stays clear forever (writers are only ever decided, never added).
  uint32_t wave_e = 0;
  if (live) {
    for (uint32_t base = T.A0; base < T.A1; base += 64) {
      const uint32_t x = base + lane;
      const bool act = x < T.A1;
      const uint32_t lt = act ? map[x - T.A0] : 0xFFu;
      const uint32_t en = act ? ent[x - T.A0] : SID_NONE;
      const bool keep = lt != 0xFFu && s_stat[wv][lt] == 3u && (en & ENT_SID) != SID_NONE &&
                        (en & (ENT_WRITE | ENT_BLOCK));
      const uint64_t km = ballot64(keep);
      const uint32_t below = (uint32_t)__builtin_popcountll(km & ((1ull << lane) - 1ull));
      // first access of a txn (txn start inside this tile)
      const bool first = act && lt != 0xFFu && (x == T.A0 || map[x - 1 - T.A0] != lt);
      if (first) s_opos[wv][lt] = wave_e + below;
      wave_e += (uint32_t)__builtin_popcountll(km);
    }
  }
  const uint64_t bm = ballot64(live && lane < T.nt && dec == 3u);
  const uint32_t wave_t = (uint32_t)__builtin_popcountll(bm);
  if (lane == 0) {
    s_wt[wv] = wave_t;
    s_we[wv] = wave_e;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    unsigned long long tt = 0, te = 0;
    for (int w = 0; w < WAVES; w++) {
      tt += s_wt[w];
      te += s_we[w];
    }
    unsigned long long base = 0;
    if (tt) base = atomicAdd(a.ctr, (tt << CTR_E_BITS) | te);
    s_base = base;
  }
  __syncthreads();
  uint64_t bt = s_base >> CTR_E_BITS, be = s_base & CTR_E_MASK;
  for (uint32_t w = 0; w < wv; w++) {
    bt += s_wt[w];
    be += s_we[w];
  }

  // ---- phase 4: emit list entries + publish owner words
  if (live) {
    if (lane < T.nt && dec == 3u) {
      const uint32_t p = (uint32_t)__builtin_popcountll(bm & ((1ull << lane) - 1ull));
      a.tid_out[bt + p] = txn;
      a.coff_out[bt + p] = (uint32_t)(be + s_opos[wv][lane]);
    }
    uint32_t run = 0;
    for (uint32_t base = T.A0; base < T.A1; base += 64) {
      const uint32_t x = base + lane;
      const bool act = x < T.A1;
      const uint32_t lt = act ? map[x - T.A0] : 0xFFu;
      const uint32_t en = act ? ent[x - T.A0] : SID_NONE;
      const uint32_t d = lt != 0xFFu ? s_stat[wv][lt] : 0u;
      const uint32_t sid = en & ENT_SID;
      const bool has = sid != SID_NONE;
      const bool keep = d == 3u && has && (en & (ENT_WRITE | ENT_BLOCK));
      const uint64_t km = ballot64(keep);
      if (keep) {
        const uint32_t below = (uint32_t)__builtin_popcountll(km & ((1ull << lane) - 1ull));
        a.cent_out[be + run + below] = en & (ENT_WRITE | ENT_SID);
      }
      run += (uint32_t)__builtin_popcountll(km);
      if (has && (en & ENT_WRITE)) {
        const uint32_t i = s_txn[wv][lt];
        if (d == 1u) {
          // committed writer: tag-0 word in both buffers (never displaced)
          atomicMin(&a.tab[sid].own[0], own_word(0, i));
          atomicMin(&a.tab[sid].own[1], own_word(0, i));
        } else if (d == 3u) {
          own_min(&a.tab[sid].own[nb], tag_n | i);
        }
      }
    }
  }
}

// --------------------------------------------------------------------------
// k_retag: after MAX_TAG_ROUND rounds, drop every non-committed owner word.
__global__ __launch_bounds__(256) void k_retag(Slot* __restrict__ tab, uint64_t cap) {
  const uint64_t sidx = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (sidx >= cap) return;
  for (int b = 0; b < 2; b++) {
    const uint32_t w = tab[sidx].own[b];
    if ((w >> IDX_BITS) != 0) tab[sidx].own[b] = OWN_EMPTY;
  }
}

// k_owner_list: publish round-`r` owners from a list (after a retag).
__global__ __launch_bounds__(256) void k_owner_list(OwnerArgs a) {
  const uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= a.m) return;
  const uint32_t i = a.tid[j];
  const uint32_t s = a.coff[j], e = (j + 1 < a.m) ? a.coff[j + 1] : a.end_total;
  const uint32_t w = own_word(round_tag(a.r), i);
  for (uint32_t x = s; x < e; x++) {
    const uint32_t en = a.cent[x];
    if (en & ENT_WRITE) own_min(&a.tab[en & ENT_SID].own[a.r & 1u], w);
  }
}

// --------------------------------------------------------------------------
// k_final: RC bytes + counts; commit flags for the tn scan.
__global__ __launch_bounds__(256) void k_final(FinalArgs a) {
  const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  uint32_t c = 0, ab = 0, ro = 0, und = 0, cw = 0;
  if (t < a.n) {
    const uint8_t st = a.state[t];
    const bool w = a.hasw[t] != 0;
    if (st == ST_COMMIT) c = 1;
    else if (st == ST_ABORT) ab = 1;
    else und = 1;
    ro = w ? 0 : 1;
    cw = (st == ST_COMMIT && w) ? 1 : 0;
    a.rc[t] = st == ST_COMMIT ? 0 /* RCOK */ : 2 /* Abort */;
    if (a.cflag) a.cflag[t] = (st == ST_COMMIT && w) ? 1u : 0u;
  }
  for (int d = 32; d > 0; d >>= 1) {
    c += __shfl_xor(c, d);
    ab += __shfl_xor(ab, d);
    ro += __shfl_xor(ro, d);
    und += __shfl_xor(und, d);
    cw += __shfl_xor(cw, d);
  }
  if ((threadIdx.x & 63) == 0) {
    if (c) atomicAdd((unsigned long long*)&a.counts[0], (unsigned long long)c);
    if (ab) atomicAdd((unsigned long long*)&a.counts[1], (unsigned long long)ab);
    if (ro) atomicAdd((unsigned long long*)&a.counts[2], (unsigned long long)ro);
    if (cw) atomicAdd((unsigned long long*)&a.counts[3], (unsigned long long)cw);
    if (und) atomicOr(a.err, ERR_UNDECIDED);
  }
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

__global__ __launch_bounds__(64) void k_scan_sums(uint64_t* __restrict__ bsum, uint64_t nb) {
  if (threadIdx.x != 0) return;
  uint64_t run = 0;
  for (uint64_t b = 0; b < nb; b++) {
    const uint64_t v = bsum[b];
    bsum[b] = run;
    run += v;
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

void launch_prep(const uint32_t* off, uint64_t n, uint64_t nnz, uint32_t* info, hipStream_t st) {
  k_prep<<<grid_for(n, 256), 256, 0, st>>>(off, n, nnz, info);
}
void launch_hist(const HistArgs& a, hipStream_t st) {
  k_hist<<<grid_for(a.n, 256), 256, 0, st>>>(a);
}
void launch_build(const BuildArgs& a, hipStream_t st) {
  const uint64_t waves = (a.n + a.tw - 1) / a.tw;
  k_build<TILE_CAP, TILE_WAVES><<<grid_for(waves, TILE_WAVES), TILE_WAVES * 64, 0, st>>>(a);
}
void launch_round(const RoundArgs& a, bool from_keys, hipStream_t st) {
  const uint64_t waves = (a.m + a.tw - 1) / a.tw;
  const unsigned g = grid_for(waves, TILE_WAVES);
  if (from_keys) k_round<true, TILE_CAP, TILE_WAVES><<<g, TILE_WAVES * 64, 0, st>>>(a);
  else k_round<false, TILE_CAP, TILE_WAVES><<<g, TILE_WAVES * 64, 0, st>>>(a);
}
void launch_retag(Slot* tab, uint64_t cap, hipStream_t st) {
  k_retag<<<grid_for(cap, 256), 256, 0, st>>>(tab, cap);
}
void launch_owner_list(const OwnerArgs& a, hipStream_t st) {
  k_owner_list<<<grid_for(a.m, 256), 256, 0, st>>>(a);
}
void launch_final(const FinalArgs& a, hipStream_t st) {
  k_final<<<grid_for(a.n, 256), 256, 0, st>>>(a);
}
void launch_commit_tn(const uint32_t* cflag, uint64_t n, uint64_t* bsum, uint64_t tnc,
                      uint64_t* tn, hipStream_t st) {
  const unsigned nb = grid_for(n, 1024);
  k_scan_blocks<<<nb, 1024, 0, st>>>(cflag, n, bsum);
  k_scan_sums<<<1, 64, 0, st>>>(bsum, nb);
  k_scan_apply<<<nb, 1024, 0, st>>>(cflag, n, bsum, tnc, tn);
}

__global__ __launch_bounds__(256) void k_count_writes(const uint8_t* __restrict__ at, uint64_t nnz,
                                                      unsigned long long* __restrict__ cnt) {
  uint32_t c = 0;
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x * 16;
  for (uint64_t x = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) * 16; x < nnz; x += stride) {
    if (x + 16 <= nnz && ((uintptr_t)(at + x) & 15) == 0) {
      const uint4 v = *reinterpret_cast<const uint4*>(at + x);
      const uint32_t w[4] = {v.x, v.y, v.z, v.w};
      for (int q = 0; q < 4; q++)
        for (int b = 0; b < 4; b++) c += ((w[q] >> (8 * b)) & 0xFF) == 1u;
    } else {
      for (uint64_t y = x; y < nnz && y < x + 16; y++) c += at[y] == 1;
    }
  }
  for (int d = 32; d > 0; d >>= 1) c += __shfl_xor(c, d);
  if ((threadIdx.x & 63) == 0 && c) atomicAdd(cnt, (unsigned long long)c);
}
void launch_count_writes(const uint8_t* at, uint64_t nnz, unsigned long long* cnt, hipStream_t st) {
  uint64_t g = (nnz / 16 + 255) / 256;
  if (g > 2048) g = 2048;
  if (g == 0) g = 1;
  k_count_writes<<<(unsigned)g, 256, 0, st>>>(at, nnz, cnt);
}

}  // namespace dcc
