// gfx950 kernels of the OCC stage solver.
//
// The serial decision (central_validate in index order, occ.cpp:116-239,
// then central_finish, :248-294) is
//
//   abort(i)  <=>  some EARLIER committed txn j wrote a key i reads or writes
//
// A txn touching a key of C, the committed write set of the txns decided
// before it, is dead; a dead txn never commits, so it neither kills nor
// blocks anyone, and the survivors can be decided in their own order.  The
// epoch is therefore decided in stages.  Stage l runs ONE kernel:
//
//   filter workgroups   stream the stage's input list (stage 0: the epoch's
//                       first P0 txns; stage 1: the rest of the epoch; stage
//                       l >= 2: the previous stage's output list minus what
//                       its decider decided), kill every txn touching the
//                       previous decider's C (rc = Abort), and write the
//                       survivors, in index order, chunk by chunk, as the
//                       stage's output list — grouped into tiles of 64 with
//                       everything the serial decision needs precomputed:
//                       per access a 32-bit key hash and (tile-local txn,
//                       W); per txn the mask of EARLIER txns of its tile that
//                       write one of its keys (an LDS write map per tile);
//   decider workgroup   (workgroup 0) takes the published chunks' tiles in
//                       order and decides them exactly: a txn is dead if a
//                       key is in C (an LDS bitmap + exact hash set of the
//                       committed write keys of this decider) or an earlier
//                       committed txn of its tile writes one of its keys (a
//                       bit-parallel fixed point over the tile's dependency
//                       masks); committed write keys join C.  It stops at
//                       pmax txns or when C would exceed its budget; its C is
//                       the next stage's filter.
//
// The decider overlaps its own stage's filter (stage 1: the epoch-long
// stream).  Hand-off: a filter workgroup publishes a chunk with the agent
// release / relaxed flag / agent acquire protocol (MI355X_MICROARCH.md,
// "Workgroup dispatch ... Valid forms"); the decider acquires twice per
// stage (the first chunks, then the rest).  Flags carry a (gen, stage) tag,
// so no per-epoch reset is needed.
//
// The decider runs on one CU, so its cost is instructions per access: it
// only loads key / hash / (txn, W), tests one bitmap bit, probes the exact
// set on a bitmap hit, and inserts committed writes; one wave runs the fixed
// point.  Everything else is done by the filter workgroups on the other CUs.
#include <hip/hip_runtime.h>

#include "dcc_device.h"
#include "occ_kernels.h"
#include "occ_stage.h"

namespace dcc {

constexpr uint8_t AT_WR = 1;   // access_t WR (system/global.h:287)
constexpr uint8_t RC_OK = 0;   // RCOK
constexpr uint8_t RC_AB = 2;   // Abort
constexpr uint32_t CT_SLOTS = 1u << ST_CT_LOG;
constexpr uint32_t CS_SLOTS = 1u << ST_CS_LOG;
constexpr uint32_t WM_SLOTS = 1u << ST_WM_LOG;

__device__ inline uint32_t st_tag(uint32_t gen, uint32_t stage) { return gen * ST_MAX_STAGES + stage + 1; }

// One 32-bit hash per key serves every structure: set slots take its top
// bits, bitmaps its low bits.
__device__ inline uint32_t st_hash(uint64_t key) {
  return (uint32_t)((key * 0x9E3779B97F4A7C15ull) >> 32);
}
__device__ inline uint32_t hslot(uint32_t h, uint32_t bits) { return h >> (32 - bits); }

// Open-addressing u64 set in LDS (linear probing from the hash's top bits;
// keys are never removed while the set is read).
__device__ inline bool lset_has(const uint64_t* t, uint32_t bits, uint64_t key, uint32_t h) {
  const uint32_t m = (1u << bits) - 1u;
  uint32_t s = hslot(h, bits);
  for (uint32_t q = 0; q <= m; q++) {
    const uint64_t v = t[s];
    if (v == key) return true;
    if (v == KEY_EMPTY) return false;
    s = (s + 1) & m;
  }
  return false;
}
// returns the slot (~0u if full); `fresh` when this call entered the key
__device__ inline uint32_t lset_put(uint64_t* t, uint32_t bits, uint64_t key, uint32_t h, bool& fresh) {
  const uint32_t m = (1u << bits) - 1u;
  uint32_t s = hslot(h, bits);
  fresh = false;
  for (uint32_t q = 0; q <= m; q++) {
    const uint64_t v = t[s];
    if (v == key) return s;
    if (v == KEY_EMPTY) {
      const unsigned long long p = atomicCAS((unsigned long long*)&t[s], (unsigned long long)KEY_EMPTY,
                                             (unsigned long long)key);
      if (p == KEY_EMPTY) {
        fresh = true;
        return s;
      }
      if (p == key) return s;
    }
    s = (s + 1) & m;
  }
  return ~0u;
}
__device__ inline uint32_t lset_slot(const uint64_t* t, uint32_t bits, uint64_t key, uint32_t h) {
  const uint32_t m = (1u << bits) - 1u;
  uint32_t s = hslot(h, bits);
  for (uint32_t q = 0; q <= m; q++) {
    const uint64_t v = t[s];
    if (v == key) return s;
    if (v == KEY_EMPTY) return ~0u;
    s = (s + 1) & m;
  }
  return ~0u;
}

// any bit of [lo, hi) in an LDS bitmap of u64 words
__device__ inline bool bits_any(const uint64_t* bm, uint32_t lo, uint32_t hi) {
  bool any = false;
  for (uint32_t w = lo >> 6; (w << 6) < hi; w++) {
    uint64_t v = bm[w];
    if ((w << 6) < lo) v &= ~0ull << (lo & 63);
    if (((w + 1) << 6) > hi) v &= ~0ull >> (64 - (hi & 63));
    any |= v != 0;
  }
  return any;
}
__device__ inline uint32_t bits_count(const uint64_t* bm, uint32_t lo, uint32_t hi) {
  uint32_t c = 0;
  for (uint32_t w = lo >> 6; (w << 6) < hi; w++) {
    uint64_t v = bm[w];
    if ((w << 6) < lo) v &= ~0ull << (lo & 63);
    if (((w + 1) << 6) > hi) v &= ~0ull >> (64 - (hi & 63));
    c += (uint32_t)__builtin_popcountll(v);
  }
  return c;
}

// first epoch txn of stage 1: stage 0's decider stop, or P0 when it decided all
__device__ inline uint32_t st_begin(const StArgs& a) {
  return a.prev->stop_tid == 0xFFFFFFFFu ? a.p0 : a.prev->stop_tid;
}

__device__ inline uint64_t lt_mask(uint32_t l) { return l ? (~0ull >> (64 - l)) : 0ull; }

// Cross-lane primitives on DPP (GFX9 row shifts / row broadcasts) and
// readlane: a __shfl is a ds_bpermute, an LDS round trip per step.
template <int CTRL, int ROW = 0xF, int BANK = 0xF>
__device__ inline uint32_t dpp0(uint32_t v) {
  return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, CTRL, ROW, BANK, false);
}
// inclusive prefix sum over the 64 lanes
__device__ inline uint32_t wave_incl_sum(uint32_t v) {
  uint32_t t = v + dpp0<0x111>(v);   // row_shr:1
  t += dpp0<0x112>(v);               // row_shr:2
  t += dpp0<0x113>(v);               // row_shr:3
  t += dpp0<0x114, 0xF, 0xE>(t);     // row_shr:4, banks 1-3
  t += dpp0<0x118, 0xF, 0xC>(t);     // row_shr:8, banks 2-3
  t += dpp0<0x142, 0xA>(t);          // row_bcast:15 into rows 1, 3
  t += dpp0<0x143, 0xC>(t);          // row_bcast:31 into rows 2, 3
  return t;
}
__device__ inline uint32_t wave_excl_sum(uint32_t v) { return wave_incl_sum(v) - v; }
__device__ inline uint32_t wave_sum_u32(uint32_t v) {
  return (uint32_t)__builtin_amdgcn_readlane((int)wave_incl_sum(v), 63);
}
// Workgroup barrier for LDS hand-offs only: waits for this wave's LDS ops,
// not for its outstanding global loads (__syncthreads() is a release fence
// too, i.e. s_waitcnt vmcnt(0): it would drain every prefetch in flight).
__device__ inline void lds_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

__device__ inline uint32_t lane_bcast(uint32_t v, uint32_t l) {
  return (uint32_t)__builtin_amdgcn_readlane((int)v, (int)l);
}

// ---------------------------------------------------------------- LDS
struct WaveTile {
  uint32_t t0, nt;   // txns [t0, t0 + nt) of the input (epoch index or list slot)
  uint32_t mode;     // 0 epoch CSR, 1 list
  uint32_t pad;
};
struct FilterLds {
  union {
    struct {                           // streaming pass: C of the previous decider
      uint32_t fb[1u << (ST_FB_LOG - 5)];  // bitmap (32 KB)
      uint64_t ct[CT_SLOTS];               // exact set (64 KB)
    } c;
    struct {                           // tile building: one write map per building wave
      uint64_t wk[ST_WM_WAVES][WM_SLOTS];  // key
      uint64_t wm[ST_WM_WAVES][WM_SLOTS];  // writer mask
    } t;
  } u;
  uint64_t he[ST_W][32];               // per wave: hits of the even / odd accesses of a wave-tile
  uint64_t ho[ST_W][32];
  uint64_t wb[ST_W][80];               // per wave: W bit per access (<= 4096 + 1024 from b16)
  uint64_t tdep[ST_WM_WAVES][ST_TILE];
  uint64_t thw[ST_WM_WAVES];
  WaveTile wt[ST_WT];
  uint64_t smask[ST_WT];               // per wave-tile: survivors
  uint32_t scnt[ST_WT], sacc[ST_WT], spos[ST_WT], sapos[ST_WT];
  uint32_t cnt[4];                     // stats partials
  uint32_t nwt, maxlen;
};
struct DeciderLds {
  uint64_t cs[CS_SLOTS];               // committed write keys of this decider (C)
  uint32_t cb[1u << (ST_CB_LOG - 5)];  // their bitmap
  uint64_t stk[ST_TILE_ACC];           // the current tile's write accesses: key
  uint32_t sth[ST_TILE_ACC];           //                                    hash
  uint8_t stt[ST_TILE_ACC];            //                                    txn
  struct Slot {                        // a tile staged by the loader waves
    uint64_t k[ST_TILE_ACC];
    uint32_t h[ST_TILE_ACC];
    uint8_t p[ST_TILE_ACC];
    uint64_t dep[ST_TILE];
  } slot[2];
  uint64_t desc[ST_MAX_TILES][ST_TILE_WORDS];
  uint32_t tpref[ST_MAX_PUB + 1];      // taken chunks: first flat tile index
  uint32_t ttb[ST_MAX_PUB];            //               first txn slot
  uint32_t wsum[ST_W];
  uint64_t dead;
  uint32_t nst, ckn, err;
  uint32_t tslot[ST_MAX_TILES];        // per decided tile: first txn slot
  uint64_t tcom[ST_MAX_TILES];         //                   commit mask
  uint64_t thw[ST_MAX_TILES];          //                   has-write mask
  uint32_t tnt[ST_MAX_TILES];          //                   txns
};
union StLds {
  FilterLds f;
  DeciderLds d;
};

// ------------------------------------------------------------------ filter
// One wave-tile: txns [t0, t0 + nt) whose accesses are one contiguous range
// (epoch CSR, or a chunk's survivors).  Sets the survivor mask and their
// access count; writes nothing to global memory.
__device__ void filter_wave_tile(const StArgs& a, FilterLds& L, uint32_t w, const WaveTile& wt,
                                 bool useC, uint32_t stats_from, uint64_t& surv, uint32_t& sacc,
                                 uint32_t& err) {
  const uint32_t lane = lane_id();
  const uint32_t nt = wt.nt, t0 = wt.t0;
  const bool own = lane < nt;
  uint32_t tid = 0, o = 0, e = 0;
  if (wt.mode == 0) {
    const uint32_t j = t0 + lane;
    tid = j;
    if (own) {
      o = a.off[j];
      e = a.off[j + 1];
      if (e < o || e > a.nnz || (j == 0 && o != 0) || (j + 1 == a.n && e != a.nnz)) {
        err |= STE_OFFSETS;
        o = min(o, (uint32_t)a.nnz);
        e = min(max(e, o), (uint32_t)a.nnz);
      }
      if (e - o > MAX_TXN_LEN) {
        err |= STE_LEN;
        e = o + MAX_TXN_LEN;
      }
    }
  } else if (own) {
    const uint32_t j = t0 + lane;
    tid = a.in.tid[j];
    o = a.in.ast[j];
    e = o + a.in.alen[j];
  }
  const uint64_t* kp = wt.mode == 0 ? a.keys : a.in.keys;
  const uint8_t* tp = wt.mode == 0 ? a.at : a.in.pk;
  const uint8_t wmatch = wt.mode == 0 ? AT_WR : 1u;  // list mode: pk bit 0 is W
  const uint8_t wmask8 = wt.mode == 0 ? 0xFFu : 1u;
  // the wave-tile's accesses [A0, A1): contiguous by construction; clamp
  // for malformed input
  const uint32_t A0 = lane_bcast(o, 0);
  uint32_t A1 = lane_bcast(e, nt - 1);
  if (A1 < A0) A1 = A0;
  if (A1 - A0 > MAX_TXN_LEN * 64) A1 = A0 + MAX_TXN_LEN * 64;
  const uint32_t base = A0 & ~1u;
  const uint32_t npair = (A1 - base + 1) >> 1;
  const uint32_t J = (npair + 63) >> 6;  // <= 32
  const uint64_t lim = wt.mode == 0 ? a.nnz : 0xFFFFFFFFull;
  // keys: two per lane (16 B), hit bits of even / odd accesses by pair index
  for (uint32_t jj = 0; jj < J; jj++) {
    const uint32_t x0 = base + 2 * (64 * jj + lane);
    uint64_t k0 = KEY_EMPTY, k1 = KEY_EMPTY;
    const bool v0 = x0 >= A0 && x0 < A1;
    const bool v1 = x0 + 1 < A1;
    if (v1 && (uint64_t)x0 + 2 <= lim && ((uintptr_t)(kp + x0) & 15) == 0) {
      const ulonglong2 kk = *(const ulonglong2*)(kp + x0);
      k0 = kk.x;
      k1 = kk.y;
    } else {
      if (v0) k0 = kp[x0];
      if (v1) k1 = kp[x0 + 1];
    }
    if ((v0 && k0 == KEY_EMPTY) || (v1 && k1 == KEY_EMPTY)) err |= STE_KEY;
    bool h0 = false, h1 = false;
    if (useC) {
      if (v0) {
        const uint32_t h = st_hash(k0), b = h & ((1u << ST_FB_LOG) - 1u);
        if ((L.u.c.fb[b >> 5] >> (b & 31)) & 1u) h0 = lset_has(L.u.c.ct, ST_CT_LOG, k0, h);
      }
      if (v1) {
        const uint32_t h = st_hash(k1), b = h & ((1u << ST_FB_LOG) - 1u);
        if ((L.u.c.fb[b >> 5] >> (b & 31)) & 1u) h1 = lset_has(L.u.c.ct, ST_CT_LOG, k1, h);
      }
    }
    const uint64_t be = __ballot(h0), bo = __ballot(h1);
    if (lane == 0) {
      L.he[w][jj] = be;
      L.ho[w][jj] = bo;
    }
  }
  // access types: 16 per lane, W bits in access order
  const uint32_t b16 = A0 & ~15u;
  const uint32_t J16 = (A1 - b16 + 1023) >> 10;  // <= 5
  for (uint32_t jj = 0; jj < J16; jj++) {
    const uint32_t x = b16 + 1024 * jj + 16 * lane;
    uint32_t m16 = 0;
    if (x < A1) {
      if ((uint64_t)x + 16 <= lim && ((uintptr_t)(tp + x) & 15) == 0) {
        const uint4 v = *(const uint4*)(tp + x);
        const uint32_t wv[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
        for (int q = 0; q < 16; q++)
          m16 |= ((((wv[q >> 2] >> (8 * (q & 3))) & wmask8) == wmatch) ? 1u : 0u) << q;
      } else {
#pragma unroll 1
        for (int q = 0; q < 16; q++)
          if (x + q < A1) m16 |= ((tp[x + q] & wmask8) == wmatch ? 1u : 0u) << q;
      }
      // drop bytes outside [A0, A1)
      if (x < A0) m16 &= ~0u << (A0 - x);
      if (x + 16 > A1) m16 &= (1u << (A1 - x)) - 1u;
    }
    ((uint16_t*)L.wb[w])[64 * jj + lane] = (uint16_t)m16;
  }
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  bool kill = false;
  uint32_t nw = 0;
  if (own) {
    const uint32_t s = o - base, t = e - base;
    // even accesses p = 2i in [s, t): i in [ceil(s/2), ceil(t/2)); odd: [floor(s/2), floor(t/2))
    kill = bits_any(L.he[w], (s + 1) >> 1, (t + 1) >> 1) || bits_any(L.ho[w], s >> 1, t >> 1);
    nw = bits_count(L.wb[w], o - b16, e - b16);
    if (a.hkill && a.hkill[tid]) kill = true;
  }
  if (wt.mode == 0) {
    const bool cnt = own && tid >= stats_from;
    const uint32_t sw = wave_sum_u32(cnt ? nw : 0u);
    const uint32_t sr = (uint32_t)__builtin_popcountll(__ballot(cnt && nw == 0));
    if (lane == 0) {
      if (sw) atomicAdd(&L.cnt[0], sw);
      if (sr) atomicAdd(&L.cnt[1], sr);
    }
  }
  const bool sv = own && !kill;
  surv = __ballot(sv);
  sacc = wave_sum_u32(sv ? e - o : 0u);
  if (sv && e - o > 16) atomicMax(&L.maxlen, e - o);
  __builtin_amdgcn_wave_barrier();
}

// Copy the survivors of one wave-tile into the output list: per txn slot
// (tid, ast, alen), per access (key, hash, pk = tile-local txn << 1 | W).
// opos / oapos: the wave-tile's first output txn / access (chunk-relative);
// tiles hold T consecutive survivors.
__device__ void filter_copy(const StArgs& a, const WaveTile& wt, uint64_t surv, uint32_t opos,
                            uint32_t oapos, uint32_t tbase, uint32_t abase, uint32_t T) {
  const uint32_t lane = lane_id();
  const bool own = lane < wt.nt;
  uint32_t tid = 0, o = 0, e = 0;
  if (own) {
    if (wt.mode == 0) {
      tid = wt.t0 + lane;
      o = a.off[wt.t0 + lane];
      e = a.off[wt.t0 + lane + 1];
      o = min(o, (uint32_t)a.nnz);
      e = min(max(e, o), (uint32_t)a.nnz);
      if (e - o > MAX_TXN_LEN) e = o + MAX_TXN_LEN;
    } else {
      tid = a.in.tid[wt.t0 + lane];
      o = a.in.ast[wt.t0 + lane];
      e = o + a.in.alen[wt.t0 + lane];
    }
  }
  const bool sv = (surv >> lane) & 1ull;
  const uint32_t len = sv ? e - o : 0u;
  const uint32_t r = (uint32_t)__builtin_popcountll(surv & lt_mask(lane));
  const uint32_t rs = wave_excl_sum(len);  // wave-tile-relative output access
  if (sv) {
    a.out.tid[tbase + opos + r] = tid;
    a.out.ast[tbase + opos + r] = abase + oapos + rs;
    a.out.alen[tbase + opos + r] = (uint8_t)len;
  }
  const uint64_t* kp = wt.mode == 0 ? a.keys : a.in.keys;
  const uint8_t* tp = wt.mode == 0 ? a.at : a.in.pk;
  const uint32_t* hp = wt.mode == 0 ? nullptr : a.in.hsh;
  // lane-strided over the survivors' accesses in output order (coalesced
  // stores, independent iterations): output access u belongs to the last
  // lane s with rs[s] <= u (non-survivors have len 0 and share the next rs)
  const uint32_t SA = lane_bcast(rs + len, 63);
  uint64_t* ok = a.out.keys + abase + oapos;
  uint32_t* oh = a.out.hsh + abase + oapos;
  uint8_t* ot = a.out.pk + abase + oapos;
  for (uint32_t ub = 0; ub < SA; ub += 64) {
    const uint32_t u = ub + lane;
    uint32_t lo = 0;
#pragma unroll
    for (uint32_t st = 32; st > 0; st >>= 1) {
      const uint32_t cand = lo + st;
      const uint32_t v = (uint32_t)__shfl((int)rs, (int)min(cand, 63u));
      if (cand < 64 && v <= u) lo = cand;
    }
    const uint32_t so = (uint32_t)__shfl((int)o, (int)lo);
    const uint32_t sr = (uint32_t)__shfl((int)rs, (int)lo);
    const uint32_t rr = (uint32_t)__builtin_popcountll(surv & lt_mask(lo));  // survivor rank
    if (u < SA) {
      const uint32_t src = so + (u - sr);
      const uint64_t k = kp[src];
      const uint8_t ty = tp[src];
      const bool wr = wt.mode == 0 ? ty == AT_WR : (ty & 1u) != 0;
      ok[u] = k;
      oh[u] = hp ? hp[src] : st_hash(k);
      ot[u] = (uint8_t)((((opos + rr) % T) << 1) | (wr ? 1u : 0u));
    }
  }
}

// Tile k of this chunk's output (survivors [T k, T k + nt), chunk-relative),
// built by ONE wave with its own LDS write map: per txn the mask of earlier
// txns of the tile writing one of its keys, the has-write mask, the write
// count, and the descriptor.  Reads back what this workgroup just wrote.
__device__ void filter_build_tile(const StArgs& a, FilterLds& L, uint32_t wv, uint32_t k,
                                  uint32_t out_t, uint32_t tbase, uint32_t T) {
  const uint32_t lane = lane_id();
  uint64_t* wk = L.u.t.wk[wv];
  uint64_t* wm = L.u.t.wm[wv];
  uint64_t* tdep = L.tdep[wv];
  const uint32_t f = tbase + T * k;  // first txn slot
  const uint32_t nt = min(T, out_t - T * k);
  const uint32_t a0 = a.out.ast[f];
  const uint32_t a1 = a.out.ast[f + nt - 1] + a.out.alen[f + nt - 1];
  const uint32_t na = a1 - a0;
  uint32_t nw = 0;
  uint64_t hw = 0;
  bool full = false;
  for (uint32_t x = lane; x < na; x += 64) {
    const uint8_t pk = a.out.pk[a0 + x];
    if (pk & 1u) {
      bool fresh;
      const uint32_t s = lset_put(wk, ST_WM_LOG, a.out.keys[a0 + x], a.out.hsh[a0 + x], fresh);
      if (s == ~0u) full = true;
      else atomicOr((unsigned long long*)&wm[s], 1ull << (pk >> 1));
      hw |= 1ull << (pk >> 1);
      nw++;
    }
  }
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  nw = wave_sum_u32(nw);
  if (hw) atomicOr((unsigned long long*)&L.thw[wv], (unsigned long long)hw);
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  hw = L.thw[wv];
  if (nw)
    for (uint32_t x = lane; x < na; x += 64) {
      const uint8_t pk = a.out.pk[a0 + x];
      const uint32_t t = pk >> 1;
      const uint32_t s = lset_slot(wk, ST_WM_LOG, a.out.keys[a0 + x], a.out.hsh[a0 + x]);
      if (s != ~0u) {
        const uint64_t m = wm[s] & lt_mask(t);
        if (m) atomicOr((unsigned long long*)&tdep[t], (unsigned long long)m);
      }
    }
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  if (lane < nt) a.out.dep[f + lane] = tdep[lane];
  if (lane == 0) {
    uint64_t* d = a.out.tile + (size_t)(tbase + k) * ST_TILE_WORDS;
    d[0] = (uint64_t)f | ((uint64_t)nt << 32);
    d[1] = (uint64_t)a0 | ((uint64_t)na << 32);
    d[2] = nw;
    d[3] = hw;
  }
  if (__any(full) && lane == 0) atomicOr(&a.cur->err, STE_WMAP);
  // empty the map and the masks for the wave's next tile
  __builtin_amdgcn_wave_barrier();
  for (uint32_t q = lane; q < WM_SLOTS; q += 64) {
    wk[q] = KEY_EMPTY;
    wm[q] = 0;
  }
  tdep[lane] = 0;
  if (lane == 0) L.thw[wv] = 0;
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
}

__device__ void stage_filter(const StArgs& a, FilterLds& L, uint32_t g, uint32_t tag) {
  const uint32_t tid = threadIdx.x, w = tid >> 6, lane = lane_id();
  if (a.dbg && tid == 0)
    atomicMin((unsigned long long*)&a.dbg[a.stage * 32 + 19],
              (unsigned long long)__builtin_amdgcn_s_memrealtime());
  // ---- C of the previous decider: bitmap + exact set
  const uint32_t cn = a.prev ? min(a.prev->ckeys_n, CT_SLOTS / 2) : 0u;
  for (uint32_t q = tid; q < (1u << (ST_FB_LOG - 5)); q += ST_B) L.u.c.fb[q] = 0;
  if (cn)
    for (uint32_t q = tid; q < CT_SLOTS; q += ST_B) L.u.c.ct[q] = KEY_EMPTY;
  if (tid < 4) L.cnt[tid] = 0;
  if (tid == 0) L.maxlen = 0;
  __syncthreads();
  for (uint32_t q = tid; q < cn; q += ST_B) {
    const uint64_t k = a.ck_prev[q];
    const uint32_t h = st_hash(k), b = h & ((1u << ST_FB_LOG) - 1u);
    atomicOr(&L.u.c.fb[b >> 5], 1u << (b & 31));
    bool fresh;
    lset_put(L.u.c.ct, ST_CT_LOG, k, h, fresh);
  }
  // ---- this workgroup's input: wave-tiles of 64 txns with contiguous accesses
  uint32_t tbase = 0, abase = 0, stats_from = 0xFFFFFFFFu;
  if (tid == 0) {
    uint32_t n = 0;
    if (a.mode == 0) {
      // stage 0: [0, e_end = P0); stage 1: [begin, n) from the first txn stage
      // 0's decider left undecided.  Stats count every txn once: stage 0 the
      // txns < P0, stage 1 the rest.
      const uint32_t begin = a.stage == 0 ? 0u : st_begin(a);
      const uint32_t b = begin + g * a.ch, e = min(b + a.ch, a.e_end);
      for (uint32_t t = b; t < e && n < ST_WT; t += 64) L.wt[n++] = WaveTile{t, min(64u, e - t), 0u, 0u};
    } else {
      const uint32_t c0 = g * ST_G, c1 = min(c0 + ST_G, a.in_chunks);
      for (uint32_t c = c0; c < c1; c++) {
        const uint32_t ht = a.in.hdr[c].tbase, hn = a.in.hdr[c].nt;
        uint32_t s = ht;
        if (c < a.prev->stop_chunk) continue;
        if (c == a.prev->stop_chunk) s += a.prev->stop_idx;
        for (uint32_t t = s; t < ht + hn; t += 64) {
          if (n == ST_WT) {
            atomicOr(&a.cur->err, STE_WMAP);  // more than 64 wave-tiles: not sized for it
            break;
          }
          L.wt[n++] = WaveTile{t, min(64u, ht + hn - t), 1u, 0u};
        }
      }
    }
    L.nwt = n;
  }
  if (a.mode == 0) {
    const uint32_t begin = a.stage == 0 ? 0u : st_begin(a);
    stats_from = a.stage == 0 ? 0u : a.p0;
    tbase = min(begin + g * a.ch, a.n);
    abase = a.off[tbase];
  } else {
    const uint32_t c0 = g * ST_G;
    tbase = a.in.hdr[c0].tbase;
    abase = a.in.hdr[c0].abase;
  }
  __syncthreads();
  const uint32_t nwt = L.nwt;
  uint32_t err = 0, in_n = 0;
  // ---- streaming pass: every wave-tile of the workgroup at once
  for (uint32_t k = w; k < nwt; k += ST_W) {
    const WaveTile wt = L.wt[k];
    in_n += lane == 0 ? wt.nt : 0u;
    uint64_t sv;
    uint32_t sa;
    filter_wave_tile(a, L, w, wt, cn != 0, stats_from, sv, sa, err);
    if (lane == 0) {
      L.smask[k] = sv;
      L.scnt[k] = (uint32_t)__builtin_popcountll(sv);
      L.sacc[k] = sa;
    }
  }
  __syncthreads();
  if (w == 0) {
    // exclusive prefix over the wave-tiles (nwt <= 64 = one wave)
    const uint32_t cc = lane < nwt ? L.scnt[lane] : 0u;
    const uint32_t ac = lane < nwt ? L.sacc[lane] : 0u;
    const uint32_t pc = wave_excl_sum(cc), pa = wave_excl_sum(ac);
    if (lane < nwt) {
      L.spos[lane] = pc;
      L.sapos[lane] = pa;
    }
  }
  __syncthreads();
  const uint32_t out_t = nwt ? L.spos[nwt - 1] + L.scnt[nwt - 1] : 0u;
  const uint32_t out_a = nwt ? L.sapos[nwt - 1] + L.sacc[nwt - 1] : 0u;
  // tiles of T survivors: <= ST_TILE_ACC accesses each (MAX_ROW_PER_TXN = 64)
  const uint32_t T = L.maxlen > 32 ? 16u : L.maxlen > 16 ? 32u : ST_TILE;
  // ---- survivors out, then the killed txns' decisions (stores last)
  for (uint32_t k = w; k < nwt; k += ST_W) {
    const WaveTile wt = L.wt[k];
    const uint64_t sm = L.smask[k];
    if (sm) filter_copy(a, wt, sm, L.spos[k], L.sapos[k], tbase, abase, T);
    if (lane < wt.nt && !((sm >> lane) & 1ull)) {
      const uint32_t x = wt.mode == 0 ? wt.t0 + lane : a.in.tid[wt.t0 + lane];
      a.rc[x] = RC_AB;
      if (a.tn) a.tn[x] = 0;
    }
  }
  // ---- tiles for the next decider (published chunks only: the others are
  // read by the next stage's filter, which needs no tiles)
  const bool pub = a.decide && g < a.gpub;
  const uint32_t ntiles = pub ? (out_t + T - 1) / T : 0u;
  if (ntiles) {
    __builtin_amdgcn_s_waitcnt(0);  // the copies above are read back below
    __syncthreads();
    for (uint32_t q = tid; q < ST_WM_WAVES * WM_SLOTS; q += ST_B) {
      (&L.u.t.wk[0][0])[q] = KEY_EMPTY;
      (&L.u.t.wm[0][0])[q] = 0;
    }
    for (uint32_t q = tid; q < ST_WM_WAVES * ST_TILE; q += ST_B) (&L.tdep[0][0])[q] = 0;
    if (tid < ST_WM_WAVES) L.thw[tid] = 0;
    __syncthreads();
    if (w < ST_WM_WAVES)
      for (uint32_t k = w; k < ntiles; k += ST_WM_WAVES) filter_build_tile(a, L, w, k, out_t, tbase, T);
  }
  // ---- chunk header, totals, publication
  if (err) atomicOr(&a.cur->err, err);
  in_n = wave_sum_u32(in_n);
  if (lane == 0 && in_n) atomicAdd(&a.cur->in_n, in_n);
  __syncthreads();
  if (tid == 0) {
    StChunk& h = a.out.hdr[g];
    h.nt = out_t;
    h.na = out_a;
    h.tbase = tbase;
    h.abase = abase;
    h.ntiles = ntiles;
    if (out_t) {
      atomicAdd(&a.cur->surv_n, out_t);
      atomicAdd(&a.cur->surv_acc, out_a);
    }
    if (L.cnt[0]) atomicAdd(&a.cur->nnz_w, L.cnt[0]);
    if (L.cnt[1]) atomicAdd(&a.cur->ro, L.cnt[1]);
  }
  if (a.dbg && tid == 0) {
    const uint64_t now = __builtin_amdgcn_s_memrealtime();
    atomicMax((unsigned long long*)&a.dbg[a.stage * 32 + 16], (unsigned long long)now);
    if (pub) atomicMax((unsigned long long*)&a.dbg[a.stage * 32 + 17], (unsigned long long)now);
    atomicMin((unsigned long long*)&a.dbg[a.stage * 32 + 18], (unsigned long long)now);
  }
  if (pub) {
    // every storing wave drains its stores, the workgroup joins, one lane
    // releases and raises the flag
    __builtin_amdgcn_s_waitcnt(0);
    __syncthreads();
    if (tid == 0) {
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __hip_atomic_store(&a.out.hdr[g].flag, tag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
}

// ------------------------------------------------------------------ decider
#define ST_STAMP(k)                                                                             \
  do {                                                                                          \
    if (a.dbg && threadIdx.x == 0) a.dbg[a.stage * 32 + (k)] = __builtin_amdgcn_s_memrealtime(); \
  } while (0)

// A loader thread's share of one tile in flight: accesses x = j + 256 i of
// the tile (j = thread index within its loader group) and dependency mask j.
struct LoadBuf {
  uint64_t k[4];
  uint32_t h[4];
  uint32_t p[4];
  uint64_t dep;
  uint32_t na, nt;
};

__device__ void stage_decider(const StArgs& a, DeciderLds& L, uint32_t tag) {
  const uint32_t tid = threadIdx.x, w = tid >> 6, lane = lane_id();
  ST_STAMP(0);
  for (uint32_t q = tid; q < CS_SLOTS; q += ST_B) L.cs[q] = KEY_EMPTY;
  for (uint32_t q = tid; q < (1u << (ST_CB_LOG - 5)); q += ST_B) L.cb[q] = 0;
  if (tid == 0) {
    L.dead = 0;
    L.nst = 0;
    L.ckn = 0;
    L.err = 0;
  }
  const uint32_t need = min(min(a.gpub, a.out_chunks), ST_MAX_PUB);
  // ---- wait for every published chunk, then one acquire
  if (tid < need) {
    uint32_t it = 0;
    while (__hip_atomic_load(&a.out.hdr[tid].flag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != tag) {
      __builtin_amdgcn_s_sleep(2);
      if (++it > (1u << 24)) {
        atomicOr(&L.err, STE_SPIN);
        break;
      }
    }
  }
  __syncthreads();
  ST_STAMP(1);
  if (tid == 0) {
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  __syncthreads();
  // ---- flat tile index over the chunks, descriptors into LDS
  {
    const uint32_t v = tid < need ? a.out.hdr[tid].ntiles : 0u;
    if (tid < need) L.ttb[tid] = a.out.hdr[tid].tbase;
    const uint32_t ex = wave_excl_sum(v);
    if (lane == 63) L.wsum[w] = ex + v;
    __syncthreads();
    uint32_t before = 0;
    for (uint32_t q = 0; q < w; q++) before += L.wsum[q];
    if (tid < need) L.tpref[tid] = before + ex;
    if (tid == 0) {
      uint32_t t = 0;
      for (uint32_t q = 0; q < ST_W; q++) t += L.wsum[q];
      L.tpref[need] = t;
    }
    __syncthreads();
  }
  const uint32_t Q = L.err ? 0u : min(L.tpref[need], ST_MAX_TILES);
  for (uint32_t q = tid; q < Q; q += ST_B) {
    uint32_t lo = 0, hi = need;  // tpref[lo] <= q < tpref[hi]
    while (hi - lo > 1) {
      const uint32_t mid = (lo + hi) >> 1;
      if (L.tpref[mid] <= q) lo = mid;
      else hi = mid;
    }
    const uint64_t* d = a.out.tile + (size_t)(L.ttb[lo] + (q - L.tpref[lo])) * ST_TILE_WORDS;
#pragma unroll
    for (uint32_t i = 0; i < ST_TILE_WORDS; i++) L.desc[q][i] = d[i];
  }
  __syncthreads();
  ST_STAMP(2);
  // ---- roles.  Waves [0, 4) decide tile t in period t from LDS slot t & 1;
  // loader group g (waves 4 + 4g .. 8 + 4g) owns tiles t = g mod 3: it
  // issues their loads in period t - 3 and writes them into the slot in
  // period t - 1, so a load has two periods to land and the deciders never
  // wait on global memory.  Every wave passes the same two barriers per
  // period (LDS-only barriers: no vmcnt drain).
  const bool decider = w < ST_DEC_WAVES;
  const uint32_t lg = decider ? 0u : (w - ST_DEC_WAVES) / 4;  // loader group
  const uint32_t lj = tid - (ST_DEC_WAVES + 4 * lg) * 64;     // thread within the group
  LoadBuf LB;
  LB.na = LB.nt = 0;
  auto lissue = [&](uint32_t t) {  // loads of tile t into LB (loader threads)
    const uint32_t tt = min(t, Q ? Q - 1 : 0u);
    const uint64_t d0 = L.desc[tt][0], d1 = L.desc[tt][1];
    const uint32_t f = (uint32_t)d0;
    LB.nt = t < Q ? (uint32_t)(d0 >> 32) : 0u;
    LB.na = t < Q ? (uint32_t)(d1 >> 32) : 0u;
    const uint32_t a0 = (uint32_t)d1;
#pragma unroll
    for (uint32_t i = 0; i < 4; i++) {
      const uint32_t x = lj + 256 * i;
      const uint32_t ix = a0 + (LB.na ? min(x, LB.na - 1) : 0u);
      LB.k[i] = a.out.keys[ix];
      LB.h[i] = a.out.hsh[ix];
      LB.p[i] = a.out.pk[ix];
    }
    LB.dep = a.out.dep[f + (LB.nt ? min(lj, LB.nt - 1) : 0u)];
  };
  auto lwrite = [&](uint32_t t) {  // LB (tile t) into slot t & 1
    DeciderLds::Slot& S = L.slot[t & 1u];
#pragma unroll
    for (uint32_t i = 0; i < 4; i++) {
      const uint32_t x = lj + 256 * i;
      if (x < LB.na) {
        S.k[x] = LB.k[i];
        S.h[x] = LB.h[i];
        S.p[x] = (uint8_t)LB.p[i];
      }
    }
    if (lj < ST_TILE) S.dep[lj] = lj < LB.nt ? LB.dep : 0ull;
  };
  if (!decider && Q) {
    if (lg < Q) lissue(lg);  // tiles 0, 1, 2
    if (lg == 0) lwrite(0);
  }
  lds_barrier();
  uint64_t cyc1 = 0, cyc2 = 0, cyc3 = 0;
  uint32_t commits = 0, cw = 0, decided = 0;
  uint32_t q = 0;
  for (; q < Q; q++) {
    const uint64_t c_a = a.dbg ? __builtin_amdgcn_s_memtime() : 0;
    const uint64_t d0 = L.desc[q][0], d1 = L.desc[q][1], nw = L.desc[q][2], hwm = L.desc[q][3];
    const uint32_t f = (uint32_t)d0, nt = (uint32_t)(d0 >> 32), na = (uint32_t)(d1 >> 32);
    // stop before C would exceed its budget or the decided txns pmax
    // (every wave evaluates the same LDS values)
    if (q > 0 && (L.ckn + nw > ST_CS_BUDGET || decided + nt > a.pmax)) break;
    uint64_t kx[4] = {0, 0, 0, 0};
    uint32_t hx[4] = {0, 0, 0, 0}, px[4] = {0, 0, 0, 0};
    if (decider) {
      // ---- probe C (dead bits); stash the write accesses for the inserts
      const DeciderLds::Slot& S = L.slot[q & 1u];
#pragma unroll
      for (uint32_t i = 0; i < 4; i++) {
        const uint32_t x = tid + 256 * i;
        if (x < na) {
          kx[i] = S.k[x];
          hx[i] = S.h[x];
          px[i] = S.p[x] | 0x100u;
        }
      }
      uint64_t dm = 0;
#pragma unroll
      for (uint32_t i = 0; i < 4; i++) {
        const uint32_t p = px[i];
        if ((p & 0x100u) && !(a.xflags & 2)) {
          const uint32_t b = hx[i] & ((1u << ST_CB_LOG) - 1u);
          if ((L.cb[b >> 5] >> (b & 31)) & 1u)
            if (lset_has(L.cs, ST_CS_LOG, kx[i], hx[i])) dm |= 1ull << ((p & 0xFFu) >> 1);
        }
        const bool wr = (p & 0x101u) == 0x101u && !(a.xflags & 4);
        const uint64_t bw = __ballot(wr);
        if (bw) {
          uint32_t base = 0;
          if (lane == 0) base = atomicAdd(&L.nst, (uint32_t)__builtin_popcountll(bw));
          base = lane_bcast(base, 0);
          if (wr) {
            const uint32_t s = base + (uint32_t)__builtin_popcountll(bw & lt_mask(lane));
            L.stk[s] = kx[i];
            L.sth[s] = hx[i];
            L.stt[s] = (uint8_t)((p & 0xFFu) >> 1);
          }
        }
      }
      if (dm) atomicOr((unsigned long long*)&L.dead, (unsigned long long)dm);  // rare: per lane
    } else if (!(a.xflags & 16)) {
      // ---- loaders: write tile q + 1 (its group's loads issued two periods
      // ago), issue tile q + 3
      if (lg == (q + 1) % ST_LOAD_GROUPS && q + 1 < Q) lwrite(q + 1);
      if (lg == q % ST_LOAD_GROUPS && q + 3 < Q) lissue(q + 3);
    }
    lds_barrier();  // B1: dead bits and the write stash are complete
    const uint64_t c_b = a.dbg ? __builtin_amdgcn_s_memtime() : 0;
    // ---- one wave: the tile's serial decision, then committed write keys join C
    if (w == 0) {
      const uint64_t vmask = nt == 64 ? ~0ull : ((1ull << nt) - 1ull);
      const uint64_t dl = lane < nt ? L.slot[q & 1u].dep[lane] : 0ull;
      // alive txns with no earlier writer in the tile commit at once; the
      // others ("contested", dep != 0) in index order, each committing iff
      // none of its in-tile earlier writers did
      const uint64_t alive = ~L.dead & vmask;
      const uint64_t contested = __ballot(dl != 0) & alive;
      uint64_t commit = alive & ~contested;
      if (!(a.xflags & 8)) {
        const uint32_t dlo = (uint32_t)dl, dhi = (uint32_t)(dl >> 32);
        uint64_t m = contested;
        while (m) {
          const uint32_t t = (uint32_t)__builtin_ctzll(m);
          m &= m - 1;
          const uint64_t dt = ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)dhi, (int)t) << 32) |
                              (uint32_t)__builtin_amdgcn_readlane((int)dlo, (int)t);
          if (!(dt & commit)) commit |= 1ull << t;
        }
      }
      const uint32_t ns = L.nst;
      uint32_t ins = 0;
      for (uint32_t s = lane; s < ns; s += 64) {
        if ((commit >> L.stt[s]) & 1ull) {
          bool fresh;
          const uint32_t h = L.sth[s];
          lset_put(L.cs, ST_CS_LOG, L.stk[s], h, fresh);
          const uint32_t b = h & ((1u << ST_CB_LOG) - 1u);
          atomicOr(&L.cb[b >> 5], 1u << (b & 31));
          ins++;
        }
      }
      ins = (uint32_t)__builtin_popcountll(__ballot(ins & 1u)) +
            2u * (uint32_t)__builtin_popcountll(__ballot(ins & 2u)) +
            4u * (uint32_t)__builtin_popcountll(__ballot(ins & 4u)) +
            8u * (uint32_t)__builtin_popcountll(__ballot(ins & ~7u));
      if (lane == 0) {
        L.ckn += ins;
        L.dead = 0;
        L.nst = 0;
        L.tslot[q] = f;
        L.tcom[q] = commit;
        L.thw[q] = hwm & vmask;
        L.tnt[q] = nt;
      }
      cw += (uint32_t)__builtin_popcountll(commit & hwm & vmask);
      commits += (uint32_t)__builtin_popcountll(commit);
    }
    decided += nt;
    const uint64_t c_c = a.dbg ? __builtin_amdgcn_s_memtime() : 0;
    lds_barrier();  // B2: C is complete, slot q + 1 written
    if (a.dbg) {
      const uint64_t c_d = __builtin_amdgcn_s_memtime();
      cyc1 += c_b - c_a;
      cyc2 += c_c - c_b;
      cyc3 += c_d - c_c;
    }
  }
  __syncthreads();  // loaders' last loads drained
  ST_STAMP(3);
  // ---- decisions of the decided tiles: rc, tn (central_finish numbering)
  commits = __shfl(commits, 0);  // wave 0 counted them
  cw = __shfl(cw, 0);
  if (w == 0) {
    L.wsum[0] = commits;
    L.wsum[1] = cw;
  }
  __syncthreads();
  commits = L.wsum[0];
  cw = L.wsum[1];
  uint64_t tnc = a.ep->tnc;
  {
    uint64_t base = tnc;
    for (uint32_t q0 = 0; q0 < q; q0 += ST_W) {
      const uint32_t qq = q0 + w;
      uint32_t before = 0;
      for (uint32_t x = q0; x < qq && x < q; x++) before += (uint32_t)__builtin_popcountll(L.tcom[x] & L.thw[x]);
      if (qq < q && lane < L.tnt[qq]) {
        const uint32_t x = a.out.tid[L.tslot[qq] + lane];
        const uint64_t cm = L.tcom[qq], hm = L.thw[qq];
        const bool c1 = (cm >> lane) & 1ull;
        a.rc[x] = c1 ? RC_OK : RC_AB;
        if (a.tn) {
          const bool h1 = (hm >> lane) & 1ull;
          a.tn[x] = (c1 && h1) ? base + before + 1 + (uint64_t)__builtin_popcountll(cm & hm & lt_mask(lane)) : 0ull;
        }
      }
      for (uint32_t x = q0; x < q0 + ST_W && x < q; x++) base += (uint32_t)__builtin_popcountll(L.tcom[x] & L.thw[x]);
    }
    tnc = base;
  }
  // ---- C: the committed keys, for the next stage's filter
  __syncthreads();
  if (tid == 0) L.ckn = 0;
  __syncthreads();
  for (uint32_t s0 = 0; s0 < CS_SLOTS; s0 += ST_B) {
    const uint64_t k = L.cs[s0 + tid];
    const bool v = k != KEY_EMPTY;
    const uint64_t bm = __ballot(v);
    uint32_t pos = 0;
    if (lane == 0 && bm) pos = atomicAdd(&L.ckn, (uint32_t)__builtin_popcountll(bm));
    pos = lane_bcast(pos, 0);
    if (v) a.ck_cur[pos + (uint32_t)__builtin_popcountll(bm & lt_mask(lane))] = k;
  }
  __syncthreads();
  if (a.dbg && tid == 0) {
    a.dbg[a.stage * 32 + 4] = cyc1;
    a.dbg[a.stage * 32 + 5] = cyc2;
    a.dbg[a.stage * 32 + 6] = cyc3;
    a.dbg[a.stage * 32 + 7] = q;
    a.dbg[a.stage * 32 + 8] = decided;
    a.dbg[a.stage * 32 + 9] = need;
  }
  // ---- the stop point (first txn not decided: a tile start), counters
  if (tid == 0) {
    StCtl* c = a.cur;
    c->ran = 1;
    c->consumed = decided;
    uint32_t sc = need, sidx = 0, stid = 0xFFFFFFFFu;
    if (q < L.tpref[need]) {
      uint32_t lo = 0, hi = need;
      while (hi - lo > 1) {
        const uint32_t mid = (lo + hi) >> 1;
        if (L.tpref[mid] <= q) lo = mid;
        else hi = mid;
      }
      const uint32_t f = q < Q ? (uint32_t)L.desc[q][0]
                               : (uint32_t)a.out.tile[(size_t)(L.ttb[lo] + (q - L.tpref[lo])) * ST_TILE_WORDS];
      sc = lo;
      sidx = f - L.ttb[lo];
      stid = a.out.tid[f];
    }
    c->stop_chunk = sc;
    c->stop_idx = sidx;
    c->stop_tid = stid;
    c->commits = commits;
    c->cw = cw;
    c->ckeys_n = L.ckn;
    c->tiles = q;
    if (L.err) atomicOr(&c->err, L.err);
    a.ep->tnc = tnc;
  }
}

__global__ __launch_bounds__(ST_B) void k_stage(StArgs a) {
  __shared__ StLds lds;
  const uint32_t tag = st_tag(a.ep->gen, a.stage);
  // Skip the stage when its input is empty or the solver handed off.
  bool skip = false, ab = false;
  if (a.stage > 0) {
    const StCtl* p = a.prev;
    if (p->err || p->abandon) {
      skip = true;
      ab = p->abandon != 0;
    }
    if (a.mode == 0) {
      if (st_begin(a) >= a.e_end) skip = true;
    } else if (p->surv_n <= p->consumed) {
      skip = true;
    } else if (p->surv_n > 65536u &&
               4ull * p->surv_n > (a.stage == 2 ? 1ull : 3ull) * (uint64_t)p->in_n) {
      // the list stopped shrinking: hand it to the round solver
      skip = true;
      ab = true;
    }
  }
  if (blockIdx.x == 0 && a.decide) {
    if (threadIdx.x == 0) {
      if (a.next) *a.next = StCtl{};
      if (ab) a.cur->abandon = 1;
    }
    if (skip) return;
    stage_decider(a, lds.d, tag);
    return;
  }
  if (skip) return;
  stage_filter(a, lds.f, blockIdx.x - (a.decide ? 1u : 0u), tag);
}

__global__ __launch_bounds__(256) void k_stage_final(StFinalArgs a) {
  const uint32_t words = (uint32_t)((sizeof(StEpoch) + a.n_ctl * sizeof(StCtl)) / 4);
  uint32_t* h = (uint32_t*)a.host;
  const uint32_t* e = (const uint32_t*)a.ep;
  const uint32_t* c = (const uint32_t*)a.ctl;
  const uint32_t ew = (uint32_t)(sizeof(StEpoch) / 4);
  for (uint32_t q = threadIdx.x; q < words; q += blockDim.x) h[q] = q < ew ? e[q] : c[q - ew];
  __syncthreads();
  if (threadIdx.x == 0) {
    a.ep->gen++;
    a.ctl[0] = StCtl{};
  }
}

void launch_stage(const StArgs& a, hipStream_t st) {
  const unsigned grid = a.out_chunks + (a.decide ? 1u : 0u);
  k_stage<<<grid, ST_B, 0, st>>>(a);
}
void launch_stage_final(const StFinalArgs& a, hipStream_t st) {
  k_stage_final<<<1, 256, 0, st>>>(a);
}

}  // namespace dcc
