// gfx950 kernels of the OCC commit/kill round solver: decides
// the list the level-0 sweep leaves behind (its survivors, in index order).
//
// The serial decision (central_validate in index order, occ.cpp:116-239,
// then central_finish) is
//
//   abort(t)  <=>  some EARLIER committed txn wrote a key t reads or writes
//
// A key's first committed writer kills every later accessor, so each key has
// at most one committed writer.  Round r decides every list txn whose fate no
// longer depends on an undecided earlier txn:
//
//   u_r(K)   the smallest writer of key K still undecided after round r - 1
//   c(K)     K's committed writer (set once)
//
//   t commits in round r   <=>  no key K of t has c(K) < t or u_r(K) < t
//   t aborts  in round r   <=>  some key K of t has c(K) < t once round r's
//                               commits are in c
//
// Every kill a round's commits cause lands in that same round (the only
// writer of K that can commit in round r is u_r(K): any later writer is
// blocked by it), so a round is two phases: commits, then kills.  Decisions
// are final and equal the serial replay's; the smallest undecided txn always
// decides, so the rounds terminate.  For the headline batch (1M YCSB txns,
// theta 0.9) the 100,800 survivors of level 0 take 8 rounds (35,896 / 14,841 /
// 5,776 / 1,871 / 490 / 80 / 5 / 0 left).
//
//   k_ck_build   (grid)  key table over the list's write accesses: each gets
//                        its key's slot (32 B: key, c, u_r for two round
//                        parities) and publishes u_1; round 1 then finds the
//                        reads' slots with read-only probes (a key no list
//                        txn writes cannot conflict)
//   k_ck_phase   (grid)  one round in two launches (commits, then kills), a
//                        16-lane group per undecided txn (lane per access);
//                        decisions go to the list's and the epoch's state
//                        bytes, survivors publish u_{r+1} (the other
//                        parity's word, tagged with the round)
//
// The table stays clean between epochs: k_final resets every slot the list
// used (its accesses' slots), so no epoch clears the table wholesale.
#include <hip/hip_runtime.h>

#include "dcc_device.h"
#include "occ_kernels.h"

namespace dcc {

// u words: (0xFFFFFFFF - round) << 32 | list position.  Newer rounds carry
// smaller high words, so one atomicMin both replaces a stale word of round
// r - 2 (same parity) and keeps the round's minimum writer; a clean slot
// (all ones) has no round.
__device__ inline uint64_t ck_uword(uint32_t r, uint32_t t) {
  return ((uint64_t)(0xFFFFFFFFu - r) << 32) | t;
}
__device__ inline bool ck_blocks(uint64_t u, uint32_t r, uint32_t t) {
  return (uint32_t)(u >> 32) == 0xFFFFFFFFu - r && (uint32_t)u < t;
}

__device__ inline uint32_t ck_hash(uint64_t key, uint32_t mask) {
  return (uint32_t)(fmix64(key) >> 32) & mask;
}

// slot of a key: linear probing over 32-B slots; a plain read first, so only
// the first accessors of a key pay an atomic (memory-side, serialised per
// word: a hot key's thousands of accessors must not all CAS).  A stale EMPTY
// (this XCD's L2 held the line before another XCD's CAS landed) costs one
// CAS, which returns the truth and drops the stale line; a slot never
// changes once set, so a non-empty read is exact.  The table is at <= 50 %
// load of the list's accesses.
__device__ inline uint32_t ck_insert(CkSlot* tab, uint32_t mask, uint64_t key) {
  uint32_t h = ck_hash(key, mask);
  for (uint32_t n = 0; n <= mask; n++) {
    const uint64_t cur = __hip_atomic_load(&tab[h].key, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (cur == key) return h;
    if (cur == KEY_EMPTY) {
      const unsigned long long prev = atomicCAS((unsigned long long*)&tab[h].key,
                                                (unsigned long long)KEY_EMPTY,
                                                (unsigned long long)key);
      if (prev == KEY_EMPTY || prev == key) return h;
    }
    h = (h + 1) & mask;
  }
  return CK_NONE;  // unreachable at <= 50 % load
}

// slot of a key entered by k_ck_build, or CK_NONE (no list txn writes it)
__device__ inline uint32_t ck_find(const CkSlot* tab, uint32_t mask, uint64_t key) {
  uint32_t h = ck_hash(key, mask);
  for (uint32_t n = 0; n <= mask; n++) {
    const uint64_t cur = tab[h].key;
    if (cur == key) return h;
    if (cur == KEY_EMPTY) return CK_NONE;
    h = (h + 1) & mask;
  }
  return CK_NONE;
}

// atomicMin behind a read filter (a stale read is only ever higher)
__device__ inline void ck_umin(uint64_t* p, uint64_t v) {
  if (v < __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT))
    atomicMin((unsigned long long*)p, (unsigned long long)v);
}

// A txn is handled by a group of CK_G lanes, lane li holding accesses
// li, li + CK_G, ... (up to CK_C per lane: MAX_ROW_PER_TXN = CK_G * CK_C).
// Group masks of ballots: bits [gi * CK_G, gi * CK_G + CK_G).
__device__ inline uint64_t ck_gmask(uint32_t gi) {
  return (CK_G == 64 ? ~0ull : ((1ull << CK_G) - 1ull)) << (gi * CK_G);
}

// ---------------------------------------------------------------------------
// k_ck_build: a group per list txn; each lane enters its WRITE accesses'
// keys in the table (slot per access) and publishes u_1 for them.
__global__ __launch_bounds__(256) void k_ck_build(CkArgs a) {
  // round 1 sets live flag 2 (rounds zero the flags two ahead)
  if (blockIdx.x == 0 && threadIdx.x == 0) a.ctl[CK_CTL_RING + 2] = 0;
  if (*a.abandon) return;
  const uint32_t m = a.lv1->m, acc = a.lv1->acc;
  if (m == 0) return;
  uint32_t bits = 10;
  while (bits < 31 && (1ull << bits) < 2ull * acc) bits++;
  if (bits > a.cap_bits) {  // list too large for the table: the round solver takes it
    if (blockIdx.x == 0 && threadIdx.x == 0) atomicMax(a.abandon_out, a.abandon_level);
    return;
  }
  const uint32_t mask = (1u << bits) - 1u;
  if (blockIdx.x == 0 && threadIdx.x == 0) a.ctl[CK_CTL_MASK] = mask;
  const uint32_t li = lane_id() % CK_G;
  const uint32_t ng = gridDim.x * (blockDim.x / CK_G);
  bool bad = false;
  for (uint32_t t = (blockIdx.x * blockDim.x + threadIdx.x) / CK_G; t < m; t += ng) {
    if (li == 0) a.s1[t] = ST_UNDECIDED;  // (u32 state word per list position)
    const uint32_t s = a.off1[t], e = a.off1[t + 1];
    uint64_t key[CK_C];
    uint8_t at[CK_C];
#pragma unroll
    for (uint32_t c = 0; c < CK_C; c++) {
      const uint32_t q = s + li + CK_G * c;
      key[c] = q < e ? a.keys1[q] : KEY_EMPTY;
      at[c] = q < e ? a.at1[q] : (uint8_t)0;
    }
#pragma unroll
    for (uint32_t c = 0; c < CK_C; c++) {
      const uint32_t q = s + li + CK_G * c;
      // writes only (WR, occ.cpp:296-317: only WR joins the write set): a
      // key no list txn writes can neither block nor kill; round 1 finds
      // the reads' keys with read-only probes
      if (q >= e || at[c] != 1) continue;
      if (key[c] == KEY_EMPTY) {  // the reserved key: reported, never a conflict
        bad = true;
        a.aslot[q] = CK_NONE;
        continue;
      }
      const uint32_t sl = ck_insert(a.tab, mask, key[c]);
      a.aslot[q] = sl | CK_WR;
      ck_umin(&a.tab[sl].u[1], ck_uword(1, t));
    }
  }
  if (bad) atomicOr(a.err, ERR_KEY);
}

// ---------------------------------------------------------------------------
// Round r in two launches over the list's undecided txns, a group of CK_G
// lanes per txn:
//   k_ck_phase<false>  t aborts if a key has a committed writer before it;
//                      commits if no key has a committed or an undecided
//                      (u_r) writer before it -- and then becomes its write
//                      keys' c;
//   k_ck_phase<true>   the txns left undecided: a committed writer before
//                      them now (this round's commits included: the only
//                      writer of K that can commit in round r is u_r(K))
//                      aborts them, the others publish u_{r+1}.
// (One launch per round with the kill read off the blockers' state words
// measured 16 rounds instead of 8 at the headline: the blockers are decided
// concurrently with the txns they block, so their commits are rarely
// visible yet.)  No list is compacted between rounds (a single list counter
// would take one memory-side atomic per wave, ~88 per us on one word): each
// wave takes 64 list positions, ballots their state words and runs its
// undecided txns four at a time.  Each phase is then one round trip for the
// txn's slots and one for their words; a wave that keeps a txn undecided
// marks the next round live with a plain store of 1 (no atomic).
template <bool KILL>
__global__ __launch_bounds__(256) void k_ck_phase(CkArgs a, uint32_t r) {
  uint32_t* live = a.ctl + CK_CTL_RING;
  // the flag two rounds on is free again (round r + 1 sets r + 2)
  if (!KILL && blockIdx.x == 0 && threadIdx.x == 0) live[(r + 2) % CK_RING] = 0;
  if (*a.abandon) return;
  const uint32_t m = a.lv1->m;
  if (m == 0 || (r > 1 && live[r % CK_RING] == 0)) return;
  const uint32_t lane = lane_id(), li = lane % CK_G, gi = lane / CK_G;
  const uint64_t gm = ck_gmask(gi);
  const uint32_t nw = gridDim.x * (blockDim.x / 64);
  const uint32_t wid = blockIdx.x * (blockDim.x / 64) + (threadIdx.x >> 6);
  const uint32_t ru = r & 1, rn = (r + 1) & 1;
  const uint32_t mask = a.ctl[CK_CTL_MASK];
  bool any_stay = false;
  for (uint32_t c0 = wid * 64; c0 < m; c0 += nw * 64) {  // wave-uniform
    const uint32_t p = c0 + lane;
    uint64_t und = ballot64(p < m && a.s1[p] == ST_UNDECIDED);
    while (und) {  // wave-uniform: four undecided txns per step, one per group
      uint64_t mk4 = und;
      uint32_t t = ~0u;
      for (uint32_t g = 0; g < 64 / CK_G && mk4; g++) {
        const uint32_t b = (uint32_t)__builtin_ctzll(mk4);
        if (g == gi) t = c0 + b;
        mk4 &= mk4 - 1;
      }
      und = mk4;
      if (t == ~0u) continue;  // this group has no txn in the step
      const uint32_t s = a.off1[t], e = a.off1[t + 1];
      uint32_t as[CK_C];
      if (!KILL && r == 1) {
        // round 1: the reads' slots (read-only probes of the write keys)
        uint64_t key[CK_C];
        uint8_t at[CK_C];
#pragma unroll
        for (uint32_t c = 0; c < CK_C; c++) {
          const uint32_t q = s + li + CK_G * c;
          key[c] = q < e ? a.keys1[q] : KEY_EMPTY;
          at[c] = q < e ? a.at1[q] : (uint8_t)1;
        }
#pragma unroll
        for (uint32_t c = 0; c < CK_C; c++) {
          const uint32_t q = s + li + CK_G * c;
          as[c] = CK_NONE;
          if (q >= e) continue;
          if (at[c] == 1) {
            as[c] = a.aslot[q];
          } else {
            if (key[c] != KEY_EMPTY) as[c] = ck_find(a.tab, mask, key[c]);
            a.aslot[q] = as[c];
          }
        }
      } else {
#pragma unroll
        for (uint32_t c = 0; c < CK_C; c++) {
          const uint32_t q = s + li + CK_G * c;
          as[c] = q < e ? a.aslot[q] : CK_NONE;
        }
      }
      bool mk = false, mb = false;
#pragma unroll
      for (uint32_t c = 0; c < CK_C; c++) {
        if (as[c] == CK_NONE) continue;
        const CkSlot* sl = a.tab + (as[c] & ~CK_WR);
        mk |= sl->c < t;
        if (!KILL) mb |= ck_blocks(sl->u[ru], r, t);
      }
      const bool kill = (ballot64(mk) & gm) != 0;
      const bool blk = (ballot64(mb) & gm) != 0;
      const bool lead = li == 0;
      if (kill) {
        if (lead) {
          a.s1[t] = ST_ABORT;
          a.state[a.tid1[t]] = ST_ABORT;
        }
      } else if (!KILL && !blk) {
#pragma unroll
        for (uint32_t c = 0; c < CK_C; c++)
          if (as[c] != CK_NONE && (as[c] & CK_WR)) atomicMin(&a.tab[as[c] & ~CK_WR].c, t);
        if (lead) {
          a.s1[t] = ST_COMMIT;
          a.state[a.tid1[t]] = ST_COMMIT;
        }
      } else if (KILL) {
        any_stay = true;
        const uint64_t w1 = ck_uword(r + 1, t);
#pragma unroll
        for (uint32_t c = 0; c < CK_C; c++)
          if (as[c] != CK_NONE && (as[c] & CK_WR)) ck_umin(&a.tab[as[c] & ~CK_WR].u[rn], w1);
      }
    }
  }
  if (KILL && ballot64(any_stay) && lane == 0) live[(r + 1) % CK_RING] = 1;
}

// k_ck_fill: every slot clean (a new or grown table)
__global__ __launch_bounds__(256) void k_ck_fill(CkSlot* tab, uint64_t n) {
  for (uint64_t q = (uint64_t)blockIdx.x * 256 + threadIdx.x; q < n; q += (uint64_t)gridDim.x * 256) {
    CkSlot s;
    s.key = KEY_EMPTY;
    s.c = ~0u;
    s.pad = 0;
    s.u[0] = ~0ull;
    s.u[1] = ~0ull;
    tab[q] = s;
  }
}

void launch_ck_build(const CkArgs& a, unsigned grid, hipStream_t st) {
  k_ck_build<<<grid ? grid : 1u, 256, 0, st>>>(a);
}
void launch_ck_round(const CkArgs& a, uint32_t r, unsigned grid, hipStream_t st) {
  k_ck_phase<false><<<grid ? grid : 1u, 256, 0, st>>>(a, r);
  k_ck_phase<true><<<grid ? grid : 1u, 256, 0, st>>>(a, r);
}
void launch_ck_fill(CkSlot* tab, uint64_t n, hipStream_t st) {
  const uint64_t g = (n + 255) / 256;
  k_ck_fill<<<(unsigned)(g < 4096 ? (g ? g : 1) : 4096), 256, 0, st>>>(tab, n);
}

}  // namespace dcc
