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
//   t aborts  in round r   <=>  some key K of t has c(K) < t, or u_r(K) = j < t
//                               and j commits in round r
//
// The second abort rule looks one hop ahead: j's round-r commit test reads
// only u_r and c, so t can evaluate it itself, and every kill a round's
// commits cause lands in that same round (the only writer of K that can
// commit in round r is u_r(K): any later writer is blocked by it).  Decisions
// are final and equal the serial replay's; the smallest undecided txn always
// decides, so the rounds terminate.  For the headline batch (1M YCSB txns,
// theta 0.9) the 100,800 survivors of level 0 take 8 rounds (35,896 / 14,841 /
// 5,776 / 1,871 / 490 / 80 / 5 / 0 left).
//
//   k_ck_build   (grid)  key table over the list's accesses: each access gets
//                        its key's slot (32 B: key, c, u_r for two round
//                        parities); writers publish u_1
//   k_ck_round   (grid)  one round: lane per undecided txn; decisions go
//                        straight to the epoch's state bytes, survivors
//                        publish u_{r+1} (the other parity's word, tagged
//                        with the round) and append themselves to the next
//                        list (wave-aggregated, unordered: the rule reads
//                        txn positions, not list order)
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

// slot of a key (linear probing over 32-B slots; the table is at <= 50 % load
// of the list's accesses)
__device__ inline uint32_t ck_insert(CkSlot* tab, uint32_t mask, uint64_t key) {
  uint32_t h = ck_hash(key, mask);
  for (uint32_t n = 0; n <= mask; n++) {
    const uint64_t cur = tab[h].key;
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

// atomicMin behind a read filter (a stale read is only ever higher)
__device__ inline void ck_umin(uint64_t* p, uint64_t v) {
  if (v < *p) atomicMin((unsigned long long*)p, (unsigned long long)v);
}

// ---------------------------------------------------------------------------
// k_ck_build: one 256-txn tile of the list per workgroup iteration; accesses
// of the tile strided over the threads, owner by binary search of the tile's
// offsets in LDS.
__global__ __launch_bounds__(256) void k_ck_build(CkArgs a) {
  __shared__ uint32_t s_off[257];
  // round 1 appends to counter 2 (rounds zero the counters two ahead)
  if (blockIdx.x == 0 && threadIdx.x == 0) a.ctl[CK_CTL_RING + 2] = 0;
  if (*a.abandon) return;
  const uint32_t m = a.lv1->m, acc = a.lv1->acc;
  if (m == 0) return;
  uint32_t bits = 10;
  while (bits < 31 && (1ull << bits) < 2ull * acc) bits++;
  if (bits > a.cap_bits) {  // list too large for the table: the round solver takes it
    if (blockIdx.x == 0 && threadIdx.x == 0) atomicMax(a.abandon_out, 1u);
    return;
  }
  const uint32_t mask = (1u << bits) - 1u;
  if (blockIdx.x == 0 && threadIdx.x == 0) a.ctl[CK_CTL_MASK] = mask;
  const uint32_t j = threadIdx.x;
  bool bad = false;
  for (uint32_t t0 = blockIdx.x * 256u; t0 < m; t0 += gridDim.x * 256u) {
    const uint32_t nt = min(256u, m - t0);
    __syncthreads();  // s_off reuse
    for (uint32_t q = j; q <= nt; q += 256) s_off[q] = a.off1[t0 + q];
    __syncthreads();
    const uint32_t A0 = s_off[0], A1 = s_off[nt];
    for (uint32_t x = A0 + j; x < A1; x += 256) {
      uint32_t lo = 0, hi = nt;  // s_off[lo] <= x < s_off[hi]
      while (hi - lo > 1) {
        const uint32_t mid = (lo + hi) >> 1;
        if (s_off[mid] <= x) lo = mid;
        else hi = mid;
      }
      const uint64_t key = a.keys1[x];
      const bool w = a.at1[x] == 1;  // WR (occ.cpp:296-317: only WR joins the write set)
      if (key == KEY_EMPTY) {        // the reserved key: reported, never a conflict
        bad = true;
        a.aslot[x] = CK_NONE;
        continue;
      }
      const uint32_t sl = ck_insert(a.tab, mask, key);
      a.aslot[x] = sl | (w ? CK_WR : 0u);
      if (w) ck_umin(&a.tab[sl].u[1], ck_uword(1, t0 + lo));
    }
  }
  if (bad) atomicOr(a.err, ERR_KEY);
}

// Does list txn j commit in round r?  (no key with a committed writer before
// j, no key with an undecided writer before j at the start of the round)
__device__ inline bool ck_commits(const CkArgs& a, uint32_t j, uint32_t r) {
  const uint32_t s = a.off1[j], e = a.off1[j + 1];
  for (uint32_t q = s; q < e; q++) {
    const uint32_t as = a.aslot[q];
    if (as == CK_NONE) continue;
    const CkSlot* sl = a.tab + (as & ~CK_WR);
    if (sl->c < j || ck_blocks(sl->u[r & 1], r, j)) return false;
  }
  return true;
}

// ---------------------------------------------------------------------------
// k_ck_round: round r over its list (round 1: the whole list, identity).
__global__ __launch_bounds__(256) void k_ck_round(CkArgs a, uint32_t r) {
  uint32_t* cnt = a.ctl + CK_CTL_RING;
  // the counter two rounds on is free again (round r + 1 appends to r + 2)
  if (blockIdx.x == 0 && threadIdx.x == 0) cnt[(r + 2) % CK_RING] = 0;
  if (*a.abandon) return;
  const uint32_t n = r == 1 ? a.lv1->m : cnt[r % CK_RING];
  if (n == 0) return;
  const uint32_t* lin = a.lst[r & 1];
  uint32_t* lout = a.lst[(r + 1) & 1];
  const uint32_t lane = lane_id();
  const uint32_t nw = gridDim.x * (blockDim.x / 64);
  const uint32_t wid = blockIdx.x * (blockDim.x / 64) + (threadIdx.x >> 6);
  for (uint32_t base = wid * 64; base < n; base += nw * 64) {
    const uint32_t i = base + lane;
    const bool valid = i < n;
    bool stay = false;
    uint32_t t = 0;
    if (valid) {
      t = r == 1 ? i : lin[i];
      const uint32_t s = a.off1[t], e = a.off1[t + 1];
      bool kill = false, blk = false;
      // every access's slot words, CK_U loads in flight per lane
      for (uint32_t q0 = s; q0 < e && !kill; q0 += CK_U) {
        uint32_t as[CK_U];
#pragma unroll
        for (uint32_t u = 0; u < CK_U; u++) as[u] = q0 + u < e ? a.aslot[q0 + u] : CK_NONE;
        uint32_t c[CK_U];
        uint64_t uw[CK_U];
#pragma unroll
        for (uint32_t u = 0; u < CK_U; u++) {
          c[u] = ~0u;
          uw[u] = ~0ull;
          if (as[u] != CK_NONE) {
            const CkSlot* sl = a.tab + (as[u] & ~CK_WR);
            c[u] = sl->c;
            uw[u] = sl->u[r & 1];
          }
        }
#pragma unroll
        for (uint32_t u = 0; u < CK_U; u++) {
          kill |= c[u] < t;
          blk |= ck_blocks(uw[u], r, t);
        }
      }
      // blocked: killed now if one of its blockers commits in this round
      if (!kill && blk) {
        uint32_t last = ~0u;
        for (uint32_t q = s; q < e && !kill; q++) {
          const uint32_t as = a.aslot[q];
          if (as == CK_NONE) continue;
          const uint64_t uw = a.tab[as & ~CK_WR].u[r & 1];
          if (!ck_blocks(uw, r, t)) continue;
          const uint32_t bj = (uint32_t)uw;
          if (bj == last) continue;
          last = bj;
          kill = ck_commits(a, bj, r);
        }
      }
      if (kill) {
        a.state[a.tid1[t]] = ST_ABORT;
      } else if (!blk) {
        a.state[a.tid1[t]] = ST_COMMIT;
        for (uint32_t q = s; q < e; q++) {
          const uint32_t as = a.aslot[q];
          if (as != CK_NONE && (as & CK_WR)) atomicMin(&a.tab[as & ~CK_WR].c, t);
        }
      } else {
        stay = true;
        const uint64_t w1 = ck_uword(r + 1, t);
        for (uint32_t q = s; q < e; q++) {
          const uint32_t as = a.aslot[q];
          if (as != CK_NONE && (as & CK_WR)) ck_umin(&a.tab[as & ~CK_WR].u[(r + 1) & 1], w1);
        }
      }
    }
    const uint64_t sm = ballot64(stay);
    if (sm) {
      uint32_t b = 0;
      if (lane == 0) b = atomicAdd(&cnt[(r + 1) % CK_RING], (uint32_t)__popcll(sm));
      b = __shfl(b, 0);
      if (stay) lout[b + (uint32_t)__popcll(sm & ((1ull << lane) - 1ull))] = t;
    }
  }
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
  k_ck_round<<<grid ? grid : 1u, 256, 0, st>>>(a, r);
}
void launch_ck_fill(CkSlot* tab, uint64_t n, hipStream_t st) {
  const uint64_t g = (n + 255) / 256;
  k_ck_fill<<<(unsigned)(g < 4096 ? (g ? g : 1) : 4096), 256, 0, st>>>(tab, n);
}

}  // namespace dcc
