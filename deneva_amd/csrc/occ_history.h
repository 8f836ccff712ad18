// Device-resident OCC history (the `history` list of committed write sets,
// concurrency_control/occ.h:62-64, pushed by central_finish, occ.cpp:277-286,
// scanned by the window check of central_validate, occ.cpp:160-180).
//
// The history is a multiset of (key, tn) pairs: one per write of a committed
// txn numbered tn.  It lives in HBM as two levels, a large `base` and a small
// `delta` (a two-level log-structured merge), each its pairs sorted by (key,
// tn) with an open-addressing key table (<= 25 % load).  An epoch appends its
// committed writes to the delta's flat pairs on the device (count, scan,
// emit: no D2H of the batch) and pushes each onto its key's chain in the
// delta's table (no re-sort per epoch); the delta is rebuilt sorted after a
// host append and merged into the base when it outgrows a quarter of it.
// A window query is one 16-B probe per level (the key and its largest tn
// answer it unless the window ends below that tn); only then the key's chain
// (newest first) and the binary search of its sorted run.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "dcc.h"

// history hash slot of a key (device build and probe agree)
__host__ __device__ inline uint64_t hist_hash_slot(uint64_t key, uint32_t bits) {
  return (key * 0x9E3779B97F4A7C15ull) >> (64 - bits);
}

namespace dcc {

struct HistLevel {
  // [2 << hbits] probe words (HistSlot per slot: key DCC_KEY_RESERVED =
  // empty), then [2 << hbits] side words per slot: the key's sorted run
  // (first | count << 32; all-ones: none) and its chain head (low word,
  // HIST_NIL: none)
  const uint64_t* hash;
  const uint64_t* tn;    // [m] the sorted pairs' tns, ascending within a key's run
  const uint64_t* ctn;   // the flat pairs' tns (chain entries), or null
  const uint32_t* next;  // the flat pairs' chain links (HIST_NIL ends), or null
  uint32_t hbits;
  uint32_t on;           // 0: the level is empty
  uint32_t walk;         // flat pairs of the level: no chain is longer, no link points past it
  uint32_t pad;
};
// A probe slot (16 B): the key and the complement of its largest tn
// (all-ones when empty, so a chain push lowers it with atomicMin).  Every key
// sits within HIST_WALK slots of its home (a build or push that walks further
// flags the table, and the host rebuilds it bigger), so probes stop there.
struct HistSlot {
  uint64_t key, ntmax;
};
constexpr uint32_t HIST_NIL = 0xFFFFFFFFu;
constexpr uint32_t HIST_WALK = 64;
__device__ inline HistSlot hist_slot_ld(const uint64_t* hash, uint64_t s) {
  const ulonglong2 a = reinterpret_cast<const ulonglong2*>(hash)[s];
  return HistSlot{a.x, a.y};
}
// does the key of found slot s (largest tn tmax) have a pair with lo < tn <= hi?
__device__ inline bool hist_found_hit(const HistLevel& L, uint64_t s, uint64_t tmax, uint64_t lo, uint64_t hi) {
  if (tmax <= lo) return false;
  if (tmax <= hi) return true;  // tmax is in the window
  const ulonglong2 side = reinterpret_cast<const ulonglong2*>(L.hash + (2ull << L.hbits))[s];
  // the chain: epochs' appends, pushed in tn order, so newest first (a walk
  // is bounded by the level's pairs even if a chain were ever corrupt: a
  // step past them ends it instead of looping)
  if (L.next)
    for (uint32_t p = (uint32_t)side.y, st = 0; p < L.walk && st < L.walk; p = L.next[p], st++) {
      const uint64_t t = L.ctn[p];
      if (t <= hi) {
        if (t > lo) return true;
        break;  // the rest are older still
      }
    }
  if (side.x == ~0ull) return false;
  const uint64_t first = (uint32_t)side.x, end = first + (side.x >> 32);
  uint64_t b = first, e = end;
  while (b < e) {  // first tn > lo
    const uint64_t m = (b + e) >> 1;
    if (L.tn[m] <= lo) b = m + 1;
    else e = m;
  }
  return b < end && L.tn[b] <= hi;
}
// One-hash bitmap of every key in the history (both levels): the window
// check loads it into LDS and probes a level's table only for keys whose bit
// is set (most reads touch keys the history never saw).
constexpr uint32_t HIST_BM_LOG = 17;  // bits (16 KiB)
__host__ __device__ inline uint32_t hist_bm_bit(uint64_t key) {
  return (uint32_t)((key * 0xD6E8FEB86659FD93ull) >> (64 - HIST_BM_LOG));
}
struct HistView {
  HistLevel lv[2];     // base, delta
  const uint32_t* bm;  // [2^HIST_BM_LOG / 32] key bitmap of both levels, or null
};

// does the level hold a pair (key, tn) with lo < tn <= hi?
__device__ inline bool hist_level_hit(const HistLevel& L, uint64_t key, uint64_t lo, uint64_t hi) {
  if (!L.on) return false;
  const uint64_t mask = (1ull << L.hbits) - 1;
  uint64_t slot = hist_hash_slot(key, L.hbits);
  for (uint32_t i = 0; i < HIST_WALK; i++) {
    const HistSlot S = hist_slot_ld(L.hash, slot);
    if (S.key == key) return hist_found_hit(L, slot, ~S.ntmax, lo, hi);
    if (S.key == DCC_KEY_RESERVED) return false;
    slot = (slot + 1) & mask;
  }
  return false;
}
__device__ inline bool hist_hit(const HistView& h, uint64_t key, uint64_t lo, uint64_t hi) {
  return hist_level_hit(h.lv[1], key, lo, hi) || hist_level_hit(h.lv[0], key, lo, hi);
}

// ---- build kernels (occ_history.hip)
// per 1024-txn block: the writes of committed txns (tn[t] != 0)
void launch_hist_count(uint64_t n, const uint32_t* off, const uint8_t* acctype, uint64_t nnz,
                       const uint64_t* tn, uint32_t* bsum, hipStream_t st);
// pairs of block b's committed writes at out + bsum[b] (scanned) + block rank
// (*kmax raised to the largest key emitted)
void launch_hist_emit(uint64_t n, const uint32_t* off, const uint64_t* keys, const uint8_t* acctype,
                      uint64_t nnz, const uint64_t* tn, const uint32_t* bsum, uint64_t* out_k,
                      uint64_t* out_t, unsigned long long* kmax, hipStream_t st);
// An epoch's append into the delta's table: each flat pair p (key, tn)
// finds or claims its key's slot within HIST_WALK of home (else *over is set
// and the pair left out: the host rebuilds the level before it is read
// again), lowers the slot's ~tmax and is pushed on the key's chain; the key
// bitmaps get its bit.  At most one committed txn of an epoch writes a key
// and tns grow from epoch to epoch, so every chain stays newest first.
struct HistInsert {
  const uint64_t* fk;
  const uint64_t* ft;
  uint64_t* hash;
  uint32_t* next;
  uint32_t* bm_level;
  uint32_t* bm_all;
  uint32_t* over;  // [0] overflow flag, [1] k_fin_insert's finished workgroups
  uint32_t hbits, pad;
};
__device__ inline void hist_insert(const HistInsert& h, uint64_t p, uint64_t key, uint64_t tn) {
  const uint64_t mask = (1ull << h.hbits) - 1;
  uint64_t s = hist_hash_slot(key, h.hbits);
  for (uint32_t i = 0;; i++) {
    if (i == HIST_WALK) {
      atomicOr(h.over, 1u);
      return;
    }
    unsigned long long* ks = (unsigned long long*)&h.hash[2 * s];
    unsigned long long k = *(volatile unsigned long long*)ks;
    if (k == DCC_KEY_RESERVED) {
      k = atomicCAS(ks, (unsigned long long)DCC_KEY_RESERVED, (unsigned long long)key);
      if (k == DCC_KEY_RESERVED) k = key;
    }
    if (k == key) break;
    s = (s + 1) & mask;
  }
  atomicMin((unsigned long long*)&h.hash[2 * s + 1], (unsigned long long)~tn);
  uint32_t* head = (uint32_t*)&h.hash[(2ull << h.hbits) + 2 * s + 1];
  h.next[p] = atomicExch(head, (uint32_t)p);
  const uint32_t b = hist_bm_bit(key);
  atomicOr(&h.bm_level[b >> 5], 1u << (b & 31u));
  atomicOr(&h.bm_all[b >> 5], 1u << (b & 31u));
}
// level build from flat pairs (fk, ft)[m]; K/V are radix-sort ping-pong buffers
struct HistBuild {
  uint64_t m;
  const uint64_t* fk;
  const uint64_t* ft;
  bool mono;            // flat tns ascend within every key (append order is tn order)
  uint64_t* K[2];
  uint32_t* V[2];
  uint32_t* scratch;
  uint64_t* skey;       // out: sorted keys
  uint64_t* stn;        // out: sorted tns
  uint64_t* hash;       // out: [4 << hbits] (HistLevel)
  uint32_t hbits;
  uint32_t kbits, tbits;  // significant bits of the keys / tns (radix passes)
  uint32_t* over;       // out: set when a key sits past HIST_WALK (rebuild bigger)
};
int hist_build_level(const HistBuild& b, hipStream_t st);
// the key bitmap of m flat keys (bm zeroed first), and out = a | b
void launch_hist_bm(const uint64_t* keys, uint64_t m, uint32_t* bm, hipStream_t st);
void launch_hist_bm_or(const uint32_t* a, const uint32_t* b, uint32_t* out, hipStream_t st);
// pairs with tn > floor of (ak, at)[na] then (bk, bt)[nb], appended at
// (ok, ot) + *cnt (atomic position: order not kept)
void launch_hist_trim(const uint64_t* ak, const uint64_t* at, uint64_t na, const uint64_t* bk,
                      const uint64_t* bt, uint64_t nb, uint64_t floor, uint64_t* ok, uint64_t* ot,
                      unsigned long long* cnt, hipStream_t st);

}  // namespace dcc
