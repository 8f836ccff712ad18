// Device-resident OCC history (the `history` list of committed write sets,
// concurrency_control/occ.h:62-64, pushed by central_finish, occ.cpp:277-286,
// scanned by the window check of central_validate, occ.cpp:160-180).
//
// The history is a multiset of (key, tn) pairs: one per write of a committed
// txn numbered tn.  It lives in HBM as two levels, a large `base` and a small
// `delta` (a two-level log-structured merge): an epoch appends its committed
// writes to the delta's flat pair array on the device (count, scan, emit: no
// D2H of the batch), the delta is rebuilt, and it is merged into the base when
// it outgrows a quarter of it.  A built level is its pairs sorted by (key, tn)
// plus an open-addressing table key -> (first pair, pair count, min tn, max
// tn) at <= 50 % load, so a window query is one probe per level, and a binary
// search of the key's run of tns only when the window lies inside the run.
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
  const uint64_t* hash;  // [4 << hbits]: HistSlot per slot (key DCC_KEY_RESERVED = empty)
  const uint64_t* tn;    // [m] tns, ascending within a key's run
  uint32_t hbits;
  uint32_t on;           // 0: the level is empty
};
// A table slot (32 B): the key, its run in the sorted pairs (first | count <<
// 32) and the run's smallest and largest tn, so a window query resolves from
// the slot alone unless the window lies strictly inside the run's tn range.
struct HistSlot {
  uint64_t key, fc, tmin, tmax;
};
__device__ inline HistSlot hist_slot_ld(const uint64_t* hash, uint64_t s) {
  const ulonglong2* p = reinterpret_cast<const ulonglong2*>(hash + 4 * s);
  const ulonglong2 a = p[0], b = p[1];
  return HistSlot{a.x, a.y, b.x, b.y};
}
// does the run of a found slot hold a tn with lo < tn <= hi?
__device__ inline bool hist_slot_hit(const HistLevel& L, const HistSlot& S, uint64_t lo, uint64_t hi) {
  if (S.tmax <= lo || S.tmin > hi) return false;
  if (S.tmax <= hi || S.tmin > lo) return true;  // tmax (resp. tmin) is in the window
  const uint64_t first = (uint32_t)S.fc, end = first + (S.fc >> 32);
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
  for (;;) {  // <= 50 % load: every probe sequence ends at an empty slot
    const HistSlot S = hist_slot_ld(L.hash, slot);
    if (S.key == key) return hist_slot_hit(L, S, lo, hi);
    if (S.key == DCC_KEY_RESERVED) return false;
    slot = (slot + 1) & mask;
  }
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
  uint64_t* hash;       // out: [4 << hbits]
  uint32_t hbits;
  uint32_t kbits, tbits;  // significant bits of the keys / tns (radix passes)
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
