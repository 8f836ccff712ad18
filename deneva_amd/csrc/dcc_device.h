// Device-side primitives shared by the gfx950 kernels of libdcc.
//
// Hash-slot layout (HBM-resident open-addressing table):
//
//   struct Slot { u64 key; u32 own; u32 aux; }   16 B, 16-B aligned, capacity 2^k
//
// `own` is a 32-bit owner word:  tag:6 | txn index:26
//   tag 0            the key's committed writer (at most one per key and epoch:
//                    every later accessor of the key aborts, occ.cpp:185-199)
//   tag 63 - r       minimum undecided writer at the start of round r (r = 1..61)
//   0xFFFFFFFF       empty (tag 63)
// Newer rounds carry SMALLER tags, so one atomicMin both replaces stale words
// of older rounds and keeps the round's minimum writer, and a committed word
// (tag 0) is never displaced.  Owner words are only consulted for accesses
// whose previous blocker aborted (or in round 1); everything else resolves
// from the per-txn state byte of the recorded blocker.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace dcc {

constexpr uint64_t KEY_EMPTY = 0xFFFFFFFFFFFFFFFFull;

// Bounded spins of cross-workgroup waits (look-back predecessors, grid
// barriers) are bounded in time, generously: processes sharing one GPU are
// time-sliced, and a workgroup dispatched before the waiter can stay
// switched out for hundreds of milliseconds (round 6: an iteration bound of
// ~0.4 s expired under four rank processes on one GPU, and k_fin numbered a
// partly published prefix).  The bound only turns a hang into an error.
constexpr uint64_t SPIN_TICKS = 2000000000ull;  // 20 s of the 100 MHz realtime clock
__device__ inline uint64_t spin_clock() { return __builtin_amdgcn_s_memrealtime(); }
constexpr uint32_t OWN_EMPTY = 0xFFFFFFFFu;
constexpr uint32_t IDX_BITS = 26;
constexpr uint32_t IDX_MASK = (1u << IDX_BITS) - 1;
constexpr uint32_t MAX_TAG_ROUND = 62;
constexpr uint32_t SID_NONE = 0x3FFFFFFFu;   // 30-bit slot index space
// List entry (u64): low word  = W:1 | B:1 | sid:30
//                   high word = blocker txn index (valid when B)
constexpr uint32_t ENT_WRITE = 0x80000000u;  // access is a write
constexpr uint32_t ENT_BLOCK = 0x40000000u;  // access is blocked by the recorded owner
constexpr uint32_t ENT_SID = 0x3FFFFFFFu;

// per-txn state byte: 0 undecided, 1 commit, 2 + (round % 64) abort.
// The abort round lets a reader tell an abort of an EARLIER round (owner
// words already republished, safe to re-read) from one of the current round
// (seen through a race; treated as still blocking until the next round).
constexpr uint8_t ST_UNDECIDED = 0;
constexpr uint8_t ST_COMMIT = 1;
constexpr uint8_t ST_ABORT = 2;  // abort in round 0 (history window)
__host__ __device__ inline uint8_t st_abort(uint32_t round) { return (uint8_t)(2u + (round & 63u)); }

// per-access / per-txn probe status bits
constexpr uint32_t PS_BLOCKED = 1;
constexpr uint32_t PS_KILLED = 2;
constexpr uint32_t PS_WRITE = 4;  // sharded rounds: the txn keeps a write entry here

struct __attribute__((aligned(16))) Slot {
  uint64_t key;
  uint32_t own;
  uint32_t aux;
};

__host__ __device__ inline uint32_t round_tag(uint32_t r) { return 63u - r; }
__host__ __device__ inline uint32_t own_word(uint32_t tag, uint32_t idx) {
  return (tag << IDX_BITS) | idx;
}

__device__ __host__ inline uint64_t fmix64(uint64_t k) {
  k ^= k >> 33;
  k *= 0xff51afd7ed558ccdull;
  k ^= k >> 33;
  k *= 0xc4ceb9fe1a85ec53ull;
  k ^= k >> 33;
  return k;
}
__device__ __host__ inline uint32_t fmix32(uint32_t h) {
  h ^= h >> 16;
  h *= 0x85ebca6bu;
  h ^= h >> 13;
  h *= 0xc2b2ae35u;
  h ^= h >> 16;
  return h;
}

// Probe sequence: double hashing.  The home slot keeps the low 32 key bits
// (offset by a hash of the high bits), so the dense, zipf-hot low rows of a
// table (YCSB row ids, TPC-C warehouse/district/customer keys under their
// table tag) sit next to each other and stay L2-resident — the analogue of
// the reference's (key / part_cnt) % buckets index hash (index_hash.h:86-92).
// Collisions jump by a key-dependent odd stride, so a dense run of occupied
// home slots never turns into a long linear probe chain.
__device__ inline uint32_t slot_home(uint64_t key, uint32_t mask) {
  return ((uint32_t)key + fmix32((uint32_t)(key >> 32))) & mask;
}
__device__ inline uint32_t slot_step(uint64_t key, uint32_t mask) {
  return ((uint32_t)(fmix64(key) >> 32) | 1u) & mask;
}

// Insert-or-find a write key.  Keys are never removed during an epoch, so a
// non-empty key read by a plain (possibly L1-stale) load is exact; a stale
// EMPTY only costs a CAS that then reports the real key.
__device__ inline uint32_t table_insert(Slot* tab, uint32_t mask, uint64_t key) {
  uint32_t h = slot_home(key, mask);
  const uint32_t st = slot_step(key, mask);
  for (uint32_t n = 0; n <= mask; n++) {
    uint64_t cur = tab[h].key;
    if (cur == key) return h;
    if (cur == KEY_EMPTY) {
      uint64_t prev = atomicCAS((unsigned long long*)&tab[h].key, (unsigned long long)KEY_EMPTY,
                                (unsigned long long)key);
      if (prev == KEY_EMPTY || prev == key) return h;
    }
    h = (h + st) & mask;
  }
  return SID_NONE;  // table full: host sizing guarantees this never happens
}

// Find a key inserted by an earlier kernel (read-only probe).
__device__ inline uint32_t table_find(const Slot* tab, uint32_t mask, uint64_t key) {
  uint32_t h = slot_home(key, mask);
  const uint32_t st = slot_step(key, mask);
  for (uint32_t n = 0; n <= mask; n++) {
    const uint64_t cur = tab[h].key;
    if (cur == key) return h;
    if (cur == KEY_EMPTY) return SID_NONE;
    h = (h + st) & mask;
  }
  return SID_NONE;
}

// atomicMin with a read filter: hot keys see one real atomic per round instead
// of one per writer.  A stale read can only be HIGHER than the true value
// (owner words only decrease between resets), so skipping is always safe.
__device__ inline void own_min(uint32_t* p, uint32_t v) {
  uint32_t cur = *p;
  if (v < cur) atomicMin(p, v);
}

// Decode an owner word for accessor txn i in round r (tag t_r).
__device__ inline uint32_t own_status(uint32_t w, uint32_t t_r, uint32_t i) {
  const uint32_t tag = w >> IDX_BITS, idx = w & IDX_MASK;
  if (tag == 0) return idx < i ? PS_KILLED : 0u;
  if (tag == t_r) return idx < i ? PS_BLOCKED : 0u;
  return 0u;
}
__device__ inline uint32_t own_idx(uint32_t w) { return w & IDX_MASK; }

// Per-workgroup LDS min-combiner for owner publishing: candidates for the
// same slot are folded in LDS first, so a key receives at most one global
// atomicMin per workgroup instead of one per writer (a single word serialises
// device atomics at ~100/us: hot keys would otherwise pile up).
template <int NT>
struct LdsMin {
  uint32_t sid[NT];
  uint32_t val[NT];
  __device__ void init() {
    for (uint32_t q = threadIdx.x; q < NT; q += blockDim.x) {
      sid[q] = SID_NONE;
      val[q] = OWN_EMPTY;
    }
  }
  // returns false when the probe window is full (caller publishes directly)
  __device__ bool add(uint32_t s, uint32_t v) {
    uint32_t h = (s * 2654435761u) >> (32 - __builtin_ctz(NT));
#pragma unroll 1
    for (int q = 0; q < 8; q++) {
      const uint32_t cur = sid[h];
      if (cur == s || (cur == SID_NONE && (atomicCAS(&sid[h], SID_NONE, s) == SID_NONE ||
                                           sid[h] == s))) {
        atomicMin(&val[h], v);
        return true;
      }
      h = (h + 1) & (NT - 1);
    }
    return false;
  }
  __device__ void flush(Slot* tab) {
    for (uint32_t q = threadIdx.x; q < NT; q += blockDim.x)
      if (sid[q] != SID_NONE) own_min(&tab[sid[q]].own, val[q]);
  }
};

__device__ inline uint64_t ballot64(bool p) { return __ballot(p); }
__device__ inline uint32_t lane_id() { return __lane_id(); }

// OR-reduce per contiguous segment of lanes.  `seg` is the segment id of the
// lane (equal ids are contiguous); returns for HEAD lanes the OR of the low
// NB bits of `bits` over the segment, 0 elsewhere, and sets is_head.
template <int NB>
__device__ inline uint32_t segment_or(uint32_t seg, uint32_t bits, bool& is_head) {
  const uint32_t lane = lane_id();
  const uint32_t prev = __shfl_up(seg, 1);
  is_head = (lane == 0) || (prev != seg);
  const uint64_t hm = ballot64(is_head);
  uint64_t b[NB];
#pragma unroll
  for (int q = 0; q < NB; q++) b[q] = ballot64(bits & (1u << q));
  if (!is_head) return 0;
  const uint64_t above = lane == 63 ? 0ull : (hm & ~((2ull << lane) - 1ull));
  const uint32_t end = above ? (uint32_t)__builtin_ctzll(above) : 64u;
  const uint64_t hi = end == 64 ? ~0ull : ((1ull << end) - 1ull);
  const uint64_t m = hi & ~((1ull << lane) - 1ull);
  uint32_t v = 0;
#pragma unroll
  for (int q = 0; q < NB; q++) v |= (b[q] & m) ? (1u << q) : 0u;
  return v;
}
__device__ inline uint32_t segment_or2(uint32_t seg, uint32_t bits, bool& is_head) {
  return segment_or<2>(seg, bits, is_head);
}

}  // namespace dcc
