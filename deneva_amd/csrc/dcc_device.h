// Device-side primitives shared by the gfx950 kernels of libdcc.
//
// Hash-slot layout (HBM-resident open-addressing table):
//
//   struct Slot { u64 key; u32 own[2]; }   16 B, 16-B aligned, capacity = 2^k
//
// own[b] is a 32-bit "owner word":  tag:6 | txn index:26
//   tag 0            the key's committed writer (at most one per key and epoch:
//                    every later accessor of the key is aborted, occ.cpp:185-199)
//   tag 63 - r       minimum undecided writer at the start of round r
//                    (r = 1..62; buffer b = r & 1)
//   0xFFFFFFFF       empty (tag 63)
// Newer rounds carry SMALLER tags, so a plain atomicMin both replaces stale
// entries of older rounds and keeps the minimum writer of the current round,
// and the committed word (tag 0) is never displaced.  Round r reads own[r&1]
// while its blocked writers publish round r+1 into own[(r+1)&1]: one kernel
// per round, no reset pass.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace dcc {

constexpr uint64_t KEY_EMPTY = 0xFFFFFFFFFFFFFFFFull;
constexpr uint32_t OWN_EMPTY = 0xFFFFFFFFu;
constexpr uint32_t IDX_BITS = 26;
constexpr uint32_t IDX_MASK = (1u << IDX_BITS) - 1;
constexpr uint32_t MAX_TAG_ROUND = 62;
constexpr uint32_t SID_NONE = 0x3FFFFFFFu;   // 30-bit slot index space
constexpr uint32_t ENT_WRITE = 0x80000000u;  // list entry: access is a write
constexpr uint32_t ENT_BLOCK = 0x40000000u;  // list entry: access was blocking
constexpr uint32_t ENT_SID = 0x3FFFFFFFu;

// per-txn state byte
constexpr uint8_t ST_UNDECIDED = 0;
constexpr uint8_t ST_COMMIT = 1;
constexpr uint8_t ST_ABORT = 2;

// per-access / per-txn probe status bits
constexpr uint32_t PS_BLOCKED = 1;
constexpr uint32_t PS_KILLED = 2;

struct __attribute__((aligned(16))) Slot {
  uint64_t key;
  uint32_t own[2];
};

__host__ __device__ inline uint32_t round_tag(uint32_t r) { return 63u - r; }
__host__ __device__ inline uint32_t own_word(uint32_t tag, uint32_t idx) {
  return (tag << IDX_BITS) | idx;
}

// Table index hash: murmur3 fmix64.  Deliberately different from the shard
// hash (dcc_key_shard) so that a shard's keys spread over all slots.
__device__ __host__ inline uint64_t fmix64(uint64_t k) {
  k ^= k >> 33;
  k *= 0xff51afd7ed558ccdull;
  k ^= k >> 33;
  k *= 0xc4ceb9fe1a85ec53ull;
  k ^= k >> 33;
  return k;
}

__device__ inline uint32_t slot_hash(uint64_t key, uint32_t mask) {
  return (uint32_t)fmix64(key) & mask;
}

// Insert-or-find a write key (linear probing).  Keys are never removed during
// an epoch, so a non-empty key read by a plain (possibly L1-stale) load is
// exact; a stale EMPTY only costs a CAS that then reports the real key.
__device__ inline uint32_t table_insert(Slot* tab, uint32_t mask, uint64_t key) {
  uint32_t h = slot_hash(key, mask);
  for (uint32_t n = 0; n <= mask; n++) {
    uint64_t cur = tab[h].key;
    if (cur == key) return h;
    if (cur == KEY_EMPTY) {
      uint64_t prev = atomicCAS((unsigned long long*)&tab[h].key, (unsigned long long)KEY_EMPTY,
                                (unsigned long long)key);
      if (prev == KEY_EMPTY || prev == key) return h;
    }
    h = (h + 1) & mask;
  }
  return SID_NONE;  // table full: host sizing guarantees this never happens
}

// Find a key after the build kernel completed (no concurrent inserts).
__device__ inline uint32_t table_find(const Slot* tab, uint32_t mask, uint64_t key) {
  uint32_t h = slot_hash(key, mask);
  for (uint32_t n = 0; n <= mask; n++) {
    uint64_t cur = tab[h].key;
    if (cur == key) return h;
    if (cur == KEY_EMPTY) return SID_NONE;
    h = (h + 1) & mask;
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

__device__ inline uint64_t ballot64(bool p) { return __ballot(p); }
__device__ inline uint32_t lane_id() { return __lane_id(); }

// OR-reduce per contiguous segment of lanes.  `seg` is the segment id of the
// lane (equal ids are contiguous); returns for HEAD lanes the OR of `bits`
// over the segment (2 bits), 0 elsewhere, and sets is_head.
__device__ inline uint32_t segment_or2(uint32_t seg, uint32_t bits, bool& is_head) {
  const uint32_t lane = lane_id();
  const uint32_t prev = __shfl_up(seg, 1);
  is_head = (lane == 0) || (prev != seg);
  const uint64_t hm = ballot64(is_head);
  const uint64_t b0 = ballot64(bits & 1u);
  const uint64_t b1 = ballot64(bits & 2u);
  if (!is_head) return 0;
  const uint64_t above = lane == 63 ? 0ull : (hm & ~((2ull << lane) - 1ull));
  const uint32_t end = above ? (uint32_t)__builtin_ctzll(above) : 64u;
  const uint64_t hi = end == 64 ? ~0ull : ((1ull << end) - 1ull);
  const uint64_t m = hi & ~((1ull << lane) - 1ull);
  return ((b0 & m) ? 1u : 0u) | ((b1 & m) ? 2u : 0u);
}

}  // namespace dcc
