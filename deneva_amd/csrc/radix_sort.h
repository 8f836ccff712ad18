// Stable LSD radix sort of (key, u32 value) pairs on gfx950, 8-bit digits.
//
// Used by the Calvin engine to put an epoch's lock requests into per-row FIFO
// order ("K4 radix sort of (key, order)") and to rank
// txns by their sequencer order (a13).  Keys are first compressed to the bits
// that actually vary across the batch, so a YCSB epoch (row*16+part < 2^28)
// sorts in 3-4 passes of 32-bit keys instead of 8 passes of 64-bit keys.
//
// Per pass (3 launches): k_rs_hist (per-tile digit counts, wave-level digit
// matching so equal digits cost one LDS atomic per wave), k_rs_scan (digit-
// major exclusive scan of the [digit][tile] counts, one workgroup per digit),
// k_rs_scatter (stable in-tile ranking, staged through LDS so global writes
// leave in digit runs).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <algorithm>

namespace dcc {

constexpr uint32_t RS_THREADS = 512;
constexpr uint32_t RS_ITEMS = 16;
constexpr uint32_t RS_TILE = RS_THREADS * RS_ITEMS;  // 8192 pairs per workgroup

constexpr uint32_t RS_ITEMS_SMALL = 4;           // sorts of <= RS_SMALL pairs: 2,048-pair tiles
constexpr uint64_t RS_SMALL = 2ull << 20;

inline uint64_t rs_tiles(uint64_t m) {
  const uint64_t t = m <= RS_SMALL ? (uint64_t)RS_THREADS * RS_ITEMS_SMALL : RS_TILE;
  return (m + t - 1) / t;
}
// u32 words of scratch a sort of up to m pairs needs: counts [256][tiles] +
// totals [256] (monotone in m: covers either tiling of any m' <= m)
inline uint64_t rs_scratch_words(uint64_t m) {
  const uint64_t ts = (uint64_t)RS_THREADS * RS_ITEMS_SMALL;
  return 256 * ((std::min<uint64_t>(m, RS_SMALL) + ts - 1) / ts + (m + RS_TILE - 1) / RS_TILE + 1);
}

// Sorts m pairs by the low `bits` key bits.  Input in k[0]/v[0]; k[1]/v[1] are
// equal-sized ping-pong buffers.  Returns the index (0 or 1) of the buffer
// pair that holds the result.  m < 2^32.
int radix_sort_u32(uint32_t* k[2], uint32_t* v[2], uint64_t m, uint32_t bits, uint32_t* scratch,
                   hipStream_t st);
int radix_sort_u64(uint64_t* k[2], uint32_t* v[2], uint64_t m, uint32_t bits, uint32_t* scratch,
                   hipStream_t st);

// Exclusive scan of one u32 row in place (one workgroup); *total = its sum.
void rs_scan_one(uint32_t* row, uint32_t len, uint32_t* total, hipStream_t st);
// The same for `rows` rows of `len` (row r at cnt + r * len); tot[r] = row sums.
void rs_scan_rows(uint32_t* cnt, uint32_t rows, uint32_t len, uint32_t* tot, hipStream_t st);

// Bit-gather: the positions where a batch's keys differ (OR ^ AND over every
// key) packed into the low bits, as at most 32 runs of contiguous bits.
struct KeyPack {
  uint32_t nruns;
  uint32_t bits;  // total packed bits
  uint8_t src[32], width[32], dst[32];
};
KeyPack make_keypack(uint64_t varying);  // host
__device__ inline uint64_t keypack_apply(const KeyPack& p, uint64_t key) {
  uint64_t out = 0;
  for (uint32_t r = 0; r < p.nruns; r++) {
    const uint64_t m = p.width[r] == 64 ? ~0ull : ((1ull << p.width[r]) - 1ull);
    out |= ((key >> p.src[r]) & m) << p.dst[r];
  }
  return out;
}

}  // namespace dcc
