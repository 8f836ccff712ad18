// Batch validation pass shared by k_prep (occ_kernels.hip) and
// the level-0 serial pass launch (occ_sweep.hip): offset validation, max txn
// length and write count over offsets + acctype, per-block partials that the
// host reduces after its one synchronisation (no same-address atomics: one
// word serialises device atomics at ~100/us, MI355X_MICROARCH.md "dequeue").
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include "occ_kernels.h"

namespace dcc {

// block reductions for workgroups of up to 16 waves (sh: 16 words)
__device__ inline uint32_t block_sum_u32(uint32_t v, uint32_t* sh) {
  for (int d = 32; d > 0; d >>= 1) v += __shfl_xor(v, d);
  __syncthreads();
  if ((threadIdx.x & 63) == 0) sh[threadIdx.x >> 6] = v;
  __syncthreads();
  uint32_t t = 0;
  for (uint32_t w = 0; w < (blockDim.x >> 6); w++) t += sh[w];
  return t;
}
__device__ inline uint32_t block_max_u32(uint32_t v, uint32_t* sh) {
  for (int d = 32; d > 0; d >>= 1) v = max(v, (uint32_t)__shfl_xor(v, d));
  __syncthreads();
  if ((threadIdx.x & 63) == 0) sh[threadIdx.x >> 6] = v;
  __syncthreads();
  uint32_t t = 0;
  for (uint32_t w = 0; w < (blockDim.x >> 6); w++) t = max(t, sh[w]);
  return t;
}

// workgroup `blk` of `nblk` (every thread of the workgroup calls it)
__device__ inline void prep_body(const uint32_t* __restrict__ off, uint64_t n, const uint8_t* __restrict__ at,
                          uint64_t nnz, uint64_t p, PrepPart* __restrict__ part, uint32_t blk,
                          uint32_t nblk) {
  __shared__ uint32_t sh[16];
  uint32_t len = 0, bad = 0, nw = 0, nwp = 0;
  const uint64_t tid = (uint64_t)blk * blockDim.x + threadIdx.x;
  const uint64_t stride = (uint64_t)nblk * blockDim.x;
  // writes inside the peel prefix [0, off[p]) size its key table
  const uint64_t lim = (p && p <= n) ? off[p] : 0;
  for (uint64_t t = tid; t < n; t += stride) {
    const uint32_t a0 = off[t], b0 = off[t + 1];
    if (b0 < a0) bad |= ERR_OFFSETS;
    else len = max(len, b0 - a0);
    if (t == 0 && a0 != 0) bad |= ERR_OFFSETS;
    if (t == n - 1 && b0 != nnz) bad |= ERR_OFFSETS;
  }
  // acctype: 16 bytes per thread per step when aligned
  for (uint64_t x = tid * 16; x < nnz; x += stride * 16) {
    if (x + 16 <= nnz && ((uintptr_t)(at + x) & 15) == 0) {
      const uint4 v = *reinterpret_cast<const uint4*>(at + x);
      const uint32_t w4[4] = {v.x, v.y, v.z, v.w};
      uint32_t c = 0, cp = 0;
      for (int q = 0; q < 4; q++)
        for (int bb = 0; bb < 4; bb++) {
          const uint32_t is = ((w4[q] >> (8 * bb)) & 0xFFu) == 1u;
          c += is;
          cp += (x + 4 * q + bb < lim) ? is : 0u;
        }
      nw += c;
      nwp += cp;
    } else {
      for (uint64_t y = x; y < nnz && y < x + 16; y++) {
        nw += at[y] == 1;
        nwp += (y < lim && at[y] == 1) ? 1u : 0u;
      }
    }
  }
  const uint32_t tl = block_max_u32(len, sh);
  const uint32_t tb = block_max_u32(bad, sh);  // error bits are 0/1 flags: max == or here
  const uint32_t tw = block_sum_u32(nw, sh);
  const uint32_t tp = block_sum_u32(nwp, sh);
  if (threadIdx.x == 0) part[blk] = PrepPart{tb, tl, tw, tp};
}

// The sweep's variant: the same checks and counts, plus the has-write byte of
// every txn (get_rw_set's wr_cnt > 0, occ.cpp:296-317), so the level filters
// never load access types.  One txn per lane: its access types are read as
// the aligned 4-byte words covering [off[t], off[t+1]) -- adjacent lanes read
// adjacent words, one ~1 KB span per wave instruction.  Txns longer than
// MAX_TXN_LEN are only measured (the host rejects the batch).
__device__ inline void prep_body_hasw(const uint32_t* __restrict__ off, uint64_t n,
                                      const uint8_t* __restrict__ at, uint64_t nnz,
                                      uint8_t* __restrict__ hasw, PrepPart* __restrict__ part,
                                      uint32_t blk, uint32_t nblk, uint32_t* errw = nullptr) {
  __shared__ uint32_t sh[16];
  uint32_t len = 0, bad = 0, nw = 0;
  const uint64_t tid = (uint64_t)blk * blockDim.x + threadIdx.x;
  const uint64_t stride = (uint64_t)nblk * blockDim.x;
  const uint32_t mis = (uint32_t)((uintptr_t)at & 3u);  // at = base + mis, base 4-aligned
  const uint32_t* base = (const uint32_t*)(at - mis);
  for (uint64_t t = tid; t < n; t += stride) {
    const uint32_t a0 = off[t], b0 = off[t + 1];
    if (b0 < a0) bad |= ERR_OFFSETS;
    else len = max(len, b0 - a0);
    if (t == 0 && a0 != 0) bad |= ERR_OFFSETS;
    if (t == n - 1 && b0 != nnz) bad |= ERR_OFFSETS;
    uint32_t c = 0;
    const uint64_t lo = a0, hi = min((uint64_t)b0, nnz);
    if (lo < hi && hi - lo <= MAX_TXN_LEN) {
      // byte positions relative to base: [lo + mis, hi + mis)
      const uint64_t p0 = lo + mis, p1 = hi + mis;
      for (uint64_t w = p0 >> 2; w < (p1 + 3) >> 2; w++) {
        const uint32_t v = base[w];
#pragma unroll
        for (uint32_t q = 0; q < 4; q++) {
          const uint64_t p = 4 * w + q;
          c += (p >= p0 && p < p1 && ((v >> (8 * q)) & 0xFFu) == 1u) ? 1u : 0u;
        }
      }
    }
    nw += c;
    hasw[t] = c ? 1 : 0;
  }
  const uint32_t tl = block_max_u32(len, sh);
  const uint32_t tb = block_max_u32(bad, sh);
  const uint32_t tw = block_sum_u32(nw, sh);
  if (threadIdx.x == 0) {
    part[blk] = PrepPart{tb, tl, tw, 0u};
    if (errw && ((tb & ERR_OFFSETS) || tl > MAX_TXN_LEN)) atomicOr(errw, ERR_PREP);
  }
}
}  // namespace dcc
