// The one-word grant-group scan state shared by the Calvin kernels
// (calvin.hip's global scan, calvin_bucket.hip's per-bucket scan).
//
// Over requests sorted by (row, sequence position), the grant group of a
// request is the number of group boundaries before it on its row, where two
// consecutive requests of a row are in different groups iff either is EX
// (row_lock.cpp:78-81, 152-170: an SH run shares the lock, every EX is alone).
// State of an interval: segment start (bit 0: the interval holds a row's first
// request), first and last lock type of its requests (2 bits each: SH, EX,
// NONE) and the boundaries since the segment's start (27 bits).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "dcc_device.h"

namespace dcc {

constexpr uint32_t CV_SH = 0, CV_EX = 1, CV_NONE = 2;

__host__ __device__ constexpr uint32_t gl_pack(uint32_t flag, uint32_t ft, uint32_t lt, uint32_t cnt) {
  return flag | (ft << 1) | (lt << 3) | (cnt << 5);
}
constexpr uint32_t GL_ID = gl_pack(0, CV_NONE, CV_NONE, 0);

__device__ inline uint32_t gl_combine(uint32_t A, uint32_t B) {
  if (B & 1u) return B;
  const uint32_t aft = (A >> 1) & 3u, alt = (A >> 3) & 3u, bft = (B >> 1) & 3u, blt = (B >> 3) & 3u;
  const bool bnd = alt != CV_NONE && bft != CV_NONE && (alt == CV_EX || bft == CV_EX);
  const uint32_t ft = aft != CV_NONE ? aft : bft;
  const uint32_t lt = blt != CV_NONE ? blt : alt;
  return (A & 1u) | (ft << 1) | (lt << 3) | (((A >> 5) + (B >> 5) + (bnd ? 1u : 0u)) << 5);
}

// Inclusive scan of a wave, then the block's exclusive prefix of each thread
// (blockDim.x / 64 waves, at most 16; the wave totals through LDS s_w); returns
// the exclusive prefix and the block total.
__device__ inline uint32_t gl_block_excl(uint32_t v, uint32_t* s_w, uint32_t& total) {
  const uint32_t lane = threadIdx.x & 63u, w = threadIdx.x >> 6, nw = blockDim.x >> 6;
  uint32_t x = v;
#pragma unroll
  for (uint32_t d = 1; d < 64; d <<= 1) {
    const uint32_t y = __shfl_up(x, d);
    if (lane >= d) x = gl_combine(y, x);
  }
  if (lane == 63) s_w[w] = x;
  __syncthreads();
  uint32_t wp = GL_ID;
  total = GL_ID;
  for (uint32_t q = 0; q < nw; q++) {
    if (q < w) wp = gl_combine(wp, s_w[q]);
    total = gl_combine(total, s_w[q]);
  }
  const uint32_t ex_in = __shfl_up(x, 1);
  __syncthreads();
  return gl_combine(wp, lane ? ex_in : GL_ID);
}

}  // namespace dcc
