// gfx950 kernels of the OCC dataflow solver: decides the txns
// level 0 of the sweep leaves undecided -- its survivors, write and read-only
// txns in index order -- without further levels, rounds or grid barriers.
//
// The serial decision (central_validate in index order, occ.cpp:116-239, then
// central_finish, occ.cpp:248-294) is
//
//   abort(t)  <=>  some EARLIER committed txn wrote a key t reads or writes
//
// (read-only txns never enter `active`, occ.cpp:151-154; only WR joins the
// write set, occ.cpp:296-317).  A key's first committed writer kills every
// later accessor, so a key has at most one committed writer, and t's fate on
// key K is settled once every writer of K with a smaller txn id is decided:
// t is killed if one of them committed, K is clear for t if all aborted.  t
// commits when all its keys are clear.  The survivors of level 0 touch no key
// level 0 committed, so only list txns matter.
//
//   k_df_list     (the level-0 compaction launch, occ_sweep.hip) the
//                 survivors by reference -- txn ids and access offsets into the
//                 batch's CSR, no keys copied -- and every write key entered in
//                 the table (tkey), its writers counted (tnw: the write's rank)
//   k_df_alloc    one exclusive scan over the table (decoupled look-back, one
//                 workgroup per CU, all resident): each key's writer entries and
//                 group words (one 64-bit word per 32 writers)
//   k_df_scatter  writers' txn ids into their key's entries; reads find their
//                 key's slot (a key no list txn writes cannot conflict)
//   k_df_solve    persistent: each wave keeps a window of chunks (the txns whose
//                 first access lies in a 64-access window of the list), a lane
//                 per access.  An access's relevant writers are a mask over its
//                 key's group words (writers with a smaller txn id); it polls
//                 the word until the mask is all decided or a committed writer
//                 shows.  A decided txn ORs its bit into each of its write
//                 keys' words (with ~txn id on commit): one atomic per write,
//                 seen by every later accessor.  The smallest undecided txn can
//                 always decide and its wave is resident, so the solver drains;
//                 a time limit hands a pathological epoch back to the levels.
#include <hip/hip_runtime.h>

#include "dcc_device.h"
#include "occ_kernels.h"
#include "occ_dataflow.h"

namespace dcc {

// ---------------------------------------------------------------------------
// 256-thread block scan of two u32 counters (exclusive; totals returned)
__device__ inline void df_block_scan2(uint32_t p, uint32_t w, uint32_t& ep, uint32_t& ew, uint32_t& tp,
                                      uint32_t& tw, uint32_t* sh /*[8]*/) {
  const uint32_t lane = lane_id(), wv = threadIdx.x >> 6;
  uint32_t ip = p, iw = w;
#pragma unroll
  for (int dd = 1; dd < 64; dd <<= 1) {
    const uint32_t yp = __shfl_up(ip, dd), yw = __shfl_up(iw, dd);
    if (lane >= (uint32_t)dd) {
      ip += yp;
      iw += yw;
    }
  }
  if (lane == 63) {
    sh[wv] = ip;
    sh[4 + wv] = iw;
  }
  __syncthreads();
  uint32_t bp = 0, bw = 0;
  tp = 0;
  tw = 0;
  for (uint32_t q = 0; q < 4; q++) {
    if (q < wv) {
      bp += sh[q];
      bw += sh[4 + q];
    }
    tp += sh[q];
    tw += sh[4 + q];
  }
  ep = bp + ip - p;
  ew = bw + iw - w;
  __syncthreads();
}

// k_df_alloc: the table's writer counts -> each key's first entry and first
// group word (slot order).  DF_SCAN_WG workgroups, one per CU: each scans its
// slot range, publishes its total, and sums the totals of the workgroups
// before it (they are all resident, so the look-back is one round trip).
__global__ __launch_bounds__(256) void k_df_alloc(DfArgs d) {
  __shared__ uint32_t sh[8];
  __shared__ uint32_t s_base[2];
  DfCtl* c = d.ctl;
  if (!c->live) return;
  const uint32_t bits = c->bits;
  const uint64_t cap = 1ull << bits;
  const uint64_t per = cap / DF_SCAN_WG;  // cap >= 2^DF_MIN_BITS
  const uint64_t lo = (uint64_t)blockIdx.x * per;
  const uint32_t T = (uint32_t)((per + 255) / 256);
  const uint64_t s0 = min(lo + (uint64_t)threadIdx.x * T, lo + per), s1 = min(s0 + T, lo + per);
  uint32_t np = 0, nw = 0;
  for (uint64_t q = s0; q < s1; q++) {
    const uint32_t v = d.tnw[q];
    np += v;
    nw += (v + 31u) / 32u;
  }
  uint32_t ep, ew, tp, tw;
  df_block_scan2(np, nw, ep, ew, tp, tw, sh);
  if (threadIdx.x == 0)
    __hip_atomic_store(&c->gran[blockIdx.x], (1ull << 63) | ((unsigned long long)tw << 32) | tp,
                       __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  // look-back: thread t < blockIdx.x waits for workgroup t's total
  uint32_t gp = 0, gw = 0;
  if (threadIdx.x < blockIdx.x) {
    unsigned long long g = 0;
    for (uint32_t spin = 0;; spin++) {
      g = __hip_atomic_load(&c->gran[threadIdx.x], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (g >> 63) break;
      if (spin > (1u << 22)) {  // a predecessor never ran (not resident): give up
        atomicOr(&c->err, DF_E_SCAN);
        break;
      }
      __builtin_amdgcn_s_sleep(1);
    }
    gp = (uint32_t)g;
    gw = (uint32_t)(g >> 32) & 0x7FFFFFFFu;
  }
  uint32_t bp_, bw_, tbp, tbw;
  df_block_scan2(gp, gw, bp_, bw_, tbp, tbw, sh);
  (void)bp_;
  (void)bw_;
  if (threadIdx.x == 0) {
    s_base[0] = tbp;
    s_base[1] = tbw;
    if (blockIdx.x == DF_SCAN_WG - 1) {
      c->npos = tbp + tp;
      c->nwords = tbw + tw;
      // group words are addressed by 27 bits in the solver
      if (tbw + tw >= (1u << 27)) atomicOr(&c->err, DF_E_FULL);
    }
  }
  __syncthreads();
  uint32_t rp = s_base[0] + ep, rw = s_base[1] + ew;
  for (uint64_t q = s0; q < s1; q++) {
    const uint32_t v = d.tnw[q];
    if (!v) continue;
    const uint32_t ng = (v + 31u) / 32u;
    d.trec[q] = make_uint4(rp, rw, v, ~0u);
    for (uint32_t k = 0; k < ng; k++) d.words[rw + k] = 0ull;
    rp += v;
    rw += ng;
  }
}

// k_df_scatter: every list access -- a write's txn id into its key's writer
// entries; a read's key slot (DF_NONE: no list txn writes the key)
__global__ __launch_bounds__(256) void k_df_scatter(DfArgs d) {
  DfCtl* c = d.ctl;
  if (!c->live) return;
  const uint32_t acc = c->acc, bits = c->bits;
  for (uint32_t a = blockIdx.x * 256 + threadIdx.x; a < acc; a += gridDim.x * 256) {
    const uint32_t sl = d.s_slot[a];
    if (sl == DF_PEND) {
      d.s_slot[a] = df_find(d.tkey, bits, d.keys[d.s_x[a]]);
    } else if (sl != DF_NONE) {
      const uint32_t r = d.s_rank[a];
      d.wtid[d.trec[sl].x + r] = d.s_x[a];
    }
  }
}

// ---------------------------------------------------------------------------
// k_df_solve.  Per lane-slot x (access x of a window chunk, x < 128: a chunk
// holds the txns whose first access is in a 64-access window, so at most 127
// accesses) the wave keeps six words in LDS (struct of arrays):
constexpr uint32_t DF_F = 6;
enum : uint32_t { F_TID = 0, F_WORD = 1, F_MASK = 2, F_INFO = 3, F_PUB = 4, F_SLOT = 5 };
// F_INFO: txn's lane-slots [x0, x1) | flags | group
constexpr uint32_t I_LIVE = 1u << 16;   // the lane-slot holds an access
constexpr uint32_t I_DONE = 1u << 17;   // every relevant writer decided, none committed
constexpr uint32_t I_MULTI = 1u << 18;  // the key has > 32 writers (groups, committed-writer word)
constexpr uint32_t I_FIN = 1u << 19;    // the txn is decided
constexpr uint32_t I_GSHIFT = 20;       // current group (12 bits)
constexpr uint32_t DF_MAX_GROUPS = 1u << 12;

// relevant-writer mask of a group: entries with a smaller txn id
__device__ inline uint32_t df_mask(const uint32_t* e, uint32_t cnt, uint32_t tid) {
  uint32_t m = 0;
#pragma unroll 8
  for (uint32_t j = 0; j < cnt; j++) m |= (e[j] < tid ? 1u : 0u) << j;
  return m;
}
// first group >= g with a relevant writer; false: none left (the key is clear)
__device__ inline bool df_group(const DfArgs& d, uint4 r, uint32_t tid, uint32_t& g, uint32_t& m) {
  const uint32_t ng = (r.z + 31u) / 32u;
  for (; g < ng; g++) {
    m = df_mask(d.wtid + r.x + 32u * g, min(32u, r.z - 32u * g), tid);
    if (m) return true;
  }
  return false;
}

__global__ __launch_bounds__(256) void k_df_solve(DfArgs d) {
  __shared__ uint32_t ls[4][DF_QW][DF_F][128];
  const uint32_t lane = lane_id(), wv = threadIdx.x >> 6;
  DfCtl* c = d.ctl;
  if (!c->live) return;
  const uint32_t nch = c->nchunks;
  const uint32_t W = gridDim.x * 4, wid = blockIdx.x * 4 + wv;
  uint32_t (*L)[DF_F][128] = ls[wv];
  uint32_t cid[DF_QW];
#pragma unroll
  for (uint32_t w = 0; w < DF_QW; w++) cid[w] = DF_NONE;
  uint32_t next = wid;
  const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
  uint32_t passes = 0;
  bool bail = false;
  for (;;) {
    // ---- refill empty window slots (their loads overlap)
    bool any = false;
#pragma unroll
    for (uint32_t w = 0; w < DF_QW; w++) {
      if (cid[w] == DF_NONE && next < nch) {
        cid[w] = next;
        next += W;
        const uint32_t ch = cid[w];
        const uint32_t p0 = d.cfirst[ch], p1 = d.cfirst[ch + 1];
        const uint32_t nt = p1 - p0;
        const uint32_t a0 = d.s_aoff[p0];
        const uint32_t na = d.s_aoff[p1] - a0;
        const uint32_t ao = lane < nt ? d.s_aoff[p0 + lane] - a0 : na;
        const uint32_t tt = lane < nt ? d.s_tid[p0 + lane] : 0u;
#pragma unroll
        for (uint32_t k = 0; k < 2; k++) {
          const uint32_t x = lane + 64 * k;
          // owner txn: the last lane l < nt with ao[l] <= x
          uint32_t l = 0;
#pragma unroll
          for (uint32_t st = 32; st > 0; st >>= 1) {
            const uint32_t v = __shfl(ao, min(l + st, 63u));
            if (l + st < nt && v <= x) l += st;
          }
          const uint32_t x0 = __shfl(ao, l);
          const uint32_t x1n = __shfl(ao, min(l + 1, 63u));
          const uint32_t x1 = l + 1 < nt ? x1n : na;
          const uint32_t tid = __shfl(tt, l);
          const bool live = x < na;
          uint32_t info = 0, word = 0, mask = 0, pub = DF_NONE, slot = DF_NONE;
          if (live) {
            info = x0 | (x1 << 8) | I_LIVE;
            slot = d.s_slot[a0 + x];
            const uint32_t rk = d.s_rank[a0 + x];
            if (slot == DF_NONE) {
              info |= I_DONE;
            } else {
              const uint4 r = d.trec[slot];
              if (rk != DF_NONE) pub = ((r.y + rk / 32u) << 5) | (rk & 31u);
              if (r.z > 32u) info |= I_MULTI;
              uint32_t g = 0, m = 0;
              if ((r.z + 31u) / 32u > DF_MAX_GROUPS) {
                atomicOr(&c->err, DF_E_FULL);
                info |= I_DONE;
              } else if (df_group(d, r, tid, g, m)) {
                word = r.y + g;
                mask = m;
                info |= g << I_GSHIFT;
              } else {
                info |= I_DONE;
              }
            }
          }
          L[w][F_TID][x] = tid;
          L[w][F_WORD][x] = word;
          L[w][F_MASK][x] = mask;
          L[w][F_INFO][x] = info;
          L[w][F_PUB][x] = pub;
          L[w][F_SLOT][x] = slot;
        }
      }
      any |= cid[w] != DF_NONE;
    }
    if (!any || bail) break;
    // ---- poll: every pending access's group word (and, for keys with more
    // than 32 writers, the committed-writer word), all in flight together
    unsigned long long pv[DF_QW][2];
    uint32_t cw[DF_QW][2];
#pragma unroll
    for (uint32_t w = 0; w < DF_QW; w++)
#pragma unroll
      for (uint32_t k = 0; k < 2; k++) {
        pv[w][k] = 0;
        cw[w][k] = ~0u;
        if (cid[w] == DF_NONE) continue;
        const uint32_t x = lane + 64 * k;
        const uint32_t info = L[w][F_INFO][x];
        if ((info & (I_LIVE | I_DONE | I_FIN)) != I_LIVE) continue;
        pv[w][k] = __hip_atomic_load(&d.words[L[w][F_WORD][x]], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (info & I_MULTI)
          cw[w][k] = __hip_atomic_load(&d.trec[L[w][F_SLOT][x]].w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
    // ---- evaluate
    bool progress = false;
#pragma unroll
    for (uint32_t w = 0; w < DF_QW; w++) {
      if (cid[w] == DF_NONE) continue;
      bool kill[2], done[2];
#pragma unroll
      for (uint32_t k = 0; k < 2; k++) {
        const uint32_t x = lane + 64 * k;
        uint32_t info = L[w][F_INFO][x];
        kill[k] = false;
        if ((info & (I_LIVE | I_DONE | I_FIN)) == I_LIVE) {
          const uint32_t tid = L[w][F_TID][x];
          const unsigned long long v = pv[w][k];
          const uint32_t hi = (uint32_t)(v >> 32);
          if ((hi && ~hi < tid) || cw[w][k] < tid) {
            kill[k] = true;
          } else {
            const uint32_t m = L[w][F_MASK][x];
            if (((uint32_t)v & m) == m) {  // this group is clear: the next one
              uint32_t g = (info >> I_GSHIFT) + 1u, nm = 0;
              bool more = false;
              uint4 r = make_uint4(0, 0, 0, 0);
              if (info & I_MULTI) {
                r = d.trec[L[w][F_SLOT][x]];
                more = df_group(d, r, tid, g, nm);
              }
              if (more) {
                L[w][F_WORD][x] = r.y + g;
                L[w][F_MASK][x] = nm;
                info = (info & ((1u << I_GSHIFT) - 1u)) | (g << I_GSHIFT);
              } else {
                info |= I_DONE;
              }
              L[w][F_INFO][x] = info;
            }
          }
        }
        done[k] = (info & I_DONE) != 0;
      }
      const uint64_t K0 = ballot64(kill[0]), K1 = ballot64(kill[1]);
      const uint64_t D0 = ballot64(done[0]), D1 = ballot64(done[1]);
      bool fin_all = true;
#pragma unroll
      for (uint32_t k = 0; k < 2; k++) {
        const uint32_t x = lane + 64 * k;
        uint32_t info = L[w][F_INFO][x];
        if ((info & (I_LIVE | I_FIN)) == I_LIVE) {
          const uint32_t x0 = info & 0xFFu, x1 = (info >> 8) & 0xFFu;
          // the txn's lane-slots [x0, x1) as two 64-bit masks
          const uint32_t a0 = min(x0, 64u), a1 = min(x1, 64u);
          const uint32_t b0 = max(x0, 64u) - 64u, b1 = max(x1, 64u) - 64u;
          const uint64_t R0 = a1 > a0 ? (((a1 - a0) == 64 ? ~0ull : ((1ull << (a1 - a0)) - 1ull)) << a0) : 0ull;
          const uint64_t R1 = b1 > b0 ? (((b1 - b0) == 64 ? ~0ull : ((1ull << (b1 - b0)) - 1ull)) << b0) : 0ull;
          const bool tk = ((K0 & R0) | (K1 & R1)) != 0;
          const bool td = (D0 & R0) == R0 && (D1 & R1) == R1;
          if (tk || td) {
            const bool commit = !tk;
            const uint32_t tid = L[w][F_TID][x];
            if (x == x0) d.state[tid] = commit ? ST_COMMIT : ST_ABORT;
            const uint32_t pub = L[w][F_PUB][x];
            if (pub != DF_NONE) {
              const uint32_t slot = L[w][F_SLOT][x];
              const unsigned long long bit = (1ull << (pub & 31u)) |
                                             (commit ? ((unsigned long long)(~tid) << 32) : 0ull);
              if (commit && (info & I_MULTI)) atomicMin(&d.trec[slot].w, tid);
              __hip_atomic_fetch_or(&d.words[pub >> 5], bit, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
              // the table back to clean for the next epoch (no reader of this
              // launch looks at tkey / tnw)
              d.tkey[slot] = KEY_EMPTY;
              d.tnw[slot] = 0u;
            }
            info |= I_FIN;
            L[w][F_INFO][x] = info;
            progress = true;
          }
        }
        if ((info & (I_LIVE | I_FIN)) == I_LIVE) fin_all = false;
      }
      if (!ballot64(!fin_all)) cid[w] = DF_NONE;  // the chunk is decided
    }
    passes++;
    (void)progress;
    if ((passes & 15u) == 1) {  // the first pass too (a 0 limit gives up at once)
      const bool late = __builtin_amdgcn_s_memrealtime() - t0 > d.limit_ticks;
      const uint32_t e = __hip_atomic_load(&c->err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (late && lane == 0) atomicOr(&c->err, DF_E_SPIN);
      bail = late || (e & (DF_E_SPIN | DF_E_SCAN)) != 0;
    }
  }
  if (wid == 0 && lane == 0) c->passes = passes;
}

// k_df_clear: the whole table clean (first use, growth, or after an epoch
// that stopped before its solver reset the slots it used)
__global__ __launch_bounds__(256) void k_df_clear(DfArgs d, uint64_t slots) {
  for (uint64_t q = (uint64_t)blockIdx.x * 256 + threadIdx.x; q < slots; q += (uint64_t)gridDim.x * 256) {
    d.tkey[q] = KEY_EMPTY;
    d.tnw[q] = 0u;
  }
}

void launch_df_alloc(const DfArgs& a, hipStream_t st) { k_df_alloc<<<DF_SCAN_WG, 256, 0, st>>>(a); }
void launch_df_scatter(const DfArgs& a, unsigned grid, hipStream_t st) {
  k_df_scatter<<<grid ? grid : 1u, 256, 0, st>>>(a);
}
void launch_df_solve(const DfArgs& a, unsigned grid, hipStream_t st) {
  k_df_solve<<<grid ? grid : 1u, 256, 0, st>>>(a);
}
int df_solve_blocks_per_cu() {
  int nb = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, k_df_solve, 256, 0) != hipSuccess) nb = 1;
  return nb;
}
void launch_df_clear(const DfArgs& a, uint64_t slots, hipStream_t st) {
  const uint64_t g = (slots + 255) / 256;
  k_df_clear<<<(unsigned)(g < 8192 ? (g ? g : 1) : 8192), 256, 0, st>>>(a, slots);
}

}  // namespace dcc
