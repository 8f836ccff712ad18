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
//   k_df_list     (the level-0 compaction launch, occ_sweep.hip) the write and
//                 the read-only survivors as two lists by reference -- txn ids
//                 and batch access indices, no keys copied -- and one count per
//                 write access into its key's hash bucket (no key table: a
//                 bucket holds the writes of every key hashing to it)
//   k_df_alloc    one exclusive scan over the buckets (decoupled look-back, one
//                 workgroup per CU, all resident): each bucket's entries and
//                 group words; the counts are cleared for the next epoch
//   k_df_scatter  each write access becomes an entry {key, txn id} of its
//                 bucket (a cursor per bucket) and learns its word and bit
//   k_df_solve    persistent: each wave keeps a window of chunks (the write
//                 txns whose first access lies in a 64-access window of the
//                 list), a lane per access.  An access's relevant writers are a
//                 mask over its bucket's group words (entries of its key with a
//                 smaller txn id); it polls the word until the mask is all
//                 decided or a committed entry shows.  A decided txn ORs its
//                 bits into each of its writes' words: one atomic per write,
//                 seen by every later accessor.  The smallest undecided txn can
//                 always decide and its wave is resident, so the solver drains;
//                 a time limit hands a pathological epoch back to the levels.
//   k_df_ro       the read-only survivors: one with a committed entry of one
//                 of its keys with a smaller txn id aborts.
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

// k_df_alloc: bucket counts -> each bucket's first entry and first group word.
// DF_SCAN_WG workgroups, one per CU: each sums its bucket range (coalesced,
// bucket lo + 256 k + thread), publishes its total, sums the totals of the
// workgroups before it (all resident: the look-back is one round trip), then
// assigns its buckets in the same order, 256 per step.  The order of
// allocation is free: a bucket only needs a contiguous range.
__global__ __launch_bounds__(256) void k_df_alloc(DfArgs d) {
  __shared__ uint32_t sh[8];
  DfCtl* c = d.ctl;
  if (!c->live || !c->m) return;
  const uint32_t t = threadIdx.x;
  const uint32_t bits = c->bits;
  const uint32_t per = (1u << bits) / DF_SCAN_WG;  // 2^bits >= 2^DF_MIN_BITS
  const uint32_t lo = blockIdx.x * per;
  uint32_t np = 0, nw = 0;
  for (uint32_t k = t; k < per; k += 256) {
    const uint32_t v = d.bcnt[lo + k];
    np += v;
    nw += (v + 31u) / 32u;
  }
  uint32_t ep, ew, tp, tw;
  df_block_scan2(np, nw, ep, ew, tp, tw, sh);
  if (t == 0)
    __hip_atomic_store(&c->gran[blockIdx.x], (1ull << 63) | ((unsigned long long)tw << 32) | tp,
                       __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  // look-back: thread t < blockIdx.x waits for workgroup t's total
  uint32_t gp = 0, gw = 0;
  if (t < blockIdx.x) {
    unsigned long long g = 0;
    for (uint32_t spin = 0;; spin++) {
      g = __hip_atomic_load(&c->gran[t], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
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
  if (t == 0 && blockIdx.x == DF_SCAN_WG - 1) {
    c->nent = tbp + tp;
    c->nwords = tbw + tw;
    // group words are addressed by 27 bits in the solver
    if (tbw + tw >= (1u << 27)) atomicOr(&c->err, DF_E_FULL);
  }
  uint32_t rp = tbp, rw = tbw;
  for (uint32_t k0 = 0; k0 < per; k0 += 256) {  // uniform trip count
    const uint32_t q = lo + k0 + t;
    const uint32_t v = k0 + t < per ? d.bcnt[q] : 0u;
    const uint32_t ng = (v + 31u) / 32u;
    uint32_t xp, xw, sp, sw;
    df_block_scan2(v, ng, xp, xw, sp, sw, sh);
    if (k0 + t < per) {
      const uint32_t seg = rp + xp, gb = rw + xw;
      d.brec[q] = make_uint4(seg, gb, v, 0u);
      d.bcur[q] = seg;
      for (uint32_t g = 0; g < ng; g++) d.words[gb + g] = 0ull;
      if (v) d.bcnt[q] = 0u;  // clean for the next epoch
    }
    rp += sp;
    rw += sw;
  }
}

// k_df_scatter: each write access of the list becomes an entry of its bucket
// and learns its group word and bit (s_pub)
__global__ __launch_bounds__(256) void k_df_scatter(DfArgs d) {
  DfCtl* c = d.ctl;
  if (!c->live || !c->m) return;
  const uint32_t acc = c->acc, bits = c->bits;
  for (uint32_t a = blockIdx.x * 256 + threadIdx.x; a < acc; a += gridDim.x * 256) {
    const uint32_t tid = d.s_pub[a];
    if (tid == DF_NONE) continue;  // a read
    const uint64_t key = d.keys[d.s_x[a]];
    const uint32_t b = df_bucket(key, bits);
    const uint32_t pos = atomicAdd(&d.bcur[b], 1u);
    const uint4 r = d.brec[b];
    const uint32_t j = pos - r.x;
    d.ent[pos] = make_uint4((uint32_t)key, (uint32_t)(key >> 32), tid, 0u);
    d.s_pub[a] = ((r.y + j / 32u) << 5) | (j & 31u);
  }
}

// ---------------------------------------------------------------------------
// k_df_solve.  Per lane-slot x (access x of a window chunk, x < 128: a chunk
// holds the txns whose first access is in a 64-access window, so at most 127
// accesses) the wave keeps six words in LDS (struct of arrays):
constexpr uint32_t DF_F = 6;
enum : uint32_t { F_TID = 0, F_WORD = 1, F_MASK = 2, F_INFO = 3, F_PUB = 4, F_BX = 5 };
// F_INFO: txn's lane-slots [x0, x1) | flags | group
constexpr uint32_t I_LIVE = 1u << 16;   // the lane-slot holds an access
constexpr uint32_t I_DONE = 1u << 17;   // every relevant entry decided, none committed
constexpr uint32_t I_FIN = 1u << 19;    // the txn is decided
constexpr uint32_t I_GSHIFT = 20;       // current group (12 bits)
constexpr uint32_t DF_MAX_GROUPS = 1u << 12;

// relevant-entry mask of a group: entries of the key with a smaller txn id
__device__ inline uint32_t df_mask(const uint4* e, uint32_t cnt, uint64_t key, uint32_t tid) {
  uint32_t m = 0;
#pragma unroll 4
  for (uint32_t j = 0; j < cnt; j++) {
    const uint4 v = e[j];
    m |= ((((uint64_t)v.y << 32) | v.x) == key && v.z < tid ? 1u : 0u) << j;
  }
  return m;
}
// first group >= g with a relevant entry; false: none left (the key is clear)
__device__ inline bool df_group(const DfArgs& d, uint4 r, uint64_t key, uint32_t tid, uint32_t& g,
                                uint32_t& m) {
  const uint32_t ng = (r.z + 31u) / 32u;
  for (; g < ng; g++) {
    m = df_mask(d.ent + r.x + 32u * g, min(32u, r.z - 32u * g), key, tid);
    if (m) return true;
  }
  return false;
}

__global__ __launch_bounds__(256) void k_df_solve(DfArgs d) {
  __shared__ uint32_t ls[4][DF_QW][DF_F][128];
  const uint32_t lane = lane_id(), wv = threadIdx.x >> 6;
  DfCtl* c = d.ctl;
  if (!c->live || !c->m) return;
  const uint32_t nch = c->nchunks, bits = c->bits;
  const uint32_t W = gridDim.x * 4, wid = blockIdx.x * 4 + wv;
  uint32_t (*L)[DF_F][128] = ls[wv];
  uint32_t cid[DF_QW];
#pragma unroll
  for (uint32_t w = 0; w < DF_QW; w++) cid[w] = DF_NONE;
  uint32_t next = wid;
  const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
  uint32_t passes = 0, refills = 0, polls = 0;
  uint64_t t_ready = 0;
  unsigned long long* dbg = (d.dbg && wid < DF_DBG_WAVES) ? d.dbg + 8 * wid : nullptr;
  bool bail = false;
  for (;;) {
    // ---- refill empty window slots (their loads overlap)
    bool any = false;
#pragma unroll
    for (uint32_t w = 0; w < DF_QW; w++) {
      if (cid[w] == DF_NONE && next < nch) {
        cid[w] = next;
        next += W;
        refills++;
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
          uint32_t info = 0, word = 0, mask = 0, pub = DF_NONE, bx = 0;
          if (live) {
            info = x0 | (x1 << 8) | I_LIVE;
            bx = d.s_x[a0 + x];
            pub = d.s_pub[a0 + x];
            const uint64_t key = d.keys[bx];
            const uint4 r = d.brec[df_bucket(key, bits)];
            uint32_t g = 0, m = 0;
            if ((r.z + 31u) / 32u > DF_MAX_GROUPS) {
              atomicOr(&c->err, DF_E_FULL);
              info |= I_DONE;
            } else if (df_group(d, r, key, tid, g, m)) {
              word = r.y + g;
              mask = m;
              info |= g << I_GSHIFT;
            } else {
              info |= I_DONE;
            }
          }
          L[w][F_TID][x] = tid;
          L[w][F_WORD][x] = word;
          L[w][F_MASK][x] = mask;
          L[w][F_INFO][x] = info;
          L[w][F_PUB][x] = pub;
          L[w][F_BX][x] = bx;
        }
      }
      any |= cid[w] != DF_NONE;
    }
    if (!any || bail) break;
    if (dbg && !t_ready) t_ready = __builtin_amdgcn_s_memrealtime();
    // ---- poll every pending access's group word, all in flight together
    unsigned long long pv[DF_QW][2];
#pragma unroll
    for (uint32_t w = 0; w < DF_QW; w++)
#pragma unroll
      for (uint32_t k = 0; k < 2; k++) {
        pv[w][k] = 0;
        if (cid[w] == DF_NONE) continue;
        const uint32_t x = lane + 64 * k;
        const uint32_t info = L[w][F_INFO][x];
        if ((info & (I_LIVE | I_DONE | I_FIN)) != I_LIVE) continue;
        pv[w][k] = __hip_atomic_load(&d.words[L[w][F_WORD][x]], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        polls++;
      }
    // ---- evaluate
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
          const unsigned long long v = pv[w][k];
          const uint32_t m = L[w][F_MASK][x];
          if ((uint32_t)(v >> 32) & m) {  // a committed entry of the key precedes the txn
            kill[k] = true;
          } else if (((uint32_t)v & m) == m) {  // this group is clear: the next one
            const uint32_t tid = L[w][F_TID][x];
            const uint64_t key = d.keys[L[w][F_BX][x]];
            const uint4 r = d.brec[df_bucket(key, bits)];
            uint32_t g = (info >> I_GSHIFT) + 1u, nm = 0;
            if (df_group(d, r, key, tid, g, nm)) {
              L[w][F_WORD][x] = r.y + g;
              L[w][F_MASK][x] = nm;
              info = (info & ((1u << I_GSHIFT) - 1u)) | (g << I_GSHIFT);
            } else {
              info |= I_DONE;
            }
            L[w][F_INFO][x] = info;
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
            if (x == x0) d.state[L[w][F_TID][x]] = commit ? ST_COMMIT : ST_ABORT;
            const uint32_t pub = L[w][F_PUB][x];
            if (pub != DF_NONE) {
              const unsigned long long bit = 1ull << (pub & 31u);
              __hip_atomic_fetch_or(&d.words[pub >> 5], commit ? (bit | (bit << 32)) : bit,
                                    __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
            info |= I_FIN;
            L[w][F_INFO][x] = info;
          }
        }
        if ((info & (I_LIVE | I_FIN)) == I_LIVE) fin_all = false;
      }
      if (!ballot64(!fin_all)) cid[w] = DF_NONE;  // the chunk is decided
    }
    passes++;
    if ((passes & 15u) == 1) {  // the first pass too (a 0 limit gives up at once)
      const bool late = __builtin_amdgcn_s_memrealtime() - t0 > d.limit_ticks;
      const uint32_t e = __hip_atomic_load(&c->err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (late && lane == 0) atomicOr(&c->err, DF_E_SPIN);
      bail = late || (e & (DF_E_SPIN | DF_E_SCAN)) != 0;
    }
  }
  if (wid == 0 && lane == 0) c->passes = passes;
  if (dbg) {
    // polls summed over the wave's lanes
    uint32_t p = polls;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) p += __shfl_xor(p, o);
    if (lane == 0) {
      dbg[0] = t0;
      dbg[1] = t_ready;
      dbg[2] = __builtin_amdgcn_s_memrealtime();
      dbg[3] = passes;
      dbg[4] = refills;
      dbg[5] = p;
      dbg[6] = 1;
    }
  }
}

// k_df_ro: the read-only survivors, an access per thread: a committed entry
// of the access's key with a smaller txn id aborts the txn (k_df_list started
// it as committed; only aborts are stored here, so threads of one txn never
// disagree).  Every writer is decided: plain loads.
__global__ __launch_bounds__(256) void k_df_ro(DfArgs d) {
  DfCtl* c = d.ctl;
  if (!c->live || !c->m) return;  // no write survivors: every read-only one commits
  const uint32_t acc = c->acc_r, bits = c->bits;
  for (uint32_t a = blockIdx.x * 256 + threadIdx.x; a < acc; a += gridDim.x * 256) {
    const uint32_t tid = d.r_t[a];
    const uint64_t key = d.keys[d.r_x[a]];
    const uint4 r = d.brec[df_bucket(key, bits)];
    bool kill = false;
    for (uint32_t j = 0; j < r.z && !kill; j++) {
      const uint4 e = d.ent[r.x + j];
      if ((((uint64_t)e.y << 32) | e.x) == key && e.z < tid)
        kill = (d.words[r.y + j / 32u] >> (32u + (j & 31u))) & 1ull;
    }
    if (kill) d.state[tid] = ST_ABORT;
  }
}

// k_df_clear: the bucket counts clean (first use, growth, or after an epoch
// that stopped before k_df_alloc cleared them)
__global__ __launch_bounds__(256) void k_df_clear(DfArgs d, uint64_t buckets) {
  for (uint64_t q = (uint64_t)blockIdx.x * 256 + threadIdx.x; q < buckets; q += (uint64_t)gridDim.x * 256)
    d.bcnt[q] = 0u;
}

void launch_df_alloc(const DfArgs& a, hipStream_t st) { k_df_alloc<<<DF_SCAN_WG, 256, 0, st>>>(a); }
void launch_df_scatter(const DfArgs& a, unsigned grid, hipStream_t st) {
  k_df_scatter<<<grid ? grid : 1u, 256, 0, st>>>(a);
}
void launch_df_solve(const DfArgs& a, unsigned grid, hipStream_t st) {
  k_df_solve<<<grid ? grid : 1u, 256, 0, st>>>(a);
}
void launch_df_ro(const DfArgs& a, unsigned grid, hipStream_t st) {
  k_df_ro<<<grid ? grid : 1u, 256, 0, st>>>(a);
}
int df_solve_blocks_per_cu() {
  int nb = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, k_df_solve, 256, 0) != hipSuccess) nb = 1;
  return nb;
}
void launch_df_clear(const DfArgs& a, uint64_t buckets, hipStream_t st) {
  const uint64_t g = (buckets + 255) / 256;
  k_df_clear<<<(unsigned)(g < 8192 ? (g ? g : 1) : 8192), 256, 0, st>>>(a, buckets);
}

}  // namespace dcc
