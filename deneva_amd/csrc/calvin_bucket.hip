// Calvin grant groups by key buckets on gfx950 (see calvin_bucket.h).
//
// Same result as calvin.hip's key sort + group scan + windowed put (grant
// group = group boundaries before the request on its row, in sequence order;
// row_lock.cpp:78-81, 152-170, 317-357), with the data moved fewer times:
//
//   k_cb_count   requests in sequence order, per tile of 64 x 1024 / ulen
//                txns: counts of the 2^bb buckets (low packed-key bits)
//   k_cb_scan    per bucket, exclusive scan of its tile counts
//   k_cb_part    the stable partition: each tile's requests -- packed key and
//                (txn, j, EX) -- ranked per wave, staged in LDS by bucket and
//                written to the buckets' runs (bucket order = sequence order)
//   k_cb_bucket  one workgroup per bucket, 4,096-request chunks in order: an
//                LDS radix sort of the chunk by the row bits above the bucket
//                bits (stable, so a row's requests stay in sequence order),
//                the grant-group scan with each row's state carried across
//                chunks in an LDS table indexed by those bits (hashed on them
//                past 13 bits, up to 17: TPC-C), and the
//                (request, group) pairs staged by output window and appended
//                to the window's region (one returning atomic per window and
//                chunk, on one of R replicated counters)
//   k_cb_put     one workgroup per window of 2^tsh txns: the window's groups
//                placed in LDS, stored whole, and the txns' readiness
//                (acquire_locks' RCOK iff every request is in group 0,
//                ycsb_txn.cpp:76-79)
#include "calvin_bucket.h"

#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdlib>

#include "calvin_gl.h"
#include "dcc.h"
#include "dcc_device.h"
#include "dcc_env.h"

// The DCC_CB_VARIANT timing variants (kernels with one phase removed, wrong
// results by design) exist only in -DDCC_EXPERIMENTS builds: in the product
// build every variant test is a compile-time 0.
#ifdef DCC_EXPERIMENTS
#define CB_VAR(v, bit) ((v) & (bit))
#else
#define CB_VAR(v, bit) 0u
#endif

namespace dcc {
namespace {

constexpr uint32_t CB_PT = 512;                 // count / partition threads (8 waves)
constexpr uint32_t CB_SUB = CB_PT * 16;         // requests per partition sub-tile (LDS staging)
constexpr uint32_t CB_NSUB = 8;                 // sub-tiles per tile
constexpr uint32_t CB_BB_MAX = 11;              // bucket bits
constexpr uint32_t CB_LB_MAX = 13;              // row bits inside a bucket (direct carry table)
constexpr uint32_t CB_LB_HASH_MAX = 17;         // ... with the hashed carry table
constexpr uint32_t CB_HSLOTS = 1u << CB_LB_MAX; // hashed table slots (the same 32 KiB of LDS)
constexpr uint32_t CB_HWALK = 64;               // longest probe of a hashed slot
constexpr uint32_t CB_HCNT_MAX = (1u << 12) - 1;  // group counts a tagged word holds (below)
constexpr uint32_t CB_BT = 256;                 // bucket workgroup
constexpr uint32_t CB_IT = 16;                  // requests per thread per chunk
constexpr uint32_t CB_CHUNK = CB_BT * CB_IT;
constexpr uint32_t CB_STG = CB_CHUNK + CB_CHUNK / 32;  // one pad slot per 32 (bank spread)
constexpr uint32_t CB_NDIG_MAX = 760;           // output windows (LDS: two bucket workgroups per CU)
constexpr uint32_t CB_WIN = 32768;              // groups per output window (128 KiB of LDS)
constexpr uint32_t CB_R = 8;                    // reservation-counter replicas
constexpr uint32_t CB_TSH_RAGGED = 11;          // ragged txns: at most 2^11 txns per output window
constexpr uint32_t NOTXN = 0xFFFFFFFFu;
// carry-table word: bit 0 "the row's last request is the chunk's last txn",
// bits 1-2 its lock type (CV_NONE: row not seen yet), bits 3.. its group count
constexpr uint32_t TAB_EMPTY = CV_NONE << 1;
// Hashed carry table (row bits 14-17: TPC-C's packed keys are 28 bits at 128
// warehouses): the word is tagged -- row bits 31..15, group count 14..3 -- in
// open addressing over the same 8,192 LDS words; a bucket's rows never leave
// it, so linear probing needs no deletion.  A row whose probe runs past
// CB_HWALK slots or whose group count outgrows 12 bits raises CB_ERR_TAB and
// the host redoes the epoch on the sort path.
constexpr uint32_t TAB_HEMPTY = 0xFFFFFFFFu;
__device__ inline uint32_t cb_hslot(uint32_t r) { return (r * 0x9E3779B1u) >> (32 - CB_LB_MAX); }
// the carry word of row r (TAB_EMPTY: not seen in this bucket yet), from its
// first probe w at slot h
__device__ inline uint32_t cb_hget(const uint32_t* t, uint32_t r, uint32_t h, uint32_t w) {
  for (uint32_t q = 1; w != TAB_HEMPTY && (w >> 15) != r && q < CB_HWALK; q++) {
    h = (h + 1) & (CB_HSLOTS - 1);
    w = *(volatile const uint32_t*)&t[h];
  }
  return (w == TAB_HEMPTY || (w >> 15) != r) ? TAB_EMPTY : (w & 0x7FFFu);
}
// store row r's carry word v (untagged); returns its slot (CB_HSLOTS: no room)
__device__ inline uint32_t cb_hput(uint32_t* t, uint32_t r, uint32_t v, uint32_t* err) {
  if ((v >> 3) >= CB_HCNT_MAX) {
    atomicOr(err, CB_ERR_TAB);
    return CB_HSLOTS;
  }
  const uint32_t wn = (r << 15) | v;
  uint32_t h = cb_hslot(r);
  for (uint32_t q = 0; q < CB_HWALK;) {
    const uint32_t w = *(volatile uint32_t*)&t[h];
    if (w == TAB_HEMPTY) {
      if (atomicCAS(&t[h], TAB_HEMPTY, wn) == TAB_HEMPTY) return h;
      continue;  // another row took the slot: look at it again
    }
    if ((w >> 15) == r) {  // this row's slot (one writer per row and chunk)
      t[h] = wn;
      return h;
    }
    h = (h + 1) & (CB_HSLOTS - 1);
    q++;
  }
  atomicOr(err, CB_ERR_TAB);
  return CB_HSLOTS;
}

__device__ inline uint32_t stg_ix(uint32_t p) { return p + (p >> 5); }

// LDS-only workgroup barrier: waits for this wave's LDS operations, not for
// its outstanding global loads, stores or returning atomics.
__device__ inline void lds_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

// Exclusive add-scan of one u32 per thread over the workgroup (LDS barriers
// only); s_w holds one word per wave.
__device__ inline uint32_t blk_excl_add(uint32_t v, uint32_t* s_w, uint32_t& total) {
  const uint32_t lane = threadIdx.x & 63u, w = threadIdx.x >> 6, nw = blockDim.x >> 6;
  uint32_t x = v;
#pragma unroll
  for (uint32_t d = 1; d < 64; d <<= 1) {
    const uint32_t y = __shfl_up(x, d);
    if (lane >= d) x += y;
  }
  lds_barrier();  // s_w free (an earlier call's readers are done)
  if (lane == 63) s_w[w] = x;
  lds_barrier();
  uint32_t off = 0;
  total = 0;
  for (uint32_t q = 0; q < nw; q++) {
    const uint32_t s = s_w[q];
    if (q < w) off += s;
    total += s;
  }
  return off + x - v;
}

// Lanes of the wave whose nbits-bit bucket equals this lane's (NB > 0: a
// compile-time bit count, the loop unrolled).
template <uint32_t NB>
__device__ inline uint64_t bucket_peers(uint32_t d, bool act, uint32_t nbits) {
  uint64_t m = ballot64(act);
  if (NB) {
#pragma unroll
    for (uint32_t b = 0; b < NB; b++) {
      const bool bit = (d >> b) & 1u;
      const uint64_t bb = ballot64(bit);
      m &= bit ? bb : ~bb;
    }
  } else {
    for (uint32_t b = 0; b < nbits; b++) {
      const bool bit = (d >> b) & 1u;
      const uint64_t bb = ballot64(bit);
      m &= bit ? bb : ~bb;
    }
  }
  return act ? m : 0ull;
}

struct CbSrc {
  const uint64_t* keys;
  const uint8_t* at;
  const uint32_t* seq;
  const uint32_t* off;  // index-order offsets (ragged txns)
  uint32_t n;     // txns
  uint32_t ulen;  // requests per txn (0: ragged, at most maxlen each)
  uint32_t um;    // (2^20 + ulen - 1) / ulen: e / ulen == (e * um) >> 20 for e <= 1024
  uint32_t wt;    // txns per wave and sub-tile (1024 / ulen, or 1024 / maxlen)
  uint32_t nnz;
  uint32_t var;   // DCC_CB_VARIANT timing variants (wrong results): 1 no partition stores,
                  // 2 no ranking, 4 no element loads
  KeyPack kp;
};

// Wave w's share of a sub-tile: sequence positions [q0, q0 + nq), nq <= wt.
// Their txn ids are staged in LDS (s_t, this wave's 1024 words; one round
// trip for nq <= 64), then element e = 64 it + lane (< nq * ulen) is request
// e % ulen of txn e / ulen: every key (and type) load of the wave is issued
// before the first is used.  FULL: the element (packed key high, txn:25 |
// j:6 | EX:1 low), else the packed key alone; past the end ~0 (sorts last).
//
// Ragged txns (s.ulen == 0, each at most 1024 / wt requests): the wave also
// stages each txn's first request (s_b) and a map from its element to (txn
// slot, request) (s_m, built from a wave scan of the lengths), so element e
// finds its request with one LDS read instead of a division.
template <bool FULL>
__device__ inline uint32_t cb_wave_elems(const CbSrc& s, uint32_t q0, uint32_t nq, uint32_t* s_t,
                                         uint32_t* s_b, uint16_t* s_m, uint64_t (&el)[16]) {
  const uint32_t lane = threadIdx.x & 63u;
  if (nq == 0) {
#pragma unroll
    for (uint32_t it = 0; it < 16; it++) el[it] = ~0ull;
    return 0;
  }
  const uint32_t nk = (nq + 63) / 64;
  uint32_t ne = nq * s.ulen;
  if (s.ulen) {
    for (uint32_t k = 0; k < nk; k++) {
      const uint32_t i = k * 64 + lane;
      if (i < nq) s_t[i] = s.seq ? s.seq[q0 + i] : q0 + i;
    }
  } else {
    uint32_t run = 0;
    for (uint32_t k = 0; k < nk; k++) {
      const uint32_t i = k * 64 + lane;
      uint32_t t = 0, b = 0, len = 0;
      if (i < nq) {
        t = s.seq ? s.seq[q0 + i] : q0 + i;
        b = min(s.off[t], s.nnz);
        const uint32_t e = min(max(s.off[t + 1], b), s.nnz);
        len = min(e - b, 64u);  // MAX_ROW_PER_TXN (the prep validated it)
        s_t[i] = t;
        s_b[i] = b;  // (the count pass passes s_b == s_t: only b is read there)
      }
      uint32_t x = len;  // inclusive wave scan of the lengths
#pragma unroll
      for (uint32_t d = 1; d < 64; d <<= 1) {
        const uint32_t y = __shfl_up(x, d);
        if (lane >= d) x += y;
      }
      const uint32_t p = run + x - len;
      // (the plan keeps wt * maxlen <= 1024; the clamp only guards the LDS)
      for (uint32_t r = 0; r < len && p + r < 1024u; r++) s_m[p + r] = (uint16_t)((i << 6) | r);
      run += __shfl(x, 63);
    }
    ne = min(run, 1024u);
  }
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  if (ne == 0) {
#pragma unroll
    for (uint32_t it = 0; it < 16; it++) el[it] = ~0ull;
    return 0;
  }
  uint64_t kk[16];
  uint32_t tj[16];
  uint8_t aa[16];
#pragma unroll
  for (uint32_t it = 0; it < 16; it++) {
    const uint32_t e = min(it * 64 + lane, ne - 1);
    uint32_t i, j;
    uint64_t x;
    if (s.ulen) {
      i = (e * s.um) >> 20;
      j = e - i * s.ulen;
      x = (uint64_t)s_t[i] * s.ulen + j;
    } else {
      const uint32_t m = s_m[e];
      i = m >> 6;
      j = m & 63u;
      x = (uint64_t)s_b[i] + j;
    }
    const uint32_t t = s_t[i];
    kk[it] = s.keys[x];
    if (FULL) aa[it] = s.at[x];
    tj[it] = (t << 7) | (j << 1);
  }
#pragma unroll
  for (uint32_t it = 0; it < 16; it++) {
    const uint32_t pk = (uint32_t)keypack_apply(s.kp, kk[it]);
    if (it * 64 + lane >= ne)
      el[it] = ~0ull;
    else if (FULL)
      el[it] = ((uint64_t)pk << 32) | tj[it] | ((aa[it] != DCC_RD && aa[it] != DCC_SCAN) ? 1u : 0u);
    else
      el[it] = pk;
  }
  return ne;
}

// ---------------------------------------------------------------- count
// A tile is CB_NSUB sub-tiles of 8 waves x wt txns in sequence order (wave w
// of sub-tile u: positions tile_q0 + (8u + w) * wt ...).  cnt[tile][b] =
// requests of the tile in bucket b (tile-major: coalesced).
__global__ __launch_bounds__(CB_PT) void k_cb_count(CbSrc s, uint32_t bmask, uint32_t* __restrict__ cnt) {
  constexpr uint32_t W = CB_PT / 64;
  __shared__ uint32_t s_h[1u << CB_BB_MAX];
  __shared__ uint32_t s_t[W][1024];  // txn ids; ragged txns: their first requests (ids are not needed here)
  __shared__ uint16_t s_m[W][1024];  // ragged txns: element -> (txn slot, request)
  const uint32_t B = bmask + 1, lane = threadIdx.x & 63u, wv = threadIdx.x >> 6;
  for (uint32_t i = threadIdx.x; i < B; i += CB_PT) s_h[i] = 0;
  __syncthreads();
  const uint64_t tq0 = (uint64_t)blockIdx.x * CB_NSUB * W * s.wt;
  for (uint32_t sub = 0; sub < CB_NSUB; sub++) {
    const uint64_t q0 = tq0 + (uint64_t)(sub * W + wv) * s.wt;
    if (q0 >= s.n) break;  // this wave (no barrier in the loop)
    const uint32_t nq = (uint32_t)min<uint64_t>(s.wt, s.n - q0);
    uint64_t el[16];
    const uint32_t ne = cb_wave_elems<false>(s, (uint32_t)q0, nq, s_t[wv], s_t[wv], s_m[wv], el);
#pragma unroll
    for (uint32_t it = 0; it < 16; it++)
      if (it * 64 + lane < ne) atomicAdd(&s_h[(uint32_t)el[it] & bmask], 1u);
  }
  __syncthreads();
  for (uint32_t i = threadIdx.x; i < B; i += CB_PT) cnt[(uint64_t)blockIdx.x * B + i] = s_h[i];
}

// ---------------------------------------------------------------- scan
// Per bucket (a lane each, 64 per workgroup), the exclusive scan of its tile
// counts in place, the four waves taking a quarter of the tiles each; tot[b]
// = the bucket's size.
__global__ __launch_bounds__(256) void k_cb_scan(uint32_t* __restrict__ cnt, uint32_t ntile, uint32_t B,
                                                 uint32_t* __restrict__ tot) {
  __shared__ uint32_t s_p[4][64];
  const uint32_t lane = threadIdx.x & 63u, w = threadIdx.x >> 6;
  const uint32_t b = blockIdx.x * 64 + lane;
  const uint32_t per = (ntile + 3) / 4, t0 = min(ntile, w * per), t1 = min(ntile, t0 + per);
  uint32_t s = 0;
  if (b < B) {
#pragma unroll 8
    for (uint32_t t = t0; t < t1; t++) s += cnt[(uint64_t)t * B + b];
  }
  s_p[w][lane] = s;
  __syncthreads();
  uint32_t run = 0;
  for (uint32_t q = 0; q < w; q++) run += s_p[q][lane];
  if (b < B) {
#pragma unroll 8
    for (uint32_t t = t0; t < t1; t++) {
      const uint32_t c = cnt[(uint64_t)t * B + b];
      cnt[(uint64_t)t * B + b] = run;
      run += c;
    }
    if (w == 3) tot[b] = run;
  }
}

// ---------------------------------------------------------------- partition
// One workgroup per tile, its sub-tiles in order.  In a sub-tile wave w
// produces its wt txns' requests (cb_wave_elems: element 64 it + lane, so
// sequence order is (wave, round, lane)) and ranks each among the wave's
// earlier requests of its bucket with a running per-bucket count in its own
// LDS row; the waves' counts become per-(bucket, wave) bases of a
// bucket-ordered LDS staging, written out as one run per bucket at the
// bucket's cursor.  Workgroup 0 also stores the buckets' bases for the
// bucket pass.  Its barriers are LDS-only: the workgroup shares nothing
// through global memory, so a sub-tile's stores and the next sub-tile's
// loads stay in flight across them.
template <uint32_t NB>  // bucket bits at compile time (0: bb at run time)
__global__ __launch_bounds__(CB_PT) void k_cb_part(CbSrc s, uint32_t bb, const uint32_t* __restrict__ cnt,
                                                   const uint32_t* __restrict__ tot,
                                                   uint32_t* __restrict__ bbase_out,
                                                   uint64_t* __restrict__ out, uint32_t ntile) {
  constexpr uint32_t BM = 1u << CB_BB_MAX, W = CB_PT / 64;
  // XCD-contiguous tiles: workgroup b runs on XCD b % 8, which takes tiles
  // [x * per, (x + 1) * per) -- a bucket's runs from consecutive tiles then
  // meet in one L2 and leave it as whole lines
  const uint32_t tpx = (ntile + 7) / 8;
  const uint32_t tile = (blockIdx.x % 8) * tpx + blockIdx.x / 8;
  if (tile >= ntile) return;  // whole workgroup (tile 0 is workgroup 0's)
  __shared__ uint64_t s_stg[CB_SUB];  // also the waves' txn ids (and ragged first requests) while the elements load
  __shared__ uint16_t s_m[CB_PT / 64][1024];  // ragged txns: element -> (txn slot, request)
  __shared__ uint32_t s_cur[BM];      // global cursor of the bucket
  __shared__ uint32_t s_gof[BM];      // global destination minus staging index
  __shared__ uint16_t s_wc[W][BM];
  __shared__ uint32_t s_w[W];
  const uint32_t B = 1u << bb, bmask = B - 1;
  const uint32_t tid = threadIdx.x, lane = tid & 63u, wv = tid >> 6;
  const uint32_t per = (B + CB_PT - 1) / CB_PT;  // buckets per thread
  const uint32_t b0 = min(B, tid * per), b1 = min(B, b0 + per);
  {
    uint32_t ls = 0;
    for (uint32_t b = b0; b < b1; b++) ls += tot[b];
    uint32_t total;
    uint32_t run = blk_excl_add(ls, s_w, total);
    for (uint32_t b = b0; b < b1; b++) {
      s_cur[b] = run + cnt[(uint64_t)tile * B + b];
      if (tile == 0) bbase_out[b] = run;
      run += tot[b];
    }
  }
  const uint64_t lt = lane ? (~0ull >> (64 - lane)) : 0ull;
  const uint64_t tq0 = (uint64_t)tile * CB_NSUB * W * s.wt;
  for (uint32_t sub = 0; sub < CB_NSUB; sub++) {
    if (tq0 + (uint64_t)sub * W * s.wt >= s.n) break;  // whole workgroup
    const uint64_t q0 = tq0 + (uint64_t)(sub * W + wv) * s.wt;
    const uint32_t nq = q0 < s.n ? (uint32_t)min<uint64_t>(s.wt, s.n - q0) : 0u;
    for (uint32_t i = tid; i < W * BM; i += CB_PT) (&s_wc[0][0])[i] = 0;
    uint64_t e[16];
    uint32_t ne;
    if (CB_VAR(s.var, 4u)) {
      ne = nq * max(s.ulen, 1u);
#pragma unroll
      for (uint32_t it = 0; it < 16; it++)
        e[it] = ((uint64_t)((((uint32_t)q0 * 16 + it * 64 + lane) * 2654435761u) >> 8) << 32) |
                ((uint32_t)min<uint64_t>(q0, s.n - 1) << 7);  // in-range row and txn
    } else {
      ne = cb_wave_elems<true>(s, (uint32_t)q0, nq, (uint32_t*)s_stg + wv * 1024,
                               (uint32_t*)s_stg + CB_SUB + wv * 1024, s_m[wv], e);
    }
    lds_barrier();
    uint16_t loc[16];
    uint16_t* my = s_wc[wv];
#pragma unroll
    for (uint32_t it = 0; it < 16; it++) {
      const bool act = it * 64 + lane < ne;
      const uint32_t b = (uint32_t)(e[it] >> 32) & bmask;
      const uint64_t peers = (CB_VAR(s.var, 2u)) ? (act ? 1ull << lane : 0ull) : bucket_peers<NB>(b, act, bb);
      const uint32_t lr = (uint32_t)__builtin_popcountll(peers & lt);
      const uint32_t before = my[b];
      loc[it] = (uint16_t)(before + lr);
      // the bucket's first lane advances the count (same wave: in order)
      if (act && lr == 0) my[b] = (uint16_t)(before + (uint32_t)__builtin_popcountll(peers));
    }
    lds_barrier();
    uint32_t n_sub;
    {
      uint32_t ls = 0;
      for (uint32_t b = b0; b < b1; b++)
#pragma unroll
        for (uint32_t w = 0; w < W; w++) ls += s_wc[w][b];
      uint32_t run = blk_excl_add(ls, s_w, n_sub);
      for (uint32_t b = b0; b < b1; b++) {
        const uint32_t lb = run;
#pragma unroll
        for (uint32_t w = 0; w < W; w++) {
          const uint32_t c = s_wc[w][b];
          s_wc[w][b] = (uint16_t)run;
          run += c;
        }
        s_gof[b] = s_cur[b] - lb;  // mod 2^32: dst = s_gof[b] + staging index
        s_cur[b] += run - lb;
      }
    }
    lds_barrier();
#pragma unroll
    for (uint32_t it = 0; it < 16; it++) {
      if (it * 64 + lane < ne) {
        const uint32_t b = (uint32_t)(e[it] >> 32) & bmask;
        s_stg[my[b] + loc[it]] = e[it];
      }
    }
    lds_barrier();
    for (uint32_t j = tid; j < n_sub; j += CB_PT) {
      const uint64_t x = s_stg[j];
      if (!(CB_VAR(s.var, 1u))) out[s_gof[(uint32_t)(x >> 32) & bmask] + j] = x;
    }
    lds_barrier();
  }
}

// ---------------------------------------------------------------- bucket
struct CbBucket {
  const uint64_t* in;
  const uint32_t* tot;
  const uint32_t* bbase;
  uint32_t bb, lbits, tsh, ndig;
  uint64_t span;
  uint32_t* gcnt;  // [R][ndig]
  uint64_t* out;   // [R][ndig][span]
  uint32_t* err;   // CB_ERR_TAB
  uint32_t var;    // DCC_CB_VARIANT (wrong results): 8 no radix passes, 16 no pair stores,
                   // 32 no grant-group scan, 64 no staging/output
};

// Thread p0 / 16's 16 consecutive requests of a chunk of nc, clamped to the
// chunk (straight-line loads, so a prefetch stays in flight); cb_mask_chunk
// then sets the ones past nc to all-ones (they sort last).
__device__ inline void cb_load_chunk(const uint64_t* src, uint32_t nc, uint32_t p0, uint64_t (&e)[CB_IT]) {
#pragma unroll
  for (uint32_t i = 0; i < CB_IT; i++) e[i] = src[min(p0 + i, nc - 1)];
}
__device__ inline void cb_mask_chunk(uint32_t nc, uint32_t p0, uint64_t (&e)[CB_IT]) {
#pragma unroll
  for (uint32_t i = 0; i < CB_IT; i++) e[i] = p0 + i < nc ? e[i] : ~0ull;
}

// calvin_gl.h's block scan with LDS-only barriers (the outstanding
// reservations and next-chunk loads stay in flight)
__device__ inline uint32_t gl_block_excl_lds(uint32_t v, uint32_t* s_w, uint32_t& total) {
  const uint32_t lane = threadIdx.x & 63u, w = threadIdx.x >> 6, nw = blockDim.x >> 6;
  uint32_t x = v;
#pragma unroll
  for (uint32_t d = 1; d < 64; d <<= 1) {
    const uint32_t y = __shfl_up(x, d);
    if (lane >= d) x = gl_combine(y, x);
  }
  lds_barrier();  // s_w free
  if (lane == 63) s_w[w] = x;
  lds_barrier();
  uint32_t wp = GL_ID;
  total = GL_ID;
  for (uint32_t q = 0; q < nw; q++) {
    if (q < w) wp = gl_combine(wp, s_w[q]);
    total = gl_combine(total, s_w[q]);
  }
  const uint32_t ex_in = __shfl_up(x, 1);
  return gl_combine(wp, lane ? ex_in : GL_ID);
}

template <bool H>  // the hashed carry table (row bits > CB_LB_MAX)
__global__ __launch_bounds__(CB_BT) void k_cb_bucket(CbBucket a) {
  __shared__ uint32_t s_tab[1u << CB_LB_MAX];
  __shared__ uint64_t s_stg[CB_STG];
  __shared__ uint16_t s_rc[16 * CB_BT];       // radix counts [digit][thread]
  __shared__ uint32_t s_dc[CB_NDIG_MAX + 1];  // window counts, then cursors (+ a spare)
  __shared__ uint32_t s_dg[CB_NDIG_MAX];      // window region offset minus staging index
  __shared__ uint32_t s_w[CB_BT / 64];
  __shared__ uint32_t s_tl;
  __shared__ uint32_t s_fl[2][64], s_fln[2];  // rows flagged per chunk (parity)
  const uint32_t tid = threadIdx.x;
  const uint32_t size = a.tot[blockIdx.x];
  if (size == 0) return;  // whole workgroup
  const uint64_t base = a.bbase[blockIdx.x];
  const uint32_t r = blockIdx.x % CB_R;
  const uint32_t ntab = H ? CB_HSLOTS : 1u << a.lbits;
  for (uint32_t i = tid; i < ntab; i += CB_BT) s_tab[i] = H ? TAB_HEMPTY : TAB_EMPTY;
  for (uint32_t d = tid; d < a.ndig; d += CB_BT) s_dc[d] = 0;
  const uint32_t npass = (CB_VAR(a.var, 8u)) ? 0u : (a.lbits + 3) / 4;
  const uint32_t dpt = (a.ndig + CB_BT - 1) / CB_BT;  // windows per thread (<= 3)
  const uint32_t d0 = min(a.ndig, tid * dpt), d1 = min(a.ndig, d0 + dpt);
  uint32_t t_prev = NOTXN;  // the previous chunk's last txn
  const uint32_t p0 = tid * CB_IT;
  uint64_t e[CB_IT];  // this thread's 16 consecutive requests (padding: all-ones, sorts last)
  cb_load_chunk(a.in + base, min(CB_CHUNK, size), p0, e);
  lds_barrier();
  if (tid < 2) s_fln[tid] = 0;
  for (uint32_t c0 = 0; c0 < size; c0 += CB_CHUNK) {
    const uint32_t nc = min(CB_CHUNK, size - c0);
    const uint32_t pc = (c0 / CB_CHUNK) & 1u;
    if (tid == 0 && c0) s_fln[pc] = 0;  // its flags were cleared in the last chunk
    cb_mask_chunk(nc, p0, e);
#pragma unroll
    for (uint32_t i = 0; i < CB_IT; i++)
      if (p0 + i == nc - 1) s_tl = (uint32_t)e[i] >> 7;
    // (2) window counts, then one reservation per window (used after the sort)
#pragma unroll
    for (uint32_t i = 0; i < CB_IT; i++)
      if (p0 + i < nc) atomicAdd(&s_dc[((uint32_t)e[i] >> 7) >> a.tsh], 1u);
    lds_barrier();
    const uint32_t t_last = s_tl;
    // straight-line: a window past this thread's range adds 0 to its last one
    uint32_t resv[3], dcn[3];
#pragma unroll
    for (uint32_t k = 0; k < 3; k++) {
      const uint32_t d = d0 + k;
      dcn[k] = d < d1 ? s_dc[min(d, a.ndig - 1)] : 0u;
    }
#pragma unroll
    for (uint32_t k = 0; k < 3; k++)
      resv[k] = k < dpt ? atomicAdd(&a.gcnt[r * a.ndig + min(d0 + k, a.ndig - 1)], dcn[k]) : 0u;
    // the next chunk's requests, in flight behind the reservations through the
    // sort and the scan (the last chunk reloads itself: no branch)
    uint64_t en[CB_IT];
    {
      const uint32_t cn = c0 + CB_CHUNK < size ? c0 + CB_CHUNK : c0;
      cb_load_chunk(a.in + base + cn, min(CB_CHUNK, size - cn), p0, en);
    }
    // (3) stable LDS radix sort of the chunk by the row bits, 4 per pass
    for (uint32_t ps = 0; ps < npass; ps++) {
      const uint32_t sh = a.bb + 4 * ps;  // in the high word
      if (a.lbits - 4 * ps == 1) {
        // a last pass of one bit (13 row bits: C4): a stable split, zeros
        // first -- one block scan of the zero counts instead of the 16-digit
        // count table (real requests have no row bit above; padding sorts last)
        uint32_t z = 0, rk[CB_IT];
#pragma unroll
        for (uint32_t i = 0; i < CB_IT; i++) {
          const uint32_t bit = ((uint32_t)(e[i] >> 32) >> sh) & 1u;
          rk[i] = bit ? i - z : z;
          z += bit ^ 1u;
        }
        uint32_t Z;
        const uint32_t zp = blk_excl_add(z, s_w, Z);
#pragma unroll
        for (uint32_t i = 0; i < CB_IT; i++) {
          const uint32_t bit = ((uint32_t)(e[i] >> 32) >> sh) & 1u;
          s_stg[stg_ix(bit ? Z + (p0 - zp) + rk[i] : zp + rk[i])] = e[i];
        }
        lds_barrier();
#pragma unroll
        for (uint32_t i = 0; i < CB_IT; i++) e[i] = s_stg[stg_ix(p0 + i)];
        lds_barrier();
        continue;
      }
      uint64_t clo = 0, chi = 0;  // 8-bit running counts of digits 0-7 / 8-15
      uint32_t rk[CB_IT];
#pragma unroll
      for (uint32_t i = 0; i < CB_IT; i++) {
        const uint32_t d = ((uint32_t)(e[i] >> 32) >> sh) & 15u;
        const uint32_t fs = (d & 7u) * 8u;
        if (d < 8) {
          rk[i] = (uint32_t)(clo >> fs) & 255u;
          clo += 1ull << fs;
        } else {
          rk[i] = (uint32_t)(chi >> fs) & 255u;
          chi += 1ull << fs;
        }
      }
#pragma unroll
      for (uint32_t d = 0; d < 16; d++)
        s_rc[d * CB_BT + tid] = (uint16_t)(((d < 8 ? clo : chi) >> ((d & 7u) * 8u)) & 255u);
      lds_barrier();
      {  // digit-major exclusive scan of the 16 x 256 counts
        uint32_t v[16], ls = 0;
#pragma unroll
        for (uint32_t k = 0; k < 16; k++) {
          v[k] = s_rc[tid * 16 + k];
          ls += v[k];
        }
        uint32_t total;
        uint32_t run = blk_excl_add(ls, s_w, total);
#pragma unroll
        for (uint32_t k = 0; k < 16; k++) {
          s_rc[tid * 16 + k] = (uint16_t)run;
          run += v[k];
        }
      }
      lds_barrier();
#pragma unroll
      for (uint32_t i = 0; i < CB_IT; i++) {
        const uint32_t d = ((uint32_t)(e[i] >> 32) >> sh) & 15u;
        s_stg[stg_ix(s_rc[d * CB_BT + tid] + rk[i])] = e[i];
      }
      lds_barrier();
#pragma unroll
      for (uint32_t i = 0; i < CB_IT; i++) e[i] = s_stg[stg_ix(p0 + i)];
      lds_barrier();
    }
    if (npass == 0) {  // one row per bucket: position order is row order
#pragma unroll
      for (uint32_t i = 0; i < CB_IT; i++) s_stg[stg_ix(p0 + i)] = e[i];
      lds_barrier();
    }
    // (4) grant-group scan; a row's first request in the chunk continues from
    // the carry table, its last one stores the row's state back
    // Row of a request: its high word past the bucket bits (32-bit shifts).
    const uint32_t bsh = a.bb;
    const uint64_t prev_e = p0 ? s_stg[stg_ix(p0 - 1)] : ~0ull;
    const uint64_t next_e = p0 + CB_IT < nc ? s_stg[stg_ix(p0 + CB_IT)] : ~0ull;
    uint32_t dupm = 0;
    uint32_t grp[CB_IT];
    if (CB_VAR(a.var, 32u)) {
#pragma unroll
      for (uint32_t i = 0; i < CB_IT; i++) grp[i] = (uint32_t)(e[i] >> 32) >> bsh;
      goto staged;
    }
    {
      // every item's carry word read up front (one LDS round trip, not one per
      // row start inside the branches below)
      uint32_t cw[CB_IT];
      if (H) {  // first probes in one round trip, then the rare longer walks
        uint32_t hs[CB_IT];
#pragma unroll
        for (uint32_t i = 0; i < CB_IT; i++) {
          hs[i] = cb_hslot((uint32_t)(e[i] >> 32) >> bsh);
          cw[i] = s_tab[hs[i]];
        }
#pragma unroll
        for (uint32_t i = 0; i < CB_IT; i++)
          cw[i] = p0 + i < nc ? cb_hget(s_tab, (uint32_t)(e[i] >> 32) >> bsh, hs[i], cw[i]) : TAB_EMPTY;
      } else {
#pragma unroll
        for (uint32_t i = 0; i < CB_IT; i++) cw[i] = s_tab[min((uint32_t)(e[i] >> 32) >> bsh, ntab - 1)];
      }
      // The thread's 16 requests folded left to right into the gl state
      // (flag, ft, lt, cnt) in separate registers; per request the inclusive
      // local count lc[i], and bit masks: a row start at or before i (startm),
      // a non-identity request at or before i (seenm), the local last type
      // after i (ltp, 2 bits each).  A row start resets the state.
      uint32_t lc[CB_IT];
      uint32_t startm = 0, seenm = 0, ltp = 0;
      uint32_t lflag = 0, lft = CV_NONE, llt = CV_NONE, lcnt = 0;
#pragma unroll
      for (uint32_t i = 0; i < CB_IT; i++) {
        const uint64_t pe = i ? e[i - 1] : prev_e;
        const uint32_t lk = (uint32_t)(e[i] >> 32) >> bsh, plk = (uint32_t)(pe >> 32) >> bsh;
        const uint32_t v = (uint32_t)e[i], tx = v >> 7;
        const uint32_t typ = (v & 1u) ? CV_EX : CV_SH;
        if (p0 + i < nc) {
          if (p0 + i == 0 || lk != plk) {
            const uint32_t c = cw[i];
            const uint32_t cl = (c >> 1) & 3u, cc = c >> 3;
            uint32_t ft;
            if (cl == CV_NONE) {
              ft = typ;
              llt = typ;
              lcnt = 0;
            } else if ((c & 1u) && tx == t_prev) {  // same txn as the row's last request
              ft = cl;
              llt = cl;
              lcnt = cc;
              dupm |= 1u << i;
            } else {
              ft = cl;
              llt = typ;
              lcnt = cc + ((cl == CV_EX || typ == CV_EX) ? 1u : 0u);
            }
            lflag = 1;
            lft = lft == CV_NONE ? ft : lft;
          } else if (tx == (uint32_t)pe >> 7) {  // duplicate row of the same txn: identity
            dupm |= 1u << i;
          } else {
            lcnt += (llt == CV_EX || (llt == CV_SH && typ == CV_EX)) ? 1u : 0u;
            lft = lft == CV_NONE ? typ : lft;
            llt = typ;
          }
        }
        lc[i] = lcnt;
        startm |= lflag << i;
        seenm |= (lft != CV_NONE ? 1u : 0u) << i;
        ltp |= llt << (2 * i);
      }
      uint32_t total;
      const uint32_t run =  // every table read is done past this
          gl_block_excl_lds(gl_pack(lflag, lft, llt, lcnt), s_w, total);
      // a "same txn" flag lives one chunk: the rows flagged by the previous
      // chunk lose it before this chunk's row states go in
      {
        const uint32_t po = pc ^ 1u;
        if (tid < s_fln[po]) atomicAnd(&s_tab[s_fl[po][tid]], ~1u);
        lds_barrier();
      }
      // inclusive state at i = prefix (x) local state at i
      const uint32_t pcnt = run >> 5, plt = (run >> 3) & 3u;
      const uint32_t pb = (plt != CV_NONE && lft != CV_NONE && (plt == CV_EX || lft == CV_EX)) ? 1u : 0u;
#pragma unroll
      for (uint32_t i = 0; i < CB_IT; i++) {
        const uint32_t cnt = ((startm >> i) & 1u) ? lc[i] : pcnt + lc[i] + (pb & (seenm >> i));
        grp[i] = ((dupm >> i) & 1u) ? DCC_GROUP_NONE : cnt;
        if (p0 + i < nc) {
          const uint64_t ne = i + 1 < CB_IT ? e[i + 1] : next_e;
          const uint32_t lk = (uint32_t)(e[i] >> 32) >> bsh;
          if (p0 + i + 1 == nc || (uint32_t)(ne >> 32) >> bsh != lk) {
            const uint32_t tx = (uint32_t)e[i] >> 7;
            const uint32_t lt_i = (ltp >> (2 * i)) & 3u;
            const uint32_t v = (cnt << 3) | ((lt_i != CV_NONE ? lt_i : plt) << 1) | (tx == t_last ? 1u : 0u);
            uint32_t slot = lk;
            if (H) slot = cb_hput(s_tab, lk, v, a.err);
            else s_tab[lk] = v;
            // <= 64 flagged: one txn's requests
            if (tx == t_last && slot < ntab) s_fl[pc][atomicAdd(&s_fln[pc], 1u)] = slot;
          }
        }
      }
    }
  staged:
    if (CB_VAR(a.var, 64u)) {
      uint32_t x = 0;
#pragma unroll
      for (uint32_t i = 0; i < CB_IT; i++) x ^= grp[i];
      if (x == 0x9e3779b9u) a.gcnt[0] = resv[0] + resv[1] + resv[2];
      goto next_chunk;
    }
    // (5) the (request, group) pairs staged by window, appended to the regions
    {
      uint32_t ls = 0;
#pragma unroll
      for (uint32_t k = 0; k < 3; k++) ls += dcn[k];
      uint32_t tt;
      uint32_t lb = blk_excl_add(ls, s_w, tt);
#pragma unroll
      for (uint32_t k = 0; k < 3; k++) {
        const uint32_t d = d0 + k;
        if (d < d1) {
          s_dc[d] = lb;
          s_dg[d] = resv[k] - lb;
          lb += dcn[k];
        }
      }
    }
    lds_barrier();
    {  // every position drawn before the first store (padding draws from a spare counter)
      uint32_t q[CB_IT];
#pragma unroll
      for (uint32_t i = 0; i < CB_IT; i++)
        q[i] = atomicAdd(&s_dc[p0 + i < nc ? ((uint32_t)e[i] >> 7) >> a.tsh : CB_NDIG_MAX], 1u);
#pragma unroll
      for (uint32_t i = 0; i < CB_IT; i++)
        if (p0 + i < nc) s_stg[q[i]] = ((uint64_t)grp[i] << 32) | (uint32_t)e[i];
    }
    lds_barrier();
    for (uint32_t j = tid; j < nc; j += CB_BT) {
      const uint64_t x = s_stg[j];
      const uint32_t d = ((uint32_t)x >> 7) >> a.tsh;
      if (!(CB_VAR(a.var, 16u))) a.out[((uint64_t)r * a.ndig + d) * a.span + (uint32_t)(s_dg[d] + j)] = x;
    }
    lds_barrier();
  next_chunk:
    for (uint32_t d = tid; d < a.ndig; d += CB_BT) s_dc[d] = 0;
    t_prev = t_last;
#pragma unroll
    for (uint32_t i = 0; i < CB_IT; i++) e[i] = en[i];
    lds_barrier();
  }
}

// ---------------------------------------------------------------- put
// Ragged txns (ulen == 0): the window's offsets are staged in LDS (s_off,
// 2^tsh + 1 words, tsh <= CB_TSH_RAGGED) and a request's place is its txn's
// offset plus its index.
__global__ __launch_bounds__(1024) void k_cb_put(const uint64_t* __restrict__ in,
                                                 const uint32_t* __restrict__ gcnt, uint32_t ndig,
                                                 uint64_t span, uint32_t n, uint32_t ulen, uint32_t tsh,
                                                 const uint32_t* __restrict__ off, uint32_t nnz,
                                                 uint32_t* __restrict__ group, uint8_t* __restrict__ rc) {
  __shared__ uint32_t win[CB_WIN];
  __shared__ uint32_t s_wait[CB_WIN / 32];
  __shared__ uint32_t s_off[(1u << CB_TSH_RAGGED) + 1];
  const uint32_t d = blockIdx.x, tid = threadIdx.x;
  const uint32_t t_lo = d << tsh, ntx = min(n - t_lo, 1u << tsh);
  uint32_t w = ntx * ulen;
  uint64_t x_lo = (uint64_t)t_lo * ulen;
  if (!ulen) {
    for (uint32_t i = tid; i <= ntx; i += 1024) s_off[i] = min(off[t_lo + i], nnz);
    __syncthreads();
    x_lo = s_off[0];
    w = min(s_off[ntx] - s_off[0], (uint32_t)CB_WIN);  // the plan bounds it; the clamp guards the LDS
  }
  for (uint32_t i = tid; i < (ntx + 31) / 32; i += 1024) s_wait[i] = 0;
  constexpr uint32_t U = 8;
  for (uint32_t r = 0; r < CB_R; r++) {
    const uint32_t m = gcnt[r * ndig + d];
    const uint64_t* src = in + ((uint64_t)r * ndig + d) * span;
    for (uint32_t p0 = tid; p0 < m; p0 += 1024 * U) {
      uint64_t x[U];
#pragma unroll
      for (uint32_t u = 0; u < U; u++) x[u] = src[min(p0 + u * 1024, m - 1)];
#pragma unroll
      for (uint32_t u = 0; u < U; u++) {
        if (p0 + u * 1024 >= m) continue;
        const uint32_t v = (uint32_t)x[u];
        const uint32_t tl = (v >> 7) - t_lo, jj = (v >> 1) & 63u;
        const uint32_t wi = ulen ? tl * ulen + jj : s_off[tl] - (uint32_t)x_lo + jj;
        if (wi < w) win[wi] = (uint32_t)(x[u] >> 32);
      }
    }
  }
  __syncthreads();
  uint32_t* dst = group + x_lo;
  for (uint32_t i = tid; i < w; i += 1024) {
    const uint32_t g = win[i];
    dst[i] = g;
    if (ulen) {
      // one atomic per txn and wave, from the txn's first lane in the wave:
      // a wave's 64 requests belong to a few txns, whose wait bits share a
      // word (64 same-word atomics serialise: SQ_LDS_BANK_CONFLICT)
      const uint64_t fm = ballot64(g != 0 && g != DCC_GROUP_NONE);
      const uint32_t tt = i / ulen, base = i - (tid & 63u);
      const uint32_t lo = max(tt * ulen, base);
      if (i == lo) {
        const uint32_t hi = min((tt + 1) * ulen, base + 64u);
        const uint64_t rm = (hi - lo >= 64u ? ~0ull : ((1ull << (hi - lo)) - 1ull)) << (lo - base);
        if (fm & rm) atomicOr(&s_wait[tt >> 5], 1u << (tt & 31u));
      }
    }
  }
  if (!ulen) {  // a thread per txn over its requests
    for (uint32_t tt = tid; tt < ntx; tt += 1024) {
      bool wait = false;
      for (uint32_t i = s_off[tt] - (uint32_t)x_lo; i < min(s_off[tt + 1] - (uint32_t)x_lo, w); i++) {
        const uint32_t g = win[i];
        wait |= g != 0 && g != DCC_GROUP_NONE;
      }
      // a wave's 64 txns are two whole words (tt of lane 0 is a multiple of
      // 64): one store per word, no same-word atomics
      const uint64_t wm = ballot64(wait);
      const uint32_t ln = tid & 63u;
      if ((ln & 31u) == 0) s_wait[tt >> 5] = (uint32_t)(wm >> ln);
    }
  }
  __syncthreads();
  for (uint32_t tt = tid; tt < ntx; tt += 1024)
    rc[t_lo + tt] = ((s_wait[tt >> 5] >> (tt & 31u)) & 1u) ? DCC_RC_WAIT : DCC_RC_RCOK;
}

}  // namespace

bool cb_plan(uint64_t n, uint64_t nnz, uint32_t ulen, uint32_t maxlen, uint32_t kbits, CbPlan* p) {
  // uniform txns (ulen requests each), or ragged ones of at most maxlen
  const uint32_t len = ulen ? ulen : maxlen;
  if (!len || len > 64 || nnz == 0 || (ulen && nnz != n * ulen) || nnz >= 0xFFFFFFFFull) return false;
  if (kbits > CB_BB_MAX + CB_LB_HASH_MAX) return false;
  CbPlan q{};
  q.bb = std::min(CB_BB_MAX, kbits);
  q.lbits = kbits - q.bb;
  q.hashed = q.lbits > CB_LB_MAX ? 1u : 0u;
  q.tsh = 0;
  while ((2ull << q.tsh) * len <= CB_WIN && (ulen || q.tsh < CB_TSH_RAGGED)) q.tsh++;
  q.span = (1ull << q.tsh) * len;
  q.ndig = (uint32_t)((n + (1ull << q.tsh) - 1) >> q.tsh);
  if (q.ndig > CB_NDIG_MAX) return false;
  q.wt = 1024 / len;
  const uint64_t tile_txn = (uint64_t)CB_NSUB * (CB_PT / 64) * q.wt;
  q.ntile = (uint32_t)((n + tile_txn - 1) / tile_txn);
  q.R = CB_R;
  const uint64_t B = 1ull << q.bb;
  q.elem_bytes = nnz * 8;
  q.out_bytes = (uint64_t)q.R * q.ndig * q.span * 8;
  q.cnt_bytes = (uint64_t)q.ntile * B * 4;
  q.small_bytes = (2 * B + (uint64_t)q.R * q.ndig) * 4;
  *p = q;
  return true;
}

hipError_t cb_run(const CbPlan& p, const CbArgs& a, hipStream_t st, hipEvent_t ev_part,
                  hipEvent_t ev_bucket) {
  const uint32_t B = 1u << p.bb;
  uint32_t* tot = a.small;
  uint32_t* bbase = tot + B;
  uint32_t* gcnt = bbase + B;
  static const uint32_t var = [] {
    const char* e = DCC_ENV("DCC_CB_VARIANT");
    return e ? (uint32_t)atoi(e) : 0u;
  }();
  const CbSrc s{a.keys,       a.acctype, a.seq, a.off, (uint32_t)a.n, a.ulen,
                a.ulen ? ((1u << 20) + a.ulen - 1) / a.ulen : 0u, p.wt, (uint32_t)a.nnz, var, a.kp};
  hipError_t e = hipMemsetAsync(gcnt, 0, (size_t)p.R * p.ndig * 4, st);
  if (e != hipSuccess) return e;
  k_cb_count<<<p.ntile, CB_PT, 0, st>>>(s, B - 1, a.cnt);
  k_cb_scan<<<(B + 63) / 64, 256, 0, st>>>(a.cnt, p.ntile, B, tot);
  if (p.bb == CB_BB_MAX)
    k_cb_part<CB_BB_MAX><<<8 * ((p.ntile + 7) / 8), CB_PT, 0, st>>>(s, p.bb, a.cnt, tot, bbase, a.elems,
                                                                    p.ntile);
  else
    k_cb_part<0><<<8 * ((p.ntile + 7) / 8), CB_PT, 0, st>>>(s, p.bb, a.cnt, tot, bbase, a.elems, p.ntile);
  if (ev_part && (e = hipEventRecord(ev_part, st)) != hipSuccess) return e;
  const CbBucket ba{a.elems, tot, bbase, p.bb, p.lbits, p.tsh, p.ndig, p.span, gcnt, a.out, a.err, var};
  if (p.hashed)
    k_cb_bucket<true><<<B, CB_BT, 0, st>>>(ba);
  else
    k_cb_bucket<false><<<B, CB_BT, 0, st>>>(ba);
  if (ev_bucket && (e = hipEventRecord(ev_bucket, st)) != hipSuccess) return e;
  k_cb_put<<<p.ndig, 1024, 0, st>>>(a.out, gcnt, p.ndig, p.span, (uint32_t)a.n, a.ulen, p.tsh, a.off,
                                    (uint32_t)a.nnz, a.group, a.rc);
  return hipGetLastError();
}

}  // namespace dcc
