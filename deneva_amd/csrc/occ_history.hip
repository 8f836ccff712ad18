// Device-resident OCC history: append, level build, trim (occ_history.h).
//
// Reference: central_finish pushes every committed write set onto `history`
// with tn = ++tnc (concurrency_control/occ.cpp:277-286); central_validate
// scans the entries with start_tn < tn <= finish_tn against the read set
// (occ.cpp:160-180).  Here an epoch's committed writes are appended on the
// device in index (= tn) order and the per-key tn runs are rebuilt by a
// stable radix sort, so the host never copies the batch back.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>

#include "dcc_device.h"
#include "dcc_env.h"
#include "occ_history.h"
#include "occ_kernels.h"
#include "radix_sort.h"

namespace dcc {

constexpr uint32_t HB = 1024;  // txns per block of the append kernels

// committed writes of txn t (0 when it did not commit or is read-only)
__device__ inline uint32_t hist_writes_of(uint64_t t, const uint32_t* off, const uint8_t* acctype,
                                          uint64_t nnz, const uint64_t* tn, uint32_t& a0) {
  a0 = 0;
  if (!tn[t]) return 0;
  const uint64_t o0 = min((uint64_t)off[t], nnz), o1 = min((uint64_t)off[t + 1], nnz);
  if (o1 <= o0) return 0;
  a0 = (uint32_t)o0;
  uint32_t c = 0;
  for (uint64_t x = o0; x < o1 && x < o0 + MAX_TXN_LEN; x++) c += acctype[x] == DCC_WR;
  return c;
}

// exclusive scan over the block (1024 threads = 16 waves); returns the block total
__device__ inline uint32_t block_excl_scan1024(uint32_t v, uint32_t& excl) {
  __shared__ uint32_t s_w[HB / 64];
  const uint32_t lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  uint32_t x = v;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const uint32_t y = __shfl_up(x, d);
    if (lane >= (uint32_t)d) x += y;
  }
  if (lane == 63) s_w[w] = x;
  __syncthreads();
  uint32_t before = 0, total = 0;
#pragma unroll
  for (uint32_t q = 0; q < HB / 64; q++) {
    const uint32_t s = s_w[q];
    if (q < w) before += s;
    total += s;
  }
  excl = before + x - v;
  return total;
}

__global__ __launch_bounds__(HB) void k_hist_count(uint64_t n, const uint32_t* off,
                                                   const uint8_t* acctype, uint64_t nnz,
                                                   const uint64_t* tn, uint32_t* bsum) {
  const uint64_t t = (uint64_t)blockIdx.x * HB + threadIdx.x;
  uint32_t a0;
  const uint32_t c = t < n ? hist_writes_of(t, off, acctype, nnz, tn, a0) : 0u;
  uint32_t ex;
  const uint32_t tot = block_excl_scan1024(c, ex);
  if (threadIdx.x == 0) bsum[blockIdx.x] = tot;
}

__global__ __launch_bounds__(HB) void k_hist_emit(uint64_t n, const uint32_t* off,
                                                  const uint64_t* keys, const uint8_t* acctype,
                                                  uint64_t nnz, const uint64_t* tn,
                                                  const uint32_t* bsum, uint64_t* out_k,
                                                  uint64_t* out_t, unsigned long long* kmax) {
  __shared__ unsigned long long s_mx;
  const uint64_t t = (uint64_t)blockIdx.x * HB + threadIdx.x;
  uint32_t a0 = 0;
  const uint32_t c = t < n ? hist_writes_of(t, off, acctype, nnz, tn, a0) : 0u;
  uint32_t ex;
  (void)block_excl_scan1024(c, ex);
  if (threadIdx.x == 0) s_mx = 0;
  __syncthreads();
  uint64_t mx = 0;
  if (c) {
    uint64_t p = (uint64_t)bsum[blockIdx.x] + ex;
    const uint64_t my_tn = tn[t];
    for (uint64_t x = a0; p < (uint64_t)bsum[blockIdx.x] + ex + c; x++) {
      if (acctype[x] != DCC_WR) continue;
      const uint64_t k = keys[x];
      out_k[p] = k;
      out_t[p] = my_tn;
      mx = max(mx, k);
      p++;
    }
  }
  for (int d = 32; d > 0; d >>= 1) mx = max(mx, (uint64_t)__shfl_xor(mx, d));
  if ((threadIdx.x & 63) == 0 && mx) atomicMax(&s_mx, (unsigned long long)mx);
  __syncthreads();
  if (threadIdx.x == 0 && s_mx) atomicMax(kmax, s_mx);  // one per workgroup
}

// ---------------------------------------------------------------------------
// central_finish in one launch (OccFinArgs, occ_kernels.h): a workgroup per
// 2,048 txns counts its committed writers (cflag) and, when appending, their
// writes and largest key; a single-pass scan with decoupled look-back gives
// its prefix (tnc and the delta's append position from the epoch parameters,
// dyn->tnc / dyn->hist_m); each committed writer takes its tn and emits its
// write set there; the workgroup's threads then push its pairs onto the
// delta's chains (a thread per pair); the last workgroup to finish copies the
// totals to pinned memory.  Only committed writers (a few per thousand under
// contention) read their access lists.
//
// Look-back words, as MaaT's round scan (maat.hip): payload and status are
// written with device-scope atomics, the status after `s_waitcnt vmcnt(0)`
// (the payload is at the coherence point first), and read in the other
// order; the status carries the epoch's tag (dyn->fin_tag), so nothing is
// reset between epochs.
struct __attribute__((aligned(64))) FinLb {
  uint64_t agg, inc;  // commits | writes << 32: the workgroup's, and through it
  uint32_t status;    // tag << 2 | 1 aggregate, | 2 inclusive
  uint32_t pad[11];
};
static_assert(sizeof(FinLb) == 64, "one line per workgroup");
struct FinTail {
  unsigned long long kmax;  // largest key appended (reset by the last workgroup)
  uint32_t done;            // finished workgroups (reset by the last one)
  uint32_t ticket;          // workgroups started (reset by the last one)
  uint32_t und;             // chained: undecided txns seen (reset by the last one)
  uint32_t capx;            // chained: a workgroup's pairs did not fit (reset by the last one)
  uint32_t pad[10];
};
static_assert(sizeof(FinTail) == 64, "one line");
template <typename T>
__device__ inline void fin_st(T* p, T v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
template <typename T>
__device__ inline T fin_ld(T* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ inline void fin_publish(FinLb* e, uint64_t v, bool incl, uint32_t tag) {
  fin_st(incl ? &e->inc : &e->agg, v);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  fin_st(&e->status, (tag << 2) | (incl ? 2u : 1u));
}

// A committed writer's accesses [o0, o1), FIN_U at a time: every type and
// key of a step loaded before any is used (one memory round trip per step
// instead of one per access).
constexpr uint32_t FIN_U = 8;
// k_fin: 2,048 txns per workgroup, as 1,024 threads x 2 consecutive txns for
// an epoch finished on its own (its pushes and write-set emission spread over
// more threads: the SHIM / HIST epochs) and as 512 x 4 for a chained finish
// beside other lanes' kernels (half the wave slots while its look-back waits;
// profiles/r06/fin_t/)
constexpr uint32_t FIN_TXN_WG = 2048;
__device__ inline void fin_step(const OccFinArgs& a, uint64_t x, uint64_t o1, uint8_t (&ty)[FIN_U],
                                uint64_t (&k)[FIN_U]) {
#pragma unroll
  for (uint32_t u = 0; u < FIN_U; u++) {
    const bool in = x + u < o1;
    ty[u] = in ? a.acctype[x + u] : (uint8_t)0;
    k[u] = in ? a.keys[x + u] : 0ull;
  }
}
__device__ inline uint32_t fin_writes(uint64_t t, const OccFinArgs& a, uint64_t& o0, uint64_t& o1,
                                      uint64_t& kmx) {
  o0 = min((uint64_t)a.off[t], a.nnz);
  o1 = min((uint64_t)a.off[t + 1], a.nnz);
  if (o1 < o0) o1 = o0;
  o1 = min(o1, o0 + MAX_TXN_LEN);
  uint32_t c = 0;
  for (uint64_t x = o0; x < o1; x += FIN_U) {
    uint8_t ty[FIN_U];
    uint64_t k[FIN_U];
    fin_step(a, x, o1, ty, k);
#pragma unroll
    for (uint32_t u = 0; u < FIN_U; u++)
      if (ty[u] == DCC_WR) {
        c++;
        kmx = max(kmx, k[u]);
      }
  }
  return c;
}

// block-wide exclusive scans of two counters (FB threads); returns both totals
template <uint32_t FB>
__device__ inline void block_excl_scan2(uint32_t v0, uint32_t v1, uint32_t& e0, uint32_t& e1,
                                        uint32_t& t0, uint32_t& t1) {
  __shared__ uint32_t s_w[2][FB / 64];
  const uint32_t lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  uint32_t x0 = v0, x1 = v1;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const uint32_t y0 = __shfl_up(x0, d), y1 = __shfl_up(x1, d);
    if (lane >= (uint32_t)d) {
      x0 += y0;
      x1 += y1;
    }
  }
  if (lane == 63) {
    s_w[0][w] = x0;
    s_w[1][w] = x1;
  }
  __syncthreads();
  uint32_t b0 = 0, b1 = 0;
  t0 = t1 = 0;
#pragma unroll
  for (uint32_t q = 0; q < FB / 64; q++) {
    if (q < w) {
      b0 += s_w[0][q];
      b1 += s_w[1][q];
    }
    t0 += s_w[0][q];
    t1 += s_w[1][q];
  }
  e0 = b0 + x0 - v0;
  e1 = b1 + x1 - v1;
}

template <uint32_t FB, uint32_t FIN_T>
__global__ __launch_bounds__(FB, 8) void k_fin(OccFinArgs a) {
  __shared__ unsigned long long s_mx;
  __shared__ uint64_t s_pre;
  __shared__ uint32_t s_last, s_id;
  const OccDyn* dy = a.dyn;
  const uint32_t tag = a.tag ? a.tag : dy->fin_tag;
  const bool chained = a.ctl != nullptr;
  if (chained && dy->pad != 1u) {
    // an epoch before this one is not finished yet (its host finish is still
    // to come): the host finishes this one too, nothing is written
    if (blockIdx.x == 0 && threadIdx.x == 0)
      for (int q = 0; q < 5; q++) a.totals[q] = 0;
    return;
  }
  // the tail first: its place must not depend on the epoch's grid size
  FinTail* tail = (FinTail*)a.part;
  FinLb* lb = (FinLb*)(tail + 1);
  // The workgroup's place in the scan is a ticket, not blockIdx: workgroups
  // are dealt to the XCDs round-robin and each XCD dispatches its share as
  // its own CUs free up, so workgroup b can run while b - 4 still waits for
  // a slot -- held, when other kernels share the GPU, by workgroups that
  // spin themselves (two key shards of one context on one GPU, or rank
  // processes sharing it: the round-5/6 "numbered 339 txns" failures).  A
  // ticket holder's predecessors all hold tickets, so all of them run.
  if (threadIdx.x == 0) s_id = atomicAdd(&tail->ticket, 1u);
  __syncthreads();
  const uint32_t bid = s_id;
  // FIN_T consecutive txns per thread (one generation of workgroups fits the
  // chip: a workgroup's chain of round trips is paid once, not twice)
  const uint64_t t_0 = ((uint64_t)bid * FB + threadIdx.x) * FIN_T;
  uint64_t* app_k = dy->app_k;
  uint64_t* app_t = dy->app_t;
  uint32_t c[FIN_T], w[FIN_T];
  uint64_t o0[FIN_T], o1[FIN_T], kmx = 0;
#pragma unroll
  for (uint32_t i = 0; i < FIN_T; i++) c[i] = (t_0 + i < a.n && a.cflag[t_0 + i]) ? 1u : 0u;
#pragma unroll
  for (uint32_t i = 0; i < FIN_T; i++) {
    o0[i] = o1[i] = 0;
    w[i] = (c[i] && app_k) ? fin_writes(t_0 + i, a, o0[i], o1[i], kmx) : 0u;
  }
  uint32_t cs = 0, ws = 0, und = 0;
#pragma unroll
  for (uint32_t i = 0; i < FIN_T; i++) {
    cs += c[i];
    ws += w[i];
    if (chained && t_0 + i < a.n) und += a.state[t_0 + i] == ST_UNDECIDED;
  }
  if (chained) {  // the epoch's undecided txns, one atomic per wave (none usually)
    for (int d = 32; d > 0; d >>= 1) und += __shfl_xor(und, d);
    if ((threadIdx.x & 63) == 0 && und) atomicAdd(&tail->und, und);
  }
  if (threadIdx.x == 0) s_mx = 0;
  uint32_t e0, e1, t0, t1;
  block_excl_scan2<FB>(cs, ws, e0, e1, t0, t1);  // its barrier orders s_mx's reset
  for (int d = 32; d > 0; d >>= 1) kmx = max(kmx, (uint64_t)__shfl_xor(kmx, d));
  if ((threadIdx.x & 63) == 0 && kmx) atomicMax(&s_mx, (unsigned long long)kmx);
  __syncthreads();
  const uint32_t lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  if (wv == 0) {
    const uint64_t tot = (uint64_t)t0 | ((uint64_t)t1 << 32);
    uint64_t P = 0;
    // the block's largest key before its publish (whose waitcnt orders it)
    if (lane == 0 && s_mx) atomicMax(&tail->kmax, s_mx);
    if (bid == 0) {
      if (lane == 0) fin_publish(&lb[0], tot, true, tag);
    } else {
      if (lane == 0) fin_publish(&lb[bid], tot, false, tag);
      bool timed_out = false;
      for (int64_t hi = (a.var & 2u) ? -1 : (int64_t)bid - 1; hi >= 0; hi -= 64) {
        const int64_t j = hi - (int64_t)lane;
        uint32_t stw = 0;
        if (j >= 0) {
          const uint64_t t0 = spin_clock();
          while (((stw = fin_ld(&lb[j].status)) >> 2) != tag) {
            __builtin_amdgcn_s_sleep(1);
            if (spin_clock() - t0 > SPIN_TICKS) {  // dispatch is in index order: a hang, not a wait
              timed_out = true;
              break;
            }
          }
        }
        if (ballot64(timed_out)) {
          P = ~0ull;  // the host sees the numbering fail (totals)
          break;
        }
        const bool inc = j >= 0 && (stw & 3u) == 2u;
        const uint64_t im = ballot64(inc);
        const uint32_t stop = im ? (uint32_t)__builtin_ctzll(im) : 63u;
        uint64_t v = (j >= 0 && lane <= stop) ? fin_ld(inc ? &lb[j].inc : &lb[j].agg) : 0ull;
        for (int d = 32; d > 0; d >>= 1) v += __shfl_xor(v, d);
        P += v;
        if (im) break;
      }
      if (lane == 0) fin_publish(&lb[bid], P == ~0ull ? ~0ull : P + tot, true, tag);
    }
    if (lane == 0) s_pre = P;
  }
  __syncthreads();
  const uint64_t P = s_pre;
  const uint64_t wbase = dy->hist_m + (P >> 32);
  // chained: the host reserved room for the epochs in flight from a bound;
  // pairs past it are not written and the host finishes the epoch itself
  const bool room = !chained || wbase + t1 <= a.cap;
  if (!room && threadIdx.x == 0) atomicOr(&tail->capx, 1u);
  if (P != ~0ull) {
    uint32_t ec = e0, ew = e1;
#pragma unroll
    for (uint32_t i = 0; i < FIN_T; i++) {
      const uint64_t t = t_0 + i;
      if (t >= a.n) break;
      const uint64_t my_tn = c[i] ? dy->tnc + (uint32_t)P + ec + 1 : 0;
      if (!(a.var & 8u)) a.tn[t] = my_tn;
      if (w[i] && room && !(a.var & 4u)) {
        uint64_t p = wbase + ew;
        for (uint64_t x = o0[i]; x < o1[i]; x += FIN_U) {
          uint8_t ty[FIN_U];
          uint64_t k[FIN_U];
          fin_step(a, x, o1[i], ty, k);
#pragma unroll
          for (uint32_t u = 0; u < FIN_U; u++)
            if (ty[u] == DCC_WR) {
              app_k[p] = k[u];
              app_t[p] = my_tn;
              p++;
            }
        }
      }
      ec += c[i];
      ew += w[i];
    }
  }
  // the block's pairs onto the delta's chains, a thread per pair
  const HistInsert ins = dy->ins;
  if (ins.hash && t1 && P != ~0ull && room && !(a.var & 1u)) {
    __syncthreads();  // the pairs written above
    for (uint32_t i = threadIdx.x; i < t1; i += FB) hist_insert(ins, wbase + i, app_k[wbase + i], app_t[wbase + i]);
  }
  // the last workgroup to finish: totals to pinned memory (every value it
  // reads was written with device-scope atomics, acknowledged before the
  // writer's arrival)
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) s_last = atomicAdd(&tail->done, 1u) == gridDim.x - 1;
  __syncthreads();
  if (s_last && threadIdx.x == 0) {
    const uint64_t g = fin_ld(&lb[gridDim.x - 1].inc);
    a.totals[0] = g == ~0ull ? ~0ull : (uint32_t)g;
    a.totals[1] = g >> 32;
    a.totals[2] = atomicExch(&tail->kmax, 0ull);
    a.totals[3] = ins.hash ? atomicAdd(ins.over, 0u) : 0u;
    if (chained) {
      // the epoch is final and numbered from the snapshot: the next one in
      // submit order may go on from here
      const bool ok = g != ~0ull && fin_ld(&tail->und) == 0 && fin_ld(&tail->capx) == 0 &&
                      (fin_ld(a.err) & ERR_NOT_FINAL) == 0 && (!a.wfull || fin_ld(a.wfull) == 0);
      if (ok) {
        fin_st(&a.ctl->tnc, dy->tnc + (uint32_t)g);
        fin_st(&a.ctl->hist_m, dy->hist_m + (g >> 32));
        __hip_atomic_store(&a.ctl->seq, a.seq + 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
      }
      a.totals[4] = ok ? 1u : 0u;
      fin_st(&tail->und, 0u);
      fin_st(&tail->capx, 0u);
    }
    fin_st(&tail->ticket, 0u);  // every workgroup took its ticket before it arrived
    fin_st(&tail->done, 0u);
  }
}

// A chained finish's parameters (OccFinArgs::ctl): the epoch's OccDyn words
// from pinned host memory, then -- once every thread's copy is in -- the
// snapshot of the device tnc / append position when *ctl is at `seq`.
__global__ __launch_bounds__(256) void k_fin_prep(const uint32_t* src, OccDyn* dyn, const FinCtl* ctl,
                                                   uint64_t seq) {
  uint32_t* d = (uint32_t*)dyn;
  for (uint32_t i = threadIdx.x; i < sizeof(OccDyn) / 4; i += 256) d[i] = src[i];
  __syncthreads();
  if (threadIdx.x == 0) {
    const uint64_t s = __hip_atomic_load(&ctl->seq, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT);
    const bool at = s == seq;
    if (at) {
      dyn->tnc = fin_ld(&ctl->tnc);
      dyn->hist_m = fin_ld(&ctl->hist_m);
    }
    dyn->pad = at ? 1u : 0u;
  }
}
__global__ void k_fin_ctl_set(FinCtl* ctl, uint64_t tnc, uint64_t hist_m, uint64_t seq) {
  fin_st(&ctl->tnc, tnc);
  fin_st(&ctl->hist_m, hist_m);
  __hip_atomic_store(&ctl->seq, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
}

void launch_fin(const OccFinArgs& a0, hipStream_t st) {
  OccFinArgs a = a0;
  // timing variants, wrong results by design: 1 no chain pushes, 2 no
  // look-back wait, 4 no write-set emission, 8 no tn stores
  if (const char* e = DCC_ENV("DCC_FIN_VAR")) a.var = (uint32_t)atoi(e);
  const uint64_t nb = (a.n + FIN_TXN_WG - 1) / FIN_TXN_WG;
  if (a.ctl)
    k_fin<512, 4><<<(unsigned)(nb ? nb : 1), 512, 0, st>>>(a);
  else
    k_fin<1024, 2><<<(unsigned)(nb ? nb : 1), 1024, 0, st>>>(a);
}

void launch_fin_prep(const uint32_t* src, OccDyn* dyn, const FinCtl* ctl, uint64_t seq, hipStream_t st) {
  k_fin_prep<<<1, 256, 0, st>>>(src, dyn, ctl, seq);
}
void launch_fin_ctl_set(FinCtl* ctl, uint64_t tnc, uint64_t hist_m, uint64_t seq, hipStream_t st) {
  k_fin_ctl_set<<<1, 1, 0, st>>>(ctl, tnc, hist_m, seq);
}

uint64_t fin_part_bytes(uint64_t n) { return (((n + FIN_TXN_WG - 1) / FIN_TXN_WG) + 2) * sizeof(FinLb); }

// A host copy of k_fin's look-back words (fin_part_bytes(n) bytes) after a
// launch with `tag`, summarised for the error message of a totals mismatch:
// workgroups whose status carries another tag or no inclusive value, and the
// first one whose inclusive prefix is not its predecessor's plus its own
// aggregate (a foreign or stale prefix taken by the look-back).
std::string fin_diag(const void* words, uint64_t n, uint32_t tag) {
  const FinLb* lb = (const FinLb*)((const FinTail*)words + 1);
  const uint64_t nb = std::max<uint64_t>(1, (n + FIN_TXN_WG - 1) / FIN_TXN_WG);
  uint64_t stale = 0, first_stale = ~0ull, bad = ~0ull;
  uint32_t stale_tag = 0;
  uint64_t prev = 0;
  for (uint64_t b = 0; b < nb; b++) {
    const FinLb& e = lb[b];
    if ((e.status >> 2) != tag || (e.status & 3u) != 2u) {
      if (!stale++) {
        first_stale = b;
        stale_tag = e.status;
      }
      continue;
    }
    const uint64_t own = b == 0 ? e.inc : e.agg;
    if (bad == ~0ull && b > 0 && e.inc != prev + own) bad = b;
    prev = e.inc;
  }
  char buf[512];
  int k = snprintf(buf, sizeof buf, "look-back of %llu workgroups, tag %u: %llu not inclusive under the tag",
                   (unsigned long long)nb, tag, (unsigned long long)stale);
  if (stale)
    k += snprintf(buf + k, sizeof buf - k, " (first: workgroup %llu, status tag %u flag %u)",
                  (unsigned long long)first_stale, stale_tag >> 2, stale_tag & 3u);
  if (bad != ~0ull) {
    const FinLb& e = lb[bad];
    snprintf(buf + k, sizeof buf - k,
             "; workgroup %llu's prefix is not its predecessor's plus its own: inclusive %llu commits, "
             "aggregate %llu, predecessor inclusive %llu",
             (unsigned long long)bad, (unsigned long long)(uint32_t)e.inc, (unsigned long long)(uint32_t)e.agg,
             (unsigned long long)(uint32_t)lb[bad - 1].inc);
  } else {
    snprintf(buf + k, sizeof buf - k, "; inclusive prefixes consistent");
  }
  return buf;
}

void launch_hist_count(uint64_t n, const uint32_t* off, const uint8_t* acctype, uint64_t nnz,
                       const uint64_t* tn, uint32_t* bsum, hipStream_t st) {
  const unsigned g = (unsigned)((n + HB - 1) / HB);
  k_hist_count<<<g ? g : 1, HB, 0, st>>>(n, off, acctype, nnz, tn, bsum);
}
void launch_hist_emit(uint64_t n, const uint32_t* off, const uint64_t* keys, const uint8_t* acctype,
                      uint64_t nnz, const uint64_t* tn, const uint32_t* bsum, uint64_t* out_k,
                      uint64_t* out_t, unsigned long long* kmax, hipStream_t st) {
  const unsigned g = (unsigned)((n + HB - 1) / HB);
  k_hist_emit<<<g ? g : 1, HB, 0, st>>>(n, off, keys, acctype, nnz, tn, bsum, out_k, out_t, kmax);
}

// ---------------------------------------------------------------- level build
__global__ __launch_bounds__(256) void k_hist_init(const uint64_t* src, uint64_t m, uint64_t* k,
                                                   uint32_t* v) {
  for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < m; i += (uint64_t)gridDim.x * 256) {
    k[i] = src[i];
    v[i] = (uint32_t)i;
  }
}
// second key of a two-pass sort: k[i] = fk[perm[i]], v[i] = perm[i]
__global__ __launch_bounds__(256) void k_hist_regather(const uint64_t* fk, const uint32_t* perm,
                                                       uint64_t m, uint64_t* k, uint32_t* v) {
  for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < m; i += (uint64_t)gridDim.x * 256) {
    const uint32_t p = perm[i];
    k[i] = fk[p];
    v[i] = p;
  }
}
__global__ __launch_bounds__(256) void k_hist_gather(const uint64_t* sk, const uint32_t* perm,
                                                     const uint64_t* ft, uint64_t m, uint64_t* skey,
                                                     uint64_t* stn) {
  for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < m; i += (uint64_t)gridDim.x * 256) {
    skey[i] = sk[i];
    stn[i] = ft[perm[i]];
  }
}
// the first pair of each key's run enters the table: (key, first)
__global__ __launch_bounds__(256) void k_hist_heads(const uint64_t* skey, uint64_t m,
                                                    uint64_t* hash, uint32_t hbits, uint32_t* over) {
  const uint64_t mask = (1ull << hbits) - 1;
  uint64_t* side = hash + (2ull << hbits);
  for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < m; i += (uint64_t)gridDim.x * 256) {
    const uint64_t key = skey[i];
    if (i > 0 && skey[i - 1] == key) continue;
    uint64_t s = hist_hash_slot(key, hbits);
    for (uint32_t w = 0;; w++) {
      if (w == HIST_WALK) atomicOr(over, 1u);  // probes stop at HIST_WALK: the host rebuilds
      const unsigned long long prev = atomicCAS((unsigned long long*)&hash[2 * s],
                                                (unsigned long long)DCC_KEY_RESERVED,
                                                (unsigned long long)key);
      if (prev == DCC_KEY_RESERVED) break;
      s = (s + 1) & mask;  // keys are unique here: a taken slot is another key's
    }
    side[2 * s] = i;
  }
}
// the last pair of each run completes its slot: the run (first | count << 32)
// and ~(its largest tn)
__global__ __launch_bounds__(256) void k_hist_tails(const uint64_t* skey, const uint64_t* stn, uint64_t m,
                                                    uint64_t* hash, uint32_t hbits) {
  const uint64_t mask = (1ull << hbits) - 1;
  uint64_t* side = hash + (2ull << hbits);
  for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < m; i += (uint64_t)gridDim.x * 256) {
    const uint64_t key = skey[i];
    if (i + 1 < m && skey[i + 1] == key) continue;
    uint64_t s = hist_hash_slot(key, hbits);
    while (hash[2 * s] != key) s = (s + 1) & mask;
    const uint64_t first = side[2 * s];
    side[2 * s] = first | ((i + 1 - first) << 32);
    hash[2 * s + 1] = ~stn[i];
  }
}

static unsigned hgrid(uint64_t m) {
  uint64_t g = (m + 255) / 256;
  return (unsigned)(g == 0 ? 1 : g > 4096 ? 4096 : g);
}

int hist_build_level(const HistBuild& b, hipStream_t st) {
  if (b.m == 0) return 0;
  uint64_t* K[2] = {b.K[0], b.K[1]};
  uint32_t* V[2] = {b.V[0], b.V[1]};
  int r;
  if (b.mono) {
    // append order is tn order within every key: one stable sort by key
    k_hist_init<<<hgrid(b.m), 256, 0, st>>>(b.fk, b.m, K[0], V[0]);
    r = radix_sort_u64(K, V, b.m, b.kbits, b.scratch, st);
  } else {
    // LSD over (key, tn): by tn, then stably by key
    k_hist_init<<<hgrid(b.m), 256, 0, st>>>(b.ft, b.m, K[0], V[0]);
    const int r1 = radix_sort_u64(K, V, b.m, b.tbits, b.scratch, st);
    k_hist_regather<<<hgrid(b.m), 256, 0, st>>>(b.fk, V[r1], b.m, K[r1 ^ 1], V[r1 ^ 1]);
    uint64_t* K2[2] = {K[r1 ^ 1], K[r1]};
    uint32_t* V2[2] = {V[r1 ^ 1], V[r1]};
    const int r2 = radix_sort_u64(K2, V2, b.m, b.kbits, b.scratch, st);
    K[0] = K2[r2];
    V[0] = V2[r2];
    r = 0;
  }
  k_hist_gather<<<hgrid(b.m), 256, 0, st>>>(K[r], V[r], b.ft, b.m, b.skey, b.stn);
  if (hipMemsetAsync(b.hash, 0xFF, (32ull << b.hbits), st) != hipSuccess) return -1;
  k_hist_heads<<<hgrid(b.m), 256, 0, st>>>(b.skey, b.m, b.hash, b.hbits, b.over);
  k_hist_tails<<<hgrid(b.m), 256, 0, st>>>(b.skey, b.stn, b.m, b.hash, b.hbits);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

// ---------------------------------------------------------------- key bitmap
__global__ __launch_bounds__(256) void k_hist_bm(const uint64_t* keys, uint64_t m, uint32_t* bm) {
  for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < m; i += (uint64_t)gridDim.x * 256) {
    const uint32_t b = hist_bm_bit(keys[i]);
    atomicOr(&bm[b >> 5], 1u << (b & 31u));
  }
}
__global__ __launch_bounds__(256) void k_hist_bm_or(const uint32_t* a, const uint32_t* b, uint32_t* out) {
  for (uint32_t i = blockIdx.x * 256 + threadIdx.x; i < (1u << HIST_BM_LOG) / 32; i += gridDim.x * 256)
    out[i] = (a ? a[i] : 0u) | (b ? b[i] : 0u);
}
void launch_hist_bm(const uint64_t* keys, uint64_t m, uint32_t* bm, hipStream_t st) {
  (void)hipMemsetAsync(bm, 0, (1u << HIST_BM_LOG) / 8, st);
  if (m) k_hist_bm<<<hgrid(m), 256, 0, st>>>(keys, m, bm);
}
void launch_hist_bm_or(const uint32_t* a, const uint32_t* b, uint32_t* out, hipStream_t st) {
  k_hist_bm_or<<<16, 256, 0, st>>>(a, b, out);
}

// ---------------------------------------------------------------- trim
__global__ __launch_bounds__(256) void k_hist_trim(const uint64_t* ak, const uint64_t* at,
                                                   uint64_t na, const uint64_t* bk,
                                                   const uint64_t* bt, uint64_t nb, uint64_t floor,
                                                   uint64_t* ok, uint64_t* ot,
                                                   unsigned long long* cnt) {
  for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < na + nb;
       i += (uint64_t)gridDim.x * 256) {
    const uint64_t k = i < na ? ak[i] : bk[i - na];
    const uint64_t t = i < na ? at[i] : bt[i - na];
    if (t <= floor) continue;
    const unsigned long long p = atomicAdd(cnt, 1ull);
    ok[p] = k;
    ot[p] = t;
  }
}
void launch_hist_trim(const uint64_t* ak, const uint64_t* at, uint64_t na, const uint64_t* bk,
                      const uint64_t* bt, uint64_t nb, uint64_t floor, uint64_t* ok, uint64_t* ot,
                      unsigned long long* cnt, hipStream_t st) {
  k_hist_trim<<<hgrid(na + nb), 256, 0, st>>>(ak, at, na, bk, bt, nb, floor, ok, ot, cnt);
}

}  // namespace dcc
