// Captured-snapshot OCC validation (C ABI
// dcc_occ_validate_snapshot in include/dcc.h).
//
// A live concurrent run decides each txn inside central_validate
// (concurrency_control/occ.cpp:116-239) against what its critical section saw
// (occ.cpp:137-158): the history head and the active list.  With those two
// captured, every txn's decision is independent of every other's, so the
// whole capture is validated in one data-parallel pass — no fixed point:
//
//   abort(i) <=> [finish_tn > start_tn and some visible history entry with
//                 start_tn < tn <= finish_tn wrote a key i READ]   (occ.cpp:167-180)
//             or [some captured active write set meets i's keys]   (occ.cpp:185-199)
//
// Grid-stride over steps of four txns; per-wave statistics are plain stores
// folded by k_snap_sum (no same-address atomics).  When all four txns have
// <= 16 accesses a 16-lane group decides each (snap_grouped); otherwise the
// wave decides them one at a time, lane l holding access l
// (MAX_ROW_PER_TXN = 64 = one wavefront, snap_full).  The history window is
// a lookup in the context's history CSR, its rows found through an
// open-addressing key table.  Captured active txns: the lanes load their
// accesses and compare the writes against i's keys, broadcast one at a time
// (v_readlane on the whole-wave path, an LDS row per wave on the grouped one).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstring>
#include <vector>

#include "dcc.h"
#include "dcc_ctx.h"
#include "dcc_device.h"
#include "occ_kernels.h"

using namespace dcc;

namespace {

constexpr int SNAP_WAVES = 4;           // waves per 256-thread workgroup
constexpr int SNAP_EPS = 2;             // captured entries per step (4 measured no faster)
constexpr uint32_t SNAP_ERR_LEN = 1;    // a txn longer than MAX_ROW_PER_TXN
constexpr uint32_t SNAP_ERR_IDX = 2;    // an active index >= n_txn
constexpr uint32_t SNAP_ERR_AOFF = 4;   // active_off decreasing

struct SnapArgs {
  uint64_t n;
  const uint32_t* off;
  const uint64_t* keys;
  const uint8_t* acctype;
  const uint64_t* start_tn;  // NULL: history window closed (TS_CLOCK)
  const uint64_t* finish_tn;
  const uint64_t* hist_top;  // NULL: whole history visible
  const uint32_t* aoff;
  const uint32_t* aidx;
  HistView hist;  // device history levels (occ_history.h); both off: no window
  uint8_t* out_rc;
  unsigned long long* part;  // [waves][SNAP_NCNT] per-wave partials (plain stores, no atomics)
};
constexpr int SNAP_NCNT = 5;  // error bits, commits, read-only, writes, bytes

// one workgroup folds the per-wave partials into cnt[SNAP_NCNT]
constexpr int SUM_THREADS = 1024;
__global__ __launch_bounds__(SUM_THREADS) void k_snap_sum(const unsigned long long* part,
                                                          uint32_t waves, unsigned long long* cnt) {
  __shared__ unsigned long long sh[SNAP_NCNT][SUM_THREADS];
  unsigned long long v[SNAP_NCNT] = {0, 0, 0, 0, 0};
  for (uint32_t w = threadIdx.x; w < waves; w += SUM_THREADS) {
    v[0] |= part[(uint64_t)w * SNAP_NCNT];
    for (int c = 1; c < SNAP_NCNT; c++) v[c] += part[(uint64_t)w * SNAP_NCNT + c];
  }
  for (int c = 0; c < SNAP_NCNT; c++) sh[c][threadIdx.x] = v[c];
  __syncthreads();
  for (int s = SUM_THREADS / 2; s >= 1; s >>= 1) {
    if (threadIdx.x < (unsigned)s) {
      sh[0][threadIdx.x] |= sh[0][threadIdx.x + s];
      for (int c = 1; c < SNAP_NCNT; c++) sh[c][threadIdx.x] += sh[c][threadIdx.x + s];
    }
    __syncthreads();
  }
  if (threadIdx.x < SNAP_NCNT) cnt[threadIdx.x] = sh[threadIdx.x][0];
}

__device__ inline uint64_t readlane64(uint64_t v, uint32_t lane) {
  const uint32_t lo = __builtin_amdgcn_readlane((uint32_t)v, lane);
  const uint32_t hi = __builtin_amdgcn_readlane((uint32_t)(v >> 32), lane);
  return ((uint64_t)hi << 32) | lo;
}

struct SnapCnt {  // per-lane partials, reduced over the wave at the end
  uint32_t err = 0, n_commit = 0, n_ro = 0, n_w = 0;
  uint64_t bytes = 0;
};

// Whole-wave path: txn t, lane l holds access l (any length <= 64).
__device__ void snap_full(const SnapArgs& a, uint64_t t, uint32_t lane, SnapCnt& c) {
  const uint32_t o0 = a.off[t], o1 = a.off[t + 1];
  uint32_t len = o1 - o0;
  if (o1 < o0 || len > MAX_TXN_LEN) {
    c.err |= SNAP_ERR_LEN;
    len = 0;
  }
  const bool have = lane < len;
  const uint64_t k = have ? a.keys[o0 + lane] : 0;
  const bool wr = have && a.acctype[o0 + lane] == DCC_WR;
  const uint64_t wmask = ballot64(wr);
  if (lane == 0) c.bytes += 4 + 9ull * len;
  bool hit = false;
  // history window, read set only (occ.cpp:167-180)
  if (a.start_tn) {
    const uint64_t s = a.start_tn[t], f = a.finish_tn[t];
    uint64_t hi = f;
    if (a.hist_top) hi = min(hi, a.hist_top[t]);
    if (lane == 0) c.bytes += a.hist_top ? 24 : 16;
    if (f > s && hi > s && have && !wr) hit = hist_hit(a.hist, k, s, hi);
  }
  bool conflict = ballot64(hit) != 0;
  // captured active list: W_j vs R_i, then W_j vs W_i (occ.cpp:185-199).
  // Four entries per step: 16-lane group g takes entry q0 + step + g, so
  // the dependent loads (aidx -> off -> accesses) of four entries overlap.
  const uint32_t q0 = a.aoff[t], q1 = a.aoff[t + 1];
  if (q1 < q0) c.err |= SNAP_ERR_AOFF;
  if (lane == 0) c.bytes += 8;
  const uint32_t g = lane >> 4, sl = lane & 15;
  for (uint32_t qb = q0; qb < q1 && !conflict; qb += 4) {
    const uint32_t q = qb + g;
    uint32_t j0 = 0, jl = 0;
    if (q < q1) {
      const uint32_t j = a.aidx[q];
      if (j >= a.n) {
        c.err |= SNAP_ERR_IDX;
      } else {
        j0 = a.off[j];
        jl = a.off[j + 1] - j0;
        if (jl > MAX_TXN_LEN) jl = 0;  // reported when txn j itself is visited
      }
      if (sl == 0) c.bytes += 4 + 8 + 9ull * jl;
    }
    bool h = false;
    for (uint32_t base = 0;; base += 16) {
      const bool act = base + sl < jl;
      if (ballot64(act) == 0) break;
      const bool jw = act && a.acctype[j0 + base + sl] == DCC_WR;
      const uint64_t kj = jw ? a.keys[j0 + base + sl] : 0;
      for (uint32_t x = 0; x < len; x++) h |= jw && readlane64(k, x) == kj;
    }
    conflict = ballot64(h) != 0;
  }
  if (lane == 0) {
    a.out_rc[t] = conflict ? DCC_RC_ABORT : DCC_RC_RCOK;
    c.n_commit += conflict ? 0 : 1;
    c.n_ro += wmask ? 0 : 1;
    c.n_w += __popcll(wmask);
  }
}

// Grouped path: four txns per wave, 16-lane group g owns txn tb + g and lane
// sl of it holds access sl (every txn of the four has <= 16 accesses, e.g.
// YCSB's REQ_PER_QUERY = 16).  Each group walks its own captured active list
// one entry per step; i's keys are read back from LDS as broadcast pairs.
__device__ void snap_grouped(const SnapArgs& a, uint64_t t, bool tv, uint32_t o0, uint32_t len,
                             uint32_t lane, uint64_t* sk, SnapCnt& c) {
  const uint32_t g = lane >> 4, sl = lane & 15;
  const bool have = tv && sl < len;
  const uint64_t k = have ? a.keys[o0 + sl] : 0;
  // the group's keys in this wave's LDS row; read back as broadcast 16-B
  // pairs (one LDS op per two keys instead of two ds_bpermute per key).
  // LDS ops of one wave complete in order; the wave barrier keeps the
  // compiler from moving the reads above the write.
  __builtin_amdgcn_wave_barrier();
  sk[lane] = k;
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  const bool wr = have && a.acctype[o0 + sl] == DCC_WR;
  const uint64_t wgrp = (ballot64(wr) >> (16 * g)) & 0xFFFFull;
  if (tv && sl == 0) c.bytes += 4 + 9ull * len;
  uint32_t q0 = 0, q1 = 0;
  if (tv) {
    q0 = a.aoff[t];
    q1 = a.aoff[t + 1];
    if (q1 < q0) {
      c.err |= SNAP_ERR_AOFF;
      q1 = q0;
    }
    if (sl == 0) c.bytes += 8;
  }
  // (issued before the history lookup: the two gather chains overlap)
  // the first 16 captured entries of every group are resolved up front, one
  // per lane (aidx -> off in parallel), so a step only loads j's accesses
  uint32_t pj0 = 0, pjl = 0;
  if (tv && q0 + sl < q1) {
    const uint32_t j = a.aidx[q0 + sl];
    if (j >= a.n) {
      c.err |= SNAP_ERR_IDX;
    } else {
      pj0 = a.off[j];
      pjl = a.off[j + 1] - pj0;
      if (pjl > MAX_TXN_LEN) pjl = 0;
    }
  }
  bool hit = false;
  if (tv && a.start_tn) {
    const uint64_t s = a.start_tn[t], f = a.finish_tn[t];
    uint64_t hi = f;
    if (a.hist_top) hi = min(hi, a.hist_top[t]);
    if (sl == 0) c.bytes += a.hist_top ? 24 : 16;
    if (f > s && hi > s && have && !wr) hit = hist_hit(a.hist, k, s, hi);
  }
  bool conflict = ((ballot64(hit) >> (16 * g)) & 0xFFFFull) != 0;
  // entry e (uniform) of this group's list: from the up-front lanes when e < 16
  auto entry = [&](uint32_t e, bool go, uint32_t& j0, uint32_t& jl) {
    j0 = 0;
    jl = 0;
    if (e < 16) {
      j0 = __shfl(pj0, (int)(g * 16 + e));
      jl = __shfl(pjl, (int)(g * 16 + e));
      if (!go) jl = 0;
    } else if (go) {
      const uint32_t j = a.aidx[q0 + e];
      if (j >= a.n) {
        c.err |= SNAP_ERR_IDX;
      } else {
        j0 = a.off[j];
        jl = a.off[j + 1] - j0;
        if (jl > MAX_TXN_LEN) jl = 0;
      }
    }
    if (go && sl == 0) c.bytes += 4 + 8 + 9ull * jl;
  };
  // SNAP_EPS entries per step: their accesses are in flight together (an
  // entry checked after a conflict cannot change the decision)
  for (uint32_t step = 0;; step += SNAP_EPS) {
    const bool go0 = tv && !conflict && q0 + step < q1;
    if (ballot64(go0) == 0) break;
    uint32_t je[SNAP_EPS], le[SNAP_EPS];
#pragma unroll
    for (int e = 0; e < SNAP_EPS; e++)
      entry(step + e, go0 && q0 + step + e < q1, je[e], le[e]);
    bool h = false;
    for (uint32_t base = 0;; base += 16) {
      bool any = false;
#pragma unroll
      for (int e = 0; e < SNAP_EPS; e++) any |= base + sl < le[e];
      if (ballot64(any) == 0) break;
      uint64_t ke[SNAP_EPS];
      bool we[SNAP_EPS];
#pragma unroll
      for (int e = 0; e < SNAP_EPS; e++) {
        const bool act = base + sl < le[e];
        we[e] = act && a.acctype[je[e] + base + sl] == DCC_WR;
        ke[e] = we[e] ? a.keys[je[e] + base + sl] : 0;
      }
      for (uint32_t x = 0; x < 16; x += 2) {
        const ulonglong2 kx = *reinterpret_cast<const ulonglong2*>(&sk[g * 16 + x]);
        const bool m0 = x < len, m1 = x + 1 < len;
#pragma unroll
        for (int e = 0; e < SNAP_EPS; e++)
          h |= we[e] && ((m0 && kx.x == ke[e]) || (m1 && kx.y == ke[e]));
      }
    }
    conflict = conflict || ((ballot64(h) >> (16 * g)) & 0xFFFFull) != 0;
  }
  if (tv && sl == 0) {
    a.out_rc[t] = conflict ? DCC_RC_ABORT : DCC_RC_RCOK;
    c.n_commit += conflict ? 0 : 1;
    c.n_ro += wgrp ? 0 : 1;
    c.n_w += __popcll(wgrp);
  }
}

__global__ __launch_bounds__(256) void k_snap(SnapArgs a) {
  const uint32_t lane = threadIdx.x & 63;
  const uint64_t wave0 = (uint64_t)blockIdx.x * SNAP_WAVES + (threadIdx.x >> 6);
  const uint64_t stride = (uint64_t)gridDim.x * SNAP_WAVES;
  __shared__ __attribute__((aligned(16))) uint64_t skeys[SNAP_WAVES][64];
  uint64_t* sk = skeys[threadIdx.x >> 6];
  SnapCnt c;
  for (uint64_t tb = wave0 * 4; tb < a.n; tb += stride * 4) {
    const uint64_t t = tb + (lane >> 4);
    const bool tv = t < a.n;
    uint32_t o0 = 0, len = 0;
    if (tv) {
      o0 = a.off[t];
      len = a.off[t + 1] - o0;  // a decreasing offset wraps to a huge length
    }
    if (ballot64(len > 16) == 0) {
      snap_grouped(a, t, tv, o0, len, lane, sk, c);
    } else {
      for (uint64_t u = tb; u < tb + 4 && u < a.n; u++) snap_full(a, u, lane, c);
    }
  }
  // per-lane partials: reduce over the wave
  uint64_t v1 = c.n_commit, v2 = c.n_ro, v3 = c.n_w;
  uint32_t err = c.err;
  uint64_t bytes = c.bytes;
  for (int m = 32; m >= 1; m >>= 1) {
    bytes += __shfl_xor(bytes, m);
    v1 += __shfl_xor(v1, m);
    v2 += __shfl_xor(v2, m);
    v3 += __shfl_xor(v3, m);
    err |= __shfl_xor(err, m);
  }
  if (lane < SNAP_NCNT) {  // every wave of the grid writes its row
    const unsigned long long v[SNAP_NCNT] = {err, v1, v2, v3, bytes};
    unsigned long long x = v[0];
    for (int q = 1; q < SNAP_NCNT; q++) x = lane == (uint32_t)q ? v[q] : x;
    a.part[wave0 * SNAP_NCNT + lane] = x;
  }
}

#define CK(expr)                                           \
  do {                                                     \
    hipError_t e_ = (expr);                                \
    if (e_ != hipSuccess) return ctx->hip_fail(e_, #expr); \
  } while (0)
#define CR(expr)                 \
  do {                           \
    int r_ = (expr);             \
    if (r_ != DCC_OK) return r_; \
  } while (0)

}  // namespace

int dcc_ctx::occ_snapshot(const dcc_batch* b, const dcc_occ_snapshot* s, uint8_t* out_rc,
                          dcc_stats* st) {
  dcc_ctx* ctx = this;
  const auto t_wall0 = std::chrono::steady_clock::now();
  if (!s || !s->active_off) return fail(DCC_EINVAL, "snapshot: null snapshot or active_off");
  // a device capture is not read on the host: its lists must be addressable
  if ((b && (b->flags & DCC_DEVICE_PTRS)) && !s->active_idx)
    return fail(DCC_EINVAL, "snapshot: device capture needs active_idx (a 1-element buffer "
                            "when every list is empty)");
  if (comm_ranks() > 1) return fail(DCC_ENOTSUP, "snapshot validation is single-GPU");
  CR(check_batch(b));
  dcc_stats S;
  memset(&S, 0, sizeof S);
  S.n_shards = 1;
  if (b->n_txn == 0) {
    if (st) *st = S;
    return DCC_OK;
  }
  if (!out_rc) return fail(DCC_EINVAL, "snapshot: null out_rc");
  const uint64_t n = b->n_txn;
  const bool dev = (b->flags & DCC_DEVICE_PTRS) != 0;
  uint64_t n_active = 0;
  if (!dev) {
    // host capture: full structural validation before any launch
    const uint32_t* ao = s->active_off;
    if (ao[0] != 0) return fail(DCC_EINVAL, "snapshot: active_off[0] must be 0");
    for (uint64_t t = 0; t < n; t++)
      if (ao[t + 1] < ao[t])
        return fail(DCC_EINVAL, "snapshot: active_off decreases at txn %llu", (unsigned long long)t);
    n_active = ao[n];
    if (n_active && !s->active_idx) return fail(DCC_EINVAL, "snapshot: null active_idx");
    for (uint64_t q = 0; q < n_active; q++)
      if (s->active_idx[q] >= n)
        return fail(DCC_EINVAL, "snapshot: active_idx[%llu] = %u >= n_txn", (unsigned long long)q,
                    s->active_idx[q]);
  }
  DevBatch d;
  CR(stage_batch(b, d));
  const uint64_t* top = s->hist_top;
  const uint32_t* aoff = s->active_off;
  const uint32_t* aidx = s->active_idx;
  if (!dev) {
    CR(snap_aoff.ensure(this, (n + 1) * 4, "snapshot active_off"));
    CR(snap_aidx.ensure(this, std::max<uint64_t>(16, n_active * 4), "snapshot active_idx"));
    CK(hipMemcpyAsync(snap_aoff.p, aoff, (n + 1) * 4, hipMemcpyHostToDevice, stream));
    if (n_active)
      CK(hipMemcpyAsync(snap_aidx.p, aidx, n_active * 4, hipMemcpyHostToDevice, stream));
    aoff = (const uint32_t*)snap_aoff.p;
    aidx = (const uint32_t*)snap_aidx.p;
    if (top) {
      CR(snap_top.ensure(this, n * 8, "snapshot hist_top"));
      CK(hipMemcpyAsync(snap_top.p, top, n * 8, hipMemcpyHostToDevice, stream));
      top = (const uint64_t*)snap_top.p;
    }
    CR(rc.ensure(this, n + 16, "rc"));
  }
  const bool hist_on = d.start_tn && hist_size() > 0;
  if (hist_on) CR(hist_prepare());
  HistView hv{};
  if (hist_on) hv = hist_view();
  const uint64_t waves_needed = (n + 3) / 4;  // four txns per wave step
  uint64_t grid = (waves_needed + SNAP_WAVES - 1) / SNAP_WAVES;
  grid = std::min<uint64_t>(grid, (uint64_t)n_cu * 16);
  const uint32_t waves = (uint32_t)grid * SNAP_WAVES;
  CR(snap_cnt.ensure(this, 64 + (uint64_t)waves * SNAP_NCNT * 8, "snapshot counters"));
  unsigned long long* cnt_dev = (unsigned long long*)snap_cnt.p;
  SnapArgs a{n,
             d.off,
             d.keys,
             d.acctype,
             hist_on ? d.start_tn : nullptr,
             hist_on ? d.finish_tn : nullptr,
             top,
             aoff,
             aidx,
             hv,
             dev ? out_rc : (uint8_t*)rc.p,
             cnt_dev + 8};
  CK(hipEventRecord(ev0, stream));
  k_snap<<<(unsigned)grid, 256, 0, stream>>>(a);
  CK(hipGetLastError());
  k_snap_sum<<<1, SUM_THREADS, 0, stream>>>(cnt_dev + 8, waves, cnt_dev);
  CK(hipGetLastError());
  CK(hipEventRecord(ev1, stream));
  unsigned long long cnt[5];
  CK(hipMemcpyAsync(cnt, cnt_dev, sizeof cnt, hipMemcpyDeviceToHost, stream));
  if (!dev) CK(hipMemcpyAsync(out_rc, rc.p, n, hipMemcpyDeviceToHost, stream));
  CK(hipStreamSynchronize(stream));
  if (cnt[0])
    return fail(DCC_EINVAL, "snapshot: malformed device capture (error bits 0x%llx)", cnt[0]);
  float ms = 0.f;
  CK(hipEventElapsedTime(&ms, ev0, ev1));
  S.n_commit = cnt[1];
  S.n_abort = n - cnt[1];
  S.n_readonly = cnt[2];
  S.nnz_w = cnt[3];
  S.alg_bytes = cnt[4];
  S.device_ms = ms;
  S.total_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t_wall0)
                   .count();
  if (st) *st = S;
  return DCC_OK;
}

extern "C" int dcc_occ_validate_snapshot(dcc_ctx* ctx, const dcc_batch* batch,
                                         const dcc_occ_snapshot* snap, uint8_t* out_rc,
                                         dcc_stats* out_stats) {
  if (!ctx) return DCC_EINVAL;
  if (ctx->multi) return dcc_multi_occ_snapshot(ctx, batch, snap, out_rc, out_stats);
  if (hipSetDevice(ctx->device) != hipSuccess) return DCC_ENODEV;
  return ctx->occ_snapshot(batch, snap, out_rc, out_stats);
}
