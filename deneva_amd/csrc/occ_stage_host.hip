// Host driver of the OCC stage solver (occ_stage.hip):
// workspaces, the per-epoch stage launch sequence (captured once in a HIP
// graph), completion / error read-back, and the hand-off to the round solver
// when the stage lists stop shrinking.
//
// Reference: OptCC::central_validate / central_finish applied to a whole
// epoch (concurrency_control/occ.cpp:116-294); entry dcc_occ_validate_epoch.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdlib>
#include <cstdio>
#include <cstring>
#include <vector>

#include "dcc.h"
#include "dcc_ctx.h"
#include "dcc_device.h"
#include "occ_kernels.h"
#include "occ_stage.h"

using namespace dcc;

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

namespace {

constexpr uint32_t ST_CH0 = 256;         // stage 0: epoch txns per chunk
constexpr uint32_t ST_CH1 = 1024;        // stage 1: epoch txns per chunk
constexpr uint32_t ST_P0 = 1024;         // stage 0 decides the epoch's first P0 txns
constexpr uint32_t ST_GPUB1 = 128;       // stage-1 chunks published to its decider
constexpr uint32_t ST_GRAPH_STAGES = 10; // stages in the captured epoch

// "a,b,c" -> values (tuning experiments)
std::vector<uint32_t> env_list(const char* name) {
  std::vector<uint32_t> v;
  if (const char* e = getenv(name))
    for (const char* c = e; *c;) {
      char* x;
      const unsigned long p = strtoul(c, &x, 10);
      if (x == c) break;
      v.push_back((uint32_t)p);
      c = *x ? x + 1 : x;
    }
  return v;
}
uint32_t env_u32(const char* name, uint32_t dflt) {
  const std::vector<uint32_t> v = env_list(name);
  return v.empty() ? dflt : v[0];
}

// txns stage l's decider may decide (l >= 1); DCC_ST_PMAX="p1,p2,..."
uint32_t st_pmax(uint32_t l) {
  static const std::vector<uint32_t> ov = env_list("DCC_ST_PMAX");
  if (l - 1 < ov.size()) return std::max<uint32_t>(64, ov[l - 1]);
  if (!ov.empty()) return std::max<uint32_t>(64, ov.back());
  static const uint32_t dflt[] = {6144, 2048, 2048, 4096};
  return dflt[std::min<uint32_t>(l - 1, 3)];
}
uint32_t st_p0(uint64_t n) { return (uint32_t)std::min<uint64_t>(n, env_u32("DCC_ST_P0", ST_P0)); }
uint32_t st_chunks(uint64_t n, uint32_t l) {
  if (l == 0) return std::max<uint32_t>(1, (st_p0(n) + ST_CH0 - 1) / ST_CH0);
  uint32_t c = (uint32_t)std::max<uint64_t>(1, (n + ST_CH1 - 1) / ST_CH1);
  for (uint32_t q = 2; q <= l; q++) c = (c + ST_G - 1) / ST_G;
  return c;
}
uint32_t st_gpub(uint64_t n, uint32_t l) {
  const uint32_t c = st_chunks(n, l);
  if (l == 0) return c;
  if (l == 1) return std::min<uint32_t>(c, env_u32("DCC_ST_GPUB", ST_GPUB1));
  return std::min<uint32_t>(c, ST_MAX_PUB);
}

struct StMirror {
  StEpoch ep;
  StCtl ctl[ST_MAX_STAGES];
};

}  // namespace

int dcc_ctx::stage_reserve(const DevBatch& d) {
  dcc_ctx* ctx = this;
  const size_t ctl_bytes = sizeof(StEpoch) + ST_MAX_STAGES * sizeof(StCtl);
  void* old = st_ctl.p;
  CR(st_ctl.ensure(this, ctl_bytes, "stage control"));
  if (st_ctl.p != old) {
    CK(hipMemsetAsync(st_ctl.p, 0, ctl_bytes, stream));
    st_tnc_dev = 0;
  }
  const uint64_t chunks = (uint64_t)st_chunks(d.n, 1) + 8;
  for (int i = 0; i < 2; i++) {
    CR(st_tid[i].ensure(this, d.n * 4 + 64, "stage list tid"));
    CR(st_ast[i].ensure(this, d.n * 4 + 64, "stage list ast"));
    CR(st_alen[i].ensure(this, d.n + 64, "stage list alen"));
    CR(st_keys[i].ensure(this, std::max<uint64_t>(64, d.nnz * 8 + 64), "stage list keys"));
    CR(st_at[i].ensure(this, std::max<uint64_t>(64, d.nnz + 64), "stage list types"));
    CR(st_hsh[i].ensure(this, std::max<uint64_t>(64, d.nnz * 4 + 64), "stage list hashes"));
    CR(st_dep[i].ensure(this, d.n * 8 + 64, "stage list dependency masks"));
    CR(st_tile[i].ensure(this, (d.n + 64) * ST_TILE_WORDS * 8, "stage tile descriptors"));
    void* oh = st_hdr[i].p;
    CR(st_hdr[i].ensure(this, chunks * sizeof(StChunk), "stage chunk headers"));
    // a fresh header block must not hold a flag a future tag could match
    if (st_hdr[i].p != oh) CK(hipMemsetAsync(st_hdr[i].p, 0, st_hdr[i].cap, stream));
    CR(st_ck[i].ensure(this, (ST_CS_BUDGET + 4096 + 64) * 8, "stage committed keys"));
  }
  return DCC_OK;
}

int dcc_ctx::stage_enqueue(const DevBatch& d, uint32_t l0, uint32_t l1, uint8_t* rc_dev,
                           uint64_t* tn_dev, const uint8_t* hkill) {
  dcc_ctx* ctx = this;
  StEpoch* ep = (StEpoch*)st_ctl.p;
  StCtl* ctl = (StCtl*)((char*)st_ctl.p + sizeof(StEpoch));
  auto list = [&](uint32_t side) {
    return StList{(uint32_t*)st_tid[side].p,  (uint32_t*)st_ast[side].p, (uint8_t*)st_alen[side].p,
                  (uint64_t*)st_dep[side].p,  (uint64_t*)st_keys[side].p, (uint32_t*)st_hsh[side].p,
                  (uint8_t*)st_at[side].p,    (uint64_t*)st_tile[side].p, (StChunk*)st_hdr[side].p};
  };
  for (uint32_t l = l0; l < l1; l++) {
    StArgs a{};
    a.stage = l;
    a.mode = l < 2 ? 0u : 1u;
    a.n = (uint32_t)d.n;
    a.nnz = d.nnz;
    a.off = d.off;
    a.keys = d.keys;
    a.at = d.acctype;
    a.p0 = st_p0(d.n);
    a.e_end = l == 0 ? a.p0 : (uint32_t)d.n;
    a.ch = l == 0 ? ST_CH0 : ST_CH1;
    if (l >= 2) {
      a.in = list((l - 1) & 1);
      a.in_chunks = st_chunks(d.n, l - 1);
    }
    a.out = list(l & 1);
    a.out_chunks = st_chunks(d.n, l);
    a.gpub = st_gpub(d.n, l);
    a.pmax = l == 0 ? a.p0 : st_pmax(l);
    a.decide = 1;
    a.prev = l ? ctl + l - 1 : nullptr;
    a.cur = ctl + l;
    a.next = l + 1 < ST_MAX_STAGES ? ctl + l + 1 : nullptr;
    a.ck_prev = l ? (const uint64_t*)st_ck[(l - 1) & 1].p : nullptr;
    a.ck_cur = (uint64_t*)st_ck[l & 1].p;
    a.ep = ep;
    a.hkill = hkill;
    a.rc = rc_dev;
    a.tn = tn_dev;
    a.dbg = st_debug ? (uint64_t*)st_dbg.p : nullptr;
    a.xflags = env_u32("DCC_ST_X", 0);
    if (profiling && l < 3) CK(hipEventRecord(pev[l], stream));
    launch_stage(a, stream);
  }
  CK(hipGetLastError());
  return DCC_OK;
}

int dcc_ctx::occ_stage_epoch(const dcc_batch* b, uint8_t* out_rc, uint64_t* out_tn, dcc_stats* st) {
  dcc_ctx* ctx = this;
  const auto t_wall0 = std::chrono::steady_clock::now();
  CR(check_batch(b));
  dcc_stats S;
  memset(&S, 0, sizeof S);
  S.n_shards = 1;
  if (b->n_txn == 0) {
    if (st) *st = S;
    return DCC_OK;
  }
  if (b->n_txn >= 0xFFFFFFFFull) return fail(DCC_ERANGE, "batch: n_txn exceeds 2^32-2");
  DevBatch d;
  CR(stage_batch(b, d));
  CR(stage_reserve(d));
  const bool dev_out = (b->flags & DCC_DEVICE_PTRS) != 0;
  CR(rc.ensure(this, d.n + 16, "rc"));
  const bool want_tn = out_tn != nullptr || (b->flags & DCC_OCC_APPEND_HISTORY);
  if (want_tn) CR(tn.ensure(this, d.n * 8 + 16, "tn"));
  uint8_t* rc_dev = (dev_out && out_rc) ? out_rc : (uint8_t*)rc.p;
  uint64_t* tn_dev = want_tn ? ((dev_out && out_tn) ? out_tn : (uint64_t*)tn.p) : nullptr;
  StEpoch* ep = (StEpoch*)st_ctl.p;
  StCtl* ctl = (StCtl*)((char*)st_ctl.p + sizeof(StEpoch));
  // the commit counter the deciders continue from (occ.h:67)
  if (st_tnc_dev != tnc) {
    st_tnc_upload = tnc;
    CK(hipMemcpyAsync(&ep->tnc, &st_tnc_upload, 8, hipMemcpyHostToDevice, stream));
    st_tnc_dev = tnc;
  }
  // history window pre-pass (occ.cpp:160-180): per-txn aborts the filters and
  // deciders treat as dead
  const bool hist_on = d.start_tn && !hist.empty();
  const uint8_t* hkill = nullptr;
  if (hist_on) {
    CR(state.ensure(this, d.n + 16, "state"));
    CK(hipMemsetAsync(state.p, 0, d.n + 16, stream));
    CR(upload_history());
    HistArgs ha{d.n, d.off, d.keys, d.acctype, d.start_tn, d.finish_tn,
                (const uint64_t*)hkeys.p, h_nkeys, (const uint64_t*)hoff.p,
                (const uint64_t*)htn.p, (uint8_t*)state.p};
    launch_hist(ha, stream);
    hkill = (const uint8_t*)state.p;
  }
  const uint32_t S_graph = std::min<uint32_t>(ST_MAX_STAGES, env_u32("DCC_ST_STAGES", ST_GRAPH_STAGES));
  StFinalArgs fa{ep, ctl, S_graph, st_host_dev};
  st_debug = getenv("DCC_ST_DEBUG") != nullptr;
  if (st_debug) {
    CR(st_dbg.ensure(this, ST_MAX_STAGES * 32 * 8, "stage debug"));
    std::vector<uint64_t> init(ST_MAX_STAGES * 32, 0);
    for (uint32_t l = 0; l < ST_MAX_STAGES; l++) init[l * 32 + 18] = init[l * 32 + 19] = ~0ull;
    CK(hipMemcpy(st_dbg.p, init.data(), init.size() * 8, hipMemcpyHostToDevice));
  }
  const bool graph_ok = !profiling && !hist_on && !st_debug && !getenv("DCC_NO_GRAPH");
  const GraphKey gkey{d.off, d.keys, d.acctype, d.n, d.nnz, rc_dev, tn_dev != nullptr, S_graph,
                      buf_gen + (uint64_t)(uintptr_t)tn_dev};
  if (graph_ok && st_graph && gkey == st_graph_key) {
    CK(hipEventRecord(ev0, stream));
    CK(hipGraphLaunch(st_graph, stream));
    CK(hipEventRecord(ev1, stream));
  } else if (graph_ok) {
    if (st_graph) {
      (void)hipGraphExecDestroy(st_graph);
      st_graph = nullptr;
    }
    CK(hipStreamBeginCapture(stream, hipStreamCaptureModeThreadLocal));
    int r = stage_enqueue(d, 0, S_graph, rc_dev, tn_dev, hkill);
    if (r == DCC_OK) launch_stage_final(fa, stream);
    hipGraph_t g = nullptr;
    const hipError_t ce = hipStreamEndCapture(stream, &g);
    if (r != DCC_OK) {
      if (g) (void)hipGraphDestroy(g);
      return r;
    }
    CK(ce);
    const hipError_t ie = hipGraphInstantiate(&st_graph, g, nullptr, nullptr, 0);
    (void)hipGraphDestroy(g);
    if (ie != hipSuccess) {
      st_graph = nullptr;
      return fail(DCC_EIO, "hipGraphInstantiate: %s", hipGetErrorString(ie));
    }
    st_graph_key = gkey;
    CK(hipEventRecord(ev0, stream));
    CK(hipGraphLaunch(st_graph, stream));
    CK(hipEventRecord(ev1, stream));
  } else {
    CK(hipEventRecord(ev0, stream));
    CR(stage_enqueue(d, 0, S_graph, rc_dev, tn_dev, hkill));
    if (profiling) CK(hipEventRecord(pev[3], stream));
    launch_stage_final(fa, stream);
    CK(hipGetLastError());
    CK(hipEventRecord(ev1, stream));
  }
  CK(hipStreamSynchronize(stream));
  StMirror M;
  memcpy(&M, st_host, sizeof(StEpoch) + S_graph * sizeof(StCtl));
  uint32_t last = S_graph - 1;
  // more stages when the captured ones did not finish the list (rare)
  auto remaining = [&](const StCtl& c) { return c.surv_n > c.consumed ? c.surv_n - c.consumed : 0u; };
  uint32_t err = 0;
  bool abandon = false;
  for (uint32_t l = 0; l <= last; l++) {
    err |= M.ctl[l].err;
    abandon |= M.ctl[l].abandon != 0;
  }
  while (!err && !abandon && remaining(M.ctl[last]) && last + 1 < ST_MAX_STAGES) {
    const uint32_t l = last + 1;
    CR(stage_enqueue(d, l, l + 1, rc_dev, tn_dev, hkill));
    StFinalArgs fx{ep, ctl, l + 1, st_host_dev};
    launch_stage_final(fx, stream);
    CK(hipGetLastError());
    CK(hipEventRecord(ev1, stream));
    CK(hipStreamSynchronize(stream));
    const StMirror* h = (const StMirror*)st_host;
    M.ctl[l] = h->ctl[l];
    M.ep = h->ep;
    err |= M.ctl[l].err;
    abandon |= M.ctl[l].abandon != 0;
    last = l;
  }
  if (st_debug) {
    std::vector<uint64_t> v(ST_MAX_STAGES * 32);
    CK(hipMemcpy(v.data(), st_dbg.p, v.size() * 8, hipMemcpyDeviceToHost));
    for (uint32_t l = 0; l <= last; l++) {
      const uint64_t* x = v.data() + l * 32;
      if (!x[0]) continue;
      const double us = 0.01;  // s_memrealtime: 100 MHz
      fprintf(stderr,
              "stage %u: decider first take %.2f us, second take at %+.2f, loop end %+.2f | tiles %llu "
              "decided %llu chunks %llu | per tile cycles probe %.0f fixpoint %.0f insert %.0f | "
              "filter first start %+.2f, first done %+.2f, last published %+.2f, last done %+.2f "
              "(us from decider start)\n",
              l, (x[1] - x[0]) * us, x[2] ? ((double)x[2] - (double)x[0]) * us : 0.0,
              ((double)x[3] - (double)x[0]) * us, (unsigned long long)x[7], (unsigned long long)x[8],
              (unsigned long long)x[9], x[7] ? (double)x[4] / x[7] : 0.0,
              x[7] ? (double)x[5] / x[7] : 0.0, x[7] ? (double)x[6] / x[7] : 0.0,
              ((double)x[19] - (double)x[0]) * us, ((double)x[18] - (double)x[0]) * us,
              ((double)x[17] - (double)x[0]) * us, ((double)x[16] - (double)x[0]) * us);
    }
  }
  if (err & STE_OFFSETS) return fail(DCC_EINVAL, "batch: malformed offsets");
  if (err & STE_LEN)
    return fail(DCC_ERANGE, "batch: a txn has more than MAX_ROW_PER_TXN=%u accesses", MAX_TXN_LEN);
  if (err & STE_KEY) return fail(DCC_EINVAL, "batch: key equal to DCC_KEY_RESERVED");
  if (err & STE_SPIN) return fail(DCC_EIO, "stage solver: chunk hand-off did not complete");
  const bool fallback = abandon || (err & STE_WMAP) || remaining(M.ctl[last]) != 0;
  if (fallback) {
    // the lists stopped shrinking (low contention) or a decider tile's write
    // map overflowed: decide the epoch with the round solver instead
    st_tnc_dev = ~0ull;
    st_fallbacks++;
    force_rounds = true;
    const int r2 = occ_epoch(b, out_rc, out_tn, st);
    force_rounds = false;
    if (st && r2 == DCC_OK) st->fallback = 1;
    return r2;
  }
  float ms = 0;
  CK(hipEventElapsedTime(&ms, ev0, ev1));
  uint64_t commits = 0, cw = 0;
  uint32_t stages = 0;
  for (uint32_t l = 0; l <= last; l++) {
    commits += M.ctl[l].commits;
    cw += M.ctl[l].cw;
    stages += M.ctl[l].ran;
  }
  S.rounds = stages;
  S.n_commit = commits;
  S.n_abort = d.n - commits;
  S.n_readonly = (uint64_t)M.ctl[0].ro + M.ctl[1].ro;
  S.nnz_w = (uint64_t)M.ctl[0].nnz_w + M.ctl[1].nnz_w;
  S.alg_bytes = dcc_alg_bytes(d.n, d.nnz, S.nnz_w);
  S.device_ms = ms;
  S.peel_prefix = M.ctl[0].consumed;
  S.n_survivors = M.ctl[1].surv_n;
  if (profiling) {
    // phases: 0 = stage 0, 1 = stage 1 (the epoch-long filter + its decider),
    // 2 = stages >= 2, 3 = final
    float t0 = 0, t1 = 0, t2 = 0;
    CK(hipEventElapsedTime(&t0, ev0, pev[1]));
    CK(hipEventElapsedTime(&t1, pev[1], pev[2]));
    CK(hipEventElapsedTime(&t2, pev[2], pev[3]));
    S.phase_ms[0] = t0;
    S.phase_ms[1] = t1;
    S.phase_ms[2] = t2;
    S.phase_ms[3] = ms - t0 - t1 - t2;
    const uint64_t p0 = st_p0(d.n);
    S.phase_bytes[1] = 4 * (d.n - p0 + 1) + 9 * (d.nnz - std::min<uint64_t>(d.nnz, p0 * 16)) + d.n;
  }
  if (tnc + cw != M.ep.tnc) return fail(DCC_EIO, "stage solver: commit counter out of step");
  tnc = M.ep.tnc;
  st_tnc_dev = tnc;
  if (!dev_out) {
    if (out_rc) CK(hipMemcpyAsync(out_rc, rc_dev, d.n, hipMemcpyDeviceToHost, stream));
    if (out_tn) CK(hipMemcpyAsync(out_tn, tn_dev, d.n * 8, hipMemcpyDeviceToHost, stream));
    CK(hipStreamSynchronize(stream));
  }
  if (b->flags & DCC_OCC_APPEND_HISTORY) CR(history_append_epoch(b, d, tn_dev, dev_out, cw));
  const auto t_wall1 = std::chrono::steady_clock::now();
  S.total_ms = std::chrono::duration<double, std::milli>(t_wall1 - t_wall0).count();
  if (st) *st = S;
  return DCC_OK;
}
