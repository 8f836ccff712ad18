// libdcc host side: context lifecycle, workspaces and the OCC epoch driver.
// C ABI declared in include/dcc.h.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdarg>
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

#include "dcc.h"
#include "dcc_ctx.h"
#include "dcc_env.h"
#include "radix_sort.h"
#include "dcc_device.h"
#include "occ_kernels.h"

using namespace dcc;

// ---------------------------------------------------------------- helpers
int dcc_ctx::fail(int code, const char* fmt, ...) {
  char buf[512];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof buf, fmt, ap);
  va_end(ap);
  last_error = buf;
  return code;
}

int dcc_ctx::hip_fail(hipError_t e, const char* what) {
  return fail(DCC_EIO, "%s: %s", what, hipGetErrorString(e));
}

int DevBuf::ensure(dcc_ctx* c, size_t bytes, const char* what) {
  if (bytes <= cap) return DCC_OK;
  c->buf_gen++;  // a captured graph holding the old address is stale
  if (p) (void)hipFree(p);
  p = nullptr;
  cap = 0;
  size_t want = bytes + bytes / 8 + 256;  // grow-only with slack
  hipError_t e = hipMalloc(&p, want);
  if (e != hipSuccess) {
    p = nullptr;
    (void)hipGetLastError();
    return c->fail(DCC_ENOMEM, "hipMalloc(%s, %zu): %s", what, want, hipGetErrorString(e));
  }
  cap = want;
  return DCC_OK;
}

void DevBuf::release() {
  if (p) (void)hipFree(p);
  p = nullptr;
  cap = 0;
}

#define CK(expr)                                           \
  do {                                                     \
    hipError_t e_ = (expr);                                \
    if (e_ != hipSuccess) return ctx->hip_fail(e_, #expr); \
  } while (0)
#define CR(expr)             \
  do {                       \
    int r_ = (expr);         \
    if (r_ != DCC_OK) return r_; \
  } while (0)

static uint64_t next_pow2(uint64_t x) {
  uint64_t p = 1;
  while (p < x) p <<= 1;
  return p;
}

// ---------------------------------------------------------------- lifecycle
extern "C" int dcc_device_count(void) {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) {
    (void)hipGetLastError();
    return 0;
  }
  int g = 0;
  for (int i = 0; i < n; i++) {
    hipDeviceProp_t p;
    if (hipGetDeviceProperties(&p, i) == hipSuccess && strncmp(p.gcnArchName, "gfx950", 6) == 0) g++;
  }
  return g;
}

extern "C" int dcc_version(void) { return 100; }

extern "C" const char* dcc_strerror(int code) {
  switch (code) {
    case DCC_OK: return "success";
    case DCC_EIO: return "HIP runtime failure";
    case DCC_ENOMEM: return "out of memory";
    case DCC_ENODEV: return "no usable gfx950 device";
    case DCC_EINVAL: return "invalid argument or malformed batch";
    case DCC_ERANGE: return "size exceeds an engine limit";
    case DCC_ECOMM: return "RCCL communicator failure";
    case DCC_ENOTSUP: return "not supported";
    default: return "unknown error";
  }
}

extern "C" const char* dcc_last_error(const dcc_ctx* ctx) {
  return ctx ? ctx->last_error.c_str() : "null context";
}

extern "C" int dcc_init(dcc_ctx** out, int device_id) {
  if (!out) return DCC_EINVAL;
  *out = nullptr;
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) {
    (void)hipGetLastError();
    return DCC_ENODEV;
  }
  if (device_id < 0) {
    if (hipGetDevice(&device_id) != hipSuccess) return DCC_ENODEV;
  }
  if (device_id >= ndev) return DCC_ENODEV;
  hipDeviceProp_t prop;
  if (hipGetDeviceProperties(&prop, device_id) != hipSuccess) return DCC_ENODEV;
  if (strncmp(prop.gcnArchName, "gfx950", 6) != 0) return DCC_ENODEV;
  if (hipSetDevice(device_id) != hipSuccess) return DCC_ENODEV;
  dcc_ctx* ctx = new dcc_ctx();
  ctx->device = device_id;
  ctx->n_cu = prop.multiProcessorCount;
  CK(hipStreamCreateWithFlags(&ctx->own_stream, hipStreamNonBlocking));
  ctx->stream = ctx->own_stream;
  CK(hipEventCreate(&ctx->ev0));
  CK(hipEventCreate(&ctx->ev1));
  for (auto& e : ctx->pev) CK(hipEventCreate(&e));
  CK(hipHostMalloc((void**)&ctx->hmisc, 16384, hipHostMallocDefault));
  CK(hipHostMalloc((void**)&ctx->hpart, 1 << 17, hipHostMallocDefault));
  CK(hipHostGetDevicePointer(&ctx->hmisc_dev, ctx->hmisc, 0));
  CK(hipHostGetDevicePointer(&ctx->hpart_dev, ctx->hpart, 0));
  ctx->hs[1].chained = true;  // the delta level (dcc_ctx.h HistStore)
  CK(hipHostMalloc((void**)&ctx->hdyn, dcc_ctx::HDYN_BYTES, hipHostMallocDefault));
  CK(hipHostGetDevicePointer(&ctx->hdyn_dev, ctx->hdyn, 0));
  memset(ctx->hdyn, 0, dcc_ctx::HDYN_BYTES);
  int rc = ctx->misc.ensure(ctx, 16384, "misc");
  if (!rc) rc = ctx->part.ensure(ctx, 1 << 17, "partials");
  // counters and barrier words start zeroed (hipMalloc memory is not)
  if (!rc && (hipMemset(ctx->misc.p, 0, 16384) != hipSuccess ||
              hipMemset(ctx->part.p, 0, 1 << 17) != hipSuccess))
    rc = DCC_EIO;
  if (rc) {
    dcc_destroy(ctx);
    return rc;
  }
  *out = ctx;
  return DCC_OK;
}

extern "C" void dcc_destroy(dcc_ctx* ctx) {
  if (!ctx) return;
  dcc_pipe_destroy(ctx);
  dcc_multi_destroy(ctx);
  (void)hipSetDevice(ctx->device);
  if (ctx->stream) (void)hipStreamSynchronize(ctx->stream);
  if (ctx->graph_exec) (void)hipGraphExecDestroy(ctx->graph_exec);
  if (ctx->cv_graph_exec) (void)hipGraphExecDestroy(ctx->cv_graph_exec);
  dcc_comm_destroy(ctx);
  for (DevBuf* b : ctx->all_bufs()) b->release();
  if (ctx->hmisc) (void)hipHostFree(ctx->hmisc);
  if (ctx->hpart) (void)hipHostFree(ctx->hpart);
  if (ctx->hdyn) (void)hipHostFree(ctx->hdyn);
  if (ctx->hfin) (void)hipHostFree(ctx->hfin);
  if (ctx->ev_done) (void)hipEventDestroy(ctx->ev_done);
  if (ctx->ev0) (void)hipEventDestroy(ctx->ev0);
  if (ctx->ev1) (void)hipEventDestroy(ctx->ev1);
  for (auto& e : ctx->pev)
    if (e) (void)hipEventDestroy(e);
  if (ctx->own_stream) (void)hipStreamDestroy(ctx->own_stream);
  delete ctx;
}

extern "C" int dcc_set_profiling(dcc_ctx* ctx, int enable) {
  if (!ctx) return DCC_EINVAL;
  if (ctx->multi)
    for (int r = 0; r < dcc_multi_size(ctx); r++) dcc_multi_sub(ctx, r)->profiling = enable != 0;
  ctx->profiling = enable != 0;
  return DCC_OK;
}

int dcc_multi_set_fail_rank(dcc_ctx* ctx, int rank);  // dcc_multi.cpp

extern "C" int dcc_set_option(dcc_ctx* ctx, int option, int64_t value) {
  if (!ctx) return DCC_EINVAL;
  if (option == DCC_OPT_FAIL_RANK) {
    if (!ctx->multi) return ctx->fail(DCC_EINVAL, "DCC_OPT_FAIL_RANK: multi-GPU contexts only");
    return dcc_multi_set_fail_rank(ctx, (int)value);
  }
  if (option == DCC_OPT_PIPELINE) {
    if (value < 1 || value > 8) return DCC_EINVAL;
    // the epochs in flight complete on their lanes (their results and
    // tickets stay until waited); the next submit resizes the lanes
    dcc_pipe_drain(ctx);
    ctx->pipe_lanes = (uint32_t)value;
    return DCC_OK;
  }
  if (option == DCC_OPT_PIPE_PARTITION) {
    if (value != 0 && value != 1) return DCC_EINVAL;
    dcc_pipe_drain(ctx);  // as DCC_OPT_PIPELINE; the lanes are re-created at the next submit
    ctx->pipe_part = (uint32_t)value;
    return DCC_OK;
  }
  if (option == DCC_OPT_PIPE_CHAIN) {
    if (value != 0 && value != 1) return DCC_EINVAL;
    dcc_pipe_drain(ctx);
    ctx->pipe_chain = (uint32_t)value;
    return DCC_OK;
  }
  if (ctx->multi)
    for (int r = 0; r < dcc_multi_size(ctx); r++) {
      const int e = dcc_set_option(dcc_multi_sub(ctx, r), option, value);
      if (e != DCC_OK) return e;
    }
  switch (option) {
    case DCC_OPT_RECHECK:
      if (value < 0) return DCC_EINVAL;
      ctx->recheck_max = (uint64_t)value;
      return DCC_OK;
    case DCC_OPT_SOLVER:
      if (value != 0 && value != 1 && value != 3) return DCC_EINVAL;
      ctx->solver = (int)value;
      return DCC_OK;
    case DCC_OPT_SWEEP_LEVELS:
      if (value < 0 || value > SW_MAX_LEVEL) return DCC_EINVAL;
      ctx->sw_levels = (uint32_t)value;
      return DCC_OK;
    case DCC_OPT_RO_SPLIT:
      // 0 off, 1 on; 4..24: on with a writer table of 2^value slots (tests
      // drive the overflow fallback with small tables)
      if (value != 0 && value != 1 && (value < 4 || value > 24)) return DCC_EINVAL;
      ctx->ro_split = value != 0;
      ctx->wt_bits = value >= 4 ? (uint32_t)value : WT_BITS_DEFAULT;
      return DCC_OK;
    case DCC_OPT_HIST_MERGE:
      if (value < 1) return DCC_EINVAL;
      ctx->hist_merge_min = (uint64_t)value;
      return DCC_OK;
    case DCC_OPT_CALVIN_PATH:
      if (value < 0 || value > 2) return DCC_EINVAL;
      ctx->cv_path = (int)value;
      return DCC_OK;
    case DCC_OPT_COMM_SOLO:
      if (value != 0 && value != 1) return DCC_EINVAL;
      if (ctx->comm) return ctx->fail(DCC_EINVAL, "DCC_OPT_COMM_SOLO: set before dcc_comm_init");
      ctx->comm_solo = value != 0;
      return DCC_OK;
    case DCC_OPT_BATCH_MAX:
      if (value < 1 || value > 32) return DCC_EINVAL;
      ctx->batch_max = (uint32_t)value;
      return DCC_OK;
    default: return DCC_EINVAL;
  }
}

extern "C" int dcc_set_stream(dcc_ctx* ctx, void* s) {
  if (!ctx) return DCC_EINVAL;
  if (ctx->multi) return ctx->fail(DCC_ENOTSUP, "multi-GPU context: one stream per sub-context");
  ctx->stream = s ? (hipStream_t)s : ctx->own_stream;
  return DCC_OK;
}

std::vector<DevBuf*> dcc_ctx::all_bufs() {
  std::vector<DevBuf*> v = {&misc, &part, &off, &keys, &acctype, &start_tn, &finish_tn, &table, &state,
                            &hasw, &cflag, &bsum, &tn, &rc, &stat, &dyn, &fin_part,
                            &order, &perm, &calvin_a, &calvin_b, &calvin_c, &calvin_d,
                            &cv_scratch, &cv_agg, &cv_group, &cv_wave, &cv_pgx, &cv_gsx,
                            &cv_gsize, &cv_done, &cv_maxl, &cv_cwmax, &cv_cwpos, &cv_cwmark, &cv_cwhot, &cv_cwpa, &cv_cwoa, &cv_cwhelp, &cv_cwrec2, &cv_seq_b, &cv_ok, &cv_len,
                            &cv_off2, &cv_tsum, &cv_hkeys, &cv_hat, &cb_e, &cb_out, &cb_cnt, &cb_small, &gst, &hasw_scr, &sw_ctl, &sw_status, &sw_dbg,
                            &sw_ckeys, &sw_gtab, &sw_rec, &sw_rk, &sw_fw, &sw_aent, &sw_mg, &sw_xcnt, &sw_xsend,
                            &sw_xrec, &sw_mcnt, &sw_moff, &sw_mkeys, &sw_mat, &sw_kill,
                            &sw_rflag, &sw_ro, &sw_wtab, &sw_cw, &sw_wtab_big,
                            &snap_top, &snap_aoff, &snap_aidx, &snap_cnt, &mt_rk,
                            &mt_misc, &mt_slot, &mt_sval, &mt_slot2, &mt_sval2, &mt_sfl,
                            &mt_stx, &mt_txn, &mt_agg, &mt_sflB, &mt_stxB, &mt_k1, &mt_tcnt, &mt_ul, &mt_lb, &mt_ptab, &ix_keys, &ix_ord, &ix_rows, &ix_cnt, &wv_buf, &ix_scr, &wv_hbuf, &wv_obuf,
                            &h_K[0], &h_K[1], &h_V[0], &h_V[1], &h_scr, &h_bsum, &h_bm,
                            &nar_keys, &nar_at, &nar_tn, &fin_ctl, &fdyn, &fin_off, &fin_keys, &fin_at, &fin_state, &fin_hasw, &fin_rc, &fin_cnt,
                            &sh_off, &sh_keys, &sh_at, &sh_src, &sh_cnt, &sh_bsum, &sh_rc, &sh_tn, &sh_grp};
  for (auto& h : hs)
    for (DevBuf* b : {&h.fk, &h.ft, &h.skey, &h.stn, &h.hash, &h.bm, &h.nx, &h.tcnt}) v.push_back(b);
  for (auto& sb : sw_list)
    for (DevBuf* b : {&sb.tid, &sb.off, &sb.keys, &sb.acctype, &sb.state}) v.push_back(b);
  for (int i = 0; i < 2; i++) {
    v.push_back(&l_tid[i]);
    v.push_back(&l_coff[i]);
    v.push_back(&l_cent[i]);
  }
  return v;
}

extern "C" int dcc_reserve(dcc_ctx* ctx, uint64_t max_txn, uint64_t max_nnz) {
  if (!ctx) return DCC_EINVAL;
  if (ctx->multi)
    for (int r = 0; r < dcc_multi_size(ctx); r++) {
      const int e = dcc_reserve(dcc_multi_sub(ctx, r), max_txn, max_nnz);
      if (e != DCC_OK) return e;
    }
  (void)hipSetDevice(ctx->device);
  const uint32_t tw = ROUND_CAP / MAX_TXN_LEN;  // worst case: MAX_ROW_PER_TXN-long txns
  int rc = ctx->state.ensure(ctx, max_txn + 16, "state");
  if (!rc) rc = ctx->hasw.ensure(ctx, max_txn + 16, "hasw");
  if (!rc) rc = ctx->rc.ensure(ctx, max_txn + 16, "rc");
  if (rc) return rc;
  return ctx->reserve_occ(max_txn, max_nnz, max_nnz, tw);
}

// ---------------------------------------------------------------- history
// The history lives on the device (occ_history.h): host appends are uploaded
// into the delta level's flat pairs, epochs append there on the device.
int dcc_ctx::hist_grow_flat(HistStore& h, uint64_t need) {
  dcc_ctx* ctx = this;
  if (need * 8 <= h.fk.cap && need * 8 <= h.ft.cap && (!h.chained || need * 4 <= h.nx.cap)) return DCC_OK;
  if (h.chained && need >= HIST_NIL) return fail(DCC_ENOMEM, "history delta level of %llu pairs",
                                                 (unsigned long long)need);
  const uint64_t want = std::max<uint64_t>(need + need / 2, 4096);
  for (DevBuf* b : {&h.fk, &h.ft, &h.nx}) {
    if (b == &h.nx && !h.chained) continue;
    const uint64_t w = b == &h.nx ? 4 : 8;
    DevBuf nb;
    CR(nb.ensure(this, want * w, "history pairs"));
    if (h.m) CK(hipMemcpyAsync(nb.p, b->p, h.m * w, hipMemcpyDeviceToDevice, stream));
    CK(hipStreamSynchronize(stream));
    b->release();
    *b = nb;
  }
  return DCC_OK;
}

// pairs with tns in [lo_tn, hi_tn] were appended after the first h.m
void dcc_ctx::hist_note(HistStore& h, uint64_t lo_tn, uint64_t hi_tn) {
  if (lo_tn < h.max_tn) h.mono = false;
  h.max_tn = std::max(h.max_tn, hi_tn);
  h.min_tn = std::min(h.min_tn, lo_tn);
  h.built = false;
}

// A level's sorted build (occ_history.h): the pairs sorted by (key, tn), the
// table (<= 25 % load; the delta's also has room for the pairs epochs push
// before its next rebuild: the merge threshold plus one more epoch like the
// last) and the key bitmap.  A table with a key past HIST_WALK of its home
// is built again twice as big.
int dcc_ctx::hist_build(HistStore& h) {
  dcc_ctx* ctx = this;
  if (h.built) return DCC_OK;
  h_bm_stale = true;
  if (h.m == 0 && !h.chained) {
    h.built = true;
    h.mono = true;
    return DCC_OK;
  }
  // experiments: DCC_HIST_SLOTS (slots per pair)
  static const uint64_t slots_per_pair = [] {
    const char* e = DCC_ENV("DCC_HIST_SLOTS");
    return e && atoi(e) >= 2 ? (uint64_t)atoi(e) : 4ull;
  }();
  uint64_t need = slots_per_pair * h.m;
  if (h.chained)
    need = std::max<uint64_t>({need, 65536,
                               4 * (std::max<uint64_t>(hist_merge_min, hs[0].m / 4) + h.last_app)});
  if (h.overflowed) need = std::max<uint64_t>(need, 4ull << h.hbits);
  h.hbits = 4;
  while ((1ull << h.hbits) < need) h.hbits++;
  const uint64_t mm = std::max<uint64_t>(h.m, 1);
  CR(h.skey.ensure(this, mm * 8, "history keys"));
  CR(h.stn.ensure(this, mm * 8, "history tns"));
  CR(h.hash.ensure(this, 32ull << h.hbits, "history table"));
  CR(h.tcnt.ensure(this, 16, "history table overflow flag"));
  CR(h.bm.ensure(this, (1u << HIST_BM_LOG) / 8, "history key bitmap"));
  CK(hipMemsetAsync(h.tcnt.p, 0, 16, stream));
  if (h.m == 0) {  // an empty delta: a clear table for the epochs' pushes
    CK(hipMemsetAsync(h.hash.p, 0xFF, 32ull << h.hbits, stream));
    CK(hipMemsetAsync(h.bm.p, 0, (1u << HIST_BM_LOG) / 8, stream));
    h.built = true;
    h.mono = true;
    h.overflowed = false;
    return DCC_OK;
  }
  for (int q = 0; q < 2; q++) {
    CR(h_K[q].ensure(this, h.m * 8, "history sort keys"));
    CR(h_V[q].ensure(this, h.m * 4, "history sort values"));
  }
  CR(h_scr.ensure(this, rs_scratch_words(h.m) * 4, "history sort scratch"));
  HistBuild b{h.m,
              (const uint64_t*)h.fk.p,
              (const uint64_t*)h.ft.p,
              h.mono,
              {(uint64_t*)h_K[0].p, (uint64_t*)h_K[1].p},
              {(uint32_t*)h_V[0].p, (uint32_t*)h_V[1].p},
              (uint32_t*)h_scr.p,
              (uint64_t*)h.skey.p,
              (uint64_t*)h.stn.p,
              (uint64_t*)h.hash.p,
              h.hbits,
              h.max_key ? 64u - (uint32_t)__builtin_clzll(h.max_key) : 1u,
              64u - (uint32_t)__builtin_clzll(h.max_tn | 1ull),
              (uint32_t*)h.tcnt.p};
  if (hist_build_level(b, stream)) CK(hipGetLastError());
  launch_hist_bm((const uint64_t*)h.fk.p, h.m, (uint32_t*)h.bm.p, stream);
  CK(hipGetLastError());
  CK(hipMemcpyAsync(hmisc, h.tcnt.p, 4, hipMemcpyDeviceToHost, stream));
  CK(hipStreamSynchronize(stream));
  if (*(const uint32_t*)hmisc) {  // a key past HIST_WALK: twice the slots
    h.overflowed = true;
    return hist_build(h);
  }
  h.overflowed = false;
  h.built = true;
  return DCC_OK;
}

HistInsert dcc_ctx::hist_insert_args(HistStore& h) {
  return HistInsert{(const uint64_t*)h.fk.p, (const uint64_t*)h.ft.p, (uint64_t*)h.hash.p,
                    (uint32_t*)h.nx.p, (uint32_t*)h.bm.p, (uint32_t*)h_bm.p, (uint32_t*)h.tcnt.p,
                    h.hbits, 0u};
}

// Merge the delta into the base once it outgrows a quarter of it (or 64K
// pairs), then rebuild whatever changed.
int dcc_ctx::hist_prepare() {
  dcc_ctx* ctx = this;
  HistStore& B = hs[0];
  HistStore& D = hs[1];
  CR(h_bm.ensure(this, (1u << HIST_BM_LOG) / 8, "history key bitmap"));
  if (D.m > std::max<uint64_t>(hist_merge_min, B.m / 4)) {
    CR(hist_grow_flat(B, B.m + D.m));
    CK(hipMemcpyAsync((uint64_t*)B.fk.p + B.m, D.fk.p, D.m * 8, hipMemcpyDeviceToDevice, stream));
    CK(hipMemcpyAsync((uint64_t*)B.ft.p + B.m, D.ft.p, D.m * 8, hipMemcpyDeviceToDevice, stream));
    // still tn-ordered within every key if the delta's tns all follow the base's
    B.mono = B.mono && D.mono && (B.m == 0 || D.min_tn >= B.max_tn);
    B.m += D.m;
    B.max_tn = std::max(B.max_tn, D.max_tn);
    B.min_tn = std::min(B.min_tn, D.min_tn);
    B.max_key = std::max(B.max_key, D.max_key);
    B.built = false;
    D.reset();  // buffers kept, level emptied (its table cleared by the build)
  }
  CR(hist_build(B));
  CR(hist_build(D));
  if (h_bm_stale) {
    launch_hist_bm_or(B.m ? (const uint32_t*)B.bm.p : nullptr, D.m ? (const uint32_t*)D.bm.p : nullptr,
                      (uint32_t*)h_bm.p, stream);
    CK(hipGetLastError());
    h_bm_stale = false;
  }
  return DCC_OK;
}

HistView dcc_ctx::hist_view() const {
  HistView v{};
  for (int q = 0; q < 2; q++) {
    const HistStore& h = hs[q];
    v.lv[q] = HistLevel{(const uint64_t*)h.hash.p, (const uint64_t*)h.stn.p,
                        h.chained ? (const uint64_t*)h.ft.p : nullptr, h.chained ? (const uint32_t*)h.nx.p : nullptr,
                        h.hbits, h.m && h.built ? 1u : 0u,
                        (uint32_t)std::min<uint64_t>(h.m, HIST_NIL), 0u};
  }
  v.bm = (const uint32_t*)h_bm.p;  // set by hist_prepare
  return v;
}

// central_finish for the epoch (occ.cpp:277-286): every write of a txn with a
// commit tn joins the delta level, in index (= tn) order, on the device.
int dcc_ctx::hist_append_epoch(const DevBatch& d, const uint64_t* tn_dev, uint64_t nnz_w,
                               uint64_t n_cw) {
  dcc_ctx* ctx = this;
  if (!n_cw || !nnz_w) return DCC_OK;
  HistStore& D = hs[1];
  CR(hist_grow_flat(D, D.m + nnz_w));
  const uint64_t nb = (d.n + 1023) / 1024;
  CR(h_bsum.ensure(this, (nb + 1) * 4 + 96, "history append scan"));
  uint32_t* bsum = (uint32_t*)h_bsum.p;
  // the total and the largest key appended share one read-back (16 B)
  uint32_t* total = bsum + ((nb + 1 + 3) & ~3ull);
  unsigned long long* kmax = (unsigned long long*)(total + 2);
  CK(hipMemsetAsync(total, 0, 16, stream));
  launch_hist_count(d.n, d.off, d.acctype, d.nnz, tn_dev, bsum, stream);
  rs_scan_one(bsum, (uint32_t)nb, total, stream);
  launch_hist_emit(d.n, d.off, d.keys, d.acctype, d.nnz, tn_dev, bsum, (uint64_t*)D.fk.p + D.m,
                   (uint64_t*)D.ft.p + D.m, kmax, stream);
  CK(hipGetLastError());
  CK(hipMemcpyAsync(hmisc, total, 16, hipMemcpyDeviceToHost, stream));
  CK(hipStreamSynchronize(stream));
  const uint32_t added = *(const uint32_t*)hmisc;
  D.max_key = std::max<uint64_t>(D.max_key, *(const uint64_t*)((const char*)hmisc + 8));
  if (added > nnz_w) return fail(DCC_EIO, "history append: %u writes > %llu", added,
                                 (unsigned long long)nnz_w);
  D.m += added;
  hist_note(D, tnc + 1, tnc + n_cw);
  return DCC_OK;
}

extern "C" int dcc_occ_history_append(dcc_ctx* ctx, const uint64_t* keys, const uint64_t* tn,
                                      uint64_t n) {
  if (!ctx || (n && (!keys || !tn))) return DCC_EINVAL;
  dcc_pipe_drain(ctx);
  if (n == 0) return DCC_OK;
  if (ctx->multi) {  // each rank keeps its key shard's history
    const int R = dcc_multi_size(ctx);
    std::vector<std::vector<uint64_t>> k(R), t(R);
    for (uint64_t i = 0; i < n; i++) {
      const uint32_t r = dcc_key_shard(keys[i], (uint32_t)R);
      k[r].push_back(keys[i]);
      t[r].push_back(tn[i]);
    }
    for (int r = 0; r < R; r++)
      if (!k[r].empty()) CR(dcc_occ_history_append(dcc_multi_sub(ctx, r), k[r].data(), t[r].data(),
                                                   k[r].size()));
    return DCC_OK;
  }
  if (hipSetDevice(ctx->device) != hipSuccess) return DCC_ENODEV;
  // stable by tn, so that the batch keeps tn order within every key
  std::vector<uint64_t> idx(n);
  for (uint64_t i = 0; i < n; i++) idx[i] = i;
  std::stable_sort(idx.begin(), idx.end(), [&](uint64_t a, uint64_t b) { return tn[a] < tn[b]; });
  std::vector<uint64_t> k2(n), t2(n);
  for (uint64_t i = 0; i < n; i++) {
    k2[i] = keys[idx[i]];
    t2[i] = tn[idx[i]];
  }
  HistStore& D = ctx->hs[1];
  CR(ctx->hist_grow_flat(D, D.m + n));
  CK(hipMemcpy((uint64_t*)D.fk.p + D.m, k2.data(), n * 8, hipMemcpyHostToDevice));
  CK(hipMemcpy((uint64_t*)D.ft.p + D.m, t2.data(), n * 8, hipMemcpyHostToDevice));
  D.m += n;
  ctx->hist_note(D, t2.front(), t2.back());
  D.max_key = std::max(D.max_key, *std::max_element(k2.begin(), k2.end()));
  return DCC_OK;
}

extern "C" int dcc_occ_history_clear(dcc_ctx* ctx) {
  if (!ctx) return DCC_EINVAL;
  dcc_pipe_drain(ctx);
  if (ctx->multi)
    for (int r = 0; r < dcc_multi_size(ctx); r++) dcc_occ_history_clear(dcc_multi_sub(ctx, r));
  for (HistStore& h : ctx->hs) h.reset();
  return DCC_OK;
}

extern "C" int dcc_occ_history_trim(dcc_ctx* ctx, uint64_t tn_floor) {
  if (!ctx) return DCC_EINVAL;
  dcc_pipe_drain(ctx);
  if (ctx->multi) {
    for (int r = 0; r < dcc_multi_size(ctx); r++) CR(dcc_occ_history_trim(dcc_multi_sub(ctx, r), tn_floor));
    return DCC_OK;
  }
  if (hipSetDevice(ctx->device) != hipSuccess) return DCC_ENODEV;
  HistStore& B = ctx->hs[0];
  HistStore& D = ctx->hs[1];
  const uint64_t tot = B.m + D.m;
  if (tot == 0) return DCC_OK;
  // survivors (tn > floor) of both levels into fresh flat arrays, then the base
  HistStore N;
  CR(ctx->hist_grow_flat(N, tot));
  CR(ctx->h_bsum.ensure(ctx, 64, "history trim count"));
  unsigned long long* cnt = (unsigned long long*)ctx->h_bsum.p;
  CK(hipMemsetAsync(cnt, 0, 8, ctx->stream));
  launch_hist_trim((const uint64_t*)B.fk.p, (const uint64_t*)B.ft.p, B.m, (const uint64_t*)D.fk.p,
                   (const uint64_t*)D.ft.p, D.m, tn_floor, (uint64_t*)N.fk.p, (uint64_t*)N.ft.p, cnt,
                   ctx->stream);
  CK(hipGetLastError());
  CK(hipMemcpyAsync(ctx->hmisc, cnt, 8, hipMemcpyDeviceToHost, ctx->stream));
  CK(hipStreamSynchronize(ctx->stream));
  const uint64_t kept = *(const uint64_t*)ctx->hmisc;
  const uint64_t mx = std::max(B.max_tn, D.max_tn);
  B.fk.release();
  B.ft.release();
  B.fk = N.fk;
  B.ft = N.ft;
  N.fk = DevBuf{};
  N.ft = DevBuf{};
  B.m = kept;
  B.max_tn = mx;
  B.max_key = std::max(B.max_key, D.max_key);
  D.max_key = 0;
  B.mono = false;  // the compaction does not keep the order
  B.built = false;
  D.reset();
  ctx->buf_gen++;
  return DCC_OK;
}

extern "C" uint64_t dcc_occ_history_size(const dcc_ctx* ctx) {
  if (!ctx) return 0;
  if (ctx->multi) {
    uint64_t s = 0;
    for (int r = 0; r < dcc_multi_size(ctx); r++) s += dcc_multi_sub((dcc_ctx*)ctx, r)->hist_size();
    return s;
  }
  return ctx->hist_size();
}

extern "C" int dcc_occ_history_export(dcc_ctx* ctx, uint64_t* keys, uint64_t* tn, uint64_t cap,
                                      uint64_t* out_n) {
  if (!ctx || !out_n) return DCC_EINVAL;
  dcc_pipe_drain(ctx);
  if (ctx->multi) {
    const uint64_t total = dcc_occ_history_size(ctx);
    *out_n = total;
    if (!keys || !tn) return DCC_OK;
    if (cap < total) return DCC_ERANGE;
    uint64_t at = 0;
    for (int r = 0; r < dcc_multi_size(ctx); r++) {
      uint64_t m = 0;
      CR(dcc_occ_history_export(dcc_multi_sub(ctx, r), keys + at, tn + at, cap - at, &m));
      at += m;
    }
    return DCC_OK;
  }
  if (hipSetDevice(ctx->device) != hipSuccess) return DCC_ENODEV;
  const uint64_t n = ctx->hist_size();
  *out_n = n;
  if (!keys || !tn) return DCC_OK;  // size query
  if (cap < n) return DCC_ERANGE;
  uint64_t at = 0;
  for (HistStore& h : ctx->hs) {
    if (!h.m) continue;
    CK(hipMemcpy(keys + at, h.fk.p, h.m * 8, hipMemcpyDeviceToHost));
    CK(hipMemcpy(tn + at, h.ft.p, h.m * 8, hipMemcpyDeviceToHost));
    at += h.m;
  }
  return DCC_OK;
}

extern "C" int dcc_occ_set_tnc(dcc_ctx* ctx, uint64_t tnc) {
  if (!ctx) return DCC_EINVAL;
  dcc_pipe_drain(ctx);
  if (ctx->multi)
    for (int r = 0; r < dcc_multi_size(ctx); r++) dcc_multi_sub(ctx, r)->tnc = tnc;
  ctx->tnc = tnc;
  return DCC_OK;
}
extern "C" uint64_t dcc_occ_get_tnc(const dcc_ctx* ctx) {
  dcc_pipe_drain(const_cast<dcc_ctx*>(ctx));  // tnc counts the epochs in flight
  if (ctx && ctx->multi) return dcc_multi_sub((dcc_ctx*)ctx, 0)->tnc;
  return ctx ? ctx->tnc : 0;
}

// ---------------------------------------------------------------- batch checks
int dcc_ctx::check_batch(const dcc_batch* b, bool scan_offsets) {
  if (!b) return fail(DCC_EINVAL, "null batch");
  if (b->n_txn == 0) return DCC_OK;
  if (!b->offsets || (b->nnz && (!b->keys || !b->acctype)))
    return fail(DCC_EINVAL, "batch: null offsets/keys/acctype");
  if ((b->start_tn == nullptr) != (b->finish_tn == nullptr))
    return fail(DCC_EINVAL, "batch: start_tn and finish_tn must both be set or both NULL");
  if (b->n_txn > (uint64_t)IDX_MASK)
    return fail(DCC_ERANGE, "batch: n_txn %llu exceeds %u per epoch and shard",
                (unsigned long long)b->n_txn, IDX_MASK);
  if (b->nnz >= 0xFFFFFFFFull) return fail(DCC_ERANGE, "batch: nnz exceeds 2^32-1");
  if (!(b->flags & DCC_DEVICE_PTRS)) {
    // host batch: full structural validation before any launch
    const uint32_t* o = b->offsets;
    if (o[0] != 0 || o[b->n_txn] != b->nnz)
      return fail(DCC_EINVAL, "batch: offsets[0] must be 0 and offsets[n_txn] == nnz");
    for (uint64_t t = 0; scan_offsets && t < b->n_txn; t++) {
      if (o[t + 1] < o[t]) return fail(DCC_EINVAL, "batch: offsets decrease at txn %llu",
                                       (unsigned long long)t);
      if (o[t + 1] - o[t] > MAX_TXN_LEN)
        return fail(DCC_ERANGE, "batch: txn %llu has %u accesses (> MAX_ROW_PER_TXN=%u)",
                    (unsigned long long)t, o[t + 1] - o[t], MAX_TXN_LEN);
    }
  }
  return DCC_OK;
}

// Upload a host batch into ctx buffers (or alias a device batch); fills `d`.
// A host batch is copied to the context's device buffers (asynchronously on
// the engine stream: from pinned memory, dcc_host_alloc, at DMA speed); a
// device batch is read in place.  Compact forms (DCC_KEYS_U32,
// DCC_ACCTYPE_2BIT, DCC_TN_U32) move their narrow arrays and are widened on
// the device (k_widen) into the context's buffers, so every engine below sees
// u64 keys, byte access types and u64 timestamps.
int dcc_ctx::stage_batch(const dcc_batch* b, DevBatch& d) {
  dcc_ctx* ctx = this;
  d.n = b->n_txn;
  d.nnz = b->nnz;
  const bool dev = (b->flags & DCC_DEVICE_PTRS) != 0;
  const bool k32 = (b->flags & DCC_KEYS_U32) != 0, a2 = (b->flags & DCC_ACCTYPE_2BIT) != 0,
             t32 = (b->flags & DCC_TN_U32) != 0;
  if (dev && !k32 && !a2 && !t32) {
    d.off = b->offsets;
    d.keys = b->keys;
    d.acctype = b->acctype;
    d.start_tn = b->start_tn;
    d.finish_tn = b->finish_tn;
    d.order = b->order;
    return DCC_OK;
  }
  const hipMemcpyKind kind = dev ? hipMemcpyDeviceToDevice : hipMemcpyHostToDevice;
  WidenArgs w{};
  w.nnz = d.nnz;
  w.n = d.n;
  // offsets: never compact (read in place from a device batch)
  if (dev) {
    d.off = b->offsets;
  } else {
    CR(off.ensure(this, (d.n + 1) * 4, "offsets"));
    CK(hipMemcpyAsync(off.p, b->offsets, (d.n + 1) * 4, kind, stream));
    d.off = (const uint32_t*)off.p;
  }
  CR(keys.ensure(this, std::max<uint64_t>(8, d.nnz * 8), "keys"));
  CR(acctype.ensure(this, std::max<uint64_t>(16, d.nnz), "acctype"));
  d.keys = (const uint64_t*)keys.p;
  d.acctype = (const uint8_t*)acctype.p;
  if (d.nnz) {
    if (k32) {
      const void* src = b->keys;
      if (!dev) {
        CR(nar_keys.ensure(this, d.nnz * 4, "compact keys"));
        CK(hipMemcpyAsync(nar_keys.p, b->keys, d.nnz * 4, kind, stream));
        src = nar_keys.p;
      }
      w.k32 = (const uint32_t*)src;
      w.k64 = (uint64_t*)keys.p;
    } else if (dev) {
      d.keys = b->keys;
    } else {
      CK(hipMemcpyAsync(keys.p, b->keys, d.nnz * 8, kind, stream));
    }
    if (a2) {
      const uint64_t pb = (d.nnz + 3) / 4;
      const void* src = b->acctype;
      if (!dev) {
        CR(nar_at.ensure(this, pb + 16, "compact access types"));
        CK(hipMemcpyAsync(nar_at.p, b->acctype, pb, kind, stream));
        src = nar_at.p;
      }
      w.a2 = (const uint8_t*)src;
      w.a8 = (uint8_t*)acctype.p;
    } else if (dev) {
      d.acctype = b->acctype;
    } else {
      CK(hipMemcpyAsync(acctype.p, b->acctype, d.nnz, kind, stream));
    }
  }
  d.start_tn = d.finish_tn = nullptr;
  if (b->start_tn) {
    CR(start_tn.ensure(this, d.n * 8, "start_tn"));
    CR(finish_tn.ensure(this, d.n * 8, "finish_tn"));
    d.start_tn = (const uint64_t*)start_tn.p;
    d.finish_tn = (const uint64_t*)finish_tn.p;
    if (t32) {
      const void *s0 = b->start_tn, *f0 = b->finish_tn;
      if (!dev) {
        CR(nar_tn.ensure(this, d.n * 8 + 16, "compact timestamps"));
        CK(hipMemcpyAsync(nar_tn.p, b->start_tn, d.n * 4, kind, stream));
        CK(hipMemcpyAsync((char*)nar_tn.p + d.n * 4, b->finish_tn, d.n * 4, kind, stream));
        s0 = nar_tn.p;
        f0 = (const char*)nar_tn.p + d.n * 4;
      }
      w.s32 = (const uint32_t*)s0;
      w.f32 = (const uint32_t*)f0;
      w.s64 = (uint64_t*)start_tn.p;
      w.f64 = (uint64_t*)finish_tn.p;
    } else if (dev) {
      d.start_tn = b->start_tn;
      d.finish_tn = b->finish_tn;
    } else {
      CK(hipMemcpyAsync(start_tn.p, b->start_tn, d.n * 8, kind, stream));
      CK(hipMemcpyAsync(finish_tn.p, b->finish_tn, d.n * 8, kind, stream));
    }
  }
  d.order = nullptr;
  if (b->order) {
    if (dev) {
      d.order = b->order;
    } else {
      CR(order.ensure(this, d.n * 8, "order"));
      CK(hipMemcpyAsync(order.p, b->order, d.n * 8, kind, stream));
      d.order = (const uint64_t*)order.p;
    }
  }
  if (w.k32 || w.a2 || w.s32) {
    launch_widen(w, n_cu, stream);
    CK(hipGetLastError());
  }
  return DCC_OK;
}

extern "C" int dcc_copy_bandwidth(dcc_ctx* ctx, uint64_t bytes, int reps, double* gbps) {
  if (!ctx || !gbps || bytes < 16 || reps < 1) return DCC_EINVAL;
  if (ctx->multi) ctx = dcc_multi_sub(ctx, 0);
  if (hipSetDevice(ctx->device) != hipSuccess) return DCC_ENODEV;
  bytes &= ~15ull;
  DevBuf a, b;
  CR(a.ensure(ctx, bytes, "copy source"));
  CR(b.ensure(ctx, bytes, "copy destination"));
  CK(hipMemsetAsync(a.p, 1, bytes, ctx->stream));
  // the best of the copy forms (grid-stride at 8 workgroups per CU; one
  // contiguous range per workgroup, non-temporal, at 2 / 4 / 8 per CU), each
  // timed over `reps` launches after two warm-up launches
  float ms = 0;
  for (int v = 0; v < 4; v++) {
    const unsigned grid = (unsigned)ctx->n_cu * (v == 0 ? 8u : (1u << v));
    auto run = [&] {
      if (v == 0) launch_copy16(a.p, b.p, bytes, grid, ctx->stream);
      else launch_copy16_chunk(a.p, b.p, bytes, grid, ctx->stream);
    };
    for (int i = 0; i < 2; i++) run();
    CK(hipEventRecord(ctx->ev0, ctx->stream));
    for (int i = 0; i < reps; i++) run();
    CK(hipEventRecord(ctx->ev1, ctx->stream));
    CK(hipEventSynchronize(ctx->ev1));
    float m = 0;
    CK(hipEventElapsedTime(&m, ctx->ev0, ctx->ev1));
    if (v == 0 || m < ms) ms = m;
  }
  *gbps = 2.0 * (double)bytes * reps / (ms * 1e-3) / 1e9;
  return DCC_OK;
}

extern "C" int dcc_host_alloc(dcc_ctx* ctx, uint64_t bytes, void** out) {
  if (!ctx || !out) return DCC_EINVAL;
  *out = nullptr;
  if (!bytes) return DCC_OK;
  const hipError_t e = hipHostMalloc(out, bytes, hipHostMallocDefault);
  if (e != hipSuccess) {
    *out = nullptr;
    return ctx->fail(DCC_ENOMEM, "hipHostMalloc(%llu): %s", (unsigned long long)bytes, hipGetErrorString(e));
  }
  return DCC_OK;
}

// ctx may be NULL (memory outliving its context)
extern "C" int dcc_host_free(dcc_ctx* ctx, void* p) {
  if (p && hipHostFree(p) != hipSuccess)
    return ctx ? ctx->fail(DCC_EINVAL, "dcc_host_free: not a dcc_host_alloc pointer") : DCC_EINVAL;
  return DCC_OK;
}

extern "C" int dcc_occ_validate_epoch(dcc_ctx* ctx, const dcc_batch* batch, uint8_t* out_rc,
                                      uint64_t* out_commit_tn, dcc_stats* out_stats) {
  if (!ctx) return DCC_EINVAL;
  dcc_pipe_drain(ctx);  // submit order
  if (ctx->multi) return dcc_multi_occ_epoch(ctx, batch, out_rc, out_commit_tn, out_stats);
  if (hipSetDevice(ctx->device) != hipSuccess) return DCC_ENODEV;
  return ctx->occ_epoch(batch, out_rc, out_commit_tn, out_stats);
}

extern "C" int dcc_occ_finish_epoch(dcc_ctx* ctx, const uint8_t* final_rc, uint64_t* out_commit_tn,
                                    uint32_t flags) {
  if (!ctx) return DCC_EINVAL;
  dcc_pipe_drain(ctx);
  if (ctx->multi) {
    // every shard appends its own keys' writes; tn numbering is alike on all.
    // Every rank is checked first (allocations, the votes): a failure there
    // leaves every rank's epoch pending, so the call can be repeated.  Only
    // the history appends follow (an allocation failure there leaves the
    // shards disagreeing: the context must then be re-created).
    const int R = dcc_multi_size(ctx);
    std::vector<uint32_t> n_cw(R, 0);
    for (int pass = 0; pass < 2; pass++)
      for (int r = 0; r < R; r++) {
        dcc_ctx* s = dcc_multi_sub(ctx, r);
        if (hipSetDevice(s->device) != hipSuccess) return DCC_ENODEV;
        const int e = pass == 0 ? s->occ_finish_prepare(final_rc, flags, n_cw[r])
                                : s->occ_finish_commit(n_cw[r], r == 0 ? out_commit_tn : nullptr, flags);
        if (e != DCC_OK) {
          ctx->last_error = "rank " + std::to_string(r) + ": " + s->last_error;
          return e;
        }
      }
    return DCC_OK;
  }
  if (hipSetDevice(ctx->device) != hipSuccess) return DCC_ENODEV;
  return ctx->occ_finish(final_rc, out_commit_tn, flags);
}
