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
  CK(hipHostMalloc((void**)&ctx->hpart, 1 << 16, hipHostMallocDefault));
  CK(hipHostGetDevicePointer(&ctx->hmisc_dev, ctx->hmisc, 0));
  CK(hipHostGetDevicePointer(&ctx->hpart_dev, ctx->hpart, 0));
  CK(hipHostMalloc((void**)&ctx->st_host, 8192, hipHostMallocDefault));
  CK(hipHostGetDevicePointer(&ctx->st_host_dev, ctx->st_host, 0));
  int rc = ctx->misc.ensure(ctx, 16384, "misc");
  if (!rc) rc = ctx->part.ensure(ctx, 1 << 16, "partials");
  if (rc) {
    dcc_destroy(ctx);
    return rc;
  }
  *out = ctx;
  return DCC_OK;
}

extern "C" void dcc_destroy(dcc_ctx* ctx) {
  if (!ctx) return;
  (void)hipSetDevice(ctx->device);
  if (ctx->stream) (void)hipStreamSynchronize(ctx->stream);
  if (ctx->graph_exec) (void)hipGraphExecDestroy(ctx->graph_exec);
  dcc_comm_destroy(ctx);
  for (DevBuf* b : ctx->all_bufs()) b->release();
  if (ctx->hmisc) (void)hipHostFree(ctx->hmisc);
  if (ctx->hpart) (void)hipHostFree(ctx->hpart);
  if (ctx->st_host) (void)hipHostFree(ctx->st_host);
  if (ctx->st_graph) (void)hipGraphExecDestroy(ctx->st_graph);
  if (ctx->ev0) (void)hipEventDestroy(ctx->ev0);
  if (ctx->ev1) (void)hipEventDestroy(ctx->ev1);
  for (auto& e : ctx->pev)
    if (e) (void)hipEventDestroy(e);
  if (ctx->own_stream) (void)hipStreamDestroy(ctx->own_stream);
  delete ctx;
}

extern "C" int dcc_set_profiling(dcc_ctx* ctx, int enable) {
  if (!ctx) return DCC_EINVAL;
  ctx->profiling = enable != 0;
  return DCC_OK;
}

extern "C" int dcc_set_option(dcc_ctx* ctx, int option, int64_t value) {
  if (!ctx) return DCC_EINVAL;
  switch (option) {
    case DCC_OPT_RECHECK:
      if (value < 0) return DCC_EINVAL;
      ctx->recheck_max = (uint64_t)value;
      return DCC_OK;
    case DCC_OPT_PEEL:
      if (value < -1) return DCC_EINVAL;
      ctx->peel_mode = value;
      return DCC_OK;
    case DCC_OPT_PEEL_MIN:
      if (value < 2) return DCC_EINVAL;
      ctx->peel_min = (uint64_t)value;
      return DCC_OK;
    case DCC_OPT_SOLVER:
      if (value < 0 || value > 4) return DCC_EINVAL;
      ctx->solver = (int)value;
      return DCC_OK;
    case DCC_OPT_SWEEP_LEVELS:
      if (value < 1 || value > SW_MAX_LEVEL) return DCC_EINVAL;
      ctx->sw_levels = (uint32_t)value;
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
  ctx->stream = s ? (hipStream_t)s : ctx->own_stream;
  return DCC_OK;
}

std::vector<DevBuf*> dcc_ctx::all_bufs() {
  std::vector<DevBuf*> v = {&misc, &part, &off, &keys, &acctype, &start_tn, &finish_tn, &table, &state,
                            &hasw, &cflag, &bsum, &tn, &rc, &hkeys, &hoff, &htn, &stat,
                            &order, &perm, &calvin_a, &calvin_b, &calvin_c, &calvin_d,
                            &cv_scratch, &cv_agg, &cv_group, &cv_wave, &cv_pgx, &cv_gsx,
                            &cv_gsize, &cv_done, &cv_maxl, &cv_seq_b, &cv_ok, &cv_len,
                            &cv_off2, &cv_tsum, &gst, &hasw_scr, &cset_tab, &cset_keys,
                            &a_cnt, &a_writers, &a_big, &a_st32, &sw_ctl, &sw_status, &sw_dbg,
                            &sw_ckeys, &sw_gtab, &sw_rec, &sw_rk, &sw_fw, &sw_aent, &sw_mg, &sw_xcnt,
                            &sw_xrec, &sw_mcnt, &sw_moff, &sw_mkeys, &sw_mat, &sw_kill,
                            &snap_top, &snap_aoff, &snap_aidx, &snap_cnt, &hhash};
  for (auto& sb : sw_list)
    for (DevBuf* b : {&sb.tid, &sb.off, &sb.keys, &sb.acctype, &sb.state}) v.push_back(b);
  v.push_back(&st_ctl);
  for (int i = 0; i < 2; i++)
    for (DevBuf* b : {&st_tid[i], &st_ast[i], &st_alen[i], &st_keys[i], &st_at[i], &st_hdr[i], &st_ck[i],
                      &st_hsh[i], &st_dep[i], &st_tile[i]})
      v.push_back(b);
  for (auto& sb : subs)
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
  (void)hipSetDevice(ctx->device);
  const uint32_t tw = ROUND_CAP / MAX_TXN_LEN;  // worst case: MAX_ROW_PER_TXN-long txns
  int rc = ctx->state.ensure(ctx, max_txn + 16, "state");
  if (!rc) rc = ctx->hasw.ensure(ctx, max_txn + 16, "hasw");
  if (!rc) rc = ctx->rc.ensure(ctx, max_txn + 16, "rc");
  if (rc) return rc;
  return ctx->reserve_occ(max_txn, max_nnz, max_nnz, tw);
}

// ---------------------------------------------------------------- history
extern "C" int dcc_occ_history_append(dcc_ctx* ctx, const uint64_t* keys, const uint64_t* tn,
                                      uint64_t n) {
  if (!ctx || (n && (!keys || !tn))) return DCC_EINVAL;
  ctx->hist.reserve(ctx->hist.size() + n);
  for (uint64_t i = 0; i < n; i++) ctx->hist.emplace_back(keys[i], tn[i]);
  if (n) ctx->hist_dirty = true;
  return DCC_OK;
}

extern "C" int dcc_occ_history_clear(dcc_ctx* ctx) {
  if (!ctx) return DCC_EINVAL;
  ctx->hist.clear();
  ctx->hist_dirty = true;
  return DCC_OK;
}

extern "C" uint64_t dcc_occ_history_size(const dcc_ctx* ctx) { return ctx ? ctx->hist.size() : 0; }
extern "C" int dcc_occ_set_tnc(dcc_ctx* ctx, uint64_t tnc) {
  if (!ctx) return DCC_EINVAL;
  ctx->tnc = tnc;
  return DCC_OK;
}
extern "C" uint64_t dcc_occ_get_tnc(const dcc_ctx* ctx) { return ctx ? ctx->tnc : 0; }

int dcc_ctx::upload_history() {
  dcc_ctx* ctx = this;
  if (!hist_dirty) return DCC_OK;
  std::sort(hist.begin(), hist.end());
  std::vector<uint64_t> hk, ho, ht;
  ht.reserve(hist.size());
  for (size_t i = 0; i < hist.size(); i++) {
    if (i == 0 || hist[i].first != hist[i - 1].first) {
      hk.push_back(hist[i].first);
      ho.push_back(ht.size());
    }
    ht.push_back(hist[i].second);
  }
  ho.push_back(ht.size());
  h_nkeys = hk.size();
  CR(hkeys.ensure(this, std::max<size_t>(8, hk.size() * 8), "hist keys"));
  CR(hoff.ensure(this, ho.size() * 8, "hist off"));
  CR(htn.ensure(this, std::max<size_t>(8, ht.size() * 8), "hist tn"));
  if (!hk.empty()) CK(hipMemcpy(hkeys.p, hk.data(), hk.size() * 8, hipMemcpyHostToDevice));
  CK(hipMemcpy(hoff.p, ho.data(), ho.size() * 8, hipMemcpyHostToDevice));
  if (!ht.empty()) CK(hipMemcpy(htn.p, ht.data(), ht.size() * 8, hipMemcpyHostToDevice));
  // key -> CSR row as an open-addressing table at <= 50% load (one probe of
  // 16 B instead of a log2(keys)-deep binary search; snapshot validation)
  h_hbits = 4;
  while ((1ull << h_hbits) < 2 * hk.size()) h_hbits++;
  std::vector<uint64_t> tab(2ull << h_hbits, DCC_KEY_RESERVED);
  const uint64_t mask = (1ull << h_hbits) - 1;
  for (size_t u = 0; u < hk.size(); u++) {
    uint64_t slot = hist_hash_slot(hk[u], h_hbits);
    while (tab[2 * slot] != DCC_KEY_RESERVED) slot = (slot + 1) & mask;
    tab[2 * slot] = hk[u];
    tab[2 * slot + 1] = u;
  }
  CR(hhash.ensure(this, tab.size() * 8, "hist hash"));
  CK(hipMemcpy(hhash.p, tab.data(), tab.size() * 8, hipMemcpyHostToDevice));
  hist_dirty = false;
  return DCC_OK;
}

// ---------------------------------------------------------------- batch checks
int dcc_ctx::check_batch(const dcc_batch* b) {
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
    for (uint64_t t = 0; t < b->n_txn; t++) {
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
int dcc_ctx::stage_batch(const dcc_batch* b, DevBatch& d) {
  dcc_ctx* ctx = this;
  d.n = b->n_txn;
  d.nnz = b->nnz;
  if (b->flags & DCC_DEVICE_PTRS) {
    d.off = b->offsets;
    d.keys = b->keys;
    d.acctype = b->acctype;
    d.start_tn = b->start_tn;
    d.finish_tn = b->finish_tn;
    d.order = b->order;
    return DCC_OK;
  }
  CR(off.ensure(this, (d.n + 1) * 4, "offsets"));
  CR(keys.ensure(this, std::max<uint64_t>(8, d.nnz * 8), "keys"));
  CR(acctype.ensure(this, std::max<uint64_t>(16, d.nnz), "acctype"));
  CK(hipMemcpyAsync(off.p, b->offsets, (d.n + 1) * 4, hipMemcpyHostToDevice, stream));
  if (d.nnz) {
    CK(hipMemcpyAsync(keys.p, b->keys, d.nnz * 8, hipMemcpyHostToDevice, stream));
    CK(hipMemcpyAsync(acctype.p, b->acctype, d.nnz, hipMemcpyHostToDevice, stream));
  }
  d.off = (const uint32_t*)off.p;
  d.keys = (const uint64_t*)keys.p;
  d.acctype = (const uint8_t*)acctype.p;
  d.start_tn = d.finish_tn = nullptr;
  if (b->start_tn) {
    CR(start_tn.ensure(this, d.n * 8, "start_tn"));
    CR(finish_tn.ensure(this, d.n * 8, "finish_tn"));
    CK(hipMemcpyAsync(start_tn.p, b->start_tn, d.n * 8, hipMemcpyHostToDevice, stream));
    CK(hipMemcpyAsync(finish_tn.p, b->finish_tn, d.n * 8, hipMemcpyHostToDevice, stream));
    d.start_tn = (const uint64_t*)start_tn.p;
    d.finish_tn = (const uint64_t*)finish_tn.p;
  }
  d.order = nullptr;
  if (b->order) {
    CR(order.ensure(this, d.n * 8, "order"));
    CK(hipMemcpyAsync(order.p, b->order, d.n * 8, hipMemcpyHostToDevice, stream));
    d.order = (const uint64_t*)order.p;
  }
  return DCC_OK;
}

extern "C" int dcc_occ_validate_epoch(dcc_ctx* ctx, const dcc_batch* batch, uint8_t* out_rc,
                                      uint64_t* out_commit_tn, dcc_stats* out_stats) {
  if (!ctx) return DCC_EINVAL;
  if (hipSetDevice(ctx->device) != hipSuccess) return DCC_ENODEV;
  return ctx->occ_epoch(batch, out_rc, out_commit_tn, out_stats);
}
