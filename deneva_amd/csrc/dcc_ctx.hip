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
  CK(hipHostMalloc((void**)&ctx->hmisc, 4096, hipHostMallocDefault));
  int rc = ctx->misc.ensure(ctx, 4096, "misc");
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
  dcc_comm_destroy(ctx);
  for (DevBuf* b : ctx->all_bufs()) b->release();
  if (ctx->hmisc) (void)hipHostFree(ctx->hmisc);
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

extern "C" int dcc_set_stream(dcc_ctx* ctx, void* s) {
  if (!ctx) return DCC_EINVAL;
  ctx->stream = s ? (hipStream_t)s : ctx->own_stream;
  return DCC_OK;
}

std::vector<DevBuf*> dcc_ctx::all_bufs() {
  std::vector<DevBuf*> v = {&misc, &off, &keys, &acctype, &start_tn, &finish_tn, &table, &state,
                            &hasw, &cflag, &bsum, &tn, &rc, &hkeys, &hoff, &htn, &stat,
                            &order, &perm, &calvin_a, &calvin_b, &calvin_c, &calvin_d};
  for (int i = 0; i < 2; i++) {
    v.push_back(&l_tid[i]);
    v.push_back(&l_coff[i]);
    v.push_back(&l_cent[i]);
  }
  return v;
}

int dcc_ctx::reserve_occ(uint64_t n, uint64_t nnz, uint64_t nnz_w) {
  dcc_ctx* ctx = this;
  CR(state.ensure(this, n, "state"));
  CR(hasw.ensure(this, n, "hasw"));
  CR(rc.ensure(this, n, "rc"));
  CR(stat.ensure(this, n, "stat"));
  for (int i = 0; i < 2; i++) {
    CR(l_tid[i].ensure(this, n * 4 + 64, "list tid"));
    CR(l_coff[i].ensure(this, n * 4 + 64, "list off"));
    CR(l_cent[i].ensure(this, nnz * 4 + 64, "list entries"));
  }
  const uint64_t cap = table_capacity(nnz_w);
  CR(table.ensure(this, cap * sizeof(Slot), "table"));
  (void)ctx;
  return DCC_OK;
}

uint64_t dcc_ctx::table_capacity(uint64_t nnz_w) {
  // load factor <= 0.8 even if every write key is distinct
  return std::max<uint64_t>(1024, next_pow2(nnz_w + nnz_w / 4 + 1));
}

extern "C" int dcc_reserve(dcc_ctx* ctx, uint64_t max_txn, uint64_t max_nnz) {
  if (!ctx) return DCC_EINVAL;
  (void)hipSetDevice(ctx->device);
  return ctx->reserve_occ(max_txn, max_nnz, max_nnz);
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

// Offsets check + max length + write count on the device (one sync).
int dcc_ctx::device_prep(const DevBatch& d, uint32_t& maxlen, uint64_t& nnz_w) {
  dcc_ctx* ctx = this;
  uint32_t* info = (uint32_t*)misc.p;  // [0] err [1] maxlen; [2..3] nnz_w (u64)
  CK(hipMemsetAsync(misc.p, 0, 64, stream));
  launch_prep(d.off, d.n, d.nnz, info, stream);
  if (d.nnz) launch_count_writes(d.acctype, d.nnz, (unsigned long long*)(info + 2), stream);
  CK(hipGetLastError());
  CK(hipMemcpyAsync(hmisc, misc.p, 64, hipMemcpyDeviceToHost, stream));
  CK(hipStreamSynchronize(stream));
  const uint32_t* h = (const uint32_t*)hmisc;
  if (h[0] & ERR_OFFSETS) return fail(DCC_EINVAL, "batch: malformed offsets");
  maxlen = h[1];
  nnz_w = *(const uint64_t*)(h + 2);
  if (maxlen > MAX_TXN_LEN)
    return fail(DCC_ERANGE, "batch: a txn has %u accesses (> MAX_ROW_PER_TXN=%u)", maxlen,
                MAX_TXN_LEN);
  return DCC_OK;
}

// ---------------------------------------------------------------- OCC epoch
int dcc_ctx::occ_epoch(const dcc_batch* b, uint8_t* out_rc, uint64_t* out_tn, dcc_stats* st) {
  dcc_ctx* ctx = this;
  const auto t_wall0 = std::chrono::steady_clock::now();
  CR(check_batch(b));
  const bool dev_out = (b->flags & DCC_DEVICE_PTRS) != 0;
  dcc_stats S;
  memset(&S, 0, sizeof S);
  S.n_shards = comm_ranks();
  if (b->n_txn == 0) {
    if (st) *st = S;
    return DCC_OK;
  }
  DevBatch d;
  CR(stage_batch(b, d));
  CK(hipEventRecord(ev0, stream));  // device clock starts with the batch resident
  uint32_t maxlen = 0;
  uint64_t nnz_w = 0;
  CR(device_prep(d, maxlen, nnz_w));
  CR(reserve_occ(d.n, d.nnz, nnz_w));
  const uint64_t cap = table_capacity(nnz_w);
  const uint32_t mask = (uint32_t)(cap - 1);
  if (cap > (1ull << 30)) return fail(DCC_ERANGE, "table capacity exceeds 2^30 slots");
  const uint32_t tw = std::min<uint32_t>(64, TILE_CAP / std::max<uint32_t>(1, maxlen));
  Slot* tab = (Slot*)table.p;
  uint32_t* err = (uint32_t*)misc.p + 16;
  unsigned long long* ctr = (unsigned long long*)((uint32_t*)misc.p + 32);
  uint64_t* counts = (uint64_t*)((uint32_t*)misc.p + 64);
  uint64_t* d_nnzw = (uint64_t*)((uint32_t*)misc.p + 96);

  CK(hipMemsetAsync(misc.p, 0, 1024, stream));
  CK(hipMemsetAsync(table.p, 0xFF, cap * sizeof(Slot), stream));
  CK(hipMemsetAsync(state.p, 0, d.n, stream));

  // history window pre-pass (occ.cpp:160-180)
  const bool use_hist = d.start_tn && !hist.empty();
  if (use_hist) {
    CR(upload_history());
    HistArgs ha{d.n, d.off, d.keys, d.acctype, d.start_tn, d.finish_tn,
                (const uint64_t*)hkeys.p, h_nkeys, (const uint64_t*)hoff.p,
                (const uint64_t*)htn.p, (uint8_t*)state.p};
    launch_hist(ha, stream);
  }

  BuildArgs ba{d.n, tw, d.off, d.keys, d.acctype, tab, mask, (const uint8_t*)state.p,
               (uint8_t*)hasw.p, d_nnzw, err};
  if (profiling) CK(hipEventRecord(pev[0], stream));
  launch_build(ba, stream);
  CK(hipGetLastError());
  if (profiling) CK(hipEventRecord(pev[1], stream));
  double ph_rest = 0;

  // ---- fixed-point rounds
  uint64_t m = d.n;
  uint32_t end_total = (uint32_t)d.nnz;
  int cur = 0;
  uint32_t rt = 1;  // round tag
  uint32_t rounds = 0;
  for (;;) {
    const bool first = rounds == 0;
    if (rt > MAX_ROUND_TAG) {
      // tag space exhausted: drop stale owner words, republish from the list
      launch_retag(tab, cap, stream);
      OwnerArgs oa{m, 1, end_total, (const uint32_t*)l_tid[cur].p,
                   (const uint32_t*)l_coff[cur].p, (const uint32_t*)l_cent[cur].p, tab};
      launch_owner_list(oa, stream);
      rt = 1;
    }
    CK(hipMemsetAsync(ctr, 0, 8, stream));
    RoundArgs ra;
    ra.m = m;
    ra.tw = tw;
    ra.r = rt;
    ra.end_total = end_total;
    ra.tid = first ? nullptr : (const uint32_t*)l_tid[cur].p;
    ra.coff = first ? d.off : (const uint32_t*)l_coff[cur].p;
    ra.keys = d.keys;
    ra.acctype = d.acctype;
    ra.cent = first ? nullptr : (const uint32_t*)l_cent[cur].p;
    ra.tab = tab;
    ra.mask = mask;
    ra.state = (uint8_t*)state.p;
    ra.tid_out = (uint32_t*)l_tid[cur ^ 1].p;
    ra.coff_out = (uint32_t*)l_coff[cur ^ 1].p;
    ra.cent_out = (uint32_t*)l_cent[cur ^ 1].p;
    ra.ctr = ctr;
    ra.err = err;
    if (profiling && !first) CK(hipEventRecord(pev[3], stream));
    launch_round(ra, first, stream);
    CK(hipGetLastError());
    if (profiling) CK(hipEventRecord(first ? pev[2] : pev[4], stream));
    rounds++;
    CK(hipMemcpyAsync(hmisc, ctr, 8, hipMemcpyDeviceToHost, stream));
    CK(hipStreamSynchronize(stream));
    if (profiling && !first) {
      float t = 0;
      CK(hipEventElapsedTime(&t, pev[3], pev[4]));
      ph_rest += t;
    }
    const unsigned long long c = *(const unsigned long long*)hmisc;
    m = c >> CTR_E_BITS;
    end_total = (uint32_t)(c & CTR_E_MASK);
    cur ^= 1;
    rt++;
    if (m == 0) break;
    if (rounds > d.n + 2) return fail(DCC_EIO, "fixed point did not converge");
  }

  // ---- finalize
  uint8_t* rc_dev = (dev_out && out_rc) ? out_rc : (uint8_t*)rc.p;
  uint32_t* cf = nullptr;
  const bool want_tn = out_tn != nullptr || (b->flags & DCC_OCC_APPEND_HISTORY);
  if (want_tn) {
    CR(cflag.ensure(this, d.n * 4, "cflag"));
    CR(bsum.ensure(this, ((d.n + 1023) / 1024 + 1) * 8, "bsum"));
    CR(tn.ensure(this, d.n * 8, "tn"));
    cf = (uint32_t*)cflag.p;
  }
  FinalArgs fa{d.n, (const uint8_t*)state.p, (const uint8_t*)hasw.p, rc_dev, cf, counts, err};
  launch_final(fa, stream);
  uint64_t* tn_dev = nullptr;
  if (want_tn) {
    tn_dev = (dev_out && out_tn) ? out_tn : (uint64_t*)tn.p;
    launch_commit_tn(cf, d.n, (uint64_t*)bsum.p, tnc, tn_dev, stream);
  }
  CK(hipGetLastError());
  CK(hipEventRecord(ev1, stream));
  if (!dev_out) {
    if (out_rc) CK(hipMemcpyAsync(out_rc, rc.p, d.n, hipMemcpyDeviceToHost, stream));
    if (out_tn) CK(hipMemcpyAsync(out_tn, tn.p, d.n * 8, hipMemcpyDeviceToHost, stream));
  }
  CK(hipMemcpyAsync(hmisc, misc.p, 1024, hipMemcpyDeviceToHost, stream));
  CK(hipStreamSynchronize(stream));
  const uint32_t* hm = (const uint32_t*)hmisc;
  const uint32_t e = hm[16];
  if (e & ERR_KEY) return fail(DCC_EINVAL, "batch: key equal to DCC_KEY_RESERVED");
  if (e & ERR_FULL) return fail(DCC_EIO, "hash table overflow");
  if (e & ERR_TILE) return fail(DCC_EIO, "tile capacity exceeded");
  if (e & ERR_UNDECIDED) return fail(DCC_EIO, "undecided transaction after convergence");
  const uint64_t* hc = (const uint64_t*)(hm + 64);
  float ms = 0;
  CK(hipEventElapsedTime(&ms, ev0, ev1));
  S.rounds = rounds;
  S.n_commit = hc[0];
  S.n_abort = hc[1];
  S.n_readonly = hc[2];
  S.nnz_w = *(const uint64_t*)(hm + 96);
  S.alg_bytes = dcc_alg_bytes(d.n, d.nnz, S.nnz_w);
  S.device_ms = ms;
  if (profiling) {
    float t0 = 0, t1 = 0;
    CK(hipEventElapsedTime(&t0, pev[0], pev[1]));
    CK(hipEventElapsedTime(&t1, pev[1], pev[2]));
    S.phase_ms[0] = t0;
    S.phase_ms[1] = t1;
    S.phase_ms[2] = ph_rest;
    S.phase_ms[3] = ms - t0 - t1 - ph_rest;
  }
  // algorithmic bytes per phase: build reads acctype for all
  // accesses and keys of writes, one 16-B slot update per write; round 1
  // reads offsets, keys+acctype, one 16-B slot per access, state byte.
  S.phase_bytes[0] = d.nnz + 8 * S.nnz_w + 16 * S.nnz_w + 4 * (d.n + 1) + d.n;
  S.phase_bytes[1] = 4 * (d.n + 1) + 9 * d.nnz + 16 * d.nnz + d.n;

  // central_finish (occ.cpp:283-286): committed non-read-only txns take
  // tn = tnc+1, tnc+2, ... in index order; their write sets join the history.
  const uint64_t n_cw = hc[3];
  if (b->flags & DCC_OCC_APPEND_HISTORY) {
    std::vector<uint64_t> htn_host(d.n);
    CK(hipMemcpy(htn_host.data(), tn_dev, d.n * 8, hipMemcpyDeviceToHost));
    std::vector<uint32_t> ho;
    std::vector<uint64_t> hk;
    std::vector<uint8_t> ha;
    const uint32_t* o = b->offsets;
    const uint64_t* k = b->keys;
    const uint8_t* at = b->acctype;
    if (dev_out) {
      ho.resize(d.n + 1);
      hk.resize(d.nnz);
      ha.resize(d.nnz);
      CK(hipMemcpy(ho.data(), d.off, (d.n + 1) * 4, hipMemcpyDeviceToHost));
      if (d.nnz) {
        CK(hipMemcpy(hk.data(), d.keys, d.nnz * 8, hipMemcpyDeviceToHost));
        CK(hipMemcpy(ha.data(), d.acctype, d.nnz, hipMemcpyDeviceToHost));
      }
      o = ho.data();
      k = hk.data();
      at = ha.data();
    }
    for (uint64_t t = 0; t < d.n; t++) {
      if (!htn_host[t]) continue;
      for (uint32_t x = o[t]; x < o[t + 1]; x++)
        if (at[x] == DCC_WR) hist.emplace_back(k[x], htn_host[t]);
    }
    if (n_cw) hist_dirty = true;
  }
  tnc += n_cw;
  const auto t_wall1 = std::chrono::steady_clock::now();
  S.total_ms = std::chrono::duration<double, std::milli>(t_wall1 - t_wall0).count();
  if (st) *st = S;
  return DCC_OK;
}

extern "C" int dcc_occ_validate_epoch(dcc_ctx* ctx, const dcc_batch* batch, uint8_t* out_rc,
                                      uint64_t* out_commit_tn, dcc_stats* out_stats) {
  if (!ctx) return DCC_EINVAL;
  if (hipSetDevice(ctx->device) != hipSuccess) return DCC_ENODEV;
  if (ctx->comm_ranks() > 1) return ctx->occ_epoch_sharded(batch, out_rc, out_commit_tn, out_stats);
  return ctx->occ_epoch(batch, out_rc, out_commit_tn, out_stats);
}
