/* stub_engine.c — TEST INFRASTRUCTURE: a host-only stand-in for the libdcc
 * calls the OccEpoch shim makes (dcc_occ_validate_epoch, dcc_occ_get_tnc),
 * deciding each epoch with the oracle's serial hash-set scan.  It lets the
 * shim's mutex / condition-variable epoch map run under ThreadSanitizer and
 * AddressSanitizer on a machine without a GPU.  Never part of libdcc. */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include "dcc.h"
#include "oracle.h"

struct dcc_ctx {
  uint64_t tnc;
};
static struct dcc_ctx g_ctx;

dcc_ctx* stub_ctx(void) { return &g_ctx; }

uint64_t dcc_occ_get_tnc(const dcc_ctx* ctx) { return ctx ? ctx->tnc : 0; }

int dcc_occ_validate_epoch(dcc_ctx* ctx, const dcc_batch* b, uint8_t* out_rc,
                           uint64_t* out_commit_tn, dcc_stats* st) {
  if (!ctx || !b || !out_rc) return DCC_EINVAL;
  /* the shim keeps one engine call in flight (a context is thread-compatible) */
  static int inflight;
  if (__atomic_fetch_add(&inflight, 1, __ATOMIC_ACQ_REL) != 0) {
    __atomic_fetch_sub(&inflight, 1, __ATOMIC_ACQ_REL);
    return DCC_EIO;
  }
  /* a device call's latency, so workers fill the next epoch meanwhile */
  const struct timespec ts = {0, 100000};
  nanosleep(&ts, NULL);
  uint64_t tn_scratch[1];
  uint64_t* tn = out_commit_tn;
  uint64_t n = b->n_txn;
  if (!tn) {
    /* the shim never asks for tns: decide into a small stack buffer in chunks
     * is not possible (serial order), so use the out array of rc as a guard */
    static __thread uint64_t buf[1 << 16];
    if (n > (1 << 16)) {
      __atomic_fetch_sub(&inflight, 1, __ATOMIC_ACQ_REL);
      return DCC_ERANGE;
    }
    tn = buf;
  }
  (void)tn_scratch;
  /* the shim hands the engine its compact transfer form (dcc.h): widen it */
  const uint64_t nnz = b->nnz;
  uint64_t* keys = (uint64_t*)malloc((nnz + 1) * 8);
  uint8_t* at = (uint8_t*)malloc(nnz + 1);
  uint64_t* s_tn = b->start_tn ? (uint64_t*)malloc((n + 1) * 8) : NULL;
  uint64_t* f_tn = b->start_tn ? (uint64_t*)malloc((n + 1) * 8) : NULL;
  for (uint64_t x = 0; x < nnz; x++) {
    keys[x] = (b->flags & DCC_KEYS_U32) ? ((const uint32_t*)(const void*)b->keys)[x] : b->keys[x];
    at[x] = (b->flags & DCC_ACCTYPE_2BIT) ? (uint8_t)((b->acctype[x >> 2] >> (2 * (x & 3))) & 3u)
                                          : b->acctype[x];
  }
  for (uint64_t t = 0; s_tn && t < n; t++) {
    s_tn[t] = (b->flags & DCC_TN_U32) ? ((const uint32_t*)(const void*)b->start_tn)[t] : b->start_tn[t];
    f_tn[t] = (b->flags & DCC_TN_U32) ? ((const uint32_t*)(const void*)b->finish_tn)[t] : b->finish_tn[t];
  }
  int r = oracle_occ_hash(n, b->offsets, keys, at, s_tn, f_tn, 0, NULL, NULL, &ctx->tnc, out_rc, tn);
  free(keys);
  free(at);
  free(s_tn);
  free(f_tn);
  if (st) memset(st, 0, sizeof *st);
  __atomic_fetch_sub(&inflight, 1, __ATOMIC_ACQ_REL);
  return r ? DCC_EIO : DCC_OK;
}

/* pinned host memory (dcc_host_alloc): plain malloc in the stub */
int dcc_host_alloc(dcc_ctx* ctx, uint64_t bytes, void** out) {
  (void)ctx;
  if (!out) return DCC_EINVAL;
  *out = bytes ? malloc(bytes) : NULL;
  return (bytes && !*out) ? DCC_ENOMEM : DCC_OK;
}
int dcc_host_free(dcc_ctx* ctx, void* p) {
  (void)ctx;
  free(p);
  return DCC_OK;
}

/* The pipeline entry points (dcc_occ_submit_epoch / dcc_occ_wait_epoch):
 * submit only records the epoch -- the shim must leave its arrays and the
 * decision buffer alone until the wait -- and a wait decides every recorded
 * epoch up to its ticket, in submit order (tnc advances in that order). */
#define STUB_RING 64
static struct {
  dcc_batch b;
  uint8_t* rc;
  int done, err;
} g_pend[STUB_RING];
static uint64_t g_next = 1, g_decided = 0;

int dcc_set_option(dcc_ctx* ctx, int option, int64_t value) {
  (void)option;
  (void)value;
  return ctx ? DCC_OK : DCC_EINVAL;
}

int dcc_occ_submit_epoch(dcc_ctx* ctx, const dcc_batch* b, uint8_t* out_rc, uint64_t* out_tn,
                         uint64_t* out_ticket) {
  if (!ctx || !b || !out_ticket || out_tn) return DCC_EINVAL;
  if (g_next - g_decided > STUB_RING) return DCC_ERANGE;
  const uint64_t t = g_next++;
  g_pend[t % STUB_RING].b = *b;
  g_pend[t % STUB_RING].rc = out_rc;
  g_pend[t % STUB_RING].done = 0;
  *out_ticket = t;
  return DCC_OK;
}

int dcc_occ_wait_epoch(dcc_ctx* ctx, uint64_t ticket, dcc_stats* st) {
  if (!ctx || ticket == 0 || ticket >= g_next) return DCC_EINVAL;
  while (g_decided < ticket) {
    const uint64_t t = ++g_decided;
    g_pend[t % STUB_RING].err = dcc_occ_validate_epoch(ctx, &g_pend[t % STUB_RING].b, g_pend[t % STUB_RING].rc,
                                                       NULL, NULL);
    g_pend[t % STUB_RING].done = 1;
  }
  if (!g_pend[ticket % STUB_RING].done) return DCC_EINVAL;
  g_pend[ticket % STUB_RING].done = 0;
  if (st) memset(st, 0, sizeof *st);
  return g_pend[ticket % STUB_RING].err;
}
