/* stub_engine.c — TEST INFRASTRUCTURE: a host-only stand-in for the libdcc
 * calls the OccEpoch shim makes (dcc_occ_validate_epoch, dcc_occ_get_tnc),
 * deciding each epoch with the oracle's serial hash-set scan.  It lets the
 * shim's mutex / condition-variable epoch map run under ThreadSanitizer and
 * AddressSanitizer on a machine without a GPU.  Never part of libdcc. */
#include <stdint.h>
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
  int r = oracle_occ_hash(n, b->offsets, b->keys, b->acctype, b->start_tn, b->finish_tn, 0, NULL,
                          NULL, &ctx->tnc, out_rc, tn);
  if (st) memset(st, 0, sizeof *st);
  __atomic_fetch_sub(&inflight, 1, __ATOMIC_ACQ_REL);
  return r ? DCC_EIO : DCC_OK;
}
