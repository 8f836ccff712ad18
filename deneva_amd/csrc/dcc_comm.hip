// Multi-GPU key sharding: one process per GPU, each owning
// the keys with dcc_key_shard(key, nranks) == rank.  The only exchange is an
// in-place all-reduce MAX of per-txn bytes once per fixed-point round (OCC
// status: 0 clear, 1 blocked, 2 killed — killed on any shard dominates, the
// 2PC AND of votes of worker_thread.cpp:328-334) and once per epoch for
// Calvin readiness.
//
// Two backends behind one call:
//   RCCL  (dcc_comm_init): ncclAllReduce(ncclUint8, ncclMax) enqueued on the
//         engine stream — no host synchronisation, rounds stay batched.
//   host  (dcc_comm_init_host): the caller's exchange function runs on a
//         pinned host copy (used by tests that put several ranks on one GPU
//         and exchange over torch.distributed/gloo).
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <cstring>

#include "dcc.h"
#include "dcc_ctx.h"

static_assert(sizeof(ncclUniqueId) == DCC_UNIQUE_ID_BYTES, "unique id size");

struct dcc_comm_state {
  int rank = 0, nranks = 1;
  ncclComm_t nccl = nullptr;
  dcc_exchange_fn fn = nullptr;
  void* user = nullptr;
  uint8_t* hbuf = nullptr;  // pinned staging for the host backend
  uint64_t hcap = 0;
  bool aborted = false;     // ncclCommAbort ran (a peer rank failed)
  bool solo = false;        // a one-rank RCCL clique running the sharded paths (DCC_OPT_COMM_SOLO)
  uint64_t calls = 0;       // collectives run (dcc_comm_calls)
};

int dcc_ctx::comm_ranks() const { return comm ? comm->nranks : 1; }
bool dcc_ctx::sharded() const { return comm && (comm->nranks > 1 || comm->solo); }
int dcc_ctx::comm_rank() const { return comm ? comm->rank : 0; }

int dcc_ctx::comm_allreduce_max_u8(uint8_t* dev, uint64_t n) {
  dcc_ctx* ctx = this;
  if (!sharded() || n == 0) return DCC_OK;
  if (comm->aborted) return fail(DCC_ECOMM, "communicator aborted (a peer rank failed)");
  comm->calls++;
  if (comm->nccl) {
    const ncclResult_t r = ncclAllReduce(dev, dev, n, ncclUint8, ncclMax, comm->nccl, stream);
    if (r != ncclSuccess) return fail(DCC_ECOMM, "ncclAllReduce: %s", ncclGetErrorString(r));
    return DCC_OK;
  }
  if (comm->hcap < n) {
    if (comm->hbuf) (void)hipHostFree(comm->hbuf);
    comm->hbuf = nullptr;
    comm->hcap = 0;
    hipError_t e = hipHostMalloc((void**)&comm->hbuf, n, hipHostMallocDefault);
    if (e != hipSuccess) return hip_fail(e, "hipHostMalloc(exchange)");
    comm->hcap = n;
  }
  hipError_t e = hipMemcpyAsync(comm->hbuf, dev, n, hipMemcpyDeviceToHost, stream);
  if (e == hipSuccess) e = hipStreamSynchronize(stream);
  if (e != hipSuccess) return ctx->hip_fail(e, "exchange D2H");
  if (comm->fn(comm->user, comm->hbuf, n) != 0) return fail(DCC_ECOMM, "exchange callback failed");
  e = hipMemcpyAsync(dev, comm->hbuf, n, hipMemcpyHostToDevice, stream);
  if (e == hipSuccess) e = hipStreamSynchronize(stream);  // hbuf is reused by the next call
  if (e != hipSuccess) return ctx->hip_fail(e, "exchange H2D");
  return DCC_OK;
}

int dcc_ctx::comm_allgather_u8(const uint8_t* send, uint8_t* recv, uint64_t bytes) {
  const int R = comm_ranks(), me = comm_rank();
  if (!sharded()) {
    const hipError_t e = hipMemcpyAsync(recv, send, bytes, hipMemcpyDeviceToDevice, stream);
    return e == hipSuccess ? DCC_OK : hip_fail(e, "allgather copy");
  }
  if (comm->aborted) return fail(DCC_ECOMM, "communicator aborted (a peer rank failed)");
  if (comm->nccl) {
    comm->calls++;
    const ncclResult_t r = ncclAllGather(send, recv, bytes, ncclUint8, comm->nccl, stream);
    if (r != ncclSuccess) return fail(DCC_ECOMM, "ncclAllGather: %s", ncclGetErrorString(r));
    return DCC_OK;
  }
  // host exchange: own slot in a zeroed buffer, then the byte-wise MAX
  hipError_t e = hipMemsetAsync(recv, 0, bytes * R, stream);
  if (e == hipSuccess)
    e = hipMemcpyAsync(recv + (uint64_t)me * bytes, send, bytes, hipMemcpyDeviceToDevice, stream);
  if (e != hipSuccess) return hip_fail(e, "allgather staging");
  return comm_allreduce_max_u8(recv, bytes * R);
}

extern "C" int dcc_comm_unique_id(void* out_id) {
  if (!out_id) return DCC_EINVAL;
  ncclUniqueId id;
  if (ncclGetUniqueId(&id) != ncclSuccess) return DCC_ECOMM;
  memcpy(out_id, &id, sizeof id);
  return DCC_OK;
}

static int comm_check(dcc_ctx* ctx, int rank, int nranks) {
  if (!ctx || nranks < 1 || rank < 0 || rank >= nranks) return DCC_EINVAL;
  if (ctx->multi) return ctx->fail(DCC_EINVAL, "multi-GPU context: its communicator is internal");
  if (ctx->comm) return ctx->fail(DCC_EINVAL, "communicator already initialised");
  return DCC_OK;
}

extern "C" int dcc_comm_init(dcc_ctx* ctx, int rank, int nranks, const void* unique_id) {
  int r = comm_check(ctx, rank, nranks);
  if (r) return r;
  if (!unique_id) return DCC_EINVAL;
  if (hipSetDevice(ctx->device) != hipSuccess) return DCC_ENODEV;
  auto* c = new dcc_comm_state;
  c->rank = rank;
  c->nranks = nranks;
  c->solo = nranks == 1 && ctx->comm_solo;
  if (nranks > 1 || c->solo) {
    ncclUniqueId id;
    memcpy(&id, unique_id, sizeof id);
    const ncclResult_t e = ncclCommInitRank(&c->nccl, nranks, id, rank);
    if (e != ncclSuccess) {
      delete c;
      return ctx->fail(DCC_ECOMM, "ncclCommInitRank: %s", ncclGetErrorString(e));
    }
  }
  ctx->comm = c;
  return DCC_OK;
}

// dcc_init_multi: a sub-context joins the clique ncclCommInitAll made
int dcc_comm_attach(dcc_ctx* ctx, int rank, int nranks, void* nccl_comm) {
  if (!ctx || !nccl_comm || ctx->comm) return DCC_EINVAL;
  auto* c = new dcc_comm_state;
  c->rank = rank;
  c->nranks = nranks;
  c->nccl = (ncclComm_t)nccl_comm;
  ctx->comm = c;
  return DCC_OK;
}

// a peer failed: end this rank's pending RCCL collectives (multi context)
void dcc_comm_abort(dcc_ctx* ctx) {
  if (!ctx || !ctx->comm || ctx->comm->aborted) return;
  ctx->comm->aborted = true;
  if (ctx->comm->nccl) {
    (void)ncclCommAbort(ctx->comm->nccl);
    ctx->comm->nccl = nullptr;
  }
}

extern "C" int dcc_comm_init_host(dcc_ctx* ctx, int rank, int nranks, dcc_exchange_fn fn,
                                  void* user) {
  int r = comm_check(ctx, rank, nranks);
  if (r) return r;
  if (!fn) return DCC_EINVAL;
  auto* c = new dcc_comm_state;
  c->rank = rank;
  c->nranks = nranks;
  c->fn = fn;
  c->user = user;
  ctx->comm = c;
  return DCC_OK;
}

extern "C" int dcc_comm_destroy(dcc_ctx* ctx) {
  if (!ctx || !ctx->comm) return DCC_OK;
  if (ctx->comm->nccl) (void)ncclCommDestroy(ctx->comm->nccl);
  if (ctx->comm->hbuf) (void)hipHostFree(ctx->comm->hbuf);
  delete ctx->comm;
  ctx->comm = nullptr;
  return DCC_OK;
}

extern "C" uint64_t dcc_comm_calls(const dcc_ctx* ctx) {
  if (!ctx) return 0;
  if (ctx->multi) {
    uint64_t s = 0;
    for (int r = 0; r < dcc_multi_size(ctx); r++) s += dcc_comm_calls(dcc_multi_sub((dcc_ctx*)ctx, r));
    return s;
  }
  return ctx->comm ? ctx->comm->calls : 0;
}

extern "C" int dcc_comm_rank(const dcc_ctx* ctx) { return ctx && ctx->comm ? ctx->comm->rank : 0; }
extern "C" int dcc_comm_size(const dcc_ctx* ctx) {
  if (ctx && ctx->multi) return dcc_multi_size(ctx);
  return ctx && ctx->comm ? ctx->comm->nranks : 1;
}
