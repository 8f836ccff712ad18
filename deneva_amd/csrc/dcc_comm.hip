// Multi-GPU key sharding over RCCL — placeholder until the
// sharded round driver lands.
#include <hip/hip_runtime.h>

#include "dcc.h"
#include "dcc_ctx.h"

struct dcc_comm_state {
  int rank = 0, nranks = 1;
};

int dcc_ctx::comm_ranks() const { return comm ? comm->nranks : 1; }

extern "C" int dcc_comm_unique_id(void*) { return DCC_ENOTSUP; }
extern "C" int dcc_comm_init(dcc_ctx*, int, int, const void*) { return DCC_ENOTSUP; }
extern "C" int dcc_comm_destroy(dcc_ctx* ctx) {
  if (!ctx || !ctx->comm) return DCC_OK;
  delete ctx->comm;
  ctx->comm = nullptr;
  return DCC_OK;
}
int dcc_ctx::occ_epoch_sharded(const dcc_batch*, uint8_t*, uint64_t*, dcc_stats*) {
  return fail(DCC_ENOTSUP, "sharded OCC not built yet");
}
