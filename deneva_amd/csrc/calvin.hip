// Calvin epoch lock ordering — placeholder until the grant-group kernels land.
#include <hip/hip_runtime.h>

#include "dcc.h"
#include "dcc_ctx.h"

int dcc_ctx::calvin_epoch(const dcc_batch*, uint32_t*, uint8_t*, uint32_t*, dcc_stats*) {
  return fail(DCC_ENOTSUP, "Calvin engine not built yet");
}

extern "C" int dcc_calvin_order_epoch(dcc_ctx* ctx, const dcc_batch* batch, uint32_t* out_group,
                                      uint8_t* out_rc, uint32_t* out_wave, dcc_stats* st) {
  if (!ctx) return DCC_EINVAL;
  if (hipSetDevice(ctx->device) != hipSuccess) return DCC_ENODEV;
  return ctx->calvin_epoch(batch, out_group, out_rc, out_wave, st);
}
