// Pipelined OCC epochs: dcc_occ_submit_epoch / dcc_occ_wait_epoch
// (include/dcc.h).
//
// One headline epoch is a chain of ~20 dependent launches whose serial passes
// run on one CU each: most of the chip idles through most of
// the epoch.  Consecutive epochs of central_validate are independent under
// TS_CLOCK (no history window; occ.cpp:160-180 never finds
// an entry) except for the commit counter tnc (occ.cpp:283-284), so they can
// share the chip: each lane is a full engine context on the same device (its
// own stream, workspaces and captured graph), epoch k goes to lane k mod L,
// and the epochs complete -- results read back, tnc advanced -- in submit
// order.  Commit tn and the history append (central_finish, occ.cpp:277-286)
// are the parent's: a lane only decides, and the parent numbers and appends
// each epoch when it completes (dcc_ctx::pipe_finish), so the history changes
// only in submit order.  An epoch that reads the history (a window over a
// non-empty history, or over appends still in flight) or defers its finish
// drains the lanes and runs on the parent context itself.
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>

#include <deque>
#include <string>
#include <unordered_map>
#include <vector>

#include "dcc.h"
#include "dcc_ctx.h"

struct OccPipe {
  std::vector<dcc_ctx*> lanes;
  struct Flight {
    uint64_t ticket;
    int lane;
  };
  std::deque<Flight> flight;  // submitted and not yet completed, submit order
  struct Result {
    int rc;
    dcc_stats st;
    std::string err;
  };
  std::unordered_map<uint64_t, Result> done;  // completed, not yet waited
  uint64_t next = 1;
  uint32_t next_lane = 0;
  hipEvent_t ready = nullptr;  // the caller's stream, before an epoch's first lane launch
  uint32_t part = 0;           // DCC_OPT_PIPE_PARTITION the lanes were made with
  uint32_t app_in_flight = 0;  // epochs in flight whose history append is still to come
};

static void pipe_complete_front(dcc_ctx* ctx) {
  OccPipe* p = ctx->pipe;
  const OccPipe::Flight f = p->flight.front();
  p->flight.pop_front();
  dcc_ctx* lane = p->lanes[f.lane];
  OccPipe::Result r{};
  (void)hipSetDevice(lane->device);
  r.rc = lane->occ_end(&r.st);
  if (r.rc != DCC_OK) {
    r.err = lane->last_error;
  } else if (lane->run.fin_later) {
    // commit tn and the history append from the parent's state, in submit
    // order (central_finish, occ.cpp:248-294)
    r.rc = ctx->pipe_finish(lane);
    if (r.rc != DCC_OK) r.err = ctx->last_error;
  } else {
    ctx->tnc += lane->run.n_cw;  // tnc advances in submit order (occ.cpp:283-284)
  }
  if (lane->run.fin_later && lane->run.app) p->app_in_flight--;
  lane->tnc = 0;
  p->done[f.ticket] = std::move(r);
}

// Complete every epoch in flight (results stay until waited).
void dcc_pipe_drain(dcc_ctx* ctx) {
  if (!ctx || !ctx->pipe) return;
  while (!ctx->pipe->flight.empty()) pipe_complete_front(ctx);
}

void dcc_pipe_destroy(dcc_ctx* ctx) {
  if (!ctx || !ctx->pipe) return;
  dcc_pipe_drain(ctx);
  for (dcc_ctx* l : ctx->pipe->lanes) dcc_destroy(l);
  if (ctx->pipe->ready) (void)hipEventDestroy(ctx->pipe->ready);
  delete ctx->pipe;
  ctx->pipe = nullptr;
}

// Lanes on their own CUs (DCC_OPT_PIPE_PARTITION): lane i of L runs on CU
// mask bits [i n / L, (i + 1) n / L), so a lane's one-workgroup serial passes
// never wait for a CU that another lane's chip-wide kernels hold.  A queue's
// workgroups are dealt round-robin to all 8 XCDs whatever its mask, so every
// XCD must keep CUs in every lane's mask (a mask that empties an XCD is
// ignored: the stream then runs on the whole chip); the driver spreads a
// range of consecutive mask bits evenly over the XCDs and their shader
// engines (bits 0-31: four CUs on each XCD, one per SE;
// tools/cumask_probe.hip, profiles/r06/cumask_probe.txt), so each lane gets
// n / (8 L) CUs of every XCD.
static int lane_partition(dcc_ctx* ctx, dcc_ctx* l, uint32_t i, uint32_t L) {
  const uint32_t n = (uint32_t)ctx->n_cu;
  if (L < 2 || n % (8 * L)) return DCC_OK;  // one lane, or CUs that do not split evenly: unmasked
  std::vector<uint32_t> mask((n + 31) / 32, 0u);
  const uint32_t b0 = i * n / L, b1 = (i + 1) * n / L;
  for (uint32_t b = b0; b < b1; b++) mask[b / 32] |= 1u << (b % 32);
  hipStream_t s = nullptr;
  const hipError_t e = hipExtStreamCreateWithCUMask(&s, (uint32_t)mask.size(), mask.data());
  if (e != hipSuccess) return ctx->hip_fail(e, "pipeline lane: hipExtStreamCreateWithCUMask");
  if (l->own_stream) (void)hipStreamDestroy(l->own_stream);
  l->own_stream = l->stream = s;
  l->n_cu = (int)(b1 - b0);  // grids are sized to the lane's CUs
  return DCC_OK;
}

static int pipe_lanes(dcc_ctx* ctx) {
  OccPipe* p = ctx->pipe;
  const size_t want = ctx->pipe_lanes;
  if (p->lanes.size() == want && p->part == ctx->pipe_part) return DCC_OK;
  dcc_pipe_drain(ctx);
  if (p->part != ctx->pipe_part) {  // every lane is re-created on its new CUs
    for (dcc_ctx* l : p->lanes) dcc_destroy(l);
    p->lanes.clear();
    p->part = ctx->pipe_part;
  }
  while (p->lanes.size() > want) {
    dcc_destroy(p->lanes.back());
    p->lanes.pop_back();
  }
  if (p->part)  // the partition depends on the lane count
    while (!p->lanes.empty() && p->lanes.size() != want) {
      dcc_destroy(p->lanes.back());
      p->lanes.pop_back();
    }
  while (p->lanes.size() < want) {
    dcc_ctx* l = nullptr;
    const int e = dcc_init(&l, ctx->device);
    if (e != DCC_OK) return ctx->fail(e, "pipeline lane on device %d: %s", ctx->device, dcc_strerror(e));
    p->lanes.push_back(l);
    if (p->part) {
      const int x = lane_partition(ctx, l, (uint32_t)p->lanes.size() - 1, (uint32_t)want);
      if (x != DCC_OK) return x;
    }
  }
  p->next_lane = 0;
  return DCC_OK;
}

// The parent's tuning knobs, at every submit (a lane's writer table keeps any
// growth it needed after an overflow).
static void lane_options(const dcc_ctx* ctx, dcc_ctx* l) {
  l->solver = ctx->solver;
  l->ro_split = ctx->ro_split;
  l->wt_bits = std::max(l->wt_bits, ctx->wt_bits);
  l->sw_levels = ctx->sw_levels;
  l->recheck_max = ctx->recheck_max;
  l->batch_max = ctx->batch_max;
}

extern "C" int dcc_occ_submit_epoch(dcc_ctx* ctx, const dcc_batch* b, uint8_t* out_rc,
                                    uint64_t* out_tn, uint64_t* out_ticket) {
  if (!ctx || !b || !out_ticket) return DCC_EINVAL;
  if (hipSetDevice(ctx->device) != hipSuccess) return DCC_ENODEV;
  if (!ctx->pipe) {
    ctx->pipe = new OccPipe();
    if (hipEventCreateWithFlags(&ctx->pipe->ready, hipEventDisableTiming) != hipSuccess) {
      (void)hipGetLastError();
      ctx->pipe->ready = nullptr;
      return ctx->fail(DCC_EIO, "pipeline event");
    }
  }
  OccPipe* p = ctx->pipe;
  const uint64_t ticket = p->next;
  // Commit tn and the history append go to lanes too (the parent runs each
  // epoch's central_finish when it completes, pipe_finish).  What needs the
  // epochs before it finished runs on the parent after a drain: a history
  // window over a non-empty history -- or over appends still in flight --
  // and the deferred 2PC finish.
  const bool shared = (b->flags & DCC_OCC_DEFER_FINISH) || ctx->fin_pending ||
                      (b->start_tn && (ctx->hist_size() > 0 || p->app_in_flight > 0));
  const bool lanes_ok = !ctx->multi && !ctx->sharded() && !ctx->profiling &&
                        ctx->use_sweep() && !shared && b->n_txn > 0;
  if (!lanes_ok) {
    // in submit order, on the parent context itself
    dcc_pipe_drain(ctx);
    OccPipe::Result r{};
    r.rc = dcc_occ_validate_epoch(ctx, b, out_rc, out_tn, &r.st);
    if (r.rc != DCC_OK) r.err = ctx->last_error;
    p->next++;
    p->done[ticket] = std::move(r);
    *out_ticket = ticket;
    return DCC_OK;
  }
  if (int e = pipe_lanes(ctx)) return e;
  const int li = (int)(p->next_lane++ % p->lanes.size());
  dcc_ctx* lane = p->lanes[li];
  // the lane's previous epoch completes first (and every epoch before it)
  while (lane->run.active && !p->flight.empty()) pipe_complete_front(ctx);
  lane_options(ctx, lane);
  // device batches may have been written on the caller's stream
  if (hipEventRecord(p->ready, ctx->stream) != hipSuccess ||
      hipStreamWaitEvent(lane->stream, p->ready, 0) != hipSuccess)
    return ctx->hip_fail(hipGetLastError(), "pipeline stream ordering");
  p->next++;
  *out_ticket = ticket;
  const int e = lane->occ_begin(b, out_rc, out_tn, true, true);
  if (e == DCC_OK && lane->run.fin_later && lane->run.app) p->app_in_flight++;
  if (e != DCC_OK) {
    OccPipe::Result r{};
    r.rc = e;
    r.err = lane->last_error;
    p->done[ticket] = std::move(r);
    return DCC_OK;
  }
  p->flight.push_back({ticket, li});
  return DCC_OK;
}

extern "C" int dcc_occ_wait_epoch(dcc_ctx* ctx, uint64_t ticket, dcc_stats* st) {
  if (!ctx) return DCC_EINVAL;
  OccPipe* p = ctx->pipe;
  if (!p || ticket == 0 || ticket >= p->next) return ctx->fail(DCC_EINVAL, "unknown epoch ticket %llu",
                                                               (unsigned long long)ticket);
  while (!p->done.count(ticket) && !p->flight.empty() && p->flight.front().ticket <= ticket)
    pipe_complete_front(ctx);
  auto it = p->done.find(ticket);
  if (it == p->done.end())
    return ctx->fail(DCC_EINVAL, "epoch ticket %llu was already waited", (unsigned long long)ticket);
  const int rc = it->second.rc;
  if (st) *st = it->second.st;
  if (rc != DCC_OK) ctx->last_error = it->second.err;
  p->done.erase(it);
  return rc;
}
