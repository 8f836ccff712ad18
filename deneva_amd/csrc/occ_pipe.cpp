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

#include <algorithm>
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
    uint64_t seq;       // submit sequence of lane epochs (the chained finishes' order)
    bool chain;         // its central_finish is chained on the device (chain_enqueue)
    bool app;           // ... and appends to the history
    uint64_t res;       // delta-level pairs reserved for that append
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
  uint64_t seq = 0;            // the last lane epoch's sequence number
  uint64_t app_res = 0;        // delta-level pairs reserved by chained appends in flight
  uint64_t app_max = 0;        // largest append seen (the reservation estimate)
  bool broken = false;         // an epoch failed after its chained finish numbered it
};

// Another chained epoch in flight (its finish may wait for fin_ctl to move).
static bool chain_behind(const OccPipe* p) {
  for (const OccPipe::Flight& f : p->flight)
    if (f.chain) return true;
  return false;
}

// Completion, in submit order.  A chained epoch's finish ran behind its
// decision on the lane: when it numbered the epoch (totals[4] == 1) the
// context's tnc and delta level follow its totals; when it did not (an epoch
// before it was not finished when it ran, or this one was not final and took
// more levels), the context finishes the epoch itself (pipe_finish) and moves
// fin_ctl past it, as it does after every other epoch it finishes on the host
// while chained epochs are in flight behind it.
static void pipe_complete_front(dcc_ctx* ctx) {
  OccPipe* p = ctx->pipe;
  const OccPipe::Flight f = p->flight.front();
  p->flight.pop_front();
  dcc_ctx* lane = p->lanes[f.lane];
  OccPipe::Result r{};
  (void)hipSetDevice(lane->device);
  r.rc = lane->occ_end(&r.st);
  if (r.rc != DCC_OK) r.err = lane->last_error;
  bool host_done = true;  // fin_ctl does not know this epoch's outcome
  if (f.chain) {
    uint64_t st = 0;
    const hipError_t e = hipEventSynchronize(lane->ev_done);  // the finish (and tn copy) passed
    if (e == hipSuccess) {
      st = ((const uint64_t*)((const char*)lane->hfin + dcc_ctx::HDYN_TOTALS))[4];
    } else if (r.rc == DCC_OK) {
      r.rc = ctx->hip_fail(e, "chained central_finish");
      r.err = ctx->last_error;
    }
    if (st == 2 && lane->run.app) ctx->hs[1].built = false;  // pushed before the epoch was final
    if (p->broken) {
      // numbered behind an epoch that failed after its finish ran
      r.rc = DCC_EIO;
      r.err = "an epoch before this one in the pipeline failed after its central_finish ran on the device";
      host_done = false;
    } else if (r.rc != DCC_OK) {
      if (st == 1) {  // the later finishes followed its numbering
        p->broken = true;
        ctx->hs[1].built = false;
        host_done = false;
      }
    } else if (st == 1) {
      r.rc = ctx->chain_accept(lane);
      r.st.fin_where = 1;
      host_done = false;
      if (r.rc != DCC_OK) {
        r.err = ctx->last_error;
        p->broken = true;
        ctx->hs[1].built = false;
      }
    } else {
      r.rc = ctx->pipe_finish(lane, true);
      r.st.fin_where = 2;
      if (r.rc != DCC_OK) r.err = ctx->last_error;
    }
  } else if (r.rc == DCC_OK && lane->run.fin_later) {
    // commit tn and the history append from the parent's state, in submit
    // order (central_finish, occ.cpp:248-294)
    // (chained epochs behind it: the delta level stays where their finishes
    // will write)
    r.rc = ctx->pipe_finish(lane, chain_behind(p));
    r.st.fin_where = 2;
    if (r.rc != DCC_OK) r.err = ctx->last_error;
  } else if (r.rc == DCC_OK) {
    ctx->tnc += lane->run.n_cw;  // tnc advances in submit order (occ.cpp:283-284)
  }
  if (host_done && !p->broken && chain_behind(p) && ctx->chain_set(lane, f.seq + 1) != DCC_OK) {
    p->broken = true;  // the chained epochs behind it cannot be trusted to follow
    ctx->hs[1].built = false;
  }
  if (lane->run.fin_later && lane->run.app) p->app_in_flight--;
  if (f.chain && f.app) {
    p->app_res -= f.res;
    p->app_max = std::max<uint64_t>(p->app_max, ctx->hs[1].last_app);
  }
  lane->tnc = 0;
  p->done[f.ticket] = std::move(r);
}

// Complete every epoch in flight (results stay until waited).
void dcc_pipe_drain(dcc_ctx* ctx) {
  if (!ctx || !ctx->pipe) return;
  while (!ctx->pipe->flight.empty()) pipe_complete_front(ctx);
  ctx->pipe->broken = false;  // the next chained epoch starts fin_ctl afresh
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
  // Chained central_finish (DCC_OPT_PIPE_CHAIN): the epoch's commit tn and
  // history append are enqueued behind its decision on its lane.  Its append
  // needs room in the delta level reserved now (the level never moves while
  // chained epochs are in flight): an estimate from the largest append seen,
  // a sixteenth of the accesses before any; a finish that does not fit leaves
  // the epoch to the host (pipe_finish).
  const bool fin = out_tn || (b->flags & DCC_OCC_APPEND_HISTORY);
  const bool chain = fin && ctx->pipe_chain;
  const bool app = chain && (b->flags & DCC_OCC_APPEND_HISTORY);
  const uint64_t res = app ? (p->app_max ? 2 * p->app_max : b->nnz / 16) + 4096 : 0;
  if (p->broken) dcc_pipe_drain(ctx);
  if (app && ctx->hs[1].m + p->app_res + res > ctx->hist_room()) dcc_pipe_drain(ctx);
  const int li = (int)(p->next_lane++ % p->lanes.size());
  dcc_ctx* lane = p->lanes[li];
  // the lane's previous epoch completes first (and every epoch before it)
  while (lane->run.active && !p->flight.empty()) pipe_complete_front(ctx);
  // with nothing in flight the host's tnc and history are exact: fin_ctl
  // starts from them (after any merge / rebuild the history is due, and room
  // for the appends of a full pipeline)
  const bool reset = chain && p->flight.empty();
  if (reset && app) {
    if (int e = ctx->hist_prepare()) return e;
    const uint64_t want = ctx->hs[1].m + 4 * (p->lanes.size() + 1) * res;
    if (want > ctx->hist_room())
      if (int e = ctx->hist_grow_flat(ctx->hs[1], want)) return e;
  }
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
  OccPipe::Flight f{ticket, li, ++p->seq, false, false, 0};
  if (ctx->pipe_chain) {
    if (!lane->ev_done && hipEventCreateWithFlags(&lane->ev_done, hipEventDisableTiming) != hipSuccess)
      return ctx->hip_fail(hipGetLastError(), "pipeline lane event");
    if (chain && lane->run.fin_later) {
      // behind the previous epoch's last work (its own finish, or its decision)
      hipEvent_t after = p->flight.empty() ? nullptr : p->lanes[p->flight.back().lane]->ev_done;
      f.chain = ctx->chain_enqueue(lane, f.seq, after, reset) == DCC_OK;
      if (!f.chain) {
        // the host finishes it at completion instead; a finish the failed
        // enqueue may still have launched can have pushed its pairs onto the
        // delta's chains: rebuilt from the flat pairs before the next read
        (void)hipGetLastError();
        ctx->hs[1].built = false;
      }
      f.app = f.chain && app;
      f.res = f.app ? res : 0;
      p->app_res += f.res;
    }
    if (hipEventRecord(lane->ev_done, lane->stream) != hipSuccess)
      return ctx->hip_fail(hipGetLastError(), "pipeline lane event");
  }
  p->flight.push_back(f);
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
