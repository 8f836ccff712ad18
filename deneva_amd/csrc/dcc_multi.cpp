// Single-process multi-GPU context (dcc_init(&ctx, n_gpus,
// device_ids), multi-GPU internal to the context).  A reference node is one
// rundb process with one occ_man (system/global.cpp:42); with this context
// that one process drives every GPU of the node.
//
// The context owns one per-device sub-context per GPU, key-sharded exactly
// like the one-process-per-GPU path (dcc_key_shard; each sub-context keeps
// only its shard's accesses, partitioned on its own GPU: shard_dev.hip).  The sub-contexts talk over one RCCL clique
// made with ncclCommInitAll when the device ids are distinct; when ids repeat
// (several shards on one GPU: tests, or a node with fewer GPUs than shards)
// over an in-process host exchange.  One host thread per sub-context runs its
// epoch, so every rank's collectives and host synchronisations proceed as in
// the multi-process path.  Decisions are identical on every rank (the kill /
// readiness bytes are all-reduced): rank 0's are returned.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <condition_variable>
#include <cstring>
#include <mutex>
#include <set>
#include <thread>
#include <vector>

#include "dcc.h"
#include "dcc_ctx.h"

int dcc_comm_attach(dcc_ctx* ctx, int rank, int nranks, void* nccl_comm);  // dcc_comm.hip
void dcc_comm_abort(dcc_ctx* ctx);                                          // dcc_comm.hip

namespace {

// Byte-wise MAX all-reduce among the host threads of one process.  Each
// generation's result (and its size-mismatch flag) lives in the slot of the
// generation's parity: a slow waiter of generation g reads slot g & 1, which
// only generation g + 2 rewrites -- and g + 1 cannot complete before that
// waiter arrives at it.  A failing rank poisons the exchange: every waiter
// and every later arrival returns at once with an error, so no rank blocks
// on a peer that will never arrive.
struct LocalExchange {
  int n = 0;
  std::mutex mu;
  std::condition_variable cv;
  uint64_t gen = 0;
  int arrived = 0;
  bool bad = false;        // the open generation's size mismatch
  bool poisoned = false;   // a rank failed this epoch
  std::vector<uint8_t> acc;
  std::vector<uint8_t> result[2];
  bool result_bad[2] = {false, false};
  void poison() {
    std::lock_guard<std::mutex> lk(mu);
    poisoned = true;
    cv.notify_all();
  }
  // between epochs (no rank inside): a clean exchange
  void reset() {
    std::lock_guard<std::mutex> lk(mu);
    poisoned = false;
    arrived = 0;
    bad = false;
    acc.clear();
    gen += 2;  // keeps the slot parity meaning of any stale waiter moot
  }
};
struct LocalPart {
  LocalExchange* x;
  int rank;
};

int local_exchange(void* user, uint8_t* buf, uint64_t nb) {
  LocalPart* p = (LocalPart*)user;
  LocalExchange* X = p->x;
  std::unique_lock<std::mutex> lk(X->mu);
  if (X->poisoned) return 1;
  const uint64_t g = X->gen;
  if (X->arrived == 0) {
    X->acc.assign(buf, buf + nb);
    X->bad = false;
  } else if (X->acc.size() != nb) {
    X->bad = true;  // ranks disagree on the exchange size: every rank fails
  } else {
    for (uint64_t i = 0; i < nb; i++) X->acc[i] = std::max(X->acc[i], buf[i]);
  }
  if (++X->arrived == X->n) {
    X->result[g & 1].swap(X->acc);
    X->result_bad[g & 1] = X->bad;
    X->arrived = 0;
    X->gen++;
    X->cv.notify_all();
  } else {
    X->cv.wait(lk, [&] { return X->gen != g || X->poisoned; });
    if (X->gen == g) return 1;  // poisoned before the generation completed
  }
  const std::vector<uint8_t>& res = X->result[g & 1];
  if (X->result_bad[g & 1] || res.size() != nb) return 1;
  memcpy(buf, res.data(), nb);
  return 0;
}

}  // namespace

struct dcc_multi {
  std::vector<dcc_ctx*> sub;
  LocalExchange lx;
  std::vector<LocalPart> parts;
  bool rccl = false;        // the sub-contexts share an RCCL clique
  bool broken = false;      // the clique was aborted after a rank failed
  int fail_rank = -1;       // DCC_OPT_FAIL_RANK (fault injection, tests)
  std::mutex fail_mu;
  bool failing = false;     // a rank of the running epoch failed
};

// A rank failed: its peers must not wait for it.  The host exchange is
// poisoned (waiters return an error at once); the RCCL clique is aborted
// (ncclCommAbort ends the peers' pending collectives) and the context stays
// unusable until it is destroyed.
static void fail_fast(dcc_multi* M) {
  std::lock_guard<std::mutex> lk(M->fail_mu);
  if (M->failing) return;
  M->failing = true;
  M->lx.poison();
  if (M->rccl) {
    for (dcc_ctx* s : M->sub) dcc_comm_abort(s);
    M->broken = true;
  }
}

// Runs fn(rank) on one host thread per sub-context; the first failure's code
// and message become the multi context's.  A failing rank makes every other
// rank fail too (fail_fast) instead of leaving it blocked in an exchange.
template <typename F>
static int run_ranks(dcc_ctx* ctx, F fn) {
  dcc_multi* M = ctx->multi;
  if (M->broken)
    return ctx->fail(DCC_ECOMM, "multi-GPU: the RCCL clique was aborted after a rank failed; "
                                "destroy and re-create the context");
  const int R = (int)M->sub.size();
  M->lx.reset();
  M->failing = false;
  const int inject = M->fail_rank;
  M->fail_rank = -1;  // one-shot
  std::vector<int> rc(R, DCC_OK);
  std::vector<std::thread> th;
  for (int r = 0; r < R; r++)
    th.emplace_back([&, r] {
      if (hipSetDevice(M->sub[r]->device) != hipSuccess) {
        rc[r] = DCC_ENODEV;
      } else if (r == inject) {
        rc[r] = M->sub[r]->fail(DCC_EIO, "injected failure (DCC_OPT_FAIL_RANK)");
      } else {
        rc[r] = fn(r, M->sub[r]);
      }
      if (rc[r] != DCC_OK) fail_fast(M);
    });
  for (auto& t : th) t.join();
  // the first rank that failed on its own (the others report the poisoning)
  int first = -1;
  for (int r = 0; r < R; r++)
    if (rc[r] != DCC_OK && (first < 0 || (rc[first] == DCC_ECOMM && rc[r] != DCC_ECOMM))) first = r;
  if (first >= 0) {
    ctx->last_error = "rank " + std::to_string(first) + ": " + M->sub[first]->last_error;
    return rc[first];
  }
  return DCC_OK;
}

int dcc_multi_set_fail_rank(dcc_ctx* ctx, int rank) {
  if (!ctx->multi || rank < -1 || rank >= (int)ctx->multi->sub.size()) return DCC_EINVAL;
  ctx->multi->fail_rank = rank;
  return DCC_OK;
}

extern "C" int dcc_init_multi(dcc_ctx** out, int n_gpus, const int* device_ids) {
  if (!out || n_gpus < 1 || !device_ids) return DCC_EINVAL;
  *out = nullptr;
  dcc_ctx* root = nullptr;
  int r = dcc_init(&root, device_ids[0]);
  if (r != DCC_OK) return r;
  dcc_multi* M = new dcc_multi;
  root->multi = M;
  for (int i = 0; i < n_gpus; i++) {
    dcc_ctx* s = nullptr;
    r = dcc_init(&s, device_ids[i]);
    if (r != DCC_OK) {
      dcc_destroy(root);
      return r;
    }
    M->sub.push_back(s);
  }
  if (n_gpus > 1) {
    const std::set<int> distinct(device_ids, device_ids + n_gpus);
    if ((int)distinct.size() == n_gpus) {
      // one RCCL clique over the node's GPUs (xGMI), one communicator per rank
      // (unverified on hardware: the test box has one GPU)
      std::vector<ncclComm_t> comms(n_gpus);
      const ncclResult_t e = ncclCommInitAll(comms.data(), n_gpus, device_ids);
      if (e != ncclSuccess) {
        root->last_error = std::string("ncclCommInitAll: ") + ncclGetErrorString(e);
        dcc_destroy(root);
        return DCC_ECOMM;
      }
      M->rccl = true;
      // peer access both ways between every pair: a rank's shard kernels read
      // a caller's device batch, and Calvin groups are written, over xGMI
      for (int i = 0; i < n_gpus; i++) {
        if (hipSetDevice(device_ids[i]) != hipSuccess) continue;
        for (int j = 0; j < n_gpus; j++) {
          if (i == j) continue;
          int can = 0;
          if (hipDeviceCanAccessPeer(&can, device_ids[i], device_ids[j]) == hipSuccess && can) {
            const hipError_t pe = hipDeviceEnablePeerAccess(device_ids[j], 0);
            if (pe != hipSuccess && pe != hipErrorPeerAccessAlreadyEnabled) (void)hipGetLastError();
          }
        }
      }
      for (int i = 0; i < n_gpus; i++) {
        r = dcc_comm_attach(M->sub[i], i, n_gpus, comms[i]);
        if (r != DCC_OK) {
          // the attached ones go with their sub-contexts; the rest here
          for (int j = i; j < n_gpus; j++) (void)ncclCommDestroy(comms[j]);
          dcc_destroy(root);
          return r;
        }
      }
    } else {
      // shards sharing a GPU: the in-process host exchange
      M->lx.n = n_gpus;
      M->parts.resize(n_gpus);
      for (int i = 0; i < n_gpus; i++) {
        M->parts[i] = LocalPart{&M->lx, i};
        r = dcc_comm_init_host(M->sub[i], i, n_gpus, local_exchange, &M->parts[i]);
        if (r != DCC_OK) {
          dcc_destroy(root);
          return r;
        }
      }
    }
  }
  *out = root;
  return DCC_OK;
}

int dcc_multi_size(const dcc_ctx* ctx) { return ctx && ctx->multi ? (int)ctx->multi->sub.size() : 1; }

void dcc_multi_destroy(dcc_ctx* ctx) {
  if (!ctx->multi) return;
  for (dcc_ctx* s : ctx->multi->sub) dcc_destroy(s);
  delete ctx->multi;
  ctx->multi = nullptr;
}

// A device batch (DCC_DEVICE_PTRS) is validated whole before it is sharded:
// check_batch only sees host arrays, and the ranks' shards always have
// well-formed offsets, so a malformed device batch would otherwise be decided
// silently (or fail on some ranks and not others, breaking the "every rank
// runs the same collectives" rule).  Rank 0's sub-context runs the offsets /
// length pass (prep_body) on the caller's arrays (over xGMI when they sit on a
// peer) and the batch is rejected before any rank starts.
static int multi_check_device_batch(dcc_ctx* ctx, const dcc_batch* b) {
  if (!(b->flags & DCC_DEVICE_PTRS) || b->n_txn == 0) return DCC_OK;
  dcc_ctx* s = ctx->multi->sub[0];
  int prev = 0;
  if (hipGetDevice(&prev) != hipSuccess || hipSetDevice(s->device) != hipSuccess)
    return ctx->fail(DCC_ENODEV, "multi-GPU: cannot select rank 0's device");
  DevBatch d;
  uint32_t maxlen = 0;
  uint64_t nnz_w = 0;
  int e = s->stage_batch(b, d);
  if (e == DCC_OK) e = s->device_prep(d, maxlen, nnz_w);
  (void)hipSetDevice(prev);
  if (e != DCC_OK) return ctx->fail(e, "%s", s->last_error.c_str());
  return DCC_OK;
}

// Every rank stages the batch (host: its own H2D copy; device: the caller's
// arrays, read over xGMI when they sit on a peer) and keeps its key shard on
// its GPU (dcc_ctx::shard_stage, shard_dev.hip); its epoch runs on that device
// batch into device outputs.  Rank 0's decisions are returned (host outputs:
// every rank's are compared first).
int dcc_multi_occ_epoch(dcc_ctx* ctx, const dcc_batch* b, uint8_t* out_rc, uint64_t* out_tn,
                        dcc_stats* st) {
  if (!b) return ctx->fail(DCC_EINVAL, "null batch");
  // the whole batch is validated before it is sharded: every rank then
  // runs the same collectives (no rank may fail alone mid-exchange)
  if (int e = ctx->check_batch(b)) return e;
  if (int e = multi_check_device_batch(ctx, b)) return e;
  const bool dev = (b->flags & DCC_DEVICE_PTRS) != 0;
  const uint64_t n = b->n_txn;
  const int R = (int)ctx->multi->sub.size();
  std::vector<std::vector<uint8_t>> rc(R);
  std::vector<uint64_t> tn0;
  std::vector<dcc_stats> S(R);
  const int e = run_ranks(ctx, [&](int r, dcc_ctx* s) -> int {
    // the whole batch: the rank keeps its key shard (partitioned on its GPU)
    // and serves its serial passes from the whole batch (DCC_SHARD_SELF)
    dcc_batch fb = *b;
    fb.flags |= DCC_SHARD_SELF;
    int x = DCC_OK;
    if ((x = s->sh_rc.ensure(s, n + 16, "shard rc")) != DCC_OK) return x;
    if (out_tn && (x = s->sh_tn.ensure(s, n * 8 + 16, "shard tn")) != DCC_OK) return x;
    uint8_t* drc = (uint8_t*)s->sh_rc.p;
    uint64_t* dtn = out_tn ? (uint64_t*)s->sh_tn.p : nullptr;
    if ((x = s->occ_epoch(&fb, drc, dtn, &S[r])) != DCC_OK) return x;
    hipError_t he = hipSuccess;
    if (!dev) {
      rc[r].resize(n + 1);
      he = hipMemcpy(rc[r].data(), drc, n, hipMemcpyDeviceToHost);
      if (he == hipSuccess && r == 0 && dtn) {
        tn0.resize(n);
        he = hipMemcpy(tn0.data(), dtn, n * 8, hipMemcpyDeviceToHost);
      }
    } else if (r == 0) {  // the caller's device arrays (this GPU or a peer)
      if (out_rc) he = hipMemcpy(out_rc, drc, n, hipMemcpyDeviceToDevice);
      if (he == hipSuccess && out_tn) he = hipMemcpy(out_tn, dtn, n * 8, hipMemcpyDeviceToDevice);
    }
    return he == hipSuccess ? DCC_OK : s->hip_fail(he, "multi-GPU: decisions out");
  });
  if (e != DCC_OK) return e;
  if (!dev) {
    for (int r = 1; r < R; r++)
      if (memcmp(rc[r].data(), rc[0].data(), n) != 0)
        return ctx->fail(DCC_EIO, "multi-GPU: ranks 0 and %d decided differently", r);
    if (out_rc) memcpy(out_rc, rc[0].data(), n);
    if (out_tn) memcpy(out_tn, tn0.data(), n * 8);
  }
  if (st) {
    *st = S[0];
    for (int r = 1; r < R; r++) st->device_ms = std::max(st->device_ms, S[r].device_ms);
    // every rank counts the whole batch's writes (its has-write pass reads it)
    st->nnz_w = S[0].nnz_w;
    st->alg_bytes = dcc_alg_bytes(n, b->nnz, st->nnz_w);
  }
  return DCC_OK;
}

int dcc_multi_calvin_epoch(dcc_ctx* ctx, const dcc_batch* b, const dcc_calvin_held* held,
                           uint32_t* out_group, uint8_t* out_rc, uint32_t* out_wave,
                           dcc_stats* st) {
  if (!b) return ctx->fail(DCC_EINVAL, "null batch");
  if (out_wave) {
    // wave levels chain through every row of the epoch (one walk in
    // sequence order, calvin_wave.h): the whole epoch runs on rank 0's GPU,
    // as one context (no exchange), reading a device batch over xGMI
    if (held && held->n)
      return ctx->fail(DCC_ENOTSUP, "calvin: wave levels need an empty lock table (no held prefix)");
    dcc_ctx* s = ctx->multi->sub[0];
    int prev = 0;
    if (hipGetDevice(&prev) != hipSuccess || hipSetDevice(s->device) != hipSuccess)
      return ctx->fail(DCC_ENODEV, "multi-GPU: cannot select rank 0's device");
    dcc_comm_state* const cm = s->comm;
    s->comm = nullptr;
    const int e = s->calvin_epoch(b, nullptr, out_group, out_rc, out_wave, st);
    s->comm = cm;
    (void)hipSetDevice(prev);
    if (e != DCC_OK) return ctx->fail(e, "%s", s->last_error.c_str());
    return DCC_OK;
  }
  if (int e = ctx->check_batch(b)) return e;
  if (int e = multi_check_device_batch(ctx, b)) return e;
  if (held && held->n && (!held->keys || !held->acctype))
    return ctx->fail(DCC_EINVAL, "calvin: null held arrays");
  const bool dev = (b->flags & DCC_DEVICE_PTRS) != 0;
  const uint64_t n = b->n_txn;
  const int R = (int)ctx->multi->sub.size();
  // the held prefix is sharded by row as well, on the host: with a device
  // batch its arrays are device arrays too (dcc.h), read back first (a few
  // requests per still-locked row, against the epoch's millions)
  std::vector<uint64_t> hkeys_h;
  std::vector<uint8_t> hat_h;
  const uint64_t* hkeys = held ? held->keys : nullptr;
  const uint8_t* hat = held ? held->acctype : nullptr;
  if (dev && held && held->n) {
    hkeys_h.resize(held->n);
    hat_h.resize(held->n);
    if (hipMemcpy(hkeys_h.data(), held->keys, held->n * 8, hipMemcpyDefault) != hipSuccess ||
        hipMemcpy(hat_h.data(), held->acctype, held->n, hipMemcpyDefault) != hipSuccess) {
      (void)hipGetLastError();
      return ctx->fail(DCC_EINVAL, "multi-GPU calvin: held arrays unreadable as device arrays");
    }
    hkeys = hkeys_h.data();
    hat = hat_h.data();
  }
  std::vector<std::vector<uint64_t>> hk(R);
  std::vector<std::vector<uint8_t>> ha(R);
  if (held)
    for (uint64_t i = 0; i < held->n; i++) {
      const int r = (int)dcc_key_shard(hkeys[i], (uint32_t)R);
      hk[r].push_back(hkeys[i]);
      ha[r].push_back(hat[i]);
    }
  std::vector<std::vector<uint8_t>> rc(R);
  std::vector<std::vector<uint32_t>> grp(R), src(R);
  std::vector<dcc_stats> S(R);
  const int e = run_ranks(ctx, [&](int r, dcc_ctx* s) -> int {
    dcc_batch sb;
    int x = s->shard_stage(b, (uint32_t)r, (uint32_t)R, sb);
    if (x != DCC_OK) return x;
    const uint64_t m = sb.nnz;
    if ((x = s->sh_rc.ensure(s, n + 16, "shard rc")) != DCC_OK) return x;
    if ((x = s->sh_grp.ensure(s, (m + 16) * 4, "shard groups")) != DCC_OK) return x;
    uint8_t* drc = (uint8_t*)s->sh_rc.p;
    uint32_t* dgrp = out_group ? (uint32_t*)s->sh_grp.p : nullptr;
    if (held && held->n) {
      // the shard's held rows go to its GPU beside its device batch
      const uint64_t nh = hk[r].size();
      if ((x = s->cv_hkeys.ensure(s, std::max<uint64_t>(8, nh * 8), "calvin held keys")) != DCC_OK ||
          (x = s->cv_hat.ensure(s, std::max<uint64_t>(16, nh), "calvin held types")) != DCC_OK)
        return x;
      hipError_t he = hipSuccess;
      if (nh) {
        he = hipMemcpy(s->cv_hkeys.p, hk[r].data(), nh * 8, hipMemcpyHostToDevice);
        if (he == hipSuccess) he = hipMemcpy(s->cv_hat.p, ha[r].data(), nh, hipMemcpyHostToDevice);
      }
      if (he != hipSuccess) return s->hip_fail(he, "multi-GPU calvin: held rows in");
      const dcc_calvin_held h{nh, (const uint64_t*)s->cv_hkeys.p, (const uint8_t*)s->cv_hat.p};
      x = s->calvin_epoch(&sb, &h, dgrp, drc, nullptr, &S[r]);
    } else {
      x = s->calvin_epoch(&sb, nullptr, dgrp, drc, nullptr, &S[r]);
    }
    if (x != DCC_OK) return x;
    hipError_t he = hipSuccess;
    if (!dev) {
      if (r == 0) {
        rc[0].resize(n + 1);
        he = hipMemcpy(rc[0].data(), drc, n, hipMemcpyDeviceToHost);
      }
      if (he == hipSuccess && dgrp && m) {
        grp[r].resize(m);
        src[r].resize(m);
        he = hipMemcpy(grp[r].data(), dgrp, m * 4, hipMemcpyDeviceToHost);
        if (he == hipSuccess) he = hipMemcpy(src[r].data(), s->sh_src.p, m * 4, hipMemcpyDeviceToHost);
      }
    } else {
      if (r == 0 && out_rc) he = hipMemcpy(out_rc, drc, n, hipMemcpyDeviceToDevice);
      if (he == hipSuccess && dgrp && (x = s->shard_groups(dgrp, m, out_group)) != DCC_OK) return x;
      if (he == hipSuccess) he = hipStreamSynchronize(s->stream);
    }
    return he == hipSuccess ? DCC_OK : s->hip_fail(he, "multi-GPU calvin: results out");
  });
  if (e != DCC_OK) return e;
  if (!dev) {
    if (out_rc) memcpy(out_rc, rc[0].data(), n);
    if (out_group)
      for (int r = 0; r < R; r++)
        for (size_t j = 0; j < src[r].size(); j++) out_group[src[r][j]] = grp[r][j];
  }
  if (st) {
    *st = S[0];
    for (int r = 1; r < R; r++) st->device_ms = std::max(st->device_ms, S[r].device_ms);
    // every rank counts the whole batch's writes (its has-write pass reads it)
    st->nnz_w = S[0].nnz_w;
    st->alg_bytes = dcc_calvin_alg_bytes(n, b->nnz, b->order != nullptr, 0);
  }
  return DCC_OK;
}

// Captured-snapshot validation (occ_snapshot.hip) key-sharded: a txn's
// decision is an OR over its accesses -- a history pair of a key it read, a
// captured active write set meeting one of its keys (occ.cpp:167-199) -- and
// every such meeting is between accesses of one key, so each rank decides its
// key shard against its own history shard and the captured lists (txn
// indices of the whole batch), and a txn commits iff it commits on every
// rank.  The snapshot arrays go to every rank's GPU beside its shard.
int dcc_multi_occ_snapshot(dcc_ctx* ctx, const dcc_batch* b, const dcc_occ_snapshot* snap,
                           uint8_t* out_rc, dcc_stats* st) {
  if (!b) return ctx->fail(DCC_EINVAL, "null batch");
  if (!snap || !snap->active_off) return ctx->fail(DCC_EINVAL, "snapshot: null snapshot or active_off");
  if (int e = ctx->check_batch(b)) return e;
  if (int e = multi_check_device_batch(ctx, b)) return e;
  const bool dev = (b->flags & DCC_DEVICE_PTRS) != 0;
  if (dev && !snap->active_idx)
    return ctx->fail(DCC_EINVAL, "snapshot: device capture needs active_idx (a 1-element buffer "
                                 "when every list is empty)");
  const uint64_t n = b->n_txn;
  dcc_stats S0{};
  S0.n_shards = (uint32_t)dcc_multi_size(ctx);
  if (n == 0) {
    if (st) *st = S0;
    return DCC_OK;
  }
  if (!out_rc) return ctx->fail(DCC_EINVAL, "snapshot: null out_rc");
  // a host capture: the structural checks of the one-GPU path, then its
  // arrays to every GPU (the shards are device batches)
  uint64_t n_active = 0;
  if (!dev) {
    const uint32_t* ao = snap->active_off;
    if (ao[0] != 0) return ctx->fail(DCC_EINVAL, "snapshot: active_off[0] must be 0");
    for (uint64_t t = 0; t < n; t++)
      if (ao[t + 1] < ao[t])
        return ctx->fail(DCC_EINVAL, "snapshot: active_off decreases at txn %llu", (unsigned long long)t);
    n_active = ao[n];
    if (n_active && !snap->active_idx) return ctx->fail(DCC_EINVAL, "snapshot: null active_idx");
    for (uint64_t q = 0; q < n_active; q++)
      if (snap->active_idx[q] >= n)
        return ctx->fail(DCC_EINVAL, "snapshot: active_idx[%llu] = %u >= n_txn", (unsigned long long)q,
                         snap->active_idx[q]);
  }
  const int R = (int)ctx->multi->sub.size();
  std::vector<std::vector<uint8_t>> rc(R);
  std::vector<dcc_stats> S(R);
  const int e = run_ranks(ctx, [&](int r, dcc_ctx* s) -> int {
    dcc_batch sb;
    int x = s->shard_stage(b, (uint32_t)r, (uint32_t)R, sb);
    if (x != DCC_OK) return x;
    dcc_occ_snapshot ds = *snap;
    if (!dev) {
      if ((x = s->snap_aoff.ensure(s, (n + 1) * 4, "snapshot active_off")) != DCC_OK ||
          (x = s->snap_aidx.ensure(s, std::max<uint64_t>(16, n_active * 4), "snapshot active_idx")) != DCC_OK)
        return x;
      hipError_t he = hipMemcpy(s->snap_aoff.p, snap->active_off, (n + 1) * 4, hipMemcpyHostToDevice);
      if (he == hipSuccess && n_active)
        he = hipMemcpy(s->snap_aidx.p, snap->active_idx, n_active * 4, hipMemcpyHostToDevice);
      if (he == hipSuccess && snap->hist_top) {
        if ((x = s->snap_top.ensure(s, n * 8, "snapshot hist_top")) != DCC_OK) return x;
        he = hipMemcpy(s->snap_top.p, snap->hist_top, n * 8, hipMemcpyHostToDevice);
      }
      if (he != hipSuccess) return s->hip_fail(he, "multi-GPU snapshot: capture in");
      ds.active_off = (const uint32_t*)s->snap_aoff.p;
      ds.active_idx = (const uint32_t*)s->snap_aidx.p;
      ds.hist_top = snap->hist_top ? (const uint64_t*)s->snap_top.p : nullptr;
    }
    if ((x = s->sh_rc.ensure(s, n + 16, "shard rc")) != DCC_OK) return x;
    // the shard's decisions alone (no collective: the ranks are combined below)
    dcc_comm_state* const cm = s->comm;
    s->comm = nullptr;
    x = s->occ_snapshot(&sb, &ds, (uint8_t*)s->sh_rc.p, &S[r]);
    s->comm = cm;
    if (x != DCC_OK) return x;
    rc[r].resize(n);
    const hipError_t he = hipMemcpy(rc[r].data(), s->sh_rc.p, n, hipMemcpyDeviceToHost);
    return he == hipSuccess ? DCC_OK : s->hip_fail(he, "multi-GPU snapshot: decisions out");
  });
  if (e != DCC_OK) return e;
  // a txn aborts if any rank aborts it (DCC_RC_ABORT > DCC_RC_RCOK)
  std::vector<uint8_t> fin(rc[0]);
  for (int r = 1; r < R; r++)
    for (uint64_t t = 0; t < n; t++) fin[t] = std::max(fin[t], rc[r][t]);
  if (dev) {
    if (hipMemcpy(out_rc, fin.data(), n, hipMemcpyHostToDevice) != hipSuccess)
      return ctx->hip_fail(hipGetLastError(), "multi-GPU snapshot: decisions to the caller");
  } else {
    memcpy(out_rc, fin.data(), n);
  }
  if (st) {
    dcc_stats T = S0;
    for (int r = 0; r < R; r++) {
      T.device_ms = std::max(T.device_ms, S[r].device_ms);
      T.nnz_w += S[r].nnz_w;
      T.alg_bytes += S[r].alg_bytes;
    }
    for (uint64_t t = 0; t < n; t++) (fin[t] == DCC_RC_RCOK ? T.n_commit : T.n_abort)++;
    if (!dev) {  // read-only txns of the whole batch (a rank sees only its shard)
      for (uint64_t t = 0; t < n; t++) {
        bool w = false;
        for (uint32_t x = b->offsets[t]; x < b->offsets[t + 1] && !w; x++) w = b->acctype[x] == DCC_WR;
        T.n_readonly += w ? 0 : 1;
      }
    }
    *st = T;
  }
  return DCC_OK;
}

// MaaT on a multi-GPU context: the whole epoch on rank 0's GPU, whose row
// table holds every row's timestamps (the bounds of a txn combine every row
// it touches; a key-sharded MaaT would all-reduce a txn's lower and upper
// bound per round -- a u64 max and min -- not built).
dcc_ctx* dcc_multi_rank0(dcc_ctx* ctx) {
  dcc_ctx* s = ctx->multi->sub[0];
  (void)hipSetDevice(s->device);
  return s;
}

// per-rank state kept identical on every rank (options, tnc, history)
int dcc_multi_each(dcc_ctx* ctx, int (*fn)(dcc_ctx*, void*), void* user) {
  for (dcc_ctx* s : ctx->multi->sub) {
    const int r = fn(s, user);
    if (r != DCC_OK) {
      ctx->last_error = s->last_error;
      return r;
    }
  }
  return DCC_OK;
}

dcc_ctx* dcc_multi_sub(dcc_ctx* ctx, int rank) { return ctx->multi->sub[rank]; }
