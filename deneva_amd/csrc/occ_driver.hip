// OCC epoch driver (host): sizes workspaces, enqueues the gfx950 kernels of
// occ_kernels.hip and synchronises once per batch of rounds.
//
// Reference: OptCC::validate / central_validate / central_finish
// (concurrency_control/occ.cpp:42-327) applied to a whole epoch; the C entry
// point is dcc_occ_validate_epoch (include/dcc.h).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstring>
#include <vector>

#include "dcc.h"
#include "dcc_ctx.h"
#include "dcc_device.h"
#include "occ_kernels.h"

using namespace dcc;

#define CK(expr)                                           \
  do {                                                     \
    hipError_t e_ = (expr);                                \
    if (e_ != hipSuccess) return ctx->hip_fail(e_, #expr); \
  } while (0)
#define CR(expr)                 \
  do {                           \
    int r_ = (expr);             \
    if (r_ != DCC_OK) return r_; \
  } while (0)

static uint64_t next_pow2(uint64_t x) {
  uint64_t p = 1;
  while (p < x) p <<= 1;
  return p;
}

uint64_t dcc_ctx::table_capacity(uint64_t nnz_w) {
  // load factor <= 0.8 even if every write key is distinct
  return std::max<uint64_t>(1024, next_pow2(nnz_w + nnz_w / 4 + 1));
}

// Undecided lists are NSEG segments; workgroup-tile g of a round appends its
// blocked txns to segment g % NSEG.  A segment holds at most seg_tiles tiles.
void dcc_ctx::list_geometry(uint64_t n, uint32_t tw, uint64_t& seg_ts, uint64_t& seg_es) const {
  const uint64_t per_tile = (uint64_t)tw * TILE_WAVES;
  const uint64_t tiles = (n + per_tile - 1) / per_tile;
  const uint64_t seg_tiles = (tiles + NSEG - 1) / NSEG + 1;
  seg_ts = seg_tiles * per_tile;
  seg_es = seg_tiles * (uint64_t)TILE_WAVES * ROUND_CAP;
}

int dcc_ctx::reserve_occ(uint64_t n, uint64_t nnz, uint64_t nnz_w, uint32_t tw) {
  (void)nnz;
  CR(state.ensure(this, n + 16, "state"));
  CR(hasw.ensure(this, n + 16, "hasw"));
  CR(rc.ensure(this, n + 16, "rc"));
  uint64_t ts, es;
  list_geometry(n, tw, ts, es);
  for (int i = 0; i < 2; i++) {
    CR(l_tid[i].ensure(this, NSEG * ts * 4, "list tid"));
    CR(l_coff[i].ensure(this, NSEG * ts * 4, "list off"));
    CR(l_cent[i].ensure(this, NSEG * es * 8, "list entries"));
  }
  CR(table.ensure(this, table_capacity(nnz_w) * sizeof(Slot), "table"));
  return DCC_OK;
}

int dcc_ctx::read_partials(size_t bytes) {
  dcc_ctx* ctx = this;
  CK(hipMemcpyAsync(hpart, part.p, bytes, hipMemcpyDeviceToHost, stream));
  return DCC_OK;
}

// Offsets check + max length + write count on the device (one sync).
int dcc_ctx::device_prep(const DevBatch& d, uint32_t& maxlen, uint64_t& nnz_w) {
  dcc_ctx* ctx = this;
  launch_prep(d.off, d.n, d.acctype, d.nnz, (PrepPart*)part.p, stream);
  CK(hipGetLastError());
  CR(read_partials(PREP_BLOCKS * sizeof(PrepPart)));
  CK(hipStreamSynchronize(stream));
  const PrepPart* pp = (const PrepPart*)hpart;
  uint32_t err = 0;
  maxlen = 0;
  nnz_w = 0;
  for (unsigned b = 0; b < PREP_BLOCKS; b++) {
    err |= pp[b].err;
    maxlen = std::max(maxlen, pp[b].maxlen);
    nnz_w += pp[b].nw;
  }
  if (err & ERR_OFFSETS) return fail(DCC_EINVAL, "batch: malformed offsets");
  if (maxlen > MAX_TXN_LEN)
    return fail(DCC_ERANGE, "batch: a txn has %u accesses (> MAX_ROW_PER_TXN=%u)", maxlen,
                MAX_TXN_LEN);
  return DCC_OK;
}

int dcc_ctx::occ_epoch(const dcc_batch* b, uint8_t* out_rc, uint64_t* out_tn, dcc_stats* st) {
  dcc_ctx* ctx = this;
  // key-sharded across ranks: this rank holds only its keys
  const bool sh = comm_ranks() > 1;
  const auto t_wall0 = std::chrono::steady_clock::now();
  CR(check_batch(b));
  const bool dev_out = (b->flags & DCC_DEVICE_PTRS) != 0;
  dcc_stats S;
  memset(&S, 0, sizeof S);
  S.n_shards = (uint32_t)comm_ranks();
  if (b->n_txn == 0) {
    if (st) *st = S;
    return DCC_OK;
  }
  DevBatch d;
  CR(stage_batch(b, d));
  CK(hipEventRecord(ev0, stream));  // device clock starts with the batch resident

  // ---- prep: validation, max length (tile width), write count (table size)
  uint32_t maxlen = 0;
  uint64_t nnz_w = 0;
  CR(device_prep(d, maxlen, nnz_w));
  // txns per wave: build tiles stage TILE_CAP accesses, round tiles ROUND_CAP
  const uint32_t tw_b = std::min<uint32_t>(64, TILE_CAP / std::max<uint32_t>(1, maxlen));
  const uint32_t tw = std::min<uint32_t>(64, ROUND_CAP / std::max<uint32_t>(1, maxlen));
  CR(reserve_occ(d.n, d.nnz, nnz_w, tw));
  const uint64_t cap = table_capacity(nnz_w);
  if (cap > (1ull << 30)) return fail(DCC_ERANGE, "table capacity exceeds 2^30 slots");
  const uint32_t mask = (uint32_t)(cap - 1);
  uint64_t seg_ts, seg_es;
  list_geometry(d.n, tw, seg_ts, seg_es);
  Slot* tab = (Slot*)table.p;
  uint32_t* err = (uint32_t*)misc.p;                                     // [0]
  uint32_t* one = (uint32_t*)misc.p + 1;                                 // constant 1
  uint32_t* kflag = (uint32_t*)((char*)misc.p + 64);                     // CTR_RING flags
  unsigned long long* ring = (unsigned long long*)((char*)misc.p + 512);  // CTR_RING x NSEG
  char* bars = (char*)misc.p + 512 + CTR_RING * NSEG * 8;                 // CTR_RING x 16 B
  uint32_t* und = (uint32_t*)((char*)misc.p + 8192);                      // CTR_RING (sharded)

  CK(hipMemsetAsync(misc.p, 0, 8192 + CTR_RING * 4, stream));
  CK(hipMemsetAsync(one, 0x01, 1, stream));
  CK(hipMemsetAsync(table.p, 0xFF, cap * sizeof(Slot), stream));
  CK(hipMemsetAsync(state.p, 0, d.n, stream));
  uint8_t* gstat = nullptr;
  if (sh) {
    CR(gst.ensure(this, d.n + 16, "shard status"));
    gstat = (uint8_t*)gst.p;
    CK(hipMemsetAsync(gstat, 0, d.n, stream));
  }

  // ---- history window pre-pass (occ.cpp:160-180)
  if (d.start_tn && !hist.empty()) {
    CR(upload_history());
    HistArgs ha{d.n, d.off, d.keys, d.acctype, d.start_tn, d.finish_tn,
                (const uint64_t*)hkeys.p, h_nkeys, (const uint64_t*)hoff.p,
                (const uint64_t*)htn.p, (uint8_t*)state.p};
    launch_hist(ha, stream);
  }
  // the history window is checked on each shard's keys: any shard's abort wins
  if (sh && d.start_tn) CR(comm_allreduce_max_u8((uint8_t*)state.p, d.n));

  // ---- key-hash build: round-1 owners
  BuildArgs ba{d.n, tw_b, d.off, d.keys, d.acctype, tab, mask, (const uint8_t*)state.p,
               (uint8_t*)hasw.p, err};
  if (profiling) CK(hipEventRecord(pev[0], stream));
  launch_build(ba, (unsigned)n_cu * 16, stream);
  CK(hipGetLastError());
  if (sh) CR(comm_allreduce_max_u8((uint8_t*)hasw.p, d.n));  // read-only is a global property
  if (profiling) CK(hipEventRecord(pev[1], stream));

  // ---- fixed-point rounds.  Round k (0-based) reads its list size from the
  // NSEG counters ring[k-1] (device), reserves its output in ring[k] and
  // zeroes ring[k+1]; k_pub republishes owner words before round k+1 only if
  // round k aborted something.  The host enqueues rounds in batches and
  // synchronises once per batch.
  int cur = 0;
  uint32_t rt = 1;  // round tag of the next round
  uint32_t k = 0;   // rounds enqueued
  uint64_t m_bound = d.n;
  uint32_t rounds = 0;
  const unsigned max_grid = (unsigned)n_cu * 8;
  // recheck (kill wave folded into the round) pays off on short lists where
  // per-round fixed costs dominate.  Such rounds keep every workgroup
  // resident for the grid barrier:
  // k_round fits 5 workgroups of 4 waves per CU (LDS ~21 KB, <= 96 VGPRs);
  // launch 4 per CU.
  const unsigned resident_grid = (unsigned)n_cu * 4;
  uint32_t batch = std::min<uint32_t>(2, batch_max);
  bool done = false;
  while (!done) {
    const uint32_t k0 = k;
    for (uint32_t q = 0; q < batch; q++, k++) {
      const bool first = k == 0;
      const unsigned long long* prev = first ? nullptr : &ring[((k - 1) % CTR_RING) * NSEG];
      if (!first) {
        PubArgs pa;
        pa.m_in = prev;
        pa.tw = tw;
        // sharded: always run (committed writers publish their tag-0 words here)
        pa.kill_flag = sh ? one : &kflag[(k - 1) % CTR_RING];
        pa.force = 0;
        pa.state = (const uint8_t*)state.p;
        if (rt > MAX_ROUND_TAG) {
          // tag space exhausted: drop stale owner words, every writer republishes
          launch_retag(tab, cap, stream);
          rt = 1;
          pa.kill_flag = one;
          pa.force = 1;
        }
        pa.r = rt;
        pa.tid = (const uint32_t*)l_tid[cur].p;
        pa.coff = (const uint32_t*)l_coff[cur].p;
        pa.cent = (const uint64_t*)l_cent[cur].p;
        pa.seg_ts = seg_ts;
        pa.seg_es = seg_es;
        pa.tab = tab;
        pa.err = err;
        launch_pub(pa, m_bound, (unsigned)n_cu * 2, stream);
      }
      RoundArgs ra;
      ra.m_in = prev;
      ra.m = d.n;
      ra.tw = tw;
      ra.r = rt;
      ra.k = k + 1;  // 1-based: abort round 0 is the history pre-pass
      ra.end_total = (uint32_t)d.nnz;
      ra.tid = first ? nullptr : (const uint32_t*)l_tid[cur].p;
      ra.coff = first ? d.off : (const uint32_t*)l_coff[cur].p;
      ra.keys = d.keys;
      ra.acctype = d.acctype;
      ra.cent = first ? nullptr : (const uint64_t*)l_cent[cur].p;
      ra.seg_ts = seg_ts;
      ra.seg_es = seg_es;
      ra.tab = tab;
      ra.mask = mask;
      ra.state = (uint8_t*)state.p;
      ra.tid_out = (uint32_t*)l_tid[cur ^ 1].p;
      ra.coff_out = (uint32_t*)l_coff[cur ^ 1].p;
      ra.cent_out = (uint64_t*)l_cent[cur ^ 1].p;
      ra.ctr = &ring[(k % CTR_RING) * NSEG];
      ra.ctr_zero = &ring[((k + 1) % CTR_RING) * NSEG];
      ra.kill_flag = &kflag[k % CTR_RING];
      ra.kill_zero = &kflag[(k + 1) % CTR_RING];
      // m_bound bounds this round's list (lists only shrink)
      const bool recheck = !sh && !first && m_bound <= recheck_max;
      ra.bar = recheck ? (GridBar*)(bars + (k % CTR_RING) * 16) : nullptr;
      ra.bar_zero = (uint32_t*)(bars + ((k + 1) % CTR_RING) * 16);
      ra.gst = gstat;
      ra.err = err;
      launch_round(ra, first, m_bound, recheck ? resident_grid : max_grid, stream);
      if (sh) {
        CR(comm_allreduce_max_u8(gstat, d.n));
        launch_decide((uint8_t*)state.p, gstat, d.n, st_abort(k + 1), &und[k % CTR_RING],
                      &und[(k + 1) % CTR_RING], stream);
      }
      if (profiling && first) CK(hipEventRecord(pev[2], stream));
      cur ^= 1;
      rt++;
    }
    CK(hipGetLastError());
    CK(hipMemcpyAsync(hmisc, ring, CTR_RING * NSEG * 8, hipMemcpyDeviceToHost, stream));
    if (sh) CK(hipMemcpyAsync((char*)hmisc + 8192, und, CTR_RING * 4, hipMemcpyDeviceToHost, stream));
    CK(hipStreamSynchronize(stream));
    const unsigned long long* hr = (const unsigned long long*)hmisc;
    const uint32_t* hu = (const uint32_t*)((const char*)hmisc + 8192);
    for (uint32_t q = k0; q < k; q++) {
      uint64_t mq = 0;
      for (uint32_t g = 0; g < NSEG; g++) mq += hr[(q % CTR_RING) * NSEG + g] >> CTR_E_BITS;
      // sharded: the local list can empty while other shards still decide;
      // the all-reduced undecided count (equal on every rank) ends the loop
      if (sh ? hu[q % CTR_RING] == 0 : mq == 0) {
        rounds = q + 1;
        done = true;
        break;
      }
      m_bound = mq;
    }
    if (!done && k > d.n + 2) return fail(DCC_EIO, "fixed point did not converge");
    batch = std::min<uint32_t>(batch * 2, batch_max);
  }
  if (profiling) CK(hipEventRecord(pev[4], stream));

  // ---- finalize: RC bytes, counts, central_finish tn numbering
  uint8_t* rc_dev = (dev_out && out_rc) ? out_rc : (uint8_t*)rc.p;
  uint32_t* cf = nullptr;
  const bool want_tn = out_tn != nullptr || (b->flags & DCC_OCC_APPEND_HISTORY);
  if (want_tn) {
    CR(cflag.ensure(this, d.n * 4, "cflag"));
    CR(bsum.ensure(this, ((d.n + 1023) / 1024 + 1) * 8, "bsum"));
    CR(tn.ensure(this, d.n * 8, "tn"));
    cf = (uint32_t*)cflag.p;
  }
  FinalArgs fa{d.n, (const uint8_t*)state.p, (const uint8_t*)hasw.p, rc_dev, cf,
               (FinalPart*)part.p};
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
  CK(hipMemcpyAsync(hmisc, misc.p, 64, hipMemcpyDeviceToHost, stream));
  CR(read_partials(FINAL_BLOCKS * sizeof(FinalPart)));
  CK(hipStreamSynchronize(stream));
  const uint32_t e = *(const uint32_t*)hmisc;
  {
    // barrier timeout words (third word of each GridBar in the ring)
    std::vector<uint32_t> bw(CTR_RING * 4);
    CK(hipMemcpy(bw.data(), bars, CTR_RING * 16, hipMemcpyDeviceToHost));
    for (uint32_t q = 0; q < CTR_RING; q++)
      if (bw[q * 4 + 2]) return fail(DCC_EIO, "grid barrier timed out (grid not co-resident)");
  }
  if (e & ERR_KEY) return fail(DCC_EINVAL, "batch: key equal to DCC_KEY_RESERVED");
  if (e & ERR_FULL) return fail(DCC_EIO, "hash table overflow");
  if (e & ERR_TILE) return fail(DCC_EIO, "tile capacity exceeded");
  const FinalPart* fp = (const FinalPart*)hpart;
  uint64_t n_commit = 0, n_abort = 0, n_ro = 0, n_cw = 0, n_und = 0;
  for (unsigned q = 0; q < FINAL_BLOCKS; q++) {
    n_commit += fp[q].commit;
    n_abort += fp[q].abort;
    n_ro += fp[q].readonly;
    n_cw += fp[q].cwriters;
    n_und += fp[q].undecided;
  }
  if (n_und) return fail(DCC_EIO, "%llu undecided transactions after convergence",
                         (unsigned long long)n_und);
  float ms = 0;
  CK(hipEventElapsedTime(&ms, ev0, ev1));
  S.rounds = rounds;
  S.n_commit = n_commit;
  S.n_abort = n_abort;
  S.n_readonly = n_ro;
  S.nnz_w = nnz_w;
  S.alg_bytes = dcc_alg_bytes(d.n, d.nnz, nnz_w);
  S.device_ms = ms;
  if (profiling) {
    float t0 = 0, t1 = 0, t2 = 0;
    CK(hipEventElapsedTime(&t0, pev[0], pev[1]));
    CK(hipEventElapsedTime(&t1, pev[1], pev[2]));
    CK(hipEventElapsedTime(&t2, pev[2], pev[4]));
    S.phase_ms[0] = t0;
    S.phase_ms[1] = t1;
    S.phase_ms[2] = t2;
    S.phase_ms[3] = ms - t0 - t1 - t2;
  }
  // algorithmic bytes per phase: the build reads acctype of
  // every access and the keys of writes, one 16-B slot update per write;
  // round 1 reads offsets, keys + acctype, one 16-B slot per access, state.
  S.phase_bytes[0] = d.nnz + 8 * nnz_w + 16 * nnz_w + 4 * (d.n + 1) + d.n;
  S.phase_bytes[1] = 4 * (d.n + 1) + 9 * d.nnz + 16 * d.nnz + d.n;

  // central_finish (occ.cpp:283-286): committed non-read-only txns take
  // tn = tnc+1, tnc+2, ... in index order; their write sets join the history.
  if (b->flags & DCC_OCC_APPEND_HISTORY) {
    std::vector<uint64_t> htn_host(d.n);
    CK(hipMemcpy(htn_host.data(), tn_dev, d.n * 8, hipMemcpyDeviceToHost));
    std::vector<uint32_t> ho;
    std::vector<uint64_t> hk;
    std::vector<uint8_t> ha;
    const uint32_t* o = b->offsets;
    const uint64_t* kk = b->keys;
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
      kk = hk.data();
      at = ha.data();
    }
    for (uint64_t t = 0; t < d.n; t++) {
      if (!htn_host[t]) continue;
      for (uint32_t x = o[t]; x < o[t + 1]; x++)
        if (at[x] == DCC_WR) hist.emplace_back(kk[x], htn_host[t]);
    }
    if (n_cw) hist_dirty = true;
  }
  tnc += n_cw;
  const auto t_wall1 = std::chrono::steady_clock::now();
  S.total_ms = std::chrono::duration<double, std::milli>(t_wall1 - t_wall0).count();
  if (st) *st = S;
  return DCC_OK;
}
