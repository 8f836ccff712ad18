// OCC epoch driver (host): sizes workspaces, enqueues the gfx950 kernels of
// occ_kernels.hip and synchronises once per batch of rounds.
//
// Reference: OptCC::validate / central_validate / central_finish
// (concurrency_control/occ.cpp:42-327) applied to a whole epoch; the C entry
// point is dcc_occ_validate_epoch (include/dcc.h).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "dcc.h"
#include "dcc_ctx.h"
#include "dcc_device.h"
#include "dcc_env.h"
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
int dcc_ctx::device_prep(const DevBatch& d, uint32_t& maxlen, uint64_t& nnz_w, uint64_t p,
                         uint64_t* nnz_w_prefix) {
  dcc_ctx* ctx = this;
  launch_prep(d.off, d.n, d.acctype, d.nnz, p, (PrepPart*)part.p, stream);
  CK(hipGetLastError());
  CR(read_partials(PREP_BLOCKS * sizeof(PrepPart)));
  CK(hipStreamSynchronize(stream));
  const PrepPart* pp = (const PrepPart*)hpart;
  uint32_t err = 0;
  maxlen = 0;
  nnz_w = 0;
  uint64_t wp = 0;
  for (unsigned b = 0; b < PREP_BLOCKS; b++) {
    err |= pp[b].err;
    maxlen = std::max(maxlen, pp[b].maxlen);
    nnz_w += pp[b].nw;
    wp += pp[b].nw_prefix;
  }
  if (nnz_w_prefix) *nnz_w_prefix = wp;
  if (err & ERR_OFFSETS) return fail(DCC_EINVAL, "batch: malformed offsets");
  if (maxlen > MAX_TXN_LEN)
    return fail(DCC_ERANGE, "batch: a txn has %u accesses (> MAX_ROW_PER_TXN=%u)", maxlen,
                MAX_TXN_LEN);
  return DCC_OK;
}

// misc layout (bytes): [0] error word, [4] constant 1, [64..) kill flags
// (CTR_RING), [512..) round counter ring (CTR_RING x NSEG), then grid barrier
// words (CTR_RING x 16 B), [8192..) sharded undecided counts (CTR_RING).
static constexpr size_t MISC_KFLAG = 64, MISC_RING = 512,
                        MISC_BARS = 512 + CTR_RING * NSEG * 8, MISC_UND = 8192;

// Build + fixed-point rounds for one (sub-)batch: txn i of the sub-batch has
// accesses [off[i], off[i+1]) and state byte state[i]; only UNDECIDED txns
// take part.  Rounds are enqueued in batches with one host synchronisation
// per batch.
int dcc_ctx::occ_rounds(const SubProb& sp, uint32_t maxlen, bool prof, uint32_t& rounds_out) {
  dcc_ctx* ctx = this;
  const bool sh = sharded();
  rounds_out = 0;
  if (sp.n == 0) return DCC_OK;
  // txns per wave: build tiles stage TILE_CAP accesses, round tiles ROUND_CAP
  const uint32_t tw_b = std::min<uint32_t>(64, TILE_CAP / std::max<uint32_t>(1, maxlen));
  const uint32_t tw = std::min<uint32_t>(64, ROUND_CAP / std::max<uint32_t>(1, maxlen));
  CR(reserve_occ(sp.n, 0, sp.w_bound, tw));
  const uint64_t cap = table_capacity(sp.w_bound);
  if (cap > (1ull << 30)) return fail(DCC_ERANGE, "table capacity exceeds 2^30 slots");
  const uint32_t mask = (uint32_t)(cap - 1);
  uint64_t seg_ts, seg_es;
  list_geometry(sp.n, tw, seg_ts, seg_es);
  Slot* tab = (Slot*)table.p;
  char* mb = (char*)misc.p;
  uint32_t* err = (uint32_t*)mb;
  uint32_t* one = (uint32_t*)mb + 1;
  uint32_t* kflag = (uint32_t*)(mb + MISC_KFLAG);
  unsigned long long* ring = (unsigned long long*)(mb + MISC_RING);
  char* bars = mb + MISC_BARS;
  uint32_t* und = (uint32_t*)(mb + MISC_UND);
  CK(hipMemsetAsync(mb + MISC_KFLAG, 0, MISC_UND + CTR_RING * 4 - MISC_KFLAG, stream));
  CK(hipMemsetAsync(table.p, 0xFF, cap * sizeof(Slot), stream));
  uint8_t* gstat = nullptr;
  if (sh) {
    CR(gst.ensure(this, sp.n + 16, "shard status"));
    gstat = (uint8_t*)gst.p;
    CK(hipMemsetAsync(gstat, 0, sp.n, stream));
  }

  // ---- key-hash build: round-1 owners
  BuildArgs ba{sp.n, tw_b, sp.off, sp.keys, sp.acctype, tab, mask, sp.state, sp.hasw, err};
  if (prof) CK(hipEventRecord(pev[0], stream));
  launch_build(ba, (unsigned)n_cu * 16, stream);
  CK(hipGetLastError());
  if (sh && sp.hasw_global) CR(comm_allreduce_max_u8(sp.hasw, sp.n));  // global property
  if (prof) CK(hipEventRecord(pev[1], stream));

  // ---- fixed-point rounds.  Round k (0-based) reads its list size from the
  // NSEG counters ring[k-1] (device), reserves its output in ring[k] and
  // zeroes ring[k+1]; k_pub republishes owner words before round k+1 only if
  // round k aborted something.  The host enqueues rounds in batches and
  // synchronises once per batch.
  int cur = 0;
  uint32_t rt = 1;  // round tag of the next round
  uint32_t k = 0;   // rounds enqueued
  uint64_t m_bound = sp.n;
  uint32_t rounds = 0;
  const unsigned max_grid = (unsigned)n_cu * 8;
  // recheck (kill wave folded into the round) pays off on short lists where
  // per-round fixed costs dominate.  Such rounds keep every workgroup
  // resident for the grid barrier:
  // k_round fits 5 workgroups of 4 waves per CU (LDS ~21 KB, <= 96 VGPRs);
  // launch 4 per CU.
  const unsigned resident_grid = (unsigned)n_cu * 4;
  uint32_t batch = std::min<uint32_t>(sp.n > 65536 ? 2 : 4, batch_max);
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
        pa.state = sp.state;
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
      ra.m = sp.n;
      ra.tw = tw;
      ra.r = rt;
      ra.k = k + 1;  // 1-based: abort round 0 is the history pre-pass
      ra.end_total = 0;  // identity lists read off[m]; later lists carry counters
      ra.tid = first ? nullptr : (const uint32_t*)l_tid[cur].p;
      ra.coff = first ? sp.off : (const uint32_t*)l_coff[cur].p;
      ra.keys = sp.keys;
      ra.acctype = sp.acctype;
      ra.cent = first ? nullptr : (const uint64_t*)l_cent[cur].p;
      ra.seg_ts = seg_ts;
      ra.seg_es = seg_es;
      ra.tab = tab;
      ra.mask = mask;
      ra.state = sp.state;
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
      bars_used |= recheck;
      ra.bar_zero = (uint32_t*)(bars + ((k + 1) % CTR_RING) * 16);
      ra.gst = gstat;
      ra.err = err;
      launch_round(ra, first, m_bound, recheck ? resident_grid : max_grid, stream);
      if (sh) {
        CR(comm_allreduce_max_u8(gstat, sp.n));
        launch_decide(sp.state, gstat, sp.n, st_abort(k + 1), &und[k % CTR_RING],
                      &und[(k + 1) % CTR_RING], stream);
      }
      if (prof && first) CK(hipEventRecord(pev[2], stream));
      cur ^= 1;
      rt++;
    }
    CK(hipGetLastError());
    CK(hipMemcpyAsync(hmisc, ring, CTR_RING * NSEG * 8, hipMemcpyDeviceToHost, stream));
    if (sh) CK(hipMemcpyAsync((char*)hmisc + MISC_UND, und, CTR_RING * 4, hipMemcpyDeviceToHost, stream));
    CK(hipStreamSynchronize(stream));
    const unsigned long long* hr = (const unsigned long long*)hmisc;
    const uint32_t* hu = (const uint32_t*)((const char*)hmisc + MISC_UND);
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
    if (!done && k > sp.n + 2) return fail(DCC_EIO, "fixed point did not converge");
    batch = std::min<uint32_t>(batch * 2, batch_max);
  }
  if (prof) CK(hipEventRecord(pev[4], stream));
  rounds_out = rounds;
  return DCC_OK;
}

// ---------------------------------------------------------------------------
// Sweep solver (occ_sweep.hip): per level, tile records + one serial pass in
// one CU + a filter/compaction pass; levels are enqueued without host
// synchronisation (list lengths live on the device), sw_levels at a time.
static constexpr size_t SW_PREP_OFF = 32768;  // prep partials inside `part` / `hpart`
static constexpr size_t SW_HCTL = 13312;      // control-block copy inside `hmisc`
static constexpr uint32_t SW_PMAX_TOP = 65536;
                                                          // the serial pass's LDS set)
// the serial prefixes per level: 1,024 txns at level 0; with the read-only
// split (lists of write txns only after level 0) 3,072 and 8,192 next, so the
// headline epoch ends in three levels (tools/sweep_model.py, measured A/B in
// DESIGN.md §3); without it 1,024 << level.  mode: 0 no split, 1 split (three
// levels per graph), 2 split with two levels per graph -- level 1 a serial
// tail of 8,192, for epochs whose level-1 list fits it (C2, C3: the last
// epoch's list decides, dcc_ctx::sw_l1_last)
static uint32_t sw_pmax(int level, int mode) {
  // DCC_SW_PMAX="p0,p1,...": per-level serial prefixes (tuning experiments)
  static const std::vector<uint32_t> ov = [] {
    std::vector<uint32_t> v;
    if (const char* e = DCC_ENV("DCC_SW_PMAX"))
      for (const char* c = e; *c;) {
        char* x;
        const unsigned long p = strtoul(c, &x, 10);
        if (x == c) break;
        v.push_back((uint32_t)std::min<unsigned long>(std::max<unsigned long>(p, SW_T), SW_PMAX_TOP));
        c = *x ? x + 1 : x;
      }
    return v;
  }();
  if (level < (int)ov.size()) return ov[level];
  if (mode == 2) {
    if (level == 0) return 1024u;
    return level >= 4 ? SW_PMAX_TOP : (8192u << (level - 1));
  }
  if (mode) {
    if (level == 0) return 1024u;
    if (level == 1) return 3072u;
    return level >= 5 ? SW_PMAX_TOP : (8192u << (level - 2));
  }
  return level >= 6 ? SW_PMAX_TOP : (1024u << level);
}
static size_t sw_ctl_bytes() { return (SW_MAX_LEVEL + 2) * sizeof(SwLevel) + 64; }
// the access budget of a level's serial range: a quarter of the smallest
// table with four slots per access of p_max 16-access txns
static uint32_t sw_budget_bits(int level, int mode) {
  uint32_t b = 12;
  while (b < SW_GBITS_MAX && (1ull << b) < 4ull * sw_pmax(level, mode) * 16) b++;
  return b;
}
static uint32_t sw_budget(int level, int mode) { return 1u << (sw_budget_bits(level, mode) - 2); }
// key-table slots of a level: sparse (2^18 at level 0, 2^19 after; the
// DCC_SW_GBITS override for experiments), so a pre-pass workgroup's ~500
// first inserts almost never meet another key at their first slot -- each
// lost slot is one more dependent round trip for the whole workgroup
static uint32_t sw_gbits(int level, int mode) {
  static const int ov = [] {
    const char* c = DCC_ENV("DCC_SW_GBITS");
    return c ? atoi(c) : 0;
  }();
  uint32_t b = ov > 0 ? (uint32_t)ov : (level == 0 ? 18u : 19u);
  b = std::max(b, sw_budget_bits(level, mode));
  return std::min<uint32_t>(b, SW_GBITS_MAX);
}

int dcc_ctx::sweep_reserve(const DevBatch& d) {
  const uint64_t tiles = SW_PMAX_TOP / SW_T;
  sw_debug = DCC_ENV("DCC_SW_DEBUG") != nullptr;
  if (sw_debug) {
    CR(sw_dbg.ensure(this, (4096 + 4 * 256 * 8 + 4 * 64 * 8) * 8, "sweep debug"));
    dcc_ctx* ctx = this;
    CK(hipMemsetAsync(sw_dbg.p, 0, (4096 + 4 * 256 * 8 + 4 * 64 * 8) * 8, stream));
  }
  CR(sw_ctl.ensure(this, sw_ctl_bytes(), "sweep control"));
  CR(sw_status.ensure(this, ((d.n + 63) / 64 + 64) * 16 + (4ull * n_cu + 64) * 8,
                        "sweep survivor bits + tile counts"));
  CR(sw_ckeys.ensure(this, ((1ull << SW_GBITS_MAX) / 32 + (1ull << SW_BLOOM_LOG) / 32) * 4 +
                                (1ull << SW_GBITS_MAX) * 8,
                     "sweep committed set"));
  CR(sw_rec.ensure(this, tiles * sizeof(SwRec), "sweep tile records"));
  CR(sw_rk.ensure(this, tiles * SW_OVF * 4, "sweep tile-list overflow"));
  CR(sw_gtab.ensure(this, 2 * (1ull << SW_GBITS_MAX) * 8, "sweep key tables"));
  CR(sw_fw.ensure(this, 2 * (1ull << SW_GBITS_MAX) * 4, "sweep first writer / last accessor"));
  CR(sw_aent.ensure(this, 2 * (1ull << (SW_GBITS_MAX - 1)) * 4, "sweep access entries"));
  CR(sw_mg.ensure(this, SW_PMAX_TILES * 8, "sweep tile commit masks"));
  if (ro_on) {
    const uint64_t n64 = (d.n + 63) / 64 + 32;
    CR(sw_rflag.ensure(this, (2 * n64 + 4ull * n_cu + 64) * 8, "sweep read-only survivor bits"));
    CR(sw_ro.ensure(this, d.n * sizeof(RoEnt) + 64, "sweep read-only list"));
    CR(sw_wtab.ensure(this, sizeof(WrSlot) << wt_bits, "committed-writer table"));
    CR(sw_cw.ensure(this, d.n * 4 + 64, "committed writers"));
  }
  for (SubBufs& b : sw_list) {
    CR(b.tid.ensure(this, d.n * 4 + 16, "sweep list tid"));
    CR(b.off.ensure(this, (d.n + 1) * 4 + 16, "sweep list offsets"));
    CR(b.keys.ensure(this, std::max<uint64_t>(8, d.nnz * 8), "sweep list keys"));
    CR(b.acctype.ensure(this, std::max<uint64_t>(16, d.nnz), "sweep list acctype"));
    CR(b.state.ensure(this, d.n + 16, "sweep list state"));
  }
  return DCC_OK;
}

// Enqueue levels [l0, l1) (list l0 must exist: the epoch, or written by the
// filter of level l0 - 1).
int dcc_ctx::sweep_enqueue(const DevBatch& d, int l0, int l1, const SwShard* shl, bool resume,
                           bool tail_serial) {
  dcc_ctx* ctx = this;
  SwLevel* ctl = (SwLevel*)sw_ctl.p;
  uint32_t* abandon = (uint32_t*)(ctl + SW_MAX_LEVEL + 1);
  uint32_t* err = (uint32_t*)misc.p;
  const uint32_t n = (uint32_t)d.n;
  // the filter / compaction grid: four workgroups per CU whatever the epoch's
  // size -- besides its tiles the filter clears the next level's key table
  // and first-writer / last-accessor words (8 MB at 2^19 slots), which on a
  // small epoch's grid (C2: 256 workgroups) would otherwise be spread over a
  // quarter of the CUs; the workgroups past the tiles clear and leave
  // (measured neutral on C2, 0.132 ms either way: the clears overlap)
  static const unsigned fgrid_ov = [] {  // DCC_SW_FGRID: experiments
    const char* e = DCC_ENV("DCC_SW_FGRID");
    return e ? (unsigned)atoi(e) : 0u;
  }();
  const unsigned fgrid = fgrid_ov ? fgrid_ov : (unsigned)std::max<uint64_t>(1, 4ull * n_cu);
  static const unsigned fgrid1_ov = [] {  // DCC_SW_FGRID1: experiments, the levels after 0
    const char* e = DCC_ENV("DCC_SW_FGRID1");
    return e ? (unsigned)atoi(e) : 0u;
  }();
  uint64_t* gtab0 = (uint64_t*)sw_gtab.p;
  uint32_t* cbits_d = (uint32_t*)sw_ckeys.p;
  uint32_t* bloom_d = cbits_d + (1u << SW_GBITS_MAX) / 32;
  uint64_t* ckeys_d = (uint64_t*)(bloom_d + (1u << SW_BLOOM_LOG) / 32);
  const uint64_t n64 = (d.n + 63) / 64;
  uint64_t* sflag_d = (uint64_t*)sw_status.p;
  unsigned long long* tcount_d = (unsigned long long*)(sflag_d + n64 + 32);
  unsigned long long* bsum_d = tcount_d + n64 + 32;
  // read-only split (one GPU): level 0 moves its read-only survivors to the
  // RO list (decided after the levels, sweep_ro)
  const bool ros = ro_on && (!shl || shl->full_off);
  const int rmode = ros ? (int)sw_mode : 0;  // the schedule (sw_pmax)
  uint32_t* const wctl = abandon;  // [0] abandon [1] writer table full [2] RO count
  for (int l = l0; l < l1; l++) {
    const bool top = l == 0;
    SwList in;
    if (top) {
      in = SwList{nullptr, d.off, d.keys, d.acctype, d.nnz};
    } else {
      const SubBufs& b = sw_list[(l - 1) & 1];
      in = SwList{(const uint32_t*)b.tid.p, (const uint32_t*)b.off.p, (const uint64_t*)b.keys.p,
                  (const uint8_t*)b.acctype.p, d.nnz};
    }
    SubBufs& out = sw_list[l & 1];
    SwLevel* lv = ctl + l;
    const uint32_t* mdev = top ? nullptr : &lv->m;
    const uint32_t pmax = sw_pmax(l, rmode);
    const uint64_t tiles = (std::min<uint64_t>(pmax, d.n) + SW_T - 1) / SW_T;
    uint32_t* fw = (uint32_t*)sw_fw.p;
    uint32_t* la = fw + (1u << SW_GBITS_MAX);
    uint32_t* aent = (uint32_t*)sw_aent.p;
    uint32_t* apos = aent + (1u << (SW_GBITS_MAX - 1));
    // key-sharded: the serial part runs on the merged serial range (every
    // shard's accesses of list txns [0, P)), identically on every rank
    const SwList sin = shl ? shl->serial : in;
    const uint32_t* smdev = shl ? shl->m_dev : mdev;
    const uint32_t sm_host = (shl && !shl->m_dev) ? shl->P : n;
    SwPreArgs pa{sin, smdev, sm_host, pmax, top ? (const uint8_t*)state.p : nullptr,
                 (SwRec*)sw_rec.p, (uint32_t*)sw_rk.p,
                 gtab0 + (size_t)(l & 1) * (1ull << SW_GBITS_MAX), sw_gbits(l, rmode),
                 sw_budget(l, rmode), fw, la, aent, apos, abandon, err, nullptr};
    if (sw_debug && l < 4) pa.dbg = (uint64_t*)sw_dbg.p + 4096 + 4 * 256 * 8 + (size_t)l * 64 * 8;
    const bool serial_part = !(resume && l == l0);
    if (serial_part) {
      launch_sw_pre(pa, (unsigned)tiles, stream);
      launch_sw_rows(pa, (unsigned)tiles, stream);
    }
    SwSeqArgs sa{smdev, sm_host, pmax, top ? 1 : 0, (const SwRec*)sw_rec.p, (const uint32_t*)sw_rk.p,
                 gtab0 + (size_t)(l & 1) * (1ull << SW_GBITS_MAX), sw_gbits(l, rmode),
                 (uint8_t*)state.p, (uint8_t*)hasw.p,
                 cbits_d, ckeys_d, bloom_d, lv, lv + 1, (uint32_t*)out.off.p, (uint64_t*)sw_mg.p,
                 abandon, err, nullptr};
    if (sw_debug && l < 4) sa.dbg = (uint64_t*)sw_dbg.p + (size_t)l * 1024;
    if (ros) {
      sa.cw_list = (uint32_t*)sw_cw.p;
      sa.cw_count = wctl + 4;
    }
    if (serial_part) launch_sw_seq(sa, stream);
    // the last level of a graph-captured epoch usually decides its whole list
    // serially: its listing, filter and compaction are enqueued only when the
    // host finds list txns past the serial range (occ_epoch)
    if (tail_serial && l == l1 - 1) break;
    SwCoutArgs ca{sin,     aent,    apos,    (const uint64_t*)sw_mg.p, lv, cbits_d, ckeys_d,
                  bloom_d, abandon, smdev, sm_host, shl ? 0 : 1};
    if (top && serial_part) {  // the epoch's validation pass rides along the level-0 listing
      // (a rank holding the whole batch takes its has-write bytes from it)
      const bool whole = shl && shl->full_off;
      ca.prep_off = whole ? shl->full_off : d.off;
      ca.prep_n = d.n;
      ca.prep_at = whole ? shl->full_at : d.acctype;
      ca.prep_nnz = whole ? shl->full_nnz : d.nnz;
      ca.prep_part = (PrepPart*)((char*)hpart_dev + SW_PREP_OFF);
      ca.hasw = (uint8_t*)hasw.p;
      ca.prep_err = err;
      if (ros) {
        ca.wclear = (uint4*)sw_wtab.p;
        ca.wclear_n16 = (sizeof(WrSlot) << wt_bits) / 16;
      }
    }
    launch_sw_cout(ca, (unsigned)std::min<uint64_t>((pa.budget + 1023) / 1024, 4ull * n_cu), stream);
    SwFilterArgs fa;
    fa.in = in;
    fa.m_dev = mdev;
    fa.m_host = n;
    fa.cand_state = top ? 1 : 0;
    fa.level = (uint32_t)l;
    fa.gtab = gtab0 + (size_t)(l & 1) * (1ull << SW_GBITS_MAX);
    fa.gbits = sw_gbits(l, rmode);
    fa.cbits = cbits_d;
    fa.bloom = bloom_d;
    fa.ckeys = ckeys_d;
    fa.sflag = sflag_d;
    fa.tcount = tcount_d;
    fa.bsum = bsum_d;
    const unsigned lgrid = (!top && fgrid1_ov) ? std::min(fgrid1_ov, fgrid) : fgrid;
    fa.nblocks = lgrid;
    fa.lv = lv;
    fa.lv_next = lv + 1;
    fa.state = (uint8_t*)state.p;
    fa.hasw = (uint8_t*)hasw.p;
    fa.tid_out = (uint32_t*)out.tid.p;
    fa.off_out = (uint32_t*)out.off.p;
    fa.keys_out = (uint64_t*)out.keys.p;
    fa.acc_out = (uint8_t*)out.acctype.p;
    fa.abandon = abandon;
    fa.abandon_out = abandon;
    // hand the survivors to the round solver when the committed keys stop
    // killing: > 1/4 of the epoch survive level 0, > 3/4 of a later list
    fa.abandon_min = 65536;
    fa.abandon_num = top ? 1 : 3;
    fa.abandon_den = 4;
    fa.gclear = gtab0 + (size_t)((l + 1) & 1) * (1ull << SW_GBITS_MAX);
    fa.gclear_n = 1ull << sw_gbits(l + 1, rmode);
    fa.fw_clear = fw;
    fa.la_clear = la;
    fa.err = err;
    fa.dbg = (sw_debug && l < 4) ? (uint64_t*)sw_dbg.p + 4096 + (size_t)l * 256 * 8 : nullptr;
    fa.cdbg = pa.dbg ? pa.dbg + 32 : nullptr;
    fa.kill_out = shl ? shl->kill_out : nullptr;
    fa.kill_in = shl ? shl->kill_all : nullptr;
    fa.kill_ranks = shl ? (uint32_t)comm_ranks() : 0u;
    fa.kill_stride = shl ? shl->kill_words : 0u;
    fa.ro_split = (ros && top) ? 1 : 0;
    fa.rflag = (uint64_t*)sw_rflag.p;
    fa.rtcount = (unsigned long long*)(fa.rflag + n64 + 32);
    fa.rbsum = fa.rtcount + n64 + 32;
    fa.ro_out = (RoEnt*)sw_ro.p;
    fa.ro_count = wctl + 2;
    // phase 1 of the profile is exactly the level-0 streaming filter
    if (top && profiling) CK(hipEventRecord(pev[1], stream));
    launch_sw_filter(fa, lgrid, stream);
    if (top && profiling) CK(hipEventRecord(pev[2], stream));
    if (shl) {
      // a kill on any shard wins (every rank's kill words gathered, OR-ed by
      // k_sw_apply); then every rank applies the same decision.  The has-write
      // bytes are global already when the rank holds the whole batch.
      CR(comm_allgather_u8((const uint8_t*)shl->kill_out, (uint8_t*)shl->kill_all, shl->kill_words * 8));
      if (top && !shl->full_off) CR(comm_allreduce_max_u8((uint8_t*)hasw.p, d.n));
      launch_sw_apply(fa, lgrid, stream);
    }
    launch_sw_compact(fa, lgrid, stream);
  }
  CK(hipGetLastError());
  return DCC_OK;
}

// Key-sharded sweep: levels one at a time.  Per level: the
// list length and this rank's share of the serial range, an all-gather of the
// shares' sizes and then of the records themselves (a byte-wise MAX
// all-reduce over a zeroed buffer in which each rank fills its slot), the
// merged serial range, then sweep_enqueue with the filter in kill-bit mode.
// On return next_level is the first level not run; its list is empty, or
// handed off (abandon), or left to the round solver.
int dcc_ctx::sweep_sharded(const DevBatch& d, int& next_level) {
  dcc_ctx* ctx = this;
  const int R = comm_ranks(), me = comm_rank();
  SwLevel* ctl = (SwLevel*)sw_ctl.p;
  const uint32_t* abandon = (const uint32_t*)(ctl + SW_MAX_LEVEL + 1);
  CR(sw_xcnt.ensure(this, 64ull * R + 64, "sweep exchange counts"));
  for (int l = 0; l < SW_MAX_LEVEL - 1; l++) {
    next_level = l;
    const bool top = l == 0;
    SwList in;
    if (top) {
      in = SwList{nullptr, d.off, d.keys, d.acctype, d.nnz};
    } else {
      const SubBufs& b = sw_list[(l - 1) & 1];
      in = SwList{(const uint32_t*)b.tid.p, (const uint32_t*)b.off.p, (const uint64_t*)b.keys.p,
                  (const uint8_t*)b.acctype.p, d.nnz};
    }
    // (1) one size exchange per level: the list length and abandon word
    // (alike on every rank) and each rank's accesses of the serial range
    uint32_t* cnt = (uint32_t*)sw_xcnt.p;
    CK(hipMemsetAsync(cnt, 0, 4ull * (R + 2), stream));
    launch_sw_share(top ? nullptr : &ctl[l].m, (uint32_t)d.n, abandon, top ? d.off : in.off,
                    sw_pmax(l, 0), (uint32_t)me, cnt, stream);
    CR(comm_allreduce_max_u8((uint8_t*)cnt, 4ull * (R + 2)));
    std::vector<uint32_t> hc(R + 2);
    CK(hipMemcpyAsync(hc.data(), cnt, 4ull * (R + 2), hipMemcpyDeviceToHost, stream));
    CK(hipStreamSynchronize(stream));
    const uint32_t m = hc[0];
    if (hc[1]) return DCC_OK;  // an earlier level handed off
    if (m == 0) return DCC_OK;
    const uint32_t P = std::min<uint32_t>(sw_pmax(l, 0), m);
    const uint32_t* share = hc.data() + 2;
    uint64_t total = 0, before = 0;
    for (int r = 0; r < R; r++) {
      if (r < me) before += share[r];
      total += share[r];
    }
    // (3) the records, all-gathered (ncclAllGather of every rank's share,
    // padded to the largest); merged by txn into one CSR
    uint32_t maxshare = 0;
    for (int r = 0; r < R; r++) maxshare = std::max(maxshare, share[r]);
    const uint64_t chunk = std::max<uint64_t>(1, maxshare) * 12;
    CR(sw_xsend.ensure(this, chunk, "sweep exchange send"));
    CR(sw_xrec.ensure(this, chunk * R, "sweep exchange records"));
    CR(sw_mcnt.ensure(this, 8ull * (P + 1) + 64, "sweep merge counts"));
    CR(sw_moff.ensure(this, 4ull * (P + 1) + 64, "sweep merged offsets"));
    CR(sw_mkeys.ensure(this, std::max<uint64_t>(64, total * 8), "sweep merged keys"));
    CR(sw_mat.ensure(this, std::max<uint64_t>(64, total), "sweep merged types"));
    // kill words: one per 64 list positions past where the serial pass
    // stopped (at most P, earlier when its access budget ran out)
    const uint64_t kw = (m + 63) / 64 + 1;
    CR(sw_kill.ensure(this, kw * 8 * (R + 1) + 64, "sweep kill bits"));
    uint32_t* xrec = (uint32_t*)sw_xrec.p;
    uint32_t* mcnt = (uint32_t*)sw_mcnt.p;
    CK(hipMemsetAsync(sw_xsend.p, 0xFF, chunk, stream));
    CK(hipMemsetAsync(mcnt, 0, 4ull * (P + 1), stream));
    launch_sw_merge(in, P, (uint32_t*)sw_xsend.p, 0, 0, nullptr, nullptr, nullptr, nullptr,
                    nullptr, true, stream);
    CR(comm_allgather_u8((const uint8_t*)sw_xsend.p, (uint8_t*)xrec, chunk));
    (void)before;
    launch_sw_merge(in, P, xrec, 0, (uint32_t)(R * (chunk / 12)), mcnt, mcnt + (P + 1),
                    (uint32_t*)sw_moff.p, (uint64_t*)sw_mkeys.p, (uint8_t*)sw_mat.p, false, stream);
    CK(hipGetLastError());
    SwShard shl{};
    shl.serial = SwList{top ? nullptr : in.tid, (const uint32_t*)sw_moff.p,
                        (const uint64_t*)sw_mkeys.p, (const uint8_t*)sw_mat.p, total};
    shl.P = P;
    shl.kill_out = (uint64_t*)sw_kill.p;
    shl.kill_all = (uint64_t*)sw_kill.p + kw;
    shl.kill_words = kw;
    CR(sweep_enqueue(d, l, l + 1, &shl));
  }
  next_level = SW_MAX_LEVEL - 1;
  return DCC_OK;
}


// Key-sharded sweep, every rank holding the whole batch (DCC_SHARD_SELF):
// the serial part of a level needs the whole access lists of the level's first
// txns, which every rank gathers from its copy of the batch
// (launch_sw_sgather) instead of exchanging records, so the ranks exchange
// only the filters' kill bits -- one all-gather of fixed size per level (the
// list's bound: the epoch at level 0, then the hand-off thresholds), with
// every list length on the device.  The levels are enqueued with no host
// synchronisation; the read-only split applies as on one GPU (every rank
// decides the read-only list from the whole batch).  Levels [0, L) are
// enqueued; next_level = L.
int dcc_ctx::sweep_sharded_full(const DevBatch& d, const DevBatch& full, int l0, int L) {
  dcc_ctx* ctx = this;
  const int R = comm_ranks();
  SwLevel* ctl = (SwLevel*)sw_ctl.p;
  uint32_t* err = (uint32_t*)misc.p;
  // kill-word capacity per level: list l holds at most cap[l] txns (the
  // compaction hands a list to the round solver past max(abandon_min, 1/4 of
  // the epoch) at level 0 and max(abandon_min, 3/4 of the list) later)
  uint64_t cap = d.n, wmax = 0;
  std::vector<uint64_t> words(std::max(L, 1));
  for (int l = 0; l < L; l++) {
    words[l] = (cap + 63) / 64 + 1;
    wmax = std::max(wmax, words[l]);
    cap = std::min<uint64_t>(cap, std::max<uint64_t>(65536, l == 0 ? (cap + 3) / 4 : (cap * 3 + 3) / 4));
  }
  CR(sw_kill.ensure(this, wmax * 8 * (R + 1) + 64, "sweep kill bits"));
  const uint32_t pm = sw_pmax(SW_MAX_LEVEL - 1, ro_on ? (int)sw_mode : 0);
  CR(sw_moff.ensure(this, 4ull * (std::min<uint64_t>(pm, d.n) + 1) + 64, "sweep serial offsets"));
  CR(sw_mkeys.ensure(this, 8ull * std::min<uint64_t>(pm, d.n) * MAX_TXN_LEN + 64, "sweep serial keys"));
  CR(sw_mat.ensure(this, std::min<uint64_t>(pm, d.n) * MAX_TXN_LEN + 64, "sweep serial types"));
  for (int l = l0; l < L; l++) {
    SwShard shl{};
    if (l == 0) {
      shl.serial = SwList{nullptr, full.off, full.keys, full.acctype, full.nnz};
      shl.P = (uint32_t)d.n;
    } else {
      const SubBufs& b = sw_list[(l - 1) & 1];
      launch_sw_sgather((const uint32_t*)b.tid.p, &ctl[l].m, sw_pmax(l, ro_on ? (int)sw_mode : 0), full.off, full.keys,
                        full.acctype, full.nnz, (uint32_t*)sw_moff.p, (uint64_t*)sw_mkeys.p,
                        (uint8_t*)sw_mat.p, err, stream);
      CK(hipGetLastError());
      shl.serial = SwList{(const uint32_t*)b.tid.p, (const uint32_t*)sw_moff.p, (const uint64_t*)sw_mkeys.p,
                          (const uint8_t*)sw_mat.p, std::min<uint64_t>(pm, d.n) * MAX_TXN_LEN};
      shl.m_dev = &ctl[l].m;
    }
    shl.kill_out = (uint64_t*)sw_kill.p;
    shl.kill_all = (uint64_t*)sw_kill.p + wmax;
    shl.kill_words = words[l];
    shl.full_off = full.off;
    shl.full_at = full.acctype;
    shl.full_nnz = full.nnz;
    CR(sweep_enqueue(d, l, l + 1, &shl));
  }
  return DCC_OK;
}

// ---------------------------------------------------------------------------
// Deferred central_finish (DCC_OCC_DEFER_FINISH): the decided epoch is kept --
// its local state and has-write bytes, and the batch itself when it was a
// host batch (the staging buffers belong to the next call) -- until
// dcc_occ_finish_epoch brings the global RC.
int dcc_ctx::fin_save(const DevBatch& d, bool host_batch, uint64_t nnz_w) {
  dcc_ctx* ctx = this;
  CR(fin_state.ensure(this, d.n + 16, "deferred finish state"));
  CR(fin_hasw.ensure(this, d.n + 16, "deferred finish has-write"));
  CK(hipMemcpyAsync(fin_state.p, state.p, d.n, hipMemcpyDeviceToDevice, stream));
  CK(hipMemcpyAsync(fin_hasw.p, hasw.p, d.n, hipMemcpyDeviceToDevice, stream));
  fin_d = d;
  // the batch must outlive this call: a host batch sits in the staging
  // buffers of the next call, and a multi-GPU rank's shard (a "device" batch
  // in this context's own sh_* buffers) is rewritten by the next epoch of any
  // kind (e.g. a Calvin epoch before dcc_occ_finish_epoch) -- copy both
  // -- and so is a device batch in compact form, whose widened keys / access
  // types sit in this context's staging buffers
  const bool own = d.off == (const uint32_t*)sh_off.p || d.keys == (const uint64_t*)sh_keys.p ||
                   d.off == (const uint32_t*)off.p || d.keys == (const uint64_t*)keys.p ||
                   d.acctype == (const uint8_t*)acctype.p;
  if (host_batch || own) {
    CR(fin_off.ensure(this, (d.n + 1) * 4, "deferred finish offsets"));
    CR(fin_keys.ensure(this, std::max<uint64_t>(8, d.nnz * 8), "deferred finish keys"));
    CR(fin_at.ensure(this, std::max<uint64_t>(16, d.nnz), "deferred finish types"));
    CK(hipMemcpyAsync(fin_off.p, d.off, (d.n + 1) * 4, hipMemcpyDeviceToDevice, stream));
    if (d.nnz) {
      CK(hipMemcpyAsync(fin_keys.p, d.keys, d.nnz * 8, hipMemcpyDeviceToDevice, stream));
      CK(hipMemcpyAsync(fin_at.p, d.acctype, d.nnz, hipMemcpyDeviceToDevice, stream));
    }
    fin_d.off = (const uint32_t*)fin_off.p;
    fin_d.keys = (const uint64_t*)fin_keys.p;
    fin_d.acctype = (const uint8_t*)fin_at.p;
  }
  CK(hipStreamSynchronize(stream));
  fin_nnz_w = nnz_w;
  fin_pending = true;
  return DCC_OK;
}

// Two phases, so a multi-GPU context can check every rank before any rank
// changes state: prepare (allocations, the finish flags, the tn numbering and
// the bad-vote check -- device scratch only) and commit (the history append,
// tnc, the tn copy-out).
int dcc_ctx::occ_finish_prepare(const uint8_t* final_rc, uint32_t flags, uint32_t& n_cw) {
  dcc_ctx* ctx = this;
  n_cw = 0;
  if (!fin_pending) return fail(DCC_EINVAL, "no epoch awaits dcc_occ_finish_epoch");
  const uint64_t n = fin_d.n;
  if (n == 0) return DCC_OK;
  if (!final_rc) return fail(DCC_EINVAL, "null final_rc");
  const bool dev = (flags & DCC_DEVICE_PTRS) != 0;
  const uint8_t* frc = final_rc;
  if (!dev) {
    CR(fin_rc.ensure(this, n + 16, "final rc"));
    CK(hipMemcpyAsync(fin_rc.p, final_rc, n, hipMemcpyHostToDevice, stream));
    frc = (const uint8_t*)fin_rc.p;
  }
  CR(cflag.ensure(this, n * 4, "cflag"));
  CR(bsum.ensure(this, ((n + 1023) / 1024 + 1) * 8, "bsum"));
  CR(tn.ensure(this, n * 8, "tn"));
  CR(fin_cnt.ensure(this, 64, "finish counts"));
  CK(hipMemsetAsync(fin_cnt.p, 0, 8, stream));
  launch_finish_flags(frc, (const uint8_t*)fin_state.p, (const uint8_t*)fin_hasw.p, n,
                      (uint32_t*)cflag.p, (uint32_t*)fin_cnt.p, stream);
  launch_commit_tn((const uint32_t*)cflag.p, n, (uint64_t*)bsum.p, tnc, (uint64_t*)tn.p, stream);
  CK(hipGetLastError());
  CK(hipMemcpyAsync(hmisc, fin_cnt.p, 8, hipMemcpyDeviceToHost, stream));
  CK(hipStreamSynchronize(stream));
  n_cw = ((const uint32_t*)hmisc)[0];
  const uint32_t bad = ((const uint32_t*)hmisc)[1];
  if (bad)
    return fail(DCC_EINVAL, "final_rc: %u txns with global RCOK aborted locally (2PC never commits them)",
                bad);
  return DCC_OK;
}

int dcc_ctx::occ_finish_commit(uint32_t n_cw, uint64_t* out_tn, uint32_t flags) {
  dcc_ctx* ctx = this;
  const uint64_t n = fin_d.n;
  if (n) {
    CR(hist_append_epoch(fin_d, (const uint64_t*)tn.p, fin_nnz_w, n_cw));
    tnc += n_cw;
    if (out_tn) {
      const bool dev = (flags & DCC_DEVICE_PTRS) != 0;
      CK(hipMemcpy(out_tn, tn.p, n * 8, dev ? hipMemcpyDeviceToDevice : hipMemcpyDeviceToHost));
    }
  }
  fin_pending = false;
  return DCC_OK;
}

int dcc_ctx::occ_finish(const uint8_t* final_rc, uint64_t* out_tn, uint32_t flags) {
  uint32_t n_cw = 0;
  CR(occ_finish_prepare(final_rc, flags, n_cw));
  return occ_finish_commit(n_cw, out_tn, flags);
}

// central_finish of a pipeline lane's epoch (occ.cpp:248-294), run by the
// parent context when the epoch completes in submit order: every epoch before
// it has finished, so this context's tnc and delta level are exactly what a
// synchronous call would see.  The lane decided the epoch (its committed-
// writer flags are in its cflag buffer, its batch still in place); k_fin
// numbers the committed writers from this context's tnc and appends their
// write sets to this context's delta level, on the lane's stream.  The lanes
// never read the history (an epoch with a window check drains the pipeline
// and runs here), so the history changes only in this host-ordered step.
// chained: the epoch's own chained finish did not number it (an epoch before
// it was not finished yet, or this one was not final), and chained epochs
// behind it may still be finishing on the device: the delta level is not
// merged, rebuilt or moved here -- only grown, once the device is idle.
int dcc_ctx::pipe_finish(dcc_ctx* l, bool chained) {
  dcc_ctx* ctx = this;
  OccRun& r = l->run;
  const DevBatch& d = r.d;
  if (r.n_txn == 0 || !r.fin_later) return DCC_OK;
  HistStore& D = hs[1];
  if (r.app) {
    if (!chained) {
      CR(hist_prepare());  // merge / rebuild as a synchronous append would
    } else if (D.m + d.nnz > hist_room()) {
      // the later chained finishes were all skipped (this epoch did not
      // advance the device control): once they have run, nothing writes the
      // level while it moves
      CK(hipDeviceSynchronize());
    }
    CR(hist_grow_flat(D, D.m + d.nnz));
    // this context's launches (merge, rebuild) before the lane's k_fin: a
    // device-side wait, the host does not block
    CK(hipEventRecord(ev1, stream));
    CK(hipStreamWaitEvent(l->stream, ev1, 0));
  }
  if (l->fin_tag + 4 >= (1u << 30)) {
    CK(hipMemsetAsync(l->fin_part.p, 0, l->fin_part.cap, l->stream));
    l->fin_tag = 0;
  }
  OccDyn& y = *(OccDyn*)l->hdyn;
  y.tnc = tnc;
  y.fin_tag = ++l->fin_tag;
  y.hist_m = D.m;
  y.app_k = r.app ? (uint64_t*)D.fk.p : nullptr;
  y.app_t = r.app ? (uint64_t*)D.ft.p : nullptr;
  y.ins = r.app ? hist_insert_args(D) : HistInsert{};
  y.view = HistView{};
  if (r.app) D.built = false;  // until the append is accepted (see occ_begin)
  FillArgs fa{};
  fa.job[fa.n++] = FillJob{(uint32_t*)l->dyn.p, sizeof(OccDyn) / 4, 0u, (const uint32_t*)l->hdyn_dev};
  launch_fill(fa, l->stream);
  launch_fin(OccFinArgs{d.n, d.nnz, r.cf, d.off, d.keys, d.acctype, (uint64_t*)l->fin_part.p,
                        (const OccDyn*)l->dyn.p, r.tn_dev, (uint64_t*)((char*)l->hdyn_dev + HDYN_TOTALS), 0u, 0u},
             l->stream);
  CK(hipGetLastError());
  if (!r.dev_out && r.out_tn) CK(hipMemcpyAsync(r.out_tn, l->tn.p, d.n * 8, hipMemcpyDeviceToHost, l->stream));
  CK(hipStreamSynchronize(l->stream));
  const uint64_t* tot = (const uint64_t*)((const char*)l->hdyn + HDYN_TOTALS);
  if (tot[0] != r.n_cw) {
    std::string why = "look-back words unreadable";
    std::vector<uint8_t> w(fin_part_bytes(d.n));
    if (hipMemcpy(w.data(), l->fin_part.p, w.size(), hipMemcpyDeviceToHost) == hipSuccess)
      why = fin_diag(w.data(), d.n, l->fin_tag);
    (void)hipGetLastError();
    return fail(DCC_EIO, "central_finish numbered %llu txns, %llu committed writers (%s)",
                (unsigned long long)tot[0], (unsigned long long)r.n_cw, why.c_str());
  }
  if (r.app) {
    if (tot[1] > d.nnz) return fail(DCC_EIO, "history append: %llu writes > %llu accesses",
                                    (unsigned long long)tot[1], (unsigned long long)d.nnz);
    if (tot[1]) {
      D.m += tot[1];
      D.max_key = std::max<uint64_t>(D.max_key, tot[2]);
      D.last_app = tot[1];
      hist_note(D, tnc + 1, tnc + r.n_cw);
    }
    if (tot[3]) D.overflowed = true;
    // chained: the table may hold pushes of a finish that ran on this epoch
    // before it was final, or of a skipped one's successors: rebuilt from the
    // flat pairs before its next read
    D.built = !tot[3] && !chained;
  }
  tnc += r.n_cw;
  return DCC_OK;
}

// flat pairs the delta level can hold without moving
uint64_t dcc_ctx::hist_room() const {
  const HistStore& D = hs[1];
  return std::min<uint64_t>({D.fk.cap / 8, D.ft.cap / 8, D.nx.cap / 4});
}

// A chained central_finish (OccFinArgs::ctl; occ_pipe.cpp): enqueued on lane
// l's stream right behind its decision, so the lane needs no host round trip
// between deciding an epoch and numbering it.  The finish waits on the device
// for the previous epoch's last work (`after`), snapshots fin_ctl and numbers
// and appends only when fin_ctl is at `seq`; the delta level's pointers are
// this context's at submit (the level does not move while chained epochs are
// in flight: occ_pipe.cpp reserves room up front).
int dcc_ctx::chain_enqueue(dcc_ctx* l, uint64_t seq, hipEvent_t after, bool reset) {
  dcc_ctx* ctx = this;
  OccRun& r = l->run;
  const DevBatch& d = r.d;
  HistStore& D = hs[1];
  CR(fin_ctl.ensure(this, sizeof(FinCtl), "chained finish control"));
  CR(l->fdyn.ensure(l, sizeof(OccDyn), "chained finish parameters"));
  if (!l->hfin) {
    CK(hipHostMalloc(&l->hfin, HDYN_BYTES, hipHostMallocDefault));
    CK(hipHostGetDevicePointer(&l->hfin_dev, l->hfin, 0));
    memset(l->hfin, 0, HDYN_BYTES);
  }
  if (l->fin_tag + 4 >= (1u << 30)) {
    CK(hipMemsetAsync(l->fin_part.p, 0, l->fin_part.cap, l->stream));
    l->fin_tag = 0;
  }
  OccDyn& y = *(OccDyn*)l->hfin;
  y.tnc = 0;
  y.hist_m = 0;
  y.fin_tag = ++l->fin_tag;
  y.pad = 0;
  y.app_k = r.app ? (uint64_t*)D.fk.p : nullptr;
  y.app_t = r.app ? (uint64_t*)D.ft.p : nullptr;
  y.ins = r.app ? hist_insert_args(D) : HistInsert{};
  y.view = HistView{};
  if (after) CK(hipStreamWaitEvent(l->stream, after, 0));
  if (reset) {
    // this context's merges / builds first, then the device control starts
    // from this context's values (no epoch is in flight)
    CK(hipEventRecord(ev1, stream));
    CK(hipStreamWaitEvent(l->stream, ev1, 0));
    launch_fin_ctl_set((FinCtl*)fin_ctl.p, tnc, D.m, seq, l->stream);
  }
  launch_fin_prep((const uint32_t*)l->hfin_dev, (OccDyn*)l->fdyn.p, (const FinCtl*)fin_ctl.p, seq, l->stream);
  OccFinArgs fa{d.n, d.nnz, r.cf, d.off, d.keys, d.acctype, (uint64_t*)l->fin_part.p,
                (const OccDyn*)l->fdyn.p, r.tn_dev, (uint64_t*)((char*)l->hfin_dev + HDYN_TOTALS),
                y.fin_tag, 0u};
  fa.ctl = (FinCtl*)fin_ctl.p;
  fa.seq = seq;
  fa.state = (const uint8_t*)l->state.p;
  fa.err = (const uint32_t*)l->misc.p;
  fa.wfull = (const uint32_t*)((const SwLevel*)l->sw_ctl.p + SW_MAX_LEVEL + 1) + 1;
  fa.cap = r.app ? hist_room() : ~0ull;
  launch_fin(fa, l->stream);
  CK(hipGetLastError());
  if (!r.dev_out && r.out_tn) CK(hipMemcpyAsync(r.out_tn, l->tn.p, d.n * 8, hipMemcpyDeviceToHost, l->stream));
  return DCC_OK;
}

// The chained finish numbered and appended lane l's epoch (its totals, read
// after the lane's stream passed it): the host's tnc and delta level follow.
int dcc_ctx::chain_accept(dcc_ctx* l) {
  OccRun& r = l->run;
  const DevBatch& d = r.d;
  const uint64_t* tot = (const uint64_t*)((const char*)l->hfin + HDYN_TOTALS);
  if (tot[0] != r.n_cw) {
    std::string why = "look-back words unreadable";
    std::vector<uint8_t> w(fin_part_bytes(d.n));
    if (hipMemcpy(w.data(), l->fin_part.p, w.size(), hipMemcpyDeviceToHost) == hipSuccess)
      why = fin_diag(w.data(), d.n, l->fin_tag);
    (void)hipGetLastError();
    return fail(DCC_EIO, "chained central_finish numbered %llu txns, %llu committed writers (%s)",
                (unsigned long long)tot[0], (unsigned long long)r.n_cw, why.c_str());
  }
  if (r.app) {
    HistStore& D = hs[1];
    if (tot[1] > d.nnz) return fail(DCC_EIO, "history append: %llu writes > %llu accesses",
                                    (unsigned long long)tot[1], (unsigned long long)d.nnz);
    if (tot[1]) {
      D.m += tot[1];
      D.max_key = std::max<uint64_t>(D.max_key, tot[2]);
      D.last_app = tot[1];
      const bool b = D.built;
      hist_note(D, tnc + 1, tnc + r.n_cw);
      D.built = b;  // the pushes went onto the chains
    }
    if (tot[3]) {
      D.overflowed = true;
      D.built = false;
    }
  }
  tnc += r.n_cw;
  return DCC_OK;
}

int dcc_ctx::chain_set(dcc_ctx* l, uint64_t seq) {
  dcc_ctx* ctx = this;
  CR(fin_ctl.ensure(this, sizeof(FinCtl), "chained finish control"));
  launch_fin_ctl_set((FinCtl*)fin_ctl.p, tnc, hs[1].m, seq, l->stream);
  CK(hipGetLastError());
  return DCC_OK;
}

// The read-only list of a split epoch, once every writer is decided: the
// writer table of the committed writes (k_sw_wall: the committed writers the
// serial passes listed, or after a hand-off to the round solver every
// committed writer of the epoch), then the list against it (k_sw_ro).  `big`:
// after an overflow, a table sized for every write of the epoch (<= 50 %
// load, unbounded probes).
int dcc_ctx::sweep_ro(const DevBatch& d0, bool big, bool scan, uint64_t nnz_w, const DevBatch* full) {
  // a key-sharded rank holding the whole batch decides every read-only txn
  // from it (the writer table then holds every committed write)
  const DevBatch& d = full ? *full : d0;
  dcc_ctx* ctx = this;
  uint32_t* wctl = (uint32_t*)((SwLevel*)sw_ctl.p + SW_MAX_LEVEL + 1);
  WrTab wt{(WrSlot*)sw_wtab.p, wt_bits, WT_PROBES, wctl + 1};
  if (big) {
    uint32_t bits = 10;
    while (bits < 31 && (1ull << bits) < 2 * std::max<uint64_t>(nnz_w, 1)) bits++;
    CR(sw_wtab_big.ensure(this, sizeof(WrSlot) << bits, "committed-writer fallback table"));
    CK(hipMemsetAsync(sw_wtab_big.p, 0xFF, sizeof(WrSlot) << bits, stream));
    wt = WrTab{(WrSlot*)sw_wtab_big.p, bits, 1u << bits, wctl + 3};
  }
  SwWallArgs wa{d.n, d.off, d.keys, d.acctype, d.nnz, (const uint8_t*)state.p,
                (const uint8_t*)hasw.p, scan ? nullptr : (const uint32_t*)sw_cw.p, wctl + 4, wt};
  launch_sw_wall(wa, (unsigned)std::max<uint64_t>(1, std::min<uint64_t>(scan ? 4096 : 256, (d.n + 255) / 256)),
                 stream);
  SwRoArgs ra{(const RoEnt*)sw_ro.p, wctl + 2, d.keys, wt, (uint8_t*)state.p, full ? full->off : nullptr};
  static const uint64_t ro_grid = [] {  // DCC_SW_ROGRID: experiments
    const char* e = DCC_ENV("DCC_SW_ROGRID");
    return e && atoi(e) > 0 ? (uint64_t)atoi(e) : 1024ull;
  }();
  launch_sw_ro(ra, (unsigned)std::max<uint64_t>(1, std::min<uint64_t>(ro_grid, (d.n + 255) / 256)), stream);
  CK(hipGetLastError());
  return DCC_OK;
}

int dcc_ctx::occ_epoch(const dcc_batch* b, uint8_t* out_rc, uint64_t* out_tn, dcc_stats* st) {
  CR(occ_begin(b, out_rc, out_tn, false));
  return occ_end(st);
}

static double wall_ms() {
  return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now().time_since_epoch())
      .count();
}

// First half of an epoch: checks, staging, and every launch up to the
// finalize (or the captured graph's replay).  With `async` and a replayable
// graph the call returns right after the graph launch (run.pending); occ_end
// synchronises and reads the results back.
int dcc_ctx::occ_begin(const dcc_batch* b, uint8_t* out_rc, uint64_t* out_tn, bool async, bool fin_later) {
  dcc_ctx* ctx = this;
  if (run.active) return fail(DCC_EINVAL, "an epoch of this context is still in flight");
  run = OccRun{};
  OccRun& r = run;
  r.out_rc = out_rc;
  r.out_tn = out_tn;
  // key-sharded across ranks: this rank holds only its keys
  r.sh = sharded();
  r.t_wall0 = wall_ms();
  // the one-GPU sweep validates a host batch's offsets on the device (its
  // level-0 launch, prep_body; every kernel before clamps its indices), so the
  // O(n) host pass is skipped there
  CR(check_batch(b, !(use_sweep() && !r.sh)));
  r.n_txn = b->n_txn;
  r.flags = b->flags;
  r.dev_out = (b->flags & DCC_DEVICE_PTRS) != 0;
  r.defer = (b->flags & DCC_OCC_DEFER_FINISH) != 0;
  if (fin_pending)
    return fail(DCC_EINVAL, "an epoch validated with DCC_OCC_DEFER_FINISH awaits dcc_occ_finish_epoch");
  if (r.defer && (out_tn || (b->flags & DCC_OCC_APPEND_HISTORY)))
    return fail(DCC_EINVAL, "DCC_OCC_DEFER_FINISH: commit tn and history come from dcc_occ_finish_epoch");
  r.S.n_shards = (uint32_t)comm_ranks();
  if (b->n_txn == 0) {
    if (r.defer) {
      fin_d = DevBatch{};
      fin_nnz_w = 0;
      fin_pending = true;
    }
    r.active = true;
    return DCC_OK;
  }
  DevBatch& d = r.d;
  const bool self_shard = r.sh && (b->flags & DCC_SHARD_SELF);
  r.whole = self_shard && use_sweep();
  if (self_shard) {
    // this rank's key shard of the whole batch, partitioned on the device;
    // the sweep keeps the whole batch for its serial passes and the
    // read-only list (the round solver needs only the shard)
    dcc_batch sb;
    CR(shard_stage(b, (uint32_t)comm_rank(), (uint32_t)comm_ranks(), sb, r.whole ? &r.full : nullptr));
    CR(stage_batch(&sb, d));
  } else {
    CR(stage_batch(b, d));
  }
  r.sweep = use_sweep();
  const bool sh = r.sh, sweep = r.sweep;
  ro_on = sweep && ro_split && (!sh || r.whole);
  if (sweep) CR(sweep_reserve(d));
  CR(state.ensure(this, d.n + 16, "state"));
  CR(hasw.ensure(this, d.n + 16, "hasw"));
  CR(rc.ensure(this, d.n + 16, "rc"));
  r.want_tn = out_tn != nullptr || (b->flags & DCC_OCC_APPEND_HISTORY);
  r.app = (b->flags & DCC_OCC_APPEND_HISTORY) != 0;
  // a pipeline lane's epoch: central_finish (commit tn, history append) is
  // left to the parent context when the epoch completes in submit order
  // (dcc_ctx::pipe_finish); the lane decides only
  r.fin_later = fin_later && r.want_tn;
  const bool app_here = r.app && !r.fin_later;
  if (r.want_tn) {
    CR(cflag.ensure(this, d.n * 4, "cflag"));
    {
      // Any reallocation is cleared, even one that returns the old address:
      // the grown tail then holds whatever the allocator's previous owner left
      // there -- for a context sharing the GPU with another one (the shards of
      // a multi-GPU context on one device), look-back words carrying the same
      // tag sequence, which k_fin would take as its own predecessors'
      // prefixes (the round-5 "numbered 339 txns, 480 committed writers").
      const size_t old_cap = fin_part.cap;
      CR(fin_part.ensure(this, fin_part_bytes(d.n), "finish look-back words"));
      if (fin_part.cap != old_cap || fin_tag + 4 >= (1u << 30)) {  // reallocated, or the tags wrap
        CK(hipMemsetAsync(fin_part.p, 0, fin_part.cap, stream));
        fin_tag = 0;
      }
    }
    CR(tn.ensure(this, d.n * 8, "tn"));
  }
  CR(dyn.ensure(this, sizeof(OccDyn), "epoch parameters"));
  // the history the window check reads (merge / level builds: launched here,
  // before any capture) and room for this epoch's append
  r.hist_on = d.start_tn && hist_size() > 0;
  if (r.hist_on || app_here) CR(hist_prepare());  // an append inserts into the delta's table
  if (app_here) CR(hist_grow_flat(hs[1], hs[1].m + d.nnz));
  static_assert(sizeof(OccDyn) <= HDYN_TOTALS, "epoch parameters overlap the totals");
  {
    OccDyn& y = *(OccDyn*)hdyn;
    y.tnc = tnc;
    y.fin_tag = ++fin_tag;
    y.hist_m = hs[1].m;
    y.app_k = app_here ? (uint64_t*)hs[1].fk.p : nullptr;
    y.app_t = app_here ? (uint64_t*)hs[1].ft.p : nullptr;
    y.ins = app_here ? hist_insert_args(hs[1]) : HistInsert{};
    y.view = hist_view();
  }
  // central_finish pushes this epoch's pairs onto the delta's chains before
  // the host learns whether the epoch succeeded: until occ_end accepts the
  // append, the delta counts as unbuilt, so an epoch that fails (and a retry
  // that pushes the same flat positions again) leaves a table the next
  // window check rebuilds from the flat pairs instead of walking
  if (app_here) hs[1].built = false;
  // The sweep's whole launch sequence (parameters ... central_finish) is
  // replayed from a captured HIP graph when the batch, the outputs and every
  // workspace are the ones it was captured with: one graph launch instead of
  // ~30 kernel launches, so the device never waits for the host between
  // kernels.  tnc, the history and its append position change every epoch;
  // the graph reads them from the epoch parameters (OccDyn).
  const bool graph_ok = sweep && !profiling && !sw_debug && !sh && !DCC_ENV("DCC_NO_GRAPH");
  // levels per captured epoch (DCC_OPT_SWEEP_LEVELS; 0 = auto: 3 with the
  // read-only split, 4 without) and the schedule.  Auto with the split: two
  // levels (level 1 a serial tail of 8,192) while the last epoch's level-1
  // list fitted comfortably, three otherwise -- a longer list in a two-level
  // epoch is still decided exactly, by more levels after a host round trip.
  if (ro_on && !sw_levels && !sh) {
    if (sw_l1_last <= 6144) sw_mode = 2;
    else if (sw_l1_last > 8192) sw_mode = 1;
  } else {
    sw_mode = 1;
  }
  r.glv = sw_levels ? sw_levels : (ro_on ? (sw_mode == 2 ? 2u : 3u) : 4u);
  // (host outputs are copied outside the graph: their addresses are not part of it)
  r.gkey = GraphKey{d.off, d.keys, d.acctype, d.n, d.nnz, r.dev_out ? out_rc : nullptr, r.dev_out,
                    r.glv | (ro_on ? 0x80u | (wt_bits << 8) : 0u), buf_gen,
                    d.start_tn, d.finish_tn, r.dev_out ? out_tn : (const void*)(uintptr_t)(out_tn != nullptr),
                    (r.want_tn ? 1u : 0u) | (r.app ? 2u : 0u) | (r.hist_on ? 4u : 0u) |
                        (r.fin_later ? 8u : 0u)};
  r.replay = graph_ok && graph_exec && r.gkey == graph_key;
  // a failure while capturing must still end the capture
  struct CaptureGuard {
    hipStream_t s;
    bool* on;
    ~CaptureGuard() {
      if (*on) {
        *on = false;
        hipGraph_t g = nullptr;
        (void)hipStreamEndCapture(s, &g);
        if (g) (void)hipGraphDestroy(g);
        (void)hipGetLastError();
      }
    }
  } capture_guard{stream, &r.capturing};
  if (graph_ok && !r.replay) {
    if (graph_exec) {
      (void)hipGraphExecDestroy(graph_exec);
      graph_exec = nullptr;
    }
    CK(hipStreamBeginCapture(stream, hipStreamCaptureModeThreadLocal));
    r.capturing = true;
  }
  // device clock starts with the batch resident (around the graph launch
  // when one is used: event timing of graph-internal records is unsupported)
  if (!r.replay && !r.capturing) CK(hipEventRecord(ev0, stream));

  // ---- prep: validation, max length (tile width), write count (table size).
  // The sweep needs none of it up front (its kernels clamp every index): its
  // partials are read back with the epoch's one synchronisation.
  if (!sweep) CR(device_prep(d, r.maxlen, r.nnz_w));
  if (!r.replay) {
    // one launch: error word 0, the constant-one word 1, words 2..15, the
    // async pass count, the state bytes, and for the sweep its control block
    // and level-0 key table
    uint32_t* mw = (uint32_t*)misc.p;
    FillArgs fa{};
    fa.job[fa.n++] = FillJob{mw, 1, 0u};
    fa.job[fa.n++] = FillJob{mw + 1, 1, 1u};
    fa.job[fa.n++] = FillJob{mw + 2, 14, 0u};
    fa.job[fa.n++] = FillJob{(uint32_t*)state.p, (d.n + 3) / 4, 0u};  // state holds n + 16
    fa.job[fa.n++] = FillJob{(uint32_t*)dyn.p, sizeof(OccDyn) / 4, 0u, (const uint32_t*)hdyn_dev};
    if (sweep) {
      fa.job[fa.n++] = FillJob{(uint32_t*)sw_ctl.p, sw_ctl_bytes() / 4, 0u};
      const int m0 = ro_on ? (int)sw_mode : 0;
      fa.job[fa.n++] = FillJob{(uint32_t*)sw_gtab.p, (1ull << sw_gbits(0, m0)) * 2, 0xFFFFFFFFu};
      fa.job[fa.n++] = FillJob{(uint32_t*)sw_fw.p, 1ull << sw_gbits(0, m0), 0xFFFFFFFFu};
      fa.job[fa.n++] = FillJob{(uint32_t*)sw_fw.p + (1u << SW_GBITS_MAX), 1ull << sw_gbits(0, m0), 0u};
    }
    launch_fill(fa, stream);  // the sweep's prep runs inside its level-0 serial pass
  }

  // ---- history window pre-pass (occ.cpp:160-180)
  if (r.hist_on && !r.replay) {
    HistArgs ha{d.n, d.nnz, d.off, d.keys, d.acctype, d.start_tn, d.finish_tn, (const OccDyn*)dyn.p, 0u,
                (uint8_t*)state.p, (uint32_t*)misc.p};
    launch_hist(ha, stream);
  }
  // the history window is checked on each shard's keys: any shard's abort wins
  if (sh && d.start_tn) CR(comm_allreduce_max_u8((uint8_t*)state.p, d.n));

  SubProb top;
  top.n = d.n;
  top.nnz = d.nnz;
  top.off = d.off;
  top.keys = d.keys;
  top.acctype = d.acctype;
  top.state = (uint8_t*)state.p;
  top.hasw = (uint8_t*)hasw.p;
  top.hasw_global = true;
  top.w_bound = r.nnz_w;
  bars_used = false;
  if (sweep) {
    if (profiling) CK(hipEventRecord(pev[0], stream));
    r.next_level = (int)std::min<uint32_t>(r.glv, SW_MAX_LEVEL - 1);
    if (!sh && r.next_level >= 2) r.serial_tail = r.next_level - 1;
    if (r.whole) {
      CR(sweep_sharded_full(d, r.full, 0, r.next_level));
      if (ro_on) CR(sweep_ro(d, false, false, 0, &r.full));
    } else if (sh) {
      CR(sweep_sharded(d, r.next_level));
    } else if (!r.replay) {
      CR(sweep_enqueue(d, 0, r.next_level, nullptr, false, r.serial_tail >= 0));
      if (ro_on) CR(sweep_ro(d, false, false, 0));
    }
  } else {
    CR(occ_rounds(top, r.maxlen, profiling, r.rounds));
  }
  if (profiling) CK(hipEventRecord(pev[3], stream));

  // ---- finalize: RC bytes, counts, central_finish tn numbering
  r.rc_dev = (r.dev_out && out_rc) ? out_rc : (uint8_t*)rc.p;
  r.cf = r.want_tn ? (uint32_t*)cflag.p : nullptr;
  r.tn_dev = r.want_tn ? ((r.dev_out && out_tn) ? out_tn : (uint64_t*)tn.p) : nullptr;
  const bool go_async = async && r.replay;
  CR(occ_final(go_async));
  r.pending = go_async;
  r.active = true;
  return DCC_OK;
}

// The finalize launches of `run` (k_final, commit tn, read-back copies), the
// end of a capture, or the replay of the captured graph; synchronises unless
// `async` (a replay only).
int dcc_ctx::occ_final(bool async) {
  dcc_ctx* ctx = this;
  OccRun& r = run;
  const DevBatch& d = r.d;
  // host outputs are copied after the epoch's launches, outside any graph:
  // one captured graph then serves every host output buffer (the pipeline's
  // callers rotate theirs), and the device time includes the copies
  auto copy_out = [&]() -> int {
    if (r.dev_out) return DCC_OK;
    if (r.out_rc) CK(hipMemcpyAsync(r.out_rc, rc.p, d.n, hipMemcpyDeviceToHost, stream));
    if (r.out_tn && !r.fin_later) CK(hipMemcpyAsync(r.out_tn, tn.p, d.n * 8, hipMemcpyDeviceToHost, stream));
    return DCC_OK;
  };
  if (r.replay) {  // once: a second finalize (after more levels) runs directly
    r.replay = false;
    if (r.want_tn) r.fin_runs = 1;  // the graph holds the epoch's first central_finish
    CK(hipEventRecord(ev0, stream));
    CK(hipGraphLaunch(graph_exec, stream));
    CR(copy_out());
    CK(hipEventRecord(ev1, stream));
    if (!async) CK(hipStreamSynchronize(stream));
    return DCC_OK;
  }
  // everything the host reads back goes to pinned memory from k_final
  // itself: its partials directly, the error words and the sweep's control
  // block copied by its last workgroup (prep wrote its partials directly)
  GatherArgs ga{};
  auto job = [&](void* hdst_dev, const void* src, size_t bytes) {
    ga.job[ga.n++] = CopyJob{(const uint32_t*)src, (uint32_t*)hdst_dev, (uint32_t)(bytes / 4)};
  };
  job(hmisc_dev, misc.p, 64);
  job((char*)hmisc_dev + MISC_BARS, (char*)misc.p + MISC_BARS, CTR_RING * 16);
  if (r.sweep) job((char*)hmisc_dev + SW_HCTL, sw_ctl.p, sw_ctl_bytes());
  FinalArgs fa{d.n, (const uint8_t*)state.p, (const uint8_t*)hasw.p, r.rc_dev, r.cf,
               (FinalPart*)hpart_dev};
  launch_final(fa, ga, stream);
  if (r.want_tn && !r.fin_later)
    // a second central_finish of the epoch (after more levels or a hand-off:
    // the graph's ran on a partly decided epoch) needs a fresh look-back tag
    launch_fin(OccFinArgs{d.n, d.nnz, r.cf, d.off, d.keys, d.acctype, (uint64_t*)fin_part.p,
                          (const OccDyn*)dyn.p, r.tn_dev, (uint64_t*)((char*)hdyn_dev + HDYN_TOTALS),
                          r.fin_runs++ ? ++fin_tag : 0u, 0u},
               stream);
  CK(hipGetLastError());
  if (r.capturing) {
    r.capturing = false;
    hipGraph_t g = nullptr;
    CK(hipStreamEndCapture(stream, &g));
    const hipError_t ie = hipGraphInstantiate(&graph_exec, g, nullptr, nullptr, 0);
    (void)hipGraphDestroy(g);
    if (ie != hipSuccess) {
      graph_exec = nullptr;
      return fail(DCC_EIO, "hipGraphInstantiate: %s", hipGetErrorString(ie));
    }
    graph_key = r.gkey;
    CK(hipEventRecord(ev0, stream));
    CK(hipGraphLaunch(graph_exec, stream));
  }
  CR(copy_out());
  CK(hipEventRecord(ev1, stream));
  CK(hipStreamSynchronize(stream));
  return DCC_OK;
}

// Second half: waits for the epoch (when occ_begin returned early), reads the
// results back, runs any further levels / hand-offs, and central_finish.
int dcc_ctx::occ_end(dcc_stats* st) {
  dcc_ctx* ctx = this;
  OccRun& r = run;
  if (!r.active) return fail(DCC_EINVAL, "no epoch of this context is in flight");
  struct Inactive {
    bool* a;
    ~Inactive() { *a = false; }
  } inactive{&r.active};
  if (r.pending) {
    r.pending = false;
    // the replayed graph's last record (ev1) marks the epoch done
    static const int wait_mode = [] {
      const char* e = DCC_ENV("DCC_WAIT_MODE");  // experiments: 0 stream sync, 1 event sync, 2 event poll
      return e ? atoi(e) : 0;
    }();
    if (wait_mode == 1) {
      CK(hipEventSynchronize(ev1));
    } else if (wait_mode == 2) {
      hipError_t q;
      while ((q = hipEventQuery(ev1)) == hipErrorNotReady) {
      }
      CK(q);
    } else {
      CK(hipStreamSynchronize(stream));
    }
  }
  dcc_stats& S = r.S;
  if (r.n_txn == 0) {
    if (st) *st = S;
    return DCC_OK;
  }
  const DevBatch& d = r.d;
  const bool sh = r.sh, sweep = r.sweep;
  const uint32_t glv = r.glv;
  uint32_t& maxlen = r.maxlen;
  uint64_t& nnz_w = r.nnz_w;
  uint32_t& rounds = r.rounds;
  uint32_t& handoffs = r.handoffs;
  int& next_level = r.next_level;
  int& serial_tail = r.serial_tail;
  if (sweep) {
    // prep results: the batch is rejected exactly as device_prep would
    const PrepPart* pp = (const PrepPart*)((const char*)hpart + SW_PREP_OFF);
    static_assert(SW_PREP_OFF + SW_PREP_BLOCKS * sizeof(PrepPart) <= (1u << 16), "hpart holds them");
    uint32_t perr = 0;
    for (unsigned q = 0; q < SW_PREP_BLOCKS; q++) {
      perr |= pp[q].err;
      maxlen = std::max(maxlen, pp[q].maxlen);
      nnz_w += pp[q].nw;
    }
    if (perr & ERR_OFFSETS) return fail(DCC_EINVAL, "batch: malformed offsets");
    if (maxlen > MAX_TXN_LEN)
      return fail(DCC_ERANGE, "batch: a txn has %u accesses (> MAX_ROW_PER_TXN=%u)", maxlen,
                  MAX_TXN_LEN);
    // more levels, or hand the remaining list to the round solver
    bool again = false, ro_fast_rerun = false;
    for (;;) {
      const SwLevel* hc = (const SwLevel*)((const char*)hmisc + SW_HCTL);
      const uint32_t ab = *(const uint32_t*)(hc + SW_MAX_LEVEL + 1);
      const uint32_t e = *(const uint32_t*)hmisc;
      if (e & (ERR_SPIN | ERR_TILE | ERR_FULL)) break;  // reported below
      if (serial_tail >= 0) {
        // the serial-only last level left list txns past its serial range:
        // its committed-set listing, filter and compaction, then more levels
        const SwLevel& t = hc[serial_tail];
        const int lt = serial_tail;
        serial_tail = -1;
        if (!ab && t.m > 0 && t.pos < t.m) {
          const int l1 = std::min(lt + 1 + (int)glv, SW_MAX_LEVEL - 1);
          CR(sweep_enqueue(d, lt, l1, nullptr, true, false));
          next_level = l1;
          GatherArgs ga{};
          ga.job[ga.n++] = CopyJob{(const uint32_t*)sw_ctl.p,
                                   (uint32_t*)((char*)hmisc_dev + SW_HCTL),
                                   (uint32_t)(sw_ctl_bytes() / 4)};
          ga.job[ga.n++] = CopyJob{(const uint32_t*)misc.p, (uint32_t*)hmisc_dev, 16};
          launch_gather(ga, stream);
          CK(hipGetLastError());
          CK(hipStreamSynchronize(stream));
          again = true;
          continue;
        }
      }
      int L = -1;
      if (ab) L = (int)ab;
      else if (hc[next_level].m == 0) break;  // every list decided
      else if ((sh && !r.whole) || next_level + (int)glv >= SW_MAX_LEVEL) L = next_level;
      if (L < 0) {
        const int l1 = next_level + (int)glv;
        if (r.whole) CR(sweep_sharded_full(d, r.full, next_level, l1));
        else CR(sweep_enqueue(d, next_level, l1));
        next_level = l1;
        GatherArgs ga{};
        ga.job[ga.n++] = CopyJob{(const uint32_t*)sw_ctl.p,
                                 (uint32_t*)((char*)hmisc_dev + SW_HCTL),
                                 (uint32_t)(sw_ctl_bytes() / 4)};
        ga.job[ga.n++] = CopyJob{(const uint32_t*)misc.p, (uint32_t*)hmisc_dev, 16};
        launch_gather(ga, stream);
        CK(hipGetLastError());
        CK(hipStreamSynchronize(stream));
        again = true;
        continue;
      }
      // list L (written by the filter of level L-1): decide it with rounds
      const SubBufs& lb = sw_list[(L - 1) & 1];
      SubProb sub;
      sub.n = hc[L].m;
      sub.nnz = hc[L].acc;
      sub.off = (const uint32_t*)lb.off.p;
      sub.keys = (const uint64_t*)lb.keys.p;
      sub.acctype = (const uint8_t*)lb.acctype.p;
      sub.state = (uint8_t*)lb.state.p;
      CR(hasw_scr.ensure(this, d.n + 16, "hasw scratch"));
      sub.hasw = (uint8_t*)hasw_scr.p;
      sub.hasw_global = false;
      sub.w_bound = std::max<uint64_t>(1, sub.nnz);
      CK(hipMemsetAsync(sub.state, 0, sub.n, stream));
      uint32_t r_sub = 0;
      CR(occ_rounds(sub, maxlen, false, r_sub));
      handoffs++;
      rounds += r_sub;
      launch_scatter(sub.state, (const uint32_t*)lb.tid.p,
                     &((SwLevel*)sw_ctl.p)[L].m, sub.n, (uint8_t*)state.p, stream);
      CK(hipGetLastError());
      again = true;
      break;
    }
    if (ro_on) {
      // the RO list: decided again after more levels (their commits joined
      // the writer table), or from the whole decided epoch when a list went
      // to the round solver (its commits never reach the table) or the table
      // overflowed (and the next epochs get a larger one)
      const uint32_t* w = (const uint32_t*)((const SwLevel*)((const char*)hmisc + SW_HCTL) +
                                            SW_MAX_LEVEL + 1);
      const bool full = w[1] != 0, ro_n = w[2] != 0;
      if (full && wt_bits < 24) wt_bits += 2;
      if (ro_n && (full || again)) {
        CR(sweep_ro(d, full, handoffs > 0, nnz_w, r.whole ? &r.full : nullptr));
        ro_fast_rerun = !full;
        again = true;
      }
    }
    if (again) {
      if (profiling) CK(hipEventRecord(pev[3], stream));
      CR(occ_final(false));
    }
    if (ro_fast_rerun) {
      // the rerun's table may have overflowed in turn (more commits than the
      // graph pass saw): then once more with the table sized for every write
      const uint32_t* w = (const uint32_t*)((const SwLevel*)((const char*)hmisc + SW_HCTL) +
                                            SW_MAX_LEVEL + 1);
      if (w[1]) {
        if (wt_bits < 24) wt_bits += 2;
        CR(sweep_ro(d, true, handoffs > 0, nnz_w, r.whole ? &r.full : nullptr));
        CR(occ_final(false));
      }
    }
    const SwLevel* hc = (const SwLevel*)((const char*)hmisc + SW_HCTL);
#ifdef DCC_EXPERIMENTS
    if (sw_debug) {
      std::vector<uint64_t> dv(4096 + 4 * 256 * 8 + 4 * 64 * 8);
      CK(hipMemcpy(dv.data(), sw_dbg.p, dv.size() * 8, hipMemcpyDeviceToHost));
      for (int l = 0; l < 4; l++) {
        // k_sw_seq stamps (s_memrealtime, 100 MHz): start, init done, loop
        // done, decisions written, end; consumer wait polls; tiles
        const uint64_t* t = dv.data() + l * 1024;
        if (t[4])
          fprintf(stderr, "sweep L%d (m %u, pos %u) seq: %llu tiles, init %.2f us, loop %.2f us, decisions "
                          "%.2f us, C out %.2f us, consumer waits %llu, producer waits %llu, "
                          "loop cycles/tile %.0f\n",
                  l, hc[l].m, hc[l].pos, (unsigned long long)t[6], (t[1] - t[0]) * 0.01, (t[2] - t[1]) * 0.01,
                  (t[3] - t[2]) * 0.01, (t[4] - t[3]) * 0.01, (unsigned long long)t[5],
                  (unsigned long long)t[7], t[6] ? (double)t[8] / t[6] : 0.0);
        if (t[6])
          fprintf(stderr, "  seq L%d: candidates/tile %.2f, fixed-point rounds after the first/tile %.2f\n",
                  l, (double)t[9] / t[6], (double)t[10] / t[6]);
        // filter: per workgroup init / first chunk local / look-back / writes / total
        const uint64_t* f = dv.data() + 4096 + l * 256 * 8;
        double fi = 0, fl = 0, fb = 0, fw = 0, ft = 0, nc = 0;
        int nw = 0, nwc = 0;
        for (int w = 0; w < 256 && f[w * 8]; w++) {
          const uint64_t* x = f + w * 8;
          if (!x[5]) continue;  // returned early (nothing to filter)
          nw++;
          fi += x[1] - x[0];
          ft += x[5] - x[0];
          nc += x[6];
          if (x[6]) {
            fl += x[2] - x[1];
            fb += x[3] - x[2];
            fw += x[4] - x[3];
            nwc++;
          }
        }
        {
          // k_sw_pre / k_sw_rows stamps of workgroup 0 (s_memrealtime, 100 MHz)
          const uint64_t* pp = dv.data() + 4096 + 4 * 256 * 8 + l * 64 * 8;
          if (pp[6])
            fprintf(stderr, "  pre L%d (us): offsets %.2f check %.2f keys+map clear %.2f "
                            "map+gid %.2f deps+out %.2f tail %.2f\n", l,
                    (pp[1] - pp[0]) * 0.01, (pp[2] - pp[1]) * 0.01, (pp[3] - pp[2]) * 0.01,
                    (pp[4] - pp[3]) * 0.01, (pp[5] - pp[4]) * 0.01, (pp[6] - pp[5]) * 0.01);
          if (pp[12] && pp[14])
            fprintf(stderr, "  pre L%d map+gid (us): LDS map %.2f first CAS %.2f second CAS %.2f rest "
                            "%.2f; first inserts %llu, lost first slots %llu\n", l, (pp[12] - pp[3]) * 0.01,
                    (pp[13] - pp[12]) * 0.01, (pp[14] - pp[13]) * 0.01, (pp[4] - pp[14]) * 0.01,
                    (unsigned long long)pp[16], (unsigned long long)pp[15]);
          if (pp[36])
            fprintf(stderr, "  compact L%d (us, workgroup 0): totals %.2f tile bases %.2f moves %.2f\n", l,
                    (pp[33] - pp[32]) * 0.01, (pp[34] - pp[33]) * 0.01, (pp[36] - pp[34]) * 0.01);
          if (pp[11])
            fprintf(stderr, "  rows L%d (us): offsets %.2f flags %.2f lists %.2f\n", l,
                    (pp[9] - pp[8]) * 0.01, (pp[10] - pp[9]) * 0.01, (pp[11] - pp[10]) * 0.01);
        }
        if (nw)
          fprintf(stderr, "  filter L%d (us, wave 0 of WGs < 256): %d WGs, tiles/wave %.2f, setup %.2f, "
                          "first tile loads %.2f exact %.2f writes %.2f, total %.2f\n", l, nw, nc / nw,
                  0.01 * fi / nw, nwc ? 0.01 * fl / nwc : 0, nwc ? 0.01 * fb / nwc : 0,
                  nwc ? 0.01 * fw / nwc : 0, 0.01 * ft / nw);
      }
    }
#endif
    r.info.prefix = hc[0].pos;
    r.info.survivors = hc[1].m;
    if (ro_on && !sh) sw_l1_last = hc[1].m;  // the next epoch's schedule (occ_begin)
    for (int l = 0; l < next_level && (l == 0 || hc[l].m); l++) rounds++;
  }

  const uint32_t e = *(const uint32_t*)hmisc;
  {
    // barrier timeout words (third word of each GridBar in the ring, read
    // back with the epoch's gather) of the rounds that used a grid barrier
    const uint32_t* bw = (const uint32_t*)((const char*)hmisc + MISC_BARS);
    for (uint32_t q = 0; q < CTR_RING && bars_used; q++)
      if (bw[q * 4 + 2]) return fail(DCC_EIO, "grid barrier timed out (grid not co-resident)");
  }
  if (e & ERR_KEY) return fail(DCC_EINVAL, "batch: key equal to DCC_KEY_RESERVED");
  if (e & ERR_FULL) return fail(DCC_EIO, "hash table overflow");
  if (e & ERR_TILE) return fail(DCC_EIO, "tile capacity exceeded");
  if (e & ERR_SPIN) return fail(DCC_EIO, "sweep look-back did not complete");
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
  S.peel_prefix = r.info.prefix;
  S.fallback = handoffs;
  S.n_survivors = r.info.survivors;
  if (profiling) {
    float t0 = 0, t1 = 0, t2 = 0;
    if (sweep) {
      // phases: 0 = level-0 records + serial pass + committed set, 1 = the
      // level-0 filter kernel, 2 = level-0 compaction + later levels (+
      // fallback), 3 = prep + finalize
      CK(hipEventElapsedTime(&t0, pev[0], pev[1]));
      CK(hipEventElapsedTime(&t1, pev[1], pev[2]));
      CK(hipEventElapsedTime(&t2, pev[2], pev[3]));
    } else {
      // phases: 0 = key-hash build, 1 = round 1, 2 = rounds >= 2, 3 = prep + finalize
      CK(hipEventElapsedTime(&t0, pev[0], pev[1]));
      CK(hipEventElapsedTime(&t1, pev[1], pev[2]));
      CK(hipEventElapsedTime(&t2, pev[2], pev[4]));
    }
    S.phase_ms[0] = t0;
    S.phase_ms[1] = t1;
    S.phase_ms[2] = t2;
    S.phase_ms[3] = ms - t0 - t1 - t2;
  }
  if (sweep) {
    // the filter pass reads offsets, keys + acctype of every access and the
    // state byte of every txn, and writes the has-write (and kill) bytes
    S.phase_bytes[1] = 4 * (d.n + 1) + 9 * d.nnz + 2 * d.n;
  } else {
    // algorithmic bytes per phase: the build reads acctype of
    // every access and the keys of writes, one 16-B slot update per write;
    // round 1 reads offsets, keys + acctype, one 16-B slot per access, state.
    S.phase_bytes[0] = d.nnz + 8 * nnz_w + 16 * nnz_w + 4 * (d.n + 1) + d.n;
    S.phase_bytes[1] = 4 * (d.n + 1) + 9 * d.nnz + 16 * d.nnz + d.n;
  }

  // central_finish (occ.cpp:277-286): committed write sets join the history
  // -- or, deferred, with the global RC (dcc_occ_finish_epoch)
  if (r.defer) {
    CR(fin_save(d, !r.dev_out, nnz_w));
  } else {
    if (r.want_tn && !r.fin_later) {
      // central_finish ran on the device (k_fin_*): its totals
      const uint64_t* tot = (const uint64_t*)((const char*)hdyn + HDYN_TOTALS);
      if (tot[0] != n_cw) {
        // the look-back words of the last launch explain the mismatch
        std::string why = "look-back words unreadable";
        std::vector<uint8_t> w(fin_part_bytes(d.n));
        if (hipMemcpy(w.data(), fin_part.p, w.size(), hipMemcpyDeviceToHost) == hipSuccess)
          why = fin_diag(w.data(), d.n, fin_tag);
        (void)hipGetLastError();
        return fail(DCC_EIO, "central_finish numbered %llu txns, %llu committed writers (%s)",
                    (unsigned long long)tot[0], (unsigned long long)n_cw, why.c_str());
      }
      if (r.app) {
        HistStore& D = hs[1];
        if (tot[1] > d.nnz) return fail(DCC_EIO, "history append: %llu writes > %llu accesses",
                                        (unsigned long long)tot[1], (unsigned long long)d.nnz);
        if (tot[1]) {
          D.m += tot[1];
          D.max_key = std::max<uint64_t>(D.max_key, tot[2]);
          D.last_app = tot[1];
          hist_note(D, tnc + 1, tnc + n_cw);
        }
        // the pairs went onto the delta's chains too (the table holds every
        // flat pair again), unless its table ran out of room (then it is
        // rebuilt bigger before its next read) or an earlier central_finish
        // of this epoch pushed pairs of a partly decided epoch (then it is
        // rebuilt from the flat pairs, which the last one rewrote)
        if (tot[3]) D.overflowed = true;
        D.built = !tot[3] && r.fin_runs <= 1;
      }
    }
    tnc += n_cw;
    r.n_cw = n_cw;
  }
  S.total_ms = wall_ms() - r.t_wall0;
  if (st) *st = S;
  return DCC_OK;
}
