// dcc_ctx: the per-process, per-device engine context behind the C ABI.
// Replaces the reference's global OptCC singleton (`occ_man`,
// system/global.cpp:42) and owns every device workspace so that a validation
// call performs no allocation once warmed up.
#pragma once
#include <hip/hip_runtime.h>

#include <string>
#include <utility>
#include <vector>

#include "dcc.h"
#include "occ_history.h"

namespace dcc {
struct SwShard;  // occ_kernels.h: one key-sharded sweep level's serial range
}

struct dcc_ctx;


struct DevBuf {
  void* p = nullptr;
  size_t cap = 0;
  int ensure(dcc_ctx* c, size_t bytes, const char* what);
  void release();
};

// A batch as device pointers (aliases the caller's or the ctx's staging).
struct DevBatch {
  uint64_t n = 0, nnz = 0;
  const uint32_t* off = nullptr;
  const uint64_t* keys = nullptr;
  const uint8_t* acctype = nullptr;
  const uint64_t* start_tn = nullptr;
  const uint64_t* finish_tn = nullptr;
  const uint64_t* order = nullptr;
};

struct dcc_comm_state;  // RCCL communicator (dcc_comm.hip)
struct dcc_multi;       // single-process multi-GPU context (dcc_multi.cpp)

// One level of the device OCC history (occ_history.h): flat (key, tn) pairs in
// append order and, once built, the pairs sorted by (key, tn) with the key
// table.
// The delta level also takes the epochs' appends as chains in its table
// (occ_history.h HistInsert), so an epoch's append needs no rebuild.
struct HistStore {
  DevBuf fk, ft;            // flat pairs
  DevBuf skey, stn, hash;   // built level
  DevBuf bm;                // key bitmap of the built level (occ_history.h HIST_BM_LOG)
  DevBuf nx, tcnt;          // delta: chain links per flat pair; the table's overflow flag
  uint64_t m = 0;           // pairs
  uint32_t hbits = 0;
  bool built = true;        // the built level (with its chains) holds every flat pair
  bool mono = true;         // append order is tn order within every key
  uint64_t max_tn = 0;      // largest tn appended
  uint64_t min_tn = ~0ull;  // smallest tn appended
  uint64_t max_key = 0;     // largest key appended (radix passes of the build)
  bool chained = false;     // the delta level
  bool overflowed = false;  // a key landed past HIST_WALK: the next build doubles the table
  uint64_t last_app = 0;    // delta: pairs the last epoch appended (table headroom)
  // empty the level, keeping its buffers (the next build clears its table)
  void reset() {
    m = 0;
    built = false;
    mono = true;
    max_tn = 0;
    min_tn = ~0ull;
    max_key = 0;
  }
};

// One OCC (sub-)batch: txn i has accesses [off[i], off[i+1]) of keys/acctype
// and the state byte state[i]; nnz bounds off[n], w_bound its write count.
struct SubProb {
  uint64_t n = 0, nnz = 0, w_bound = 0;
  const uint32_t* off = nullptr;
  const uint64_t* keys = nullptr;
  const uint8_t* acctype = nullptr;
  uint8_t* state = nullptr;
  uint8_t* hasw = nullptr;   // has-write bytes out
  bool hasw_global = false;  // hasw is the epoch's (all-reduced when sharded)
};
struct PeelInfo {
  uint64_t prefix = 0, survivors = 0;
};
// Dense survivor sub-batch of one peel level.
struct SubBufs {
  DevBuf tid, off, keys, acctype, state;
};

struct dcc_ctx {
  int device = 0;
  int n_cu = 256;
  hipStream_t own_stream = nullptr;
  hipStream_t stream = nullptr;
  hipEvent_t ev0 = nullptr, ev1 = nullptr;
  bool profiling = false;
  uint64_t recheck_max = 16384;   // fold the kill wave into rounds with lists <= this
  uint32_t batch_max = 8;       // rounds enqueued between host synchronisations
  bool bars_used = false;       // this epoch's rounds used grid-barrier words
  int solver = 0;               // 0 auto (= 3), 1 fixed-point rounds, 3 sweep
  bool use_sweep() const { return solver != 1; }
  bool ro_split = true;           // DCC_OPT_RO_SPLIT
  bool ro_on = false;             // this epoch splits read-only txns off (sweep, one GPU)
  uint32_t wt_bits = 18;          // committed-writer table slots (WT_BITS_DEFAULT; grows after an overflow)
  uint32_t wf_bits = 0;           // fallback table (k_sw_wall) slots
  uint32_t sw_levels = 0;          // DCC_OPT_SWEEP_LEVELS (0: auto)
  uint32_t sw_mode = 1;            // this epoch's level schedule (occ_driver.hip sw_pmax)
  uint32_t sw_l1_last = ~0u;       // level-1 list length of the last one-GPU split epoch
  bool sw_debug = false;        // DCC_SW_DEBUG: per-tile clock stamps of the serial pass       // sweep levels enqueued between host synchronisations
  hipEvent_t pev[8] = {};  // phase boundary events (profiling only)
  std::string last_error;
  void* hmisc = nullptr;  // pinned host mirror of `misc`
  void* hpart = nullptr;  // pinned host mirror of `part`
  // the sweep epoch's captured launch sequence (occ_epoch) and what it was
  // captured with; buf_gen counts workspace reallocations
  struct GraphKey {
    const void *off, *keys, *acc;
    uint64_t n, nnz;
    const void* out_rc;
    bool dev_out;
    uint32_t levels;
    uint64_t gen;
    const void *start_tn, *finish_tn, *out_tn;
    uint32_t fin;  // want tn | append << 1 | window check << 2
    bool operator==(const GraphKey& o) const {
      return off == o.off && keys == o.keys && acc == o.acc && n == o.n && nnz == o.nnz &&
             out_rc == o.out_rc && dev_out == o.dev_out && levels == o.levels && gen == o.gen &&
             start_tn == o.start_tn && finish_tn == o.finish_tn && out_tn == o.out_tn && fin == o.fin;
    }
  };
  hipGraphExec_t graph_exec = nullptr;
  // the Calvin epoch's launch sequence after its prep read-back (calvin.hip):
  // captured the second time a shape is seen, replayed while it repeats
  struct CvGraphKey {
    const void *off, *keys, *acc, *order, *grp, *rc;
    uint64_t n, nnz, gen;
    uint32_t ulen, have_seq, bucket;
    uint8_t kp[112], op[112];  // KeyPack images (memcmp)
  };
  hipGraphExec_t cv_graph_exec = nullptr;
  CvGraphKey cv_graph_key{}, cv_seen_key{};
  bool cv_seen = false;
  bool cv_last_sorted = false, cv_last_bucket = false;  // the last Calvin epoch's order / path
  uint64_t cv_spec_miss = 0;  // speculative Calvin replays whose prep results differed
  GraphKey graph_key{};
  uint64_t buf_gen = 0;
  void* hmisc_dev = nullptr;  // device-visible addresses of the two (k_gather targets)
  void* hpart_dev = nullptr;
  // per-epoch values of a captured OCC epoch (dcc::OccDyn at offset 0, written
  // by the host before each launch) and the central_finish totals (offset
  // HDYN_TOTALS, written by the device); pinned
  void* hdyn = nullptr;
  void* hdyn_dev = nullptr;
  static constexpr size_t HDYN_TOTALS = 256, HDYN_BYTES = 512;

  // device workspaces (grow-only)
  DevBuf misc;                                   // counters / error words
  DevBuf part;                                   // per-block partial reductions
  DevBuf off, keys, acctype, start_tn, finish_tn, order;  // staged host batch
  DevBuf nar_keys, nar_at, nar_tn;                 // compact forms before widening (host batches)
  DevBuf table;                                  // Slot[cap]
  DevBuf state, hasw, rc, stat;                  // per-txn bytes
  DevBuf cflag, bsum, tn;                        // commit-tn scan
  DevBuf dyn, fin_part;                          // OccDyn (device copy), central_finish block counts
  DevBuf gst;                                    // sharded per-txn status
  DevBuf hasw_scr;                               // round-solver hand-off
  DevBuf sw_ctl, sw_status, sw_ckeys, sw_dbg;            // sweep solver: level control, look-back, C
  DevBuf sw_rec, sw_rk, sw_gtab, sw_fw, sw_aent, sw_mg;
  DevBuf sw_rflag, sw_ro, sw_wtab, sw_cw, sw_wtab_big;  // read-only split: survivor bits, RO
                                                        // list, writer tables, committed writers
  DevBuf sw_xcnt, sw_xsend, sw_xrec, sw_mcnt, sw_moff, sw_mkeys, sw_mat, sw_kill;  // key-sharded sweep  // sweep tile records
  SubBufs sw_list[2];                            // sweep level lists (ping-pong)
  DevBuf l_tid[2], l_coff[2], l_cent[2];         // ping-pong undecided lists
  // OCC history (occ.h:62-64) on the device: base + delta levels
  HistStore hs[2];
  uint64_t hist_merge_min = 65536;  // DCC_OPT_HIST_MERGE
  DevBuf h_K[2], h_V[2], h_scr, h_bsum;          // level-build sort buffers, append scan
  DevBuf h_bm;                                   // key bitmap of both levels (window check)
  bool h_bm_stale = true;                        // h_bm is not B.bm | D.bm
  uint32_t fin_tag = 0;                          // k_fin's look-back tag of the last epoch
  DevBuf perm, calvin_a, calvin_b, calvin_c, calvin_d;  // Calvin workspaces
  DevBuf cv_scratch, cv_agg, cv_group, cv_wave, cv_pgx, cv_gsx, cv_gsize, cv_done, cv_maxl, cv_cwmax, cv_cwpos, cv_cwmark, cv_cwhot, cv_cwpa, cv_cwoa, cv_cwhelp, cv_cwrec2;
  DevBuf cv_seq_b, cv_ok, cv_len, cv_off2, cv_tsum, cv_hkeys, cv_hat;
  DevBuf cb_e, cb_out, cb_cnt, cb_small;           // Calvin bucket path (calvin_bucket.h)
  DevBuf snap_top, snap_aoff, snap_aidx, snap_cnt;  // captured-snapshot validation
  DevBuf mt_rk;                                  // MaaT row table: 32-B {key, last read, last write} slots
  uint32_t mt_bits = 0;                          // log2 row-table slots (0: none yet)
  uint64_t mt_rows = 0;                          // rows in the table
  uint64_t mt_new_last = 0;                      // rows the last epoch added (table sizing)
  uint64_t mt_full_redo = 0;                     // epochs run again on a bigger row table
  uint32_t mt_rows32 = 0;                        // upload source of the row counter
  DevBuf mt_misc, mt_slot, mt_sval, mt_slot2, mt_sval2, mt_sfl, mt_stx, mt_txn, mt_agg;
  DevBuf mt_sflB, mt_stxB, mt_k1, mt_tcnt, mt_ul;
  DevBuf mt_lb;          // fused round scan: look-back status per tile (k_mt_round)
  DevBuf mt_ptab;        // prefix level: per-row commit bounds of the prefix (MtPTab)
  uint32_t mt_tag = 0;   // its round tag (monotone; the buffer is zeroed when it wraps)
  // GPU index (index.hip): key table, newest insert ordinal per key, rows
  DevBuf ix_keys, ix_ord, ix_rows, ix_cnt, wv_buf, ix_scr, wv_hbuf, wv_obuf;
  uint32_t ix_bits = 0;
  uint64_t ix_nkeys = 0, ix_nrows = 0;
  double ix_last_ms = 0;
  // commit counter tnc (occ.h:67)
  uint64_t tnc = 0;

  dcc_comm_state* comm = nullptr;
  dcc_multi* multi = nullptr;  // non-null: this context drives per-GPU sub-contexts
  int comm_ranks() const;
  bool sharded() const;    // the key-sharded paths run (ranks > 1, or a one-rank RCCL clique)
  bool comm_solo = false;  // DCC_OPT_COMM_SOLO
  int comm_allreduce_max_u8(uint8_t* dev, uint64_t n);  // in place, on `stream`
  // every rank's `bytes` from send into recv[rank * bytes ...], on `stream`
  int comm_allgather_u8(const uint8_t* send, uint8_t* recv, uint64_t bytes);
  int comm_rank() const;

  int fail(int code, const char* fmt, ...);
  int hip_fail(hipError_t e, const char* what);
  std::vector<DevBuf*> all_bufs();
  int reserve_occ(uint64_t n, uint64_t nnz, uint64_t nnz_w, uint32_t tw);
  void list_geometry(uint64_t n, uint32_t tw, uint64_t& seg_ts, uint64_t& seg_es) const;
  static uint64_t table_capacity(uint64_t nnz_w);
  // device history (occ_history.h / dcc_ctx.hip)
  uint64_t hist_size() const { return hs[0].m + hs[1].m; }
  int hist_grow_flat(HistStore& h, uint64_t need);
  dcc::HistInsert hist_insert_args(HistStore& h);
  void hist_note(HistStore& h, uint64_t lo_tn, uint64_t hi_tn);
  int hist_build(HistStore& h);
  int hist_prepare();  // merge policy + rebuild: call before a window check
  dcc::HistView hist_view() const;
  int hist_append_epoch(const DevBatch& d, const uint64_t* tn_dev, uint64_t nnz_w, uint64_t n_cw);
  // scan_offsets: the O(n) host pass over a host batch's offsets (the sweep
  // validates them on the device instead, inside its level-0 launch)
  int check_batch(const dcc_batch* b, bool scan_offsets = true);
  int stage_batch(const dcc_batch* b, DevBatch& d);
  int device_prep(const DevBatch& d, uint32_t& maxlen, uint64_t& nnz_w, uint64_t p = 0,
                  uint64_t* nnz_w_prefix = nullptr);
  int read_partials(size_t bytes);
  int occ_epoch(const dcc_batch* b, uint8_t* out_rc, uint64_t* out_tn, dcc_stats* st);
  // The epoch in two halves (occ_pipe.cpp overlaps epochs of several lane
  // contexts): begin enqueues; with `async` and a replayable graph it returns
  // right after the graph launch (run.pending) and end synchronises.
  struct OccRun {
    uint64_t n_txn = 0;
    uint32_t flags = 0;
    uint8_t* out_rc = nullptr;
    uint64_t* out_tn = nullptr;
    DevBatch d;
    bool sh = false, dev_out = false, defer = false, sweep = false, want_tn = false;
    bool app = false, hist_on = false;  // history append (central_finish) / window check
    bool whole = false;                 // key-sharded rank holding the whole batch (DCC_SHARD_SELF)
    DevBatch full;                      // that batch
    bool replay = false, capturing = false, pending = false, active = false;
    uint32_t glv = 0, maxlen = 0, rounds = 0, handoffs = 0;
    uint64_t nnz_w = 0;
    int next_level = 0, serial_tail = -1;
    uint8_t* rc_dev = nullptr;
    uint32_t* cf = nullptr;
    uint64_t* tn_dev = nullptr;
    PeelInfo info;
    GraphKey gkey{};
    dcc_stats S;
    double t_wall0 = 0;
    uint64_t n_cw = 0;  // committed writers of the finished epoch (tnc advance)
    uint32_t fin_runs = 0;  // central_finish launches (a second one after more levels)
    bool fin_later = false; // pipeline lane: central_finish runs at completion (pipe_finish)
  };
  OccRun run;
  int occ_begin(const dcc_batch* b, uint8_t* out_rc, uint64_t* out_tn, bool async, bool fin_later = false);
  // the central_finish of lane `l`'s completed epoch (decided with fin_later):
  // commit tn from this context's tnc, the history append into this
  // context's delta level -- run by the parent in submit order (occ_pipe.cpp)
  // chained: other chained epochs may be in flight behind it (their finishes
  // write into the delta level): no merge, rebuild or growth here
  int pipe_finish(dcc_ctx* l, bool chained = false);
  // Chained central_finish (occ_pipe.cpp, DCC_OPT_PIPE_CHAIN): lane l's epoch
  // `seq` numbered and appended on the device right after its decision, from
  // this context's device tnc / append position (fin_ctl), which the finish
  // advances; `after`: the previous epoch's last work (its finish) is waited
  // for on the device; reset: fin_ctl starts at this context's values
  int chain_enqueue(dcc_ctx* l, uint64_t seq, hipEvent_t after, bool reset);
  // fin_ctl = {tnc, delta size, seq} after lane l's work: the host finished
  // the epoch before `seq` itself
  int chain_set(dcc_ctx* l, uint64_t seq);
  // the chained finish of lane l's epoch numbered it: tnc and the delta level follow
  int chain_accept(dcc_ctx* l);
  uint64_t hist_room() const;  // flat pairs the delta level holds without moving
  DevBuf fin_ctl;                  // parent: dcc::FinCtl
  DevBuf fdyn;                     // lane: the chained finish's OccDyn
  void* hfin = nullptr;            // lane: its staging and totals (pinned, HDYN_BYTES)
  void* hfin_dev = nullptr;
  hipEvent_t ev_done = nullptr;    // lane: after the work of its last submitted epoch
  uint32_t pipe_chain = 1;         // DCC_OPT_PIPE_CHAIN
  int occ_end(dcc_stats* st);
  int occ_final(bool async);  // finalize launches (or the graph replay) of `run`
  // pipelined epochs over lane contexts on this device (occ_pipe.cpp)
  struct OccPipe* pipe = nullptr;
  uint32_t pipe_lanes = 3;  // DCC_OPT_PIPELINE
  uint32_t pipe_part = 0;   // DCC_OPT_PIPE_PARTITION
  int cv_path = 0;          // DCC_OPT_CALVIN_PATH: 0 auto, 1 sort, 2 bucket
  bool cb_hash_off = false; // a hashed bucket carry table overflowed: sort path for such epochs
  // DCC_OCC_DEFER_FINISH: the decided epoch waiting for its global RC
  bool fin_pending = false;
  DevBatch fin_d;
  uint64_t fin_nnz_w = 0;
  DevBuf fin_off, fin_keys, fin_at, fin_state, fin_hasw, fin_rc, fin_cnt;
  int fin_save(const DevBatch& d, bool host_batch, uint64_t nnz_w);
  int occ_finish(const uint8_t* final_rc, uint64_t* out_tn, uint32_t flags);
  int occ_finish_prepare(const uint8_t* final_rc, uint32_t flags, uint32_t& n_cw);
  int occ_finish_commit(uint32_t n_cw, uint64_t* out_tn, uint32_t flags);
  int occ_rounds(const SubProb& sp, uint32_t maxlen, bool prof, uint32_t& rounds);
  int sweep_reserve(const DevBatch& d);
  // levels [l0, l1); resume: level l0's serial part already ran (start at its
  // committed-set listing); tail_serial: level l1 - 1 runs its serial part only
  int sweep_enqueue(const DevBatch& d, int l0, int l1, const dcc::SwShard* shard = nullptr,
                    bool resume = false, bool tail_serial = false);
  int sweep_sharded(const DevBatch& d, int& next_level);
  int sweep_sharded_full(const DevBatch& d, const DevBatch& full, int l0, int l1);  // levels [l0, l1)
  // decide the RO list (full: a key-sharded rank's whole batch)
  int sweep_ro(const DevBatch& d, bool big, bool scan, uint64_t nnz_w, const DevBatch* full = nullptr);
  int occ_sweep_finish(const DevBatch& d, int& next_level, bool& done, uint32_t maxlen);
  int occ_snapshot(const dcc_batch* b, const dcc_occ_snapshot* s, uint8_t* out_rc, dcc_stats* st);
  // MaaT (maat.hip): row timestamp table + epoch workspaces
  int maat_rows_reserve(uint64_t want);
  int index_reserve(uint64_t want);
  int maat_epoch(const dcc_batch* b, uint8_t* out_rc, uint64_t* out_cts, dcc_stats* st);
  int maat_epoch_try(const dcc_batch* b, uint8_t* out_rc, uint64_t* out_cts, dcc_stats* st, bool all_rows,
                     bool* full);
  int calvin_epoch(const dcc_batch* b, const dcc_calvin_held* held, uint32_t* out_group,
                   uint8_t* out_rc, uint32_t* out_wave, dcc_stats* st);
  // device-side key-shard partition (shard_dev.hip): rank `rank` of R of a
  // multi-GPU context; sb is the shard as a device batch
  DevBuf sh_off, sh_keys, sh_at, sh_src, sh_cnt, sh_bsum, sh_rc, sh_tn, sh_grp;
  int shard_stage(const dcc_batch* b, uint32_t rank, uint32_t R, dcc_batch& sb, DevBatch* full_out = nullptr);
  int shard_groups(const uint32_t* grp, uint64_t m, uint32_t* out_dev);  // groups to batch order
};

// multi-GPU context (dcc_multi.cpp)
int dcc_multi_size(const dcc_ctx* ctx);
void dcc_multi_destroy(dcc_ctx* ctx);
int dcc_multi_occ_epoch(dcc_ctx* ctx, const dcc_batch* b, uint8_t* out_rc, uint64_t* out_tn,
                        dcc_stats* st);
int dcc_multi_calvin_epoch(dcc_ctx* ctx, const dcc_batch* b, const dcc_calvin_held* held,
                           uint32_t* out_group, uint8_t* out_rc, uint32_t* out_wave, dcc_stats* st);
int dcc_multi_each(dcc_ctx* ctx, int (*fn)(dcc_ctx*, void*), void* user);
int dcc_multi_occ_snapshot(dcc_ctx* ctx, const dcc_batch* b, const dcc_occ_snapshot* snap,
                           uint8_t* out_rc, dcc_stats* st);
dcc_ctx* dcc_multi_rank0(dcc_ctx* ctx);  // rank 0's sub-context, its device selected
// pipelined epochs (occ_pipe.cpp): complete every epoch in flight / tear down
void dcc_pipe_drain(dcc_ctx* ctx);
void dcc_pipe_destroy(dcc_ctx* ctx);
dcc_ctx* dcc_multi_sub(dcc_ctx* ctx, int rank);
