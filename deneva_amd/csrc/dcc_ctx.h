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

namespace dcc {
struct SwShard;  // occ_kernels.h: one key-sharded sweep level's serial range
}

struct dcc_ctx;

// history hash slot of a key (host build and device probe must agree)
__host__ __device__ inline uint64_t hist_hash_slot(uint64_t key, uint32_t bits) {
  return (key * 0x9E3779B97F4A7C15ull) >> (64 - bits);
}

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
constexpr int PEEL_MAX_LEVEL = 3;

struct dcc_ctx {
  int device = 0;
  int n_cu = 256;
  hipStream_t own_stream = nullptr;
  hipStream_t stream = nullptr;
  hipEvent_t ev0 = nullptr, ev1 = nullptr;
  bool profiling = false;
  uint64_t recheck_max = 16384;   // fold the kill wave into rounds with lists <= this
  uint32_t batch_max = 8;       // rounds enqueued between host synchronisations
  int64_t peel_mode = -1;       // -1 auto prefix, 0 off, > 0 fixed prefix length
  uint64_t peel_min = 32768;    // auto: peel (sub-)batches of at least this many txns
  int solver = 0;               // 0 auto (sweep when unsharded), 1 rounds, 2 async, 3 sweep
  bool force_rounds = false;    // retry after an async-solver limit
  uint32_t* async_passes_dev = nullptr;
  uint64_t prefix_w_top = 0;    // write accesses in the top-level peel prefix
  bool use_async() const { return !force_rounds && solver != 1 && comm_ranks() <= 1; }
  bool use_sweep() const {
    return !force_rounds && (solver == 3 || (solver == 0 && peel_mode == -1));
  }
  uint32_t sw_levels = 4;
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
    bool operator==(const GraphKey& o) const {
      return off == o.off && keys == o.keys && acc == o.acc && n == o.n && nnz == o.nnz &&
             out_rc == o.out_rc && dev_out == o.dev_out && levels == o.levels && gen == o.gen;
    }
  };
  hipGraphExec_t graph_exec = nullptr;
  GraphKey graph_key{};
  uint64_t buf_gen = 0;
  void* hmisc_dev = nullptr;  // device-visible addresses of the two (k_gather targets)
  void* hpart_dev = nullptr;

  // device workspaces (grow-only)
  DevBuf misc;                                   // counters / error words
  DevBuf part;                                   // per-block partial reductions
  DevBuf off, keys, acctype, start_tn, finish_tn, order;  // staged host batch
  DevBuf table;                                  // Slot[cap]
  DevBuf state, hasw, rc, stat;                  // per-txn bytes
  DevBuf cflag, bsum, tn;                        // commit-tn scan
  DevBuf gst;                                    // sharded per-txn status
  DevBuf hasw_scr, cset_tab, cset_keys;          // prefix peel
  DevBuf a_cnt, a_writers, a_big, a_st32;        // async solver
  DevBuf sw_ctl, sw_status, sw_ckeys, sw_dbg;            // sweep solver: level control, look-back, C
  DevBuf sw_rec, sw_rk, sw_gtab, sw_fw, sw_aent, sw_mg;
  DevBuf sw_xcnt, sw_xrec, sw_mcnt, sw_moff, sw_mkeys, sw_mat, sw_kill;  // key-sharded sweep  // sweep tile records
  SubBufs sw_list[2];                            // sweep level lists (ping-pong)
  SubBufs subs[PEEL_MAX_LEVEL];
  DevBuf l_tid[2], l_coff[2], l_cent[2];         // ping-pong undecided lists
  DevBuf hkeys, hoff, htn;                       // history CSR
  DevBuf hhash;                                  // history key -> CSR row, open addressing
  DevBuf perm, calvin_a, calvin_b, calvin_c, calvin_d;  // Calvin workspaces
  DevBuf cv_scratch, cv_agg, cv_group, cv_wave, cv_pgx, cv_gsx, cv_gsize, cv_done, cv_maxl;
  DevBuf cv_seq_b, cv_ok, cv_len, cv_off2, cv_tsum;
  DevBuf snap_top, snap_aoff, snap_aidx, snap_cnt;  // captured-snapshot validation
  // OCC stage solver (occ_stage.hip): per-stage control + epoch state, the
  // ping-pong stage lists, the deciders' committed-key lists
  DevBuf st_ctl;
  DevBuf st_tid[2], st_ast[2], st_alen[2], st_keys[2], st_at[2], st_hdr[2], st_ck[2];
  DevBuf st_hsh[2], st_dep[2], st_tile[2];
  void* st_host = nullptr;      // pinned mirror of StEpoch + StCtl[] (k_stage_final)
  void* st_host_dev = nullptr;
  uint64_t st_tnc_dev = ~0ull;  // tnc the device StEpoch holds (~0: unknown)
  hipGraphExec_t st_graph = nullptr;
  GraphKey st_graph_key{};
  uint32_t st_fallbacks = 0;    // epochs handed to the round solver (lifetime)
  bool st_debug = false;        // DCC_ST_DEBUG: decider / filter stamps to stderr
  DevBuf st_dbg;

  // OCC history (occ.h:62-64) and commit counter tnc (occ.h:67)
  std::vector<std::pair<uint64_t, uint64_t>> hist;
  bool hist_dirty = false;
  uint64_t h_nkeys = 0;
  uint32_t h_hbits = 0;  // log2 of hhash slots (16 B each: key, row)
  uint64_t tnc = 0;

  dcc_comm_state* comm = nullptr;
  int comm_ranks() const;
  int comm_allreduce_max_u8(uint8_t* dev, uint64_t n);  // in place, on `stream`
  int comm_rank() const;

  int fail(int code, const char* fmt, ...);
  int hip_fail(hipError_t e, const char* what);
  std::vector<DevBuf*> all_bufs();
  int reserve_occ(uint64_t n, uint64_t nnz, uint64_t nnz_w, uint32_t tw);
  void list_geometry(uint64_t n, uint32_t tw, uint64_t& seg_ts, uint64_t& seg_es) const;
  static uint64_t table_capacity(uint64_t nnz_w);
  int upload_history();
  int check_batch(const dcc_batch* b);
  int stage_batch(const dcc_batch* b, DevBatch& d);
  int device_prep(const DevBatch& d, uint32_t& maxlen, uint64_t& nnz_w, uint64_t p = 0,
                  uint64_t* nnz_w_prefix = nullptr);
  int read_partials(size_t bytes);
  int occ_epoch(const dcc_batch* b, uint8_t* out_rc, uint64_t* out_tn, dcc_stats* st);
  bool use_stage() const { return !force_rounds && solver == 4 && comm_ranks() <= 1; }
  int stage_reserve(const DevBatch& d);
  int stage_enqueue(const DevBatch& d, uint32_t l0, uint32_t l1, uint8_t* rc_dev, uint64_t* tn_dev,
                    const uint8_t* hkill);
  int occ_stage_epoch(const dcc_batch* b, uint8_t* out_rc, uint64_t* out_tn, dcc_stats* st);
  uint64_t st_tnc_upload = 0;   // host source of the tnc upload (must outlive the copy)
  int history_append_epoch(const dcc_batch* b, const DevBatch& d, const uint64_t* tn_dev, bool dev_out,
                           uint64_t n_cw);
  int occ_rounds(const SubProb& sp, uint32_t maxlen, bool prof, uint32_t& rounds);
  int occ_async(const SubProb& sp, uint32_t maxlen, uint32_t& passes);
  int occ_peel(const SubProb& sp, uint32_t maxlen, int level, uint32_t& rounds, PeelInfo& info);
  int sweep_reserve(const DevBatch& d);
  int sweep_enqueue(const DevBatch& d, int l0, int l1, const dcc::SwShard* shard = nullptr);
  int sweep_sharded(const DevBatch& d, int& next_level);
  int occ_sweep_finish(const DevBatch& d, int& next_level, bool& done, uint32_t maxlen);
  uint64_t peel_prefix(uint64_t m, int level) const;
  int occ_snapshot(const dcc_batch* b, const dcc_occ_snapshot* s, uint8_t* out_rc, dcc_stats* st);
  int calvin_epoch(const dcc_batch* b, uint32_t* out_group, uint8_t* out_rc, uint32_t* out_wave,
                   dcc_stats* st);
};
