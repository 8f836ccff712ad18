/*
 * dcc.h — C ABI of the MI355X-native batched concurrency-control engine
 * (libdcc.so).  Everything a Deneva-style host binds to for the one hot path
 * SURVEY.md §8 scopes: deciding commit/abort (OCC) and lock-grant order
 * (Calvin) for a whole epoch of transactions at once.
 *
 * Conventions:
 *   - extern "C", plain pointers and sizes, no torch / HIP types in signatures
 *     (streams are passed as opaque `void*`).
 *   - every entry point returns int: 0 = success, < 0 = -errno-style code
 *     (DCC_E*).  Nothing aborts the process; batch validation (offset
 *     monotonicity, nnz bound, reserved key) runs on the host before launch.
 *   - all pointers are caller-owned; nothing is retained after return.
 *   - a dcc_ctx is thread-compatible, not thread-safe: the host shim
 *     serialises calls per context (reference OptCC serialises its list
 *     mutations with `_semaphore`, concurrency_control/occ.cpp:137-158).
 *
 * Reference interfaces each entry point replaces are cited per declaration
 * (paths relative to the reference tree).
 */
#ifndef DCC_H_
#define DCC_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---------------------------------------------------------------- errors */
#define DCC_OK 0
#define DCC_EIO (-5)       /* HIP runtime failure (message via dcc_last_error) */
#define DCC_ENOMEM (-12)   /* device or host allocation failed                  */
#define DCC_ENODEV (-19)   /* no usable gfx950 device / bad device id           */
#define DCC_EINVAL (-22)   /* malformed batch or argument                       */
#define DCC_ERANGE (-34)   /* size exceeds an engine limit                      */
#define DCC_ECOMM (-70)    /* RCCL failure                                       */
#define DCC_ENOTSUP (-95)  /* feature not available in this build / mode        */

/* ------------------------------------------------------ reference enums */
/* access_t, system/global.h:287  {RD, WR, XP, SCAN}.  OCC puts only WR into
 * the write set (concurrency_control/occ.cpp:296-317, get_rw_set: `get_access_type(i) == WR`, line 308); Calvin
 * maps RD/SCAN to LOCK_SH and everything else to LOCK_EX (storage/row.cpp:191). */
#define DCC_RD 0
#define DCC_WR 1
#define DCC_XP 2
#define DCC_SCAN 3

/* RC, system/global.h:236  {RCOK=0, Commit, Abort, WAIT, ...}.  The engine
 * reports per-transaction RCs with the reference's numeric values. */
#define DCC_RC_RCOK 0
#define DCC_RC_ABORT 2
#define DCC_RC_WAIT 3

/* Keys are canonical 64-bit row identities.  This
 * one value is reserved as the empty-slot marker of the device hash table. */
#define DCC_KEY_RESERVED 0xFFFFFFFFFFFFFFFFull

/* group value for a Calvin request removed by per-txn row de-duplication
 * (TxnManager::get_lock, system/txn.cpp:778-782). */
#define DCC_GROUP_NONE 0xFFFFFFFFu

/* --------------------------------------------------------------- batch  */
/* dcc_batch.flags */
#define DCC_DEVICE_PTRS 0x1u      /* every batch AND output pointer is device memory */
#define DCC_MAAT_READ_AND_PREWRITE 0x4u /* MaaT: every access both reads and prewrites its row
                                          (the TPC-C path, Row_maat::read_and_prewrite,
                                          row_maat.cpp:40-41, 54-96)                     */
#define DCC_OCC_APPEND_HISTORY 0x2u /* central_finish semantics: committed write sets
                                     of this epoch are appended to the history with
                                     tn = tnc+1, tnc+2, ... in index order
                                     (occ.cpp:248-294) */
#define DCC_OCC_DEFER_FINISH 0x8u   /* 2PC participants: decide only.  Commit tn and the
                                     history follow the GLOBAL RC passed later to
                                     dcc_occ_finish_epoch (OptCC::finish after RFIN,
                                     worker_thread.cpp:286-297, occ.cpp:248-294).  Not
                                     with DCC_OCC_APPEND_HISTORY or out_commit_tn. */

/* Compact transfer forms (host or device batches; widened on the device before
 * any kernel reads them).  They shrink what a host batch moves over PCIe:
 * u32 keys halve the largest array when the key universe fits (YCSB row ids),
 * packed access types and u32 timestamps cut the rest. */
#define DCC_KEYS_U32 0x10u      /* keys points to uint32_t keys                            */
#define DCC_ACCTYPE_2BIT 0x20u  /* acctype holds 2-bit access types, four per byte: access x
                                   in bits 2(x%4)..2(x%4)+1 of byte x/4                     */
#define DCC_TN_U32 0x40u        /* start_tn / finish_tn point to uint32_t timestamps        */
#define DCC_COMPACT_FLAGS (DCC_KEYS_U32 | DCC_ACCTYPE_2BIT | DCC_TN_U32)
/* Key-sharded contexts (dcc_comm_init*): the batch is the WHOLE epoch; the
 * rank keeps its key shard of the accesses itself (partitioned on the device)
 * and the whole batch for the serial passes, so ranks exchange only kill bits
 * (one fixed-size all-gather per sweep level, no host synchronisation between
 * levels).  Without the flag a rank passes only its own accesses
 * (dcc_shard_filter) and the ranks exchange the serial ranges' records.
 * A multi-GPU context (dcc_init_multi) always shards this way. */
#define DCC_SHARD_SELF 0x80u

/* One epoch as a CSR of per-transaction access lists in capture order
 * (Access list of TxnManager, system/txn.h:39-70; txn.cpp:818-847). */
typedef struct dcc_batch {
  uint64_t n_txn;
  uint64_t nnz;
  const uint32_t* offsets;   /* [n_txn+1]; offsets[0]=0, non-decreasing, offsets[n_txn]=nnz */
  const uint64_t* keys;      /* [nnz] canonical keys, != DCC_KEY_RESERVED                */
  const uint8_t* acctype;    /* [nnz] access_t                                           */
  const uint64_t* start_tn;  /* [n_txn] txn start ts (worker_thread.cpp:500-502) or NULL */
  const uint64_t* finish_tn; /* [n_txn] validation ts (occ.cpp:142) or NULL.  Both NULL
                                disables the history window check, which is exactly
                                the reference behaviour under TS_CLOCK */
  const uint64_t* order;     /* Calvin: [n_txn] sequence key (epoch<<48|origin<<32|seq,
                                any monotone encoding) or NULL = index order             */
  uint32_t flags;
  uint32_t reserved;
} dcc_batch;

typedef struct dcc_stats {
  uint32_t rounds;       /* fixed-point rounds executed                                */
  uint32_t n_shards;     /* GPUs that took part                                        */
  uint64_t n_commit;     /* RCOK decisions (Calvin: ready at acquire)                  */
  uint64_t n_abort;      /* Abort decisions (Calvin: WAIT)                             */
  uint64_t n_readonly;   /* txns with an empty write set                               */
  uint64_t nnz_w;        /* write accesses                                             */
  uint64_t alg_bytes;    /* algorithmic bytes of one pass, SURVEY.md §8(d)             */
  double device_ms;      /* device time of the decision, batch resident                */
  double total_ms;       /* wall time of the call incl. H2D/D2H when host pointers      */
  /* Per-phase device time (HIP events on the engine stream; filled only when
   * profiling is enabled with dcc_set_profiling) and the algorithmic bytes
   * of each phase.  OCC sweep: 0 = level-0 tile records + serial pass,
   * 1 = level-0 filter, 2 = later levels (and any round-solver hand-off),
   * 3 = prep + finalize; round solver only: 0 = key-hash build, 1 = round 1,
   * 2 = rounds >= 2, 3 = prep + finalize.  Calvin: 0 = build, 1 = grant
   * groups, 2 = waves, 3 = prep + finalize. */
  double phase_ms[4];
  uint64_t phase_bytes[4];
  /* OCC sweep: the level-0 serial prefix (0 = the epoch was
   * decided by rounds alone) and the txns that survived the level-0 filter.
   * The sweep reports its levels in `rounds`. */
  uint64_t peel_prefix;
  uint64_t n_survivors;
  uint32_t fallback;     /* sweep lists handed to the round solver (they stopped
                            shrinking); the decisions are the same                    */
  uint32_t fin_where;    /* pipelined epochs with commit tn / append (dcc_occ_wait_epoch):
                            1 numbered on the device behind the decision (chained),
                            2 by the context at completion; 0 otherwise              */
} dcc_stats;

/* ------------------------------------------------------------- context  */
typedef struct dcc_ctx dcc_ctx;

/* Replaces OptCC::init (occ.cpp:33-40) and the global occ_man singleton
 * (system/global.cpp:42): one context per process and device.
 * device_id < 0 selects the current HIP device. */
int dcc_init(dcc_ctx** out, int device_id);
/* One process, n GPUs (multi-GPU internal to the context):
 * the context key-shards every epoch over n per-device sub-contexts
 * (dcc_key_shard) that exchange over one RCCL clique (ncclCommInitAll) when
 * the ids are distinct, else over an in-process host exchange (shards sharing
 * a GPU).  Each sub-context partitions the batch on its own GPU (a host batch
 * is copied to every GPU; a device batch, DCC_DEVICE_PTRS, is read where it
 * lies -- peer access between distinct GPUs is enabled here).  OCC and Calvin
 * epochs return the same decisions as one GPU (device outputs are written by
 * rank 0); options, tnc and history apply to every shard.  Captured-snapshot
 * validation is key-sharded too (each rank against its history shard; a txn
 * commits iff every rank commits it).  Calvin wave levels and MaaT run the
 * whole epoch on rank 0's GPU (the levels chain through every row; MaaT's
 * bounds combine every row of a txn; its row table lives on rank 0).
 * dcc_set_stream is DCC_ENOTSUP on it. */
int dcc_init_multi(dcc_ctx** out, int n_gpus, const int* device_ids);
void dcc_destroy(dcc_ctx* ctx);
const char* dcc_strerror(int code);
const char* dcc_last_error(const dcc_ctx* ctx); /* detail of the last failure */
int dcc_version(void);                            /* 100*major + minor */
int dcc_device_count(void);                       /* gfx950 devices visible (0 if none) */

/* Run on an external HIP stream (opaque hipStream_t, e.g. torch's current
 * stream).  NULL restores the context's own stream. */
int dcc_set_stream(dcc_ctx* ctx, void* hip_stream);
/* Record per-phase HIP events inside every call (dcc_stats.phase_ms). */
int dcc_set_profiling(dcc_ctx* ctx, int enable);
/* Tuning knobs (defaults are the tuned values; for A/B measurement). */
#define DCC_OPT_RECHECK 1     /* fold kill waves into rounds whose list has <= value txns */
#define DCC_OPT_BATCH_MAX 2   /* max rounds enqueued between host synchronisations        */
#define DCC_OPT_SOLVER 5      /* OCC solver: 0 auto (= 3), 1 fixed-point rounds only, 3 sweep
                                 (levels of serial passes + filters; hands lists that stop
                                 shrinking to the round solver)                              */
#define DCC_OPT_SWEEP_LEVELS 6 /* sweep levels enqueued between host synchronisations (0:
                                  auto, 3 with DCC_OPT_RO_SPLIT, 4 without)                  */
#define DCC_OPT_HIST_MERGE 7  /* device history: delta pairs above which the delta merges into
                                 the base (default 65536; the base/4 rule also applies)      */
#define DCC_OPT_RO_SPLIT 10   /* sweep: read-only txns that survive the first level's filter
                                 leave the level lists and are decided once every writer is
                                 (1, default) or stay in the lists (0); one-GPU epochs only.
                                 4..24: on, with 2^value committed-writer table slots (the
                                 table grows after an overflow; tests use small ones)        */
#define DCC_OPT_FAIL_RANK 8   /* fault injection (tests): rank `value` of a multi-GPU context
                                 fails its next epoch before its first exchange; the other
                                 ranks must return DCC_ECOMM instead of waiting for it      */
#define DCC_OPT_PIPELINE 11   /* lanes of dcc_occ_submit_epoch: epochs in flight at once
                                 (1..8, default 3).  Each lane is a HIP stream that needs a
                                 hardware queue of its own: run with GPU_MAX_HW_QUEUES >=
                                 lanes + the caller's streams (HIP's default of 4 makes
                                 lanes share queues, which serialises them)                 */
#define DCC_OPT_CALVIN_PATH 12 /* Calvin grant groups: 0 auto (the bucket path for epochs of
                                  >= 2M requests it applies to), 1 the global key sort + scan,
                                  2 the bucket path wherever it applies                       */
#define DCC_OPT_COMM_SOLO 13  /* tests: with 1, a later dcc_comm_init(ctx, 0, 1, id) forms a
                                 one-rank RCCL clique and the context runs the key-sharded
                                 paths with their collectives (ncclAllReduce / ncclAllGather
                                 over the one rank) instead of the one-GPU paths: the RCCL
                                 call path executes on a one-GPU box                         */
#define DCC_OPT_PIPE_PARTITION 14 /* pipeline lanes on their own CUs: 0 every lane on the whole
                                  chip; 1 lane i of L on 1/L of the CUs of every XCD (its
                                  stream CU-masked), so a lane's serial passes never queue
                                  behind another lane's chip-wide kernels (L must divide
                                  n_CU / 8; otherwise the lanes stay unmasked)             */
#define DCC_OPT_PIPE_CHAIN 15 /* pipelined epochs with commit tn / history append: 1 (default)
                                 each lane numbers and appends its epoch on the device right
                                 after deciding it, from a device copy of tnc and the append
                                 position that the epochs advance in submit order; 0 the
                                 context finishes each epoch on its lane's completion     */
int dcc_set_option(dcc_ctx* ctx, int option, int64_t value);
/* Pre-size device workspaces so a later call performs no allocation. */
int dcc_reserve(dcc_ctx* ctx, uint64_t max_txn, uint64_t max_nnz);
/* Achievable HBM bandwidth on this device (measurement aid):
 * hand-written 16-byte-per-lane copy kernels over two `bytes`-sized device
 * buffers (grid-stride; one contiguous range per workgroup with non-temporal
 * loads and stores at 2 / 4 / 8 workgroups per CU), `reps` launches of each
 * timed with HIP events; *gbps = 2 * bytes / time of the fastest form. */
int dcc_copy_bandwidth(dcc_ctx* ctx, uint64_t bytes, int reps, double* gbps);
/* Pinned (page-locked) host memory for batches and outputs: a host batch in it
 * is copied at DMA speed with no staging copy.  Free with dcc_host_free. */
int dcc_host_alloc(dcc_ctx* ctx, uint64_t bytes, void** out);
int dcc_host_free(dcc_ctx* ctx, void* p);  /* ctx may be NULL */

/* ------------------------------------------------------- multi-GPU     */
/* Key sharding across the GPUs of one node, one process per GPU
 * (SURVEY.md §8(e)).  Each rank owns keys with dcc_key_shard(key, n) == rank,
 * receives the full per-txn offsets plus only its own accesses, and joins a
 * per-round RCCL ncclMax allreduce of per-txn state bytes — the MI355X form
 * of 2PC's AND of per-node OK bits (worker_thread.cpp:328-334). */
#define DCC_UNIQUE_ID_BYTES 128
int dcc_comm_unique_id(void* out_id /* DCC_UNIQUE_ID_BYTES */);
/* RCCL communicator: every rank passes rank 0's unique id. */
int dcc_comm_init(dcc_ctx* ctx, int rank, int nranks, const void* unique_id);
/* Host-exchange communicator: `fn` all-reduces n bytes in place with MAX
 * across the ranks (returns 0 on success).  For harnesses whose ranks cannot
 * form an RCCL clique, e.g. several ranks sharing one GPU in tests. */
typedef int (*dcc_exchange_fn)(void* user, uint8_t* host_buf, uint64_t n);
int dcc_comm_init_host(dcc_ctx* ctx, int rank, int nranks, dcc_exchange_fn fn, void* user);
int dcc_comm_destroy(dcc_ctx* ctx);
int dcc_comm_rank(const dcc_ctx* ctx);
int dcc_comm_size(const dcc_ctx* ctx);
/* Collectives this context's communicator has run since dcc_comm_init (RCCL
 * calls enqueued, or host exchanges); 0 without a communicator. */
uint64_t dcc_comm_calls(const dcc_ctx* ctx);
uint32_t dcc_key_shard(uint64_t key, uint32_t nranks);
/* dcc_key_shard of n keys (host arrays): out[i] = shard of keys[i] */
int dcc_key_shard_n(const uint64_t* keys, uint64_t n, uint32_t nranks, uint32_t* out);
/* Host helper: keep only the accesses of `rank` (same n_txn, same order).
 * out_offsets [n_txn+1]; out_keys/out_acctype sized >= in nnz; *out_nnz set. */
int dcc_shard_filter(const dcc_batch* in, uint32_t rank, uint32_t nranks,
                     uint32_t* out_offsets, uint64_t* out_keys,
                     uint8_t* out_acctype, uint64_t* out_nnz);

/* ------------------------------------------------------------------ OCC */
/* Epoch validation: the result equals validating every txn of the batch in
 * index order with OptCC::central_validate (occ.cpp:116-239) and only then
 * finishing all of them with central_finish (occ.cpp:248-294).
 *   out_rc[i]        = DCC_RC_RCOK or DCC_RC_ABORT (TxnManager::validate, txn.cpp:935)
 *   out_commit_tn[i] = history tn given to committed non-read-only txns, else 0
 *                      (tnc++ / wset->tn = tnc, occ.cpp:283-284); may be NULL. */
int dcc_occ_validate_epoch(dcc_ctx* ctx, const dcc_batch* batch, uint8_t* out_rc,
                           uint64_t* out_commit_tn, dcc_stats* out_stats);
/* (Any entry point: when a call returns an error, the contents of its output
 * arrays are unspecified -- e.g. a malformed host batch, whose offsets the
 * device checks, may already have been decided into out_rc.) */
/* Pipelined epochs (one GPU).  dcc_occ_submit_epoch enqueues an epoch and
 * returns without waiting for it.  Consecutive epochs run on separate lanes
 * (DCC_OPT_PIPELINE of them, each with its own stream, workspaces and
 * captured graph), so one epoch's latency-bound serial passes overlap the
 * next epoch's streaming passes.  The results are exactly those of calling
 * dcc_occ_validate_epoch on the epochs in submit order: under TS_CLOCK (no
 * history window) epochs of central_validate are
 * independent except for central_finish's commit counter and history
 * (occ.cpp:277-286), so each lane decides its epoch and its central_finish --
 * commit tn (out_commit_tn) and the DCC_OCC_APPEND_HISTORY append -- runs in
 * submit order: on the device right after the decision, once the epoch before
 * it has finished (DCC_OPT_PIPE_CHAIN), or by the context when the epoch
 * completes.  An epoch that fails after its finish ran on the device fails
 * the epochs in flight behind it too (their numbering followed it).  An epoch that needs the epochs before it finished -- a window
 * against a non-empty history or against appends still in flight,
 * DCC_OCC_DEFER_FINISH -- or profiling, the round solver, or a multi-GPU or
 * key-sharded context first drains the pipeline and then runs
 * synchronously, still in submit order.  The batch arrays and the outputs
 * must stay valid and unchanged until the epoch's dcc_occ_wait_epoch
 * returns.  *out_ticket (1, 2, ...) names the epoch.  Argument errors are
 * returned by submit; the epoch's own result by wait.
 * dcc_occ_wait_epoch completes, in submit order, every epoch up to `ticket`
 * and returns that epoch's status and stats.  Each ticket is waited once;
 * earlier tickets keep their results until they are waited.  Every other
 * OCC entry point on the context (validate, finish, history, tnc) first
 * completes the epochs in flight. */
int dcc_occ_submit_epoch(dcc_ctx* ctx, const dcc_batch* batch, uint8_t* out_rc,
                         uint64_t* out_commit_tn, uint64_t* out_ticket);
int dcc_occ_wait_epoch(dcc_ctx* ctx, uint64_t ticket, dcc_stats* out_stats);
/* central_finish with the global decision, for an epoch validated with
 * DCC_OCC_DEFER_FINISH (each node votes with its local RC; 2PC's coordinator
 * commits only if every participant voted RCOK, worker_thread.cpp:328-334,
 * and RFIN carries that RC back, worker_thread.cpp:286-297):
 *   final_rc[i] = DCC_RC_RCOK or DCC_RC_ABORT, the global RC of txn i;
 * committed non-read-only txns (global RCOK) take tn = tnc+1, tnc+2, ... in
 * index order and their write sets join the history; a txn aborted globally
 * leaves no trace even if it validated locally.  DCC_EINVAL if a txn has
 * final RCOK but aborted locally (2PC never commits it) or no epoch is
 * pending.  flags: DCC_DEVICE_PTRS when final_rc / out_commit_tn are device
 * memory.  The deferred epoch's device batch (DCC_DEVICE_PTRS) must stay
 * valid until this call; every other OCC epoch is refused meanwhile. */
int dcc_occ_finish_epoch(dcc_ctx* ctx, const uint8_t* final_rc, uint64_t* out_commit_tn,
                         uint32_t flags);
/* Committed write sets of earlier epochs (the `history` list, occ.h:62-64).
 * keys/tn are host arrays of n (key, tn) pairs; each pair is one write of the
 * committed txn numbered tn.  The history is device-resident: epochs with
 * DCC_OCC_APPEND_HISTORY append their committed writes on the device. */
int dcc_occ_history_append(dcc_ctx* ctx, const uint64_t* keys, const uint64_t* tn, uint64_t n);
int dcc_occ_history_clear(dcc_ctx* ctx);
uint64_t dcc_occ_history_size(const dcc_ctx* ctx);
/* Drop every history entry with tn <= tn_floor.  The reference never frees
 * history (occ.cpp:277-286 only pushes); an entry is visible to
 * a window (start_tn, finish_tn] only if tn > start_tn, so a caller that knows
 * no txn will ever validate with start_tn < tn_floor can bound the history. */
int dcc_occ_history_trim(dcc_ctx* ctx, uint64_t tn_floor);
/* Copy the history's (key, tn) pairs to host arrays of cap entries (any
 * order); *out_n = the history size.  DCC_ERANGE when cap is too small. */
int dcc_occ_history_export(dcc_ctx* ctx, uint64_t* keys, uint64_t* tn, uint64_t cap,
                           uint64_t* out_n);
/* The commit counter `tnc` (occ.h:67). */
int dcc_occ_set_tnc(dcc_ctx* ctx, uint64_t tnc);
uint64_t dcc_occ_get_tnc(const dcc_ctx* ctx);

/* Captured-snapshot validation.  A live, genuinely
 * concurrent run records, for every validating txn, what its critical section
 * saw (occ.cpp:137-158): the history head and the active list.  Every txn is
 * then validated independently and in parallel against exactly that snapshot,
 * reproducing central_validate's decision (occ.cpp:116-239) bit for bit.
 *   hist_top[i]   tn of the history head at i's critical section: entries with
 *                 tn > hist_top[i] were pushed later and are invisible to i.
 *                 NULL = the whole context history is visible.
 *   active_off    [n_txn+1] CSR; active_idx[active_off[i] .. active_off[i+1])
 *                 are the batch indices of the txns whose write sets were on the
 *                 active list (finish_active, occ.cpp:146-150) when i entered.
 * The history itself is the context's (dcc_occ_history_append).  start_tn /
 * finish_tn of the batch open the window exactly as in central_validate
 * (checked against the read set only, occ.cpp:167-180); the active check is
 * against the read set, then the write set (occ.cpp:185-199).  Pointers are
 * device memory when batch->flags has DCC_DEVICE_PTRS (then out_rc too).
 * Nothing is committed: central_finish of a live run is the caller's.
 * Stats: n_commit, n_abort, n_readonly, nnz_w, device_ms, total_ms, alg_bytes. */
typedef struct dcc_occ_snapshot {
  const uint64_t* hist_top;   /* [n_txn] or NULL */
  const uint32_t* active_off; /* [n_txn+1] */
  const uint32_t* active_idx; /* [active_off[n_txn]] indices < n_txn */
} dcc_occ_snapshot;
int dcc_occ_validate_snapshot(dcc_ctx* ctx, const dcc_batch* batch, const dcc_occ_snapshot* snap,
                              uint8_t* out_rc, dcc_stats* out_stats);

/* ----------------------------------------------------------------- MaaT */
/* MaaT epoch validation.  Epoch model: every txn of
 * the batch is initialised in the time table ([0, UINT64_MAX], RUNNING;
 * worker_thread.cpp:503-508) and performs its Row_maat accesses in index
 * order (RD -> read, WR -> prewrite, XP/SCAN -> none; with
 * DCC_MAAT_READ_AND_PREWRITE every access does read_and_prewrite,
 * row_maat.cpp:38-164); then, in index order, each txn runs Maat::validate
 * and find_bound (maat.cpp:29-191; the node is the home node) and commits
 * (Row_maat::commit with the forward validation of the later txns still on
 * its rows, row_maat.cpp:189-314) or aborts (row_maat.cpp:167-187).
 *   out_rc[i]        = DCC_RC_RCOK or DCC_RC_ABORT
 *   out_commit_ts[i] = commit_timestamp (the lower bound find_bound picks) or 0
 * Row timestamps (timestamp_last_read / _write, row_maat.h:38-39) persist in
 * the context across epochs; rows never seen start at 0.
 * Stats: n_commit, n_abort, nnz_w, rounds (of the GPU fixed point),
 * device_ms, total_ms, alg_bytes (dcc_maat_alg_bytes). */
int dcc_maat_validate_epoch(dcc_ctx* ctx, const dcc_batch* batch, uint8_t* out_rc,
                            uint64_t* out_commit_ts, dcc_stats* out_stats);
/* Row timestamps: seed (overwrite) / read (0 for unknown rows) / forget.
 * Host arrays of n entries. */
int dcc_maat_rows_set(dcc_ctx* ctx, const uint64_t* keys, const uint64_t* last_read,
                      const uint64_t* last_write, uint64_t n);
int dcc_maat_rows_get(dcc_ctx* ctx, const uint64_t* keys, uint64_t* last_read,
                      uint64_t* last_write, uint64_t n);
int dcc_maat_rows_clear(dcc_ctx* ctx);
uint64_t dcc_maat_rows_size(const dcc_ctx* ctx);
/* Algorithmic bytes of one MaaT epoch: 4(N+1) offsets + 9 nnz (key, type)
 * + 24 nnz (row slot: key, last read, last write) + 8 nnz (timestamp update)
 * + N (RC) + 8 N (commit timestamp). */
uint64_t dcc_maat_alg_bytes(uint64_t n_txn, uint64_t nnz);

/* --------------------------------------------------------------- Calvin */
/* Epoch lock ordering: the result equals the epoch's txns calling
 * acquire_locks (ycsb_txn.cpp:49-88) in sequence order against an empty
 * Row_lock table in CALVIN mode (row_lock.cpp:52-216), with per-txn row
 * de-duplication (txn.cpp:778-782) and RD/SCAN->SH, else EX (row.cpp:191).
 *   out_group[a] = grant group of request a on its row: 0 = granted at
 *                  acquire, g = granted when group g-1 has fully released
 *                  (lock_release promotion, row_lock.cpp:317-357);
 *                  DCC_GROUP_NONE for a de-duplicated request.  May be NULL.
 *   out_rc[i]    = DCC_RC_RCOK if every request is in group 0, else DCC_RC_WAIT
 *                  (acquire_locks' return).
 *   out_wave[i]  = wave in which txn i runs when every txn releases all its
 *                  locks one wave after it became ready (may be NULL).
 * batch->order (may be NULL = index order) is the sequencer's order key
 * (origin << 32 | seq); ties keep index order.
 * n_txn < 2^25.  Stats: n_commit = txns ready at acquire (RCOK), n_abort =
 * txns that WAIT, nnz_w = EX requests, rounds = number of waves (0 when
 * out_wave is NULL). */
int dcc_calvin_order_epoch(dcc_ctx* ctx, const dcc_batch* batch, uint32_t* out_group,
                           uint8_t* out_rc, uint32_t* out_wave, dcc_stats* out_stats);

/* Rows still locked when the epoch starts.  Releases are asynchronous
 * (Row_lock::lock_release, row_lock.cpp:219-372), so the lock thread may
 * acquire an epoch while rows are still owned, or queued for, by txns of an
 * earlier epoch.  The held prefix lists those requests per row in FIFO order:
 * the current owners first, then the waiters (any interleaving of rows; the
 * order among one row's requests is the queue order).  They enter the same
 * per-row order ahead of the epoch's requests, so:
 *   out_group[a] counts group boundaries from the row's owners (group 0 = the
 *                current owners; an epoch request in group 0 joins them),
 *   out_rc[i]    = RCOK iff every request of txn i joins its row's owners.
 * Equal to replaying the prefix requests, then the epoch, through Row_lock in
 * CALVIN mode.  Host arrays, or device arrays when batch->flags has
 * DCC_DEVICE_PTRS.  Wave levels need an empty table: out_wave must be NULL
 * (DCC_ENOTSUP otherwise).  Key-sharded: each rank passes its own rows. */
typedef struct dcc_calvin_held {
  uint64_t n;              /* held requests                                 */
  const uint64_t* keys;    /* [n] rows                                      */
  const uint8_t* acctype;  /* [n] access_t (RD/SCAN -> SH, else EX)         */
} dcc_calvin_held;
int dcc_calvin_order_epoch_held(dcc_ctx* ctx, const dcc_batch* batch, const dcc_calvin_held* held,
                                uint32_t* out_group, uint8_t* out_rc, uint32_t* out_wave,
                                dcc_stats* out_stats);

/* Wave dispatch: the wave levels of an epoch
 * (out_wave of dcc_calvin_order_epoch) as the lists a dispatcher releases:
 * out_txn[out_wave_off[w] .. out_wave_off[w+1]) = the txns of wave w in
 * sequence order (order = the batch's sequencer key, NULL = index order;
 * ties keep index order).  Wave w+1 starts once every txn of wave w has
 * released its locks (TxnTable::restart_txn, txn_table.cpp:151-176, after the
 * lock_release promotions of row_lock.cpp:317-357).  *out_n_waves = max
 * wave + 1; out_wave_off needs *out_n_waves + 1 entries (off_cap; may be NULL
 * to query the count).  Device pointers with DCC_DEVICE_PTRS in flags. */
int dcc_calvin_dispatch(dcc_ctx* ctx, const uint32_t* wave, const uint64_t* order, uint64_t n,
                        uint32_t flags, uint32_t* out_wave_off, uint64_t off_cap,
                        uint32_t* out_txn, uint32_t* out_n_waves);

/* ------------------------------------------------------------ GPU index */
/* The key -> row lookups execution does through IndexHash (index_insert /
 * index_read, storage/index_hash.cpp:58-137, 160-231) as one HBM table probed
 * for a whole epoch's accesses at once.  A key inserted more than once reads
 * as its newest insert (insert_item prepends, read_item takes the head); a
 * missing key (the reference's M_ASSERT_V, index_hash.cpp:221) reads as
 * DCC_ROW_NONE and is counted in *out_missing. */
#define DCC_ROW_NONE 0xFFFFFFFFFFFFFFFFull
int dcc_index_insert(dcc_ctx* ctx, const uint64_t* keys, const uint64_t* rows, uint64_t n);
/* keys / out_rows: host arrays, or device arrays with DCC_DEVICE_PTRS in flags */
int dcc_index_probe(dcc_ctx* ctx, const uint64_t* keys, uint64_t n, uint64_t* out_rows,
                    uint32_t flags, uint64_t* out_missing);
int dcc_index_clear(dcc_ctx* ctx);
uint64_t dcc_index_size(const dcc_ctx* ctx);      /* distinct keys            */
double dcc_index_last_ms(const dcc_ctx* ctx);     /* device ms of the last probe */

/* ----------------------------------------------------- batch producers */
/* Deterministic restatements of the reference workload generators
 * (SURVEY.md §8(a) a17/a18).  The reference seeds from the clock
 * (ycsb_query.cpp:31); here every chunk of `chunk_txns` transactions draws
 * from its own myrand stream (helper.cpp:144-147) seeded from `seed` and the
 * chunk index, so batches are reproducible and can be generated in parallel. */
typedef struct dcc_ycsb_params {
  uint64_t n_txn;
  uint32_t req_per_query;   /* REQ_PER_QUERY (config.h:177)                    */
  uint32_t part_cnt;        /* PART_CNT                                        */
  uint64_t table_size;      /* SYNTH_TABLE_SIZE (config.h:169)                 */
  double zipf_theta;        /* ZIPF_THETA                                      */
  double txn_write_perc;    /* TXN_WRITE_PERC                                  */
  double tup_write_perc;    /* TUP_WRITE_PERC                                  */
  uint32_t part_per_txn;    /* PART_PER_TXN (used with strict_ppt)             */
  uint32_t strict_ppt;      /* STRICT_PPT                                      */
  uint32_t first_part_local;/* FIRST_PART_LOCAL                                */
  uint32_t chunk_txns;      /* txns per generator stream; also the txns per
                               origin node for Calvin (home partition =
                               chunk index % part_cnt)                         */
  uint64_t seed;
  uint32_t n_threads;       /* host threads used to generate (0 = auto)        */
  uint32_t reserved;
} dcc_ycsb_params;
void dcc_ycsb_params_default(dcc_ycsb_params* p);
/* offsets [n_txn+1], keys/acctype [n_txn*req_per_query]; home may be NULL. */
int dcc_gen_ycsb(const dcc_ycsb_params* p, uint32_t* offsets, uint64_t* keys,
                 uint8_t* acctype, uint32_t* home);

typedef struct dcc_tpcc_params {
  uint64_t n_txn;
  uint32_t num_wh;          /* NUM_WH                                          */
  uint32_t part_cnt;        /* PART_CNT (wh_to_part, tpcc_helper.cpp:161-164)  */
  double perc_payment;      /* PERC_PAYMENT                                    */
  uint32_t wh_update;       /* WH_UPDATE (config.h:194)                        */
  uint32_t max_items;       /* MAX_ITEMS_NORM (config.h:187)                   */
  uint32_t cust_per_dist;   /* CUST_PER_DIST_NORM (config.h:188)               */
  uint32_t dist_per_wh;     /* DIST_PER_WH (config.h:223)                      */
  uint32_t max_items_per_txn; /* MAX_ITEMS_PER_TXN (config.h:189)              */
  uint32_t part_per_txn;
  double mpr;               /* MPR                                             */
  uint32_t first_part_local;
  uint32_t chunk_txns;
  uint64_t seed;
  uint32_t n_threads;
  uint32_t reserved;
} dcc_tpcc_params;
void dcc_tpcc_params_default(dcc_tpcc_params* p);
/* Upper bound of accesses per TPC-C txn (NewOrder: 3 + 2*MAX_ITEMS_PER_TXN). */
uint32_t dcc_tpcc_max_access(const dcc_tpcc_params* p);
/* offsets [n_txn+1]; keys/acctype sized n_txn*dcc_tpcc_max_access(p);
 * txn_type [n_txn] (TPCCTxnType: 1 = PAYMENT, 2 = NEW_ORDER) may be NULL. */
int dcc_gen_tpcc(const dcc_tpcc_params* p, uint32_t* offsets, uint64_t* keys,
                 uint8_t* acctype, uint8_t* txn_type, uint64_t* out_nnz);

/* Canonical TPC-C key: (table_id << 56) | index key. */
#define DCC_TPCC_KEY(table_id, ikey) ((((uint64_t)(table_id)) << 56) | ((uint64_t)(ikey)))

/* ------------------------------------------------- batch files (.dccb) */
/* One captured epoch on disk: the CSR access lists,
 * optional timestamps / sequencer order, optional decisions.  Versioned,
 * checksummed (FNV-1a 64), little-endian; layout in batch_file.cpp.  Host
 * pointers only.  Version 2's checksum also covers the header fields. */
#define DCC_FILE_VERSION 2   /* written; version 1 files are still read */
#define DCC_FILE_OCC 1
#define DCC_FILE_CALVIN 2
#define DCC_FILE_HAS_TN 0x1u         /* start_tn + finish_tn                     */
#define DCC_FILE_HAS_ORDER 0x2u      /* Calvin sequencer order                   */
#define DCC_FILE_HAS_RC 0x4u         /* per-txn RC                               */
#define DCC_FILE_HAS_COMMIT_TN 0x8u  /* OCC history tn of committed writers      */
#define DCC_FILE_HAS_GROUP 0x10u     /* Calvin grant group per request           */
#define DCC_FILE_HAS_WAVE 0x20u      /* Calvin wave per txn                      */
typedef struct dcc_file_info {
  uint32_t version;     /* DCC_FILE_VERSION                                      */
  uint32_t kind;        /* DCC_FILE_OCC / DCC_FILE_CALVIN                        */
  uint32_t sections;    /* DCC_FILE_HAS_* bits present (read); ignored on write  */
  uint32_t reserved;
  uint64_t n_txn, nnz;  /* read only (taken from the batch on write)             */
  uint64_t seed;        /* generator seed or capture id                          */
  uint64_t epoch;       /* epoch number within a capture                         */
  uint64_t tnc_before;  /* OCC commit counter before the epoch (occ.h:67)        */
} dcc_file_info;
/* Sections are written for every non-NULL array (start_tn/finish_tn/order from
 * the batch).  Returns DCC_EIO on a file error. */
int dcc_file_write(const char* path, const dcc_file_info* info, const dcc_batch* batch,
                   const uint8_t* rc, const uint64_t* commit_tn, const uint32_t* group,
                   const uint32_t* wave);
int dcc_file_read_info(const char* path, dcc_file_info* info);
/* Fills every non-NULL destination whose section is present (size them from
 * dcc_file_read_info).  DCC_EINVAL: bad magic, truncated, checksum or offsets
 * mismatch; DCC_ENOTSUP: another format version. */
int dcc_file_read(const char* path, uint32_t* offsets, uint64_t* keys, uint8_t* acctype,
                  uint64_t* start_tn, uint64_t* finish_tn, uint64_t* order, uint8_t* rc,
                  uint64_t* commit_tn, uint32_t* group, uint32_t* wave);

/* Algorithmic bytes of one epoch pass:
 * 4(N+1) + 9 nnz + 16 nnz_w + 16 nnz + N. */
uint64_t dcc_alg_bytes(uint64_t n_txn, uint64_t nnz, uint64_t nnz_w);
/* Algorithmic bytes of one Calvin epoch: 4(N+1) offsets + 9 nnz (key, type)
 * + 4 nnz (grant group) + N (RC) [+ 8N order] [+ 4N wave]. */
uint64_t dcc_calvin_alg_bytes(uint64_t n_txn, uint64_t nnz, int with_order, int with_wave);

#ifdef __cplusplus
}
#endif
#endif /* DCC_H_ */
