/*
 * oracle.h — CPU restatements of the reference's hot-path algorithms.
 *
 * TEST INFRASTRUCTURE ONLY.  Nothing under oracle/ is linked into, loaded by
 * or called from libdcc or the deneva_amd package; only tests/,
 * __graft_entry__.smoke() and bench.py's cpu_baseline leg use it, as the
 * checker.
 *
 * Pinning: the reference repository holds no tests, fixtures or golden
 * vectors for this path, its full build needs boost/lockfree,
 * nanomsg and jemalloc, which this image lacks, and there
 * is no Python reference.  The restatements are therefore "parity unpinned"
 * against reference outputs: each function cites the file:line it follows,
 * two independent restatements per algorithm cross-check each other, and
 * hand-derived known-answer cases from the reference source are committed
 * under tests/golden/.
 */
#ifndef DCC_ORACLE_H_
#define DCC_ORACLE_H_
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* Literal epoch replay of OptCC central validation:
 *   for i in index order: central_validate(i)   concurrency_control/occ.cpp:116-239
 *   then  for i in index order: central_finish(rc_i, i)   occ.cpp:248-294
 * with active/history as singly linked stacks (occ.h:62-64) and test_valid as
 * the |set1|x|set2| pointer-compare loop (occ.cpp:319-327).
 * start_tn/finish_tn may be NULL (TS_CLOCK: the history window never opens).
 * hist_keys/hist_tn: n_hist (key, tn) pairs of earlier committed write sets.
 * out_rc[i] = 0 (RCOK) or 2 (Abort); out_tn[i] = history tn or 0; *tnc updated.
 * Returns 0, or -1 on allocation failure. */
int oracle_occ_replay(uint64_t n, const uint32_t* off, const uint64_t* keys, const uint8_t* acctype,
                      const uint64_t* start_tn, const uint64_t* finish_tn, uint64_t n_hist,
                      const uint64_t* hist_keys, const uint64_t* hist_tn, uint64_t* tnc,
                      uint8_t* out_rc, uint64_t* out_tn);

/* Independent restatement: serial hash-set scan.  i aborts iff its history
 * window hits, or (R_i ∪ W_i) meets the union of W_j of earlier committed j. */
int oracle_occ_hash(uint64_t n, const uint32_t* off, const uint64_t* keys, const uint8_t* acctype,
                    const uint64_t* start_tn, const uint64_t* finish_tn, uint64_t n_hist,
                    const uint64_t* hist_keys, const uint64_t* hist_tn, uint64_t* tnc,
                    uint8_t* out_rc, uint64_t* out_tn);

/* ROUNDS-MT (occ_mt.c): the round-based fixed point on `nthreads` host
 * threads, the parallel CPU baseline of SURVEY.md §8(d).  Same decisions as
 * oracle_occ_hash without a history window; out_tn / *tnc as there.
 * *out_rounds = rounds executed.  Returns 0, -1 on allocation failure. */
int oracle_occ_rounds_mt(uint64_t n, const uint32_t* off, const uint64_t* keys,
                         const uint8_t* acctype, int nthreads, uint64_t* tnc, uint8_t* out_rc,
                         uint64_t* out_tn, uint32_t* out_rounds);

/* SWEEP-MT (occ_sweep_mt.c): the CPU form of the GPU sweep on `nthreads`
 * host threads -- per level a serial prefix (one thread) building the
 * committed write-key set, then a parallel read-only filter of the rest.
 * Same decisions and out_tn / *tnc as oracle_occ_hash without a history
 * window; *out_levels = levels run.  Returns 0, -1 on allocation failure. */
int oracle_occ_sweep_mt(uint64_t n, const uint32_t* off, const uint64_t* keys,
                        const uint8_t* acctype, int nthreads, uint64_t* tnc, uint8_t* out_rc,
                        uint64_t* out_tn, uint32_t* out_levels);

/* Captured-snapshot validation, literal (central_validate, occ.cpp:116-239,
 * against each txn's captured critical-section view, occ.cpp:137-158):
 * hist_top[t] = tn of the history head t saw (NULL = all visible);
 * active_idx[active_off[t] .. active_off[t+1]) = finish_active of t.
 * out_rc[t] = 0 (RCOK) or 2 (Abort).  Returns 0, or -1 on allocation failure. */
int oracle_occ_snapshot(uint64_t n, const uint32_t* off, const uint64_t* keys,
                        const uint8_t* acctype, const uint64_t* start_tn,
                        const uint64_t* finish_tn, const uint64_t* hist_top,
                        const uint32_t* active_off, const uint32_t* active_idx, uint64_t n_hist,
                        const uint64_t* hist_keys, const uint64_t* hist_tn, uint8_t* out_rc);

/* Round-based fixed point (the algorithm the GPU runs), one shard's view:
 * given the global per-txn state (0 undecided, 1 commit, 2 abort) at the start
 * of a round and this shard's accesses, return per-txn status bits
 * (1 = blocked by an undecided earlier writer, 2 = killed by a committed
 * earlier writer) for every undecided txn.  Used by the gloo multi-rank tests
 * of the sharded protocol. */
int oracle_occ_round_status(uint64_t n, const uint32_t* off, const uint64_t* keys,
                            const uint8_t* acctype, const uint8_t* state, uint8_t* out_status);

/* Calvin, literal: every txn in sequence order calls acquire_locks
 * (ycsb_txn.cpp:49-88) against Row_lock in CALVIN mode (row_lock.cpp:52-216),
 * de-duplicating rows per txn (txn.cpp:778-782, first type wins) and mapping
 * RD/SCAN->SH, else EX (row.cpp:191); then ready txns run in waves and release
 * all their locks (lock_release + promotion, row_lock.cpp:219-372).
 * order may be NULL (index order).  out_group [nnz] (0xFFFFFFFF for a
 * de-duplicated request), out_rc [n] (0 RCOK / 3 WAIT), out_wave [n]. */
int oracle_calvin_replay(uint64_t n, const uint32_t* off, const uint64_t* keys,
                         const uint8_t* acctype, const uint64_t* order, uint32_t* out_group,
                         uint8_t* out_rc, uint32_t* out_wave);

/* Independent restatement: per-key FIFO formula:
 * group = index of the request's run (SH runs / EX singletons) on its row;
 * wave(i) = max over its rows of EX: max(lastEX, maxSH_since)+1, SH: lastEX+1. */
int oracle_calvin_formula(uint64_t n, const uint32_t* off, const uint64_t* keys,
                          const uint8_t* acctype, const uint64_t* order, uint32_t* out_group,
                          uint8_t* out_rc, uint32_t* out_wave);

/* MaaT epoch validation (maat_ref.c): every txn of the epoch executes its
 * Row_maat accesses in index order (row_maat.cpp:38-164), then, in index
 * order, Maat::validate + find_bound (maat.cpp:29-191) and commit
 * (Row_maat::commit, row_maat.cpp:189-314, cleanup in reverse access order)
 * or abort (row_maat.cpp:167-187), with time_table.release after each.
 * rw_all != 0: the TPC-C path (read_and_prewrite for every access).
 * row_keys/row_lr/row_lw [n_rows]: timestamp_last_read / _write per row, in
 * (before the epoch; unlisted rows start at 0) and out (after it).
 * out_rc[i] = 0 RCOK / 2 Abort; out_cts[i] = commit timestamp or 0. */
int oracle_maat_replay(uint64_t n, const uint32_t* off, const uint64_t* keys, const uint8_t* acctype,
                       int rw_all, uint64_t n_rows, const uint64_t* row_keys, uint64_t* row_lr,
                       uint64_t* row_lw, uint8_t* out_rc, uint64_t* out_cts);
/* Independent restatement of the same epoch: the per-row running maxima /
 * minima of committed readers' / writers' commit timestamps (see maat_ref.c). */
int oracle_maat_formula(uint64_t n, const uint32_t* off, const uint64_t* keys, const uint8_t* acctype,
                        int rw_all, uint64_t n_rows, const uint64_t* row_keys, uint64_t* row_lr,
                        uint64_t* row_lw, uint8_t* out_rc, uint64_t* out_cts);

#ifdef __cplusplus
}
#endif
#endif
