/* maat_ref.c — CPU restatements of MaaT validation for one epoch.
 *
 * TEST INFRASTRUCTURE ONLY (see oracle.h): the checker of the GPU MaaT
 * engine, never linked into libdcc.
 *
 * The epoch model (include/dcc.h, dcc_maat_validate_epoch): every txn of the
 * epoch is initialised in the time table (lower 0, upper UINT64_MAX, RUNNING;
 * worker_thread.cpp:503-508) and executes its accesses in index order
 * (Row_maat::access, row_maat.cpp:38-52); then, in index order, each txn
 * validates (Maat::validate, maat.cpp:29-174, then find_bound, maat.cpp:
 * 176-190, TxnManager::validate, txn.cpp:946-951) and is committed
 * (TxnManager::commit, txn.cpp:427-432: cleanup in reverse access order,
 * txn.cpp:747-760, Row_maat::commit row_maat.cpp:189-314, time_table.release)
 * or aborted (txn.cpp:445-463, Row_maat::abort row_maat.cpp:167-187).
 *
 * Row timestamps (timestamp_last_read / _write, row_maat.h:38-39) carry over
 * between epochs: row_keys[n_rows] with row_lr / row_lw in/out (keys the batch
 * touches must all be listed; unlisted rows start at 0).
 *
 * out_rc[i] = 0 (RCOK) or 2 (Abort); out_cts[i] = commit_timestamp (the lower
 * bound find_bound picks) or 0.
 */
#include <stdlib.h>
#include <string.h>

#include "kmap.h"
#include "oracle.h"

#define RC_RCOK 0
#define RC_ABORT 2
enum { MAAT_RUNNING = 0, MAAT_VALIDATED, MAAT_ABORTED, MAAT_COMMITTED };
#define ACC_RD 0
#define ACC_WR 1
#define U64MAX 0xFFFFFFFFFFFFFFFFull

/* ---- sorted unique id sets (std::set<uint64_t> of the reference) */
typedef struct {
  uint64_t* v;
  uint64_t n, cap;
} idset;

static int is_push(idset* s, uint64_t x) {
  if (s->n == s->cap) {
    uint64_t c = s->cap ? 2 * s->cap : 8;
    uint64_t* nv = (uint64_t*)realloc(s->v, c * 8);
    if (!nv) return -1;
    s->v = nv;
    s->cap = c;
  }
  s->v[s->n++] = x;
  return 0;
}
static int64_t is_find(const idset* s, uint64_t x) {
  uint64_t lo = 0, hi = s->n;
  while (lo < hi) {
    const uint64_t m = (lo + hi) / 2;
    if (s->v[m] < x) lo = m + 1;
    else hi = m;
  }
  return (lo < s->n && s->v[lo] == x) ? (int64_t)lo : -1;
}
static int is_count(const idset* s, uint64_t x) { return is_find(s, x) >= 0; }
static int is_insert(idset* s, uint64_t x) {
  if (s->n == 0 || s->v[s->n - 1] < x) return is_push(s, x);
  if (is_find(s, x) >= 0) return 0;
  if (is_push(s, x)) return -1;
  uint64_t p = s->n - 1;
  while (p > 0 && s->v[p - 1] > x) {
    s->v[p] = s->v[p - 1];
    p--;
  }
  s->v[p] = x;
  return 0;
}
static void is_erase(idset* s, uint64_t x) {
  const int64_t p = is_find(s, x);
  if (p < 0) return;
  memmove(s->v + p, s->v + p + 1, (s->n - (uint64_t)p - 1) * 8);
  s->n--;
}
/* dst |= src (both sorted) */
static int is_union(idset* dst, const idset* src) {
  if (!src->n) return 0;
  idset r = {NULL, 0, 0};
  uint64_t a = 0, b = 0;
  while (a < dst->n || b < src->n) {
    uint64_t x;
    if (b >= src->n || (a < dst->n && dst->v[a] < src->v[b])) x = dst->v[a++];
    else if (a >= dst->n || src->v[b] < dst->v[a]) x = src->v[b++];
    else {
      x = dst->v[a++];
      b++;
    }
    if (is_push(&r, x)) return -1;
  }
  free(dst->v);
  *dst = r;
  return 0;
}

typedef struct { /* Row_maat (row_maat.h) */
  uint64_t lr, lw;
  idset ur, uw;
} mrow;

typedef struct { /* the MaaT parts of TxnManager (txn.h) */
  idset uw, uwy, ur;
  uint64_t gwts, grts, cts;
} mtxn;

typedef struct { /* TimeTable entries (maat.h) */
  uint8_t* present;
  uint64_t *lower, *upper;
  uint8_t* state;
} ttab;

static uint64_t tt_lower(const ttab* t, uint64_t i) { return t->present[i] ? t->lower[i] : 0; }
static uint64_t tt_upper(const ttab* t, uint64_t i) { return t->present[i] ? t->upper[i] : U64MAX; }
static int tt_state(const ttab* t, uint64_t i) {
  return t->present[i] ? t->state[i] : MAAT_ABORTED;
}
static void tt_set_lower(ttab* t, uint64_t i, uint64_t v) {
  if (t->present[i]) t->lower[i] = v;
}
static void tt_set_upper(ttab* t, uint64_t i, uint64_t v) {
  if (t->present[i]) t->upper[i] = v;
}
static void tt_set_state(ttab* t, uint64_t i, int v) {
  if (t->present[i]) t->state[i] = (uint8_t)v;
}

/* Maat::validate, maat.cpp:29-174 (the semaphore serialises it) */
static int maat_validate(ttab* tt, mtxn* tx, uint64_t id, idset* before, idset* after) {
  int rc = RC_RCOK;
  uint64_t lower = tt_lower(tt, id), upper = tt_upper(tt, id);
  before->n = after->n = 0;
  if (lower <= tx->gwts) lower = tx->gwts + 1; /* :46-49 */
  for (uint64_t q = 0; q < tx->uw.n; q++) {    /* :51-67 */
    const uint64_t it = tx->uw.v[q];
    const uint64_t it_lower = tt_lower(tt, it);
    if (upper >= it_lower) {
      const int st = tt_state(tt, it);
      if (st == MAAT_VALIDATED || st == MAAT_COMMITTED) upper = it_lower > 0 ? it_lower - 1 : it_lower;
      if (st == MAAT_RUNNING && is_insert(after, it)) return -1;
    }
  }
  if (lower <= tx->grts) lower = tx->grts + 1; /* :69-72 */
  for (uint64_t q = 0; q < tx->ur.n; q++) {    /* :74-90 */
    const uint64_t it = tx->ur.v[q];
    const uint64_t it_upper = tt_upper(tt, it);
    if (lower <= it_upper) {
      const int st = tt_state(tt, it);
      if (st == MAAT_VALIDATED || st == MAAT_COMMITTED) lower = it_upper < U64MAX ? it_upper + 1 : it_upper;
      if (st == MAAT_RUNNING && is_insert(before, it)) return -1;
    }
  }
  for (uint64_t q = 0; q < tx->uwy.n; q++) { /* :92-111 */
    const uint64_t it = tx->uwy.v[q];
    const int st = tt_state(tt, it);
    const uint64_t it_upper = tt_upper(tt, it);
    if (st == MAAT_ABORTED) continue;
    if ((st == MAAT_VALIDATED || st == MAAT_COMMITTED) && lower <= it_upper)
      lower = it_upper < U64MAX ? it_upper + 1 : it_upper;
    if (st == MAAT_RUNNING && is_insert(after, it)) return -1;
  }
  if (lower >= upper) { /* :112-115 */
    tt_set_state(tt, id, MAAT_ABORTED);
    rc = RC_ABORT;
  } else { /* :116-162 */
    tt_set_state(tt, id, MAAT_VALIDATED);
    for (uint64_t q = 0; q < before->n; q++) {
      const uint64_t it_upper = tt_upper(tt, before->v[q]);
      if (it_upper > lower && it_upper < upper - 1) lower = it_upper + 1;
    }
    for (uint64_t q = 0; q < before->n; q++) {
      const uint64_t it_upper = tt_upper(tt, before->v[q]);
      if (it_upper >= lower) tt_set_upper(tt, before->v[q], lower > 0 ? lower - 1 : lower);
    }
    for (uint64_t q = 0; q < after->n; q++) {
      const uint64_t it_lower = tt_lower(tt, after->v[q]);
      const uint64_t it_upper = tt_upper(tt, after->v[q]);
      if (it_upper != U64MAX && it_upper > lower + 2 && it_upper < upper) upper = it_upper - 2;
      if (it_lower < upper && it_lower > lower + 1) upper = it_lower - 1;
    }
    for (uint64_t q = 0; q < after->n; q++) {
      const uint64_t it_lower = tt_lower(tt, after->v[q]);
      if (it_lower <= upper) tt_set_lower(tt, after->v[q], upper < U64MAX ? upper + 1 : upper);
    }
  }
  tt_set_lower(tt, id, lower); /* :163-164 */
  tt_set_upper(tt, id, upper);
  return rc;
}

/* Maat::find_bound, maat.cpp:176-190 */
static int maat_find_bound(ttab* tt, mtxn* tx, uint64_t id) {
  const uint64_t lower = tt_lower(tt, id), upper = tt_upper(tt, id);
  if (lower >= upper) {
    tt_set_state(tt, id, MAAT_VALIDATED);
    return RC_ABORT;
  }
  tt_set_state(tt, id, MAAT_COMMITTED);
  tx->cts = lower;
  return RC_RCOK;
}

/* Row_maat::commit, row_maat.cpp:189-314 (both the TPCC and the RD/WR paths) */
static void row_commit(ttab* tt, mrow* r, mtxn* tx, uint64_t id, int type, int rw_all) {
  const uint64_t cts = tx->cts;
  const int rd = rw_all || type == ACC_RD, wr = rw_all || type == ACC_WR;
  if (rw_all) {
    if (cts > r->lr) r->lr = cts;
    is_erase(&r->ur, id);
    if (cts > r->lw) r->lw = cts;
    is_erase(&r->uw, id);
  }
  if (rd) {
    if (!rw_all) {
      if (cts > r->lr) r->lr = cts;
      is_erase(&r->ur, id);
    }
    for (uint64_t q = 0; q < r->uw.n; q++) { /* these writers come AFTER this txn */
      const uint64_t it = r->uw.v[q];
      if (!is_count(&tx->uw, it) && tt_lower(tt, it) <= cts) tt_set_lower(tt, it, cts + 1);
    }
  }
  if (wr) {
    if (!rw_all) {
      if (cts > r->lw) r->lw = cts;
      is_erase(&r->uw, id);
    }
    const uint64_t lower = tt_lower(tt, id);
    for (uint64_t q = 0; q < r->uw.n; q++) { /* these writers come BEFORE this txn */
      const uint64_t it = r->uw.v[q];
      if (!is_count(&tx->uwy, it) && tt_upper(tt, it) >= cts) tt_set_upper(tt, it, cts - 1);
    }
    for (uint64_t q = 0; q < r->ur.n; q++) {
      const uint64_t it = r->ur.v[q];
      if (!is_count(&tx->ur, it) && tt_upper(tt, it) >= lower) tt_set_upper(tt, it, lower - 1);
    }
  }
}

/* Row_maat::abort, row_maat.cpp:167-187 */
static void row_abort(mrow* r, uint64_t id, int type, int rw_all) {
  if (rw_all || type == ACC_RD) is_erase(&r->ur, id);
  if (rw_all || type == ACC_WR) is_erase(&r->uw, id);
}

int oracle_maat_replay(uint64_t n, const uint32_t* off, const uint64_t* keys, const uint8_t* acctype,
                       int rw_all, uint64_t n_rows, const uint64_t* row_keys, uint64_t* row_lr,
                       uint64_t* row_lw, uint8_t* out_rc, uint64_t* out_cts) {
  const uint64_t nnz = n ? off[n] : 0;
  kmap rows;
  if (kmap_init(&rows, n_rows + nnz + 1)) return -1;
  mrow* R = (mrow*)calloc(n_rows + nnz + 1, sizeof(mrow));
  uint64_t* rix = (uint64_t*)malloc((nnz + 1) * 8);
  mtxn* T = (mtxn*)calloc(n + 1, sizeof(mtxn));
  ttab tt = {(uint8_t*)calloc(n + 1, 1), (uint64_t*)calloc(n + 1, 8), (uint64_t*)calloc(n + 1, 8),
             (uint8_t*)calloc(n + 1, 1)};
  idset before = {NULL, 0, 0}, after = {NULL, 0, 0};
  int ret = 0;
  if (!R || !rix || !T || !tt.present || !tt.lower || !tt.upper || !tt.state) return -1;
  uint64_t nr = 0;
  for (uint64_t q = 0; q < n_rows; q++) {
    uint64_t* v = kmap_get(&rows, row_keys[q], nr);
    if (*v == nr) {
      R[nr].lr = row_lr[q];
      R[nr].lw = row_lw[q];
      nr++;
    }
  }
  /* time_table.init (worker_thread.cpp:503-508) */
  for (uint64_t i = 0; i < n; i++) {
    tt.present[i] = 1;
    tt.lower[i] = 0;
    tt.upper[i] = U64MAX;
    tt.state[i] = MAAT_RUNNING;
  }
  /* access phase: Row_maat::access (row_maat.cpp:38-52), index order */
  for (uint64_t i = 0; i < n && !ret; i++) {
    mtxn* tx = &T[i];
    for (uint32_t x = off[i]; x < off[i + 1]; x++) {
      uint64_t* v = kmap_get(&rows, keys[x], nr);
      if (*v == nr) nr++;
      mrow* r = &R[*v];
      rix[x] = *v;
      const int type = acctype[x];
      if (rw_all) { /* read_and_prewrite, :54-96 */
        if (is_union(&tx->uw, &r->uw) || is_union(&tx->uwy, &r->uw) || is_union(&tx->ur, &r->ur))
          ret = -1;
        if (tx->grts < r->lr) tx->grts = r->lr;
        if (tx->gwts < r->lw) tx->gwts = r->lw;
        if (is_insert(&r->ur, i) || is_insert(&r->uw, i)) ret = -1;
      } else if (type == ACC_RD) { /* read, :99-125 */
        if (is_union(&tx->uw, &r->uw)) ret = -1;
        if (tx->gwts < r->lw) tx->gwts = r->lw;
        if (is_insert(&r->ur, i)) ret = -1;
      } else if (type == ACC_WR) { /* prewrite, :127-164 */
        if (is_union(&tx->ur, &r->ur) || is_union(&tx->uwy, &r->uw)) ret = -1;
        if (tx->grts < r->lr) tx->grts = r->lr;
        if (tx->gwts < r->lw) tx->gwts = r->lw;
        if (is_insert(&r->uw, i)) ret = -1;
      }
    }
  }
  /* validation + commit/abort, index order */
  for (uint64_t i = 0; i < n && !ret; i++) {
    mtxn* tx = &T[i];
    int rc = maat_validate(&tt, tx, i, &before, &after);
    if (rc < 0) {
      ret = -1;
      break;
    }
    if (rc == RC_RCOK) rc = maat_find_bound(&tt, tx, i); /* home node validates last */
    out_rc[i] = (uint8_t)rc;
    out_cts[i] = rc == RC_RCOK ? tx->cts : 0;
    for (int64_t x = (int64_t)off[i + 1] - 1; x >= (int64_t)off[i]; x--) { /* cleanup, reverse */
      if (rc == RC_RCOK) row_commit(&tt, &R[rix[x]], tx, i, acctype[x], rw_all);
      else row_abort(&R[rix[x]], i, acctype[x], rw_all);
    }
    tt.present[i] = 0; /* time_table.release, txn.cpp:431 / :463 */
    free(tx->uw.v);
    free(tx->uwy.v);
    free(tx->ur.v);
    memset(tx, 0, sizeof *tx);
  }
  for (uint64_t q = 0; q < n_rows && !ret; q++) {
    const uint64_t* v = kmap_find(&rows, row_keys[q]);
    row_lr[q] = R[*v].lr;
    row_lw[q] = R[*v].lw;
  }
  for (uint64_t r = 0; r < nr; r++) {
    free(R[r].ur.v);
    free(R[r].uw.v);
  }
  for (uint64_t i = 0; i < n; i++) {
    free(T[i].uw.v);
    free(T[i].uwy.v);
    free(T[i].ur.v);
  }
  free(before.v);
  free(after.v);
  free(R);
  free(rix);
  free(T);
  free(tt.present);
  free(tt.lower);
  free(tt.upper);
  free(tt.state);
  kmap_free(&rows);
  return ret;
}

/* ------------------------------------------------------------ formula
 * Independent restatement.  In the epoch model a txn's copied sets hold only
 * earlier txns, which are decided and released (time_table defaults: state
 * ABORTED) when it validates, so the set loops of Maat::validate never fire;
 * what reaches txn i is the forward validation of earlier commits
 * (Row_maat::commit) and the row timestamps copied at access time:
 *   L_i = max(gwts_i + 1, grts_i + 1, max{cts_j + 1 : j < i committed, j read a row i wrote})
 *   U_i = min(UINT64_MAX, min{cts_j - 1 : j < i committed, j wrote a row i accessed})
 *   commit iff L_i < U_i, cts_i = L_i
 * (rw_all: every access both reads and writes, the TPC-C path).  Kept per row
 * as running maxima / minima over the committed txns in index order. */
int oracle_maat_formula(uint64_t n, const uint32_t* off, const uint64_t* keys, const uint8_t* acctype,
                        int rw_all, uint64_t n_rows, const uint64_t* row_keys, uint64_t* row_lr,
                        uint64_t* row_lw, uint8_t* out_rc, uint64_t* out_cts) {
  const uint64_t nnz = n ? off[n] : 0;
  kmap rows;
  if (kmap_init(&rows, n_rows + nnz + 1)) return -1;
  const uint64_t cap = n_rows + nnz + 1;
  uint64_t* lr = (uint64_t*)calloc(cap, 8);   /* pre-epoch timestamps */
  uint64_t* lw = (uint64_t*)calloc(cap, 8);
  uint64_t* nlr = (uint64_t*)calloc(cap, 8);  /* after the epoch */
  uint64_t* nlw = (uint64_t*)calloc(cap, 8);
  uint64_t* rmax = (uint64_t*)calloc(cap, 8); /* max cts of committed readers (0 = none) */
  uint64_t* wmin = (uint64_t*)malloc(cap * 8);
  if (!lr || !lw || !nlr || !nlw || !rmax || !wmin) return -1;
  for (uint64_t q = 0; q < cap; q++) wmin[q] = U64MAX;
  uint64_t nr = 0;
  for (uint64_t q = 0; q < n_rows; q++) {
    uint64_t* v = kmap_get(&rows, row_keys[q], nr);
    if (*v == nr) {
      lr[nr] = nlr[nr] = row_lr[q];
      lw[nr] = nlw[nr] = row_lw[q];
      nr++;
    }
  }
  for (uint64_t i = 0; i < n; i++) {
    uint64_t L = 0, U = U64MAX;
    uint64_t gw = 0, gr = 0;
    for (uint32_t x = off[i]; x < off[i + 1]; x++) {
      uint64_t* v = kmap_get(&rows, keys[x], nr);
      if (*v == nr) nr++;
      const uint64_t r = *v;
      const int rd = rw_all || acctype[x] == ACC_RD, wr = rw_all || acctype[x] == ACC_WR;
      if (rd || wr) {
        if (lw[r] > gw) gw = lw[r];
        if (wmin[r] != U64MAX && wmin[r] - 1 < U) U = wmin[r] - 1;
      }
      if (wr) {
        if (lr[r] > gr) gr = lr[r];
        if (rmax[r] && rmax[r] + 1 > L) L = rmax[r] + 1;
      }
    }
    if (gw + 1 > L) L = gw + 1;
    if (gr + 1 > L) L = gr + 1;
    if (L < U) {
      out_rc[i] = RC_RCOK;
      out_cts[i] = L;
      for (uint32_t x = off[i]; x < off[i + 1]; x++) {
        const uint64_t r = *kmap_find(&rows, keys[x]);
        const int rd = rw_all || acctype[x] == ACC_RD, wr = rw_all || acctype[x] == ACC_WR;
        if (rd) {
          if (L > rmax[r]) rmax[r] = L;
          if (L > nlr[r]) nlr[r] = L;
        }
        if (wr) {
          if (L < wmin[r]) wmin[r] = L;
          if (L > nlw[r]) nlw[r] = L;
        }
      }
    } else {
      out_rc[i] = RC_ABORT;
      out_cts[i] = 0;
    }
  }
  for (uint64_t q = 0; q < n_rows; q++) {
    const uint64_t r = *kmap_find(&rows, row_keys[q]);
    row_lr[q] = nlr[r];
    row_lw[q] = nlw[r];
  }
  free(lr);
  free(lw);
  free(nlr);
  free(nlw);
  free(rmax);
  free(wmin);
  kmap_free(&rows);
  return 0;
}
