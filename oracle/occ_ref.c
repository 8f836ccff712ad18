/*
 * occ_ref.c — CPU restatements of OptCC central validation (test infrastructure
 * only; see oracle.h for the pinning status).
 *
 *   oracle_occ_replay   literal: linked active/history stacks + nested-loop
 *                        test_valid, validate-all-then-finish-all epoch replay
 *   oracle_occ_hash     independent: serial hash-set scan
 *   oracle_occ_round_status  one round of the GPU fixed point, per shard
 */
#include <stdlib.h>
#include <string.h>

#include "kmap.h"
#include "oracle.h"

#define AT_WR 1 /* access_t WR, system/global.h:287 */
#define RC_RCOK 0
#define RC_ABORT 2

/* set_ent, concurrency_control/occ.h:33-41 */
typedef struct set_ent {
  uint64_t tn;
  int64_t txn;
  uint32_t set_size;
  uint64_t* rows;
  struct set_ent* next;
} set_ent;

/* OptCC::test_valid, occ.cpp:319-327: false iff the two sets share a row */
static int test_valid(const set_ent* s1, const set_ent* s2) {
  for (uint32_t i = 0; i < s1->set_size; i++)
    for (uint32_t j = 0; j < s2->set_size; j++)
      if (s1->rows[i] == s2->rows[j]) return 0;
  return 1;
}

/* OptCC::get_rw_set, occ.cpp:296-317: WR accesses -> wset, all others -> rset */
static int get_rw_set(int64_t txn, const uint32_t* off, const uint64_t* keys,
                      const uint8_t* acctype, set_ent** rset, set_ent** wset) {
  set_ent* w = (set_ent*)calloc(1, sizeof(set_ent));
  set_ent* r = (set_ent*)calloc(1, sizeof(set_ent));
  if (!w || !r) return -1;
  uint32_t nw = 0, nr = 0;
  for (uint32_t x = off[txn]; x < off[txn + 1]; x++) (acctype[x] == AT_WR ? nw++ : nr++);
  w->rows = (uint64_t*)malloc(sizeof(uint64_t) * (nw ? nw : 1));
  r->rows = (uint64_t*)malloc(sizeof(uint64_t) * (nr ? nr : 1));
  if (!w->rows || !r->rows) return -1;
  for (uint32_t x = off[txn]; x < off[txn + 1]; x++) {
    if (acctype[x] == AT_WR) w->rows[w->set_size++] = keys[x];
    else r->rows[r->set_size++] = keys[x];
  }
  w->txn = r->txn = txn;
  *rset = r;
  *wset = w;
  return 0;
}

static void free_ent(set_ent* e) {
  if (!e) return;
  free(e->rows);
  free(e);
}

int oracle_occ_replay(uint64_t n, const uint32_t* off, const uint64_t* keys, const uint8_t* acctype,
                      const uint64_t* start_tn, const uint64_t* finish_tn, uint64_t n_hist,
                      const uint64_t* hist_keys, const uint64_t* hist_tn, uint64_t* tnc,
                      uint8_t* out_rc, uint64_t* out_tn) {
  set_ent* active = NULL;  /* occ.h:64 */
  set_ent* history = NULL; /* occ.h:63, head = latest (largest tn) */
  uint64_t active_len = 0;
  int ret = 0;

  /* Seed history from (key, tn) pairs: one set_ent per distinct tn, pushed
   * in ascending tn so the head holds the largest (STACK_PUSH order of
   * central_finish, occ.cpp:283-286). */
  if (n_hist) {
    uint64_t* idx = (uint64_t*)malloc(n_hist * sizeof(uint64_t));
    if (!idx) return -1;
    for (uint64_t i = 0; i < n_hist; i++) idx[i] = i;
    { /* shell sort of pair indices by tn */
      uint64_t gap = n_hist / 2;
      while (gap) {
        for (uint64_t i = gap; i < n_hist; i++) {
          uint64_t t = idx[i], j = i;
          while (j >= gap && hist_tn[idx[j - gap]] > hist_tn[t]) {
            idx[j] = idx[j - gap];
            j -= gap;
          }
          idx[j] = t;
        }
        gap /= 2;
      }
    }
    uint64_t i = 0;
    while (i < n_hist) {
      uint64_t j = i;
      while (j < n_hist && hist_tn[idx[j]] == hist_tn[idx[i]]) j++;
      set_ent* e = (set_ent*)calloc(1, sizeof(set_ent));
      if (!e) return -1;
      e->tn = hist_tn[idx[i]];
      e->txn = -1;
      e->rows = (uint64_t*)malloc(sizeof(uint64_t) * (j - i));
      for (uint64_t q = i; q < j; q++) e->rows[e->set_size++] = hist_keys[idx[q]];
      e->next = history;
      history = e;
      i = j;
    }
    free(idx);
  }

  set_ent** snap = (set_ent**)malloc(sizeof(set_ent*) * (n + 1));
  uint8_t* ro = (uint8_t*)malloc(n ? n : 1);
  if (!snap || !ro) return -1;

  /* ---- validate every txn in index order: central_validate, occ.cpp:116-239 */
  for (uint64_t t = 0; t < n; t++) {
    set_ent *rset, *wset;
    if (get_rw_set((int64_t)t, off, keys, acctype, &rset, &wset)) return -1;
    const int readonly = wset->set_size == 0; /* occ.cpp:130 */
    ro[t] = (uint8_t)readonly;
    /* critical section, occ.cpp:137-158: snapshot active, push own wset */
    uint64_t f_active_len = 0;
    for (set_ent* e = active; e; e = e->next) snap[f_active_len++] = e;
    if (!readonly) {
      active_len++;
      wset->next = active;
      active = wset;
    }
    int valid = 1;
    /* history window, occ.cpp:167-180 (checked against the READ set only) */
    if (start_tn && finish_tn && finish_tn[t] > start_tn[t]) {
      set_ent* his = history;
      while (his && his->tn > finish_tn[t]) his = his->next;
      while (his && his->tn > start_tn[t]) {
        valid = test_valid(his, rset);
        if (!valid) break;
        his = his->next;
      }
    }
    /* active set, occ.cpp:185-199: vs R, then vs W */
    if (valid) {
      for (uint64_t q = 0; q < f_active_len; q++) {
        valid = test_valid(snap[q], rset);
        if (valid) valid = test_valid(snap[q], wset);
        if (!valid) break;
      }
    }
    free_ent(rset);
    out_rc[t] = valid ? RC_RCOK : RC_ABORT;
    if (!valid) {
      /* occ.cpp:219-235: unlink own wset from active immediately */
      set_ent *act = active, *prev = NULL;
      while (act && act->txn != (int64_t)t) {
        prev = act;
        act = act->next;
      }
      if (act && act->txn == (int64_t)t) {
        if (prev) prev->next = act->next;
        else active = act->next;
        active_len--;
        free_ent(act);
      } else {
        free_ent(wset); /* read-only: never pushed */
      }
    } else if (readonly) {
      free_ent(wset);
    }
  }

  /* ---- finish every txn in index order: central_finish, occ.cpp:248-294 */
  for (uint64_t t = 0; t < n; t++) {
    if (out_tn) out_tn[t] = 0;
    if (ro[t]) continue; /* occ.cpp:254: read-only txns skip the finish */
    set_ent *act = active, *prev = NULL;
    while (act && act->txn != (int64_t)t) {
      prev = act;
      act = act->next;
    }
    if (!act) {
      if (out_rc[t] != RC_ABORT) ret = -2; /* assert(rc == Abort), occ.cpp:265-266 */
      continue;
    }
    if (prev) prev->next = act->next;
    else active = act->next;
    active_len--;
    if (out_rc[t] == RC_RCOK) {
      (*tnc)++;             /* occ.cpp:283 */
      act->tn = *tnc;       /* occ.cpp:284 */
      act->next = history;  /* STACK_PUSH(history, wset) */
      history = act;
      if (out_tn) out_tn[t] = act->tn;
    } else {
      free_ent(act);
    }
  }
  while (history) {
    set_ent* nx = history->next;
    free_ent(history);
    history = nx;
  }
  free(snap);
  free(ro);
  (void)active_len;
  return ret;
}

/* ---------------------------------------------------------------- hash-set */
int oracle_occ_hash(uint64_t n, const uint32_t* off, const uint64_t* keys, const uint8_t* acctype,
                    const uint64_t* start_tn, const uint64_t* finish_tn, uint64_t n_hist,
                    const uint64_t* hist_keys, const uint64_t* hist_tn, uint64_t* tnc,
                    uint8_t* out_rc, uint64_t* out_tn) {
  kmap committed; /* keys written by committed txns of this epoch */
  if (kmap_init(&committed, 1024)) return -1;
  kmap hk; /* history: key -> list index */
  uint64_t** lists = NULL;
  uint32_t* lc = NULL;
  uint64_t nl = 0;
  if (kmap_init(&hk, n_hist + 1)) return -1;
  if (n_hist) {
    lists = (uint64_t**)calloc(n_hist, sizeof(uint64_t*));
    lc = (uint32_t*)calloc(n_hist, sizeof(uint32_t));
    uint32_t* lcap = (uint32_t*)calloc(n_hist, sizeof(uint32_t));
    for (uint64_t i = 0; i < n_hist; i++) {
      uint64_t* v = kmap_get(&hk, hist_keys[i], (uint64_t)-1);
      if (*v == (uint64_t)-1) *v = nl++;
      const uint64_t l = *v;
      if (lc[l] == lcap[l]) {
        lcap[l] = lcap[l] ? 2 * lcap[l] : 4;
        lists[l] = (uint64_t*)realloc(lists[l], lcap[l] * sizeof(uint64_t));
      }
      lists[l][lc[l]++] = hist_tn[i];
    }
    free(lcap);
  }
  for (uint64_t t = 0; t < n; t++) {
    int abort = 0, has_w = 0;
    for (uint32_t x = off[t]; x < off[t + 1]; x++) {
      if (acctype[x] == AT_WR) has_w = 1;
      if (kmap_find(&committed, keys[x])) abort = 1;
      if (!abort && start_tn && finish_tn && finish_tn[t] > start_tn[t] && acctype[x] != AT_WR) {
        const uint64_t* l = kmap_find(&hk, keys[x]);
        if (l)
          for (uint32_t q = 0; q < lc[*l]; q++)
            if (lists[*l][q] > start_tn[t] && lists[*l][q] <= finish_tn[t]) abort = 1;
      }
    }
    out_rc[t] = abort ? RC_ABORT : RC_RCOK;
    if (out_tn) out_tn[t] = 0;
    if (!abort) {
      for (uint32_t x = off[t]; x < off[t + 1]; x++)
        if (acctype[x] == AT_WR) *kmap_get(&committed, keys[x], 0) = t;
      if (has_w) {
        (*tnc)++;
        if (out_tn) out_tn[t] = *tnc;
      }
    }
  }
  for (uint64_t l = 0; l < nl; l++) free(lists[l]);
  free(lists);
  free(lc);
  kmap_free(&hk);
  kmap_free(&committed);
  return 0;
}

/* ------------------------------------------------------- round status */
int oracle_occ_round_status(uint64_t n, const uint32_t* off, const uint64_t* keys,
                            const uint8_t* acctype, const uint8_t* state, uint8_t* out_status) {
  /* per key: minimum undecided writer and the committed writer */
  kmap und, com;
  if (kmap_init(&und, 1024) || kmap_init(&com, 1024)) return -1;
  for (uint64_t t = 0; t < n; t++) {
    if (state[t] == 2) continue;
    for (uint32_t x = off[t]; x < off[t + 1]; x++) {
      if (acctype[x] != AT_WR) continue;
      if (state[t] == 0) {
        uint64_t* v = kmap_get(&und, keys[x], (uint64_t)-1);
        if (t < *v) *v = t;
      } else {
        uint64_t* v = kmap_get(&com, keys[x], (uint64_t)-1);
        if (t < *v) *v = t;
      }
    }
  }
  for (uint64_t t = 0; t < n; t++) {
    uint8_t s = 0;
    if (state[t] == 0) {
      for (uint32_t x = off[t]; x < off[t + 1]; x++) {
        const uint64_t* c = kmap_find(&com, keys[x]);
        if (c && *c < t) s |= 2;
        const uint64_t* u = kmap_find(&und, keys[x]);
        if (u && *u < t) s |= 1;
      }
    }
    out_status[t] = s;
  }
  kmap_free(&und);
  kmap_free(&com);
  return 0;
}

/* Captured-snapshot validation, literal: for each txn t, central_validate
 * (occ.cpp:116-239) against what its critical section captured
 * (occ.cpp:137-158) — the history stack from the entry with the largest
 * tn <= hist_top[t] downwards (his = history; NULL hist_top = whole history),
 * and the write sets of active_idx[active_off[t] .. active_off[t+1]) as
 * finish_active.  History pairs form one set_ent per distinct tn. */
int oracle_occ_snapshot(uint64_t n, const uint32_t* off, const uint64_t* keys,
                        const uint8_t* acctype, const uint64_t* start_tn,
                        const uint64_t* finish_tn, const uint64_t* hist_top,
                        const uint32_t* active_off, const uint32_t* active_idx, uint64_t n_hist,
                        const uint64_t* hist_keys, const uint64_t* hist_tn, uint8_t* out_rc) {
  /* history as an array of entries in descending tn (the stack, head first) */
  set_ent* hv = NULL;
  uint64_t nh = 0;
  if (n_hist) {
    uint64_t* idx = (uint64_t*)malloc(n_hist * sizeof(uint64_t));
    hv = (set_ent*)calloc(n_hist, sizeof(set_ent));
    if (!idx || !hv) return -1;
    for (uint64_t i = 0; i < n_hist; i++) idx[i] = i;
    for (uint64_t gap = n_hist / 2; gap; gap /= 2) /* shell sort, descending tn */
      for (uint64_t i = gap; i < n_hist; i++) {
        uint64_t t = idx[i], j = i;
        while (j >= gap && hist_tn[idx[j - gap]] < hist_tn[t]) {
          idx[j] = idx[j - gap];
          j -= gap;
        }
        idx[j] = t;
      }
    for (uint64_t i = 0; i < n_hist;) {
      uint64_t j = i;
      while (j < n_hist && hist_tn[idx[j]] == hist_tn[idx[i]]) j++;
      set_ent* e = &hv[nh++];
      e->tn = hist_tn[idx[i]];
      e->rows = (uint64_t*)malloc(sizeof(uint64_t) * (j - i));
      if (!e->rows) return -1;
      for (uint64_t q = i; q < j; q++) e->rows[e->set_size++] = hist_keys[idx[q]];
      i = j;
    }
    free(idx);
  }
  set_ent** wsets = (set_ent**)calloc(n ? n : 1, sizeof(set_ent*));
  set_ent** rsets = (set_ent**)calloc(n ? n : 1, sizeof(set_ent*));
  if (!wsets || !rsets) return -1;
  for (uint64_t t = 0; t < n; t++)
    if (get_rw_set((int64_t)t, off, keys, acctype, &rsets[t], &wsets[t])) return -1;
  for (uint64_t t = 0; t < n; t++) {
    int valid = 1;
    uint64_t h = 0; /* his = history, as seen at t's critical section */
    if (hist_top)
      while (h < nh && hv[h].tn > hist_top[t]) h++;
    if (start_tn && finish_tn && finish_tn[t] > start_tn[t]) { /* occ.cpp:167-180 */
      while (h < nh && hv[h].tn > finish_tn[t]) h++;
      while (h < nh && hv[h].tn > start_tn[t]) {
        valid = test_valid(&hv[h], rsets[t]);
        if (!valid) break;
        h++;
      }
    }
    if (valid) /* occ.cpp:185-199 */
      for (uint32_t q = active_off[t]; q < active_off[t + 1]; q++) {
        const set_ent* wact = wsets[active_idx[q]];
        valid = test_valid(wact, rsets[t]);
        if (valid) valid = test_valid(wact, wsets[t]);
        if (!valid) break;
      }
    out_rc[t] = valid ? RC_RCOK : RC_ABORT;
  }
  for (uint64_t t = 0; t < n; t++) {
    free_ent(rsets[t]);
    free_ent(wsets[t]);
  }
  free(rsets);
  free(wsets);
  for (uint64_t i = 0; i < nh; i++) free(hv[i].rows);
  free(hv);
  return 0;
}
