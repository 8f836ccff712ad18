/*
 * calvin_ref.c — CPU restatements of Calvin epoch lock ordering (test
 * infrastructure only; see oracle.h for the pinning status).
 *
 *   oracle_calvin_replay   literal Row_lock (CALVIN) simulation: FIFO waiters,
 *                          no barging, promotion on release, waves of releases
 *   oracle_calvin_formula  independent per-key run/level formula
 */
#include <stdlib.h>
#include <string.h>

#include "kmap.h"
#include "oracle.h"

/* lock_t, system/global.h:289 */
#define LOCK_EX 0
#define LOCK_SH 1
#define LOCK_NONE 2
#define AT_RD 0
#define AT_SCAN 3
#define GROUP_NONE 0xFFFFFFFFu
#define RC_RCOK 0
#define RC_WAIT 3

/* row_t::get_lock, storage/row.cpp:191 */
static int lock_type_of(uint8_t at) { return (at == AT_RD || at == AT_SCAN) ? LOCK_SH : LOCK_EX; }

/* Row_lock::conflict_lock, row_lock.cpp:374-381 */
static int conflict_lock(int l1, int l2) {
  if (l1 == LOCK_NONE || l2 == LOCK_NONE) return 0;
  if (l1 == LOCK_EX || l2 == LOCK_EX) return 1;
  return 0;
}

/* sequence order: stable argsort of `order` (sched_dequeue's
 * (epoch, origin, FIFO) order, work_queue.cpp:105-151) */
static uint64_t* seq_order(uint64_t n, const uint64_t* order) {
  uint64_t* p = (uint64_t*)malloc(sizeof(uint64_t) * (n ? n : 1));
  if (!p) return NULL;
  for (uint64_t i = 0; i < n; i++) p[i] = i;
  if (!order) return p;
  /* stable merge sort */
  uint64_t* tmp = (uint64_t*)malloc(sizeof(uint64_t) * (n ? n : 1));
  for (uint64_t w = 1; w < n; w *= 2) {
    for (uint64_t lo = 0; lo < n; lo += 2 * w) {
      uint64_t mid = lo + w < n ? lo + w : n, hi = lo + 2 * w < n ? lo + 2 * w : n;
      uint64_t a = lo, b = mid, k = lo;
      while (a < mid && b < hi) tmp[k++] = (order[p[b]] < order[p[a]]) ? p[b++] : p[a++];
      while (a < mid) tmp[k++] = p[a++];
      while (b < hi) tmp[k++] = p[b++];
    }
    memcpy(p, tmp, sizeof(uint64_t) * n);
  }
  free(tmp);
  return p;
}

/* per-txn de-duplication: TxnManager::get_lock, txn.cpp:778-782 (first wins) */
static int is_dup(const uint64_t* keys, uint32_t s, uint32_t x) {
  for (uint32_t y = s; y < x; y++)
    if (keys[y] == keys[x]) return 1;
  return 0;
}

typedef struct {
  int owner_cnt, lock_type;
  uint32_t cur_group;
  int64_t wh, wt; /* waiter FIFO through request indices */
} row_lock;

int oracle_calvin_replay(uint64_t n, const uint32_t* off, const uint64_t* keys,
                         const uint8_t* acctype, const uint64_t* order, uint32_t* out_group,
                         uint8_t* out_rc, uint32_t* out_wave) {
  const uint64_t nnz = n ? off[n] : 0;
  uint64_t* seq = seq_order(n, order);
  kmap rows;
  if (!seq || kmap_init(&rows, nnz + 1)) return -1;
  row_lock* rl = (row_lock*)calloc(nnz + 1, sizeof(row_lock));
  uint64_t* rrow = (uint64_t*)malloc(sizeof(uint64_t) * (nnz + 1));
  int64_t* wnext = (int64_t*)malloc(sizeof(int64_t) * (nnz + 1));
  uint32_t* req_txn = (uint32_t*)malloc(sizeof(uint32_t) * (nnz + 1));
  int64_t* lr = (int64_t*)calloc(n + 1, sizeof(int64_t));
  uint64_t* wave_a = (uint64_t*)malloc(sizeof(uint64_t) * (n + 1));
  uint64_t* wave_b = (uint64_t*)malloc(sizeof(uint64_t) * (n + 1));
  if (!rl || !rrow || !wnext || !req_txn || !lr || !wave_a || !wave_b) return -1;
  uint64_t nrows = 0, na = 0;

  /* ---- acquisition in sequence order: acquire_locks, ycsb_txn.cpp:49-88 */
  for (uint64_t q = 0; q < n; q++) {
    const uint64_t t = seq[q];
    lr[t] = 1; /* incr_lr(), ycsb_txn.cpp:55 */
    for (uint32_t x = off[t]; x < off[t + 1]; x++) {
      req_txn[x] = (uint32_t)t;
      if (is_dup(keys, off[t], x)) {
        out_group[x] = GROUP_NONE;
        continue;
      }
      uint64_t* rv = kmap_get(&rows, keys[x], (uint64_t)-1);
      if (*rv == (uint64_t)-1) {
        *rv = nrows;
        rl[nrows].lock_type = LOCK_NONE;
        rl[nrows].wh = rl[nrows].wt = -1;
        nrows++;
      }
      const uint64_t r = *rv;
      rrow[x] = r;
      const int type = lock_type_of(acctype[x]);
      /* Row_lock::lock_get, row_lock.cpp:66-81: conflict with owners, or
       * (CALVIN) any waiter present -> no barging */
      int conflict = conflict_lock(rl[r].lock_type, type);
      if (!conflict && rl[r].wh >= 0) conflict = 1;
      if (conflict) {
        /* row_lock.cpp:152-170: LIST_PUT_TAIL(waiters), incr_lr, WAIT */
        wnext[x] = -1;
        if (rl[r].wt >= 0) wnext[rl[r].wt] = x;
        else rl[r].wh = x;
        rl[r].wt = x;
        lr[t]++;
      } else {
        /* row_lock.cpp:171-196: join the owners */
        rl[r].owner_cnt++;
        rl[r].lock_type = type;
        out_group[x] = rl[r].cur_group;
      }
    }
    /* decr_lr() == 0 -> lock_ready (ycsb_txn.cpp:76-79) */
    if (--lr[t] == 0) {
      out_rc[t] = RC_RCOK;
      wave_a[na++] = t;
    } else {
      out_rc[t] = RC_WAIT;
    }
  }

  /* ---- waves: every ready txn runs, then releases all its locks */
  uint32_t w = 0;
  while (na) {
    uint64_t nb = 0;
    for (uint64_t q = 0; q < na; q++) {
      const uint64_t t = wave_a[q];
      out_wave[t] = w;
      for (uint32_t x = off[t]; x < off[t + 1]; x++) {
        if (out_group[x] == GROUP_NONE) continue;
        const uint64_t r = rrow[x];
        /* Row_lock::lock_release, row_lock.cpp:258-287 */
        rl[r].owner_cnt--;
        if (rl[r].owner_cnt == 0) rl[r].lock_type = LOCK_NONE;
        /* promotion, row_lock.cpp:317-357 */
        int opened = rl[r].lock_type == LOCK_NONE;
        while (rl[r].wh >= 0) {
          const int64_t h = rl[r].wh;
          const int ht = lock_type_of(acctype[h]);
          if (conflict_lock(rl[r].lock_type, ht)) break;
          rl[r].wh = wnext[h];
          if (rl[r].wh < 0) rl[r].wt = -1;
          if (opened) {
            rl[r].cur_group++;
            opened = 0;
          }
          out_group[h] = rl[r].cur_group;
          rl[r].owner_cnt++;
          rl[r].lock_type = ht;
          const uint32_t ht_txn = req_txn[h];
          if (--lr[ht_txn] == 0) wave_b[nb++] = ht_txn; /* restart_txn */
        }
      }
    }
    uint64_t* tmp = wave_a;
    wave_a = wave_b;
    wave_b = tmp;
    na = nb;
    w++;
  }
  int ret = 0;
  for (uint64_t t = 0; t < n; t++)
    if (lr[t] != 0) ret = -2; /* a txn never became ready: impossible for a DAG */
  kmap_free(&rows);
  free(rl);
  free(rrow);
  free(wnext);
  free(req_txn);
  free(lr);
  free(wave_a);
  free(wave_b);
  free(seq);
  return ret;
}

/* ------------------------------------------------------------ formula */
typedef struct {
  uint32_t group;
  int last_type; /* LOCK_NONE = no request yet */
  int64_t last_ex_lvl, max_sh_since;
} key_state;

int oracle_calvin_formula(uint64_t n, const uint32_t* off, const uint64_t* keys,
                          const uint8_t* acctype, const uint64_t* order, uint32_t* out_group,
                          uint8_t* out_rc, uint32_t* out_wave) {
  const uint64_t nnz = n ? off[n] : 0;
  uint64_t* seq = seq_order(n, order);
  kmap km;
  if (!seq || kmap_init(&km, nnz + 1)) return -1;
  key_state* ks = (key_state*)calloc(nnz + 1, sizeof(key_state));
  uint64_t nk = 0;
  for (uint64_t q = 0; q < n; q++) {
    const uint64_t t = seq[q];
    int64_t lvl = 0;
    int ready = 1;
    /* pass 1: groups and the txn's level */
    for (uint32_t x = off[t]; x < off[t + 1]; x++) {
      if (is_dup(keys, off[t], x)) {
        out_group[x] = GROUP_NONE;
        continue;
      }
      uint64_t* v = kmap_get(&km, keys[x], (uint64_t)-1);
      if (*v == (uint64_t)-1) {
        *v = nk;
        ks[nk].last_type = LOCK_NONE;
        ks[nk].last_ex_lvl = -1;
        ks[nk].max_sh_since = -1;
        nk++;
      }
      key_state* s = &ks[*v];
      const int type = lock_type_of(acctype[x]);
      uint32_t g;
      if (s->last_type == LOCK_NONE) g = 0;
      else if (type == LOCK_EX || s->last_type == LOCK_EX) g = s->group + 1;
      else g = s->group;
      out_group[x] = g;
      if (g) ready = 0;
      int64_t need;
      if (type == LOCK_EX) need = (s->last_ex_lvl > s->max_sh_since ? s->last_ex_lvl : s->max_sh_since) + 1;
      else need = s->last_ex_lvl + 1;
      if (need > lvl) lvl = need;
    }
    /* pass 2: publish */
    for (uint32_t x = off[t]; x < off[t + 1]; x++) {
      if (out_group[x] == GROUP_NONE) continue;
      key_state* s = &ks[*kmap_find(&km, keys[x])];
      const int type = lock_type_of(acctype[x]);
      s->group = out_group[x];
      s->last_type = type;
      if (type == LOCK_EX) {
        s->last_ex_lvl = lvl;
        s->max_sh_since = -1;
      } else if (lvl > s->max_sh_since) {
        s->max_sh_since = lvl;
      }
    }
    out_rc[t] = ready ? RC_RCOK : RC_WAIT;
    out_wave[t] = (uint32_t)lvl;
  }
  kmap_free(&km);
  free(ks);
  free(seq);
  return 0;
}
