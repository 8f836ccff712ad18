/*
 * occ_sweep_mt.c — SWEEP-MT: the strongest host-core CPU baseline this build
 * knows for the OCC epoch, the CPU form of the GPU sweep.
 * TEST INFRASTRUCTURE ONLY (oracle.h): bench.py's cpu_baseline leg times it
 * beside the literal replay, the serial hash scan and ROUNDS-MT;
 * tests/test_oracle.py checks it against the serial scan.
 *
 * Decisions equal the serial epoch replay of central_validate /
 * central_finish (concurrency_control/occ.cpp:116-294) without a history
 * window: txn i aborts iff some earlier committed txn wrote a key i accesses.
 * Per level, over a list of txns in index order (level 0: the epoch):
 *   1. one thread decides the list's first P txns serially, adding committed
 *      write keys to the committed set C (a hash set);
 *   2. every thread filters its share of the rest against C, read-only: a
 *      txn touching a key of C is dead (its committed writer is earlier);
 *      the survivors, still in index order, form the next level's list.
 * A dead txn never commits, so it neither kills nor blocks anyone, and
 * deciding the survivors in their own order reproduces the serial replay.
 * P doubles per level (1,024, 2,048, ...); a list that stops shrinking is
 * decided serially whole.
 */
#define _GNU_SOURCE
#include <pthread.h>
#include <stdlib.h>
#include <string.h>

#include "kmap.h"
#include "oracle.h"

#define AT_WR 1
#define EMPTY 0xFFFFFFFFFFFFFFFFull

typedef struct {
  uint64_t* k;
  uint64_t mask;
  uint64_t n;
} cset;

static int cset_has(const cset* c, uint64_t key) {
  uint64_t h = kmap_h(key) & c->mask;
  for (;;) {
    const uint64_t v = c->k[h];
    if (v == key) return 1;
    if (v == EMPTY) return 0;
    h = (h + 1) & c->mask;
  }
}

static int cset_add(cset* c, uint64_t key) {
  if (2 * (c->n + 1) > c->mask + 1) { /* grow: keep <= 50 % load */
    const uint64_t cap = 2 * (c->mask + 1);
    uint64_t* nk = (uint64_t*)malloc(cap * 8);
    if (!nk) return -1;
    memset(nk, 0xFF, cap * 8);
    for (uint64_t q = 0; q <= c->mask; q++) {
      if (c->k[q] == EMPTY) continue;
      uint64_t h = kmap_h(c->k[q]) & (cap - 1);
      while (nk[h] != EMPTY) h = (h + 1) & (cap - 1);
      nk[h] = c->k[q];
    }
    free(c->k);
    c->k = nk;
    c->mask = cap - 1;
  }
  uint64_t h = kmap_h(key) & c->mask;
  for (;;) {
    if (c->k[h] == key) return 0;
    if (c->k[h] == EMPTY) {
      c->k[h] = key;
      c->n++;
      return 0;
    }
    h = (h + 1) & c->mask;
  }
}

typedef struct {
  const uint32_t* off;
  const uint64_t* keys;
  const uint8_t* at;
  uint8_t* state; /* [n] 0 undecided, 1 commit, 2 abort */
  cset C;
  uint32_t* list[2];
  uint64_t len, pos; /* current list length; txns [0, pos) decided serially */
  uint64_t* part;    /* [T] survivors per thread */
  int cur, nthreads, done, err;
  uint32_t levels;
  pthread_barrier_t bar;
} Shared;

typedef struct {
  Shared* s;
  int id;
} Arg;

static void range(uint64_t lo, uint64_t hi, int T, int id, uint64_t* b, uint64_t* e) {
  const uint64_t len = hi - lo, per = (len + T - 1) / T;
  *b = lo + (per * id < len ? per * id : len);
  *e = *b + per < hi ? *b + per : hi;
}

/* thread 0: the serial part of a level */
static void serial(Shared* s, uint64_t P) {
  const uint32_t* L = s->list[s->cur];
  for (uint64_t q = 0; q < P; q++) {
    const uint32_t t = L[q];
    int dead = 0, w = 0;
    for (uint32_t x = s->off[t]; x < s->off[t + 1] && !dead; x++) {
      dead = cset_has(&s->C, s->keys[x]);
      w |= s->at[x] == AT_WR;
    }
    if (dead) {
      s->state[t] = 2;
      continue;
    }
    s->state[t] = 1;
    if (w)
      for (uint32_t x = s->off[t]; x < s->off[t + 1]; x++)
        if (s->at[x] == AT_WR && cset_add(&s->C, s->keys[x])) s->err = 1;
  }
}

static void* worker(void* p) {
  Arg* a = (Arg*)p;
  Shared* s = a->s;
  const int T = s->nthreads, id = a->id;
  uint64_t P = 1024;
  for (;;) {
    if (id == 0) {
      const uint64_t pp = P < s->len ? P : s->len;
      serial(s, pp);
      s->pos = pp;
      s->levels++;
    }
    pthread_barrier_wait(&s->bar);
    /* filter [pos, len) against C, compact each share at its range start */
    const uint32_t* L = s->list[s->cur];
    uint32_t* out = s->list[s->cur ^ 1];
    uint64_t b, e;
    range(s->pos, s->len, T, id, &b, &e);
    uint64_t keep = b;
    for (uint64_t q = b; q < e; q++) {
      const uint32_t t = L[q];
      int dead = 0;
      for (uint32_t x = s->off[t]; x < s->off[t + 1] && !dead; x++) dead = cset_has(&s->C, s->keys[x]);
      if (dead) s->state[t] = 2;
      else out[keep++] = t;
    }
    s->part[id] = keep - b;
    pthread_barrier_wait(&s->bar);
    if (id == 0) {
      uint64_t w = 0;
      for (int r = 0; r < T; r++) {
        uint64_t rb, re;
        range(s->pos, s->len, T, r, &rb, &re);
        memmove(out + w, out + rb, s->part[r] * sizeof(uint32_t));
        w += s->part[r];
      }
      /* a list that stops shrinking is decided serially whole next level */
      const uint64_t rest = s->len - s->pos;
      s->len = w;
      s->cur ^= 1;
      s->done = w == 0 || s->err;
      if (4 * w > 3 * rest) s->pos = ~0ull; /* marker: next P = whole list */
    }
    pthread_barrier_wait(&s->bar);
    if (s->done) break;
    P = s->pos == ~0ull ? s->len : 2 * P;
  }
  return NULL;
}

int oracle_occ_sweep_mt(uint64_t n, const uint32_t* off, const uint64_t* keys,
                        const uint8_t* acctype, int nthreads, uint64_t* tnc, uint8_t* out_rc,
                        uint64_t* out_tn, uint32_t* out_levels) {
  if (nthreads < 1) nthreads = 1;
  if (n >= 0xFFFFFFFFull) return -1;
  Shared s;
  memset(&s, 0, sizeof s);
  s.off = off;
  s.keys = keys;
  s.at = acctype;
  s.nthreads = nthreads;
  s.len = n;
  s.C.mask = 4095;
  s.C.k = (uint64_t*)malloc(4096 * 8);
  s.state = (uint8_t*)calloc(n ? n : 1, 1);
  s.list[0] = (uint32_t*)malloc((n ? n : 1) * 4);
  s.list[1] = (uint32_t*)malloc((n ? n : 1) * 4);
  s.part = (uint64_t*)calloc(nthreads, 8);
  pthread_t* th = (pthread_t*)malloc(sizeof(pthread_t) * nthreads);
  Arg* args = (Arg*)malloc(sizeof(Arg) * nthreads);
  int ret = 0;
  if (!s.C.k || !s.state || !s.list[0] || !s.list[1] || !s.part || !th || !args) {
    ret = -1;
    goto out;
  }
  memset(s.C.k, 0xFF, 4096 * 8);
  for (uint64_t t = 0; t < n; t++) s.list[0][t] = (uint32_t)t;
  if (n) {
    pthread_barrier_init(&s.bar, NULL, (unsigned)nthreads);
    for (int i = 0; i < nthreads; i++) {
      args[i].s = &s;
      args[i].id = i;
      pthread_create(&th[i], NULL, worker, &args[i]);
    }
    for (int i = 0; i < nthreads; i++) pthread_join(th[i], NULL);
    pthread_barrier_destroy(&s.bar);
  }
  if (s.err) {
    ret = -1;
    goto out;
  }
  /* central_finish numbering (occ.cpp:283-284): committed non-read-only
   * txns take tnc+1, tnc+2, ... in index order */
  for (uint64_t t = 0; t < n; t++) {
    out_rc[t] = s.state[t] == 1 ? 0 : 2;
    uint64_t v = 0;
    if (s.state[t] == 1) {
      int w = 0;
      for (uint32_t x = off[t]; x < off[t + 1]; x++) w |= acctype[x] == AT_WR;
      if (w) v = ++*tnc;
    }
    if (out_tn) out_tn[t] = v;
  }
  if (out_levels) *out_levels = s.levels;
out:
  free(s.C.k);
  free(s.state);
  free(s.list[0]);
  free(s.list[1]);
  free(s.part);
  free(th);
  free(args);
  return ret;
}
