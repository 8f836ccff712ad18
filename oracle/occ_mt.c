/*
 * occ_mt.c — ROUNDS-MT: the round-based OCC fixed point on all host cores
 * (SURVEY.md §8(d) CPU variant (iii)).  TEST INFRASTRUCTURE ONLY (oracle.h):
 * bench.py's cpu_baseline leg times it beside the literal replay and the
 * serial hash scan; tests/test_oracle.py checks it against both.
 *
 * Decisions equal the serial epoch replay of central_validate /
 * central_finish (concurrency_control/occ.cpp:116-294) without a history
 * window: txn i aborts iff some earlier committed txn wrote a key i accesses.
 * Round r, for every undecided txn i and each of its keys K, with o(K) the
 * smallest non-aborted writer of K:
 *   o(K) < i committed   -> i aborts (the key's committed writer, occ.cpp:185-199)
 *   o(K) < i undecided   -> i is blocked this round
 *   otherwise, all keys  -> i commits (and is then o(K) of its write keys)
 * Every decision is final, and the smallest undecided txn decides each
 * round, so the loop terminates.
 *
 * Per key: a slot of a lock-free open-addressing table (CAS on the key word)
 * holding com[s] (its committed writer, written once) and und[s] (min over
 * the undecided writers of the current round, reset per round for the
 * writers of the previous list).  Threads: a static split of the undecided
 * list, pthread barriers between the phases.
 */
#define _GNU_SOURCE
#include <pthread.h>
#include <stdlib.h>
#include <string.h>

#include "kmap.h"
#include "oracle.h"

#define AT_WR 1
#define NONE 0xFFFFFFFFu
#define EMPTY 0xFFFFFFFFFFFFFFFFull

typedef struct {
  uint64_t n;
  const uint32_t* off;
  const uint64_t* keys;
  const uint8_t* at;
  uint64_t* tkey; /* slot keys */
  uint64_t mask;
  uint32_t* aslot; /* [nnz] slot of each access */
  uint32_t* com;   /* [slots] committed writer */
  uint32_t* und;   /* [slots] min undecided writer this round */
  uint8_t* state;  /* [n] 0 undecided, 1 commit, 2 abort */
  uint32_t* list[2];
  uint64_t len;      /* current list length */
  uint64_t* part;    /* [T] survivors per thread */
  int nthreads;
  int done;
  uint32_t rounds;
  int err;
  pthread_barrier_t bar;
} Shared;

typedef struct {
  Shared* s;
  int id;
} Arg;

static uint32_t slot_of(Shared* s, uint64_t key) {
  uint64_t h = kmap_h(key) & s->mask;
  for (;;) {
    uint64_t cur = __atomic_load_n(&s->tkey[h], __ATOMIC_ACQUIRE);
    if (cur == key) return (uint32_t)h;
    if (cur == EMPTY) {
      uint64_t exp = EMPTY;
      if (__atomic_compare_exchange_n(&s->tkey[h], &exp, key, 0, __ATOMIC_ACQ_REL,
                                      __ATOMIC_ACQUIRE))
        return (uint32_t)h;
      if (exp == key) return (uint32_t)h;
    }
    h = (h + 1) & s->mask;
  }
}

static void amin(uint32_t* p, uint32_t v) {
  uint32_t cur = __atomic_load_n(p, __ATOMIC_RELAXED);
  while (v < cur && !__atomic_compare_exchange_n(p, &cur, v, 1, __ATOMIC_RELAXED, __ATOMIC_RELAXED)) {
  }
}

static void range(uint64_t len, int T, int id, uint64_t* b, uint64_t* e) {
  const uint64_t per = (len + T - 1) / T;
  *b = per * id < len ? per * id : len;
  *e = *b + per < len ? *b + per : len;
}

static void* worker(void* p) {
  Arg* a = (Arg*)p;
  Shared* s = a->s;
  const int T = s->nthreads, id = a->id;
  uint64_t b, e;
  /* first touch of the key tables, split across the threads */
  range(s->mask + 1, T, id, &b, &e);
  memset(s->tkey + b, 0xFF, (e - b) * 8);
  memset(s->com + b, 0xFF, (e - b) * 4);
  memset(s->und + b, 0xFF, (e - b) * 4);
  pthread_barrier_wait(&s->bar);
  /* phase 0: slots of every access; the initial list is 0..n-1 */
  range(s->n, T, id, &b, &e);
  for (uint64_t t = b; t < e; t++) {
    for (uint32_t x = s->off[t]; x < s->off[t + 1]; x++) s->aslot[x] = slot_of(s, s->keys[x]);
    s->list[0][t] = (uint32_t)t;
  }
  pthread_barrier_wait(&s->bar);
  int cur = 0;
  for (;;) {
    const uint64_t len = s->len;
    const uint32_t* L = s->list[cur];
    range(len, T, id, &b, &e);
    /* (a) min undecided writer per key */
    for (uint64_t q = b; q < e; q++) {
      const uint32_t t = L[q];
      for (uint32_t x = s->off[t]; x < s->off[t + 1]; x++)
        if (s->at[x] == AT_WR) amin(&s->und[s->aslot[x]], t);
    }
    pthread_barrier_wait(&s->bar);
    /* (b) decide; (c) compact this thread's share in place at its range start */
    uint64_t keep = b;
    uint32_t* out = s->list[cur ^ 1];
    for (uint64_t q = b; q < e; q++) {
      const uint32_t t = L[q];
      int kill = 0, block = 0;
      for (uint32_t x = s->off[t]; x < s->off[t + 1] && !kill; x++) {
        const uint32_t sl = s->aslot[x];
        const uint32_t c = __atomic_load_n(&s->com[sl], __ATOMIC_ACQUIRE);
        if (c < t) kill = 1;
        else if (s->und[sl] < t) block = 1;
      }
      if (kill) {
        s->state[t] = 2;
      } else if (!block) {
        s->state[t] = 1;
        for (uint32_t x = s->off[t]; x < s->off[t + 1]; x++)
          if (s->at[x] == AT_WR) __atomic_store_n(&s->com[s->aslot[x]], t, __ATOMIC_RELEASE);
      } else {
        out[keep++] = t;
      }
    }
    s->part[id] = keep - b;
    pthread_barrier_wait(&s->bar);
    /* (d) reset und for every writer of this round's list */
    for (uint64_t q = b; q < e; q++) {
      const uint32_t t = L[q];
      for (uint32_t x = s->off[t]; x < s->off[t + 1]; x++)
        if (s->at[x] == AT_WR)  /* several threads may reset one key: atomic (TSan) */
          __atomic_store_n(&s->und[s->aslot[x]], NONE, __ATOMIC_RELAXED);
    }
    pthread_barrier_wait(&s->bar);
    if (id == 0) {
      /* close the gaps between the threads' survivor runs (in list order) */
      uint64_t w = 0;
      for (int r = 0; r < T; r++) {
        uint64_t rb, re;
        range(len, T, r, &rb, &re);
        memmove(out + w, out + rb, s->part[r] * sizeof(uint32_t));
        w += s->part[r];
      }
      s->rounds++;
      if (len && w == len) s->err = 1; /* no progress: cannot happen */
      s->len = w;
      s->done = w == 0 || s->err;
    }
    pthread_barrier_wait(&s->bar);
    cur ^= 1;
    if (s->done) break;
  }
  return NULL;
}

int oracle_occ_rounds_mt(uint64_t n, const uint32_t* off, const uint64_t* keys,
                         const uint8_t* acctype, int nthreads, uint64_t* tnc, uint8_t* out_rc,
                         uint64_t* out_tn, uint32_t* out_rounds) {
  if (nthreads < 1) nthreads = 1;
  if (n >= NONE) return -1;
  const uint64_t nnz = off[n];
  uint64_t cap = 1024;
  while (cap < 2 * nnz + 2) cap <<= 1;
  Shared s;
  memset(&s, 0, sizeof s);
  s.n = n;
  s.off = off;
  s.keys = keys;
  s.at = acctype;
  s.mask = cap - 1;
  s.nthreads = nthreads;
  s.len = n;
  s.tkey = (uint64_t*)malloc(cap * 8);
  s.aslot = (uint32_t*)malloc((nnz ? nnz : 1) * 4);
  s.com = (uint32_t*)malloc(cap * 4);
  s.und = (uint32_t*)malloc(cap * 4);
  s.state = (uint8_t*)calloc(n ? n : 1, 1);
  s.list[0] = (uint32_t*)malloc((n ? n : 1) * 4);
  s.list[1] = (uint32_t*)malloc((n ? n : 1) * 4);
  s.part = (uint64_t*)calloc(nthreads, 8);
  pthread_t* th = (pthread_t*)malloc(sizeof(pthread_t) * nthreads);
  Arg* args = (Arg*)malloc(sizeof(Arg) * nthreads);
  int ret = 0;
  if (!s.tkey || !s.aslot || !s.com || !s.und || !s.state || !s.list[0] || !s.list[1] || !s.part ||
      !th || !args) {
    ret = -1;
    goto out;
  }
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
    ret = -2;
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
  if (out_rounds) *out_rounds = s.rounds;
out:
  free(s.tkey);
  free(s.aslot);
  free(s.com);
  free(s.und);
  free(s.state);
  free(s.list[0]);
  free(s.list[1]);
  free(s.part);
  free(th);
  free(args);
  return ret;
}
