/* kmap.h — tiny open-addressing u64 -> u64 map for the oracle (test infrastructure). */
#ifndef DCC_ORACLE_KMAP_H_
#define DCC_ORACLE_KMAP_H_
#include <stdint.h>
#include <stdlib.h>

typedef struct {
  uint64_t* k;
  uint64_t* v;
  uint8_t* used;
  uint64_t cap, n;
} kmap;

static inline uint64_t kmap_h(uint64_t x) {
  x ^= x >> 31;
  x *= 0x7fb5d329728ea185ull;
  x ^= x >> 27;
  x *= 0x81dadef4bc2dd44dull;
  x ^= x >> 33;
  return x;
}

static inline int kmap_init(kmap* m, uint64_t expect) {
  uint64_t cap = 16;
  while (cap < 2 * expect + 2) cap <<= 1;
  m->k = (uint64_t*)malloc(cap * 8);
  m->v = (uint64_t*)malloc(cap * 8);
  m->used = (uint8_t*)calloc(cap, 1);
  m->cap = cap;
  m->n = 0;
  return (m->k && m->v && m->used) ? 0 : -1;
}

static inline void kmap_free(kmap* m) {
  free(m->k);
  free(m->v);
  free(m->used);
}

static inline int kmap_grow(kmap* m);

/* pointer to the value slot of key; inserts (value = dflt) when absent */
static inline uint64_t* kmap_get(kmap* m, uint64_t key, uint64_t dflt) {
  if (2 * (m->n + 1) > m->cap && kmap_grow(m)) return NULL;
  uint64_t h = kmap_h(key) & (m->cap - 1);
  while (m->used[h]) {
    if (m->k[h] == key) return &m->v[h];
    h = (h + 1) & (m->cap - 1);
  }
  m->used[h] = 1;
  m->k[h] = key;
  m->v[h] = dflt;
  m->n++;
  return &m->v[h];
}

static inline const uint64_t* kmap_find(const kmap* m, uint64_t key) {
  uint64_t h = kmap_h(key) & (m->cap - 1);
  while (m->used[h]) {
    if (m->k[h] == key) return &m->v[h];
    h = (h + 1) & (m->cap - 1);
  }
  return NULL;
}

static inline int kmap_grow(kmap* m) {
  kmap o = *m;
  if (kmap_init(m, o.cap)) return -1;
  for (uint64_t i = 0; i < o.cap; i++)
    if (o.used[i]) *kmap_get(m, o.k[i], 0) = o.v[i];
  kmap_free(&o);
  return 0;
}

#endif
