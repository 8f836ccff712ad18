// TPC-C NewOrder + Payment batch producer.
//
// Restates the reference's query generators and the access sets the two
// transactions record through get_row / get_lock:
//
//   create_query            tpcc_query.cpp:26-33   (x < PERC_PAYMENT -> Payment)
//   gen_payment             tpcc_query.cpp:149-203
//   gen_new_order           tpcc_query.cpp:205-263
//   URand / NURand / RAND   tpcc_helper.cpp:93-134 (rand() -> per-chunk myrand stream)
//   key functions           tpcc_helper.cpp:19-47, wh_to_part :161-164
//   Payment accesses        tpcc_txn.cpp:140-183 / 517-662:
//       WAREHOUSE w_id        WR if WH_UPDATE else RD
//       DISTRICT distKey      WR
//       CUSTOMER custKey      WR  (by last name: the middle row of the
//                                  i_customer_last chain, :594-625)
//   NewOrder accesses       tpcc_txn.cpp:189-230 / 717-874:
//       WAREHOUSE w_id RD, CUSTOMER custKey RD, DISTRICT distKey WR,
//       per item: ITEM ol_i_id RD, STOCK stockKey WR
//   Inserts (order, new-order, order-line, history) are not accesses
//   (txn.cpp:899-904).
//
// Canonical key = DCC_TPCC_KEY(TPCCTable enum value, index key) (config.h:200).
//
// Determinism: the reference draws from the process-global rand() and
// loads the customer table with g_init_parallelism threads, so neither its
// streams nor its by-last-name chains are reproducible.  Here every chunk of
// `chunk_txns` queries has its own myrand stream, the NURand C constants come
// from the seed, and the customer table is "loaded" once in cid order (so a
// name chain is ordered by descending cid: index_insert pushes at the chain
// head, index_hash.cpp:197-199).
#include <algorithm>
#include <atomic>
#include <cstring>
#include <vector>

#include "dcc.h"
#include "dcc_internal.h"

using namespace dcc;

namespace {

enum : uint64_t { T_WAREHOUSE = 0, T_DISTRICT = 1, T_CUSTOMER = 2, T_ITEM = 7, T_STOCK = 8 };

struct TpccRand {
  MyRand r;
  uint64_t c255, c1023, c8191;  // NURand run-time constants
  uint64_t rand_() { return r.next(); }                      // rand()
  uint64_t RAND(uint64_t max) { return rand_() % max; }       // tpcc_helper.cpp:93
  uint64_t URand(uint64_t x, uint64_t y) { return x + RAND(y - x + 1); }
  uint64_t NURand(uint64_t A, uint64_t x, uint64_t y) {       // tpcc_helper.cpp:101-134
    const uint64_t C = A == 255 ? c255 : A == 1023 ? c1023 : c8191;
    return (((URand(0, A) | URand(x, y)) + C) % (y - x + 1)) + x;
  }
};

// Lastname(num) (tpcc_helper.cpp:83-91) and the name part of custNPKey
// (tpcc_helper.cpp:35-43): key = sum of (c - 'A') shifted left one bit per char.
const char* const kSyl[10] = {"BAR", "OUGHT", "ABLE", "PRI", "PRES",
                              "ESE", "ANTI", "CALLY", "ATION", "EING"};
uint64_t name_key(uint32_t num) {
  char name[32];
  strcpy(name, kSyl[num / 100]);
  strcat(name, kSyl[(num / 10) % 10]);
  strcat(name, kSyl[num % 10]);
  uint64_t key = 0;
  for (const char* c = name; *c; c++) key = (key << 1) + (uint64_t)(*c - 'A');
  return key;
}

struct Params {
  uint64_t num_wh, dist, cust, items, max_ol, part_cnt, part_per_txn;
  double perc_payment, mpr;
  bool wh_update, first_local;
};

uint64_t wh_to_part(const Params& P, uint64_t w) { return (w - 1) % P.part_cnt; }
uint64_t dist_key(const Params& P, uint64_t d, uint64_t w) { return w * P.dist + d; }
uint64_t cust_key(const Params& P, uint64_t c, uint64_t d, uint64_t w) {
  return dist_key(P, d, w) * P.cust + c;
}
uint64_t stock_key(const Params& P, uint64_t i, uint64_t w) { return w * P.items + i; }

// Customer last-name index: per (w, d) and per distinct name key, the cids
// carrying it in descending order (the chain walk order).
struct CustIndex {
  uint64_t dist = 0, cust = 0;
  std::vector<uint32_t> nameclass;    // name number -> class id (equal name keys)
  uint32_t nclass = 0;
  std::vector<uint32_t> start;        // [(w*dist + d-1) * nclass + class] -> offset
  std::vector<uint32_t> cids;
  uint32_t pick(uint64_t w, uint64_t d, uint32_t num) const {  // middle of the chain
    const uint64_t base = ((w - 1) * dist + (d - 1)) * nclass + nameclass[num];
    const uint32_t s = start[base], e = start[base + 1];
    if (s == e) return 0;
    return cids[s + (e - s) / 2];
  }
};

bool build_cust_index(const Params& P, uint64_t seed, unsigned threads, CustIndex& ix) {
  ix.dist = P.dist;
  ix.cust = P.cust;
  // name numbers with equal name keys share a chain (custNPKey collisions)
  ix.nameclass.assign(1000, 0);
  std::vector<uint64_t> keys(1000);
  for (uint32_t i = 0; i < 1000; i++) keys[i] = name_key(i);
  std::vector<uint64_t> uniq(keys);
  std::sort(uniq.begin(), uniq.end());
  uniq.erase(std::unique(uniq.begin(), uniq.end()), uniq.end());
  ix.nclass = (uint32_t)uniq.size();
  for (uint32_t i = 0; i < 1000; i++)
    ix.nameclass[i] = (uint32_t)(std::lower_bound(uniq.begin(), uniq.end(), keys[i]) - uniq.begin());
  const uint64_t nwd = P.num_wh * P.dist;
  if (nwd * ix.nclass + 1 > 0xFFFFFFFFull || nwd * P.cust > 0xFFFFFFFFull) return false;
  ix.start.assign(nwd * ix.nclass + 1, 0);
  ix.cids.assign(nwd * P.cust, 0);
  // load-time NURand constant (tpcc_wl.cpp:369-374 draws from the loader's rand())
  MyRand cr;
  cr.init(chunk_seed(seed ^ 0x10ADull, 0));
  const uint64_t c_load = cr.next() % 256;
  parallel_for(nwd, threads, [&](uint64_t wd) {
    TpccRand tr;
    tr.r.init(chunk_seed(seed ^ 0x10ADull, wd + 1));
    tr.c255 = c_load;
    std::vector<uint32_t> cls(P.cust);
    std::vector<uint32_t> cnt(ix.nclass, 0);
    for (uint64_t cid = 1; cid <= P.cust; cid++) {
      const uint32_t num = cid <= 1000 ? (uint32_t)(cid - 1) : (uint32_t)tr.NURand(255, 0, 999);
      cls[cid - 1] = ix.nameclass[num];
      cnt[cls[cid - 1]]++;
    }
    // local offsets (the global start array is filled below)
    std::vector<uint32_t> off(ix.nclass + 1, 0);
    for (uint32_t c = 0; c < ix.nclass; c++) off[c + 1] = off[c] + cnt[c];
    uint32_t* out = &ix.cids[wd * P.cust];
    std::vector<uint32_t> fill(off.begin(), off.end() - 1);
    for (uint64_t cid = P.cust; cid >= 1; cid--) out[fill[cls[cid - 1]]++] = (uint32_t)cid;
    for (uint32_t c = 0; c < ix.nclass; c++)
      ix.start[wd * ix.nclass + c] = (uint32_t)(wd * P.cust + off[c]);
  });
  ix.start[nwd * ix.nclass] = (uint32_t)(nwd * P.cust);
  return true;
}

}  // namespace

extern "C" void dcc_tpcc_params_default(dcc_tpcc_params* p) {
  memset(p, 0, sizeof(*p));
  p->n_txn = 262144;
  p->num_wh = 128;
  p->part_cnt = 1;
  p->perc_payment = 0.5;
  p->wh_update = 1;
  p->max_items = 100000;
  p->cust_per_dist = 3000;
  p->dist_per_wh = 10;
  p->max_items_per_txn = 15;
  p->part_per_txn = 1;
  p->mpr = 1.0;
  p->first_part_local = 1;
  p->chunk_txns = 65536;
  p->seed = 0xD3E7A003ull;
}

extern "C" uint32_t dcc_tpcc_max_access(const dcc_tpcc_params* p) {
  return 3 + 2 * (p ? p->max_items_per_txn : 15);
}

extern "C" int dcc_gen_tpcc(const dcc_tpcc_params* p, uint32_t* offsets, uint64_t* keys,
                            uint8_t* acctype, uint8_t* txn_type, uint64_t* out_nnz) {
  if (!p || !offsets || !keys || !acctype || !out_nnz) return DCC_EINVAL;
  Params P{p->num_wh, p->dist_per_wh, p->cust_per_dist, p->max_items, p->max_items_per_txn,
           p->part_cnt, p->part_per_txn, p->perc_payment, p->mpr, p->wh_update != 0,
           p->first_part_local != 0};
  if (P.num_wh == 0 || P.dist == 0 || P.cust == 0 || P.items == 0 || P.part_cnt == 0 ||
      P.part_cnt > P.num_wh || P.max_ol < 5 || P.max_ol > 30 || P.items < P.max_ol ||
      P.num_wh > 1023)
    return DCC_EINVAL;
  const uint32_t maxa = dcc_tpcc_max_access(p);
  if (p->n_txn * maxa > 0xFFFFFFFFull) return DCC_ERANGE;
  CustIndex ix;
  if (!build_cust_index(P, p->seed, p->n_threads, ix)) return DCC_ERANGE;

  // run-time NURand constants, fixed by the seed for the whole batch
  MyRand cr;
  cr.init(chunk_seed(p->seed ^ 0xC0417ull, 0));
  const uint64_t c255 = cr.next() % 256, c1023 = cr.next() % 1024, c8191 = cr.next() % 8192;

  const uint64_t chunk = p->chunk_txns ? p->chunk_txns : p->n_txn;
  const uint64_t n_chunks = p->n_txn ? (p->n_txn + chunk - 1) / chunk : 0;
  // per-txn lengths first (slots of maxa per txn), compacted afterwards
  std::vector<uint8_t> len(p->n_txn);
  std::atomic<int> err{0};
  parallel_for(n_chunks, p->n_threads, [&](uint64_t c) {
    TpccRand R;
    R.r.init(chunk_seed(p->seed, c));
    R.c255 = c255;
    R.c1023 = c1023;
    R.c8191 = c8191;
    const uint64_t home_part = c % P.part_cnt;
    const uint64_t t0 = c * chunk, t1 = std::min<uint64_t>(p->n_txn, t0 + chunk);
    for (uint64_t t = t0; t < t1; t++) {
      uint64_t* k = keys + t * maxa;
      uint8_t* a = acctype + t * maxa;
      uint32_t n = 0;
      auto put = [&](uint64_t table, uint64_t ikey, uint8_t at) {
        k[n] = DCC_TPCC_KEY(table, ikey);
        a[n] = at;
        n++;
      };
      const double x = (double)(R.rand_() % 100) / 100.0;  // create_query
      uint64_t w;
      auto pick_home = [&]() {
        if (P.first_local) {
          uint64_t guard = 0;
          while (wh_to_part(P, w = R.URand(1, P.num_wh)) != home_part)
            if (++guard > 100000000) { err = DCC_EINVAL; return false; }
        } else {
          w = R.URand(1, P.num_wh);
        }
        return true;
      };
      if (x < P.perc_payment) {
        // ---- gen_payment (tpcc_query.cpp:149-203)
        if (txn_type) txn_type[t] = 1;  // TPCC_PAYMENT
        if (!pick_home()) return;
        const uint64_t d = R.URand(1, P.dist);
        (void)R.URand(1, 5000);  // h_amount
        const double xr = (double)(R.rand_() % 10000) / 10000;
        const uint64_t y = R.URand(1, 100);
        uint64_t c_d = d, c_w = w;
        if (!(xr > 0.15)) {  // remote customer warehouse
          c_d = R.URand(1, P.dist);
          if (P.num_wh > 1) {
            while ((c_w = R.URand(1, P.num_wh)) == w) {}
          } else {
            c_w = w;
          }
        }
        uint64_t cid;
        if (y <= 60) {
          const uint32_t num = (uint32_t)R.NURand(255, 0, 999);  // by last name
          cid = ix.pick(c_w, c_d, num);
          if (cid == 0) { err = DCC_EINVAL; return; }  // the reference asserts (:615)
        } else {
          cid = R.NURand(1023, 1, P.cust);
        }
        put(T_WAREHOUSE, w, P.wh_update ? DCC_WR : DCC_RD);
        put(T_DISTRICT, dist_key(P, d, w), DCC_WR);
        put(T_CUSTOMER, cust_key(P, cid, c_d, c_w), DCC_WR);
      } else {
        // ---- gen_new_order (tpcc_query.cpp:205-263)
        if (txn_type) txn_type[t] = 2;  // TPCC_NEW_ORDER
        if (!pick_home()) return;
        const uint64_t d = R.URand(1, P.dist);
        const uint64_t cid = R.NURand(1023, 1, P.cust);
        const uint64_t ol_cnt = R.URand(5, P.max_ol);
        const double r_mpr = (double)(R.rand_() % 10000) / 10000;
        const uint64_t part_limit = r_mpr < P.mpr ? P.part_per_txn : 1;
        uint64_t parts[64];
        uint32_t nparts = 0;
        parts[nparts++] = wh_to_part(P, w);
        auto has_part = [&](uint64_t q) {
          for (uint32_t i = 0; i < nparts; i++)
            if (parts[i] == q) return true;
          return false;
        };
        uint64_t item[32], supply[32];
        for (uint64_t i = 0; i < ol_cnt; i++) {
          uint64_t id;
          bool dup;
          do {
            id = R.NURand(8191, 1, P.items);
            dup = false;
            for (uint64_t j = 0; j < i; j++) dup |= item[j] == id;
          } while (dup);
          item[i] = id;
          (void)R.URand(1, 10);  // ol_quantity
          const double r_rem = (double)(R.rand_() % 100000) / 100000;
          if (r_rem > 0.01 || r_mpr > P.mpr || P.num_wh == 1) {
            supply[i] = w;
          } else if (nparts < part_limit) {
            supply[i] = R.URand(1, P.num_wh);
            if (!has_part(wh_to_part(P, supply[i])) && nparts < 64)
              parts[nparts++] = wh_to_part(P, supply[i]);
          } else {
            while (!has_part(wh_to_part(P, supply[i] = R.URand(1, P.num_wh)))) {}
          }
        }
        put(T_WAREHOUSE, w, DCC_RD);
        put(T_CUSTOMER, cust_key(P, cid, d, w), DCC_RD);
        put(T_DISTRICT, dist_key(P, d, w), DCC_WR);
        for (uint64_t i = 0; i < ol_cnt; i++) {
          put(T_ITEM, item[i], DCC_RD);
          put(T_STOCK, stock_key(P, item[i], supply[i]), DCC_WR);
        }
      }
      len[t] = (uint8_t)n;
    }
  });
  if (err.load()) return err.load();
  // compact the fixed-stride slots into CSR (in place, forward)
  uint64_t w = 0;
  offsets[0] = 0;
  for (uint64_t t = 0; t < p->n_txn; t++) {
    const uint64_t src = t * maxa;
    if (src != w) {
      memmove(keys + w, keys + src, len[t] * sizeof(uint64_t));
      memmove(acctype + w, acctype + src, len[t]);
    }
    w += len[t];
    offsets[t + 1] = (uint32_t)w;
  }
  *out_nnz = w;
  return DCC_OK;
}
