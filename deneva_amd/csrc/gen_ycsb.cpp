// YCSB batch producer — deterministic restatement of the reference generator.
//
//   myrand           system/helper.cpp:144-147
//   zeta / zipf      benchmarks/ycsb_query.cpp:181-202 (init: :29-38)
//   gen_requests_zipf benchmarks/ycsb_query.cpp:303-376
//   key_to_part      benchmarks/ycsb_wl.cpp:69-74 (key % part_cnt)
//
// The draw sequence per transaction is the reference's: r_twr, then per
// request r, [partition], zipf, value — duplicates consume their draws and
// retry (ycsb_query.cpp:342-350).  Only the seeding differs: the reference
// seeds from the clock (ycsb_query.cpp:31); here each chunk of chunk_txns
// transactions owns a stream seeded from (seed, chunk index).
#include <cmath>
#include <cstring>
#include <map>
#include <mutex>
#include <thread>
#include <vector>

#include "dcc.h"
#include "dcc_internal.h"

namespace dcc {

double zeta_cached(uint64_t n, double theta) {
  // zeta(n, theta) = sum_{i=1..n} (1/i)^theta, summed in the reference's
  // order (ycsb_query.cpp:181-186) so the double is bit-identical.
  static std::mutex mu;
  static std::map<std::pair<uint64_t, double>, double> cache;
  {
    std::lock_guard<std::mutex> g(mu);
    auto it = cache.find({n, theta});
    if (it != cache.end()) return it->second;
  }
  double sum = 0;
  for (uint64_t i = 1; i <= n; i++) sum += pow(1.0 / i, theta);
  std::lock_guard<std::mutex> g(mu);
  cache[{n, theta}] = sum;
  return sum;
}

namespace {

struct Zipf {
  uint64_t n;
  double theta, alpha, zetan, eta, half_pow;
  Zipf(uint64_t n_, double theta_) : n(n_), theta(theta_) {
    const double zeta_2 = zeta_cached(2, theta);
    zetan = zeta_cached(n, theta);
    alpha = 1 / (1 - theta);
    eta = (1 - pow(2.0 / n, 1 - theta)) / (1 - zeta_2 / zetan);
    half_pow = pow(0.5, theta);
  }
  // ycsb_query.cpp:188-202; returns a value in [1, n]
  uint64_t draw(MyRand& r) const {
    double u = (double)(r.next() % 10000000) / 10000000;
    double uz = u * zetan;
    if (uz < 1) return 1;
    if (uz < 1 + half_pow) return 2;
    return 1 + (uint64_t)(n * pow(eta * u - eta + 1, alpha));
  }
};

struct SmallSet {  // <= MAX_ROW_PER_TXN entries; linear scan beats std::set here
  uint64_t v[128];
  uint32_t n = 0;
  bool has(uint64_t x) const {
    for (uint32_t i = 0; i < n; i++)
      if (v[i] == x) return true;
    return false;
  }
  void add(uint64_t x) { v[n++] = x; }
};

}  // namespace
}  // namespace dcc

using namespace dcc;

extern "C" void dcc_ycsb_params_default(dcc_ycsb_params* p) {
  memset(p, 0, sizeof(*p));
  p->n_txn = 65536;
  p->req_per_query = 16;
  p->part_cnt = 1;
  p->table_size = 16777216;
  p->zipf_theta = 0.9;
  p->txn_write_perc = 0.5;
  p->tup_write_perc = 0.5;
  p->part_per_txn = 1;
  p->strict_ppt = 0;
  p->first_part_local = 1;
  p->chunk_txns = 65536;
  p->seed = 0xD3E7A001ull;
  p->n_threads = 0;
}

extern "C" int dcc_gen_ycsb(const dcc_ycsb_params* p, uint32_t* offsets, uint64_t* keys,
                            uint8_t* acctype, uint32_t* home) {
  if (!p || !offsets || !keys || !acctype) return DCC_EINVAL;
  const uint64_t k = p->req_per_query;
  if (k == 0 || k > 64 || p->part_cnt == 0 || p->zipf_theta < 0 || p->zipf_theta >= 1)
    return DCC_EINVAL;
  if (p->n_txn * k > 0xFFFFFFFFull) return DCC_ERANGE;
  const uint64_t part_rows = p->table_size / p->part_cnt;  // ycsb_query.cpp:309
  if (part_rows < 3 || part_rows - 1 < k) return DCC_EINVAL;
  const Zipf zipf(part_rows - 1, p->zipf_theta);           // the_n = table_size-1 (:35)
  const double txn_read_perc = 1.0 - p->txn_write_perc;    // global.cpp:86
  const double tup_read_perc = 1.0 - p->tup_write_perc;    // global.cpp:88
  const uint64_t chunk = p->chunk_txns ? p->chunk_txns : p->n_txn;
  const uint64_t n_chunks = p->n_txn ? (p->n_txn + chunk - 1) / chunk : 0;

  for (uint64_t t = 0; t <= p->n_txn; t++) offsets[t] = (uint32_t)(t * k);

  std::atomic<int> err{0};
  auto run_chunk = [&](uint64_t c) {
    MyRand rng;
    rng.init(chunk_seed(p->seed, c));
    const uint32_t home_part = (uint32_t)(c % p->part_cnt);
    const uint64_t t0 = c * chunk, t1 = std::min(p->n_txn, t0 + chunk);
    for (uint64_t t = t0; t < t1; t++) {
      SmallSet all_keys, parts;
      const double r_twr = (double)(rng.next() % 10000) / 10000;
      uint32_t rid = 0, guard = 0;
      for (uint32_t i = 0; i < k; i++) {
        if (++guard > 1000000) { err = DCC_EINVAL; return; }
        const double r = (double)(rng.next() % 10000) / 10000;
        uint64_t pid;
        if (p->first_part_local && rid == 0) {
          pid = home_part;
        } else {
          pid = rng.next() % p->part_cnt;
          if (p->strict_ppt && p->part_per_txn <= p->part_cnt) {
            while ((parts.n < p->part_per_txn && parts.has(pid)) ||
                   (parts.n == p->part_per_txn && !parts.has(pid)))
              pid = rng.next() % p->part_cnt;
          }
        }
        const uint8_t at = (r_twr < txn_read_perc || r < tup_read_perc) ? DCC_RD : DCC_WR;
        const uint64_t row_id = zipf.draw(rng);
        const uint64_t key = row_id * p->part_cnt + pid;
        (void)(rng.next() % (1 << 8));  // req->value draw (ycsb_query.cpp:339)
        if (all_keys.has(key)) { i--; continue; }
        all_keys.add(key);
        if (!parts.has(pid)) parts.add(pid);
        keys[t * k + rid] = key;
        acctype[t * k + rid] = at;
        rid++;
      }
      if (home) home[t] = home_part;
    }
  };
  parallel_for(n_chunks, p->n_threads, run_chunk);
  return err.load();
}

extern "C" uint64_t dcc_alg_bytes(uint64_t n_txn, uint64_t nnz, uint64_t nnz_w) {
  return 4 * (n_txn + 1) + 9 * nnz + 16 * nnz_w + 16 * nnz + n_txn;
}
