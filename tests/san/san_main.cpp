// san_main.cpp — TEST INFRASTRUCTURE: host code under sanitizers (SURVEY.md §5
// build counterpart).  Exercises, with no GPU:
//   1. the OccEpoch shim (deneva_amd/csrc/host/occ_epoch.h): THREAD_CNT
//      workers validating concurrently through its mutex / condvar epoch map,
//      against the stub engine (stub_engine.c), capture files included;
//   2. the .dccb reader / writer (batch_file.cpp): round trips, then every
//      truncation and single-byte corruption of a file must be rejected
//      cleanly;
//   3. the oracle (oracle/*.c): literal and hash OCC, rounds-MT (threads),
//      Calvin, MaaT on random batches, cross-checked.
// Built twice by tests/san/Makefile: ASan+UBSan and TSan.  Exit 0 = clean.
#include <atomic>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <string>
#include <thread>
#include <vector>

#include "dcc.h"
#include "occ_epoch.h"
#include "oracle.h"

extern "C" dcc_ctx* stub_ctx(void);

static int fails = 0;
#define CHECK(c)                                                        \
  do {                                                                  \
    if (!(c)) {                                                         \
      fprintf(stderr, "CHECK failed %s:%d: %s\n", __FILE__, __LINE__, #c); \
      fails++;                                                          \
    }                                                                   \
  } while (0)

static void shim_threads(const char* dir, bool overlap, int depth = 4, int workers = 4) {
  dcc_host::OccEpoch::Options o;
  o.overlap = overlap;
  o.depth = depth;
  o.max_txns = 64;
  o.n_workers = workers;
  o.timer_ms = 1.0;
  o.capture_dir = dir;
  dcc_host::OccEpoch ep(stub_ctx(), o);
  std::atomic<uint64_t> commits{0}, aborts{0}, errs{0};
  std::vector<std::thread> th;
  for (int w = 0; w < workers; w++)
    th.emplace_back([&, w] {
      std::mt19937_64 rng(100 + w);
      for (int i = 0; i < 400; i++) {
        std::vector<dcc_host::Access> acc;
        const int len = 1 + (int)(rng() % 8);
        for (int k = 0; k < len; k++)
          acc.push_back({(uint64_t)(rng() % 64) * 4 + (uint64_t)k % 4, (uint8_t)(rng() % 2)});
        uint8_t rc = 0;
        const int e = ep.validate(acc.data(), acc.size(), &rc);
        if (e) errs++;
        else (rc == DCC_RC_RCOK ? commits : aborts)++;
      }
      ep.leave();
    });
  for (auto& t : th) t.join();
  const auto s = ep.stats();
  CHECK(errs == 0);
  CHECK(commits + aborts == 400ull * workers);
  CHECK(s.txns == 400ull * workers);
  CHECK(s.capture_errors == 0);
}

static void batch_files(const char* dir) {
  std::mt19937_64 rng(7);
  const uint64_t n = 300;
  std::vector<uint32_t> off(n + 1, 0);
  for (uint64_t t = 0; t < n; t++) off[t + 1] = off[t] + (uint32_t)(rng() % 9);
  const uint64_t nnz = off[n];
  std::vector<uint64_t> keys(nnz), st(n), ft(n), ord(n), ctn(n);
  std::vector<uint8_t> at(nnz), rc(n);
  std::vector<uint32_t> grp(nnz), wave(n);
  for (auto& k : keys) k = rng() % 1000;
  for (auto& a : at) a = (uint8_t)(rng() % 4);
  for (uint64_t t = 0; t < n; t++) {
    st[t] = rng() % 50;
    ft[t] = st[t] + rng() % 50;
    ord[t] = rng();
    rc[t] = (uint8_t)(rng() % 3);
    ctn[t] = rng() % 99;
    wave[t] = (uint32_t)(rng() % 5);
  }
  for (auto& g : grp) g = (uint32_t)(rng() % 4);
  dcc_batch b{};
  b.n_txn = n;
  b.nnz = nnz;
  b.offsets = off.data();
  b.keys = keys.data();
  b.acctype = at.data();
  b.start_tn = st.data();
  b.finish_tn = ft.data();
  b.order = ord.data();
  dcc_file_info fi{};
  fi.kind = DCC_FILE_OCC;
  fi.seed = 5;
  const std::string path = std::string(dir) + "/t.dccb";
  CHECK(dcc_file_write(path.c_str(), &fi, &b, rc.data(), ctn.data(), grp.data(), wave.data()) == 0);
  dcc_file_info ri{};
  CHECK(dcc_file_read_info(path.c_str(), &ri) == 0);
  CHECK(ri.n_txn == n && ri.nnz == nnz);
  std::vector<uint32_t> o2(n + 1), g2(nnz), w2(n);
  std::vector<uint64_t> k2(nnz), s2(n), f2(n), r2(n), c2(n);
  std::vector<uint8_t> a2(nnz), rc2(n);
  CHECK(dcc_file_read(path.c_str(), o2.data(), k2.data(), a2.data(), s2.data(), f2.data(), r2.data(),
                      rc2.data(), c2.data(), g2.data(), w2.data()) == 0);
  CHECK(o2 == off && k2 == keys && a2 == at && s2 == st && f2 == ft && r2 == ord && rc2 == rc &&
        c2 == ctn && g2 == grp && w2 == wave);
  // every truncation and a sweep of single-byte corruptions must fail cleanly
  std::vector<uint8_t> raw;
  {
    FILE* f = fopen(path.c_str(), "rb");
    int c;
    while ((c = fgetc(f)) != EOF) raw.push_back((uint8_t)c);
    fclose(f);
  }
  const std::string bad = std::string(dir) + "/bad.dccb";
  auto try_read = [&](const std::vector<uint8_t>& bytes) {
    FILE* f = fopen(bad.c_str(), "wb");
    if (!bytes.empty()) fwrite(bytes.data(), 1, bytes.size(), f);
    fclose(f);
    dcc_file_info bi{};
    if (dcc_file_read_info(bad.c_str(), &bi) != 0) return -1;
    if (bi.n_txn != n || bi.nnz != nnz) return -1;  // sizes from the header only
    return dcc_file_read(bad.c_str(), o2.data(), k2.data(), a2.data(), s2.data(), f2.data(),
                         r2.data(), rc2.data(), c2.data(), g2.data(), w2.data());
  };
  for (size_t cut = 0; cut < raw.size(); cut += 1 + cut / 8) {
    std::vector<uint8_t> t(raw.begin(), raw.begin() + cut);
    CHECK(try_read(t) != 0);
  }
  for (size_t pos = 0; pos < raw.size(); pos += 1 + pos / 16) {
    std::vector<uint8_t> t = raw;
    t[pos] ^= 0x5A;
    CHECK(try_read(t) != 0);
  }
}

static void oracles() {
  std::mt19937_64 rng(11);
  for (int it = 0; it < 30; it++) {
    const uint64_t n = 1 + rng() % 500, nk = 1 + rng() % 300;
    std::vector<uint32_t> off(n + 1, 0);
    for (uint64_t t = 0; t < n; t++) off[t + 1] = off[t] + (uint32_t)(rng() % 12);
    const uint64_t nnz = off[n];
    std::vector<uint64_t> keys(nnz + 1);
    std::vector<uint8_t> at(nnz + 1);
    for (uint64_t x = 0; x < nnz; x++) {
      keys[x] = rng() % nk;
      at[x] = (uint8_t)(rng() % 4);
    }
    std::vector<uint8_t> r1(n), r2(n), r3(n);
    std::vector<uint64_t> t1(n), t2(n), t3(n);
    uint64_t c1 = 0, c2 = 0, c3 = 0;
    uint32_t rounds = 0;
    CHECK(oracle_occ_replay(n, off.data(), keys.data(), at.data(), nullptr, nullptr, 0, nullptr,
                            nullptr, &c1, r1.data(), t1.data()) == 0);
    CHECK(oracle_occ_hash(n, off.data(), keys.data(), at.data(), nullptr, nullptr, 0, nullptr,
                          nullptr, &c2, r2.data(), t2.data()) == 0);
    CHECK(oracle_occ_rounds_mt(n, off.data(), keys.data(), at.data(), 4, &c3, r3.data(), t3.data(),
                               &rounds) == 0);
    CHECK(r1 == r2 && r2 == r3 && t1 == t2 && t2 == t3 && c1 == c2 && c2 == c3);
    std::vector<uint32_t> g1(nnz + 1), g2(nnz + 1), w1(n), w2(n);
    std::vector<uint8_t> q1(n), q2(n);
    CHECK(oracle_calvin_replay(n, off.data(), keys.data(), at.data(), nullptr, g1.data(), q1.data(),
                               w1.data()) == 0);
    CHECK(oracle_calvin_formula(n, off.data(), keys.data(), at.data(), nullptr, g2.data(),
                                q2.data(), w2.data()) == 0);
    CHECK(g1 == g2 && q1 == q2 && w1 == w2);
    std::vector<uint64_t> rk(nk), lr1(nk), lw1(nk), lr2(nk), lw2(nk), m1(n), m2(n);
    for (uint64_t k = 0; k < nk; k++) {
      rk[k] = k;
      lr1[k] = lr2[k] = rng() % 20;
      lw1[k] = lw2[k] = rng() % 20;
    }
    std::vector<uint8_t> mr1(n), mr2(n);
    CHECK(oracle_maat_replay(n, off.data(), keys.data(), at.data(), it & 1, nk, rk.data(), lr1.data(),
                             lw1.data(), mr1.data(), m1.data()) == 0);
    CHECK(oracle_maat_formula(n, off.data(), keys.data(), at.data(), it & 1, nk, rk.data(),
                              lr2.data(), lw2.data(), mr2.data(), m2.data()) == 0);
    CHECK(mr1 == mr2 && m1 == m2 && lr1 == lr2 && lw1 == lw2);
  }
}

int main(int argc, char** argv) {
  const char* dir = argc > 1 ? argv[1] : ".";
  shim_threads(dir, true);         // 4 epochs in flight
  shim_threads(dir, true, 1);      // one in flight
  shim_threads(dir, true, 4, 12);  // 12 workers: epochs close while others are in flight
  shim_threads(dir, false);
  batch_files(dir);
  oracles();
  if (fails) {
    fprintf(stderr, "%d checks failed\n", fails);
    return 1;
  }
  printf("sanitizer harness clean\n");
  return 0;
}
