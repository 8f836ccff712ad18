// c1_driver — the C1 configuration's host driver (BASELINE.json configs[0]:
// YCSB, one server node, CC_ALG=OCC, THREAD_CNT=4, 10 req/txn, theta=0.6).
//
// THREAD_CNT worker threads each generate their txns with the restated YCSB
// generator (dcc_gen_ycsb: gen_requests_zipf, benchmarks/ycsb_query.cpp:
// 303-376) and validate them through the OccEpoch shim exactly where the
// reference's workers call TxnManager::validate; an aborted txn is restarted
// (re-validated in a later epoch, as WorkerThread restarts it).  Every decided
// epoch can be captured as a .dccb file with its decisions (--capture DIR),
// which tests/test_host_shim.py checks against the oracle.  --calvin runs the
// same workload through the CalvinEpoch sequencer hand-off instead (each
// worker is an origin node).  Prints one JSON line.
#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

#include "calvin_epoch.h"
#include "dcc.h"
#include "occ_epoch.h"
#include "occ_live.h"

using namespace dcc_host;

struct Cfg {
  int threads = 4;             // THREAD_CNT
  uint64_t txns = 2000;        // txns per worker
  double theta = 0.6;          // ZIPF_THETA
  uint32_t req = 10;           // REQ_PER_QUERY
  uint64_t table = 65536;      // SYNTH_TABLE_SIZE of C1 (config.h:169)
  uint64_t epoch_max = 256;    // txns per epoch (cap)
  double timer_ms = 5.0;
  uint64_t seed = 7;
  int device = 0;
  int gpus = 0;                // > 0: one process drives this many shards (dcc_init_multi)
  int max_retries = 1000;
  bool calvin = false;
  bool live = false;           // live OptCC run on the workers, capture replayed on the GPU
  bool overlap = true;         // OccEpoch fills epoch N+1 while N is on the GPU
  int depth = 4;               // OccEpoch: closed epochs on the GPU at once
  std::string capture;
};

static void usage() {
  fprintf(stderr,
          "c1_driver [--threads N] [--txns N] [--theta T] [--req N] [--table N]\n"
          "          [--epoch-max N] [--timer-ms T] [--seed S] [--device D] [--gpus N]\n"
          "          [--capture DIR] [--calvin | --live] [--no-overlap] [--depth N]\n");
}

static int parse(int argc, char** argv, Cfg& c) {
  for (int i = 1; i < argc; i++) {
    const std::string a = argv[i];
    auto val = [&](void) -> const char* { return i + 1 < argc ? argv[++i] : nullptr; };
    const char* v = nullptr;
    if (a == "--help" || a == "-h") return 1;
    if (a == "--calvin") { c.calvin = true; continue; }
    if (a == "--live") { c.live = true; continue; }
    if (a == "--no-overlap") { c.overlap = false; continue; }
    if (!(v = val())) return 2;
    if (a == "--threads") c.threads = atoi(v);
    else if (a == "--txns") c.txns = strtoull(v, nullptr, 0);
    else if (a == "--theta") c.theta = atof(v);
    else if (a == "--req") c.req = (uint32_t)atoi(v);
    else if (a == "--table") c.table = strtoull(v, nullptr, 0);
    else if (a == "--epoch-max") c.epoch_max = strtoull(v, nullptr, 0);
    else if (a == "--timer-ms") c.timer_ms = atof(v);
    else if (a == "--seed") c.seed = strtoull(v, nullptr, 0);
    else if (a == "--device") c.device = atoi(v);
    else if (a == "--gpus") c.gpus = atoi(v);
    else if (a == "--capture") c.capture = v;
    else if (a == "--depth") c.depth = atoi(v);
    else return 2;
  }
  return (c.threads > 0 && c.txns > 0 && c.req > 0 && c.depth >= 1) ? 0 : 2;
}

// one worker's txns from the restated generator (its own stream)
static int gen(const Cfg& c, int w, std::vector<uint32_t>& off, std::vector<uint64_t>& keys,
               std::vector<uint8_t>& at) {
  dcc_ycsb_params p;
  dcc_ycsb_params_default(&p);
  p.n_txn = c.txns;
  p.req_per_query = c.req;
  p.part_cnt = 1;
  p.table_size = c.table;
  p.zipf_theta = c.theta;
  p.chunk_txns = (uint32_t)c.txns;
  p.seed = c.seed * 1000003ull + (uint64_t)w;
  p.n_threads = 1;
  off.resize(c.txns + 1);
  keys.resize(c.txns * c.req);
  at.resize(c.txns * c.req);
  return dcc_gen_ycsb(&p, off.data(), keys.data(), at.data(), nullptr);
}

int main(int argc, char** argv) {
  Cfg c;
  if (int r = parse(argc, argv, c)) {
    usage();
    return r == 1 ? 0 : 2;
  }
  dcc_ctx* ctx = nullptr;
  int e = 0;
  if (c.gpus > 0) {
    // the node's GPUs inside one context: devices 0..N-1 when present, else
    // the shards share the GPUs there are (in-process exchange)
    int ndev = dcc_device_count();
    if (ndev < 1) ndev = 1;
    std::vector<int> ids(c.gpus);
    for (int g = 0; g < c.gpus; g++) ids[g] = g % ndev;
    e = dcc_init_multi(&ctx, c.gpus, ids.data());
  } else {
    e = dcc_init(&ctx, c.device);
  }
  if (e) {
    fprintf(stderr, "dcc_init: %s %s\n", dcc_strerror(e), ctx ? dcc_last_error(ctx) : "");
    return 1;
  }
  std::vector<std::vector<uint32_t>> off(c.threads);
  std::vector<std::vector<uint64_t>> keys(c.threads);
  std::vector<std::vector<uint8_t>> at(c.threads);
  for (int w = 0; w < c.threads; w++)
    if (int e = gen(c, w, off[w], keys[w], at[w])) {
      fprintf(stderr, "dcc_gen_ycsb: %s\n", dcc_strerror(e));
      return 1;
    }
  const auto t0 = std::chrono::steady_clock::now();
  std::atomic<int> failed{0};
  std::atomic<uint64_t> commits{0}, restarts{0}, ready{0}, waits{0}, gave_up{0};
  uint64_t epochs = 0;
  double device_ms = 0;
  long long live_mismatch = -1;

  if (c.live) {
    // live, concurrent OptCC on the worker threads (occ_live.h), then the
    // whole capture decided again by dcc_occ_validate_snapshot
    LiveOcc occ;
    std::vector<std::thread> ws;
    for (int w = 0; w < c.threads; w++)
      ws.emplace_back([&, w] {
        std::vector<Access> acc;
        uint64_t spin = c.seed * 2654435761ull + (uint64_t)w;
        for (uint64_t i = 0; i < c.txns && !failed; i++) {
          acc.clear();
          for (uint32_t x = off[w][i]; x < off[w][i + 1]; x++) acc.push_back({keys[w][x], at[w][x]});
          for (int attempt = 0;; attempt++) {  // WorkerThread: restart on Abort
            const uint64_t st = occ.get_ts();
            spin = spin * 6364136223846793005ull + 1442695040888963407ull;
            for (volatile uint64_t z = 0; z < ((spin >> 33) & 1023); z = z + 1) {}  // execution
            uint8_t rc = DCC_RC_ABORT;
            const uint32_t rec = occ.validate(acc.data(), acc.size(), st, &rc);
            if (rc == DCC_RC_RCOK) {
              occ.finish_commit(rec);
              commits++;
              break;
            }
            restarts++;
            if (attempt >= c.max_retries) {  // starved by hot writers: the live
              gave_up++;                     // run moves on (not an engine error)
              break;
            }
          }
        }
      });
    for (auto& t : ws) t.join();
    const LiveCapture cap = occ.take();
    uint64_t bad = 0;
    dcc_stats s{};
    if (int e = validate_capture(ctx, cap, &bad, &s)) {
      fprintf(stderr, "dcc_occ_validate_snapshot: %s (%s)\n", dcc_strerror(e), dcc_last_error(ctx));
      failed = 1;
    } else {
      live_mismatch = (long long)bad;
      if (bad) failed = 3;
      if (s.n_commit != commits.load()) failed = 4;
    }
    epochs = 1;
    device_ms = s.device_ms;
  } else if (!c.calvin) {
    OccEpoch::Options o;
    o.max_txns = c.epoch_max;
    o.n_workers = c.threads;
    o.timer_ms = c.timer_ms;
    o.capture_dir = c.capture;
    o.overlap = c.overlap;
    o.depth = c.depth;
    OccEpoch occ(ctx, o);
    std::vector<std::thread> ws;
    for (int w = 0; w < c.threads; w++)
      ws.emplace_back([&, w] {
        std::vector<Access> acc;
        for (uint64_t i = 0; i < c.txns && !failed; i++) {
          acc.clear();
          for (uint32_t x = off[w][i]; x < off[w][i + 1]; x++) acc.push_back({keys[w][x], at[w][x]});
          for (int attempt = 0;; attempt++) {  // WorkerThread: restart on Abort
            uint8_t rc = DCC_RC_ABORT;
            if (occ.validate(acc.data(), acc.size(), &rc)) {
              failed = 1;
              break;
            }
            if (rc == DCC_RC_RCOK) {
              commits++;
              break;
            }
            restarts++;
            if (attempt >= c.max_retries) {
              failed = 2;
              break;
            }
          }
        }
        // a worker that leaves no longer counts toward "every worker waits"
        occ.leave();
      });
    for (auto& t : ws) t.join();
    const OccEpoch::Stats s = occ.stats();
    epochs = s.epochs;
    device_ms = s.device_ms;
  } else {
    // each worker is an origin node; an epoch is every worker's next chunk
    CalvinEpoch cal(ctx, c.capture);
    const uint64_t chunk = std::max<uint64_t>(1, c.epoch_max / (uint64_t)c.threads);
    for (uint64_t base = 0; base < c.txns && !failed; base += chunk) {
      std::vector<std::thread> ws;
      for (int w = 0; w < c.threads; w++)
        ws.emplace_back([&, w] {
          std::vector<Access> acc;
          for (uint64_t i = base; i < std::min(c.txns, base + chunk); i++) {
            acc.clear();
            for (uint32_t x = off[w][i]; x < off[w][i + 1]; x++)
              acc.push_back({keys[w][x], at[w][x]});
            cal.submit((uint32_t)w, acc.data(), acc.size());
          }
        });
      for (auto& t : ws) t.join();
      CalvinEpoch::Result r = cal.close();
      if (r.err) {
        fprintf(stderr, "dcc_calvin_order_epoch: %s\n", dcc_strerror(r.err));
        failed = 1;
        break;
      }
      if (r.capture_err) fprintf(stderr, "calvin capture: .dccb write failed\n");
      for (uint8_t x : r.rc) (x == DCC_RC_RCOK ? ready : waits)++;
      epochs++;
      device_ms += r.stats.device_ms;
    }
  }
  const double wall =
      std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
  const uint64_t total = c.txns * (uint64_t)c.threads;
  printf("{\"driver\": \"c1\", \"cc\": \"%s\", \"threads\": %d, \"txns\": %llu, "
         "\"epochs\": %llu, \"commits\": %llu, \"restarts\": %llu, \"ready\": %llu, "
         "\"waits\": %llu, \"device_ms\": %.3f, \"wall_s\": %.3f, \"txns_per_s\": %.1f, "
         "\"live_mismatch\": %lld, \"gave_up\": %llu, \"overlap\": %d, \"depth\": %d, \"failed\": %d}\n",
         c.calvin ? "CALVIN" : (c.live ? "OCC-live" : "OCC"), c.threads, (unsigned long long)total,
         (unsigned long long)epochs, (unsigned long long)commits.load(),
         (unsigned long long)restarts.load(), (unsigned long long)ready.load(),
         (unsigned long long)waits.load(), device_ms, wall, total / wall, live_mismatch,
         (unsigned long long)gave_up.load(), c.overlap ? 1 : 0, c.depth, failed.load());
  dcc_destroy(ctx);
  return failed ? 1 : 0;
}
