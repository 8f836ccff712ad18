// occ_epoch.h — host-side OCC plugin shim over libdcc.
//
// Mirrors the reference's validation surface for the OCC branch: every worker
// thread calls validate() the way it calls TxnManager::validate()
// (system/txn.cpp:935) -> OptCC::validate (concurrency_control/occ.cpp:42),
// with the access set its execution captured (Access list, system/txn.h:39-70)
// and gets RCOK or Abort (system/global.h:236).  Instead of validating one
// txn at a time against the active/history lists, the shim appends the txn to
// the open epoch and blocks until the epoch is decided on the GPU by
// dcc_occ_validate_epoch, whose decisions equal central_validate in epoch
// (index) order followed by central_finish (occ.cpp:116-294).
//
// An epoch closes when it holds max_txns txns, when every registered worker is
// waiting in validate() (nobody else can add to it), or when the oldest waiter
// has waited timer_ms.  Decided epochs can be captured as .dccb files
// (dcc_file_write) with their decisions, for offline parity checks.
//
// Capture and validation overlap: the closing thread swaps the open epoch's
// CSR into the in-flight buffer and releases the mutex for the engine call,
// so workers fill epoch N+1 while epoch N is on the GPU.  Engine calls stay
// serialized (one in flight; the context is thread-compatible), and an epoch
// closes only when the previous one is decided, which keeps tnc and the
// history in epoch order.  Options::overlap = false holds the mutex across
// the call (the pre-overlap behaviour, kept for A/B measurement).
//
// Timestamps: with the reference's default TS_CLOCK (config.h:124) the history
// window of central_validate never fires, so by
// default the shim passes no start/finish timestamps and keeps no history (the
// reference's history would only grow).  With
// Options::ts_window (TS_CAS-style timestamps) every validate() passes the
// txn's start_tn / finish_tn (occ.cpp:142) and committed write sets join the
// context's history (central_finish, occ.cpp:277-286), so later epochs'
// windows see them.  The class is thread-safe; the dcc_ctx it
// drives must not be used by anyone else meanwhile (a context is
// thread-compatible, dcc.h).
#pragma once

#include <chrono>
#include <condition_variable>
#include <cstdint>
#include <cstdio>
#include <map>
#include <mutex>
#include <string>
#include <vector>

#include "dcc.h"

namespace dcc_host {

struct Access {   // one entry of a txn's access list
  uint64_t key;   // canonical row key
  uint8_t type;   // access_t: DCC_RD / DCC_WR / DCC_XP / DCC_SCAN
};

class OccEpoch {
 public:
  struct Options {
    uint64_t max_txns = 65536;   // epoch size cap
    int n_workers = 1;           // threads that call validate()
    double timer_ms = 5.0;       // SEQ_BATCH_TIMER-like close timer (config.h:348)
    std::string capture_dir;     // "" = no capture
    bool ts_window = false;      // pass start/finish tn and keep the history
    bool overlap = true;         // fill epoch N+1 while epoch N is decided
  };
  struct Stats {
    uint64_t epochs = 0, txns = 0, commits = 0, aborts = 0;
    uint64_t capture_errors = 0;  // .dccb writes that failed (decisions unaffected)
    double device_ms = 0, wall_ms = 0;
  };

  OccEpoch(dcc_ctx* ctx, const Options& o) : ctx_(ctx), opt_(o) { open_.off.push_back(0); }

  // TxnManager::validate for CC_ALG == OCC: DCC_RC_RCOK or DCC_RC_ABORT in *rc.
  // start_tn / finish_tn are read only with Options::ts_window.
  // Returns a dcc error code (0 = ok).
  int validate(const Access* acc, size_t n, uint8_t* rc, uint64_t start_tn = 0,
               uint64_t finish_tn = 0) {
    std::unique_lock<std::mutex> lk(mu_);
    const uint64_t ep = epoch_;
    const uint64_t slot = open_.off.size() - 1;
    for (size_t i = 0; i < n; i++) {
      open_.keys.push_back(acc[i].key);
      open_.at.push_back(acc[i].type);
    }
    open_.off.push_back((uint32_t)open_.keys.size());
    if (opt_.ts_window) {
      open_.start.push_back(start_tn);
      open_.finish.push_back(finish_tn);
    }
    if (slot == 0) opened_ = std::chrono::steady_clock::now();
    // waiting for the OPEN epoch: a worker blocked on the in-flight one will
    // add its next txn to the open epoch once that one is decided, so it does
    // not count towards "every worker is in" (the open epoch would otherwise
    // close early, right after the in-flight call returns and before its
    // waiters have woken)
    open_waiting_++;
    int err = 0;
    while (decided_.find(ep) == decided_.end()) {
      const bool full = open_.off.size() - 1 >= opt_.max_txns;
      const bool all_in = open_waiting_ >= opt_.n_workers;
      const auto age = std::chrono::duration<double, std::milli>(
                           std::chrono::steady_clock::now() - opened_).count();
      if (ep == epoch_ && !busy_ && (full || all_in || age >= opt_.timer_ms)) {
        err = close(lk);
        continue;  // decided (or failed) now
      }
      // a system_clock deadline (pthread_cond_timedwait: the wait ThreadSanitizer
      // intercepts; a 200 us poll does not care about clock steps)
      cv_.wait_until(lk, std::chrono::system_clock::now() + std::chrono::microseconds(200));
    }
    auto it = decided_.find(ep);
    if (it == decided_.end()) return err ? err : DCC_EIO;
    if (it->second.err) err = it->second.err;
    *rc = err ? (uint8_t)DCC_RC_ABORT : it->second.rc[slot];
    if (--it->second.readers == 0) decided_.erase(it);
    return err;
  }

  // a worker that stops calling validate() (end of its run): the epoch no
  // longer waits for it
  void leave() {
    std::lock_guard<std::mutex> lk(mu_);
    opt_.n_workers--;
    cv_.notify_all();
  }

  Stats stats() {
    std::lock_guard<std::mutex> lk(mu_);
    return stats_;
  }

 private:
  struct Decided {
    std::vector<uint8_t> rc;
    uint64_t readers = 0;
    int err = 0;
  };

  struct Csr {  // an epoch's access sets
    std::vector<uint32_t> off;
    std::vector<uint64_t> keys;
    std::vector<uint8_t> at;
    std::vector<uint64_t> start, finish;
  };

  // decide the open epoch: it moves to the in-flight buffer, the mutex is
  // released for the engine call (Options::overlap), then everyone wakes.
  // Called with lk held and no call in flight; returns with lk held.
  int close(std::unique_lock<std::mutex>& lk) {
    std::swap(open_, fly_);
    open_.off.assign(1, 0);
    open_.keys.clear();
    open_.at.clear();
    open_.start.clear();
    open_.finish.clear();
    const uint64_t id = epoch_++;
    open_waiting_ = 0;  // they wait for the closed epoch now
    busy_ = true;
    if (opt_.overlap) lk.unlock();
    const uint64_t n = fly_.off.size() - 1;
    Decided d;
    d.rc.assign(n, DCC_RC_ABORT);
    d.readers = n;
    dcc_batch b{};
    b.n_txn = n;
    b.nnz = fly_.keys.size();
    b.offsets = fly_.off.data();
    b.keys = fly_.keys.data();
    b.acctype = fly_.at.data();
    if (opt_.ts_window) {
      b.start_tn = fly_.start.data();
      b.finish_tn = fly_.finish.data();
      b.flags = DCC_OCC_APPEND_HISTORY;  // central_finish: commit tn + history
    }
    dcc_stats st{};
    const uint64_t tnc0 = dcc_occ_get_tnc(ctx_);
    const auto t0 = std::chrono::steady_clock::now();
    d.err = n ? dcc_occ_validate_epoch(ctx_, &b, d.rc.data(), nullptr, &st) : 0;
    const auto t1 = std::chrono::steady_clock::now();
    bool cap_err = false;
    if (!d.err && !opt_.capture_dir.empty()) {
      dcc_file_info fi{};
      fi.kind = DCC_FILE_OCC;
      fi.epoch = id;
      fi.tnc_before = tnc0;
      char path[4096];
      snprintf(path, sizeof path, "%s/epoch_%06llu.dccb", opt_.capture_dir.c_str(),
               (unsigned long long)id);
      // the epoch is decided (tnc and history advanced): a failed capture is
      // counted, never turned into aborts
      cap_err = dcc_file_write(path, &fi, &b, d.rc.data(), nullptr, nullptr, nullptr) != DCC_OK;
    }
    if (opt_.overlap) lk.lock();
    busy_ = false;
    stats_.capture_errors += cap_err ? 1 : 0;
    stats_.epochs++;
    stats_.txns += n;
    for (uint8_t r : d.rc) (r == DCC_RC_RCOK ? stats_.commits : stats_.aborts)++;
    stats_.device_ms += st.device_ms;
    stats_.wall_ms += std::chrono::duration<double, std::milli>(t1 - t0).count();
    const int err = d.err;
    decided_.emplace(id, std::move(d));
    cv_.notify_all();
    return err;
  }

  dcc_ctx* ctx_;
  Options opt_;
  std::mutex mu_;
  std::condition_variable cv_;
  Csr open_, fly_;     // the epoch workers fill; the one on the GPU
  bool busy_ = false;  // an engine call is in flight
  std::chrono::steady_clock::time_point opened_{};
  uint64_t epoch_ = 0;
  int open_waiting_ = 0;  // workers in validate() for the open epoch
  std::map<uint64_t, Decided> decided_;
  Stats stats_;
};

}  // namespace dcc_host
