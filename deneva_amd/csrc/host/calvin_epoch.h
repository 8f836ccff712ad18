// calvin_epoch.h — host-side Calvin sequencer hand-off over libdcc
// (SURVEY.md §8(b) (ii)).
//
// The reference's sequencer numbers txns per origin node (txn_id = node +
// node_cnt * next_txn_id, system/sequencer.cpp:207), closes an epoch every
// SEQ_BATCH_TIMER (sequencer.cpp:283-326) and the lock thread dequeues it in
// (epoch, origin, FIFO) order (work_queue.cpp:105-151) calling acquire_locks
// one txn at a time (calvin_thread.cpp:40-100).  CalvinEpoch collects the
// epoch the same way -- submit(origin, accesses) appends to the origin's FIFO
// -- and close() decides the whole epoch with dcc_calvin_order_epoch: per txn
// RCOK (runnable at acquire) or WAIT, and the wave at which it runs when
// every txn releases its locks one wave after it became ready.
#pragma once

#include <cstdint>
#include <cstdio>
#include <mutex>
#include <string>
#include <vector>

#include "dcc.h"
#include "occ_epoch.h"

namespace dcc_host {

class CalvinEpoch {
 public:
  struct Result {
    std::vector<uint32_t> origin, seq;  // per txn of the epoch, submission order
    std::vector<uint8_t> rc;            // DCC_RC_RCOK / DCC_RC_WAIT
    std::vector<uint32_t> wave;
    std::vector<uint32_t> group;        // grant group per request (capture only)
    dcc_stats stats{};
    int err = 0;
    bool capture_err = false;           // the .dccb write failed (decisions unaffected)
  };

  // capture_dir: every closed epoch is written as a .dccb file (batch in
  // submission order with the sequencer order, grant groups, readiness and
  // wave levels) for offline parity checks against the Row_lock replay
  explicit CalvinEpoch(dcc_ctx* ctx, std::string capture_dir = "")
      : ctx_(ctx), capture_(std::move(capture_dir)) {
    off_.push_back(0);
  }

  // Sequencer::process_txn: the txn joins its origin's FIFO for this epoch.
  void submit(uint32_t origin, const Access* acc, size_t n) {
    std::lock_guard<std::mutex> lk(mu_);
    if (origin >= next_seq_.size()) next_seq_.resize(origin + 1, 0);
    origin_.push_back(origin);
    seq_.push_back(next_seq_[origin]++);
    for (size_t i = 0; i < n; i++) {
      keys_.push_back(acc[i].key);
      at_.push_back(acc[i].type);
    }
    off_.push_back((uint32_t)keys_.size());
  }

  // Sequencer::send_next_batch + the lock thread's walk over the epoch.
  Result close() {
    std::lock_guard<std::mutex> lk(mu_);
    Result r;
    const uint64_t n = off_.size() - 1;
    std::vector<uint64_t> order(n);
    for (uint64_t i = 0; i < n; i++) order[i] = ((uint64_t)origin_[i] << 32) | seq_[i];
    r.rc.assign(n, DCC_RC_WAIT);
    r.wave.assign(n, 0);
    dcc_batch b{};
    b.n_txn = n;
    b.nnz = keys_.size();
    b.offsets = off_.data();
    b.keys = keys_.data();
    b.acctype = at_.data();
    b.order = order.data();
    const bool cap = !capture_.empty();
    if (cap) r.group.assign(b.nnz ? b.nnz : 1, 0);
    if (n)
      r.err = dcc_calvin_order_epoch(ctx_, &b, cap ? r.group.data() : nullptr, r.rc.data(), r.wave.data(),
                                     &r.stats);
    if (n && cap && !r.err) {
      dcc_file_info fi{};
      fi.kind = DCC_FILE_CALVIN;
      fi.epoch = epoch_;
      char path[4096];
      snprintf(path, sizeof path, "%s/calvin_%06llu.dccb", capture_.c_str(), (unsigned long long)epoch_);
      r.capture_err =
          dcc_file_write(path, &fi, &b, r.rc.data(), nullptr, r.group.data(), r.wave.data()) != DCC_OK;
    }
    epoch_++;
    r.origin.swap(origin_);
    r.seq.swap(seq_);
    off_.assign(1, 0);
    keys_.clear();
    at_.clear();
    next_seq_.assign(next_seq_.size(), 0);  // per-epoch numbering (sequencer.cpp:325)
    return r;
  }

 private:
  dcc_ctx* ctx_;
  std::string capture_;
  uint64_t epoch_ = 0;
  std::mutex mu_;
  std::vector<uint32_t> off_, origin_, seq_, next_seq_;
  std::vector<uint64_t> keys_;
  std::vector<uint8_t> at_;
};

}  // namespace dcc_host
