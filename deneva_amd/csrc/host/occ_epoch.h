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
// Epochs in flight (Options::depth, default 4): a closed epoch is submitted
// to the engine's pipeline (dcc_occ_submit_epoch: its own lane, stream and
// captured graph) and the workers fill the next one at once; up to `depth`
// closed epochs are on the GPU together.  They complete in close order
// (dcc_occ_wait_epoch), driven by one of the threads waiting on the oldest,
// so decisions, tnc and the history are those of validating the epochs one
// after another (occ.cpp:116-294).  Engine calls are serialised by their own
// mutex (the context is thread-compatible), never under the shim's state
// mutex.  Counting "every worker is waiting" takes the workers blocked on
// closed epochs into account: an epoch closes when every worker is either in
// it or waiting on an epoch already closed.  depth = 1 is one epoch in flight
// (the round-4 shim); Options::overlap = false additionally holds the state
// mutex across the engine calls (the pre-overlap behaviour, for A/B).
// An epoch that needs shared state in order (the TS_CAS history below) runs
// synchronously inside dcc_occ_submit_epoch: the pipeline drains first.
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
#include <cstdlib>
#include <cstring>
#include <algorithm>
#include <deque>
#include <map>
#include <memory>
#include <mutex>
#include <new>
#include <string>
#include <utility>
#include <vector>

#include "dcc.h"

namespace dcc_host {

struct Access {   // one entry of a txn's access list
  uint64_t key;   // canonical row key
  uint8_t type;   // access_t: DCC_RD / DCC_WR / DCC_XP / DCC_SCAN
};

// A growable array in pinned host memory (dcc_host_alloc): the epoch's CSR is
// built in place, so the engine's H2D copy runs at DMA speed with no staging
// copy.  Falls back to ordinary memory if pinning fails (slower copy, same
// result).
template <class T>
class PinnedVec {
 public:
  explicit PinnedVec(dcc_ctx* ctx = nullptr) : ctx_(ctx) {}
  ~PinnedVec() { release(); }
  PinnedVec(const PinnedVec&) = delete;
  PinnedVec& operator=(const PinnedVec&) = delete;
  PinnedVec(PinnedVec&& o) noexcept { take(o); }
  PinnedVec& operator=(PinnedVec&& o) noexcept {
    if (this != &o) {
      release();
      take(o);
    }
    return *this;
  }
  void push_back(T v) {
    if (n_ == cap_) grow(n_ ? 2 * n_ : 4096);
    p_[n_++] = v;
  }
  void resize(size_t n) {
    if (n > cap_) grow(n);
    n_ = n;
  }
  void clear() { n_ = 0; }
  size_t size() const { return n_; }
  T* data() { return p_; }
  const T* data() const { return p_; }
  T& operator[](size_t i) { return p_[i]; }
  const T& operator[](size_t i) const { return p_[i]; }
  T& back() { return p_[n_ - 1]; }

 private:
  void grow(size_t cap) {
    void* q = nullptr;
    bool pinned = ctx_ && dcc_host_alloc(ctx_, cap * sizeof(T), &q) == DCC_OK && q;
    if (!pinned) {
      q = std::malloc(cap * sizeof(T));
      if (!q) throw std::bad_alloc();
    }
    if (n_) std::memcpy(q, p_, n_ * sizeof(T));
    release();
    p_ = (T*)q;
    cap_ = cap;
    pinned_ = pinned;
  }
  void release() {
    if (p_) {
      if (pinned_) (void)dcc_host_free(ctx_, p_);
      else std::free(p_);
    }
    p_ = nullptr;
    cap_ = 0;
  }
  void take(PinnedVec& o) {
    ctx_ = o.ctx_;
    p_ = o.p_;
    n_ = o.n_;
    cap_ = o.cap_;
    pinned_ = o.pinned_;
    o.p_ = nullptr;
    o.n_ = o.cap_ = 0;
  }
  dcc_ctx* ctx_ = nullptr;
  T* p_ = nullptr;
  size_t n_ = 0, cap_ = 0;
  bool pinned_ = false;
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
    int depth = 4;               // closed epochs on the GPU at once (engine pipeline lanes)
  };
  struct Stats {
    uint64_t epochs = 0, txns = 0, commits = 0, aborts = 0;
    uint64_t capture_errors = 0;  // .dccb writes that failed (decisions unaffected)
    double device_ms = 0, wall_ms = 0;
  };

  OccEpoch(dcc_ctx* ctx, const Options& o)
      : ctx_(ctx), opt_(o), depth_((size_t)std::max(1, o.overlap ? o.depth : 1)), open_(new Csr(ctx)) {
    open_->clear();  // offsets start at 0
    tnc_done_ = dcc_occ_get_tnc(ctx);
    // one engine lane per epoch in flight (DCC_OPT_PIPELINE, 1..8)
    if (depth_ > 1) (void)dcc_set_option(ctx, DCC_OPT_PIPELINE, (int64_t)std::min<size_t>(depth_, 8));
  }

  // TxnManager::validate for CC_ALG == OCC: DCC_RC_RCOK or DCC_RC_ABORT in *rc.
  // start_tn / finish_tn are read only with Options::ts_window.
  // Returns a dcc error code (0 = ok).
  int validate(const Access* acc, size_t n, uint8_t* rc, uint64_t start_tn = 0,
               uint64_t finish_tn = 0) {
    std::unique_lock<std::mutex> lk(mu_);
    const uint64_t ep = epoch_;
    const uint64_t slot = open_->off.size() - 1;
    for (size_t i = 0; i < n; i++) open_->add(acc[i].key, acc[i].type);
    open_->off.push_back((uint32_t)open_->nnz);
    if (opt_.ts_window) open_->add_tn(start_tn, finish_tn);
    if (slot == 0) opened_ = std::chrono::steady_clock::now();
    // waiting for the OPEN epoch; once it closes, its waiters count as
    // waiting on a closed epoch (closed_waiting_) until it is decided
    open_waiting_++;
    int err = 0;
    while (decided_.find(ep) == decided_.end()) {
      const size_t open_n = open_->off.size() - 1;
      const bool full = open_n >= opt_.max_txns;
      const bool all_in = open_waiting_ + closed_waiting_ >= opt_.n_workers;
      const auto age = std::chrono::duration<double, std::milli>(
                           std::chrono::steady_clock::now() - opened_).count();
      if (ep == epoch_ && open_n > 0 && !submitting_ && fly_.size() < depth_ &&
          (full || all_in || age >= opt_.timer_ms)) {
        err = submit(lk);
        continue;
      }
      // complete the oldest closed epoch: this thread's own, an earlier one,
      // or one that holds the slot the open epoch needs
      if (!driving_ && !fly_.empty() && fly_.front().submitted &&
          (ep < epoch_ || fly_.size() >= depth_)) {
        err = drive(lk);
        continue;
      }
      // a system_clock deadline (pthread_cond_timedwait: the wait ThreadSanitizer
      // intercepts; a 200 us poll does not care about clock steps)
      cv_.wait_until(lk, std::chrono::system_clock::now() + std::chrono::microseconds(200));
    }
    auto it = decided_.find(ep);
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

  // An epoch's access sets in pinned memory and in the engine's compact
  // transfer form (dcc.h): u32 keys while every key fits (widened in place on
  // the first one that does not), 2-bit access types four per byte, u32
  // timestamps while they fit -- a third of the full-width PCIe bytes for YCSB.
  struct Csr {
    explicit Csr(dcc_ctx* c)
        : off(c), k32(c), k64(c), at2(c), s32(c), f32(c), s64(c), f64(c) {}
    PinnedVec<uint32_t> off;
    PinnedVec<uint32_t> k32;
    PinnedVec<uint64_t> k64;
    PinnedVec<uint8_t> at2;
    PinnedVec<uint32_t> s32, f32;
    PinnedVec<uint64_t> s64, f64;
    uint64_t nnz = 0, ntn = 0;
    bool wide = false, tn_wide = false;

    void add(uint64_t key, uint8_t type) {
      if (!wide && (key >> 32)) {
        k64.resize(k32.size());
        for (size_t i = 0; i < k32.size(); i++) k64[i] = k32[i];
        wide = true;
      }
      if (wide) k64.push_back(key);
      else k32.push_back((uint32_t)key);
      if ((nnz & 3) == 0) at2.push_back(0);
      at2.back() = (uint8_t)(at2.back() | ((type & 3u) << (2 * (nnz & 3))));
      nnz++;
    }
    void add_tn(uint64_t s, uint64_t f) {
      if (!tn_wide && ((s | f) >> 32)) {
        s64.resize(s32.size());
        f64.resize(f32.size());
        for (size_t i = 0; i < s32.size(); i++) {
          s64[i] = s32[i];
          f64[i] = f32[i];
        }
        tn_wide = true;
      }
      if (tn_wide) {
        s64.push_back(s);
        f64.push_back(f);
      } else {
        s32.push_back((uint32_t)s);
        f32.push_back((uint32_t)f);
      }
      ntn++;
    }
    void clear() {
      off.clear();
      off.push_back(0);
      k32.clear();
      k64.clear();
      at2.clear();
      s32.clear();
      f32.clear();
      s64.clear();
      f64.clear();
      nnz = ntn = 0;
      wide = tn_wide = false;
    }
    void to_batch(dcc_batch& b) const {
      b.n_txn = off.size() - 1;
      b.nnz = nnz;
      b.offsets = off.data();
      b.keys = wide ? k64.data() : (const uint64_t*)(const void*)k32.data();
      b.acctype = at2.data();
      b.flags |= DCC_ACCTYPE_2BIT | (wide ? 0u : DCC_KEYS_U32);
      if (ntn) {
        b.start_tn = tn_wide ? s64.data() : (const uint64_t*)(const void*)s32.data();
        b.finish_tn = tn_wide ? f64.data() : (const uint64_t*)(const void*)f32.data();
        b.flags |= tn_wide ? 0u : DCC_TN_U32;
      }
    }
    // full-width copies for a .dccb capture (the file holds the engine's
    // canonical layout)
    void full(std::vector<uint64_t>& keys, std::vector<uint8_t>& at, std::vector<uint64_t>& st,
              std::vector<uint64_t>& ft) const {
      keys.resize(nnz);
      at.resize(nnz);
      for (uint64_t x = 0; x < nnz; x++) {
        keys[x] = wide ? k64[x] : k32[x];
        at[x] = (uint8_t)((at2[x >> 2] >> (2 * (x & 3))) & 3u);
      }
      st.resize(ntn);
      ft.resize(ntn);
      for (uint64_t t = 0; t < ntn; t++) {
        st[t] = tn_wide ? s64[t] : s32[t];
        ft[t] = tn_wide ? f64[t] : f32[t];
      }
    }
  };

  // A closed epoch on its way through the engine: its CSR and decision
  // buffers (pinned; they stay untouched until it completes) and ticket.
  struct Flight {
    uint64_t id = 0, ticket = 0, n = 0;
    std::unique_ptr<Csr> csr;
    std::unique_ptr<PinnedVec<uint8_t>> rc;
    dcc_batch b{};
    bool submitted = false;
    int err = 0;
    std::chrono::steady_clock::time_point t0{};
  };

  std::unique_ptr<Csr> take_csr() {
    std::unique_ptr<Csr> c;
    if (free_csr_.empty()) {
      c.reset(new Csr(ctx_));
    } else {
      c = std::move(free_csr_.back());
      free_csr_.pop_back();
    }
    c->clear();  // offsets start at 0
    return c;
  }

  // Close the open epoch and submit it.  Called with lk held, the open epoch
  // non-empty and a slot free; returns with lk held.
  int submit(std::unique_lock<std::mutex>& lk) {
    fly_.emplace_back();
    Flight& f = fly_.back();  // deque: stays put while others append
    f.csr = std::move(open_);
    open_ = take_csr();
    f.id = epoch_++;
    f.n = f.csr->off.size() - 1;
    closed_waiting_ += open_waiting_;  // they wait for the closed epoch now (one per txn)
    open_waiting_ = 0;
    if (!free_rc_.empty()) {
      f.rc = std::move(free_rc_.back());
      free_rc_.pop_back();
    } else {
      f.rc.reset(new PinnedVec<uint8_t>(ctx_));
    }
    f.rc->resize(f.n);
    if (opt_.ts_window) f.b.flags = DCC_OCC_APPEND_HISTORY;  // central_finish: commit tn + history
    f.csr->to_batch(f.b);
    submitting_ = true;
    if (opt_.overlap) lk.unlock();
    uint64_t ticket = 0;
    int e;
    {
      std::lock_guard<std::mutex> eg(eng_mu_);
      f.t0 = std::chrono::steady_clock::now();
      e = dcc_occ_submit_epoch(ctx_, &f.b, f.rc->data(), nullptr, &ticket);
    }
    if (opt_.overlap) lk.lock();
    f.ticket = ticket;
    f.err = e;
    f.submitted = true;
    submitting_ = false;
    cv_.notify_all();
    return 0;
  }

  // Complete the oldest closed epoch (dcc_occ_wait_epoch), capture it, and
  // hand its decisions to its waiters.  Called with lk held; returns with it.
  int drive(std::unique_lock<std::mutex>& lk) {
    driving_ = true;
    Flight& f = fly_.front();  // only the driver removes entries
    if (opt_.overlap) lk.unlock();
    dcc_stats st{};
    int err = f.err;
    if (!err) {
      std::lock_guard<std::mutex> eg(eng_mu_);
      err = dcc_occ_wait_epoch(ctx_, f.ticket, &st);
    }
    const auto t1 = std::chrono::steady_clock::now();
    // tnc before this epoch: the epochs complete in close order, each
    // advancing tnc by its committed writers (occ.cpp:283-284)
    const uint64_t tnc0 = tnc_done_;
    uint64_t n_cw = 0;
    if (!err) {
      const Csr& c = *f.csr;
      for (uint64_t t = 0; t < f.n; t++) {
        if ((*f.rc)[t] != DCC_RC_RCOK) continue;
        for (uint64_t x = c.off[t]; x < c.off[t + 1]; x++)
          if (((c.at2[x >> 2] >> (2 * (x & 3))) & 3u) == DCC_WR) {
            n_cw++;
            break;
          }
      }
      tnc_done_ += n_cw;
    }
    bool cap_err = false;
    if (!err && !opt_.capture_dir.empty()) {
      dcc_file_info fi{};
      fi.kind = DCC_FILE_OCC;
      fi.epoch = f.id;
      fi.tnc_before = tnc0;
      char path[4096];
      snprintf(path, sizeof path, "%s/epoch_%06llu.dccb", opt_.capture_dir.c_str(),
               (unsigned long long)f.id);
      // the epoch is decided (tnc and history advanced): a failed capture is
      // counted, never turned into aborts
      std::vector<uint64_t> fk, fs, ff;
      std::vector<uint8_t> fa;
      f.csr->full(fk, fa, fs, ff);
      dcc_batch fb = f.b;
      fb.flags &= ~DCC_COMPACT_FLAGS;
      fb.keys = fk.data();
      fb.acctype = fa.data();
      if (f.csr->ntn) {
        fb.start_tn = fs.data();
        fb.finish_tn = ff.data();
      }
      cap_err = dcc_file_write(path, &fi, &fb, f.rc->data(), nullptr, nullptr, nullptr) != DCC_OK;
    }
    if (opt_.overlap) lk.lock();
    Decided d;
    d.rc.assign(f.rc->data(), f.rc->data() + f.n);
    if (err) std::fill(d.rc.begin(), d.rc.end(), (uint8_t)DCC_RC_ABORT);
    d.readers = f.n;
    d.err = err;
    closed_waiting_ -= (int)f.n;
    stats_.capture_errors += cap_err ? 1 : 0;
    stats_.epochs++;
    stats_.txns += f.n;
    for (uint8_t r : d.rc) (r == DCC_RC_RCOK ? stats_.commits : stats_.aborts)++;
    stats_.device_ms += st.device_ms;
    stats_.wall_ms += std::chrono::duration<double, std::milli>(t1 - f.t0).count();
    decided_.emplace(f.id, std::move(d));
    free_csr_.push_back(std::move(f.csr));
    free_rc_.push_back(std::move(f.rc));
    fly_.pop_front();
    driving_ = false;
    cv_.notify_all();
    return err;
  }

  dcc_ctx* ctx_;
  Options opt_;
  size_t depth_ = 1;
  std::mutex mu_;      // the shim's state
  std::mutex eng_mu_;  // engine calls (the context is thread-compatible)
  std::condition_variable cv_;
  std::unique_ptr<Csr> open_;  // the epoch the workers fill
  std::deque<Flight> fly_;     // closed epochs in close order
  std::vector<std::unique_ptr<Csr>> free_csr_;
  std::vector<std::unique_ptr<PinnedVec<uint8_t>>> free_rc_;
  bool submitting_ = false, driving_ = false;
  std::chrono::steady_clock::time_point opened_{};
  uint64_t epoch_ = 0;
  int open_waiting_ = 0;    // workers in validate() for the open epoch
  int closed_waiting_ = 0;  // workers in validate() for closed, undecided epochs
  uint64_t tnc_done_ = 0;   // commit counter after the last completed epoch
  std::map<uint64_t, Decided> decided_;
  Stats stats_;
};

}  // namespace dcc_host
