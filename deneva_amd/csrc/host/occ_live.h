// occ_live.h — a live, genuinely concurrent OptCC run on host threads, with
// the critical-section capture that dcc_occ_validate_snapshot replays on the
// GPU ("OCC: validating a captured live run").
//
// The host side stays the reference's own engine: worker threads take
// start_tn = get_ts() (worker_thread.cpp:500-502, TS_CAS: manager.cpp:41-70),
// enter central_validate's critical section (occ.cpp:137-158) — finish_tn,
// finish_active, his = history, push of the own write set — decide
// (occ.cpp:160-199), unlink on abort in a second critical section
// (occ.cpp:219-235), and on commit run central_finish (occ.cpp:248-294:
// tn = ++tnc, push on history).  Every validation appends one capture record:
// its accesses, start/finish tn, the history head's tn and the record indices
// of the active write sets it saw.  Header-only C++17 over dcc.h.
#pragma once
#include <algorithm>
#include <cstdint>
#include <mutex>
#include <vector>

#include "dcc.h"
#include "occ_epoch.h"  // dcc_host::Access

namespace dcc_host {

struct LiveCapture {
  std::vector<uint32_t> off{0};
  std::vector<uint64_t> keys;
  std::vector<uint8_t> acctype;
  std::vector<uint64_t> start_tn, finish_tn, hist_top;
  std::vector<uint32_t> active_off{0}, active_idx;
  std::vector<uint8_t> rc;                // the live decisions
  std::vector<uint64_t> hist_keys, hist_tn;  // committed write sets (central_finish)
  uint64_t n() const { return start_tn.size(); }
};

class LiveOcc {
 public:
  // Manager::get_ts under TS_CAS: a global counter, +1 per call
  uint64_t get_ts() {
    std::lock_guard<std::mutex> g(ts_mu_);
    return ++clock_;
  }

  // central_validate; returns the capture record index, *rc = RCOK / Abort
  uint32_t validate(const Access* a, size_t n, uint64_t start_tn, uint8_t* rc) {
    std::vector<uint64_t> r, w;
    for (size_t i = 0; i < n; i++) (a[i].type == DCC_WR ? w : r).push_back(a[i].key);
    bool valid = true;
    uint32_t rec;
    {
      std::lock_guard<std::mutex> g(mu_);  // sem_wait(&_semaphore), occ.cpp:136
      rec = (uint32_t)cap_.n();
      for (size_t i = 0; i < n; i++) {
        cap_.keys.push_back(a[i].key);
        cap_.acctype.push_back(a[i].type);
      }
      cap_.off.push_back((uint32_t)cap_.keys.size());
      const uint64_t finish_tn = get_ts();  // occ.cpp:142
      cap_.start_tn.push_back(start_tn);
      cap_.finish_tn.push_back(finish_tn);
      cap_.hist_top.push_back(history_.empty() ? 0 : history_.back().tn);
      for (const Ent& e : active_) cap_.active_idx.push_back(e.rec);  // finish_active
      cap_.active_off.push_back((uint32_t)cap_.active_idx.size());
      cap_.rc.push_back(DCC_RC_RCOK);
      // the checks read only this snapshot (decided here so that the
      // append-only history needs no second lock; the decision is the same)
      if (finish_tn > start_tn)  // occ.cpp:167-180, read set only
        for (auto h = history_.rbegin(); h != history_.rend() && valid; ++h) {
          if (h->tn > finish_tn) continue;
          if (h->tn <= start_tn) break;
          valid = !meets(h->w, r);
        }
      for (size_t q = 0; valid && q < active_.size(); q++)  // occ.cpp:185-199
        valid = !meets(active_[q].w, r) && !meets(active_[q].w, w);
      if (!w.empty()) active_.push_back(Ent{rec, w});  // STACK_PUSH(active, wset)
      if (!valid) cap_.rc[rec] = DCC_RC_ABORT;
    }
    // sem_post: others may now see this write set on the active list
    if (!valid && !w.empty()) unlink(rec);  // occ.cpp:219-235
    *rc = valid ? DCC_RC_RCOK : DCC_RC_ABORT;
    return rec;
  }

  // central_finish for a committed txn (occ.cpp:248-294)
  void finish_commit(uint32_t rec) {
    std::lock_guard<std::mutex> g(mu_);
    auto it = std::find_if(active_.begin(), active_.end(),
                           [&](const Ent& e) { return e.rec == rec; });
    if (it == active_.end()) return;  // read-only: never on the active list
    Hist h{++tnc_, it->w};
    for (uint64_t k : h.w) {
      cap_.hist_keys.push_back(k);
      cap_.hist_tn.push_back(h.tn);
    }
    history_.push_back(std::move(h));
    active_.erase(it);
  }

  LiveCapture take() {
    std::lock_guard<std::mutex> g(mu_);
    return std::move(cap_);
  }

 private:
  struct Ent {
    uint32_t rec;
    std::vector<uint64_t> w;
  };
  struct Hist {
    uint64_t tn;
    std::vector<uint64_t> w;
  };
  static bool meets(const std::vector<uint64_t>& a, const std::vector<uint64_t>& b) {
    for (uint64_t x : a)  // OptCC::test_valid, occ.cpp:319-327
      for (uint64_t y : b)
        if (x == y) return true;
    return false;
  }
  void unlink(uint32_t rec) {
    std::lock_guard<std::mutex> g(mu_);
    auto it = std::find_if(active_.begin(), active_.end(),
                           [&](const Ent& e) { return e.rec == rec; });
    if (it != active_.end()) active_.erase(it);
  }

  std::mutex mu_, ts_mu_;
  uint64_t clock_ = 0, tnc_ = 0;
  std::vector<Ent> active_;
  std::vector<Hist> history_;
  LiveCapture cap_;
};

// Replays a capture on the GPU; returns DCC_OK and the number of records
// whose GPU decision differs from the live one in *mismatch.
inline int validate_capture(dcc_ctx* ctx, const LiveCapture& c, uint64_t* mismatch,
                            dcc_stats* st) {
  int e = dcc_occ_history_clear(ctx);
  if (!e && !c.hist_keys.empty())
    e = dcc_occ_history_append(ctx, c.hist_keys.data(), c.hist_tn.data(), c.hist_keys.size());
  if (e) return e;
  dcc_batch b{};
  b.n_txn = c.n();
  b.nnz = c.keys.size();
  b.offsets = c.off.data();
  b.keys = c.keys.data();
  b.acctype = c.acctype.data();
  b.start_tn = c.start_tn.data();
  b.finish_tn = c.finish_tn.data();
  dcc_occ_snapshot s{c.hist_top.data(), c.active_off.data(), c.active_idx.data()};
  std::vector<uint8_t> rc(c.n() + 1);
  e = dcc_occ_validate_snapshot(ctx, &b, &s, rc.data(), st);
  if (e) return e;
  uint64_t bad = 0;
  for (uint64_t i = 0; i < c.n(); i++) bad += rc[i] != c.rc[i];
  *mismatch = bad;
  return DCC_OK;
}

}  // namespace dcc_host
