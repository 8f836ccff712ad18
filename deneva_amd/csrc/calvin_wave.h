// Calvin wave levels in one CU (calvin_wave.hip): the longest-path pass
// behind dcc_calvin_order_epoch's out_wave.
//
//   wave(t) = max over t's requests in a group g > 0 of 1 + M(row, g - 1),
//   M(row, g) = max wave over the members of the row's group g
// (oracle_calvin_formula, calvin_ref.c:196-257; row_lock.cpp:317-357 released
// in waves).  Every member of a row's group g - 1 precedes every member of
// group g in sequence order, so sequence order is a topological order and a
// single walk over it is exact.  The walk is a chain of ~50,000 dependent
// steps at C4 size; one cross-CU hand-off per step (the dataflow grid this
// replaces) costs ~2 us each, an LDS round trip ~0.1 us.  So the walk runs in
// one workgroup:
//
// * slots: txn at sequence position q, request j -> slot q * Lp + j (Lp = the
//   txn length rounded up to a power of two, at most 32); a group's maximum
//   lives at the slot of its sequence-last member (the sorted element before
//   the next group's start), so every request names two slots: its previous
//   group's (read) and its own group's (max-accumulated);
// * chunks of C sequence positions (H = C * Lp slots) walked in order by one
//   wave, 64 txns (a sub-chunk) at a time, one lane per txn: LDS holds the
//   group maxima of the current and the previous chunk; a sub-chunk iterates
//   (Jacobi, LDS only) until none of its lanes changes -- only when one of its
//   txns depends on another of the same sub-chunk;
// * the other 7 waves stage the next chunk meanwhile: each txn's bound from
//   groups that ended two or more chunks back (LDS or the global maxima), the
//   global maxima's share of the next chunk's slots, the outputs of the last
//   chunk, and the maxima of groups ending beyond the window (global atomics);
// * with helper workgroups (CwArgs::nh, the default: 16 more CUs) the
//   scattered part of that -- the global maxima of groups ending three or
//   more chunks ahead, and the bounds from groups that ended three or more
//   chunks back -- runs on the helpers a whole chunk ahead of its use, handed
//   over through global memory (sc1 stores and loads, counters), and the
//   two-chunk cases go through LDS; the walk no longer waits for the staging
//   (C4: 34.7 -> 18.1 ms).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace dcc {

constexpr uint32_t CW_HMAX = 16383;  // slots per chunk (two chunks: 15-bit LDS slot)
constexpr uint32_t CW_CMAX = 1024;   // txns per chunk
constexpr uint32_t CW_LMAX = 32;     // slots per txn

struct CwPlan {
  uint32_t lg;   // log2 Lp
  uint32_t C;    // txns per chunk (multiple of 64)
  uint32_t H;    // slots per chunk = C << lg
  uint32_t nch;  // chunks
  uint64_t slots;  // nch * H
};

// false when the txns are longer than CW_LMAX (the dataflow grid takes them)
bool cw_plan(uint64_t n, uint32_t maxlen, CwPlan* p);

struct CwArgs {
  uint64_t n;
  const uint32_t* seq;    // sequence position -> txn, or null (index order)
  const uint32_t* off;    // index-order offsets (ragged), or null
  uint32_t ulen;          // uniform length, or 0
  const uint32_t* gsx;    // [nnz] own group start | has-previous-group << 31, or ~0 (dup)
  const uint32_t* glast;  // [m] by group start: sorted position of the group's last element, or ~0
  const uint32_t* sv;     // [m] sorted values (txn << 7 | j << 1 | EX)
  // workspaces: seqpos [n] (only with seq), rec16 / recp / reco / mg [slots]
  uint32_t* seqpos;
  uint32_t* rec16;
  uint32_t* recp;
  uint32_t* reco;
  uint32_t* mg;
  uint8_t* mark;   // [slots] the slot is read by a request of its own sub-chunk
  uint32_t* pa;    // [slots] walker: LDS byte address read for the previous group
  uint32_t* oa;    // [slots] walker: LDS byte address the own group's max goes to
  uint32_t* cr;    // [nch * C * 8] walker: per txn its intra reads / hot publications
  uint32_t* wave;  // [n] out
  uint32_t* err;   // ERR word (bit: helper spin limit)
  uint64_t* dbg;   // experiments builds: walker timing counters (or null)
  uint32_t* help;  // [cw_help_words] helper hand-offs (nh > 0)
  uint32_t* rec2;  // [slots] (nh > 0) LDS slots of groups ending two chunks back / ahead
  uint32_t nh;     // helper workgroups (0: the walker's workgroup alone)
};

// words of CwArgs::help for a plan
__host__ __device__ inline uint64_t cw_help_words(const CwPlan& p) { return 64 + 2ull * p.nch * p.C; }

constexpr uint32_t CW_ERR_SPIN = 1u << 9;

hipError_t cw_run(const CwPlan& p, const CwArgs& a, hipStream_t st);

}  // namespace dcc
