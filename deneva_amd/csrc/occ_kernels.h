// Kernel argument blocks shared by occ_kernels.hip and the host driver.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace dcc {

struct Slot;

constexpr int TILE_CAP = 1024;  // accesses staged per wave (LDS), build kernel
constexpr int ROUND_CAP = 512;  // accesses staged per wave, round / publish kernels
constexpr int TILE_WAVES = 4;   // waves per workgroup
constexpr int PUB_LDS = 2048;   // LDS owner-combiner slots per workgroup
constexpr int PUB_WAVES = 16;   // waves per workgroup of the build / publish kernels
constexpr uint32_t MAX_TXN_LEN = 64;  // MAX_ROW_PER_TXN (config.h:155)
constexpr uint32_t MAX_ROUND_TAG = 61;  // largest round tag a k_round may run with

// list-reservation counter: txns in the high bits, entries in the low bits
constexpr uint32_t CTR_E_BITS = 38;
constexpr unsigned long long CTR_E_MASK = (1ull << CTR_E_BITS) - 1ull;
constexpr uint32_t CTR_RING = 64;  // per-round counter sets kept on the device
constexpr uint32_t NSEG = 8;       // list segments (one reservation counter each)

// error bits reported by kernels
constexpr uint32_t ERR_OFFSETS = 1;
constexpr uint32_t ERR_TILE = 2;
constexpr uint32_t ERR_KEY = 4;
constexpr uint32_t ERR_FULL = 8;
constexpr uint32_t ERR_UNDECIDED = 16;
constexpr uint32_t ERR_SEG = 32;    // async solver: a key segment too long to sort in LDS
constexpr uint32_t ERR_ASYNC = 64;  // async solver: pass limit reached

constexpr unsigned PREP_BLOCKS = 512;
constexpr unsigned FINAL_BLOCKS = 512;
struct PrepPart {
  uint32_t err, maxlen, nw, nw_prefix;
};
struct FinalPart {
  uint32_t commit, abort, readonly, cwriters, undecided, pad0, pad1, pad2;
};

struct GridBar;
constexpr uint32_t RECHECK_TILES = 32;  // tiles a workgroup can recheck per round
struct TileOut {
  uint32_t og, bt, nt, be, ne;
};

struct HistArgs {
  uint64_t n;
  const uint32_t* off;
  const uint64_t* keys;
  const uint8_t* acctype;
  const uint64_t* start_tn;
  const uint64_t* finish_tn;
  const uint64_t* hkeys;
  uint64_t nkeys;
  const uint64_t* hoff;
  const uint64_t* htn;
  uint8_t* state;
};

struct BuildArgs {
  uint64_t n;
  uint32_t tw;
  const uint32_t* off;
  const uint64_t* keys;
  const uint8_t* acctype;
  Slot* tab;
  uint32_t mask;
  const uint8_t* state;
  uint8_t* hasw;
  uint32_t* err;
};

struct RoundArgs {
  const unsigned long long* m_in;  // previous round's NSEG counters (list size) or null
  uint64_t m;             // txns in the input list (when m_in is null)
  uint32_t tw;            // txns per wave
  uint32_t r;             // round tag (1..MAX_ROUND_TAG)
  uint32_t k;             // round index (0-based, never reset)
  uint32_t end_total;     // coff[m] (entries in the input list)
  const uint32_t* tid;    // list txn ids (nullptr: identity, round 1)
  const uint32_t* coff;   // list offsets
  const uint64_t* keys;   // round 1 input
  const uint8_t* acctype; // round 1 input
  const uint64_t* cent;   // rounds >= 2 input entries (see dcc_device.h)
  uint64_t seg_ts;        // segment stride of tid/coff arrays
  uint64_t seg_es;        // segment stride of entry arrays
  Slot* tab;
  uint32_t mask;
  uint8_t* state;
  uint32_t* tid_out;
  uint32_t* coff_out;
  uint64_t* cent_out;
  unsigned long long* ctr;       // this round's NSEG reservation counters
  unsigned long long* ctr_zero;  // next round's NSEG counters, zeroed here
  uint32_t* kill_flag;           // set when this round aborted a txn
  uint32_t* kill_zero;           // next round's flag, zeroed here
  GridBar* bar;                  // grid barrier words (recheck enabled) or null
  uint32_t* bar_zero;            // next round's barrier words, zeroed here
  uint8_t* gst;                  // sharded: per-txn local status out (1 blocked, 2 killed)
  uint32_t* err;
};

struct PubArgs {
  const unsigned long long* m_in;  // NSEG counters of the list
  uint32_t r;                      // round whose owner words are published
  uint32_t tw;
  const uint32_t* kill_flag;       // previous round's abort flag (always-one word to force)
  uint32_t force;                  // publish every write entry (after a retag)
  const uint8_t* state;
  const uint32_t* tid;
  const uint32_t* coff;
  const uint64_t* cent;
  uint64_t seg_ts, seg_es;
  Slot* tab;
  uint32_t* err;
};

struct FinalArgs {
  uint64_t n;
  const uint8_t* state;
  const uint8_t* hasw;
  uint8_t* rc;
  uint32_t* cflag;
  FinalPart* part;  // [FINAL_BLOCKS]
};

// ---- prefix peel (occ_peel.hip)
constexpr int FILTER_CAP = 1024;  // accesses staged per wave
constexpr int FILTER_WAVES = 8;
constexpr int FILTER_ILP = 16;  // all of a wave tile's accesses in flight at once
constexpr unsigned FILTER_MAX_GRID = 2048;  // per-block partials fit `part`

struct SurvPart {
  uint32_t t, a, w, pad;  // survivors: txns, accesses, writes (scanned: bases)
};

struct CsetArgs {
  uint64_t p;  // prefix length
  uint32_t tw;  // txns per wave tile
  const uint32_t* off;
  const uint64_t* keys;
  const uint8_t* acctype;
  const uint8_t* state;
  uint64_t* gset;  // exact set, capacity gmask + 1, pre-filled with KEY_EMPTY
  uint32_t gmask;
  uint64_t* ckeys;  // compact list of the set's keys
  uint32_t* ccount;
};

struct FilterArgs {
  uint64_t t0, n;    // kill candidates [t0, n); has-write bytes for [0, n)
  uint64_t per_blk;  // txns per block (block b: [b*per_blk, (b+1)*per_blk))
  uint32_t tw;       // txns per wave tile
  const uint32_t* off;
  const uint64_t* keys;
  const uint8_t* acctype;
  const uint64_t* ckeys;
  const uint32_t* ccount;
  const uint64_t* gset;
  uint32_t gmask;
  uint8_t* state;
  uint8_t* kill;  // sharded: local kill byte out (all-reduced MAX), else null
  uint8_t* hasw;
  SurvPart* part;  // [grid]
  uint32_t* err;
};

struct CompactArgs {
  uint64_t t0, n, per_blk;
  const uint32_t* off;
  const uint64_t* keys;
  const uint8_t* acctype;
  const uint8_t* state;
  const SurvPart* part;  // scanned bases per block
  uint32_t* sub_tid;
  uint32_t* sub_off;
  uint64_t* sub_keys;
  uint8_t* sub_acctype;
};

void launch_cset(const CsetArgs& a, hipStream_t st);
void launch_filter(const FilterArgs& a, unsigned grid, hipStream_t st);
void launch_survivors(const FilterArgs& a, unsigned grid, hipStream_t st);
void launch_surv_scan(SurvPart* part, uint32_t nb, uint32_t* tot, uint32_t* sub_off,
                      hipStream_t st);
void launch_compact(const CompactArgs& a, unsigned grid, hipStream_t st);
void launch_scatter(const uint8_t* sub_state, const uint32_t* sub_tid, const uint32_t* n_sub,
                    uint64_t m_bound, uint8_t* state, hipStream_t st);

// ---- asynchronous solver (occ_async.hip)
constexpr int ASYNC_CAP = 1024;   // accesses staged per wave (preprocessing)
constexpr int ASYNC_KCAP = 512;   // accesses staged per wave (k_async)
constexpr int ASYNC_WAVES = 8;
constexpr uint32_t ASORT_SMALL = 16;   // segments sorted by one thread
constexpr uint32_t ASORT_BIG = 32768;  // longest segment the LDS sort takes
constexpr uint32_t ASYNC_MAX_PASS = 1u << 20;

struct AsyncArgs {
  uint64_t m;   // txns of the (sub-)batch
  uint32_t tw;  // txns per wave chunk (k_async)
  uint32_t tw_pre;  // txns per wave tile (preprocessing)
  const uint32_t* off;
  const uint64_t* keys;
  const uint8_t* acctype;
  uint8_t* state;   // u8 decisions in (history aborts) / out
  uint32_t* st32;   // working state words (agent-scope atomics)
  Slot* tab;
  uint32_t mask;
  uint32_t* wcnt;     // [cap] writers per key
  uint32_t* wstart;   // [cap] segment start
  uint32_t* wfill;    // [cap] fill counters
  uint32_t* cursor;   // [cap] first writer not known aborted
  uint32_t* writers;  // segments of writer txn ids, sorted per key
  uint32_t* bump;
  uint32_t* big;      // keys with long segments
  uint32_t* nbig;
  unsigned long long* ticket;
  uint32_t* passes;
  uint32_t* err;
  uint8_t* hasw;  // has-write byte per txn out (may be null)
};
void launch_async(const AsyncArgs& a, uint64_t cap, unsigned n_cu, hipStream_t st);

// launchers (occ_kernels.hip)
void launch_prep(const uint32_t* off, uint64_t n, const uint8_t* at, uint64_t nnz, uint64_t p,
                 PrepPart* part, hipStream_t st);
void launch_hist(const HistArgs& a, hipStream_t st);
void launch_build(const BuildArgs& a, unsigned max_grid, hipStream_t st);
void launch_round(const RoundArgs& a, bool from_keys, uint64_t m_bound, unsigned max_grid,
                  hipStream_t st);
void launch_retag(Slot* tab, uint64_t cap, hipStream_t st);
void launch_pub(const PubArgs& a, uint64_t m_bound, unsigned max_grid, hipStream_t st);
void launch_final(const FinalArgs& a, hipStream_t st);
// sharded rounds: apply the all-reduced status (0 commit, 1 stay, >=2 abort),
// clear it for the next round, add the undecided count to *und.
void launch_decide(uint8_t* state, uint8_t* gst, uint64_t n, uint8_t abort_byte, uint32_t* und,
                   uint32_t* und_next, hipStream_t st);
void launch_commit_tn(const uint32_t* cflag, uint64_t n, uint64_t* bsum, uint64_t tnc,
                      uint64_t* tn, hipStream_t st);

}  // namespace dcc
