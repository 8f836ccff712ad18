// Kernel argument blocks shared by occ_kernels.hip and the host driver.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <string>
#include "occ_history.h"

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
constexpr uint32_t ERR_SPIN = 128;  // sweep filter: look-back spin limit reached
// the level-0 validation pass found malformed offsets or an over-long txn (the
// host reports it from the pass's partials; the bit tells a chained
// central_finish not to number the epoch, occ_history.hip k_fin)
constexpr uint32_t ERR_PREP = 256;
// error bits after which an epoch's decisions are not final
constexpr uint32_t ERR_NOT_FINAL = ERR_OFFSETS | ERR_TILE | ERR_KEY | ERR_FULL | ERR_SPIN | ERR_PREP;

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

// Per-epoch values a captured epoch graph reads when it runs -- the commit
// counter, the delta level's append position and arrays, the history levels
// of the window check -- so one graph serves every epoch of a shape: the
// host writes them to pinned memory before each launch and the epoch's first
// kernel (k_fill) copies them to device memory.
struct OccDyn {
  uint64_t tnc;     // commit counter before the epoch (occ.cpp:283-284)
  uint32_t fin_tag; // central_finish's look-back tag (never 0; occ_history.hip k_fin)
  uint32_t pad;
  uint64_t hist_m;  // pairs in the delta level before the epoch's append
  uint64_t* app_k;  // delta level flat pairs (null: no append this epoch)
  uint64_t* app_t;
  HistInsert ins;   // the delta's table, updated by the append (hash null: none)
  HistView view;    // history levels (occ_history.h)
};
static_assert(sizeof(OccDyn) % 4 == 0, "copied as words");
struct HistArgs {
  uint64_t n, nnz;
  const uint32_t* off;
  const uint64_t* keys;
  const uint8_t* acctype;
  const uint64_t* start_tn;
  const uint64_t* finish_tn;
  const OccDyn* dyn;  // device history levels (dyn->view)
  uint32_t var;       // DCC_HIST_VAR timing variants (DCC_EXPERIMENTS builds only; 0)
  uint8_t* state;
  uint32_t* err;   // ERR_OFFSETS on a malformed device batch
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
  FinalPart* part;  // [FINAL_BLOCKS] (pinned host memory: read back directly)
};

// sub-list decisions back to the epoch's state bytes (round-solver hand-off)
void launch_scatter(const uint8_t* sub_state, const uint32_t* sub_tid, const uint32_t* n_sub,
                    uint64_t m_bound, uint8_t* state, hipStream_t st);

// ---- sweep solver (occ_sweep.hip)
constexpr uint32_t SW_T = 64;        // txns per serial tile (one 64-bit mask word)
constexpr uint32_t SW_TA = 4096;     // accesses per tile (SW_T x MAX_ROW_PER_TXN)
constexpr uint32_t SW_PL = 640;      // probe entries held in a tile record (more: lst_ovf)
constexpr uint32_t SW_IL = 312;      // insert entries held in a tile record (more: lst_ovf)
constexpr uint32_t SW_OVF = 2 * SW_TA;  // overflow entries per tile: probes, then inserts
constexpr uint32_t SW_WA = 4096;     // accesses of one filter wave (64 txns x MAX_ROW_PER_TXN)
constexpr uint32_t SW_CHUNK = 256;   // txns per filter chunk (4 waves x 64)
constexpr uint32_t SW_BLOOM_LOG = 17; // Bloom filter of a level's committed keys (16 KiB)
constexpr int SW_MAX_LEVEL = 24;
constexpr uint32_t SW_PMAX_TILES = 1024;  // tiles one serial pass may decide (65,536 txns)
constexpr uint32_t SW_GBITS_MAX = 19;  // key-table slots of one level (LDS bitmap: 64 KiB)
// Per-access key ids (slots of the level's key table) as k_sw_pre records
// them: id << 6 | WR << 5.
__host__ __device__ constexpr uint32_t sw_apack(uint32_t id, bool w) {
  return (id << 6) | (w ? 32u : 0u);
}
__host__ __device__ constexpr uint32_t sw_aid(uint32_t e) { return e >> 6; }
// Tile-list entries as the serial pass reads them, laid out so that one
// shift gives the LDS byte address of the committed bitmap's word and the
// bit / txn fields sit where the shift instructions read them (their low 5
// or 6 bits):
//   probe:  word << 7  | bit            address e >> 5,  bit e & 31
//   insert: word << 13 | bit << 6 | t   address e >> 11, bit (e >> 6) & 31,
//                                       txn of the tile e & 63
__host__ __device__ constexpr uint32_t sw_ppack(uint32_t id) {
  return ((id >> 5) << 7) | (id & 31u);
}
__host__ __device__ constexpr uint32_t sw_ipack(uint32_t id, uint32_t t) {
  return ((id >> 5) << 13) | ((id & 31u) << 6) | t;
}
// an id one past the largest table slot: the always-zero word that ends the
// serial pass's committed bitmap (64 spare words follow it: lane q of an
// unused insert slot ORs 0 into spare word q)
constexpr uint32_t SW_ID_NONE = 1u << SW_GBITS_MAX;
constexpr uint32_t SW_A_NONE = sw_apack(SW_ID_NONE, false);
constexpr uint32_t SW_P_NONE = sw_ppack(SW_ID_NONE);
__host__ __device__ constexpr uint32_t sw_idummy(uint32_t q) {
  return sw_ipack(SW_ID_NONE + 32u * (1u + (q & 63u)), 0);
}
// per-txn meta word of a tile record
constexpr uint32_t SWM_VALID = 1, SWM_PRE = 2, SWM_HASW = 4, SWM_STOP = 16;
// list chunks the serial pass holds in registers: the first SW_RC * 64
// entries of each list (padded with no-op entries by k_sw_rows).  Three: the
// headline's serial ranges hold 107-161 probes per 64-txn tile on average,
// and a tile past the register chunks takes the long path (an LDS loop per
// chunk); 2 -> 3 took the passes from 17 / 33 / 55 to 14 / 25 / 48 us, 4 was
// slower again at level 2 (14 / 28 / 54).
constexpr uint32_t SW_RC = 3;
// insert chunks held in registers (the needed writes are fewer: 58-92 per
// tile at the headline's levels; a third insert chunk is a dummy atomic)
constexpr uint32_t SW_RC_I = 2;
// One 64-txn tile of a level's serial range as k_sw_seq reads it (7,168 B).
// Only the accesses the serial pass must look at, as two tile-wide lists:
// probes (accesses whose key an earlier txn of the range writes), grouped by
// txn (txn t's are [pspan & 0xFFFF, pspan >> 16)), and inserts (writes whose
// key a later txn of the range accesses).
struct SwRec {
  uint32_t probe[SW_PL];
  uint32_t ins[SW_IL];
  uint64_t dep[SW_T];     // dep[t]: earlier txns of the tile writing a key t touches
  uint32_t meta[SW_T];    // SWM_* (SWM_STOP on every txn: the access budget ends here)
  uint32_t rtid[SW_T];    // original txn index
  uint32_t pspan[SW_T];
  // seg[c][t]: txn t's probe entries among list positions [64c, 64c + 64)
  uint64_t seg[SW_RC][SW_T];
  uint32_t np, ni;
  uint32_t hdr;  // SWH_*: the serial pass's per-tile branches
  uint32_t pad[5 + 128];  // whole KiB (the ring copy moves 16 B per lane)
};
constexpr uint32_t SWH_PLONG = 1, SWH_ILONG = 2, SWH_STOP = 4;
struct SwLevel {     // device control words of one level
  uint32_t m;        // list length (written by the previous level's filter)
  uint32_t acc;      // accesses of the list
  uint32_t pos;      // list txns decided by the level's sequential pass
  uint32_t ccount;   // committed write keys of the pass (k_sw_cout's fill counter)
  uint32_t ticket;   // filter chunk ticket
  uint32_t pad[3];
};
struct SwList {
  const uint32_t* tid;  // original txn index per list position (null: identity)
  const uint32_t* off;
  const uint64_t* keys;
  const uint8_t* acctype;
  uint64_t nnz;         // accesses addressable through keys/acctype
};
// The epoch's committed writers: key -> the txn id of its committed writer.
// A key has at most one (the first committed writer of a key kills every
// later accessor, occ.cpp:185-199), so a slot is written once.  Open
// addressing, linear probes over 16-B slots (key and writer read together),
// KEY_EMPTY-filled per epoch; an insert that finds no slot within `probes`
// sets *full (the host then rebuilds a table sized for every write).
struct __attribute__((aligned(16))) WrSlot {
  uint64_t key;
  uint32_t tid;
  uint32_t pad;
};
struct WrTab {
  WrSlot* slot;     // [1 << bits]
  uint32_t bits;
  uint32_t probes;  // longest probe sequence (WT_PROBES; the whole table for the fallback)
  uint32_t* full;
};
constexpr uint32_t WT_PROBES = 64;
constexpr uint32_t WT_BITS_DEFAULT = 18;  // 2^18 slots (4 MiB): ~10 % load at the headline (2^16 measured slower)
// A read-only txn the level-0 compaction split off: its id and access range.
struct RoEnt {
  uint32_t tid, s, e, pad;
};
// k_sw_ro: the split-off read-only txns, decided once every writer is: abort
// iff a key has a committed writer with a smaller txn id (occ.cpp:185-199
// with only earlier txns' writes in `active`; read-only txns never enter it).
struct SwRoArgs {
  const RoEnt* ro;
  const uint32_t* ro_count;
  const uint64_t* keys;
  WrTab wt;
  uint8_t* state;
  const uint32_t* full_off;  // key-sharded with the whole batch: a txn's accesses are
                             // [full_off[t], full_off[t + 1]) of keys, not the entry's range
};
// k_sw_wall: the committed writers' writes into wt -- the txns the serial
// passes listed (cw_list, cw_count), or (cw_list null) every committed txn
// with a write of the decided epoch (after a hand-off to the round solver)
struct SwWallArgs {
  uint64_t n;
  const uint32_t* off;
  const uint64_t* keys;
  const uint8_t* acctype;
  uint64_t nnz;
  const uint8_t* state;
  const uint8_t* hasw;
  const uint32_t* cw_list;
  const uint32_t* cw_count;
  WrTab wt;
};
void launch_sw_ro(const SwRoArgs& a, unsigned grid, hipStream_t st);
void launch_sw_wall(const SwWallArgs& a, unsigned grid, hipStream_t st);

struct SwPreArgs {
  SwList in;
  const uint32_t* m_dev;  // list length on the device (null: m_host)
  uint32_t m_host;
  uint32_t p_max;
  const uint8_t* state;   // identity list: decisions made before the solver, else null
  SwRec* rec;             // [tiles]
  uint32_t* lst_ovf;      // [tiles][SW_OVF] list entries past the record's
  uint64_t* gtab;         // [1 << gbits] key table (KEY_EMPTY-filled), slot = key id
  uint32_t gbits;
  uint32_t budget;        // accesses the level's tiles may hold (gtab at <= 50% load)
  uint32_t* first_w;      // [1 << gbits] first writer (list position) per key id, ~0u-filled
  uint32_t* last_a;       // [1 << gbits] last accessor per key id, 0-filled
  uint32_t* aent;         // [budget] sw_apack(key id, WR) per access of the serial range
  uint32_t* apos;         // [budget] list position of the access's txn
  const uint32_t* abandon;
  uint32_t* err;
  uint64_t* dbg;          // workgroup-0 stamps (DCC_SW_DEBUG) or null
};
struct SwSeqArgs {
  const uint32_t* m_dev;
  uint32_t m_host;
  uint32_t p_max;
  int write_hasw;
  const SwRec* rec;
  const uint32_t* lst_ovf;
  const uint64_t* gtab;
  uint32_t gbits;
  uint8_t* state;
  uint8_t* hasw;
  uint32_t* cbits_out;    // out: committed ids (bitmap over the key table's slots)
  uint64_t* ckeys_out;    // out: the committed keys (lv->ccount of them)
  uint32_t* bloom_out;    // out: Bloom filter of the committed keys
  SwLevel* lv;
  SwLevel* lv_next;
  uint32_t* next_off;     // the next list's offsets (off[0] = 0 written here)
  uint64_t* mg;           // out: commit mask per decided tile
  const uint32_t* abandon;
  uint32_t* err;
  uint64_t* dbg;          // per-tile clock stamps (DCC_SW_DEBUG) or null
  // read-only split: committed txns with a write are appended here (their
  // writes enter the writer table after the levels, k_sw_wall); null: none
  uint32_t* cw_list;
  uint32_t* cw_count;
};
// prep workgroups beside the level-0 committed-set listing (k_sw_cout)
#ifndef DCC_SW_PREP_BLOCKS
#define DCC_SW_PREP_BLOCKS 1024
#endif
constexpr unsigned SW_PREP_BLOCKS = DCC_SW_PREP_BLOCKS;
struct SwCoutArgs {
  SwList in;
  const uint32_t* aent;
  const uint32_t* apos;
  const uint64_t* mg;
  SwLevel* lv;            // pos in, ccount out
  uint32_t* cbits_out;
  uint64_t* ckeys_out;
  uint32_t* bloom_out;
  const uint32_t* abandon;
  const uint32_t* m_dev;  // list length: with skip_done, a level whose serial
  uint32_t m_host;        // pass decided the whole list lists nothing (no
  int skip_done;          // filter follows)
  uint32_t cout_grid;     // workgroups of the listing; the launch's others (level 0):
  // the epoch's batch validation (prep_body.h) -- offsets, lengths, write
  // count, and every txn's has-write byte into `hasw` (read first by the
  // level-0 filter) -- on 0-LDS workgroups beside the listing rather than
  // beside the serial pass, whose 160 KB of LDS made each of them hold a
  // whole CU (prep_part null: none)
  const uint32_t* prep_off;
  uint64_t prep_n;
  const uint8_t* prep_at;
  uint64_t prep_nnz;
  PrepPart* prep_part;    // [SW_PREP_BLOCKS] (pinned host memory)
  uint8_t* hasw;
  uint4* wclear;          // the writer table, cleared by the prep workgroups
  uint64_t wclear_n16;    // its size in 16-B words (0: none)
  uint32_t* prep_err;     // ERR_PREP joins the epoch's error word (null: none)
};
// k_sw_filter / k_sw_scan / k_sw_compact (one argument block for the three)
struct SwFilterArgs {
  SwList in;
  const uint32_t* m_dev;
  uint32_t m_host;
  int cand_state;         // identity list: only UNDECIDED txns are candidates
  uint32_t level;
  const uint64_t* gtab;   // the level's key table / committed ids / Bloom filter /
  uint32_t gbits;         // committed keys (k_sw_seq's outputs): the committed set C
  const uint32_t* cbits;
  const uint32_t* bloom;
  const uint64_t* ckeys;
  SwLevel* lv;
  SwLevel* lv_next;
  uint8_t* state;
  uint8_t* hasw;
  uint64_t* sflag;        // survivor bit per list position past pos (64 per word)
  unsigned long long* tcount;  // per 64-txn tile: survivors << 34 | their accesses
  unsigned long long* bsum;    // per filter workgroup: its tiles' total (scanned in place)
  uint32_t nblocks;            // filter / compaction grid
  uint32_t* tid_out;
  uint32_t* off_out;
  uint64_t* keys_out;
  uint8_t* acc_out;
  const uint32_t* abandon;
  uint32_t* abandon_out;  // = level + 1 when the survivors stay too many
  uint32_t abandon_min, abandon_num, abandon_den;
  // key-sharded: this shard's kill bits, one 64-bit word per list tile of 64
  // positions after the serial range (bit = lane), else null; k_sw_apply ORs
  // the kill_ranks contributions of kill_stride words each in kill_in
  uint64_t* kill_out;
  const uint64_t* kill_in;
  uint32_t kill_ranks;
  uint64_t kill_stride;
  // read-only split (level 0, one GPU): read-only survivors (hasw[txn] == 0)
  // go to ro_out (txn ids, any order) instead of the next list -- no later
  // level holds them; k_sw_ro decides them once every writer is decided
  int ro_split;
  uint64_t* rflag;        // read-only survivor bits per tile
  unsigned long long* rtcount;  // per tile: read-only survivors << 34 | their accesses
  unsigned long long* rbsum;    // per filter workgroup: read-only total
  RoEnt* ro_out;
  uint32_t* ro_count;     // out: length of ro_out (0 when the level hands off)
  uint64_t* gclear;       // the next level's key table, KEY_EMPTY-filled here
  uint64_t gclear_n;
  uint32_t* fw_clear;     // the next level's first-writer / last-accessor words
  uint32_t* la_clear;
  uint32_t* err;
  uint64_t* dbg;          // per-workgroup clock stamps (DCC_SW_DEBUG) or null
  uint64_t* cdbg;         // k_sw_compact's workgroup-0 stamps (DCC_SW_DEBUG) or null
};
// One key-sharded sweep level (the host side of SURVEY.md §8(e)): the merged
// serial range, its txn count, the list length and the kill-bit buffer.
// One key-sharded sweep level: the serial range every rank decides alike
// (merged records, or gathered from the whole batch each rank holds), and the
// kill-bit exchange of the level's filter.
struct SwShard {
  SwList serial;
  const uint32_t* m_dev;  // the serial list's length on the device (null: P)
  uint32_t P;             // its length on the host (m_dev null)
  uint64_t* kill_out;     // this rank's kill words (kill_words of them)
  uint64_t* kill_all;     // every rank's, rank-major
  uint64_t kill_words;    // words exchanged per rank
  // the whole batch (DCC_SHARD_SELF): the serial part's has-write bytes come
  // from it, so no has-write exchange is needed
  const uint32_t* full_off;
  const uint8_t* full_at;
  uint64_t full_nnz;
};
// The first min(p_max, *m) list txns' whole access lists (the serial range of
// a key-sharded level, gathered from the whole batch): offsets soff[0..P],
// keys / types at soff; two launches, no host synchronisation.
void launch_sw_sgather(const uint32_t* tid, const uint32_t* m_dev, uint32_t p_max,
                       const uint32_t* full_off, const uint64_t* full_keys, const uint8_t* full_at,
                       uint64_t full_nnz, uint32_t* soff, uint64_t* skeys, uint8_t* sat,
                       uint32_t* err, hipStream_t st);
void launch_sw_pre(const SwPreArgs& a, unsigned grid, hipStream_t st);
void launch_sw_seq(const SwSeqArgs& a, hipStream_t st);
void launch_sw_rows(const SwPreArgs& a, unsigned grid, hipStream_t st);
void launch_sw_cout(const SwCoutArgs& a, unsigned grid, hipStream_t st);
void launch_sw_filter(const SwFilterArgs& a, unsigned grid, hipStream_t st);
void launch_sw_compact(const SwFilterArgs& a, unsigned grid, hipStream_t st);
void launch_sw_apply(const SwFilterArgs& a, unsigned grid, hipStream_t st);
void launch_sw_share(const uint32_t* m_dev, uint32_t m_host, const uint32_t* abandon,
                     const uint32_t* off, uint32_t p_max, uint32_t rank, uint32_t* cnt,
                     hipStream_t st);
// key-sharded serial range: export this rank's records at xbuf + xoff_words
// (export_only), or merge the all-gathered n_all records into one CSR
void launch_sw_merge(const SwList& in, uint32_t P, uint32_t* xbuf, uint32_t xoff_words,
                     uint32_t n_all, uint32_t* cnt, uint32_t* cur, uint32_t* moff,
                     uint64_t* mkeys, uint8_t* mat, bool export_only, hipStream_t st);

// Compact transfer forms widened on the device (dcc_ctx::stage_batch): u32
// keys -> u64, 2-bit packed access types -> bytes, u32 timestamps -> u64.
// A null source skips that part.
struct WidenArgs {
  uint64_t n, nnz;
  const uint32_t* k32;
  uint64_t* k64;
  const uint8_t* a2;
  uint8_t* a8;
  const uint32_t *s32, *f32;
  uint64_t *s64, *f64;
};
void launch_widen(const WidenArgs& a, unsigned n_cu, hipStream_t st);
void launch_copy16(const void* src, void* dst, uint64_t bytes, unsigned grid, hipStream_t st);
void launch_copy16_chunk(const void* src, void* dst, uint64_t bytes, unsigned grid, hipStream_t st);

// Several word fills in one launch (replaces a run of hipMemsetAsync calls,
// each of which costs a dispatch and an idle gap on the stream).
struct FillJob {
  uint32_t* p;
  uint64_t words;
  uint32_t value;
  const uint32_t* src = nullptr;  // copy `words` words from here instead of filling
};
struct FillArgs {
  FillJob job[12];
  uint32_t n;
};
void launch_fill(const FillArgs& a, hipStream_t st);
// Several small device -> pinned-host copies in one launch (word granular):
// the control words, counters and partials the host reads after an epoch.
struct CopyJob {
  const uint32_t* src;
  uint32_t* dst;  // device-visible pointer of pinned host memory
  uint32_t words;
};
struct GatherArgs {
  CopyJob job[12];
  uint32_t n;
};
void launch_gather(const GatherArgs& a, hipStream_t st);

// launchers (occ_kernels.hip)
void launch_prep(const uint32_t* off, uint64_t n, const uint8_t* at, uint64_t nnz, uint64_t p,
                 PrepPart* part, hipStream_t st);
void launch_hist(const HistArgs& a, hipStream_t st);
void launch_build(const BuildArgs& a, unsigned max_grid, hipStream_t st);
void launch_round(const RoundArgs& a, bool from_keys, uint64_t m_bound, unsigned max_grid,
                  hipStream_t st);
void launch_retag(Slot* tab, uint64_t cap, hipStream_t st);
void launch_pub(const PubArgs& a, uint64_t m_bound, unsigned max_grid, hipStream_t st);
// k_final also performs the read-back copies of g (pinned host targets)
void launch_final(const FinalArgs& a, const GatherArgs& g, hipStream_t st);
// sharded rounds: apply the all-reduced status (0 commit, 1 stay, >=2 abort),
// clear it for the next round, add the undecided count to *und.
void launch_decide(uint8_t* state, uint8_t* gst, uint64_t n, uint8_t abort_byte, uint32_t* und,
                   uint32_t* und_next, hipStream_t st);
// central_finish of a decided epoch in three launches, every per-epoch value
// read from `dyn` (graph-replayable): commit tn in index order for the txns
// with cflag set (tn = dyn->tnc + 1, ...) and, when dyn->app_k is set, their
// write sets appended to the delta level at dyn->hist_m in tn order
// (occ.cpp:277-286).  totals (pinned): [0] committed writers, [1] pairs
// appended, [2] largest key appended.
// The device copy of the commit counter and the delta level's append position
// that chained central_finish launches advance in submit order (seq: the next
// epoch entitled to them).
struct FinCtl {
  uint64_t tnc, hist_m, seq, pad;
};
struct OccFinArgs {
  uint64_t n, nnz;
  const uint32_t* cflag;
  const uint32_t* off;
  const uint64_t* keys;
  const uint8_t* acctype;
  uint64_t* part;      // fin_part_bytes(n): look-back words (zeroed when allocated)
  const OccDyn* dyn;
  uint64_t* tn;        // out: commit tn per txn (0 = none)
  uint64_t* totals;    // out: pinned host memory: [0] numbered, [1] appended, [2] largest
                       // key appended, [3] the delta table's overflow flag
  uint32_t tag;        // look-back tag; 0: the epoch's (dyn->fin_tag).  A second launch
                       // for the same epoch takes a fresh one.
  uint32_t var;        // DCC_FIN_VAR timing variants (DCC_EXPERIMENTS builds only; 0)
  // Chained (a pipeline lane's epoch, finished on the device in submit order;
  // ctl null: not chained).  dyn->tnc / hist_m are then the snapshot of *ctl
  // taken by k_fin_prep, dyn->pad 1 when *ctl was at `seq` (every epoch before
  // this one finished): only then does k_fin number the epoch, and it advances
  // *ctl past it when the epoch was final -- no undecided txn (state), no
  // ERR_NOT_FINAL bit in *err, no overflow of the committed-writer table
  // (*wfull), every pair within `cap` -- reporting totals[4] = 1.  Otherwise
  // totals[4] = 0 and the host finishes the epoch itself.
  FinCtl* ctl;
  uint64_t seq;
  const uint8_t* state;
  const uint32_t* err;
  const uint32_t* wfull;
  uint64_t cap;
};
void launch_fin(const OccFinArgs& a, hipStream_t st);
// a chained finish's parameters: the OccDyn words from pinned `src` into
// `dyn`, then the snapshot of *ctl (occ_history.hip)
void launch_fin_prep(const uint32_t* src, OccDyn* dyn, const FinCtl* ctl, uint64_t seq, hipStream_t st);
// *ctl = {tnc, hist_m, seq} (seq stored last, release)
void launch_fin_ctl_set(FinCtl* ctl, uint64_t tnc, uint64_t hist_m, uint64_t seq, hipStream_t st);
uint64_t fin_part_bytes(uint64_t n);
// summary of a host copy of the look-back words after a launch with `tag`
// (the totals-mismatch error message)
std::string fin_diag(const void* words, uint64_t n, uint32_t tag);
void launch_commit_tn(const uint32_t* cflag, uint64_t n, uint64_t* bsum, uint64_t tnc,
                      uint64_t* tn, hipStream_t st);
// deferred central_finish: cflag[t] = global RCOK && local commit && has a
// write; cnt[0] += their number, cnt[1] += txns with global RCOK that
// aborted locally
void launch_finish_flags(const uint8_t* final_rc, const uint8_t* state, const uint8_t* hasw,
                         uint64_t n, uint32_t* cflag, uint32_t* cnt, hipStream_t st);

}  // namespace dcc
