// The OCC stage solver (occ_stage.hip): argument blocks and constants shared
// with the host driver (occ_driver.hip).  DESIGN.md §3 describes the solver.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace dcc {

constexpr uint32_t ST_B = 1024;          // threads per workgroup (16 waves, one per CU)
constexpr uint32_t ST_W = ST_B / 64;     // waves per workgroup
constexpr uint32_t ST_WT = 64;           // wave-tiles (of 64 txns) per filter round
constexpr uint32_t ST_MAX_PUB = 1024;    // chunks a decider can take in
constexpr uint32_t ST_MAX_STAGES = 64;   // stages per epoch before the round-solver fallback
constexpr uint32_t ST_G = 4;             // input chunks per filter workgroup, list stages
constexpr uint32_t ST_CS_LOG = 13;       // decider: committed-key set, 8192 slots (64 KB)
constexpr uint32_t ST_CS_BUDGET = 3800;  // committed keys a decider may collect (<= 47% load)
constexpr uint32_t ST_CB_LOG = 16;       // decider: committed-key bitmap bits (8 KB)
constexpr uint32_t ST_WM_LOG = 10;       // filter: per-wave tile write map, 1024 slots (16 KB)
constexpr uint32_t ST_WM_WAVES = 4;      // filter waves building tiles concurrently
constexpr uint32_t ST_FB_LOG = 18;       // filter: committed-key bitmap bits (32 KB)
constexpr uint32_t ST_CT_LOG = 13;       // filter: exact committed-key set, 8192 slots
constexpr uint32_t ST_TILE = 64;         // txns per decider tile (32 when a chunk has a txn > 32 accesses)
constexpr uint32_t ST_TILE_ACC = 1024;   // accesses per decider tile: 64 txns of <= 16, 32 of <= 32, 16 of <= 64
constexpr uint32_t ST_DEC_WAVES = 4;     // decider workgroup: waves deciding tiles (the rest load them)
constexpr uint32_t ST_LOAD_GROUPS = 3;   // loader groups: each keeps one tile in flight
constexpr uint32_t ST_MAX_TILES = 256;   // tiles one decider may decide (16K txns)

// error bits (StCtl::err)
constexpr uint32_t STE_OFFSETS = 1;  // malformed offsets
constexpr uint32_t STE_KEY = 4;      // DCC_KEY_RESERVED in the batch
constexpr uint32_t STE_LEN = 8;      // a txn longer than MAX_ROW_PER_TXN
constexpr uint32_t STE_SPIN = 16;    // decider: chunk hand-off spin limit
constexpr uint32_t STE_WMAP = 32;    // decider: tile write map full

// One stage's control record.  Stage l's filter workgroups add to the
// counters; its decider writes the rest.  Zeroed for stage l + 1 by stage
// l's decider, for stage 0 by the epoch's final kernel.
struct StCtl {
  uint32_t in_n;        // list txns the filter examined
  uint32_t surv_n;      // survivors written (this stage's output list)
  uint32_t surv_acc;    // their accesses
  uint32_t nnz_w;       // write accesses (stages 0/1: the epoch's, for the stats)
  uint32_t ro;          // read-only txns (idem)
  uint32_t err;
  uint32_t ran;         // 1 when the decider ran
  uint32_t consumed;    // survivors the decider decided (a prefix of the output list)
  uint32_t stop_chunk;  // first chunk / index in it that the decider did not decide
  uint32_t stop_idx;
  uint32_t stop_tid;    // epoch index of that txn (0xFFFFFFFF: none)
  uint32_t commits;     // RCOK decisions of the decider
  uint32_t cw;          // of which with a write set (tn given, central_finish)
  uint32_t ckeys_n;     // committed write keys collected (the next filter's C)
  uint32_t tiles;       // decider tiles
  uint32_t abandon;     // 1: the list stopped shrinking, hand off to the round solver
};

// Epoch-persistent device state.
struct StEpoch {
  uint32_t gen;         // bumped by the final kernel: hand-off tags are (gen, stage)
  uint32_t pad;
  uint64_t tnc;         // the commit counter tnc (occ.h:67), carried by the deciders
};

// Chunk header of a stage's output list (written before its flag).
struct StChunk {
  uint32_t nt, na;      // survivors and their accesses
  uint32_t tbase;       // first txn slot of the chunk's region
  uint32_t abase;       // first access slot
  uint32_t flag;        // hand-off tag (gen, stage) once the chunk is published
  uint32_t ntiles;      // decider tiles of the chunk (64 survivors each, the last partial)
  uint32_t pad[2];
};

// A stage's output list: survivors in index order, chunk by chunk.  Txn slot
// j holds the epoch index tid[j], its accesses [ast[j], ast[j] + alen[j]) of
// keys / at.  Chunk regions never overlap and stay in index order.
struct StList {
  uint32_t* tid;
  uint32_t* ast;
  uint8_t* alen;
  uint64_t* dep;     // per txn slot: intra-tile dependency mask (earlier writers of its keys)
  uint64_t* keys;
  uint32_t* hsh;     // per access: st_hash(key)
  uint8_t* pk;       // per access: tile-local txn << 1 | W
  uint64_t* tile;    // per tile (at the chunk's txn base + k): 4 words, see StTile
  StChunk* hdr;
};
// Tile descriptor, 4 u64 words: [0] first txn slot | nt << 32,
// [1] first access slot | na << 32, [2] write accesses, [3] has-write mask.
constexpr uint32_t ST_TILE_WORDS = 4;

struct StArgs {
  uint32_t stage;
  uint32_t mode;         // 0: epoch range (stages 0, 1), 1: list (stages >= 2)
  uint32_t n;            // epoch txns
  uint64_t nnz;          // epoch accesses
  const uint32_t* off;   // epoch CSR
  const uint64_t* keys;
  const uint8_t* at;
  uint32_t e_end;        // mode 0: end of the epoch range (stage 0: P0, stage 1: n)
  uint32_t p0;           // P0: the epoch prefix stage 0 covers
  uint32_t ch;           // mode 0: epoch txns per chunk
  StList in;             // mode 1: the previous stage's output list
  uint32_t in_chunks;
  StList out;
  uint32_t out_chunks;   // = filter workgroups
  uint32_t gpub;         // chunks [0, gpub) are published to the decider
  uint32_t pmax;         // txns the decider may decide
  uint32_t decide;       // 1: workgroup 0 is the decider
  const StCtl* prev;     // previous stage (nullptr for stage 0)
  StCtl* cur;
  StCtl* next;           // zeroed by the decider
  const uint64_t* ck_prev;  // the previous decider's committed write keys (C)
  uint64_t* ck_cur;
  StEpoch* ep;
  const uint8_t* hkill;  // per-txn history-window aborts (nullptr: none)
  uint8_t* rc;           // per-txn RC out (RCOK / Abort)
  uint64_t* tn;          // per-txn commit tn out (nullptr: not wanted)
  uint32_t xflags;       // DCC_ST_X: experiment switches (0 = production)
  uint64_t* dbg;         // DCC_ST_DEBUG: s_memrealtime stamps, [stage][32] (nullptr: off)
};

struct StFinalArgs {
  StEpoch* ep;
  StCtl* ctl;            // [ST_MAX_STAGES]
  uint32_t n_ctl;        // records copied
  void* host;            // device-visible pinned host mirror: StEpoch then StCtl[n_ctl]
};

void launch_stage(const StArgs& a, hipStream_t st);
void launch_stage_final(const StFinalArgs& a, hipStream_t st);

}  // namespace dcc
