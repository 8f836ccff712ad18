// Calvin wave levels in one CU -- see calvin_wave.h for the formulation.
//
//   k_cw_seqpos  inverse of the sequencer order (txn -> sequence position)
//   k_cw_link    per slot: the previous group's and the own group's max slot
//                (global slot codes), their 16-bit LDS forms (staging) and
//                LDS byte addresses (walker)
//   k_cw_mark / k_cw_cr  the slots read inside their own sub-chunk, and per
//                txn its (at most two) such reads and publications
//   k_cw_walk    one workgroup: wave 0 walks, the other waves stage (with
//                helper workgroups on other CUs taking the scattered part)
//
// LDS and global group maxima hold (max wave + 1): 0 is "no member yet", and
// a request's bound is the value it reads.
#include "calvin_wave.h"

#include <algorithm>

#include "dcc_device.h"

namespace dcc {
namespace {

constexpr uint32_t NONE = 0xFFFFFFFFu;
// 8 waves (2 per SIMD: 256 VGPRs each -- the walker's three record
// buffers fit without spills)
constexpr uint32_t CW_T = 512;
constexpr uint32_t CW_HELP = CW_T - 64;                            // staging threads
constexpr uint32_t CW_HWAVES = CW_HELP / 64;                       // staging waves
constexpr uint32_t CW_K = 36;                                      // slots per staging thread
constexpr uint32_t CW_HPLAN = CW_K * CW_HELP;                      // slots per chunk (cw_plan)
constexpr uint32_t F_NONE = 0xFFFFu;                               // 16-bit field: no slot
constexpr uint32_t F_FAR = 0xFFFEu;  // prev: ended 2+ chunks back; own: ends 2+ chunks ahead
constexpr uint32_t F_FLAG = 0x8000u;  // prev: same sub-chunk; own: next chunk's region
constexpr uint32_t CW_ZERO = 0x7FFFu;  // LDS slot that stays 0 (F_NONE's read target)
constexpr uint32_t CW_SINK = CW_ZERO - 65;  // 64 write-only slots (one per walker lane)
static_assert(2 * CW_K * CW_HELP <= CW_SINK, "LDS slot space");

// Staging loads through buffer descriptors: a 32-bit offset per load (one
// VGPR, not a 64-bit address pair); aux 16 = sc1 (read in the L2, past this
// CU's L1: the global maxima are written by other waves of the workgroup).
__device__ inline __amdgpu_buffer_rsrc_t cw_rsrc(const void* p, uint64_t bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), (short)0,
                                           (int)(bytes < 0x7FFFFFFFull ? bytes : 0x7FFFFFFFull),
                                           0x00020000);
}
__device__ inline uint32_t cw_ld(__amdgpu_buffer_rsrc_t r, uint32_t idx) {
  return __builtin_amdgcn_raw_buffer_load_b32(r, idx * 4u, 0, 0);
}
__device__ inline uint32_t cw_ld_l2(__amdgpu_buffer_rsrc_t r, uint32_t idx) {
  return __builtin_amdgcn_raw_buffer_load_b32(r, idx * 4u, 0, 16);
}
// (helpers) a write-through store: sc1, like an agent-scope relaxed store
__device__ inline void cw_st_l2(__amdgpu_buffer_rsrc_t r, uint32_t idx, uint32_t v) {
  __builtin_amdgcn_raw_buffer_store_b32(v, r, idx * 4u, 0, 16);
}

__device__ inline void lds_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

// Hand-offs between the walker's workgroup and the helper workgroups (other
// CUs, any XCD): every handed-off word is stored and loaded with agent-scope
// relaxed atomics (global_store / global_load sc1: past the L1, write-through)
// or changed by agent-scope atomics; a storing wave waits for its stores
// (vmcnt 0) before the flag that covers them is raised (MI355X_MICROARCH.md,
// inter-workgroup visibility, the sc1 hand-off row).
__device__ inline uint32_t ag_ld(const uint32_t* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ inline void ag_st(uint32_t* p, uint32_t v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ inline void vm_drain() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }
// help block: [0] chunks published by the walker's workgroup, [16] helper
// iterations done (summed over helpers), [32] abort (a poll gave up), then the
// bounds of every chunk's txns and the waves of every chunk, in sequence order
constexpr uint32_t CW_HP = 0, CW_HR = 16, CW_HAB = 32, CW_HDATA = 64;
constexpr uint32_t CW_POLL_MAX = 1u << 22;  // ~0.2 s of s_sleep(2) per poll
// wait until *ctr >= target; false when this or another poll gave up
__device__ inline bool cw_poll(uint32_t* help, uint32_t at, uint32_t target) {
  for (uint32_t k = 0; ag_ld(help + at) < target; k++) {
    if (ag_ld(help + CW_HAB)) return false;
    if (k >= CW_POLL_MAX) {
      __hip_atomic_fetch_or(help + CW_HAB, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      return false;
    }
    __builtin_amdgcn_s_sleep(2);
  }
  return true;
}

__global__ __launch_bounds__(256) void k_cw_seqpos(const uint32_t* __restrict__ seq, uint64_t n,
                                                   uint32_t* __restrict__ seqpos) {
  const uint64_t q = (uint64_t)blockIdx.x * 256 + threadIdx.x;
  if (q < n) seqpos[seq[q]] = (uint32_t)q;
}

struct LinkArgs {
  CwPlan p;
  CwArgs a;
};

// One thread per slot, in slot order (coalesced writes).  A slot's code is
// seqpos(txn) << lg | j; its chunk is code / H.
__global__ __launch_bounds__(256) void k_cw_link(LinkArgs A) {
  const CwPlan& p = A.p;
  const CwArgs& a = A.a;
  const uint64_t s = (uint64_t)blockIdx.x * 256 + threadIdx.x;
  if (s >= p.slots) return;
  const uint32_t q = (uint32_t)(s >> p.lg), j = (uint32_t)s & ((1u << p.lg) - 1u);
  uint32_t prevc = NONE, ownc = NONE;
  if (q < a.n) {
    const uint32_t t = a.seq ? a.seq[q] : q;
    const uint32_t x0 = a.ulen ? t * a.ulen : a.off[t];
    const uint32_t len = a.ulen ? a.ulen : a.off[t + 1] - x0;
    if (j < len) {
      const uint32_t g = a.gsx[x0 + j];
      if (g != NONE) {
        const uint32_t gs = g & 0x7FFFFFFFu;
        auto code = [&](uint32_t v) {
          const uint32_t tt = v >> 7;
          return ((a.seq ? a.seqpos[tt] : tt) << p.lg) | ((v >> 1) & 63u);
        };
        if (g >> 31) prevc = code(a.sv[gs - 1]);
        const uint32_t gl = a.glast[gs];
        if (gl != NONE) ownc = code(a.sv[gl]);
      }
    }
  }
  const uint32_t c = q / p.C;
  uint32_t f_prev = F_NONE, f_own = F_NONE;
  if (prevc != NONE) {
    const uint32_t pc = prevc / p.H, loc = prevc - pc * p.H;
    if (pc + 1 >= c) {  // the current or the previous chunk: LDS
      const bool intra = pc == c && ((loc >> p.lg) >> 6) == ((q - c * p.C) >> 6);
      f_prev = ((pc & 1u) * p.H + loc) | (intra ? F_FLAG : 0u);
    } else {
      f_prev = F_FAR;
    }
  }
  if (ownc != NONE) {
    const uint32_t oc = ownc / p.H, loc = ownc - oc * p.H;
    if (oc == c) f_own = (c & 1u) * p.H + loc;
    else if (oc == c + 1) f_own = (((c + 1) & 1u) * p.H + loc) | F_FLAG;
    else f_own = F_FAR;
  }
  a.rec16[s] = f_prev | (f_own << 16);
  a.recp[s] = prevc;
  a.reco[s] = ownc;
  if (a.rec2) {
    // (helpers) the staging record: low half, the LDS slot of a previous
    // group that ended exactly two chunks back; high half, the LDS slot an
    // own group ending in the next chunk (F_FLAG clear) or two chunks ahead
    // (F_FLAG set) is added to at a boundary; F_NONE: none
    uint32_t p2 = F_NONE, o2 = F_NONE;
    if (prevc != NONE) {
      const uint32_t pc = prevc / p.H;
      if (pc + 2 == c) p2 = (pc & 1u) * p.H + (prevc - pc * p.H);
    }
    if (ownc != NONE) {
      const uint32_t oc = ownc / p.H;
      if (oc == c + 1 || oc == c + 2)
        o2 = ((oc & 1u) * p.H + (ownc - oc * p.H)) | (oc == c + 2 ? F_FLAG : 0u);
    }
    a.rec2[s] = p2 | (o2 << 16);
  }
  // the walker's addresses: a far / absent previous group reads the zero
  // slot; an own group not in this chunk publishes to the lane's sink
  a.pa[s] = 4u * (f_prev < F_FAR ? (f_prev & 0x7FFFu) : CW_ZERO);
  a.oa[s] = 4u * (f_own < F_FLAG ? f_own : CW_SINK + (q & 63u));
}

// Marks every slot that a request of the same sub-chunk reads (an intra
// previous group), then per txn the own slots that publish to a marked slot:
// the walker's per-round publications are those (the rest publish once, with
// the final wave).
__global__ __launch_bounds__(256) void k_cw_mark(const uint32_t* __restrict__ rec16,
                                                 const uint32_t* __restrict__ recp, uint64_t slots,
                                                 uint8_t* __restrict__ mark) {
  const uint64_t s = (uint64_t)blockIdx.x * 256 + threadIdx.x;
  if (s >= slots) return;
  const uint32_t f = rec16[s] & F_NONE;
  if (f < F_FAR && (f & F_FLAG)) mark[recp[s]] = 1;
}

// Per txn: its intra reads (previous groups whose last member is in the
// same sub-chunk) and hot publications (own groups some request of the same
// sub-chunk reads), at most CR_K of each as LDS byte addresses (the zero slot
// / the lane's sink when fewer); flags in the top bits of word 0: CR_INTRA
// (an intra read), CR_HOT (a hot publication), CR_OVF (more than CR_K of
// either).  Record: CR_K read addresses, then CR_K publication addresses.
constexpr uint32_t CR_K = 4, CR_W = 2 * CR_K;
constexpr uint32_t CR_INTRA = 1u << 30, CR_HOT = 1u << 29, CR_OVF = 1u << 31, CR_ADDR = 0x1FFFFu;
__global__ __launch_bounds__(256) void k_cw_cr(const uint32_t* __restrict__ rec16,
                                               const uint32_t* __restrict__ reco,
                                               const uint8_t* __restrict__ mark, uint64_t nq,
                                               uint32_t lg, uint32_t* __restrict__ cr) {
  const uint64_t q = (uint64_t)blockIdx.x * 256 + threadIdx.x;
  if (q >= nq) return;
  uint32_t r[CR_W];
  for (uint32_t k = 0; k < CR_K; k++) {
    r[k] = 4u * CW_ZERO;
    r[CR_K + k] = 4u * (CW_SINK + ((uint32_t)q & 63u));
  }
  uint32_t ni = 0, no = 0;
  for (uint32_t j = 0; j < (1u << lg); j++) {
    const uint64_t s = (q << lg) + j;
    const uint32_t w = rec16[s], fp = w & F_NONE, fo = w >> 16;
    if (fp < F_FAR && (fp & F_FLAG)) {
      if (ni < CR_K) r[ni] = 4u * (fp & 0x7FFFu);
      ni++;
    }
    if (fo < F_FLAG && mark[reco[s]]) {
      if (no < CR_K) r[CR_K + no] = 4u * fo;
      no++;
    }
  }
  r[0] |= (ni ? CR_INTRA : 0u) | (no ? CR_HOT : 0u) | (ni > CR_K || no > CR_K ? CR_OVF : 0u);
  for (uint32_t k = 0; k < CR_W; k++) cr[CR_W * q + k] = r[k];
}

__device__ inline void cw_sync(uint32_t* ctr, uint32_t target, bool& spun) {
  if (lane_id() == 0) __hip_atomic_fetch_add(ctr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
  uint32_t k = 0;
  while (__hip_atomic_load(ctr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) < target) {
    __builtin_amdgcn_s_sleep(1);
    if (++k > (1u << 24)) {
      spun = true;
      break;
    }
  }
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
}

// Entries b .. b+N-1 of txn q's slots (NONE past the txn's Lp slots or when !ok).
template <int N>
__device__ inline void cw_load(uint32_t (&r)[N], const uint32_t* base, uint32_t q, bool ok,
                               uint32_t lg, uint32_t b = 0) {
  const uint32_t L = 1u << lg;
  const uint32_t* src = base + ((uint64_t)q << lg) + b;
  if (ok && b + N <= L) {
    const uint4* v = (const uint4*)src;
#pragma unroll
    for (int i = 0; i < N / 4; i++) {
      const uint4 w = v[i];
      r[4 * i] = w.x;
      r[4 * i + 1] = w.y;
      r[4 * i + 2] = w.z;
      r[4 * i + 3] = w.w;
    }
  } else {
#pragma unroll
    for (int i = 0; i < N; i++) r[i] = (ok && b + i < L) ? src[i] : NONE;
  }
}

// experiments builds: a staging wave's time per step (h_m: the last stamp)
#ifdef DCC_EXPERIMENTS
#define CW_H(v)                                           \
  do {                                                    \
    const uint64_t m_ = __builtin_amdgcn_s_memrealtime(); \
    v += m_ - h_m;                                        \
    h_m = m_;                                             \
  } while (0)
#else
#define CW_H(v) ((void)0)
#endif
// The walk (see calvin_wave.h).  Iteration c: wave 0 walks chunk c while the
// staging waves (1) add chunk c-1's maxima of groups ending two or more chunks
// ahead to the global maxima, (2) read chunk c+1's records: own fields, and
// each txn's bound from groups that ended in chunk c-1 (LDS) or earlier
// (global maxima), (3) read the global maxima's share of chunk c+1's slots,
// (4) store chunk c-1's waves.  Then, between barriers: chunk c-1's region is
// flushed to the global maxima and refilled as chunk c+1's, and chunk c's
// members of groups ending in chunk c+1 add themselves.  The two roles run
// their own loops (same barrier count per iteration), so neither's registers
// are live in the other's.
//
// HELP (a.nh helper workgroups, blockIdx 1..nh): the scattered part moves to
// helpers on other CUs, a whole chunk ahead of where it is needed.  Groups
// ending exactly two chunks away go through LDS (rec2): a request whose
// previous group ended two chunks back reads chunk c-1's region while chunk
// c+1 is staged, and a member of a group ending two chunks ahead adds itself
// to that chunk's region at the boundary after its refill.  What is three or
// more chunks away goes through the global maxima: at iteration c the
// staging waves publish chunk c-1 (its region -- final once walk c-1 is done
// -- and its waves) and raise P = c; helper iteration c then adds chunk
// c-1's members to groups ending three or more chunks ahead and gathers the
// bounds of chunk c+2's requests from groups that ended three or more chunks
// back, and counts itself in R; staging iteration c+1 waits for R, loads
// chunk c+2's bounds and its maxima share, and the boundary refills the
// region without a flush.
template <int LR, bool HELP>
__global__ __launch_bounds__(CW_T) void k_cw_walk(CwPlan p, CwArgs a) {
  __shared__ uint32_t sgm[CW_ZERO + 1];
  __shared__ uint32_t sE[2][CW_CMAX];
  __shared__ uint32_t swt[2][CW_CMAX];
  __shared__ uint32_t s_ctr, s_pub;
  const uint32_t tid = threadIdx.x, lane = lane_id(), wid = tid >> 6;
  const uint32_t H = p.H, C = p.C, lg = p.lg, nch = p.nch;
  const uint32_t n = (uint32_t)a.n;
  if (HELP && blockIdx.x > 0) {
    // ---------------------------------------------------------------- helper
    const uint32_t nh = gridDim.x - 1, hid = blockIdx.x - 1, L = 1u << lg;
    uint32_t* const sEg = a.help + CW_HDATA;
    uint32_t* const wsq = sEg + (uint64_t)nch * C;
    bool spun = false;
#ifdef DCC_EXPERIMENTS
    uint64_t hw_wait = 0, hw_busy = 0, hw_m = __builtin_amdgcn_s_memrealtime();
#endif
    for (uint32_t c = 0; c + 2 < nch; c++) {
      const uint32_t c2 = c + 2, cp = c ? c - 1 : 0u;
      // (H and the stride are multiples of 64: the loop is wave-uniform, and a
      // txn's L slots sit in one wave)
      for (uint32_t l = hid * CW_T + tid, it = 0; l < H; l += nh * CW_T, it++) {
        const uint64_t s1 = (uint64_t)cp * H + l, s2 = (uint64_t)c2 * H + l;
        // the records (inputs) before the wait for the hand-off
        const uint32_t w1 = c ? a.rec16[s1] : F_NONE << 16, x1 = a.rec2[s1], o1 = a.reco[s1];
        const uint32_t w2 = a.rec16[s2], x2 = a.rec2[s2], p2 = a.recp[s2];
        if (it == 0) {  // chunks < c published
#ifdef DCC_EXPERIMENTS
          const uint64_t m0 = __builtin_amdgcn_s_memrealtime();
          hw_busy += m0 - hw_m;
#endif
          if (wid == 0 && !cw_poll(a.help, CW_HP, c)) spun = true;
          __syncthreads();
#ifdef DCC_EXPERIMENTS
          hw_m = __builtin_amdgcn_s_memrealtime();
          hw_wait += hw_m - m0;
#endif
        }
        // chunk c-1's member of a group ending three or more chunks ahead
        if ((w1 >> 16) == F_FAR && (x1 >> 16) == F_NONE)
          __hip_atomic_fetch_max(a.mg + o1, ag_ld(wsq + (uint64_t)cp * C + (l >> lg)) + 1u,
                                 __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        // chunk c+2's request after a group that ended three or more chunks back
        uint32_t v = ((w2 & F_NONE) == F_FAR && (x2 & F_NONE) == F_NONE) ? ag_ld(a.mg + p2) : 0u;
        for (uint32_t d = 1; d < L; d <<= 1) v = max(v, (uint32_t)__shfl_xor(v, d));
        if ((l & (L - 1u)) == 0) ag_st(sEg + (uint64_t)c2 * C + (l >> lg), v);
      }
      if (hid * CW_T >= H) {  // no slots this iteration: only the wait
        if (wid == 0 && !cw_poll(a.help, CW_HP, c)) spun = true;
        __syncthreads();
      }
      vm_drain();
      __syncthreads();
      if (tid == 0) __hip_atomic_fetch_add(a.help + CW_HR, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
#ifdef DCC_EXPERIMENTS
    if (a.dbg && hid == 0 && tid == 0) {
      a.dbg[14] = hw_wait;
      a.dbg[15] = hw_busy + (__builtin_amdgcn_s_memrealtime() - hw_m);
    }
#endif
    if (spun && lane == 0) atomicOr(a.err, CW_ERR_SPIN);
    return;
  }
  for (uint32_t i = tid; i < H; i += CW_T) sgm[i] = 0;
  for (uint32_t i = tid; i < C; i += CW_T) sE[0][i] = 0;
  if (tid == 0) {
    s_ctr = 0;
    s_pub = 0;
    sgm[CW_ZERO] = 0;
  }
  __syncthreads();
  if (wid == 0) {
    // ---------------------------------------------------------------- walker
    // Sub-chunk G covers sequence positions 64G .. 64G+63 (a chunk holds a
    // whole number of them); lane = txn.  A sub-chunk's records: the LDS
    // addresses of its LR previous-group reads and own-group publications and
    // (LR == 16) its compact record; three buffers, the records of sub-chunk
    // G+2 loaded while G is walked (G mod 3 picks the buffers: no copies).
    constexpr bool CMP = LR == 16;  // compact intra rounds
    constexpr int NR = 2 * LR + CR_W;
    uint32_t b0[NR], b1[CMP ? NR : 1], b2[CMP ? NR : 1];
#ifdef DCC_EXPERIMENTS
    uint64_t t_walk = 0, t_rounds = 0, t_bar = 0, n_rounds = 0;
    uint64_t n_multi = 0, n_ovf = 0, n_plain = 0;
    const uint64_t clk0 = __builtin_amdgcn_s_memtime(), rt0 = __builtin_amdgcn_s_memrealtime();
#define CW_CNT(v) v++
#else
#define CW_CNT(v) ((void)0)
#endif
    // txn q's records (an absent txn or slot: the zero slot / the lane's sink)
    const uint32_t qcap = nch * C;  // records exist for every position of every chunk
    // txn q's records; a position past the last chunk loads the last one's
    // (only a prefetch past the walk's end does, and it is never walked)
    auto load = [&](uint32_t (&r)[NR], uint32_t q) {
      const uint64_t qq = min(q, qcap - 1u);
      if constexpr (CMP) {  // Lp == LR: whole-record vector loads, no branch
#pragma unroll
        for (int i = 0; i < LR / 4; i++) {
          const uint4 x = ((const uint4*)(a.pa + (qq << lg)))[i];
          const uint4 y = ((const uint4*)(a.oa + (qq << lg)))[i];
          r[4 * i] = x.x, r[4 * i + 1] = x.y, r[4 * i + 2] = x.z, r[4 * i + 3] = x.w;
          r[LR + 4 * i] = y.x, r[LR + 4 * i + 1] = y.y, r[LR + 4 * i + 2] = y.z, r[LR + 4 * i + 3] = y.w;
        }
#pragma unroll
        for (int i = 0; i < (int)CR_W / 4; i++) {
          const uint4 z = ((const uint4*)(a.cr + (uint64_t)CR_W * qq))[i];
          r[2 * LR + 4 * i] = z.x, r[2 * LR + 4 * i + 1] = z.y, r[2 * LR + 4 * i + 2] = z.z,
                       r[2 * LR + 4 * i + 3] = z.w;
        }
      } else {
        const uint32_t L = 1u << lg;
#pragma unroll
        for (int i = 0; i < LR; i++) {
          r[i] = (uint32_t)i < L ? a.pa[(qq << lg) + i] : 4u * CW_ZERO;
          r[LR + i] = (uint32_t)i < L ? a.oa[(qq << lg) + i] : 4u * (CW_SINK + lane);
        }
      }
    };
    auto lds_ld = [&](uint32_t addr) { return *(const uint32_t*)((const char*)sgm + addr); };
    auto lds_max = [&](uint32_t addr, uint32_t v) { atomicMax((uint32_t*)((char*)sgm + addr), v); };
    // walk sub-chunk G (chunk c, LDS buffers of parity r) from cb; load G+2 into pb
    auto step = [&](uint32_t (&cb)[NR], uint32_t (&pb)[NR], uint32_t G, uint32_t c, uint32_t r) {
      if constexpr (CMP) load(pb, 64 * (G + 2) + lane);
      else load(cb, 64 * G + lane);  // (LR 32: one buffer, no prefetch)
      const uint32_t ql = 64 * G + lane - c * C;
      const bool act = 64 * G + lane < n;
      const uint32_t e = act ? sE[r][ql] : 0u;
      // first round: every previous group (all reads before the first use)
      uint32_t v[LR];
#pragma unroll
      for (int i = 0; i < LR; i++) v[i] = lds_ld(cb[i]);
      uint32_t w = e;
#pragma unroll
      for (int i = 0; i < LR; i++) w = max(w, v[i]);
      CW_CNT(n_rounds);
      const uint32_t fl = CMP ? cb[2 * LR] : CR_INTRA | CR_OVF;
      if (ballot64(act && (fl & CR_INTRA))) {
        CW_CNT(n_multi);
        if (!CMP || ballot64(act && (fl & CR_OVF))) {
          // plain rounds: every group read and published until no lane changes
          CW_CNT(n_ovf);
          for (;;) {
#pragma unroll
            for (int i = 0; i < LR; i++) lds_max(cb[LR + i], w + 1u);
#pragma unroll
            for (int i = 0; i < LR; i++) v[i] = lds_ld(cb[i]);
            uint32_t nw = e;
#pragma unroll
            for (int i = 0; i < LR; i++) nw = max(nw, v[i]);
            const bool ch = nw != w;
            w = nw;
            CW_CNT(n_rounds);
            CW_CNT(n_plain);
            if (ballot64(ch) == 0) break;
          }
        } else {
          // intra rounds: a lane's value moves only through its intra reads
          // and matters inside the sub-chunk only through its hot
          // publications; stop when no lane with one changed
          uint32_t ia[CR_K];
#pragma unroll
          for (int k = 0; k < (int)CR_K; k++) ia[k] = cb[2 * LR + k] & CR_ADDR;
          const bool hot = (fl & CR_HOT) != 0;
          for (;;) {
#pragma unroll
            for (int k = 0; k < (int)CR_K; k++) lds_max(cb[2 * LR + CR_K + k], w + 1u);
            uint32_t iv[CR_K];
#pragma unroll
            for (int k = 0; k < (int)CR_K; k++) iv[k] = lds_ld(ia[k]);
            uint32_t nw = w;
#pragma unroll
            for (int k = 0; k < (int)CR_K; k++) nw = max(nw, iv[k]);
            const bool ch = nw != w;
            w = nw;
            CW_CNT(n_rounds);
            if (ballot64(ch && hot) == 0) break;
          }
        }
      }
      // the final wave to every own group of this chunk
#pragma unroll
      for (int i = 0; i < LR; i++) lds_max(cb[LR + i], w + 1u);
      if (act) swt[r][ql] = w;
    };
    __builtin_amdgcn_s_setprio(3);
    if constexpr (CMP) {
      load(b0, lane);
      load(b1, 64 + lane);
    }
    for (uint32_t c = 0; c <= nch; c++) {
#ifdef DCC_EXPERIMENTS
      const uint64_t tw0 = __builtin_amdgcn_s_memrealtime();
#endif
      if (c < nch) {
        const uint32_t r = c & 1u, G1 = (c * C + min(C, n - c * C) + 63) / 64;
        if constexpr (CMP) {  // (a chunk is a multiple of three sub-chunks)
          for (uint32_t G = c * C / 64; G < G1; G += 3) {
            step(b0, b2, G, c, r);
            if (G + 1 < G1) step(b1, b0, G + 1, c, r);
            if (G + 2 < G1) step(b2, b1, G + 2, c, r);
          }
        } else {
          for (uint32_t G = c * C / 64; G < G1; G++) step(b0, b0, G, c, r);
        }
      }
#ifdef DCC_EXPERIMENTS
      const uint64_t tb0 = __builtin_amdgcn_s_memrealtime();
      t_walk += tb0 - tw0;
#endif
      lds_barrier();  // walk done / staging done
      if constexpr (!HELP) lds_barrier();  // region refilled (HELP: among the staging waves)
      lds_barrier();  // next-chunk members added
#ifdef DCC_EXPERIMENTS
      t_bar += __builtin_amdgcn_s_memrealtime() - tb0;
#endif
    }
#ifdef DCC_EXPERIMENTS
    if (a.dbg && lane == 0) {
      a.dbg[0] = t_walk;
      a.dbg[1] = t_rounds;
      a.dbg[2] = t_bar;
      a.dbg[3] = n_rounds;
      a.dbg[8] = __builtin_amdgcn_s_memtime() - clk0;
      a.dbg[9] = __builtin_amdgcn_s_memrealtime() - rt0;
      a.dbg[10] = n_multi;
      a.dbg[11] = n_ovf;
      a.dbg[12] = n_plain;
    }
#endif
  } else if (HELP) {
    // ------------------------------------------------- staging (with helpers)
    const uint32_t h0 = tid - 64, nh = gridDim.x - 1;
    constexpr uint32_t LG = LR == 16 ? 4u : 5u;  // == lg (cw_plan; cw_run picks LR by it)
    // buffer loads / stores, sc1 (32-bit offsets: one VGPR per access in flight)
    const __amdgpu_buffer_rsrc_t rs_mg = cw_rsrc(a.mg, (uint64_t)p.slots * 4),
                                 rs_hp = cw_rsrc(a.help, cw_help_words(p) * 4);
    const uint32_t o_sE = CW_HDATA, o_wsq = CW_HDATA + nch * C;
    // staging records' high halves (16-bit, two per word): boundary-add
    // targets of chunk c+1 (ownp), c (own) and c-1 (ownq)
    uint32_t own[CW_K / 2], ownp[CW_K / 2], ownq[CW_K / 2], ini[CW_K];
    const __amdgpu_buffer_rsrc_t rs_r2 = cw_rsrc(a.rec2, (uint64_t)p.slots * 4);
    bool spun = false;
    uint32_t target = 0;
#ifdef DCC_EXPERIMENTS
    uint64_t h_t1 = 0, h_sync = 0, h_t2 = 0, h_rest = 0, h_m = 0, h_poll = 0, h_b1 = 0, h_b2 = 0;
#endif
    auto put16 = [](uint32_t (&w)[CW_K / 2], uint32_t k, uint32_t f) {
      if (k & 1) w[k >> 1] |= f << 16;
      else w[k >> 1] = f;
    };
    auto get16 = [](const uint32_t (&w)[CW_K / 2], uint32_t k) { return (w[k >> 1] >> (16 * (k & 1))) & F_NONE; };
#pragma unroll
    for (uint32_t k = 0; k < CW_K; k++) {  // chunk 0's
      const uint32_t l = h0 + k * CW_HELP;
      put16(own, k, l < H ? a.rec2[l] >> 16 : F_NONE);
      put16(ownq, k, F_NONE);
    }
    for (uint32_t c = 0; c <= nch; c++) {
      // a fresh copy of the thread's slot base each iteration: the per-slot
      // offsets are recomputed, not hoisted out of the loop (and spilled)
      uint32_t h = h0;
      asm volatile("" : "+v"(h));
#ifdef DCC_EXPERIMENTS
      h_m = __builtin_amdgcn_s_memrealtime();
#endif
      // (A) chunk c-1 to the helpers: its region and its waves, then P = c
      if (c >= 1) {
        const uint32_t cp = c - 1, rp = cp & 1u, nqp = min(C, n - cp * C);
#pragma unroll
        for (uint32_t k = 0; k < CW_K; k++) {
          const uint32_t l = h + k * CW_HELP;
          if (l < H) cw_st_l2(rs_mg, cp * H + l, sgm[rp * H + l]);
        }
        for (uint32_t ql = h; ql < nqp; ql += CW_HELP) cw_st_l2(rs_hp, o_wsq + cp * C + ql, swt[rp][ql]);
        vm_drain();
        // the staging wave whose count completes this iteration's raises P
        // (a counter of its own: a wave may reach the sync in (B) before
        // another has counted here)
        if (lane == 0 && atomicAdd(&s_pub, 1u) == CW_HWAVES * c - 1u) ag_st(a.help + CW_HP, c);
        // the outputs (not handed off)
        for (uint32_t ql = h; ql < nqp; ql += CW_HELP) {
          const uint32_t q = cp * C + ql;
          a.wave[a.seq ? a.seq[q] : q] = swt[rp][ql];
        }
      }
      CW_H(h_t1);
      // (B) chunk c+1: its staging records; its requests' bounds from groups
      // that ended in chunk c-1 (LDS: that region is refilled only at this
      // iteration's boundary) and, once helper iteration c-1 is done, from
      // older ones (sEg) and its maxima share
      if (c + 1 < nch) {
        const uint32_t c1 = c + 1, r1 = c1 & 1u, base = c1 * H;
        uint32_t p2[CW_K / 2];  // the two-back LDS slots of chunk c+1's requests
        {
          uint32_t x[CW_K];
#pragma unroll
          for (uint32_t k = 0; k < CW_K; k++) {
            const uint32_t l = h + k * CW_HELP;
            x[k] = cw_ld(rs_r2, base + (l < H ? l : 0u));
          }
#pragma unroll
          for (uint32_t k = 0; k < CW_K; k++) {
            const bool in = h + k * CW_HELP < H;
            put16(ownp, k, in ? x[k] >> 16 : F_NONE);
            put16(p2, k, in ? x[k] & F_NONE : F_NONE);
          }
        }
#ifdef DCC_EXPERIMENTS
        const uint64_t pw0 = __builtin_amdgcn_s_memrealtime();
#endif
        if (c1 >= 2 && !cw_poll(a.help, CW_HR, nh * c)) spun = true;
        asm volatile("" ::: "memory");  // the loads below stay behind the poll
#ifdef DCC_EXPERIMENTS
        h_poll += __builtin_amdgcn_s_memrealtime() - pw0;
#endif
        CW_H(h_sync);
#pragma unroll
        for (uint32_t k = 0; k < CW_K; k++) {
          const uint32_t l = h + k * CW_HELP;
          ini[k] = cw_ld_l2(rs_mg, base + (l < H ? l : 0u));
        }
        for (uint32_t ql = h; ql < C; ql += CW_HELP)
          sE[r1][ql] = c1 >= 2 ? cw_ld_l2(rs_hp, o_sE + c1 * C + ql) : 0u;
        // every staging wave's sE stores before the LDS maxima below
        target += CW_HWAVES;
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        cw_sync(&s_ctr, target, spun);
        // (LDS reads in batches ahead of their maxima: one wait per batch)
#pragma unroll
        for (uint32_t k0 = 0; k0 < CW_K; k0 += 12) {
          uint32_t v[12];
#pragma unroll
          for (uint32_t k = 0; k < 12; k++) {
            const uint32_t x = get16(p2, k0 + k);
            v[k] = sgm[x == F_NONE ? CW_ZERO : x];
          }
#pragma unroll
          for (uint32_t k = 0; k < 12; k++)
            if (v[k]) atomicMax(&sE[r1][(h + (k0 + k) * CW_HELP) >> LG], v[k]);
        }
      } else {
#pragma unroll
        for (uint32_t k = 0; k < CW_K; k++) put16(ownp, k, F_NONE);
      }
      CW_H(h_t2);
      lds_barrier();  // walk done / staging done
      CW_H(h_b1);
      if (c + 1 < nch) {  // chunk c-1's region (published in (A)) <- chunk c+1's
        const uint32_t rn = (c + 1) & 1u;
#pragma unroll
        for (uint32_t k = 0; k < CW_K; k++) {
          const uint32_t l = h + k * CW_HELP;
          if (l < H) sgm[rn * H + l] = ini[k];
        }
      }
      // the refill before the adds: a sync of the staging waves only (the
      // walker waits for the adds)
      target += CW_HWAVES;
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      cw_sync(&s_ctr, target, spun);
      CW_H(h_b2);
      if (c < nch) {
        // chunk c's members of groups ending in chunk c+1, and chunk c-1's of
        // groups ending in chunk c+1 (its waves are still in swt until walk
        // c+1)
        const uint32_t r = c & 1u, rq = (c + 1) & 1u;
        // (LDS reads in batches ahead of their maxima: one wait per batch)
#pragma unroll
        for (uint32_t k0 = 0; k0 < CW_K; k0 += 12) {
          uint32_t wf[12], wg[12];
#pragma unroll
          for (uint32_t k = 0; k < 12; k++) {
            const uint32_t t = (h + (k0 + k) * CW_HELP) >> LG;  // (< CW_CMAX: l < CW_HPLAN)
            wf[k] = swt[r][t];
            wg[k] = swt[rq][t];
          }
#pragma unroll
          for (uint32_t k = 0; k < 12; k++) {
            const uint32_t f = get16(own, k0 + k), g = get16(ownq, k0 + k);
            if (f != F_NONE && !(f & F_FLAG)) atomicMax(&sgm[f], wf[k] + 1u);
            if (g != F_NONE && (g & F_FLAG)) atomicMax(&sgm[g & 0x7FFFu], wg[k] + 1u);
          }
        }
      }
      lds_barrier();
      CW_H(h_rest);
#pragma unroll
      for (uint32_t k = 0; k < CW_K / 2; k++) {
        ownq[k] = own[k];
        own[k] = ownp[k];
      }
    }
    if (spun && lane == 0) atomicOr(a.err, CW_ERR_SPIN);
#ifdef DCC_EXPERIMENTS
    if (a.dbg && h0 == 0) {
      a.dbg[4] = h_t1;
      a.dbg[5] = h_sync;
      a.dbg[6] = h_t2;
      a.dbg[7] = h_rest;
      a.dbg[13] = h_poll;
      a.dbg[16] = h_b1;
      a.dbg[17] = h_b2;
    }
#endif
  } else {
    // --------------------------------------------------------------- staging
    const uint32_t h = tid - 64;
    const uint64_t sb = (uint64_t)p.slots * 4;  // (cw_plan: below 2^31 bytes)
    const __amdgpu_buffer_rsrc_t rs_reco = cw_rsrc(a.reco, sb), rs_recp = cw_rsrc(a.recp, sb),
                                 rs_rec16 = cw_rsrc(a.rec16, sb), rs_mg = cw_rsrc(a.mg, sb);
    // own fields (two 16-bit fields per word): own = chunk c's (for the
    // boundary after walk c), ownp = chunk c-1's (its far maxima, during walk
    // c), then chunk c+1's; swapped after each iteration
    uint32_t own[CW_K / 2], ownp[CW_K / 2], ini[CW_K];
    uint32_t target = 0;
    bool spun = false;
#ifdef DCC_EXPERIMENTS
    uint64_t h_t1 = 0, h_sync = 0, h_t2 = 0, h_rest = 0, h_m = 0;  // staging wave 1's steps
#endif
#pragma unroll
    for (uint32_t k = 0; k < CW_K; k++) {  // chunk 0's own fields
      const uint32_t l = h + k * CW_HELP;
      const uint32_t f = l < H ? a.rec16[l] >> 16 : F_NONE;
      if (k & 1) own[k >> 1] |= f << 16;
      else own[k >> 1] = f;
    }
#pragma unroll
    for (uint32_t k = 0; k < CW_K / 2; k++) ownp[k] = NONE;
    for (uint32_t c = 0; c <= nch; c++) {
#ifdef DCC_EXPERIMENTS
      h_m = __builtin_amdgcn_s_memrealtime();
#endif
      // (0) chunk c+1's bounds start at 0 (its buffer was chunk c-1's)
      if (c + 1 < nch)
        for (uint32_t i = h; i < C; i += CW_HELP) sE[(c + 1) & 1u][i] = 0;
      // (1) chunk c-1's members of groups ending two or more chunks ahead
      // (every load issued before the first use: no branch around a load)
      if (c >= 1) {
        const uint32_t cp = c - 1;
#pragma unroll
        for (uint32_t k0 = 0; k0 < CW_K; k0 += 12) {
          bool any = false;
#pragma unroll
          for (uint32_t k = 0; k < 12; k++)
            any |= ((ownp[(k0 + k) >> 1] >> (16 * ((k0 + k) & 1))) & F_NONE) == F_FAR;
          if (!ballot64(any)) continue;  // (far groups are rare: skip the loads)
          uint32_t oc[12];
#pragma unroll
          for (uint32_t k = 0; k < 12; k++) {
            const uint32_t l = h + (k0 + k) * CW_HELP;
            oc[k] = cw_ld(rs_reco, cp * H + (l < H ? l : 0u));
          }
#pragma unroll
          for (uint32_t k = 0; k < 12; k++) {
            const uint32_t kk = k0 + k, l = h + kk * CW_HELP;
            if (((ownp[kk >> 1] >> (16 * (kk & 1))) & F_NONE) == F_FAR)
              __hip_atomic_fetch_max(a.mg + oc[k], swt[cp & 1u][l >> lg] + 1u, __ATOMIC_RELAXED,
                                     __HIP_MEMORY_SCOPE_AGENT);
          }
        }
      }
      // (the flush stores of the last boundary and these maxima, complete in
      // the L2: every reader is a wave of this workgroup, so workgroup scope --
      // an agent-scope release would write the L2 back -- and the readers'
      // loads skip the L1 (agent-scope loads))
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
      CW_H(h_t1);
      target += CW_HWAVES;
      cw_sync(&s_ctr, target, spun);
      CW_H(h_sync);
      // (2) chunk c+1's records: the own fields (replacing chunk c-1's), and
      // each request's bound from a group that ended two or more chunks back
      // -- chunk c-1's maxima are in LDS, older ones in the global maxima --
      // max-accumulated per txn in LDS; (3) the global maxima's share of
      // chunk c+1's slots
      if (c + 1 < nch) {
        const uint32_t c1 = c + 1;
        const uint64_t base = (uint64_t)c1 * H;
        // the global maxima's share first, then in two halves: the records
        // and the previous groups' codes, then every bound's source (a slot
        // without a far bound reads its own global slot) -- each half's loads
        // issued before its first use
#pragma unroll
        for (uint32_t k = 0; k < CW_K; k++) {
          const uint32_t l = h + k * CW_HELP;
          ini[k] = cw_ld_l2(rs_mg, (uint32_t)base + (l < H ? l : 0u));
        }
        constexpr uint32_t KB = CW_K / 2;
#pragma unroll
        for (uint32_t k0 = 0; k0 < CW_K; k0 += KB) {
          uint32_t w16[KB], pcs[KB], vg[KB], vl[KB];
#pragma unroll
          for (uint32_t k = 0; k < KB; k++) {
            const uint32_t l = h + (k0 + k) * CW_HELP;
            const uint32_t o = (uint32_t)base + (l < H ? l : 0u);
            w16[k] = l < H ? cw_ld(rs_rec16, o) : NONE;
            pcs[k] = cw_ld(rs_recp, o);
          }
#pragma unroll
          for (uint32_t k = 0; k < KB; k++) {
            const uint32_t kk = k0 + k, l = h + kk * CW_HELP;
            if (kk & 1) ownp[kk >> 1] |= (w16[k] >> 16) << 16;
            else ownp[kk >> 1] = w16[k] >> 16;
            const bool f = (w16[k] & F_NONE) == F_FAR;
            const uint32_t pc = pcs[k], ch = f ? pc / H : 0u;
            const bool lds = f && ch + 1 == c;
            vl[k] = sgm[lds ? ((c - 1) & 1u) * H + (pc - ch * H) : CW_ZERO];
            vg[k] = cw_ld_l2(rs_mg, f && !lds ? pc : (uint32_t)base + (l < H ? l : 0u));
            pcs[k] = lds ? 1u : f ? 2u : 0u;
          }
#pragma unroll
          for (uint32_t k = 0; k < KB; k++) {
            const uint32_t l = h + (k0 + k) * CW_HELP;
            if (pcs[k]) atomicMax(&sE[c1 & 1u][l >> lg], pcs[k] == 1u ? vl[k] : vg[k]);
          }
        }
      }
      CW_H(h_t2);
      // (4) chunk c-1's waves
      if (c >= 1) {
        const uint32_t cp = c - 1, nqp = min(C, n - cp * C);
        for (uint32_t ql = h; ql < nqp; ql += CW_HELP) {
          const uint32_t q = cp * C + ql;
          a.wave[a.seq ? a.seq[q] : q] = swt[cp & 1u][ql];
        }
      }
#ifdef DCC_EXPERIMENTS
      __builtin_amdgcn_s_waitcnt(0);
#endif
      CW_H(h_rest);
      // (the LDS barriers do not wait for global stores: the flush stores and
      // the maxima are fenced before the staging waves' next sync)
      lds_barrier();  // walk done / staging done
      {  // region of chunk c-1 -> global maxima; the same region <- chunk c+1
        const uint32_t rn = (c + 1) & 1u;
#pragma unroll
        for (uint32_t k = 0; k < CW_K; k++) {
          const uint32_t l = h + k * CW_HELP;
          if (l < H) {
            if (c >= 1) a.mg[(uint64_t)(c - 1) * H + l] = sgm[rn * H + l];
            if (c + 1 < nch) sgm[rn * H + l] = ini[k];
          }
        }
      }
      lds_barrier();
      if (c < nch) {  // chunk c's members of groups ending in chunk c+1
        const uint32_t r = c & 1u;
#pragma unroll
        for (uint32_t k = 0; k < CW_K; k++) {
          const uint32_t l = h + k * CW_HELP;
          const uint32_t f = (own[k >> 1] >> (16 * (k & 1))) & F_NONE;
          if (f < F_FAR && (f & F_FLAG)) atomicMax(&sgm[f & 0x7FFFu], swt[r][l >> lg] + 1u);
        }
      }
      lds_barrier();
#pragma unroll
      for (uint32_t k = 0; k < CW_K / 2; k++) {
        const uint32_t t = own[k];
        own[k] = ownp[k];
        ownp[k] = t;
      }
    }
    if (spun && lane == 0) atomicOr(a.err, CW_ERR_SPIN);
#ifdef DCC_EXPERIMENTS
    if (a.dbg && h == 0) {
      a.dbg[4] = h_t1;
      a.dbg[5] = h_sync;
      a.dbg[6] = h_t2;
      a.dbg[7] = h_rest;
    }
#endif
  }
}

}  // namespace

bool cw_plan(uint64_t n, uint32_t maxlen, CwPlan* p) {
  if (maxlen == 0 || maxlen > CW_LMAX || n == 0 || n >= (1ull << 26)) return false;
  // 16 slots per txn for txns of at most 16 requests (the walker's compact
  // form), else 32; a chunk is a multiple of three 64-txn sub-chunks
  const uint32_t lg = maxlen <= 16 ? 4u : 5u;
  const uint32_t C = std::min<uint32_t>(CW_CMAX, CW_HPLAN >> lg) / 192u * 192u;
  const uint64_t nch = (n + C - 1) / C;
  p->lg = lg;
  p->C = C;
  p->H = C << lg;
  p->nch = (uint32_t)nch;
  p->slots = nch * p->H;
  return p->slots * 4 < 0x7FFFFFFFull;  // (the staging waves' 32-bit buffer offsets)
}

hipError_t cw_run(const CwPlan& p, const CwArgs& a, hipStream_t st) {
  if (a.seq) k_cw_seqpos<<<(unsigned)((a.n + 255) / 256), 256, 0, st>>>(a.seq, a.n, a.seqpos);
  k_cw_link<<<(unsigned)((p.slots + 255) / 256), 256, 0, st>>>(LinkArgs{p, a});
  hipError_t e = hipMemsetAsync(a.mg, 0, p.slots * 4, st);
  if (e != hipSuccess) return e;
  e = hipMemsetAsync(a.mark, 0, p.slots, st);
  if (e != hipSuccess) return e;
  k_cw_mark<<<(unsigned)((p.slots + 255) / 256), 256, 0, st>>>(a.rec16, a.recp, p.slots, a.mark);
  const uint64_t nq = (uint64_t)p.nch * p.C;
  if (p.lg == 4)
    k_cw_cr<<<(unsigned)((nq + 255) / 256), 256, 0, st>>>(a.rec16, a.reco, a.mark, nq, p.lg, a.cr);
  if (a.nh && a.rec2 && p.nch > 2) {
    // the walker's workgroup and a.nh helpers (each a CU of its own: the
    // kernel's LDS); the helpers' counters start at 0
    e = hipMemsetAsync(a.help, 0, CW_HDATA * 4, st);
    if (e != hipSuccess) return e;
    if (p.lg <= 4)
      k_cw_walk<16, true><<<1 + a.nh, CW_T, 0, st>>>(p, a);
    else
      k_cw_walk<32, true><<<1 + a.nh, CW_T, 0, st>>>(p, a);
  } else if (p.lg <= 4) {
    k_cw_walk<16, false><<<1, CW_T, 0, st>>>(p, a);
  } else {
    k_cw_walk<32, false><<<1, CW_T, 0, st>>>(p, a);
  }
  return hipGetLastError();
}

}  // namespace dcc
