// pack_dev.h — the packed small-frontier search (included by search.hip after
// search_dev.h).
//
// Most histories of a DST batch have a tiny frontier (C4: at most 1
// configuration in 93 % of histories, at most 4 in 99.8 %), so a workgroup- or
// wave-per-history kernel leaves 60+ of 64 lanes idle and is VALU-issue bound
// (round-1 PROF build: ~38k cycles per round, 64 % of them in a one-lane
// closure). Here a GROUP of L lanes (L = 8, 16 or 32, a power of two >= K)
// owns one history, so a wave checks 64/L histories at once (C4: K <= 8, eight
// histories per wave), and inside a group lane l owns chain l:
//   - expand: lane l tries the head of chain l as the next non-identity op
//     (the candidates of porcupine's checkSingle loop, upstream checker.go),
//     folding the record hashes (main.go:227-244) only when the tail matches;
//   - closure: every pass is one head load per lane plus a group min-reduce of
//     the heads' return events (minret) and required tails (P1 bound); legal
//     minimal identity ops advance in parallel (rule 1);
//   - children are consumed one at a time straight from the producing lane
//     (shuffles), closed by the whole group and deduplicated against the next
//     frontier (at most F configurations in LDS) by a lane-parallel compare.
// A history whose frontier outgrows F is flagged S2LC_R_FRONTIER and re-run by
// search_kernel's HBM-slab passes. Each lane caches the record at its chain's
// last count in registers, so a chain that did not move costs no load.
//
// All control flow that reaches a cross-lane operation is uniform within a
// group (lanes l >= K take part with a null chain), so ballots and shuffles
// never read a disabled lane. Groups of one wave diverge freely.
#pragma once
#include <type_traits>

namespace s2lc {
namespace {

constexpr int PACK_F = 8;       // frontier capacity per group (configurations)
#ifndef S2LC_PACK_PF
#define S2LC_PACK_PF 8
#endif
constexpr int PACK_PF = S2LC_PACK_PF;  // record hashes prefetched per lane for the next round's first expansion

// fold with the first PACK_PF hashes already in registers
__device__ __forceinline__ uint64_t fold_hashes_pf(uint64_t h, const uint64_t (&pf)[PACK_PF],
                                                   const uint64_t* __restrict__ rs, uint32_t n) {
#pragma unroll
  for (int q = 0; q < PACK_PF; ++q)
    if ((uint32_t)q < n) h = chain_hash(h, pf[q]);
  return n > (uint32_t)PACK_PF ? fold_hashes_blk(h, rs + PACK_PF, n - PACK_PF) : h;
}
constexpr int PACK_BLOCK = 256; // threads per workgroup
// per-launch totals (Params::agg[0..7]): the run's statistics without reading
// every history's result back (batch_run's fast path)
enum { PACK_AGG_CONFIGS, PACK_AGG_CHILDREN, PACK_AGG_ROUNDS, PACK_AGG_SEARCH_BYTES, PACK_AGG_OVERFLOW, PACK_AGG_SETTLED };

template <int L>
struct __attribute__((aligned(8))) PCfg {
  uint64_t tail;
  uint64_t hash;
  uint32_t tok;
  uint32_t minret;  // exact minret of the closed configuration
  uint32_t trace;   // own trace index
  uint32_t ptrace;  // parent's trace index
  uint32_t move;    // move that produced it
  uint32_t _pad;
  uint16_t cnt[L];
};

template <int L>
constexpr size_t pack_group_bytes() { return 2 * PACK_F * sizeof(PCfg<L>); }

template <int L>
constexpr size_t pack_smem_bytes() { return (PACK_BLOCK / L) * pack_group_bytes<L>(); }

// LDS accesses of one wave execute in program order; this keeps the compiler
// from reordering them across lanes (a store by lane a, a load by lane b).
__device__ __forceinline__ void wave_lds_sync() {
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  __builtin_amdgcn_wave_barrier();
}

// Group min-reductions. A 16-lane group is one DPP row: quad_perm [1,0,3,2],
// quad_perm [2,3,0,1], row_ror:4, row_ror:8 leave the row minimum in every
// lane with VALU data-parallel moves (no LDS round trip, unlike ds_bpermute,
// which __shfl_xor compiles to). An 8-lane group (half a row) ends with
// row_half_mirror; a 32-lane group adds one bpermute (lane ^ 16).
template <int CTRL>
__device__ __forceinline__ uint32_t dpp_u32(uint32_t v) {
  return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, CTRL, 0xF, 0xF, false);
}
template <int CTRL>
__device__ __forceinline__ uint64_t dpp_min_u64(uint64_t v) {
  const uint64_t w = ((uint64_t)dpp_u32<CTRL>((uint32_t)(v >> 32)) << 32) | dpp_u32<CTRL>((uint32_t)v);
  return w < v ? w : v;
}

template <int L>
__device__ __forceinline__ uint32_t gmin_u32(uint32_t v) {
  v = min(v, dpp_u32<0xB1>(v));
  v = min(v, dpp_u32<0x4E>(v));
  if (L == 8) return min(v, dpp_u32<0x141>(v));  // row_half_mirror: the other quad of the 8-lane group
  v = min(v, dpp_u32<0x124>(v));
  v = min(v, dpp_u32<0x128>(v));
  if (L == 32) v = min(v, (uint32_t)__shfl_xor((int)v, 16, 64));
  return v;
}

template <int L>
__device__ __forceinline__ uint64_t gmin_u64(uint64_t v) {
  v = dpp_min_u64<0xB1>(v);
  v = dpp_min_u64<0x4E>(v);
  if (L == 8) return dpp_min_u64<0x141>(v);
  v = dpp_min_u64<0x124>(v);
  v = dpp_min_u64<0x128>(v);
  if (L == 32) {
    const uint32_t lo = (uint32_t)__shfl_xor((int)(uint32_t)v, 16, 64);
    const uint32_t hi = (uint32_t)__shfl_xor((int)(uint32_t)(v >> 32), 16, 64);
    const uint64_t w = ((uint64_t)hi << 32) | lo;
    v = w < v ? w : v;
  }
  return v;
}

__device__ __forceinline__ uint32_t bcast_u32(uint32_t v, int src) { return (uint32_t)__shfl((int)v, src, 64); }
__device__ __forceinline__ uint64_t bcast_u64(uint64_t v, int src) {
  return ((uint64_t)bcast_u32((uint32_t)(v >> 32), src) << 32) | bcast_u32((uint32_t)v, src);
}

// Per-lane view of chain l of the group's history with a register window of
// PACK_W consecutive records. A closure that advances a chain by several
// identity ops, and the next rounds' expansions, read them from registers: a
// window refill issues PACK_W independent loads (one memory latency) where a
// one-record cache paid one dependent latency per advanced op. Two records
// (161 VGPRs: 3 waves per SIMD) beat four (193: 2 waves) on C4 by 1-4 %
// (tools/variant_sweep.sh, profiles/r03/pack_variants.txt); every record a
// pass selects costs 16 v_cndmask per extra window slot.
#ifndef S2LC_PACK_W
#define S2LC_PACK_W 2
#endif
constexpr int PACK_W = S2LC_PACK_W;
// Read-ahead: a window refill at count c also loads one dword of records
// c+PD .. c+PD+PN-1 (the lines of the chain's next window), so that the next
// refill finds them in L2 instead of HBM. The dwords are consumed (folded into
// sink) only at the refill after, by when they have long arrived, and sink is
// consumed by an empty asm at the history's end. C4 10k launch
// (tools/pack_ab.sh, profiles/r05/pack_readahead.txt): 1.363 -> 1.287 ms at
// PD = 2, PN = 2; PN = 4 / 8 and PD = 3 / 4 are no better, and touching the
// next record's hashes as well (PH = 1) is slower (1.455 ms): vmcnt retires
// in order, so a later load that misses to HBM delays every wait behind it.
#ifndef S2LC_PACK_PD
#define S2LC_PACK_PD 2
#endif
constexpr int PACK_PD = S2LC_PACK_PD;  // read-ahead distance (records); 0 = off
#ifndef S2LC_PACK_PN
#define S2LC_PACK_PN 2
#endif
constexpr int PACK_PN = S2LC_PACK_PN;  // read-ahead records per refill
#ifndef S2LC_PACK_PH
#define S2LC_PACK_PH 0
#endif
constexpr int PACK_PH = S2LC_PACK_PH;  // 1: a refill also touches the window's second record's hashes
template <bool SMALL>
struct ChainLane {
  using Rec = typename std::conditional<SMALL, SRec, OpRec>::type;
  static constexpr int NW = SMALL ? 2 : 4;  // uint4 words per record
  const Rec* __restrict__ base;    // first record of chain l (valid iff on)
  bool on;                         // l < K
  uint32_t len;                    // records of chain l, its sentinel included
  uint32_t w0;                     // count of the window's first record
  uint32_t cc;                     // count of r
  uint4 w[PACK_W][NW];             // window: records at counts w0 .. w0+PACK_W-1
  OpRec r;                         // record at count cc (null record when !on)
  uint32_t pfx[PACK_PN];           // read-ahead dwords of the last refill (PACK_PD)
  uint32_t sink;                   // read-ahead dwords consumed
  uint32_t phx;                    // PACK_PH read-ahead dword
  const uint32_t* pool32;          // the hash pool (PACK_PH)
#ifdef S2LC_PROF
  bool refilled;                   // the last at() reloaded the window
#endif
  __device__ __forceinline__ void reset(const Rec* b, bool on_, uint32_t len_) {
    base = b;
    on = on_;
    len = len_;
    w0 = 0xFFFF0000u;
    cc = 0xFFFFFFFFu;
#pragma unroll
    for (int i = 0; i < PACK_PN; ++i) pfx[i] = 0;
    sink = 0;
    phx = 0;
    r.num_records = 0; r.msn = 0; r.out_tail = 0; r.out_hash = 0;
    r.sufmin = REQ_NONE; r.call_ev = EV_INF; r.ret_ev = EV_INF;
    r.hash_off = 0; r.hash_cnt = 0; r.batch_tok = 0; r.set_tok = 0;
    r.flags = OPF_SENTINEL;
  }
  __device__ __forceinline__ void at(uint32_t c) {
#ifdef S2LC_PROF
    refilled = false;
#endif
    if (!on || c == cc) return;
    uint32_t o = c - w0;
    if (o >= (uint32_t)PACK_W) {
#ifdef S2LC_PROF
      refilled = true;
#endif
      // clamp to the chain: a record past its sentinel is never selected
      const Rec* q = base + c;
      const uint32_t last = len - 1 - c;  // c < len always (sentinel included)
#pragma unroll
      for (int i = 0; i < PACK_W; ++i) {
        const uint4* qi = reinterpret_cast<const uint4*>(q + min((uint32_t)i, last));
#pragma unroll
        for (int k = 0; k < NW; ++k) w[i][k] = qi[k];
      }
      if (PACK_PD > 0) {
#pragma unroll
        for (int i = 0; i < PACK_PN; ++i) sink ^= pfx[i];
#pragma unroll
        for (int i = 0; i < PACK_PN; ++i)
          pfx[i] = *reinterpret_cast<const uint32_t*>(q + min((uint32_t)(PACK_PD + i), last));
      }
      if constexpr (PACK_PH && !SMALL) {
        sink ^= phx;
        phx = w[1][3].y ? pool32[2 * w[1][3].x] : 0u;  // hash_cnt, hash_off of record c+1
      }
      w0 = c;
      o = 0;
    }
    // select dword-wise in registers (a struct-typed select goes through scratch)
    uint4 sel[NW];
#pragma unroll
    for (int k = 0; k < NW; ++k) {
      sel[k] = w[0][k];
#pragma unroll
      for (int i = 1; i < PACK_W; ++i) {
        const bool t = o == (uint32_t)i;
        sel[k].x = t ? w[i][k].x : sel[k].x;
        sel[k].y = t ? w[i][k].y : sel[k].y;
        sel[k].z = t ? w[i][k].z : sel[k].z;
        sel[k].w = t ? w[i][k].w : sel[k].w;
      }
    }
    if constexpr (SMALL) {  // widen (search.h, SRec)
      r.out_hash = (uint64_t)sel[0].x | ((uint64_t)sel[0].y << 32);
      r.hash_off = sel[0].z;
      r.num_records = sel[0].w & 0xFFFFu;
      // msn / out_tail 0xFFFF and a bound 0xFFFD stay as they are: no
      // reachable tail (<= 65,532) equals or passes them; REQ_NONE,
      // REQ_HASH_ONLY and EV_INF widen to their 64 / 32-bit values
      const uint32_t sf = sel[1].x >> 16;
      r.msn = sel[0].w >> 16;
      r.out_tail = sel[1].x & 0xFFFFu;
      r.sufmin = (uint64_t)sf | (sf >= 0xFFFEu ? 0xFFFFFFFFFFFF0000ull : 0ull);
      const uint32_t ce = sel[1].y & 0xFFFFu, re = sel[1].y >> 16;
      r.call_ev = ce | (ce == 0xFFFFu ? 0xFFFF0000u : 0u);
      r.ret_ev = re | (re == 0xFFFFu ? 0xFFFF0000u : 0u);
      r.hash_cnt = sel[1].z & 0xFFFFu;
      r.flags = sel[1].z >> 16;
      r.batch_tok = (uint16_t)(sel[1].w & 0xFFFFu);
      r.set_tok = (uint16_t)(sel[1].w >> 16);
    } else {
      __builtin_memcpy(&r, sel, sizeof(OpRec));
    }
    cc = c;
  }
};

// Group closure of one configuration (state s, lane count cnt) under minimal,
// legal identity ops + P1/P2/P4; returns CL_* and the exact minret.
template <int L, class CL>
__device__ __forceinline__ int pack_closure(CL& ch, const uint64_t* __restrict__ pool, uint32_t& cnt,
                                            const State& s, uint32_t hflags,
                                            uint64_t gmask, uint32_t& minret_out,
                                            unsigned long long* prof_pass = nullptr) {
  const bool nowrap = hflags & H_NOWRAP;
  const bool p2 = hflags & H_P2OK;
  const bool p4 = hflags & H_P4;
  for (;;) {
    ch.at(cnt);
#ifdef S2LC_PROF
    if (prof_pass) {  // [0] passes, [1] passes that reloaded a window (the group waited on memory)
      prof_pass[0]++;
      if (__ballot(ch.refilled) & gmask) prof_pass[1]++;
    }
#endif
    const OpRec& r = ch.r;
    const uint32_t minret = gmin_u32<L>(r.ret_ev);
    // P1 bound in 32 bits (H_TAIL32 histories only: every reachable tail is
    // below 2^32 - 3): REQ_NONE -> 0xFFFFFFFF, REQ_HASH_ONLY -> 0xFFFFFFFE, a
    // larger requirement (never reachable) -> 0xFFFFFFFD; one DPP min per step
    const uint32_t s_lo = (uint32_t)r.sufmin, s_hi = (uint32_t)(r.sufmin >> 32);
    const uint32_t b32 = s_hi == 0 ? min(s_lo, 0xFFFFFFFDu)
                         : s_hi == 0xFFFFFFFFu && s_lo >= 0xFFFFFFFEu ? s_lo : 0xFFFFFFFDu;
    const uint32_t bound = gmin_u32<L>(b32);
    const uint32_t f = r.flags;
    const bool minimal_e = (f & OPF_CLS_E) && r.call_ev < minret;
    bool legal = false, dead = false;
    if (minimal_e) {
      legal = true;
      if ((f & OPF_KIND_MASK) != 0) {
        const bool hash_bad = (f & OPF_HAS_HASH) && s.hash != r.out_hash;
        const bool tail_bad = !(f & OPF_FAIL) && s.tail != r.out_tail;
        legal = !hash_bad && !tail_bad;
        // P2: a minimal successful read at this tail with another hash can never pass
        dead = p2 && hash_bad && !(f & OPF_FAIL) && r.out_tail == s.tail;
      }
    }
    minret_out = minret;
    if ((__ballot(dead) & gmask) || (nowrap && s.tail > (uint64_t)bound)) return CL_DEAD;
    if (!(__ballot(legal) & gmask)) {
      if (minret == EV_INF) return CL_COMPLETE;
      return (p4 && bound == 0xFFFFFFFFu) ? CL_P4 : CL_ALIVE;
    }
    cnt += legal ? 1u : 0u;
  }
}

// S2LC_PROF: per-phase cycle counts of the pack kernel (lane 0 of each group),
// summed into g_prof[10..15]: expand, closure, dedupe+insert, rounds, closure
// passes, children.
#ifdef S2LC_PROF
#define PK_T0() pk_t = clock64()
#define PK_LAP(i) do { const unsigned long long t_ = clock64(); pk_acc[i] += t_ - pk_t; pk_t = t_; } while (0)
#else
#define PK_T0() do { } while (0)
#define PK_LAP(i) do { } while (0)
#endif

#ifndef S2LC_PACK_MINW
#define S2LC_PACK_MINW 1
#endif
template <int L, bool SMALL = false>
__global__ __launch_bounds__(PACK_BLOCK, S2LC_PACK_MINW) void pack_kernel(Params p) {
#ifdef S2LC_PROF
  unsigned long long pk_acc[6] = {0, 0, 0, 0, 0, 0};
  unsigned long long pk_pass[2] = {0, 0};
  unsigned long long pk_t = 0;
#endif
  using C = PCfg<L>;
  S2LC_DYNAMIC_LDS(smem);
  const int lane = (int)(threadIdx.x & 63);
  const int gl = lane & (L - 1);           // lane within the group = chain index
  const int gbase = lane & ~(L - 1);       // first wave lane of the group
  const uint64_t gmask = (L == 64 ? ~0ull : ((1ull << L) - 1)) << gbase;
  C* const fr = reinterpret_cast<C*>(smem + (threadIdx.x / L) * pack_group_bytes<L>());

  // Only the first gpw groups of each wave take histories: the groups of a
  // wave run in lockstep (every round costs the wave the most any of its
  // groups spends), so fewer histories per wave shorten every round, at the
  // price of fewer histories in flight (the host picks gpw from the batch)
  if (p.zero_ctr && blockIdx.x == 0 && threadIdx.x < 32) {  // the next run's counters (this run uses the other set)
    p.zero_ctr[threadIdx.x] = 0;
    p.zero_agg[threadIdx.x] = 0;
  }
  if (p.gpw && (uint32_t)(lane / L) >= p.gpw) return;
  uint32_t tbase = 0, tleft = 0;  // group's trace chunk (uniform)
  // this group's totals (lane gl == 0), added to p.agg once at the end
  unsigned long long a_cfg = 0, a_ch = 0, a_rounds = 0, a_bytes = 0, a_ovf = 0, a_set = 0;
  for (;;) {
    uint32_t hi = 0;
    if (gl == 0) hi = atomicAdd(p.counter, 1u);
    hi = bcast_u32(hi, gbase);
    if (hi >= p.n_hist) break;
    const uint32_t h = p.order[hi];
    const HistDesc hd = p.hist[h];
    const int K = hd.K;
    if (K > L) {  // never listed by the host; re-run by a workgroup pass if it were
      if (gl == 0) { p.res[h].verdict = V_UNKNOWN; p.res[h].reason = S2LC_R_FRONTIER; }
      continue;
    }
    const bool on = gl < K;
    const bool idefer = hd.flags & H_IDEFER;
    const uint64_t deadline = p.deadline ? *p.deadline : 0ull;
    uint32_t* const rc = p.rcounts ? p.rcounts + p.res[h].witness_off : nullptr;
    const uint32_t cs = on ? p.chain_start[hd.cs_base + gl] : 0u;
    const uint32_t ce = on ? p.chain_start[hd.cs_base + gl + 1] : 0u;
    ChainLane<SMALL> ch;
    if constexpr (SMALL) ch.reset(p.srecs + cs, on, ce - cs);
    else ch.reset(p.recs + cs, on, ce - cs);
    ch.pool32 = reinterpret_cast<const uint32_t*>(p.pool);
    bool witness_ok = p.witness != 0;
    // the first record hashes of this lane's head in the next round's first
    // configuration, loaded right after that configuration's closure so the
    // load overlaps the round's dedupe / insert / bookkeeping (pf_cc: the count
    // they belong to; PACK_PF hashes)
    uint64_t pf[PACK_PF];
    uint32_t pf_cc = 0xFFFFFFFFu;
    // witness moves: while every round leaves exactly one configuration the
    // path is the sequence of those configurations' moves, written as the
    // rounds go (rounds 1 .. lin_len); from the first round that keeps several
    // configurations on, their trace entries are written and lane 0 walks the
    // parent chain at the end, down to round lin_len + 1. A history that stays
    // linear (93 % of C4) writes no trace entry at all.
    uint32_t* const wout = p.moves ? p.moves + p.res[h].witness_off : nullptr;
    bool linear = wout != nullptr;
    uint32_t lin_len = 0;

    uint32_t verdict = V_ILLEGAL, reason = S2LC_R_SEARCH_EXHAUSTED;
    uint32_t found_parent = TRACE_NONE, found_move = TRACE_NONE, found_p4 = 0;
    uint32_t deep_trace = TRACE_NONE, deep_len = 0;
    uint64_t configs = 0, children = 0;
    uint32_t rounds = 0;
    int cur = 0;  // frontier parity: fr[cur*F ..] current, fr[(1-cur)*F ..] next
    uint32_t nf = 0;

    // ---- round 0: the initial configuration (∅, (0, 0, nil)) -------------
    {
      uint32_t cnt = 0, mr = 0;
      const State s0{0, 0, 0};
      const int cr = pack_closure<L>(ch, p.pool, cnt, s0, hd.flags, gmask, mr);
      if (cr == CL_DEAD) {
        nf = 0;
      } else if (cr != CL_ALIVE) {
        verdict = V_OK; reason = 0; found_p4 = cr == CL_P4;
        nf = 0xFFFFFFFFu;  // done
      } else {
        C& c = fr[0];
        if (gl == 0) {
          c.tail = 0; c.hash = 0; c.tok = 0; c.minret = mr;
          c.trace = TRACE_NONE; c.ptrace = TRACE_NONE; c.move = TRACE_NONE;
        }
        if (gl < L) c.cnt[gl] = on ? (uint16_t)cnt : 0;
        nf = 1;
        configs = 1;
        if (rc && gl == 0) rc[0] = 1;
      }
      wave_lds_sync();
    }

    // ---- rounds: each linearizes one durable / indefinite append ----------
    while (nf != 0 && nf != 0xFFFFFFFFu) {
      // s_memrealtime is a scalar read: the same value in every lane of the wave
      if (deadline && wall_clock64() > deadline) { verdict = V_UNKNOWN; reason = S2LC_R_TIMEOUT; break; }
      C* const curf = fr + cur * PACK_F;
      C* const nxt = fr + (1 - cur) * PACK_F;
      uint32_t nn = 0;
      bool found = false, overflow = false;
      for (uint32_t f = 0; f < nf && !found && !overflow; ++f) {
        const C& pc = curf[f];
        const State s{pc.tail, pc.hash, pc.tok};
        const uint32_t pmin = pc.minret;
        const uint32_t ptrace = pc.trace;
        const uint32_t pcnt = on ? pc.cnt[gl] : 0u;
        PK_T0();
        // expand: lane l tries the head of chain l
        ch.at(pcnt);
        const OpRec& r = ch.r;
        const bool cand = on && !(r.flags & (OPF_SENTINEL | OPF_CLS_E)) && r.call_ev < pmin;
        bool take_opt = false, take_id = false, pre_dead = false;
        State opt = s;
        // P1 precheck: the smallest required tail among the OTHER chains'
        // heads (the group's smallest, or its second smallest in the lane
        // holding the smallest). Lane j's opt child above it is dead at its
        // closure's first pass (that pass's bound is the min over the same
        // heads and chain j's next one, never larger), so it is counted as a
        // child and dropped here: no broadcast, closure pass or window load
        uint32_t p1x = 0xFFFFFFFFu;
        if (hd.flags & H_NOWRAP) {
          const uint32_t s_lo = (uint32_t)r.sufmin, s_hi = (uint32_t)(r.sufmin >> 32);
          const uint32_t b32 = s_hi == 0 ? min(s_lo, 0xFFFFFFFDu)
                               : s_hi == 0xFFFFFFFFu && s_lo >= 0xFFFFFFFEu ? s_lo : 0xFFFFFFFDu;
          const uint32_t m1 = gmin_u32<L>(b32);
          const int fl = __ffsll((unsigned long long)(__ballot(b32 == m1) & gmask)) - 1;
          const uint32_t m2 = gmin_u32<L>(lane == fl ? 0xFFFFFFFFu : b32);
          p1x = lane == fl ? m2 : m1;
        }
        if (cand) {
          const bool g = append_guards_ok(r, s);
          opt.tail = s.tail + r.num_records;
          opt.tok = r.set_tok ? r.set_tok : s.tok;
          if (r.flags & OPF_CLS_D) {
            take_opt = g && opt.tail == r.out_tail;
          } else {
            take_opt = g;
          }
          if (take_opt && opt.tail > (uint64_t)p1x) { take_opt = false; pre_dead = true; }
          if (take_opt) {
            if (f == 0 && pcnt == pf_cc)
              opt.hash = fold_hashes_pf(s.hash, pf, p.pool + r.hash_off, r.hash_cnt);
            else
              opt.hash = fold_hashes_blk(s.hash, p.pool + r.hash_off, r.hash_cnt);
          }
          if (r.flags & OPF_CLS_I) take_id = (!idefer || r.ret_ev == pmin) && !(g && state_eq(opt, s));
        }
        PK_LAP(0);
        uint64_t mo = __ballot(take_opt) & gmask;
        uint64_t mi = __ballot(take_id) & gmask;
        children += __popcll(mo) + __popcll(mi) + __popcll(__ballot(pre_dead) & gmask);
        // consume the children one at a time: close, dedupe, insert
        while ((mo | mi) && !found && !overflow) {
          const bool is_id = mo == 0;
          const uint64_t m = is_id ? mi : mo;
          const int src = __ffsll((unsigned long long)m) - 1;
          if (is_id) mi &= mi - 1; else mo &= mo - 1;
          const int j = src - gbase;
          State ks;
          ks.tail = bcast_u64(is_id ? s.tail : opt.tail, src);
          ks.hash = bcast_u64(is_id ? s.hash : opt.hash, src);
          ks.tok = bcast_u32(is_id ? s.tok : opt.tok, src);
          uint32_t cnt = pcnt + (gl == j ? 1u : 0u);
          uint32_t mr = 0;
          PK_LAP(2);
#ifdef S2LC_PROF
          const int cr = pack_closure<L>(ch, p.pool, cnt, ks, hd.flags, gmask, mr, pk_pass);
#else
          const int cr = pack_closure<L>(ch, p.pool, cnt, ks, hd.flags, gmask, mr);
#endif
          if (cr == CL_ALIVE && nn == 0) {
            // this child becomes the next round's first configuration: start
            // loading its candidate heads' record hashes now
            const OpRec& hr = ch.r;  // the head at cnt (the closure's last pass selected it)
            pf_cc = 0xFFFFFFFFu;
            if (on && !(hr.flags & (OPF_SENTINEL | OPF_CLS_E)) && hr.call_ev < mr) {
              const uint64_t* src = p.pool + hr.hash_off;
#pragma unroll
              for (int q = 0; q < PACK_PF; ++q) pf[q] = (uint32_t)q < hr.hash_cnt ? src[q] : 0ull;
              pf_cc = cnt;
            }
          }
          PK_LAP(1);
          const uint32_t mv = is_id ? ((uint32_t)j | MOVE_IDENT) : (uint32_t)j;
          if (cr == CL_COMPLETE || cr == CL_P4) {
            found = true;
            found_parent = ptrace; found_move = mv; found_p4 = cr == CL_P4;
            break;
          }
          if (cr == CL_DEAD) continue;
          // dedupe against the next frontier
          bool dup = false;
          for (uint32_t e = 0; e < nn; ++e) {
            const C& o = nxt[e];
            if (o.tail != ks.tail || o.hash != ks.hash || o.tok != ks.tok) continue;
            const bool ne = on && o.cnt[gl] != (uint16_t)cnt;
            if (!(__ballot(ne) & gmask)) { dup = true; break; }
          }
          if (dup) continue;
          if (nn == PACK_F) { overflow = true; break; }
          C& o = nxt[nn];
          if (gl == 0) {
            o.tail = ks.tail; o.hash = ks.hash; o.tok = ks.tok; o.minret = mr;
            o.ptrace = ptrace; o.move = mv;
          }
          o.cnt[gl] = on ? (uint16_t)cnt : 0;
          wave_lds_sync();
          ++nn;
        }
      }
      PK_LAP(2);
      if (found) { verdict = V_OK; reason = 0; rounds++; break; }
      if (overflow) { verdict = V_UNKNOWN; reason = S2LC_R_FRONTIER; break; }
      rounds++;
      if (rc && gl == 0) rc[rounds] = nn;
      if (linear && nn == 1 && gl == 0) wout[rounds - 1] = nxt[0].move;
      if (linear && nn == 1) lin_len = rounds;
      if (nn > 1) linear = false;
      if (nn == 0) {
        verdict = V_ILLEGAL; reason = S2LC_R_SEARCH_EXHAUSTED;
        deep_trace = curf[0].trace;  // a configuration of the deepest non-empty round
        deep_len = rounds - 1;
        break;
      }
      // trace entries (parent, move) of the surviving configurations
      uint32_t tb = TRACE_NONE;
      if (witness_ok && !linear) {
        if (tleft < nn) {
          unsigned long long b = 0;
          if (gl == 0) b = atomicAdd(p.trace_head, (unsigned long long)TRACE_CHUNK);
          b = bcast_u64(b, gbase);
          if (b + TRACE_CHUNK <= p.trace_cap) { tbase = (uint32_t)b; tleft = TRACE_CHUNK; }
          else { witness_ok = false; tleft = 0; }
        }
        if (witness_ok) { tb = tbase; tbase += nn; tleft -= nn; }
      }
      if ((uint32_t)gl < nn) {
        C& o = nxt[gl];
        if (tb != TRACE_NONE) {
          o.trace = tb + gl;
          p.trace[tb + gl] = TraceEnt{o.ptrace, o.move};
        } else {
          o.trace = TRACE_NONE;
        }
      }
      wave_lds_sync();
      configs += nn;
      if (p.max_configs && configs > p.max_configs) { verdict = V_UNKNOWN; reason = S2LC_R_BUDGET; break; }
      cur = 1 - cur;
      nf = nn;
    }
    if (PACK_PD > 0) {  // the read-ahead's last loads
#pragma unroll
      for (int i = 0; i < PACK_PN; ++i) ch.sink ^= ch.pfx[i];
      asm volatile("" ::"v"(ch.sink ^ ch.phx));
    }
#ifdef S2LC_PROF
    if (gl == 0) {
      for (int i_ = 0; i_ < 3; ++i_) { atomicAdd(&g_prof[10 + i_], pk_acc[i_]); pk_acc[i_] = 0; }
      atomicAdd(&g_prof[13], (unsigned long long)rounds);
      atomicAdd(&g_prof[8], pk_pass[0]);
      atomicAdd(&g_prof[9], pk_pass[1]);
      pk_pass[0] = pk_pass[1] = 0;
      atomicAdd(&g_prof[15], (unsigned long long)children);
    }
#endif
    if (gl == 0) {
      if (verdict == V_UNKNOWN && reason == S2LC_R_FRONTIER) {
        ++a_ovf;
      } else {
        const uint64_t S = 8 * ((2 * (uint64_t)K + 20 + 7) / 8);  // DESIGN.md §5 accounting
        a_cfg += configs; a_ch += children; a_rounds += rounds; ++a_set;
        a_bytes += 2 * S * configs + 8 * children;
      }
      HistResult& R = p.res[h];
      R.verdict = verdict;
      R.reason = reason;
      R.rounds = rounds;
      R.configs = configs;
      R.children = children;
      R.p4 = found_p4;
      R.final_parent = (verdict == V_OK && witness_ok) ? found_parent : TRACE_NONE;
      R.final_move = found_move;
      R.witness_len = 0;
      // (a history linear to the end has its whole path in wout already: no trace entry)
      const bool deep = verdict == V_ILLEGAL && witness_ok && (linear ? deep_len > 0 : deep_trace != TRACE_NONE);
      R.deep_trace = deep ? (linear ? 0u : deep_trace) : TRACE_NONE;
      R.deep_len = deep_len;
      const bool want = (verdict == V_OK || deep) && witness_ok;
      uint32_t hw = 0;
      if (want && wout) {
        // Ok: the completing move after the path to its parent; Illegal: the
        // path to a configuration of the deepest non-empty round (walk_kernel's
        // output, produced here)
        uint32_t len, pos, idx;
        if (verdict == V_OK) {
          len = found_move == TRACE_NONE ? 0u : rounds;
          if (len) wout[len - 1] = found_move;
          pos = len ? len - 1 : 0;
          idx = found_parent;
        } else {
          len = deep_len;
          pos = len;
          idx = deep_trace;
        }
        if (linear) {
          pos = 0;  // rounds 1 .. len-1 (Ok) / 1 .. len (Illegal) were written as they closed
        } else {
          // rounds lin_len + 1 .. pos from the trace (the ones before were written as they closed)
          while (pos > lin_len && idx != TRACE_NONE) {
            const TraceEnt e = p.trace[idx];
            wout[--pos] = e.move;
            idx = e.parent;
          }
        }
        if (!linear && pos == lin_len) pos = 0;
        hw = pos == 0 ? 1u : 0u;
        R.witness_len = hw ? len : 0u;
      } else if (want) {
        hw = 2u;  // no move buffer: resolved by walk_kernel
      }
      R.has_witness = hw;
    }
  }
  if (p.agg && gl == 0 && (a_set | a_ovf)) {
    atomicAdd(p.agg + PACK_AGG_CONFIGS, a_cfg);
    atomicAdd(p.agg + PACK_AGG_CHILDREN, a_ch);
    atomicAdd(p.agg + PACK_AGG_ROUNDS, a_rounds);
    atomicAdd(p.agg + PACK_AGG_SEARCH_BYTES, a_bytes);
    atomicAdd(p.agg + PACK_AGG_SETTLED, a_set);
    if (a_ovf) atomicAdd(p.agg + PACK_AGG_OVERFLOW, a_ovf);
  }
}

}  // namespace
}  // namespace s2lc
