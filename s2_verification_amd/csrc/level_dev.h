// level_dev.h — device-wide level-synchronous search of ONE history (included
// by level.hip). Used for the histories the per-workgroup passes cannot hold:
// frontiers beyond a workgroup's capacity and histories with more than 128
// chains (single hard histories, BASELINE config C5). Same search as
// search_dev.h (rounds of one durable/indefinite append, E-closure,
// I-identity deferral, P1/P2/P4), replacing porcupine v1.0.3 checkSingle
// (called at golang/s2-porcupine/main.go:606). A round is two grid-wide
// kernels:
//
//   lv_round  : one WAVE per (frontier configuration, slice of its candidate
//               moves). Lane l owns chains l, l+64, ..., l+64(NQ-1) and loads
//               their head records ONCE into registers. For every child in its
//               slice (a minimal durable/indefinite append at a chain head, and
//               its outcome) the wave runs the E-closure against those cached
//               heads: only the chains the closure advances load a record. The
//               closed child is staged in HBM with an incrementally updated
//               fingerprint (the parent's chain terms XOR the changed ones).
//   lv_insert : one lane per staged configuration; 64-bit atomicCAS
//               open-addressing table (32-bit tag | staging index), full-key
//               compare on a tag hit; the winners form the next frontier (an
//               index list into the staging array) and get a trace entry.
//               Its last block closes the round on the device (counters,
//               Ok / Illegal / budget / overflow decisions, per-round counts)
//               and publishes the run state to host-mapped memory.
//
// Because the round's bookkeeping is on the device, the host enqueues many
// rounds back to back and reads the run state once per batch (level.hip);
// every kernel of a finished run returns at once.
//
// Layout: NQ = ceil(K / 64) register slots per lane; a configuration holds
// 64 * NQ u16 chain counters, so K = 319 stores 320 counters (not 512).
#pragma once

namespace s2lc {
namespace {

constexpr uint32_t LV_NONE = 0xFFFFFFFFu;
constexpr uint32_t LV_HOLE = 0xFFFFFFFEu;  // LCfg::move of a reserved, unused staging slot
constexpr int LV_BLOCK = 256;
constexpr uint32_t LV_RESERVE = 8;          // staging slots a wave reserves per atomic
constexpr unsigned long long LV_PENDING = 1ull << 31;  // table entry whose configuration is still landing (lv_persist)

// A staged / frontier configuration: 128 + 128 * NQ bytes. The header fills
// one 128-byte line and every 64-counter block another, so no two
// configurations share a line: the persistent kernel hands a freshly staged
// configuration to another workgroup inside the launch (write-through stores,
// then the table CAS), and a reader must never have pulled a neighbour's
// not-yet-written bytes into its caches.
template <int NQ>
struct __attribute__((aligned(128))) LCfg {
  uint64_t tail;
  uint64_t hash;
  uint64_t fp;      // fingerprint (dedupe / ownership)
  uint32_t tok;
  uint32_t minret;  // exact minret of the closed configuration
  uint32_t ptrace;  // trace id of the parent
  uint32_t move;    // chain | MOVE_IDENT; LV_NONE initial configuration; LV_HOLE unused slot
  uint32_t trace;   // own trace id once in a frontier
  uint32_t slot;    // table slot (cleared when this configuration is expanded)
  uint32_t _pad[20];
  uint16_t cnt[64 * NQ];
};
static_assert(offsetof(LCfg<1>, trace) == 40, "LCfg::trace offset");
static_assert(offsetof(LCfg<1>, cnt) == 128 && sizeof(LCfg<5>) == 128 * 6, "LCfg line layout");

// Per-round device counters (double buffered by round parity). Staging is
// split into LV_STRIPES stripes with a counter each, 64 bytes apart: a single
// counter serializes same-address atomics (~11 ns each on MI355X), and a wide
// round stages millions of configurations.
constexpr int LV_STRIPES = 64;
struct LvCtl {
  uint32_t nnext;     // unique configurations inserted by lv_insert
  uint32_t found;     // a child completed (Ok)
  uint32_t overflow;  // a staging stripe over capacity
  uint32_t done_blocks;  // lv_insert blocks finished (the last one closes the round)
  uint32_t found_parent, found_move, found_p4, _p0;
  unsigned long long children;  // children generated this round
  unsigned long long prof_end;  // S2LC_PROF: latest expansion end of the round (wall clock)
  uint32_t _pad[4];
  uint32_t lo[LV_STRIPES];        // lv_insert: first slot of each stripe not inserted yet (chunked rounds)
  uint32_t cnt[LV_STRIPES * 16];  // stripe s reserves slots at cnt[16 s] (holes included)
};
static_assert(sizeof(LvCtl) == 64 + 4 * LV_STRIPES + 64 * LV_STRIPES, "LvCtl layout");

__device__ __forceinline__ uint32_t ld_agent(const uint32_t* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ unsigned long long ld_agent64(const unsigned long long* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// State of one level search, kept on the device across rounds and published
// to host-mapped memory by the last lv_insert block of every round.
enum : uint32_t { LVR_RUNNING = 0, LVR_FOUND = 1, LVR_EMPTY = 2, LVR_BUDGET = 3, LVR_OVERFLOW = 4, LVR_ABORT = 5 };
struct LvRun {
  uint32_t done;           // LVR_*
  uint32_t round;          // expansion rounds completed (round 0 = the initial closure)
  uint32_t nf;             // current frontier size
  uint32_t max_frontier;
  unsigned long long configs;   // sum of the frontiers (round 0 included)
  unsigned long long children;
  unsigned long long tnext;     // next trace index of this process's pool
  unsigned long long max_configs;  // budget (0 = none)
  uint32_t found_parent, found_move, found_p4;
  uint32_t witness;        // recording trace entries
  uint32_t deep_trace, deep_len;  // Illegal: a configuration of the deepest non-empty round
  uint32_t last_tbase;     // trace index of the first winner of the last non-empty round
  uint32_t last_nf;        // frontier expanded by the last round
  unsigned long long last_children;  // children it generated (slices per configuration)
  uint32_t _pad[2];
};
static_assert(sizeof(LvRun) == 96, "LvRun layout");

struct LvParams {
  const OpRec* __restrict__ recs;
  const uint64_t* __restrict__ pool;
  const uint32_t* __restrict__ cs;  // K+1 absolute chain starts of this history
  uint32_t K;
  uint32_t hflags;
  // current frontier: positions [f0, f1) of cur_idx index cur (staging array);
  // f1 = LV_NONE: the whole frontier, size read from run->nf on the device
  const uint8_t* cur;
  const uint32_t* cur_idx;
  uint32_t f0, f1;
  // staging of this round (becomes the next frontier) + its index list
  uint8_t* stg;
  uint32_t* nxt_idx;
  uint32_t scap;
  uint32_t scs;          // staging slots per stripe (scap / LV_STRIPES); slot = stripe * scs + index
  uint32_t dense;        // lv_insert: a dense input of this many configurations (distributed receive), else striped
  unsigned long long* ht;        // this round's table (the staged configurations are inserted here)
  unsigned long long* ht_clear;  // the table holding the expanded frontier's slots (round parity)
  uint32_t ht_mask;
  uint32_t clear_slots;  // lv_round clears the table slots of the frontier it expands
  uint32_t init;         // lv_round: round 0 (close the initial configuration)
  uint32_t round;        // the round this launch belongs to (host count)
  LvCtl* ctl;            // this round's counters
  LvCtl* ctl_next;       // lv_round zeroes the next round's counters (double buffer)
  LvRun* run;            // device run state
  LvRun* publish;        // host-mapped mirror of *run (the last lv_insert block copies it)
  uint32_t close_round;  // lv_insert's last block closes the round (0: a chunk of a host-driven round)
  uint32_t publish_always;  // publish the run state after this round (else only when the search ends)
  uint32_t* rcounts;     // per-round unique configurations (nullable)
  TraceEnt* trace;
  uint64_t trace_cap;
  uint32_t tgid;         // added to pool indices to form trace ids (distributed: rank << 29)
  uint32_t tbase_host;   // distributed / host-driven: trace index of nxt_idx[0] when run == nullptr
  uint32_t witness_host; // trace recording when run == nullptr
  // distributed search: ownership buckets of the staged configurations
  uint32_t world;
  uint32_t* own_cnt;     // [world] configurations per owner rank
  uint32_t* own_pos;     // per staged configuration: owner << 27 | position within the owner's bucket
  uint8_t* send;         // bucketed configurations, owner-major
  uint64_t own_off[8];   // first configuration of each owner's bucket in send
  unsigned long long* prof;  // S2LC_PROF builds: lv_round phase cycles (nullable)
};

template <int NQ>
__device__ __forceinline__ const LCfg<NQ>* lv_cfg(const uint8_t* base, uint32_t i) {
  return reinterpret_cast<const LCfg<NQ>*>(base + (size_t)i * sizeof(LCfg<NQ>));
}
template <int NQ>
__device__ __forceinline__ LCfg<NQ>* lv_cfg(uint8_t* base, uint32_t i) {
  return reinterpret_cast<LCfg<NQ>*>(base + (size_t)i * sizeof(LCfg<NQ>));
}

// ---- wave reductions: DPP inside each 16-lane row, then one readlane per row
// (the result is wave-uniform, in scalar registers) ------------------------
template <int CTRL>
__device__ __forceinline__ uint32_t lv_dpp(uint32_t v) {
  return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, CTRL, 0xF, 0xF, false);
}
__device__ __forceinline__ uint32_t rl(uint32_t v, int lane) { return (uint32_t)__builtin_amdgcn_readlane((int)v, lane); }

__device__ __forceinline__ uint32_t wave_min_u32(uint32_t v) {
  v = min(v, lv_dpp<0xB1>(v));   // quad_perm [1,0,3,2]
  v = min(v, lv_dpp<0x4E>(v));   // quad_perm [2,3,0,1]
  v = min(v, lv_dpp<0x124>(v));  // row_ror:4
  v = min(v, lv_dpp<0x128>(v));  // row_ror:8
  return min(min(rl(v, 0), rl(v, 16)), min(rl(v, 32), rl(v, 48)));
}
__device__ __forceinline__ uint32_t wave_max_u32(uint32_t v) {
  v = max(v, lv_dpp<0xB1>(v));
  v = max(v, lv_dpp<0x4E>(v));
  v = max(v, lv_dpp<0x124>(v));
  v = max(v, lv_dpp<0x128>(v));
  return max(max(rl(v, 0), rl(v, 16)), max(rl(v, 32), rl(v, 48)));
}
__device__ __forceinline__ uint64_t lv_min64(uint64_t a, uint64_t b) { return a < b ? a : b; }
template <int CTRL>
__device__ __forceinline__ uint64_t lv_dpp64(uint64_t v) {
  return ((uint64_t)lv_dpp<CTRL>((uint32_t)(v >> 32)) << 32) | lv_dpp<CTRL>((uint32_t)v);
}
__device__ __forceinline__ uint64_t rl64(uint64_t v, int lane) {
  return ((uint64_t)rl((uint32_t)(v >> 32), lane) << 32) | rl((uint32_t)v, lane);
}
__device__ __forceinline__ uint64_t wave_min_u64(uint64_t v) {
  v = lv_min64(v, lv_dpp64<0xB1>(v));
  v = lv_min64(v, lv_dpp64<0x4E>(v));
  v = lv_min64(v, lv_dpp64<0x124>(v));
  v = lv_min64(v, lv_dpp64<0x128>(v));
  return lv_min64(lv_min64(rl64(v, 0), rl64(v, 16)), lv_min64(rl64(v, 32), rl64(v, 48)));
}
__device__ __forceinline__ uint64_t wave_xor_u64(uint64_t v) {
  v ^= lv_dpp64<0xB1>(v);
  v ^= lv_dpp64<0x4E>(v);
  v ^= lv_dpp64<0x124>(v);
  v ^= lv_dpp64<0x128>(v);
  return rl64(v, 0) ^ rl64(v, 16) ^ rl64(v, 32) ^ rl64(v, 48);
}

// Wave-aggregated bump allocation: lane asks for `want` entries; returns its
// first index (one atomic per wave). All 64 lanes must call it.
__device__ __forceinline__ uint32_t wave_alloc(uint32_t* ctr, uint32_t want) {
  const int lane = (int)(threadIdx.x & 63);
  uint32_t incl = want;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const uint32_t v = (uint32_t)__shfl_up((int)incl, o, 64);
    if (lane >= o) incl += v;
  }
  const uint32_t total = (uint32_t)__shfl((int)incl, 63, 64);
  uint32_t base = 0;
  if (lane == 63 && total) base = atomicAdd(ctr, total);
  base = (uint32_t)__shfl((int)base, 63, 64);
  return base + incl - want;
}

// Configuration fingerprint: state term ^ XOR over chains of a per-(chain,
// count) term. Commutative over chains, so a wave computes it with one XOR
// reduction, and a child's differs from its parent's only in the chains the
// move and its closure advanced.
__device__ __forceinline__ uint64_t lv_chain_term(uint32_t j, uint32_t c) {
  return mix64(((uint64_t)j << 32 | c) * 0x9E3779B97F4A7C15ull + 0x2545F4914F6CDD1Dull);
}
__device__ __forceinline__ uint64_t lv_state_term(uint64_t tail, uint64_t hash, uint32_t tok) {
  return mix64(tail ^ 0x9E3779B97F4A7C15ull) ^ mix64(hash + 0x632BE59BD9B4E019ull * (tok + 1));
}

// The hot fields of a chain head the closure reads every pass; a head's
// observation (out_tail / out_hash) is only read when it is an eligible
// identity op. For a head loaded during a child's closure the state is fixed,
// so its legality at that state (and the P2 verdict) is computed once at load
// time and kept as flag bits.
struct LvHot {
  uint64_t suf;
  uint32_t call, ret, fl;
};
constexpr uint32_t HB_KNOWN = 1u << 31;   // legality bits below are valid (a head loaded by this child)
constexpr uint32_t HB_LEGAL = 1u << 30;   // legal at the child's state
constexpr uint32_t HB_P2DEAD = 1u << 29;  // P2: a successful read at this tail with another hash

// legality of an identity-class head at s (ident_legal) + the P2 condition
__device__ __forceinline__ uint32_t lv_legal_bits(uint32_t fl, uint64_t otail, uint64_t ohash, const State& s) {
  if ((fl & OPF_KIND_MASK) == 0) return HB_LEGAL;  // definite append failure: {s}
  const bool hash_bad = (fl & OPF_HAS_HASH) && s.hash != ohash;
  const bool tail_bad = !(fl & OPF_FAIL) && s.tail != otail;
  uint32_t b = (!hash_bad && !tail_bad) ? HB_LEGAL : 0u;
  if (hash_bad && !(fl & OPF_FAIL) && otail == s.tail) b |= HB_P2DEAD;
  return b;
}

__device__ __forceinline__ LvHot lv_hot_null() {
  LvHot h;
  h.suf = REQ_NONE; h.call = EV_INF; h.ret = EV_INF; h.fl = OPF_SENTINEL;
  return h;
}

// The parent's heads of one wave, in LDS (structure of arrays: lane-indexed,
// so every access is conflict-free).
template <int NQ>
struct LvHeadsLds {
  uint64_t otail[NQ][64], ohash[NQ][64], suf[NQ][64];
  uint32_t call[NQ][64], ret[NQ][64], fl[NQ][64];
};

// Load the head at rec into LDS slot q and return its hot fields.
template <int NQ>
__device__ __forceinline__ LvHot lv_load_parent_head(const OpRec* r, LvHeadsLds<NQ>& L, int q, int lane) {
  const uint4 a = ld16(r, 16);
  const uint4 b = ld16(r, 32);
  LvHot h;
  h.suf = (uint64_t)b.x | ((uint64_t)b.y << 32);
  h.call = b.z;
  h.ret = b.w;
  h.fl = r->flags;
  L.otail[q][lane] = (uint64_t)a.x | ((uint64_t)a.y << 32);
  L.ohash[q][lane] = (uint64_t)a.z | ((uint64_t)a.w << 32);
  L.suf[q][lane] = h.suf;
  L.call[q][lane] = h.call;
  L.ret[q][lane] = h.ret;
  L.fl[q][lane] = h.fl;
  return h;
}
template <int NQ>
__device__ __forceinline__ LvHot lv_parent_hot(const LvHeadsLds<NQ>& L, int q, int lane) {
  LvHot h;
  h.suf = L.suf[q][lane]; h.call = L.call[q][lane]; h.ret = L.ret[q][lane]; h.fl = L.fl[q][lane];
  return h;
}
// A head loaded during a child's closure: hot fields + legality at s.
__device__ __forceinline__ LvHot lv_load_child_head(const OpRec* r, const State& s) {
  const uint4 a = ld16(r, 16);
  const uint4 b = ld16(r, 32);
  LvHot h;
  h.suf = (uint64_t)b.x | ((uint64_t)b.y << 32);
  h.call = b.z;
  h.ret = b.w;
  const uint32_t fl = r->flags;
  h.fl = fl | HB_KNOWN |
         lv_legal_bits(fl, (uint64_t)a.x | ((uint64_t)a.y << 32), (uint64_t)a.z | ((uint64_t)a.w << 32), s);
  return h;
}

// E-closure of one child. H[q] = hot fields of the child's current head on
// slot q (the parent's, unless the move or the closure advanced that chain),
// d[q] = ops the child linearized on slot q beyond the parent's count.
// A pass takes every identity head that is minimal under the previous pass's
// minret (a lower bound of the current one: minret only grows, so such an op
// is minimal now) and legal at s; all of them advance together (the closure
// is order-independent). A pass that changes nothing has read exactly the
// final heads, so its minret / P1 bound are exact; it ends the closure once
// its eligibility test also used that exact minret. Seeded with the parent's
// minret. Only advancing chains load a record.
template <int NQ>
__device__ __forceinline__ int lv_closure(LvHot (&H)[NQ], uint32_t (&d)[NQ], const uint32_t (&cnt)[NQ],
                                          const uint32_t* s_cs, const LvHeadsLds<NQ>& PL, int lane, const State& s,
                                          uint32_t hflags, uint32_t minret_seed, const OpRec* __restrict__ recs,
                                          uint32_t& minret_out) {
  const bool nowrap = hflags & H_NOWRAP;
  const bool p2 = hflags & H_P2OK;
  const bool p4 = hflags & H_P4;
  uint32_t minret_prev = minret_seed;
  for (;;) {
    uint32_t mr = EV_INF;
    uint64_t bd = REQ_NONE;
    uint32_t adv = 0;
    bool dead = false;
#pragma unroll
    for (int q = 0; q < NQ; ++q) {
      const LvHot& h = H[q];
      mr = min(mr, h.ret);
      bd = lv_min64(bd, h.suf);
      if (!(h.fl & OPF_CLS_E) || h.call >= minret_prev) continue;
      uint32_t bits = h.fl;
      if (!(bits & HB_KNOWN)) bits = lv_legal_bits(h.fl, PL.otail[q][lane], PL.ohash[q][lane], s);
      if (bits & HB_LEGAL) adv |= 1u << q;
      else if (p2 && (bits & HB_P2DEAD)) dead = true;
    }
    const uint32_t minret = wave_min_u32(mr);
    const uint64_t bound = wave_min_u64(bd);
    if (__ballot(dead) || (nowrap && s.tail > bound)) return CL_DEAD;
    const bool changed = __ballot(adv != 0) != 0;
    if (!changed && minret == minret_prev) {
      minret_out = minret;
      return minret == EV_INF ? CL_COMPLETE : ((p4 && bound == REQ_NONE) ? CL_P4 : CL_ALIVE);
    }
#pragma unroll
    for (int q = 0; q < NQ; ++q) {
      if ((adv >> q) & 1u) {
        d[q] += 1;
        H[q] = lv_load_child_head(recs + s_cs[64 * q + lane] + cnt[q] + d[q], s);
      }
    }
    minret_prev = minret;
  }
}

// Stage one closed child into stripe `st` of the staging array; the wave
// reserves LV_RESERVE slots of its stripe at a time (rk / rleft, wave-uniform).
template <int NQ>
__device__ __forceinline__ void lv_stage(const LvParams& p, uint32_t st, uint32_t& rk, uint32_t& rleft, const State& s,
                                         uint64_t fp, uint32_t minret, uint32_t ptrace, uint32_t move,
                                         const uint32_t (&cnt)[NQ], const uint32_t (&d)[NQ]) {
  const int lane = (int)(threadIdx.x & 63);
  if (rleft == 0) {
    uint32_t b = 0;
    if (lane == 0) b = atomicAdd(&p.ctl->cnt[16 * st], LV_RESERVE);
    rk = (uint32_t)__shfl((int)b, 0, 64);
    rleft = LV_RESERVE;
  }
  const uint32_t i = rk++;
  rleft--;
  if (i >= p.scs) {
    if (lane == 0) atomicExch(&p.ctl->overflow, 1u);
    return;
  }
  LCfg<NQ>* o = lv_cfg<NQ>(p.stg, st * p.scs + i);
  if (lane == 0) {
    o->tail = s.tail; o->hash = s.hash; o->fp = fp; o->tok = s.tok;
    o->minret = minret; o->ptrace = ptrace; o->move = move;
    o->trace = TRACE_NONE; o->slot = LV_NONE;
  }
#pragma unroll
  for (int q = 0; q < NQ; ++q) o->cnt[lane + 64 * q] = (uint16_t)(cnt[q] + d[q]);
}

// Unused reserved slots become holes (lv_insert and the distributed kernels skip them).
template <int NQ>
__device__ __forceinline__ void lv_release(const LvParams& p, uint32_t st, uint32_t rk, uint32_t rleft) {
  const int lane = (int)(threadIdx.x & 63);
  for (uint32_t i = lane; i < rleft; i += 64)
    if (rk + i < p.scs) lv_cfg<NQ>(p.stg, st * p.scs + rk + i)->move = LV_HOLE;
}

// S2LC_PROF: per-phase cycle counts of lv_expand (lane 0 of every wave, summed
// into p.prof by the waves that had items; every lap first waits for the
// wave's outstanding loads): [0] parent load, [1] heads + fingerprint, [2]
// move states, [3] closures, [4] stage (+ insert) + restore, [5] items, [6]
// children, [12] move selection, [13] move record loads (the rest of [2] is
// the hash fold). [9..11]: persistent round timing (lv_persist).
#ifdef S2LC_PROF
#define LV_T0() lv_t = clock64()
#define LV_LAP(i) do { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); const unsigned long long t_ = clock64(); lv_acc[i] += t_ - lv_t; lv_t = t_; } while (0)
#define LV_ADD(i, v) lv_acc[i] += (v)
#else
#define LV_T0() do { } while (0)
#define LV_LAP(i) do { } while (0)
#define LV_ADD(i, v) do { } while (0)
#endif

// cnt[q] for a wave-uniform runtime slot q (a select chain, no scratch)
template <int NQ>
__device__ __forceinline__ uint32_t sel_cnt(const uint32_t (&cnt)[NQ], uint32_t q) {
  uint32_t v = cnt[0];
#pragma unroll
  for (int i = 1; i < NQ; ++i) v = q == (uint32_t)i ? cnt[i] : v;
  return v;
}

template <int N>
__device__ __forceinline__ uint32_t sel_u32(const uint32_t (&a)[N], uint32_t q) {
  uint32_t v = a[0];
#pragma unroll
  for (int i = 1; i < N; ++i) v = q == (uint32_t)i ? a[i] : v;
  return v;
}
template <int N>
__device__ __forceinline__ uint64_t sel_u64(const uint64_t (&a)[N], uint32_t q) {
  uint64_t v = a[0];
#pragma unroll
  for (int i = 1; i < N; ++i) v = q == (uint32_t)i ? a[i] : v;
  return v;
}

typedef __attribute__((address_space(1))) uint16_t lv_g16;
typedef __attribute__((address_space(1))) uint32_t lv_g32;
typedef __attribute__((address_space(1))) unsigned long long lv_g64;
// write-through (agent-scope) stores and loads: the hand-off forms of the
// persistent kernel (a configuration staged by one workgroup is compared by
// another inside the same round)
__device__ __forceinline__ void st_wt16(uint16_t* p, uint16_t v) {
  __hip_atomic_store((lv_g16*)p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st_wt32(uint32_t* p, uint32_t v) {
  __hip_atomic_store((lv_g32*)p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st_wt64(void* p, unsigned long long v) {
  __hip_atomic_store((lv_g64*)p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ uint16_t ld_wt16(const uint16_t* p) {
  return __hip_atomic_load((lv_g16*)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ unsigned long long ld_wt64(const void* p) {
  return __hip_atomic_load((lv_g64*)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void lv_drain() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }

// What one round's expansion takes besides LvParams: the frontier range, the
// slices per configuration, and (fused insert) the round's trace base.
struct LvRoundIn {
  uint32_t f0, nf;  // frontier positions [f0, f0 + nf) of cur_idx (init: the initial configuration)
  uint32_t S;       // slices per configuration
  uint32_t tbase;   // trace index of the round's first winner (fused insert)
  uint32_t wit;     // record trace entries (fused insert)
};

// Slices per configuration: narrow frontiers spread a configuration's moves
// over several waves (down to about one child per wave), wide ones give a wave
// whole configurations. The expected moves per configuration come from the
// previous round.
__device__ __forceinline__ uint32_t lv_slices(uint32_t K, uint32_t nf, uint32_t nwaves, uint32_t last_nf,
                                              unsigned long long last_children) {
  uint32_t c_est = K;
  if (last_nf) c_est = (uint32_t)min<unsigned long long>(K, last_children / last_nf + 1);
  return max(1u, min(c_est + (c_est >> 2) + 1, (2u * nwaves + nf - 1) / max(nf, 1u)));
}

// Persistent kernel: stage one closed child with write-through stores and
// insert it at once (the producing wave deduplicates its own child: a 64-bit
// CAS, and on a tag hit a wave-parallel compare against the resident entry).
template <int NQ>
__device__ __forceinline__ void lv_stage_insert(const LvParams& p, const LvRoundIn& in, uint32_t st, uint32_t& rk,
                                                uint32_t& rleft, const State& s, uint64_t fp, uint32_t minret,
                                                uint32_t ptrace, uint32_t move, const uint32_t (&cnt)[NQ],
                                                const uint32_t (&d)[NQ]) {
  const int lane = (int)(threadIdx.x & 63);
  if (rleft == 0) {
    uint32_t b = 0;
    if (lane == 0) b = atomicAdd(&p.ctl->cnt[16 * st], LV_RESERVE);
    rk = rl(b, 0);
    rleft = LV_RESERVE;
  }
  const uint32_t i = rk++;
  rleft--;
  if (i >= p.scs) {
    if (lane == 0) atomicExch(&p.ctl->overflow, 1u);
    return;
  }
  const uint32_t k = st * p.scs + i;
  LCfg<NQ>* o = lv_cfg<NQ>(p.stg, k);
  // the header line: lanes 0..15 store one 8-byte word each (one whole-line store)
  const unsigned long long w = lane == 0 ? s.tail
                             : lane == 1 ? s.hash
                             : lane == 2 ? fp
                             : lane == 3 ? ((unsigned long long)minret << 32 | s.tok)
                             : lane == 4 ? ((unsigned long long)move << 32 | ptrace)
                             : lane == 5 ? ((unsigned long long)LV_NONE << 32 | TRACE_NONE)
                                         : 0ull;
  if (lane < 16) st_wt64(reinterpret_cast<unsigned long long*>(o) + lane, w);
#pragma unroll
  for (int q = 0; q < NQ; ++q) st_wt16(&o->cnt[lane + 64 * q], (uint16_t)(cnt[q] + d[q]));
  // The CAS goes out with the stores: the entry is published PENDING (bit 31
  // of the index) and made final once this wave's stores have landed. A wave
  // that meets a pending entry with its tag waits for the final form before
  // it reads the configuration. A duplicate never waits for its own stores.
  const uint32_t tag = (uint32_t)(fp >> 32);
  const unsigned long long mine = ((unsigned long long)tag << 32) | k;
  uint32_t slot = (uint32_t)fp & p.ht_mask;
  for (;;) {
    unsigned long long prev = 0;
    if (lane == 0) prev = atomicCAS(&p.ht[slot], HT_EMPTY, mine | LV_PENDING);
    prev = rl64(prev, 0);
    if (prev == HT_EMPTY) break;
    if ((uint32_t)(prev >> 32) == tag) {
      while (prev & LV_PENDING) {  // its producer is between its CAS and its final store
        __builtin_amdgcn_s_sleep(1);
        unsigned long long x = 0;
        if (lane == 0) x = ld_agent64(&p.ht[slot]);
        prev = rl64(x, 0);
      }
      const LCfg<NQ>* e = lv_cfg<NQ>(p.stg, (uint32_t)prev);
      const unsigned long long et = ld_wt64(&e->tail), eh = ld_wt64(&e->hash), ek = ld_wt64(&e->tok);
      bool ne = et != s.tail || eh != s.hash || (uint32_t)ek != s.tok;
#pragma unroll
      for (int q = 0; q < NQ; ++q) ne |= ld_wt16(&e->cnt[lane + 64 * q]) != (uint16_t)(cnt[q] + d[q]);
      if (__ballot(ne) == 0) return;  // an equal configuration is already in the round
    }
    slot = (slot + 1) & p.ht_mask;
  }
  // the winner: its stores land, then the entry loses its PENDING bit
  lv_drain();
  if (lane == 0) atomicExch(&p.ht[slot], mine);
  // next-frontier position, table slot, trace entry
  uint32_t n = 0;
  if (lane == 0) n = atomicAdd(&p.ctl->nnext, 1u);
  n = rl(n, 0);
  if (lane == 0) {
    st_wt32(&p.nxt_idx[n], k);
    st_wt32(&o->slot, slot);
    if (in.wit) {
      st_wt32(&o->trace, p.tgid + in.tbase + n);
      p.trace[in.tbase + n] = TraceEnt{ptrace, move};
    }
  }
}

// ---- expansion: one wave per (frontier configuration, slice of its candidates)
// FUSED = false: stage into the striped staging array (lv_insert deduplicates);
// FUSED = true: the persistent kernel's stage-and-insert.
template <int NQ, bool FUSED>
__device__ __forceinline__ bool lv_expand(const LvParams& p, const LvRoundIn& in, LvHeadsLds<NQ>& PL,
                                          const uint32_t* s_cs) {
  const int lane = (int)(threadIdx.x & 63);
  const uint32_t K = p.K;
  const bool idefer = p.hflags & H_IDEFER;
  const uint32_t f0 = in.f0, nf = in.nf, S = in.S;
  const uint32_t nwaves = gridDim.x * (LV_BLOCK / 64);
  const uint32_t items = nf * S;
  uint32_t rk = 0, rleft = 0;  // reserved staging slots (wave-uniform)
  const uint32_t wave_id = blockIdx.x * (LV_BLOCK / 64) + (threadIdx.x >> 6);
  const uint32_t stripe = wave_id & (LV_STRIPES - 1);
  if (wave_id < items) {  // the first reservation, in flight with the first item's loads
    uint32_t b0 = 0;
    if (lane == 0) b0 = atomicAdd(&p.ctl->cnt[16 * stripe], LV_RESERVE);
    rk = rl(b0, 0);
    rleft = LV_RESERVE;
  }
  unsigned long long kids = 0;
#ifdef S2LC_PROF
  unsigned long long lv_acc[10] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0}, lv_t = 0;
#endif
  for (uint32_t it = wave_id; it < items; it += nwaves) {
    LV_T0();
    LV_ADD(5, 1);
    const uint32_t f = f0 + it / S;
    const uint32_t slice = it % S;
    // parent configuration (round 0: the all-zero initial one)
    const LCfg<NQ>* pc = p.init ? nullptr : lv_cfg<NQ>(p.cur, p.cur_idx[f]);
    State ps{0, 0, 0};
    uint32_t pmin = 0, ptrace = TRACE_NONE;
    if (pc) {
      ps = State{pc->tail, pc->hash, pc->tok};
      pmin = pc->minret;
      ptrace = pc->trace;
      if (slice == 0 && lane == 0 && p.clear_slots && pc->slot <= p.ht_mask)
        st_wt64(&p.ht_clear[pc->slot], HT_EMPTY);
    }
    uint32_t cnt[NQ], d[NQ];
    LvHot H[NQ];
    LV_LAP(0);
    uint64_t chx = 0;  // this lane's part of the parent's chain fingerprint
    uint32_t cand = 0;
#pragma unroll
    for (int q = 0; q < NQ; ++q) {
      const uint32_t j = (uint32_t)lane + 64u * q;
      cnt[q] = (j < K && pc) ? (uint32_t)pc->cnt[j] : 0u;
      d[q] = 0;
      if (j < K) {
        H[q] = lv_load_parent_head<NQ>(p.recs + s_cs[64 * q + lane] + cnt[q], PL, q, lane);
      } else {
        H[q] = lv_hot_null();
        PL.fl[q][lane] = OPF_SENTINEL; PL.call[q][lane] = EV_INF; PL.ret[q][lane] = EV_INF; PL.suf[q][lane] = REQ_NONE;
      }
      if (j < K) chx ^= lv_chain_term(j, cnt[q]);
      // candidate moves: minimal durable / indefinite appends at the chain heads
      if (pc && !(H[q].fl & (OPF_SENTINEL | OPF_CLS_E)) && H[q].call < pmin) cand |= 1u << q;
    }
    const uint64_t parent_chx = wave_xor_u64(chx);
    LV_LAP(1);
    // candidate moves in (slot, lane) order; this slice takes moves [c0, c1)
    uint32_t n_cand = 0, my_idx[NQ];
    const uint64_t lt_mask = (1ull << lane) - 1;
#pragma unroll
    for (int q = 0; q < NQ; ++q) {
      const uint64_t bq = __ballot((cand >> q) & 1u);
      my_idx[q] = n_cand + (uint32_t)__popcll(bq & lt_mask);
      n_cand += (uint32_t)__popcll(bq);
    }
    // round 0 has one pseudo-move: the initial configuration itself
    const uint32_t n_moves = pc ? n_cand : 1u;
    const uint32_t c0 = (uint32_t)(((uint64_t)n_moves * slice) / S);
    const uint32_t c1 = (uint32_t)(((uint64_t)n_moves * (slice + 1)) / S);
    // The outcome of every move of this slice at once (lane l, slot q: the
    // append at the head of chain l + 64 q): the rest of its record, guards,
    // outcome and hash fold, for those moves in parallel, so a move in the
    // loop below costs only its next head's load. Registers: 5 per slot
    // (NQ <= 6).
    constexpr bool PRE = NQ <= 6;
    constexpr int NP = PRE ? NQ : 1;
    uint64_t mv_tail[NP], mv_hash[NP];
    uint32_t mv_pk[NP];  // take_opt | take_id << 1 | token << 16
#pragma unroll
    for (int q = 0; q < NP; ++q) {
      mv_tail[q] = ps.tail;
      mv_hash[q] = ps.hash;
      mv_pk[q] = ps.tok << 16;
      if (PRE && ((cand >> q) & 1u) && my_idx[q] >= c0 && my_idx[q] < c1) {
        const OpRec r = load_rec(p.recs + s_cs[64 * q + lane] + cnt[q]);  // the head: just loaded, cached
        const bool g = append_guards_ok(r, ps);
        State opt = ps;
        opt.tail = ps.tail + r.num_records;
        opt.tok = r.set_tok ? r.set_tok : ps.tok;
        const bool to = (r.flags & OPF_CLS_D) ? (g && opt.tail == r.out_tail) : g;
        if (to || ((r.flags & OPF_CLS_I) && g)) opt.hash = fold_hashes_blk(ps.hash, p.pool + r.hash_off, r.hash_cnt);
        const bool ti = (r.flags & OPF_CLS_I) && (!idefer || r.ret_ev == pmin) && !(g && state_eq(opt, ps));
        mv_tail[q] = opt.tail;
        mv_hash[q] = opt.hash;
        mv_pk[q] = (to ? 1u : 0u) | (ti ? 2u : 0u) | (opt.tok << 16);
      }
    }
    uint32_t ord = 0, q_cur = 0;
    uint64_t m = pc ? __ballot(cand & 1u) : 1ull;
    for (;;) {
      // next move (wave-uniform): slot q_cur, owner lane src
      while (m == 0 && q_cur + 1 < (uint32_t)NQ && pc) {
        ++q_cur;
        m = __ballot((cand >> q_cur) & 1u);
      }
      if (m == 0 || ord >= c1) break;
      const int src = __ffsll((unsigned long long)m) - 1;
      m &= m - 1;
      const uint32_t o = ord++;
      if (o < c0) continue;
      // children of the move: on the owner lane (round 0: the unchanged initial state)
      bool take_opt = !pc, take_id = false;
      State opt = ps;
      uint4 nx_obs = make_uint4(0, 0, 0, 0), nx_mid = make_uint4(0, 0, 0, 0);
      uint32_t nx_fl = 0;
      LV_LAP(7);
      uint32_t fl2;
      State so;
      if (PRE) {
        if (pc && lane == src) {
          // the chain's next head (the child's first new head)
          const OpRec* nx = p.recs + s_cs[64 * q_cur + lane] + sel_cnt<NQ>(cnt, q_cur) + 1;
          nx_obs = ld16(nx, 16);
          nx_mid = ld16(nx, 32);
          nx_fl = nx->flags;
        }
        const uint32_t pk = rl(sel_u32<NP>(mv_pk, q_cur), src);
        fl2 = pc ? (pk & 3u) : 1u;
        so = pc ? State{rl64(sel_u64<NP>(mv_tail, q_cur), src), rl64(sel_u64<NP>(mv_hash, q_cur), src), pk >> 16} : ps;
      } else {
        if (pc && lane == src) {
          // the move's record, and the chain's next head (the child's first new head) with it
          const OpRec* mrec = p.recs + s_cs[64 * q_cur + lane] + sel_cnt<NQ>(cnt, q_cur);
          const OpRec* nx = mrec + 1;
          nx_obs = ld16(nx, 16);
          nx_mid = ld16(nx, 32);
          nx_fl = nx->flags;
          const OpRec r = load_rec(mrec);
          const bool g = append_guards_ok(r, ps);
          LV_LAP(8);
          opt.tail = ps.tail + r.num_records;
          opt.tok = r.set_tok ? r.set_tok : ps.tok;
          take_opt = (r.flags & OPF_CLS_D) ? (g && opt.tail == r.out_tail) : g;
          if (take_opt || ((r.flags & OPF_CLS_I) && g)) opt.hash = fold_hashes_blk(ps.hash, p.pool + r.hash_off, r.hash_cnt);
          if (r.flags & OPF_CLS_I) take_id = (!idefer || r.ret_ev == pmin) && !(g && state_eq(opt, ps));
        }
        fl2 = pc ? rl((take_opt ? 1u : 0u) | (take_id ? 2u : 0u), src) : 1u;
        so = State{rl64(opt.tail, src), rl64(opt.hash, src), rl(opt.tok, src)};
      }
      const uint32_t j = (uint32_t)src + 64u * q_cur;
      LV_LAP(2);
#pragma unroll 1
      for (int w = 0; w < 2; ++w) {
        if (!((fl2 >> w) & 1u)) continue;
        const State cs_ = w == 0 ? so : ps;
        const uint32_t mv = !pc ? LV_NONE : (w == 0 ? j : (j | MOVE_IDENT));
        if (pc) {
          kids++;
#pragma unroll
          for (int q = 0; q < NQ; ++q)
            if ((uint32_t)q == q_cur && lane == src) {
              d[q] = 1;
              H[q].suf = (uint64_t)nx_mid.x | ((uint64_t)nx_mid.y << 32);
              H[q].call = nx_mid.z;
              H[q].ret = nx_mid.w;
              H[q].fl = nx_fl | HB_KNOWN |
                        lv_legal_bits(nx_fl, (uint64_t)nx_obs.x | ((uint64_t)nx_obs.y << 32),
                                      (uint64_t)nx_obs.z | ((uint64_t)nx_obs.w << 32), cs_);
            }
        }
        uint32_t mr = 0;
        LV_LAP(4);
        LV_ADD(6, 1);
        const int cr = lv_closure<NQ>(H, d, cnt, s_cs, PL, lane, cs_, p.hflags, pmin, p.recs, mr);
        LV_LAP(3);
        if (cr == CL_COMPLETE || cr == CL_P4) {
          if (lane == 0 && atomicCAS(&p.ctl->found, 0u, 1u) == 0u) {
            atomicExch(&p.ctl->found_parent, ptrace);
            atomicExch(&p.ctl->found_move, mv);
            atomicExch(&p.ctl->found_p4, cr == CL_P4 ? 1u : 0u);
          }
        } else if (cr == CL_ALIVE) {
          uint64_t dx = 0;
#pragma unroll
          for (int q = 0; q < NQ; ++q) {
            const uint32_t jj = (uint32_t)lane + 64u * q;
            if (d[q]) dx ^= lv_chain_term(jj, cnt[q]) ^ lv_chain_term(jj, cnt[q] + d[q]);
          }
          const uint64_t fp = mix64(parent_chx ^ wave_xor_u64(dx) ^ lv_state_term(cs_.tail, cs_.hash, cs_.tok));
          if (FUSED)
            lv_stage_insert<NQ>(p, in, stripe, rk, rleft, cs_, fp, mr, ptrace, mv, cnt, d);
          else
            lv_stage<NQ>(p, stripe, rk, rleft, cs_, fp, mr, ptrace, mv, cnt, d);
        }
        // back to the parent's heads on the chains this child advanced
#pragma unroll
        for (int q = 0; q < NQ; ++q)
          if (d[q]) {
            d[q] = 0;
            H[q] = lv_parent_hot<NQ>(PL, q, lane);
          }
      }
    }
  }
#ifdef S2LC_PROF
  if (lane == 0 && p.prof && lv_acc[5])  // only waves that had work (idle waves would swamp the counters)
    for (int i_ = 0; i_ < 9; ++i_) atomicAdd(&p.prof[i_ < 7 ? i_ : i_ + 5], lv_acc[i_]);
#endif
  if (!FUSED && rleft) lv_release<NQ>(p, stripe, rk, rleft);
  if (lane == 0 && kids) atomicAdd(&p.ctl->children, kids);
  return wave_id < items;
}

// ---- round kernel (host-enqueued rounds): expand + close + stage ----------
template <int NQ>
__global__ __launch_bounds__(LV_BLOCK) void lv_round(LvParams p) {
  if (p.run && p.run->done) return;  // the search ended in an earlier round of this batch
  if (p.ctl_next && blockIdx.x == 0)
    for (uint32_t i = threadIdx.x; i < sizeof(LvCtl) / 4; i += LV_BLOCK) reinterpret_cast<uint32_t*>(p.ctl_next)[i] = 0;
  __shared__ LvHeadsLds<NQ> s_heads[LV_BLOCK / 64];
  __shared__ uint32_t s_cs[64 * NQ];  // chain starts (slot q of lane l = chain l + 64 q), shared by the block
  for (uint32_t x = threadIdx.x; x < 64u * NQ; x += LV_BLOCK) s_cs[x] = x < p.K ? p.cs[x] : 0u;
  __syncthreads();
  LvRoundIn in;
  in.f0 = p.f0;
  in.nf = p.f1 == LV_NONE ? p.run->nf : p.f1 - p.f0;
  if (p.f1 == LV_NONE) in.f0 = 0;
  if (p.init) in.nf = 1;
  const uint32_t nwaves = gridDim.x * (LV_BLOCK / 64);
  in.S = p.init ? 1u : lv_slices(p.K, in.nf, nwaves, p.run ? p.run->last_nf : 0u, p.run ? p.run->last_children : 0ull);
  in.tbase = 0;
  in.wit = 0;
  lv_expand<NQ, false>(p, in, s_heads[threadIdx.x >> 6], s_cs);
}

template <int NQ>
__device__ __forceinline__ bool lv_eq(const LCfg<NQ>* a, const LCfg<NQ>* b, uint32_t K) {
  if (a->tail != b->tail || a->hash != b->hash || a->tok != b->tok) return false;
  const uint4* x = reinterpret_cast<const uint4*>(a->cnt);
  const uint4* y = reinterpret_cast<const uint4*>(b->cnt);
  const uint32_t nw = (K + 7) >> 3;
  for (uint32_t q = 0; q < nw; ++q) {
    const uint4 u = x[q], v = y[q];
    if (u.x != v.x || u.y != v.y || u.z != v.z || u.w != v.w) return false;
  }
  return true;
}

// A round's counters, read by the closer (every word was written by
// device-scope atomics: read as such, issued together).
struct LvCounts {
  uint32_t nn, ovf, fnd, fpar, fmov, fp4;
  unsigned long long ch;
};
__device__ __forceinline__ LvCounts lv_read_counts(LvCtl* c) {
  LvCounts k;
  k.nn = ld_agent(&c->nnext);
  k.ovf = ld_agent(&c->overflow);
  k.fnd = ld_agent(&c->found);
  k.fpar = ld_agent(&c->found_parent);
  k.fmov = ld_agent(&c->found_move);
  k.fp4 = ld_agent(&c->found_p4);
  k.ch = ld_agent64(&c->children);
  return k;
}

// Close round `rnd` on the run state R: per-round count, run counters, and
// the decision (found / empty / budget / overflow / witness off).
__device__ __forceinline__ void lv_close_state(LvRun& R, const LvCounts& k, uint32_t rnd, uint32_t* rcounts,
                                               uint32_t scap, uint64_t trace_cap) {
  R.children += k.ch;
  R.last_nf = rnd == 0 ? 0u : R.nf;
  R.last_children = k.ch;
  if (k.ovf) {
    R.done = LVR_OVERFLOW;  // the host re-runs this round in frontier chunks
  } else if (k.fnd) {
    R.done = LVR_FOUND;
    R.round = rnd;
    R.found_parent = R.witness ? k.fpar : TRACE_NONE;
    R.found_move = k.fmov;
    R.found_p4 = k.fp4;
  } else {
    if (rcounts) rcounts[rnd] = k.nn;
    R.round = rnd;
    if (k.nn == 0) {
      R.done = LVR_EMPTY;
      if (rnd > 0 && R.witness) { R.deep_trace = R.last_tbase; R.deep_len = rnd - 1; }
    } else {
      R.nf = k.nn;
      R.max_frontier = max(R.max_frontier, k.nn);
      R.configs += k.nn;
      if (R.witness) {
        R.last_tbase = (uint32_t)R.tnext;
        R.tnext += k.nn;
        if (R.tnext + scap > trace_cap) R.witness = 0;
      }
      if (R.max_configs && R.configs > R.max_configs) R.done = LVR_BUDGET;
    }
  }
}

__device__ __forceinline__ void lv_publish(const LvRun& R, LvRun* pub) {
  const uint32_t* src = reinterpret_cast<const uint32_t*>(&R);
  volatile uint32_t* dst = reinterpret_cast<volatile uint32_t*>(pub);
  for (uint32_t i = 0; i < sizeof(LvRun) / 4; ++i) dst[i] = src[i];
  __threadfence_system();
}

// The last block of lv_insert closes the round on the device, then publishes
// the run state to the host-mapped mirror when the host will look (the last
// round of a batch, or the end of the search): every word is a write over the link.
__device__ __forceinline__ void lv_close_round(const LvParams& p) {
  const LvCounts k = lv_read_counts(p.ctl);
  LvRun& R = *p.run;
  lv_close_state(R, k, p.round, p.rcounts, p.scap, p.trace_cap);
  if (p.publish && (p.publish_always || R.done)) lv_publish(R, p.publish);
}

// ---- insert: one lane per staged configuration -----------------------------
// Striped staging: lane l of every wave walks stripe l (slot l * scs + i for
// i = lo[l] .. cnt[l]); the grid strides over i. Winners take next-frontier
// positions with one atomic per block.
template <int NQ>
__global__ __launch_bounds__(LV_BLOCK) void lv_insert(LvParams p) {
  if (p.run && p.run->done) return;
  __shared__ uint32_t s_wcnt[LV_BLOCK / 64], s_base, s_hi, s_last;
  const int lane = (int)(threadIdx.x & 63), wv = (int)(threadIdx.x >> 6);
  const bool wit = p.run ? p.run->witness != 0 : p.witness_host != 0;
  const uint32_t tbase = p.run ? (uint32_t)p.run->tnext : p.tbase_host;
  uint32_t lo = 0, hi = 0;  // this lane's stripe range (striped mode)
  if (p.dense) {
    hi = p.dense;
  } else if (!ld_agent(&p.ctl->overflow)) {
    lo = p.ctl->lo[lane];
    hi = min(ld_agent(&p.ctl->cnt[16 * lane]), p.scs);
  }
  // iterations: the longest stripe (striped) / the dense range, block-uniform
  uint32_t n_it;
  if (p.dense) {
    n_it = (p.dense + LV_BLOCK - 1) / LV_BLOCK;
  } else {
    const uint32_t m = wave_max_u32(hi);
    n_it = (m + LV_BLOCK / 64 - 1) / (LV_BLOCK / 64);  // rows of 4 slots per stripe per block iteration
  }
  for (uint32_t itb = blockIdx.x; itb < n_it; itb += gridDim.x) {
    bool win = false;
    uint32_t slot = 0, k = 0;
    LCfg<NQ>* c = nullptr;
    bool valid;
    if (p.dense) {
      k = itb * LV_BLOCK + threadIdx.x;
      valid = k < p.dense;
    } else {
      const uint32_t i = itb * (LV_BLOCK / 64) + (uint32_t)wv;
      valid = i >= lo && i < hi;
      k = (uint32_t)lane * p.scs + i;
    }
    if (valid) {
      c = lv_cfg<NQ>(p.stg, k);
      if (c->move != LV_HOLE) {
        const uint64_t fp = c->fp;
        const uint32_t tag = (uint32_t)(fp >> 32);
        const unsigned long long mine = ((unsigned long long)tag << 32) | k;
        slot = (uint32_t)fp & p.ht_mask;
        for (;;) {
          const unsigned long long prev = atomicCAS(&p.ht[slot], HT_EMPTY, mine);
          if (prev == HT_EMPTY) { win = true; break; }
          if ((uint32_t)(prev >> 32) == tag && lv_eq<NQ>(lv_cfg<NQ>(p.stg, (uint32_t)prev), c, p.K)) break;
          slot = (slot + 1) & p.ht_mask;
        }
      }
    }
    // next-frontier positions: one atomic per block
    const uint64_t bw = __ballot(win);
    if (lane == 0) s_wcnt[wv] = (uint32_t)__popcll(bw);
    __syncthreads();
    if (threadIdx.x == 0) {
      uint32_t t = 0;
      for (int w = 0; w < LV_BLOCK / 64; ++w) t += s_wcnt[w];
      s_base = t ? atomicAdd(&p.ctl->nnext, t) : 0u;
    }
    __syncthreads();
    uint32_t n = s_base;
    for (int w = 0; w < wv; ++w) n += s_wcnt[w];
    n += (uint32_t)__popcll(bw & ((1ull << lane) - 1));
    __syncthreads();  // s_wcnt / s_base are rewritten next iteration
    if (win) {
      p.nxt_idx[n] = k;
      c->slot = slot;
      if (wit) {
        c->trace = p.tgid + tbase + n;
        p.trace[tbase + n] = TraceEnt{c->ptrace, c->move};
      }
    }
  }
  (void)s_hi;
  if (!p.close_round) return;
  // the last block to finish closes the round (it only reads atomics: no fence)
  __syncthreads();
  if (threadIdx.x == 0) s_last = atomicAdd(&p.ctl->done_blocks, 1u) == gridDim.x - 1;
  __syncthreads();
  if (s_last && threadIdx.x == 0) lv_close_round(p);
}

// ---- persistent narrow rounds ---------------------------------------------
// While the frontier is narrow, a round's work is a few microseconds of
// dependent loads per wave, and two kernel launches per round (each starting
// with cold instruction / scalar / data caches on every CU) cost far more than
// the work. lv_persist keeps one resident workgroup per CU and runs round
// after round: lv_expand<FUSED> stages every closed child with write-through
// stores and inserts it at once, then a grid barrier ends the round, and
// every workgroup closes it identically from the round's atomic counters (its
// own copy of the run state, in LDS). It stops when the search ends, the
// frontier outgrows it (the host goes on with lv_round / lv_insert), or after
// max_rounds rounds (the host checks its deadline between launches).
//
// Memory protocol (inter-workgroup hand-offs inside one launch): everything a
// workgroup writes that another reads in this launch is stored write-through
// (agent-scope stores) and drained (vmcnt(0)) before the atomic that
// publishes it; inside a round, staged configurations are read back only with
// agent-scope loads; across rounds, every workgroup runs one agent-scope
// acquire after the barrier before any plain load. Counters and the tables are
// atomics only.

// Barrier words (zeroed by the host before every launch), one per 128-byte line.
struct LvBar {
  uint32_t grp[8][32];  // arrivals of blocks b with b % 8 == g (block-to-XCD placement is only a speed hint)
  uint32_t top[32];     // arrivals of the group leaders
  uint32_t gen[32];     // the last completed barrier epoch
  uint32_t abort[32];   // set by a block whose wait timed out: every block leaves
};

struct LvPersist {
  LvCtl* ctl3;                // round r counts in ctl3[r % 3]
  LvBar* bar;
  uint8_t* stg[2];            // round r stages into stg[r & 1]; its frontier is stg[(r + 1) & 1]
  uint32_t* idx[2];
  unsigned long long* ht[2];  // round r inserts into ht[r & 1]
  uint32_t max_rounds;        // rounds per launch
  uint32_t nf_max;            // leave when the frontier is wider
  unsigned long long spin_ticks;  // barrier wait limit (wall-clock ticks)
};

// Grid barrier for epoch e = 1, 2, ... (monotonic counters: no reset inside a
// launch). Returns false when the wait timed out or another block gave up.
__device__ __forceinline__ bool lv_grid_sync(LvBar* B, uint32_t e, unsigned long long spin_ticks) {
  __shared__ uint32_t s_ok;
  lv_drain();  // this wave's write-through stores have landed
  __syncthreads();
  if (threadIdx.x == 0) {
    const uint32_t G = gridDim.x, g = blockIdx.x & 7u;
    const uint32_t ng = min(G, 8u);
    const uint32_t gsz = G / 8u + (g < G % 8u ? 1u : 0u);
    const uint32_t v = atomicAdd(&B->grp[g][0], 1u) + 1u;
    if (v == e * gsz) {
      const uint32_t t = atomicAdd(&B->top[0], 1u) + 1u;
      if (t == e * ng) st_wt32(&B->gen[0], e);
    }
    uint32_t ok = 1;
    const unsigned long long t0 = wall_clock64();
    while (ld_agent(&B->gen[0]) < e) {
      if (ld_agent(&B->abort[0])) { ok = 0; break; }
      __builtin_amdgcn_s_sleep(2);
      if (wall_clock64() - t0 > spin_ticks) {
        atomicExch(&B->abort[0], 1u);
        ok = 0;
        break;
      }
    }
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");  // this CU's stale lines go
    lv_drain();                                        // ... before any wave of the block loads
    s_ok = ok;
  }
  __syncthreads();
  return s_ok != 0;
}

template <int NQ>
__global__ __launch_bounds__(LV_BLOCK) void lv_persist(LvParams p, LvPersist q) {
  __shared__ LvHeadsLds<NQ> s_heads[LV_BLOCK / 64];
  __shared__ uint32_t s_cs[64 * NQ];
  __shared__ LvRun s_run;
  for (uint32_t x = threadIdx.x; x < 64u * NQ; x += LV_BLOCK) s_cs[x] = x < p.K ? p.cs[x] : 0u;
  if (threadIdx.x == 0) s_run = *p.run;  // written by an earlier launch
  __syncthreads();
  if (s_run.done != LVR_RUNNING) return;
  const uint32_t nwaves = gridDim.x * (LV_BLOCK / 64);
  bool ok = true;
#ifdef S2LC_PROF
  unsigned long long t_round = wall_clock64();
#endif
  for (uint32_t it = 0; ok; ++it) {
    const uint32_t r = s_run.round + 1;  // the round this iteration expands
    LvParams rp = p;
    rp.round = r;
    rp.cur = q.stg[(r + 1) & 1]; rp.cur_idx = q.idx[(r + 1) & 1];
    rp.stg = q.stg[r & 1]; rp.nxt_idx = q.idx[r & 1];
    rp.ht = q.ht[r & 1]; rp.ht_clear = q.ht[(r + 1) & 1];
    rp.ctl = q.ctl3 + (r % 3);
    rp.clear_slots = 1;
    rp.init = 0;
    if (blockIdx.x == 0) {  // the counters of round r + 1 (last read in round r - 2's close)
      uint32_t* z = reinterpret_cast<uint32_t*>(q.ctl3 + ((r + 1) % 3));
      for (uint32_t i = threadIdx.x; i < sizeof(LvCtl) / 4; i += LV_BLOCK) st_wt32(z + i, 0u);
    }
    LvRoundIn in;
    in.f0 = 0;
    in.nf = s_run.nf;
    in.S = lv_slices(p.K, in.nf, nwaves, s_run.last_nf, s_run.last_children);
    in.tbase = (uint32_t)s_run.tnext;
    in.wit = s_run.witness;
    const bool worked = lv_expand<NQ, true>(rp, in, s_heads[threadIdx.x >> 6], s_cs);
#ifdef S2LC_PROF
    if (worked && (threadIdx.x & 63) == 0 && p.prof) atomicMax(&rp.ctl->prof_end, wall_clock64());
#else
    (void)worked;
#endif
    ok = lv_grid_sync(q.bar, it + 1, q.spin_ticks);
#ifdef S2LC_PROF
    if (blockIdx.x == 0 && threadIdx.x == 0 && p.prof) {
      // [9] round time, [10] expansion critical path, [11] rounds (wall-clock ticks)
      const unsigned long long t_b = wall_clock64(), e = ld_agent64(&rp.ctl->prof_end);
      atomicAdd(&p.prof[9], t_b - t_round);
      atomicAdd(&p.prof[10], e > t_round ? e - t_round : 0ull);
      atomicAdd(&p.prof[11], 1ull);
      t_round = t_b;
    }
#endif
    if (threadIdx.x == 0) {
      if (ok) {
        const LvCounts k = lv_read_counts(rp.ctl);
        lv_close_state(s_run, k, r, blockIdx.x == 0 ? p.rcounts : nullptr, p.scap, p.trace_cap);
      } else {
        s_run.done = LVR_ABORT;
      }
    }
    __syncthreads();
    if (s_run.done != LVR_RUNNING || it + 1 >= q.max_rounds || s_run.nf > q.nf_max) break;
  }
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    if (ld_agent(&q.bar->abort[0])) s_run.done = LVR_ABORT;  // some block left early: nothing here is valid
    *p.run = s_run;
    if (p.publish) lv_publish(s_run, p.publish);
  }
}

// Round 0 setup on the device: the run state of a fresh search.
__global__ __attribute__((unused)) void lv_run_init(LvRun* R, unsigned long long tnext, uint32_t witness,
                                                    unsigned long long max_configs) {
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  R->done = LVR_RUNNING; R->round = 0; R->nf = 0; R->max_frontier = 0;
  R->configs = 0; R->children = 0; R->tnext = tnext; R->max_configs = max_configs;
  R->found_parent = TRACE_NONE; R->found_move = LV_NONE; R->found_p4 = 0;
  R->witness = witness; R->deep_trace = TRACE_NONE; R->deep_len = 0; R->last_tbase = TRACE_NONE;
  R->last_nf = 0; R->last_children = 0;
}

// ---- distributed: owner of a configuration ---------------------------------
// Independent of the table slot (low fingerprint bits) and tag (high bits).
__host__ __device__ __forceinline__ uint32_t lv_owner(uint64_t fp, uint32_t world) {
  return (uint32_t)(((fp * 0xD6E8FEB86659FD93ull) >> 40) % world);
}

// Distributed staging walk: k -> stripe k & 63, index k >> 6, for k below
// p.dense = 64 * (the longest stripe) (set by the host from the round's counters).
// one lane per staging slot: owner bucket and position within it (LV_NONE for holes)
template <int NQ>
__global__ __launch_bounds__(LV_BLOCK) void lv_bucket(LvParams p) {
  for (uint32_t k = blockIdx.x * LV_BLOCK + threadIdx.x; k < p.dense; k += gridDim.x * LV_BLOCK) {
    const uint32_t st = k & (LV_STRIPES - 1), i = k / LV_STRIPES, slot = st * p.scs + i;
    if (i >= min(p.ctl->cnt[16 * st], p.scs)) continue;
    const LCfg<NQ>* c = lv_cfg<NQ>(p.stg, slot);
    if (c->move == LV_HOLE) { p.own_pos[slot] = LV_NONE; continue; }
    const uint32_t o = lv_owner(c->fp, p.world);
    const uint32_t pos = atomicAdd(&p.own_cnt[o], 1u);
    p.own_pos[slot] = (o << 27) | pos;
  }
}

// one lane per 16-byte piece: copy staged configurations into their owner's bucket
template <int NQ>
__global__ __launch_bounds__(LV_BLOCK) void lv_scatter(LvParams p) {
  constexpr uint32_t PER = sizeof(LCfg<NQ>) / 16;
  const uint64_t total = (uint64_t)p.dense * PER;
  for (uint64_t x = (uint64_t)blockIdx.x * LV_BLOCK + threadIdx.x; x < total; x += (uint64_t)gridDim.x * LV_BLOCK) {
    const uint32_t k = (uint32_t)(x / PER), c = (uint32_t)(x % PER);
    const uint32_t st = k & (LV_STRIPES - 1), i = k / LV_STRIPES, slot = st * p.scs + i;
    if (i >= min(p.ctl->cnt[16 * st], p.scs)) continue;
    const uint32_t op = p.own_pos[slot];
    if (op == LV_NONE) continue;
    const uint64_t dst = p.own_off[op >> 27] + (op & ((1u << 27) - 1));
    const uint4* src = reinterpret_cast<const uint4*>(lv_cfg<NQ>(p.stg, slot));
    reinterpret_cast<uint4*>(p.send + dst * sizeof(LCfg<NQ>))[c] = src[c];
  }
}

// keep the frontier configurations this rank owns (replicated -> partitioned)
template <int NQ>
__global__ __launch_bounds__(LV_BLOCK) void lv_keep(LvParams p, uint32_t rank) {
  const uint32_t nf = p.f1;
  for (uint32_t b0 = blockIdx.x * LV_BLOCK; b0 < nf; b0 += gridDim.x * LV_BLOCK) {
    const uint32_t i = b0 + threadIdx.x;
    uint32_t k = 0;
    bool mine = false;
    if (i < nf) {
      k = p.cur_idx[i];
      mine = lv_owner(lv_cfg<NQ>(p.cur, k)->fp, p.world) == rank;
    }
    const uint32_t n = wave_alloc(&p.ctl->nnext, mine ? 1u : 0u);
    if (mine) p.nxt_idx[n] = k;
  }
}

// copy the frontier's configurations contiguously into p.send (16 B per lane)
template <int NQ>
__global__ __launch_bounds__(LV_BLOCK) void lv_gather_frontier(LvParams p) {
  constexpr uint32_t PER = sizeof(LCfg<NQ>) / 16;
  const uint64_t total = (uint64_t)p.f1 * PER;
  for (uint64_t i = (uint64_t)blockIdx.x * LV_BLOCK + threadIdx.x; i < total; i += (uint64_t)gridDim.x * LV_BLOCK) {
    const uint32_t f = (uint32_t)(i / PER), c = (uint32_t)(i % PER);
    const uint4* src = reinterpret_cast<const uint4*>(lv_cfg<NQ>(p.cur, p.cur_idx[f]));
    reinterpret_cast<uint4*>(p.send + (uint64_t)f * sizeof(LCfg<NQ>))[c] = src[c];
  }
}

__global__ __attribute__((unused)) void lv_iota(uint32_t* out, uint32_t n) {
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) out[i] = i;
}

}  // namespace
}  // namespace s2lc
