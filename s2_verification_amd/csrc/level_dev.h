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
// Index bit of a frontier / table entry in a partitioned round (distributed
// search): the configuration lives in the rank's local staging (its own share
// of what it expanded, never sent), not in the received exchange blocks.
constexpr uint32_t LV_LOCAL = 1u << 30;

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
  uint64_t chx;     // XOR of its chain terms (lv_chain_term): its children's fingerprints start here
  uint32_t _pad[18];
  uint16_t cnt[64 * NQ];
};
static_assert(offsetof(LCfg<1>, trace) == 40 && offsetof(LCfg<1>, chx) == 48, "LCfg header offsets");
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
  uint32_t found_parent, found_move, found_p4, closed;  // closed: children closed (the rest failed the P1 precheck)
  unsigned long long children;  // children generated this round
  unsigned long long prof_end;  // S2LC_PROF: latest expansion end of the round (wall clock)
  uint32_t stop;      // lv_persist: the run's deadline passed (set by workgroup 0 before the round's barrier)
  uint32_t xblocks;   // lv_xsend blocks finished (the last one writes the exchange headers)
  uint32_t staged;    // closed children staged this round (lv_round, grid rounds)
  uint32_t _pad;
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
enum : uint32_t { LVR_RUNNING = 0, LVR_FOUND = 1, LVR_EMPTY = 2, LVR_BUDGET = 3, LVR_OVERFLOW = 4, LVR_ABORT = 5,
                  LVR_TIMEOUT = 6 };  // (timeout: the run's device deadline passed inside lv_persist)
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
  unsigned long long last_closed;  // children it closed (slices per configuration)
  uint32_t solo_rounds;    // rounds run as solo rounds (LvSolo)
  uint32_t solo_skip;      // a round a solo phase handed to the grid (too many live moves)
  // wall-clock ticks of the rounds by their frontier (the configurations they
  // expand): narrower than LV_WIDE_NF (the rounds the distributed search
  // replicates) or not (the ones it partitions); t_last = the last close
  unsigned long long t_last, narrow_ticks, wide_ticks, solo_ticks;  // (solo rounds: part of narrow)
};
static_assert(sizeof(LvRun) == 128, "LvRun layout");
constexpr uint32_t LV_WIDE_NF = 4096;  // (distributed.py's default `wide`)

struct LvParams {
  // test knob (S2LC_TAG_DROP, zero in production): bits cleared from every
  // dedupe table tag and first probe slot, so that distinct configurations
  // meet on one tag and the compare-and-probe paths run all the time
  uint32_t tag_drop;
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
  uint32_t fused;        // lv_round inserts its children itself (lv_stage_insert); lv_insert only closes
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
  // host-free partitioned rounds: fixed-capacity exchange blocks (xcap
  // configurations per owner, header in the block's first slot; 0 = the
  // variable-size buckets above) and the host-mapped status ring
  uint32_t xcap;
  struct LvXStat* xstat;
  // partitioned rounds: the rank keeps its own share of what it staged
  // (LV_LOCAL): cur_loc holds the current frontier's local part, stg_loc this
  // round's local staging (lv_insert), xself the rank's own exchange header
  uint32_t rank;
  const uint8_t* cur_loc;
  uint8_t* stg_loc;
  struct LvXHdr* xself;
  unsigned long long* prof;  // S2LC_PROF builds: lv_round phase cycles (nullable)
  // per-op longest partial linearizations (s2lc_check_partials): for every
  // inserted configuration c and chain j, pmax[cs[j] + cnt_c[j]] = max of
  // (|c| << 32 | c's trace id), |c| = its linearized ops (nullable)
  unsigned long long* pmax;
};

// ---- distributed: owner of a configuration ---------------------------------
// Independent of the table slot (low fingerprint bits) and tag (high bits).
__host__ __device__ __forceinline__ uint32_t lv_owner(uint64_t fp, uint32_t world) {
  return (uint32_t)(((fp * 0xD6E8FEB86659FD93ull) >> 40) % world);
}

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
// P1 bounds in 32 bits for H_TAIL32 histories (every reachable tail is below
// 2^32 - 3): a monotone map, so minima commute with it, and every comparison
// the search makes against a reachable tail (and P4's "no bound left") gives
// the same answer: a real requirement at or above 2^32 - 3 -> 0xFFFFFFFD,
// REQ_HASH_ONLY -> 0xFFFFFFFE, REQ_NONE -> 0xFFFFFFFF (as pack_closure).
__device__ __forceinline__ uint32_t suf32(uint64_t v) {
  const uint32_t lo = (uint32_t)v, hi = (uint32_t)(v >> 32);
  return hi == 0 ? min(lo, 0xFFFFFFFDu) : (hi == 0xFFFFFFFFu && lo >= 0xFFFFFFFEu) ? lo : 0xFFFFFFFDu;
}
__device__ __forceinline__ uint64_t suf64_of32(uint32_t b) {
  return b == 0xFFFFFFFFu ? REQ_NONE : b == 0xFFFFFFFEu ? REQ_HASH_ONLY : (uint64_t)b;
}
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

// A parent's head (record bytes 16..47 and its flags, already loaded) into
// LDS slot q; returns its hot fields.
template <int NQ>
__device__ __forceinline__ LvHot lv_put_parent_head(const uint4& a, const uint4& b, uint32_t fl, LvHeadsLds<NQ>& L,
                                                    int q, int lane) {
  LvHot h;
  h.suf = (uint64_t)b.x | ((uint64_t)b.y << 32);
  h.call = b.z;
  h.ret = b.w;
  h.fl = fl;
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
  const bool t32 = hflags & H_TAIL32;  // the P1 bound reduces in 32 bits (suf32)
  uint32_t minret_prev = minret_seed;
  for (;;) {
    uint32_t mr = EV_INF;
    uint64_t bd = REQ_NONE;
    uint32_t bd32 = 0xFFFFFFFFu;
    uint32_t adv = 0;
    bool dead = false;
#pragma unroll
    for (int q = 0; q < NQ; ++q) {
      const LvHot& h = H[q];
      mr = min(mr, h.ret);
      if (t32) bd32 = min(bd32, suf32(h.suf));
      else bd = lv_min64(bd, h.suf);
      if (!(h.fl & OPF_CLS_E) || h.call >= minret_prev) continue;
      uint32_t bits = h.fl;
      if (!(bits & HB_KNOWN)) bits = lv_legal_bits(h.fl, PL.otail[q][lane], PL.ohash[q][lane], s);
      if (bits & HB_LEGAL) adv |= 1u << q;
      else if (p2 && (bits & HB_P2DEAD)) dead = true;
    }
    const uint32_t minret = wave_min_u32(mr);
    const uint64_t bound = t32 ? suf64_of32(wave_min_u32(bd32)) : wave_min_u64(bd);
    if (__ballot(dead) || (nowrap && s.tail > bound)) return CL_DEAD;
    const bool changed = __ballot(adv != 0) != 0;
    if (!changed && minret == minret_prev) {
      minret_out = minret;
      return minret == EV_INF ? CL_COMPLETE : ((p4 && bound == REQ_NONE) ? CL_P4 : CL_ALIVE);
    }
    if (NQ <= 5) {
      // grid rounds (NQ <= 5): every slot's next head loaded at once, unconditionally
      // (a slot that does not advance reloads its current head, cached), so
      // the pass waits one memory latency, not one or two per advancing slot
      uint4 ca[NQ], cb[NQ];
      uint32_t cf[NQ];
#pragma unroll
      for (int q = 0; q < NQ; ++q) {
        const OpRec* r = recs + s_cs[64 * q + lane] + cnt[q] + d[q] + ((adv >> q) & 1u);
        ca[q] = ld16(r, 16);
        cb[q] = ld16(r, 32);
        cf[q] = r->flags;
      }
#pragma unroll
      for (int q = 0; q < NQ; ++q) {
        if ((adv >> q) & 1u) {
          d[q] += 1;
          H[q].suf = (uint64_t)cb[q].x | ((uint64_t)cb[q].y << 32);
          H[q].call = cb[q].z;
          H[q].ret = cb[q].w;
          H[q].fl = cf[q] | HB_KNOWN |
                    lv_legal_bits(cf[q], (uint64_t)ca[q].x | ((uint64_t)ca[q].y << 32),
                                  (uint64_t)ca[q].z | ((uint64_t)ca[q].w << 32), s);
        }
      }
      minret_prev = minret;
      continue;
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
                                         uint64_t fp, uint64_t chx, uint32_t minret, uint32_t ptrace, uint32_t move,
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
    o->trace = TRACE_NONE; o->slot = LV_NONE; o->chx = chx;
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

constexpr uint32_t LV_PROF_ROUNDS = 16384;  // S2LC_PROF: persistent grid rounds logged one by one
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
  // (masks, not a select chain: the compiler turned that back into an
  // indexed private array, i.e. a scratch store per update and a scratch
  // load per move on the round's critical path)
  uint32_t v = 0;
#pragma unroll
  for (int i = 0; i < NQ; ++i) v |= cnt[i] & (0u - (uint32_t)(q == (uint32_t)i));
  return v;
}

template <int N>
__device__ __forceinline__ uint32_t sel_u32(const uint32_t (&a)[N], uint32_t q) {
  uint32_t v = 0;
#pragma unroll
  for (int i = 0; i < N; ++i) v |= a[i] & (0u - (uint32_t)(q == (uint32_t)i));
  return v;
}
template <int N>
__device__ __forceinline__ uint64_t sel_u64(const uint64_t (&a)[N], uint32_t q) {
  uint64_t v = 0;
#pragma unroll
  for (int i = 0; i < N; ++i) v |= a[i] & (0ull - (uint64_t)(q == (uint32_t)i));
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
// Plain loads / stores through a global (address space 1) pointer. A pointer
// that reaches a noinline function (the solo rounds) is generic, and generic
// accesses compile to flat_* instructions, which count on lgkmcnt as well as
// vmcnt: every later LDS wait (s_waitcnt lgkmcnt(0)) then also waits for the
// memory access (round 6: C5's solo rounds 61.2 -> 60.5 ms with these,
// profiles/r06/solo_args_ab.txt).
typedef unsigned int lv_u32x4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ uint4 lv_gld16(const void* p) {
  const lv_u32x4 v = *(const __attribute__((address_space(1))) lv_u32x4*)p;
  return make_uint4(v.x, v.y, v.z, v.w);
}
__device__ __forceinline__ uint32_t lv_gld32(const void* p) { return *(const lv_g32*)p; }
__device__ __forceinline__ unsigned long long lv_gld64(const void* p) { return *(const lv_g64*)p; }
__device__ __forceinline__ void lv_gst32(void* p, uint32_t v) { *(lv_g32*)p = v; }
__device__ __forceinline__ void lv_gst64(void* p, unsigned long long v) { *(lv_g64*)p = v; }
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
  uint32_t par;     // solo rounds: the round's counter slot (LvSolo::c)
  uint32_t S;       // slices per configuration
  uint32_t tbase;   // trace index of the round's first winner (fused insert)
  uint32_t wit;     // record trace entries (fused insert)
};

// Slices per configuration: narrow frontiers spread a configuration's moves
// over several waves (down to about one child per wave), wide ones give a wave
// whole configurations. The expected moves per configuration come from the
// previous round.
#ifndef S2LC_SLICE_WAVES
#define S2LC_SLICE_WAVES 2  // items per wave a round may make (x the waves)
#endif
#ifndef S2LC_SLICE_KIDS
#define S2LC_SLICE_KIDS 1   // expected closed children per item
#endif
__device__ __forceinline__ uint32_t lv_slices(uint32_t K, uint32_t nf, uint32_t nwaves, uint32_t last_nf,
                                              unsigned long long last_closed) {
  uint32_t c_est = K;
  if (last_nf) c_est = (uint32_t)min<unsigned long long>(K, last_closed / last_nf + 1);
  c_est = (c_est + S2LC_SLICE_KIDS - 1) / S2LC_SLICE_KIDS;
  return max(1u, min(c_est + (c_est >> 2) + 1, (S2LC_SLICE_WAVES * nwaves + nf - 1) / max(nf, 1u)));
}

// A configuration's counters (lane l holds chains l + 64 q) with 8-byte
// write-through stores: lanes l = 0 mod 4 store chains l .. l+3 of each slot
// (a 2-byte write-through store per lane costs a memory write per request).
template <int NQ>
__device__ __forceinline__ void lv_store_cnt_wt(uint16_t* dst, const uint32_t (&cnt)[NQ], const uint32_t (&d)[NQ]) {
  const int lane = (int)(threadIdx.x & 63);
#pragma unroll
  for (int q = 0; q < NQ; ++q) {
    const uint32_t v = (cnt[q] + d[q]) & 0xFFFFu;
    const uint32_t p2 = v | ((uint32_t)__shfl_xor((int)v, 1, 64) << 16);  // chains l, l+1 (l even)
    const uint32_t o2 = (uint32_t)__shfl_xor((int)p2, 2, 64);              // chains l+2, l+3
    if ((lane & 3) == 0) st_wt64(dst + 64 * q + lane, ((unsigned long long)o2 << 32) | p2);
  }
}

// Persistent kernel: stage one closed child with write-through stores and
// insert it at once (the producing wave deduplicates its own child: a 64-bit
// CAS, and on a tag hit a wave-parallel compare against the resident entry).
template <int NQ>
__device__ __forceinline__ void lv_stage_insert(const LvParams& p, const LvRoundIn& in, uint32_t st, uint32_t& rk,
                                                uint32_t& rleft, const State& s, uint64_t fp, uint64_t chx,
                                                uint32_t minret, uint32_t ptrace, uint32_t move,
                                                const uint32_t (&cnt)[NQ], const uint32_t (&d)[NQ]) {
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
  // The CAS goes first: the entry is published PENDING (bit 31 of the index)
  // and made final once the winner's stores have landed, so a duplicate writes
  // nothing at all (wide rounds stage several copies of most configurations).
  // A wave that meets a pending entry with its tag waits for the final form
  // before it reads the configuration.
  const uint32_t tag = (uint32_t)(fp >> 32) & ~p.tag_drop;
  const unsigned long long mine = ((unsigned long long)tag << 32) | k;
  uint32_t slot = (uint32_t)fp & p.ht_mask & ~p.tag_drop;
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
  // the winner: next-frontier position, then the configuration (header line:
  // lanes 0..15 store one 8-byte word each, one whole-line store), its index
  // and trace entry; its stores land, then the entry loses its PENDING bit
  uint32_t n = 0;
  if (lane == 0) n = atomicAdd(&p.ctl->nnext, 1u);
  n = rl(n, 0);
  const uint32_t tr = in.wit ? p.tgid + in.tbase + n : TRACE_NONE;
  const unsigned long long w = lane == 0 ? s.tail
                             : lane == 1 ? s.hash
                             : lane == 2 ? fp
                             : lane == 3 ? ((unsigned long long)minret << 32 | s.tok)
                             : lane == 4 ? ((unsigned long long)move << 32 | ptrace)
                             : lane == 5 ? ((unsigned long long)slot << 32 | tr)
                             : lane == 6 ? chx
                                         : 0ull;
  if (lane < 16) st_wt64(reinterpret_cast<unsigned long long*>(o) + lane, w);
  lv_store_cnt_wt<NQ>(o->cnt, cnt, d);
  if (lane == 0) {
    st_wt32(&p.nxt_idx[n], k);
    if (in.wit) p.trace[in.tbase + n] = TraceEnt{ptrace, move};
  }
  lv_drain();
  if (lane == 0) atomicExch(&p.ht[slot], mine);
}

// S2LC_BATCH_INSERT (default on): the persistent rounds' children are staged
// first (the whole configuration, drained once per batch) and inserted LV_PEND
// at a time, one lane per child: one CAS latency for the batch, tag hits
// compared four at a time, one next-frontier atomic for the batch's winners.
// Inserting each child on its own cost a chain of device-scope round trips per
// child (~4.6 us each in C5's slowest grid rounds). C5 0.0913 -> 0.0905 s,
// C5wide 0.0369 -> 0.0362 s (profiles/r05/c5_batch_insert_ab.txt); the
// configurations and rounds are unchanged.
#ifndef S2LC_BATCH_INSERT
#define S2LC_BATCH_INSERT 1
#endif
constexpr uint32_t LV_PEND = 32;
struct LvPend {
  unsigned long long fp[LV_PEND];
  uint32_t k[LV_PEND], mv[LV_PEND], pt[LV_PEND];
};

template <int NQ>
__device__ __forceinline__ void lv_flush_pend(const LvParams& p, const LvRoundIn& in, LvPend& P, uint32_t& np) {
  if (np == 0) return;
  const int lane = (int)(threadIdx.x & 63);
  lv_drain();  // every pending configuration has landed
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  __builtin_amdgcn_wave_barrier();
  const bool act = (uint32_t)lane < np;
  const unsigned long long fp = act ? P.fp[lane] : 0ull;
  const uint32_t k = act ? P.k[lane] : 0u;
  const uint32_t tag = (uint32_t)(fp >> 32) & ~p.tag_drop;
  const unsigned long long mine = ((unsigned long long)tag << 32) | k;
  uint32_t slot = (uint32_t)fp & p.ht_mask & ~p.tag_drop;
  bool probing = act, win = false;
  while (__ballot(probing)) {
    unsigned long long prev = HT_EMPTY;
    if (probing) prev = atomicCAS(&p.ht[slot], HT_EMPTY, mine);
    const bool hit = probing && prev != HT_EMPTY && (uint32_t)(prev >> 32) == tag;
    if (probing && prev == HT_EMPTY) {
      win = true;
      probing = false;
    } else if (probing && !hit) {
      slot = (slot + 1) & p.ht_mask;  // another configuration's entry: the next slot
    }
    // the tag hits: each resident configuration compared with the pending one,
    // wave-parallel, LV_CMP of them with their loads in flight together
    constexpr int LV_CMP = 4;
    uint64_t hm = __ballot(hit);
    while (hm) {
      int jj[LV_CMP];
      bool ne[LV_CMP];
#pragma unroll
      for (int c = 0; c < LV_CMP; ++c) {
        jj[c] = hm ? __ffsll((unsigned long long)hm) - 1 : -1;
        if (hm) hm &= hm - 1;
      }
#pragma unroll
      for (int c = 0; c < LV_CMP; ++c) {
        ne[c] = false;
        if (jj[c] < 0) continue;
        const LCfg<NQ>* e = lv_cfg<NQ>(p.stg, (uint32_t)rl64(prev, jj[c]));
        const LCfg<NQ>* m = lv_cfg<NQ>(p.stg, rl(k, jj[c]));
        const unsigned long long et = ld_wt64(&e->tail), eh = ld_wt64(&e->hash), ek = ld_wt64(&e->tok);
        const unsigned long long mt = ld_wt64(&m->tail), mh = ld_wt64(&m->hash), mk = ld_wt64(&m->tok);
        bool x = et != mt || eh != mh || (uint32_t)ek != (uint32_t)mk;
#pragma unroll
        for (int q = 0; q < NQ; ++q) x |= ld_wt16(&e->cnt[lane + 64 * q]) != ld_wt16(&m->cnt[lane + 64 * q]);
        ne[c] = x;
      }
#pragma unroll
      for (int c = 0; c < LV_CMP; ++c) {
        if (jj[c] < 0) continue;
        const bool eq = __ballot(ne[c]) == 0;
        if (lane == jj[c]) {
          if (eq) probing = false;  // an equal configuration is already in the round
          else slot = (slot + 1) & p.ht_mask;
        }
      }
    }
  }
  // the winners' next-frontier positions: one atomic for the batch
  const uint64_t wm = __ballot(win);
  uint32_t base = 0;
  if (lane == 0 && wm) base = atomicAdd(&p.ctl->nnext, (uint32_t)__popcll(wm));
  base = rl(base, 0);
  if (win) {
    const uint32_t n = base + (uint32_t)__popcll(wm & ((1ull << lane) - 1));
    const uint32_t tr = in.wit ? p.tgid + in.tbase + n : TRACE_NONE;
    st_wt64(reinterpret_cast<unsigned long long*>(lv_cfg<NQ>(p.stg, k)) + 5, (unsigned long long)slot << 32 | tr);
    st_wt32(&p.nxt_idx[n], k);
    if (in.wit) p.trace[in.tbase + n] = TraceEnt{P.pt[lane], P.mv[lane]};
  }
  np = 0;
}

// Stage one closed child for a batched insert: the configuration (all but its
// slot / trace word) with write-through stores, its key in the wave's list.
template <int NQ>
__device__ __forceinline__ void lv_stage_pend(const LvParams& p, const LvRoundIn& in, uint32_t st, uint32_t& rk,
                                              uint32_t& rleft, const State& s, uint64_t fp, uint64_t chx,
                                              uint32_t minret, uint32_t ptrace, uint32_t move,
                                              const uint32_t (&cnt)[NQ], const uint32_t (&d)[NQ], LvPend& P,
                                              uint32_t& np) {
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
  const unsigned long long w = lane == 0 ? s.tail
                             : lane == 1 ? s.hash
                             : lane == 2 ? fp
                             : lane == 3 ? ((unsigned long long)minret << 32 | s.tok)
                             : lane == 4 ? ((unsigned long long)move << 32 | ptrace)
                             : lane == 6 ? chx
                                         : 0ull;
  if (lane < 16 && lane != 5) st_wt64(reinterpret_cast<unsigned long long*>(o) + lane, w);
  lv_store_cnt_wt<NQ>(o->cnt, cnt, d);
  if (lane == 0) {
    P.fp[np] = fp;
    P.k[np] = k;
    P.mv[np] = move;
    P.pt[np] = ptrace;
  }
  if (++np == LV_PEND) lv_flush_pend<NQ>(p, in, P, np);
}

// Workgroup barrier over LDS only: waits for this wave's LDS operations, not
// for its global loads and write-through stores (a __syncthreads release
// would drain those too). Solo rounds share only LDS between their waves.
__device__ __forceinline__ void lv_sync_lds() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

// (smallest, second smallest) of the heads' P1 bounds over the wave's chains
// (a value held by two chains is both), in every lane.
template <int CTRL>
__device__ __forceinline__ void lv_min2_step(uint64_t& a, uint64_t& b) {
  const uint64_t oa = lv_dpp64<CTRL>(a), ob = lv_dpp64<CTRL>(b);
  const uint64_t lo = lv_min64(a, oa), hi = a < oa ? oa : a;
  b = lv_min64(hi, lv_min64(b, ob));
  a = lo;
}
template <int NQ>
__device__ __forceinline__ void wave_min2_hot(const LvHot (&H)[NQ], uint64_t& m1, uint64_t& m2) {
  uint64_t a = REQ_NONE, b = REQ_NONE;
#pragma unroll
  for (int q = 0; q < NQ; ++q) {
    const uint64_t v = H[q].suf;
    if (v < a) { b = a; a = v; } else if (v < b) { b = v; }
  }
  lv_min2_step<0xB1>(a, b);
  lv_min2_step<0x4E>(a, b);
  lv_min2_step<0x124>(a, b);
  lv_min2_step<0x128>(a, b);
  m1 = REQ_NONE; m2 = REQ_NONE;
#pragma unroll
  for (int row = 0; row < 4; ++row) {
    const uint64_t ra = rl64(a, 16 * row), rb = rl64(b, 16 * row);
    const uint64_t lo = lv_min64(m1, ra), hi = m1 < ra ? ra : m1;
    m2 = lv_min64(hi, lv_min64(m2, rb));
    m1 = lo;
  }
}

template <int CTRL>
__device__ __forceinline__ void lv_min2_step32(uint32_t& a, uint32_t& b) {
  const uint32_t oa = lv_dpp<CTRL>(a), ob = lv_dpp<CTRL>(b);
  const uint32_t lo = min(a, oa), hi = max(a, oa);
  b = min(hi, min(b, ob));
  a = lo;
}
template <int NQ>
__device__ __forceinline__ void wave_min2_hot32(const LvHot (&H)[NQ], uint32_t& m1, uint32_t& m2) {
  uint32_t a = 0xFFFFFFFFu, b = 0xFFFFFFFFu;
#pragma unroll
  for (int q = 0; q < NQ; ++q) {
    const uint32_t v = suf32(H[q].suf);
    if (v < a) { b = a; a = v; } else if (v < b) { b = v; }
  }
  lv_min2_step32<0xB1>(a, b);
  lv_min2_step32<0x4E>(a, b);
  lv_min2_step32<0x124>(a, b);
  lv_min2_step32<0x128>(a, b);
  m1 = 0xFFFFFFFFu; m2 = 0xFFFFFFFFu;
#pragma unroll
  for (int row = 0; row < 4; ++row) {
    const uint32_t ra = rl(a, 16 * row), rb = rl(b, 16 * row);
    const uint32_t lo = min(m1, ra), hi = max(m1, ra);
    m2 = min(hi, min(m2, rb));
    m1 = lo;
  }
}

// P1 bound (sufmin) of a record
__device__ __forceinline__ uint64_t ld_suf(const OpRec* r) {
  return *reinterpret_cast<const uint64_t*>(reinterpret_cast<const uint8_t*>(r) + 32);
}

// ---- expansion: one wave per (frontier configuration, slice of its candidates)
// MODE 0: stage into the striped staging array (lv_insert deduplicates);
// MODE 1: the persistent kernel's stage-and-insert.
#ifndef S2LC_FUSED_PRE_NQ
#define S2LC_FUSED_PRE_NQ 6  // the widest layout whose persistent rounds precheck every move at once
#endif
// (A frontier of one configuration runs as solo rounds: solo_dev.h.)
template <int NQ, int MODE>
__device__ __forceinline__ bool lv_expand(const LvParams& p, const LvRoundIn& in, LvHeadsLds<NQ>& PL,
                                          const uint32_t* s_cs) {
  constexpr bool FUSED = MODE == 1;
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
  uint32_t closed = 0;  // children closed by this wave (wave-uniform)
  uint32_t staged = 0;  // children it staged (grid rounds)
  // (S2LC_BATCH_INSERT: the wave's children waiting for their batched insert)
  __shared__ LvPend s_pend[FUSED && S2LC_BATCH_INSERT ? LV_BLOCK / 64 : 1];
  LvPend& PP = s_pend[FUSED && S2LC_BATCH_INSERT ? (threadIdx.x >> 6) : 0];
  uint32_t np = 0;
#ifdef S2LC_PROF
  unsigned long long lv_acc[10] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0}, lv_t = 0;
  const unsigned long long w_t0 = clock64();
  unsigned long long w_ins = 0, w_cl = 0, w_items = 0, w_pend = 0;
#endif
  for (uint32_t it = wave_id; it < items; it += nwaves) {
#ifdef S2LC_PROF
    ++w_items;
#endif
    LV_T0();
    LV_ADD(5, 1);
    const uint32_t f = f0 + it / S;
    const uint32_t slice = it % S;
    // parent configuration (round 0: the all-zero initial one)
    const LCfg<NQ>* pc = nullptr;
    if (!p.init) {
      const uint32_t ci = p.cur_idx[f];
      // (a partitioned round's frontier: its local part in cur_loc; lv_round only)
      pc = (!FUSED && (ci & LV_LOCAL)) ? lv_cfg<NQ>(p.cur_loc, ci & ~LV_LOCAL) : lv_cfg<NQ>(p.cur, ci);
    }
    const bool has_parent = pc != nullptr;
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
    // Grid rounds: every slot's count, then every slot's head record, each
    // group issued before any is used: one memory latency per group. (Loads
    // under a per-slot condition were compiled into a wait per slot, two
    // serialized latencies per slot: ~12.6 k cycles per item for NQ = 5.)
    // Unconditional loads stay in bounds: a configuration holds 64 * NQ
    // counts, and a slot past K reads record 0 (s_cs is 0 there).
    // (NQ <= 5: wider layouts would spill the grouped registers; they load
    // per slot)
    constexpr bool HG = NQ <= 5;
    uint4 ha[HG ? NQ : 1], hb[HG ? NQ : 1];
    uint32_t hf[HG ? NQ : 1];
    if (HG) {
#pragma unroll
      for (int q = 0; q < NQ; ++q) {
        const uint32_t j = (uint32_t)lane + 64u * q;
        const uint32_t c = pc ? (uint32_t)pc->cnt[j] : 0u;
        cnt[q] = j < K ? c : 0u;
      }
#pragma unroll
      for (int q = 0; q < NQ; ++q) {
        const OpRec* r = p.recs + s_cs[64 * q + lane] + cnt[q];
        ha[HG ? q : 0] = ld16(r, 16);
        hb[HG ? q : 0] = ld16(r, 32);
        hf[HG ? q : 0] = r->flags;
      }
    }
#pragma unroll
    for (int q = 0; q < NQ; ++q) {
      const uint32_t j = (uint32_t)lane + 64u * q;
      d[q] = 0;
      if (!HG) cnt[q] = (j < K && pc) ? (uint32_t)pc->cnt[j] : 0u;
      if (j < K) {
        if (HG) {
          H[q] = lv_put_parent_head<NQ>(ha[HG ? q : 0], hb[HG ? q : 0], hf[HG ? q : 0], PL, q, lane);
        } else {
          const OpRec* r = p.recs + s_cs[64 * q + lane] + cnt[q];
          H[q] = lv_put_parent_head<NQ>(ld16(r, 16), ld16(r, 32), r->flags, PL, q, lane);
        }
      } else {
        H[q] = lv_hot_null();
        PL.fl[q][lane] = OPF_SENTINEL; PL.call[q][lane] = EV_INF; PL.ret[q][lane] = EV_INF; PL.suf[q][lane] = REQ_NONE;
      }
      if (j < K && !pc) chx ^= lv_chain_term(j, cnt[q]);  // (round 0; a staged parent carries it)
      // candidate moves: minimal durable / indefinite appends at the chain heads
      if (has_parent && !(H[q].fl & (OPF_SENTINEL | OPF_CLS_E)) && H[q].call < pmin) cand |= 1u << q;
    }
    const uint64_t parent_chx = pc ? pc->chx : wave_xor_u64(chx);
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
    const uint32_t n_moves = has_parent ? n_cand : 1u;
    const uint32_t c0 = (uint32_t)(((uint64_t)n_moves * slice) / S);
    const uint32_t c1 = (uint32_t)(((uint64_t)n_moves * (slice + 1)) / S);
    // The outcome of every move of this slice at once (lane l, slot q: the
    // append at the head of chain l + 64 q): the rest of its record, guards,
    // outcome and hash fold, for those moves in parallel, so a move in the
    // loop below costs only its next head's load. Registers: 5 per slot
    // (NQ <= 6).
    constexpr bool PRE = FUSED ? NQ <= S2LC_FUSED_PRE_NQ : NQ <= 6;
    constexpr int NP = PRE ? NQ : 1;
    uint64_t mv_tail[NP], mv_hash[NP];
    uint32_t mv_pk[NP];  // take_opt | take_id << 1 | P1-dead opt child << 2 | token << 16
    // P1 precheck: a child's P1 bound is the parent's with the moved chain's
    // head replaced by its next record, so (smallest, second smallest) head
    // bound over all chains gives every child's bound without its chain; an
    // opt child past it dies in its closure's first pass, and is counted but
    // not closed (most children of a hard history end this way)
    const bool p1 = PRE && (p.hflags & H_NOWRAP);
    const bool t32 = p.hflags & H_TAIL32;
    uint64_t b_min = REQ_NONE, b_2nd = REQ_NONE;
    uint32_t b_min32 = 0xFFFFFFFFu, b_2nd32 = 0xFFFFFFFFu;
    if (p1) {
      if (t32) wave_min2_hot32<NQ>(H, b_min32, b_2nd32);
      else wave_min2_hot<NQ>(H, b_min, b_2nd);
    }
#ifndef S2LC_PRE_GROUP
#define S2LC_PRE_GROUP 1
#endif
#ifndef S2LC_PRE_GROUP_NQ
#define S2LC_PRE_GROUP_NQ 4
#endif
    // grid rounds: the rest of every candidate's record and its next record's
    // P1 bound loaded for all slots before the precheck uses any (one latency
    // instead of one per slot with a candidate). NQ <= 4: C5wide (NQ = 4)
    // 0.0394 -> 0.0361 s; at NQ = 5 the 50 more live VGPRs cost C5 0.6 %
    // (profiles/r04/pre_group_ab.txt)
    constexpr bool PG = NQ <= S2LC_PRE_GROUP_NQ && S2LC_PRE_GROUP;
    uint4 pm0[PG ? NP : 1], pm3[PG ? NP : 1];
    uint64_t pns[PG ? NP : 1];
    if (PG) {
#pragma unroll
      for (int q = 0; q < NP; ++q) {
        const OpRec* hp = p.recs + s_cs[64 * q + lane] + cnt[q];
        pm0[q] = ld16(hp, 0);
        pm3[q] = ld16(hp, 48);
        // (a non-candidate head may be its chain's sentinel: no next record)
        pns[q] = p1 ? ld_suf(hp + ((cand >> q) & 1u)) : REQ_NONE;
      }
    }

#pragma unroll
    for (int q = 0; q < NP; ++q) {
      mv_tail[q] = ps.tail;
      mv_hash[q] = ps.hash;
      mv_pk[q] = ps.tok << 16;
      if (PRE && ((cand >> q) & 1u) && my_idx[q] >= c0 && my_idx[q] < c1) {
        const OpRec* hp = p.recs + s_cs[64 * q + lane] + cnt[q];
        // the chain's next record's P1 bound
        const uint64_t nx_suf = PG ? pns[PG ? q : 0] : (p1 ? ld_suf(hp + 1) : REQ_NONE);
        // the head: its hot part was just loaded (cached)
        OpRec r;
        if (PG) {  // bytes 0..15 and 48..63 just loaded; 16..47 in PL / H
          const uint4 a0 = pm0[PG ? q : 0], a3 = pm3[PG ? q : 0];
          r.num_records = (uint64_t)a0.x | ((uint64_t)a0.y << 32);
          r.msn = (uint64_t)a0.z | ((uint64_t)a0.w << 32);
          r.out_tail = PL.otail[q][lane]; r.out_hash = PL.ohash[q][lane]; r.sufmin = H[q].suf;
          r.call_ev = H[q].call; r.ret_ev = H[q].ret;
          r.hash_off = a3.x; r.hash_cnt = a3.y;
          r.batch_tok = (uint16_t)a3.z; r.set_tok = (uint16_t)(a3.z >> 16);
          r.flags = a3.w;
        } else {
          r = load_rec(hp);
        }
        const bool g = append_guards_ok(r, ps);
        State opt = ps;
        opt.tail = ps.tail + r.num_records;
        opt.tok = r.set_tok ? r.set_tok : ps.tok;
        bool to = (r.flags & OPF_CLS_D) ? (g && opt.tail == r.out_tail) : g;
        const uint64_t others = t32 ? suf64_of32(suf32(H[q].suf) == b_min32 ? b_2nd32 : b_min32)
                                    : (H[q].suf == b_min ? b_2nd : b_min);
        const bool p1dead = p1 && to && opt.tail > lv_min64(others, nx_suf);
        // the fold: for a live opt child, or for an indefinite append's
        // identity test (opt == s needs equal tails)
        const bool fold = (to && !p1dead) || ((r.flags & OPF_CLS_I) && g && opt.tail == ps.tail);
        if (fold) opt.hash = fold_hashes_blk(ps.hash, p.pool + r.hash_off, r.hash_cnt);
        const bool ti = (r.flags & OPF_CLS_I) && (!idefer || r.ret_ev == pmin) && !(g && state_eq(opt, ps));
        mv_tail[q] = opt.tail;
        mv_hash[q] = opt.hash;
        mv_pk[q] = (to && !p1dead ? 1u : 0u) | (ti ? 2u : 0u) | (p1dead ? 4u : 0u) | (opt.tok << 16);
      }
    }
    // the loop below visits only this slice's moves with a child to close;
    // the P1-dead opt children are counted here
    uint32_t live = cand;
    if (PRE) {
      live = 0;
#pragma unroll
      for (int q = 0; q < NP; ++q) {
        if (mv_pk[q] & 3u) live |= 1u << q;
        const uint32_t nd = (uint32_t)__popcll(__ballot((mv_pk[q] >> 2) & 1u));
        kids += nd;
        LV_ADD(9, nd);
      }
    }
    uint32_t ord = 0, q_cur = 0;
    uint64_t m = has_parent ? __ballot(live & 1u) : 1ull;
    for (;;) {
      // next move (wave-uniform): slot q_cur, owner lane src
      while (m == 0 && q_cur + 1 < (uint32_t)NQ && has_parent) {
        ++q_cur;
        m = __ballot((live >> q_cur) & 1u);
      }
      if (m == 0 || (!PRE && ord >= c1)) break;
      const int src = __ffsll((unsigned long long)m) - 1;
      m &= m - 1;
      const uint32_t o = ord++;
      if (!PRE && o < c0) continue;  // (PRE: live holds this slice's moves only)
      // children of the move: on the owner lane (round 0: the unchanged initial state)
      bool take_opt = !has_parent, take_id = false;
      State opt = ps;
      uint4 nx_obs = make_uint4(0, 0, 0, 0), nx_mid = make_uint4(0, 0, 0, 0);
      uint32_t nx_fl = 0;
      LV_LAP(7);
      uint32_t fl2;
      State so;
      if (PRE) {
        if (has_parent && lane == src) {
          // the chain's next head (the child's first new head)
          const OpRec* nx = p.recs + s_cs[64 * q_cur + lane] + sel_cnt<NQ>(cnt, q_cur) + 1;
          nx_obs = ld16(nx, 16);
          nx_mid = ld16(nx, 32);
          nx_fl = nx->flags;
        }
        const uint32_t pk = rl(sel_u32<NP>(mv_pk, q_cur), src);
        fl2 = has_parent ? (pk & 3u) : 1u;
        so = has_parent ? State{rl64(sel_u64<NP>(mv_tail, q_cur), src), rl64(sel_u64<NP>(mv_hash, q_cur), src), pk >> 16} : ps;
      } else {
        if (has_parent && lane == src) {
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
        fl2 = has_parent ? rl((take_opt ? 1u : 0u) | (take_id ? 2u : 0u), src) : 1u;
        so = State{rl64(opt.tail, src), rl64(opt.hash, src), rl(opt.tok, src)};
      }
      const uint32_t j = (uint32_t)src + 64u * q_cur;
      LV_LAP(2);
#pragma unroll 1
      for (int w = 0; w < 2; ++w) {
        if (!((fl2 >> w) & 1u)) continue;
        const State cs_ = w == 0 ? so : ps;
        const uint32_t mv = !has_parent ? LV_NONE : (w == 0 ? j : (j | MOVE_IDENT));
        if (has_parent) {
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
        ++closed;
#ifdef S2LC_PROF
        const unsigned long long w_c0 = clock64();
#endif
        const int cr = lv_closure<NQ>(H, d, cnt, s_cs, PL, lane, cs_, p.hflags, pmin, p.recs, mr);
#ifdef S2LC_PROF
        w_cl += clock64() - w_c0;
#endif
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
          const uint64_t cdx = parent_chx ^ wave_xor_u64(dx);
          auto fp_of = [&]() { return mix64(cdx ^ lv_state_term(cs_.tail, cs_.hash, cs_.tok)); };
          if (FUSED) {
#ifdef S2LC_PROF
            const unsigned long long w_i0 = clock64();
#endif
            if (S2LC_BATCH_INSERT) lv_stage_pend<NQ>(p, in, stripe, rk, rleft, cs_, fp_of(), cdx, mr, ptrace, mv, cnt, d, PP, np);
            else lv_stage_insert<NQ>(p, in, stripe, rk, rleft, cs_, fp_of(), cdx, mr, ptrace, mv, cnt, d);
#ifdef S2LC_PROF
            w_ins += clock64() - w_i0;
            ++w_pend;
#endif
          } else {
            lv_stage<NQ>(p, stripe, rk, rleft, cs_, fp_of(), cdx, mr, ptrace, mv, cnt, d);
            ++staged;
          }
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
  if (FUSED && S2LC_BATCH_INSERT) lv_flush_pend<NQ>(p, in, PP, np);
#ifdef S2LC_PROF
  if (lane == 0 && p.prof && lv_acc[5])  // only waves that had work (idle waves would swamp the counters)
    for (int i_ = 0; i_ < 9; ++i_) atomicAdd(&p.prof[i_ < 7 ? i_ : i_ + 5], lv_acc[i_]);
  if (FUSED && lane == 0 && p.prof && w_items && p.round < LV_PROF_ROUNDS) {  // per round: the busiest wave's split
    unsigned long long* pr = p.prof + 48 + 6 * LV_PROF_ROUNDS;
    atomicMax(&pr[p.round], clock64() - w_t0);
    atomicMax(&pr[LV_PROF_ROUNDS + p.round], w_ins);
    atomicMax(&pr[2 * LV_PROF_ROUNDS + p.round], w_cl);
    atomicMax(&pr[3 * LV_PROF_ROUNDS + p.round], w_items);
    atomicMax(&pr[4 * LV_PROF_ROUNDS + p.round], w_pend);
  }
#endif
  if (MODE == 0 && rleft) lv_release<NQ>(p, stripe, rk, rleft);
  if (lane == 0 && kids) atomicAdd(&p.ctl->children, kids);
  if (lane == 0 && closed) atomicAdd(&p.ctl->closed, closed);
  if (!FUSED && lane == 0 && staged) atomicAdd(&p.ctl->staged, staged);
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
  in.par = 0;
  in.f0 = p.f0;
  in.nf = p.f1 == LV_NONE ? p.run->nf : p.f1 - p.f0;
  if (p.f1 == LV_NONE) in.f0 = 0;
  if (p.init) in.nf = 1;
  const uint32_t nwaves = gridDim.x * (LV_BLOCK / 64);
  in.S = p.init ? 1u : lv_slices(p.K, in.nf, nwaves, p.run ? p.run->last_nf : 0u, p.run ? p.run->last_closed : 0ull);
  if (p.fused) {
    in.tbase = (uint32_t)p.run->tnext;
    in.wit = p.run->witness;
    lv_expand<NQ, 1>(p, in, s_heads[threadIdx.x >> 6], s_cs);
  } else {
    in.tbase = 0;
    in.wit = 0;
    lv_expand<NQ, 0>(p, in, s_heads[threadIdx.x >> 6], s_cs);
  }
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
  uint32_t closed;
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
  k.closed = ld_agent(&c->closed);
  return k;
}

// Close round `rnd` on the run state R: per-round count, run counters, and
// the decision (found / empty / budget / overflow / witness off).
__device__ __forceinline__ void lv_close_state(LvRun& R, const LvCounts& k, uint32_t rnd, uint32_t* rcounts,
                                               uint32_t scap, uint64_t trace_cap, bool clock = true) {
  if (clock) {  // (solo rounds account their phase's time once, at its end)
    const unsigned long long now = wall_clock64();
    if (rnd > 0) (R.nf >= LV_WIDE_NF ? R.wide_ticks : R.narrow_ticks) += now - R.t_last;
    R.t_last = now;
  }
  R.children += k.ch;
  R.last_nf = rnd == 0 ? 0u : R.nf;
  R.last_closed = k.closed;
  if (k.ovf) {
    R.done = LVR_OVERFLOW;  // the host re-runs this round in frontier chunks
  } else if (k.fnd) {
    R.done = LVR_FOUND;
    R.round = rnd;
    R.found_parent = R.witness ? k.fpar : TRACE_NONE;
    R.found_move = k.fmov;
    R.found_p4 = k.fp4;
  } else {
    if (rcounts) lv_gst32(rcounts + rnd, k.nn);
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

// ---- fixed-capacity exchange blocks (host-free partitioned rounds; the kernels
// that fill and read them follow lv_scatter) ----
struct LvXHdr {
  uint32_t count;     // configurations the sender staged for this block's owner (> xcap: overflow)
  uint32_t maxblk;    // the sender's largest block this round
  uint32_t found, fpar, fmov, fp4;  // a closed child completed (Ok) on the sender
  uint32_t sovf;      // the sender's staging overflowed (the round is incomplete)
  uint32_t nf;        // the frontier the sender expanded this round
  unsigned long long staged;  // the sender's staged configurations, all owners
};
struct LvXStat {       // one per round in a ring of LV_XRING (host-mapped)
  uint32_t round;      // written last: the entry is complete when it equals the round
  uint32_t done;       // LVR_* once the search stopped in this round (0: running)
  uint32_t nf;         // this rank's next frontier
  uint32_t maxblk;     // the largest block of any sender: the capacity this round needed
  unsigned long long nf_global;  // the global frontier this round expanded
  unsigned long long staged;     // configurations staged this round, all ranks
  uint32_t found_parent, found_move, found_p4, _pad;
};
constexpr uint32_t LV_XRING = 8;

template <int NQ>
__device__ __forceinline__ LvXHdr* lv_xhdr(uint8_t* buf, uint32_t o, uint32_t cap) {
  return reinterpret_cast<LvXHdr*>(buf + (size_t)o * (cap + 1) * sizeof(LCfg<NQ>));
}

struct LvXDecision {
  uint32_t halt;      // LVR_* (0: insert the round)
  uint32_t maxblk;
  uint32_t fpar, fmov, fp4;
  unsigned long long nf_global, staged;
};
template <int NQ>
__device__ __forceinline__ LvXDecision lv_xdecide(const LvParams& p);
template <int NQ>
__device__ __forceinline__ void lv_xhalt(const LvParams& p, const LvXDecision& d);
template <int NQ>
__device__ __forceinline__ void lv_xclose(const LvParams& p, const LvXDecision& d);

// ---- insert: one lane per staged configuration -----------------------------
// Striped staging: lane l of every wave walks stripe l (slot l * scs + i for
// i = lo[l] .. cnt[l]); the grid strides over i. Winners take next-frontier
// positions with one atomic per block. Dense mode (p.dense): configurations
// 0 .. dense-1 of p.stg (a distributed receive; with p.xcap, exchange blocks).
template <int NQ>
__global__ __launch_bounds__(LV_BLOCK) void lv_insert(LvParams p) {
  __shared__ uint32_t s_wcnt[LV_BLOCK / 64], s_base, s_hi, s_last;
  __shared__ LvXDecision xd;  // (thread 0: the exchanged round's decision, reused by the close; in LDS, not a private frame)
  if (p.xcap) {
    // exchanged round: every block takes the round's decision from the
    // received headers; a halting round inserts nothing (block 0 records it).
    // One thread reads the run state for the whole block: block 0 may stop
    // the run while other blocks start, and every wave of a block must leave
    // or stay together
    __shared__ uint32_t s_halt;
    if (threadIdx.x == 0) {
      uint32_t h = p.run->done ? LVR_ABORT : 0u;  // (stopped in an earlier round)
      if (!h) {
        xd = lv_xdecide<NQ>(p);
        h = xd.halt;
        if (h && blockIdx.x == 0) lv_xhalt<NQ>(p, xd);
      }
      s_halt = h;
    }
    __syncthreads();
    if (s_halt) return;
  } else if (p.run && p.run->done) {
    return;
  }
  const int lane = (int)(threadIdx.x & 63), wv = (int)(threadIdx.x >> 6);
  const bool wit = p.run ? p.run->witness != 0 : p.witness_host != 0;
  const uint32_t tbase = p.run ? (uint32_t)p.run->tnext : p.tbase_host;
  // an exchanged round (p.xcap) inserts two sources: the exchange blocks it
  // received (p.stg, p.dense slots: the other ranks' children this rank
  // owns) and its own share of what it staged itself (p.stg_loc, striped,
  // never sent: entries marked LV_LOCAL)
  const bool xm = p.xcap != 0;
  uint32_t lo = 0, hi = 0;  // this lane's stripe range (striped mode; exchanged rounds: the local staging)
  if (p.fused) {
    // lv_round inserted the children itself: only the round's close is left
  } else if (p.dense && !xm) {
    hi = p.dense;
  } else if (!ld_agent(&p.ctl->overflow)) {
    lo = p.ctl->lo[lane];
    hi = min(ld_agent(&p.ctl->cnt[16 * lane]), p.scs);
  }
  // iterations, block-uniform: the dense range, then the longest stripe (rows
  // of 4 slots per stripe per block iteration)
  const uint32_t n_dense = p.dense ? (p.dense + LV_BLOCK - 1) / LV_BLOCK : 0u;
  const uint32_t n_str = (p.dense && !xm) ? 0u : (wave_max_u32(hi) + LV_BLOCK / 64 - 1) / (LV_BLOCK / 64);
  const uint32_t n_it = n_dense + n_str;
  uint8_t* const loc = xm ? p.stg_loc : p.stg;  // the striped source
  for (uint32_t itb = blockIdx.x; itb < n_it; itb += gridDim.x) {
    bool win = false;
    uint32_t slot = 0, k = 0;
    LCfg<NQ>* c = nullptr;
    bool valid;
    if (itb < n_dense) {
      k = itb * LV_BLOCK + threadIdx.x;
      valid = k < p.dense;
      if (valid && xm) {  // exchange blocks: slot 0 is the header, then the block's count
        const uint32_t b = k / (p.xcap + 1), i = k - b * (p.xcap + 1);
        valid = i >= 1 && i - 1 < min(lv_xhdr<NQ>(p.stg, b, p.xcap)->count, p.xcap);
      }
      if (valid) c = lv_cfg<NQ>(p.stg, k);
    } else {
      const uint32_t i = (itb - n_dense) * (LV_BLOCK / 64) + (uint32_t)wv;
      valid = i >= lo && i < hi;
      k = (uint32_t)lane * p.scs + i;
      if (valid) {
        c = lv_cfg<NQ>(loc, k);
        // exchanged rounds: only the configurations this rank owns (lv_xsend sent the rest)
        if (xm) {
          valid = c->move == LV_HOLE || lv_owner(c->fp, p.world) == p.rank;
          k |= LV_LOCAL;
        }
      }
    }
    if (valid) {
      if (c->move != LV_HOLE) {
        const uint64_t fp = c->fp;
        const uint32_t tag = (uint32_t)(fp >> 32) & ~p.tag_drop;
        const unsigned long long mine = ((unsigned long long)tag << 32) | k;
        slot = (uint32_t)fp & p.ht_mask & ~p.tag_drop;
        for (;;) {
          const unsigned long long prev = atomicCAS(&p.ht[slot], HT_EMPTY, mine);
          if (prev == HT_EMPTY) { win = true; break; }
          if ((uint32_t)(prev >> 32) == tag) {
            const uint32_t pk = (uint32_t)prev;
            const LCfg<NQ>* o = (pk & LV_LOCAL) ? lv_cfg<NQ>(loc, pk & ~LV_LOCAL) : lv_cfg<NQ>(p.stg, pk);
            if (lv_eq<NQ>(o, c, p.K)) break;
          }
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
      // An exchanged round inserts its whole local share plus the received
      // blocks, so n can pass scap. Winners there are dropped: the close stops
      // the run (lv_xclose), and the witness cutoff (tnext + scap <= trace_cap)
      // only covers n < scap, so no index or trace entry is written for them.
      const bool kept = n < p.scap;
      if (kept) p.nxt_idx[n] = k;
      c->slot = slot;
      if (wit) {
        c->trace = kept ? p.tgid + tbase + n : TRACE_NONE;
        if (kept) p.trace[tbase + n] = TraceEnt{c->ptrace, c->move};
      }
      if (p.pmax) {  // LinearizationInfo: this configuration as the longest one holding each chain's prefix
        uint32_t size = 0;
        for (uint32_t j = 0; j < p.K; ++j) size += c->cnt[j];
        const unsigned long long v = ((unsigned long long)size << 32) | (wit ? c->trace : 0xFFFFFFFFu);
        for (uint32_t j = 0; j < p.K; ++j) atomicMax(&p.pmax[p.cs[j] + c->cnt[j]], v);
      }
    }
  }
  (void)s_hi;
  if (!p.close_round) return;
  // the last block to finish closes the round (it only reads atomics: no fence)
  __syncthreads();
  if (threadIdx.x == 0) s_last = atomicAdd(&p.ctl->done_blocks, 1u) == gridDim.x - 1;
  __syncthreads();
  if (s_last && threadIdx.x == 0) {
    if (p.xcap) lv_xclose<NQ>(p, xd);
    else lv_close_round(p);
  }
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
  LvCtl* ctl3;                // round r counts in ctl3[(r + co) % 3] (co: lv_persist)
  LvBar* bar;
  uint8_t* stg[2];            // round r stages into stg[r & 1]; its frontier is stg[(r + 1) & 1]
  uint32_t* idx[2];
  unsigned long long* ht[2];  // round r inserts into ht[r & 1]
  uint32_t max_rounds;        // rounds per launch
  uint32_t nf_max;            // leave when the frontier is wider
  uint32_t solo;              // one-configuration frontiers run as solo rounds (workgroup 0)
  uint32_t solo_maxlive;      // a solo round with more live moves goes to the grid (0: default)
  const unsigned long long* deadline;  // the run's deadline (device wall clock; nullable, 0 = none)
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

#include "solo_dev.h"

template <int NQ>
// (one workgroup per CU: the launch is one per CU anyway, and the whole
// 512-register file of a SIMD lane goes to its one wave: the grid rounds'
// pressure spills to AGPRs, not to scratch; round 4's two-per-CU bound left
// lv_persist<5> ~300 scratch accesses in its grid rounds)
__global__ __launch_bounds__(LV_BLOCK, 1) void lv_persist(LvParams p, LvPersist q) {
  // solo rounds use s_heads[0] (the configuration's heads), s_heads[1] (the
  // moves' next heads) and s_heads[2..3] as the move records (LvSoloExt)
  __shared__ __attribute__((aligned(16))) LvHeadsLds<NQ> s_heads[LV_BLOCK / 64];
  static_assert(2 * sizeof(LvHeadsLds<NQ>) >= sizeof(LvSoloExt<NQ>), "solo move records fit in s_heads[2..3]");
  static_assert(sizeof(LvHeadsLds<NQ>) >= sizeof(LvSoloHeads<NQ>), "solo heads fit in s_heads[0], s_heads[1]");
  __shared__ uint32_t s_cs[64 * NQ];
  __shared__ LvRun s_run;
  __shared__ LvSolo<(NQ <= 5 ? NQ : 1)> s_solo;  // (solo rounds only for NQ <= 5)
  for (uint32_t x = threadIdx.x; x < 64u * NQ; x += LV_BLOCK) s_cs[x] = x < p.K ? p.cs[x] : 0u;
  if (threadIdx.x == 0) s_run = *p.run;  // written by an earlier launch
  __syncthreads();
  if (s_run.done != LVR_RUNNING) return;
  const uint32_t nwaves = gridDim.x * (LV_BLOCK / 64);
  const unsigned long long dl = q.deadline ? *q.deadline : 0ull;  // (deadline_kernel wrote it earlier on the stream)
  bool ok = true;
#ifdef S2LC_PROF
  unsigned long long t_round = wall_clock64();
#endif
  uint32_t it = 0, ep = 0;  // rounds run by this launch, barrier epochs
  // grid round r counts in ctl3[(r + co) % 3]; co changes only across a solo
  // phase (the same on every workgroup: it follows from the run state)
  uint32_t co = 0;
  while (ok) {
    const uint32_t r_before = s_run.round;
    // solo rounds for NQ <= 5 (K <= 320): wider layouts would lose the second
    // resident workgroup per CU the grid barrier relies on (VGPRs)
    // (H_TAIL32 histories only: their tails are 32-bit in solo rounds)
    if (NQ <= 5 && q.solo && (p.hflags & H_TAIL32) && s_run.nf == 1 && s_run.solo_skip != s_run.round + 1) {
      if (blockIdx.x == 0) {
        if constexpr (NQ <= 5) {
          lv_solo_rounds<NQ>(p, q, s_run, *reinterpret_cast<LvSoloHeads<NQ>*>(&s_heads[0]),
                             *reinterpret_cast<LvSoloHeads<NQ>*>(&s_heads[1]),
                             *reinterpret_cast<LvSoloExt<NQ>*>(&s_heads[2]), s_cs, s_solo, max(1u, q.max_rounds - it),
                             dl);
        }
        // the next grid round's counters start at zero: the slot after
        // r_before's, never r_before's own (a workgroup that left round
        // r_before's barrier late may still be reading it: ADVICE r2); the
        // other workgroups take the run state from here after the barrier
        uint32_t* z = reinterpret_cast<uint32_t*>(q.ctl3 + (r_before + co + 1) % 3);
        for (uint32_t i = threadIdx.x; i < sizeof(LvCtl) / 4; i += LV_BLOCK) st_wt32(z + i, 0u);
        if (threadIdx.x < sizeof(LvRun) / 4)
          st_wt32(reinterpret_cast<uint32_t*>(p.run) + threadIdx.x, reinterpret_cast<const uint32_t*>(&s_run)[threadIdx.x]);
      }
      ok = lv_grid_sync(q.bar, ++ep, q.spin_ticks);
      if (ok && blockIdx.x != 0 && threadIdx.x < sizeof(LvRun) / 4)
        reinterpret_cast<uint32_t*>(&s_run)[threadIdx.x] = ld_agent(reinterpret_cast<const uint32_t*>(p.run) + threadIdx.x);
      if (!ok && threadIdx.x == 0) s_run.done = LVR_ABORT;
      __syncthreads();
      // round s_run.round + 1 counts in slot (r_before + co + 1) % 3 (zeroed above)
      co = (r_before + co + 1 + 3 * 3 - (s_run.round + 1) % 3) % 3;
#ifdef S2LC_PROF
      t_round = wall_clock64();  // (the grid rounds' timing excludes the solo phases)
#endif
      it += max(1u, s_run.round - r_before);
      if (s_run.done != LVR_RUNNING || it >= q.max_rounds || s_run.nf > q.nf_max) break;
      continue;
    }
    const uint32_t r = s_run.round + 1;  // the round this iteration expands
    LvParams rp = p;
    rp.round = r;
    rp.cur = q.stg[(r + 1) & 1]; rp.cur_idx = q.idx[(r + 1) & 1];
    rp.stg = q.stg[r & 1]; rp.nxt_idx = q.idx[r & 1];
    rp.ht = q.ht[r & 1]; rp.ht_clear = q.ht[(r + 1) & 1];
    rp.ctl = q.ctl3 + (r + co) % 3;
    rp.clear_slots = 1;
    rp.init = 0;
    if (blockIdx.x == 0) {  // the counters of round r + 1 (last read in round r - 2's close)
      uint32_t* z = reinterpret_cast<uint32_t*>(q.ctl3 + (r + 1 + co) % 3);
      for (uint32_t i = threadIdx.x; i < sizeof(LvCtl) / 4; i += LV_BLOCK) st_wt32(z + i, 0u);
    }
    LvRoundIn in;
    in.par = 0;
    in.f0 = 0;
    in.nf = s_run.nf;
    in.S = lv_slices(p.K, in.nf, nwaves, s_run.last_nf, s_run.last_closed);
    in.tbase = (uint32_t)s_run.tnext;
    in.wit = s_run.witness;
    const bool worked = lv_expand<NQ, 1>(rp, in, s_heads[threadIdx.x >> 6], s_cs);
    // the run's deadline: workgroup 0 decides before the barrier, every
    // workgroup reads the decision with the round's counters
    if (dl && blockIdx.x == 0 && threadIdx.x == 0 && wall_clock64() > dl) atomicExch(&rp.ctl->stop, 1u);
#ifdef S2LC_PROF
    if (worked && (threadIdx.x & 63) == 0 && p.prof) atomicMax(&rp.ctl->prof_end, wall_clock64());
#else
    (void)worked;
#endif
    ok = lv_grid_sync(q.bar, ++ep, q.spin_ticks);
#ifdef S2LC_PROF
    if (blockIdx.x == 0 && threadIdx.x == 0 && p.prof) {
      // [9] round time, [10] expansion critical path, [11] rounds (wall-clock ticks)
      const unsigned long long t_b = wall_clock64(), e = ld_agent64(&rp.ctl->prof_end);
      atomicAdd(&p.prof[9], t_b - t_round);
      atomicAdd(&p.prof[10], e > t_round ? e - t_round : 0ull);
      atomicAdd(&p.prof[11], 1ull);
      if (r < LV_PROF_ROUNDS) {  // per round: time, expansion critical path, frontier (wall-clock ticks)
        p.prof[48 + r] = t_b - t_round;
        p.prof[48 + LV_PROF_ROUNDS + r] = e > t_round ? e - t_round : 0ull;
        p.prof[48 + 2 * LV_PROF_ROUNDS + r] = in.nf;
      }
      t_round = t_b;
    }
#endif
    if (threadIdx.x == 0) {
      if (ok) {
        const LvCounts k = lv_read_counts(rp.ctl);
#ifdef S2LC_PROF
        if (blockIdx.x == 0 && p.prof && r < LV_PROF_ROUNDS) {  // per round: closed, children, slices
          p.prof[48 + 3 * LV_PROF_ROUNDS + r] = k.closed;
          p.prof[48 + 4 * LV_PROF_ROUNDS + r] = k.ch;
          p.prof[48 + 5 * LV_PROF_ROUNDS + r] = in.S;
        }
#endif
        lv_close_state(s_run, k, r, blockIdx.x == 0 ? p.rcounts : nullptr, p.scap, p.trace_cap);
        if (ld_agent(&rp.ctl->stop) && s_run.done == LVR_RUNNING) s_run.done = LVR_TIMEOUT;
      } else {
        s_run.done = LVR_ABORT;
      }
    }
    __syncthreads();
    ++it;
    if (s_run.done != LVR_RUNNING || it >= q.max_rounds || s_run.nf > q.nf_max) break;
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
  R->last_nf = 0; R->last_closed = 0; R->solo_rounds = 0; R->solo_skip = 0;
  R->t_last = wall_clock64(); R->narrow_ticks = 0; R->wide_ticks = 0; R->solo_ticks = 0;
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

// ---- host-free partitioned rounds (distributed.py) ---------
// Every rank sends every other rank a block of fixed capacity (xcap
// configurations) through one equal-split all-to-all, so no size travels to
// the host. Block o of a send buffer is sizeof(LCfg) * (xcap + 1) bytes: an
// LvXHdr in slot 0, then the configurations this rank staged for owner o.
// Every header carries what all ranks need to take the same decision after
// the exchange (found, the largest block, staging overflow, the staged
// total), so termination and capacity overflow are decided on the device,
// identically on every rank, and published to a host-mapped status ring the
// host reads a round or two behind while the next rounds are already queued.

// stripe walk bound of the round's staging (64 x the longest stripe), from
// the device counters (every wave computes it)
__device__ __forceinline__ uint32_t lv_stage_dense(const LvParams& p) {
  const uint32_t lane = threadIdx.x & 63;
  return 64u * wave_max_u32(min(ld_agent(&p.ctl->cnt[16 * lane]), p.scs));
}

// Block of owner / sender o in a rank's send / receive buffer: the world - 1
// other ranks in rank order (the rank's own share never travels)
__host__ __device__ __forceinline__ uint32_t lv_xblk(uint32_t o, uint32_t rank) { return o < rank ? o : o - 1; }

// the exchange headers (one wave): block o's count, the sender's largest
// block and staged total, the round's found / staging-overflow flags; clears
// the owner counters for the next round. The rank's own header goes to
// p.xself (its share stays in its local staging)
template <int NQ>
__device__ __forceinline__ void lv_xhdr_wave(const LvParams& p) {
  const uint32_t lane = threadIdx.x & 63;
  const uint32_t c = (lane < p.world && lane != p.rank) ? atomicExch(&p.own_cnt[lane], 0u) : 0u;
  const uint32_t mb = wave_max_u32(c);
  if (lane < p.world) {
    LvXHdr h;
    h.count = c; h.maxblk = mb;
    h.found = ld_agent(&p.ctl->found);
    h.fpar = ld_agent(&p.ctl->found_parent); h.fmov = ld_agent(&p.ctl->found_move);
    h.fp4 = ld_agent(&p.ctl->found_p4);
    h.sovf = ld_agent(&p.ctl->overflow);
    h.nf = p.run->nf;
    h.staged = ld_agent(&p.ctl->staged);
    *(lane == p.rank ? p.xself : lv_xhdr<NQ>(p.send, lv_xblk(lane, p.rank), p.xcap)) = h;
  }
}

// stage -> fixed-capacity blocks of the OTHER ranks: one wave per 64
// staging slots (lane = stripe) takes owner positions (one atomic per owner
// per wave), then the wave copies its configurations as one flat stream of
// 16-byte pieces, every lane's loads in flight together; the rank's own
// share stays in its staging (lv_insert reads it there). With one rank
// nothing is copied: only the own header is written. The last block to
// finish writes the headers. It reads only the owner counters (device-scope
// atomics, complete before each block's arrival) and values earlier kernels
// wrote, so the hand-off needs no fence (an agent-scope __threadfence per
// block cost ~60 us per round at 4 blocks per CU: MI355X_MICROARCH.md).
template <int NQ>
__global__ __launch_bounds__(LV_BLOCK) void lv_xsend(LvParams p) {
  if (p.run->done) return;
  __shared__ uint32_t s_last;
  __shared__ uint32_t s_to[LV_BLOCK], s_sl[LV_BLOCK];  // per wave: destination / source of its kept configurations
  constexpr uint32_t PER = sizeof(LCfg<NQ>) / 16;
  const uint32_t lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const uint32_t dense = p.world > 1 ? lv_stage_dense(p) : 0u, cap = p.xcap;
  const uint4* src = reinterpret_cast<const uint4*>(p.stg);
  uint4* dst = reinterpret_cast<uint4*>(p.send);
  for (uint32_t k0 = (blockIdx.x * (LV_BLOCK / 64) + wv) * 64; k0 < dense; k0 += gridDim.x * LV_BLOCK) {
    const uint32_t i = k0 / 64, slot = lane * p.scs + i;
    bool v = i < min(ld_agent(&p.ctl->cnt[16 * lane]), p.scs);
    uint32_t o = p.rank;
    if (v) {
      const LCfg<NQ>* c = lv_cfg<NQ>(p.stg, slot);
      v = c->move != LV_HOLE;
      if (v) o = lv_owner(c->fp, p.world);
    }
    v = v && o != p.rank;
    // positions: one atomic per owner present in the wave
    uint32_t to = 0;
    bool keep = false;
    for (uint32_t w = 0; w < p.world; ++w) {
      const uint64_t bw = __ballot(v && o == w);
      if (!bw) continue;
      uint32_t base = 0;
      if (lane == (uint32_t)(__ffsll((unsigned long long)bw) - 1)) base = atomicAdd(&p.own_cnt[w], (uint32_t)__popcll(bw));
      base = (uint32_t)__shfl((int)base, __ffsll((unsigned long long)bw) - 1, 64);
      if (v && o == w) {
        const uint32_t pos = base + (uint32_t)__popcll(bw & ((1ull << lane) - 1));
        keep = pos < cap;
        to = lv_xblk(w, p.rank) * (cap + 1) + 1 + pos;
      }
    }
    // the wave's kept configurations, as one stream of pieces: piece x of the
    // n kept ones is piece x % PER of configuration x / PER
    const uint64_t km = __ballot(keep);
    const uint32_t nk = (uint32_t)__popcll(km);
    const uint32_t my = (uint32_t)__popcll(km & ((1ull << lane) - 1));  // my rank among the kept lanes
    if (keep) { s_to[wv * 64 + my] = to; s_sl[wv * 64 + my] = slot; }
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
#pragma unroll 4
    for (uint32_t x = lane; x < nk * PER; x += 64) {
      const uint32_t e = x / PER, c = x - e * PER;
      dst[(size_t)s_to[wv * 64 + e] * PER + c] = src[(size_t)s_sl[wv * 64 + e] * PER + c];
    }
    __builtin_amdgcn_wave_barrier();
  }
  __syncthreads();  // (every wave's owner atomics have returned)
  if (threadIdx.x == 0) s_last = atomicAdd(&p.ctl->xblocks, 1u) == gridDim.x - 1;
  __syncthreads();
  if (s_last && threadIdx.x < 64) lv_xhdr_wave<NQ>(p);
}

// the decision of an exchanged round, from the received headers (every rank
// reads the same values, so every rank decides the same)
template <int NQ>
__device__ __forceinline__ LvXDecision lv_xdecide(const LvParams& p) {
  LvXDecision d;
  d.halt = 0; d.maxblk = 0; d.fpar = TRACE_NONE; d.fmov = LV_NONE; d.fp4 = 0; d.nf_global = 0; d.staged = 0;
  bool found = false, sovf = false;
  for (uint32_t s = 0; s < p.world; ++s) {  // (in rank order: every rank takes the same found child)
    uint32_t mb, nf, sv, fnd, fpar, fmov, fp4;
    unsigned long long stg;
    if (p.world == 1) {  // one rank: its header from its counters (no lv_xsend ran; nothing was sent)
      mb = 0; nf = p.run->nf; stg = ld_agent(&p.ctl->staged); sv = ld_agent(&p.ctl->overflow);
      fnd = ld_agent(&p.ctl->found); fpar = ld_agent(&p.ctl->found_parent); fmov = ld_agent(&p.ctl->found_move);
      fp4 = ld_agent(&p.ctl->found_p4);
    } else {
      const LvXHdr* h = s != p.rank ? lv_xhdr<NQ>(const_cast<uint8_t*>(p.stg), lv_xblk(s, p.rank), p.xcap) : p.xself;
      mb = h->maxblk; nf = h->nf; stg = h->staged; sv = h->sovf;
      fnd = h->found; fpar = h->fpar; fmov = h->fmov; fp4 = h->fp4;
    }
    d.maxblk = max(d.maxblk, mb);
    d.nf_global += nf;
    d.staged += stg;
    sovf |= sv != 0;
    if (fnd && !found) { found = true; d.fpar = fpar; d.fmov = fmov; d.fp4 = fp4; }
  }
  d.halt = found ? LVR_FOUND : sovf ? LVR_ABORT : d.maxblk > p.xcap ? LVR_OVERFLOW : d.staged == 0 ? LVR_EMPTY : 0u;
  return d;
}

// publish round p.round's status to the host-mapped ring (the round last)
__device__ __forceinline__ void lv_xpublish(const LvParams& p, const LvRun& R, const LvXDecision& d) {
  volatile LvXStat* x = p.xstat + (p.round % LV_XRING);
  x->done = R.done; x->nf = R.nf; x->maxblk = d.maxblk;
  x->nf_global = d.nf_global; x->staged = d.staged;
  x->found_parent = R.found_parent; x->found_move = R.found_move; x->found_p4 = R.found_p4;
  __threadfence_system();
  x->round = p.round;  // (the kernel's end makes it visible; the host reads after the round's event)
}

// a halting exchanged round (block 0 of lv_insert): the run stops, nothing inserted
template <int NQ>
__device__ __forceinline__ void lv_xhalt(const LvParams& p, const LvXDecision& d) {
  LvRun& R = *p.run;
  R.done = d.halt;
  if (d.halt == LVR_FOUND) {
    R.round = p.round;
    R.found_parent = R.witness ? d.fpar : TRACE_NONE;
    R.found_move = d.fmov;
    R.found_p4 = d.fp4;
  } else if (d.halt == LVR_EMPTY) {
    R.round = p.round;
  }
  lv_xpublish(p, R, d);
}

// the close of an exchanged round (the last lv_insert block): this rank's
// share of the next frontier
template <int NQ>
__device__ __forceinline__ void lv_xclose(const LvParams& p, const LvXDecision& d) {
  const LvCounts k = lv_read_counts(p.ctl);
  LvRun& R = *p.run;
  R.children += k.ch;
  R.last_nf = R.nf;
  R.last_closed = k.closed;
  R.nf = k.nn;
  R.round = p.round;
  R.configs += k.nn;
  R.max_frontier = max(R.max_frontier, k.nn);
  if (k.nn > p.scap) R.done = LVR_ABORT;  // (the next frontier's index list is full)
  if (R.witness) {
    R.last_tbase = (uint32_t)R.tnext;
    R.tnext += k.nn;
    if (R.tnext + p.scap > p.trace_cap) R.witness = 0;
  }
  lv_xpublish(p, R, d);
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
      const uint8_t* base = (k & LV_LOCAL) ? p.cur_loc : p.cur;
      mine = lv_owner(lv_cfg<NQ>(base, k & ~LV_LOCAL)->fp, p.world) == rank;
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
    const uint32_t k = p.cur_idx[f];
    const uint4* src = reinterpret_cast<const uint4*>(lv_cfg<NQ>((k & LV_LOCAL) ? p.cur_loc : p.cur, k & ~LV_LOCAL));
    reinterpret_cast<uint4*>(p.send + (uint64_t)f * sizeof(LCfg<NQ>))[c] = src[c];
  }
}

// clear the table slots of the frontier's configurations in both tables (a
// phase switch of the distributed search: the tables then hold no entry at
// all, since at a switch their only entries are the current frontier's,
// each at its configuration's slot; a slot another rank's configuration
// names is empty here or this rank's frontier entry, cleared either way)
template <int NQ>
__global__ __launch_bounds__(LV_BLOCK) void lv_clear_slots(LvParams p) {
  const uint32_t nf = p.f1;
  for (uint32_t i = blockIdx.x * LV_BLOCK + threadIdx.x; i < nf; i += gridDim.x * LV_BLOCK) {
    const uint32_t k = p.cur_idx[i];
    const uint32_t s = lv_cfg<NQ>((k & LV_LOCAL) ? p.cur_loc : p.cur, k & ~LV_LOCAL)->slot;
    if (s <= p.ht_mask) {
      p.ht[s] = HT_EMPTY;
      p.ht_clear[s] = HT_EMPTY;
    }
  }
}

__global__ __attribute__((unused)) void lv_iota(uint32_t* out, uint32_t n) {
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) out[i] = i;
}

}  // namespace
}  // namespace s2lc
