// search_dev.h — device side of the frontier search (included by search.hip).
// See search.hip for the algorithm overview.
#pragma once
#include "s2lincheck.h"
#include "search.h"

namespace s2lc {
namespace {

constexpr uint64_t HT_EMPTY = ~0ull;
constexpr uint32_t STAGE_BIT = 0x80000000u;
constexpr uint32_t SLOT_DEAD = 0xFFFFFFFFu;
constexpr uint32_t TRACE_CHUNK = 4096;

enum : int { CL_ALIVE = 0, CL_DEAD = 1, CL_COMPLETE = 2, CL_P4 = 3 };

#ifdef S2LC_DEBUG
#define DCHECK(cond, ...)                                                    \
  do {                                                                       \
    if (!(cond)) {                                                           \
      printf("S2LC DCHECK %s:%d: " #cond " | ", __FILE__, __LINE__);         \
      printf(__VA_ARGS__);                                                   \
      printf("\n");                                                          \
    }                                                                        \
  } while (0)
#else
#define DCHECK(cond, ...) do { } while (0)
#endif

// S2LC_GUARD: diagnostic build. Every computed index is range-checked; the
// first violation is recorded in g_guard (read back by the host) and the
// access is redirected to a safe index instead of faulting.
#ifdef S2LC_GUARD
__device__ uint32_t g_guard[8];
__device__ __forceinline__ bool guard_ok(bool cond, uint32_t line, uint32_t a, uint32_t b) {
  if (!cond && atomicAdd(&g_guard[0], 1u) == 0u) { g_guard[1] = line; g_guard[2] = a; g_guard[3] = b; }
  return cond;
}
#define GUARD(cond, a, b) guard_ok((cond), __LINE__, (uint32_t)(a), (uint32_t)(b))
#else
#define GUARD(cond, a, b) true
#endif

// S2LC_PROF: diagnostic build. Lane 0 of every workgroup stamps clock64()
// after each phase barrier and adds the per-phase cycles to g_prof (read back
// and printed by the host); closure passes / calls are counted too.
//   g_prof[0..5]: setup, expand, close, dedupe, compact, finalize (cycles)
//   g_prof[6]: closure passes  g_prof[7]: closure calls  g_prof[8]: rounds
//   g_prof[9]: record-window refills
#ifdef S2LC_PROF
__device__ unsigned long long g_prof[16];
__shared__ uint32_t s_prof_cl[3];  // per-workgroup closure passes / calls / window refills
#define PROF_DECL unsigned long long prof_t = clock64(), prof_acc[6] = {0, 0, 0, 0, 0, 0}; \
  if (tid == 0) { s_prof_cl[0] = 0; s_prof_cl[1] = 0; s_prof_cl[2] = 0; }
#define PROF_STAMP(i) do { if (tid == 0) { const unsigned long long t_ = clock64(); prof_acc[i] += t_ - prof_t; prof_t = t_; } } while (0)
#define PROF_FLUSH() do { if (tid == 0) { for (int i_ = 0; i_ < 6; ++i_) { atomicAdd(&g_prof[i_], prof_acc[i_]); prof_acc[i_] = 0; } \
  atomicAdd(&g_prof[6], (unsigned long long)s_prof_cl[0]); atomicAdd(&g_prof[7], (unsigned long long)s_prof_cl[1]); \
  atomicAdd(&g_prof[9], (unsigned long long)s_prof_cl[2]); s_prof_cl[0] = 0; s_prof_cl[1] = 0; s_prof_cl[2] = 0; } } while (0)
#define PROF_ADD(i, v) atomicAdd(&g_prof[i], (unsigned long long)(v))
#else
#define PROF_DECL do { } while (0)
#define PROF_STAMP(i) do { } while (0)
#define PROF_FLUSH() do { } while (0)
#define PROF_ADD(i, v) do { } while (0)
#endif

template <int KMAX>
struct __attribute__((aligned(16))) Cfg {
  uint64_t tail;
  uint64_t hash;
  uint32_t tok;
  uint32_t minret;  // min return event over unlinearized ops (closure output)
  uint32_t ptrace;  // trace index of the parent
  uint32_t move;    // move that produced this configuration
  uint32_t trace;   // own trace index (once in a frontier)
  uint32_t slot;    // claimed table slot, SLOT_DEAD if dropped
  uint64_t fp;      // fingerprint
  uint16_t cnt[KMAX];
};
static_assert(sizeof(Cfg<16>) == 80, "cfg16");
static_assert(sizeof(Cfg<32>) == 112, "cfg32");

struct Params {
  const OpRec* recs;
  const SRec* srecs;   // the same records in 32 bytes (H_SMALL histories; the packed kernels' SMALL instances)
  const uint64_t* pool;
  const uint32_t* chain_start;
  const HistDesc* hist;
  const uint32_t* order;
  uint32_t n_hist;
  uint32_t* counter;
  uint8_t* slab;
  size_t slab_bytes;
  uint32_t fcap, chunk, ht_mask;
  uint32_t stage_cap;  // staging entries (2 * chunk in HBM mode; may be smaller in LDS mode)
  TraceEnt* trace;
  unsigned long long* trace_head;
  uint64_t trace_cap;
  HistResult* res;
  uint32_t* moves;     // witness move lists (pack_kernel resolves its own; nullable)
  uint64_t max_configs;
  uint32_t witness;
  uint32_t n_recs, n_pool, n_res;  // buffer sizes (guard build checks)
  uint32_t win_recs;               // LDS record-window capacity (SHARED mode; 0 = none)
  uint32_t* rcounts;               // per-round unique configurations at res[h].witness_off (nullable)
  const unsigned long long* deadline;  // wall_clock64() value after which histories give Unknown (nullable)
  uint32_t gpw;                    // pack kernels: lane groups per wave that take histories (0 = all)
  unsigned long long* agg;         // pack kernels: this launch's totals (PACK_AGG_*; nullable)
  uint32_t* zero_ctr;              // (nullable) the next run's counter set (32 words) and
  unsigned long long* zero_agg;    // totals (32), zeroed by block 0: no reset dispatch before it
};

// The run's deadline in device wall-clock ticks (written once per run, read by
// the search kernels; see batch_run).
__global__ __attribute__((unused)) void deadline_kernel(unsigned long long* d, unsigned long long ticks) { *d = wall_clock64() + ticks; }

// Every history of the batch starts a run undecided (a history that no engine
// reaches in this run, e.g. after a timeout, must not keep a stale verdict).
__global__ __attribute__((unused)) void reset_results_kernel(HistResult* res, uint32_t n, uint32_t* counter,
                                                             unsigned long long* agg) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (counter && i < 64) counter[i] = 0;  // both sets: work counters, deadline, trace head
  if (agg && i < 64) agg[i] = 0;          // both sets: packed launches' totals
  if (i >= n) return;
  HistResult& r = res[i];
  r.verdict = V_UNKNOWN;
  r.reason = S2LC_R_NONE;
  r.rounds = 0;
  r.has_witness = 0;
  r.witness_len = 0;
  r.configs = 0;
  r.children = 0;
}

__device__ __forceinline__ uint64_t mix64(uint64_t x) {
  x ^= x >> 33;
  x *= 0xff51afd7ed558ccdull;
  x ^= x >> 33;
  x *= 0xc4ceb9fe1a85ec53ull;
  x ^= x >> 33;
  return x;
}

__device__ __forceinline__ OpRec load_rec(const OpRec* p) {
  // 64-byte record as four 16-byte loads
  OpRec r;
  const uint4* s = reinterpret_cast<const uint4*>(p);
  uint4* d = reinterpret_cast<uint4*>(&r);
  d[0] = s[0]; d[1] = s[1]; d[2] = s[2]; d[3] = s[3];
  return r;
}

// Closure under minimal, legal identity ops + the P1/P2/P4 rules.
//
// Latency-oriented: each pass fetches every chain head with independent loads
// (blocks of 8 chains in flight) and, in the same pass, takes each head that is
// an identity op, minimal under the previous pass's minret and legal at s.
// Using the previous pass's minret is sound: minret only grows as ops are
// linearized, so an op minimal under an older (smaller) minret is minimal now.
// A pass that changes nothing has loaded exactly the final heads, so its
// minret / bound are exact; it ends the closure once its eligibility test also
// used that exact minret. Seeded with the parent's minret (a lower bound).
//   OpRec bytes 16..31 = out_tail, out_hash; 32..47 = sufmin, call_ev, ret_ev;
//   60..63 = flags.
__device__ __forceinline__ uint4 ld16(const OpRec* r, int off) {
  return *reinterpret_cast<const uint4*>(reinterpret_cast<const uint8_t*>(r) + off);
}

// Where a chain's records are read from. In LDS mode the workgroup keeps a
// window of W records per chain (chain j's records wb[j] .. wb[j]+W-1, copied
// from HBM by all lanes when the frontier nears the window's end); a record
// outside the window is read from HBM. W = 0 disables the window.
struct RecSrc {
  const OpRec* __restrict__ recs;  // HBM, chain-major
  const uint32_t* cs;              // LDS chain starts
  const OpRec* win;                // LDS window, chain j at win[j * W]
  const uint32_t* wb;              // LDS per-chain window base (count)
  uint32_t W;
  __device__ __forceinline__ const OpRec* at(int j, uint32_t c) const {
    const uint32_t o = c - wb[j];
    return o < W ? &win[j * W + o] : &recs[cs[j] + c];
  }
};

// One pass over a block of B chains: load every head (out_tail/out_hash,
// sufmin/call/ret, flags) with independent loads, fold minret / bound, and
// mark the heads that are identity ops, minimal under minret_prev and legal.
template <int B, int KMAX_CS>
__device__ __forceinline__ uint32_t closure_block(const uint32_t* cb, int nq, int b, const RecSrc& src, const State& s,
                                                  uint32_t minret_prev, bool p2, uint32_t& minret, uint64_t& bound,
                                                  bool& dead) {
  uint4 obs[B], mid[B];
  uint32_t fl[B];
#pragma unroll
  for (int q = 0; q < B; ++q) {
    // unconditional: chains >= K read the history's last sentinel (cs[KMAX],
    // see the kernel's chain-start fill); their results are ignored
    const uint32_t* cs = src.cs;
    DCHECK(q >= nq || cs[b + q] + cb[q] < cs[b + q + 1], "closure chain %d cnt %u end %u", b + q, cb[q], cs[b + q + 1]);
    const bool ok = q < nq && GUARD(cs[b + q] + cb[q] < cs[b + q + 1], cs[b + q] + cb[q], cs[b + q + 1]);
    const OpRec* r = ok ? src.at(b + q, cb[q]) : &src.recs[cs[KMAX_CS]];
    obs[q] = ld16(r, 16);
    mid[q] = ld16(r, 32);
    fl[q] = r->flags;
  }
  uint32_t adv = 0;
#pragma unroll
  for (int q = 0; q < B; ++q) {
    if (q >= nq) continue;
    minret = min(minret, mid[q].w);
    bound = min(bound, (uint64_t)mid[q].x | ((uint64_t)mid[q].y << 32));
    const uint32_t f = fl[q];
    if (!(f & OPF_CLS_E) || mid[q].z >= minret_prev) continue;
    const uint64_t ot = (uint64_t)obs[q].x | ((uint64_t)obs[q].y << 32);
    const uint64_t oh = (uint64_t)obs[q].z | ((uint64_t)obs[q].w << 32);
    bool legal = true;
    if ((f & OPF_KIND_MASK) != 0) {
      if ((f & OPF_HAS_HASH) && s.hash != oh) legal = false;
      if (!(f & OPF_FAIL) && s.tail != ot) legal = false;
    }
    if (legal) adv |= 1u << q;
    // P2: a minimal successful read at this tail with another hash can never pass
    else if (p2 && (f & OPF_KIND_MASK) != 0 && !(f & OPF_FAIL) && (f & OPF_HAS_HASH) && ot == s.tail)
      dead = true;
  }
  return adv;
}

template <int KMAX>
__device__ __forceinline__ int closure(Cfg<KMAX>* c, int K, const RecSrc& src, uint32_t hflags, uint32_t minret_seed) {
  constexpr int B = 8;
  constexpr bool REG = KMAX <= 32;  // counts held in registers (packed u16 pairs)
  constexpr int NP = REG ? KMAX / 2 : 1;
  const State s{c->tail, c->hash, c->tok};
  const bool nowrap = hflags & H_NOWRAP;
  const bool p2 = hflags & H_P2OK;
  const bool p4 = hflags & H_P4;
  uint32_t pk[NP];
  if constexpr (REG) {
    const uint4* w = reinterpret_cast<const uint4*>(c->cnt);
#pragma unroll
    for (int q = 0; q < KMAX / 8; ++q) {
      const uint4 v = w[q];
      pk[4 * q] = v.x; pk[4 * q + 1] = v.y; pk[4 * q + 2] = v.z; pk[4 * q + 3] = v.w;
    }
  }
  uint32_t minret_prev = minret_seed;
  uint32_t minret = EV_INF;
  uint64_t bound = REQ_NONE;
  int result = CL_ALIVE;
#ifdef S2LC_PROF
  uint32_t passes = 0;
#endif
  for (;;) {
#ifdef S2LC_PROF
    ++passes;
#endif
    minret = EV_INF;
    bound = REQ_NONE;
    bool changed = false, dead = false;
    if constexpr (REG) {
#pragma unroll
      for (int b = 0; b < KMAX; b += B) {
        if (b >= K) break;
        uint32_t cb[B];
#pragma unroll
        for (int q = 0; q < B; ++q) cb[q] = ((b + q) & 1) ? (pk[(b + q) >> 1] >> 16) : (pk[(b + q) >> 1] & 0xFFFFu);
        const uint32_t adv = closure_block<B, KMAX>(cb, min(B, K - b), b, src, s, minret_prev, p2, minret, bound, dead);
        if (adv) {
          changed = true;
#pragma unroll
          for (int q = 0; q < B; ++q)
            if (adv & (1u << q)) pk[(b + q) >> 1] += ((b + q) & 1) ? 0x10000u : 1u;
        }
      }
    } else {
      for (int b = 0; b < K; b += B) {
        const uint4 v = *reinterpret_cast<const uint4*>(&c->cnt[b]);
        uint32_t cb[B] = {v.x & 0xFFFFu, v.x >> 16, v.y & 0xFFFFu, v.y >> 16,
                          v.z & 0xFFFFu, v.z >> 16, v.w & 0xFFFFu, v.w >> 16};
        const uint32_t adv = closure_block<B, KMAX>(cb, min(B, K - b), b, src, s, minret_prev, p2, minret, bound, dead);
        if (adv) {
          changed = true;
          uint4 o;
          o.x = (cb[0] + ((adv >> 0) & 1)) | ((cb[1] + ((adv >> 1) & 1)) << 16);
          o.y = (cb[2] + ((adv >> 2) & 1)) | ((cb[3] + ((adv >> 3) & 1)) << 16);
          o.z = (cb[4] + ((adv >> 4) & 1)) | ((cb[5] + ((adv >> 5) & 1)) << 16);
          o.w = (cb[6] + ((adv >> 6) & 1)) | ((cb[7] + ((adv >> 7) & 1)) << 16);
          *reinterpret_cast<uint4*>(&c->cnt[b]) = o;
        }
      }
    }
    if (dead) { result = CL_DEAD; break; }
    if (nowrap && s.tail > bound) { result = CL_DEAD; break; }  // P1: a pending observer needs a smaller tail
    // Final only if nothing changed AND eligibility was judged with the exact minret.
    if (!changed && minret == minret_prev) {
      if (minret == EV_INF) result = CL_COMPLETE;
      else if (p4 && bound == REQ_NONE) result = CL_P4;     // P4: nothing left constrains the state
      break;
    }
    minret_prev = minret;
  }
  if constexpr (REG) {
    uint4* w = reinterpret_cast<uint4*>(c->cnt);
#pragma unroll
    for (int q = 0; q < KMAX / 8; ++q) w[q] = make_uint4(pk[4 * q], pk[4 * q + 1], pk[4 * q + 2], pk[4 * q + 3]);
  }
  c->minret = minret;
#ifdef S2LC_PROF
  atomicAdd(&s_prof_cl[0], passes);
  atomicAdd(&s_prof_cl[1], 1u);
#endif
  return result;
}

template <int KMAX>
__device__ __forceinline__ uint64_t fingerprint(const Cfg<KMAX>* c, int nw) {
  uint64_t h = mix64(c->tail ^ 0x9E3779B97F4A7C15ull) ^ mix64(c->hash + 0x632BE59BD9B4E019ull * (c->tok + 1));
  const uint4* w = reinterpret_cast<const uint4*>(c->cnt);
  for (int q = 0; q < nw; ++q) {
    const uint4 v = w[q];
    h = mix64(h ^ ((uint64_t)v.x | ((uint64_t)v.y << 32)));
    h = mix64(h + ((uint64_t)v.z | ((uint64_t)v.w << 32)));
  }
  return h;
}

template <int KMAX>
__device__ __forceinline__ bool cfg_eq(const Cfg<KMAX>* a, const Cfg<KMAX>* b, int nw) {
  if (a->tail != b->tail || a->hash != b->hash || a->tok != b->tok) return false;
  const uint4* x = reinterpret_cast<const uint4*>(a->cnt);
  const uint4* y = reinterpret_cast<const uint4*>(b->cnt);
  for (int q = 0; q < nw; ++q) {
    const uint4 u = x[q], v = y[q];
    if (u.x != v.x || u.y != v.y || u.z != v.z || u.w != v.w) return false;
  }
  return true;
}

template <int KMAX>
__device__ __forceinline__ void cfg_copy(Cfg<KMAX>* d, const Cfg<KMAX>* s) {
  const uint4* x = reinterpret_cast<const uint4*>(s);
  uint4* y = reinterpret_cast<uint4*>(d);
#pragma unroll
  for (int q = 0; q < (int)(sizeof(Cfg<KMAX>) / 16); ++q) y[q] = x[q];
}

// Per-workgroup scalars, at the start of dynamic LDS (one 16-byte-aligned
// object, so the configuration arrays that follow stay 16-byte aligned).
template <int KMAX>
struct __attribute__((aligned(16))) WgState {
  uint32_t cs[KMAX + 1];  // chain starts; entries > K point at a sentinel
  uint32_t wb[KMAX];      // record-window base (count) per chain
  uint32_t h, nstage, nnext, found, overflow, children;
  uint32_t found_parent, found_move, found_p4;
  uint32_t tb, tleft, witness_ok, timed_out;
  unsigned long long tbase;
  HistDesc hd;
};

// Dynamic LDS declaration (overridable only by the test-only CPU emulator).
#ifndef S2LC_DYNAMIC_LDS
#define S2LC_DYNAMIC_LDS(name) extern __shared__ __attribute__((aligned(16))) uint8_t name[]
#endif

template <int KMAX>
constexpr size_t wg_state_bytes() { return (sizeof(WgState<KMAX>) + 15) & ~(size_t)15; }

// 16-byte global -> LDS copy without a register round trip (overridable only by
// the test-only CPU emulator).
#ifndef S2LC_GLDS16
#define S2LC_GLDS16(gsrc, lds_base) \
  __builtin_amdgcn_global_load_lds((gsrc), (__attribute__((address_space(3))) void*)(lds_base), 16, 0, 0)
#define S2LC_WAIT_ALL() __builtin_amdgcn_s_waitcnt(0)
#endif

// Record-window refill (LDS mode). Chain j's window
// must start at or below every frontier configuration's count on j (counts only
// grow, so every later configuration stays at or above it); it is re-based to
// the frontier minimum when some configuration has come within a quarter
// window of its end. All lanes copy, at most WIN_ITEMS 16-byte pieces each, by
// LDS-DMA: every piece is in flight at once, so a refill costs one HBM latency.
constexpr int WIN_ITEMS = 8;
template <int KMAX, int BT>
__device__ __noinline__ void window_refill(WgState<KMAX>& S, OpRec* win, const OpRec* __restrict__ recs,
                                              const Cfg<KMAX>* cur, uint32_t ncur, int K, uint32_t W, bool init) {
  const int tid = threadIdx.x;
  bool flag = false;
  uint32_t lo = 0;
  if (tid < K) {
    if (init) {
      flag = true;
    } else {
      lo = 0xFFFFu;
      uint32_t hi = 0;
#pragma unroll 1
      for (uint32_t i = 0; i < ncur; ++i) {
        const uint32_t c = cur[i].cnt[tid];
        lo = min(lo, c);
        hi = max(hi, c);
      }
      flag = hi + (W >> 2) >= S.wb[tid] + W;
    }
  }
  if (!__syncthreads_or(flag)) return;
#ifdef S2LC_PROF
  if (tid == 0) ++s_prof_cl[2];
#endif
  if (tid < K) S.wb[tid] = lo;
  __syncthreads();
  // LDS-DMA: lane l of a wave-instruction writes window bytes base + 16*l, so
  // piece `it` lands at win + 16*it; the global source address is per lane.
  const uint32_t per = W * 4, n = (uint32_t)K * per;
  const uint4* __restrict__ src = reinterpret_cast<const uint4*>(recs);
  uint4* w4 = reinterpret_cast<uint4*>(win);
  // not unrolled: an LDS-DMA has no destination register, so iterations never wait
#pragma unroll 1
  for (int k = 0; k < WIN_ITEMS; ++k) {
    const uint32_t base = k * BT;
    if (base >= n) break;
    const uint32_t it = base + tid;
    if (it < n) {
      const uint32_t j = it / per;
      const uint32_t o = it - j * per;  // 16-byte piece within the chain's window
      const uint32_t g = S.cs[j] + S.wb[j] + (o >> 2);
      if (g < S.cs[j + 1]) S2LC_GLDS16(&src[4 * (size_t)g + (o & 3)], w4 + base);
    }
  }
  S2LC_WAIT_ALL();
  __syncthreads();
}

// SHARED = true: frontier A/B, staging and the dedupe table live in LDS right
// after WgState (sized by the host: fcap / stage_cap / ht_mask); a history that
// outgrows them is flagged S2LC_R_FRONTIER and re-run in HBM mode.
// SHARED = false: the same arrays live in a per-workgroup HBM slab.
template <int KMAX, int BT, bool SHARED>
__global__ __launch_bounds__(BT) void search_kernel(Params p) {
  using C = Cfg<KMAX>;
  S2LC_DYNAMIC_LDS(smem);
  WgState<KMAX>& S = *reinterpret_cast<WgState<KMAX>*>(smem);

  const int tid = threadIdx.x;
  uint8_t* slab = SHARED ? smem + wg_state_bytes<KMAX>() : p.slab + (size_t)blockIdx.x * p.slab_bytes;
  C* const fa = reinterpret_cast<C*>(slab);
  C* const fb = fa + p.fcap;
  C* const stage = fb + p.fcap;
  unsigned long long* const ht = reinterpret_cast<unsigned long long*>(stage + p.stage_cap);
  const uint32_t mask = p.ht_mask;
  OpRec* const win = SHARED ? reinterpret_cast<OpRec*>(ht + mask + 1) : nullptr;

  for (uint32_t i = tid; i <= mask; i += BT) ht[i] = HT_EMPTY;
  if (tid == 0) { S.tleft = 0; S.tbase = 0; }
  __syncthreads();
  PROF_DECL;

  for (;;) {
    if (tid == 0) S.h = atomicAdd(p.counter, 1u);
    __syncthreads();
    const uint32_t hi = S.h;
    if (hi >= p.n_hist) break;
    uint32_t h = p.order[hi];
    if (!GUARD(h < p.n_res, h, hi)) h = 0;
    if (tid == 0) S.hd = p.hist[h];
    __syncthreads();
    const HistDesc hd = S.hd;
    const int K = hd.K;
    if (K > KMAX) {  // the host sizes KMAX to the batch; never taken
      if (tid == 0) { p.res[h].verdict = V_UNKNOWN; p.res[h].reason = S2LC_R_FRONTIER; }
      __syncthreads();
      continue;
    }
    const bool idefer = hd.flags & H_IDEFER;
    const unsigned long long deadline = p.deadline ? *p.deadline : 0ull;
    uint32_t* const rc = p.rcounts ? p.rcounts + p.res[h].witness_off : nullptr;
    const int nw = (K + 7) >> 3;
    const OpRec* __restrict__ recs = p.recs;
    // cs[0..K] are the chain starts (cs[K] = end); cs[K+1..KMAX] hold the index
    // of the history's last sentinel, which closure loads for unused chain
    // slots so that every head load is in bounds and unconditional.
    for (int j = tid; j <= KMAX; j += BT) {
      const uint32_t end = p.chain_start[hd.cs_base + K];
      S.cs[j] = j <= K ? p.chain_start[hd.cs_base + j] : (end > 0 ? end - 1 : 0);
      if (j < KMAX) S.wb[j] = 0;
    }
    // record window: W records per chain (0 in HBM mode or when K is too large)
    const uint32_t W = SHARED ? min(p.win_recs / (uint32_t)K, (uint32_t)(WIN_ITEMS * BT / 4) / (uint32_t)K) : 0u;
    const RecSrc src{recs, S.cs, win, S.wb, W};
    if (tid == 0) {
      S.found = 0; S.overflow = 0; S.children = 0;
      S.witness_ok = p.witness;
      S.found_parent = TRACE_NONE; S.found_move = TRACE_NONE; S.found_p4 = 0;
    }
    __syncthreads();
    PROF_STAMP(0);

    // Round 0 stages the initial configuration (∅, (0, 0, nil)) as its only
    // "child"; every later round stages the children of the frontier. Each
    // round then runs: close (one lane per staged child) -> dedupe -> compact.
    C* cur = fa;
    C* nxt = fb;
    uint32_t ncur = 0;
    uint64_t configs = 0;
    uint32_t rounds = 0;
    uint32_t verdict = V_ILLEGAL, reason = S2LC_R_SEARCH_EXHAUSTED;
    uint32_t deep_trace = TRACE_NONE, deep_len = 0;
    for (bool init = true;; init = false) {
      if (!init && ncur == 0) {
        verdict = V_ILLEGAL; reason = S2LC_R_SEARCH_EXHAUSTED;
        // nxt holds the previous (deepest non-empty) frontier after the swap
        deep_trace = rounds > 0 ? nxt[0].trace : TRACE_NONE;
        deep_len = rounds > 0 ? rounds - 1 : 0;
        break;
      }
      if (deadline) {  // one lane reads the clock: waves of a workgroup may see different values
        if (tid == 0) S.timed_out = wall_clock64() > deadline ? 1u : 0u;
        __syncthreads();
        if (S.timed_out) { verdict = V_UNKNOWN; reason = S2LC_R_TIMEOUT; break; }
      }
      if (tid == 0) S.nnext = 0;
      if (SHARED && W) window_refill<KMAX, BT>(S, win, recs, cur, ncur, K, W, init);
      const uint32_t total = init ? 1u : ncur * (uint32_t)K;
      for (uint32_t base = 0; base < total; base += p.chunk) {
        if (tid == 0) S.nstage = 0;
        __syncthreads();
        PROF_STAMP(5);
        // ---- expand: one lane per (configuration, chain); raw children ---
        if (init) {
          if (tid == 0) {
            C* c = &stage[0];
#pragma unroll
            for (int w = 0; w < KMAX / 8; ++w) reinterpret_cast<uint4*>(c->cnt)[w] = make_uint4(0, 0, 0, 0);
            c->tail = 0; c->hash = 0; c->tok = 0;
            c->minret = 0;  // closure seed: a lower bound of the true minret
            c->ptrace = TRACE_NONE; c->move = TRACE_NONE;
            S.nstage = 1;
          }
        } else {
          const uint32_t lim = min(total, base + p.chunk);
          for (uint32_t it = base + tid; it < lim; it += BT) {
            const uint32_t i = it / (uint32_t)K;
            const uint32_t j = it - i * (uint32_t)K;
            const C* pc = &cur[i];
            const uint32_t cj = (reinterpret_cast<const uint32_t*>(pc->cnt)[j >> 1] >> (16 * (j & 1))) & 0xFFFFu;
            DCHECK(i < ncur && S.cs[j] + cj < S.cs[j + 1], "expand i %u ncur %u j %u cnt %u", i, ncur, j, cj);
            if (!GUARD(i < ncur && S.cs[j] + cj < S.cs[j + 1] && S.cs[j + 1] <= p.n_recs, i * 65536u + j, cj)) continue;
            const OpRec r = load_rec(src.at(j, cj));
            if ((r.flags & (OPF_SENTINEL | OPF_CLS_E)) || r.call_ev >= pc->minret) continue;
            const State s{pc->tail, pc->hash, pc->tok};
            const bool g = append_guards_ok(r, s);
            State opt{0, 0, 0};
            if (!GUARD((uint64_t)r.hash_off + r.hash_cnt <= p.n_pool, r.hash_off, r.hash_cnt)) continue;
            if (g) {
              opt.tail = s.tail + r.num_records;
              opt.hash = fold_hashes_blk(s.hash, p.pool + r.hash_off, r.hash_cnt);
              opt.tok = r.set_tok ? r.set_tok : s.tok;
            }
            // children as two named slots (a runtime-indexed array would go to scratch)
            bool take_opt, take_id;
            if (r.flags & OPF_CLS_D) {
              take_opt = g && opt.tail == r.out_tail;
              take_id = false;
            } else {  // indefinite: opt any time; identity only when it holds the minimal return
              take_opt = g;
              take_id = (!idefer || r.ret_ev == pc->minret) && !(g && state_eq(opt, s));
            }
            const int nk = (int)take_opt + (int)take_id;
            if (nk) atomicAdd(&S.children, (uint32_t)nk);
#pragma unroll
            for (int q = 0; q < 2; ++q) {
              if (q >= nk) break;
              const bool is_opt = (q == 0) && take_opt;
              const State kid = is_opt ? opt : s;
              const uint32_t k = atomicAdd(&S.nstage, 1u);
              if (k >= p.stage_cap) { S.overflow = 1; break; }  // staging full: re-run in a bigger pass
              C* ch = &stage[k];
              // child counts = parent counts with chain j advanced, built in
              // registers and written with the same 16-byte type used to read them
              const uint4* src = reinterpret_cast<const uint4*>(pc->cnt);
              uint4* dst = reinterpret_cast<uint4*>(ch->cnt);
#pragma unroll
              for (int w = 0; w < KMAX / 8; ++w) {
                uint4 v = src[w];
                if ((int)(j >> 3) == w) {
                  const uint32_t inc = (j & 1) ? 0x10000u : 1u;
                  switch ((j >> 1) & 3) {
                    case 0: v.x += inc; break;
                    case 1: v.y += inc; break;
                    case 2: v.z += inc; break;
                    default: v.w += inc; break;
                  }
                }
                dst[w] = v;
              }
              ch->tail = kid.tail; ch->hash = kid.hash; ch->tok = kid.tok;
              ch->minret = pc->minret;  // closure seed
              ch->ptrace = pc->trace;
              ch->move = is_opt ? j : (j | MOVE_IDENT);
            }
          }
        }
        __syncthreads();
        PROF_STAMP(1);
        const uint32_t ns = min(S.nstage, p.stage_cap);
        // ---- close: one lane per staged child ------------------------------
        for (uint32_t k = tid; k < ns; k += BT) {
          C* ch = &stage[k];
          const int cr = closure<KMAX>(ch, K, src, hd.flags, ch->minret);
          if (cr == CL_ALIVE) {
            ch->fp = fingerprint<KMAX>(ch, nw);
            ch->slot = 0;
          } else {
            ch->slot = SLOT_DEAD;
            if (cr >= CL_COMPLETE && atomicCAS(&S.found, 0u, 1u) == 0u) {
              S.found_parent = ch->ptrace; S.found_move = ch->move; S.found_p4 = (cr == CL_P4);
            }
          }
        }
        __syncthreads();
        PROF_STAMP(2);
        // ---- dedupe: 64-bit CAS open addressing, full-key compare on tag hit
        for (uint32_t k = tid; k < ns; k += BT) {
          C* ch = &stage[k];
          if (ch->slot == SLOT_DEAD) continue;
          const uint64_t fp = ch->fp;
          const uint32_t tag = (uint32_t)(fp >> 32);
          const unsigned long long mine = ((unsigned long long)tag << 32) | (k | STAGE_BIT);
          uint32_t slot = (uint32_t)fp & mask;
          for (;;) {
            const unsigned long long prev = atomicCAS(&ht[slot], HT_EMPTY, mine);
            if (prev == HT_EMPTY) { ch->slot = slot; break; }
            if ((uint32_t)(prev >> 32) == tag) {
              const uint32_t ref = (uint32_t)prev;
              DCHECK((ref & STAGE_BIT) ? (ref & ~STAGE_BIT) < p.stage_cap : ref < p.fcap, "ht ref %x slot %u", ref, slot);
              if (GUARD((ref & STAGE_BIT) ? (ref & ~STAGE_BIT) < p.stage_cap : ref < p.fcap, ref, slot)) {
                const C* o = (ref & STAGE_BIT) ? &stage[ref & ~STAGE_BIT] : &nxt[ref];
                if (cfg_eq<KMAX>(o, ch, nw)) { ch->slot = SLOT_DEAD; break; }
              }
            }
            slot = (slot + 1) & mask;
          }
        }
        __syncthreads();
        PROF_STAMP(3);
        // ---- compact survivors into the next frontier ---------------------
        for (uint32_t k = tid; k < ns; k += BT) {
          C* ch = &stage[k];
          if (ch->slot == SLOT_DEAD) continue;
          const uint32_t n = atomicAdd(&S.nnext, 1u);
          if (n < p.fcap) {
            cfg_copy<KMAX>(&nxt[n], ch);
            if (GUARD(ch->slot <= mask, ch->slot, n))
              ht[ch->slot] = ((unsigned long long)(uint32_t)(ch->fp >> 32) << 32) | n;
          } else {
            S.overflow = 1;
          }
        }
        __syncthreads();
        PROF_STAMP(4);
        if (S.found || S.overflow) break;
      }
      if (S.overflow) {
        for (uint32_t i = tid; i <= mask; i += BT) ht[i] = HT_EMPTY;
        if (S.found) { verdict = V_OK; reason = 0; rounds += init ? 0u : 1u; }
        else { verdict = V_UNKNOWN; reason = S2LC_R_FRONTIER; }
        __syncthreads();
        PROF_STAMP(5);
        break;
      }
      const uint32_t nn = min(S.nnext, p.fcap);
      if (tid == 0) {
        S.tb = TRACE_NONE;
        if (S.witness_ok) {
          if (S.tleft < nn) {
            const unsigned long long want = max((unsigned long long)nn, (unsigned long long)TRACE_CHUNK);
            const unsigned long long b = atomicAdd(p.trace_head, want);
            if (b + want <= p.trace_cap) { S.tbase = b; S.tleft = (uint32_t)want; }
            else S.witness_ok = 0;
          }
          if (S.witness_ok) { S.tb = (uint32_t)S.tbase; S.tbase += nn; S.tleft -= nn; }
        }
      }
      __syncthreads();
      PROF_STAMP(5);
      const uint32_t tb = S.tb;
      for (uint32_t n = tid; n < nn; n += BT) {
        C* c = &nxt[n];
        DCHECK(c->slot <= mask && (tb == TRACE_NONE || tb + n < p.trace_cap), "clear slot %u tb %u n %u", c->slot, tb, n);
        if (GUARD(c->slot <= mask, c->slot, n)) ht[c->slot] = HT_EMPTY;
        if (tb != TRACE_NONE && GUARD((uint64_t)tb + n < p.trace_cap, tb, n)) {
          c->trace = tb + n;
          p.trace[tb + n].parent = c->ptrace;
          p.trace[tb + n].move = c->move;
        } else {
          c->trace = TRACE_NONE;
        }
      }
      __syncthreads();
      PROF_STAMP(5);
      configs += nn;
      rounds += init ? 0u : 1u;
      if (rc && tid == 0) rc[rounds] = nn;
      if (S.found) { verdict = V_OK; reason = 0; break; }
      if (p.max_configs && configs > p.max_configs) { verdict = V_UNKNOWN; reason = S2LC_R_BUDGET; break; }
      C* t = cur; cur = nxt; nxt = t;
      ncur = nn;
    }
    if (tid == 0) {
      HistResult& R = p.res[h];
      R.verdict = verdict;
      R.reason = reason;
      R.rounds = rounds;
      R.configs = configs;
      R.children = S.children;
      R.p4 = S.found_p4;
      R.final_parent = (verdict == V_OK && S.witness_ok) ? S.found_parent : TRACE_NONE;
      R.final_move = S.found_move;
      R.witness_len = 0;
      R.deep_trace = (verdict == V_ILLEGAL && S.witness_ok) ? deep_trace : TRACE_NONE;
      R.deep_len = deep_len;
      R.has_witness = ((verdict == V_OK || R.deep_trace != TRACE_NONE) && S.witness_ok) ? 2u : 0u;  // resolved by walk_kernel
      PROF_ADD(8, rounds);
    }
    __syncthreads();
    PROF_STAMP(5);
    PROF_FLUSH();
  }
}

// Witness extraction: one lane per history walks the parent chain backwards
// and writes the move list in order. Ok: the completing move after the path
// to its parent. Illegal: the path to a configuration of the deepest
// non-empty round (the partial linearization the visualization shows).
// One WAVE per history (launch: 4 waves per 256-thread block): lane i reads
// the entry i steps below the current one, and a ballot finds how far the
// chain runs through consecutive entries (a parent is usually the entry just
// before its child: the level search's one-configuration rounds append one
// entry per round), so those moves are written in one step instead of one
// dependent load each.
__global__ __attribute__((unused)) void walk_kernel(uint32_t n, HistResult* res, const TraceEnt* trace, uint32_t* moves) {
  const uint32_t h = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
  const uint32_t lane = threadIdx.x & 63;
  if (h >= n) return;
  const HistResult r = res[h];
  if (r.has_witness != 2u) return;
  uint32_t* out = moves + r.witness_off;
  uint32_t len, pos, idx;
  if (r.verdict == V_OK) {
    len = (r.final_move == TRACE_NONE) ? 0u : r.rounds;
    if (len && lane == 0) out[len - 1] = r.final_move;
    pos = len ? len - 1 : 0;
    idx = r.final_parent;
  } else {
    len = r.deep_len;
    pos = len;
    idx = r.deep_trace;
  }
  while (pos > 0 && idx != TRACE_NONE) {
    const uint32_t my = idx - lane;
    const bool valid = lane <= idx && lane < pos;
    TraceEnt e{TRACE_NONE, TRACE_NONE};
    if (valid) e = trace[my];
    // lane i's entry ends the consecutive run when its parent is elsewhere
    const bool brk = !valid || e.parent == TRACE_NONE || e.parent != my - 1;
    const unsigned long long bm = __ballot(brk);
    // the run ends at the first breaking lane (all 64 lanes consecutive: lane 63)
    const uint32_t last = bm ? (uint32_t)__ffsll(bm) - 1 : 63u;
    const bool last_valid = __shfl((int)valid, (int)last, 64) != 0;
    const uint32_t cnt = last_valid ? last + 1 : last;
    if (lane < cnt) out[pos - 1 - lane] = e.move;
    const uint32_t nidx = (uint32_t)__shfl((int)e.parent, (int)last, 64);
    pos -= cnt;
    idx = last_valid ? nidx : TRACE_NONE;
  }
  if (lane == 0) {
    const bool ok = pos == 0;
    res[h].witness_len = ok ? len : 0u;
    res[h].has_witness = ok ? 1u : 0u;
  }
}

}  // namespace
}  // namespace s2lc
