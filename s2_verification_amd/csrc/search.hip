// search.hip — frontier-parallel linearizability search for the S2 model on
// gfx950 (MI355X). Replaces porcupine v1.0.3 checkSingle (WGL backtracking DFS
// with a (bitset, state) cache, called at golang/s2-porcupine/main.go:606).
//
// Search space: configurations (L, s) with L a down-set of the real-time
// order, encoded as K per-chain prefix counters (greedy interval colouring,
// history.cpp), and s a single S2 state (the powerset state is exploded).
// One ROUND linearizes exactly one non-identity op (durable or indefinite
// append) per configuration, then closes the child under the identity ops
// (reads, check-tails, definite failures) that are minimal and legal — a
// verdict-exact reduction. Configurations are deduplicated per
// round in an open-addressing table with 64-bit atomicCAS; survivors are
// compacted into the next frontier.
//
// Work mapping: one workgroup owns one history at a time (persistent grid,
// atomic work counter, longest-first order); inside a round, one lane per
// (configuration, chain) candidate. Frontier, staging and table live in a
// per-workgroup HBM slab (L2-resident at these sizes); chain offsets in LDS.
#include <hip/hip_runtime.h>
#include <string.h>

#include <algorithm>
#include <chrono>
#include <numeric>
#include <string>

#include "s2lincheck.h"
#include "search.h"

namespace s2lc {

namespace {

constexpr uint64_t HT_EMPTY = ~0ull;
constexpr uint32_t STAGE_BIT = 0x80000000u;
constexpr uint32_t SLOT_DEAD = 0xFFFFFFFFu;
constexpr uint32_t TRACE_CHUNK = 4096;

enum : int { CL_ALIVE = 0, CL_DEAD = 1, CL_COMPLETE = 2, CL_P4 = 3 };

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
  const uint64_t* pool;
  const uint32_t* chain_start;
  const HistDesc* hist;
  const uint32_t* order;
  uint32_t n_hist;
  uint32_t* counter;
  uint8_t* slab;
  size_t slab_bytes;
  uint32_t fcap, chunk, ht_mask;
  TraceEnt* trace;
  unsigned long long* trace_head;
  uint64_t trace_cap;
  HistResult* res;
  uint64_t max_configs;
  uint32_t witness;
};

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
template <int KMAX>
__device__ int closure(Cfg<KMAX>* c, int K, const uint32_t* cs, const OpRec* __restrict__ recs, uint32_t hflags) {
  const State s{c->tail, c->hash, c->tok};
  const bool nowrap = hflags & H_NOWRAP;
  const bool p2 = hflags & H_P2OK;
  for (;;) {
    uint32_t minret = EV_INF;
    uint64_t bound = REQ_NONE;
    for (int q = 0; q < K; ++q) {
      const OpRec* r = &recs[cs[q] + c->cnt[q]];
      minret = min(minret, r->ret_ev);
      bound = min(bound, r->sufmin);
    }
    if (minret == EV_INF) return CL_COMPLETE;
    if (nowrap && s.tail > bound) return CL_DEAD;  // P1: a pending observer needs a smaller tail
    if (bound == REQ_NONE) return CL_P4;          // P4: nothing left constrains the state
    bool changed = false;
    for (int q = 0; q < K; ++q) {
      uint32_t cq = c->cnt[q];
      const uint32_t c0 = cq;
      for (;;) {
        const OpRec r = load_rec(&recs[cs[q] + cq]);
        if (!(r.flags & OPF_CLS_E) || r.call_ev >= minret) break;
        if (!ident_legal(r, s)) {
          // P2: a minimal successful read at this tail with another hash can never pass
          if (p2 && (r.flags & OPF_KIND_MASK) != 0 && !(r.flags & OPF_FAIL) && (r.flags & OPF_HAS_HASH) &&
              r.out_tail == s.tail)
            return CL_DEAD;
          break;
        }
        ++cq;
      }
      if (cq != c0) { c->cnt[q] = (uint16_t)cq; changed = true; }
    }
    if (!changed) { c->minret = minret; return CL_ALIVE; }
  }
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

template <int KMAX, int BT>
__global__ __launch_bounds__(BT) void search_kernel(Params p) {
  using C = Cfg<KMAX>;
  __shared__ uint32_t s_cs[KMAX + 1];
  __shared__ uint32_t s_h, s_nstage, s_nnext, s_found, s_overflow, s_children;
  __shared__ uint32_t s_found_parent, s_found_move, s_found_p4;
  __shared__ uint32_t s_tb, s_tleft, s_witness_ok;
  __shared__ unsigned long long s_tbase;
  __shared__ HistDesc s_hd;

  const int tid = threadIdx.x;
  uint8_t* slab = p.slab + (size_t)blockIdx.x * p.slab_bytes;
  C* const fa = reinterpret_cast<C*>(slab);
  C* const fb = fa + p.fcap;
  C* const stage = fb + p.fcap;
  unsigned long long* const ht = reinterpret_cast<unsigned long long*>(stage + 2 * p.chunk);
  const uint32_t mask = p.ht_mask;

  for (uint32_t i = tid; i <= mask; i += BT) ht[i] = HT_EMPTY;
  if (tid == 0) { s_tleft = 0; s_tbase = 0; }
  __syncthreads();

  for (;;) {
    if (tid == 0) s_h = atomicAdd(p.counter, 1u);
    __syncthreads();
    const uint32_t hi = s_h;
    if (hi >= p.n_hist) break;
    const uint32_t h = p.order[hi];
    if (tid == 0) s_hd = p.hist[h];
    __syncthreads();
    const HistDesc hd = s_hd;
    const int K = hd.K;
    const int nw = (K + 7) >> 3;
    const OpRec* __restrict__ recs = p.recs;
    for (int j = tid; j <= K; j += BT) s_cs[j] = p.chain_start[hd.cs_base + j];
    if (tid == 0) {
      s_found = 0; s_overflow = 0; s_children = 0;
      s_witness_ok = p.witness;
      s_found_parent = TRACE_NONE; s_found_move = TRACE_NONE; s_found_p4 = 0;
    }
    __syncthreads();

    // ---- initial configuration: (∅, (0, 0, nil)) closed ------------------
    if (tid == 0) {
      C* c = &fa[0];
      for (int q = 0; q < KMAX; ++q) c->cnt[q] = 0;
      c->tail = 0; c->hash = 0; c->tok = 0;
      c->ptrace = TRACE_NONE; c->move = TRACE_NONE; c->slot = 0;
      const int r = closure<KMAX>(c, K, s_cs, recs, hd.flags);
      if (r == CL_DEAD) s_nnext = 0;
      else s_nnext = 1;
      if (r >= CL_COMPLETE) { s_found = 1; s_found_p4 = (r == CL_P4); }
      uint32_t t = TRACE_NONE;
      if (s_witness_ok) {
        if (s_tleft == 0) {
          const unsigned long long b = atomicAdd(p.trace_head, (unsigned long long)TRACE_CHUNK);
          if (b + TRACE_CHUNK <= p.trace_cap) { s_tbase = b; s_tleft = TRACE_CHUNK; }
          else s_witness_ok = 0;
        }
        if (s_witness_ok) {
          t = (uint32_t)s_tbase; s_tbase += 1; s_tleft -= 1;
          p.trace[t].parent = TRACE_NONE; p.trace[t].move = TRACE_NONE;
        }
      }
      c->trace = t;
    }
    __syncthreads();

    C* cur = fa;
    C* nxt = fb;
    uint32_t ncur = s_nnext;
    uint64_t configs = ncur;
    uint32_t rounds = 0;
    uint32_t verdict = V_ILLEGAL, reason = S2LC_R_SEARCH_EXHAUSTED;
    if (s_found) verdict = V_OK, reason = 0;

    while (!s_found) {
      if (ncur == 0) { verdict = V_ILLEGAL; reason = S2LC_R_SEARCH_EXHAUSTED; break; }
      if (tid == 0) s_nnext = 0;
      const uint32_t total = ncur * (uint32_t)K;
      for (uint32_t base = 0; base < total; base += p.chunk) {
        if (tid == 0) s_nstage = 0;
        __syncthreads();
        // ---- expand: one lane per (configuration, chain) -----------------
        const uint32_t lim = min(total, base + p.chunk);
        for (uint32_t it = base + tid; it < lim; it += BT) {
          const uint32_t i = it / (uint32_t)K;
          const uint32_t j = it - i * (uint32_t)K;
          const C* pc = &cur[i];
          const OpRec r = load_rec(&recs[s_cs[j] + pc->cnt[j]]);
          if ((r.flags & (OPF_SENTINEL | OPF_CLS_E)) || r.call_ev >= pc->minret) continue;
          const State s{pc->tail, pc->hash, pc->tok};
          const bool g = append_guards_ok(r, s);
          State kids[2];
          uint32_t moves[2];
          int nk = 0;
          State opt{0, 0, 0};
          if (g) opt = append_opt(r, s, p.pool);
          if (r.flags & OPF_CLS_D) {
            if (g && opt.tail == r.out_tail) { kids[nk] = opt; moves[nk++] = j; }
          } else {  // indefinite: opt any time; identity only when it holds the minimal return
            if (g) { kids[nk] = opt; moves[nk++] = j; }
            if (r.ret_ev == pc->minret && !(g && state_eq(opt, s))) { kids[nk] = s; moves[nk++] = j | MOVE_IDENT; }
          }
          for (int q = 0; q < nk; ++q) {
            const uint32_t k = atomicAdd(&s_nstage, 1u);
            C* ch = &stage[k];
            const uint4* src = reinterpret_cast<const uint4*>(pc->cnt);
            uint4* dst = reinterpret_cast<uint4*>(ch->cnt);
#pragma unroll
            for (int w = 0; w < KMAX / 8; ++w) dst[w] = src[w];
            ch->cnt[j] = (uint16_t)(ch->cnt[j] + 1);
            ch->tail = kids[q].tail; ch->hash = kids[q].hash; ch->tok = kids[q].tok;
            ch->ptrace = pc->trace;
            ch->move = moves[q];
            const int cr = closure<KMAX>(ch, K, s_cs, recs, hd.flags);
            if (cr == CL_ALIVE) {
              ch->fp = fingerprint<KMAX>(ch, nw);
              ch->slot = 0;
            } else {
              ch->slot = SLOT_DEAD;
              if (cr >= CL_COMPLETE && atomicCAS(&s_found, 0u, 1u) == 0u) {
                s_found_parent = pc->trace; s_found_move = moves[q]; s_found_p4 = (cr == CL_P4);
              }
            }
          }
          if (nk) atomicAdd(&s_children, (uint32_t)nk);
        }
        __syncthreads();
        const uint32_t ns = s_nstage;
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
              const C* o = (ref & STAGE_BIT) ? &stage[ref & ~STAGE_BIT] : &nxt[ref];
              if (cfg_eq<KMAX>(o, ch, nw)) { ch->slot = SLOT_DEAD; break; }
            }
            slot = (slot + 1) & mask;
          }
        }
        __syncthreads();
        // ---- compact survivors into the next frontier ---------------------
        for (uint32_t k = tid; k < ns; k += BT) {
          C* ch = &stage[k];
          if (ch->slot == SLOT_DEAD) continue;
          const uint32_t n = atomicAdd(&s_nnext, 1u);
          if (n < p.fcap) {
            cfg_copy<KMAX>(&nxt[n], ch);
            ht[ch->slot] = ((unsigned long long)(uint32_t)(ch->fp >> 32) << 32) | n;
          } else {
            s_overflow = 1;
          }
        }
        __syncthreads();
        if (s_found || s_overflow) break;
      }
      if (s_overflow) {
        for (uint32_t i = tid; i <= mask; i += BT) ht[i] = HT_EMPTY;
        if (s_found) { verdict = V_OK; reason = 0; ++rounds; }
        else { verdict = V_UNKNOWN; reason = S2LC_R_FRONTIER; }
        __syncthreads();
        break;
      }
      const uint32_t nn = min(s_nnext, p.fcap);
      if (tid == 0) {
        s_tb = TRACE_NONE;
        if (s_witness_ok) {
          if (s_tleft < nn) {
            const unsigned long long want = max((unsigned long long)nn, (unsigned long long)TRACE_CHUNK);
            const unsigned long long b = atomicAdd(p.trace_head, want);
            if (b + want <= p.trace_cap) { s_tbase = b; s_tleft = (uint32_t)want; }
            else s_witness_ok = 0;
          }
          if (s_witness_ok) { s_tb = (uint32_t)s_tbase; s_tbase += nn; s_tleft -= nn; }
        }
      }
      __syncthreads();
      const uint32_t tb = s_tb;
      for (uint32_t n = tid; n < nn; n += BT) {
        C* c = &nxt[n];
        ht[c->slot] = HT_EMPTY;
        if (tb != TRACE_NONE) {
          c->trace = tb + n;
          p.trace[tb + n].parent = c->ptrace;
          p.trace[tb + n].move = c->move;
        } else {
          c->trace = TRACE_NONE;
        }
      }
      __syncthreads();
      configs += nn;
      ++rounds;
      if (s_found) { verdict = V_OK; reason = 0; break; }
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
      R.children = s_children;
      R.p4 = s_found_p4;
      R.final_parent = (verdict == V_OK && s_witness_ok) ? s_found_parent : TRACE_NONE;
      R.final_move = s_found_move;
      R.witness_len = 0;
      R.has_witness = (verdict == V_OK && s_witness_ok) ? 2u : 0u;  // resolved by walk_kernel
    }
    __syncthreads();
  }
}

// Witness extraction: one lane per history walks the parent chain backwards
// and writes the move list in order.
__global__ void walk_kernel(uint32_t n, HistResult* res, const TraceEnt* trace, uint32_t* moves) {
  const uint32_t h = blockIdx.x * blockDim.x + threadIdx.x;
  if (h >= n) return;
  HistResult r = res[h];
  if (r.verdict != V_OK || r.has_witness != 2u) return;
  const uint32_t len = (r.final_move == TRACE_NONE) ? 0u : r.rounds;
  uint32_t* out = moves + r.witness_off;
  bool ok = true;
  if (len) {
    out[len - 1] = r.final_move;
    uint32_t idx = r.final_parent;
    uint32_t pos = len - 1;
    while (pos > 0 && idx != TRACE_NONE) {
      const TraceEnt e = trace[idx];
      out[--pos] = e.move;
      idx = e.parent;
    }
    ok = (pos == 0);
  }
  res[h].witness_len = ok ? len : 0u;
  res[h].has_witness = ok ? 1u : 0u;
}

#define HIPCHK(x)                                                        \
  do {                                                                   \
    hipError_t e_ = (x);                                                 \
    if (e_ != hipSuccess) {                                              \
      err = std::string(#x) + ": " + hipGetErrorString(e_);              \
      return S2LC_EHIP;                                                  \
    }                                                                    \
  } while (0)

template <int KMAX, int BT>
hipError_t launch_search(const Params& prm, uint32_t grid, hipStream_t st) {
  hipLaunchKernelGGL((search_kernel<KMAX, BT>), dim3(grid), dim3(BT), 0, st, prm);
  return hipGetLastError();
}

hipError_t launch_dispatch(uint32_t kmax, uint32_t block, const Params& prm, uint32_t grid, hipStream_t st) {
  if (block == 64) {
    switch (kmax) {
      case 16: return launch_search<16, 64>(prm, grid, st);
      case 32: return launch_search<32, 64>(prm, grid, st);
      case 64: return launch_search<64, 64>(prm, grid, st);
      default: return launch_search<128, 64>(prm, grid, st);
    }
  }
  switch (kmax) {
    case 16: return launch_search<16, 256>(prm, grid, st);
    case 32: return launch_search<32, 256>(prm, grid, st);
    case 64: return launch_search<64, 256>(prm, grid, st);
    default: return launch_search<128, 256>(prm, grid, st);
  }
}

size_t cfg_bytes(uint32_t kmax) { return 48 + 2 * (size_t)kmax; }

SearchGeom make_geom(uint32_t kmax, uint32_t block, uint32_t fcap, uint32_t chunk, uint32_t grid) {
  SearchGeom g;
  g.block = block;
  g.kmax = kmax;
  g.fcap = fcap;
  g.chunk = chunk;
  uint32_t ht = 16;
  while (ht < 2 * (fcap + 2 * chunk)) ht <<= 1;
  g.ht_slots = ht;
  g.grid = grid;
  g.cfg_bytes = cfg_bytes(kmax);
  g.slab_bytes = (2 * (size_t)fcap + 2 * (size_t)chunk) * g.cfg_bytes + (size_t)ht * 8;
  g.slab_bytes = (g.slab_bytes + 255) & ~(size_t)255;
  return g;
}

}  // namespace

int batch_upload(DevBatch& b, const std::vector<const History*>& hs, std::string& err) {
  b.n_hist = (uint32_t)hs.size();
  b.src = hs;
  b.forced.assign(hs.size(), 0);
  uint32_t kmax_needed = 1;
  size_t n_recs = 0, n_pool = 0, n_cs = 0;
  uint64_t moves_total = 0;
  b.h_hist.resize(hs.size());
  b.h_moves_off.resize(hs.size());
  for (size_t i = 0; i < hs.size(); ++i) {
    const History& h = *hs[i];
    if (h.status != 0) { err = "history " + std::to_string(i) + ": " + h.error; return h.status; }
    if (h.structural) { b.forced[i] = 1; }
    if (h.K > 128) { err = "history has more than 128 concurrent chains"; return S2LC_EUNSUPPORTED; }
    if (h.max_chain_len >= 0xFFFF) { err = "chain longer than 65534 ops"; return S2LC_EUNSUPPORTED; }
    kmax_needed = std::max(kmax_needed, h.K);
    HistDesc& d = b.h_hist[i];
    d.rec_base = (uint32_t)n_recs;
    d.cs_base = (uint32_t)n_cs;
    d.K = (uint16_t)h.K;
    d.flags = h.hflags;
    d.n_ops = h.n_ops;
    n_recs += h.recs.size();
    n_cs += h.K + 1;
    n_pool += h.pool.size();
    b.h_moves_off[i] = (uint32_t)moves_total;
    moves_total += h.n_ops + 1;
    b.algo_bytes_inputs += 48ull * h.n_ops;
    for (const OpRec& r : h.recs) b.algo_bytes_inputs += 8ull * r.hash_cnt;
  }
  if (n_recs >= 0xFFFFFFFFull || n_pool >= 0xFFFFFFFFull || moves_total >= 0xFFFFFFFFull) {
    err = "batch too large for 32-bit indices";
    return S2LC_EUNSUPPORTED;
  }
  b.kmax = kmax_needed <= 16 ? 16 : kmax_needed <= 32 ? 32 : kmax_needed <= 64 ? 64 : 128;
  std::vector<OpRec> recs(std::max<size_t>(n_recs, 1));
  std::vector<uint64_t> pool(std::max<size_t>(n_pool, 1));
  std::vector<uint32_t> cs(std::max<size_t>(n_cs, 1));
  size_t pr = 0, pp = 0, pc = 0;
  for (size_t i = 0; i < hs.size(); ++i) {
    const History& h = *hs[i];
    for (const OpRec& r0 : h.recs) {
      OpRec r = r0;
      r.hash_off = (uint32_t)(r0.hash_off + pp);
      recs[pr++] = r;
    }
    for (uint32_t j = 0; j <= h.K && !h.chain_start.empty(); ++j) cs[pc++] = b.h_hist[i].rec_base + h.chain_start[j];
    if (h.chain_start.empty()) cs[pc++] = b.h_hist[i].rec_base;
    std::copy(h.pool.begin(), h.pool.end(), pool.begin() + pp);
    pp += h.pool.size();
  }
  // longest-first processing order (LPT): work ~ ops x chains
  std::vector<uint32_t> order;
  order.reserve(hs.size());
  for (uint32_t i = 0; i < hs.size(); ++i)
    if (!b.forced[i]) order.push_back(i);
  std::stable_sort(order.begin(), order.end(), [&](uint32_t x, uint32_t y) {
    return (uint64_t)b.h_hist[x].n_ops * b.h_hist[x].K > (uint64_t)b.h_hist[y].n_ops * b.h_hist[y].K;
  });
  b.moves_cap = moves_total;
  HIPCHK(hipMalloc(&b.recs, recs.size() * sizeof(OpRec)));
  HIPCHK(hipMalloc(&b.pool, pool.size() * sizeof(uint64_t)));
  HIPCHK(hipMalloc(&b.chain_start, cs.size() * sizeof(uint32_t)));
  HIPCHK(hipMalloc(&b.hist, std::max<size_t>(hs.size(), 1) * sizeof(HistDesc)));
  HIPCHK(hipMalloc(&b.order, std::max<size_t>(order.size(), 1) * sizeof(uint32_t)));
  HIPCHK(hipMalloc(&b.res, std::max<size_t>(hs.size(), 1) * sizeof(HistResult)));
  HIPCHK(hipMalloc(&b.moves, std::max<uint64_t>(moves_total, 1) * sizeof(uint32_t)));
  HIPCHK(hipMalloc(&b.counter, 16 * sizeof(uint32_t)));
  HIPCHK(hipMalloc(&b.trace_head, sizeof(unsigned long long)));
  HIPCHK(hipMemcpy(b.recs, recs.data(), recs.size() * sizeof(OpRec), hipMemcpyHostToDevice));
  HIPCHK(hipMemcpy(b.pool, pool.data(), pool.size() * sizeof(uint64_t), hipMemcpyHostToDevice));
  HIPCHK(hipMemcpy(b.chain_start, cs.data(), cs.size() * sizeof(uint32_t), hipMemcpyHostToDevice));
  if (!hs.empty()) HIPCHK(hipMemcpy(b.hist, b.h_hist.data(), hs.size() * sizeof(HistDesc), hipMemcpyHostToDevice));
  if (!order.empty()) HIPCHK(hipMemcpy(b.order, order.data(), order.size() * sizeof(uint32_t), hipMemcpyHostToDevice));
  b.h_res.assign(hs.size(), HistResult{});
  for (size_t i = 0; i < hs.size(); ++i) b.h_res[i].witness_off = b.h_moves_off[i];
  if (!hs.empty()) HIPCHK(hipMemcpy(b.res, b.h_res.data(), hs.size() * sizeof(HistResult), hipMemcpyHostToDevice));
  return 0;
}

void batch_release(DevBatch& b) {
  void* ptrs[] = {b.recs, b.pool, b.chain_start, b.hist, b.order, b.res, b.moves, b.counter, b.trace, b.trace_head, b.slab};
  for (void* q : ptrs) if (q) (void)hipFree(q);
  b.recs = nullptr; b.pool = nullptr; b.chain_start = nullptr; b.hist = nullptr; b.order = nullptr;
  b.res = nullptr; b.moves = nullptr; b.counter = nullptr; b.trace = nullptr; b.trace_head = nullptr;
  b.slab = nullptr; b.slab_cap = 0; b.trace_cap = 0;
}

static int ensure(void** p, size_t& cap, size_t need, std::string& err) {
  if (need <= cap) return 0;
  if (*p) (void)hipFree(*p);
  *p = nullptr;
  cap = 0;
  HIPCHK(hipMalloc(p, need));
  cap = need;
  return 0;
}

int batch_run(DevBatch& b, hipStream_t stream, uint64_t max_configs, bool witness, RunStats& st, std::string& err) {
  st = RunStats{};
  auto t0 = std::chrono::steady_clock::now();
  const uint32_t n_search = (uint32_t)std::count(b.forced.begin(), b.forced.end(), 0u);
  int dev = 0;
  HIPCHK(hipGetDevice(&dev));
  int n_cu = 256;
  (void)hipDeviceGetAttribute(&n_cu, hipDeviceAttributeMultiprocessorCount, dev);

  // trace pool: generous, reused across runs
  if (witness && b.trace_cap == 0) {
    size_t free_b = 0, total_b = 0;
    HIPCHK(hipMemGetInfo(&free_b, &total_b));
    uint64_t want = std::min<uint64_t>(1ull << 28, (uint64_t)(free_b / 8) / sizeof(TraceEnt));
    want = std::min<uint64_t>(want, 0xFFFFFFF0ull);
    HIPCHK(hipMalloc(&b.trace, want * sizeof(TraceEnt)));
    b.trace_cap = want;
  }
  // main pass: 64-lane workgroups, small frontier slabs, persistent grid
  const uint32_t grid0 = std::max<uint32_t>(1, std::min<uint32_t>(n_search, (uint32_t)n_cu * 16));
  SearchGeom g = make_geom(b.kmax, 64, 1024, 256, grid0);
  size_t cap = b.slab_cap;
  if (ensure((void**)&b.slab, cap, g.slab_bytes * g.grid, err)) return S2LC_EHIP;
  b.slab_cap = cap;

  Params prm;
  prm.recs = b.recs; prm.pool = b.pool; prm.chain_start = b.chain_start; prm.hist = b.hist;
  prm.order = b.order; prm.n_hist = n_search; prm.counter = b.counter;
  prm.slab = b.slab; prm.slab_bytes = g.slab_bytes;
  prm.fcap = g.fcap; prm.chunk = g.chunk; prm.ht_mask = g.ht_slots - 1;
  prm.trace = b.trace; prm.trace_head = b.trace_head; prm.trace_cap = witness ? b.trace_cap : 0;
  prm.res = b.res; prm.max_configs = max_configs; prm.witness = witness ? 1 : 0;

  hipEvent_t e0, e1;
  HIPCHK(hipEventCreate(&e0));
  HIPCHK(hipEventCreate(&e1));
  HIPCHK(hipMemsetAsync(b.counter, 0, 16 * sizeof(uint32_t), stream));
  HIPCHK(hipMemsetAsync(b.trace_head, 0, sizeof(unsigned long long), stream));
  HIPCHK(hipEventRecord(e0, stream));
  if (n_search) {
    HIPCHK(launch_dispatch(g.kmax, g.block, prm, g.grid, stream));
    st.launches++;
  }
  HIPCHK(hipEventRecord(e1, stream));
  HIPCHK(hipMemcpyAsync(b.h_res.data(), b.res, b.n_hist * sizeof(HistResult), hipMemcpyDeviceToHost, stream));
  HIPCHK(hipStreamSynchronize(stream));
  float ms = 0;
  HIPCHK(hipEventElapsedTime(&ms, e0, e1));
  st.kernel_ms = ms;

  // wide pass for frontier overflows: 256-lane workgroups, large slabs
  std::vector<uint32_t> over;
  for (uint32_t i = 0; i < b.n_hist; ++i)
    if (!b.forced[i] && b.h_res[i].verdict == V_UNKNOWN && b.h_res[i].reason == S2LC_R_FRONTIER) over.push_back(i);
  st.n_overflow = (uint32_t)over.size();
  if (!over.empty()) {
    size_t free_b = 0, total_b = 0;
    HIPCHK(hipMemGetInfo(&free_b, &total_b));
    uint32_t fcap = 1u << 20;
    SearchGeom gw = make_geom(b.kmax, 256, fcap, 16384, 1);
    while (gw.slab_bytes > free_b / 2 && fcap > 4096) { fcap >>= 1; gw = make_geom(b.kmax, 256, fcap, 16384, 1); }
    uint32_t gridw = (uint32_t)std::min<size_t>(over.size(), std::max<size_t>(1, (free_b / 2) / gw.slab_bytes));
    gridw = std::min<uint32_t>(gridw, (uint32_t)n_cu);
    gw.grid = gridw;
    if (ensure((void**)&b.slab, b.slab_cap, gw.slab_bytes * gw.grid, err)) return S2LC_EHIP;
    uint32_t* d_over = nullptr;
    HIPCHK(hipMalloc(&d_over, over.size() * sizeof(uint32_t)));
    HIPCHK(hipMemcpyAsync(d_over, over.data(), over.size() * sizeof(uint32_t), hipMemcpyHostToDevice, stream));
    Params pw = prm;
    pw.order = d_over; pw.n_hist = (uint32_t)over.size(); pw.counter = b.counter + 4;
    pw.slab = b.slab; pw.slab_bytes = gw.slab_bytes;
    pw.fcap = gw.fcap; pw.chunk = gw.chunk; pw.ht_mask = gw.ht_slots - 1;
    HIPCHK(launch_dispatch(gw.kmax, gw.block, pw, gw.grid, stream));
    st.launches++;
    HIPCHK(hipMemcpyAsync(b.h_res.data(), b.res, b.n_hist * sizeof(HistResult), hipMemcpyDeviceToHost, stream));
    HIPCHK(hipStreamSynchronize(stream));
    (void)hipFree(d_over);
  }
  if (witness && b.n_hist) {
    hipLaunchKernelGGL(walk_kernel, dim3((b.n_hist + 255) / 256), dim3(256), 0, stream, b.n_hist, b.res,
                       (const TraceEnt*)b.trace, b.moves);
    HIPCHK(hipGetLastError());
    HIPCHK(hipMemcpyAsync(b.h_res.data(), b.res, b.n_hist * sizeof(HistResult), hipMemcpyDeviceToHost, stream));
    HIPCHK(hipStreamSynchronize(stream));
  }
  HIPCHK(hipEventDestroy(e0));
  HIPCHK(hipEventDestroy(e1));
  for (uint32_t i = 0; i < b.n_hist; ++i) {
    if (b.forced[i]) {
      b.h_res[i] = HistResult{};
      b.h_res[i].verdict = V_ILLEGAL;
      b.h_res[i].reason = S2LC_R_UNMATCHED;
      b.h_res[i].witness_off = b.h_moves_off[i];
      continue;
    }
    const HistResult& r = b.h_res[i];
    st.configs += r.configs;
    st.children += r.children;
    st.rounds += r.rounds;
    const uint64_t S = 8 * ((2 * (uint64_t)b.h_hist[i].K + 20 + 7) / 8);
    st.algo_bytes += 2 * S * r.configs + 8 * r.children;
  }
  st.algo_bytes += b.algo_bytes_inputs;
  st.total_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
  return 0;
}

}  // namespace s2lc
