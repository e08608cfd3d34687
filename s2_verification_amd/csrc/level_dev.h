// level_dev.h — device-wide level-synchronous search of ONE history (included
// by level.hip). Used for the histories the per-workgroup passes cannot hold:
// frontiers beyond a workgroup's capacity and histories with more than 128
// chains (single hard histories, BASELINE config C5). Same search as
// search_dev.h (rounds of one durable/indefinite append, E-closure,
// I-identity deferral, P1/P2/P4), replacing porcupine v1.0.3 checkSingle
// (called at golang/s2-porcupine/main.go:606), but every phase of a round is a
// grid-wide launch over the whole chip:
//
//   lv_expand : one lane per (frontier configuration, chain) candidate
//               -> raw children (parent, move, successor state), 32 B each
//   lv_close  : one WAVE per child; lane l owns chains l, l+64, ...; a closure
//               pass is one head load per owned chain + wave min-reductions of
//               minret (return events) and the P1 bound; all legal minimal
//               identity ops advance together -> closed configuration staged
//               in HBM with its fingerprint
//   lv_insert : one lane per staged configuration; 64-bit atomicCAS
//               open-addressing table (32-bit tag | staging index), full-key
//               compare on a tag hit; winners form the next frontier (an
//               index list into the staging array) and get a trace entry
//
// The frontier of round r is the staging array written in round r (double
// buffered), so a surviving configuration is written exactly once.
#pragma once

namespace s2lc {
namespace {

constexpr uint32_t LV_NONE = 0xFFFFFFFFu;
constexpr int LV_BLOCK = 256;

// A staged / frontier configuration: 48 + 2*KMAX bytes.
template <int KMAX>
struct __attribute__((aligned(16))) LCfg {
  uint64_t tail;
  uint64_t hash;
  uint64_t fp;      // fingerprint (dedupe / ownership)
  uint32_t tok;
  uint32_t minret;  // exact minret of the closed configuration
  uint32_t ptrace;  // trace index of the parent
  uint32_t move;    // chain | MOVE_IDENT, LV_NONE for the initial configuration
  uint32_t trace;   // own trace index once in a frontier
  uint32_t slot;    // table slot (cleared when this configuration is expanded)
  uint16_t cnt[KMAX];
};
static_assert(offsetof(LCfg<64>, trace) == 40, "LCfg::trace offset (read by the host)");

// A raw child: successor state of frontier configuration `parent` (staging
// index) after the op at the head of chain move & 0xFFFF.
struct __attribute__((aligned(16))) LChild {
  uint64_t tail;
  uint64_t hash;
  uint32_t tok;
  uint32_t parent;  // staging index of the parent, LV_NONE = the all-zero initial configuration
  uint32_t move;
  uint32_t _pad;
};

// Device-side counters of one round.
struct LvCtl {
  uint32_t nchild;    // children produced by lv_expand
  uint32_t nstage;    // closed configurations staged by lv_close
  uint32_t nnext;     // unique configurations inserted by lv_insert
  uint32_t found;     // a child completed (Ok)
  uint32_t overflow;  // 1: children over capacity, 2: staging over capacity
  uint32_t found_parent, found_move, found_p4;
  unsigned long long children;  // running total
  uint32_t done_blocks;         // lv_insert blocks finished (the last one publishes)
  uint32_t _pad[5];
};

struct LvParams {
  const OpRec* __restrict__ recs;
  const uint64_t* __restrict__ pool;
  const uint32_t* __restrict__ cs;  // K+1 absolute chain starts of this history
  uint32_t K;
  uint32_t hflags;
  // current frontier: positions [f0, f1) of cur_idx index cur (staging array)
  const uint8_t* cur;
  const uint32_t* cur_idx;
  uint32_t f0, f1;
  // children
  LChild* child;
  uint32_t ccap;
  // staging of this round (becomes the next frontier) + its index list
  uint8_t* stg;
  uint32_t* nxt_idx;
  uint32_t scap;
  uint32_t st_lo;  // lv_insert: first staged configuration of this chunk
  unsigned long long* ht;
  uint32_t ht_mask;
  uint32_t clear_slots;  // lv_expand clears the table slots of the frontier it expands
  LvCtl* ctl_next;       // lv_expand zeroes the next round's control block (double buffer)
  LvCtl* publish;        // host-mapped mirror lv_insert's last block copies the control block to
  TraceEnt* trace;
  uint32_t tbase;        // trace index of nxt_idx[0] (in this process's pool)
  uint32_t witness;
  uint32_t tgid;         // added to pool indices to form trace ids (distributed: rank << 29)
  LvCtl* ctl;
  // distributed search: ownership buckets of the staged configurations
  uint32_t world;
  uint32_t* own_cnt;     // [world] configurations per owner rank
  uint32_t* own_pos;     // per staged configuration: owner << 27 | position within the owner's bucket
  uint8_t* send;         // bucketed configurations, owner-major
  uint64_t own_off[8];   // first configuration of each owner's bucket in send
};

template <int KMAX>
__device__ __forceinline__ const LCfg<KMAX>* lv_cfg(const uint8_t* base, uint32_t i) {
  return reinterpret_cast<const LCfg<KMAX>*>(base + (size_t)i * sizeof(LCfg<KMAX>));
}
template <int KMAX>
__device__ __forceinline__ LCfg<KMAX>* lv_cfg(uint8_t* base, uint32_t i) {
  return reinterpret_cast<LCfg<KMAX>*>(base + (size_t)i * sizeof(LCfg<KMAX>));
}

__device__ __forceinline__ uint32_t wave_min_u32(uint32_t v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = min(v, (uint32_t)__shfl_xor((int)v, o, 64));
  return v;
}
__device__ __forceinline__ uint64_t wave_min_u64(uint64_t v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const uint32_t lo = (uint32_t)__shfl_xor((int)(uint32_t)v, o, 64);
    const uint32_t hi = (uint32_t)__shfl_xor((int)(uint32_t)(v >> 32), o, 64);
    const uint64_t w = ((uint64_t)hi << 32) | lo;
    v = w < v ? w : v;
  }
  return v;
}
__device__ __forceinline__ uint64_t wave_xor_u64(uint64_t v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const uint32_t lo = (uint32_t)__shfl_xor((int)(uint32_t)v, o, 64);
    const uint32_t hi = (uint32_t)__shfl_xor((int)(uint32_t)(v >> 32), o, 64);
    v ^= ((uint64_t)hi << 32) | lo;
  }
  return v;
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

// Configuration fingerprint: state mix ^ XOR over chains of mix(chain, count).
// Commutative over chains, so a wave computes it with one XOR reduction.
__device__ __forceinline__ uint64_t lv_chain_term(uint32_t j, uint32_t c) {
  return mix64(((uint64_t)j << 32 | c) * 0x9E3779B97F4A7C15ull + 0x2545F4914F6CDD1Dull);
}
__device__ __forceinline__ uint64_t lv_state_term(uint64_t tail, uint64_t hash, uint32_t tok) {
  return mix64(tail ^ 0x9E3779B97F4A7C15ull) ^ mix64(hash + 0x632BE59BD9B4E019ull * (tok + 1));
}

// ---- expand: one lane per (frontier position, chain) ----------------------
template <int KMAX>
__global__ __launch_bounds__(LV_BLOCK) void lv_expand(LvParams p) {
  if (p.ctl_next && blockIdx.x == 0 && threadIdx.x < sizeof(LvCtl) / 4)
    reinterpret_cast<uint32_t*>(p.ctl_next)[threadIdx.x] = 0;
  const uint32_t K = p.K;
  const uint64_t total = (uint64_t)(p.f1 - p.f0) * K;
  const uint64_t stride = (uint64_t)gridDim.x * LV_BLOCK;
  for (uint64_t b0 = (uint64_t)blockIdx.x * LV_BLOCK; b0 < total; b0 += stride) {
    const uint64_t it = b0 + threadIdx.x;
    const bool act = it < total;
    uint32_t nk = 0;
    bool take_opt = false, take_id = false;
    State opt{0, 0, 0}, s{0, 0, 0};
    uint32_t k = 0, j = 0;
    if (act) {
      const uint32_t i = p.f0 + (uint32_t)(it / K);
      j = (uint32_t)(it % K);
      k = p.cur_idx[i];
      const LCfg<KMAX>* pc = lv_cfg<KMAX>(p.cur, k);
      if (j == 0 && p.clear_slots && pc->slot <= p.ht_mask) p.ht[pc->slot] = HT_EMPTY;
      const uint32_t c = pc->cnt[j];
      const OpRec* rp = p.recs + p.cs[j] + c;
      const uint32_t f = rp->flags;
      const uint32_t pmin = pc->minret;
      if (!(f & (OPF_SENTINEL | OPF_CLS_E)) && rp->call_ev < pmin) {
        const OpRec r = load_rec(rp);
        s = State{pc->tail, pc->hash, pc->tok};
        const bool g = append_guards_ok(r, s);
        opt.tail = s.tail + r.num_records;
        opt.tok = r.set_tok ? r.set_tok : s.tok;
        opt.hash = s.hash;
        if (r.flags & OPF_CLS_D) take_opt = g && opt.tail == r.out_tail;
        else take_opt = g;
        if (take_opt || (r.flags & OPF_CLS_I)) {
          if (g) opt.hash = fold_hashes_blk(s.hash, p.pool + r.hash_off, r.hash_cnt);
        }
        if (r.flags & OPF_CLS_I) take_id = (!(p.hflags & H_IDEFER) || r.ret_ev == pmin) && !(g && state_eq(opt, s));
        nk = (uint32_t)take_opt + (uint32_t)take_id;
      }
    }
    const uint32_t base = wave_alloc(&p.ctl->nchild, nk);
    if (nk) {
      uint32_t q = base;
      if (take_opt) {
        if (q < p.ccap) p.child[q] = LChild{opt.tail, opt.hash, opt.tok, k, j, 0};
        ++q;
      }
      if (take_id) {
        if (q < p.ccap) p.child[q] = LChild{s.tail, s.hash, s.tok, k, j | MOVE_IDENT, 0};
        ++q;
      }
      if (q > p.ccap) p.ctl->overflow = 1;
    }
  }
}

// ---- close: one wave per child --------------------------------------------
template <int KMAX>
__global__ __launch_bounds__(LV_BLOCK) void lv_close(LvParams p) {
  constexpr int NQ = KMAX / 64;
  const int lane = (int)(threadIdx.x & 63);
  const uint32_t K = p.K;
  const bool nowrap = p.hflags & H_NOWRAP;
  const bool p2 = p.hflags & H_P2OK;
  const bool p4 = p.hflags & H_P4;
  uint32_t csj[NQ];
#pragma unroll
  for (int q = 0; q < NQ; ++q) {
    const uint32_t j = (uint32_t)lane + 64u * q;
    csj[q] = j < K ? p.cs[j] : 0u;
  }
  const uint32_t nch = min(p.ctl->nchild, p.ccap);
  const uint32_t nwaves = gridDim.x * (LV_BLOCK / 64);
  for (uint32_t ci = blockIdx.x * (LV_BLOCK / 64) + (threadIdx.x >> 6); ci < nch; ci += nwaves) {
    const LChild ch = p.child[ci];
    const State s{ch.tail, ch.hash, ch.tok};
    const LCfg<KMAX>* pc = ch.parent == LV_NONE ? nullptr : lv_cfg<KMAX>(p.cur, ch.parent);
    const uint32_t mj = ch.move == LV_NONE ? LV_NONE : (ch.move & 0xFFFFu);
    uint32_t cnt[NQ];
#pragma unroll
    for (int q = 0; q < NQ; ++q) {
      const uint32_t j = (uint32_t)lane + 64u * q;
      cnt[q] = (j < K && pc) ? (uint32_t)pc->cnt[j] : 0u;
      if (j == mj) cnt[q] += 1;
    }
    int res;
    uint32_t minret;
    // Head fields of the owned chains, kept in registers across passes: a pass
    // reloads only the chains the previous pass advanced (the first pass loads
    // every head), so the closure's L2 traffic is one head per chain plus one
    // per advanced op instead of one per chain per pass.
    uint32_t callv[NQ], flv[NQ], retv[NQ];
    uint64_t otl[NQ], ohs[NQ], smv[NQ];
    uint32_t need = (1u << NQ) - 1u;
    for (;;) {
      uint32_t mr = EV_INF;
      uint64_t bd = REQ_NONE;
#pragma unroll
      for (int q = 0; q < NQ; ++q) {
        const uint32_t j = (uint32_t)lane + 64u * q;
        if (j < K) {
          if ((need >> q) & 1u) {
            const OpRec* r = p.recs + csj[q] + cnt[q];
            const uint4 obs = ld16(r, 16);
            const uint4 mid = ld16(r, 32);
            flv[q] = r->flags;
            otl[q] = (uint64_t)obs.x | ((uint64_t)obs.y << 32);
            ohs[q] = (uint64_t)obs.z | ((uint64_t)obs.w << 32);
            callv[q] = mid.z;
            retv[q] = mid.w;
            smv[q] = (uint64_t)mid.x | ((uint64_t)mid.y << 32);
          }
          mr = min(mr, retv[q]);
          bd = smv[q] < bd ? smv[q] : bd;
        } else {
          flv[q] = OPF_SENTINEL; otl[q] = 0; ohs[q] = 0; callv[q] = EV_INF; retv[q] = EV_INF; smv[q] = REQ_NONE;
        }
      }
      minret = wave_min_u32(mr);
      const uint64_t bound = wave_min_u64(bd);
      uint32_t adv = 0;
      bool dead = false;
#pragma unroll
      for (int q = 0; q < NQ; ++q) {
        const uint32_t f = flv[q];
        if (!(f & OPF_CLS_E) || callv[q] >= minret) continue;
        bool legal = true;
        if ((f & OPF_KIND_MASK) != 0) {
          const bool hash_bad = (f & OPF_HAS_HASH) && s.hash != ohs[q];
          const bool tail_bad = !(f & OPF_FAIL) && s.tail != otl[q];
          legal = !hash_bad && !tail_bad;
          // P2: a minimal successful read at this tail with another hash can never pass
          if (p2 && hash_bad && !(f & OPF_FAIL) && otl[q] == s.tail) dead = true;
        }
        if (legal) adv |= 1u << q;
      }
      if (__ballot(dead) || (nowrap && s.tail > bound)) { res = CL_DEAD; break; }
      if (!__ballot(adv != 0)) {
        res = minret == EV_INF ? CL_COMPLETE : ((p4 && bound == REQ_NONE) ? CL_P4 : CL_ALIVE);
        break;
      }
#pragma unroll
      for (int q = 0; q < NQ; ++q) cnt[q] += (adv >> q) & 1u;
      need = adv;
    }
    if (res == CL_DEAD) continue;
    const uint32_t ptrace = pc ? pc->trace : TRACE_NONE;
    if (res != CL_ALIVE) {
      if (lane == 0 && atomicCAS(&p.ctl->found, 0u, 1u) == 0u) {
        p.ctl->found_parent = ptrace;
        p.ctl->found_move = ch.move;
        p.ctl->found_p4 = res == CL_P4;
      }
      continue;
    }
    uint64_t h = 0;
#pragma unroll
    for (int q = 0; q < NQ; ++q) {
      const uint32_t j = (uint32_t)lane + 64u * q;
      if (j < K) h ^= lv_chain_term(j, cnt[q]);
    }
    const uint64_t fp = mix64(wave_xor_u64(h) ^ lv_state_term(s.tail, s.hash, s.tok));
    uint32_t k = 0;
    if (lane == 0) k = atomicAdd(&p.ctl->nstage, 1u);
    k = (uint32_t)__shfl((int)k, 0, 64);
    if (k >= p.scap) {
      if (lane == 0) p.ctl->overflow = 2;
      continue;
    }
    LCfg<KMAX>* o = lv_cfg<KMAX>(p.stg, k);
    if (lane == 0) {
      o->tail = s.tail; o->hash = s.hash; o->fp = fp; o->tok = s.tok;
      o->minret = minret; o->ptrace = ptrace; o->move = ch.move;
      o->trace = TRACE_NONE; o->slot = LV_NONE;
    }
#pragma unroll
    for (int q = 0; q < NQ; ++q) {
      const uint32_t j = (uint32_t)lane + 64u * q;
      o->cnt[j] = j < K ? (uint16_t)cnt[q] : (uint16_t)0;
    }
  }
}

template <int KMAX>
__device__ __forceinline__ bool lv_eq(const LCfg<KMAX>* a, const LCfg<KMAX>* b, uint32_t K) {
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

// ---- insert: one lane per staged configuration -----------------------------
template <int KMAX>
__global__ __launch_bounds__(LV_BLOCK) void lv_insert(LvParams p) {
  const uint32_t hi = p.ctl->overflow ? 0u : min(p.ctl->nstage, p.scap);
  const uint32_t stride = gridDim.x * LV_BLOCK;
  for (uint32_t b0 = p.st_lo + blockIdx.x * LV_BLOCK; b0 < hi; b0 += stride) {
    const uint32_t k = b0 + threadIdx.x;
    bool win = false;
    uint32_t slot = 0;
    LCfg<KMAX>* c = nullptr;
    if (k < hi) {
      c = lv_cfg<KMAX>(p.stg, k);
      const uint64_t fp = c->fp;
      const uint32_t tag = (uint32_t)(fp >> 32);
      const unsigned long long mine = ((unsigned long long)tag << 32) | k;
      slot = (uint32_t)fp & p.ht_mask;
      for (;;) {
        const unsigned long long prev = atomicCAS(&p.ht[slot], HT_EMPTY, mine);
        if (prev == HT_EMPTY) { win = true; break; }
        if ((uint32_t)(prev >> 32) == tag && lv_eq<KMAX>(lv_cfg<KMAX>(p.stg, (uint32_t)prev), c, p.K)) break;
        slot = (slot + 1) & p.ht_mask;
      }
    }
    const uint32_t n = wave_alloc(&p.ctl->nnext, win ? 1u : 0u);
    if (win) {
      p.nxt_idx[n] = k;
      c->slot = slot;
      if (p.witness) {
        c->trace = p.tgid + p.tbase + n;
        p.trace[p.tbase + n] = TraceEnt{c->ptrace, c->move};
      }
    }
  }
  // the last block to finish copies the control block to the host-mapped
  // mirror: the host then needs no copy, only the stream sync
  if (p.publish) {
    __syncthreads();
    __shared__ uint32_t s_last;
    if (threadIdx.x == 0) {
      __threadfence();
      s_last = atomicAdd(&p.ctl->done_blocks, 1u) == gridDim.x - 1;
    }
    __syncthreads();
    if (s_last && threadIdx.x < sizeof(LvCtl) / 4) {
      __threadfence();
      const uint32_t v = atomicAdd(reinterpret_cast<uint32_t*>(p.ctl) + threadIdx.x, 0u);
      reinterpret_cast<volatile uint32_t*>(p.publish)[threadIdx.x] = v;
      __threadfence_system();
    }
  }
}

// ---- distributed: owner of a configuration ---------------------------------
// Independent of the table slot (low fingerprint bits) and tag (high bits).
__host__ __device__ __forceinline__ uint32_t lv_owner(uint64_t fp, uint32_t world) {
  return (uint32_t)(((fp * 0xD6E8FEB86659FD93ull) >> 40) % world);
}

// one lane per staged configuration: owner bucket and position within it
template <int KMAX>
__global__ __launch_bounds__(LV_BLOCK) void lv_bucket(LvParams p) {
  const uint32_t n = min(p.ctl->nstage, p.scap);
  for (uint32_t k = blockIdx.x * LV_BLOCK + threadIdx.x; k < n; k += gridDim.x * LV_BLOCK) {
    const uint32_t o = lv_owner(lv_cfg<KMAX>(p.stg, k)->fp, p.world);
    const uint32_t pos = atomicAdd(&p.own_cnt[o], 1u);
    p.own_pos[k] = (o << 27) | pos;
  }
}

// one lane per 16-byte piece: copy staged configurations into their owner's bucket
template <int KMAX>
__global__ __launch_bounds__(LV_BLOCK) void lv_scatter(LvParams p) {
  constexpr uint32_t PER = sizeof(LCfg<KMAX>) / 16;
  const uint32_t n = min(p.ctl->nstage, p.scap);
  const uint64_t total = (uint64_t)n * PER;
  for (uint64_t i = (uint64_t)blockIdx.x * LV_BLOCK + threadIdx.x; i < total; i += (uint64_t)gridDim.x * LV_BLOCK) {
    const uint32_t k = (uint32_t)(i / PER), c = (uint32_t)(i % PER);
    const uint32_t op = p.own_pos[k];
    const uint64_t dst = p.own_off[op >> 27] + (op & ((1u << 27) - 1));
    const uint4* src = reinterpret_cast<const uint4*>(lv_cfg<KMAX>(p.stg, k));
    reinterpret_cast<uint4*>(p.send + dst * sizeof(LCfg<KMAX>))[c] = src[c];
  }
}

// keep the frontier configurations this rank owns (replicated -> partitioned)
template <int KMAX>
__global__ __launch_bounds__(LV_BLOCK) void lv_keep(LvParams p, uint32_t rank) {
  const uint32_t nf = p.f1;
  for (uint32_t b0 = blockIdx.x * LV_BLOCK; b0 < nf; b0 += gridDim.x * LV_BLOCK) {
    const uint32_t i = b0 + threadIdx.x;
    uint32_t k = 0;
    bool mine = false;
    if (i < nf) {
      k = p.cur_idx[i];
      mine = lv_owner(lv_cfg<KMAX>(p.cur, k)->fp, p.world) == rank;
    }
    const uint32_t n = wave_alloc(&p.ctl->nnext, mine ? 1u : 0u);
    if (mine) p.nxt_idx[n] = k;
  }
}

// copy the frontier's configurations contiguously into p.send (16 B per lane)
template <int KMAX>
__global__ __launch_bounds__(LV_BLOCK) void lv_gather_frontier(LvParams p) {
  constexpr uint32_t PER = sizeof(LCfg<KMAX>) / 16;
  const uint64_t total = (uint64_t)p.f1 * PER;
  for (uint64_t i = (uint64_t)blockIdx.x * LV_BLOCK + threadIdx.x; i < total; i += (uint64_t)gridDim.x * LV_BLOCK) {
    const uint32_t f = (uint32_t)(i / PER), c = (uint32_t)(i % PER);
    const uint4* src = reinterpret_cast<const uint4*>(lv_cfg<KMAX>(p.cur, p.cur_idx[f]));
    reinterpret_cast<uint4*>(p.send + (uint64_t)f * sizeof(LCfg<KMAX>))[c] = src[c];
  }
}

__global__ void lv_iota(uint32_t* out, uint32_t n) {
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) out[i] = i;
}

}  // namespace
}  // namespace s2lc
