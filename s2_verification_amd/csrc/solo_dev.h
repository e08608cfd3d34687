// solo_dev.h — solo rounds of the level search: rounds whose frontier is ONE
// configuration (included by level_dev.h inside its namespace, after the
// grid barrier).
//
// Most rounds of a hard history keep exactly one configuration (C5: 9,937 of
// 10,493; H174: 10,129 of 10,285). The children of one configuration are
// pairwise distinct (each linearizes a different durable / indefinite op, or
// the same indefinite op with two different states), so such a round needs no
// dedupe table and no grid: workgroup 0 of lv_persist runs it alone while the
// other workgroups wait at the grid barrier. Same search as lv_expand
// (E-closure, I-identity deferral, P1/P2/P4), replacing
// porcupine v1.0.3 checkSingle (golang/s2-porcupine/main.go:606); every
// round's configuration count equals the grid mappings' and oracle/reduced.c's.
//
// A round's work is about one closure (C5: 77 candidate moves per round, 97 %
// of them P1-dead in the precheck, ~1.1 with a child to close), so a round is
// run by ONE wave, with no barrier per round, and written for latency:
//   - histories whose reachable tails fit 32 bits (H_TAIL32; every hard
//     history here) only: tails, record counts, match_seq_nums and P1 bounds
//     are 32-bit (a value that cannot be a reachable tail maps to one that
//     never equals one); other histories run their narrow rounds on the grid;
//   - the configuration lives in LDS (structure of arrays, conflict-free):
//     every chain's head (closure fields, the move's fields, its first 8
//     record hashes) and the record after it (a child's first new head on
//     that chain), read by each round once, with one wait. Only the
//     chains the surviving child advanced are reloaded, at the carry; each
//     reload then touches what that chain's next advance will load (the
//     record after the next one, the next one's record hashes) with loads
//     into an LDS sink, so the next reload hits the caches;
//   - the precheck of every candidate move (guards, outcome, the P1 bound
//     without the move's own chain) is branch-free over the chain slots, its
//     results per-lane bit masks;
//   - a move's record hashes are folded on the scalar unit (wave-uniform
//     inputs: the chain of 64-bit multiplies runs as s_mul_* instead of
//     quarter-rate vector multiplies);
//   - a child's closure keeps its heads in registers with a key per head (its
//     call event if it is an identity op legal at the child's state): a pass
//     is a compare per slot and one DPP reduction;
//   - the fingerprint's chain terms are recomputed only when a configuration
//     is staged (a round with several survivors, or the phase's end);
//   - a round with more than 16 live moves (S2LC_SOLO_MAXLIVE) goes to the
//     grid, which spreads its moves over many waves;
//   - the round loop is its own (not inlined) function, its rare paths too:
//     registers are allocated for the loop alone.
#pragma once

// A carry round's close on registers (the run state's per-round fields held
// by the solo wave for the phase, written back before its last close and at
// its exit; S2LC_SOLO_REGRUN=0: every round closes on the LDS run state)
#ifndef S2LC_SOLO_REGRUN
#define S2LC_SOLO_REGRUN 1
#endif
// The child setup's flag tests kept in the move loop (an opaque copy of each
// slot's flags; S2LC_SOLO_NOHOIST=0 lets the compiler hoist them out of it:
// profiles/r06/solo_nohoist_ab.txt)
#ifndef S2LC_SOLO_NOHOIST
#define S2LC_SOLO_NOHOIST 1
#endif
// After a carry, touch the records the advanced chains' next advance will
// load (S2LC_SOLO_TOUCH=0 turns it off; profiles/r06/solo_touch_ab.txt)
#ifndef S2LC_SOLO_TOUCH
#define S2LC_SOLO_TOUCH 1
#endif
constexpr int LV_SOLO_HP = 4;   // record hashes of each head kept in LvSolo
constexpr int LV_SOLO_HP2 = 4;  // the next ones, in LvSoloExt (8 in LDS: 91 % of C5's appends)
constexpr int LV_SOLO_HPT = LV_SOLO_HP + LV_SOLO_HP2;

// 32-bit forms of a record's values for H_TAIL32 histories (every reachable
// tail is below 2^32 - 3): a tail / match_seq_num / out_tail that cannot be a
// reachable tail maps to 0xFFFFFFFF, which never equals one; P1 bounds map by
// suf32 (monotone, exact against every reachable tail).
__host__ __device__ __forceinline__ uint32_t tail32(uint64_t v) { return v >> 32 ? 0xFFFFFFFFu : (uint32_t)v; }

// Per-chain head data beside the closure fields (structure of arrays).
template <int NQ>
struct LvSoloExt {
  uint32_t nr[64 * NQ];                     // num_records (< 2^32 under H_TAIL32)
  uint32_t msn[64 * NQ];                    // tail32(match_seq_num)
  uint32_t hoff[64 * NQ], hcnt[64 * NQ];    // record-hash range
  uint32_t toks[64 * NQ];                   // batch_tok | set_tok << 16 (OpRec bytes 56..59)
  uint64_t hp2[LV_SOLO_HP2][64 * NQ];       // record hashes LV_SOLO_HP.. of each head
};
// The closure fields of the heads (PL) and of the records after them (NX):
// LvHeadsLds's memory (the grid rounds' per-wave heads), viewed 32-bit.
template <int NQ>
struct LvSoloHeads {
  uint32_t ot[64 * NQ];   // tail32(out_tail)
  uint32_t suf[64 * NQ];  // suf32(sufmin)
  uint32_t call[64 * NQ], ret[64 * NQ], fl[64 * NQ];
  uint64_t oh[64 * NQ];   // out_hash
};
template <int NQ>
struct LvSolo {
  uint64_t hp[LV_SOLO_HP][64 * NQ];  // the heads' first record hashes
  uint32_t nx_hoff[64 * NQ], nx_hcnt[64 * NQ];  // record-hash range of each head's next record
  uint16_t cnt[64 * NQ];   // the configuration's chain counts
  uint16_t keep[64 * NQ];  // advance per chain (a staged child's; the phase's kept child at its end)
  uint64_t tail, hash, chx;        // the configuration: state, XOR of its chain terms
  uint64_t ktail, khash, kchx;     // the kept child
  uint32_t tok, pmin, ptrace, ktok, kmr, kmv, cs_end, xtrace;
  uint64_t wx[LV_BLOCK / 64];
#if S2LC_SOLO_TOUCH
  uint32_t sink[64];  // destination of the cache-touch loads (never read)
#endif
#ifdef S2LC_PROF
  unsigned long long pt[8];  // wave 0 phase cycles: [0] start [1] setup [2] pre [3] moves [4] close [5] next [6] wait; [7] last stamp
  unsigned long long pc[6];  // closure cycles (ALIVE, other), ALIVE closures, stage cycles, closure passes, closure head loads
  unsigned long long pm[5];  // moves: fold, child setup, closure loop, keep + prefetch cycles; moves
#endif
};

// (the ballot builtin on a bool: HIP's __ballot(int) had the compiler
// materialize the condition as 0 / 1 in a VGPR and compare it again)
__device__ __forceinline__ uint64_t wballot(bool b) { return __builtin_amdgcn_ballot_w64(b); }
__device__ __forceinline__ uint32_t uni32(uint32_t v) { return (uint32_t)__builtin_amdgcn_readfirstlane((int)v); }
__device__ __forceinline__ uint64_t uni64(uint64_t v) {
  return ((uint64_t)uni32((uint32_t)(v >> 32)) << 32) | uni32((uint32_t)v);
}

// Wave reductions that finish with row broadcasts (row_bcast:15 into rows 1
// and 3, row_bcast:31 into rows 2 and 3: lane 63 holds the result, one
// readlane) instead of four readlanes and scalar combines
// (profiles/r06/solo_rbcast_ab.txt)
template <int CTRL, int ROWS>
__device__ __forceinline__ uint32_t solo_bcast(uint32_t v, uint32_t old) {
  return (uint32_t)__builtin_amdgcn_update_dpp((int)old, (int)v, CTRL, ROWS, 0xF, false);
}
__device__ __forceinline__ uint32_t solo_wave_min(uint32_t v) {
  v = min(v, lv_dpp<0xB1>(v));
  v = min(v, lv_dpp<0x4E>(v));
  v = min(v, lv_dpp<0x124>(v));
  v = min(v, lv_dpp<0x128>(v));
  v = min(v, solo_bcast<0x142, 0xA>(v, v));
  v = min(v, solo_bcast<0x143, 0xC>(v, v));
  return rl(v, 63);
}
__device__ __forceinline__ uint32_t solo_wave_sum(uint32_t c) {
  c += lv_dpp<0xB1>(c);
  c += lv_dpp<0x4E>(c);
  c += lv_dpp<0x124>(c);
  c += lv_dpp<0x128>(c);
  c += solo_bcast<0x142, 0xA>(c, 0u);
  c += solo_bcast<0x143, 0xC>(c, 0u);
  return rl(c, 63);
}

// (smallest, second smallest) of v over the wave's chain slots (a value held
// by two chains is both), wave-uniform
template <int CTRL>
__device__ __forceinline__ void min2_step32(uint32_t& a, uint32_t& b) {
  const uint32_t oa = lv_dpp<CTRL>(a), ob = lv_dpp<CTRL>(b);
  b = min(max(a, oa), min(b, ob));
  a = min(a, oa);
}
template <int NQ>
__device__ __forceinline__ void wave_min2_32(const uint32_t (&v)[NQ], uint32_t& m1, uint32_t& m2) {
  uint32_t a = 0xFFFFFFFFu, b = 0xFFFFFFFFu;
#pragma unroll
  for (int q = 0; q < NQ; ++q) {
    b = min(b, max(a, v[q]));
    a = min(a, v[q]);
  }
  min2_step32<0xB1>(a, b);
  min2_step32<0x4E>(a, b);
  min2_step32<0x124>(a, b);
  min2_step32<0x128>(a, b);
  {  // (rows a bcast does not write combine with (INF, INF): unchanged)
    const uint32_t oa = solo_bcast<0x142, 0xA>(a, 0xFFFFFFFFu), ob = solo_bcast<0x142, 0xA>(b, 0xFFFFFFFFu);
    b = min(max(a, oa), min(b, ob));
    a = min(a, oa);
  }
  {
    const uint32_t oa = solo_bcast<0x143, 0xC>(a, 0xFFFFFFFFu), ob = solo_bcast<0x143, 0xC>(b, 0xFFFFFFFFu);
    b = min(max(a, oa), min(b, ob));
    a = min(a, oa);
  }
  m1 = rl(a, 63);
  m2 = rl(b, 63);
}

// Closure keys of a head at the child's state (tail t, hash h): its call
// event if it is an identity op legal there (ident_legal, main.go:320-331 and
// :283-285), resp. an identity op that kills the child once minimal (P2: a
// successful read at the state's tail with another hash), else EV_INF. One
// compare against the previous pass's minret then gives the lanes that act.
struct SoloKeys { uint32_t ekey, dkey; };
__device__ __forceinline__ SoloKeys solo_keys(uint32_t fl, uint32_t call, uint32_t ot, uint64_t oh, uint32_t t,
                                              uint64_t h, bool p2) {
  const bool e = (fl & OPF_CLS_E) != 0;
  const bool defin = (fl & OPF_KIND_MASK) == 0;  // a definite append failure (the only E append): {s}
  const bool fail = (fl & OPF_FAIL) != 0;
  const bool hash_bad = ((fl & OPF_HAS_HASH) != 0) & (h != oh);
  const bool tail_eq = ot == t;
  const bool legal = defin | (!hash_bad & (fail | tail_eq));
  const bool p2d = p2 & !defin & hash_bad & !fail & tail_eq;
  return SoloKeys{(e & legal) ? call : EV_INF, (e & p2d) ? call : EV_INF};
}

// A head's first 8 record hashes (range [ho, ho + hc)), loaded together:
// unconditional loads with clamped indices (a guarded load per hash would be
// compiled into a wait per hash); pool index 0 always exists.
__device__ __forceinline__ void lv_solo_hashes(const uint64_t* __restrict__ pool, uint32_t ho, uint32_t hc,
                                               uint64_t (&hv)[LV_SOLO_HPT]) {
#pragma unroll
  for (int k = 0; k < LV_SOLO_HPT; ++k) hv[k] = lv_gld64(pool + (hc ? ho + min((uint32_t)k, hc - 1u) : 0u));
}

// A solo configuration's head on chain j (record x = bytes 0..63, its next
// record y = bytes 16..63, the head's first record hashes hv) into LDS.
template <int NQ>
__device__ __forceinline__ void lv_solo_head_put(const uint4& x0, const uint4& x1, const uint4& x2, const uint4& x3,
                                                 const uint4& y1, const uint4& y2, const uint4& y3,
                                                 const uint64_t (&hv)[LV_SOLO_HPT], uint32_t j, LvSoloHeads<NQ>& PL,
                                                 LvSoloHeads<NQ>& NX, LvSoloExt<NQ>& FR, LvSolo<NQ>& S) {
  FR.nr[j] = x0.x;  // (x0.y == 0 under H_TAIL32)
  FR.msn[j] = x0.w ? 0xFFFFFFFFu : x0.z;
  FR.hoff[j] = x3.x;
  FR.hcnt[j] = x3.y;
  FR.toks[j] = x3.z;
  PL.ot[j] = x1.y ? 0xFFFFFFFFu : x1.x;
  PL.oh[j] = (uint64_t)x1.z | ((uint64_t)x1.w << 32);
  PL.suf[j] = suf32((uint64_t)x2.x | ((uint64_t)x2.y << 32));
  PL.call[j] = x2.z;
  PL.ret[j] = x2.w;
  PL.fl[j] = x3.w;
  NX.ot[j] = y1.y ? 0xFFFFFFFFu : y1.x;
  NX.oh[j] = (uint64_t)y1.z | ((uint64_t)y1.w << 32);
  NX.suf[j] = suf32((uint64_t)y2.x | ((uint64_t)y2.y << 32));
  NX.call[j] = y2.z;
  NX.ret[j] = y2.w;
  NX.fl[j] = y3.w;
  S.nx_hoff[j] = y3.x;
  S.nx_hcnt[j] = y3.y;
#pragma unroll
  for (int k = 0; k < LV_SOLO_HP; ++k) S.hp[k][j] = hv[k];
#pragma unroll
  for (int k = 0; k < LV_SOLO_HP2; ++k) FR.hp2[k][j] = hv[LV_SOLO_HP + k];
}

// The head on chain j at record h (chain end: `end`, its sentinel's index + 1)
// loaded and put. `known`: the head's hash range is already known (it was the
// previous head's next record), so the hash loads go out with the record
// loads instead of after them.
#if S2LC_SOLO_TOUCH
// (inline asm, not the builtin: the compiler tracks the builtin's LDS write
// and waits for it before every later LDS read it cannot tell apart from the
// sink, which makes the touch a blocking load. Untracked, it only makes a
// later counted vmcnt wait over-wait, never under-wait: loads retire in order.)
__device__ __forceinline__ void lv_touch(const void* g, uint32_t* sink) {
  const uint32_t dst = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) uint32_t*)sink;
  uint32_t keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dword %1, off\n\ts_mov_b32 m0, %0"
               : "=&s"(keep) : "v"(g), "s"(dst));
}
#endif
template <int NQ>
__device__ __forceinline__ void lv_solo_head(const uint64_t* pool, const OpRec* h, const OpRec* end, uint32_t j,
                                             bool known, LvSoloHeads<NQ>& PL, LvSoloHeads<NQ>& NX,
                                             LvSoloExt<NQ>& FR, LvSolo<NQ>& S, bool touch = false) {
  const uint4* a = reinterpret_cast<const uint4*>(h);
  const uint4* b = reinterpret_cast<const uint4*>(h + 1 < end ? h + 1 : h);  // (the sentinel has no next record)
  const uint4 x0 = lv_gld16(a), x1 = lv_gld16(a + 1), x2 = lv_gld16(a + 2), x3 = lv_gld16(a + 3);
  const uint4 y1 = lv_gld16(b + 1), y2 = lv_gld16(b + 2), y3 = lv_gld16(b + 3);
  uint64_t hv[LV_SOLO_HPT];
  if (known) lv_solo_hashes(pool, S.nx_hoff[j], S.nx_hcnt[j], hv);
  else lv_solo_hashes(pool, x3.x, x3.y, hv);
  lv_solo_head_put<NQ>(x0, x1, x2, x3, y1, y2, y3, hv, j, PL, NX, FR, S);
#if S2LC_SOLO_TOUCH
  if (touch) {
    // what this chain's next advance loads (the record after the next one,
    // the next one's record hashes), pulled into the caches by loads that
    // write LDS (no register waits for them)
    lv_touch(h + 2 < end ? h + 2 : h, S.sink);
    const uint32_t ho = y3.y ? y3.x : 0u;
    lv_touch(pool + ho, S.sink);
    lv_touch(pool + ho + (y3.y > 8u ? 7u : (y3.y ? y3.y - 1u : 0u)), S.sink);
  }
#endif
}

// What the solo round loop reads besides LDS (kernel-parameter values; the
// loop is a function of its own). A by-value argument: the caller writes it to
// the call frame right before the call and the callee reads it in its
// prologue (tests/test_kernel_resources.py checks exactly that). No field is
// indexed dynamically (the staging arrays by round parity are two fields,
// selected by a ternary): a dynamic index would keep the struct in scratch
// inside the round loop. (Handing it over through LDS instead was measured in
// round 6: C5's solo rounds 63.5 -> 64.8 ms, the callee's registers allocated
// differently; profiles/r06/solo_args_ab.txt.)
struct SoloArgs {
  const OpRec* recs;
  const uint64_t* pool;
  TraceEnt* trace;
  uint32_t* rcounts;
  unsigned long long* prof;
  uint8_t* stg0;
  uint8_t* stg1;
  uint32_t* idx0;
  uint32_t* idx1;
  uint64_t trace_cap;
  unsigned long long deadline;  // device wall clock; 0 = none
  uint32_t K, hflags, scap, scs, tgid, max_rounds, max_live;
};

// ---- rare paths of a solo round, out of line (noinline): their lane masks
// and addressing stay out of the round loop's registers ----------------------

// A second (third, ...) survivor of a round: staged at slot k of the round's
// staging array with its fingerprint (the parent's chain terms are recomputed
// when S.chx is stale: chx_ok == 0). Its advance per slot is in S.keep, the
// parent's counts in S.cnt. Written in the form lv_stage_insert leaves.
template <int NQ>
__device__ __attribute__((noinline)) void lv_solo_stage(LvSolo<NQ>& S, uint8_t* stg, uint32_t* nxt_idx,
                                                        TraceEnt* trace, uint32_t tgid, uint32_t K, uint32_t k,
                                                        uint64_t tail, uint64_t hash, uint32_t tok, uint32_t minret,
                                                        uint32_t ptrace, uint32_t move, uint32_t tbase, uint32_t wit,
                                                        uint32_t chx_ok) {
  const int lane = (int)(threadIdx.x & 63);
  uint32_t cnt[NQ], d[NQ];
  uint64_t x = 0, dx = 0;
#pragma unroll
  for (int q = 0; q < NQ; ++q) {
    const uint32_t j = (uint32_t)lane + 64u * q;
    cnt[q] = S.cnt[j];
    d[q] = S.keep[j];
    if (!chx_ok && j < K) x ^= lv_chain_term(j, cnt[q]);
    if (d[q]) dx ^= lv_chain_term(j, cnt[q]) ^ lv_chain_term(j, cnt[q] + d[q]);
  }
  uint64_t pchx;
  if (!chx_ok) {
    pchx = wave_xor_u64(x);
    if (lane == 0) S.chx = pchx;
  } else {
    pchx = uni64(S.chx);
  }
  const uint64_t cdx = pchx ^ wave_xor_u64(dx);
  const uint64_t fp = mix64(cdx ^ lv_state_term(tail, hash, tok));
  LCfg<NQ>* o = lv_cfg<NQ>(stg, k);
  const uint32_t tr = wit ? tgid + tbase + k : TRACE_NONE;
  if (lane == 0) {  // the header line
    unsigned long long* h = reinterpret_cast<unsigned long long*>(o);
    st_wt64(h + 0, tail);
    st_wt64(h + 1, hash);
    st_wt64(h + 2, fp);
    st_wt64(h + 3, (unsigned long long)minret << 32 | tok);
    st_wt64(h + 4, (unsigned long long)move << 32 | ptrace);
    st_wt64(h + 5, (unsigned long long)LV_NONE << 32 | tr);
    st_wt64(h + 6, cdx);
    for (int i = 7; i < 16; ++i) st_wt64(h + i, 0ull);
  }
  lv_store_cnt_wt<NQ>(o->cnt, cnt, d);
  if (lane == 0) {
    st_wt32(&nxt_idx[k], k);
    if (wit) trace[tbase + k] = TraceEnt{ptrace, move};
  }
}

// A lane whose kept child advanced two or more of its chain slots reloads
// them after the round (the early loads hold one chain per lane); the
// advances are in S.keep.
template <int NQ>
__device__ __attribute__((noinline)) void lv_solo_reload_lane(const OpRec* recs, const uint64_t* pool,
                                                              const uint32_t* s_cs, uint32_t K, LvSoloHeads<NQ>& PL,
                                                              LvSoloHeads<NQ>& NX, LvSoloExt<NQ>& FR, LvSolo<NQ>& S) {
  const int lane = (int)(threadIdx.x & 63);
  for (int q = 0; q < NQ; ++q) {
    const uint32_t j = (uint32_t)lane + 64u * q;
    const uint32_t dj = S.keep[j];
    if (!dj) continue;
    const uint32_t c = S.cnt[j] + dj;
    S.cnt[j] = (uint16_t)c;
    lv_solo_head<NQ>(pool, recs + s_cs[j] + c, recs + (j + 1 < K ? s_cs[j + 1] : S.cs_end), j, dj == 1, PL, NX, FR, S);
  }
}

// A closure's head after a chain's second advance (not in LDS): its closure fields
struct SoloHead { uint64_t oh; uint32_t ot, suf, call, ret, fl; };
__device__ __attribute__((noinline)) SoloHead lv_solo_load_head(const OpRec* r) {
  const uint8_t* rb = reinterpret_cast<const uint8_t*>(r);
  const uint4 o = lv_gld16(rb + 16), mm = lv_gld16(rb + 32);
  SoloHead h;
  h.fl = lv_gld32(&r->flags);
  h.ot = o.y ? 0xFFFFFFFFu : o.x;
  h.oh = (uint64_t)o.z | ((uint64_t)o.w << 32);
  h.suf = suf32((uint64_t)mm.x | ((uint64_t)mm.y << 32));
  h.call = mm.z;
  h.ret = mm.w;
  return h;
}

// chain terms of the configuration in S.cnt (+ d), XORed over the wave
template <int NQ>
__device__ __forceinline__ uint64_t lv_solo_chx(const LvSolo<NQ>& S, uint32_t K, const uint32_t (&d)[NQ]) {
  const int lane = (int)(threadIdx.x & 63);
  uint64_t x = 0;
#pragma unroll
  for (int q = 0; q < NQ; ++q) {
    const uint32_t j = (uint32_t)lane + 64u * q;
    if (j < K) x ^= lv_chain_term(j, (uint32_t)S.cnt[j] + d[q]);
  }
  return wave_xor_u64(x);
}

enum : uint32_t { SX_END = 0, SX_OVF = 1, SX_STAGED = 2, SX_MAX = 3, SX_GRID = 4 };

#ifdef S2LC_PROF
#define LV_SOLO_T(i) do { if (lane == 0) { const unsigned long long t_ = clock64(); S.pt[i] += t_ - S.pt[7]; S.pt[7] = t_; } } while (0)
#else
#define LV_SOLO_T(i) do { } while (0)
#endif

// The solo rounds of one phase, run by wave 0 of workgroup 0 alone (no
// barrier per round; waves 1..3 wait for the phase's end). Returns how the
// phase ended (SX_*); the configuration / kept child to write is left in S.
template <int NQ>
__device__ __attribute__((noinline)) uint32_t lv_solo_wave(const SoloArgs pa, LvRun& R, LvSoloHeads<NQ>& PL,
                                                           LvSoloHeads<NQ>& NX, LvSoloExt<NQ>& FR,
                                                           const uint32_t* s_cs, LvSolo<NQ>& S) {
  const SoloArgs& p = pa;
  const int lane = (int)(threadIdx.x & 63);
  const uint32_t K = p.K, hf = p.hflags;
  const bool p1 = hf & H_NOWRAP, p2 = hf & H_P2OK, p4 = hf & H_P4, idefer = hf & H_IDEFER;
  // the configuration (wave-uniform) and its heads' closure fields (registers)
  uint32_t ptail = tail32(uni64(S.tail)), ptok = uni32(S.tok), pmin = uni32(S.pmin), ptrace = uni32(S.ptrace);
  uint64_t phash = uni64(S.hash);
  bool chx_ok = true;  // S.chx is the configuration's (false after a carry: recomputed on demand)
  uint32_t ex = SX_END;
#ifdef S2LC_PROF
  unsigned long long pf_closures = 0, pf_dead = 0;
#endif
#if S2LC_SOLO_REGRUN
  // the run state's fields a carry round's close changes (lv_close_state with
  // one new configuration, no overflow, not found), wave-uniform; R is behind
  // by `nfast` such closes until flush() writes them back (lane 0)
  uint32_t g_round = uni32(R.round), g_wit = uni32(R.witness), g_ltb = uni32(R.last_tbase), g_done = uni32(R.done);
  uint64_t g_tnext = uni64(R.tnext), g_ch = 0;
  uint32_t nfast = 0;  // (each adds one configuration: R.configs += nfast)
  // fast rounds the budget allows (lv_close_state: configs > max_configs)
  uint32_t fast_cap;
  {
    const uint64_t mc = uni64(R.max_configs), cf = uni64(R.configs);
    fast_cap = !mc ? 0xFFFFFFFFu : cf >= mc ? 0u : (uint32_t)min<uint64_t>(mc - cf, 0xFFFFFFFFull);
  }
  auto flush = [&]() {
    if (nfast && lane == 0) {
      R.round = g_round; R.witness = g_wit; R.last_tbase = g_ltb; R.done = g_done;
      R.tnext = g_tnext; R.configs += nfast; R.children += g_ch;
      R.nf = 1; R.last_nf = 1; R.last_closed = 0; R.max_frontier = max(R.max_frontier, 1u);
      R.solo_rounds += nfast;
    }
    nfast = 0;
    g_ch = 0;
  };
#endif
  for (uint32_t n = 0;; ++n) {
#if S2LC_SOLO_REGRUN
    const uint32_t r = g_round + 1;
    const uint32_t tbase = (uint32_t)g_tnext, wit = g_wit;
#else
    const uint32_t r = uni32(R.round) + 1;
    const uint32_t tbase = uni32((uint32_t)R.tnext), wit = uni32(R.witness);
#endif
    if (p.deadline && (n & 15) == 15 && uni64(wall_clock64()) > p.deadline) {
      // the run's deadline (checked every 16 rounds): Unknown (timeout)
#if S2LC_SOLO_REGRUN
      flush();
#endif
      if (lane == 0) R.done = LVR_TIMEOUT;
      ex = SX_END;
      break;
    }
    // the heads' closure fields and the precheck's values, read from LDS at
    // the round's start with one wait (held in registers across rounds, they
    // cost the loop ~30 back-edge copies and a register update per carry:
    // profiles/r06/solo_ldsheads_ab.txt)
    uint32_t hcall[NQ], hret[NQ], hfl[NQ], hsuf[NQ];
    uint32_t a_nr[NQ], a_msn[NQ], a_toks[NQ], a_ot[NQ], a_nxs[NQ];
#pragma unroll
    for (int q = 0; q < NQ; ++q) {
      const uint32_t j = (uint32_t)(64 * q + lane);
      hcall[q] = PL.call[j]; hret[q] = PL.ret[j]; hfl[q] = PL.fl[j]; hsuf[q] = PL.suf[j];
      a_nr[q] = FR.nr[j]; a_msn[q] = FR.msn[j]; a_toks[q] = FR.toks[j]; a_ot[q] = PL.ot[j]; a_nxs[q] = NX.suf[j];
    }
#pragma unroll
    for (int q = 0; q < NQ; ++q) {
      asm volatile("" : "+v"(hcall[q]), "+v"(hret[q]), "+v"(hfl[q]), "+v"(hsuf[q]));
      asm volatile("" : "+v"(a_nr[q]), "+v"(a_msn[q]), "+v"(a_toks[q]), "+v"(a_ot[q]), "+v"(a_nxs[q]));
    }
    LV_SOLO_T(0);
    // P1: a child's bound is the parent's with the moved chain's head
    // replaced by its next record, so (smallest, second smallest) over all
    // heads gives every child's bound without its own chain
    uint32_t b1 = 0xFFFFFFFFu, b2 = 0xFFFFFFFFu;
    if (p1) wave_min2_32<NQ>(hsuf, b1, b2);
    LV_SOLO_T(1);
    // Precheck of every candidate (minimal durable / indefinite appends at
    // the heads), branch-free: guards, the opt child's tail, P1. Per-lane bit
    // masks over the slots: opt child to close, identity child possible
    // (I-op, deferral), the identity child's existence needs the fold (opt ==
    // s on everything but the hash).
    uint32_t b_opt = 0, b_tip = 0, b_eqn = 0, b_dead = 0;
    // every slot's values read first, with one wait for all of them: a value
    // only some lanes need (msn) would otherwise be loaded under a branch,
    // one LDS round trip after another
#pragma unroll
    for (int q = 0; q < NQ; ++q) {
      const uint32_t nr = a_nr[q], msn = a_msn[q], toks = a_toks[q], otl = a_ot[q], nxs = a_nxs[q];
      const uint32_t fl = hfl[q];
      // (bitwise & | on the conditions, not && ||: the short-circuit forms
      // were compiled into exec-mask branches per slot)
      const bool cand = ((fl & (OPF_SENTINEL | OPF_CLS_E)) == 0) & (hcall[q] < pmin);
      const uint32_t bt = toks & 0xFFFFu, st = toks >> 16;
      const bool g = ((bt == 0) | ((ptok != 0) & (ptok == bt))) & (((fl & OPF_HAS_MSN) == 0) | (msn == ptail));
      const uint32_t ot = ptail + nr;  // (no wrap under H_TAIL32)
      const bool to = g & (((fl & OPF_CLS_D) == 0) | (ot == otl));
      const uint32_t others = hsuf[q] == b1 ? b2 : b1;
      const bool dead = p1 & to & (ot > min(others, nxs));
      const bool tip = ((fl & OPF_CLS_I) != 0) & (!idefer | (hret[q] == pmin));
      const bool eqn = g & (nr == 0) & ((st == 0) | (st == ptok));
      const uint32_t bit = cand ? 1u << q : 0u;
      b_opt |= (to & !dead) ? bit : 0u;
      b_tip |= tip ? bit : 0u;
      b_eqn |= (tip & eqn) ? bit : 0u;
      b_dead |= (cand & dead) ? bit : 0u;
    }
    uint32_t b_live = b_opt | b_tip;
    LV_SOLO_T(2);
    uint32_t n_dead, tot;
    {
      // live moves of the round and P1-dead opt children (wave-wide sums of
      // the per-lane counts, one reduction: 16 bits each, at most 320)
      const uint32_t sum = solo_wave_sum((uint32_t)__popc(b_live) | ((uint32_t)__popc(b_dead) << 16));
      tot = sum & 0xFFFFu;
      n_dead = sum >> 16;
      if (tot > p.max_live) {
        // a wide round: the grid expands it (its moves spread over many waves)
        ex = SX_GRID;
#if S2LC_SOLO_REGRUN
        flush();  // (before the writes below: the grid round's slices read last_closed)
#endif
        if (lane == 0) { R.solo_skip = r; R.last_nf = 1; R.last_closed = tot; }
        break;
      }
    }

    // the moves with a child to close; the first survivor (the kept child:
    // the next configuration when it is the only one) stays in registers
    uint32_t alive = 0, found = 0, ovf = 0, fpar = 0, fmov = 0, fp4 = 0;
    uint32_t kd[NQ];  // the kept child's advance per slot
#pragma unroll
    for (int q = 0; q < NQ; ++q) kd[q] = 0;
    uint32_t ktail = ptail, ktok = ptok, kmr = 0, kmv = 0;
    uint64_t khash = phash;
    unsigned long long kids = n_dead;  // (P1-dead opt children: counted, never closed)
    for (;;) {
      const uint64_t m = wballot(b_live != 0);
      if (m == 0 || found) break;
      const int src = __ffsll((unsigned long long)m) - 1;
      const uint32_t lb = rl(b_live, src);
      const uint32_t q_cur = (uint32_t)__ffs(lb) - 1;
      if (lane == src) b_live &= b_live - 1;
      const uint32_t j = 64u * q_cur + (uint32_t)src;
#ifdef S2LC_PROF
      const unsigned long long tm0_ = clock64();
#endif
      // the move (wave-uniform): its outcome, the fold on the scalar unit;
      // the 8 LDS hashes and the next record's fields read together
      const bool m_opt = (rl(b_opt, src) >> q_cur) & 1u, m_tip = (rl(b_tip, src) >> q_cur) & 1u,
                 m_eqn = (rl(b_eqn, src) >> q_cur) & 1u;
      const uint32_t nr = uni32(FR.nr[j]), toks = uni32(FR.toks[j]), hcnt = uni32(FR.hcnt[j]), hoff = uni32(FR.hoff[j]);
      uint64_t hv[LV_SOLO_HPT];
#pragma unroll
      for (int k = 0; k < LV_SOLO_HP; ++k) hv[k] = S.hp[k][j];
#pragma unroll
      for (int k = 0; k < LV_SOLO_HP2; ++k) hv[LV_SOLO_HP + k] = FR.hp2[k][j];
      const uint32_t nx_call = NX.call[j], nx_ret = NX.ret[j], nx_fl = NX.fl[j], nx_suf = NX.suf[j], nx_ot = NX.ot[j];
      const uint64_t nx_oh = NX.oh[j];
      // (all 8 hash loads issued here, with the move's other reads: the
      // compiler sank the first one into the fold, a wait of its own)
#pragma unroll
      for (int k = 0; k < LV_SOLO_HPT; ++k) asm volatile("" : "+v"(hv[k]));
      const uint32_t otail = ptail + nr, otok = (toks >> 16) ? (toks >> 16) : ptok;
      uint64_t ohash = phash;
      if (m_opt || m_eqn) {
        // (uni64 at every step: phash is a loop-carried VGPR value, so
        // without it the chain of 64-bit multiplies is selected as VALU code)
        uint64_t h = uni64(phash);
#pragma unroll
        for (int k = 0; k < LV_SOLO_HPT; ++k)
          if ((uint32_t)k < hcnt) h = uni64(chain_hash(h, uni64(hv[k])));
        for (uint32_t k = LV_SOLO_HPT; k < hcnt; ++k) h = uni64(chain_hash(h, uni64(lv_gld64(p.pool + hoff + k))));
        ohash = h;
      }
#ifdef S2LC_PROF
      if (lane == 0) { S.pm[0] += clock64() - tm0_; S.pm[4] += 1; }
#endif
      const bool c_id = m_tip && !(m_eqn && ohash == phash);
#pragma unroll 1
      for (int w = 0; w < 2 && !found; ++w) {
        if (!(w == 0 ? m_opt : c_id)) continue;
        const uint32_t ct = w == 0 ? otail : ptail, ck = w == 0 ? otok : ptok;
        const uint64_t ch = w == 0 ? ohash : phash;
        const uint32_t mv = w == 0 ? j : (j | MOVE_IDENT);
        ++kids;
#ifdef S2LC_PROF
        ++pf_closures;
        const unsigned long long tc0_ = clock64();
#endif
        // the child's heads: the parent's, but the moved chain's next
        // record on (q_cur, src); their closure keys at the child's state
        uint32_t ccall[NQ], cret[NQ], csuf[NQ], ek[NQ], dk[NQ], d[NQ];
        const SoloKeys nk = solo_keys(nx_fl, nx_call, nx_ot, nx_oh, ct, ch, p2);
#pragma unroll
        for (int q = 0; q < NQ; ++q) {
          const uint32_t jq = (uint32_t)(64 * q + lane);
          const bool mvd = (uint32_t)q == q_cur && lane == src;
#if S2LC_SOLO_NOHOIST
          // (an opaque copy of the flags: the compiler would hoist their
          // per-slot tests out of the move loop, which runs ~1.1 times a
          // round, and hold ~20 VGPRs and 10 SGPR masks across it)
          uint32_t flq = hfl[q];
          asm volatile("" : "+v"(flq));
          const SoloKeys k0 = solo_keys(flq, hcall[q], a_ot[q], PL.oh[jq], ct, ch, p2);  // (a_ot: PL.ot, read at the round's start)
#else
          const SoloKeys k0 = solo_keys(hfl[q], hcall[q], PL.ot[jq], PL.oh[jq], ct, ch, p2);
#endif
          ccall[q] = mvd ? nx_call : hcall[q];
          cret[q] = mvd ? nx_ret : hret[q];
          csuf[q] = mvd ? nx_suf : hsuf[q];
          ek[q] = mvd ? nk.ekey : k0.ekey;
          dk[q] = mvd ? nk.dkey : k0.dkey;
          d[q] = mvd ? 1u : 0u;
        }
#ifdef S2LC_PROF
        const unsigned long long tcs_ = clock64();
        if (lane == 0) S.pm[1] += tcs_ - tc0_;
#endif
        // E-closure: every identity head minimal under the previous pass's
        // minret and legal at the child's state advances; a pass that
        // changes nothing read exactly the final heads (lv_closure). P1: a
        // pending observer needs a smaller tail; P2: a minimal read at the
        // child's tail with another hash.
        uint32_t mprev = pmin, minret = pmin;
        int res;
        for (;;) {
          uint32_t mr = EV_INF, advb = 0, bad = 0;
#pragma unroll
          for (int q = 0; q < NQ; ++q) {
            mr = min(mr, cret[q]);
            advb |= ek[q] < mprev ? 1u << q : 0u;
            bad |= (uint32_t)((dk[q] < mprev) | (p1 & (csuf[q] < ct)));
          }
          minret = solo_wave_min(mr);
#ifdef S2LC_PROF
          if (lane == 0) S.pc[4] += 1;
#endif
          if (wballot(bad != 0)) { res = CL_DEAD; break; }
          const uint64_t am = wballot(advb != 0);
          if (am == 0 && minret == mprev) {
            if (minret == EV_INF) {
              res = CL_COMPLETE;
            } else {
              bool con = false;  // P4: no pending op constrains the state
#pragma unroll
              for (int q = 0; q < NQ; ++q) con |= csuf[q] != 0xFFFFFFFFu;
              res = (p4 && wballot(con) == 0) ? CL_P4 : CL_ALIVE;
            }
            break;
          }
#pragma unroll
          for (int q = 0; q < NQ; ++q) {
            const bool a = (advb >> q) & 1u;
            if (wballot(a) == 0) continue;
            // the head after the current one: the next record (LDS) after
            // the parent's head, else a load (a chain advanced twice: rare)
            const uint32_t jq = (uint32_t)(64 * q + lane);
            uint32_t n_call = NX.call[jq], n_ret = NX.ret[jq], n_fl = NX.fl[jq], n_suf = NX.suf[jq], n_ot = NX.ot[jq];
            uint64_t n_oh = NX.oh[jq];
            const bool gl = a && d[q] != 0;
            if (wballot(gl)) {
              if (gl) {
                const SoloHead hh = lv_solo_load_head(p.recs + s_cs[jq] + S.cnt[jq] + d[q] + 1);
                n_fl = hh.fl; n_ot = hh.ot; n_oh = hh.oh; n_suf = hh.suf; n_call = hh.call; n_ret = hh.ret;
#ifdef S2LC_PROF
                atomicAdd(&S.pc[5], 1ull);
#endif
              }
            }
            const SoloKeys k1 = solo_keys(n_fl, n_call, n_ot, n_oh, ct, ch, p2);
            ccall[q] = a ? n_call : ccall[q];
            cret[q] = a ? n_ret : cret[q];
            csuf[q] = a ? n_suf : csuf[q];
            ek[q] = a ? k1.ekey : ek[q];
            dk[q] = a ? k1.dkey : dk[q];
            d[q] += a ? 1u : 0u;
          }
          mprev = minret;
        }
#ifdef S2LC_PROF
        const unsigned long long tc1_ = clock64();
        if (lane == 0) {
          S.pm[2] += tc1_ - tcs_;
          S.pc[res == CL_ALIVE ? 0 : 1] += tc1_ - tc0_;
          if (res == CL_ALIVE) S.pc[2] += 1;
        }
#endif
        if (res == CL_COMPLETE || res == CL_P4) {
          found = 1; fpar = ptrace; fmov = mv; fp4 = res == CL_P4 ? 1u : 0u;
        } else if (res == CL_ALIVE) {
          // distinct children: staging slot = arrival order; the first one
          // stays in registers (the next configuration when it is the only one)
          const uint32_t k = alive++;
          if (k == 0) {
            ktail = ct; khash = ch; ktok = ck; kmr = minret; kmv = mv;
#pragma unroll
            for (int q = 0; q < NQ; ++q) kd[q] = d[q];
          } else if (k < pa.scs) {
#pragma unroll
            for (int q = 0; q < NQ; ++q) S.keep[lane + 64 * q] = (uint16_t)d[q];
            lv_solo_stage<NQ>(S, (r & 1) ? pa.stg1 : pa.stg0, (r & 1) ? pa.idx1 : pa.idx0, p.trace, p.tgid, K, k, ct, ch, ck, minret, ptrace, mv,
                              tbase, wit, chx_ok ? 1u : 0u);
            chx_ok = true;
          } else {
            ovf = 1;
          }
#ifdef S2LC_PROF
          if (lane == 0) { const unsigned long long t_ = clock64() - tc1_; S.pc[3] += t_; S.pm[3] += t_; }
#endif
        }
      }
    }
    LV_SOLO_T(3);
#ifdef S2LC_PROF
    pf_dead += n_dead;
#endif
    const bool carry = !found && !ovf && alive == 1;
#if S2LC_SOLO_REGRUN
    if (carry) {
      // lv_close_state for one new configuration, on the registers
      g_ch += kids;
      g_round = r;
      if (g_wit) {
        g_ltb = (uint32_t)g_tnext;
        g_tnext += 1;
        if (g_tnext + p.scap > p.trace_cap) g_wit = 0;
      }
      ++nfast;
      if (nfast > fast_cap) g_done = LVR_BUDGET;
      if (lane == 0) {
        if (p.rcounts) lv_gst32(p.rcounts + r, 1u);
        if (wit) lv_gst64(p.trace + tbase, (unsigned long long)kmv << 32 | ptrace);
      }
    } else {
      flush();
    }
    if (!carry && lane == 0) {
#else
    // close the round on the run state (lane 0; every lane reads it back)
    if (lane == 0) {
#endif
      LvCounts kc;
      kc.nn = alive; kc.ovf = ovf; kc.fnd = found;
      kc.fpar = fpar; kc.fmov = fmov; kc.fp4 = fp4; kc.ch = kids; kc.closed = 0;
      // (no clock read per round: s_memrealtime is a scalar-memory round
      // trip; the phase's time is added at its end)
      lv_close_state(R, kc, r, p.rcounts, p.scap, p.trace_cap, false);
      R.solo_rounds++;
      // the first survivor's trace entry (it was not staged)
      if (!found && !ovf && alive && wit) lv_gst64(p.trace + tbase, (unsigned long long)kmv << 32 | ptrace);
#ifdef S2LC_PROF
      if (p.prof) { atomicAdd(&p.prof[29], (unsigned long long)alive); atomicAdd(&p.prof[30], alive == 1 ? 1ull : 0ull); }
#endif
    }
#if S2LC_SOLO_REGRUN && defined(S2LC_PROF)
    if (carry && lane == 0 && p.prof) { atomicAdd(&p.prof[29], 1ull); atomicAdd(&p.prof[30], 1ull); }
#endif
    if (carry) {
      // the kept child becomes the configuration: its advanced chains into
      // LDS (early loads; a lane with two advanced slots loads them now) and
      // their closure fields into registers
      uint32_t nmine = 0, qm = 0;
#pragma unroll
      for (int q = 0; q < NQ; ++q)
        if (kd[q]) { ++nmine; qm = (uint32_t)q; }
      if (nmine == 1) {
        const uint32_t jj = (uint32_t)lane + 64u * qm, dd = sel_u32<NQ>(kd, qm);
        const uint32_t c = (uint32_t)S.cnt[jj] + dd;
        S.cnt[jj] = (uint16_t)c;
        lv_solo_head<NQ>(p.pool, p.recs + s_cs[jj] + c, p.recs + (jj + 1 < K ? s_cs[jj + 1] : S.cs_end), jj, dd == 1,
                         PL, NX, FR, S, true);
      } else if (nmine > 1) {
#pragma unroll
        for (int q = 0; q < NQ; ++q) S.keep[lane + 64 * q] = (uint16_t)kd[q];
        lv_solo_reload_lane<NQ>(p.recs, p.pool, s_cs, K, PL, NX, FR, S);
      }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      ptail = ktail; phash = khash; ptok = ktok; pmin = kmr;
      ptrace = wit ? p.tgid + tbase : TRACE_NONE;
      chx_ok = false;
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // (lane 0's close, read back by every lane)
    LV_SOLO_T(4);
#if S2LC_SOLO_REGRUN
    const uint32_t done = carry ? g_done : uni32(R.done), nf = carry ? 1u : uni32(R.nf);
#else
    const uint32_t done = uni32(R.done), nf = uni32(R.nf);
#endif
    if (found || done != LVR_RUNNING) { ex = (ovf && !found) ? SX_OVF : SX_END; break; }
    if (alive >= 2) {
      // the kept child joins the staged ones at the phase's exit (S.keep, S.k*)
      ex = SX_STAGED;
      const uint64_t kx = lv_solo_chx<NQ>(S, K, kd);
#pragma unroll
      for (int q = 0; q < NQ; ++q) S.keep[lane + 64 * q] = (uint16_t)kd[q];
      if (lane == 0) {
        S.kchx = kx;
        S.ktail = ktail; S.khash = khash; S.ktok = ktok; S.kmr = kmr; S.kmv = kmv;
        S.xtrace = wit ? p.tgid + tbase : TRACE_NONE;
      }
      break;
    }
    if (nf != 1) { ex = SX_END; break; }
    if (n + 1 >= p.max_rounds) { ex = SX_MAX; break; }
  }
#if S2LC_SOLO_REGRUN
  flush();
#endif
  // leave the configuration (and the kept child) in S for the phase's exit writes
  if (ex != SX_END) {
    uint32_t z[NQ];
#pragma unroll
    for (int q = 0; q < NQ; ++q) z[q] = 0;
    if (!chx_ok) {
      const uint64_t x = lv_solo_chx<NQ>(S, K, z);
      if (lane == 0) S.chx = x;
    }
  }
  if (lane == 0) {
    // the phase's rounds (narrow, solo) in the run's wall-clock split
    const unsigned long long now = wall_clock64();
    R.narrow_ticks += now - R.t_last;
    R.solo_ticks += now - R.t_last;
    R.t_last = now;
    S.tail = ptail; S.hash = phash; S.tok = ptok; S.pmin = pmin; S.ptrace = ptrace;
#ifdef S2LC_PROF
    if (p.prof) {
      atomicAdd(&p.prof[14], pf_closures);
      atomicAdd(&p.prof[15], pf_dead);
    }
#endif
  }
#if S2LC_SOLO_TOUCH
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // (the touches land before the phase ends)
#endif
  return ex;
}

// The whole workgroup writes a solo configuration held in LDS (counts
// S.cnt[j] + (child ? S.keep[j] : 0), the configuration's or the kept child's
// header) into staging slot 0 of `stg` / index list `idx`: the form a grid
// round leaves its frontier in.
template <int NQ>
__device__ void lv_solo_write(const LvSolo<NQ>& S, bool child, uint8_t* stg, uint32_t* idx, uint32_t trace_id,
                              uint32_t K) {
  LCfg<NQ>* o = lv_cfg<NQ>(stg, 0);
  for (uint32_t j = threadIdx.x; j < 64u * NQ; j += LV_BLOCK)
    st_wt16(&o->cnt[j], (uint16_t)(j < K ? S.cnt[j] + (child ? S.keep[j] : 0u) : 0u));
  if (threadIdx.x < 16) {
    const uint32_t l = threadIdx.x;
    const uint64_t tail = child ? S.ktail : S.tail, hash = child ? S.khash : S.hash;
    const uint32_t tok = child ? S.ktok : S.tok, mr = child ? S.kmr : S.pmin;
    const uint64_t fp = mix64((child ? S.kchx : S.chx) ^ lv_state_term(tail, hash, tok));
    const unsigned long long w = l == 0 ? tail
                               : l == 1 ? hash
                               : l == 2 ? fp
                               : l == 3 ? ((unsigned long long)mr << 32 | tok)
                               : l == 4 ? ((unsigned long long)(child ? S.kmv : LV_NONE) << 32 | (child ? S.ptrace : TRACE_NONE))
                               : l == 5 ? ((unsigned long long)LV_NONE << 32 | trace_id)
                               : l == 6 ? (child ? S.kchx : S.chx)
                                        : 0ull;
    st_wt64(reinterpret_cast<unsigned long long*>(o) + l, w);
  }
  if (threadIdx.x == 0) st_wt32(&idx[0], 0u);
}

// Solo rounds (H_TAIL32 histories, NQ <= 5), run by workgroup 0 of
// lv_persist while the others wait at the grid barrier: enter from the
// frontier's one configuration, go on while every round keeps exactly one,
// and stop when a round keeps none or several, completes, overflows, has
// more live moves than max_live (the grid expands that round), or after
// max_rounds. R is the workgroup's run state; every round is closed on it
// exactly as a grid round is. The LDS views: PL = s_heads[0], NX =
// s_heads[1], FR = s_heads[2..3] (lv_persist).
template <int NQ>
__device__ void lv_solo_rounds(const LvParams& p, const LvPersist& q, LvRun& R, LvSoloHeads<NQ>& PL,
                               LvSoloHeads<NQ>& NX, LvSoloExt<NQ>& FR, const uint32_t* s_cs, LvSolo<NQ>& S,
                               uint32_t max_rounds, unsigned long long deadline) {
  const uint32_t K = p.K;
  if (threadIdx.x == 0) S.cs_end = p.cs[K];
  lv_sync_lds();
  const uint32_t r0 = R.round + 1;
  {  // the configuration: counts, heads, state, chain terms (the whole workgroup)
    const LCfg<NQ>* pc = lv_cfg<NQ>(q.stg[(r0 + 1) & 1], q.idx[(r0 + 1) & 1][0]);
    uint64_t chx = 0;
    for (uint32_t j = threadIdx.x; j < 64u * NQ; j += LV_BLOCK) {
      const uint32_t c = j < K ? (uint32_t)pc->cnt[j] : 0u;
      S.cnt[j] = (uint16_t)c;
      S.keep[j] = 0;
      if (j < K) {
        lv_solo_head<NQ>(p.pool, p.recs + s_cs[j] + c, p.recs + (j + 1 < K ? s_cs[j + 1] : S.cs_end), j, false, PL, NX,
                         FR, S);
        chx ^= lv_chain_term(j, c);
      } else {  // (no chain: a sentinel-like head; its P1 bound is REQ_NONE: suf32 0xFFFFFFFF)
        PL.fl[j] = OPF_SENTINEL; PL.call[j] = EV_INF; PL.ret[j] = EV_INF; PL.suf[j] = 0xFFFFFFFFu;
        NX.fl[j] = OPF_SENTINEL; NX.call[j] = EV_INF; NX.ret[j] = EV_INF; NX.suf[j] = 0xFFFFFFFFu;
      }
    }
    chx = wave_xor_u64(chx);
    if ((threadIdx.x & 63) == 0) S.wx[threadIdx.x >> 6] = chx;
    if (threadIdx.x == 0) {
      S.tail = pc->tail; S.hash = pc->hash; S.tok = pc->tok;
      S.pmin = pc->minret; S.ptrace = pc->trace;
      if (pc->slot <= p.ht_mask) st_wt64(&q.ht[(r0 + 1) & 1][pc->slot], HT_EMPTY);
    }
    lv_sync_lds();
    if (threadIdx.x == 0) {
      uint64_t x = 0;
      for (int w = 0; w < LV_BLOCK / 64; ++w) x ^= S.wx[w];
      S.chx = x;
#ifdef S2LC_PROF
      for (int i_ = 0; i_ < 8; ++i_) S.pt[i_] = 0;
      for (int i_ = 0; i_ < 6; ++i_) S.pc[i_] = 0;
      for (int i_ = 0; i_ < 5; ++i_) S.pm[i_] = 0;
      S.pt[7] = clock64();
#endif
    }
    lv_sync_lds();
  }
#ifdef S2LC_PROF
  const unsigned long long t_solo = wall_clock64();
  const uint32_t rounds0 = R.solo_rounds;
#endif
  // the rounds: wave 0 alone (waves 1..3 wait here)
  __shared__ uint32_t s_ex;
  if (threadIdx.x < 64) {
    SoloArgs a;
    a.recs = p.recs; a.pool = p.pool; a.trace = p.trace; a.rcounts = p.rcounts; a.prof = p.prof;
    a.stg0 = q.stg[0]; a.stg1 = q.stg[1]; a.idx0 = q.idx[0]; a.idx1 = q.idx[1];
    a.trace_cap = p.trace_cap;
    a.deadline = deadline;
    a.K = p.K; a.hflags = p.hflags; a.scap = p.scap; a.scs = p.scs; a.tgid = p.tgid;
    a.max_rounds = max_rounds;
    // more live moves than this in a round: the grid expands it (S2LC_SOLO_MAXLIVE)
    a.max_live = q.solo_maxlive ? q.solo_maxlive : 8u;  // (sweep: profiles/r04/maxlive_sweep.txt)
    const uint32_t ex = lv_solo_wave<NQ>(a, R, PL, NX, FR, s_cs, S);
    if (threadIdx.x == 0) s_ex = ex;
  }
  __syncthreads();
  const uint32_t ex = s_ex;
  const uint32_t r = R.round + 1;  // (after the phase: the next round)
  if (ex == SX_OVF || ex == SX_GRID) {
    // round r (overflowed: the host re-runs it; or wide: the grid runs it),
    // from its frontier: this configuration, in the staging array round r
    // reads its frontier from
    lv_solo_write<NQ>(S, false, q.stg[(r + 1) & 1], q.idx[(r + 1) & 1], S.ptrace, K);
  } else if (ex == SX_STAGED) {
    // the kept child joins the staged ones at slot 0 of round r - 1's staging
    lv_solo_write<NQ>(S, true, q.stg[(r - 1) & 1], q.idx[(r - 1) & 1], S.xtrace, K);
  } else if (ex == SX_MAX) {
    // leaving with one configuration: the next round's frontier
    lv_solo_write<NQ>(S, false, q.stg[(r + 1) & 1], q.idx[(r + 1) & 1], S.ptrace, K);
  }
#ifdef S2LC_PROF
  if (threadIdx.x == 0 && p.prof) {  // [7] solo rounds, [8] their wall-clock ticks, [16..21] phase cycles
    atomicAdd(&p.prof[7], (unsigned long long)(R.solo_rounds - rounds0));
    atomicAdd(&p.prof[8], wall_clock64() - t_solo);
    for (int i_ = 0; i_ < 6; ++i_) atomicAdd(&p.prof[16 + i_], S.pt[i_]);
    for (int i_ = 0; i_ < 6; ++i_) atomicAdd(&p.prof[22 + i_], S.pc[i_]);
    for (int i_ = 0; i_ < 5; ++i_) atomicAdd(&p.prof[32 + i_], S.pm[i_]);
  }
#endif
}
#undef LV_SOLO_T
