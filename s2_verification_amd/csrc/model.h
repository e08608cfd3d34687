// model.h — S2 stream model shared by the gfx950 search kernels and the host
// (witness replay, s2lc_step_cpu). Compiled as HIP everywhere.
//
// Reference: s2Model (golang/s2-porcupine/main.go:253-340), chainHash /
// foldRecordHashes (main.go:227-244) over zeebo/xxh3 HashSeed (8-byte path).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace s2lc {

constexpr uint32_t EV_INF = 0xFFFFFFFFu;     // "no event" (chain sentinel call/ret)
constexpr uint64_t REQ_NONE = ~0ull;         // no constraining op remains
constexpr uint64_t REQ_HASH_ONLY = ~0ull - 1; // constraining, but on the hash only

// Op record flags ------------------------------------------------------------
enum : uint32_t {
  OPF_KIND_MASK = 0x3u,    // s2lc_input_type
  OPF_FAIL = 0x4u,         // StreamOutput.Failure
  OPF_DEF = 0x8u,          // StreamOutput.DefiniteFailure
  OPF_HAS_TAIL = 0x10u,
  OPF_HAS_HASH = 0x20u,
  OPF_HAS_MSN = 0x40u,
  OPF_CLS_E = 0x100u,      // Step(s) ⊆ {s} for every s: reads, check-tails, definite failures
  OPF_CLS_D = 0x200u,      // durable append: Step(s) ∈ {∅, {opt(s)}}
  OPF_CLS_I = 0x400u,      // indefinite append: s ∈ Step(s) for every s, maybe also opt(s)
  OPF_SENTINEL = 0x800u,   // end-of-chain marker
  OPF_CONSTRAIN = 0x1000u, // must observe the state when linearized (success ops, hash checks)
};

// One operation (call + matched return), 64 bytes = one half cache line.
// Stored chain-major on the device: chain j's ops are contiguous, followed by
// a sentinel record, so "head of chain j at count c" is one indexed load.
struct __attribute__((aligned(64))) OpRec {
  uint64_t num_records;  // *StreamInput.NumRecords
  uint64_t msn;          // *StreamInput.MatchSeqNum (valid iff OPF_HAS_MSN)
  uint64_t out_tail;     // *StreamOutput.Tail (valid iff OPF_HAS_TAIL)
  uint64_t out_hash;     // *StreamOutput.StreamHash (valid iff OPF_HAS_HASH)
  uint64_t sufmin;       // min required pre-tail over constraining ops from here to chain end
  uint32_t call_ev;      // event index of the call
  uint32_t ret_ev;       // event index of the return
  uint32_t hash_off;     // first record hash in the (batch-wide) hash pool
  uint32_t hash_cnt;     // len(RecordHashes) — independent of num_records
  uint16_t batch_tok;    // BatchFencingToken id, 0 = nil
  uint16_t set_tok;      // SetFencingToken id, 0 = nil
  uint32_t flags;
};
static_assert(sizeof(OpRec) == 64, "OpRec must be 64 bytes");

struct State {
  uint64_t tail;
  uint64_t hash;
  uint32_t tok;  // interned token id, 0 = nil (stringPtrEqual <=> id equality)
};

__host__ __device__ inline uint64_t rotl64(uint64_t x, int r) { return (x << r) | (x >> (64 - r)); }

// chainHash(h, r) = xxh3.HashSeed(le64(r), h): XXH3's 4..8-byte path with
// len = 8. Two 64-bit multiplies per record.
__host__ __device__ inline uint64_t chain_hash(uint64_t h, uint64_t r) {
  const uint32_t lo = (uint32_t)h;
  const uint32_t sw = (lo >> 24) | ((lo >> 8) & 0xff00u) | ((lo << 8) & 0xff0000u) | (lo << 24);
  const uint64_t seed = h ^ ((uint64_t)sw << 32);
  uint64_t k = rotl64(r, 32) ^ (0xc73ab174c5ecd5a2ull - seed);
  k ^= rotl64(k, 49) ^ rotl64(k, 24);
  k *= 0x9FB21C651E98DF25ull;
  k ^= (k >> 35) + 8;
  k *= 0x9FB21C651E98DF25ull;
  return k ^ (k >> 28);
}

__host__ __device__ inline uint64_t fold_hashes(uint64_t h, const uint64_t* rs, uint32_t n) {
  for (uint32_t i = 0; i < n; ++i) h = chain_hash(h, rs[i]);
  return h;
}

// Device fold with the record-hash loads issued 8 at a time: the fold is a
// dependent chain of multiplies, but its loads are independent, and a loop that
// loads inside the chain pays one memory latency per record. The 8 loads are
// unconditional (indices clamped to the last record): a guarded load becomes a
// branch per record, and gfx950 code then waits for each load before the
// next one issues (8 memory latencies instead of one).
__device__ inline uint64_t fold_hashes_blk(uint64_t h, const uint64_t* __restrict__ rs, uint32_t n) {
  for (uint32_t b = 0; b < n; b += 8) {
    uint64_t v[8];
    const uint32_t last = n - 1 - b;
#pragma unroll
    for (int q = 0; q < 8; ++q) v[q] = rs[b + min((uint32_t)q, last)];
#pragma unroll
    for (int q = 0; q < 8; ++q)
      if (b + q < n) h = chain_hash(h, v[q]);
  }
  return h;
}

__host__ __device__ inline bool state_eq(const State& a, const State& b) {
  return a.tail == b.tail && a.hash == b.hash && a.tok == b.tok;
}

// Guards of an append at state s (main.go:287-298, 303-312).
__host__ __device__ inline bool append_guards_ok(const OpRec& o, const State& s) {
  if (o.batch_tok && (s.tok == 0 || s.tok != o.batch_tok)) return false;
  if ((o.flags & OPF_HAS_MSN) && o.msn != s.tail) return false;
  return true;
}

// Optimistic post-append state (main.go:272-282).
__host__ __device__ inline State append_opt(const OpRec& o, const State& s, const uint64_t* pool) {
  State r;
  r.tail = s.tail + o.num_records;  // Go uint64 wraparound
  r.hash = fold_hashes(s.hash, pool + o.hash_off, o.hash_cnt);
  r.tok = o.set_tok ? o.set_tok : s.tok;
  return r;
}

// Legality of an identity-class op (OPF_CLS_E) at s: Step(s) == {s}.
__host__ __device__ inline bool ident_legal(const OpRec& o, const State& s) {
  if ((o.flags & OPF_KIND_MASK) == 0) return true;  // definite append failure: {s}
  if ((o.flags & OPF_HAS_HASH) && s.hash != o.out_hash) return false;
  return (o.flags & OPF_FAIL) || s.tail == o.out_tail;
}

// s2Model.Step (main.go:264-335) for one op from one state; writes 0..2
// successors (deduplicated by Equal, like the powerset merge) and returns
// the count. Histories whose Step would panic in Go are rejected at build.
__host__ __device__ inline int s2_step(const OpRec& o, const State& s, const uint64_t* pool, State out[2]) {
  const uint32_t kind = o.flags & OPF_KIND_MASK;
  if (kind == 0) {
    const bool fail = o.flags & OPF_FAIL;
    if (fail && (o.flags & OPF_DEF)) { out[0] = s; return 1; }
    const bool ok = append_guards_ok(o, s);
    if (fail) {
      if (!ok) { out[0] = s; return 1; }
      out[0] = append_opt(o, s, pool);
      out[1] = s;
      return state_eq(out[0], s) ? 1 : 2;
    }
    if (!ok) return 0;
    State opt = append_opt(o, s, pool);
    if (o.out_tail != opt.tail) return 0;
    out[0] = opt;
    return 1;
  }
  if (!ident_legal(o, s)) return 0;
  out[0] = s;
  return 1;
}

}  // namespace s2lc
