// literal.hip — porcupine's checkSingle run as written, one GPU thread per
// history, for histories with duplicate op ids.
//
// With more than one Start or Finish per op_id, porcupine links each call to
// the nearest later return with its id (makeLinkedEntries; two calls can
// share a return) and keys its linearized bitset and its cache by that id, so
// two ops with one id share a bit. Its verdict then depends on the order of
// its depth-first search, which the frontier search cannot
// reproduce. These histories take this engine instead: the same doubly
// linked entry list, lift / unlift, (bitset, powerset state) cache and
// backtracking stack as checkSingle (porcupine v1.0.3, upstream; restated on
// the CPU in oracle/oracle.c), over the S2 model's Step (model.h s2_step,
// main.go:264-335) merged into powerset states as NondeterministicModel.
// ToModel does. A batch's duplicate-id histories run side by side, one
// thread each, every one in its own slice of device memory; a history that
// outgrows its slice gives Unknown (budget).
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <string>
#include <vector>

#include "s2lincheck.h"
#include "search.h"

namespace s2lc {
namespace {

#define LITCHK(x)                                                                 \
  do {                                                                            \
    hipError_t e_ = (x);                                                          \
    if (e_ != hipSuccess) {                                                       \
      err = std::string("literal: ") + #x + ": " + hipGetErrorString(e_);         \
      return S2LC_EHIP;                                                           \
    }                                                                             \
  } while (0)

struct LitState {
  uint64_t tail, hash;
  uint32_t tok, _pad;
};
struct LitEntry {  // a cache entry: (bitset, state set), chained per hash
  int32_t next;
  uint32_t bits;   // first word in the bitset pool
  uint32_t s_off, s_n;
};
struct LitSlot {
  unsigned long long key;
  int32_t head;    // -1: empty
  int32_t _pad;
};
struct LitCall {
  int32_t entry;   // node
  uint32_t s_off, s_n;
  uint32_t _pad;
};

// one history's work region, carved from its slice of the literal buffer
struct LitWork {
  int32_t* next;  // node links: 0 = head, event i = node i + 1, -1 = nil
  int32_t* prev;
  unsigned long long* lin;
  LitCall* calls;
  LitSlot* table;
  uint32_t table_mask;
  LitEntry* ent;
  uint32_t ent_cap;
  unsigned long long* bits;
  LitState* st;
  uint32_t st_cap;
};

__device__ inline bool lit_carve(uint8_t* base, uint64_t bytes, uint32_t n_ev, uint32_t W, LitWork& w) {
  uint64_t o = 0;
  auto take = [&](uint64_t sz) { const uint64_t at = (o + 15) & ~15ull; o = at + sz; return base + at; };
  w.next = reinterpret_cast<int32_t*>(take(4ull * (n_ev + 1)));
  w.prev = reinterpret_cast<int32_t*>(take(4ull * (n_ev + 1)));
  w.lin = reinterpret_cast<unsigned long long*>(take(8ull * W));
  w.calls = reinterpret_cast<LitCall*>(take(sizeof(LitCall) * (n_ev / 2 + 1)));
  if (o + 4096 > bytes) return false;
  // the rest: per cache entry two table slots, the entry, its bitset and
  // four states of the state pool
  const uint64_t per = 2 * sizeof(LitSlot) + sizeof(LitEntry) + 8ull * W + 4 * sizeof(LitState);
  uint64_t e = (bytes - o - 1024) / per;
  if (e < 8) return false;
  e = std::min<uint64_t>(e, 1ull << 30);
  uint64_t t = 16;
  while (t < e) t <<= 1;  // (<= 2e slots)
  w.table = reinterpret_cast<LitSlot*>(take(sizeof(LitSlot) * t));
  w.table_mask = (uint32_t)(t - 1);
  w.ent = reinterpret_cast<LitEntry*>(take(sizeof(LitEntry) * e));
  w.ent_cap = (uint32_t)e;
  w.bits = reinterpret_cast<unsigned long long*>(take(8ull * W * e));
  const uint64_t left = bytes > o ? (bytes - o) / sizeof(LitState) : 0;
  w.st = reinterpret_cast<LitState*>(take(0));
  w.st_cap = (uint32_t)std::min<uint64_t>(left > 16 ? left - 16 : 0, 0xFFFFFFF0ull);
  return w.st_cap >= 4;
}

__device__ inline bool lit_contains(const LitState* v, uint32_t n, const LitState& x) {
  for (uint32_t i = 0; i < n; ++i)
    if (v[i].tail == x.tail && v[i].hash == x.hash && v[i].tok == x.tok) return true;
  return false;
}

// bitset.hash: popcount of the words, then XOR of the words
__device__ inline unsigned long long lit_bits_hash(const unsigned long long* b, uint32_t W, uint32_t id) {
  unsigned long long pc = 0, x = 0;
  for (uint32_t i = 0; i < W; ++i) {
    const unsigned long long v = b[i] | (i == id / 64 ? 1ull << (id % 64) : 0ull);
    pc += (unsigned long long)__popcll(v);
    x ^= v;
  }
  return pc ^ x;
}

enum : uint32_t { LIT_OK = 0, LIT_ILLEGAL = 1, LIT_BUDGET = 2, LIT_PANIC = 3 };

__global__ void literal_kernel(const LitDesc* __restrict__ descs, uint32_t n, const LitEv* __restrict__ evs,
                               const uint64_t* __restrict__ pool, uint8_t* mem, HistResult* res, uint32_t* moves,
                               unsigned long long max_configs, unsigned long long max_iters,
                               const unsigned long long* deadline) {
  const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= n) return;
  const LitDesc D = descs[t];
  const LitEv* ev = evs + D.ev_off;
  const uint32_t n_ev = D.n_ev, W = D.W;
  LitWork w;
  HistResult& R = res[D.h];
  if (!lit_carve(mem + D.mem_off, D.mem_bytes, n_ev, W, w)) {
    R.verdict = V_UNKNOWN; R.reason = S2LC_R_BUDGET; R.has_witness = 0;
    return;
  }
  // makeLinkedEntries' list, then insertBefore(head, first entry)
  for (uint32_t i = 0; i <= n_ev; ++i) {
    w.next[i] = i < n_ev ? (int32_t)(i + 1) : -1;
    w.prev[i] = i == 0 ? -1 : (int32_t)(i - 1);
  }
  for (uint32_t i = 0; i < W; ++i) w.lin[i] = 0;
  for (uint32_t i = 0; i <= w.table_mask; ++i) w.table[i].head = -1;
  uint32_t n_ent = 0, st_top = 0, ncalls = 0, max_calls = 0;
  unsigned long long steps = 0;
  // Init: the powerset state {(0, 0, nil)}
  uint32_t s_off = st_top, s_n = 1;
  w.st[st_top++] = LitState{0, 0, 0, 0};
  int32_t entry = w.next[0];
  uint32_t outcome = LIT_ILLEGAL;
  // Every thread leaves: porcupine's list surgery on a return shared by two
  // calls can send its search round a cycle (it would then never return),
  // so the loop is bounded by an iteration count and the run's deadline.
  const unsigned long long dl = deadline ? *deadline : 0ull;
  unsigned long long iters = 0;
  bool timed_out = false;
  for (;;) {
    if (w.next[0] == -1) { outcome = LIT_OK; break; }
    if (++iters > max_iters) { outcome = LIT_BUDGET; break; }
    if (dl && (iters & 1023) == 0 && wall_clock64() > dl) { outcome = LIT_BUDGET; timed_out = true; break; }
    if (entry <= 0) { outcome = LIT_PANIC; break; }  // (porcupine: nil entry dereference)
    const LitEv& E = ev[entry - 1];
    if (E.kind == 0 && E.match > 0) {
      // ToModel().Step: every state's successors, merged (first occurrence kept)
      const uint32_t ns_off = st_top;
      uint32_t ns_n = 0;
      bool full = false;
      for (uint32_t k = 0; k < s_n && !full; ++k) {
        State kids[2];
        const LitState& s = w.st[s_off + k];
        const int c = s2_step(E.rec, State{s.tail, s.hash, s.tok}, pool, kids);
        for (int q = 0; q < c; ++q) {
          const LitState x{kids[q].tail, kids[q].hash, kids[q].tok, 0};
          if (lit_contains(w.st + ns_off, ns_n, x)) continue;
          if (ns_off + ns_n >= w.st_cap) { full = true; break; }
          w.st[ns_off + ns_n++] = x;
        }
      }
      if (full) { outcome = LIT_BUDGET; break; }
      ++steps;
      if (ns_n > 0) {
        const uint32_t id = (uint32_t)E.id;
        if (id >= W * 64) { outcome = LIT_PANIC; break; }  // (porcupine: bitset index out of range)
        const unsigned long long hk = lit_bits_hash(w.lin, W, id);
        // cacheContains: an entry with this bitset and an Equal state set
        uint32_t slot = (uint32_t)((hk * 0x9E3779B97F4A7C15ull) >> 20) & w.table_mask;
        while (w.table[slot].head >= 0 && w.table[slot].key != hk) slot = (slot + 1) & w.table_mask;
        bool found = false;
        for (int32_t c = w.table[slot].head; c >= 0 && !found; c = w.ent[c].next) {
          const LitEntry& ce = w.ent[c];
          bool same = true;
          for (uint32_t i = 0; i < W && same; ++i)
            same = w.bits[(uint64_t)ce.bits + i] == (w.lin[i] | (i == id / 64 ? 1ull << (id % 64) : 0ull));
          if (!same) continue;
          bool eq = true;  // sets equal: containsAll both ways
          for (uint32_t i = 0; i < ns_n && eq; ++i) eq = lit_contains(w.st + ce.s_off, ce.s_n, w.st[ns_off + i]);
          for (uint32_t i = 0; i < ce.s_n && eq; ++i) eq = lit_contains(w.st + ns_off, ns_n, w.st[ce.s_off + i]);
          found = eq;
        }
        if (!found) {
          if (n_ent >= w.ent_cap || n_ent >= w.table_mask / 2) { outcome = LIT_BUDGET; break; }
          // (more calls on the stack than calls in the history: only a
          // shared-return list can get here; porcupine's slice would grow)
          if (ncalls >= n_ev / 2 + 1) { outcome = LIT_BUDGET; break; }
          LitEntry& ne = w.ent[n_ent];
          ne.bits = n_ent * W;
          for (uint32_t i = 0; i < W; ++i)
            w.bits[(uint64_t)ne.bits + i] = w.lin[i] | (i == id / 64 ? 1ull << (id % 64) : 0ull);
          ne.s_off = ns_off; ne.s_n = ns_n;
          if (w.table[slot].head < 0) w.table[slot].key = hk;
          ne.next = w.table[slot].head;
          w.table[slot].head = (int32_t)n_ent;
          ++n_ent;
          st_top = ns_off + ns_n;  // the set is the cache's now
          w.calls[ncalls] = LitCall{entry, s_off, s_n, 0};
          ++ncalls;
          max_calls = max(max_calls, ncalls);
          s_off = ns_off; s_n = ns_n;
          w.lin[id / 64] |= 1ull << (id % 64);
          // lift(entry): porcupine writes entry.next.prev unconditionally, so
          // a call left last in the list (two calls sharing one return) is
          // its nil dereference
          const int32_t m = E.match;
          if (w.next[entry] < 0) { outcome = LIT_PANIC; break; }
          w.next[w.prev[entry]] = w.next[entry];
          w.prev[w.next[entry]] = w.prev[entry];
          w.next[w.prev[m]] = w.next[m];
          if (w.next[m] >= 0) w.prev[w.next[m]] = w.prev[m];
          entry = w.next[0];
          if (max_configs && n_ent > max_configs) { outcome = LIT_BUDGET; break; }
          continue;
        }
      }
      entry = w.next[entry];  // (the tentative set is dropped: st_top unchanged)
    } else {
      if (ncalls == 0) { outcome = LIT_ILLEGAL; break; }
      const LitCall top = w.calls[--ncalls];
      entry = top.entry;
      s_off = top.s_off; s_n = top.s_n;
      const uint32_t id = (uint32_t)ev[entry - 1].id;
      w.lin[id / 64] &= ~(1ull << (id % 64));
      // unlift(entry)
      const int32_t m = ev[entry - 1].match;
      w.next[w.prev[m]] = m;
      if (w.next[m] >= 0) w.prev[w.next[m]] = m;
      w.next[w.prev[entry]] = entry;
      if (w.next[entry] < 0) { outcome = LIT_PANIC; break; }  // (entry.next.prev: unconditional)
      w.prev[w.next[entry]] = entry;
      entry = w.next[entry];
    }
  }
  R.verdict = outcome == LIT_OK ? V_OK : outcome == LIT_ILLEGAL ? V_ILLEGAL : V_UNKNOWN;
  R.reason = outcome == LIT_OK ? 0u
           : outcome == LIT_ILLEGAL ? (uint32_t)S2LC_R_SEARCH_EXHAUSTED
           : outcome == LIT_BUDGET ? (timed_out ? (uint32_t)S2LC_R_TIMEOUT : (uint32_t)S2LC_R_BUDGET)
                                   : (uint32_t)S2LC_R_NONE;
  R.rounds = max_calls;
  R.configs = n_ent;
  R.children = steps;
  R.p4 = 0;
  R.final_parent = TRACE_NONE;
  R.final_move = TRACE_NONE;
  R.deep_trace = TRACE_NONE;
  R.deep_len = 0;
  if (outcome == LIT_OK && moves) {
    // the linearization: the call events in the order the search took them
    // (clamped to the history's n_ops + 1 slot; a longer stack can only come
    // from a shared-return list and fails certification)
    uint32_t* out = moves + R.witness_off;
    const uint32_t nw = min(ncalls, D.moves_cap);
    for (uint32_t k = 0; k < nw; ++k) out[k] = (uint32_t)(w.calls[k].entry - 1);
    R.witness_len = nw;
    R.has_witness = 1;
  } else {
    R.witness_len = 0;
    R.has_witness = 0;
  }
}

}  // namespace

// Build the literal engine's event table for history i of the batch (its
// record hashes at pool_off in the batch pool).
void literal_prepare(const History& h, uint32_t i, uint64_t pool_off, std::vector<LitDesc>& descs,
                     std::vector<LitEv>& evs) {
  const uint32_t n_ev = (uint32_t)h.events.size();
  LitDesc d{};
  d.h = i;
  d.n_ev = n_ev;
  d.ev_off = (uint32_t)evs.size();
  d.W = std::max<uint32_t>(1, (n_ev / 2 + 63) / 64);
  d.moves_cap = h.n_ops + 1;
  descs.push_back(d);
  std::vector<uint32_t> op_of_call(n_ev, EV_INF);
  for (uint32_t k = 0; k < h.n_ops; ++k) op_of_call[h.op_call[k]] = k;
  for (uint32_t e = 0; e < n_ev; ++e) {
    LitEv x{};
    x.kind = (uint32_t)h.events[e].kind;
    x.id = h.lit_id[e];
    x.match = -1;
    if (x.kind == 0) {
      const int32_t m = h.lit_match[e];
      x.match = m >= 0 ? m + 1 : 0;  // node index of the matched return (0: none)
      if (m >= 0) {
        x.rec = h.rec_of(op_of_call[e]);
        x.rec.hash_off = (uint32_t)(x.rec.hash_off + pool_off);
      }
    }
    evs.push_back(x);
  }
}

int literal_run(DevBatch& b, hipStream_t stream, const RunOpts& ro, const unsigned long long* deadline,
                std::string& err) {
  const uint32_t n = (uint32_t)b.lit_desc.size();
  if (!n) return 0;
  if (!b.lit_dev_ready) {
    // One slice of device memory per history, from a fixed share of free HBM
    // (1/8, at least 64 MiB): that share over the histories, between 16 MiB
    // and 2 GiB each. When the histories need more slices than the share
    // holds (about 2,000 histories on an empty MI355X), they run in chunks
    // that reuse one buffer, so the literal engine never takes more than its
    // share from the other engines and never fails a batch for memory.
    size_t free_b = 0, total_b = 0;
    LITCHK(hipMemGetInfo(&free_b, &total_b));
    uint64_t share = std::max<uint64_t>(64ull << 20, free_b / 8);
    if (const char* e_ = getenv("S2LC_LITERAL_SHARE")) share = std::max<uint64_t>(16ull << 20, strtoull(e_, nullptr, 10));  // (tests)
    const uint64_t slice = std::max<uint64_t>(16ull << 20, std::min<uint64_t>(2ull << 30, share / n)) & ~255ull;
    b.lit_chunk = (uint32_t)std::max<uint64_t>(1, std::min<uint64_t>(n, share / slice));
    for (uint32_t k = 0; k < n; ++k) {
      b.lit_desc[k].mem_off = (uint64_t)(k % b.lit_chunk) * slice;
      b.lit_desc[k].mem_bytes = slice;
    }
    // (the events start 256-byte aligned: LitEv holds a 64-byte aligned OpRec)
    const size_t need_d = (n * sizeof(LitDesc) + 255) & ~(size_t)255,
                 need_e = std::max<size_t>(1, b.lit_ev.size()) * sizeof(LitEv);
    if (b.lit_bytes < need_d + need_e || !b.lit_meta) {
      if (b.lit_meta) (void)hipFree(b.lit_meta);
      b.lit_meta = nullptr;
      LITCHK(hipMalloc(&b.lit_meta, need_d + need_e));
      b.lit_bytes = need_d + need_e;
    }
    const uint64_t need_m = slice * b.lit_chunk;
    if (b.lit_mem_bytes < need_m || !b.lit_mem) {
      if (b.lit_mem) (void)hipFree(b.lit_mem);
      b.lit_mem = nullptr;
      LITCHK(hipMalloc(&b.lit_mem, need_m));
      b.lit_mem_bytes = need_m;
    }
    LITCHK(hipMemcpy(b.lit_meta, b.lit_desc.data(), n * sizeof(LitDesc), hipMemcpyHostToDevice));
    if (!b.lit_ev.empty()) LITCHK(hipMemcpy(b.lit_meta + need_d, b.lit_ev.data(), b.lit_ev.size() * sizeof(LitEv), hipMemcpyHostToDevice));
    b.lit_dev_ready = true;
  }
  const LitDesc* d = reinterpret_cast<const LitDesc*>(b.lit_meta);
  const LitEv* e = reinterpret_cast<const LitEv*>(b.lit_meta + ((n * sizeof(LitDesc) + 255) & ~(size_t)255));
  // loop iterations per history (S2LC_LITERAL_ITERS; a single GPU thread
  // runs ~1 M per second)
  unsigned long long iters = 1ull << 22;
  if (const char* ev_ = getenv("S2LC_LITERAL_ITERS")) iters = std::max<unsigned long long>(1, strtoull(ev_, nullptr, 10));
  // chunks of lit_chunk histories, one launch each, in stream order (each
  // chunk's slices are the previous chunk's)
  for (uint32_t c0 = 0; c0 < n; c0 += b.lit_chunk) {
    const uint32_t m = std::min(b.lit_chunk, n - c0);
    hipLaunchKernelGGL(literal_kernel, dim3((m + 63) / 64), dim3(64), 0, stream, d + c0, m, e, (const uint64_t*)b.pool,
                       b.lit_mem, b.res, ro.witness ? b.moves : nullptr, (unsigned long long)ro.max_configs, iters,
                       deadline);
    LITCHK(hipGetLastError());
  }
  return 0;
}

void literal_release(DevBatch& b) {
  if (b.lit_meta) (void)hipFree(b.lit_meta);
  if (b.lit_mem) (void)hipFree(b.lit_mem);
  b.lit_meta = nullptr;
  b.lit_mem = nullptr;
  b.lit_bytes = b.lit_mem_bytes = 0;
  b.lit_dev_ready = false;
}

}  // namespace s2lc
