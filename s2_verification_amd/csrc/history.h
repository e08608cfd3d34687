// history.h — host-side history representation (C++).
//
// A History holds the porcupine event list (main.go:529-563 output) and the
// derived search layout: dense op ids (porcupine renumber: first appearance),
// greedy interval-colouring chains, and the chain-major OpRec table that the
// gfx950 kernels read.
#pragma once
#include <stdint.h>

#include <memory>
#include <mutex>
#include <string>
#include <unordered_map>
#include <vector>

#include "model.h"

namespace s2lc {

struct Event {  // (80 bytes: the 8-byte fields first, no padding holes)
  int64_t op_id = 0;
  int64_t client_id = 0;
  uint64_t num_records = 0, msn = 0;
  uint64_t hash_off = 0, hash_cnt = 0;  // into History::pool
  uint64_t tail = 0, stream_hash = 0;
  uint32_t set_tok = 0, batch_tok = 0;  // interned ids, 0 = nil
  uint8_t kind = 0;                     // 0 call, 1 return
  uint8_t input_type = 0, has_num_records = 0, has_msn = 0;
  uint8_t failure = 0, definite = 0, has_tail = 0, has_hash = 0;
};
static_assert(sizeof(Event) == 80, "Event layout");

// Per-history search flags (HistDesc.flags). Each gates one verdict-exact
// reduction; batch_upload clears the ones a context disables
// (s2lc_opts.reductions_off) for ablation tests.
enum : uint16_t {
  H_NOWRAP = 0x1,  // P1: sum of all num_records <= 2^63: tails never wrap, tail-bound prune valid
  H_P2OK = 0x2,    // P2: NOWRAP and no 0-record append carries hashes: equal tail => equal hash needed
  H_P4 = 0x4,      // P4: no pending observer left => complete
  H_IDEFER = 0x8,  // indefinite append's identity outcome only when it holds minret
  H_TAIL32 = 0x10, // sum of all num_records < 2^32 - 3: every reachable tail fits 32 bits (packed kernels)
};

struct History {
  // ---- porcupine events ----
  // (a history loaded from the binary cache builds this list on first use:
  // the check reads only the records; use n_events() / ensure_events())
  mutable std::vector<Event> events;
  std::vector<uint64_t> pool;         // record hashes
  std::vector<std::string> tokens;    // token id i+1 -> string
  // token -> id index for histories with many distinct tokens (intern():
  // a scan below 32 tokens); it covers tokens[0, tok_ix_n) and is rebuilt
  // when tokens shrank (a cache load refills them)
  std::unordered_map<std::string, uint32_t> tok_ix;
  size_t tok_ix_n = 0;

  uint32_t intern(const std::string& s);

  // ---- derived by finalize() ----
  int status = 0;                     // 0 ok, else s2lc_status (EINVAL / EUNSUPPORTED)
  std::string error;
  int structural = 0;                 // 0 or S2LC_R_UNMATCHED
  uint32_t n_ops = 0;
  uint32_t n_ident = 0;
  std::vector<uint32_t> op_call, op_ret;   // event index per dense op id
  std::vector<int64_t> op_ids;            // original Event.Id per dense op id
  uint32_t K = 0;                          // chains
  std::vector<uint32_t> chain_start;       // K+1 record positions (sentinels included)
  std::vector<OpRec> recs;                 // chain-major, hash_off relative to pool
  std::vector<uint32_t> rec_op;            // record position -> dense op id (UINT32_MAX = sentinel)
  std::vector<uint32_t> op_rec;            // dense op id -> record position
  uint16_t hflags = 0;
  uint32_t max_chain_len = 0;
  // Duplicate op ids (more than one Start or Finish per op_id): porcupine's
  // checkSingle is run literally (literal.hip), on its own linked entry list.
  // Ops are then the call events in order (op_call), op_ret their porcupine
  // match (makeLinkedEntries: the nearest later return with the same id;
  // EV_INF when none), op_ids their Event.Id; there are no chains.
  bool literal = false;
  std::vector<int32_t> lit_id;     // per event: porcupine's dense id (renumber)
  std::vector<int32_t> lit_match;  // per event: a call's matched return event (-1: none / a return)

  // Validate, renumber, classify, decompose into chains. Idempotent.
  int finalize();
  // OpRec of dense op d built from its call/return events (sufmin unset).
  OpRec rec_of(uint32_t d) const;

  // ---- binary cache (cache.cpp) ----
  std::vector<int64_t> lazy_client;          // per event client id while `events` is not built
  std::unique_ptr<std::once_flag> lazy_once;  // builds `events` once (thread-safe)
  size_t n_events() const { return lazy_once ? lazy_client.size() : events.size(); }
  void ensure_events() const;                 // no-op unless loaded from the cache

  // ---- recycling (history_acquire / history_release) ----
  // Back to the freshly constructed state, keeping every array's capacity.
  void recycle();
  size_t used_bytes() const;
  size_t capacity_bytes() const;  // what its arrays hold allocated (the pool's accounting)
  size_t pooled_bytes = 0;        // capacity_bytes() when it was parked
};

// OpRec flags of an op from its call's and return's fields (History::rec_of
// and the direct JSONL decoder; s2Model.Step's cases, main.go:264-335).
inline uint32_t op_flags(uint8_t input_type, bool has_msn, bool failure, bool definite, bool has_tail, bool has_hash) {
  uint32_t f = input_type & OPF_KIND_MASK;
  if (failure) f |= OPF_FAIL;
  if (definite) f |= OPF_DEF;
  if (has_tail) f |= OPF_HAS_TAIL;
  if (has_hash) f |= OPF_HAS_HASH;
  if (has_msn) f |= OPF_HAS_MSN;
  if (input_type == 0) {  // S2LC_INPUT_APPEND
    if (failure && definite) f |= OPF_CLS_E;  // main.go:283-285: {s}
    else if (failure) f |= OPF_CLS_I;         // main.go:286-300: {s} or {opt, s}
    else f |= OPF_CLS_D | OPF_CONSTRAIN;      // main.go:301-318: {} or {opt}
  } else {
    f |= OPF_CLS_E;                           // main.go:320-331: {} or {s}
    if (!failure || has_hash) f |= OPF_CONSTRAIN;
  }
  return f;
}

// JSONL loader (eventsFromReader, main.go:529-563). Returns 0 or S2LC_EDECODE.
int load_jsonl(const uint8_t* buf, size_t len, History& h, std::string& err);
// load_jsonl + History::finalize. A history entirely in the collector's form
// (each record as serde writes it, op ids 0, 1, 2, ... in call order, every op
// returned once) is decoded straight into the finalized form: records, chains
// and op tables, with the event list built on first use (as a cache load
// leaves it). Anything else goes through load_jsonl and finalize, which also
// own every error message. Returns 0 or the status; the message in err.
int load_jsonl_finalized(const uint8_t* buf, size_t len, History& h, std::string& err);

// Deterministic simulator (collector workload, history.rs + collect-history.rs).
struct SimParams;
}  // namespace s2lc

// The opaque C-ABI handle (include/s2lincheck.h) is a History.
struct s2lc_history {
  s2lc::History h;
};

namespace s2lc {
// Decoders take their History from a process-wide pool of released ones, and
// s2lc_history_free parks a history there (cleared, capacity kept) instead of
// returning its arrays to the C heap. A long-running checker decodes batch N+1
// into batch N's storage: no page faults, no heap growth or trim, no
// address-space lock shared by the decoder threads. The pool is
// bounded by S2LC_HISTORY_POOL_MB of array capacity (default 2048; 0 = off);
// s2lc_history_pool_trim empties it.
s2lc_history* history_acquire();
// n histories under one lock (the parallel loaders take theirs up front)
void history_acquire_many(size_t n, s2lc_history** out);
void history_release(s2lc_history* h);
size_t history_pool_trim();
// this thread's decode / finalize scratch (jsonl.cpp, history.cpp) back to the heap
void load_scratch_trim();
void finalize_scratch_trim();
}  // namespace s2lc
