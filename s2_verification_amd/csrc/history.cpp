// history.cpp — History::finalize: validation, porcupine renumbering, op
// classification and chain decomposition.
//
// Reference semantics:
//   renumber / makeLinkedEntries / checkSingle  porcupine v1.0.3 (upstream)
//   s2Model.Step                                main.go:264-335
#include <stdlib.h>

#include <algorithm>
#include <queue>

#include "history.h"
#include "s2lincheck.h"

namespace s2lc {

uint32_t History::intern(const std::string& s) {
  const size_t n = tokens.size();
  if (n < 32) {  // the collector's histories: a handful of tokens
    for (size_t i = 0; i < n; ++i)
      if (tokens[i] == s) return (uint32_t)(i + 1);
    tokens.push_back(s);
    return (uint32_t)tokens.size();
  }
  // many distinct tokens (one per append, say): a hash index instead of a
  // scan per token, which would make the decode quadratic
  if (tok_ix_n > n) {
    tok_ix.clear();
    tok_ix_n = 0;
  }
  for (; tok_ix_n < n; ++tok_ix_n) tok_ix.emplace(tokens[tok_ix_n], (uint32_t)(tok_ix_n + 1));  // (first id wins)
  const auto it = tok_ix.find(s);
  if (it != tok_ix.end()) return it->second;
  tokens.push_back(s);
  tok_ix.emplace(s, (uint32_t)tokens.size());
  tok_ix_n = tokens.size();
  return (uint32_t)tokens.size();
}

static uint32_t classify(const Event& in, const Event& out) {
  return op_flags(in.input_type, in.has_msn, out.failure, out.definite, out.has_tail, out.has_hash);
}

OpRec History::rec_of(uint32_t d) const {
  ensure_events();
  const Event& in = events[op_call[d]];
  const Event& out = events[op_ret[d]];
  OpRec r{};
  r.num_records = in.num_records;
  r.msn = in.msn;
  r.out_tail = out.tail;
  r.out_hash = out.stream_hash;
  r.sufmin = REQ_NONE;
  r.call_ev = op_call[d];
  r.ret_ev = op_ret[d];
  r.hash_off = (uint32_t)in.hash_off;
  r.hash_cnt = (uint32_t)in.hash_cnt;
  r.batch_tok = (uint16_t)in.batch_tok;
  r.set_tok = (uint16_t)in.set_tok;
  r.flags = classify(in, out);
  return r;
}

// finalize's working arrays: per decoder thread, reused from history to history
namespace {
struct FinalizeScratch {
  std::vector<uint32_t> dense, dir, val, ncall, nret, call, ret, chain_of, chain_len, last, fill;
  std::vector<int64_t> ids, key;
  std::vector<int32_t> reg;
};
thread_local FinalizeScratch fin_scratch;
}  // namespace

void finalize_scratch_trim() { fin_scratch = FinalizeScratch(); }

int History::finalize() {
  status = 0;
  error.clear();
  structural = 0;
  const size_t E = events.size();
  if (E >= (size_t)EV_INF) { status = S2LC_EUNSUPPORTED; error = "too many events"; return status; }

  FinalizeScratch& S = fin_scratch;
  // porcupine renumber(): ids -> 0..m-1 in order of first appearance
  // (an open-addressing map, no per-id nodes)
  std::vector<uint32_t>& dense = S.dense;
  std::vector<int64_t>& ids = S.ids;
  dense.resize(E);
  ids.clear();
  {
    size_t cap = 16;
    while (cap < 2 * E) cap <<= 1;
    std::vector<int64_t>& key = S.key;
    std::vector<uint32_t>& val = S.val;
    std::vector<uint32_t>& dir = S.dir;  // ids in [0, cap) (the collector's: 0, 1, 2, ...) index directly
    dir.assign(cap, EV_INF);
    bool hashed = false;
    const size_t mask = cap - 1;
    for (size_t i = 0; i < E; ++i) {
      const int64_t id = events[i].op_id;
      if ((uint64_t)id < (uint64_t)cap) {
        uint32_t& d = dir[(size_t)id];
        if (d == EV_INF) {
          d = (uint32_t)ids.size();
          ids.push_back(id);
        }
        dense[i] = d;
        continue;
      }
      if (!hashed) {
        key.resize(cap);
        val.assign(cap, EV_INF);
        hashed = true;
      }
      uint64_t x = (uint64_t)id * 0x9E3779B97F4A7C15ull;
      size_t s_ = (size_t)(x ^ (x >> 29)) & mask;
      while (val[s_] != EV_INF && key[s_] != id) s_ = (s_ + 1) & mask;
      if (val[s_] == EV_INF) {
        key[s_] = id;
        val[s_] = (uint32_t)ids.size();
        ids.push_back(id);
      }
      dense[i] = val[s_];
    }
  }
  const uint32_t m = (uint32_t)ids.size();
  std::vector<uint32_t>&ncall = S.ncall, &nret = S.nret, &call = S.call, &ret = S.ret;
  ncall.assign(m, 0);
  nret.assign(m, 0);
  call.assign(m, EV_INF);
  ret.assign(m, EV_INF);
  for (size_t i = 0; i < E; ++i) {
    const uint32_t d = dense[i];
    if (events[i].kind == 0) { ncall[d]++; call[d] = (uint32_t)i; }
    else { nret[d]++; ret[d] = (uint32_t)i; }
  }
  literal = false;
  lit_id.clear();
  lit_match.clear();
  for (uint32_t d = 0; d < m && !literal; ++d)
    if (ncall[d] > 1 || nret[d] > 1) literal = true;
  // Validate what the Go model would dereference (main.go:279, 313, 327).
  for (size_t i = 0; i < E; ++i) {
    const Event& e = events[i];
    if (e.kind == 0) {
      if (e.input_type > 2) { status = S2LC_EINVAL; error = "unknown input type"; return status; }
      if (e.input_type == S2LC_INPUT_APPEND && !e.has_num_records) {
        status = S2LC_EINVAL; error = "append without num_records"; return status;
      }
    } else if (!e.failure && !e.has_tail) {
      status = S2LC_EINVAL; error = "success output without tail"; return status;
    }
  }
  if (literal) {
    // porcupine makeLinkedEntries: walk the events backwards; a return
    // registers itself for its id, a call takes the registered return (the
    // nearest later one with its id; two calls may take the same return)
    lit_id.assign(dense.begin(), dense.end());
    lit_match.assign(E, -1);
    std::vector<int32_t>& reg = S.reg;
    reg.assign(m, -1);
    for (size_t i = E; i-- > 0;) {
      if (events[i].kind == 1) reg[dense[i]] = (int32_t)i;
      else lit_match[i] = reg[dense[i]];
    }
    recs.clear(); rec_op.clear(); chain_start.clear(); K = 0;
    n_ident = 0; hflags = 0; max_chain_len = 0;
    op_ids.clear(); op_call.clear(); op_ret.clear();
    for (size_t i = 0; i < E; ++i)
      if (events[i].kind == 0) {
        op_call.push_back((uint32_t)i);
        op_ret.push_back(lit_match[i] >= 0 ? (uint32_t)lit_match[i] : EV_INF);
        op_ids.push_back(events[i].op_id);
      }
    n_ops = (uint32_t)op_call.size();
    op_rec.assign(n_ops, EV_INF);
    if (tokens.size() > 0xFFFF) { status = S2LC_EUNSUPPORTED; error = "more than 65535 distinct fencing tokens"; }
    if (pool.size() > 0xFFFFFFFFull) { status = S2LC_EUNSUPPORTED; error = "more than 2^32 record hashes"; }
    return status;
  }
  for (uint32_t d = 0; d < m; ++d)
    if (ncall[d] != 1 || nret[d] != 1 || ret[d] < call[d]) structural = S2LC_R_UNMATCHED;

  n_ops = m;
  op_ids = ids;
  op_call = call;
  op_ret = ret;
  recs.clear(); rec_op.clear(); op_rec.assign(m, EV_INF); chain_start.clear(); K = 0;
  n_ident = 0; hflags = 0; max_chain_len = 0;
  if (structural) return 0;  // verdict fixed: checkSingle's list can never empty

  // Well formed: each id's first event is its call, so dense order == call order.
  // Overflow-free tail bound (enables the P1 prune).
  uint64_t total = 0;
  bool nowrap = true, zero_with_hashes = false;
  for (uint32_t d = 0; d < m; ++d) {
    const Event& in = events[call[d]];
    if (in.input_type != S2LC_INPUT_APPEND) continue;
    if (in.num_records > (1ull << 63) - total) nowrap = false;
    else total += in.num_records;
    if (in.num_records == 0 && in.hash_cnt > 0) zero_with_hashes = true;
  }
  hflags |= H_P4 | H_IDEFER;
  if (nowrap) hflags |= H_NOWRAP;
  if (nowrap && !zero_with_hashes) hflags |= H_P2OK;
  if (nowrap && total <= 0xFFFFFFFCull) hflags |= H_TAIL32;

  // Greedy interval colouring (ops by call order; reuse the chain that
  // finished earliest if it finished before this call): K = max overlap.
  std::vector<uint32_t>&chain_of = S.chain_of, &chain_len = S.chain_len;
  chain_of.resize(m);
  chain_len.clear();
  {
    // the chain with the smallest (last ret, index) that ended before the call
    std::vector<uint32_t>& last = S.last;  // last ret of each chain
    last.clear();
    using P = std::pair<uint32_t, uint32_t>;  // (last ret, chain), for wide histories
    std::priority_queue<P, std::vector<P>, std::greater<P>> heap;
    bool use_heap = false;
    for (uint32_t d = 0; d < m; ++d) {
      uint32_t c = EV_INF;
      if (!use_heap) {
        uint32_t best = EV_INF;
        for (uint32_t k = 0; k < (uint32_t)last.size(); ++k)
          if (last[k] < best) { best = last[k]; c = k; }
        if (best >= call[d]) c = EV_INF;
      } else if (!heap.empty() && heap.top().first < call[d]) {
        c = heap.top().second;
        heap.pop();
      }
      if (c == EV_INF) {
        c = (uint32_t)chain_len.size();
        chain_len.push_back(0);
        last.push_back(0);
      }
      chain_of[d] = c;
      chain_len[c]++;
      last[c] = ret[d];
      if (use_heap) heap.push({ret[d], c});
      if (!use_heap && last.size() > 32) {  // many chains: switch to the heap (same choices)
        use_heap = true;
        for (uint32_t k = 0; k < (uint32_t)last.size(); ++k) heap.push({last[k], k});
      }
    }
  }
  K = (uint32_t)chain_len.size();
  chain_start.resize(K + 1);
  uint32_t pos = 0;
  for (uint32_t c = 0; c < K; ++c) {
    chain_start[c] = pos;
    pos += chain_len[c] + 1;
    max_chain_len = std::max<uint32_t>(max_chain_len, chain_len[c]);
  }
  chain_start[K] = pos;
  rec_op.assign(pos, EV_INF);
  {
    std::vector<uint32_t>& fill = S.fill;  // next slot of each chain
    fill.assign(chain_start.begin(), chain_start.end() - 1);
    for (uint32_t d = 0; d < m; ++d) {  // call order within every chain
      const uint32_t p = fill[chain_of[d]]++;
      rec_op[p] = d;
      op_rec[d] = p;
    }
  }
  // the records in position order, each written once (assign() would zero
  // them first); a sentinel is completed below
  recs.clear();
  recs.reserve(pos);
  for (uint32_t p = 0; p < pos; ++p) {
    const uint32_t d = rec_op[p];
    if (d == EV_INF) {
      recs.push_back(OpRec{});
      continue;
    }
    recs.push_back(rec_of(d));
    if (recs.back().flags & OPF_CLS_E) n_ident++;
  }
  for (uint32_t c = 0; c < K; ++c) {
    const uint32_t p = chain_start[c + 1] - 1;
    OpRec& s = recs[p];  // sentinel
    s.call_ev = EV_INF;
    s.ret_ev = EV_INF;
    s.flags = OPF_SENTINEL;
    s.sufmin = REQ_NONE;
    // suffix minimum of the pre-tail each constraining op requires
    uint64_t run = REQ_NONE;
    for (uint32_t q = p; q-- > chain_start[c];) {
      OpRec& r = recs[q];
      if (r.flags & OPF_CONSTRAIN) {
        uint64_t req;
        if ((r.flags & OPF_KIND_MASK) == S2LC_INPUT_APPEND)
          req = r.out_tail >= r.num_records ? r.out_tail - r.num_records : 0;  // 0: unsatisfiable
        else if (!(r.flags & OPF_FAIL))
          req = r.out_tail;
        else
          req = REQ_HASH_ONLY;
        if (req > REQ_HASH_ONLY) req = REQ_HASH_ONLY;
        run = std::min(run, req);
      }
      r.sufmin = run;
    }
  }
  if (tokens.size() > 0xFFFF) { status = S2LC_EUNSUPPORTED; error = "more than 65535 distinct fencing tokens"; }
  if (pool.size() > 0xFFFFFFFFull) { status = S2LC_EUNSUPPORTED; error = "more than 2^32 record hashes"; }
  return status;
}

// ------------------------------------------------------------- recycling ---
template <class V>
static size_t used(const V& v) {
  return v.size() * sizeof(typename V::value_type);
}

template <class V>
static size_t cap(const V& v) {
  return v.capacity() * sizeof(typename V::value_type);
}

size_t History::capacity_bytes() const {
  size_t b = cap(events) + cap(pool) + cap(op_call) + cap(op_ret) + cap(op_ids) + cap(chain_start) + cap(recs) +
             cap(rec_op) + cap(op_rec) + cap(lit_id) + cap(lit_match) + cap(lazy_client) + cap(tokens);
  for (const std::string& t : tokens) b += t.capacity();
  return b;
}

size_t History::used_bytes() const {
  return used(events) + used(pool) + used(op_call) + used(op_ret) + used(op_ids) + used(chain_start) + used(recs) +
         used(rec_op) + used(op_rec) + used(lit_id) + used(lit_match) + used(lazy_client) + used(tokens);
}

void History::recycle() {
  History f;  // every scalar and member back to its default ...
  auto keep = [](auto& dst, auto& src) {  // ... and every array to empty with its capacity
    src.clear();
    dst.swap(src);
  };
  keep(f.events, events);
  keep(f.pool, pool);
  keep(f.op_call, op_call);
  keep(f.op_ret, op_ret);
  keep(f.op_ids, op_ids);
  keep(f.chain_start, chain_start);
  keep(f.recs, recs);
  keep(f.rec_op, rec_op);
  keep(f.op_rec, op_rec);
  keep(f.lit_id, lit_id);
  keep(f.lit_match, lit_match);
  keep(f.lazy_client, lazy_client);
  *this = std::move(f);
  pooled_bytes = 0;
}

namespace {
struct HistoryPool {
  std::mutex mu;
  std::vector<s2lc_history*> free;
  size_t bytes = 0;
  size_t budget;
  HistoryPool() {
    const char* e = getenv("S2LC_HISTORY_POOL_MB");
    budget = (size_t)(e && *e ? strtoull(e, nullptr, 10) : 2048ull) << 20;
  }
};
// never destroyed: a history freed by another static destructor at exit must
// still find it
HistoryPool& hpool() {
  static HistoryPool* p = new HistoryPool();
  return *p;
}
}  // namespace

s2lc_history* history_acquire() {
  HistoryPool& P = hpool();
  {
    std::lock_guard<std::mutex> g(P.mu);
    if (!P.free.empty()) {
      s2lc_history* h = P.free.back();
      P.free.pop_back();
      P.bytes -= h->h.pooled_bytes;
      return h;
    }
  }
  return new s2lc_history();
}

void history_acquire_many(size_t n, s2lc_history** out) {
  HistoryPool& P = hpool();
  size_t k = 0;
  {
    std::lock_guard<std::mutex> g(P.mu);
    for (; k < n && !P.free.empty(); ++k) {
      out[k] = P.free.back();
      P.free.pop_back();
      P.bytes -= out[k]->h.pooled_bytes;
    }
  }
  try {
    for (; k < n; ++k) out[k] = new s2lc_history();
  } catch (...) {
    for (size_t i = 0; i < k; ++i) history_release(out[i]);
    throw;
  }
}

void history_release(s2lc_history* h) {
  if (!h) return;
  HistoryPool& P = hpool();
  // (accounted by capacity: an upper bound on what the parked arrays keep resident)
  if (P.budget) {
    h->h.recycle();  // outside the lock: frees the token strings, keeps the arrays
    const size_t b = h->h.capacity_bytes();
    if (b > P.budget) {
      delete h;
      return;
    }
    h->h.pooled_bytes = b;
    std::lock_guard<std::mutex> g(P.mu);
    if (P.bytes + b <= P.budget) {
      P.free.push_back(h);
      P.bytes += b;
      return;
    }
  }
  delete h;
}

size_t history_pool_trim() {
  HistoryPool& P = hpool();
  std::vector<s2lc_history*> v;
  {
    std::lock_guard<std::mutex> g(P.mu);
    v.swap(P.free);
    P.bytes = 0;
  }
  size_t b = 0;
  for (s2lc_history* h : v) {
    b += h->h.pooled_bytes;
    delete h;
  }
  load_scratch_trim();
  finalize_scratch_trim();
  return b;
}

}  // namespace s2lc
