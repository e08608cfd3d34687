// witness.cpp — host-side witness reconstruction and CPU-model replay.
//
// The device records, per round, the move (chain, outcome) that produced each
// surviving configuration. For an Ok verdict the move list is expanded here
// into a full linearization (identity ops re-derived by the same closure) and
// then replayed through the CPU model with porcupine's powerset semantics
// (NondeterministicModel.ToModel, main.go:253-361) plus a real-time check:
// every GPU witness must replay cleanly (BASELINE.json north_star).
#include <algorithm>
#include <vector>

#include "search.h"

namespace s2lc {

namespace {

// The outcome a linearization claims for op r at state s is one of
// s2Model.Step(s, r)'s successors (main.go:264-335): `applied` = the
// optimistic post-append state, else the unchanged state. Exactly s2_step's
// membership test, with the record hashes folded at most once.
bool claim_ok(const OpRec& r, const State& s, const uint64_t* pool, bool applied, State& next) {
  const uint32_t kind = r.flags & OPF_KIND_MASK;
  if (kind != 0) {  // read / check-tail: identity or reject
    next = s;
    return !applied && ident_legal(r, s);
  }
  const bool fail = r.flags & OPF_FAIL;
  if (fail && (r.flags & OPF_DEF)) { next = s; return !applied; }  // definite failure: {s}
  const bool ok = append_guards_ok(r, s);
  if (fail) {  // indefinite: {s} when the guards fail, else {opt, s}
    if (!applied) { next = s; return true; }
    if (!ok) return false;
    next = append_opt(r, s, pool);
    return true;
  }
  if (!ok) return false;  // success: {opt} when the guards pass and the tail matches, else {}
  const State opt = append_opt(r, s, pool);
  if (opt.tail != r.out_tail) return false;
  if (!applied && !state_eq(opt, s)) return false;
  next = opt;
  return true;
}

// One step of the certifying replay (replay_states): order's next op, with the
// outcome the linearization claims, from the replay's own state.
inline bool replay_step(const History& h, uint32_t op, uint8_t ident, State& s) {
  const OpRec& r = h.recs[h.op_rec[op]];
  // the outcome this linearization claims: the optimistic successor for an
  // append taken as applied, the unchanged state otherwise
  const bool applied = !ident && !(r.flags & OPF_CLS_E) && (r.flags & OPF_KIND_MASK) == 0;
  State next;
  if (!claim_ok(r, s, h.pool.data(), applied, next)) return false;
  s = next;
  return true;
}

void prefetch_range(const void* p, size_t bytes) {
  const char* c = static_cast<const char*>(p);
  for (size_t o = 0; o < bytes; o += 64) __builtin_prefetch(c + o, 0, 3);
}

// Per-thread scratch of the rebuild (no allocation per history once warm).
struct Head {  // a chain's head, as the closure tests it
  uint32_t call, ret;
  uint32_t need;  // bit 0: identity class; bit 1: tail must match; bit 2: hash must match
  uint32_t _pad;
  uint64_t tail, hash;
  const OpRec* rec;
};
struct Scratch {
  std::vector<Head> head;
  std::vector<uint8_t> seen;
};
thread_local Scratch t_scr;

// The device's closure and moves over one history, host side. The heads are
// kept as a small array of what the closure tests (call, return, and the
// observation an identity op must match), so a closure pass is a short loop
// with no record loads; a chain's next head is its next record. The
// linearization is written by index into buffers sized n_ops.
struct Rebuild {
  const History& h;
  const OpRec* recs;
  Head* hd;
  const uint32_t K;
  uint32_t* order;
  uint8_t* ident;
  uint32_t n = 0;  // ops written
  State s{0, 0, 0};
  // the certifying replay run alongside (rebuild_and_replay): its own state,
  // stepped through each op as the rebuild writes it, so the two folds of the
  // record hashes (the rebuild's and the replay's) are independent dependency
  // chains in flight together instead of two passes
  bool rep = false, rep_ok = true;
  State rs{0, 0, 0};
  Rebuild(const History& h_, Head* hd_, uint32_t* ord, uint8_t* id)
      : h(h_), recs(h_.recs.data()), hd(hd_), K(h_.K), order(ord), ident(id) {
    for (uint32_t q = 0; q < K; ++q) load(q, recs + h.chain_start[q]);
  }
  void load(uint32_t q, const OpRec* r) {
    Head& x = hd[q];
    x.rec = r;
    x.call = r->call_ev;
    x.ret = r->ret_ev;
    const uint32_t f = r->flags;
    uint32_t need = 0;
    if (f & OPF_CLS_E) {
      need = 1;
      if ((f & OPF_KIND_MASK) != 0) {  // read / check-tail (ident_legal)
        if (!(f & OPF_FAIL)) need |= 2;
        if (f & OPF_HAS_HASH) need |= 4;
      }
    }
    x.need = need;
    x.tail = r->out_tail;
    x.hash = r->out_hash;
  }
  uint32_t min_ret() const {
    uint32_t m = EV_INF;
    for (uint32_t q = 0; q < K; ++q) m = std::min(m, hd[q].ret);
    return m;
  }
  bool eligible(const Head& x, uint32_t mr) const {
    return (x.need & 1) && x.call < mr && (!(x.need & 2) || x.tail == s.tail) && (!(x.need & 4) || x.hash == s.hash);
  }
  void take(uint32_t q, uint8_t id) {
    const OpRec* r = hd[q].rec;
    order[n] = h.rec_op[(size_t)(r - recs)];
    ident[n] = id;
    if (rep && rep_ok) rep_ok = replay_step(h, order[n], id, rs);
    ++n;
    load(q, r + 1);
  }
  // legal minimal identity ops, to the fixpoint (search.hip's closure)
  void close() {
    for (;;) {
      const uint32_t mr = min_ret();
      if (mr == EV_INF) return;
      bool changed = false;
      for (uint32_t q = 0; q < K; ++q)
        while (eligible(hd[q], mr)) {
          take(q, 1);
          changed = true;
        }
      if (!changed) return;
    }
  }
};

}  // namespace

static bool rebuild(const History& h, const uint32_t* moves, uint32_t n_moves, bool p4, std::vector<uint32_t>& order,
                    std::vector<uint8_t>& ident, bool partial, bool replay) {
  order.clear();
  ident.clear();
  if (h.structural) return false;
  // The history's records are read chain by chain (K interleaved streams),
  // and in a batch they are cold (last touched by the upload): stream them
  // (and the record-hash pool and record -> op map) into the cache first, with
  // all misses in flight at once, instead of one miss per closure step.
  prefetch_range(h.recs.data(), h.recs.size() * sizeof(OpRec));
  prefetch_range(h.rec_op.data(), h.rec_op.size() * sizeof(uint32_t));
  prefetch_range(h.pool.data(), h.pool.size() * sizeof(uint64_t));
  order.resize(h.n_ops);
  ident.resize(h.n_ops);
  t_scr.head.resize(h.K);
  Rebuild c(h, t_scr.head.data(), order.data(), ident.data());
  c.rep = replay;
  c.close();
  for (uint32_t m = 0; m < n_moves; ++m) {
    const uint32_t j = moves[m] & 0xFFFFu;
    const bool is_id = moves[m] & MOVE_IDENT;
    if (j >= h.K || c.n >= h.n_ops) { order.resize(c.n); ident.resize(c.n); return false; }
    const OpRec& r = *c.hd[j].rec;
    State next;
    if ((r.flags & (OPF_SENTINEL | OPF_CLS_E)) || r.call_ev >= c.min_ret() ||  // a minimal non-identity op
        !claim_ok(r, c.s, h.pool.data(), !is_id, next)) {
      order.resize(c.n);
      ident.resize(c.n);
      return false;
    }
    c.s = next;
    c.take(j, is_id ? 1 : 0);
    c.close();
  }
  order.resize(c.n);
  ident.resize(c.n);
  if (partial) return true;
  if (order.size() != h.n_ops) {
    if (!p4) return false;
    // P4 completion: nothing left constrains the state; finish in return order.
    std::vector<uint32_t> rest;
    for (uint32_t q = 0; q < h.K; ++q)
      for (const OpRec* x = c.hd[q].rec; !(x->flags & OPF_SENTINEL); ++x) rest.push_back(h.rec_op[(size_t)(x - c.recs)]);
    std::sort(rest.begin(), rest.end(), [&](uint32_t a, uint32_t b) { return h.op_ret[a] < h.op_ret[b]; });
    order.insert(order.end(), rest.begin(), rest.end());
    ident.resize(order.size(), 1);
    if (replay)
      for (uint32_t op : rest)
        if (c.rep_ok) c.rep_ok = replay_step(h, op, 1, c.rs);
  }
  return order.size() == h.n_ops && (!replay || c.rep_ok);
}

bool rebuild_linearization(const History& h, const uint32_t* moves, uint32_t n_moves, bool p4,
                           std::vector<uint32_t>& order, std::vector<uint8_t>& ident, bool partial) {
  return rebuild(h, moves, n_moves, p4, order, ident, partial, false);
}

bool rebuild_and_replay(const History& h, const uint32_t* moves, uint32_t n_moves, bool p4,
                        std::vector<uint32_t>& order, std::vector<uint8_t>& ident) {
  return rebuild(h, moves, n_moves, p4, order, ident, false, true) &&
         real_time_ok(h, order.data(), order.size());
}

// (The op's record is recs[op_rec[d]]: History::finalize builds it with
// rec_of(d) from the op's call and return events (history.cpp), and the
// rebuild has just read it, so the replay runs from cache.)
static bool replay_states(const History& h, const uint32_t* order, const uint8_t* ident, size_t n) {
  State s{0, 0, 0};
  for (size_t i = 0; i < n; ++i)
    if (!replay_step(h, order[i], ident[i], s)) return false;
  return true;
}

bool replay_path(const History& h, const uint32_t* order, const uint8_t* ident, size_t n) {
  return real_time_ok(h, order, n) && replay_states(h, order, ident, n);
}

bool replay_prefix(const History& h, const uint32_t* order, const uint8_t* ident, size_t n) {
  if (h.structural || n > h.n_ops) return false;
  std::vector<uint8_t> in(h.n_ops, 0);
  uint32_t max_call = 0;
  for (size_t i = 0; i < n; ++i) {
    if (order[i] >= h.n_ops || in[order[i]]) return false;
    in[order[i]] = 1;
    max_call = std::max(max_call, h.op_call[order[i]]);
  }
  // closed under real-time predecessors: nothing outside returned before an op inside was called
  for (uint32_t d = 0; d < h.n_ops; ++d)
    if (!in[d] && h.op_ret[d] < max_call) return false;
  uint32_t later_min_ret = EV_INF;
  for (size_t i = n; i-- > 0;) {
    if (h.op_call[order[i]] >= later_min_ret) return false;
    later_min_ret = std::min(later_min_ret, h.op_ret[order[i]]);
  }
  return replay_states(h, order, ident, n);
}

bool real_time_ok(const History& h, const uint32_t* order, size_t n) {
  if (h.structural || n != h.n_ops) return false;
  std::vector<uint8_t>& seen = t_scr.seen;
  seen.assign(h.n_ops, 0);
  for (size_t i = 0; i < n; ++i) {
    if (order[i] >= h.n_ops || seen[order[i]]) return false;
    seen[order[i]] = 1;
  }
  // real time: call(order[i]) < ret(order[k]) for all k > i
  uint32_t later_min_ret = EV_INF;
  for (size_t i = n; i-- > 0;) {
    if (h.op_call[order[i]] >= later_min_ret) return false;
    later_min_ret = std::min(later_min_ret, h.op_ret[order[i]]);
  }
  return true;
}

bool replay_order(const History& h, const uint32_t* order, size_t n) {
  if (!real_time_ok(h, order, n)) return false;
  // powerset replay (ToModel().Step + merge)
  std::vector<State> set{State{0, 0, 0}}, next;
  for (size_t i = 0; i < n; ++i) {
    const OpRec r = h.rec_of(order[i]);
    next.clear();
    for (const State& s : set) {
      State kids[2];
      const int nk = s2_step(r, s, h.pool.data(), kids);
      for (int k = 0; k < nk; ++k) {
        bool dup = false;
        for (const State& x : next) if (state_eq(x, kids[k])) { dup = true; break; }
        if (!dup) next.push_back(kids[k]);
      }
    }
    if (next.empty()) return false;
    if (next.size() > (1u << 16)) return false;
    set.swap(next);
  }
  return true;
}

// Duplicate-id histories (History::literal): the literal engine's order is
// porcupine's own calls stack, a sequence of (call, matched return) ops that
// its DFS stepped through ToModel().Step; certify it by replaying those steps
// through the CPU model, the powerset state never empty. (Real-time order is
// porcupine's list discipline there: two calls may share one return.)
bool replay_literal(const History& h, const uint32_t* order, size_t n) {
  if (!h.literal || n != h.n_ops) return false;
  std::vector<uint8_t> seen(h.n_ops, 0);
  std::vector<State> set{State{0, 0, 0}}, next;
  for (size_t i = 0; i < n; ++i) {
    const uint32_t d = order[i];
    if (d >= h.n_ops || seen[d] || h.op_ret[d] == EV_INF) return false;
    seen[d] = 1;
    const OpRec r = h.rec_of(d);
    next.clear();
    for (const State& s : set) {
      State kids[2];
      const int nk = s2_step(r, s, h.pool.data(), kids);
      for (int k = 0; k < nk; ++k) {
        bool dup = false;
        for (const State& x : next) if (state_eq(x, kids[k])) { dup = true; break; }
        if (!dup) next.push_back(kids[k]);
      }
    }
    if (next.empty() || next.size() > (1u << 20)) return false;
    set.swap(next);
  }
  return true;
}

}  // namespace s2lc
