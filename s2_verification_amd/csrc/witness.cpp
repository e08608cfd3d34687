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
#include "cert_prof.h"

static_assert(s2lc::OPF_CLS_E == 0x100u && s2lc::OPF_FAIL == 0x4u && s2lc::OPF_HAS_HASH == 0x20u,
              "witness.cpp's head bits");

namespace s2lc {

#ifdef S2LC_CERT_PROF
std::atomic<uint64_t> g_cert_prof[16];
#endif

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
  const uint32_t f = r.flags;
  if (f & OPF_CLS_E) {
    // Step(s) is {s} or {} (main.go:283-285, 320-331): ident_legal, without a
    // branch per field (the closure takes these ops in data-dependent kinds)
    const int any = (f & OPF_KIND_MASK) == 0;  // definite append failure
    const int hash_ok = !(f & OPF_HAS_HASH) | (s.hash == r.out_hash);
    const int tail_ok = ((f & OPF_FAIL) != 0) | (s.tail == r.out_tail);
    return any | (hash_ok & tail_ok);
  }
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
// The chains' heads as the closure tests them, one array per field: a pass's
// min-return and its "called before mr" test are straight loops over K
// entries, and only the heads that pass the second get the observation test.
struct Heads {
  std::vector<uint32_t> ccall;  // call event of an identity-class head, EV_INF otherwise (never closure-taken)
  std::vector<uint32_t> ret;
  std::vector<uint32_t> need;   // bit 1: tail must match; bit 2: hash must match
  std::vector<uint64_t> tail, hash;
  std::vector<const OpRec*> rec;
  void resize(uint32_t K) {
    ccall.resize(K);
    ret.resize(K);
    need.resize(K);
    tail.resize(K);
    hash.resize(K);
    rec.resize(K);
  }
};
struct Scratch {
  Heads head;
  std::vector<uint8_t> seen;
};
thread_local Scratch t_scr;

// The device's closure and moves over one history, host side. The heads are
// kept as what the closure tests (call, return, and the observation an
// identity op must match), so a closure pass is a few loops with no record
// loads; a chain's next head is its next record. The linearization is written
// by index into buffers sized n_ops.
struct Rebuild {
  const History& h;
  const OpRec* recs;
  Heads& hd;
  uint32_t* const ccall;
  uint32_t* const ret;
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
  Rebuild(const History& h_, Heads& hd_, uint32_t* ord, uint8_t* id)
      : h(h_), recs(h_.recs.data()), hd(hd_), ccall(hd_.ccall.data()), ret(hd_.ret.data()), K(h_.K), order(ord),
        ident(id) {
    for (uint32_t q = 0; q < K; ++q) load(q, recs + h.chain_start[q]);
  }
  void load(uint32_t q, const OpRec* r) {
    hd.rec[q] = r;
    ret[q] = r->ret_ev;
    const uint32_t f = r->flags;
    // read / check-tail (ident_legal): bit 1 unless failed, bit 2 if it carries
    // a hash; none for an append (bit arithmetic: the kinds come in data order)
    const uint32_t ce = (f >> 8) & 1u;                          // OPF_CLS_E
    const uint32_t rd = ce & (uint32_t)((f & OPF_KIND_MASK) != 0);
    const uint32_t need = rd * ((((f >> 2) & 1u) ^ 1u) << 1 | ((f >> 5) & 1u) << 2);  // OPF_FAIL, OPF_HAS_HASH
    ccall[q] = ce ? r->call_ev : EV_INF;
    hd.need[q] = need;
    hd.tail[q] = r->out_tail;
    hd.hash[q] = r->out_hash;
  }
  uint32_t min_ret() const {
    uint32_t m = EV_INF;
    for (uint32_t q = 0; q < K; ++q) m = ret[q] < m ? ret[q] : m;
    return m;
  }
  // head q (called before mr) observes the current state
  bool obs_ok(uint32_t q) const {
    const uint32_t nd = hd.need[q];
    const int tail_ok = !(nd & 2) | (hd.tail[q] == s.tail), hash_ok = !(nd & 4) | (hd.hash[q] == s.hash);
    return tail_ok & hash_ok;
  }
  void take(uint32_t q, uint8_t id) {
    const OpRec* r = hd.rec[q];
    order[n] = h.rec_op[(size_t)(r - recs)];
    ident[n] = id;
    if (rep && rep_ok) rep_ok = replay_step(h, order[n], id, rs);
    ++n;
    load(q, r + 1);
  }
  // record x (a chain's next head) is an identity op called before mr that
  // observes the state: the test obs_ok makes on a loaded head
  bool ident_ok(const OpRec& x, uint32_t mr) const {
    const uint32_t f = x.flags;
    const int ce = (f & OPF_CLS_E) != 0, before = x.call_ev < mr, rd = (f & OPF_KIND_MASK) != 0;
    const int tail_ok = !rd | ((f & OPF_FAIL) != 0) | (x.out_tail == s.tail);
    const int hash_ok = !rd | ((f & OPF_HAS_HASH) == 0) | (x.out_hash == s.hash);
    return ce & before & tail_ok & hash_ok;
  }
  // the run of chain q's identity ops a pass takes, read straight from the
  // chain's consecutive records, then the head loaded once (a sentinel ends
  // every run: it is not identity-class)
  bool take_run(uint32_t q, uint32_t mr) {
    if (!((ccall[q] < mr) & obs_ok(q))) return false;
    const OpRec* r = hd.rec[q];
    const uint32_t* ro = h.rec_op.data() + (size_t)(r - recs);
    size_t k = 0;
    do {
      const uint32_t op = ro[k];
      order[n] = op;
      ident[n] = 1;
      if (rep) rep_ok &= replay_step(h, op, 1, rs);
      ++n;
      ++k;
    } while (ident_ok(r[k], mr));
    load(q, r + k);
    return true;
  }
  // legal minimal identity ops, to the fixpoint (search.hip's closure). A pass
  // holds mr fixed and takes, chain by chain in order, every head that was
  // called before it and observes the state; a take changes only its own
  // chain's head, so the heads that pass the call test at the pass's start are
  // exactly the ones the pass can take. The state is fixed too (identity ops),
  // so a pass after one that left mr where it was would take nothing: the
  // fixpoint is reached when a pass takes nothing or mr does not move.
  void close() {
#ifdef S2LC_CERT_PROF
    CP_DECL(tq);
    const uint32_t n0 = n;
    uint32_t passes = 0;
    struct Done {
      uint64_t& t; const uint32_t& n; uint32_t n0; uint32_t& passes;
      ~Done() { CP_LAP(11, t); CP_CNT(10, n - n0); CP_CNT(9, passes); CP_CNT(8, 1); }
    } done{tq, n, n0, passes};
#endif
    uint32_t mr = min_ret();
    for (;;) {
#ifdef S2LC_CERT_PROF
      ++passes;
#endif
      if (mr == EV_INF) return;
      bool changed = false;
      for (uint32_t q0 = 0; q0 < K; q0 += 64) {
        const uint32_t nq = K - q0 < 64 ? K - q0 : 64;
        uint64_t m = 0;
        for (uint32_t j = 0; j < nq; ++j) m |= (uint64_t)(ccall[q0 + j] < mr) << j;
        while (m) {
          const uint32_t q = q0 + (uint32_t)__builtin_ctzll(m);
          m &= m - 1;
          if (take_run(q, mr)) changed = true;
        }
      }
      if (!changed) return;
      const uint32_t mr2 = min_ret();
      if (mr2 == mr) return;
      mr = mr2;
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
  CP_DECL(t0);
  prefetch_range(h.recs.data(), h.recs.size() * sizeof(OpRec));
  prefetch_range(h.rec_op.data(), h.rec_op.size() * sizeof(uint32_t));
  prefetch_range(h.pool.data(), h.pool.size() * sizeof(uint64_t));
  CP_LAP(0, t0);
  order.resize(h.n_ops);
  ident.resize(h.n_ops);
  t_scr.head.resize(h.K);
  Rebuild c(h, t_scr.head, order.data(), ident.data());
  c.rep = replay;
  c.close();
  for (uint32_t m = 0; m < n_moves; ++m) {
    const uint32_t j = moves[m] & 0xFFFFu;
    const bool is_id = moves[m] & MOVE_IDENT;
    if (j >= h.K || c.n >= h.n_ops) { order.resize(c.n); ident.resize(c.n); return false; }
    const OpRec& r = *c.hd.rec[j];
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
  CP_LAP(1, t0);
  if (partial) return true;
  if (order.size() != h.n_ops) {
    if (!p4) return false;
    // P4 completion: nothing left constrains the state; finish in return order.
    std::vector<uint32_t> rest;
    for (uint32_t q = 0; q < h.K; ++q)
      for (const OpRec* x = c.hd.rec[q]; !(x->flags & OPF_SENTINEL); ++x) rest.push_back(h.rec_op[(size_t)(x - c.recs)]);
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
#ifdef S2LC_CERT_PROF
  static const bool norep = getenv("S2LC_CERT_NOREPLAY") != nullptr;
  if (!rebuild(h, moves, n_moves, p4, order, ident, false, !norep)) return false;
  CP_DECL(t0);
  const bool ok = real_time_ok(h, order.data(), order.size());
  CP_LAP(2, t0);
  return ok;
#else
  return rebuild(h, moves, n_moves, p4, order, ident, false, true) &&
         real_time_ok(h, order.data(), order.size());
#endif
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
