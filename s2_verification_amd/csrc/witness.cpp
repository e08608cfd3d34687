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

struct HostCfg {
  std::vector<uint32_t> cnt;
  State s{0, 0, 0};
};

const OpRec& head(const History& h, const HostCfg& c, uint32_t q) { return h.recs[h.chain_start[q] + c.cnt[q]]; }

uint32_t min_ret(const History& h, const HostCfg& c) {
  uint32_t m = EV_INF;
  for (uint32_t q = 0; q < h.K; ++q) m = std::min(m, head(h, c, q).ret_ev);
  return m;
}

// Same closure as the device (search.hip), recording the ops it linearizes.
void close(const History& h, HostCfg& c, std::vector<uint32_t>& order, std::vector<uint8_t>& ident) {
  for (;;) {
    const uint32_t mr = min_ret(h, c);
    if (mr == EV_INF) return;
    bool changed = false;
    for (uint32_t q = 0; q < h.K; ++q) {
      for (;;) {
        const OpRec& r = head(h, c, q);
        if (!(r.flags & OPF_CLS_E) || r.call_ev >= mr || !ident_legal(r, c.s)) break;
        order.push_back(h.rec_op[h.chain_start[q] + c.cnt[q]]);
        ident.push_back(1);
        c.cnt[q]++;
        changed = true;
      }
    }
    if (!changed) return;
  }
}

}  // namespace

bool rebuild_linearization(const History& h, const uint32_t* moves, uint32_t n_moves, bool p4,
                           std::vector<uint32_t>& order, std::vector<uint8_t>& ident, bool partial) {
  order.clear();
  ident.clear();
  if (h.structural) return false;
  HostCfg c;
  c.cnt.assign(h.K, 0);
  close(h, c, order, ident);
  for (uint32_t m = 0; m < n_moves; ++m) {
    const uint32_t j = moves[m] & 0xFFFFu;
    const bool is_id = moves[m] & MOVE_IDENT;
    if (j >= h.K) return false;
    const OpRec& r = head(h, c, j);
    if (r.flags & (OPF_SENTINEL | OPF_CLS_E)) return false;
    if (r.call_ev >= min_ret(h, c)) return false;  // not minimal
    State kids[2];
    const int nk = s2_step(r, c.s, h.pool.data(), kids);
    State want = c.s;
    if (!is_id) {
      if (!append_guards_ok(r, c.s)) return false;
      want = append_opt(r, c.s, h.pool.data());
    }
    bool found = false;
    for (int k = 0; k < nk; ++k) found |= state_eq(kids[k], want);
    if (!found) return false;
    c.s = want;
    order.push_back(h.rec_op[h.chain_start[j] + c.cnt[j]]);
    ident.push_back(is_id ? 1 : 0);
    c.cnt[j]++;
    close(h, c, order, ident);
  }
  if (partial) return true;
  if (order.size() != h.n_ops) {
    if (!p4) return false;
    // P4 completion: nothing left constrains the state; finish in return order.
    std::vector<uint32_t> rest;
    for (uint32_t q = 0; q < h.K; ++q)
      for (uint32_t p = h.chain_start[q] + c.cnt[q]; p + 1 < h.chain_start[q + 1]; ++p) rest.push_back(h.rec_op[p]);
    std::sort(rest.begin(), rest.end(), [&](uint32_t a, uint32_t b) { return h.op_ret[a] < h.op_ret[b]; });
    order.insert(order.end(), rest.begin(), rest.end());
    ident.resize(order.size(), 1);
  }
  return order.size() == h.n_ops;
}

static bool replay_states(const History& h, const uint32_t* order, const uint8_t* ident, size_t n) {
  State s{0, 0, 0};
  for (size_t i = 0; i < n; ++i) {
    const OpRec r = h.rec_of(order[i]);
    State kids[2];
    const int nk = s2_step(r, s, h.pool.data(), kids);
    // the outcome this linearization claims: the optimistic successor for an
    // append taken as applied, the unchanged state otherwise
    const bool applied = !ident[i] && !(r.flags & OPF_CLS_E) && (r.flags & OPF_KIND_MASK) == 0;
    const State want = applied ? append_opt(r, s, h.pool.data()) : s;
    bool found = false;
    for (int k = 0; k < nk; ++k) found |= state_eq(kids[k], want);
    if (!found) return false;
    s = want;
  }
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
  std::vector<uint8_t> seen(h.n_ops, 0);
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

}  // namespace s2lc
