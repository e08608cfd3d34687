// TEST INFRASTRUCTURE: host cost of witness certification (rebuild the
// linearization from a move list + replay it through the CPU model), per
// history, single thread. Move lists come from a small CPU breadth-first
// search written here (the GPU search's rounds, no reductions but the
// E-closure), so the timing needs no GPU:
//   make -C tests/witness_bench && tests/witness_bench/bench [n]
// Exit status 0 when every witness certifies and every broken move list is
// rejected (tests/test_witness_cpu.py runs it at a small n).
#include <chrono>
#include <map>
#include <stdio.h>
#include <stdlib.h>
#include <string>
#include <string.h>
#include <vector>

#include "history.h"
#include "s2lincheck.h"
#include "search.h"

using namespace s2lc;

struct Cfg { std::vector<uint16_t> cnt; State s; int parent; uint32_t move; };

static const OpRec& head(const History& h, const std::vector<uint16_t>& c, uint32_t q) {
  return h.recs[h.chain_start[q] + c[q]];
}
static uint32_t min_ret(const History& h, const std::vector<uint16_t>& c) {
  uint32_t m = EV_INF;
  for (uint32_t q = 0; q < h.K; ++q) m = std::min(m, head(h, c, q).ret_ev);
  return m;
}
static void close_cfg(const History& h, Cfg& c) {
  for (;;) {
    const uint32_t mr = min_ret(h, c.cnt);
    bool ch = false;
    for (uint32_t q = 0; q < h.K; ++q)
      for (;;) {
        const OpRec& r = head(h, c.cnt, q);
        if (!(r.flags & OPF_CLS_E) || r.call_ev >= mr || !ident_legal(r, c.s)) break;
        c.cnt[q]++;
        ch = true;
      }
    if (!ch) return;
  }
}
static bool complete(const History& h, const Cfg& c) {
  for (uint32_t q = 0; q < h.K; ++q) if (h.chain_start[q] + c.cnt[q] + 1 < h.chain_start[q + 1]) return false;
  return true;
}

// moves of a completing path, or false (Illegal / too wide)
static bool find_moves(const History& h, std::vector<uint32_t>& moves) {
  std::vector<Cfg> all;
  Cfg c0{std::vector<uint16_t>(h.K, 0), State{0, 0, 0}, -1, 0};
  close_cfg(h, c0);
  all.push_back(c0);
  std::vector<int> cur{0};
  int done = complete(h, c0) ? 0 : -1;
  while (done < 0 && !cur.empty() && all.size() < 200000) {
    std::map<std::string, int> seen;
    std::vector<int> nxt;
    for (int ci : cur) {
      const uint32_t mr = min_ret(h, all[ci].cnt);
      for (uint32_t j = 0; j < h.K && done < 0; ++j) {
        const OpRec& r = head(h, all[ci].cnt, j);
        if (r.flags & (OPF_SENTINEL | OPF_CLS_E) || r.call_ev >= mr) continue;
        State kids[2];
        const int nk = s2_step(r, all[ci].s, h.pool.data(), kids);
        for (int k = 0; k < nk && done < 0; ++k) {
          const bool ident = state_eq(kids[k], all[ci].s) && !(r.flags & OPF_CLS_D);
          Cfg c{all[ci].cnt, kids[k], ci, j | (ident ? MOVE_IDENT : 0u)};
          if (ident && !state_eq(append_opt(r, all[ci].s, h.pool.data()), all[ci].s) == false && (r.flags & OPF_CLS_D)) continue;
          c.cnt[j]++;
          close_cfg(h, c);
          std::string key((const char*)c.cnt.data(), c.cnt.size() * 2);
          key.append((const char*)&c.s.tail, 8).append((const char*)&c.s.hash, 8).append((const char*)&c.s.tok, 4);
          if (seen.count(key)) continue;
          seen[key] = (int)all.size();
          all.push_back(c);
          if (complete(h, c)) { done = (int)all.size() - 1; break; }
          nxt.push_back((int)all.size() - 1);
        }
      }
    }
    cur.swap(nxt);
  }
  if (done < 0) return false;
  moves.clear();
  for (int i = done; all[i].parent >= 0; i = all[i].parent) moves.push_back(all[i].move);
  std::reverse(moves.begin(), moves.end());
  return true;
}

int main(int argc, char** argv) {
  const int n = argc > 1 ? atoi(argv[1]) : 2000;
  std::vector<s2lc_history*> hs;
  std::vector<std::vector<uint32_t>> mv;
  for (int sd = 0; (int)hs.size() < n && sd < 10 * n; ++sd) {
    s2lc_sim_params p;
    s2lc_sim_params_default(&p);
    const uint32_t wf[3] = {S2LC_WF_REGULAR, S2LC_WF_MATCH_SEQ_NUM, S2LC_WF_FENCING};
    p.workflow = wf[sd % 3];
    p.num_clients = 5 + sd % 4;
    p.ops_per_client = 100;
    p.seed = (uint64_t)sd;
    p.p_indefinite = 0.01; p.p_definite = 0.02; p.p_read_failure = 0.01; p.p_check_tail_failure = 0.01;
    s2lc_history* h = nullptr;
    if (s2lc_simulate_history(&p, &h)) return 1;
    std::vector<uint32_t> m;
    if (!find_moves(h->h, m)) { s2lc_history_free(h); continue; }
    hs.push_back(h);
    mv.push_back(m);
  }
  std::vector<int64_t> ids(1 << 16);
  int bad = 0;
  {  // one history, repeated (warm caches)
    std::vector<uint32_t> order;
    std::vector<uint8_t> ident;
    const auto a = std::chrono::steady_clock::now();
    for (int k = 0; k < 1000; ++k)
      bad += !rebuild_linearization(hs[0]->h, mv[0].data(), (uint32_t)mv[0].size(), false, order, ident, false);
    const auto b = std::chrono::steady_clock::now();
    printf("{\"warm_rebuild_us\": %.2f, \"moves\": %zu, \"n_ops\": %u, \"K\": %u}\n",
           1e3 * std::chrono::duration<double>(b - a).count(), mv[0].size(), hs[0]->h.n_ops, hs[0]->h.K);
  }
  {  // the two halves separately
    std::vector<uint32_t> order;
    std::vector<uint8_t> ident;
    double t_rb = 0, t_rp = 0;
    for (size_t i = 0; i < hs.size(); ++i) {
      const auto a = std::chrono::steady_clock::now();
      bad += !rebuild_linearization(hs[i]->h, mv[i].data(), (uint32_t)mv[i].size(), false, order, ident, false);
      const auto b = std::chrono::steady_clock::now();
      bad += !replay_path(hs[i]->h, order.data(), ident.data(), order.size());
      const auto c = std::chrono::steady_clock::now();
      t_rb += std::chrono::duration<double>(b - a).count();
      t_rp += std::chrono::duration<double>(c - b).count();
    }
    printf("{\"rebuild_us\": %.2f, \"replay_us\": %.2f}\n", 1e6 * t_rb / hs.size(), 1e6 * t_rp / hs.size());
  }
  for (int rep = 0; rep < 3; ++rep) {
    const auto t0 = std::chrono::steady_clock::now();
    for (size_t i = 0; i < hs.size(); ++i)
      bad += s2lc_witness_from_moves(hs[i], mv[i].data(), mv[i].size(), 0, ids.data(), ids.size()) != 0;
    const double s = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    printf("{\"histories\": %zu, \"us_per_history\": %.2f, \"failed\": %d}\n", hs.size(), 1e6 * s / hs.size(), bad);
  }
  {  // a digest of every certified witness (op ids in order), to compare builds
    uint64_t fnv = 0xcbf29ce484222325ull;
    for (size_t i = 0; i < hs.size(); ++i) {
      if (s2lc_witness_from_moves(hs[i], mv[i].data(), mv[i].size(), 0, ids.data(), ids.size()) != 0) { ++bad; continue; }
      for (uint32_t k = 0; k < hs[i]->h.n_ops; ++k) fnv = (fnv ^ (uint64_t)ids[k]) * 0x100000001b3ull;
    }
    printf("{\"witness_digest\": \"%016llx\"}\n", (unsigned long long)fnv);
  }
  {  // broken move lists must fail certification: an unknown chain first, or the last move dropped
    int negatives = 0, rejected = 0;
    for (size_t i = 0; i < hs.size() && i < 100; ++i) {
      if (mv[i].empty()) continue;
      std::vector<uint32_t> m = mv[i];
      m[0] = 0xFFFFu;
      ++negatives;
      rejected += s2lc_witness_from_moves(hs[i], m.data(), m.size(), 0, ids.data(), ids.size()) != 0;
      m = mv[i];
      m.pop_back();
      ++negatives;
      rejected += s2lc_witness_from_moves(hs[i], m.data(), m.size(), 0, ids.data(), ids.size()) != 0;
    }
    printf("{\"negatives\": %d, \"rejected\": %d}\n", negatives, rejected);
    bad += negatives - rejected;
  }
  for (auto* h : hs) s2lc_history_free(h);
  return bad != 0;
}
