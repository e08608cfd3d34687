// viz.cpp — the visualization the reference CLI writes after every check
// (golang/s2-porcupine/main.go:608-631: porcupine.Visualize(model, info, file)
// into ./porcupine-outputs/<input>-*.html).
//
// Porcupine's page shows each client's operations on a time axis, labelled
// with DescribeOperation, and the (partial) linearization with the model state
// after each step (DescribeState of the powerset state). This is a
// self-contained HTML page with the same information: the op rectangles
// (call .. return event index) per client, the witness order (Ok) or the
// deepest certified prefix (Illegal), and the powerset state after each
// linearized op. Describe strings follow main.go:341-426 exactly.
#include <stdio.h>
#include <string.h>

#include <algorithm>
#include <string>
#include <unordered_map>
#include <vector>

#include "history.h"
#include "s2lincheck.h"
#include "search.h"

namespace s2lc {
namespace {

std::string u64s(uint64_t v) { return std::to_string(v); }

std::string tok_str(const History& h, uint32_t id) { return id ? h.tokens[id - 1] : std::string(); }

// DescribeOperation (main.go:341-352) with formatAppendCall / formatReadCall /
// formatCheckTailCall (main.go:362-426).
std::string describe_op(const History& h, uint32_t d) {
  static const Event no_return{};  // (a call without a return: duplicate-id histories)
  const Event& in = h.events[h.op_call[d]];
  const Event& out = h.op_ret[d] < h.events.size() ? h.events[h.op_ret[d]] : no_return;
  if (in.input_type == 0) {
    std::string failure = "none";
    if (out.definite) failure = "definite";
    else if (out.failure) failure = "indefinite";
    std::string s = "append(len[" + u64s(in.num_records) + "]";
    if (in.set_tok) s += ", set_token[" + tok_str(h, in.set_tok) + "]";
    if (in.batch_tok) s += ", batch_token[" + tok_str(h, in.batch_tok) + "]";
    if (in.has_msn) s += ", match_seq_num[" + u64s(in.msn) + "]";
    if (in.hash_cnt) s += ", rh_last[" + u64s(h.pool[in.hash_off + in.hash_cnt - 1]) + "]";
    s += ")";
    return s + " -> " + (out.failure ? "FAILED[" + failure + "]" : "tail[" + u64s(out.tail) + "]");
  }
  if (in.input_type == 1) {
    if (out.failure) return "read() -> failed";
    if (out.has_hash) return "read() -> tail[" + u64s(out.tail) + "], hash[" + u64s(out.stream_hash) + "]";
    return "read() -> tail[" + u64s(out.tail) + "]";
  }
  if (out.failure) return "check_tail() -> failed";
  return "check_tail() -> tail[" + u64s(out.tail) + "]";
}

// DescribeState (main.go:353-360)
std::string describe_state(const History& h, const State& s) {
  std::string r = "tail[" + u64s(s.tail) + "],hash[" + u64s(s.hash) + "]";
  if (s.tok) r += ",token[" + tok_str(h, s.tok) + "]";
  return r;
}

std::string html_esc(const std::string& s) {
  std::string o;
  for (char c : s) {
    if (c == '<') o += "&lt;";
    else if (c == '>') o += "&gt;";
    else if (c == '&') o += "&amp;";
    else if (c == '"') o += "&quot;";
    else o += c;
  }
  return o;
}

}  // namespace
}  // namespace s2lc

using namespace s2lc;

static int render(const s2lc_history* hh, const s2lc_result* r, const s2lc_partials* info, const char* path);

static int put_str(const std::string& s, char* buf, size_t cap) {
  if (buf && cap) {
    const size_t n = std::min(s.size(), cap - 1);
    memcpy(buf, s.data(), n);
    buf[n] = 0;
  }
  return (int)std::min<size_t>(s.size(), 0x7FFFFFFF);
}

extern "C" int s2lc_describe_operation(const s2lc_history* hh, uint32_t op, char* buf, size_t cap) {
  if (!hh) return S2LC_EINVAL;
  const History& h = hh->h;
  h.ensure_events();
  if (op >= h.n_ops || h.op_call[op] >= h.events.size()) return S2LC_EINVAL;
  return put_str(describe_op(h, op), buf, cap);
}

extern "C" int s2lc_describe_state(const s2lc_history* hh, const s2lc_state* s, char* buf, size_t cap) {
  if (!hh || !s) return S2LC_EINVAL;
  const History& h = hh->h;
  if (s->token > h.tokens.size()) return S2LC_EINVAL;
  return put_str(describe_state(h, State{s->tail, s->stream_hash, s->token}), buf, cap);
}

extern "C" int s2lc_visualize(const s2lc_history* hh, const s2lc_result* r, const char* path) {
  return render(hh, r, nullptr, path);
}

extern "C" int s2lc_visualize_info(const s2lc_history* hh, const s2lc_result* r, const s2lc_partials* info,
                                   const char* path) {
  return render(hh, r, info, path);
}

static int render(const s2lc_history* hh, const s2lc_result* r, const s2lc_partials* info, const char* path) {
  if (!hh || !r || !path) return S2LC_EINVAL;
  const History& h = hh->h;
  if (h.status) return h.status;
  h.ensure_events();
  FILE* f = fopen(path, "w");
  if (!f) return S2LC_EIO;
  try {
    // the linearized ops (witness or deepest certified prefix), as dense ids
    std::unordered_map<int64_t, uint32_t> dense;
    for (uint32_t d = 0; d < h.n_ops; ++d) dense[h.op_ids[d]] = d;
    std::vector<uint32_t> order;
    const int64_t* ids = r->verdict == S2LC_OK ? r->witness : r->partial;
    const uint32_t nids = r->verdict == S2LC_OK ? r->witness_len : r->partial_len;
    for (uint32_t k = 0; k < nids && ids; ++k) {
      auto it = dense.find(ids[k]);
      if (it != dense.end()) order.push_back(it->second);
    }
    std::vector<int> pos(h.n_ops, -1);
    for (size_t k = 0; k < order.size(); ++k) pos[order[k]] = (int)k;
    // powerset state after each linearized op (porcupine's state for ToModel())
    std::vector<std::string> after(order.size());
    {
      std::vector<State> set{State{0, 0, 0}}, next;
      bool tracked = true;
      for (size_t k = 0; k < order.size(); ++k) {
        if (!tracked) { after[k] = "(state set not tracked)"; continue; }
        const OpRec rec = h.rec_of(order[k]);
        next.clear();
        for (const State& s : set) {
          State kids[2];
          const int nk = s2_step(rec, s, h.pool.data(), kids);
          for (int q = 0; q < nk; ++q) {
            bool dup = false;
            for (const State& x : next) dup |= state_eq(x, kids[q]);
            if (!dup) next.push_back(kids[q]);
          }
        }
        set.swap(next);
        std::string d = "[";
        for (size_t q = 0; q < set.size() && q < 4; ++q) d += (q ? ", " : "") + describe_state(h, set[q]);
        if (set.size() > 4) d += ", … " + std::to_string(set.size()) + " states";
        after[k] = d + "]";
        if (set.size() > 256) tracked = false;  // porcupine would track it; the page stays readable
      }
    }
    // clients
    std::vector<int64_t> clients;
    for (uint32_t d = 0; d < h.n_ops; ++d) clients.push_back(h.events[h.op_call[d]].client_id);
    std::sort(clients.begin(), clients.end());
    clients.erase(std::unique(clients.begin(), clients.end()), clients.end());
    std::unordered_map<int64_t, int> row;
    for (size_t i = 0; i < clients.size(); ++i) row[clients[i]] = (int)i;

    const char* verdict = r->verdict == S2LC_OK ? "Ok" : r->verdict == S2LC_ILLEGAL ? "Illegal" : "Unknown";
    const double xs = 6.0;  // px per event
    const int rh = 22;      // px per client row
    const size_t n_ev = h.events.size();
    fprintf(f,
            "<!DOCTYPE html>\n<html><head><meta charset=\"utf-8\"><title>s2-porcupine: %s</title>\n"
            "<style>body{font-family:monospace;font-size:12px}rect.lin{fill:#9fd89f}rect.out{fill:#f2a0a0}"
            "rect.ok{fill:#cfe3ff}text{font-size:10px}table{border-collapse:collapse}td,th{border:1px solid #ccc;"
            "padding:2px 6px}</style></head><body>\n",
            verdict);
    fprintf(f, "<h2>%s</h2>\n<p>%u operations, %zu clients, %zu events. ", verdict, h.n_ops, clients.size(), n_ev);
    if (r->verdict == S2LC_OK)
      fprintf(f, "Linearization found (%zu ops, certified through the CPU model).</p>\n", order.size());
    else
      fprintf(f, "Deepest linearized prefix the search reached: %zu of %u ops (red: not in it).</p>\n", order.size(),
              h.n_ops);
    fprintf(f, "<div style=\"overflow-x:scroll\"><svg width=\"%.0f\" height=\"%zu\">\n", xs * (double)n_ev + 80.0,
            (clients.size() + 1) * (size_t)rh);
    for (size_t i = 0; i < clients.size(); ++i)
      fprintf(f, "<text x=\"0\" y=\"%zu\">c%lld</text>\n", i * rh + 15, (long long)clients[i]);
    for (uint32_t d = 0; d < h.n_ops; ++d) {
      const int y = row[h.events[h.op_call[d]].client_id] * rh + 3;
      const double x0 = 60.0 + xs * h.op_call[d],
                   x1 = 60.0 + xs * std::min<size_t>(h.op_ret[d], n_ev ? n_ev - 1 : 0) + xs * 0.8;
      const char* cls = pos[d] >= 0 ? "lin" : (r->verdict == S2LC_OK ? "ok" : "out");
      std::string tip = "op " + std::to_string(h.op_ids[d]) + ": " + describe_op(h, d);
      if (pos[d] >= 0) tip += "\nlinearized #" + std::to_string(pos[d]) + ", state after: " + after[(size_t)pos[d]];
      const uint32_t lp = info && d < info->n_ops ? info->op_partial[d] : 0xFFFFFFFFu;
      if (lp != 0xFFFFFFFFu)
        tip += "\nlongest partial linearization containing it: #" + std::to_string(lp) + " (" +
               std::to_string(info->offs[lp + 1] - info->offs[lp]) + " ops)";
      fprintf(f, "<g onmouseenter=\"hl(%u)\" onmouseleave=\"hl(-1)\"><title>%s</title><rect id=\"op%u\" class=\"%s\" x=\"%.1f\" y=\"%d\" width=\"%.1f\" height=\"%d\"/>",
              d, html_esc(tip).c_str(), d, cls, x0, y, std::max(1.0, x1 - x0), rh - 6);
      if (pos[d] >= 0) fprintf(f, "<text x=\"%.1f\" y=\"%d\">%d</text>", x0 + 1, y + 11, pos[d]);
      fprintf(f, "</g>\n");
    }
    fprintf(f, "</svg></div>\n<h3>%s</h3>\n<table><tr><th>#</th><th>op id</th><th>client</th><th>operation</th>"
               "<th>state after</th></tr>\n",
            r->verdict == S2LC_OK ? "Linearization" : "Deepest linearized prefix");
    for (size_t k = 0; k < order.size(); ++k) {
      const uint32_t d = order[k];
      fprintf(f, "<tr><td>%zu</td><td>%lld</td><td>%lld</td><td>%s</td><td>%s</td></tr>\n", k,
              (long long)h.op_ids[d], (long long)h.events[h.op_call[d]].client_id, html_esc(describe_op(h, d)).c_str(),
              html_esc(after[k]).c_str());
    }
    fprintf(f, "</table>\n");
    // LinearizationInfo (porcupine's Visualize: hovering an op shows the
    // longest partial linearization containing it)
    fprintf(f, "<script>\nconst P=[");
    if (info) {
      for (uint32_t k = 0; k < info->n_partials; ++k) {
        fprintf(f, "%s[", k ? "," : "");
        for (uint64_t x = info->offs[k]; x < info->offs[k + 1]; ++x) {
          auto it = dense.find(info->ids[x]);
          fprintf(f, "%s%u", x > info->offs[k] ? "," : "", it != dense.end() ? it->second : 0u);
        }
        fprintf(f, "]");
      }
    }
    fprintf(f, "];\nconst L=[");
    for (uint32_t d = 0; d < h.n_ops; ++d)
      fprintf(f, "%s%d", d ? "," : "", info && d < info->n_ops && info->op_partial[d] != 0xFFFFFFFFu ? (int)info->op_partial[d] : -1);
    fprintf(f, "];\nfunction hl(d){document.querySelectorAll('rect').forEach(r=>r.style.stroke='');"
               "if(d<0||L[d]<0)return;P[L[d]].forEach(o=>{const e=document.getElementById('op'+o);"
               "if(e){e.style.stroke='#000';e.style.strokeWidth='2';}});}\n</script>\n");
    if (info && info->n_partials) {
      fprintf(f, "<h3>Longest partial linearizations (LinearizationInfo%s)</h3>\n<table><tr><th>#</th><th>ops</th>"
                 "<th>ops whose longest it is</th></tr>\n", info->exact ? "" : ", search budget reached: lower bounds");
      std::vector<uint32_t> owners(info->n_partials, 0);
      for (uint32_t d = 0; d < info->n_ops; ++d)
        if (info->op_partial[d] != 0xFFFFFFFFu) owners[info->op_partial[d]]++;
      for (uint32_t k = 0; k < info->n_partials; ++k)
        fprintf(f, "<tr><td>%u</td><td>%llu</td><td>%u</td></tr>\n", k,
                (unsigned long long)(info->offs[k + 1] - info->offs[k]), owners[k]);
      fprintf(f, "</table>\n");
    }
    fprintf(f, "</body></html>\n");
  } catch (...) {
    fclose(f);
    return S2LC_ENOMEM;
  }
  return fclose(f) == 0 ? 0 : S2LC_EIO;
}
