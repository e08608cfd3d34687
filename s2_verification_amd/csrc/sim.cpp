// sim.cpp — deterministic S2 simulator emitting collector-format histories.
//
// Reproduces the workload of rust/s2-verification (collect-history.rs +
// history.rs) without a live S2: N sequential clients over one virtual-clock
// stream with one atomic linearization point per op inside [call, return].
//   random_op            history.rs:140-147   uniform {append, read, check_tail}
//   generate_records     history.rs:55-83     U[1,999] records under 1024 metered bytes
//   client               history.rs:357-407   regular: no guards
//   match_seq_num_client history.rs:290-348   msn = last observed tail
//   fencing_token_client history.rs:182-281   set-token every 100 ops (msn-guarded), else own token
//   handle_indefinite_failure history.rs:153-169: defer Finish, 1 s backoff, rotate id < 20
//   client ids from 1, op ids from 0          collect-history.rs:103-104
//   deferred Finishes appended at the end     collect-history.rs:191-199
//   rectifying append (client 0, op 0)        history.rs:641-670
// Record bodies are not materialised: their xxh3 hashes are i.i.d. uniform,
// so a seeded generator stands in for them. The fence-command body hash is
// the real XXH3-64 of the 6-byte token (history.rs:202).
#include <math.h>
#include <string.h>

#include <algorithm>
#include <queue>
#include <string>
#include <vector>

#include "history.h"
#include "s2lincheck.h"

namespace s2lc {
namespace {

struct Rng {
  uint64_t s[4];
  explicit Rng(uint64_t seed) {
    uint64_t x = seed;
    for (int i = 0; i < 4; ++i) {  // splitmix64 seeding
      x += 0x9E3779B97F4A7C15ull;
      uint64_t z = x;
      z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
      z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
      s[i] = z ^ (z >> 31);
    }
  }
  uint64_t next() {  // xoshiro256**
    const uint64_t r = rotl64(s[1] * 5, 7) * 9;
    const uint64_t t = s[1] << 17;
    s[2] ^= s[0]; s[3] ^= s[1]; s[1] ^= s[2]; s[0] ^= s[3];
    s[2] ^= t;
    s[3] = rotl64(s[3], 45);
    return r;
  }
  double uniform() { return (double)(next() >> 11) * (1.0 / 9007199254740992.0); }
  uint64_t range(uint64_t lo, uint64_t hi) { return lo + next() % (hi - lo + 1); }  // inclusive
  double expo(double mean) { return -mean * log(1.0 - uniform()); }
};

// XXH3-64 (seed 0) of a 4..8-byte input: the fence-command body hash.
uint64_t xxh3_4to8(const uint8_t* in, size_t len) {
  uint32_t in1, in2;
  memcpy(&in1, in, 4);
  memcpy(&in2, in + len - 4, 4);
  uint64_t k = ((uint64_t)in2 + ((uint64_t)in1 << 32)) ^ 0xc73ab174c5ecd5a2ull;
  k ^= rotl64(k, 49) ^ rotl64(k, 24);
  k *= 0x9FB21C651E98DF25ull;
  k ^= (k >> 35) + len;
  k *= 0x9FB21C651E98DF25ull;
  return k ^ (k >> 28);
}

enum Fin : uint8_t { F_APP_OK, F_APP_DEF, F_APP_INDEF, F_READ_OK, F_READ_FAIL, F_CT_OK, F_CT_FAIL };

struct SimOp {
  uint64_t op_id;
  uint64_t client_id;
  uint8_t type;  // 0 append 1 read 2 check-tail
  uint64_t num_records = 0;
  std::vector<uint64_t> hashes;
  int set_tok = -1, batch_tok = -1;  // index into token strings, -1 = nil
  bool has_msn = false;
  uint64_t msn = 0;
  Fin fin = F_READ_OK;
  uint64_t tail = 0, stream_hash = 0;
};

struct Rec {  // one LabeledEvent
  uint32_t op;  // index into ops
  bool finish;
};

enum Action : uint8_t { A_START, A_APPLY, A_FINISH };
struct QItem {
  double t;
  uint64_t seq;
  Action a;
  uint32_t who;  // client for START, op for APPLY/FINISH
  bool operator>(const QItem& o) const { return t > o.t || (t == o.t && seq > o.seq); }
};

struct Client {
  uint64_t id;
  uint32_t sample = 0;
  uint64_t expected = 0;
  int token = -1;
  bool stopped = false;
  double finished_at = 0;
  std::vector<uint32_t> deferred;
};

struct Sim {
  const s2lc_sim_params& P;
  Rng rng;
  std::vector<SimOp> ops;
  std::vector<Rec> recs;
  std::vector<std::string> toks;
  std::vector<uint64_t> tok_hash;
  std::vector<Client> clients;
  std::vector<uint32_t> op_client;  // op -> client index
  uint64_t next_client_id = 1, next_op_id = 0;
  // server state
  uint64_t tail = 0, hash = 0;
  int token = -1;
  // violation bookkeeping
  uint64_t total_ops_planned;
  bool violated = false;

  explicit Sim(const s2lc_sim_params& p) : P(p), rng(p.seed * 0x2545F4914F6CDD1Dull + 0x1234567ull) {
    total_ops_planned = (uint64_t)p.num_clients * p.ops_per_client;
  }

  uint32_t max_ids() const { return P.max_client_ids ? P.max_client_ids : 20; }

  void gen_records(SimOp& o) {  // generate_records(U[1,999]), history.rs:55-83
    const uint64_t want = rng.range(1, 999);
    uint64_t bytes = 0;
    while (o.hashes.size() < want && bytes + 8 < 1024) {
      const uint64_t budget = 1024 - bytes - 8;
      const uint64_t size = rng.range(1, budget);
      o.hashes.push_back(rng.next());
      bytes += size + 8;  // metered size: body + per-record overhead
    }
    o.num_records = o.hashes.size();
  }

  uint32_t new_op(uint32_t ci, uint8_t type) {
    SimOp o;
    o.op_id = next_op_id++;
    o.client_id = clients[ci].id;
    o.type = type;
    ops.push_back(std::move(o));
    op_client.push_back(ci);
    return (uint32_t)ops.size() - 1;
  }

  // Client issues its next op (one iteration of the client loops).
  uint32_t issue(uint32_t ci) {
    Client& c = clients[ci];
    const uint32_t wf = P.workflow;
    if (wf == S2LC_WF_FENCING && c.sample % 100 == 0) {  // history.rs:198-231
      uint32_t oi = new_op(ci, 0);
      SimOp& o = ops[oi];
      o.num_records = 1;
      o.hashes.push_back(tok_hash[c.token]);
      o.set_tok = c.token;
      o.has_msn = true;
      o.msn = c.expected;
      return oi;
    }
    const uint64_t r = rng.next() % 3;  // random_op
    uint32_t oi = new_op(ci, (uint8_t)r);
    SimOp& o = ops[oi];
    if (r == 0) {
      gen_records(o);
      if (wf == S2LC_WF_MATCH_SEQ_NUM) { o.has_msn = true; o.msn = c.expected; }
      if (wf == S2LC_WF_FENCING) o.batch_tok = c.token;
    }
    return oi;
  }

  void apply_append(const SimOp& o) {
    tail += o.num_records;
    for (uint64_t h : o.hashes) hash = chain_hash(hash, h);
    if (o.set_tok >= 0) token = o.set_tok;
  }

  bool stale_msn_target(const SimOp& o) const {
    return P.violation == S2LC_VIOL_STALE_MSN && !violated && o.has_msn && o.msn != tail &&
           next_op_id > total_ops_planned / 3;
  }

  // Server-side linearization point.
  void server_apply(uint32_t oi) {
    SimOp& o = ops[oi];
    if (o.type == 0) {
      bool guards = true;
      if (o.batch_tok >= 0 && token != o.batch_tok) guards = false;
      if (o.has_msn && o.msn != tail) guards = false;
      const double u = rng.uniform();
      if (u < P.p_indefinite) {
        o.fin = F_APP_INDEF;
        if (guards && (rng.next() & 1)) apply_append(o);
        return;
      }
      if (!guards) {
        if (stale_msn_target(o)) {  // injected: applied despite a stale msn, reported success
          violated = true;
          apply_append(o);
          o.fin = F_APP_OK;
          o.tail = tail;
          return;
        }
        o.fin = F_APP_DEF;
        return;
      }
      if (u < P.p_indefinite + P.p_definite) { o.fin = F_APP_DEF; return; }
      if (P.violation == S2LC_VIOL_DEFINITE_APPLIED && !violated && next_op_id > total_ops_planned / 3) {
        violated = true;  // injected: applied but reported as a definite failure
        apply_append(o);
        o.fin = F_APP_DEF;
        return;
      }
      apply_append(o);
      o.fin = F_APP_OK;
      o.tail = tail;
    } else if (o.type == 1) {
      if (rng.uniform() < P.p_read_failure) { o.fin = F_READ_FAIL; return; }
      o.fin = F_READ_OK;
      o.tail = tail;
      o.stream_hash = hash;
    } else {
      if (rng.uniform() < P.p_check_tail_failure) { o.fin = F_CT_FAIL; return; }
      o.fin = F_CT_OK;
      o.tail = tail;
    }
  }

  void run() {
    std::priority_queue<QItem, std::vector<QItem>, std::greater<QItem>> q;
    uint64_t seq = 0;
    const double kReq = 10.0, kResp = 10.0, kThink = 1.0, kBackoff = 1000.0;  // ms
    if (P.initial_records) {  // rectifying append, history.rs:641-670
      SimOp o;
      o.op_id = next_op_id++;
      o.client_id = 0;
      o.type = 0;
      o.num_records = P.initial_records;
      for (uint64_t i = 0; i < P.initial_records; ++i) o.hashes.push_back(rng.next());
      ops.push_back(o);
      op_client.push_back(UINT32_MAX);
      apply_append(ops.back());
      ops.back().fin = F_APP_OK;
      ops.back().tail = tail;
      recs.push_back({0, false});
      recs.push_back({0, true});
    }
    for (uint32_t i = 0; i < P.num_clients; ++i) {
      Client c;
      c.id = next_client_id++;
      if (P.workflow == S2LC_WF_FENCING) {  // FencingToken::generate(6)
        static const char al[] = "abcdefghijklmnopqrstuvwxyzABCDEFGHIJKLMNOPQRSTUVWXYZ0123456789";
        std::string s;
        for (int k = 0; k < 6; ++k) s.push_back(al[rng.next() % 62]);
        c.token = (int)toks.size();
        toks.push_back(s);
        tok_hash.push_back(xxh3_4to8((const uint8_t*)s.data(), s.size()));
      }
      clients.push_back(c);
      q.push({rng.uniform(), seq++, A_START, i});
    }
    while (!q.empty()) {
      QItem it = q.top();
      q.pop();
      if (it.a == A_START) {
        Client& c = clients[it.who];
        if (c.stopped || c.sample >= P.ops_per_client) { c.finished_at = it.t; continue; }
        uint32_t oi = issue(it.who);
        recs.push_back({oi, false});
        q.push({it.t + rng.expo(kReq), seq++, A_APPLY, oi});
      } else if (it.a == A_APPLY) {
        server_apply(it.who);
        q.push({it.t + rng.expo(kResp), seq++, A_FINISH, it.who});
      } else {
        const uint32_t oi = it.who;
        const uint32_t ci = op_client[oi];
        Client& c = clients[ci];
        SimOp& o = ops[oi];
        double next_t = it.t + rng.expo(kThink);
        if (o.fin == F_APP_INDEF) {  // handle_indefinite_failure, history.rs:153-169
          c.deferred.push_back(oi);
          next_t = it.t + kBackoff;
          const uint64_t cand = next_client_id++;
          if (cand < max_ids()) c.id = cand;
          else c.stopped = true;
        } else {
          recs.push_back({oi, true});
          const bool track = P.workflow != S2LC_WF_REGULAR;
          if (track && (o.fin == F_APP_OK || o.fin == F_READ_OK || o.fin == F_CT_OK)) c.expected = o.tail;
        }
        c.sample++;
        q.push({next_t, seq++, A_START, ci});
      }
    }
    // deferred indefinite Finishes, in client completion order (collect-history.rs:191-199)
    std::vector<uint32_t> order(clients.size());
    for (uint32_t i = 0; i < order.size(); ++i) order[i] = i;
    std::stable_sort(order.begin(), order.end(),
                     [&](uint32_t a, uint32_t b) { return clients[a].finished_at < clients[b].finished_at; });
    for (uint32_t ci : order)
      for (uint32_t oi : clients[ci].deferred) recs.push_back({oi, true});
    inject_post_hoc();
  }

  void inject_post_hoc() {
    const uint32_t v = P.violation;
    if (v == S2LC_VIOL_NONE || violated) return;
    uint32_t want = v;
    if (want == S2LC_VIOL_STALE_MSN || want == S2LC_VIOL_DEFINITE_APPLIED) want = S2LC_VIOL_TAIL;  // not triggered
    std::vector<uint32_t> cand;
    for (uint32_t i = 0; i < ops.size(); ++i) {
      const Fin f = ops[i].fin;
      if (want == S2LC_VIOL_READ_HASH && f == F_READ_OK) cand.push_back(i);
      if (want == S2LC_VIOL_TAIL && (f == F_APP_OK || f == F_READ_OK || f == F_CT_OK) && ops[i].client_id != 0)
        cand.push_back(i);
    }
    if (cand.empty()) return;
    const uint32_t lo = (uint32_t)(cand.size() / 5), hi = (uint32_t)(cand.size() * 4 / 5);
    const uint32_t pick = cand[hi > lo ? lo + (uint32_t)(rng.next() % (hi - lo)) : 0];
    if (want == S2LC_VIOL_READ_HASH) ops[pick].stream_hash ^= (rng.next() | 1);
    else ops[pick].tail += 1;
    violated = true;
  }
};

void append_u64(std::string& s, uint64_t v) {
  char buf[24];
  int n = 0;
  do { buf[n++] = (char)('0' + v % 10); v /= 10; } while (v);
  while (n) s.push_back(buf[--n]);
}

void render_jsonl(const Sim& S, std::string& out) {
  for (const Rec& r : S.recs) {
    const SimOp& o = S.ops[r.op];
    out += "{\"event\":{";
    if (!r.finish) {
      out += "\"Start\":";
      if (o.type == 1) out += "\"Read\"";
      else if (o.type == 2) out += "\"CheckTail\"";
      else {
        out += "{\"Append\":{\"num_records\":";
        append_u64(out, o.num_records);
        out += ",\"record_hashes\":[";
        for (size_t i = 0; i < o.hashes.size(); ++i) {
          if (i) out.push_back(',');
          append_u64(out, o.hashes[i]);
        }
        out += "],\"set_fencing_token\":";
        if (o.set_tok >= 0) { out += '"'; out += S.toks[o.set_tok]; out += '"'; } else out += "null";
        out += ",\"fencing_token\":";
        if (o.batch_tok >= 0) { out += '"'; out += S.toks[o.batch_tok]; out += '"'; } else out += "null";
        out += ",\"match_seq_num\":";
        if (o.has_msn) append_u64(out, o.msn); else out += "null";
        out += "}}";
      }
    } else {
      out += "\"Finish\":";
      switch (o.fin) {
        case F_APP_OK: out += "{\"AppendSuccess\":{\"tail\":"; append_u64(out, o.tail); out += "}}"; break;
        case F_APP_DEF: out += "\"AppendDefiniteFailure\""; break;
        case F_APP_INDEF: out += "\"AppendIndefiniteFailure\""; break;
        case F_READ_OK:
          out += "{\"ReadSuccess\":{\"tail\":"; append_u64(out, o.tail);
          out += ",\"stream_hash\":"; append_u64(out, o.stream_hash); out += "}}"; break;
        case F_READ_FAIL: out += "\"ReadFailure\""; break;
        case F_CT_OK: out += "{\"CheckTailSuccess\":{\"tail\":"; append_u64(out, o.tail); out += "}}"; break;
        case F_CT_FAIL: out += "\"CheckTailFailure\""; break;
      }
    }
    out += "},\"client_id\":";
    append_u64(out, o.client_id);
    out += ",\"op_id\":";
    append_u64(out, o.op_id);
    out += "}\n";
  }
}

void to_history(const Sim& S, History& h) {
  h.events.reserve(S.recs.size());
  std::vector<uint32_t> tok_id(S.toks.size());
  for (size_t i = 0; i < S.toks.size(); ++i) tok_id[i] = h.intern(S.toks[i]);
  for (const Rec& r : S.recs) {
    const SimOp& o = S.ops[r.op];
    Event e;
    e.op_id = (int64_t)o.op_id;
    e.client_id = (int64_t)o.client_id;
    if (!r.finish) {
      e.kind = 0;
      e.input_type = o.type;
      if (o.type == 0) {
        e.has_num_records = 1;
        e.num_records = o.num_records;
        e.hash_off = h.pool.size();
        e.hash_cnt = o.hashes.size();
        h.pool.insert(h.pool.end(), o.hashes.begin(), o.hashes.end());
        e.set_tok = o.set_tok >= 0 ? tok_id[o.set_tok] : 0;
        e.batch_tok = o.batch_tok >= 0 ? tok_id[o.batch_tok] : 0;
        e.has_msn = o.has_msn;
        e.msn = o.msn;
      }
    } else {
      e.kind = 1;
      switch (o.fin) {
        case F_APP_OK: case F_CT_OK: e.has_tail = 1; e.tail = o.tail; break;
        case F_READ_OK: e.has_tail = 1; e.tail = o.tail; e.has_hash = 1; e.stream_hash = o.stream_hash; break;
        case F_APP_INDEF: e.failure = 1; break;
        default: e.failure = 1; e.definite = 1; break;
      }
    }
    h.events.push_back(e);
  }
}

}  // namespace

int simulate(const s2lc_sim_params& p, History* h, std::string* jsonl) {
  if (p.workflow > S2LC_WF_FENCING || p.num_clients == 0) return S2LC_EINVAL;
  Sim S(p);
  S.run();
  if (jsonl) render_jsonl(S, *jsonl);
  if (h) to_history(S, *h);
  return 0;
}

uint64_t xxh3_64_small(const uint8_t* in, size_t len) { return xxh3_4to8(in, len); }

}  // namespace s2lc
