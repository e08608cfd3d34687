// cache.cpp — binary SoA history cache.
//
// eventsFromReader (golang/s2-porcupine/main.go:529-563) decodes a history
// from JSONL on every run. A checker that re-checks the same histories (DST
// seeds re-run, a regression corpus) pays that decode, plus renumber / chain
// decomposition (History::finalize), each time. The cache is the decoded and
// finalized form as one byte image: the event array, the record-hash pool,
// the token strings and the chain-major OpRec table with its index arrays.
// Loading it is a bounds-checked copy per array, in parallel over histories.
//
// Image layout (little endian, every array 8-byte aligned):
//   "S2LCSOA1" | u32 version | u32 sizeof(Event) | u64 n | u64 off[n + 1]
//   then per history, at payload + off[i]:
//     u32 status, structural, n_ops, n_ident, K, hflags, max_chain_len, n_tokens
//     u64 n_events, n_pool, n_recs, mode
//     mode 0 (compact): i64 client_id[n_events]   (every other event field
//        is the op's record: a finalized history's events are exactly its
//        ops' call / return pairs, rebuilt on load)
//     mode 1 (full, structurally odd or unfinalized histories): Event[n_events]
//     u64 pool[n_pool] | tokens (u32 len, bytes, pad)
//     u32 chain_start[K + 1] | OpRec[n_recs] | u32 rec_op[n_recs] | i64 op_ids[n_ops]
//   (op_rec, op_call and op_ret follow from rec_op and the records.)
// About 92 bytes per op plus 8 per record hash: ~0.55x the collector JSONL.
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <atomic>
#include <string>
#include <thread>
#include <vector>

#include "history.h"
#include "host_par.h"
#include "s2lincheck.h"

namespace s2lc {
namespace {

constexpr char kMagic[8] = {'S', '2', 'L', 'C', 'S', 'O', 'A', '1'};
constexpr uint32_t kVersion = 1;

size_t pad8(size_t x) { return (x + 7) & ~(size_t)7; }

// The call and return events of dense op d, from its record (what the JSONL
// loader and the simulator produce for it: History::rec_of's inverse).
void event_pair(const History& h, uint32_t d, int64_t c_client, int64_t r_client, Event& c, Event& r) {
  const OpRec& o = h.recs[h.op_rec[d]];
  c = Event{};
  r = Event{};
  c.kind = 0;
  c.op_id = h.op_ids[d];
  c.client_id = c_client;
  c.input_type = (uint8_t)(o.flags & OPF_KIND_MASK);
  c.has_num_records = c.input_type == S2LC_INPUT_APPEND ? 1 : 0;
  c.has_msn = (o.flags & OPF_HAS_MSN) ? 1 : 0;
  c.num_records = o.num_records;
  c.msn = o.msn;
  c.set_tok = o.set_tok;
  c.batch_tok = o.batch_tok;
  c.hash_off = o.hash_off;
  c.hash_cnt = o.hash_cnt;
  r.kind = 1;
  r.op_id = h.op_ids[d];
  r.client_id = r_client;
  r.failure = (o.flags & OPF_FAIL) ? 1 : 0;
  r.definite = (o.flags & OPF_DEF) ? 1 : 0;
  r.has_tail = (o.flags & OPF_HAS_TAIL) ? 1 : 0;
  r.has_hash = (o.flags & OPF_HAS_HASH) ? 1 : 0;
  r.tail = o.out_tail;
  r.stream_hash = o.out_hash;
}

// [off, off + cnt) inside a pool of n entries, without the u64 sum (a
// crafted image could make off + cnt wrap past n)
bool pool_range_ok(uint64_t off, uint64_t cnt, uint64_t n) { return cnt <= n && off <= n - cnt; }

bool event_eq(const Event& a, const Event& b) {  // field by field (padding bytes are not data)
  return a.kind == b.kind && a.op_id == b.op_id && a.client_id == b.client_id && a.input_type == b.input_type &&
         a.has_num_records == b.has_num_records && a.has_msn == b.has_msn && a.num_records == b.num_records &&
         a.msn == b.msn && a.set_tok == b.set_tok && a.batch_tok == b.batch_tok && a.hash_off == b.hash_off &&
         a.hash_cnt == b.hash_cnt && a.failure == b.failure && a.definite == b.definite && a.has_tail == b.has_tail &&
         a.has_hash == b.has_hash && a.tail == b.tail && a.stream_hash == b.stream_hash;
}

struct Head {
  uint32_t status, structural, n_ops, n_ident, K, hflags, max_chain_len, n_tokens;
  uint64_t n_events, n_pool, n_recs, mode, n_cs;  // n_cs: chain_start entries (K + 1, or 0 unfinalized)
};

// A history whose events are exactly its ops' call / return pairs, each
// event's fields those of its op's record (true for every finalized history
// the loader or the simulator makes): stored without the event array.
bool compactable(const History& h) {
  h.ensure_events();
  if (h.status || h.structural || h.literal || h.events.size() != 2ull * h.n_ops || h.op_rec.size() != h.n_ops) return false;
  for (uint32_t d = 0; d < h.n_ops; ++d) {
    Event c, r;
    event_pair(h, d, h.events[h.op_call[d]].client_id, h.events[h.op_ret[d]].client_id, c, r);
    if (!event_eq(c, h.events[h.op_call[d]]) || !event_eq(r, h.events[h.op_ret[d]])) return false;
  }
  return true;
}

size_t section_bytes(const History& h, bool compact) {
  size_t b = sizeof(Head);
  b += compact ? h.n_events() * 8 : pad8(h.n_events() * sizeof(Event));
  b += h.pool.size() * 8;
  for (const std::string& t : h.tokens) b += pad8(4 + t.size());
  b += pad8(h.chain_start.size() * 4);
  b += h.recs.size() * sizeof(OpRec);
  b += pad8(h.rec_op.size() * 4);
  b += (size_t)h.n_ops * 8;
  if (!compact) b += 3 * pad8((size_t)h.n_ops * 4);  // op_rec, op_call, op_ret as they are
  return b;
}

struct Writer {
  uint8_t* p;
  template <typename T>
  void arr(const T* v, size_t n) {
    if (n) memcpy(p, v, n * sizeof(T));
    const size_t b = n * sizeof(T);
    memset(p + b, 0, pad8(b) - b);
    p += pad8(b);
  }
};

void write_section(const History& h, bool compact, uint8_t* dst) {
  Head hd{(uint32_t)h.status, (uint32_t)h.structural, h.n_ops, h.n_ident, h.K, h.hflags, h.max_chain_len,
          (uint32_t)h.tokens.size(), (uint64_t)h.n_events(), h.pool.size(), h.recs.size(), compact ? 0u : 1u,
          h.chain_start.size()};
  memcpy(dst, &hd, sizeof hd);
  Writer w{dst + sizeof hd};
  if (compact) {
    int64_t* c = reinterpret_cast<int64_t*>(w.p);
    for (size_t e = 0; e < h.events.size(); ++e) memcpy(c + e, &h.events[e].client_id, 8);
    w.p += h.events.size() * 8;
  } else {
    w.arr(h.events.data(), h.events.size());
  }
  w.arr(h.pool.data(), h.pool.size());
  for (const std::string& t : h.tokens) {
    const uint32_t len = (uint32_t)t.size();
    memcpy(w.p, &len, 4);
    memcpy(w.p + 4, t.data(), len);
    memset(w.p + 4 + len, 0, pad8(4 + len) - 4 - len);
    w.p += pad8(4 + len);
  }
  w.arr(h.chain_start.data(), h.chain_start.size());
  w.arr(h.recs.data(), h.recs.size());
  w.arr(h.rec_op.data(), h.rec_op.size());
  w.arr(h.op_ids.data(), h.n_ops);
  if (!compact) {
    w.arr(h.op_rec.data(), h.n_ops);
    w.arr(h.op_call.data(), h.n_ops);
    w.arr(h.op_ret.data(), h.n_ops);
  }
}

struct Reader {
  const uint8_t* p;
  const uint8_t* end;
  bool ok = true;
  template <typename T>
  void arr(std::vector<T>& v, uint64_t n) {
    const uint64_t b = n * sizeof(T);
    if (!ok || n > (uint64_t)(end - p) / sizeof(T) || pad8(b) > (uint64_t)(end - p)) { ok = false; return; }
    v.resize(n);
    if (n) memcpy(v.data(), p, b);
    p += pad8(b);
  }
};

// One history from its section [p, end); false on a malformed section.
bool read_section(const uint8_t* p, const uint8_t* end, History& h) {
  if ((size_t)(end - p) < sizeof(Head)) return false;
  Head hd;
  memcpy(&hd, p, sizeof hd);
  if (hd.mode > 1 || hd.K == 0xFFFFFFFFu) return false;
  Reader r{p + sizeof hd, end};
  std::vector<int64_t> client;
  if (hd.mode == 0) r.arr(client, hd.n_events);
  else r.arr(h.events, hd.n_events);
  r.arr(h.pool, hd.n_pool);
  h.tokens.clear();
  h.tok_ix.clear();
  h.tok_ix_n = 0;
  for (uint32_t i = 0; i < hd.n_tokens && r.ok; ++i) {
    uint32_t len = 0;
    if ((size_t)(end - r.p) < 4) { r.ok = false; break; }
    memcpy(&len, r.p, 4);
    if (pad8(4 + (size_t)len) > (size_t)(end - r.p)) { r.ok = false; break; }
    h.tokens.emplace_back(reinterpret_cast<const char*>(r.p + 4), len);
    r.p += pad8(4 + (size_t)len);
  }
  r.arr(h.chain_start, hd.n_cs);
  r.arr(h.recs, hd.n_recs);
  r.arr(h.rec_op, hd.n_recs);
  r.arr(h.op_ids, hd.n_ops);
  if (hd.mode == 1) {
    r.arr(h.op_rec, hd.n_ops);
    r.arr(h.op_call, hd.n_ops);
    r.arr(h.op_ret, hd.n_ops);
  }
  if (!r.ok) return false;
  h.status = (int)hd.status;
  h.structural = (int)hd.structural;
  h.n_ops = hd.n_ops;
  h.n_ident = hd.n_ident;
  h.K = hd.K;
  h.hflags = (uint16_t)hd.hflags;
  h.max_chain_len = hd.max_chain_len;
  const bool searchable = hd.status == 0 && hd.structural == 0;
  if (searchable && hd.mode == 1 && hd.n_cs == 0 && hd.n_recs == 0 && hd.K == 0) {
    // a duplicate-id history (History::literal): no chains; its porcupine
    // linking is rebuilt from the events by finalize, which must agree
    for (const Event& e : h.events)
      if (!pool_range_ok(e.hash_off, e.hash_cnt, hd.n_pool) || e.set_tok > hd.n_tokens || e.batch_tok > hd.n_tokens) return false;
    const uint32_t n_ops = hd.n_ops;
    const std::vector<int64_t> ids = h.op_ids;
    if (h.finalize() != 0 || !h.literal || h.n_ops != n_ops || h.op_ids != ids) return false;
    return true;
  }
  if (!searchable) {
    // the check never reads records here (the verdict is fixed or the history
    // refused); only what the event API reads must be in range
    if (hd.mode != 1 || hd.n_cs || hd.n_recs) return false;
    for (const Event& e : h.events)
      if (!pool_range_ok(e.hash_off, e.hash_cnt, hd.n_pool) || e.set_tok > hd.n_tokens || e.batch_tok > hd.n_tokens) return false;
    return true;
  }
  // the index arrays must stay inside the tables they index (the checker
  // trusts them): chain starts ascending within the records (each chain ends
  // with its sentinel), record hashes within the pool, op maps within range
  // (n_recs = n_ops + K with exactly K sentinels: one per chain, at its end;
  // the chain-length bound of the device's u16 counters is recomputed)
  if (hd.n_cs != (uint64_t)hd.K + 1 || h.chain_start[0] != 0 || h.chain_start[h.K] != hd.n_recs ||
      hd.n_recs != (uint64_t)hd.n_ops + hd.K)
    return false;
  uint32_t mcl = 0;
  for (uint32_t q = 0; q < h.K; ++q) {
    if (h.chain_start[q + 1] <= h.chain_start[q] || !(h.recs[h.chain_start[q + 1] - 1].flags & OPF_SENTINEL)) return false;
    mcl = std::max<uint32_t>(mcl, h.chain_start[q + 1] - h.chain_start[q] - 1);
  }
  if (mcl != hd.max_chain_len) return false;
  uint32_t n_e = 0;
  for (const OpRec& o : h.recs) n_e += (!(o.flags & OPF_SENTINEL) && (o.flags & OPF_CLS_E)) ? 1u : 0u;
  if (n_e != hd.n_ident) return false;
  for (const OpRec& o : h.recs)
    if (!pool_range_ok(o.hash_off, o.hash_cnt, hd.n_pool) || o.set_tok > hd.n_tokens || o.batch_tok > hd.n_tokens ||
        (!(o.flags & OPF_SENTINEL) && (o.call_ev >= hd.n_events || o.ret_ev >= hd.n_events)))
      return false;
  std::vector<uint32_t> orec(hd.n_ops, UINT32_MAX);
  for (uint64_t x = 0; x < hd.n_recs; ++x) {
    const uint32_t d = h.rec_op[x];
    if (d == UINT32_MAX) {  // a sentinel, exactly as finalize writes it (the kernels stop at it)
      const OpRec& o = h.recs[x];
      if (o.flags != OPF_SENTINEL || o.call_ev != EV_INF || o.ret_ev != EV_INF || o.sufmin != REQ_NONE) return false;
      continue;
    }
    if (d >= hd.n_ops || orec[d] != UINT32_MAX || (h.recs[x].flags & OPF_SENTINEL)) return false;
    orec[d] = (uint32_t)x;
  }
  for (uint32_t d = 0; d < hd.n_ops; ++d)
    if (orec[d] == UINT32_MAX) return false;
  if (hd.mode == 1) {
    for (uint32_t d = 0; d < hd.n_ops; ++d)
      if (h.op_rec[d] != orec[d] || h.op_call[d] != h.recs[orec[d]].call_ev || h.op_ret[d] != h.recs[orec[d]].ret_ev)
        return false;
  } else {
    h.op_rec.swap(orec);
    h.op_call.resize(hd.n_ops);
    h.op_ret.resize(hd.n_ops);
    for (uint32_t d = 0; d < hd.n_ops; ++d) {
      h.op_call[d] = h.recs[h.op_rec[d]].call_ev;
      h.op_ret[d] = h.recs[h.op_rec[d]].ret_ev;
    }
  }
  if (hd.mode == 0) {
    // every event is one op's call or return: the list is built on first use
    if (hd.n_events != 2ull * hd.n_ops) return false;
    std::vector<uint8_t> seen(hd.n_events, 0);
    for (uint32_t d = 0; d < hd.n_ops; ++d) {
      const uint32_t c = h.op_call[d], t = h.op_ret[d];
      if (seen[c] || seen[t] || c == t) return false;
      seen[c] = seen[t] = 1;
    }
    h.events.clear();
    h.lazy_client = std::move(client);
    h.lazy_once = std::make_unique<std::once_flag>();
  } else {
    for (const Event& e : h.events)
      if (!pool_range_ok(e.hash_off, e.hash_cnt, hd.n_pool) || e.set_tok > hd.n_tokens || e.batch_tok > hd.n_tokens) return false;
    // the searched records must be the events' own (rec_of): witness
    // certification replays the record table, so a section whose records and
    // events disagree would certify a history other than the one the event
    // API shows. Every field but sufmin (the chain's P1 bound).
    for (uint32_t d = 0; d < hd.n_ops; ++d) {
      const OpRec a = h.rec_of(d), &b = h.recs[h.op_rec[d]];
      if (a.num_records != b.num_records || a.msn != b.msn || a.out_tail != b.out_tail || a.out_hash != b.out_hash ||
          a.call_ev != b.call_ev || a.ret_ev != b.ret_ev || a.hash_off != b.hash_off || a.hash_cnt != b.hash_cnt ||
          a.batch_tok != b.batch_tok || a.set_tok != b.set_tok || a.flags != b.flags)
        return false;
    }
  }
  return true;
}

}  // namespace

void History::ensure_events() const {
  if (!lazy_once) return;
  std::call_once(*lazy_once, [this]() {
    std::vector<Event> ev(lazy_client.size());
    for (uint32_t d = 0; d < n_ops; ++d)
      event_pair(*this, d, lazy_client[op_call[d]], lazy_client[op_ret[d]], ev[op_call[d]], ev[op_ret[d]]);
    events.swap(ev);
  });
}

}  // namespace s2lc

using namespace s2lc;

extern "C" {

int s2lc_history_save_many(const s2lc_history* const* hs, size_t n, uint8_t** out, size_t* out_len) {
  if (!out || !out_len || (n && !hs)) return S2LC_EINVAL;
  *out = nullptr;
  *out_len = 0;
  try {
    std::vector<uint64_t> off(n + 1, 0);
    std::vector<uint8_t> compact(n, 0);
    for (size_t i = 0; i < n; ++i)
      if (!hs[i]) return S2LC_EINVAL;
    parallel_for(n, 64, [&](size_t i) { compact[i] = compactable(hs[i]->h) ? 1 : 0; });
    for (size_t i = 0; i < n; ++i) off[i + 1] = off[i] + section_bytes(hs[i]->h, compact[i]);
    const size_t head = 8 + 4 + 4 + 8 + 8 * (n + 1);
    const size_t len = pad8(head) + off[n];
    uint8_t* buf = (uint8_t*)malloc(len ? len : 1);
    if (!buf) return S2LC_ENOMEM;
    memcpy(buf, kMagic, 8);
    const uint32_t ver = kVersion, esz = (uint32_t)sizeof(Event);
    const uint64_t nn = n;
    memcpy(buf + 8, &ver, 4);
    memcpy(buf + 12, &esz, 4);
    memcpy(buf + 16, &nn, 8);
    memcpy(buf + 24, off.data(), 8 * (n + 1));
    memset(buf + head, 0, pad8(head) - head);
    uint8_t* payload = buf + pad8(head);
    parallel_for(n, 64, [&](size_t i) { write_section(hs[i]->h, compact[i], payload + off[i]); });
    *out = buf;
    *out_len = len;
    return 0;
  } catch (...) {
    return S2LC_ENOMEM;
  }
}

int s2lc_history_load_many(const uint8_t* buf, size_t len, int n_threads, s2lc_history** out, size_t cap, size_t* n) {
  if (!buf || !n) return S2LC_EINVAL;
  *n = 0;
  if (len < 24 || memcmp(buf, kMagic, 8) != 0) return S2LC_EDECODE;
  uint32_t ver = 0, esz = 0;
  uint64_t nn = 0;
  memcpy(&ver, buf + 8, 4);
  memcpy(&esz, buf + 12, 4);
  memcpy(&nn, buf + 16, 8);
  if (ver != kVersion || esz != sizeof(Event)) return S2LC_EDECODE;
  if (nn > (len - 24) / 8) return S2LC_EDECODE;
  const size_t head = 8 + 4 + 4 + 8 + 8 * (nn + 1);
  if (pad8(head) > len) return S2LC_EDECODE;
  *n = (size_t)nn;
  if (!out) return 0;  // size query
  if (cap < nn) return S2LC_EINVAL;
  std::vector<uint64_t> off(nn + 1);
  memcpy(off.data(), buf + 24, 8 * (nn + 1));
  const uint8_t* payload = buf + pad8(head);
  const uint64_t plen = len - pad8(head);
  for (uint64_t i = 0; i < nn; ++i)
    if (off[i] > off[i + 1] || off[i + 1] > plen || (off[i] & 7)) return S2LC_EDECODE;
  for (uint64_t i = 0; i < nn; ++i) out[i] = nullptr;
  std::atomic<int> bad{0};
  std::vector<s2lc_history*> pre(nn, nullptr);
  try {
    history_acquire_many(nn, pre.data());
  } catch (...) {
    *n = 0;
    return S2LC_ENOMEM;
  }
  auto one = [&](size_t i) {
    if (bad.load(std::memory_order_relaxed)) return;
    try {
      s2lc_history* h = pre[i];  // (stays in pre[] until it is out[i] or released: an exception leaks nothing)
      const bool ok = read_section(payload + off[i], payload + off[i + 1], h->h);
      pre[i] = nullptr;
      if (!ok) {
        history_release(h);
        bad = S2LC_EDECODE;
        return;
      }
      out[i] = h;
    } catch (...) {
      bad = S2LC_ENOMEM;
    }
  };
  if (n_threads == 1) {
    for (size_t i = 0; i < nn; ++i) one(i);
  } else {
    parallel_for(nn, 64, one);
  }
  for (uint64_t i = 0; i < nn; ++i) history_release(pre[i]);  // (taken up front, not reached)
  if (bad) {
    for (uint64_t i = 0; i < nn; ++i) {
      history_release(out[i]);
      out[i] = nullptr;
    }
    *n = 0;
    return bad;
  }
  return 0;
}

}  // extern "C"
