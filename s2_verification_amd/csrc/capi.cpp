// capi.cpp — the extern "C" boundary (include/s2lincheck.h). No exception
// crosses it; every failure becomes a negative status + message.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <memory>
#include <new>
#include <stddef.h>
#include <atomic>
#include <string>
#include <thread>
#include <stdexcept>
#include <unordered_map>
#include <vector>

#include "history.h"
#include "s2lincheck.h"
#include "search.h"
#include "cert_prof.h"
#include "host_par.h"

namespace s2lc {
int simulate(const s2lc_sim_params& p, History* h, std::string* jsonl);
}

using namespace s2lc;


// One device shard of a context: its stream and a scratch batch reused by
// every s2lc_check / s2lc_check_batch (no device allocation per call once the
// scratch has grown to the working set).
struct Shard {
  int device = 0;
  hipStream_t stream = nullptr;
  bool own_stream = false;
  DevBatch scratch;
  RunStats stats;
  std::string err;
};

struct s2lc_ctx {
  int device = 0;
  hipStream_t stream = nullptr;
  bool own_stream = false;
  uint32_t flags = 0;
  uint64_t max_configs = 0;
  uint64_t timeout_us = 0;
  uint32_t engine = S2LC_ENGINE_AUTO;
  uint32_t red_off = 0;
  std::vector<int> devices;                    // s2lc_check_batch shards (>= 1 entries)
  std::vector<std::unique_ptr<Shard>> shards;  // created lazily, one per devices entry
  std::string err;

  RunOpts run_opts() const {
    RunOpts r;
    r.max_configs = max_configs;
    r.witness = !(flags & S2LC_F_NO_WITNESS);
    r.round_counts = (flags & S2LC_F_ROUND_COUNTS) != 0;
    r.engine = engine;
    r.timeout_us = timeout_us;
    return r;
  }
};

struct s2lc_batch {
  DevBatch b;
  RunStats stats;
  bool ran = false;
  bool witness = false;
  // s2lc_batch_run_totals
  uint64_t runs = 0;
  double kernel_ms_sum = 0, pack16_ms_sum = 0, pack8_ms_sum = 0;
};

static void set_err(char* err, size_t errlen, const std::string& msg) {
  if (err && errlen) {
    size_t n = std::min(errlen - 1, msg.size());
    memcpy(err, msg.data(), n);
    err[n] = 0;
  }
}

extern "C" {

const char* s2lc_version(void) { return "s2lincheck 0.2.0 (gfx950, ABI 2)"; }

s2lc_ctx* s2lc_create(const s2lc_opts* opts, int* status) {
  s2lc_ctx* c = nullptr;
  static const bool timing = getenv("S2LC_CREATE_TIMING") != nullptr;  // diagnostics
  const int64_t t0 = timing ? steady_ns() : 0;
  try {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || n <= 0) {
      if (status) *status = S2LC_ENODEV;
      return nullptr;
    }
    c = new s2lc_ctx();
    int dev = -1;
    if (opts && opts->struct_size >= offsetof(s2lc_opts, flags)) dev = opts->device;
    if (dev < 0) {
      if (hipGetDevice(&dev) != hipSuccess) dev = 0;
    }
    if (dev >= n) { delete c; if (status) *status = S2LC_ENODEV; return nullptr; }
    if (hipSetDevice(dev) != hipSuccess) { delete c; if (status) *status = S2LC_EHIP; return nullptr; }
    c->device = dev;
    // ABI 1 callers pass the layout up to `stream`; the ABI 2 fields keep their defaults
    if (opts && opts->struct_size >= offsetof(s2lc_opts, timeout_us)) {
      c->flags = opts->flags;
      c->max_configs = opts->max_configs;
      c->stream = (hipStream_t)opts->stream;
    }
    if (opts && opts->struct_size >= sizeof(s2lc_opts)) {
      c->timeout_us = opts->timeout_us;
      c->engine = opts->engine;
      c->red_off = opts->reductions_off;
      if (c->engine > S2LC_ENGINE_LEVEL) { delete c; if (status) *status = S2LC_EINVAL; return nullptr; }
      if (opts->devices && opts->n_devices) {
        if (opts->n_devices > 16) { delete c; if (status) *status = S2LC_EINVAL; return nullptr; }
        for (uint32_t i = 0; i < opts->n_devices; ++i) {
          const int d = opts->devices[i];
          if (d < 0 || d >= n) { delete c; if (status) *status = S2LC_ENODEV; return nullptr; }
          c->devices.push_back(d);
        }
      }
    }
    if (c->devices.empty()) c->devices.push_back(dev);
    const int64_t t1 = timing ? steady_ns() : 0;
    if (!c->stream) {
      if (hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) != hipSuccess) {
        delete c;
        if (status) *status = S2LC_EHIP;
        return nullptr;
      }
      c->own_stream = true;
    }
    if (timing)
      fprintf(stderr, "{\"s2lc_create_ms\":{\"runtime_init\":%.2f,\"stream\":%.2f}}\n", 1e-6 * (t1 - t0),
              1e-6 * (steady_ns() - t1));
  } catch (...) {
    delete c;
    if (status) *status = S2LC_ENOMEM;
    return nullptr;
  }
  if (status) *status = 0;
  return c;
}

void s2lc_destroy(s2lc_ctx* c) {
  if (!c) return;
  for (auto& sh : c->shards) {
    if (!sh) continue;
    (void)hipSetDevice(sh->device);
    batch_release(sh->scratch);
    if (sh->own_stream && sh->stream) (void)hipStreamDestroy(sh->stream);
  }
  (void)hipSetDevice(c->device);
  if (c->own_stream && c->stream) (void)hipStreamDestroy(c->stream);
  delete c;
}

const char* s2lc_last_error(const s2lc_ctx* c) { return c ? c->err.c_str() : "null context"; }

// ------------------------------------------------------------- histories ---
int s2lc_load_jsonl(const char* path, const uint8_t* buf, size_t len, s2lc_history** out, char* err,
                    size_t errlen) {
  if (!out) return S2LC_EINVAL;
  *out = nullptr;
  try {
    std::vector<uint8_t> data;
    if (!buf) {
      if (!path) return S2LC_EINVAL;
      FILE* f = strcmp(path, "-") == 0 ? stdin : fopen(path, "rb");
      if (!f) {
        set_err(err, errlen, std::string("open ") + path + ": " + strerror(errno));
        return S2LC_EIO;
      }
      uint8_t tmp[1 << 16];
      size_t n;
      while ((n = fread(tmp, 1, sizeof tmp, f)) > 0) data.insert(data.end(), tmp, tmp + n);
      const bool bad = ferror(f);
      if (f != stdin) fclose(f);
      if (bad) { set_err(err, errlen, std::string("read ") + path); return S2LC_EIO; }
      buf = data.data();
      len = data.size();
    }
    s2lc_history* h = history_acquire();
    std::string e;
    const int rc = load_jsonl_finalized(buf, len, h->h, e);
    if (rc) { set_err(err, errlen, e); history_release(h); return rc; }
    *out = h;
    return 0;
  } catch (const std::bad_alloc&) {
    set_err(err, errlen, "out of memory");
    return S2LC_ENOMEM;
  } catch (...) {
    set_err(err, errlen, "internal error");
    return S2LC_EINVAL;
  }
}

int s2lc_load_jsonl_many(const uint8_t* const* bufs, const size_t* lens, size_t n, int n_threads,
                         s2lc_history** out, size_t* err_index, char* err, size_t errlen) {
  if (!out || (n && (!bufs || !lens))) return S2LC_EINVAL;
  for (size_t i = 0; i < n; ++i) out[i] = nullptr;
  if (n_threads <= 0) n_threads = (int)std::max(1u, std::thread::hardware_concurrency());
  n_threads = (int)std::min<size_t>((size_t)n_threads, std::max<size_t>(n, 1));
  std::atomic<size_t> next{0};
  std::atomic<size_t> first_bad{SIZE_MAX};
  std::vector<int> rcs(n, 0);
  std::vector<std::string> errs(n);
  std::vector<s2lc_history*> pre(n, nullptr);
  try {
    history_acquire_many(n, pre.data());
  } catch (...) {
    set_err(err, errlen, "out of memory");
    return S2LC_ENOMEM;
  }
  auto work = [&]() {
    for (;;) {
      const size_t i = next.fetch_add(1);
      if (i >= n) return;
      try {
        s2lc_history* h = pre[i];  // (stays in pre[] until it is out[i] or released: an exception leaks nothing)
        const int rc = load_jsonl_finalized(bufs[i], lens[i], h->h, errs[i]);
        pre[i] = nullptr;
        if (rc) {
          history_release(h);
          rcs[i] = rc;
          size_t cur = first_bad.load();
          while (i < cur && !first_bad.compare_exchange_weak(cur, i)) {}
        } else {
          out[i] = h;
        }
      } catch (...) {
        rcs[i] = S2LC_ENOMEM;
        errs[i] = "out of memory";
        size_t cur = first_bad.load();
        while (i < cur && !first_bad.compare_exchange_weak(cur, i)) {}
      }
    }
  };
  std::vector<std::thread> ts;
  for (int t = 1; t < n_threads; ++t) ts.emplace_back(work);
  work();
  for (auto& t : ts) t.join();
  const size_t bad = first_bad.load();
  for (size_t i = 0; i < n; ++i) history_release(pre[i]);  // (taken up front, not reached)
  if (bad != SIZE_MAX) {
    for (size_t i = 0; i < n; ++i) {
      history_release(out[i]);
      out[i] = nullptr;
    }
    if (err_index) *err_index = bad;
    set_err(err, errlen, "history " + std::to_string(bad) + ": " + errs[bad]);
    return rcs[bad];
  }
  return 0;
}

int s2lc_history_from_events(const s2lc_event* ev, size_t n, s2lc_history** out, char* err, size_t errlen) {
  if (!out || (!ev && n)) return S2LC_EINVAL;
  *out = nullptr;
  try {
    s2lc_history* h = history_acquire();
    History& H = h->h;
    H.events.reserve(n);
    for (size_t i = 0; i < n; ++i) {
      const s2lc_event& x = ev[i];
      Event e;
      if (x.kind != S2LC_CALL_EVENT && x.kind != S2LC_RETURN_EVENT) {
        set_err(err, errlen, "event " + std::to_string(i) + ": bad kind");
        history_release(h);
        return S2LC_EINVAL;
      }
      e.kind = x.kind;
      e.op_id = x.op_id;
      e.client_id = x.client_id;
      if (x.kind == S2LC_CALL_EVENT) {
        e.input_type = x.input_type;
        e.has_num_records = x.has_num_records;
        e.num_records = x.num_records;
        e.has_msn = x.has_match_seq_num;
        e.msn = x.match_seq_num;
        e.set_tok = x.set_fencing_token ? H.intern(x.set_fencing_token) : 0;
        e.batch_tok = x.fencing_token ? H.intern(x.fencing_token) : 0;
        e.hash_off = H.pool.size();
        e.hash_cnt = x.n_record_hashes;
        if (x.n_record_hashes) {
          if (!x.record_hashes) { history_release(h); set_err(err, errlen, "null record_hashes"); return S2LC_EINVAL; }
          H.pool.insert(H.pool.end(), x.record_hashes, x.record_hashes + x.n_record_hashes);
        }
      } else {
        e.failure = x.failure;
        e.definite = x.definite_failure;
        e.has_tail = x.has_tail;
        e.tail = x.tail;
        e.has_hash = x.has_stream_hash;
        e.stream_hash = x.stream_hash;
      }
      H.events.push_back(e);
    }
    int rc = H.finalize();
    if (rc) { set_err(err, errlen, H.error); history_release(h); return rc; }
    *out = h;
    return 0;
  } catch (const std::bad_alloc&) {
    set_err(err, errlen, "out of memory");
    return S2LC_ENOMEM;
  } catch (...) {
    set_err(err, errlen, "internal error");
    return S2LC_EINVAL;
  }
}

void s2lc_history_free(s2lc_history* h) { history_release(h); }
size_t s2lc_history_pool_trim(void) { return history_pool_trim(); }

size_t s2lc_history_event_count(const s2lc_history* h) { return h ? h->h.n_events() : 0; }

int s2lc_history_get_event(const s2lc_history* h, size_t i, s2lc_event* out) {
  if (!h || !out || i >= h->h.n_events()) return S2LC_EINVAL;
  h->h.ensure_events();
  const History& H = h->h;
  const Event& e = H.events[i];
  memset(out, 0, sizeof *out);
  out->kind = e.kind;
  out->op_id = e.op_id;
  out->client_id = e.client_id;
  if (e.kind == 0) {
    out->input_type = e.input_type;
    out->has_num_records = e.has_num_records;
    out->num_records = e.num_records;
    out->has_match_seq_num = e.has_msn;
    out->match_seq_num = e.msn;
    out->set_fencing_token = e.set_tok ? H.tokens[e.set_tok - 1].c_str() : nullptr;
    out->fencing_token = e.batch_tok ? H.tokens[e.batch_tok - 1].c_str() : nullptr;
    out->record_hashes = e.hash_cnt ? H.pool.data() + e.hash_off : nullptr;
    out->n_record_hashes = e.hash_cnt;
  } else {
    out->failure = e.failure;
    out->definite_failure = e.definite;
    out->has_tail = e.has_tail;
    out->tail = e.tail;
    out->has_stream_hash = e.has_hash;
    out->stream_hash = e.stream_hash;
  }
  return 0;
}

int s2lc_history_get_events(const s2lc_history* h, s2lc_event* out, size_t n) {
  if (!h || (!out && n) || n > h->h.n_events()) return S2LC_EINVAL;
  h->h.ensure_events();
  for (size_t i = 0; i < n; ++i) s2lc_history_get_event(h, i, &out[i]);
  return 0;
}

int s2lc_history_info_get(const s2lc_history* h, s2lc_history_info* out) {
  if (!h || !out) return S2LC_EINVAL;
  const History& H = h->h;
  out->n_events = (uint32_t)H.n_events();
  out->n_ops = H.n_ops;
  out->n_chains = H.K;
  out->n_tokens = (uint32_t)H.tokens.size();
  out->n_record_hashes = H.pool.size();
  out->structural = H.structural;
  out->n_identity_ops = H.n_ident;
  return 0;
}

// --------------------------------------------------------------- checker ---
}  // extern "C"

namespace {

// Results of a run (+ witness rebuild and CPU-model certification) into
// out[0 .. B.n_hist). Every Ok witness must replay through s2Model.Step
// (main.go:264-335); one that does not is a checker bug: that history becomes
// Unknown (S2LC_R_WITNESS_INVALID) and the call returns S2LC_EWITNESS.
// flat_ids (nullable): Ok witnesses go straight to flat_ids + flat_offs[i]
// (no per-history allocation; out[i].witness stays null, witness_len is set).
int collect_results(DevBatch& B, const RunStats& stats, bool witness_recorded, s2lc_result* out, int with_witness,
                    std::string& err, int64_t* flat_ids = nullptr, const uint64_t* flat_offs = nullptr) {
  const bool want_w = with_witness && witness_recorded;
  CP_DECL(tc0);
  {
    const int rc = batch_host_results(B, err);
    if (rc) return rc;
  }
  if (want_w && B.n_hist) {
    const int rc = batch_fetch_moves(B, err);
    if (rc) return rc;
  }
  // test hook: corrupt every Ok witness before certification (the failure path
  // of the certificate must be loud; tests/test_gpu.py)
  CP_LAP(5, tc0);
  const char* fault = getenv("S2LC_FAULT_WITNESS");
  const bool corrupt = fault && fault[0] == '1';
  std::atomic<uint32_t> next{0};
  std::atomic<int> oom{0}, invalid{0};
  auto work = [&]() {
    std::vector<uint32_t> order, mv;
    std::vector<uint8_t> ident;
    for (;;) {
      const uint32_t i = next.fetch_add(1);
      if (i >= B.n_hist) return;
      const HistResult& r = B.h_res[i];
      s2lc_result& o = out[i];
      memset(&o, 0, sizeof o);
      o.verdict = (int32_t)r.verdict;
      o.reason = (int32_t)r.reason;
      o.configs_explored = r.configs;
      o.rounds = r.rounds;
      o.n_ops = B.src[i]->n_ops;
      o.device_ms = stats.kernel_ms;
      if (!want_w || r.has_witness != 1 || (r.verdict != V_OK && r.verdict != V_ILLEGAL)) continue;
      const History& H = *B.src[i];
      const uint32_t* moves = B.h_moves + r.witness_off;
      try {
        if (corrupt && r.verdict == V_OK) {
          mv.assign(moves, moves + r.witness_len);
          if (mv.empty()) mv.push_back(0xFFFFu); else mv[0] = 0xFFFFu;  // no such chain
          moves = mv.data();
        }
        const uint32_t n_moves = corrupt && r.verdict == V_OK ? (uint32_t)mv.size() : r.witness_len;
        if (H.literal) {
          // the literal engine wrote the call events of porcupine's calls
          // stack; ops are the call events in order (History::op_call)
          if (r.verdict != V_OK) continue;
          order.resize(n_moves);
          bool ok = true;
          for (uint32_t k = 0; k < n_moves && ok; ++k) {
            const auto it = std::lower_bound(H.op_call.begin(), H.op_call.end(), moves[k]);
            ok = it != H.op_call.end() && *it == moves[k];
            if (ok) order[k] = (uint32_t)(it - H.op_call.begin());
          }
          if (!ok || !replay_literal(H, order.data(), order.size())) {
            o.verdict = S2LC_UNKNOWN;
            o.reason = S2LC_R_WITNESS_INVALID;
            invalid = 1;
            continue;
          }
          if (flat_ids) {
            int64_t* w = flat_ids + flat_offs[i];
            for (size_t k = 0; k < order.size(); ++k) w[k] = H.op_ids[order[k]];
            o.witness_len = (uint32_t)order.size();
            continue;
          }
          o.witness = (int64_t*)malloc(sizeof(int64_t) * (order.size() ? order.size() : 1));
          if (!o.witness) { oom = 1; continue; }
          for (size_t k = 0; k < order.size(); ++k) o.witness[k] = H.op_ids[order[k]];
          o.witness_len = (uint32_t)order.size();
          continue;
        }
        if (r.verdict == V_OK) {
          CP_DECL(th0);
          const bool ok = rebuild_and_replay(H, moves, n_moves, r.p4 != 0, order, ident);
          CP_LAP(3, th0);
          if (!ok) {
            o.verdict = S2LC_UNKNOWN;
            o.reason = S2LC_R_WITNESS_INVALID;
            invalid = 1;
            continue;
          }
          if (flat_ids) {
            int64_t* w = flat_ids + flat_offs[i];
            for (size_t k = 0; k < order.size(); ++k) w[k] = H.op_ids[order[k]];
            o.witness_len = (uint32_t)order.size();
            CP_LAP(4, th0);
#ifdef S2LC_CERT_PROF
            g_cert_prof[7].fetch_add(1);
#endif
            continue;
          }
          o.witness = (int64_t*)malloc(sizeof(int64_t) * (order.size() ? order.size() : 1));
          if (!o.witness) { oom = 1; continue; }
          for (size_t k = 0; k < order.size(); ++k) o.witness[k] = H.op_ids[order[k]];
          o.witness_len = (uint32_t)order.size();
        } else if (flat_ids) {
          continue;  // (the flat form carries no Illegal partials)
        } else if (rebuild_linearization(H, moves, n_moves, false, order, ident, true) &&
                   replay_prefix(H, order.data(), ident.data(), order.size())) {
          o.partial = (int64_t*)malloc(sizeof(int64_t) * (order.size() ? order.size() : 1));
          if (!o.partial) { oom = 1; continue; }
          for (size_t k = 0; k < order.size(); ++k) o.partial[k] = H.op_ids[order[k]];
          o.partial_len = (uint32_t)order.size();
        }
      } catch (...) {
        oom = 1;
      }
    }
  };
  // Witness rebuild + certification is independent per history: worker
  // threads (S2LC_THREADS, default min(16, cores)).
  int n_threads = 1;
  if (want_w) {
    const char* e = getenv("S2LC_THREADS");
    n_threads = e ? atoi(e) : (int)std::min(16u, std::max(1u, std::thread::hardware_concurrency()));
    n_threads = std::max(1, std::min<int>(n_threads, (int)(B.n_hist / 64 + 1)));
  }
  std::vector<std::thread> ts;
  for (int t = 1; t < n_threads; ++t) ts.emplace_back(work);
  work();
  for (auto& t : ts) t.join();
#ifdef S2LC_CERT_PROF
  CP_LAP(6, tc0);
  fprintf(stderr, "{\"cert_prof\": [");
  for (int k = 0; k < 16; ++k) fprintf(stderr, "%s%llu", k ? ", " : "", (unsigned long long)g_cert_prof[k].exchange(0));
  fprintf(stderr, "], \"threads\": %d}\n", n_threads);
#endif
  if (oom) { err = "out of memory"; return S2LC_ENOMEM; }
  if (invalid) { err = "an Ok witness failed CPU-model certification (checker bug)"; return S2LC_EWITNESS; }
  return 0;
}

Shard& shard_of(s2lc_ctx* c, size_t k) {
  if (c->shards.size() < c->devices.size()) c->shards.resize(c->devices.size());
  if (!c->shards[k]) {
    auto sh = std::make_unique<Shard>();
    sh->device = c->devices[k];
    sh->scratch.device = sh->device;
    if (k == 0 && sh->device == c->device) {
      sh->stream = c->stream;  // the context's (or caller's) stream
    } else {
      if (hipSetDevice(sh->device) != hipSuccess || hipStreamCreateWithFlags(&sh->stream, hipStreamNonBlocking) != hipSuccess)
        throw std::runtime_error("stream");
      sh->own_stream = true;
    }
    c->shards[k] = std::move(sh);
  }
  return *c->shards[k];
}

// upload + run + results of `hs` on one shard, into out[0 .. hs.size())
int shard_check(s2lc_ctx* c, Shard& sh, const std::vector<const History*>& hs, s2lc_result* out) {
  if (hipSetDevice(sh.device) != hipSuccess) { sh.err = "hipSetDevice failed"; return S2LC_EHIP; }
  const RunOpts ro = c->run_opts();
  int rc = batch_upload(sh.scratch, hs, c->red_off, sh.err);
  if (!rc) rc = batch_run(sh.scratch, sh.stream, ro, sh.stats, sh.err);
  if (!rc) rc = collect_results(sh.scratch, sh.stats, ro.witness, out, 1, sh.err);
  return rc;
}

}  // namespace

extern "C" {

int s2lc_batch_create(s2lc_ctx* c, const s2lc_history* const* hs, size_t n, s2lc_batch** out) {
  if (!c || !out || (!hs && n)) return S2LC_EINVAL;
  *out = nullptr;
  try {
    if (hipSetDevice(c->device) != hipSuccess) { c->err = "hipSetDevice failed"; return S2LC_EHIP; }
    s2lc_batch* b = new s2lc_batch();
    b->b.device = c->device;
    std::vector<const History*> v(n);
    for (size_t i = 0; i < n; ++i) {
      if (!hs[i]) { delete b; c->err = "null history"; return S2LC_EINVAL; }
      v[i] = &hs[i]->h;
    }
    std::string e;
    int rc = batch_upload(b->b, v, c->red_off, e);
    if (rc) { c->err = e; batch_release(b->b); delete b; return rc; }
    *out = b;
    return 0;
  } catch (const std::bad_alloc&) {
    c->err = "out of memory";
    return S2LC_ENOMEM;
  } catch (...) {
    c->err = "internal error";
    return S2LC_EINVAL;
  }
}

int s2lc_batch_load(s2lc_ctx* c, s2lc_batch* b, const s2lc_history* const* hs, size_t n) {
  if (!c || !b || (!hs && n)) return S2LC_EINVAL;
  try {
    if (hipSetDevice(b->b.device) != hipSuccess) { c->err = "hipSetDevice failed"; return S2LC_EHIP; }
    std::vector<const History*> v(n);
    for (size_t i = 0; i < n; ++i) {
      if (!hs[i]) { c->err = "null history"; return S2LC_EINVAL; }
      v[i] = &hs[i]->h;
    }
    b->ran = false;
    return batch_upload(b->b, v, c->red_off, c->err);
  } catch (const std::bad_alloc&) {
    c->err = "out of memory";
    return S2LC_ENOMEM;
  } catch (...) {
    c->err = "internal error";
    return S2LC_EINVAL;
  }
}

void s2lc_batch_free(s2lc_batch* b) {
  if (!b) return;
  (void)hipSetDevice(b->b.device);
  batch_release(b->b);
  delete b;
}

int s2lc_batch_run(s2lc_ctx* c, s2lc_batch* b) {
  if (!c || !b) return S2LC_EINVAL;
  try {
    if (hipSetDevice(b->b.device) != hipSuccess) { c->err = "hipSetDevice failed"; return S2LC_EHIP; }
    const RunOpts ro = c->run_opts();
    std::string e;
    int rc = batch_run(b->b, c->stream, ro, b->stats, e);
    if (rc) { c->err = e; return rc; }
    b->ran = true;
    b->witness = ro.witness;
    b->runs++;
    b->kernel_ms_sum += b->stats.kernel_ms;
    b->pack16_ms_sum += b->stats.pack16_ms;
    b->pack8_ms_sum += b->stats.pack8_ms;
    return 0;
  } catch (...) {
    c->err = "internal error";
    return S2LC_EINVAL;
  }
}

int s2lc_batch_results_flat(s2lc_ctx* c, s2lc_batch* b, int32_t* verdicts, int32_t* reasons, uint64_t* configs,
                            uint64_t* rounds, int64_t* witness_ids, size_t ids_cap, uint64_t* witness_offs) {
  if (!c || !b || !witness_offs) return S2LC_EINVAL;
  if (!b->ran) { c->err = "batch has not been run"; return S2LC_EINVAL; }
  try {
    if (hipSetDevice(b->b.device) != hipSuccess) { c->err = "hipSetDevice failed"; return S2LC_EHIP; }
    const size_t n = b->b.n_hist;
    DevBatch& B = b->b;
    std::vector<s2lc_result> res(std::max<size_t>(n, 1));
    // offsets first: a certified Ok witness is every op of its history, so
    // the witnesses are written in place by the certifying threads
    const bool want = witness_ids != nullptr && b->witness;
    if (const int rc0 = batch_host_results(B, c->err)) return rc0;
    uint64_t total = 0;
    for (size_t i = 0; i < n; ++i) {
      witness_offs[i] = total;
      if (want && B.h_res[i].verdict == V_OK && B.h_res[i].has_witness == 1) total += B.src[i]->n_ops;
    }
    witness_offs[n] = total;
    if (want && total > ids_cap) {
      c->err = "witness buffer too small";
      return S2LC_EINVAL;
    }
    const int rc = collect_results(B, b->stats, b->witness, res.data(), witness_ids != nullptr, c->err,
                                   want ? witness_ids : nullptr, witness_offs);
    if (rc && rc != S2LC_EWITNESS) return rc;
    // a witness that failed certification (checker bug: rc = EWITNESS) has no
    // ids: close its gap
    if (want && rc == S2LC_EWITNESS) {
      uint64_t w = 0;
      for (size_t i = 0; i < n; ++i) {
        const uint64_t o = witness_offs[i], len = res[i].witness_len;
        if (w != o && len) memmove(witness_ids + w, witness_ids + o, sizeof(int64_t) * len);
        witness_offs[i] = w;
        w += len;
      }
      witness_offs[n] = w;
    }
    for (size_t i = 0; i < n; ++i) {
      const s2lc_result& r = res[i];
      if (verdicts) verdicts[i] = r.verdict;
      if (reasons) reasons[i] = r.reason;
      if (configs) configs[i] = r.configs_explored;
      if (rounds) rounds[i] = r.rounds;
    }
    return rc;
  } catch (const std::bad_alloc&) {
    c->err = "out of memory";
    return S2LC_ENOMEM;
  } catch (...) {
    c->err = "internal error";
    return S2LC_EINVAL;
  }
}

int s2lc_batch_results(s2lc_ctx* c, s2lc_batch* b, s2lc_result* out, int with_witness) {
  if (!c || !b || (!out && b->b.n_hist)) return S2LC_EINVAL;
  if (!b->ran) { c->err = "batch has not been run"; return S2LC_EINVAL; }
  try {
    if (hipSetDevice(b->b.device) != hipSuccess) { c->err = "hipSetDevice failed"; return S2LC_EHIP; }
    return collect_results(b->b, b->stats, b->witness, out, with_witness, c->err);
  } catch (const std::bad_alloc&) {
    c->err = "out of memory";
    return S2LC_ENOMEM;
  } catch (...) {
    c->err = "internal error";
    return S2LC_EINVAL;
  }
}

int s2lc_batch_check(s2lc_ctx* c, s2lc_batch* b, s2lc_result* out) {
  int rc = s2lc_batch_run(c, b);
  if (rc) return rc;
  return s2lc_batch_results(c, b, out, 1);
}

int s2lc_batch_run_totals(const s2lc_batch* b, uint64_t* runs, double* kernel_ms_sum, double* pack16_ms_sum,
                          double* pack8_ms_sum) {
  if (!b) return S2LC_EINVAL;
  if (runs) *runs = b->runs;
  if (kernel_ms_sum) *kernel_ms_sum = b->kernel_ms_sum;
  if (pack16_ms_sum) *pack16_ms_sum = b->pack16_ms_sum;
  if (pack8_ms_sum) *pack8_ms_sum = b->pack8_ms_sum;
  return 0;
}

int s2lc_batch_stats_get(const s2lc_batch* b, s2lc_batch_stats* out) {
  if (!b || !out) return S2LC_EINVAL;
  out->kernel_ms = b->stats.kernel_ms;
  out->total_ms = b->stats.total_ms;
  out->configs_explored = b->stats.configs;
  out->children_generated = b->stats.children;
  out->rounds = b->stats.rounds;
  out->algo_bytes = b->stats.algo_bytes;
  out->n_overflow = b->stats.n_overflow;
  out->launches = b->stats.launches;
  out->level_ms = b->stats.level.ms;
  out->level_histories = b->stats.level.histories;
  out->level_max_frontier = b->stats.level.max_frontier;
  out->level_rounds = b->stats.level.rounds;
  out->level_configs = b->stats.level.configs;
  out->level_children = b->stats.level.children;
  out->pack16_ms = b->stats.pack16_ms;
  out->pack16_algo_bytes = b->stats.pack16_algo_bytes;
  out->pack16_histories = b->stats.pack16_histories;
  out->pack16_small = b->stats.pack16_small;
  out->level_persist_rounds = b->stats.level.persist_rounds;
  out->level_persist_launches = (uint32_t)b->stats.level.persist_launches;
  out->level_chunk_retries = b->stats.level.chunk_retries;
  out->level_syncs = b->stats.level.syncs;
  out->level_solo_rounds = (uint32_t)b->stats.level.solo_rounds;
  out->n_ops_total = b->b.n_ops_total;
  out->pack8_ms = b->stats.pack8_ms;
  out->pack8_algo_bytes = b->stats.pack8_algo_bytes;
  out->pack8_histories = b->stats.pack8_histories;
  out->level_persist_fallbacks = b->stats.level.persist_fallbacks;
  out->level_narrow_ms = b->stats.level.narrow_ms;
  out->level_wide_ms = b->stats.level.wide_ms;
  out->level_solo_ms = b->stats.level.solo_ms;
  out->level_grows = b->stats.level.grows;
  return 0;
}

int s2lc_batch_round_counts(const s2lc_batch* b, size_t i, uint32_t* out, size_t cap, size_t* n) {
  if (!b || !n || i >= b->b.n_hist) return S2LC_EINVAL;
  const DevBatch& B = b->b;
  if (!b->ran || !B.rc_valid) return S2LC_EINVAL;
  const size_t k = B.forced[i] ? 0 : B.h_res[i].rounds;
  *n = k;
  if (!out) return 0;
  if (cap < k) return S2LC_EINVAL;
  for (size_t r = 0; r < k; ++r) out[r] = B.h_rcounts[B.h_moves_off[i] + r];
  return 0;
}

// porcupine.CheckEventsVerbose over many histories (main.go:606 per history).
// One device: the context's scratch batch. Several (s2lc_opts.devices): the
// histories are placed longest-processing-time first (n_ops x K) on the least
// loaded shard, every shard checks its part on its own thread and device, and
// the verdicts land in out[] in input order.
int s2lc_check_batch(s2lc_ctx* c, const s2lc_history* const* hs, size_t n, s2lc_result* out) {
  if (!c || (!hs && n) || (!out && n)) return S2LC_EINVAL;
  if (n) memset(out, 0, n * sizeof *out);  // (an error below frees whatever was filled in)
  try {
    std::vector<const History*> v(n);
    for (size_t i = 0; i < n; ++i) {
      if (!hs[i]) { c->err = "null history"; return S2LC_EINVAL; }
      v[i] = &hs[i]->h;
    }
    const size_t S = c->devices.size();
    if (S <= 1) {
      Shard& sh = shard_of(c, 0);
      const int rc = shard_check(c, sh, v, out);
      if (rc) c->err = sh.err;
      // like the sharded path: on an error other than a failed certificate
      // nothing is returned, so nothing stays allocated
      if (rc && rc != S2LC_EWITNESS)
        for (size_t i = 0; i < n; ++i) s2lc_result_free(&out[i]);
      return rc;
    }
    // LPT placement
    std::vector<size_t> idx(n);
    for (size_t i = 0; i < n; ++i) idx[i] = i;
    auto work = [&](size_t i) { return (uint64_t)v[i]->n_ops * std::max<uint32_t>(v[i]->K, 1); };
    std::stable_sort(idx.begin(), idx.end(), [&](size_t a, size_t b) { return work(a) > work(b); });
    std::vector<uint64_t> load(S, 0);
    std::vector<std::vector<size_t>> part(S);
    for (size_t i : idx) {
      const size_t k = (size_t)(std::min_element(load.begin(), load.end()) - load.begin());
      part[k].push_back(i);
      load[k] += work(i);
    }
    for (size_t k = 0; k < S; ++k) (void)shard_of(c, k);
    std::vector<std::vector<s2lc_result>> res(S);
    std::vector<int> rcs(S, 0);
    std::vector<std::thread> ts;
    for (size_t k = 0; k < S; ++k) {
      ts.emplace_back([&, k]() {
        try {
          std::vector<const History*> sub;
          for (size_t i : part[k]) sub.push_back(v[i]);
          res[k].resize(sub.size());
          rcs[k] = sub.empty() ? 0 : shard_check(c, *c->shards[k], sub, res[k].data());
        } catch (...) {
          rcs[k] = S2LC_ENOMEM;
          c->shards[k]->err = "out of memory";
        }
      });
    }
    for (auto& t : ts) t.join();
    (void)hipSetDevice(c->device);
    int rc = 0;
    for (size_t k = 0; k < S; ++k)  // verdict gather, input order
      for (size_t q = 0; q < part[k].size(); ++q) out[part[k][q]] = res[k][q];
    for (size_t k = 0; k < S && !rc; ++k)
      if (rcs[k] && rcs[k] != S2LC_EWITNESS) { rc = rcs[k]; c->err = c->shards[k]->err; }
    for (size_t k = 0; k < S && !rc; ++k)
      if (rcs[k]) { rc = rcs[k]; c->err = c->shards[k]->err; }
    if (rc && rc != S2LC_EWITNESS) {
      for (size_t i = 0; i < n; ++i) s2lc_result_free(&out[i]);
    }
    return rc;
  } catch (const std::bad_alloc&) {
    c->err = "out of memory";
    return S2LC_ENOMEM;
  } catch (...) {
    c->err = "internal error";
    return S2LC_EHIP;
  }
}

int s2lc_check(s2lc_ctx* c, const s2lc_history* h, s2lc_result* out) {
  if (!h) return S2LC_EINVAL;
  const s2lc_history* one[1] = {h};
  return s2lc_check_batch(c, one, 1, out);
}

int s2lc_device_fold(s2lc_ctx* c, const uint64_t* seeds, const uint64_t* pool, size_t pool_len, const uint32_t* offs,
                     const uint32_t* cnts, size_t n, uint64_t* out) {
  if (!c || (n && (!seeds || !offs || !cnts || !out)) || (pool_len && !pool)) return S2LC_EINVAL;
  if (hipSetDevice(c->device) != hipSuccess) { c->err = "hipSetDevice failed"; return S2LC_EHIP; }
  return device_fold(seeds, pool, pool_len, offs, cnts, n, out, c->stream, c->err);
}

void s2lc_partials_free(s2lc_partials* p) {
  if (!p) return;
  free(p->op_ids);
  free(p->op_partial);
  free(p->offs);
  free(p->ids);
  memset(p, 0, sizeof *p);
}

int s2lc_check_partials(s2lc_ctx* c, const s2lc_history* h, s2lc_partials* out) {
  if (!c || !h || !out) return S2LC_EINVAL;
  memset(out, 0, sizeof *out);
  const History& H = h->h;
  if (H.status) { c->err = H.error; return H.status; }
  if (H.literal) {  // (porcupine's own partials there come from its id-keyed DFS: not restated)
    c->err = "partial linearizations of histories with duplicate op ids";
    return S2LC_EUNSUPPORTED;
  }
  s2lc_result r;
  int rc = s2lc_check(c, h, &r);
  if (rc) { s2lc_result_free(&r); return rc; }
  out->verdict = r.verdict;
  out->n_ops = H.n_ops;
  out->exact = 1;
  std::vector<uint32_t> op_part(H.n_ops, UINT32_MAX);
  std::vector<uint64_t> offs{0};
  std::vector<int64_t> ids;
  try {
    if (r.verdict == S2LC_OK && r.witness) {
      // porcupine on success: every op's longest partial is the linearization
      ids.assign(r.witness, r.witness + r.witness_len);
      offs.push_back(ids.size());
      std::fill(op_part.begin(), op_part.end(), 0u);
    } else if (r.verdict == S2LC_ILLEGAL && !H.structural && H.n_ops) {
      Shard& sh = shard_of(c, 0);
      if (hipSetDevice(sh.device) != hipSuccess) { c->err = "hipSetDevice failed"; s2lc_result_free(&r); return S2LC_EHIP; }
      DevBatch& B = sh.scratch;
      std::vector<const History*> one{&H};
      rc = batch_upload(B, one, S2LC_RED_P1 | S2LC_RED_P2 | S2LC_RED_P4 | S2LC_RED_IDEFER, sh.err);
      unsigned long long* dmax = nullptr;
      const size_t n_recs = H.recs.size();
      if (!rc && hipMalloc(&dmax, n_recs * sizeof(unsigned long long)) != hipSuccess) { sh.err = "hipMalloc"; rc = S2LC_EHIP; }
      if (!rc && hipMemsetAsync(dmax, 0, n_recs * sizeof(unsigned long long), sh.stream) != hipSuccess) rc = S2LC_EHIP;
      if (!rc) {
        RunOpts ro = c->run_opts();
        ro.engine = S2LC_ENGINE_LEVEL;
        ro.witness = true;
        ro.round_counts = false;
        ro.max_configs = c->max_configs ? c->max_configs : (1ull << 22);
        ro.partial_max = dmax;
        RunStats st;
        rc = batch_run(B, sh.stream, ro, st, sh.err);
      }
      std::vector<unsigned long long> hmax(n_recs, 0);
      std::vector<TraceEnt> tr;
      if (!rc) {
        unsigned long long th = 0;
        if (hipMemcpy(hmax.data(), dmax, n_recs * sizeof(unsigned long long), hipMemcpyDeviceToHost) != hipSuccess ||
            hipMemcpy(&th, B.trace_head, sizeof th, hipMemcpyDeviceToHost) != hipSuccess) {
          sh.err = "hipMemcpy";
          rc = S2LC_EHIP;
        } else {
          tr.resize(std::min<unsigned long long>(th, B.trace_cap));
          if (!tr.empty() && hipMemcpy(tr.data(), B.trace, tr.size() * sizeof(TraceEnt), hipMemcpyDeviceToHost) != hipSuccess) {
            sh.err = "hipMemcpy";
            rc = S2LC_EHIP;
          }
        }
      }
      if (dmax) (void)hipFree(dmax);
      if (rc) { c->err = sh.err; s2lc_result_free(&r); return rc; }
      const uint32_t v2 = B.h_res[0].verdict;
      if (v2 == V_OK) {  // the unreduced search disagrees with the verdict: a checker bug
        c->err = "the unreduced search found a linearization of an Illegal history";
        s2lc_result_free(&r);
        return S2LC_EWITNESS;
      }
      out->exact = v2 == V_ILLEGAL ? 1u : 0u;
      // per op: the largest configuration holding it = the suffix maximum of
      // its chain's (count -> largest configuration) maxima past its position
      std::vector<unsigned long long> best(H.n_ops, 0);
      for (uint32_t q = 0; q < H.K; ++q) {
        unsigned long long run = 0;
        for (uint32_t pos = H.chain_start[q + 1] - 1; pos > H.chain_start[q]; --pos) {
          run = std::max(run, hmax[pos]);  // configurations with count >= pos - start hold the op at pos - 1
          best[H.rec_op[pos - 1]] = run;
        }
      }
      // each distinct configuration: its path from the trace, rebuilt and certified
      std::unordered_map<uint32_t, uint32_t> part_of;  // trace id -> partial index
      std::vector<uint32_t> moves, order;
      std::vector<uint8_t> ident;
      for (uint32_t d = 0; d < H.n_ops; ++d) {
        if (!best[d]) continue;
        const uint32_t t = (uint32_t)best[d], len = (uint32_t)(best[d] >> 32);
        auto it = part_of.find(t);
        if (it != part_of.end()) { op_part[d] = it->second; continue; }
        moves.clear();
        bool ok = t != 0xFFFFFFFFu;
        for (uint32_t x = t, steps = 0; ok && x != TRACE_NONE; ++steps) {
          if (x >= tr.size() || steps > H.n_ops + 1) { ok = false; break; }
          if (tr[x].move != 0xFFFFFFFFu) moves.push_back(tr[x].move);  // (LV_NONE: the initial configuration)
          x = tr[x].parent;
        }
        std::reverse(moves.begin(), moves.end());
        ok = ok && rebuild_linearization(H, moves.data(), (uint32_t)moves.size(), false, order, ident, true) &&
             order.size() == len && replay_prefix(H, order.data(), ident.data(), order.size());
        if (!ok) {
          c->err = "a partial linearization failed CPU-model certification (checker bug)";
          s2lc_result_free(&r);
          return S2LC_EWITNESS;
        }
        const uint32_t k = (uint32_t)(offs.size() - 1);
        part_of[t] = k;
        op_part[d] = k;
        for (uint32_t x : order) ids.push_back(H.op_ids[x]);
        offs.push_back(ids.size());
      }
    }
    s2lc_result_free(&r);
    out->n_partials = (uint32_t)(offs.size() - 1);
    out->op_ids = (int64_t*)malloc(sizeof(int64_t) * std::max<size_t>(1, H.n_ops));
    out->op_partial = (uint32_t*)malloc(sizeof(uint32_t) * std::max<size_t>(1, H.n_ops));
    out->offs = (uint64_t*)malloc(sizeof(uint64_t) * offs.size());
    out->ids = (int64_t*)malloc(sizeof(int64_t) * std::max<size_t>(1, ids.size()));
    if (!out->op_ids || !out->op_partial || !out->offs || !out->ids) { s2lc_partials_free(out); return S2LC_ENOMEM; }
    if (H.n_ops) memcpy(out->op_ids, H.op_ids.data(), sizeof(int64_t) * H.n_ops);
    if (H.n_ops) memcpy(out->op_partial, op_part.data(), sizeof(uint32_t) * H.n_ops);
    memcpy(out->offs, offs.data(), sizeof(uint64_t) * offs.size());
    if (!ids.empty()) memcpy(out->ids, ids.data(), sizeof(int64_t) * ids.size());
    return 0;
  } catch (const std::bad_alloc&) {
    s2lc_result_free(&r);
    s2lc_partials_free(out);
    c->err = "out of memory";
    return S2LC_ENOMEM;
  }
}

void s2lc_result_free(s2lc_result* r) {
  if (!r) return;
  free(r->witness);
  r->witness = nullptr;
  r->witness_len = 0;
  free(r->partial);
  r->partial = nullptr;
  r->partial_len = 0;
}

// ----------------------------------------------------------------- model ---
int s2lc_step_cpu(const s2lc_history* h, const s2lc_state* s, uint32_t op, s2lc_state out[2]) {
  if (!h || !s || !out) return S2LC_EINVAL;
  const History& H = h->h;
  if (op >= H.n_ops || H.op_call[op] == EV_INF || H.op_ret[op] == EV_INF) return S2LC_EINVAL;
  const OpRec r = H.rec_of(op);
  State st{s->tail, s->stream_hash, s->token};
  State kids[2];
  const int n = s2_step(r, st, H.pool.data(), kids);
  for (int k = 0; k < n; ++k) {
    out[k].tail = kids[k].tail;
    out[k].stream_hash = kids[k].hash;
    out[k].token = kids[k].tok;
    out[k]._pad = 0;
  }
  return n;
}

uint64_t s2lc_chain_hash(uint64_t h, uint64_t r) { return chain_hash(h, r); }

uint64_t s2lc_fold_record_hashes(uint64_t h, const uint64_t* r, size_t n) {
  for (size_t i = 0; i < n; ++i) h = chain_hash(h, r[i]);
  return h;
}

int s2lc_replay(const s2lc_history* h, const uint32_t* order, size_t n) {
  if (!h || (!order && n)) return S2LC_EINVAL;
  return replay_order(h->h, order, n) ? 0 : -1;
}

int s2lc_witness_from_moves(const s2lc_history* h, const uint32_t* moves, size_t n_moves, int p4, int64_t* out_ids,
                            size_t cap) {
  if (!h || (!moves && n_moves)) return S2LC_EINVAL;
  try {
    std::vector<uint32_t> order;
    std::vector<uint8_t> ident;
    if (!rebuild_linearization(h->h, moves, (uint32_t)n_moves, p4 != 0, order, ident, false) ||
        !replay_path(h->h, order.data(), ident.data(), order.size()))
      return -1;
    if (out_ids) {
      if (cap < order.size()) return S2LC_EINVAL;
      for (size_t k = 0; k < order.size(); ++k) out_ids[k] = h->h.op_ids[order[k]];
    }
    return 0;
  } catch (...) {
    return S2LC_ENOMEM;
  }
}

// ------------------------------------------------------- distributed search --
struct s2lc_dist {
  s2lc_ctx* ctx;
  DistLevel d;
};

int s2lc_dist_create(s2lc_ctx* c, const s2lc_history* h, int rank, int world, s2lc_dist** out) {
  if (!c || !h || !out || rank < 0 || world < 1) return S2LC_EINVAL;
  *out = nullptr;
  try {
    if (hipSetDevice(c->device) != hipSuccess) { c->err = "hipSetDevice"; return S2LC_EHIP; }
    auto* x = new s2lc_dist();
    x->ctx = c;
    const int rc = dist_create(x->d, &h->h, (uint32_t)rank, (uint32_t)world, c->red_off,
                               c->own_stream ? nullptr : c->stream, c->err);
    if (rc) { dist_release(x->d); delete x; return rc; }
    *out = x;
    return 0;
  } catch (const std::bad_alloc&) {
    c->err = "out of memory";
    return S2LC_ENOMEM;
  }
}

void s2lc_dist_free(s2lc_dist* x) {
  if (!x) return;
  (void)hipSetDevice(x->ctx->device);
  dist_release(x->d);
  delete x;
}

int s2lc_dist_expand(s2lc_dist* x, uint64_t* counts, int32_t* found) {
  if (!x || !counts || !found) return S2LC_EINVAL;
  int f = 0;
  const int rc = dist_expand(x->d, counts, &f, x->ctx->err);
  *found = f;
  return rc;
}

int s2lc_dist_pack(s2lc_dist* x, void* send, const uint64_t* counts) {
  if (!x || !counts) return S2LC_EINVAL;
  return dist_pack(x->d, (uint8_t*)send, counts, x->ctx->err);
}

int s2lc_dist_insert(s2lc_dist* x, void* recv, uint64_t n_recv, uint64_t* n_next) {
  if (!x || !n_next || (!recv && n_recv)) return S2LC_EINVAL;
  return dist_insert(x->d, (uint8_t*)recv, n_recv, n_next, x->ctx->err);
}

int s2lc_dist_local_round(s2lc_dist* x, uint64_t* n_next, int32_t* found) {
  if (!x || !n_next || !found) return S2LC_EINVAL;
  int f = 0;
  const int rc = dist_local_round(x->d, n_next, &f, x->ctx->err);
  *found = f;
  return rc;
}

int s2lc_dist_local_run(s2lc_dist* x, uint32_t wide, uint64_t* n_next, int32_t* found, uint32_t* rounds) {
  if (!x || !n_next || !found || !rounds) return S2LC_EINVAL;
  int f = 0;
  const int rc = dist_local_run(x->d, wide, n_next, &f, rounds, x->ctx->err);
  *found = f;
  return rc;
}

int s2lc_dist_keep_owned(s2lc_dist* x, uint64_t* n_kept) {
  if (!x || !n_kept) return S2LC_EINVAL;
  return dist_keep_owned(x->d, n_kept, x->ctx->err);
}

int s2lc_dist_x_begin(s2lc_dist* x) {
  if (!x) return S2LC_EINVAL;
  return dist_x_begin(x->d, x->ctx->err);
}

int s2lc_dist_x_send(s2lc_dist* x, void* send, uint32_t cap) {
  if (!x) return S2LC_EINVAL;  // (send / cap: checked by dist_x_send; NULL send with world 1)
  return dist_x_send(x->d, (uint8_t*)send, cap, x->ctx->err);
}

int s2lc_dist_x_recv(s2lc_dist* x, void* recv, uint32_t cap, uint32_t* round) {
  if (!x) return S2LC_EINVAL;  // (recv / cap: checked by dist_x_recv; NULL recv with world 1)
  return dist_x_recv(x->d, (uint8_t*)recv, cap, round, x->ctx->err);
}

int s2lc_dist_x_wait(s2lc_dist* x, uint32_t round, s2lc_dist_xstat* out) {
  if (!x || !out) return S2LC_EINVAL;
  DistXStat st;
  const int rc = dist_x_wait(x->d, round, &st, x->ctx->err);
  if (rc) return rc;
  out->ran = st.ran; out->done = st.done; out->nf = st.nf; out->maxblk = st.maxblk;
  out->nf_global = st.nf_global; out->staged = st.staged;
  return 0;
}

int s2lc_dist_x_rewind(s2lc_dist* x, uint32_t round) {
  if (!x) return S2LC_EINVAL;
  return dist_x_rewind(x->d, round, x->ctx->err);
}

int s2lc_dist_x_end(s2lc_dist* x, uint32_t* done, uint64_t* configs) {
  if (!x || !done || !configs) return S2LC_EINVAL;
  return dist_x_end(x->d, done, configs, x->ctx->err);
}

int s2lc_dist_frontier_pack(s2lc_dist* x, void* buf) {
  if (!x || (!buf && x->d.nf)) return S2LC_EINVAL;
  return dist_frontier_pack(x->d, (uint8_t*)buf, x->ctx->err);
}

int s2lc_dist_frontier_load(s2lc_dist* x, void* buf, uint64_t n) {
  if (!x || (!buf && n)) return S2LC_EINVAL;
  return dist_frontier_load(x->d, (uint8_t*)buf, n, x->ctx->err);
}

int s2lc_dist_info(const s2lc_dist* x, s2lc_dist_info_t* out) {
  if (!x || !out) return S2LC_EINVAL;
  const DistLevel& d = x->d;
  out->config_bytes = d.cb;
  out->n_chains = d.K;
  out->round = d.round;
  out->frontier = d.nf;
  out->found_parent = d.found_parent;
  out->found_move = d.found_move;
  out->found_p4 = d.found_p4;
  out->configs = d.configs;
  out->children = d.children;
  out->max_frontier = d.max_frontier;
  out->device_ms = d.ms;
  out->trace_len = d.tnext;
  out->frontier_cap = d.b.lv.scap;
  return 0;
}

int s2lc_dist_trace(s2lc_dist* x, uint32_t* out_pairs, uint64_t cap_entries, uint64_t* n) {
  if (!x || !n) return S2LC_EINVAL;
  return dist_trace(x->d, out_pairs, cap_entries, n, x->ctx->err);
}

// ------------------------------------------------------------- simulator ---
void s2lc_sim_params_default(s2lc_sim_params* p) {
  if (!p) return;
  memset(p, 0, sizeof *p);
  p->struct_size = sizeof *p;
  p->workflow = S2LC_WF_REGULAR;
  p->num_clients = 5;       // collect-history.rs defaults
  p->ops_per_client = 100;
  p->seed = 1;
  p->p_indefinite = 0.01;
  p->p_definite = 0.02;
  p->p_read_failure = 0.01;
  p->p_check_tail_failure = 0.01;
  p->max_client_ids = 20;
}

int s2lc_simulate_jsonl(const s2lc_sim_params* p, uint8_t** out, size_t* len) {
  if (!p || !out || !len) return S2LC_EINVAL;
  try {
    std::string s;
    int rc = simulate(*p, nullptr, &s);
    if (rc) return rc;
    uint8_t* m = (uint8_t*)malloc(s.size() + 1);
    if (!m) return S2LC_ENOMEM;
    memcpy(m, s.data(), s.size());
    m[s.size()] = 0;
    *out = m;
    *len = s.size();
    return 0;
  } catch (...) {
    return S2LC_ENOMEM;
  }
}

int s2lc_simulate_history(const s2lc_sim_params* p, s2lc_history** out) {
  if (!p || !out) return S2LC_EINVAL;
  *out = nullptr;
  try {
    s2lc_history* h = history_acquire();
    int rc = simulate(*p, &h->h, nullptr);
    if (!rc) rc = h->h.finalize();
    if (rc) { history_release(h); return rc; }
    *out = h;
    return 0;
  } catch (...) {
    return S2LC_ENOMEM;
  }
}

void s2lc_free(void* p) { free(p); }

}  // extern "C"
