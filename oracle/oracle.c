/*
 * oracle.c — TEST INFRASTRUCTURE ONLY (see oracle.h). CPU restatement of:
 *   - zeebo/xxh3 v1.1.0 HashSeed on 8 little-endian bytes, as used by
 *     chainHash (golang/s2-porcupine/main.go:232-236); closed form of XXH3's
 *     4..8-byte path — third-party, not in /root/reference.
 *   - s2Model (main.go:253-340) and porcupine's NondeterministicModel
 *     powerset wrapper (porcupine v1.0.3 model.go, upstream).
 *   - porcupine v1.0.3 checkSingle (checker.go, upstream): the WGL DFS over a
 *     doubly linked call/return list with a (bitset, state) cache.
 * Restated from the published algorithm; the module source is
 * not in the container, so behaviour is pinned by the reference tests
 * (main_test.go) via tests/golden/ fixtures.
 */
#include "oracle.h"

#include <stdlib.h>
#include <string.h>
#include <time.h>

/* ---------------------------------------------------------------- hash --- */
static inline uint64_t rotl64(uint64_t x, int r) { return (x << r) | (x >> (64 - r)); }
static inline uint32_t bswap32(uint32_t x) {
  return (x >> 24) | ((x >> 8) & 0xff00u) | ((x << 8) & 0xff0000u) | (x << 24);
}

/* XXH3_len_4to8_64b(le64(record_hash), 8, kSecret, seed=stream_hash) — the
 * path zeebo/xxh3 HashSeed takes for an 8-byte input (main.go:235). */
uint64_t or_chain_hash(uint64_t h, uint64_t r) {
  uint64_t seed = h ^ ((uint64_t)bswap32((uint32_t)h) << 32);
  /* (kSecret[8..16] ^ kSecret[16..24]) - seed */
  uint64_t bitflip = 0xc73ab174c5ecd5a2ULL - seed;
  /* input1 = lo32(r), input2 = hi32(r); input64 = input2 + (input1 << 32) */
  uint64_t k = rotl64(r, 32) ^ bitflip;
  /* XXH3_rrmxmx(k, len = 8) */
  k ^= rotl64(k, 49) ^ rotl64(k, 24);
  k *= 0x9FB21C651E98DF25ULL;
  k ^= (k >> 35) + 8;
  k *= 0x9FB21C651E98DF25ULL;
  return k ^ (k >> 28);
}

/* foldRecordHashes, main.go:238-244 */
uint64_t or_fold(uint64_t h, const uint64_t* hs, uint64_t n) {
  for (uint64_t i = 0; i < n; i++) h = or_chain_hash(h, hs[i]);
  return h;
}

/* --------------------------------------------------------------- model --- */
typedef struct ost { uint64_t tail, hash; int32_t tok; } ost; /* StreamState main.go:196-204 */

static inline int ost_equal(const ost* a, const ost* b) { /* s2Model.Equal main.go:336-340 */
  return a->tail == b->tail && a->hash == b->hash && a->tok == b->tok;
}

/* s2Model.Step, main.go:264-335. Returns the number of successors written
 * (0..2) or OR_PANIC where Go would dereference a nil pointer. */
static int nm_step(const ost* s, const or_event* in, const or_event* out, ost res[2]) {
  if (in->input_type == 0) {
    if (!in->has_num_records) return OR_PANIC;          /* *inp.NumRecords, :279 */
    ost opt;
    opt.tail = s->tail + in->num_records;                /* uint64 wraparound, :279 */
    opt.hash = or_fold(s->hash, in->hashes, in->n_hashes); /* :280 */
    opt.tok = in->set_tok ? in->set_tok : s->tok;        /* :272-277 */
    if (out->failure && out->definite) { res[0] = *s; return 1; } /* :283-285 */
    if (out->failure) {                                  /* :286-300 */
      if (in->batch_tok && (s->tok == 0 || in->batch_tok != s->tok)) { res[0] = *s; return 1; }
      if (in->has_msn && in->msn != s->tail) { res[0] = *s; return 1; }
      res[0] = opt; res[1] = *s; return 2;
    }
    /* durable, :301-318 */
    if (in->batch_tok && (s->tok == 0 || s->tok != in->batch_tok)) return 0;
    if (in->has_msn && in->msn != s->tail) return 0;
    if (!out->has_tail) return OR_PANIC;                 /* *out.Tail, :313 */
    if (out->tail != opt.tail) return 0;
    res[0] = opt; return 1;
  } else if (in->input_type == 1 || in->input_type == 2) { /* :320-331 */
    if (out->has_hash && s->hash != out->stream_hash) return 0;
    if (out->failure) { res[0] = *s; return 1; }
    if (!out->has_tail) return OR_PANIC;
    if (s->tail == out->tail) { res[0] = *s; return 1; }
    return 0;
  }
  return OR_PANIC; /* panic("unknown input type"), :333 */
}

typedef struct sset { ost* v; int n; } sset; /* powerset state: []interface{} */

static int sset_contains(const sset* a, const ost* x) {
  for (int i = 0; i < a->n; i++) if (ost_equal(&a->v[i], x)) return 1;
  return 0;
}
/* NondeterministicModel.ToModel().Equal: containsAll both ways */
static int sset_equal(const sset* a, const sset* b) {
  for (int i = 0; i < a->n; i++) if (!sset_contains(b, &a->v[i])) return 0;
  for (int i = 0; i < b->n; i++) if (!sset_contains(a, &b->v[i])) return 0;
  return 1;
}
/* ToModel().Step: map nm.Step over the set, then merge (O(k^2) Equal dedupe,
 * first occurrence kept); ok iff non-empty. */
static int ps_step(const sset* s, const or_event* in, const or_event* out, sset* res) {
  res->v = (ost*)malloc(sizeof(ost) * (size_t)(2 * s->n + 1));
  res->n = 0;
  for (int i = 0; i < s->n; i++) {
    ost nx[2];
    int c = nm_step(&s->v[i], in, out, nx);
    if (c < 0) { free(res->v); res->v = NULL; return c; }
    for (int k = 0; k < c; k++)
      if (!sset_contains(res, &nx[k])) res->v[res->n++] = nx[k];
  }
  return res->n > 0;
}

/* ------------------------------------------------------------- history --- */
/* renumber (ids -> 0..m-1 by first appearance) via an open-addressing map */
typedef struct idmap { int64_t* keys; int32_t* vals; uint8_t* used; size_t cap; } idmap;
static size_t idmap_slot(const idmap* m, int64_t k) {
  uint64_t x = (uint64_t)k * 0x9E3779B97F4A7C15ULL;
  size_t i = (size_t)(x >> 17) & (m->cap - 1);
  while (m->used[i] && m->keys[i] != k) i = (i + 1) & (m->cap - 1);
  return i;
}
static int32_t* renumber(const or_event* ev, size_t n, int32_t* n_ids) {
  idmap m;
  m.cap = 16;
  while (m.cap < 2 * n + 2) m.cap <<= 1;
  m.keys = (int64_t*)calloc(m.cap, sizeof(int64_t));
  m.vals = (int32_t*)calloc(m.cap, sizeof(int32_t));
  m.used = (uint8_t*)calloc(m.cap, 1);
  int32_t* ids = (int32_t*)malloc(sizeof(int32_t) * (n + 1));
  int32_t next = 0;
  for (size_t i = 0; i < n; i++) {
    size_t s = idmap_slot(&m, ev[i].op_id);
    if (!m.used[s]) { m.used[s] = 1; m.keys[s] = ev[i].op_id; m.vals[s] = next++; }
    ids[i] = m.vals[s];
  }
  free(m.keys); free(m.vals); free(m.used);
  *n_ids = next;
  return ids;
}

/* ------------------------------------------------------------------ WGL --- */
typedef struct node {
  const or_event* value;   /* call: input event; return: output event */
  struct node* match;      /* call -> its return; NULL for returns (and unmatched calls) */
  int32_t id;
  struct node* next;
  struct node* prev;
} node;

typedef struct centry { uint64_t* bits; sset st; } centry;
typedef struct cbucket { uint64_t key; centry* e; int n, cap; int used; } cbucket;
typedef struct cache { cbucket* b; size_t cap, nb; } cache;

static cbucket* cache_bucket(cache* c, uint64_t key, int create) {
  if (create && (c->nb + 1) * 2 > c->cap) {
    size_t ncap = c->cap ? c->cap * 2 : 1024;
    cbucket* nb = (cbucket*)calloc(ncap, sizeof(cbucket));
    for (size_t i = 0; i < c->cap; i++) if (c->b[i].used) {
      size_t j = (size_t)((c->b[i].key * 0x9E3779B97F4A7C15ULL) >> 20) & (ncap - 1);
      while (nb[j].used) j = (j + 1) & (ncap - 1);
      nb[j] = c->b[i];
    }
    free(c->b); c->b = nb; c->cap = ncap;
  }
  if (!c->cap) return NULL;
  size_t j = (size_t)((key * 0x9E3779B97F4A7C15ULL) >> 20) & (c->cap - 1);
  while (c->b[j].used && c->b[j].key != key) j = (j + 1) & (c->cap - 1);
  if (!c->b[j].used) {
    if (!create) return NULL;
    c->b[j].used = 1; c->b[j].key = key; c->nb++;
  }
  return &c->b[j];
}

static uint64_t bits_hash(const uint64_t* b, int w) { /* bitset.hash: popcnt ^ xor of words */
  uint64_t h = 0, pc = 0;
  for (int i = 0; i < w; i++) { pc += (uint64_t)__builtin_popcountll(b[i]); }
  h = pc;
  for (int i = 0; i < w; i++) h ^= b[i];
  return h;
}

/* lift / unlift as porcupine writes them: the call's next node is
 * dereferenced unconditionally (entry.next.prev = ...), the return's only when
 * non-nil. With two calls sharing one return, a call can end up last in the
 * list; porcupine then panics on the nil dereference, which is returned here
 * as -1 (the caller maps it to OR_PANIC) instead of dereferencing NULL. */
static int lift(node* e) {
  if (!e->next) return -1;
  e->prev->next = e->next;
  e->next->prev = e->prev;
  node* m = e->match;
  m->prev->next = m->next;
  if (m->next) m->next->prev = m->prev;
  return 0;
}
static int unlift(node* e) {
  node* m = e->match;
  m->prev->next = m;
  if (m->next) m->next->prev = m;
  e->prev->next = e;
  if (!e->next) return -1;
  e->next->prev = e;
  return 0;
}

typedef struct callsent { node* entry; sset st; } callsent;
typedef struct seqv { int32_t* v; int n; } seqv;

static double now_s(void) {
  struct timespec ts;
  clock_gettime(CLOCK_MONOTONIC, &ts);
  return (double)ts.tv_sec + 1e-9 * (double)ts.tv_nsec;
}

/* porcupine checkEvents -> renumber -> convertEntries (time = slice index)
 * -> checkSingle(model, entries, computePartial, kill). */
static int check_wgl_impl(const or_event* ev, size_t n_ev, int compute_partial, double timeout_s,
                          uint64_t max_entries, or_stats* st, int32_t* longest_out);

int or_check_wgl(const or_event* ev, size_t n_ev, int compute_partial, double timeout_s,
                 uint64_t max_entries, or_stats* st) {
  return check_wgl_impl(ev, n_ev, compute_partial, timeout_s, max_entries, st, NULL);
}

/* LinearizationInfo's lengths: longest_out[id] = length of the longest partial
 * linearization porcupine records for dense op id (0: in none). */
int or_check_wgl_longest(const or_event* ev, size_t n_ev, double timeout_s, uint64_t max_entries, or_stats* st,
                         int32_t* longest_out) {
  return check_wgl_impl(ev, n_ev, 1, timeout_s, max_entries, st, longest_out);
}

static int check_wgl_impl(const or_event* ev, size_t n_ev, int compute_partial, double timeout_s,
                          uint64_t max_entries, or_stats* st, int32_t* longest_out) {
  or_stats local;
  memset(&local, 0, sizeof(local));
  double t0 = now_s();
  int32_t n_ids = 0;
  int32_t* ids = renumber(ev, n_ev, &n_ids);

  /* makeLinkedEntries: walk entries backwards; a return registers itself in
   * match[id]; a call takes match[id] (the nearest later return, or NULL). */
  node* nodes = (node*)calloc(n_ev + 1, sizeof(node));
  node** match = (node**)calloc((size_t)n_ids + 1, sizeof(node*));
  node* root = NULL;
  for (size_t ii = n_ev; ii-- > 0;) {
    node* nd = &nodes[ii + 1];
    nd->value = &ev[ii];
    nd->id = ids[ii];
    nd->match = (ev[ii].kind == 1) ? NULL : match[ids[ii]];
    if (ev[ii].kind == 1) match[ids[ii]] = nd;
    if (root) { /* insertBefore(nd, root) */
      node* before = root->prev;
      root->prev = nd; nd->next = root;
      if (before) { nd->prev = before; before->next = nd; }
    }
    root = nd;
  }
  node* head = &nodes[0]; /* headEntry := insertBefore(&node{id:-1}, entry) */
  head->id = -1;
  if (root) { root->prev = head; head->next = root; }

  int n = (int)(n_ev / 2); /* length(entry) / 2 */
  int W = (n + 63) / 64;
  uint64_t* lin = (uint64_t*)calloc((size_t)W + 1, sizeof(uint64_t));
  cache c = {0, 0, 0};
  callsent* calls = (callsent*)malloc(sizeof(callsent) * ((size_t)n + 1));
  int ncalls = 0;
  seqv* longest = compute_partial ? (seqv*)calloc((size_t)n + 1, sizeof(seqv)) : NULL;
  int32_t** seq_arena = NULL; size_t n_arena = 0, cap_arena = 0;

  sset state; /* Init: merge({(0,0,nil)}) */
  state.v = (ost*)malloc(sizeof(ost)); state.n = 1;
  state.v[0].tail = 0; state.v[0].hash = 0; state.v[0].tok = 0;
  sset init_state = state;

  node* entry = root;
  int result = OR_ILLEGAL;
  uint64_t iter = 0;
  for (;;) {
    if (head->next == NULL) {
      result = OR_OK;
      if (compute_partial) /* success: every op's longest partial is the linearization */
        for (int id = 0; id < n; id++) longest[id].n = ncalls;
      break;
    }
    if ((++iter & 0xFFF) == 0 && timeout_s > 0 && now_s() - t0 > timeout_s) { result = OR_UNKNOWN; break; }
    if (entry->match) {
      node* matching = entry->match;
      sset ns;
      local.steps++;
      int ok = ps_step(&state, entry->value, matching->value, &ns);
      if (ok < 0) { result = OR_PANIC; break; }
      if (ok) {
        if ((size_t)entry->id >= (size_t)W * 64) { free(ns.v); result = OR_PANIC; break; } /* bitset index panic */
        uint64_t* nl = (uint64_t*)malloc(sizeof(uint64_t) * ((size_t)W + 1));
        memcpy(nl, lin, sizeof(uint64_t) * (size_t)W);
        nl[entry->id / 64] |= 1ULL << (entry->id % 64);
        uint64_t hk = bits_hash(nl, W);
        cbucket* b = cache_bucket(&c, hk, 0);
        int found = 0;
        if (b) for (int k = 0; k < b->n && !found; k++)
          if (memcmp(b->e[k].bits, nl, sizeof(uint64_t) * (size_t)W) == 0 && sset_equal(&b->e[k].st, &ns)) found = 1;
        if (!found && ncalls >= n + 1) {
          /* more calls on the stack than calls in the history: only a return
           * shared by two calls (duplicate ids) gets here; porcupine's calls
           * slice would grow, this restatement stops (Unknown) */
          free(nl); free(ns.v);
          result = OR_UNKNOWN;
          break;
        }
        if (!found) {
          b = cache_bucket(&c, hk, 1);
          if (b->n == b->cap) { b->cap = b->cap ? b->cap * 2 : 2; b->e = (centry*)realloc(b->e, sizeof(centry) * (size_t)b->cap); }
          b->e[b->n].bits = nl; b->e[b->n].st = ns; b->n++;
          local.cache_inserts++;
          if ((uint64_t)ns.n > local.max_state_set) local.max_state_set = (uint64_t)ns.n;
          calls[ncalls].entry = entry; calls[ncalls].st = state; ncalls++;
          state = ns;
          lin[entry->id / 64] |= 1ULL << (entry->id % 64);
          if (lift(entry) < 0) { result = OR_PANIC; break; }
          entry = head->next;
          if (max_entries && local.cache_inserts > max_entries) { result = OR_UNKNOWN; break; }
        } else {
          free(nl); free(ns.v);
          entry = entry->next;
        }
      } else {
        free(ns.v);
        entry = entry->next;
      }
    } else {
      if (ncalls == 0) { result = OR_ILLEGAL; break; }
      local.backtracks++;
      if (compute_partial) { /* longest[] update on every backtrack */
        int32_t* seq = NULL;
        for (int k = 0; k < ncalls; k++) {
          int id = calls[k].entry->id;
          if (longest[id].v == NULL || ncalls > longest[id].n) {
            if (!seq) {
              seq = (int32_t*)malloc(sizeof(int32_t) * (size_t)ncalls);
              for (int q = 0; q < ncalls; q++) seq[q] = calls[q].entry->id;
              if (n_arena == cap_arena) { cap_arena = cap_arena ? 2 * cap_arena : 64; seq_arena = (int32_t**)realloc(seq_arena, sizeof(int32_t*) * cap_arena); }
              seq_arena[n_arena++] = seq;
            }
            longest[id].v = seq; longest[id].n = ncalls;
          }
        }
      }
      callsent top = calls[--ncalls];
      entry = top.entry;
      state = top.st;
      lin[entry->id / 64] &= ~(1ULL << (entry->id % 64));
      if (unlift(entry) < 0) { result = OR_PANIC; break; }
      entry = entry->next;
    }
  }

  if (longest_out && longest)
    for (int id = 0; id < n; id++) longest_out[id] = (int32_t)longest[id].n;
  /* free: cached sets own every state except init */
  for (size_t i = 0; i < c.cap; i++) if (c.b[i].used) {
    for (int k = 0; k < c.b[i].n; k++) { free(c.b[i].e[k].bits); free(c.b[i].e[k].st.v); }
    free(c.b[i].e);
  }
  free(c.b);
  free(init_state.v);
  for (size_t i = 0; i < n_arena; i++) free(seq_arena[i]);
  free(seq_arena); free(longest);
  free(calls); free(lin); free(match); free(nodes); free(ids);
  local.seconds = now_s() - t0;
  if (st) *st = local;
  return result;
}

/* ---------------------------------------------------------- brute force --- */
typedef struct bop { const or_event* in; const or_event* out; size_t call, ret; } bop;

static int brute_rec(const bop* ops, int m, uint32_t done, const sset* s, or_stats* st) {
  if (done == ((m == 32) ? 0xFFFFFFFFu : ((1u << m) - 1))) return 1;
  for (int o = 0; o < m; o++) {
    if (done & (1u << o)) continue;
    int minimal = 1; /* no pending q with ret(q) < call(o) */
    for (int q = 0; q < m && minimal; q++)
      if (q != o && !(done & (1u << q)) && ops[q].ret < ops[o].call) minimal = 0;
    if (!minimal) continue;
    sset ns;
    st->steps++;
    int ok = ps_step(s, ops[o].in, ops[o].out, &ns);
    if (ok < 0) return ok;
    if (ok) {
      int r = brute_rec(ops, m, done | (1u << o), &ns, st);
      free(ns.v);
      if (r != 0) return r;
    } else free(ns.v);
  }
  return 0;
}

int or_check_brute(const or_event* ev, size_t n_ev, or_stats* st) {
  or_stats local;
  memset(&local, 0, sizeof(local));
  int32_t m = 0;
  int32_t* ids = renumber(ev, n_ev, &m);
  if (m > 20) { free(ids); return OR_EINVAL; }
  bop ops[32];
  int ncall[32] = {0}, nret[32] = {0};
  for (size_t i = 0; i < n_ev; i++) {
    int id = ids[i];
    if (ev[i].kind == 0) { ops[id].in = &ev[i]; ops[id].call = i; ncall[id]++; }
    else { ops[id].out = &ev[i]; ops[id].ret = i; nret[id]++; }
  }
  free(ids);
  for (int i = 0; i < m; i++) {
    if (ncall[i] != 1 || nret[i] != 1) return (ncall[i] > 1 || nret[i] > 1) ? OR_EINVAL : OR_ILLEGAL;
    if (ops[i].ret < ops[i].call) return OR_ILLEGAL; /* unmatched in the linked list */
  }
  sset s0; ost init = {0, 0, 0}; s0.v = &init; s0.n = 1;
  int r = brute_rec(ops, m, 0, &s0, &local);
  if (st) *st = local;
  if (r < 0) return r;
  return r ? OR_OK : OR_ILLEGAL;
}
