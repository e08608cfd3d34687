/*
 * reduced.c — TEST INFRASTRUCTURE ONLY. An independent, single-threaded CPU
 * implementation of the *reduced* configuration search that the GPU runs
 * (DESIGN.md §3): rounds of one non-identity op, E-closure, I-identity
 * deferral, P1 tail bound, P2 hash at equal tail, P4 completion, each of
 * which can be switched off (ablation parity with the GPU engines, which take
 * the same switches: include/s2lincheck.h S2LC_RED_*). It is NOT a restatement of the
 * reference; the reductions themselves are validated against the WGL
 * restatement (oracle.c, = porcupine checkSingle) and brute force on
 * histories where those finish. This file exists to cross-check the GPU on
 * histories where porcupine's DFS does not finish (e.g. 32 clients x 1000).
 *
 * Written from the design, not from search_dev.h: plain arrays, a
 * std-free open-addressing set, sets of ops as per-chain counters.
 */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include "oracle.h"

/* allocation failure in the search loop: fail loudly (an exploded ablation
 * must not read as a verdict) */
static void* r_chk(void* p) {
  if (!p) { fprintf(stderr, "oracle/reduced.c: out of memory in the round loop\n"); abort(); }
  return p;
}

typedef struct rop {
  const or_event* in;
  const or_event* out;
  size_t call, ret;
  int cls;        /* 0 = E, 1 = D, 2 = I */
  int constrain;  /* observes the state when linearized */
  uint64_t req;   /* required pre-tail (constraining ops) */
} rop;

typedef struct rst { uint64_t tail, hash; int32_t tok; } rst;

static uint64_t mixr(uint64_t x);
static int rs_eq(const rst* a, const rst* b) { return a->tail == b->tail && a->hash == b->hash && a->tok == b->tok; }

/* s2Model.Step for one state (main.go:264-335); returns count (0..2). */
static int r_step(const rop* o, const rst* s, rst out[2]) {
  const or_event* in = o->in;
  const or_event* ou = o->out;
  if (in->input_type == 0) {
    rst opt;
    opt.tail = s->tail + in->num_records;
    opt.hash = or_fold(s->hash, in->hashes, in->n_hashes);
    opt.tok = in->set_tok ? in->set_tok : s->tok;
    if (ou->failure && ou->definite) { out[0] = *s; return 1; }
    int ok = 1;
    if (in->batch_tok && (s->tok == 0 || s->tok != in->batch_tok)) ok = 0;
    if (in->has_msn && in->msn != s->tail) ok = 0;
    if (ou->failure) {
      if (!ok) { out[0] = *s; return 1; }
      out[0] = opt;
      out[1] = *s;
      return rs_eq(&opt, s) ? 1 : 2;
    }
    if (!ok || ou->tail != opt.tail) return 0;
    out[0] = opt;
    return 1;
  }
  if (ou->has_hash && s->hash != ou->stream_hash) return 0;
  if (ou->failure || s->tail == ou->tail) { out[0] = *s; return 1; }
  return 0;
}

typedef struct rcfg { uint16_t* cnt; rst s; } rcfg;

typedef struct rctx {
  rop* ops;
  int n, K;
  int* chain;      /* op indices, chain-major */
  int* cstart;     /* K+1 */
  uint64_t* sufmin;/* per chain position (len+1 per chain incl. sentinel) */
  int nowrap;      /* P1 on (tails never wrap) */
  int p2;          /* P2 on (nowrap, no 0-record append with hashes) */
  int p4;          /* P4 on */
  int idefer;      /* indefinite identity deferral on */
} rctx;

static int head(const rctx* c, const uint16_t* cnt, int q) {
  int p = c->cstart[q] + cnt[q];
  return p < c->cstart[q + 1] ? c->chain[p] : -1;
}

static size_t min_ret(const rctx* c, const uint16_t* cnt) {
  size_t m = (size_t)-1;
  for (int q = 0; q < c->K; q++) {
    int h = head(c, cnt, q);
    if (h >= 0 && c->ops[h].ret < m) m = c->ops[h].ret;
  }
  return m;
}

static uint64_t bound_of(const rctx* c, const uint16_t* cnt) {
  uint64_t b = ~0ull;
  for (int q = 0; q < c->K; q++) {
    uint64_t v = c->sufmin[c->cstart[q] + q + cnt[q]];
    if (v < b) b = v;
  }
  return b;
}

/* closure: 0 alive, 1 dead, 2 complete (all ops or nothing constrains) */
static int r_close(const rctx* c, uint16_t* cnt, const rst* s) {
  for (;;) {
    size_t mr = min_ret(c, cnt);
    if (mr == (size_t)-1) return 2;
    uint64_t b = bound_of(c, cnt);
    if (c->nowrap && s->tail > b) return 1;
    if (c->p4 && b == ~0ull) return 2;
    if (c->p2) { /* a minimal successful hash-checking read at this very tail with another hash never passes */
      for (int q = 0; q < c->K; q++) {
        int h = head(c, cnt, q);
        if (h < 0) continue;
        const rop* o = &c->ops[h];
        if (o->cls != 0 || o->call >= mr || o->in->input_type == 0) continue;
        if (!o->out->failure && o->out->has_hash && o->out->tail == s->tail && o->out->stream_hash != s->hash) return 1;
      }
    }
    int changed = 0;
    for (int q = 0; q < c->K; q++) {
      for (;;) {
        int h = head(c, cnt, q);
        if (h < 0) break;
        const rop* o = &c->ops[h];
        if (o->cls != 0 || o->call >= mr) break;
        rst nx[2];
        if (r_step(o, s, nx) == 0) break;
        cnt[q]++;
        changed = 1;
      }
    }
    if (!changed) return 0;
  }
}

/* open-addressing set of configurations */
typedef struct rset { uint64_t* fp; int32_t* idx; size_t cap, n; } rset;

static uint64_t mixr(uint64_t x) {
  x ^= x >> 31; x *= 0x7fb5d329728ea185ull; x ^= x >> 27; x *= 0x81dadef4bc2dd44dull; x ^= x >> 33;
  return x;
}

int or_check_reduced(const or_event* ev, size_t n_ev, uint64_t max_configs, uint32_t red_off, uint32_t* rc_out,
                     size_t rc_cap, or_stats* st) {
  or_stats local;
  memset(&local, 0, sizeof local);
  struct timespec t0, t1;
  clock_gettime(CLOCK_MONOTONIC, &t0);
  /* pair calls and returns by op_id (first appearance order) */
  int cap = (int)n_ev + 1;
  rop* ops = (rop*)calloc((size_t)cap, sizeof(rop));
  int64_t* ids = (int64_t*)malloc(sizeof(int64_t) * (size_t)cap);
  int n = 0, result = OR_ILLEGAL;
  int* ncall = (int*)calloc((size_t)cap, sizeof(int));
  int* nret = (int*)calloc((size_t)cap, sizeof(int));
  size_t mcap = 16;
  while (mcap < 2 * n_ev + 2) mcap <<= 1;
  int32_t* mslot = (int32_t*)malloc(sizeof(int32_t) * mcap);  /* op_id -> dense index */
  for (size_t z = 0; z < mcap; z++) mslot[z] = -1;
  for (size_t i = 0; i < n_ev; i++) {
    size_t j = (size_t)(mixr((uint64_t)ev[i].op_id) & (mcap - 1));
    while (mslot[j] >= 0 && ids[mslot[j]] != ev[i].op_id) j = (j + 1) & (mcap - 1);
    int k = mslot[j];
    if (k < 0) { k = n++; ids[k] = ev[i].op_id; mslot[j] = k; }
    if (ev[i].kind == 0) { ops[k].in = &ev[i]; ops[k].call = i; ncall[k]++; }
    else { ops[k].out = &ev[i]; ops[k].ret = i; nret[k]++; }
  }
  for (int k = 0; k < n; k++)
    if (ncall[k] != 1 || nret[k] != 1 || ops[k].ret < ops[k].call) {
      const int bad = (ncall[k] > 1 || nret[k] > 1) ? OR_EINVAL : OR_ILLEGAL;
      free(ops); free(ids); free(ncall); free(nret); free(mslot);
      return bad;
    }
  free(ncall); free(nret); free(ids); free(mslot);
  uint64_t total = 0;
  int nowrap = 1, zero_with_hashes = 0;
  for (int k = 0; k < n; k++) {
    rop* o = &ops[k];
    const or_event* in = o->in;
    const or_event* ou = o->out;
    if (in->input_type == 0) {
      if (!in->has_num_records) { free(ops); return OR_PANIC; }
      if (in->num_records > (1ull << 63) - total) nowrap = 0; else total += in->num_records;
      if (in->num_records == 0 && in->n_hashes > 0) zero_with_hashes = 1;
      o->cls = (ou->failure && ou->definite) ? 0 : (ou->failure ? 2 : 1);
      o->constrain = !ou->failure;
      o->req = ou->tail >= in->num_records ? ou->tail - in->num_records : 0;
    } else {
      o->cls = 0;
      o->constrain = !ou->failure || ou->has_hash;
      o->req = !ou->failure ? ou->tail : ~0ull - 1;
    }
    if (!ou->failure && !ou->has_tail) { free(ops); return OR_PANIC; }
    if (o->req > ~0ull - 1) o->req = ~0ull - 1;
  }
  /* chains: ops are in call order already (first appearance = call) */
  rctx c;
  memset(&c, 0, sizeof c);
  c.ops = ops; c.n = n;
  c.nowrap = nowrap && !(red_off & 1u);
  c.p2 = nowrap && !zero_with_hashes && !(red_off & 2u);
  c.p4 = !(red_off & 4u);
  c.idefer = !(red_off & 8u);
  int* chain_of = (int*)malloc(sizeof(int) * (size_t)(n + 1));
  size_t* last_ret = (size_t*)malloc(sizeof(size_t) * (size_t)(n + 1));
  int K = 0;
  for (int k = 0; k < n; k++) {
    int best = -1;
    for (int q = 0; q < K; q++)
      if (last_ret[q] < ops[k].call && (best < 0 || last_ret[q] < last_ret[best])) best = q;
    if (best < 0) best = K++;
    chain_of[k] = best;
    last_ret[best] = ops[k].ret;
  }
  c.K = K;
  c.cstart = (int*)calloc((size_t)K + 1, sizeof(int));
  for (int k = 0; k < n; k++) c.cstart[chain_of[k] + 1]++;
  for (int q = 0; q < K; q++) c.cstart[q + 1] += c.cstart[q];
  c.chain = (int*)malloc(sizeof(int) * (size_t)(n + 1));
  int* fill = (int*)calloc((size_t)K + 1, sizeof(int));
  for (int k = 0; k < n; k++) { int q = chain_of[k]; c.chain[c.cstart[q] + fill[q]++] = k; }
  free(fill); free(chain_of); free(last_ret);
  c.sufmin = (uint64_t*)malloc(sizeof(uint64_t) * (size_t)(n + K + 1));
  for (int q = 0; q < K; q++) {
    int len = c.cstart[q + 1] - c.cstart[q];
    uint64_t run = ~0ull;
    c.sufmin[c.cstart[q] + q + len] = run;
    for (int p = len - 1; p >= 0; p--) {
      const rop* o = &ops[c.chain[c.cstart[q] + p]];
      if (o->constrain && o->req < run) run = o->req;
      c.sufmin[c.cstart[q] + q + p] = run;
    }
  }
  /* BFS by rounds */
  size_t cw = (size_t)(K ? K : 1);
  size_t fcap = 1024, nf = 0;
  uint16_t* fcnt = (uint16_t*)r_chk(calloc(fcap * cw, sizeof(uint16_t)));
  rst* fst = (rst*)r_chk(calloc(fcap, sizeof(rst)));
  rst s0 = {0, 0, 0};
  int r0 = r_close(&c, fcnt, &s0);
  if (r0 == 2) result = OR_OK;
  else if (r0 == 0) { fst[0] = s0; nf = 1; if (rc_out && rc_cap > 0) rc_out[0] = 1; }
  size_t round = 0;
  uint16_t* tmp = (uint16_t*)r_chk(malloc(sizeof(uint16_t) * cw));
  while (result != OR_OK && nf > 0) {
    size_t ncap = 1024, nn = 0;
    uint16_t* ncnt = (uint16_t*)r_chk(malloc(ncap * cw * sizeof(uint16_t)));
    rst* nst = (rst*)r_chk(malloc(ncap * sizeof(rst)));
    rset set;
    set.cap = 4096; set.n = 0;
    set.fp = (uint64_t*)r_chk(calloc(set.cap, sizeof(uint64_t)));
    set.idx = (int32_t*)r_chk(malloc(set.cap * sizeof(int32_t)));
    for (size_t i = 0; i < nf && result != OR_OK; i++) {
      const uint16_t* pc = fcnt + i * cw;
      const rst* ps = &fst[i];
      size_t mr = min_ret(&c, pc);
      for (int q = 0; q < K && result != OR_OK; q++) {
        int h = head(&c, pc, q);
        if (h < 0) continue;
        const rop* o = &ops[h];
        if (o->cls == 0 || o->call >= mr) continue;
        rst kids[2];
        int nk = r_step(o, ps, kids);
        for (int k = 0; k < nk; k++) {
          /* I-op identity child only when the op holds minret */
          if (c.idefer && o->cls == 2 && rs_eq(&kids[k], ps) && o->ret != mr) {
            /* unless it is also the opt outcome (guards pass and opt == s: a
             * 0-record append with no hashes); with failing guards the
             * child is the identity outcome alone, deferred like any other */
            const or_event* in = o->in;
            const int guards = !(in->batch_tok && (ps->tok == 0 || ps->tok != in->batch_tok)) &&
                               !(in->has_msn && in->msn != ps->tail);
            rst opt;
            opt.tail = ps->tail + in->num_records;
            opt.hash = or_fold(ps->hash, in->hashes, in->n_hashes);
            opt.tok = in->set_tok ? in->set_tok : ps->tok;
            if (!guards || !rs_eq(&opt, ps)) continue;
          }
          memcpy(tmp, pc, cw * sizeof(uint16_t));
          tmp[q]++;
          local.steps++;
          int r = r_close(&c, tmp, &kids[k]);
          if (r == 1) continue;
          if (r == 2) { result = OR_OK; break; }
          uint64_t fp = mixr(kids[k].tail ^ mixr(kids[k].hash + (uint64_t)kids[k].tok * 0x9E3779B97F4A7C15ull));
          for (int w = 0; w < K; w++) fp = mixr(fp ^ ((uint64_t)tmp[w] << 17 ^ (uint64_t)w));
          if (fp == 0) fp = 1;
          if ((set.n + 1) * 2 > set.cap) { /* grow */
            size_t oc = set.cap;
            uint64_t* of = set.fp; int32_t* oi = set.idx;
            set.cap *= 2;
            set.fp = (uint64_t*)r_chk(calloc(set.cap, sizeof(uint64_t)));
            set.idx = (int32_t*)r_chk(malloc(set.cap * sizeof(int32_t)));
            for (size_t z = 0; z < oc; z++) if (of[z]) {
              size_t j = of[z] & (set.cap - 1);
              while (set.fp[j]) j = (j + 1) & (set.cap - 1);
              set.fp[j] = of[z]; set.idx[j] = oi[z];
            }
            free(of); free(oi);
          }
          size_t j = fp & (set.cap - 1);
          int dup = 0;
          while (set.fp[j]) {
            if (set.fp[j] == fp) {
              int32_t x = set.idx[j];
              if (rs_eq(&nst[x], &kids[k]) && memcmp(ncnt + (size_t)x * cw, tmp, cw * sizeof(uint16_t)) == 0) { dup = 1; break; }
            }
            j = (j + 1) & (set.cap - 1);
          }
          if (dup) continue;
          if (nn == ncap) {
            ncap *= 2;
            ncnt = (uint16_t*)r_chk(realloc(ncnt, ncap * cw * sizeof(uint16_t)));
            nst = (rst*)r_chk(realloc(nst, ncap * sizeof(rst)));
          }
          memcpy(ncnt + nn * cw, tmp, cw * sizeof(uint16_t));
          nst[nn] = kids[k];
          set.fp[j] = fp; set.idx[j] = (int32_t)nn; set.n++;
          nn++;
        }
      }
    }
    free(set.fp); free(set.idx);
    free(fcnt); free(fst);
    fcnt = ncnt; fst = nst; nf = nn;
    round++;
    if (result != OR_OK && rc_out && round < rc_cap) rc_out[round] = (uint32_t)nn;
    local.cache_inserts += nn;
    local.backtracks++; /* rounds */
    if (nn > local.max_state_set) local.max_state_set = nn;
    if (max_configs && local.cache_inserts > max_configs) { result = OR_UNKNOWN; break; }
  }
  if (result != OR_OK && result != OR_UNKNOWN) result = OR_ILLEGAL;
  free(tmp); free(fcnt); free(fst);
  free(c.cstart); free(c.chain); free(c.sufmin); free(ops);
  clock_gettime(CLOCK_MONOTONIC, &t1);
  local.seconds = (double)(t1.tv_sec - t0.tv_sec) + 1e-9 * (double)(t1.tv_nsec - t0.tv_nsec);
  if (st) *st = local;
  return result;
}
