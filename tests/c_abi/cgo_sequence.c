/*
 * cgo_sequence.c — a plain C99 caller of include/s2lincheck.h making exactly
 * the calls of the Go cgo shim in INTEGRATION.md §2 (checkEventsGPU): calloc'd
 * s2lc_event[], s2lc_history_from_events, s2lc_create, s2lc_check,
 * s2lc_result_free, s2lc_history_free, s2lc_destroy. It proves the header is
 * C-clean (gcc -std=c99 -pedantic -Werror) and that the ABI works from a
 * non-C++ caller; Go itself is absent from this image.
 *
 * The histories are main_test.go's TestBasicNoConcurrency (Ok, main_test.go:
 * 128-152) and TestBasicNoConcurrencyDefiniteFailure2 (Illegal, :192-232),
 * built event by event the way the shim converts porcupine.Events.
 *
 *   cgo_sequence          full sequence on the GPU; exit 0 = every check held
 *   cgo_sequence --no-gpu the ctx-free part (history build, model step, hash)
 *                         and s2lc_create's "no device" status
 */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "s2lincheck.h"

static int failures = 0;
#define EXPECT(cond, ...)                                   \
  do {                                                      \
    if (!(cond)) {                                          \
      fprintf(stderr, "FAIL %s:%d: ", __FILE__, __LINE__);  \
      fprintf(stderr, __VA_ARGS__);                         \
      fprintf(stderr, "\n");                                \
      failures++;                                           \
    }                                                       \
  } while (0)

/* append(batch) -> AppendSuccess(tail) ; read -> ReadSuccess(tail, hash) ;
 * check_tail -> CheckTailSuccess(tail). definite_fail: the append's Finish is
 * AppendDefiniteFailure (TestBasicNoConcurrencyDefiniteFailure2 shape). */
static s2lc_event* build_events(const uint64_t* batch, size_t nb, uint64_t read_tail, uint64_t read_hash,
                                int definite_fail, size_t* n_out) {
  const size_t n = 6;
  s2lc_event* ev = (s2lc_event*)calloc(n, sizeof(s2lc_event));
  if (!ev) return NULL;
  /* op 0: append */
  ev[0].kind = S2LC_CALL_EVENT;
  ev[0].op_id = 0;
  ev[0].input_type = S2LC_INPUT_APPEND;
  ev[0].has_num_records = 1;
  ev[0].num_records = nb;
  ev[0].record_hashes = batch;
  ev[0].n_record_hashes = nb;
  ev[1].kind = S2LC_RETURN_EVENT;
  ev[1].op_id = 0;
  if (definite_fail) {
    ev[1].failure = 1;
    ev[1].definite_failure = 1;
  } else {
    ev[1].has_tail = 1;
    ev[1].tail = nb;
  }
  /* op 1: read */
  ev[2].kind = S2LC_CALL_EVENT;
  ev[2].op_id = 1;
  ev[2].input_type = S2LC_INPUT_READ;
  ev[3].kind = S2LC_RETURN_EVENT;
  ev[3].op_id = 1;
  ev[3].has_tail = 1;
  ev[3].tail = read_tail;
  ev[3].has_stream_hash = 1;
  ev[3].stream_hash = read_hash;
  /* op 2: check tail */
  ev[4].kind = S2LC_CALL_EVENT;
  ev[4].op_id = 2;
  ev[4].input_type = S2LC_INPUT_CHECK_TAIL;
  ev[5].kind = S2LC_RETURN_EVENT;
  ev[5].op_id = 2;
  ev[5].has_tail = 1;
  ev[5].tail = read_tail;
  *n_out = n;
  return ev;
}

/* checkEventsGPU: returns the verdict (or -1 on an error), fills the witness */
static int check_events_gpu(const s2lc_event* cev, size_t n, int64_t* witness, uint32_t* witness_len) {
  char errbuf[512];
  s2lc_history* h = NULL;
  int rc = s2lc_history_from_events(cev, n, &h, errbuf, sizeof errbuf);
  if (rc != 0) {
    fprintf(stderr, "s2lc_history_from_events: %d %s\n", rc, errbuf);
    return -1;
  }
  s2lc_opts opts;
  memset(&opts, 0, sizeof opts);
  opts.struct_size = (uint32_t)sizeof opts;
  opts.device = -1;
  int st = 0;
  s2lc_ctx* ctx = s2lc_create(&opts, &st);
  if (!ctx) {
    fprintf(stderr, "s2lc_create: %d (no GPU)\n", st);
    s2lc_history_free(h);
    return -1;
  }
  s2lc_result res;
  memset(&res, 0, sizeof res);
  rc = s2lc_check(ctx, h, &res);
  int verdict = -1;
  if (rc != 0) {
    fprintf(stderr, "s2lc_check: %s\n", s2lc_last_error(ctx));
  } else {
    verdict = res.verdict;
    *witness_len = res.witness ? res.witness_len : 0;
    for (uint32_t i = 0; i < *witness_len && i < 16; ++i) witness[i] = res.witness[i];
  }
  s2lc_result_free(&res);
  s2lc_destroy(ctx);
  s2lc_history_free(h);
  return verdict;
}

int main(int argc, char** argv) {
  const int no_gpu = argc > 1 && strcmp(argv[1], "--no-gpu") == 0;
  const uint64_t batch[4] = {11, 22, 33, 44};
  const uint64_t h4 = s2lc_fold_record_hashes(0, batch, 4);
  /* main_test.go:15-32 vectors through the C entry points */
  EXPECT(s2lc_chain_hash(0, 0xab6e5f64077e7d8aull) == 0x4d2b003ee417c3a5ull, "chain hash vector h1");
  size_t n = 0;
  s2lc_event* ok_ev = build_events(batch, 4, 4, h4, 0, &n);
  s2lc_event* bad_ev = build_events(batch, 4, 4, h4, 1, &n); /* read observes a definite-failed append */
  if (!ok_ev || !bad_ev) return 2;

  /* ctx-free: build the history and step the model from Init */
  char err[256];
  s2lc_history* h = NULL;
  EXPECT(s2lc_history_from_events(ok_ev, n, &h, err, sizeof err) == 0, "history_from_events: %s", err);
  if (h) {
    s2lc_history_info info;
    EXPECT(s2lc_history_info_get(h, &info) == 0 && info.n_ops == 3 && info.n_events == 6, "history info");
    s2lc_state s0, out[2];
    memset(&s0, 0, sizeof s0);
    EXPECT(s2lc_step_cpu(h, &s0, 0, out) == 1 && out[0].tail == 4 && out[0].stream_hash == h4, "append step");
    EXPECT(s2lc_step_cpu(h, &out[0], 1, out) == 1, "read step after the append");
    EXPECT(s2lc_step_cpu(h, &s0, 1, out) == 0, "read step before the append is rejected");
    const uint32_t order[3] = {0, 1, 2};
    EXPECT(s2lc_replay(h, order, 3) == 0, "replay of the sequential order");
    s2lc_history_free(h);
  }

  if (no_gpu) {
    s2lc_opts opts;
    memset(&opts, 0, sizeof opts);
    opts.struct_size = (uint32_t)sizeof opts;
    opts.device = -1;
    int st = 0;
    s2lc_ctx* ctx = s2lc_create(&opts, &st);
    EXPECT(ctx == NULL && st == S2LC_ENODEV, "no device: s2lc_create must fail with ENODEV (got %d)", st);
    if (ctx) s2lc_destroy(ctx);
  } else {
    int64_t w[16];
    uint32_t wl = 0;
    const int v_ok = check_events_gpu(ok_ev, n, w, &wl);
    EXPECT(v_ok == S2LC_OK, "TestBasicNoConcurrency: verdict %d", v_ok);
    EXPECT(wl == 3 && w[0] == 0 && w[1] == 1 && w[2] == 2, "witness = op ids 0, 1, 2 (len %u)", wl);
    const int v_bad = check_events_gpu(bad_ev, n, w, &wl);
    EXPECT(v_bad == S2LC_ILLEGAL, "TestBasicNoConcurrencyDefiniteFailure2: verdict %d", v_bad);
    /* an ABI-1 caller (struct_size up to `stream`) still gets a working context */
    s2lc_opts old;
    memset(&old, 0, sizeof old);
    old.struct_size = (uint32_t)offsetof(s2lc_opts, timeout_us);
    old.device = -1;
    int st = 0;
    s2lc_ctx* ctx = s2lc_create(&old, &st);
    EXPECT(ctx != NULL, "ABI-1 sized opts: %d", st);
    if (ctx) s2lc_destroy(ctx);
  }
  free(ok_ev);
  free(bad_ev);
  if (failures) {
    fprintf(stderr, "%d failure(s)\n", failures);
    return 1;
  }
  printf("cgo_sequence: all checks passed (%s)\n", no_gpu ? "no-gpu" : "gpu");
  return 0;
}
