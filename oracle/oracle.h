/*
 * oracle.h — TEST INFRASTRUCTURE ONLY. CPU restatement of the reference hot
 * path (s2-porcupine model + porcupine v1.0.3 WGL checker + zeebo/xxh3
 * 8-byte path), used as the parity checker by tests/, by
 * __graft_entry__.smoke() and as bench.py's cpu_baseline ("port").
 * Nothing in the product (s2_verification_amd/, include/) links or calls it.
 *
 * Pinning: the hash is pinned by the reference's chain-hash vectors
 * (golang/s2-porcupine/main_test.go:15-32, rust history.rs:678-687) and by
 * python-xxhash golden vectors (tests/golden/chain_hash_vectors.json); the
 * model + checker are pinned by the reference's 9 verdict tests and the
 * large-line loader test (main_test.go:34-400), re-expressed as fixtures in
 * tests/golden/reference_cases.json. Concurrent interleavings have no
 * reference fixture: there the WGL restatement is
 * cross-checked against the brute-force enumerator below.
 */
#ifndef S2_ORACLE_H
#define S2_ORACLE_H
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* One porcupine.Event (main.go:545-558). Tokens are interned by the caller:
 * 0 = nil, equal strings -> equal positive ids. */
typedef struct or_event {
  int32_t kind;        /* 0 = call, 1 = return */
  int32_t _pad0;
  int64_t op_id;
  int64_t client_id;
  uint8_t input_type;  /* 0 append, 1 read, 2 check-tail (main.go:207-208) */
  uint8_t has_num_records;
  uint8_t has_msn;
  uint8_t _pad1;
  int32_t set_tok;     /* SetFencingToken */
  int32_t batch_tok;   /* BatchFencingToken */
  int32_t _pad2;
  uint64_t num_records;
  uint64_t msn;
  const uint64_t* hashes;
  uint64_t n_hashes;
  uint8_t failure;
  uint8_t definite;
  uint8_t has_tail;
  uint8_t has_hash;
  uint32_t _pad3;
  uint64_t tail;
  uint64_t stream_hash;
} or_event;

typedef struct or_stats {
  uint64_t cache_inserts;   /* porcupine "configs explored" */
  uint64_t steps;           /* model.Step calls */
  uint64_t backtracks;
  uint64_t max_state_set;   /* largest powerset state */
  double seconds;
} or_stats;

/* Return codes of the checkers */
#define OR_OK 0
#define OR_ILLEGAL 1
#define OR_UNKNOWN 2      /* timeout / budget hit */
#define OR_PANIC (-2)     /* the Go model would panic (nil NumRecords / nil Tail) */
#define OR_EINVAL (-1)

uint64_t or_chain_hash(uint64_t stream_hash, uint64_t record_hash);
uint64_t or_fold(uint64_t stream_hash, const uint64_t* hashes, uint64_t n);

/* porcupine.CheckEventsVerbose(s2Model.ToModel(), events, 0), restated. */
int or_check_wgl(const or_event* ev, size_t n, int compute_partial, double timeout_s,
                 uint64_t max_entries, or_stats* st);
/* The same search; longest_out[id] (n_ops entries, dense ids in first-appearance
 * order) = length of the longest partial linearization containing op id that
 * computePartial recorded (LinearizationInfo), 0 if none. */
int or_check_wgl_longest(const or_event* ev, size_t n, double timeout_s, uint64_t max_entries, or_stats* st,
                         int32_t* longest_out);
/* Independent brute force: every real-time-respecting order, powerset model.
 * Only for small histories (n_ops <= 20). */
int or_check_brute(const or_event* ev, size_t n, or_stats* st);
/* Independent CPU implementation of the GPU's reduced search (reduced.c):
 * NOT a restatement of the reference; a cross-check where WGL cannot finish.
 * st->cache_inserts = configurations, st->backtracks = rounds,
 * st->max_state_set = widest frontier. */
/* reductions_off: bits of the product's S2LC_RED_* (1 P1 tail bound, 2 P2 hash
 * at equal tail, 4 P4 nothing constrains, 8 indefinite identity deferral).
 * rc_out (nullable, rc_cap entries): unique configurations of rounds 0, 1, ...
 * (st->backtracks = the number of completed rounds). */
int or_check_reduced(const or_event* ev, size_t n, uint64_t max_configs, uint32_t reductions_off,
                     uint32_t* rc_out, size_t rc_cap, or_stats* st);

#ifdef __cplusplus
}
#endif
#endif
