/*
 * s2lincheck.h — C ABI of libs2lincheck, the MI355X (gfx950) linearizability
 * checker for the S2 stream model.
 *
 * This is the drop-in boundary for the hot path of s2-streamstore/s2-verification:
 *
 *   reference                                                 replaced by
 *   ---------------------------------------------------------------------------------
 *   eventsFromReader(r io.Reader) ([]porcupine.Event, error)  s2lc_load_jsonl
 *       golang/s2-porcupine/main.go:529-563 (+ UnmarshalJSON variants main.go:32-188)
 *   porcupine.Event{Kind, Value: StreamInput|StreamOutput,     s2lc_event / s2lc_history_from_events
 *       Id, ClientId}  main.go:206-225, main.go:545-558
 *   s2Model.ToModel()  main.go:253-361, 605                    (built in: S2 model on device)
 *   porcupine.CheckEventsVerbose(model, events, 0)             s2lc_check / s2lc_check_batch
 *       main.go:606 (porcupine v1.0.3 checkSingle, upstream)
 *   s2Model.Step  main.go:264-335                              s2lc_step_cpu
 *   chainHash / foldRecordHashes  main.go:227-244              s2lc_chain_hash / s2lc_fold_record_hashes
 *
 * Conventions
 *   - Every entry point returns 0 (S2LC_SUCCESS) or a negative s2lc_status.
 *     A human-readable message is available from s2lc_last_error(ctx) (ctx
 *     calls) or written into the caller's err buffer (ctx-free calls).
 *   - No C++ exception crosses this ABI and the library never calls exit().
 *   - Objects returned through out-pointers are owned by the library and are
 *     released with the matching *_free function.
 *   - A context is single-threaded; distinct contexts may be used
 *     concurrently from different threads. All calls block.
 *   - The checker itself runs only on the GPU. With no usable HIP device,
 *     s2lc_create fails with S2LC_ENODEV: there is no CPU fallback.
 */
#ifndef S2LINCHECK_H
#define S2LINCHECK_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define S2LC_ABI_VERSION 2

/* CheckResult (porcupine: Ok / Illegal / Unknown). Unknown only when a
 * timeout or configuration budget was set and hit (the reference CLI passes
 * timeout 0, main.go:606, so it never sees Unknown). */
enum s2lc_verdict { S2LC_OK = 0, S2LC_ILLEGAL = 1, S2LC_UNKNOWN = 2 };

enum s2lc_status {
  S2LC_SUCCESS = 0,
  S2LC_EINVAL = -1,       /* bad argument / malformed event array */
  S2LC_EDECODE = -2,      /* JSONL decode error (eventsFromReader error, main.go:539,560) */
  S2LC_EIO = -3,          /* cannot open / read the file (main.go:591-595) */
  S2LC_ENODEV = -4,       /* no usable HIP device */
  S2LC_EHIP = -5,         /* HIP runtime error */
  S2LC_EUNSUPPORTED = -6, /* history outside the supported envelope */
  S2LC_ENOMEM = -7,
  S2LC_EWITNESS = -8      /* an Ok witness failed CPU-model certification: a checker bug.
                             The results are still written; the affected histories carry
                             verdict Unknown, reason S2LC_R_WITNESS_INVALID. */
};

/* StreamInput.InputType, main.go:207-208 */
enum s2lc_input_type { S2LC_INPUT_APPEND = 0, S2LC_INPUT_READ = 1, S2LC_INPUT_CHECK_TAIL = 2 };
/* porcupine.EventKind */
enum s2lc_event_kind { S2LC_CALL_EVENT = 0, S2LC_RETURN_EVENT = 1 };

/* One porcupine.Event. For a CALL the input fields mirror StreamInput
 * (main.go:206-215); for a RETURN the output fields mirror StreamOutput
 * (main.go:217-225). Pointer-typed Go fields become has_* flags or NULL. */
typedef struct s2lc_event {
  int32_t kind;                  /* S2LC_CALL_EVENT / S2LC_RETURN_EVENT */
  int64_t op_id;                 /* Event.Id */
  int64_t client_id;             /* Event.ClientId (visualization only) */
  /* --- call: StreamInput --- */
  uint8_t input_type;            /* s2lc_input_type */
  uint8_t has_num_records;       /* NumRecords != nil (required for appends) */
  uint8_t has_match_seq_num;     /* MatchSeqNum != nil */
  uint8_t _pad0;
  uint64_t num_records;
  uint64_t match_seq_num;
  const char* set_fencing_token; /* SetFencingToken, NULL = nil */
  const char* fencing_token;     /* BatchFencingToken, NULL = nil */
  const uint64_t* record_hashes; /* RecordHashes */
  uint64_t n_record_hashes;      /* independent of num_records (main_test.go:322) */
  /* --- return: StreamOutput --- */
  uint8_t failure;               /* Failure */
  uint8_t definite_failure;      /* DefiniteFailure */
  uint8_t has_tail;              /* Tail != nil */
  uint8_t has_stream_hash;       /* StreamHash != nil */
  uint32_t _pad1;
  uint64_t tail;
  uint64_t stream_hash;
} s2lc_event;

/* Model state. token is an id interned per history: 0 = nil; equal token
 * strings get equal ids, so id equality is stringPtrEqual (main.go:246-251). */
typedef struct s2lc_state {
  uint64_t tail;
  uint64_t stream_hash;
  uint32_t token;
  uint32_t _pad;
} s2lc_state;

typedef struct s2lc_history s2lc_history;
typedef struct s2lc_ctx s2lc_ctx;
typedef struct s2lc_batch s2lc_batch;

/* Context options. Zero-initialise, set struct_size = sizeof(s2lc_opts).
 * A caller built against the first layout (up to `stream`) still works: the
 * fields after it then keep their zero defaults. */
#define S2LC_F_NO_WITNESS 0x1u     /* do not record the witness trace */
#define S2LC_F_ROUND_COUNTS 0x2u   /* record every round's unique-configuration count
                                      (s2lc_batch_round_counts; search-parity tests) */

/* Search engine routing (tests / diagnostics). AUTO picks per history:
 * packed lane groups (K <= 32), one workgroup per history (K <= 128), the
 * device-wide level search (K > 128, or a frontier beyond a workgroup). */
enum s2lc_engine {
  S2LC_ENGINE_AUTO = 0,
  S2LC_ENGINE_WORKGROUP = 1,     /* skip the packed kernels: workgroup passes (LDS, then HBM slab) */
  S2LC_ENGINE_WORKGROUP_HBM = 2, /* skip the packed kernels and the LDS pass: HBM-slab pass only */
  S2LC_ENGINE_LEVEL = 3          /* every history through the device-wide level search */
};

/* Verdict-exact search reductions that can be switched off for
 * ablation tests; the E-closure is the search's definition and stays on. */
#define S2LC_RED_P1 0x1u     /* tail lower bound of pending observers */
#define S2LC_RED_P2 0x2u     /* minimal read at the current tail with another hash */
#define S2LC_RED_P4 0x4u     /* nothing left constrains the state: complete */
#define S2LC_RED_IDEFER 0x8u /* indefinite append's identity outcome deferred to minret */

typedef struct s2lc_opts {
  uint32_t struct_size;
  int32_t device;          /* HIP device ordinal; -1 = current device */
  uint32_t flags;          /* S2LC_F_* */
  uint32_t _pad;
  uint64_t max_configs;    /* per-history budget of unique configurations; 0 = unlimited
                              (the search always terminates: it is bounded by n rounds) */
  void* stream;            /* hipStream_t to launch on; NULL = context-owned stream */
  /* ---- since ABI 2 ---- */
  uint64_t timeout_us;     /* CheckEventsVerbose's timeout (main.go:606) per s2lc_check /
                              s2lc_check_batch / s2lc_batch_run call: histories not decided
                              when it expires get Unknown (S2LC_R_TIMEOUT). 0 = none, the
                              reference CLI's setting: the result is then Ok or Illegal. */
  uint32_t engine;         /* s2lc_engine */
  uint32_t reductions_off; /* S2LC_RED_* bits to disable */
  const int32_t* devices;  /* s2lc_check_batch over several GPUs: HIP ordinals (an ordinal may
                              repeat: two shards on one GPU); NULL / n_devices 0 = {device}.
                              Histories are placed longest-processing-time first by
                              n_ops x chains; verdicts are gathered in input order. */
  uint32_t n_devices;      /* at most 16 */
  uint32_t _pad2;
} s2lc_opts;

/* Result of one history check. */
typedef struct s2lc_result {
  int32_t verdict;            /* s2lc_verdict */
  int32_t reason;             /* 0; or S2LC_R_* explaining Illegal/Unknown */
  uint64_t configs_explored;  /* unique (linearized set, state) configurations inserted */
  uint32_t rounds;            /* search rounds run (one non-identity op per round) */
  uint32_t n_ops;             /* operations in the history */
  uint32_t witness_len;       /* ops in *witness (n_ops when verdict == OK and witness on) */
  uint32_t _pad;
  int64_t* witness;           /* Event.Id of each op in linearization order; library-owned */
  double device_ms;           /* device time of the search launch(es) */
  /* Illegal: the linearized prefix of a configuration of the deepest round the
   * search reached (what porcupine's LinearizationInfo partial linearizations
   * show, main.go:607-611), certified like a witness; library-owned */
  int64_t* partial;
  uint32_t partial_len;
  uint32_t _pad2;
} s2lc_result;

#define S2LC_R_NONE 0
#define S2LC_R_UNMATCHED 1       /* a call without a later return, or a return without an
                                    earlier call: checkSingle can never empty its list */
#define S2LC_R_SEARCH_EXHAUSTED 2 /* no configuration survived */
#define S2LC_R_BUDGET 3          /* max_configs exceeded (Unknown) */
#define S2LC_R_FRONTIER 4        /* frontier exceeded device capacity (Unknown) */
#define S2LC_R_WITNESS_INVALID 5 /* the search found a linearization whose witness failed CPU
                                    replay (a checker bug; never expected): verdict Unknown and
                                    the call returns S2LC_EWITNESS */
#define S2LC_R_TIMEOUT 6         /* s2lc_opts.timeout_us expired before the verdict (Unknown) */

/* ----- LinearizationInfo: per-op longest partial linearizations ------------
 * porcupine.CheckEventsVerbose returns, beside the verdict, the longest
 * partial linearization containing each op (its DFS records one at every
 * backtrack; main.go:606), which Visualize renders (main.go:627).
 *   Ok: the certified witness, for every op (as porcupine records on success).
 *   Illegal: a second level search of the history with the pruning
 *     reductions off (P1, P2, P4 and the indefinite deferral: porcupine's DFS
 *     visits every reachable configuration of an Illegal history, and so must
 *     this one for the lengths to be porcupine's), recording per op the
 *     largest configuration that contains it. Each distinct one is rebuilt
 *     from the device trace and certified like a witness (a real-time-closed
 *     prefix whose every step the CPU model accepts).
 *   exact = 0 when that search stopped at its budget (the context's
 *     max_configs, else 2^22 configurations) or the device capacity: the
 *     partials are certified but may be shorter than porcupine's.
 * Free with s2lc_partials_free. */
typedef struct s2lc_partials {
  int32_t verdict;      /* the history's verdict (s2lc_verdict) */
  uint32_t exact;
  uint32_t n_ops;
  uint32_t n_partials;  /* distinct partial linearizations */
  int64_t* op_ids;      /* [n_ops] Event.Id of dense op d (first-appearance order) */
  uint32_t* op_partial; /* [n_ops] index of op d's longest partial, UINT32_MAX: in none */
  uint64_t* offs;       /* [n_partials + 1] */
  int64_t* ids;         /* Event.Ids of partial k in linearization order: ids[offs[k] .. offs[k+1]) */
} s2lc_partials;

/* ----- context ----------------------------------------------------------- */
s2lc_ctx* s2lc_create(const s2lc_opts* opts, int* status);
void s2lc_destroy(s2lc_ctx* ctx);
const char* s2lc_last_error(const s2lc_ctx* ctx);
const char* s2lc_version(void);

/* ----- histories (loader; main.go:529-563) --------------------------------- */
/* Decode a JSONL history: from path (or "-" = stdin) when buf == NULL, else
 * from buf[0..len). Accepts and rejects exactly what eventsFromReader does
 * (SURVEY.md A1). On error returns S2LC_EDECODE / S2LC_EIO and writes a
 * message into err. */
int s2lc_load_jsonl(const char* path_or_dash, const uint8_t* buf, size_t len,
                    s2lc_history** out, char* err, size_t errlen);
/* Decode n JSONL histories (DST seeds, C4) from memory, one worker thread per
 * core (n_threads <= 0) or n_threads: eventsFromReader per buffer, histories
 * being independent. All or nothing: on the first (lowest-index) failure every
 * out[i] is NULL, *err_index names the buffer and err its decode error. */
int s2lc_load_jsonl_many(const uint8_t* const* bufs, const size_t* lens, size_t n, int n_threads,
                         s2lc_history** out, size_t* err_index, char* err, size_t errlen);
/* Build a history from porcupine-style events; all buffers are copied. */
int s2lc_history_from_events(const s2lc_event* events, size_t n_events,
                             s2lc_history** out, char* err, size_t errlen);
/* Release a history. Its arrays are parked in a process-wide pool of released
 * histories (capacity kept) that the loaders decode the next histories into,
 * up to S2LC_HISTORY_POOL_MB of array capacity (default 2048; 0 = off: arrays
 * go back to the C heap here). */
void s2lc_history_free(s2lc_history* h);
/* Return every parked history's arrays to the C heap, and this thread's
 * decode / finalize scratch; returns the array bytes (capacity) released.
 * (s2lc_load_jsonl_many's other decoder threads live for one call: their
 * scratch is released when they exit; the calling thread's stays until this
 * call.) */
size_t s2lc_history_pool_trim(void);
size_t s2lc_history_event_count(const s2lc_history* h);
/* Export event i (pointers stay valid while h lives). */
int s2lc_history_get_event(const s2lc_history* h, size_t i, s2lc_event* out);
/* Bulk export of events [0, n); equal token strings share one pointer. */
int s2lc_history_get_events(const s2lc_history* h, s2lc_event* out, size_t n);

/* ----- binary SoA history cache --------------------
 * eventsFromReader (main.go:529-563) decodes every history from JSONL on every
 * run. The cache is the decoded, finalized form (events, record-hash pool,
 * tokens, the chain-major record table and its index arrays) as one byte
 * image; loading it skips JSON decode and the chain decomposition.
 * save_many: *out (free with s2lc_free) holds n histories.
 * load_many: out[0 .. *n) get new histories (free each with
 * s2lc_history_free); out == NULL only sets *n. Parallel over histories
 * (n_threads == 1: serial). Every array is bounds-checked against the image;
 * a malformed image gives S2LC_EDECODE and no histories. */
int s2lc_history_save_many(const s2lc_history* const* hs, size_t n, uint8_t** out, size_t* out_len);
int s2lc_history_load_many(const uint8_t* buf, size_t len, int n_threads, s2lc_history** out, size_t cap,
                           size_t* n);

typedef struct s2lc_history_info {
  uint32_t n_events;
  uint32_t n_ops;
  uint32_t n_chains;        /* K: greedy interval-colouring chain count */
  uint32_t n_tokens;
  uint64_t n_record_hashes;
  int32_t structural;       /* 0 = well formed, S2LC_R_UNMATCHED */
  uint32_t n_identity_ops;  /* reads, check-tails, definite failures */
} s2lc_history_info;
int s2lc_history_info_get(const s2lc_history* h, s2lc_history_info* out);

/* ----- checker (porcupine.CheckEventsVerbose, main.go:606) ------------------ */
int s2lc_check(s2lc_ctx* ctx, const s2lc_history* h, s2lc_result* out);
int s2lc_check_batch(s2lc_ctx* ctx, const s2lc_history* const* hs, size_t n, s2lc_result* out);
void s2lc_result_free(s2lc_result* r);
/* LinearizationInfo (above) of one history; 0 or an s2lc_status. */
int s2lc_check_partials(s2lc_ctx* ctx, const s2lc_history* h, s2lc_partials* out);
void s2lc_partials_free(s2lc_partials* p); /* frees r->witness; r itself is caller storage */

/* Device-resident batches: upload once, check many times (bench / DST loops). */
int s2lc_batch_create(s2lc_ctx* ctx, const s2lc_history* const* hs, size_t n, s2lc_batch** out);
/* Replace the batch's histories with hs[0..n) on the same device buffers
 * (grown only when hs needs more): a DST loop streams history batches
 * through one device batch without reallocating. */
int s2lc_batch_load(s2lc_ctx* ctx, s2lc_batch* b, const s2lc_history* const* hs, size_t n);
/* s2lc_batch_run + s2lc_batch_results(..., with_witness = 1). */
int s2lc_batch_check(s2lc_ctx* ctx, s2lc_batch* b, s2lc_result* out /* [n] */);
/* Device work only: search every history, copy verdicts back. */
int s2lc_batch_run(s2lc_ctx* ctx, s2lc_batch* b);
/* Results of the last run; with_witness expands and replay-verifies witnesses
 * on the host (CPU model, powerset semantics). */
int s2lc_batch_results(s2lc_ctx* ctx, s2lc_batch* b, s2lc_result* out /* [n] */, int with_witness);
/* The same results as flat arrays, for bulk callers (no per-history
 * allocation crosses the boundary): per history verdict, reason, configs and
 * rounds; the Ok witnesses (certified exactly as by s2lc_batch_results)
 * concatenated into witness_ids, history i's at [witness_offs[i],
 * witness_offs[i+1]) (empty unless Ok). witness_offs has n + 1 entries;
 * with witness_ids NULL no witness is rebuilt (every range empty), else it
 * must hold ids_cap >= the total (the sum of the histories' n_ops always
 * suffices). Any output pointer but witness_offs may be NULL. Returns
 * S2LC_EWITNESS like s2lc_batch_results. */
int s2lc_batch_results_flat(s2lc_ctx* ctx, s2lc_batch* b, int32_t* verdicts, int32_t* reasons, uint64_t* configs,
                            uint64_t* rounds, int64_t* witness_ids, size_t ids_cap, uint64_t* witness_offs);
void s2lc_batch_free(s2lc_batch* b);

typedef struct s2lc_batch_stats {
  double kernel_ms;          /* main search launch, HIP events on the ctx stream */
  double total_ms;           /* whole s2lc_batch_check including overflow reruns */
  uint64_t configs_explored; /* sum over histories */
  uint64_t children_generated;
  uint64_t rounds;           /* sum over histories */
  uint64_t algo_bytes;       /* algorithmic bytes of the main launch */
  uint32_t n_overflow;       /* histories re-run on the wide path */
  uint32_t launches;
  /* device-wide level search (histories with > 128 chains or a frontier
   * beyond the per-workgroup passes) */
  double level_ms;           /* device time of the level search, included in kernel_ms */
  uint32_t level_histories;
  uint32_t level_max_frontier;
  uint64_t level_rounds;
  uint64_t level_configs;
  uint64_t level_children;
  /* the dominant kernel of small-history batches: pack_kernel<16> (one 16-lane
   * group per history with <= 16 chains) */
  double pack16_ms;          /* its launch, HIP events on the ctx stream */
  uint64_t pack16_algo_bytes;/* algorithmic bytes of the histories it settled */
  uint32_t pack16_histories;
  uint32_t pack16_small;     /* of pack16_histories: settled from 32-byte records (every history of the list has
                                tails <= 65,532, < 65,535 events and hash counts < 65,536; S2LC_PACK_SMALL=0: never) */
  /* level search round modes: rounds run inside the persistent kernel, its
   * launches, frontier-chunk re-runs after a staging overflow, host syncs */
  uint64_t level_persist_rounds;
  uint32_t level_persist_launches;
  uint32_t level_chunk_retries;
  uint32_t level_syncs;
  uint32_t level_solo_rounds;/* one-configuration rounds run by one workgroup (LvSolo) */
  uint64_t n_ops_total;      /* ops over the batch's histories (sizes s2lc_batch_results_flat's ids) */
  /* pack_kernel<8>: histories with at most 8 chains (every C4 history), one
   * 8-lane group each */
  double pack8_ms;
  uint64_t pack8_algo_bytes;
  uint32_t pack8_histories;
  uint32_t _pad3;
  /* level searches restarted with host-driven rounds because a persistent
   * launch was refused or its grid barrier timed out (a workgroup never became
   * resident: another process holding CUs). Not an error: same verdict. */
  uint32_t level_persist_fallbacks;
  uint32_t _pad4;
  /* level search time by round width (device wall clock, per round): rounds
   * on frontiers narrower than 4,096 configurations (persistent, solo and
   * host-driven narrow rounds: the part the distributed search replicates on
   * every rank) and wider ones (the part it partitions) */
  double level_narrow_ms;
  double level_wide_ms;
  double level_solo_ms;      /* of level_narrow_ms: the one-configuration (solo) rounds */
  uint32_t level_grows;      /* staging capacity raised after an overflowing round (starts at 2 GiB) */
  uint32_t _pad5;
} s2lc_batch_stats;
int s2lc_batch_stats_get(const s2lc_batch* b, s2lc_batch_stats* out);
/* Totals over every successful s2lc_batch_run of b since it was created:
 * runs, and the sums of their kernel_ms / pack16_ms / pack8_ms (a caller that
 * times many runs reads these once before and once after, instead of the
 * stats after every run). Any pointer may be NULL. */
int s2lc_batch_run_totals(const s2lc_batch* b, uint64_t* runs, double* kernel_ms_sum, double* pack16_ms_sum,
                          double* pack8_ms_sum);
/* With S2LC_F_ROUND_COUNTS: the unique-configuration count of each completed
 * round of history i's last search, rounds 0 .. *n-1 (round 0 = the closed
 * initial configuration). With out == NULL only *n is set. */
int s2lc_batch_round_counts(const s2lc_batch* b, size_t i, uint32_t* out, size_t cap, size_t* n);

/* ----- model (s2Model, main.go:253-340) ------------------------------------ */
/* Step op op_index (dense id, first-appearance order) of history h from
 * state *s; writes 0, 1 or 2 successor states, returns the count. */
int s2lc_step_cpu(const s2lc_history* h, const s2lc_state* s, uint32_t op_index, s2lc_state out[2]);
uint64_t s2lc_chain_hash(uint64_t stream_hash, uint64_t record_hash);
uint64_t s2lc_fold_record_hashes(uint64_t stream_hash, const uint64_t* record_hashes, size_t n);
/* foldRecordHashes on the GPU, through the same device routine the search
 * kernels use: out[i] = fold(seeds[i], pool[offs[i] .. offs[i] + cnts[i])).
 * Host buffers in and out (known-answer tests of the device hash). */
int s2lc_device_fold(s2lc_ctx* ctx, const uint64_t* seeds, const uint64_t* pool, size_t pool_len,
                     const uint32_t* offs, const uint32_t* cnts, size_t n, uint64_t* out);
/* Replay a linearization (op indices) through the CPU model; 0 if every op
 * is accepted in order and every op appears exactly once, else -1. */
int s2lc_replay(const s2lc_history* h, const uint32_t* order, size_t n);

/* Rebuild a full linearization from a witness move list (one u32 per round:
 * chain | 0x10000 for an indefinite append taken as not applied), re-deriving
 * the identity ops, and certify it: real-time order + every op's claimed
 * outcome is a successor under s2Model.Step (main.go:264-335). Writes the
 * Event.Ids in order into out_ids[cap >= n_ops] when out_ids != NULL.
 * 0 = valid, -1 = not a valid linearization. */
int s2lc_witness_from_moves(const s2lc_history* h, const uint32_t* moves, size_t n_moves, int p4,
                            int64_t* out_ids, size_t cap);

/* s2Model.DescribeOperation (main.go:341-352, formatAppendCall /
 * formatReadCall / formatCheckTailCall main.go:362-426) of op op_index (dense,
 * as s2lc_step_cpu): written NUL-terminated into buf[cap] (truncated to fit);
 * returns the full length without the NUL, or a negative error. */
int s2lc_describe_operation(const s2lc_history* h, uint32_t op_index, char* buf, size_t cap);
/* s2Model.DescribeState (main.go:353-360) of s, whose token is an interned id
 * of h (0 = nil); same buffer convention. */
int s2lc_describe_state(const s2lc_history* h, const s2lc_state* s, char* buf, size_t cap);

/* porcupine.Visualize(model, info, file) (main.go:608-631): write an HTML page
 * for a checked history — each client's ops on the event axis, labelled with
 * DescribeOperation (main.go:341-426), and the witness (Ok) or the deepest
 * certified prefix (Illegal) with the powerset state after each op
 * (DescribeState). r is the s2lc_check result for h. */
int s2lc_visualize(const s2lc_history* h, const s2lc_result* r, const char* path);
/* The same page with LinearizationInfo (s2lc_check_partials): hovering an op
 * outlines the longest partial linearization containing it, as porcupine's
 * Visualize does; info may be NULL. */
int s2lc_visualize_info(const s2lc_history* h, const s2lc_result* r, const s2lc_partials* info, const char* path);

/* ----- distributed search of ONE history (BASELINE config C5) --------------
 * One rank per GPU; configurations are owned by a hash of their fingerprint.
 * The library does the device work; the caller owns the exchange (RCCL
 * all-to-all through torch.distributed in s2_verification_amd.distributed,
 * or any transport) and the device buffers it exchanges. Per round:
 *   s2lc_dist_expand  -> counts[w] configurations for each owner rank w, and
 *                        whether a child completed (Ok anywhere ends the search)
 *   (exchange counts; send buffer of sum(counts) * config_bytes)
 *   s2lc_dist_pack    -> owner-major configurations into the send buffer
 *   (all-to-all(v) of the configurations)
 *   s2lc_dist_insert  -> dedupe the received configurations (device buffer,
 *                        kept alive by the caller until the next insert):
 *                        they are this rank's next frontier; n_next = its size
 *   an all-reduce of n_next decides Illegal (0 on every rank).
 * Trace ids: rank << 29 | index into that rank's pool (s2lc_dist_trace). */
typedef struct s2lc_dist s2lc_dist;
typedef struct s2lc_dist_info_t {
  uint64_t config_bytes;   /* bytes per configuration on the wire */
  uint32_t n_chains;
  uint32_t round;          /* rounds completed (inserts) */
  uint32_t frontier;       /* local frontier size */
  uint32_t found_parent;   /* trace id of the completing child's parent (after expand reported found) */
  uint32_t found_move;
  uint32_t found_p4;
  uint64_t configs;        /* unique configurations owned by this rank so far */
  uint64_t children;       /* children generated by this rank */
  uint64_t max_frontier;
  double device_ms;        /* device time of this rank's kernels */
  uint64_t trace_len;
  uint64_t frontier_cap;   /* configurations one round may insert on this rank (world x exchange cap <= this) */
} s2lc_dist_info_t;
int s2lc_dist_create(s2lc_ctx* ctx, const s2lc_history* h, int rank, int world, s2lc_dist** out);
void s2lc_dist_free(s2lc_dist* d);
int s2lc_dist_expand(s2lc_dist* d, uint64_t* counts /* [world] */, int32_t* found);
int s2lc_dist_pack(s2lc_dist* d, void* send /* device */, const uint64_t* counts /* [world] */);
int s2lc_dist_insert(s2lc_dist* d, void* recv /* device */, uint64_t n_recv, uint64_t* n_next);
int s2lc_dist_info(const s2lc_dist* d, s2lc_dist_info_t* out);
/* Narrow frontiers run REPLICATED: every rank runs the same round on the whole
 * frontier with no exchange (the configuration set, and so every decision, is
 * identical on all ranks); the driver switches to the partitioned rounds above
 * when the frontier is wide and back when it is narrow again.
 *   s2lc_dist_local_round   one replicated round (round 0 included);
 *                           n_next = frontier size, found = a child completed
 *   s2lc_dist_local_run     replicated rounds inside one resident kernel (the
 *                           single-GPU engine's persistent and solo rounds)
 *                           until the frontier reaches `wide` or the search
 *                           ends; rounds = rounds run; S2LC_EUNSUPPORTED when
 *                           not available (before round 0, or a layout without
 *                           the persistent kernel): use s2lc_dist_local_round
 *   s2lc_dist_keep_owned    replicated -> partitioned: keep the owned configurations
 *   s2lc_dist_frontier_pack partitioned -> replicated: this rank's frontier,
 *                           frontier * config_bytes bytes, into a device buffer
 *   s2lc_dist_frontier_load the all-gathered frontier (device buffer kept alive
 *                           by the caller) becomes every rank's frontier */
int s2lc_dist_local_round(s2lc_dist* d, uint64_t* n_next, int32_t* found);
int s2lc_dist_local_run(s2lc_dist* d, uint32_t wide, uint64_t* n_next, int32_t* found, uint32_t* rounds);
int s2lc_dist_keep_owned(s2lc_dist* d, uint64_t* n_kept);
int s2lc_dist_frontier_pack(s2lc_dist* d, void* buf);
int s2lc_dist_frontier_load(s2lc_dist* d, void* buf, uint64_t n);
/* Host-free partitioned rounds: the driver queues rounds with no host
 * synchronization and reads each round's status a round or two later.
 *   s2lc_dist_x_begin   the device run state from this rank's frontier (after
 *                       s2lc_dist_keep_owned or a partitioned round)
 *   s2lc_dist_x_send    expand + close the frontier and copy the staged
 *                       children the OTHER ranks own into world - 1
 *                       fixed-capacity blocks of (cap + 1) * config_bytes
 *                       bytes, in rank order without this rank, a header in
 *                       each block's first slot (count, found, staging
 *                       overflow, the sender's largest block and staged
 *                       total); this rank's own share stays in its staging
 *                       (send may be NULL with world 1: nothing travels)
 *   (caller)            all-to-all of one block to every other rank (fixed
 *                       split sizes, none for itself: no sizes on the host)
 *   s2lc_dist_x_recv    decide the round from the received headers and its
 *                       own, insert the received configurations and its own
 *                       share; *round = its number; recv and the library's
 *                       staging are the next frontier (recv kept alive by the
 *                       caller for at least 8 rounds: a re-run reads it;
 *                       NULL with world 1)
 *   s2lc_dist_x_wait    wait for a queued round and read its status; every
 *                       rank reads the same decision
 *   s2lc_dist_x_rewind  a round whose status is S2LC_DIST_X_CAPACITY inserted
 *                       nothing: drop it and the rounds queued after it, so
 *                       the next send re-runs it (with a larger cap)
 *   s2lc_dist_x_end     wait for everything queued; the host-side state
 *                       (s2lc_dist_info, the frontier) catches up; *done =
 *                       the stop (S2LC_DIST_X_*), *configs = configurations
 *                       this rank inserted since s2lc_dist_x_begin */
enum {
  S2LC_DIST_X_RUNNING = 0,
  S2LC_DIST_X_FOUND = 1,     /* a child completed on some rank: Ok */
  S2LC_DIST_X_EMPTY = 2,     /* no rank staged a child: Illegal */
  S2LC_DIST_X_CAPACITY = 4,  /* an exchange block over its capacity: rewind and re-run */
  S2LC_DIST_X_ABORT = 5      /* a rank's staging overflowed (device buffers) */
};
typedef struct s2lc_dist_xstat {
  uint32_t ran;        /* the round ran and published its status (0: the run had stopped before it) */
  uint32_t done;       /* S2LC_DIST_X_* decided in this round */
  uint32_t nf;         /* this rank's next frontier */
  uint32_t maxblk;     /* the largest block any rank sent: the capacity this round needed */
  uint64_t nf_global;  /* the global frontier this round expanded */
  uint64_t staged;     /* configurations staged by all ranks this round */
} s2lc_dist_xstat;
int s2lc_dist_x_begin(s2lc_dist* d);
int s2lc_dist_x_send(s2lc_dist* d, void* send /* device */, uint32_t cap);
int s2lc_dist_x_recv(s2lc_dist* d, void* recv /* device */, uint32_t cap, uint32_t* round);
int s2lc_dist_x_wait(s2lc_dist* d, uint32_t round, s2lc_dist_xstat* out);
int s2lc_dist_x_rewind(s2lc_dist* d, uint32_t round);
int s2lc_dist_x_end(s2lc_dist* d, uint32_t* done, uint64_t* configs);
/* Copy this rank's trace pool ({parent id, move} u32 pairs) to host memory;
 * with out_pairs == NULL only *n is set. */
int s2lc_dist_trace(s2lc_dist* d, uint32_t* out_pairs, uint64_t cap_entries, uint64_t* n);

/* ----- deterministic S2 simulator (collector workload, history.rs) ---------- */
enum s2lc_workflow { S2LC_WF_REGULAR = 0, S2LC_WF_MATCH_SEQ_NUM = 1, S2LC_WF_FENCING = 2 };
enum s2lc_violation {
  S2LC_VIOL_NONE = 0,
  S2LC_VIOL_READ_HASH = 1,     /* perturb one ReadSuccess stream_hash (cf. main_test.go:349-374) */
  S2LC_VIOL_DEFINITE_APPLIED = 2, /* a definite failure that was applied (cf. :192-232) */
  S2LC_VIOL_TAIL = 3,          /* one success tail off by one */
  S2LC_VIOL_STALE_MSN = 4      /* msn append applied despite a stale msn (cf. :315-343) */
};
typedef struct s2lc_sim_params {
  uint32_t struct_size;
  uint32_t workflow;           /* s2lc_workflow */
  uint32_t num_clients;        /* --num-concurrent-clients (collect-history.rs) */
  uint32_t ops_per_client;     /* --num-ops-per-client */
  uint64_t seed;
  double p_indefinite;         /* append -> AppendIndefiniteFailure */
  double p_definite;           /* append -> AppendDefiniteFailure (transient) */
  double p_read_failure;
  double p_check_tail_failure;
  uint64_t initial_records;    /* > 0: pre-existing stream, rectifying append (history.rs:641-670) */
  uint32_t violation;          /* s2lc_violation */
  uint32_t max_client_ids;     /* 0 = 20 (history.rs:33) */
} s2lc_sim_params;
void s2lc_sim_params_default(s2lc_sim_params* p);
/* Emit a collector-format JSONL history (library-owned buffer, s2lc_free). */
int s2lc_simulate_jsonl(const s2lc_sim_params* p, uint8_t** out, size_t* len);
/* Same history, directly as an s2lc_history (no JSON round trip). */
int s2lc_simulate_history(const s2lc_sim_params* p, s2lc_history** out);
void s2lc_free(void* p);

#ifdef __cplusplus
}
#endif
#endif /* S2LINCHECK_H */
