// search.h — device data layout of the frontier search and its host launcher.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <vector>

#include "history.h"

namespace s2lc {

constexpr uint32_t TRACE_NONE = 0xFFFFFFFFu;
constexpr uint32_t MOVE_IDENT = 0x10000u;   // I-op taken with its identity outcome

struct HistDesc {
  uint32_t rec_base;   // first OpRec of the history in the batch table
  uint32_t cs_base;    // chain_start entries (K+1, absolute rec indices)
  uint16_t K;
  uint16_t flags;      // H_NOWRAP | H_P2OK
  uint32_t n_ops;
};

// A history's op record in 32 bytes, for histories whose tails, event
// indices and per-op hash counts fit 16 bits (HistDesc flag H_SMALL, set at
// upload): the packed kernels read these (a window of two records is 16
// registers instead of 32). Values the packed search only compares with
// reachable tails (msn, out_tail) saturate to 0xFFFF above 65,532, which no
// reachable tail equals; a P1 bound above 65,532 (never pruning) is 0xFFFD,
// REQ_HASH_ONLY 0xFFFE, REQ_NONE 0xFFFF; EV_INF is 0xFFFF.
struct __attribute__((aligned(32))) SRec {
  uint64_t out_hash;
  uint32_t hash_off;     // batch-wide pool offset
  uint16_t num_records, msn, out_tail, suf;
  uint16_t call_ev, ret_ev, hash_cnt, flags;
  uint16_t batch_tok, set_tok;
};
static_assert(sizeof(SRec) == 32, "SRec is 32 bytes");
constexpr uint16_t H_SMALL = 0x20;  // HistDesc.flags: the history's SRec table is exact (above)

// OpRec -> SRec (the host packs H_SMALL histories' records in this form)
inline SRec to_srec(const OpRec& x) {
  auto sat = [](uint64_t v) -> uint16_t { return v <= 65532u ? (uint16_t)v : (uint16_t)0xFFFFu; };
  SRec y;
  y.out_hash = x.out_hash;
  y.hash_off = x.hash_off;
  y.num_records = (uint16_t)(x.num_records < 0xFFFFu ? x.num_records : 0xFFFFu);
  y.msn = sat(x.msn);
  y.out_tail = sat(x.out_tail);
  y.suf = x.sufmin == REQ_NONE ? (uint16_t)0xFFFFu
        : x.sufmin == REQ_HASH_ONLY ? (uint16_t)0xFFFEu
        : x.sufmin <= 65532u ? (uint16_t)x.sufmin : (uint16_t)0xFFFDu;
  y.call_ev = (uint16_t)(x.call_ev < 0xFFFFu ? x.call_ev : 0xFFFFu);
  y.ret_ev = (uint16_t)(x.ret_ev < 0xFFFFu ? x.ret_ev : 0xFFFFu);
  y.hash_cnt = (uint16_t)(x.hash_cnt < 0xFFFFu ? x.hash_cnt : 0xFFFFu);
  y.flags = (uint16_t)x.flags;
  y.batch_tok = x.batch_tok;
  y.set_tok = x.set_tok;
  return y;
}

// SRec -> OpRec (on the device, for the engines that read 64-byte records).
// Not bit-exact where SRec saturates, but equal in every comparison the
// search makes for an H_SMALL history: a saturated msn / out_tail (0xFFFF)
// equals no reachable tail, as the original did not, and a P1 bound of
// 0xFFFD passes every reachable tail, as the original did.
__host__ __device__ inline OpRec from_srec(const SRec& y) {
  OpRec x;
  x.num_records = y.num_records;
  x.msn = y.msn;
  x.out_tail = y.out_tail;
  x.out_hash = y.out_hash;
  x.sufmin = y.suf == 0xFFFFu ? REQ_NONE : y.suf == 0xFFFEu ? REQ_HASH_ONLY : (uint64_t)y.suf;
  x.call_ev = y.call_ev == 0xFFFFu ? EV_INF : y.call_ev;
  x.ret_ev = y.ret_ev == 0xFFFFu ? EV_INF : y.ret_ev;
  x.hash_off = y.hash_off;
  x.hash_cnt = y.hash_cnt;
  x.batch_tok = y.batch_tok;
  x.set_tok = y.set_tok;
  x.flags = y.flags;
  return x;
}

struct TraceEnt {
  uint32_t parent;  // trace index of the parent configuration
  uint32_t move;    // chain | MOVE_IDENT
};

enum : uint32_t { V_OK = 0, V_ILLEGAL = 1, V_UNKNOWN = 2 };

struct HistResult {
  uint32_t verdict;
  uint32_t reason;
  uint32_t rounds;
  uint32_t final_parent;  // trace index of the parent of the completing config
  uint32_t final_move;    // move that produced it
  uint32_t p4;            // completed by the "no constraining op left" rule
  uint64_t configs;       // unique configurations inserted
  uint64_t children;      // successor configurations generated
  uint32_t witness_off;   // into the witness move buffer
  uint32_t witness_len;   // moves written (rounds on the path)
  uint32_t has_witness;   // 0 none, 1 moves valid, 2 pending (set by search, resolved by walk)
  uint32_t deep_trace;    // Illegal: trace index of a configuration of the deepest non-empty round
  uint32_t deep_len;      // Illegal: its depth (moves on its path); the walk writes them as a partial
  uint32_t _pad;
};
static_assert(sizeof(HistResult) == 64, "HistResult is 64 bytes");

// The literal engine (literal.hip: porcupine's checkSingle, one thread per
// duplicate-id history).
struct LitDesc {
  uint32_t h;         // batch history index
  uint32_t n_ev;      // events
  uint32_t ev_off;    // first LitEv
  uint32_t W;         // bitset words (porcupine: len(entries) / 2 bits)
  uint64_t mem_off;   // this history's work slice in the literal buffer
  uint64_t mem_bytes;
  uint32_t moves_cap;  // witness slots (n_ops + 1)
  uint32_t _pad;
};
struct LitEv {
  OpRec rec;          // a call with a matched return: the op's record (batch pool offsets)
  int32_t id;         // porcupine's dense id (renumber)
  int32_t match;      // call: node of its matched return (event + 1), 0 = none; return: -1
  uint32_t kind;      // 0 call, 1 return
  uint32_t _pad;
};
static_assert(sizeof(LitEv) == 128, "LitEv layout (OpRec is 64-byte aligned)");

struct SearchGeom {
  bool shared;         // arrays in LDS (true) or in a per-workgroup HBM slab
  uint32_t block;      // threads per workgroup (64 or 256)
  uint32_t kmax;       // 16 / 32 / 64 / 128
  uint32_t fcap;       // frontier capacity per workgroup
  uint32_t stage_cap;  // staging entries
  uint32_t chunk;      // expansion items per chunk
  uint32_t ht_slots;   // power of two
  uint32_t grid;       // workgroups
  uint32_t win_recs;   // LDS record window (records; shared mode only)
  size_t cfg_bytes;
  size_t slab_bytes;   // HBM bytes per workgroup (0 when shared)
  size_t smem_bytes;   // dynamic LDS bytes per workgroup
};

// Buffers of the device-wide level search (level.hip), reused across histories.
struct LevelBufs {
  uint32_t nq = 0, scap = 0, ht_mask = 0;
  uint32_t scap_max = 0;                    // what the budget allows (a quarter of free HBM, <= 48 GiB)
  uint8_t* stg[2] = {nullptr, nullptr};     // staging arrays (frontier of round r = staging of round r-1)
  uint32_t* idx[2] = {nullptr, nullptr};    // frontier index lists
  unsigned long long* ht[2] = {nullptr, nullptr};  // dedupe tables: round r inserts into ht[r & 1]
  void* ctl = nullptr;                      // LvCtl[3] (host-enqueued rounds: ctl[r & 1]; persistent: ctl[r % 3])
  void* bar = nullptr;                      // LvBar (persistent rounds)
  void* run = nullptr;                      // LvRun (device)
  void* h_run = nullptr;                    // pinned host-mapped mirror of the run state
  void* h_ctl = nullptr;                    // pinned host copy of a control block (chunked rounds)
  hipEvent_t ev[2] = {nullptr, nullptr};
  size_t stg_bytes[2] = {0, 0}, idx_bytes[2] = {0, 0}, ht_bytes[2] = {0, 0};
  uint32_t grid_round = 0, grid_insert = 0, grid_nq = 0;  // resident grids (for grid_nq)
  uint32_t grid_persist = 0;                // lv_persist: one workgroup per CU
  bool coop = false;                        // lv_persist launched cooperatively (residency guaranteed)
  bool persist_refused = false;             // a persistent launch was refused or timed out: host-driven rounds
};

struct LevelStats {
  double ms = 0;
  uint64_t rounds = 0, configs = 0, children = 0;
  uint32_t max_frontier = 0, histories = 0, chunk_retries = 0;
  uint32_t grows = 0;  // staging capacity raised after an overflowing round
  uint32_t syncs = 0;  // host synchronizations (one per batch of device-driven rounds)
  uint64_t persist_rounds = 0, persist_launches = 0;  // rounds run inside lv_persist
  uint64_t solo_rounds = 0;  // of those, one-configuration rounds run by one workgroup
  uint32_t persist_fallbacks = 0;  // searches restarted host-driven (persistent launch refused / timed out)
  double narrow_ms = 0, wide_ms = 0;  // device wall time of rounds on frontiers < 4096 / >= 4096
  double solo_ms = 0;                 // of narrow: the solo rounds
};

// A batch of histories resident on one device. Every buffer is grown on
// demand and reused by later uploads/runs (a context's scratch batch serves
// s2lc_check with no device allocation once it is large enough):
//   device arena : recs | srecs | pool | chain_start | hist | order | res | moves | rcounts | list
//   pinned stage : recs | srecs | pool | chain_start | hist | order | res   (the uploaded prefix)
// An H_SMALL history's records are packed and uploaded as SRec only (half
// the bytes); a device kernel widens them into recs for the other engines.
// Every other history's records go up as OpRec; its srecs are never read.
struct DevBatch {
  int device = 0;
  uint32_t n_hist = 0;
  uint32_t kmax = 16;               // template KMAX of the workgroup passes (max K <= 128)
  uint32_t n_recs = 0, n_pool = 0;
  uint8_t* arena = nullptr;
  size_t arena_cap = 0;
  uint8_t* stage = nullptr;         // pinned host memory
  size_t stage_cap = 0;
  OpRec* recs = nullptr;
  SRec* srecs = nullptr;            // the same records in 32 bytes (H_SMALL histories: uploaded as such)
  uint64_t* pool = nullptr;
  uint32_t* chain_start = nullptr;
  HistDesc* hist = nullptr;
  uint32_t* order = nullptr;        // packed-kernel lists, LPT order: [K<=16 | 16<K<=32]
  HistResult* res = nullptr;
  uint32_t* moves = nullptr;        // witness moves (per history at witness_off)
  uint32_t* rcounts = nullptr;      // per-round unique configurations (same offsets as moves)
  uint32_t* list = nullptr;         // histories of a workgroup pass
  uint32_t n_pack8 = 0, n_pack16 = 0, n_pack32 = 0;  // packed-kernel lists (order[]: pack8 | pack16 | pack32)
  uint32_t pack8_kmax = 8;                            // K bound of the pack8 list (0: none)
  int pack_bpc[3] = {0, 0, 0};                        // resident pack_kernel<8/16/32> blocks per CU (0: not queried)
  int pack_bpc_s[3] = {0, 0, 0};                      // ... of the SRec (H_SMALL) instances
  bool list_small[3] = {false, false, false};         // every history of the packed list is H_SMALL
  uint64_t n_ops_total = 0;                           // ops over the uploaded histories
  std::vector<uint32_t> lpt;        // searchable histories, longest (n_ops x K) first
  std::vector<uint64_t> h_in_bytes; // per history: input SoA bytes (48 per op + 8 per record hash)
  LevelBufs lv;
  uint32_t* counter = nullptr;      // 2 x 32: work counters (scheduling) + the run's deadline (u64 at [16]) +
                                    // trace head ([24]), one set per run parity
  uint32_t run_par = 0;             // the next run's counter set
  TraceEnt* trace = nullptr;
  unsigned long long* trace_head = nullptr;
  uint64_t trace_cap = 0;
  uint8_t* slab = nullptr;
  size_t slab_cap = 0;
  hipEvent_t ev[8] = {nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr};
  // host views
  HistDesc* h_hist = nullptr;        // in stage
  HistResult* h_res = nullptr;       // in stage (pinned: the per-run read-back is a direct DMA)
  std::vector<uint32_t> h_moves_off; // witness_off per history
  uint64_t moves_cap = 0;
  uint32_t* h_moves = nullptr;       // pinned copy of the witness moves (results with witnesses)
  size_t h_moves_cap = 0;
  std::vector<uint32_t> h_rcounts;   // host copy of rcounts after a run with round counts
  bool rc_valid = false;
  // h_res not read back by the last run (every history settled by the packed
  // kernels: the run read their per-launch totals only); batch_host_results
  // copies it on first use
  bool h_res_stale = false;
  // duplicate-id histories (History::literal): the literal engine's tables
  std::vector<uint8_t> literal;      // per history
  std::vector<LitDesc> lit_desc;
  std::vector<LitEv> lit_ev;
  uint8_t* lit_meta = nullptr;       // device: descs | events
  uint8_t* lit_mem = nullptr;        // device: one work slice per literal history
  size_t lit_bytes = 0, lit_mem_bytes = 0;
  bool lit_dev_ready = false;
  bool force_reset = false;  // the next run must zero its counters with the reset dispatch
  // batch_run's engine routing of this load (the same for every run until
  // the key changes: the engine after the environment's override and
  // S2LC_MIDK_LEVEL_MAX), and the device's CU count: a C4 run's host
  // preparation was ~26 us of routing loops and attribute queries per run
  bool route_valid = false;
  uint32_t route_engine = 0, route_midk_max = 0, route_n_forced = 0;
  std::vector<uint32_t> route_todo, route_level;
  int route_dev = -1, route_n_cu = 0;
  uint32_t lit_chunk = 1;  // literal histories per launch (their slices share one buffer)
  unsigned long long* agg = nullptr;   // device: per packed launch, 8 totals (pack_kernel PackAgg)
  unsigned long long* h_agg = nullptr; // pinned copy
  uint64_t in_bytes_list[3] = {0, 0, 0};  // input SoA bytes of each packed list
  std::vector<const History*> src;   // host histories (not owned)
  std::vector<uint32_t> forced;      // per history: 0 search, else verdict fixed on host
  uint64_t algo_bytes_inputs = 0;
};

// Options of one batch_run (from the context, include/s2lincheck.h s2lc_opts).
struct RunOpts {
  uint64_t max_configs = 0;
  bool witness = true;
  bool round_counts = false;
  uint32_t engine = 0;               // s2lc_engine
  uint64_t timeout_us = 0;           // 0 = none
  unsigned long long* partial_max = nullptr;  // level search only: per-record longest-partial maxima (LvParams::pmax)
};

struct RunStats {
  double kernel_ms = 0, total_ms = 0, pass0_ms = 0;
  uint32_t n_overflow2 = 0;
  uint64_t configs = 0, children = 0, rounds = 0;
  uint64_t algo_bytes = 0;
  uint32_t n_overflow = 0, launches = 0;
  double pack_ms = 0;
  double pack16_ms = 0;              // pack_kernel<16> launch (HIP events)
  uint64_t pack16_algo_bytes = 0;    // algorithmic bytes of the histories it settled
  uint32_t pack16_histories = 0;
  uint32_t pack16_small = 0;     // of those: settled by the SRec instance (32-byte records)
  double pack8_ms = 0;               // pack_kernel<8> (K <= 8: every C4 history)
  uint64_t pack8_algo_bytes = 0;
  uint32_t pack8_histories = 0;
  LevelStats level;
};

// reductions_off: S2LC_RED_* bits cleared from every history's flags.
int batch_upload(DevBatch& b, const std::vector<const History*>& hs, uint32_t reductions_off, std::string& err);
void batch_release(DevBatch& b);
// Copy the witness moves of the last run into b.h_moves (pinned).
int batch_fetch_moves(DevBatch& b, std::string& err);
// the literal engine (literal.hip)
void literal_prepare(const History& h, uint32_t i, uint64_t pool_off, std::vector<LitDesc>& descs,
                     std::vector<LitEv>& evs);
int literal_run(DevBatch& b, hipStream_t stream, const RunOpts& ro, const unsigned long long* deadline,
                std::string& err);
void literal_release(DevBatch& b);
// h_res valid on the host (copies it if the last run left it on the device)
int batch_host_results(DevBatch& b, std::string& err);
// out[i] = fold_hashes_blk(seeds[i], pool[offs[i] ..+ cnts[i]]) on the device.
int device_fold(const uint64_t* seeds, const uint64_t* pool, size_t pool_len, const uint32_t* offs, const uint32_t* cnts,
                size_t n, uint64_t* out, hipStream_t stream, std::string& err);
int batch_run(DevBatch& b, hipStream_t stream, const RunOpts& ro, RunStats& st, std::string& err);

constexpr uint32_t LEVEL_KMAX = 512;  // most chains the level search handles
uint32_t level_nq(uint32_t K);  // register slots per lane: ceil(K / 64)
// deadline: steady-clock time in ns since epoch after which the search gives
// Unknown (S2LC_R_TIMEOUT); 0 = none.
// (d_deadline: the run's deadline on the device wall clock, nullable)
int level_search(DevBatch& b, uint32_t h, hipStream_t st, const RunOpts& ro, int64_t deadline_ns,
                 const unsigned long long* d_deadline, LevelStats& ls, std::string& err);
void level_release(DevBatch& b);
int64_t steady_ns();

// One rank's part of the distributed level search of a single history.
struct DistLevel {
  DevBatch b;                    // the history (one entry) + level buffers
  uint32_t rank = 0, world = 1, K = 0, nq = 0;
  size_t cb = 0;                 // bytes per configuration on the wire
  uint32_t* own_cnt = nullptr;
  uint32_t* own_pos = nullptr;
  TraceEnt* trace = nullptr;     // this rank's trace pool
  uint64_t trace_cap = 0, tnext = 0;
  hipStream_t stream = nullptr;
  bool own_stream = true;        // false: the context's (caller's) stream
  const uint8_t* cur = nullptr;  // current frontier: received buffer (caller-owned)
  const uint8_t* cur_loc = nullptr;  // partitioned rounds: its local part (LV_LOCAL entries, a staging array)
  int cur_sel = 0;               // index list of the current frontier: b.lv.idx[cur_sel]
  uint32_t nf = 0, slot_hi = 0, round = 0;  // slot_hi: staging walk bound (64 x longest stripe)
  uint32_t found_parent = TRACE_NONE, found_move = TRACE_NONE, found_p4 = 0;
  uint64_t configs = 0, children = 0, max_frontier = 0;
  double ms = 0;
  uint8_t* snap = nullptr;       // the frontier entering persistent replicated rounds (restored if they abort)
  size_t snap_cap = 0;
  // host-free partitioned rounds (dist_x_*): device run state, host-mapped
  // status ring, one event per ring entry, and the frontier each queued round
  // started from (a capacity overflow re-runs that round)
  void* xrun = nullptr;
  void* xstat = nullptr;
  hipEvent_t xev[8] = {};
  const uint8_t* xcur[8] = {};
  const uint8_t* xcur_loc[8] = {};
  int xsel[8] = {};
  void* xself = nullptr;         // this rank's own exchange header (its share is never sent)
  uint32_t xround = 0;           // the next round to queue
  bool xfresh = true;            // the next queued round zeroes its counters on the host
};
int dist_create(DistLevel& d, const History* h, uint32_t rank, uint32_t world, uint32_t reductions_off,
                hipStream_t stream, std::string& err);
void dist_release(DistLevel& d);
int dist_expand(DistLevel& d, uint64_t* counts, int* found, std::string& err);
int dist_pack(DistLevel& d, uint8_t* send, const uint64_t* counts, std::string& err);
int dist_insert(DistLevel& d, uint8_t* recv, uint64_t n_recv, uint64_t* n_next, std::string& err);
int dist_trace(DistLevel& d, uint32_t* out, uint64_t cap, uint64_t* n, std::string& err);
int dist_local_round(DistLevel& d, uint64_t* n_next, int* found, std::string& err);
int dist_local_run(DistLevel& d, uint32_t wide, uint64_t* n_next, int* found, uint32_t* rounds, std::string& err);
int dist_keep_owned(DistLevel& d, uint64_t* n_kept, std::string& err);
int dist_frontier_pack(DistLevel& d, uint8_t* buf, std::string& err);
int dist_frontier_load(DistLevel& d, uint8_t* buf, uint64_t n, std::string& err);
struct DistXStat { uint32_t ran, done, nf, maxblk; uint64_t nf_global, staged; };
int dist_x_begin(DistLevel& d, std::string& err);
int dist_x_send(DistLevel& d, uint8_t* send, uint32_t cap, std::string& err);
int dist_x_recv(DistLevel& d, uint8_t* recv, uint32_t cap, uint32_t* round, std::string& err);
int dist_x_wait(DistLevel& d, uint32_t round, DistXStat* out, std::string& err);
int dist_x_rewind(DistLevel& d, uint32_t round, std::string& err);
int dist_x_end(DistLevel& d, uint32_t* done, uint64_t* configs, std::string& err);

// Host reconstruction of a full linearization (dense op ids) from the device
// move list; returns false if any move is not a legal successor.
// ident[i] = 1 when order[i] took its identity outcome (E ops, indefinite
// appends taken as not applied).
// partial = true: a prefix (the path to a non-final configuration) is accepted.
bool rebuild_linearization(const History& h, const uint32_t* moves, uint32_t n_moves, bool p4,
                           std::vector<uint32_t>& order, std::vector<uint8_t>& ident, bool partial);
// A linearized prefix: distinct ops, real-time order within it, closed under
// real-time predecessors, and every claimed outcome a Step successor.
bool replay_prefix(const History& h, const uint32_t* order, const uint8_t* ident, size_t n);
// Every op exactly once, in an order that respects real time.
bool real_time_ok(const History& h, const uint32_t* order, size_t n);
// Powerset replay of a linearization through the CPU model (+ real-time
// check), porcupine's ToModel().Step semantics; false if the state set would
// exceed 2^16 states.
bool replay_order(const History& h, const uint32_t* order, size_t n);
// A duplicate-id history's literal-engine order through the powerset model.
bool replay_literal(const History& h, const uint32_t* order, size_t n);
// Single-path replay: real-time check, then every op's claimed outcome must be
// one of s2Model.Step's successors (main.go:264-335). A path of states is a
// certificate that the powerset run never empties.
bool replay_path(const History& h, const uint32_t* order, const uint8_t* ident, size_t n);
// rebuild_linearization (full, not partial) + replay_path in one pass: the
// replay steps each op with its own state as the rebuild writes it (the same
// checks, the two hash folds overlapped), then the real-time check.
bool rebuild_and_replay(const History& h, const uint32_t* moves, uint32_t n_moves, bool p4,
                        std::vector<uint32_t>& order, std::vector<uint8_t>& ident);

}  // namespace s2lc
