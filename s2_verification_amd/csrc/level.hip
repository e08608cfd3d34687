// level.hip — host driver of the device-wide level-synchronous search of one
// history (kernels in level_dev.h). Called by batch_run for histories with
// more than 128 chains and for histories whose frontier outgrew the
// per-workgroup passes. A round is lv_round (expand + close + stage) then
// lv_insert (dedupe; its last block closes the round on the device).
//
// Rounds are enqueued in batches with no host synchronization in between:
// every kernel reads the frontier size and the run state from device memory,
// and the kernels of a finished search return immediately. The host reads the
// host-mapped run state once per batch. Narrow frontiers use long batches
// (the round latency is then a few kernel launches); wide frontiers one round
// per batch, so the launch grids follow the frontier. A round whose staged
// configurations exceed the device buffers is re-run over chunks of its
// frontier (host-driven).
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <string>

#include "s2lincheck.h"
#include "search.h"
#include "search_dev.h"
#include "level_dev.h"

namespace s2lc {

namespace {

#define LVCHK(x)                                                         \
  do {                                                                   \
    hipError_t e_ = (x);                                                 \
    if (e_ != hipSuccess) {                                              \
      err = std::string(#x) + ": " + hipGetErrorString(e_);              \
      return S2LC_EHIP;                                                  \
    }                                                                    \
  } while (0)

enum LvKernel { LK_ROUND = 0, LK_INSERT, LK_BUCKET, LK_SCATTER, LK_KEEP, LK_GATHER, LK_CLOSE, LK_XSEND, LK_CLEAR };

size_t lv_cfg_bytes(uint32_t nq) { return 128 + 128 * (size_t)nq; }

// a host-driven round's bookkeeping, after its last chunk (one thread)
// S2LC_TAG_DROP (tests): bits cleared from the dedupe tables' tags and first
// slots (LvParams::tag_drop); unset or 0 in production
uint32_t lv_tag_drop() {
  const char* e = getenv("S2LC_TAG_DROP");
  return e ? (uint32_t)strtoul(e, nullptr, 0) : 0u;
}

__global__ void lv_close_kernel(LvParams p) { lv_close_round(p); }

template <int NQ>
hipError_t lv_launch(int which, uint32_t grid, const LvParams& p, hipStream_t st) {
  switch (which) {
    case LK_ROUND: hipLaunchKernelGGL(lv_round<NQ>, dim3(grid), dim3(LV_BLOCK), 0, st, p); break;
    case LK_INSERT: hipLaunchKernelGGL(lv_insert<NQ>, dim3(grid), dim3(LV_BLOCK), 0, st, p); break;
    case LK_BUCKET: hipLaunchKernelGGL(lv_bucket<NQ>, dim3(grid), dim3(LV_BLOCK), 0, st, p); break;
    case LK_SCATTER: hipLaunchKernelGGL(lv_scatter<NQ>, dim3(grid), dim3(LV_BLOCK), 0, st, p); break;
    case LK_KEEP: hipLaunchKernelGGL(lv_keep<NQ>, dim3(grid), dim3(LV_BLOCK), 0, st, p, (uint32_t)(p.tgid >> 29)); break;
    case LK_GATHER: hipLaunchKernelGGL(lv_gather_frontier<NQ>, dim3(grid), dim3(LV_BLOCK), 0, st, p); break;
    case LK_XSEND: hipLaunchKernelGGL(lv_xsend<NQ>, dim3(grid), dim3(LV_BLOCK), 0, st, p); break;
    case LK_CLEAR: hipLaunchKernelGGL(lv_clear_slots<NQ>, dim3(grid), dim3(LV_BLOCK), 0, st, p); break;
    default: hipLaunchKernelGGL(lv_close_kernel, dim3(1), dim3(1), 0, st, p); break;
  }
  return hipGetLastError();
}

// lv_persist's grid barrier needs every workgroup resident at once. A
// cooperative launch guarantees that or is refused before any work runs
// (hipErrorCooperativeLaunchTooLarge); a plain launch (devices without
// cooperative launches) relies on the occupancy query, and a workgroup that
// never becomes resident ends in the barrier's time-out (LVR_ABORT). Either
// way the caller goes on with host-driven rounds: neither is an error.
template <int NQ>
hipError_t lv_persist_t(uint32_t grid, const LvParams& p, const LvPersist& q, bool coop, hipStream_t st) {
  if (coop) {
    LvParams pp = p;
    LvPersist qq = q;
    void* args[] = {&pp, &qq};
    return hipLaunchCooperativeKernel(reinterpret_cast<const void*>(lv_persist<NQ>), dim3(grid), dim3(LV_BLOCK), args, 0, st);
  }
  hipLaunchKernelGGL(lv_persist<NQ>, dim3(grid), dim3(LV_BLOCK), 0, st, p, q);
  return hipGetLastError();
}

hipError_t lv_persist_launch(uint32_t nq, uint32_t grid, const LvParams& p, const LvPersist& q, bool coop,
                             hipStream_t st) {
  switch (nq) {
    case 1: return lv_persist_t<1>(grid, p, q, coop, st);
    case 2: return lv_persist_t<2>(grid, p, q, coop, st);
    case 3: return lv_persist_t<3>(grid, p, q, coop, st);
    case 4: return lv_persist_t<4>(grid, p, q, coop, st);
    case 5: return lv_persist_t<5>(grid, p, q, coop, st);
    case 6: return lv_persist_t<6>(grid, p, q, coop, st);
    case 7: return lv_persist_t<7>(grid, p, q, coop, st);
    default: return lv_persist_t<8>(grid, p, q, coop, st);
  }
}

hipError_t lv_dispatch(uint32_t nq, int which, uint32_t grid, const LvParams& p, hipStream_t st) {
  grid = std::max<uint32_t>(grid, 1);
  switch (nq) {
    case 1: return lv_launch<1>(which, grid, p, st);
    case 2: return lv_launch<2>(which, grid, p, st);
    case 3: return lv_launch<3>(which, grid, p, st);
    case 4: return lv_launch<4>(which, grid, p, st);
    case 5: return lv_launch<5>(which, grid, p, st);
    case 6: return lv_launch<6>(which, grid, p, st);
    case 7: return lv_launch<7>(which, grid, p, st);
    default: return lv_launch<8>(which, grid, p, st);
  }
}

int lv_ensure(void** p, size_t& cap, size_t need, std::string& err) {
  if (need <= cap && *p) return 0;
  if (*p) (void)hipFree(*p);
  *p = nullptr;
  cap = 0;
  LVCHK(hipMalloc(p, need));
  cap = need;
  return 0;
}

int n_cus(std::string& err) {
  int dev = 0, n = 256;
  LVCHK(hipGetDevice(&dev));
  (void)hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev);
  return n;
}

// persistent grids of lv_round<NQ> / lv_insert<NQ>: the blocks the chip holds at once
template <int NQ>
int lv_grids_t(LevelBufs& L, std::string& err) {
  const int n_cu = n_cus(err);
  int br = 1, bi = 1, bp = 0;
  LVCHK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&br, lv_round<NQ>, LV_BLOCK, 0));
  LVCHK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&bi, lv_insert<NQ>, LV_BLOCK, 0));
  LVCHK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&bp, lv_persist<NQ>, LV_BLOCK, 0));
  L.grid_round = (uint32_t)(std::max(1, br) * n_cu);
  L.grid_insert = (uint32_t)(std::max(1, bi) * n_cu);
  // lv_persist's grid barrier needs every block resident: one per CU (its
  // launch bound: one workgroup per CU, the whole register file). A
  // cooperative launch is refused when its grid cannot be co-resident; a
  // plain launch whose workgroup never becomes resident (another process
  // holding the CUs) times out at the barrier: either way the search goes on
  // host-driven (LVR_ABORT / persist_refused)
  L.grid_persist = bp >= 1 ? (uint32_t)n_cu : 0u;
  // (S2LC_PERSIST_GRID: fewer persistent workgroups; diagnostics: with 1,
  // the SQ counters of lv_persist are those of the solo rounds' workgroup)
  if (const char* e = getenv("S2LC_PERSIST_GRID"))
    if (L.grid_persist) L.grid_persist = std::max<uint32_t>(1, std::min<uint32_t>(L.grid_persist, (uint32_t)strtoul(e, nullptr, 10)));
  L.grid_nq = (uint32_t)NQ;
  int dev = 0, coop = 0;
  LVCHK(hipGetDevice(&dev));
  (void)hipDeviceGetAttribute(&coop, hipDeviceAttributeCooperativeLaunch, dev);
  L.coop = coop != 0 && !getenv("S2LC_PERSIST_PLAIN");  // S2LC_PERSIST_PLAIN=1: plain launches (tests)
  return 0;
}

int lv_grids(LevelBufs& L, uint32_t nq, std::string& err) {
  if (L.grid_nq == nq) return 0;
  switch (nq) {
    case 1: return lv_grids_t<1>(L, err);
    case 2: return lv_grids_t<2>(L, err);
    case 3: return lv_grids_t<3>(L, err);
    case 4: return lv_grids_t<4>(L, err);
    case 5: return lv_grids_t<5>(L, err);
    case 6: return lv_grids_t<6>(L, err);
    case 7: return lv_grids_t<7>(L, err);
    default: return lv_grids_t<8>(L, err);
  }
}

}  // namespace

uint32_t level_nq(uint32_t K) { return std::max<uint32_t>(1, std::min<uint32_t>(8, (K + 63) / 64)); }

// Staging capacity for `budget` bytes: two staging arrays and their index
// lists plus two tables of 2 slots per staged configuration (cb: the widest
// layout, so one allocation serves every history).
static uint64_t lv_scap_for(size_t budget, size_t cb) {
  uint64_t scap = std::min<uint64_t>(1ull << 25, (uint64_t)budget / (2 * cb + 2 * 4 + 2 * 2 * 8));
  scap = std::max<uint64_t>(scap, 64 * LV_STRIPES);
  if (const char* e = getenv("S2LC_LEVEL_SCAP")) {  // (tests) a small staging capacity: the overflow paths
    const uint64_t v = strtoull(e, nullptr, 10);
    if (v >= LV_STRIPES) scap = std::min<uint64_t>(scap, v);
  }
  return scap - scap % LV_STRIPES;  // whole stripes
}

static int lv_tables(LevelBufs& L, uint64_t scap, std::string& err) {
  uint64_t ht = 1024;
  while (ht < 2 * scap) ht <<= 1;
  for (int i = 0; i < 2; ++i)
    if (lv_ensure((void**)&L.ht[i], L.ht_bytes[i], ht * 8, err)) return S2LC_EHIP;
  for (int i = 0; i < 2; ++i) LVCHK(hipMemset(L.ht[i], 0xFF, ht * 8));
  LVCHK(hipStreamSynchronize(nullptr));  // (the null stream does not order the search's non-blocking one)
  L.ht_mask = (uint32_t)(ht - 1);
  return 0;
}

// The buffers start at 2 GiB (S2LC_LEVEL_BUDGET_MB overrides) and grow on a
// staging overflow (level_grow) up to the full budget: the first kernel
// after an allocation commits it, ~54 ms per GB on the MI355X box
// (tools/startup/big_alloc.cpp: 2.7 s for 50 GB), which a history that never
// needs the capacity should not pay.
int level_buffers(DevBatch& b, uint32_t nq, std::string& err, bool full) {
  LevelBufs& L = b.lv;
  (void)nq;
  if (L.ctl && (!full || L.scap >= L.scap_max)) return 0;
  size_t free_b = 0, total_b = 0;
  LVCHK(hipMemGetInfo(&free_b, &total_b));
  const size_t cb = lv_cfg_bytes(8);  // sized for the widest layout: reused by every history
  if (!L.scap_max) L.scap_max = (uint32_t)lv_scap_for(std::min<size_t>(free_b / 4, 48ull << 30), cb);
  size_t first = 2ull << 30;
  if (const char* e = getenv("S2LC_LEVEL_BUDGET_MB")) first = (size_t)strtoull(e, nullptr, 10) << 20;
  const uint64_t scap = full ? L.scap_max : std::min<uint64_t>(L.scap_max, lv_scap_for(first, cb));
  for (int i = 0; i < 2; ++i) {
    if (lv_ensure((void**)&L.stg[i], L.stg_bytes[i], scap * cb, err)) return S2LC_EHIP;
    if (lv_ensure((void**)&L.idx[i], L.idx_bytes[i], scap * sizeof(uint32_t), err)) return S2LC_EHIP;
  }
  if (lv_tables(L, scap, err)) return S2LC_EHIP;
  if (!L.ctl) LVCHK(hipMalloc(&L.ctl, 3 * sizeof(LvCtl)));
  if (!L.bar) LVCHK(hipMalloc(&L.bar, sizeof(LvBar)));
  if (!L.run) LVCHK(hipMalloc(&L.run, sizeof(LvRun)));
  if (!L.h_run) LVCHK(hipHostMalloc(&L.h_run, sizeof(LvRun), hipHostMallocMapped));
  if (!L.h_ctl) LVCHK(hipHostMalloc(&L.h_ctl, sizeof(LvCtl), hipHostMallocDefault));
  for (hipEvent_t& e : L.ev)
    if (!e) LVCHK(hipEventCreate(&e));
  L.nq = 8;
  L.scap = (uint32_t)scap;
  return 0;
}

// Raise the staging capacity (x8, up to the budget), keeping staging array
// `keep` and its index list (the frontier of the round to re-run); the tables
// are new and empty. Returns 1 when the capacity is already at the budget.
int level_grow(DevBatch& b, int keep, hipStream_t st, std::string& err) {
  LevelBufs& L = b.lv;
  if (L.scap >= L.scap_max) return 1;
  const size_t cb = lv_cfg_bytes(8);
  uint64_t scap = std::min<uint64_t>(L.scap_max, (uint64_t)L.scap * 8);
  scap -= scap % LV_STRIPES;
  LVCHK(hipStreamSynchronize(st));
  for (int i = 0; i < 2; ++i) {
    uint8_t* ns = nullptr;
    uint32_t* ni = nullptr;
    LVCHK(hipMalloc(&ns, scap * cb));
    LVCHK(hipMalloc(&ni, scap * sizeof(uint32_t)));
    if (i == keep) {
      LVCHK(hipMemcpy(ns, L.stg[i], (size_t)L.scap * cb, hipMemcpyDeviceToDevice));
      LVCHK(hipMemcpy(ni, L.idx[i], (size_t)L.scap * sizeof(uint32_t), hipMemcpyDeviceToDevice));
    }
    (void)hipFree(L.stg[i]);
    (void)hipFree(L.idx[i]);
    L.stg[i] = ns; L.stg_bytes[i] = scap * cb;
    L.idx[i] = ni; L.idx_bytes[i] = scap * sizeof(uint32_t);
  }
  if (lv_tables(L, scap, err)) return S2LC_EHIP;
  L.scap = (uint32_t)scap;
  return 0;
}

void level_release(DevBatch& b) {
  LevelBufs& L = b.lv;
  void* ptrs[] = {L.stg[0], L.stg[1], L.idx[0], L.idx[1], L.ht[0], L.ht[1], L.ctl, L.bar, L.run};
  for (void* q : ptrs) if (q) (void)hipFree(q);
  if (L.h_run) (void)hipHostFree(L.h_run);
  if (L.h_ctl) (void)hipHostFree(L.h_ctl);
  for (hipEvent_t e : L.ev) if (e) (void)hipEventDestroy(e);
  L = LevelBufs{};
}

int level_search(DevBatch& b, uint32_t h, hipStream_t st, const RunOpts& ro, int64_t deadline_ns,
                 const unsigned long long* d_deadline, LevelStats& ls, std::string& err) {
  const HistDesc& hd = b.h_hist[h];
  const uint32_t K = hd.K;
  const uint32_t nq = level_nq(K);
  if (level_buffers(b, nq, err, false)) return S2LC_EHIP;
  LevelBufs& L = b.lv;
  if (lv_grids(L, nq, err)) return S2LC_EHIP;
  LvRun* hr = reinterpret_cast<LvRun*>(L.h_run);
  LvRun* d_pub = nullptr;  // device view of the host-mapped mirror
  LVCHK(hipHostGetDevicePointer((void**)&d_pub, hr, 0));
  LvRun* const run = reinterpret_cast<LvRun*>(L.run);
  LvCtl* const ctl = reinterpret_cast<LvCtl*>(L.ctl);
  size_t ht_bytes = ((size_t)L.ht_mask + 1) * 8;  // (grows with the staging capacity)

  // trace entries continue after what earlier passes / histories used
  unsigned long long tb0 = 0;
  if (ro.witness && b.trace) {
    LVCHK(hipMemcpyAsync(&tb0, b.trace_head, sizeof tb0, hipMemcpyDeviceToHost, st));
    LVCHK(hipStreamSynchronize(st));
  }
  const bool wit0 = ro.witness && b.trace != nullptr && tb0 + L.scap <= b.trace_cap;

  LvParams p;
  memset(&p, 0, sizeof p);
  p.tag_drop = lv_tag_drop();
  p.recs = b.recs; p.pool = b.pool; p.cs = b.chain_start + hd.cs_base; p.K = K; p.hflags = hd.flags;
  p.scap = L.scap; p.scs = L.scap / LV_STRIPES; p.ht_mask = L.ht_mask;
  p.trace = b.trace; p.trace_cap = b.trace_cap;
  p.run = run; p.publish = d_pub; p.close_round = 1; p.publish_always = 1;
  p.rcounts = ro.round_counts ? b.rcounts + b.h_moves_off[h] : nullptr;
  p.pmax = ro.partial_max;  // (every configuration goes through lv_insert: host-driven rounds, no fusion)

  // persistent narrow rounds (lv_persist): S2LC_NO_PERSIST=1 turns them off,
  // S2LC_PERSIST_NF sets the widest frontier they take (default: one wave each)
  bool persist_on = L.grid_persist > 0 && !L.persist_refused && !getenv("S2LC_NO_PERSIST") && !ro.partial_max;
  uint32_t persist_nf = L.grid_persist * (LV_BLOCK / 64);
  if (const char* e = getenv("S2LC_PERSIST_NF")) persist_nf = (uint32_t)strtoul(e, nullptr, 10);
  LvPersist pq;
  memset(&pq, 0, sizeof pq);
  pq.ctl3 = ctl; pq.bar = reinterpret_cast<LvBar*>(L.bar);
  for (int i = 0; i < 2; ++i) { pq.stg[i] = L.stg[i]; pq.idx[i] = L.idx[i]; pq.ht[i] = L.ht[i]; }
  // rounds per launch (the run's deadline is checked inside the launch too:
  // every grid round, every 16 solo rounds)
  pq.max_rounds = 4096;
  pq.deadline = d_deadline;
  pq.nf_max = persist_nf;
  pq.solo = getenv("S2LC_NO_SOLO") ? 0u : 1u;  // S2LC_NO_SOLO=1: one-configuration rounds on the grid too
  if (const char* e = getenv("S2LC_SOLO_MAXLIVE")) pq.solo_maxlive = (uint32_t)strtoul(e, nullptr, 10);
  // wide rounds: stage every child, then lv_insert dedupes (plain stores,
  // combined in L2); S2LC_WIDE_FUSED=1: lv_round inserts as it expands (CAS
  // first, so a duplicate is never written; measured slower on C5 / C5wide:
  // its write-through stores cost more HBM writes than the duplicates do)
  const uint32_t fused_wide = (getenv("S2LC_WIDE_FUSED") && !ro.partial_max) ? 1u : 0u;
  {
    int dev = 0, khz = 100000;
    LVCHK(hipGetDevice(&dev));
    (void)hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, dev);
    // a barrier wait above 2 s means a workgroup is not resident (plain launches;
    // S2LC_PERSIST_SPIN_US: a shorter limit, for the fallback's tests)
    unsigned long long us_ = 2000000;
    if (const char* e = getenv("S2LC_PERSIST_SPIN_US")) us_ = std::max<unsigned long long>(1, strtoull(e, nullptr, 10));
    pq.spin_ticks = std::max<unsigned long long>(1, (unsigned long long)khz * us_ / 1000);
  }

#ifdef S2LC_PROF
  unsigned long long* d_prof = nullptr;
  const size_t prof_n = 48 + 11 * (size_t)LV_PROF_ROUNDS;
  LVCHK(hipMalloc(&d_prof, prof_n * sizeof(unsigned long long)));
  LVCHK(hipMemset(d_prof, 0, prof_n * sizeof(unsigned long long)));
  LVCHK(hipStreamSynchronize(nullptr));
  p.prof = d_prof;
#endif
  LVCHK(hipEventRecord(L.ev[0], st));
  auto set_round = [&](uint32_t r) {
    const int w = (int)(r & 1), pr = (int)((r + 1) & 1);  // round r stages into w; its frontier is in pr
    p.round = r;
    p.cur = L.stg[pr]; p.cur_idx = L.idx[pr];
    p.stg = L.stg[w]; p.nxt_idx = L.idx[w];
    p.ht = L.ht[w]; p.ht_clear = L.ht[pr];
    p.ctl = ctl + w; p.ctl_next = ctl + pr;
  };
  bool timed_out = false;
  uint32_t syncs = 0;
  // A search runs once; when a persistent launch is refused or its barrier
  // times out (a workgroup never became resident: another process holding
  // CUs) it is run again from round 0 with host-driven rounds only.
  for (;;) {
    bool aborted = false;
    memset(hr, 0, sizeof(LvRun));
    LVCHK(hipMemsetAsync(L.ctl, 0, 3 * sizeof(LvCtl), st));
    hipLaunchKernelGGL(lv_run_init, dim3(1), dim3(1), 0, st, run, tb0, wit0 ? 1u : 0u,
                       (unsigned long long)ro.max_configs);
    LVCHK(hipGetLastError());
    // round 0: the closed initial configuration, staged into stg[0]
    set_round(0);
    p.init = 1; p.f0 = 0; p.f1 = 1; p.clear_slots = 0; p.close_round = 1; p.fused = 0;
    LVCHK(lv_dispatch(nq, LK_ROUND, 1, p, st));
    LVCHK(lv_dispatch(nq, LK_INSERT, 1, p, st));
    LVCHK(hipStreamSynchronize(st));
    p.init = 0;
    ++syncs;

    uint32_t next_round = 1;         // first round not yet enqueued
    uint32_t nf_last = hr->nf;        // frontier size at the last sync
    bool ctl_dirty = false;           // lv_persist left the double-buffer convention of ctl behind
    while (hr->done == LVR_RUNNING) {
      if (deadline_ns && steady_ns() > deadline_ns) { timed_out = true; break; }
      if (persist_on && nf_last <= persist_nf) {
        // narrow: rounds inside one resident launch until the frontier widens
        LVCHK(hipMemsetAsync(L.bar, 0, sizeof(LvBar), st));
        LVCHK(hipMemsetAsync(L.ctl, 0, 3 * sizeof(LvCtl), st));
        const uint32_t r0 = next_round;
        const hipError_t le = lv_persist_launch(nq, L.grid_persist, p, pq, L.coop, st);
        if (le != hipSuccess) {  // refused before it ran (residency not available)
          (void)hipGetLastError();
          aborted = true;
          break;
        }
        LVCHK(hipStreamSynchronize(st));
        ++syncs;
        ++ls.persist_launches;
        if (hr->done == LVR_ABORT) { aborted = true; break; }
        next_round = hr->round + 1;
        ls.persist_rounds += next_round - r0 + (hr->done == LVR_OVERFLOW ? 1 : 0);
        ctl_dirty = true;
      } else {
        if (ctl_dirty) {  // back from lv_persist: round r's counters must start at zero in ctl[r & 1]
          LVCHK(hipMemsetAsync(L.ctl, 0, 3 * sizeof(LvCtl), st));
          ctl_dirty = false;
        }
        // batch length from the last known frontier; the kernels are persistent
        // (grid = what the chip holds at once) and size their work on the device
        const bool narrow = nf_last < 4096;
        const uint32_t batch = narrow ? 16 : 1;
        const uint32_t g_round = L.grid_round;
        // lv_insert's last block closes the round: its done-counter atomics grow
        // with the grid (~11 ns each), so narrow rounds use a small grid
        const uint32_t g_ins = narrow ? std::min<uint32_t>(L.grid_insert, 128) : L.grid_insert;
        p.f0 = 0; p.f1 = LV_NONE; p.clear_slots = 1;
        p.fused = fused_wide;
        for (uint32_t k = 0; k < batch; ++k) {
          set_round(next_round + k);
          p.publish_always = k + 1 == batch;  // the host reads the state after the batch
          LVCHK(lv_dispatch(nq, LK_ROUND, g_round, p, st));
          LVCHK(lv_dispatch(nq, LK_INSERT, g_ins, p, st));
        }
        p.publish_always = 1;
        next_round += batch;
        LVCHK(hipStreamSynchronize(st));
        ++syncs;
      }
      if (hr->done == LVR_OVERFLOW) {
        // round r overflowed the staging array: its frontier (stg[(r+1)&1]) is
        // intact; raise the capacity if the budget allows, then re-run the
        // round host-driven, over halves of the frontier while it still does
        // not fit, into a clean table (an aborted persistent round left
        // entries behind)
        const uint32_t r = hr->round + 1;
        const uint32_t nf = hr->nf;
        {
          const int g = level_grow(b, (int)((r + 1) & 1), st, err);
          if (g < 0) return g;
          if (g == 0) {
            ++ls.grows;
            p.scap = L.scap; p.scs = L.scap / LV_STRIPES; p.ht_mask = L.ht_mask;
            for (int i = 0; i < 2; ++i) { pq.stg[i] = L.stg[i]; pq.idx[i] = L.idx[i]; pq.ht[i] = L.ht[i]; }
            ht_bytes = ((size_t)L.ht_mask + 1) * 8;
          }
        }
        LvRun cont = *hr;
        cont.done = LVR_RUNNING;
        LVCHK(hipMemcpyAsync(run, &cont, sizeof cont, hipMemcpyHostToDevice, st));
        set_round(r);
        LVCHK(hipMemsetAsync(p.ht, 0xFF, ht_bytes, st));
        p.clear_slots = 0;  // a chunk must not break the probe chains of earlier chunks' entries
        p.close_round = 0;
        p.fused = 0;        // (a chunk that overflows is re-run: its children must not be in the table yet)
        uint32_t f0 = 0, chunk = nf;
        LvCtl* hc = reinterpret_cast<LvCtl*>(L.h_ctl);
        LvCtl snap;  // the counters before the current chunk (restored when it overflows)
        memset(&snap, 0, sizeof snap);
        bool stop = false;
        while (f0 < nf) {
          const uint32_t f1 = (uint32_t)std::min<uint64_t>(nf, (uint64_t)f0 + chunk);
          LVCHK(hipMemcpyAsync(p.ctl, &snap, sizeof(LvCtl), hipMemcpyHostToDevice, st));
          p.f0 = f0; p.f1 = f1;
          LVCHK(lv_dispatch(nq, LK_ROUND, L.grid_round, p, st));
          LVCHK(lv_dispatch(nq, LK_INSERT, L.grid_insert, p, st));
          LVCHK(hipMemcpyAsync(hc, p.ctl, sizeof(LvCtl), hipMemcpyDeviceToHost, st));
          LVCHK(hipStreamSynchronize(st));
          ++syncs;
          if (hc->found) break;
          if (hc->overflow) {
            if (f1 - f0 == 1) { stop = true; break; }
            chunk = std::max<uint32_t>(1, (f1 - f0) / 2);
            ++ls.chunk_retries;
            continue;
          }
          // this chunk's staging is inserted: the next chunk inserts from here on
          snap = *hc;
          for (int s_ = 0; s_ < LV_STRIPES; ++s_) snap.lo[s_] = std::min(snap.cnt[16 * s_], p.scs);
          snap.done_blocks = 0;
          f0 = f1;
        }
        if (stop) break;  // hr->done stays LVR_OVERFLOW: Unknown (frontier)
        LVCHK(lv_dispatch(nq, LK_CLOSE, 1, p, st));  // the round's bookkeeping (publishes hr)
        // chunked rounds did not clear their frontier's table slots: reset the tables
        for (int i = 0; i < 2; ++i) LVCHK(hipMemsetAsync(L.ht[i], 0xFF, ht_bytes, st));
        LVCHK(hipMemsetAsync(L.ctl, 0, 3 * sizeof(LvCtl), st));
        ctl_dirty = false;
        LVCHK(hipStreamSynchronize(st));
        p.close_round = 1;
        next_round = r + 1;
      }
      nf_last = hr->nf;
    }
    if (!aborted) break;
    // start over, host-driven: clean tables; the round counts and trace
    // entries of the aborted attempt are overwritten round by round
    persist_on = false;
    L.persist_refused = true;  // (this context's later searches too)
    ++ls.persist_fallbacks;
    for (int i = 0; i < 2; ++i) LVCHK(hipMemsetAsync(L.ht[i], 0xFF, ht_bytes, st));
    LVCHK(hipStreamSynchronize(st));
  }
  LVCHK(hipEventRecord(L.ev[1], st));
  LVCHK(hipEventSynchronize(L.ev[1]));
  float ms = 0;
  LVCHK(hipEventElapsedTime(&ms, L.ev[0], L.ev[1]));
  const LvRun fin = *hr;
#ifdef S2LC_PROF
  {
    unsigned long long g[48];
    LVCHK(hipMemcpy(g, d_prof, sizeof g, hipMemcpyDeviceToHost));
    if (const char* path = getenv("S2LC_LVPROF_ROUNDS")) {  // one line per persistent grid round
      std::vector<unsigned long long> pr(11 * (size_t)LV_PROF_ROUNDS);
      LVCHK(hipMemcpy(pr.data(), d_prof + 48, pr.size() * sizeof(unsigned long long), hipMemcpyDeviceToHost));
      if (FILE* f = fopen(path, "a")) {
        for (uint32_t r = 0; r < LV_PROF_ROUNDS; ++r)
          if (pr[r])
            fprintf(f, "%u %llu %llu %llu %llu %llu %llu %llu %llu %llu %llu %llu\n", r, pr[r], pr[LV_PROF_ROUNDS + r],
                    pr[2 * LV_PROF_ROUNDS + r], pr[3 * LV_PROF_ROUNDS + r], pr[4 * LV_PROF_ROUNDS + r],
                    pr[5 * LV_PROF_ROUNDS + r], pr[6 * LV_PROF_ROUNDS + r], pr[7 * LV_PROF_ROUNDS + r],
                    pr[8 * LV_PROF_ROUNDS + r], pr[9 * LV_PROF_ROUNDS + r], pr[10 * LV_PROF_ROUNDS + r]);
        fclose(f);
      }
    }
    (void)hipFree(d_prof);
    const double it = g[5] ? (double)g[5] : 1.0, ch = g[6] ? (double)g[6] : 1.0;
    fprintf(stderr,
            "[s2lc lvprof] items %llu children %llu syncs %u persist %llu rounds / %llu launches | cycles/item "
            "parent %.0f heads+fp %.0f moves %.0f | cycles/child closure %.0f stage+restore %.0f | total Gcycles %.2f\n",
            g[5], g[6], syncs, (unsigned long long)ls.persist_rounds, (unsigned long long)ls.persist_launches,
            g[0] / it, g[1] / it, g[2] / it, g[3] / ch, g[4] / ch, (g[0] + g[1] + g[2] + g[3] + g[4]) * 1e-9);
    int khz = 100000;
    (void)hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, 0);
    const double us = 1e3 / khz, nr = g[11] ? (double)g[11] : 1.0;
    fprintf(stderr, "[s2lc lvprof] persistent rounds %llu: %.2f us/round, expansion critical path %.2f us/round | "
            "cycles/item move selection %.0f move record loads %.0f\n",
            g[11], g[9] * us / nr, g[10] * us / nr, g[12] / it, g[13] / it);
    fprintf(stderr, "[s2lc lvprof] solo rounds %llu: %.2f us/round | closures run %llu, opt children dropped by the P1 "
            "precheck %llu\n", g[7], g[8] * us / (g[7] ? (double)g[7] : 1.0), g[14], g[15]);
    const double ns = g[7] ? (double)g[7] : 1.0;
    fprintf(stderr, "[s2lc lvprof] solo cycles/round (wave 0): start %.0f setup %.0f pre %.0f moves %.0f reload+close %.0f barrier %.0f\n",
            g[16] / ns, g[17] / ns, g[18] / ns, g[19] / ns, g[20] / ns, g[21] / ns);
    fprintf(stderr, "[s2lc lvprof] solo closures: ALIVE %llu at %.0f cycles, others %.0f cycles/round; stage %.0f cycles per ALIVE"
            " | closures %llu: %.2f passes and %.2f head loads (lanes) each\n",
            g[24], g[22] / (g[24] ? (double)g[24] : 1.0), g[23] / ns, g[25] / (g[24] ? (double)g[24] : 1.0), g[14],
            g[26] / (g[14] ? (double)g[14] : 1.0), g[27] / (g[14] ? (double)g[14] : 1.0));
    fprintf(stderr, "[s2lc lvprof] solo round: slowest wave's expansion %.0f cycles, wave 0's wait at the first barrier %.0f"
            " | survivors per round %.3f, rounds with one survivor %llu\n", g[28] / ns, g[31] / ns, g[29] / ns, g[30]);
    fprintf(stderr, "[s2lc lvprof] solo moves (all waves, cycles/round): fold %.0f child setup %.0f closure loop %.0f keep+prefetch %.0f"
            " | moves %.3f/round\n", g[32] / ns, g[33] / ns, g[34] / ns, g[35] / ns, g[36] / ns);
  }
#endif
  // clear the tables for the next search
  for (int i = 0; i < 2; ++i) LVCHK(hipMemsetAsync(L.ht[i], 0xFF, ht_bytes, st));

  uint32_t verdict, reason;
  switch (fin.done) {
    case LVR_FOUND: verdict = V_OK; reason = 0; break;
    case LVR_EMPTY: verdict = V_ILLEGAL; reason = S2LC_R_SEARCH_EXHAUSTED; break;
    case LVR_BUDGET: verdict = V_UNKNOWN; reason = S2LC_R_BUDGET; break;
    case LVR_OVERFLOW: verdict = V_UNKNOWN; reason = S2LC_R_FRONTIER; break;
    case LVR_TIMEOUT: verdict = V_UNKNOWN; reason = S2LC_R_TIMEOUT; break;
    default: verdict = V_UNKNOWN; reason = timed_out ? S2LC_R_TIMEOUT : S2LC_R_FRONTIER; break;
  }
  HistResult& R = b.h_res[h];
  const uint32_t woff = R.witness_off;
  R = HistResult{};
  R.witness_off = woff;
  R.verdict = verdict;
  R.reason = reason;
  // rounds: expansion rounds run (the found / empty round included; an
  // overflowing round counts, a timed-out search stops after a completed one)
  R.rounds = fin.done == LVR_OVERFLOW ? fin.round + 1 : fin.round;
  R.configs = fin.configs;
  R.children = fin.children;
  R.p4 = verdict == V_OK ? fin.found_p4 : 0;
  const bool have_w = verdict == V_OK && fin.witness && fin.found_parent != TRACE_NONE;
  const bool root_w = verdict == V_OK && fin.witness && fin.round == 0;  // completed by the initial closure
  R.final_parent = have_w ? fin.found_parent : TRACE_NONE;
  R.final_move = verdict == V_OK ? fin.found_move : TRACE_NONE;
  R.deep_trace = verdict == V_ILLEGAL ? fin.deep_trace : TRACE_NONE;
  R.deep_len = fin.deep_len;
  R.has_witness = (have_w || root_w || R.deep_trace != TRACE_NONE) ? 2u : 0u;
  LVCHK(hipMemcpyAsync(b.res + h, &R, sizeof R, hipMemcpyHostToDevice, st));
  if (ro.witness && b.trace) {
    unsigned long long th = fin.tnext;
    LVCHK(hipMemcpyAsync(b.trace_head, &th, sizeof th, hipMemcpyHostToDevice, st));
  }
  LVCHK(hipStreamSynchronize(st));
  ls.ms += ms;
  {
    int khz = 100000;  // device wall clock
    int dev_ = 0;
    (void)hipGetDevice(&dev_);
    (void)hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, dev_);
    ls.narrow_ms += (double)fin.narrow_ticks / std::max(1, khz);
    ls.wide_ms += (double)fin.wide_ticks / std::max(1, khz);
    ls.solo_ms += (double)fin.solo_ticks / std::max(1, khz);
  }
  ls.rounds += R.rounds;
  ls.configs += fin.configs;
  ls.children += fin.children;
  ls.max_frontier = std::max(ls.max_frontier, fin.max_frontier);
  ls.histories++;
  ls.syncs += syncs;
  ls.solo_rounds += fin.solo_rounds;
  return 0;
}


// ============================================================================
// Distributed level search of one history (BASELINE config C5 over several
// GPUs). Configurations are owned by rank lv_owner(fp). A round
// on each rank:
//   dist_expand : expand + close the local frontier (lv_round) into local
//                 staging, count the staged configurations per owner rank
//   (caller)    : all-to-all of the counts, allocate the send buffer
//   dist_pack   : copy the staged configurations into owner-major buckets
//   (caller)    : all-to-all(v) of the buckets over RCCL / xGMI
//   dist_insert : deduplicate what this rank received (it owns all of it) in
//                 the local table; the winners are its next frontier
// The received buffer stays the frontier of the next round (the caller keeps
// it alive). Trace ids are rank << 29 | local pool index, so the parent chain
// of a witness crosses ranks; the caller gathers the pools at the end. These
// rounds are host-driven (the caller's collectives sit between the kernels).
// ============================================================================

int dist_create(DistLevel& d, const History* h, uint32_t rank, uint32_t world, uint32_t reductions_off,
                hipStream_t stream, std::string& err) {
  if (world < 1 || world > 8 || rank >= world) { err = "world must be 1..8"; return S2LC_EINVAL; }
  std::vector<const History*> hs{h};
  int rc = batch_upload(d.b, hs, reductions_off, err);
  if (rc) return rc;
  d.rank = rank;
  d.world = world;
  d.K = d.b.h_hist[0].K;
  d.nq = level_nq(d.K);
  d.cb = lv_cfg_bytes(d.nq);
  if (d.b.forced[0]) { err = "history is structurally illegal (unmatched events)"; return S2LC_EINVAL; }
  if (level_buffers(d.b, d.nq, err, true)) return S2LC_EHIP;
  if (lv_grids(d.b.lv, d.nq, err)) return S2LC_EHIP;
  LVCHK(hipMalloc(&d.own_cnt, 8 * sizeof(uint32_t)));
  LVCHK(hipMalloc(&d.own_pos, (size_t)d.b.lv.scap * sizeof(uint32_t)));
  size_t free_b = 0, total_b = 0;
  LVCHK(hipMemGetInfo(&free_b, &total_b));
  d.trace_cap = std::min<uint64_t>(1ull << 29, (uint64_t)(free_b / 16) / sizeof(TraceEnt));
  LVCHK(hipMalloc(&d.trace, d.trace_cap * sizeof(TraceEnt)));
  // the caller's stream (its collectives and the search are then ordered on
  // the device), else a stream of its own
  if (stream) {
    d.stream = stream;
    d.own_stream = false;
  } else {
    LVCHK(hipStreamCreateWithFlags(&d.stream, hipStreamNonBlocking));
    d.own_stream = true;
  }
  d.round = 0;
  return 0;
}

void dist_release(DistLevel& d) {
  if (d.xrun) (void)hipFree(d.xrun);
  if (d.xself) (void)hipFree(d.xself);
  d.xself = nullptr;
  if (d.xstat) (void)hipHostFree(d.xstat);
  for (hipEvent_t& e : d.xev) {
    if (e) (void)hipEventDestroy(e);
    e = nullptr;
  }
  d.xrun = nullptr;
  d.xstat = nullptr;
  if (d.snap) (void)hipFree(d.snap);
  d.snap = nullptr;
  d.snap_cap = 0;
  if (d.own_cnt) (void)hipFree(d.own_cnt);
  if (d.own_pos) (void)hipFree(d.own_pos);
  if (d.trace) (void)hipFree(d.trace);
  if (d.stream && d.own_stream) (void)hipStreamDestroy(d.stream);
  d.own_cnt = nullptr; d.own_pos = nullptr; d.trace = nullptr; d.stream = nullptr;
  batch_release(d.b);
}

static LvParams dist_params(DistLevel& d) {
  LevelBufs& L = d.b.lv;
  const HistDesc& hd = d.b.h_hist[0];
  LvParams p;
  memset(&p, 0, sizeof p);
  p.tag_drop = lv_tag_drop();
  p.recs = d.b.recs; p.pool = d.b.pool; p.cs = d.b.chain_start + hd.cs_base; p.K = d.K; p.hflags = hd.flags;
  p.scap = L.scap; p.scs = L.scap / LV_STRIPES; p.ht = L.ht[0]; p.ht_clear = L.ht[0]; p.ht_mask = L.ht_mask;
  p.trace = d.trace; p.trace_cap = d.trace_cap;
  p.ctl = reinterpret_cast<LvCtl*>(L.ctl);
  p.world = d.world; p.own_cnt = d.own_cnt; p.own_pos = d.own_pos;
  // local staging (the closed children of this rank): the array that holds
  // no part of the current frontier
  p.stg = (d.cur == L.stg[0] || d.cur_loc == L.stg[0]) ? L.stg[1] : L.stg[0];
  p.cur = d.cur; p.cur_loc = d.cur_loc; p.cur_idx = L.idx[d.cur_sel];
  p.rank = d.rank;
  p.tgid = d.rank << 29;
  p.witness_host = 1;
  return p;
}

// Phase switches of the distributed search (replicated <-> partitioned) clean
// the two tables by clearing the current frontier's slots (lv_clear_slots),
// not by resetting them: every round inserts its winners and clears its
// parents' slots, so at a switch the frontier's entries are all the tables
// hold (a reset of both tables cost ~90 us each at their full size, six per
// switch; C5wide switches 11 times)
static int dist_clear_frontier_slots(DistLevel& d, std::string& err) {
  if (!d.nf) return 0;
  LevelBufs& L = d.b.lv;
  LvParams p = dist_params(d);
  p.f1 = d.nf;
  p.ht = L.ht[0];
  p.ht_clear = L.ht[1];
  LVCHK(lv_dispatch(d.nq, LK_CLEAR, (uint32_t)std::min<uint64_t>(1024, (d.nf + LV_BLOCK - 1) / LV_BLOCK), p, d.stream));
  return 0;
}

// expand + close this rank's frontier (round 0: the initial configuration, on
// rank 0 only) into local staging; host-driven, control block 0
static int dist_stage(DistLevel& d, LvParams& p, std::string& err) {
  hipStream_t st = d.stream;
  LVCHK(hipMemsetAsync(p.ctl, 0, sizeof(LvCtl), st));
  if (d.round == 0) {
    if (d.rank == 0) {
      p.init = 1; p.f0 = 0; p.f1 = 1;
      LVCHK(lv_dispatch(d.nq, LK_ROUND, 1, p, st));
      p.init = 0;
    }
  } else if (d.nf) {
    p.f0 = 0; p.f1 = d.nf; p.clear_slots = 1;
    LVCHK(lv_dispatch(d.nq, LK_ROUND, d.b.lv.grid_round, p, st));
  }
  return 0;
}

int dist_expand(DistLevel& d, uint64_t* counts, int* found, std::string& err) {
  LevelBufs& L = d.b.lv;
  LvCtl* hc = reinterpret_cast<LvCtl*>(L.h_ctl);
  const uint32_t max_grid = (uint32_t)n_cus(err) * 8;
  hipStream_t st = d.stream;
  LvParams p = dist_params(d);
  LVCHK(hipEventRecord(L.ev[0], st));
  LVCHK(hipMemsetAsync(d.own_cnt, 0, 8 * sizeof(uint32_t), st));
  if (dist_stage(d, p, err)) return S2LC_EHIP;
  LVCHK(hipMemcpyAsync(hc, L.ctl, sizeof(LvCtl), hipMemcpyDeviceToHost, st));
  LVCHK(hipStreamSynchronize(st));
  uint32_t maxc = 0;  // the longest staging stripe
  for (int s_ = 0; s_ < LV_STRIPES; ++s_) maxc = std::max(maxc, std::min(hc->cnt[16 * s_], p.scs));
  d.slot_hi = maxc * LV_STRIPES;
  p.dense = d.slot_hi;
  if (d.slot_hi)
    LVCHK(lv_dispatch(d.nq, LK_BUCKET, (uint32_t)std::min<uint64_t>(max_grid, (d.slot_hi + LV_BLOCK - 1) / LV_BLOCK), p, st));
  uint32_t cnt[8] = {0};
  LVCHK(hipMemcpyAsync(cnt, d.own_cnt, sizeof cnt, hipMemcpyDeviceToHost, st));
  LVCHK(hipEventRecord(L.ev[1], st));
  LVCHK(hipStreamSynchronize(st));
  float ms = 0;
  LVCHK(hipEventElapsedTime(&ms, L.ev[0], L.ev[1]));
  d.ms += ms;
  if (hc->overflow) { err = "distributed round exceeds the device buffers"; return S2LC_ENOMEM; }
  d.children += hc->children;
  for (uint32_t o = 0; o < d.world; ++o) counts[o] = cnt[o];
  *found = hc->found ? 1 : 0;
  if (hc->found) { d.found_parent = hc->found_parent; d.found_move = hc->found_move; d.found_p4 = hc->found_p4; }
  return 0;
}

int dist_pack(DistLevel& d, uint8_t* send, const uint64_t* counts, std::string& err) {
  LvParams p = dist_params(d);
  uint64_t off = 0;
  for (uint32_t o = 0; o < d.world; ++o) { p.own_off[o] = off; off += counts[o]; }
  if (off > d.slot_hi) { err = "bucket counts exceed the staged configurations"; return S2LC_EINVAL; }
  if (off && !send) { err = "null send buffer"; return S2LC_EINVAL; }
  p.send = send;
  p.dense = d.slot_hi;
  if (d.slot_hi && off) {
    const uint64_t pieces = (uint64_t)d.slot_hi * (d.cb / 16);
    LVCHK(lv_dispatch(d.nq, LK_SCATTER, (uint32_t)std::min<uint64_t>(2048, (pieces + LV_BLOCK - 1) / LV_BLOCK), p, d.stream));
  }
  LVCHK(hipStreamSynchronize(d.stream));
  return 0;
}

int dist_insert(DistLevel& d, uint8_t* recv, uint64_t n_recv, uint64_t* n_next, std::string& err) {
  LevelBufs& L = d.b.lv;
  LvCtl* hc = reinterpret_cast<LvCtl*>(L.h_ctl);
  if (n_recv > L.scap) { err = "received configurations exceed the frontier capacity"; return S2LC_ENOMEM; }
  hipStream_t st = d.stream;
  const int sel = d.cur_sel ^ 1;
  LvParams p = dist_params(d);
  p.stg = recv; p.nxt_idx = L.idx[sel]; p.dense = (uint32_t)n_recv;
  if (d.tnext + n_recv > d.trace_cap) { err = "trace pool full"; return S2LC_ENOMEM; }
  p.tbase_host = (uint32_t)d.tnext;
  memset(hc, 0, sizeof(LvCtl));
  LVCHK(hipEventRecord(L.ev[0], st));
  LVCHK(hipMemcpyAsync(L.ctl, hc, sizeof(LvCtl), hipMemcpyHostToDevice, st));
  if (n_recv) {
    const uint32_t max_grid = (uint32_t)n_cus(err) * 8;
    LVCHK(lv_dispatch(d.nq, LK_INSERT, (uint32_t)std::min<uint64_t>(max_grid, (n_recv + LV_BLOCK - 1) / LV_BLOCK), p, st));
  }
  LVCHK(hipMemcpyAsync(hc, L.ctl, sizeof(LvCtl), hipMemcpyDeviceToHost, st));
  LVCHK(hipEventRecord(L.ev[1], st));
  LVCHK(hipStreamSynchronize(st));
  float ms = 0;
  LVCHK(hipEventElapsedTime(&ms, L.ev[0], L.ev[1]));
  d.ms += ms;
  d.cur = recv;
  d.cur_loc = nullptr;
  d.cur_sel = sel;
  d.nf = hc->nnext;
  d.tnext += hc->nnext;
  d.configs += hc->nnext;
  d.max_frontier = std::max<uint64_t>(d.max_frontier, hc->nnext);
  d.round++;
  *n_next = hc->nnext;
  return 0;
}

// ---- host-free partitioned rounds -------------------------------------------
// The caller queues rounds back to back with no host synchronization:
//   dist_x_send(send, cap)  expand + close this rank's frontier (lv_round) and
//                           copy the staged children into fixed-capacity
//                           blocks, one per owner, header first (lv_xsend)
//   (caller)                equal-split all-to-all of the blocks
//   dist_x_recv(recv, cap)  decide the round from the received headers, then
//                           insert what this rank received (lv_insert, xcap
//                           mode); the last block closes the round and
//                           publishes its status to the host-mapped ring
// and reads a round's status with dist_x_wait a round or two later. Every
// rank decides the same from the same headers: found (Ok), nothing staged
// anywhere (Illegal), staging overflow on any rank (abort), or a block over
// its capacity (nothing inserted: dist_x_rewind(round) and re-run it with a
// larger cap). A stopped run turns the rounds queued after it into no-ops.
// S2LC_XSYNC=1 (diagnostics): wait after every queued step, so a fault is
// reported by the call that queued it
static const bool g_xsync = getenv("S2LC_XSYNC") != nullptr;

static int dist_x_alloc(DistLevel& d, std::string& err) {
  if (d.xrun) return 0;
  LVCHK(hipMalloc(&d.xrun, sizeof(LvRun)));
  LVCHK(hipMalloc(&d.xself, sizeof(LvXHdr)));
  LVCHK(hipHostMalloc(&d.xstat, LV_XRING * sizeof(LvXStat), hipHostMallocMapped));
  for (hipEvent_t& e : d.xev) LVCHK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
  return 0;
}

int dist_x_begin(DistLevel& d, std::string& err) {
  if (d.round == 0) { err = "partitioned rounds start after round 0"; return S2LC_EINVAL; }
  if (dist_x_alloc(d, err)) return S2LC_EHIP;
  LvRun R;
  memset(&R, 0, sizeof R);
  R.round = d.round;
  R.nf = d.nf;
  R.tnext = d.tnext;
  R.witness = d.tnext + d.b.lv.scap <= d.trace_cap ? 1u : 0u;
  R.found_parent = TRACE_NONE;
  R.found_move = LV_NONE;
  R.deep_trace = TRACE_NONE;
  R.last_tbase = TRACE_NONE;
  LVCHK(hipMemcpyAsync(d.xrun, &R, sizeof R, hipMemcpyHostToDevice, d.stream));
  // the owner counters start at zero (lv_xsend's last block clears them for
  // the round after; the sized rounds leave them counted)
  LVCHK(hipMemsetAsync(d.own_cnt, 0, 8 * sizeof(uint32_t), d.stream));
  LVCHK(hipStreamSynchronize(d.stream));
  LvXStat* x = reinterpret_cast<LvXStat*>(d.xstat);
  for (uint32_t i = 0; i < LV_XRING; ++i) x[i].round = 0xFFFFFFFFu;
  d.xround = d.round + 1;
  d.xfresh = true;
  return 0;
}

// exchanged round r counts in ctl[r & 1]; its lv_round zeroes ctl[(r + 1) & 1]
// for the round after (whose last user, round r - 1, has ended)
static LvParams dist_x_params(DistLevel& d, uint32_t cap) {
  LvParams p = dist_params(d);
  p.run = reinterpret_cast<LvRun*>(d.xrun);
  p.xcap = cap;
  p.round = d.xround;
  p.ctl = reinterpret_cast<LvCtl*>(d.b.lv.ctl) + (d.xround & 1);
  p.xself = reinterpret_cast<LvXHdr*>(d.xself);
  return p;
}

// (smallest frontier, staged count) of the latest status the host can see
// without waiting: sizes the grids of the next queued round (any grid is
// correct, the kernels stride)
static void dist_x_hint(const DistLevel& d, uint32_t& hint_nf, uint64_t& hint_staged) {
  hint_nf = UINT32_MAX;
  hint_staged = UINT64_MAX;
  const volatile LvXStat* xs = reinterpret_cast<const volatile LvXStat*>(d.xstat);
  for (uint32_t back = 1; back <= 2 && back < d.xround; ++back) {
    const uint32_t r = d.xround - back;
    const volatile LvXStat& e = xs[r % LV_XRING];
    if (e.round == r && !e.done) { hint_nf = back == 1 ? e.nf : UINT32_MAX; hint_staged = e.staged; break; }
  }
}

int dist_x_send(DistLevel& d, uint8_t* send, uint32_t cap, std::string& err) {
  if (!d.xrun) { err = "dist_x_begin first"; return S2LC_EINVAL; }
  if (cap == 0 || (!send && d.world > 1)) { err = "exchange capacity 0 / null send buffer"; return S2LC_EINVAL; }
  hipStream_t st = d.stream;
  LvParams p = dist_x_params(d, cap);
  p.f0 = 0;
  p.f1 = LV_NONE;  // the frontier size lives on the device
  p.clear_slots = 1;
  p.send = send;
  if (d.xfresh) {  // the first round after x_begin / x_rewind: its counters
    LVCHK(hipMemsetAsync(p.ctl, 0, sizeof(LvCtl), st));
    d.xfresh = false;
  }
  // grids from the latest status the host can see without waiting (this
  // rank's frontier after the previous round, when published): a narrow
  // round gets small grids (any grid is correct; the kernels stride)
  uint32_t hint_nf;
  uint64_t hint_staged;
  dist_x_hint(d, hint_nf, hint_staged);
  const uint32_t ncu = (uint32_t)n_cus(err);
  const uint32_t g_round = hint_nf <= 16 ? std::min<uint32_t>(d.b.lv.grid_round, ncu / 4) : d.b.lv.grid_round;
  // (one rank: lv_xsend copies nothing, it only writes the own header)
  const uint32_t g_send = d.world == 1 ? 1u : hint_staged <= 4096 ? std::max<uint32_t>(1, ncu / 16) : ncu;
  p.ctl_next = reinterpret_cast<LvCtl*>(d.b.lv.ctl) + ((d.xround + 1) & 1);
  LVCHK(lv_dispatch(d.nq, LK_ROUND, g_round, p, st));
  p.ctl_next = nullptr;
  // (one rank sends nothing: lv_insert takes its header from the counters)
  if (d.world > 1) LVCHK(lv_dispatch(d.nq, LK_XSEND, g_send, p, st));
  // on a stream of its own the caller's collective is not ordered after these
  // kernels on the device: the host waits (the gloo tests; one process per
  // GPU passes its stream and queues with no wait)
  if (d.own_stream || g_xsync) LVCHK(hipStreamSynchronize(st));
  return 0;
}

int dist_x_recv(DistLevel& d, uint8_t* recv, uint32_t cap, uint32_t* round, std::string& err) {
  if (!d.xrun) { err = "dist_x_begin first"; return S2LC_EINVAL; }
  if (cap == 0 || (!recv && d.world > 1)) { err = "exchange capacity 0 / null receive buffer"; return S2LC_EINVAL; }
  // the other ranks' blocks (the own share stays in the local staging)
  const uint64_t slots = (uint64_t)(d.world - 1) * (cap + 1);
  // (what one round inserts: at most the local staging plus the received
  // blocks, which the table holds at under 3/4 load; the close stops the run
  // if the next frontier's index list overflows, and the device stops
  // recording the trace before the pool fills)
  if ((uint64_t)(d.world - 1) * cap > d.b.lv.scap / 2) { err = "exchange blocks exceed the frontier capacity"; return S2LC_ENOMEM; }
  hipStream_t st = d.stream;
  const uint32_t r = d.xround % LV_XRING;
  d.xcur[r] = d.cur;
  d.xcur_loc[r] = d.cur_loc;
  d.xsel[r] = d.cur_sel;
  const int sel = d.cur_sel ^ 1;
  LvParams p = dist_x_params(d, cap);
  uint8_t* const loc = p.stg;  // this round's local staging (lv_round of dist_x_send staged there)
  p.stg = recv;
  p.stg_loc = loc;
  p.nxt_idx = d.b.lv.idx[sel];
  p.dense = (uint32_t)slots;
  p.close_round = 1;
  void* xs = nullptr;
  LVCHK(hipHostGetDevicePointer(&xs, d.xstat, 0));
  p.xstat = reinterpret_cast<LvXStat*>(xs);
  uint32_t hint_nf;
  uint64_t hint_staged;
  dist_x_hint(d, hint_nf, hint_staged);
  // grid: from the latest visible status; with none visible (rounds queued
  // ahead) two blocks per CU: the close is the last block's, and its
  // done-counter atomics grow with the grid (~11 ns each: 2,048 blocks cost a
  // narrow round ~40 us)
  const uint32_t ncu = (uint32_t)n_cus(err), max_grid = ncu * 8;
  const uint64_t want = slots + (hint_staged == UINT64_MAX ? (uint64_t)2 * ncu * LV_BLOCK : hint_staged);
  LVCHK(lv_dispatch(d.nq, LK_INSERT, (uint32_t)std::max<uint64_t>(1, std::min<uint64_t>(max_grid, (want + LV_BLOCK - 1) / LV_BLOCK)), p, st));
  LVCHK(hipEventRecord(d.xev[r], st));
  if (g_xsync) LVCHK(hipStreamSynchronize(st));
  if (round) *round = d.xround;
  d.cur = recv;
  d.cur_loc = loc;
  d.cur_sel = sel;
  d.xround++;
  return 0;
}

int dist_x_wait(DistLevel& d, uint32_t round, DistXStat* out, std::string& err) {
  if (!d.xrun || round >= d.xround || round + LV_XRING < d.xround) {
    err = "round not queued (or no longer in the status ring)";
    return S2LC_EINVAL;
  }
  LVCHK(hipEventSynchronize(d.xev[round % LV_XRING]));
  const volatile LvXStat* x = reinterpret_cast<const volatile LvXStat*>(d.xstat) + round % LV_XRING;
  out->ran = x->round == round ? 1u : 0u;
  out->done = out->ran ? x->done : 0u;
  out->nf = x->nf;
  out->maxblk = x->maxblk;
  out->nf_global = x->nf_global;
  out->staged = x->staged;
  return 0;
}

int dist_x_rewind(DistLevel& d, uint32_t round, std::string& err) {
  if (!d.xrun || round >= d.xround || round + LV_XRING < d.xround) {
    err = "round not queued (or no longer in the status ring)";
    return S2LC_EINVAL;
  }
  LVCHK(hipStreamSynchronize(d.stream));
  d.cur = d.xcur[round % LV_XRING];
  d.cur_loc = d.xcur_loc[round % LV_XRING];
  d.cur_sel = d.xsel[round % LV_XRING];
  d.xround = round;
  d.xfresh = true;
  const uint32_t zero = LVR_RUNNING;
  LVCHK(hipMemcpy(d.xrun, &zero, sizeof zero, hipMemcpyHostToDevice));  // (LvRun::done)
  return 0;
}

int dist_x_end(DistLevel& d, uint32_t* done, uint64_t* configs, std::string& err) {
  if (!d.xrun) { err = "dist_x_begin first"; return S2LC_EINVAL; }
  LVCHK(hipStreamSynchronize(d.stream));
  LvRun R;
  LVCHK(hipMemcpy(&R, d.xrun, sizeof R, hipMemcpyDeviceToHost));
  d.round = R.round;
  d.nf = R.done ? 0u : R.nf;
  d.tnext = R.tnext;
  d.configs += R.configs;
  d.children += R.children;
  d.max_frontier = std::max<uint64_t>(d.max_frontier, R.max_frontier);
  if (R.done == LVR_FOUND) { d.found_parent = R.found_parent; d.found_move = R.found_move; d.found_p4 = R.found_p4; }
  *done = R.done;
  *configs = R.configs;
  return 0;
}

// ---- replicated rounds (narrow frontiers): every rank runs the same round on
// the whole frontier, with no exchange; the set of configurations, and so
// every decision, is the same on all ranks.
int dist_local_round(DistLevel& d, uint64_t* n_next, int* found, std::string& err) {
  LevelBufs& L = d.b.lv;
  if (d.cur_loc) { err = "the frontier is partitioned: gather it (frontier_pack / frontier_load) first"; return S2LC_EINVAL; }
  LvCtl* hc = reinterpret_cast<LvCtl*>(L.h_ctl);
  const uint32_t max_grid = (uint32_t)n_cus(err) * 8;
  hipStream_t st = d.stream;
  LvParams p = dist_params(d);
  p.nxt_idx = L.idx[d.cur_sel ^ 1];
  if (d.tnext + L.scap > d.trace_cap) { err = "trace pool full"; return S2LC_ENOMEM; }
  p.tbase_host = (uint32_t)d.tnext;
  LVCHK(hipEventRecord(L.ev[0], st));
  const bool first = d.round == 0;
  const uint32_t rank = d.rank;
  d.rank = 0;  // replicated: every rank closes the initial configuration
  const int rc = dist_stage(d, p, err);
  d.rank = rank;
  if (rc) return rc;
  const uint64_t ins = first ? 1 : std::min<uint64_t>(max_grid, std::max<uint64_t>(4, (uint64_t)d.nf * 64 / LV_BLOCK));
  LVCHK(lv_dispatch(d.nq, LK_INSERT, (uint32_t)ins, p, st));
  LVCHK(hipMemcpyAsync(hc, L.ctl, sizeof(LvCtl), hipMemcpyDeviceToHost, st));
  LVCHK(hipEventRecord(L.ev[1], st));
  LVCHK(hipStreamSynchronize(st));
  float ms = 0;
  LVCHK(hipEventElapsedTime(&ms, L.ev[0], L.ev[1]));
  d.ms += ms;
  if (hc->overflow && !hc->found) { err = "replicated round exceeds the device buffers"; return S2LC_ENOMEM; }
  d.children += hc->children;
  *found = hc->found ? 1 : 0;
  if (hc->found) {
    d.found_parent = hc->found_parent; d.found_move = hc->found_move; d.found_p4 = hc->found_p4;
    *n_next = 0;
    return 0;
  }
  d.cur = p.stg;
  d.cur_loc = nullptr;
  d.cur_sel ^= 1;
  d.nf = hc->nnext;
  d.tnext += hc->nnext;
  d.configs += hc->nnext;
  d.max_frontier = std::max<uint64_t>(d.max_frontier, hc->nnext);
  d.round++;
  *n_next = hc->nnext;
  return 0;
}

// Replicated rounds inside lv_persist (solo rounds included), on the
// single-GPU engine's conventions: round r reads its frontier from stg /
// idx[(r + 1) & 1] and stages into stg / idx[r & 1]. The frontier is copied
// contiguously into the staging array it does not live in (x), and the run
// state starts at round R0 with R0 & 1 == x, so round R0 + 1 reads it there;
// the launches run until the frontier reaches `wide` configurations or the
// search ends, and the last closed round R leaves the frontier in stg /
// idx[R & 1]. Every rank runs the same rounds on the same configurations, so
// every rank reaches the same state. Returns S2LC_EUNSUPPORTED when the
// persistent kernel is not available for this layout, or when a launch was
// refused or its barrier timed out: then the frontier is restored and the
// caller runs host-driven replicated rounds (dist_local_round) instead.
int dist_local_run(DistLevel& d, uint32_t wide, uint64_t* n_next, int* found, uint32_t* rounds, std::string& err) {
  LevelBufs& L = d.b.lv;
  *rounds = 0;
  *found = 0;
  if (d.cur_loc) { err = "the frontier is partitioned: gather it (frontier_pack / frontier_load) first"; return S2LC_EINVAL; }
  if (!L.grid_persist || L.persist_refused || d.round == 0 || wide < 2) {
    err = "persistent replicated rounds unavailable";
    return S2LC_EUNSUPPORTED;
  }
  hipStream_t st = d.stream;
  const size_t ht_bytes = ((size_t)L.ht_mask + 1) * 8;
  // the frontier, contiguous, into the staging array it does not live in, and
  // into the snapshot (the persistent rounds overwrite both staging arrays)
  const int x = d.cur == L.stg[0] ? 1 : 0;
  const uint32_t R0 = 2u + (uint32_t)x;  // R0 & 1 == x: round R0 + 1 reads stg / idx[x]
  LvParams p = dist_params(d);
  p.f1 = d.nf;
  p.send = L.stg[x];
  const size_t fb = (size_t)d.nf * d.cb;
  if (fb > d.snap_cap) {
    if (d.snap) (void)hipFree(d.snap);
    d.snap = nullptr;
    d.snap_cap = 0;
    LVCHK(hipMalloc(&d.snap, fb));
    d.snap_cap = fb;
  }
  if (d.nf) {
    const uint64_t pieces = (uint64_t)d.nf * (d.cb / 16);
    LVCHK(lv_dispatch(d.nq, LK_GATHER, (uint32_t)std::min<uint64_t>(2048, (pieces + LV_BLOCK - 1) / LV_BLOCK), p, st));
    LVCHK(hipMemcpyAsync(d.snap, L.stg[x], fb, hipMemcpyDeviceToDevice, st));
    hipLaunchKernelGGL(lv_iota, dim3((uint32_t)std::min<uint64_t>(1024, (d.nf + 255) / 256)), dim3(256), 0, st, L.idx[x], d.nf);
    LVCHK(hipGetLastError());
  }
  // clean tables for the persistent rounds (the frontier's entries are all
  // they hold; its configurations are still in place in d.cur)
  if (dist_clear_frontier_slots(d, err)) return S2LC_EHIP;
  LvRun* hr = reinterpret_cast<LvRun*>(L.h_run);
  LvRun* d_pub = nullptr;
  LVCHK(hipHostGetDevicePointer((void**)&d_pub, hr, 0));
  LvRun r0;
  memset(&r0, 0, sizeof r0);
  r0.done = LVR_RUNNING; r0.round = R0; r0.nf = d.nf; r0.max_frontier = (uint32_t)d.max_frontier;
  r0.tnext = d.tnext; r0.witness = d.tnext + L.scap <= d.trace_cap ? 1u : 0u;
  r0.found_parent = TRACE_NONE; r0.found_move = LV_NONE; r0.deep_trace = TRACE_NONE; r0.last_tbase = TRACE_NONE;
  LVCHK(hipMemcpyAsync(L.run, &r0, sizeof r0, hipMemcpyHostToDevice, st));
  p.run = reinterpret_cast<LvRun*>(L.run); p.publish = d_pub; p.close_round = 1; p.publish_always = 1;
  p.rcounts = nullptr; p.init = 0;
  LvPersist pq;
  memset(&pq, 0, sizeof pq);
  pq.ctl3 = reinterpret_cast<LvCtl*>(L.ctl); pq.bar = reinterpret_cast<LvBar*>(L.bar);
  for (int i = 0; i < 2; ++i) { pq.stg[i] = L.stg[i]; pq.idx[i] = L.idx[i]; pq.ht[i] = L.ht[i]; }
  pq.max_rounds = 4096;
  pq.nf_max = wide - 1;
  pq.solo = getenv("S2LC_NO_SOLO") ? 0u : 1u;
  if (const char* e = getenv("S2LC_SOLO_MAXLIVE")) pq.solo_maxlive = (uint32_t)strtoul(e, nullptr, 10);
  {
    int dev = 0, khz = 100000;
    LVCHK(hipGetDevice(&dev));
    (void)hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, dev);
    unsigned long long us_ = 2000000;
    if (const char* e = getenv("S2LC_PERSIST_SPIN_US")) us_ = std::max<unsigned long long>(1, strtoull(e, nullptr, 10));
    pq.spin_ticks = std::max<unsigned long long>(1, (unsigned long long)khz * us_ / 1000);
  }
  LVCHK(hipEventRecord(L.ev[0], st));
  memset(hr, 0, sizeof(LvRun));
  bool aborted = false;
  for (;;) {
    LVCHK(hipMemsetAsync(L.bar, 0, sizeof(LvBar), st));
    LVCHK(hipMemsetAsync(L.ctl, 0, 3 * sizeof(LvCtl), st));
    if (lv_persist_launch(d.nq, L.grid_persist, p, pq, L.coop, st) != hipSuccess) {
      (void)hipGetLastError();
      aborted = true;
      break;
    }
    LVCHK(hipStreamSynchronize(st));
    if (hr->done == LVR_ABORT) { aborted = true; break; }
    if (hr->done != LVR_RUNNING || hr->nf >= wide) break;
  }
  LVCHK(hipEventRecord(L.ev[1], st));
  // (the last round's winners stay in its table, every other slot is clear:
  // the next switch clears the frontier's slots. An aborted launch left
  // entries anywhere: reset both tables for the host-driven rounds)
  if (aborted)
    for (int i = 0; i < 2; ++i) LVCHK(hipMemsetAsync(L.ht[i], 0xFF, ht_bytes, st));
  LVCHK(hipStreamSynchronize(st));
  float ms = 0;
  LVCHK(hipEventElapsedTime(&ms, L.ev[0], L.ev[1]));
  d.ms += ms;
  if (aborted) {
    // the frontier from the snapshot, as a caller-side buffer (no staging
    // array: the host-driven rounds stage into stg[0] and index into idx[1]);
    // trace entries from d.tnext on are overwritten by those rounds
    L.persist_refused = true;
    if (d.nf) {
      hipLaunchKernelGGL(lv_iota, dim3((uint32_t)std::min<uint64_t>(1024, (d.nf + 255) / 256)), dim3(256), 0, st, L.idx[0], d.nf);
      LVCHK(hipGetLastError());
    }
    LVCHK(hipStreamSynchronize(st));
    d.cur = d.snap;
    d.cur_loc = nullptr;
    d.cur_sel = 0;
    err = "persistent replicated rounds refused or timed out: host-driven rounds";
    return S2LC_EUNSUPPORTED;
  }
  const LvRun fin = *hr;
  if (fin.done == LVR_OVERFLOW) { err = "replicated round exceeds the device buffers"; return S2LC_ENOMEM; }
  d.children += fin.children;
  d.configs += fin.configs;
  d.max_frontier = std::max<uint64_t>(d.max_frontier, fin.max_frontier);
  *rounds = fin.round - R0;
  d.round += *rounds;
  d.tnext = fin.tnext;  // (trace entries written by these rounds: the witness walk reads them)
  if (fin.done == LVR_FOUND) {
    d.found_parent = fin.found_parent; d.found_move = fin.found_move; d.found_p4 = fin.found_p4;
    *found = 1;
    *n_next = 0;
    return 0;
  }
  if (fin.done == LVR_EMPTY) { d.nf = 0; *n_next = 0; return 0; }
  d.cur_sel = (int)(fin.round & 1);  // the last closed round's staging and index list
  d.cur = L.stg[d.cur_sel];
  d.cur_loc = nullptr;
  d.nf = fin.nf;
  *n_next = fin.nf;
  return 0;
}

// replicated -> partitioned: keep only the frontier configurations this rank owns
int dist_keep_owned(DistLevel& d, uint64_t* n_kept, std::string& err) {
  LevelBufs& L = d.b.lv;
  LvCtl* hc = reinterpret_cast<LvCtl*>(L.h_ctl);
  hipStream_t st = d.stream;
  LvParams p = dist_params(d);
  p.f1 = d.nf;
  p.nxt_idx = L.idx[d.cur_sel ^ 1];
  memset(hc, 0, sizeof(LvCtl));
  LVCHK(hipMemcpyAsync(L.ctl, hc, sizeof(LvCtl), hipMemcpyHostToDevice, st));
  // the tables hold the whole replicated frontier's entries (the dropped
  // configurations' too): clear them before the partitioned rounds
  if (dist_clear_frontier_slots(d, err)) return S2LC_EHIP;
  if (d.nf) LVCHK(lv_dispatch(d.nq, LK_KEEP, (uint32_t)std::min<uint64_t>(2048, (d.nf + LV_BLOCK - 1) / LV_BLOCK), p, st));
  LVCHK(hipMemcpyAsync(hc, L.ctl, sizeof(LvCtl), hipMemcpyDeviceToHost, st));
  LVCHK(hipStreamSynchronize(st));
  d.cur_sel ^= 1;
  d.nf = hc->nnext;
  *n_kept = d.nf;
  return 0;
}

// partitioned -> replicated, step 1: this rank's frontier, contiguous, into buf
int dist_frontier_pack(DistLevel& d, uint8_t* buf, std::string& err) {
  LvParams p = dist_params(d);
  p.f1 = d.nf;
  p.send = buf;
  if (d.nf) {
    const uint64_t pieces = (uint64_t)d.nf * (d.cb / 16);
    LVCHK(lv_dispatch(d.nq, LK_GATHER, (uint32_t)std::min<uint64_t>(2048, (pieces + LV_BLOCK - 1) / LV_BLOCK), p, d.stream));
  }
  LVCHK(hipStreamSynchronize(d.stream));
  return 0;
}

// partitioned -> replicated, step 2: the gathered frontier of all ranks
// (caller-owned device buffer, kept alive until the next round) becomes the
// frontier of every rank
int dist_frontier_load(DistLevel& d, uint8_t* buf, uint64_t n, std::string& err) {
  LevelBufs& L = d.b.lv;
  if (n > L.scap) { err = "gathered frontier exceeds the frontier capacity"; return S2LC_ENOMEM; }
  hipStream_t st = d.stream;
  const int sel = d.cur_sel ^ 1;
  if (n) hipLaunchKernelGGL(lv_iota, dim3((uint32_t)std::min<uint64_t>(1024, (n + 255) / 256)), dim3(256), 0, st, L.idx[sel], (uint32_t)n);
  LVCHK(hipGetLastError());
  // (ht[0] holds this rank's share of the gathered frontier, which is in the
  // new frontier with its slots: the next round's expansion, or the next
  // switch, clears them; ht[1] is clear)
  LVCHK(hipStreamSynchronize(st));
  d.cur = buf;
  d.cur_loc = nullptr;
  d.cur_sel = sel;
  d.nf = (uint32_t)n;
  return 0;
}

int dist_trace(DistLevel& d, uint32_t* out, uint64_t cap, uint64_t* n, std::string& err) {
  *n = d.tnext;
  if (!out) return 0;
  if (cap < d.tnext) { err = "trace buffer too small"; return S2LC_EINVAL; }
  if (d.tnext) LVCHK(hipMemcpy(out, d.trace, d.tnext * sizeof(TraceEnt), hipMemcpyDeviceToHost));
  return 0;
}

}  // namespace s2lc
