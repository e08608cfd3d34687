// level.hip — host driver of the device-wide level-synchronous search of one
// history (kernels in level_dev.h). Called by batch_run for histories with
// more than 128 chains and for histories whose frontier outgrew the
// per-workgroup passes. One round = lv_expand -> lv_close -> lv_insert, then
// one 64-byte control read-back decides: found (Ok), empty (Illegal), or the
// next round. A round whose children or staged configurations exceed the
// device buffers is re-run over halves of its frontier.
#include <hip/hip_runtime.h>
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

size_t lv_cfg_bytes(uint32_t kmax) { return 48 + 2 * (size_t)kmax; }

template <int KMAX>
hipError_t lv_launch(int which, uint32_t grid, const LvParams& p, hipStream_t st) {
  if (which == 0) hipLaunchKernelGGL(lv_expand<KMAX>, dim3(grid), dim3(LV_BLOCK), 0, st, p);
  else if (which == 1) hipLaunchKernelGGL(lv_close<KMAX>, dim3(grid), dim3(LV_BLOCK), 0, st, p);
  else if (which == 2) hipLaunchKernelGGL(lv_insert<KMAX>, dim3(grid), dim3(LV_BLOCK), 0, st, p);
  else if (which == 3) hipLaunchKernelGGL(lv_bucket<KMAX>, dim3(grid), dim3(LV_BLOCK), 0, st, p);
  else if (which == 4) hipLaunchKernelGGL(lv_scatter<KMAX>, dim3(grid), dim3(LV_BLOCK), 0, st, p);
  else if (which == 5) hipLaunchKernelGGL(lv_keep<KMAX>, dim3(grid), dim3(LV_BLOCK), 0, st, p, (uint32_t)(p.tgid >> 29));
  else hipLaunchKernelGGL(lv_gather_frontier<KMAX>, dim3(grid), dim3(LV_BLOCK), 0, st, p);
  return hipGetLastError();
}

hipError_t lv_dispatch(uint32_t kmax, int which, uint32_t grid, const LvParams& p, hipStream_t st) {
  switch (kmax) {
    case 64: return lv_launch<64>(which, grid, p, st);
    case 128: return lv_launch<128>(which, grid, p, st);
    case 256: return lv_launch<256>(which, grid, p, st);
    default: return lv_launch<512>(which, grid, p, st);
  }
}

int lv_ensure(void** p, size_t& cap, size_t need, std::string& err) {
  if (need <= cap) return 0;
  if (*p) (void)hipFree(*p);
  *p = nullptr;
  cap = 0;
  LVCHK(hipMalloc(p, need));
  cap = need;
  return 0;
}

}  // namespace

uint32_t level_kmax(uint32_t K) { return K <= 64 ? 64 : K <= 128 ? 128 : K <= 256 ? 256 : 512; }

int level_buffers(DevBatch& b, uint32_t kmax, std::string& err) {
  LevelBufs& L = b.lv;
  if (L.kmax >= kmax && L.ctl) return 0;
  size_t free_b = 0, total_b = 0;
  LVCHK(hipMemGetInfo(&free_b, &total_b));
  // a quarter of free HBM (at most 48 GiB): two staging arrays + index
  // lists + table, and the children array
  const size_t budget = std::min<size_t>(free_b / 4, 48ull << 30);
  const size_t cb = lv_cfg_bytes(kmax);
  uint64_t scap = std::min<uint64_t>(1ull << 24, (uint64_t)(budget * 6 / 10) / (2 * cb + 2 * 4 + 2 * 8));
  uint64_t ccap = std::min<uint64_t>(1ull << 26, (uint64_t)(budget * 3 / 10) / sizeof(LChild));
  scap = std::max<uint64_t>(scap, 1024);
  ccap = std::max<uint64_t>(ccap, 4096);
  // S2LC_LEVEL_SCAP (tests): a small staging capacity, to reach the
  // frontier-overflow paths with small histories
  if (const char* e = getenv("S2LC_LEVEL_SCAP")) {
    const uint64_t v = strtoull(e, nullptr, 10);
    if (v >= 64) scap = std::min<uint64_t>(scap, v);
  }
  uint64_t ht = 1024;
  while (ht < 2 * scap) ht <<= 1;
  if (lv_ensure((void**)&L.child, L.child_bytes, ccap * sizeof(LChild), err)) return S2LC_EHIP;
  for (int i = 0; i < 2; ++i) {
    if (lv_ensure((void**)&L.stg[i], L.stg_bytes[i], scap * cb, err)) return S2LC_EHIP;
    if (lv_ensure((void**)&L.idx[i], L.idx_bytes[i], scap * sizeof(uint32_t), err)) return S2LC_EHIP;
  }
  if (lv_ensure((void**)&L.ht, L.ht_bytes, ht * 8, err)) return S2LC_EHIP;
  if (!L.ctl) LVCHK(hipMalloc(&L.ctl, 2 * sizeof(LvCtl)));  // double buffered by round
  if (!L.h_ctl) LVCHK(hipHostMalloc(&L.h_ctl, sizeof(LvCtl), hipHostMallocDefault));
  LVCHK(hipMemset(L.ht, 0xFF, ht * 8));
  L.kmax = kmax;
  L.scap = (uint32_t)scap;
  L.ccap = (uint32_t)ccap;
  L.ht_mask = (uint32_t)(ht - 1);
  return 0;
}

void level_release(DevBatch& b) {
  LevelBufs& L = b.lv;
  void* ptrs[] = {L.child, L.stg[0], L.stg[1], L.idx[0], L.idx[1], L.ht, L.ctl};
  for (void* q : ptrs) if (q) (void)hipFree(q);
  if (L.h_ctl) (void)hipHostFree(L.h_ctl);
  L = LevelBufs{};
}

int level_search(DevBatch& b, uint32_t h, hipStream_t st, const RunOpts& ro, int64_t deadline_ns, LevelStats& ls,
                 std::string& err) {
  const uint64_t max_configs = ro.max_configs;
  const bool witness = ro.witness;
  uint32_t* const rc = ro.round_counts && !b.h_rcounts.empty() ? b.h_rcounts.data() + b.h_moves_off[h] : nullptr;
  const HistDesc& hd = b.h_hist[h];
  const uint32_t K = hd.K;
  const uint32_t kmax = level_kmax(K);
  if (level_buffers(b, kmax, err)) return S2LC_EHIP;
  LevelBufs& L = b.lv;
  LvCtl* hc = reinterpret_cast<LvCtl*>(L.h_ctl);
  int dev = 0;
  LVCHK(hipGetDevice(&dev));
  int n_cu = 256;
  (void)hipDeviceGetAttribute(&n_cu, hipDeviceAttributeMultiprocessorCount, dev);
  const uint32_t max_grid = (uint32_t)n_cu * 8;

  // trace entries continue after what earlier passes / histories used
  unsigned long long tb0 = 0;
  if (witness && b.trace) {
    LVCHK(hipMemcpyAsync(&tb0, b.trace_head, sizeof tb0, hipMemcpyDeviceToHost, st));
    LVCHK(hipStreamSynchronize(st));
  }
  bool wit = witness && b.trace != nullptr;

  LvCtl* d_hc = nullptr;  // device view of the host-mapped control mirror
  LVCHK(hipHostGetDevicePointer((void**)&d_hc, hc, 0));
  LVCHK(hipMemsetAsync(L.ctl, 0, 2 * sizeof(LvCtl), st));

  LvParams p;
  memset(&p, 0, sizeof p);
  p.recs = b.recs; p.pool = b.pool; p.cs = b.chain_start + hd.cs_base; p.K = K; p.hflags = hd.flags;
  p.child = reinterpret_cast<LChild*>(L.child); p.ccap = L.ccap; p.scap = L.scap; p.ht = L.ht; p.ht_mask = L.ht_mask;
  p.trace = b.trace; p.ctl = reinterpret_cast<LvCtl*>(L.ctl);

  hipEvent_t e0, e1;
  LVCHK(hipEventCreate(&e0));
  LVCHK(hipEventCreate(&e1));
  LVCHK(hipEventRecord(e0, st));

  // round 0: the initial configuration as the only child, closed + inserted
  memset(hc, 0, sizeof(LvCtl));
  hc->nchild = 1;
  const LChild c0{0, 0, 0, LV_NONE, LV_NONE, 0};
  LVCHK(hipMemcpyAsync(L.child, &c0, sizeof c0, hipMemcpyHostToDevice, st));
  LVCHK(hipMemcpyAsync(L.ctl, hc, sizeof(LvCtl), hipMemcpyHostToDevice, st));
  int cur = 0;  // round r stages into stg[cur ^ 1]; its frontier is stg[cur]
  p.cur = L.stg[cur]; p.cur_idx = L.idx[cur];
  p.stg = L.stg[cur ^ 1]; p.nxt_idx = L.idx[cur ^ 1];
  p.tbase = (uint32_t)tb0; p.witness = wit ? 1u : 0u;
  if (wit && tb0 + 1 > b.trace_cap) { wit = false; p.witness = 0; }
  LVCHK(lv_dispatch(kmax, 1, 1, p, st));
  LVCHK(lv_dispatch(kmax, 2, 1, p, st));
  LVCHK(hipMemcpyAsync(hc, L.ctl, sizeof(LvCtl), hipMemcpyDeviceToHost, st));
  LVCHK(hipStreamSynchronize(st));

  uint64_t configs = 0, children = 0, tnext = tb0;
  uint32_t rounds = 0, max_frontier = 0;
  uint32_t verdict = V_ILLEGAL, reason = S2LC_R_SEARCH_EXHAUSTED;
  uint32_t deep_trace = TRACE_NONE, deep_len = 0;
  for (;;) {
    if (hc->found) { verdict = V_OK; reason = 0; break; }
    const uint32_t nf = hc->nnext;
    if (rc) rc[rounds] = nf;
    if (nf == 0) {
      verdict = V_ILLEGAL; reason = S2LC_R_SEARCH_EXHAUSTED;
      if (rounds > 0 && p.witness) {
        // a configuration of the deepest non-empty round (the input of the last one)
        uint32_t k = 0;
        LVCHK(hipMemcpy(&k, L.idx[cur], sizeof k, hipMemcpyDeviceToHost));
        LVCHK(hipMemcpy(&deep_trace, L.stg[cur] + (size_t)k * lv_cfg_bytes(kmax) + 40, sizeof deep_trace,
                        hipMemcpyDeviceToHost));  // LCfg::trace
        deep_len = rounds - 1;
      }
      break;
    }
    configs += nf;
    max_frontier = std::max(max_frontier, nf);
    if (p.witness) tnext += nf;
    if (max_configs && configs > max_configs) { verdict = V_UNKNOWN; reason = S2LC_R_BUDGET; break; }
    if (deadline_ns && steady_ns() > deadline_ns) { verdict = V_UNKNOWN; reason = S2LC_R_TIMEOUT; break; }
    cur ^= 1;
    p.cur = L.stg[cur]; p.cur_idx = L.idx[cur];
    p.stg = L.stg[cur ^ 1]; p.nxt_idx = L.idx[cur ^ 1];
    p.clear_slots = 1;
    if (wit && tnext + L.scap > b.trace_cap) wit = false;
    p.witness = wit ? 1u : 0u;
    p.tbase = (uint32_t)tnext;
    ++rounds;
    // one round, in frontier chunks (normally one). Round r uses control
    // block r & 1, which round r-1's lv_expand zeroed, and lv_insert publishes
    // it to the host-mapped mirror hc: the single-chunk round needs no copies.
    LvCtl* const ctl_r = reinterpret_cast<LvCtl*>(L.ctl) + (rounds & 1);
    p.ctl = ctl_r;
    p.ctl_next = reinterpret_cast<LvCtl*>(L.ctl) + ((rounds + 1) & 1);
    p.publish = d_hc;
    uint32_t f0 = 0, chunk = nf, st_lo = 0, nn_lo = 0;
    bool stop = false;
    bool first = true;
    while (f0 < nf) {
      const uint32_t f1 = (uint32_t)std::min<uint64_t>(nf, (uint64_t)f0 + chunk);
      if (!first) {
        memset(hc, 0, sizeof(LvCtl));
        hc->nchild = 0; hc->nstage = st_lo; hc->nnext = nn_lo; hc->overflow = 0;
        LVCHK(hipMemcpyAsync(ctl_r, hc, sizeof(LvCtl), hipMemcpyHostToDevice, st));
      }
      first = false;
      p.f0 = f0; p.f1 = f1; p.st_lo = st_lo;
      const uint64_t lanes = (uint64_t)(f1 - f0) * K;
      const uint32_t g_exp = (uint32_t)std::min<uint64_t>(max_grid, (lanes + LV_BLOCK - 1) / LV_BLOCK);
      const uint64_t kids_ub = std::min<uint64_t>(2 * lanes, L.ccap);
      const uint32_t g_cls = (uint32_t)std::min<uint64_t>(max_grid, (kids_ub + 3) / 4);
      const uint32_t g_ins = (uint32_t)std::min<uint64_t>(max_grid, (std::min<uint64_t>(kids_ub, L.scap) + LV_BLOCK - 1) / LV_BLOCK);
      LVCHK(lv_dispatch(kmax, 0, std::max<uint32_t>(1, g_exp), p, st));
      LVCHK(lv_dispatch(kmax, 1, std::max<uint32_t>(1, g_cls), p, st));
      LVCHK(lv_dispatch(kmax, 2, std::max<uint32_t>(1, g_ins), p, st));
      LVCHK(hipStreamSynchronize(st));  // hc was published by lv_insert's last block
      if (hc->found) break;
      if (hc->overflow) {
        if (f1 - f0 == 1) { verdict = V_UNKNOWN; reason = S2LC_R_FRONTIER; stop = true; break; }
        chunk = std::max<uint32_t>(1, (f1 - f0) / 2);
        ++ls.chunk_retries;
        continue;
      }
      children += std::min(hc->nchild, L.ccap);
      st_lo = std::min(hc->nstage, L.scap);
      nn_lo = hc->nnext;
      f0 = f1;
    }
    if (hc->found) children += std::min(hc->nchild, L.ccap);
    if (stop) break;
  }
  LVCHK(hipEventRecord(e1, st));
  LVCHK(hipEventSynchronize(e1));
  float ms = 0;
  LVCHK(hipEventElapsedTime(&ms, e0, e1));
  LVCHK(hipEventDestroy(e0));
  LVCHK(hipEventDestroy(e1));
  // clear the table for the next search (slots of the last frontier; cheap
  // enough to reset whole when the frontier was large)
  LVCHK(hipMemsetAsync(L.ht, 0xFF, ((size_t)L.ht_mask + 1) * 8, st));

  HistResult& R = b.h_res[h];
  const uint32_t woff = R.witness_off;
  R = HistResult{};
  R.witness_off = woff;
  R.verdict = verdict;
  R.reason = reason;
  R.rounds = rounds;
  R.configs = configs;
  R.children = children;
  R.p4 = verdict == V_OK ? hc->found_p4 : 0;
  const bool have_w = verdict == V_OK && wit;
  R.final_parent = have_w ? hc->found_parent : TRACE_NONE;
  R.final_move = verdict == V_OK ? hc->found_move : TRACE_NONE;
  R.deep_trace = deep_trace;
  R.deep_len = deep_len;
  R.has_witness = (have_w || deep_trace != TRACE_NONE) ? 2u : 0u;
  LVCHK(hipMemcpyAsync(b.res + h, &R, sizeof R, hipMemcpyHostToDevice, st));
  if (witness && b.trace) {
    unsigned long long th = tnext;
    LVCHK(hipMemcpyAsync(b.trace_head, &th, sizeof th, hipMemcpyHostToDevice, st));
  }
  LVCHK(hipStreamSynchronize(st));
  ls.ms += ms;
  ls.rounds += rounds;
  ls.configs += configs;
  ls.children += children;
  ls.max_frontier = std::max(ls.max_frontier, max_frontier);
  ls.histories++;
  return 0;
}


// ============================================================================
// Distributed level search of one history (BASELINE config C5 over several
// GPUs). Configurations are owned by rank lv_owner(fp). A round
// on each rank:
//   dist_expand : expand + close the local frontier (as above) into local
//                 staging, count the staged configurations per owner rank
//   (caller)    : all-to-all of the counts, allocate the send buffer
//   dist_pack   : copy the staged configurations into owner-major buckets
//   (caller)    : all-to-all(v) of the buckets over RCCL / xGMI
//   dist_insert : deduplicate what this rank received (it owns all of it) in
//                 the local table; the winners are its next frontier
// The received buffer stays the frontier of the next round (the caller keeps
// it alive). Trace ids are rank << 29 | local pool index, so the parent chain
// of a witness crosses ranks; the caller gathers the pools at the end.
// ============================================================================

int dist_create(DistLevel& d, const History* h, uint32_t rank, uint32_t world, uint32_t reductions_off,
                std::string& err) {
  if (world < 1 || world > 8 || rank >= world) { err = "world must be 1..8"; return S2LC_EINVAL; }
  std::vector<const History*> hs{h};
  int rc = batch_upload(d.b, hs, reductions_off, err);
  if (rc) return rc;
  d.rank = rank;
  d.world = world;
  d.K = d.b.h_hist[0].K;
  d.kmax = level_kmax(d.K);
  d.cb = lv_cfg_bytes(d.kmax);
  if (d.b.forced[0]) { err = "history is structurally illegal (unmatched events)"; return S2LC_EINVAL; }
  if (level_buffers(d.b, d.kmax, err)) return S2LC_EHIP;
  LVCHK(hipMalloc(&d.own_cnt, 8 * sizeof(uint32_t)));
  LVCHK(hipMalloc(&d.own_pos, (size_t)d.b.lv.scap * sizeof(uint32_t)));
  size_t free_b = 0, total_b = 0;
  LVCHK(hipMemGetInfo(&free_b, &total_b));
  d.trace_cap = std::min<uint64_t>(1ull << 29, (uint64_t)(free_b / 16) / sizeof(TraceEnt));
  LVCHK(hipMalloc(&d.trace, d.trace_cap * sizeof(TraceEnt)));
  LVCHK(hipStreamCreateWithFlags(&d.stream, hipStreamNonBlocking));
  d.round = 0;
  return 0;
}

void dist_release(DistLevel& d) {
  if (d.own_cnt) (void)hipFree(d.own_cnt);
  if (d.own_pos) (void)hipFree(d.own_pos);
  if (d.trace) (void)hipFree(d.trace);
  if (d.stream) (void)hipStreamDestroy(d.stream);
  d.own_cnt = nullptr; d.own_pos = nullptr; d.trace = nullptr; d.stream = nullptr;
  batch_release(d.b);
}

static LvParams dist_params(DistLevel& d) {
  LevelBufs& L = d.b.lv;
  const HistDesc& hd = d.b.h_hist[0];
  LvParams p;
  memset(&p, 0, sizeof p);
  p.recs = d.b.recs; p.pool = d.b.pool; p.cs = d.b.chain_start + hd.cs_base; p.K = d.K; p.hflags = hd.flags;
  p.child = reinterpret_cast<LChild*>(L.child); p.ccap = L.ccap; p.scap = L.scap;
  p.ht = L.ht; p.ht_mask = L.ht_mask;
  p.trace = d.trace; p.ctl = reinterpret_cast<LvCtl*>(L.ctl);
  p.world = d.world; p.own_cnt = d.own_cnt; p.own_pos = d.own_pos;
  // local staging (the closed children of this rank): the array that does not
  // hold the current frontier
  p.stg = d.cur == L.stg[0] ? L.stg[1] : L.stg[0];
  p.cur = d.cur; p.cur_idx = L.idx[d.cur_sel];
  p.tgid = d.rank << 29;
  return p;
}

int dist_expand(DistLevel& d, uint64_t* counts, int* found, std::string& err) {
  LevelBufs& L = d.b.lv;
  LvCtl* hc = reinterpret_cast<LvCtl*>(L.h_ctl);
  int dev = 0;
  LVCHK(hipGetDevice(&dev));
  int n_cu = 256;
  (void)hipDeviceGetAttribute(&n_cu, hipDeviceAttributeMultiprocessorCount, dev);
  const uint32_t max_grid = (uint32_t)n_cu * 8;
  hipStream_t st = d.stream;
  LvParams p = dist_params(d);
  hipEvent_t e0, e1;
  LVCHK(hipEventCreate(&e0));
  LVCHK(hipEventCreate(&e1));
  LVCHK(hipEventRecord(e0, st));
  memset(hc, 0, sizeof(LvCtl));
  LVCHK(hipMemsetAsync(d.own_cnt, 0, 8 * sizeof(uint32_t), st));
  if (d.round == 0) {
    // the initial configuration: closed on rank 0 only
    if (d.rank == 0) {
      hc->nchild = 1;
      const LChild c0{0, 0, 0, LV_NONE, LV_NONE, 0};
      LVCHK(hipMemcpyAsync(L.child, &c0, sizeof c0, hipMemcpyHostToDevice, st));
    }
    LVCHK(hipMemcpyAsync(L.ctl, hc, sizeof(LvCtl), hipMemcpyHostToDevice, st));
    if (d.rank == 0) LVCHK(lv_dispatch(d.kmax, 1, 1, p, st));
  } else {
    LVCHK(hipMemcpyAsync(L.ctl, hc, sizeof(LvCtl), hipMemcpyHostToDevice, st));
    if (d.nf) {
      p.f0 = 0; p.f1 = d.nf; p.clear_slots = 1;
      const uint64_t lanes = (uint64_t)d.nf * d.K;
      const uint64_t kids_ub = std::min<uint64_t>(2 * lanes, L.ccap);
      LVCHK(lv_dispatch(d.kmax, 0, (uint32_t)std::max<uint64_t>(1, std::min<uint64_t>(max_grid, (lanes + LV_BLOCK - 1) / LV_BLOCK)), p, st));
      LVCHK(lv_dispatch(d.kmax, 1, (uint32_t)std::max<uint64_t>(1, std::min<uint64_t>(max_grid, (kids_ub + 3) / 4)), p, st));
    }
  }
  // ownership buckets
  const uint32_t g_b = max_grid;
  LVCHK(lv_dispatch(d.kmax, 3, g_b, p, st));
  uint32_t cnt[8] = {0};
  LVCHK(hipMemcpyAsync(cnt, d.own_cnt, sizeof cnt, hipMemcpyDeviceToHost, st));
  LVCHK(hipMemcpyAsync(hc, L.ctl, sizeof(LvCtl), hipMemcpyDeviceToHost, st));
  LVCHK(hipEventRecord(e1, st));
  LVCHK(hipStreamSynchronize(st));
  float ms = 0;
  LVCHK(hipEventElapsedTime(&ms, e0, e1));
  (void)hipEventDestroy(e0);
  (void)hipEventDestroy(e1);
  d.ms += ms;
  if (hc->overflow) { err = "distributed round exceeds the device buffers"; return S2LC_ENOMEM; }
  d.children += std::min(hc->nchild, L.ccap);
  d.nstage = std::min(hc->nstage, L.scap);
  for (uint32_t o = 0; o < d.world; ++o) counts[o] = cnt[o];
  *found = hc->found ? 1 : 0;
  if (hc->found) { d.found_parent = hc->found_parent; d.found_move = hc->found_move; d.found_p4 = hc->found_p4; }
  return 0;
}

int dist_pack(DistLevel& d, uint8_t* send, const uint64_t* counts, std::string& err) {
  LvParams p = dist_params(d);
  uint64_t off = 0;
  for (uint32_t o = 0; o < d.world; ++o) { p.own_off[o] = off; off += counts[o]; }
  if (off != d.nstage) { err = "bucket counts do not match the staged configurations"; return S2LC_EINVAL; }
  p.send = send;
  if (d.nstage) {
    const uint64_t pieces = (uint64_t)d.nstage * (d.cb / 16);
    LVCHK(lv_dispatch(d.kmax, 4, (uint32_t)std::max<uint64_t>(1, std::min<uint64_t>(2048, (pieces + LV_BLOCK - 1) / LV_BLOCK)), p, d.stream));
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
  p.stg = recv; p.nxt_idx = L.idx[sel]; p.st_lo = 0;
  p.witness = 1;
  if (d.tnext + n_recv > d.trace_cap) { err = "trace pool full"; return S2LC_ENOMEM; }
  p.tbase = (uint32_t)d.tnext;
  memset(hc, 0, sizeof(LvCtl));
  hc->nstage = (uint32_t)n_recv;
  hipEvent_t e0, e1;
  LVCHK(hipEventCreate(&e0));
  LVCHK(hipEventCreate(&e1));
  LVCHK(hipEventRecord(e0, st));
  LVCHK(hipMemcpyAsync(L.ctl, hc, sizeof(LvCtl), hipMemcpyHostToDevice, st));
  if (n_recv) {
    int dev = 0, n_cu = 256;
    LVCHK(hipGetDevice(&dev));
    (void)hipDeviceGetAttribute(&n_cu, hipDeviceAttributeMultiprocessorCount, dev);
    LVCHK(lv_dispatch(d.kmax, 2, (uint32_t)std::max<uint64_t>(1, std::min<uint64_t>((uint64_t)n_cu * 8, (n_recv + LV_BLOCK - 1) / LV_BLOCK)), p, st));
  }
  LVCHK(hipMemcpyAsync(hc, L.ctl, sizeof(LvCtl), hipMemcpyDeviceToHost, st));
  LVCHK(hipEventRecord(e1, st));
  LVCHK(hipStreamSynchronize(st));
  float ms = 0;
  LVCHK(hipEventElapsedTime(&ms, e0, e1));
  (void)hipEventDestroy(e0);
  (void)hipEventDestroy(e1);
  d.ms += ms;
  d.cur = recv;
  d.cur_sel = sel;
  d.nf = hc->nnext;
  d.tnext += hc->nnext;
  d.configs += hc->nnext;
  d.max_frontier = std::max<uint64_t>(d.max_frontier, hc->nnext);
  d.round++;
  *n_next = hc->nnext;
  return 0;
}

// ---- replicated rounds (narrow frontiers): every rank runs the same round on
// the whole frontier, with no exchange; the set of configurations, and so
// every decision, is the same on all ranks.
int dist_local_round(DistLevel& d, uint64_t* n_next, int* found, std::string& err) {
  LevelBufs& L = d.b.lv;
  LvCtl* hc = reinterpret_cast<LvCtl*>(L.h_ctl);
  int dev = 0, n_cu = 256;
  LVCHK(hipGetDevice(&dev));
  (void)hipDeviceGetAttribute(&n_cu, hipDeviceAttributeMultiprocessorCount, dev);
  const uint64_t max_grid = (uint64_t)n_cu * 8;
  hipStream_t st = d.stream;
  LvParams p = dist_params(d);
  p.nxt_idx = L.idx[d.cur_sel ^ 1];
  p.witness = 1;
  if (d.tnext + L.scap > d.trace_cap) { err = "trace pool full"; return S2LC_ENOMEM; }
  p.tbase = (uint32_t)d.tnext;
  hipEvent_t e0, e1;
  LVCHK(hipEventCreate(&e0));
  LVCHK(hipEventCreate(&e1));
  LVCHK(hipEventRecord(e0, st));
  memset(hc, 0, sizeof(LvCtl));
  if (d.round == 0) {
    hc->nchild = 1;
    const LChild c0{0, 0, 0, LV_NONE, LV_NONE, 0};
    LVCHK(hipMemcpyAsync(L.child, &c0, sizeof c0, hipMemcpyHostToDevice, st));
    LVCHK(hipMemcpyAsync(L.ctl, hc, sizeof(LvCtl), hipMemcpyHostToDevice, st));
    LVCHK(lv_dispatch(d.kmax, 1, 1, p, st));
    LVCHK(lv_dispatch(d.kmax, 2, 1, p, st));
  } else {
    LVCHK(hipMemcpyAsync(L.ctl, hc, sizeof(LvCtl), hipMemcpyHostToDevice, st));
    p.f0 = 0; p.f1 = d.nf; p.clear_slots = 1;
    const uint64_t lanes = (uint64_t)d.nf * d.K;
    const uint64_t kids_ub = std::min<uint64_t>(2 * lanes, L.ccap);
    LVCHK(lv_dispatch(d.kmax, 0, (uint32_t)std::max<uint64_t>(1, std::min(max_grid, (lanes + LV_BLOCK - 1) / LV_BLOCK)), p, st));
    LVCHK(lv_dispatch(d.kmax, 1, (uint32_t)std::max<uint64_t>(1, std::min(max_grid, (kids_ub + 3) / 4)), p, st));
    LVCHK(lv_dispatch(d.kmax, 2, (uint32_t)std::max<uint64_t>(1, std::min(max_grid, (std::min<uint64_t>(kids_ub, L.scap) + LV_BLOCK - 1) / LV_BLOCK)), p, st));
  }
  LVCHK(hipMemcpyAsync(hc, L.ctl, sizeof(LvCtl), hipMemcpyDeviceToHost, st));
  LVCHK(hipEventRecord(e1, st));
  LVCHK(hipStreamSynchronize(st));
  float ms = 0;
  LVCHK(hipEventElapsedTime(&ms, e0, e1));
  (void)hipEventDestroy(e0);
  (void)hipEventDestroy(e1);
  d.ms += ms;
  if (hc->overflow && !hc->found) { err = "replicated round exceeds the device buffers"; return S2LC_ENOMEM; }
  d.children += std::min(hc->nchild, L.ccap);
  *found = hc->found ? 1 : 0;
  if (hc->found) {
    d.found_parent = hc->found_parent; d.found_move = hc->found_move; d.found_p4 = hc->found_p4;
    *n_next = 0;
    return 0;
  }
  d.cur = p.stg;
  d.cur_sel ^= 1;
  d.nf = hc->nnext;
  d.tnext += hc->nnext;
  d.configs += hc->nnext;
  d.max_frontier = std::max<uint64_t>(d.max_frontier, hc->nnext);
  d.round++;
  *n_next = hc->nnext;
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
  if (d.nf) LVCHK(lv_dispatch(d.kmax, 5, (uint32_t)std::min<uint64_t>(2048, (d.nf + LV_BLOCK - 1) / LV_BLOCK), p, st));
  // the table still holds the dropped configurations' slots: reset it
  LVCHK(hipMemsetAsync(L.ht, 0xFF, ((size_t)L.ht_mask + 1) * 8, st));
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
    LVCHK(lv_dispatch(d.kmax, 6, (uint32_t)std::max<uint64_t>(1, std::min<uint64_t>(2048, (pieces + LV_BLOCK - 1) / LV_BLOCK)), p, d.stream));
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
  LVCHK(hipMemsetAsync(L.ht, 0xFF, ((size_t)L.ht_mask + 1) * 8, st));
  LVCHK(hipStreamSynchronize(st));
  d.cur = buf;
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
