// search.hip — frontier-parallel linearizability search for the S2 model on
// gfx950 (MI355X). Replaces porcupine v1.0.3 checkSingle (WGL backtracking DFS
// with a (bitset, state) cache, called at golang/s2-porcupine/main.go:606).
//
// Search space: configurations (L, s) with L a down-set of the real-time
// order, encoded as K per-chain prefix counters (greedy interval colouring,
// history.cpp), and s a single S2 state (the powerset state is exploded).
// One ROUND linearizes exactly one non-identity op (durable or indefinite
// append) per configuration, then closes the child under the identity ops
// (reads, check-tails, definite failures) that are minimal and legal — a
// verdict-exact reduction. Configurations are deduplicated per
// round in an open-addressing table with 64-bit atomicCAS; survivors are
// compacted into the next frontier.
//
// Work mapping: one workgroup owns one history at a time (persistent grid,
// atomic work counter, longest-first order); inside a round, one lane per
// (configuration, chain) candidate. Frontier, staging and table live in a
// per-workgroup HBM slab (L2-resident at these sizes); chain offsets in LDS.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <chrono>
#include <numeric>
#include <string>

#include "s2lincheck.h"
#include "search.h"
#include "search_dev.h"
#include "pack_dev.h"

namespace s2lc {

namespace {

#define HIPCHK(x)                                                        \
  do {                                                                   \
    hipError_t e_ = (x);                                                 \
    if (e_ != hipSuccess) {                                              \
      err = std::string(#x) + ": " + hipGetErrorString(e_);              \
      return S2LC_EHIP;                                                  \
    }                                                                    \
  } while (0)

template <int KMAX, int BT, bool SHARED>
hipError_t launch_search(const Params& prm, uint32_t grid, size_t smem, hipStream_t st) {
  hipLaunchKernelGGL((search_kernel<KMAX, BT, SHARED>), dim3(grid), dim3(BT), smem, st, prm);
  return hipGetLastError();
}

template <bool SHARED>
hipError_t launch_kmax(uint32_t kmax, uint32_t block, const Params& prm, uint32_t grid, size_t smem, hipStream_t st) {
  if (block == 64) {
    switch (kmax) {
      case 16: return launch_search<16, 64, SHARED>(prm, grid, smem, st);
      case 32: return launch_search<32, 64, SHARED>(prm, grid, smem, st);
      case 64: return launch_search<64, 64, SHARED>(prm, grid, smem, st);
      default: return launch_search<128, 64, SHARED>(prm, grid, smem, st);
    }
  }
  switch (kmax) {
    case 16: return launch_search<16, 256, SHARED>(prm, grid, smem, st);
    case 32: return launch_search<32, 256, SHARED>(prm, grid, smem, st);
    case 64: return launch_search<64, 256, SHARED>(prm, grid, smem, st);
    default: return launch_search<128, 256, SHARED>(prm, grid, smem, st);
  }
}

size_t cfg_bytes(uint32_t kmax) { return 48 + 2 * (size_t)kmax; }

size_t state_bytes(uint32_t kmax) {
  switch (kmax) {
    case 16: return wg_state_bytes<16>();
    case 32: return wg_state_bytes<32>();
    case 64: return wg_state_bytes<64>();
    default: return wg_state_bytes<128>();
  }
}

SearchGeom make_geom(uint32_t kmax, bool shared, uint32_t block, uint32_t fcap, uint32_t stage_cap, uint32_t chunk,
                     uint32_t grid, size_t lds_budget) {
  SearchGeom g;
  g.block = block;
  g.kmax = kmax;
  g.fcap = fcap;
  g.chunk = chunk;
  g.stage_cap = stage_cap;
  g.shared = shared;
  uint32_t ht = 16;
  while (ht < 2 * (fcap + stage_cap)) ht <<= 1;
  g.ht_slots = ht;
  g.grid = grid;
  g.cfg_bytes = cfg_bytes(kmax);
  size_t arrays = (2 * (size_t)fcap + stage_cap) * g.cfg_bytes + (size_t)ht * 8;
  g.win_recs = 0;
  if (shared) {
    // the rest of the per-workgroup LDS budget holds the record window
    // (at most WIN_ITEMS 16-byte pieces per lane, i.e. 2 records per lane)
    const size_t used = state_bytes(kmax) + arrays;
    const size_t cap = (size_t)WIN_ITEMS * block / 4;
    g.win_recs = used < lds_budget ? (uint32_t)std::min(cap, (lds_budget - used) / sizeof(OpRec)) : 0;
    arrays += (size_t)g.win_recs * sizeof(OpRec);
  }
  arrays = (arrays + 255) & ~(size_t)255;
  g.smem_bytes = state_bytes(kmax) + (shared ? arrays : 0);
  g.slab_bytes = shared ? 0 : arrays;
  return g;
}

hipError_t launch_geom(const SearchGeom& g, const Params& prm, hipStream_t st) {
  return g.shared ? launch_kmax<true>(g.kmax, g.block, prm, g.grid, g.smem_bytes, st)
                  : launch_kmax<false>(g.kmax, g.block, prm, g.grid, g.smem_bytes, st);
}

}  // namespace

int batch_upload(DevBatch& b, const std::vector<const History*>& hs, std::string& err) {
  b.n_hist = (uint32_t)hs.size();
  b.src = hs;
  b.forced.assign(hs.size(), 0);
  uint32_t kmax_needed = 1;
  size_t n_recs = 0, n_pool = 0, n_cs = 0;
  uint64_t moves_total = 0;
  b.h_hist.resize(hs.size());
  b.h_moves_off.resize(hs.size());
  b.h_in_bytes.assign(hs.size(), 0);
  for (size_t i = 0; i < hs.size(); ++i) {
    const History& h = *hs[i];
    if (h.status != 0) { err = "history " + std::to_string(i) + ": " + h.error; return h.status; }
    if (h.structural) { b.forced[i] = 1; }
    if (h.K > LEVEL_KMAX) { err = "history has more than 512 concurrent chains"; return S2LC_EUNSUPPORTED; }
    if (h.max_chain_len >= 0xFFFF) { err = "chain longer than 65534 ops"; return S2LC_EUNSUPPORTED; }
    if (h.K <= 128) kmax_needed = std::max(kmax_needed, h.K);
    HistDesc& d = b.h_hist[i];
    d.rec_base = (uint32_t)n_recs;
    d.cs_base = (uint32_t)n_cs;
    d.K = (uint16_t)h.K;
    d.flags = h.hflags;
    d.n_ops = h.n_ops;
    n_recs += h.recs.size();
    n_cs += h.K + 1;
    n_pool += h.pool.size();
    b.h_moves_off[i] = (uint32_t)moves_total;
    moves_total += h.n_ops + 1;
    uint64_t in_bytes = 48ull * h.n_ops;
    for (const OpRec& r : h.recs) in_bytes += 8ull * r.hash_cnt;
    b.h_in_bytes[i] = in_bytes;
    b.algo_bytes_inputs += in_bytes;
  }
  if (n_recs >= 0xFFFFFFFFull || n_pool >= 0xFFFFFFFFull || moves_total >= 0xFFFFFFFFull) {
    err = "batch too large for 32-bit indices";
    return S2LC_EUNSUPPORTED;
  }
  b.kmax = kmax_needed <= 16 ? 16 : kmax_needed <= 32 ? 32 : kmax_needed <= 64 ? 64 : 128;
  std::vector<OpRec> recs(std::max<size_t>(n_recs, 1));
  std::vector<uint64_t> pool(std::max<size_t>(n_pool, 1));
  std::vector<uint32_t> cs(std::max<size_t>(n_cs, 1));
  size_t pr = 0, pp = 0, pc = 0;
  for (size_t i = 0; i < hs.size(); ++i) {
    const History& h = *hs[i];
    for (const OpRec& r0 : h.recs) {
      OpRec r = r0;
      r.hash_off = (uint32_t)(r0.hash_off + pp);
      recs[pr++] = r;
    }
    for (uint32_t j = 0; j <= h.K && !h.chain_start.empty(); ++j) cs[pc++] = b.h_hist[i].rec_base + h.chain_start[j];
    if (h.chain_start.empty()) cs[pc++] = b.h_hist[i].rec_base;
    std::copy(h.pool.begin(), h.pool.end(), pool.begin() + pp);
    pp += h.pool.size();
  }
  // longest-first processing order (LPT): work ~ ops x chains; split into the
  // packed-group lists (K <= 16, K <= 32) and the rest (workgroup per history)
  std::vector<uint32_t> order;
  order.reserve(hs.size());
  for (uint32_t i = 0; i < hs.size(); ++i)
    if (!b.forced[i]) order.push_back(i);
  std::stable_sort(order.begin(), order.end(), [&](uint32_t x, uint32_t y) {
    return (uint64_t)b.h_hist[x].n_ops * b.h_hist[x].K > (uint64_t)b.h_hist[y].n_ops * b.h_hist[y].K;
  });
  {
    std::vector<uint32_t> l16, l32, rest;
    b.h_level.clear();
    // S2LC_LEVEL_ONLY=1 (tests): every history through the level search
    const char* lo = getenv("S2LC_LEVEL_ONLY");
    const bool level_only = lo && lo[0] == '1';
    for (uint32_t i : order) {
      const uint32_t K = b.h_hist[i].K;
      if (level_only) b.h_level.push_back(i);
      else (K <= 16 ? l16 : K <= 32 ? l32 : K <= 128 ? rest : b.h_level).push_back(i);
    }
    b.n_pack16 = (uint32_t)l16.size();
    b.in_pack16.assign(hs.size(), 0);
    for (uint32_t i : l16) b.in_pack16[i] = 1;
    b.n_pack32 = (uint32_t)l32.size();
    b.h_rest = rest;
    order = l16;
    order.insert(order.end(), l32.begin(), l32.end());
    order.insert(order.end(), rest.begin(), rest.end());
  }
  b.moves_cap = moves_total;
  b.n_recs = (uint32_t)recs.size();
  b.n_pool = (uint32_t)pool.size();
  HIPCHK(hipMalloc(&b.recs, recs.size() * sizeof(OpRec)));
  HIPCHK(hipMalloc(&b.pool, pool.size() * sizeof(uint64_t)));
  HIPCHK(hipMalloc(&b.chain_start, cs.size() * sizeof(uint32_t)));
  HIPCHK(hipMalloc(&b.hist, std::max<size_t>(hs.size(), 1) * sizeof(HistDesc)));
  HIPCHK(hipMalloc(&b.order, std::max<size_t>(order.size(), 1) * sizeof(uint32_t)));
  HIPCHK(hipMalloc(&b.res, std::max<size_t>(hs.size(), 1) * sizeof(HistResult)));
  HIPCHK(hipMalloc(&b.moves, std::max<uint64_t>(moves_total, 1) * sizeof(uint32_t)));
  HIPCHK(hipMalloc(&b.counter, 16 * sizeof(uint32_t)));
  HIPCHK(hipMalloc(&b.trace_head, sizeof(unsigned long long)));
  HIPCHK(hipMemcpy(b.recs, recs.data(), recs.size() * sizeof(OpRec), hipMemcpyHostToDevice));
  HIPCHK(hipMemcpy(b.pool, pool.data(), pool.size() * sizeof(uint64_t), hipMemcpyHostToDevice));
  HIPCHK(hipMemcpy(b.chain_start, cs.data(), cs.size() * sizeof(uint32_t), hipMemcpyHostToDevice));
  if (!hs.empty()) HIPCHK(hipMemcpy(b.hist, b.h_hist.data(), hs.size() * sizeof(HistDesc), hipMemcpyHostToDevice));
  if (!order.empty()) HIPCHK(hipMemcpy(b.order, order.data(), order.size() * sizeof(uint32_t), hipMemcpyHostToDevice));
  if (b.h_res_pinned) { (void)hipHostUnregister(b.h_res.data()); b.h_res_pinned = false; }
  b.h_res.assign(hs.size(), HistResult{});
  for (size_t i = 0; i < hs.size(); ++i) b.h_res[i].witness_off = b.h_moves_off[i];
  // every run reads the results back: page-lock them so that copy is a direct DMA
  if (!hs.empty() && hipHostRegister(b.h_res.data(), hs.size() * sizeof(HistResult), hipHostRegisterDefault) == hipSuccess)
    b.h_res_pinned = true;
  (void)hipGetLastError();  // a failed registration only costs the staged copy
  if (!hs.empty()) HIPCHK(hipMemcpy(b.res, b.h_res.data(), hs.size() * sizeof(HistResult), hipMemcpyHostToDevice));
  return 0;
}

void batch_release(DevBatch& b) {
  level_release(b);
  if (b.h_res_pinned) { (void)hipHostUnregister(b.h_res.data()); b.h_res_pinned = false; }
  void* ptrs[] = {b.recs, b.pool, b.chain_start, b.hist, b.order, b.res, b.moves, b.counter, b.trace, b.trace_head, b.slab};
  for (void* q : ptrs) if (q) (void)hipFree(q);
  b.recs = nullptr; b.pool = nullptr; b.chain_start = nullptr; b.hist = nullptr; b.order = nullptr;
  b.res = nullptr; b.moves = nullptr; b.counter = nullptr; b.trace = nullptr; b.trace_head = nullptr;
  b.slab = nullptr; b.slab_cap = 0; b.trace_cap = 0;
}

static int ensure(void** p, size_t& cap, size_t need, std::string& err) {
  if (need <= cap) return 0;
  if (*p) (void)hipFree(*p);
  *p = nullptr;
  cap = 0;
  HIPCHK(hipMalloc(p, need));
  cap = need;
  return 0;
}

int batch_run(DevBatch& b, hipStream_t stream, uint64_t max_configs, bool witness, RunStats& st, std::string& err) {
  st = RunStats{};
  auto t0 = std::chrono::steady_clock::now();
  int dev = 0;
  HIPCHK(hipGetDevice(&dev));
  int n_cu = 256;
  (void)hipDeviceGetAttribute(&n_cu, hipDeviceAttributeMultiprocessorCount, dev);

  // trace pool: generous, reused across runs
  if (witness && b.trace_cap == 0) {
    size_t free_b = 0, total_b = 0;
    HIPCHK(hipMemGetInfo(&free_b, &total_b));
    uint64_t want = std::min<uint64_t>(1ull << 28, (uint64_t)(free_b / 8) / sizeof(TraceEnt));
    want = std::min<uint64_t>(want, 0xFFFFFFF0ull);
    HIPCHK(hipMalloc(&b.trace, want * sizeof(TraceEnt)));
    b.trace_cap = want;
  }

  Params prm;
  memset(&prm, 0, sizeof prm);
  prm.recs = b.recs; prm.pool = b.pool; prm.chain_start = b.chain_start; prm.hist = b.hist;
  prm.trace = b.trace; prm.trace_head = b.trace_head; prm.trace_cap = witness ? b.trace_cap : 0;
  prm.res = b.res; prm.max_configs = max_configs; prm.witness = witness ? 1 : 0;
  prm.n_recs = b.n_recs; prm.n_pool = b.n_pool; prm.n_res = b.n_hist;

  hipEvent_t e0, e1;
  HIPCHK(hipEventCreate(&e0));
  HIPCHK(hipEventCreate(&e1));
  HIPCHK(hipMemsetAsync(b.counter, 0, 16 * sizeof(uint32_t), stream));
  HIPCHK(hipMemsetAsync(b.trace_head, 0, sizeof(unsigned long long), stream));

  // Packed passes: one L-lane group per history (K <= 16: L = 16, K <= 32:
  // L = 32), frontier <= PACK_F. Histories that outgrow that frontier, and
  // those with K > 32, go on to the workgroup-per-history passes:
  // Pass 0: LDS-resident search (small frontier / staging).
  // Pass 1: HBM slab, 64 lanes, frontier 1024, for the ones that outgrew LDS.
  // Pass 2: HBM slab, 256 lanes, frontier up to 2^20.
  // Pass 0 sizing: one wave per workgroup; the LDS budget per workgroup is
  // what the kernel's register occupancy allows (16 / 12 workgroups per CU for
  // KMAX 16 / 32), so LDS never limits residency below the register limit.
  const bool use_pack = getenv("S2LC_NO_PACK") == nullptr;
  // histories settled by pack_kernel<16> (roofline accounting of that kernel)
  std::vector<uint8_t> pack16_done(b.n_hist, 0);
  if (use_pack)
    for (uint32_t i = 0; i < b.n_hist; ++i) pack16_done[i] = b.in_pack16[i];
  std::vector<uint32_t> todo;  // histories for the workgroup-per-history passes
  if (use_pack) {
#ifdef S2LC_PROF
    {
      unsigned long long z[16] = {0};
      HIPCHK(hipMemcpyToSymbol(HIP_SYMBOL(g_prof), z, sizeof z));
    }
#endif
    // Both packed launches, then (witness on) the walk of the histories they
    // settled, then one results read-back: a batch that needs no other pass
    // (all of C4) costs a single host sync per run.
    hipEvent_t pe[4];
    for (hipEvent_t& e : pe) HIPCHK(hipEventCreate(&e));
    bool launched[2] = {false, false};
    for (int li = 0; li < 2; ++li) {
      const uint32_t n_l = li == 0 ? b.n_pack16 : b.n_pack32;
      if (n_l == 0) continue;
      Params pp = prm;
      pp.order = b.order + (li == 0 ? 0 : b.n_pack16);
      pp.n_hist = n_l;
      pp.counter = b.counter + 12 + li;
      const uint32_t L = li == 0 ? 16 : 32;
      const size_t smem = li == 0 ? pack_smem_bytes<16>() : pack_smem_bytes<32>();
      int bpc = 1;
      if (li == 0) HIPCHK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&bpc, pack_kernel<16>, PACK_BLOCK, smem));
      else HIPCHK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&bpc, pack_kernel<32>, PACK_BLOCK, smem));
      const uint32_t groups = PACK_BLOCK / L;
      const uint32_t grid = std::max<uint32_t>(
          1, std::min<uint32_t>((n_l + groups - 1) / groups, (uint32_t)n_cu * (uint32_t)std::max(1, bpc)));
      HIPCHK(hipEventRecord(pe[2 * li], stream));
      if (li == 0) hipLaunchKernelGGL(pack_kernel<16>, dim3(grid), dim3(PACK_BLOCK), smem, stream, pp);
      else hipLaunchKernelGGL(pack_kernel<32>, dim3(grid), dim3(PACK_BLOCK), smem, stream, pp);
      HIPCHK(hipGetLastError());
      HIPCHK(hipEventRecord(pe[2 * li + 1], stream));
      launched[li] = true;
      st.launches++;
    }
    if (b.n_pack16 + b.n_pack32) {
      if (witness) {
        hipLaunchKernelGGL(walk_kernel, dim3((b.n_hist + 255) / 256), dim3(256), 0, stream, b.n_hist, b.res,
                           (const TraceEnt*)b.trace, b.moves);
        HIPCHK(hipGetLastError());
      }
      HIPCHK(hipMemcpyAsync(b.h_res.data(), b.res, b.n_hist * sizeof(HistResult), hipMemcpyDeviceToHost, stream));
      HIPCHK(hipStreamSynchronize(stream));
    }
    for (int li = 0; li < 2; ++li) {
      if (!launched[li]) continue;
      float ms = 0;
      HIPCHK(hipEventElapsedTime(&ms, pe[2 * li], pe[2 * li + 1]));
      st.kernel_ms += ms;
      st.pack_ms += ms;
      if (li == 0) st.pack16_ms = ms;
    }
    for (hipEvent_t e : pe) (void)hipEventDestroy(e);
#ifdef S2LC_PROF
    {
      unsigned long long gp[16];
      HIPCHK(hipMemcpyFromSymbol(gp, HIP_SYMBOL(g_prof), sizeof gp));
      const double rd = gp[13] ? (double)gp[13] : 1.0;
      fprintf(stderr, "[s2lc prof] pack: rounds %llu children %llu | cycles/round expand %.0f closure %.0f dedupe+rest %.0f\n",
              gp[13], gp[15], gp[10] / rd, gp[11] / rd, gp[12] / rd);
    }
#endif
    for (uint32_t i = 0; i < b.n_hist; ++i)
      if (!b.forced[i] && b.h_hist[i].K <= 32 && b.h_res[i].verdict == V_UNKNOWN && b.h_res[i].reason == S2LC_R_FRONTIER)
        todo.push_back(i);
    st.n_overflow = (uint32_t)todo.size();
    for (uint32_t i : todo) pack16_done[i] = 0;
    todo.insert(todo.end(), b.h_rest.begin(), b.h_rest.end());
  } else {
    std::vector<uint32_t> all(b.n_pack16 + b.n_pack32 + b.h_rest.size());
    if (!all.empty()) HIPCHK(hipMemcpy(all.data(), b.order, all.size() * sizeof(uint32_t), hipMemcpyDeviceToHost));
    todo = all;
  }
  const uint32_t lds_fcap = 8;
  const uint32_t lds_stage = 32;
  const size_t lds_budget = b.kmax <= 16 ? 10240 : b.kmax <= 32 ? 13312 : 0;
  uint32_t* d_list = nullptr;
  int n_passes_run = 0;
  for (int pass = 0; pass < 2; ++pass) {
    uint32_t n_pass = (uint32_t)todo.size();
    if (n_pass == 0) break;
    ++n_passes_run;
    SearchGeom g;
    if (pass == 0) {
      g = make_geom(b.kmax, true, 64, lds_fcap, lds_stage, lds_stage, 1, lds_budget);
      const uint32_t per_cu = std::max<uint32_t>(1, std::min<uint32_t>(16, (uint32_t)((160 * 1024) / g.smem_bytes)));
      g.grid = std::max<uint32_t>(1, std::min<uint32_t>(n_pass, (uint32_t)n_cu * per_cu));
    } else {
      g = make_geom(b.kmax, false, 64, 1024, 512, 256, 1, 0);
      g.grid = std::max<uint32_t>(1, std::min<uint32_t>(n_pass, (uint32_t)n_cu * 16));
    }
    if (!g.shared && ensure((void**)&b.slab, b.slab_cap, g.slab_bytes * g.grid, err)) return S2LC_EHIP;
    Params pp = prm;
    if (d_list) (void)hipFree(d_list);
    d_list = nullptr;
    HIPCHK(hipMalloc(&d_list, todo.size() * sizeof(uint32_t)));
    HIPCHK(hipMemcpyAsync(d_list, todo.data(), todo.size() * sizeof(uint32_t), hipMemcpyHostToDevice, stream));
    pp.order = d_list;
    pp.n_hist = n_pass;
    pp.counter = b.counter + 4 * pass;
    pp.slab = b.slab;
    pp.slab_bytes = g.slab_bytes;
    pp.fcap = g.fcap; pp.chunk = g.chunk; pp.stage_cap = g.stage_cap; pp.ht_mask = g.ht_slots - 1;
    pp.win_recs = g.win_recs;
#ifdef S2LC_GUARD
    {
      uint32_t z[8] = {0};
      HIPCHK(hipMemcpyToSymbol(HIP_SYMBOL(g_guard), z, sizeof z));
    }
#endif
#ifdef S2LC_PROF
    {
      unsigned long long z[16] = {0};
      HIPCHK(hipMemcpyToSymbol(HIP_SYMBOL(g_prof), z, sizeof z));
    }
#endif
    HIPCHK(hipEventRecord(e0, stream));
    HIPCHK(launch_geom(g, pp, stream));
    HIPCHK(hipEventRecord(e1, stream));
    st.launches++;
    HIPCHK(hipMemcpyAsync(b.h_res.data(), b.res, b.n_hist * sizeof(HistResult), hipMemcpyDeviceToHost, stream));
    HIPCHK(hipStreamSynchronize(stream));
#ifdef S2LC_GUARD
    {
      uint32_t gg[8];
      HIPCHK(hipMemcpyFromSymbol(gg, HIP_SYMBOL(g_guard), sizeof gg));
      if (gg[0]) {
        err = "guard: " + std::to_string(gg[0]) + " violations, first at search_dev.h:" + std::to_string(gg[1]) +
              " a=" + std::to_string(gg[2]) + " b=" + std::to_string(gg[3]);
        return S2LC_EHIP;
      }
    }
#endif
    float ms = 0;
    HIPCHK(hipEventElapsedTime(&ms, e0, e1));
#ifdef S2LC_PROF
    {
      unsigned long long gp[16];
      HIPCHK(hipMemcpyFromSymbol(gp, HIP_SYMBOL(g_prof), sizeof gp));
      const double rounds = gp[8] ? (double)gp[8] : 1.0;
      fprintf(stderr,
              "[s2lc prof] pass %d kmax %d hist %u ms %.3f rounds %llu | cycles/round setup %.0f expand %.0f close %.0f "
              "dedupe %.0f compact %.0f finalize %.0f | closure passes/call %.2f calls/round %.2f | refills/round %.3f "
              "win_recs %u smem %zu grid %u\n",
              pass, g.kmax, n_pass, ms, gp[8], gp[0] / rounds, gp[1] / rounds, gp[2] / rounds, gp[3] / rounds,
              gp[4] / rounds, gp[5] / rounds, gp[7] ? (double)gp[6] / gp[7] : 0.0, gp[7] / rounds, gp[9] / rounds,
              g.win_recs, g.smem_bytes, g.grid);
    }
#endif
    st.kernel_ms += ms;
    if (pass == 0) st.pass0_ms = ms;
    // histories that outgrew this pass's frontier go to the next pass
    std::vector<uint32_t> next;
    for (uint32_t i = 0; i < b.n_hist; ++i)
      if (!b.forced[i] && b.h_res[i].verdict == V_UNKNOWN && b.h_res[i].reason == S2LC_R_FRONTIER) next.push_back(i);
    if (pass == 0) st.n_overflow += (uint32_t)next.size();
    else st.n_overflow2 += (uint32_t)next.size();
    todo.swap(next);
  }
  if (d_list) (void)hipFree(d_list);
  // Pass 2: the device-wide level search, one history at a time: histories
  // with more than 128 chains and those whose frontier outgrew pass 1.
  todo.insert(todo.end(), b.h_level.begin(), b.h_level.end());
  for (uint32_t h : todo) {
    const int rc = level_search(b, h, stream, max_configs, witness, st.level, err);
    if (rc) return rc;
  }
  st.kernel_ms += st.level.ms;
  // the packed histories were walked with the packed launches; walk again only
  // for what the other passes settled (walk_kernel skips walked histories)
  const bool other_work = !use_pack || n_passes_run > 0 || !todo.empty();
  if (witness && b.n_hist && other_work) {
    hipLaunchKernelGGL(walk_kernel, dim3((b.n_hist + 255) / 256), dim3(256), 0, stream, b.n_hist, b.res,
                       (const TraceEnt*)b.trace, b.moves);
    HIPCHK(hipGetLastError());
    HIPCHK(hipMemcpyAsync(b.h_res.data(), b.res, b.n_hist * sizeof(HistResult), hipMemcpyDeviceToHost, stream));
    HIPCHK(hipStreamSynchronize(stream));
  }
  HIPCHK(hipEventDestroy(e0));
  HIPCHK(hipEventDestroy(e1));
  for (uint32_t i = 0; i < b.n_hist; ++i) {
    if (b.forced[i]) {
      b.h_res[i] = HistResult{};
      b.h_res[i].verdict = V_ILLEGAL;
      b.h_res[i].reason = S2LC_R_UNMATCHED;
      b.h_res[i].witness_off = b.h_moves_off[i];
      continue;
    }
    const HistResult& r = b.h_res[i];
    st.configs += r.configs;
    st.children += r.children;
    st.rounds += r.rounds;
    const uint64_t S = 8 * ((2 * (uint64_t)b.h_hist[i].K + 20 + 7) / 8);
    st.algo_bytes += 2 * S * r.configs + 8 * r.children;
    if (pack16_done[i]) {
      // pack_kernel<16> alone: its histories' search bytes + their input SoA
      st.pack16_algo_bytes += 2 * S * r.configs + 8 * r.children + b.h_in_bytes[i];
      st.pack16_histories++;
    }
  }
  st.algo_bytes += b.algo_bytes_inputs;
  st.total_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
  return 0;
}

}  // namespace s2lc
