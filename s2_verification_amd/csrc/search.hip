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
#include <hip/hip_ext.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <chrono>
#include <memory>
#include <thread>
#include <numeric>
#include <string>

#include "s2lincheck.h"
#include "search.h"
#include "host_par.h"
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

int64_t steady_ns() {
  return std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now().time_since_epoch())
      .count();
}

namespace {

size_t align256(size_t x) { return (x + 255) & ~(size_t)255; }

// Grow-only device / pinned-host buffers (a context's scratch batch is reused
// by every s2lc_check, so steady-state calls allocate nothing).
int grow_device(uint8_t** p, size_t& cap, size_t need, std::string& err) {
  if (need <= cap && *p) return 0;
  if (*p) (void)hipFree(*p);
  *p = nullptr;
  cap = 0;
  const size_t want = std::max<size_t>(need + need / 4, 1 << 16);
  HIPCHK(hipMalloc(p, want));
  cap = want;
  return 0;
}

int grow_pinned(uint8_t** p, size_t& cap, size_t need, std::string& err) {
  if (need <= cap && *p) return 0;
  if (*p) (void)hipHostFree(*p);
  *p = nullptr;
  cap = 0;
  const size_t want = std::max<size_t>(need + need / 4, 1 << 16);
  HIPCHK(hipHostMalloc(p, want, hipHostMallocDefault));
  cap = want;
  return 0;
}

// The 64-byte records of the H_SMALL histories, from their uploaded SRec
// (search.h from_srec): one block per history at a time
__global__ void widen_kernel(const HistDesc* __restrict__ hist, const SRec* __restrict__ in, OpRec* __restrict__ out,
                             uint32_t n_hist, uint32_t n_recs) {
  for (uint32_t i = blockIdx.x; i < n_hist; i += gridDim.x) {
    const HistDesc d = hist[i];
    if (!(d.flags & H_SMALL)) continue;
    const uint32_t end = i + 1 < n_hist ? hist[i + 1].rec_base : n_recs;
    for (uint32_t r = d.rec_base + threadIdx.x; r < end; r += blockDim.x) {
      const uint4* q = reinterpret_cast<const uint4*>(in + r);
      SRec y;
      uint4 w[2] = {q[0], q[1]};
      __builtin_memcpy(&y, w, sizeof(SRec));
      const OpRec x = from_srec(y);
      uint4 o[4];
      __builtin_memcpy(o, &x, sizeof(OpRec));
      uint4* dst = reinterpret_cast<uint4*>(out + r);
#pragma unroll
      for (int k = 0; k < 4; ++k) dst[k] = o[k];
    }
  }
}

}  // namespace

int batch_upload(DevBatch& b, const std::vector<const History*>& hs, uint32_t red_off, std::string& err) {
  const uint16_t clear = (uint16_t)(((red_off & S2LC_RED_P1) ? H_NOWRAP : 0) | ((red_off & S2LC_RED_P2) ? H_P2OK : 0) |
                                    ((red_off & S2LC_RED_P4) ? H_P4 : 0) | ((red_off & S2LC_RED_IDEFER) ? H_IDEFER : 0));
  const size_t n = hs.size();
  b.n_hist = (uint32_t)n;
  b.src = hs;
  b.forced.assign(n, 0);
  b.literal.assign(n, 0);
  b.lit_desc.clear();
  b.lit_ev.clear();
  b.lit_dev_ready = false;
  b.rc_valid = false;
  b.route_valid = false;
  uint32_t kmax_needed = 1;
  size_t n_recs = 0, n_pool = 0, n_cs = 0;
  uint64_t moves_total = 0;
  b.h_moves_off.resize(n);
  b.h_in_bytes.assign(n, 0);
  b.algo_bytes_inputs = 0;
  // per-history offsets into the batch arrays (a sequential prefix pass; the
  // packing below runs in parallel from them)
  std::vector<size_t> off_rec(n), off_pool(n), off_cs(n);
  for (size_t i = 0; i < n; ++i) {
    const History& h = *hs[i];
    if (h.status != 0) { err = "history " + std::to_string(i) + ": " + h.error; return h.status; }
    if (h.structural) b.forced[i] = 1;
    if (h.literal) b.literal[i] = 1;
    if (h.K > LEVEL_KMAX) { err = "history has more than 512 concurrent chains"; return S2LC_EUNSUPPORTED; }
    if (h.max_chain_len >= 0xFFFF) { err = "chain longer than 65534 ops"; return S2LC_EUNSUPPORTED; }
    if (h.K <= 128) kmax_needed = std::max(kmax_needed, h.K);
    off_rec[i] = n_recs;
    off_pool[i] = n_pool;
    off_cs[i] = n_cs;
    n_recs += h.recs.size();
    n_cs += h.chain_start.empty() ? 1 : h.K + 1;
    n_pool += h.pool.size();
    b.h_moves_off[i] = (uint32_t)moves_total;
    moves_total += h.n_ops + 1;
  }
  b.n_ops_total = moves_total - n;
  if (n_recs >= 0xFFFFFFFFull || n_pool >= 0xFFFFFFFFull || moves_total >= 0xFFFFFFFFull) {
    err = "batch too large for 32-bit indices";
    return S2LC_EUNSUPPORTED;
  }
  b.kmax = kmax_needed <= 16 ? 16 : kmax_needed <= 32 ? 32 : kmax_needed <= 64 ? 64 : 128;
  b.moves_cap = moves_total;
  b.n_recs = (uint32_t)std::max<size_t>(n_recs, 1);
  b.n_pool = (uint32_t)std::max<size_t>(n_pool, 1);
  // layout (stage = the uploaded prefix of the arena)
  const size_t o_recs = 0;
  const size_t o_srec = align256(o_recs + b.n_recs * sizeof(OpRec));
  const size_t o_pool = align256(o_srec + (size_t)b.n_recs * sizeof(SRec));
  const size_t o_cs = align256(o_pool + b.n_pool * sizeof(uint64_t));
  const size_t o_hist = align256(o_cs + std::max<size_t>(n_cs, 1) * sizeof(uint32_t));
  const size_t o_order = align256(o_hist + std::max<size_t>(n, 1) * sizeof(HistDesc));
  const size_t o_res = align256(o_order + std::max<size_t>(n, 1) * sizeof(uint32_t));
  const size_t stage_bytes = align256(o_res + std::max<size_t>(n, 1) * sizeof(HistResult));
  const size_t o_moves = stage_bytes;
  const size_t o_rc = align256(o_moves + std::max<uint64_t>(moves_total, 1) * sizeof(uint32_t));
  const size_t o_list = align256(o_rc + std::max<uint64_t>(moves_total, 1) * sizeof(uint32_t));
  const size_t arena_bytes = align256(o_list + std::max<size_t>(n, 1) * sizeof(uint32_t));
  if (grow_pinned(&b.stage, b.stage_cap, stage_bytes, err)) return S2LC_EHIP;
  if (grow_device(&b.arena, b.arena_cap, arena_bytes, err)) return S2LC_EHIP;
  OpRec* s_recs = reinterpret_cast<OpRec*>(b.stage + o_recs);
  SRec* s_srecs = reinterpret_cast<SRec*>(b.stage + o_srec);
  uint64_t* s_pool = reinterpret_cast<uint64_t*>(b.stage + o_pool);
  uint32_t* s_cs = reinterpret_cast<uint32_t*>(b.stage + o_cs);
  b.h_hist = reinterpret_cast<HistDesc*>(b.stage + o_hist);
  uint32_t* s_order = reinterpret_cast<uint32_t*>(b.stage + o_order);
  b.h_res = reinterpret_cast<HistResult*>(b.stage + o_res);
  b.recs = reinterpret_cast<OpRec*>(b.arena + o_recs);
  b.pool = reinterpret_cast<uint64_t*>(b.arena + o_pool);
  b.chain_start = reinterpret_cast<uint32_t*>(b.arena + o_cs);
  b.hist = reinterpret_cast<HistDesc*>(b.arena + o_hist);
  b.order = reinterpret_cast<uint32_t*>(b.arena + o_order);
  b.res = reinterpret_cast<HistResult*>(b.arena + o_res);
  b.moves = reinterpret_cast<uint32_t*>(b.arena + o_moves);
  b.rcounts = reinterpret_cast<uint32_t*>(b.arena + o_rc);
  b.list = reinterpret_cast<uint32_t*>(b.arena + o_list);
  b.srecs = reinterpret_cast<SRec*>(b.arena + o_srec);
  std::atomic<uint32_t> n_small{0};
  // Pack every history into the pinned stage (in parallel: ~0.5 GB for C4).
  // The records and the hash pool (nearly all of the stage) go up in slices
  // of histories as the slices complete: this thread queues each slice's two
  // ranges (async from pinned memory) while the packer threads fill the next,
  // so the DMA overlaps the packing; the small sections follow at the end.
  const size_t n_sl = n >= 2048 ? 16 : 1;
  const size_t sl_len = (n + n_sl - 1) / std::max<size_t>(n_sl, 1);
  std::unique_ptr<std::atomic<uint32_t>[]> sl_left(new std::atomic<uint32_t>[n_sl]);
  // per slice: histories packed as SRec / as OpRec (which record ranges go up)
  std::unique_ptr<std::atomic<uint32_t>[]> sl_small(new std::atomic<uint32_t>[n_sl]);
  std::unique_ptr<std::atomic<uint32_t>[]> sl_big(new std::atomic<uint32_t>[n_sl]);
  for (size_t k = 0; k < n_sl; ++k) {
    sl_left[k] = (uint32_t)(std::min(n, (k + 1) * sl_len) - std::min(n, k * sl_len));
    sl_small[k] = 0;
    sl_big[k] = 0;
  }
  // S2LC_PACK_SMALL=0: every history as OpRec, the packed kernels' 64-byte instances
  const bool small_on = !(getenv("S2LC_PACK_SMALL") && getenv("S2LC_PACK_SMALL")[0] == '0');
  auto pack_one = [&](size_t i) {
    const History& h = *hs[i];
    HistDesc& d = b.h_hist[i];
    size_t pr = off_rec[i], pc = off_cs[i];
    const size_t pp = off_pool[i];
    d.rec_base = (uint32_t)pr;
    d.cs_base = (uint32_t)pc;
    d.K = (uint16_t)h.K;
    d.flags = (uint16_t)(h.hflags & ~clear);
    d.n_ops = h.n_ops;
    uint64_t in_bytes = 48ull * h.n_ops;
    uint64_t tot_nr = 0;  // every reachable tail is at most the sum of the appends' num_records
    uint32_t max_hc = 0;
    for (const OpRec& r0 : h.recs) {
      in_bytes += 8ull * r0.hash_cnt;
      if (!(r0.flags & OPF_SENTINEL) && (r0.flags & OPF_KIND_MASK) == S2LC_INPUT_APPEND)
        tot_nr += std::min<uint64_t>(r0.num_records, 1ull << 32);
      max_hc = std::max(max_hc, r0.hash_cnt);
    }
    // the 32-byte records (SRec) are exact for this history: packed and
    // uploaded as such (widened on the device), else as OpRec
    if (small_on && (d.flags & H_TAIL32) && !h.literal && !h.structural && h.n_events() < 0xFFFFu &&
        tot_nr <= 65532u && max_hc <= 0xFFFFu) {
      d.flags |= H_SMALL;
      n_small.fetch_add(1, std::memory_order_relaxed);
      sl_small[i / sl_len].store(1, std::memory_order_relaxed);
      for (const OpRec& r0 : h.recs) {
        SRec y = to_srec(r0);
        y.hash_off = (uint32_t)(r0.hash_off + pp);
        s_srecs[pr++] = y;
      }
    } else {
      sl_big[i / sl_len].store(1, std::memory_order_relaxed);
      for (const OpRec& r0 : h.recs) {
        OpRec r = r0;
        r.hash_off = (uint32_t)(r0.hash_off + pp);
        s_recs[pr++] = r;
      }
    }
    b.h_in_bytes[i] = in_bytes;
    if (h.chain_start.empty()) s_cs[pc++] = d.rec_base;
    else for (uint32_t j = 0; j <= h.K; ++j) s_cs[pc++] = d.rec_base + h.chain_start[j];
    if (!h.pool.empty()) memcpy(s_pool + pp, h.pool.data(), h.pool.size() * sizeof(uint64_t));
    HistResult& R = b.h_res[i];
    R = HistResult{};
    R.verdict = V_UNKNOWN;
    R.witness_off = b.h_moves_off[i];
    sl_left[i / sl_len].fetch_sub(1, std::memory_order_release);
  };
  if (n_sl == 1) {
    parallel_for(n, 64, pack_one);
  } else {
    std::thread packer([&]() { parallel_for(n, 64, pack_one); });
    hipError_t ce = hipSuccess;
    for (size_t k = 0; k < n_sl; ++k) {
      while (sl_left[k].load(std::memory_order_acquire) != 0) std::this_thread::yield();
      const size_t i0 = k * sl_len, i1 = std::min(n, (k + 1) * sl_len);
      if (i0 >= i1 || ce != hipSuccess) continue;
      const size_t r0 = off_rec[i0], r1 = i1 < n ? off_rec[i1] : n_recs;
      const size_t p0 = off_pool[i0], p1 = i1 < n ? off_pool[i1] : n_pool;
      if (r1 > r0 && sl_big[k].load(std::memory_order_relaxed))
        ce = hipMemcpyAsync(b.arena + o_recs + r0 * sizeof(OpRec), b.stage + o_recs + r0 * sizeof(OpRec),
                            (r1 - r0) * sizeof(OpRec), hipMemcpyHostToDevice, 0);
      if (ce == hipSuccess && r1 > r0 && sl_small[k].load(std::memory_order_relaxed))
        ce = hipMemcpyAsync(b.arena + o_srec + r0 * sizeof(SRec), b.stage + o_srec + r0 * sizeof(SRec),
                            (r1 - r0) * sizeof(SRec), hipMemcpyHostToDevice, 0);
      if (ce == hipSuccess && p1 > p0)
        ce = hipMemcpyAsync(b.arena + o_pool + p0 * sizeof(uint64_t), b.stage + o_pool + p0 * sizeof(uint64_t),
                            (p1 - p0) * sizeof(uint64_t), hipMemcpyHostToDevice, 0);
    }
    packer.join();
    HIPCHK(ce);
  }
  for (size_t i = 0; i < n; ++i) b.algo_bytes_inputs += b.h_in_bytes[i];
  for (size_t i = 0; i < n; ++i)
    if (b.literal[i]) literal_prepare(*hs[i], (uint32_t)i, off_pool[i], b.lit_desc, b.lit_ev);
  // LPT order, longest first. A history's search runs one round per
  // non-identity op it linearizes (appends: n_ops - n_ident), a dependent
  // chain whatever the engine, so that count leads the key; n_ops x K breaks
  // ties (a round's width). On C4 this order ends the packed launch 16 %
  // sooner than n_ops x K alone, which ties every history with the same
  // client count (tools/pack_sweep.py).
  b.lpt.clear();
  std::vector<uint64_t> key(n, 0);
  for (uint32_t i = 0; i < n; ++i) {
    if (b.forced[i] || b.literal[i]) continue;
    b.lpt.push_back(i);
    const History& h = *hs[i];
    key[i] = ((uint64_t)(h.n_ops - h.n_ident) << 40) | ((uint64_t)h.n_ops * h.K & ((1ull << 40) - 1));
  }
  std::stable_sort(b.lpt.begin(), b.lpt.end(), [&](uint32_t x, uint32_t y) { return key[x] > key[y]; });
  // the packed-kernel lists (engine AUTO): K <= 16, 16 < K <= 32, and with
  // S2LC_PACK8=1 the K <= 8 histories in 8-lane groups first. Off by default:
  // at C4's 10k histories a launch lasts about one history's chain of rounds
  // (~2.3 ms either way), and the 8-lane launch runs before the
  // 16-lane one for the rest; 8-lane groups pay off only on batches several
  // times larger (twice the histories per wave).
  const char* e8 = getenv("S2LC_PACK8");
  const uint32_t k8 = (e8 && e8[0] == '1') ? 8u : 0u;
  // S2LC_PACK32_TOP=n (diagnostics): the n longest K <= 16 histories run in
  // 32-lane groups (two histories per wave instead of four)
  const char* e32 = getenv("S2LC_PACK32_TOP");
  const uint32_t top32 = e32 ? (uint32_t)strtoul(e32, nullptr, 10) : 0u;
  std::vector<uint8_t> to32(n, 0);
  {
    uint32_t c = 0;
    for (uint32_t i : b.lpt)
      if (c < top32 && b.h_hist[i].K > k8 && b.h_hist[i].K <= 16) { to32[i] = 1; ++c; }
  }
  b.pack8_kmax = k8;
  // (the packed kernels keep tail bounds in 32 bits: histories whose tails
  // can pass 2^32 take the workgroup engine)
  auto t32 = [&](uint32_t i) { return (b.h_hist[i].flags & H_TAIL32) != 0; };
  uint32_t no = 0;
  for (uint32_t i : b.lpt) if (b.h_hist[i].K <= k8 && t32(i)) s_order[no++] = i;
  b.n_pack8 = no;
  for (uint32_t i : b.lpt) if (b.h_hist[i].K > k8 && b.h_hist[i].K <= 16 && !to32[i] && t32(i)) s_order[no++] = i;
  b.n_pack16 = no - b.n_pack8;
  for (uint32_t i : b.lpt) if (((b.h_hist[i].K > 16 && b.h_hist[i].K <= 32) || to32[i]) && t32(i)) s_order[no++] = i;
  b.n_pack32 = no - b.n_pack8 - b.n_pack16;
  {
    const uint32_t lim[3] = {b.n_pack8, b.n_pack8 + b.n_pack16, no};
    uint32_t k = 0;
    for (int li = 0; li < 3; ++li) {
      b.in_bytes_list[li] = 0;
      bool all_small = k < lim[li];
      for (; k < lim[li]; ++k) {
        b.in_bytes_list[li] += b.h_in_bytes[s_order[k]];
        all_small = all_small && (b.h_hist[s_order[k]].flags & H_SMALL);
      }
      b.list_small[li] = all_small;
    }
  }
  b.h_res_stale = false;
  if (n_sl == 1) {
    // only the record region(s) this batch filled (64-byte OpRec, 32-byte
    // SRec, or both), then the pool and the small sections (the
    // whole stage had gone up, both record regions included)
    if (n_recs && sl_big[0].load(std::memory_order_relaxed))
      HIPCHK(hipMemcpyAsync(b.arena + o_recs, b.stage + o_recs, n_recs * sizeof(OpRec), hipMemcpyHostToDevice, 0));
    if (n_recs && sl_small[0].load(std::memory_order_relaxed))
      HIPCHK(hipMemcpyAsync(b.arena + o_srec, b.stage + o_srec, n_recs * sizeof(SRec), hipMemcpyHostToDevice, 0));
    HIPCHK(hipMemcpyAsync(b.arena + o_pool, b.stage + o_pool, stage_bytes - o_pool, hipMemcpyHostToDevice, 0));
  } else {  // the rest of the stage after the records and the pool, then wait for every slice
    HIPCHK(hipMemcpyAsync(b.arena + o_cs, b.stage + o_cs, stage_bytes - o_cs, hipMemcpyHostToDevice, 0));
  }
  // the 64-byte records of the H_SMALL histories, from their uploaded SRec
  if (n_small.load() > 0) {
    hipLaunchKernelGGL(widen_kernel, dim3((uint32_t)std::min<size_t>(n, 4096)), dim3(256), 0, 0, b.hist, b.srecs,
                       b.recs, (uint32_t)n, (uint32_t)n_recs);
    HIPCHK(hipGetLastError());
  }
  HIPCHK(hipStreamSynchronize(0));
  return 0;
}

void batch_release(DevBatch& b) {
  level_release(b);
  literal_release(b);
  if (b.agg) (void)hipFree(b.agg);
  if (b.h_agg) (void)hipHostFree(b.h_agg);
  b.agg = nullptr;
  b.h_agg = nullptr;
  void* dptrs[] = {b.arena, b.counter, b.trace, b.slab};  // trace_head lives inside counter
  for (void* q : dptrs) if (q) (void)hipFree(q);
  if (b.stage) (void)hipHostFree(b.stage);
  if (b.h_moves) (void)hipHostFree(b.h_moves);
  for (hipEvent_t& e : b.ev) {
    if (e) (void)hipEventDestroy(e);
    e = nullptr;
  }
  b.arena = nullptr; b.arena_cap = 0; b.stage = nullptr; b.stage_cap = 0;
  b.h_moves = nullptr; b.h_moves_cap = 0;
  b.recs = nullptr; b.pool = nullptr; b.chain_start = nullptr; b.hist = nullptr; b.order = nullptr;
  b.res = nullptr; b.moves = nullptr; b.rcounts = nullptr; b.list = nullptr; b.h_hist = nullptr; b.h_res = nullptr;
  b.counter = nullptr; b.trace = nullptr; b.trace_head = nullptr; b.trace_cap = 0;
  b.slab = nullptr; b.slab_cap = 0;
}

// Wait for the stream. S2LC_SYNC=spin polls an event recorded at its end
// instead of the blocking hipStreamSynchronize (measured on C4: the blocking
// wait returns ~23 us after the kernel; polling made the next step's enqueue
// 200 us slower, so blocking is the default).
static hipError_t stream_wait(hipStream_t stream, hipEvent_t ev) {
  static const int mode = [] {
    const char* e = getenv("S2LC_SYNC");
    return e && !strcmp(e, "spin") ? 0 : 1;
  }();
  if (mode == 0 && ev) {
    hipError_t e = hipEventRecord(ev, stream);
    if (e != hipSuccess) return e;
    while ((e = hipEventQuery(ev)) == hipErrorNotReady) {
    }
    if (e != hipSuccess) return e;
  }
  return hipStreamSynchronize(stream);
}

int batch_run(DevBatch& b, hipStream_t stream, const RunOpts& ro, RunStats& st, std::string& err) {
  st = RunStats{};
  const int64_t t0 = steady_ns();
  static const bool step_timing = getenv("S2LC_STEP_TIMING") != nullptr;
  int64_t t_enq = 0, t_wait = 0, t_ev = 0, t_over = 0, t_tail = 0;
  const int64_t deadline_ns = ro.timeout_us ? t0 + (int64_t)std::min<uint64_t>(ro.timeout_us, 1ull << 40) * 1000 : 0;
  const bool witness = ro.witness;
  int dev = 0;
  HIPCHK(hipGetDevice(&dev));
  if (b.route_dev != dev) {
    b.route_n_cu = 256;
    (void)hipDeviceGetAttribute(&b.route_n_cu, hipDeviceAttributeMultiprocessorCount, dev);
    b.route_dev = dev;
  }
  const int n_cu = b.route_n_cu;
  b.rc_valid = false;

  // Counters, by run parity: [0..15] work counters, [16..17] deadline,
  // [24..25] trace head; the packed totals likewise. A run zeroes the other
  // parity's set for the next run: in the reset dispatch, or (a batch every
  // history of which the packed kernels settle) in the first packed launch,
  // so that such a run needs no dispatch before its search.
  if (!b.counter) {
    HIPCHK(hipMalloc(&b.counter, 64 * sizeof(uint32_t)));
    HIPCHK(hipMemsetAsync(b.counter, 0, 64 * sizeof(uint32_t), stream));  // (on the stream: the
    // null stream does not order a non-blocking one, and a run that needs no reset dispatch reads these first)
  }
  if (!b.agg) {
    HIPCHK(hipMalloc(&b.agg, 64 * sizeof(unsigned long long)));
    HIPCHK(hipMemsetAsync(b.agg, 0, 64 * sizeof(unsigned long long), stream));
    HIPCHK(hipHostMalloc(&b.h_agg, 32 * sizeof(unsigned long long), hipHostMallocDefault));
  }
  const uint32_t par = b.run_par;
  b.run_par ^= 1u;
  uint32_t* const ctr = b.counter + 32 * par;
  unsigned long long* const agg = b.agg + 32 * par;
  b.trace_head = reinterpret_cast<unsigned long long*>(ctr + 24);
  for (hipEvent_t& e : b.ev)
    if (!e) HIPCHK(hipEventCreate(&e));
  // trace pool: generous, allocated once per batch and reused across runs
  if (witness && b.trace_cap == 0) {
    size_t free_b = 0, total_b = 0;
    HIPCHK(hipMemGetInfo(&free_b, &total_b));
    uint64_t want = std::min<uint64_t>(1ull << 28, (uint64_t)(free_b / 8) / sizeof(TraceEnt));
    want = std::min<uint64_t>(want, 0xFFFFFFF0ull);
    HIPCHK(hipMalloc(&b.trace, want * sizeof(TraceEnt)));
    b.trace_cap = want;
  }

  // engine routing; the environment overrides the context (diagnostics)
  uint32_t engine = ro.engine;
  {
    const char* lo = getenv("S2LC_LEVEL_ONLY");
    const char* np = getenv("S2LC_NO_PACK");
    if (lo && lo[0] == '1') engine = S2LC_ENGINE_LEVEL;
    else if (np && np[0] == '1' && engine == S2LC_ENGINE_AUTO) engine = S2LC_ENGINE_WORKGROUP;
  }

  Params prm;
  memset(&prm, 0, sizeof prm);
  prm.recs = b.recs; prm.srecs = b.srecs; prm.pool = b.pool; prm.chain_start = b.chain_start; prm.hist = b.hist;
  prm.trace = b.trace; prm.trace_head = b.trace_head; prm.trace_cap = witness ? b.trace_cap : 0;
  prm.res = b.res; prm.max_configs = ro.max_configs; prm.witness = witness ? 1 : 0;
  prm.moves = b.moves;
  prm.n_recs = b.n_recs; prm.n_pool = b.n_pool; prm.n_res = b.n_hist;
  prm.rcounts = ro.round_counts ? b.rcounts : nullptr;

  b.h_res_stale = false;
  // Every history settled by the packed kernels (they write all of their
  // results) or fixed on the host: no reset dispatch; the first packed launch
  // zeroes the next run's counters. Otherwise one dispatch resets the
  // results and zeroes both counter sets.
  uint32_t midk_level_max = 8;
  if (const char* e = getenv("S2LC_MIDK_LEVEL_MAX")) midk_level_max = (uint32_t)strtoul(e, nullptr, 10);
  if (!b.route_valid || b.route_engine != engine || b.route_midk_max != midk_level_max) {
    // the histories of each engine, LPT order
    b.route_todo.clear();   // workgroup passes
    b.route_level.clear();  // device-wide level search
    b.route_n_forced = 0;
    for (uint32_t i = 0; i < b.n_hist; ++i) b.route_n_forced += b.forced[i] ? 1u : 0u;
    const bool use_pack_r = engine == S2LC_ENGINE_AUTO;
    // A few histories with 32 < K <= 128 go to the level search too: one
    // workgroup per history (search_kernel) pays every round's latency in one
    // workgroup, while the level search runs each round on the whole device
    // (H96: 182 ms against 14 ms); a batch of many of them keeps the workgroup
    // engine, which checks them side by side. S2LC_MIDK_LEVEL_MAX overrides
    // the count (default 8).
    uint32_t n_midk = 0;
    for (uint32_t i : b.lpt)
      if (b.h_hist[i].K > 32 && b.h_hist[i].K <= 128) ++n_midk;
    const bool midk_level = engine == S2LC_ENGINE_AUTO && n_midk <= midk_level_max;
    for (uint32_t i : b.lpt) {
      const uint32_t K = b.h_hist[i].K;
      if (engine == S2LC_ENGINE_LEVEL || K > 128 || (midk_level && K > 32)) b.route_level.push_back(i);
      else if (!use_pack_r || K > 32 || !(b.h_hist[i].flags & H_TAIL32)) b.route_todo.push_back(i);
    }
    b.route_engine = engine;
    b.route_midk_max = midk_level_max;
    b.route_valid = true;
  }
  const uint32_t n_forced = b.route_n_forced;
  const uint32_t n_packed_all = b.n_pack8 + b.n_pack16 + b.n_pack32;
  // (force_reset: a run that flipped the parity but returned before it had
  // enqueued the zeroing of the other set leaves that set unzeroed)
  const bool no_reset = engine == S2LC_ENGINE_AUTO && b.lit_desc.empty() && !ro.round_counts && !deadline_ns &&
                        !b.force_reset &&
                        n_packed_all > 0 && n_packed_all + n_forced == b.n_hist && !getenv("S2LC_RESET_ALWAYS");
  if (!no_reset) {
    b.force_reset = true;
    hipLaunchKernelGGL(reset_results_kernel, dim3(std::max<uint32_t>(1, (b.n_hist + 255) / 256)), dim3(256), 0,
                       stream, b.res, b.n_hist, b.counter, b.agg);
    HIPCHK(hipGetLastError());
    b.force_reset = false;
  } else {
    b.force_reset = true;  // until the first packed launch (it zeroes the next run's set) is enqueued
  }
  if (deadline_ns) {
    int rate_khz = 100000;  // device wall clock (s_memrealtime); 100 MHz on gfx950
    (void)hipDeviceGetAttribute(&rate_khz, hipDeviceAttributeWallClockRate, dev);
    const int64_t left_ns = std::max<int64_t>(0, deadline_ns - steady_ns());
    const unsigned long long ticks = (unsigned long long)((double)left_ns * 1e-6 * rate_khz);
    unsigned long long* d = reinterpret_cast<unsigned long long*>(ctr + 16);
    hipLaunchKernelGGL(deadline_kernel, dim3(1), dim3(1), 0, stream, d, std::max<unsigned long long>(ticks, 1));
    HIPCHK(hipGetLastError());
    prm.deadline = d;
  }

  // duplicate-id histories: porcupine's own search (literal.hip), first on
  // the stream, so every later read-back of the results includes them
  if (!b.lit_desc.empty()) {
    const int rc = literal_run(b, stream, ro, prm.deadline, err);
    if (rc) return rc;
  }

  // the histories of each engine, LPT order (the cached routing)
  std::vector<uint32_t> todo = b.route_todo;    // workgroup passes
  const std::vector<uint32_t>& level = b.route_level;  // device-wide level search
  const bool use_pack = engine == S2LC_ENGINE_AUTO;
  // histories settled by pack_kernel<8> / <16> (roofline accounting of those kernels)
  std::vector<uint8_t> pack_done(b.n_hist, 0);  // 8 or 16: the kernel that settled it
  const uint32_t n_packed = b.n_pack8 + b.n_pack16 + b.n_pack32;
  if (use_pack && n_packed) {
#ifdef S2LC_PROF
    {
      unsigned long long z[16] = {0};
      HIPCHK(hipMemcpyToSymbol(HIP_SYMBOL(g_prof), z, sizeof z));
    }
#endif
    // Packed passes: one L-lane group per history (K <= 8: L = 8, K <= 16:
    // L = 16, K <= 32: L = 32), frontier <= PACK_F. All launches, then
    // (witness on) the walk of the histories they settled, then one results
    // read-back: a batch that needs no other pass (all of C4) costs a single
    // host sync per run.
    bool launched[3] = {false, false, false};
    const uint32_t n_list[3] = {b.n_pack8, b.n_pack16, b.n_pack32};
    const uint32_t first[3] = {0, b.n_pack8, b.n_pack8 + b.n_pack16};
    for (int li = 0; li < 3; ++li) {
      const uint32_t n_l = n_list[li];
      if (n_l == 0) continue;
      Params pp = prm;
      pp.order = b.order + first[li];
      pp.n_hist = n_l;
      pp.counter = ctr + 12 + li;
      pp.agg = agg + 8 * li;
      const bool first_launch = !(launched[0] || launched[1] || launched[2]);
      pp.zero_ctr = no_reset && first_launch ? b.counter + 32 * (par ^ 1u) : nullptr;
      pp.zero_agg = no_reset && first_launch ? b.agg + 32 * (par ^ 1u) : nullptr;
      const uint32_t L = 8u << li;
      const size_t smem = li == 0 ? pack_smem_bytes<8>() : li == 1 ? pack_smem_bytes<16>() : pack_smem_bytes<32>();
      // SMALL: every history of the list reads its 32-byte records (H_SMALL)
      const bool sm = b.list_small[li];
      int& bpc_c = sm ? b.pack_bpc_s[li] : b.pack_bpc[li];
      int bpc = bpc_c;  // resident blocks per CU (queried once per batch)
      if (bpc == 0) {
        if (li == 0) HIPCHK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&bpc, sm ? pack_kernel<8, true> : pack_kernel<8>, PACK_BLOCK, smem));
        else if (li == 1) HIPCHK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&bpc, sm ? pack_kernel<16, true> : pack_kernel<16>, PACK_BLOCK, smem));
        else HIPCHK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&bpc, sm ? pack_kernel<32, true> : pack_kernel<32>, PACK_BLOCK, smem));
        bpc = std::max(1, bpc);
        if (const char* e = getenv("S2LC_PACK_BPC")) bpc = std::max(1, atoi(e));  // (diagnostics: grid blocks per CU)
        bpc_c = bpc;
      }
      // lane groups per wave that take histories: 1 up to half a history per
      // resident wave, 2 up to 4, then 4 (x2 per x8). The groups of a wave
      // run in lockstep, so fewer per wave give shorter rounds; more groups
      // per wave issue one instruction stream for several histories, which
      // wins once the SIMDs are shared. C4 sweeps (tools/gpw_sweep.sh), ms at
      // 1 / 2 / 4 groups. 64-byte records, 2 blocks per CU (2,048 waves;
      // profiles/r04/gpw_sweep.txt): 1,000 histories 0.97 / 1.10 / 1.26;
      // 2,500 1.53 / 1.10 / 1.27; 6,000 1.90 / 1.28 / 1.34; 10,000 2.38 /
      // 1.63 / 1.35. 32-byte records, 3 blocks per CU (3,072 waves;
      // profiles/r05/gpw_sweep_srec.txt): 1,000 0.92 / 1.01 / 1.16; 4,000
      // 1.30 / 0.98 / 1.12; 10,000 1.66 / 1.09 / 1.18.
      const uint32_t gpw_all = 64 / L;
      const uint64_t waves = (uint64_t)n_cu * (uint64_t)bpc * (PACK_BLOCK / 64);
      uint32_t gpw = 1;
      for (uint64_t lim2 = 1; gpw < gpw_all && (uint64_t)n_l * 2 > waves * lim2; lim2 *= 8) gpw *= 2;
      if (const char* e = getenv("S2LC_PACK_GPW")) gpw = std::max<uint32_t>(1, std::min<uint32_t>(gpw_all, (uint32_t)atoi(e)));
      pp.gpw = gpw < gpw_all ? gpw : 0u;
      const uint32_t groups = (PACK_BLOCK / 64) * gpw;
      const uint32_t grid = std::max<uint32_t>(
          1, std::min<uint32_t>((n_l + groups - 1) / groups, (uint32_t)n_cu * (uint32_t)std::max(1, bpc)));
      // start / stop timestamps taken by the dispatch itself (no marker packets
      // around it: with hipEventRecord the launch started 20-30 us after the
      // previous kernel ended, rocprofv3 trace r03a)
      hipEvent_t e0 = b.ev[2 * li], e1 = b.ev[2 * li + 1];
      if (li == 0) hipExtLaunchKernelGGL(sm ? pack_kernel<8, true> : pack_kernel<8>, dim3(grid), dim3(PACK_BLOCK), smem, stream, e0, e1, 0, pp);
      else if (li == 1) hipExtLaunchKernelGGL(sm ? pack_kernel<16, true> : pack_kernel<16>, dim3(grid), dim3(PACK_BLOCK), smem, stream, e0, e1, 0, pp);
      else hipExtLaunchKernelGGL(sm ? pack_kernel<32, true> : pack_kernel<32>, dim3(grid), dim3(PACK_BLOCK), smem, stream, e0, e1, 0, pp);
      HIPCHK(hipGetLastError());
      if (pp.zero_ctr) b.force_reset = false;
      launched[li] = true;
      st.launches++;
    }
    // (pack_kernel resolves its histories' witnesses itself: no walk here)
    // Fast path: every history of the batch is in a packed list and no
    // round counts are wanted. The run then reads back only the launches'
    // totals; the per-history results stay on the device until asked for
    // (batch_host_results). A history that outgrew its packed frontier sends
    // the run down the full path (results read back, overflow scan).
    const bool fast = todo.empty() && level.empty() && !ro.round_counts && b.lit_desc.empty() &&
                      n_packed + n_forced == b.n_hist;
    if (fast)
      HIPCHK(hipMemcpyAsync(b.h_agg, agg, 24 * sizeof(unsigned long long), hipMemcpyDeviceToHost, stream));
    else
      HIPCHK(hipMemcpyAsync(b.h_res, b.res, b.n_hist * sizeof(HistResult), hipMemcpyDeviceToHost, stream));
    t_enq = steady_ns();
    HIPCHK(stream_wait(stream, b.ev[6]));
    t_wait = steady_ns();
#ifdef S2LC_PROF
    {
      unsigned long long gp[16];
      HIPCHK(hipMemcpyFromSymbol(gp, HIP_SYMBOL(g_prof), sizeof gp));
      const double rd = gp[13] ? (double)gp[13] : 1.0;
      fprintf(stderr, "[s2lc prof] pack: rounds %llu children %llu | cycles/round expand %.0f closure %.0f dedupe+rest %.0f"
              " | closure passes/round %.2f, of which with a window reload %.2f\n",
              gp[13], gp[15], gp[10] / rd, gp[11] / rd, gp[12] / rd, gp[8] / rd, gp[9] / rd);
    }
#endif
    if (fast && b.h_agg[PACK_AGG_OVERFLOW] + b.h_agg[8 + PACK_AGG_OVERFLOW] + b.h_agg[16 + PACK_AGG_OVERFLOW] == 0) {
      for (int li = 0; li < 3; ++li) {
        if (!launched[li]) continue;
        float ms = 0;
        HIPCHK(hipEventElapsedTime(&ms, b.ev[2 * li], b.ev[2 * li + 1]));
        st.kernel_ms += ms;
        st.pack_ms += ms;
        if (li == 0) st.pack8_ms = ms;
        if (li == 1) st.pack16_ms = ms;
        const unsigned long long* a = b.h_agg + 8 * li;
        st.configs += a[PACK_AGG_CONFIGS];
        st.children += a[PACK_AGG_CHILDREN];
        st.rounds += a[PACK_AGG_ROUNDS];
        st.algo_bytes += a[PACK_AGG_SEARCH_BYTES];
        // (S2LC_PACK8 lists settle in pack_kernel<8>; the 32-lane list is not a roofline line)
        if (li == 0) { st.pack8_algo_bytes = a[PACK_AGG_SEARCH_BYTES] + b.in_bytes_list[0]; st.pack8_histories = (uint32_t)a[PACK_AGG_SETTLED]; }
        if (li == 1) {
          st.pack16_algo_bytes = a[PACK_AGG_SEARCH_BYTES] + b.in_bytes_list[1];
          st.pack16_histories = (uint32_t)a[PACK_AGG_SETTLED];
          st.pack16_small = b.list_small[1] ? st.pack16_histories : 0u;
        }
      }
      st.algo_bytes += b.algo_bytes_inputs;
      b.h_res_stale = true;
      const int64_t t_end = steady_ns();
      st.total_ms = (double)(t_end - t0) * 1e-6;
      if (step_timing)
        fprintf(stderr, "[s2lc step] enqueue %.1f us, wait %.1f us (kernel %.1f us), after %.1f us (totals only); "
                "pack16 blocks/CU %d\n",
                1e-3 * (t_enq - t0), 1e-3 * (t_wait - t_enq), 1e3 * st.pack_ms, 1e-3 * (t_end - t_wait),
                b.list_small[1] ? b.pack_bpc_s[1] : b.pack_bpc[1]);
      return 0;
    }
    if (fast)  // a packed frontier overflowed: the full path needs every result
      HIPCHK(hipMemcpy(b.h_res, b.res, b.n_hist * sizeof(HistResult), hipMemcpyDeviceToHost));
    for (int li = 0; li < 3; ++li) {
      if (!launched[li]) continue;
      float ms = 0;
      HIPCHK(hipEventElapsedTime(&ms, b.ev[2 * li], b.ev[2 * li + 1]));
      st.kernel_ms += ms;
      st.pack_ms += ms;
      if (li == 0) st.pack8_ms = ms;
      if (li == 1) st.pack16_ms = ms;
    }
    t_ev = steady_ns();
    // histories that outgrew the packed frontier go on to the workgroup passes
    // (in history order: h_hist / h_res are pinned host memory, slow to read
    // in LPT order — 180-240 us per C4 step — and fast sequentially)
    std::vector<uint32_t> over;
    for (uint32_t i = 0; i < b.n_hist; ++i) {
      const HistDesc& hd = b.h_hist[i];
      if (hd.K > 32 || !(hd.flags & H_TAIL32) || b.forced[i]) continue;
      if (b.h_res[i].verdict == V_UNKNOWN && b.h_res[i].reason == S2LC_R_FRONTIER) over.push_back(i);
      else if (hd.K <= b.pack8_kmax) pack_done[i] = 8;
      else if (hd.K <= 16) pack_done[i] = 16;
    }
    if (over.size() > 1) {  // back to LPT order for the workgroup passes
      std::vector<uint32_t> rank(b.n_hist);
      for (uint32_t k = 0; k < (uint32_t)b.lpt.size(); ++k) rank[b.lpt[k]] = k;
      std::sort(over.begin(), over.end(), [&](uint32_t x, uint32_t y) { return rank[x] < rank[y]; });
    }
    st.n_overflow = (uint32_t)over.size();
    over.insert(over.end(), todo.begin(), todo.end());
    todo.swap(over);
    t_over = steady_ns();
  }
  const uint32_t lds_fcap = 8;
  const uint32_t lds_stage = 32;
  const size_t lds_budget = b.kmax <= 16 ? 10240 : b.kmax <= 32 ? 13312 : 0;
  int n_passes_run = 0;
  for (int pass = engine == S2LC_ENGINE_WORKGROUP_HBM ? 1 : 0; pass < 2; ++pass) {
    const uint32_t n_pass = (uint32_t)todo.size();
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
    if (!g.shared && grow_device(&b.slab, b.slab_cap, g.slab_bytes * g.grid, err)) return S2LC_EHIP;
    Params pp = prm;
    HIPCHK(hipMemcpyAsync(b.list, todo.data(), todo.size() * sizeof(uint32_t), hipMemcpyHostToDevice, stream));
    pp.order = b.list;
    pp.n_hist = n_pass;
    pp.counter = ctr + 4 * pass;
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
    HIPCHK(hipEventRecord(b.ev[4], stream));
    HIPCHK(launch_geom(g, pp, stream));
    HIPCHK(hipEventRecord(b.ev[5], stream));
    st.launches++;
    HIPCHK(hipMemcpyAsync(b.h_res, b.res, b.n_hist * sizeof(HistResult), hipMemcpyDeviceToHost, stream));
    HIPCHK(stream_wait(stream, b.ev[6]));
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
    HIPCHK(hipEventElapsedTime(&ms, b.ev[4], b.ev[5]));
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
    // histories of THIS pass that outgrew its frontier go to the next pass
    std::vector<uint32_t> next;
    for (uint32_t i : todo)
      if (b.h_res[i].verdict == V_UNKNOWN && b.h_res[i].reason == S2LC_R_FRONTIER) next.push_back(i);
    if (pass == 0) st.n_overflow += (uint32_t)next.size();
    else st.n_overflow2 += (uint32_t)next.size();
    todo.swap(next);
  }
  // the device-wide level search, one history at a time: histories with more
  // than 128 chains and those whose frontier outgrew the workgroup passes
  todo.insert(todo.end(), level.begin(), level.end());
  for (uint32_t h : todo) {
    const int rc = level_search(b, h, stream, ro, deadline_ns, prm.deadline, st.level, err);
    if (rc) return rc;
  }
  st.kernel_ms += st.level.ms;
  // the packed histories were walked with the packed launches; walk again only
  // for what the other passes settled (walk_kernel skips walked histories)
  const bool other_work = n_passes_run > 0 || !todo.empty() || !use_pack;
  if (witness && b.n_hist && other_work) {
    hipLaunchKernelGGL(walk_kernel, dim3((b.n_hist + 3) / 4), dim3(256), 0, stream, b.n_hist, b.res,
                       (const TraceEnt*)b.trace, b.moves);
    HIPCHK(hipGetLastError());
  }
  if (b.n_hist && (other_work || !(b.n_pack8 + b.n_pack16 + b.n_pack32)))
    HIPCHK(hipMemcpyAsync(b.h_res, b.res, b.n_hist * sizeof(HistResult), hipMemcpyDeviceToHost, stream));
  bool tail_work = false;
  if (witness && b.n_hist && other_work) tail_work = true;
  if (b.n_hist && (other_work || !(b.n_pack8 + b.n_pack16 + b.n_pack32))) tail_work = true;
  if (ro.round_counts) {  // every engine wrote its rounds' counts on the device
    b.h_rcounts.resize(std::max<uint64_t>(b.moves_cap, 1));
    HIPCHK(hipMemcpyAsync(b.h_rcounts.data(), b.rcounts, b.moves_cap * sizeof(uint32_t), hipMemcpyDeviceToHost, stream));
    tail_work = true;
  }
  if (tail_work) HIPCHK(stream_wait(stream, b.ev[6]));
  t_tail = steady_ns();
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
    if (pack_done[i] == 16) {
      // pack_kernel<16> alone: its histories' search bytes + their input SoA
      st.pack16_algo_bytes += 2 * S * r.configs + 8 * r.children + b.h_in_bytes[i];
      st.pack16_histories++;
      if (b.list_small[1]) st.pack16_small++;
    } else if (pack_done[i] == 8) {
      st.pack8_algo_bytes += 2 * S * r.configs + 8 * r.children + b.h_in_bytes[i];
      st.pack8_histories++;
    }
  }
  b.rc_valid = ro.round_counts;
  st.algo_bytes += b.algo_bytes_inputs;
  const int64_t t_end = steady_ns();
  st.total_ms = (double)(t_end - t0) * 1e-6;
  if (step_timing && t_enq)
    fprintf(stderr, "[s2lc step] enqueue %.1f us, wait %.1f us (kernel %.1f us), after %.1f us: events %.1f, overflow scan %.1f, "
            "tail %.1f, stats %.1f\n", 1e-3 * (t_enq - t0), 1e-3 * (t_wait - t_enq), 1e3 * st.pack_ms,
            1e-3 * (t_end - t_wait), 1e-3 * (t_ev - t_wait), 1e-3 * (t_over - t_ev), 1e-3 * (t_tail - t_over),
            1e-3 * (t_end - t_tail));
  return 0;
}


int batch_host_results(DevBatch& b, std::string& err) {
  if (!b.h_res_stale) return 0;
  HIPCHK(hipMemcpy(b.h_res, b.res, b.n_hist * sizeof(HistResult), hipMemcpyDeviceToHost));
  for (uint32_t i = 0; i < b.n_hist; ++i)
    if (b.forced[i]) {
      b.h_res[i] = HistResult{};
      b.h_res[i].verdict = V_ILLEGAL;
      b.h_res[i].reason = S2LC_R_UNMATCHED;
      b.h_res[i].witness_off = b.h_moves_off[i];
    }
  b.h_res_stale = false;
  return 0;
}

int batch_fetch_moves(DevBatch& b, std::string& err) {
  if (grow_pinned(reinterpret_cast<uint8_t**>(&b.h_moves), b.h_moves_cap, std::max<uint64_t>(b.moves_cap, 1) * sizeof(uint32_t),
                  err))
    return S2LC_EHIP;
  if (b.moves_cap) HIPCHK(hipMemcpy(b.h_moves, b.moves, b.moves_cap * sizeof(uint32_t), hipMemcpyDeviceToHost));
  return 0;
}

namespace {
// foldRecordHashes through the search kernels' own device routine
__global__ void fold_kernel(uint32_t n, const uint64_t* seeds, const uint64_t* pool, const uint32_t* offs,
                            const uint32_t* cnts, uint64_t* out) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) out[i] = fold_hashes_blk(seeds[i], pool + offs[i], cnts[i]);
}
}  // namespace

int device_fold(const uint64_t* seeds, const uint64_t* pool, size_t pool_len, const uint32_t* offs, const uint32_t* cnts,
                size_t n, uint64_t* out, hipStream_t stream, std::string& err) {
  for (size_t i = 0; i < n; ++i)
    if ((uint64_t)offs[i] + cnts[i] > pool_len) { err = "fold range outside the pool"; return S2LC_EINVAL; }
  if (n == 0) return 0;
  uint8_t* d = nullptr;
  const size_t o_pool = align256(n * 8), o_offs = align256(o_pool + std::max<size_t>(pool_len, 1) * 8),
               o_cnts = align256(o_offs + n * 4), o_out = align256(o_cnts + n * 4), total = o_out + n * 8;
  HIPCHK(hipMalloc(&d, total));
  hipError_t e = hipMemcpyAsync(d, seeds, n * 8, hipMemcpyHostToDevice, stream);
  if (e == hipSuccess && pool_len) e = hipMemcpyAsync(d + o_pool, pool, pool_len * 8, hipMemcpyHostToDevice, stream);
  if (e == hipSuccess) e = hipMemcpyAsync(d + o_offs, offs, n * 4, hipMemcpyHostToDevice, stream);
  if (e == hipSuccess) e = hipMemcpyAsync(d + o_cnts, cnts, n * 4, hipMemcpyHostToDevice, stream);
  if (e == hipSuccess) {
    hipLaunchKernelGGL(fold_kernel, dim3((uint32_t)((n + 255) / 256)), dim3(256), 0, stream, (uint32_t)n,
                       (const uint64_t*)d, (const uint64_t*)(d + o_pool), (const uint32_t*)(d + o_offs),
                       (const uint32_t*)(d + o_cnts), (uint64_t*)(d + o_out));
    e = hipGetLastError();
  }
  if (e == hipSuccess) e = hipMemcpyAsync(out, d + o_out, n * 8, hipMemcpyDeviceToHost, stream);
  if (e == hipSuccess) e = hipStreamSynchronize(stream);
  (void)hipFree(d);
  if (e != hipSuccess) { err = std::string("device fold: ") + hipGetErrorString(e); return S2LC_EHIP; }
  return 0;
}

}  // namespace s2lc
