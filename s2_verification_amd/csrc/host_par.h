// host_par.h — a small parallel-for over [0, n) for the host-side stages of a
// batch (packing the device SoA, rebuilding and certifying witnesses). Threads
// = S2LC_HOST_THREADS, else min(16, hardware threads) (16 = one GPU's CPU
// share on the MI355X boxes); small ranges run inline.
#pragma once
#include <stdlib.h>

#include <algorithm>
#include <atomic>
#include <thread>
#include <vector>

namespace s2lc {

inline unsigned host_threads() {
  if (const char* e = getenv("S2LC_HOST_THREADS")) {
    const long v = strtol(e, nullptr, 10);
    if (v >= 1) return (unsigned)std::min<long>(v, 256);
  }
  return std::max(1u, std::min(16u, std::thread::hardware_concurrency()));
}

// fn(i) for every i in [0, n), in chunks of `grain` handed out dynamically.
template <typename F>
void parallel_for(size_t n, size_t grain, F&& fn) {
  const unsigned nt = (unsigned)std::min<size_t>(host_threads(), (n + grain - 1) / std::max<size_t>(grain, 1));
  if (nt <= 1) {
    for (size_t i = 0; i < n; ++i) fn(i);
    return;
  }
  std::atomic<size_t> next{0};
  auto work = [&]() {
    for (;;) {
      const size_t b = next.fetch_add(grain);
      if (b >= n) return;
      const size_t e = std::min(n, b + grain);
      for (size_t i = b; i < e; ++i) fn(i);
    }
  };
  std::vector<std::thread> ts;
  ts.reserve(nt - 1);
  for (unsigned t = 1; t < nt; ++t) ts.emplace_back(work);
  work();
  for (auto& t : ts) t.join();
}

}  // namespace s2lc
